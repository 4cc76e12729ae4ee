#!/bin/bash
# flash-head ring fix: parity tests, then the C2 bench (kernel_ms) and the sampled GEMM stamps
cd $GRAFT_REPO_ROOT
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_sampled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flash.log 2>&1; rc=$?; tail -3 gpurun_out/t_flash.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-native-side > gpurun_out/b_flash.json 2> gpurun_out/b_flash.err || { tail gpurun_out/b_flash.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_flash.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['kernel_ms']);print(d['north_star_target'])"
IKEA_REC_HIP_LIB=$PWD/variants/lib_STAMP.so timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 --parts --stamps
