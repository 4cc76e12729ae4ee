#!/bin/bash
# flash ring fix + sharded embedding: affected GPU tests, C2 bench, sampled GEMM stamps
cd $GRAFT_REPO_ROOT
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_sampled.py tests/test_gpu_dist.py tests/test_gpu_dist_q.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_b.log 2>&1; rc=$?; tail -3 gpurun_out/t_b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-native-side > gpurun_out/b_flash.json 2> gpurun_out/b_flash.err || { tail gpurun_out/b_flash.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_flash.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['kernel_ms']);print(d['north_star_target'])"
IKEA_REC_HIP_LIB=$PWD/variants/lib_STAMP.so timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 --parts --stamps
