#!/bin/bash
# north-star pieces: gather parity tests, sampled logits base vs no-store variant, then the C2 bench target line
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_supervised.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ns.log 2>&1; rc=$?; tail -2 gpurun_out/t_ns.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 --fused || exit 1
IKEA_REC_HIP_LIB=$PWD/variants/lib_NOSTORE.so timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 --fused || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/b_ns.json 2> gpurun_out/b_ns.err || { tail gpurun_out/b_ns.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_ns.json'));print(d['value'],d['kernel_ms']);print(d['north_star_target'])"
