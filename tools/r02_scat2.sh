#!/bin/bash
# scatter parity + timings, trainer tests, then short C2/C3 benches
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_supervised.py tests/test_gpu_sampled.py tests/test_gpu_ckpt_eval.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sc2.log 2>&1; rc=$?; tail -3 gpurun_out/t_sc2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/scatbench.py || exit 1
./tools/r02_c23.sh
