#!/bin/bash
# trunk changes (pack sort, bidir single launch): kernel + trainer parity, then short C2/C3 benches
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_supervised.py tests/test_gpu_sampled.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_tr.log 2>&1; rc=$?; tail -3 gpurun_out/t_tr.log; [ $rc -eq 0 ] || exit $rc
./tools/r02_c23.sh
