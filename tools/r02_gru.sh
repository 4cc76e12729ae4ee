#!/bin/bash
# persistent wide GRU (H 256): kernel parity, then the H 256 trainers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_qlearning.py tests/test_gpu_supervised.py -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gru.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gru.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gru.log | tail -3
