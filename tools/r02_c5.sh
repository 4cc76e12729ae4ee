#!/bin/bash
# round-2 C5 checks: flash head (HF 256, fused top-k), SMORL C5 shape, sharded fp16 / fused SMORL
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_qlearning.py tests/test_gpu_dist_q.py -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pytest_c5.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_c5.log | tail -30; tail -60 gpurun_out/pytest_c5.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_c5.log | tail -3
