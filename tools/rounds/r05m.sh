#!/bin/bash
# round 4: Q-head / sampled changes' tests, then the C3 A/B (tools/rounds/r05l.sh)
set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 600 python -u -m pytest tests/test_gpu_qlearning.py tests/test_gpu_dist_q.py tests/test_gpu_ckpt_eval.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05m/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05m/pytest.txt | tail -20; tail -30 gpurun_out/r05m/pytest.txt; exit 1; }
tail -2 gpurun_out/r05m/pytest.txt
bash tools/rounds/r05l.sh
