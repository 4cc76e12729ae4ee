#!/bin/bash
# full snapshot after the pre-gathered negatives + XCD mapping
set -o pipefail
bash tools/gpu_snapshot.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread -m gpu tests/test_gpu_long_horizon.py > gpurun_out/snap/long.txt 2>&1; tail -1 gpurun_out/snap/long.txt
