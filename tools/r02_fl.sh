#!/bin/bash
# fused head: parity tests, then pass timings at C2 shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_flash_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_fl.log 2>&1; rc=$?; tail -3 gpurun_out/t_fl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/flashx.py --terms 6 --iters 3
