#!/bin/bash
# fused head parity + pass timings, then the hipBLASLt bf16 GEMM ceiling on the same box
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_flash_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_fl.log 2>&1; rc=$?; tail -2 gpurun_out/t_fl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/flashx.py --terms 6 --iters 3 && timeout -k 10 120 python tools/mm_peak.py
