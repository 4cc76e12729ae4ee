#!/bin/bash
# sampled head: GPU parity tests, then the forward timings (two-launch Zᵀ path and the one-launch fused path)
cd $GRAFT_REPO_ROOT
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sampled.log 2>&1; rc=$?; tail -3 gpurun_out/t_sampled.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 f32x9 --fused --iters 100
