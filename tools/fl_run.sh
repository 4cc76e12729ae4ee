#!/bin/bash
# Fused split-bf16 head (csrc/head_flash.hip) on the GPU box: parity tests,
# then C2 bench lines at f32x6 / f32x9.  Usage: bash tools/fl_run.sh [tag]
set -e
tag=${1:-fl}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 420 python -u -m pytest tests/test_gpu_flash_head.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
for p in f32x6 f32x9; do
  timeout -k 10 300 python bench.py --precision $p --no-cpu-baseline --no-target \
    > gpurun_out/bench_${tag}_${p}.json 2> gpurun_out/bench_${tag}_${p}.err
done
