#!/bin/bash
# Fused head: accuracy + 2-rank sharded parity, then a rocprofv3 kernel-stats
# profile of the C2 bench at f32x6.  Usage: bash tools/fl_check.sh [tag]
set -e
tag=${1:-flc}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_dist.py -m gpu -x -v -s \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run -- \
  python bench.py --precision f32x6 --steps 5 --warmup 2 --no-cpu-baseline --no-target \
  > gpurun_out/bench_${tag}_prof.json 2> gpurun_out/bench_${tag}_prof.err
