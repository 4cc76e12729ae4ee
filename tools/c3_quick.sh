#!/bin/bash
# Sampled-softmax parity (+ split-head forward) and the C3 bench line.
set -e
tag=${1:-c3q}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampled.py tests/test_gpu_split_head.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_${tag}_c3.json 2> gpurun_out/bench_${tag}_c3.err
