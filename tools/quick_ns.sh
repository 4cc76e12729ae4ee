#!/bin/bash
# Quick north-star iteration: sampled parity tests, then the C2 bench's
# gather + sampled-logits side run per precision and a rocprofv3 kernel-trace of C3.
set -e
tag=${1:-q}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampled.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
for p in f32 f32x9 f32x6; do
timeout -k 10 300 python bench.py --no-cpu-baseline --precision $p > gpurun_out/bench_${tag}_c2_$p.json 2> gpurun_out/bench_${tag}_c2_$p.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_c3 -o c3 -- python3 bench.py --config c3 --no-cpu-baseline --precision f32x9 > gpurun_out/prof_${tag}_c3.log 2>&1
