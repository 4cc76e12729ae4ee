#!/bin/bash
# Sampled forward microbench + per-kernel rocprof stats (prep vs logits kernel)
set -e
tag=${1:-sbs}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/sampbench.py --prec f32 f32x6 > gpurun_out/${tag}.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o s -- python3 tools/sampbench.py --prec f32x6 --iters 20 > gpurun_out/prof_${tag}.log 2>&1
