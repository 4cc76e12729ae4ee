#!/bin/bash
# sampled-forward microbench + its rocprofv3 kernel-trace summary
set -e
tag=${1:-sb}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/sampbench.py > gpurun_out/${tag}.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o sb -- python3 tools/sampbench.py --iters 20 > gpurun_out/prof_${tag}.log 2>&1
