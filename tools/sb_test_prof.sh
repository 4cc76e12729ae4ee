#!/bin/bash
# sampled parity tests, then microbench + rocprofv3 summary
set -e
tag=${1:-sb}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampled.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
bash tools/sb_prof.sh $tag
