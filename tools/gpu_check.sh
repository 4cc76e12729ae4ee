#!/bin/bash
# Full GPU verification of a tree: gpu test suite, smoke, C2/C3 bench lines,
# rocprofv3 kernel-trace summaries.  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -e
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${tag}.log 2>&1
bash tools/prof_bench.sh $tag
