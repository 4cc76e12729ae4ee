#!/bin/bash
set -e
tag=${1:-hx}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_head.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
timeout -k 10 120 python tools/headx.py > gpurun_out/${tag}.log 2>&1
