#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_head.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_hx.log 2>&1
bash tools/hx_variants.sh
