#!/bin/bash
# Fused head: parity tests + stage microbench.  Usage: bash tools/fl_quick.sh tag
set -e
tag=${1:-flq}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_head.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
timeout -k 10 120 python tools/flashx.py > gpurun_out/fx_${tag}.log 2>&1
