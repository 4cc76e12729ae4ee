#!/bin/bash
# Fused-head microbench: base library, then each variants/lib_fx*.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 120 python tools/flashx.py > gpurun_out/fx_base.log 2>&1
for f in variants/lib_fx*.so; do
  v=$(basename $f .so); v=${v#lib_}
  IKEA_REC_HIP_LIB=$PWD/$f timeout -k 10 120 python tools/flashx.py --terms 6 > gpurun_out/fx_$v.log 2>&1
done
