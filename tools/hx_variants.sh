#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 120 python tools/headx.py > gpurun_out/hxv_base.log 2>&1
for f in variants/lib_*.so; do
v=$(basename $f .so); v=${v#lib_}
IKEA_REC_HIP_LIB=$PWD/$f timeout -k 10 120 python tools/headx.py > gpurun_out/hxv_$v.log 2>&1
done
