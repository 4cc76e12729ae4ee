#!/bin/bash
# time every variants/lib_*.so with the sampled-forward microbench (split precisions)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 120 python tools/sampbench.py --prec f32x9 f32x6 > gpurun_out/sbv_base.log 2>&1
for f in variants/lib_*.so; do
v=$(basename $f .so); v=${v#lib_}
IKEA_REC_HIP_LIB=$PWD/$f timeout -k 10 120 python tools/sampbench.py --prec f32x9 f32x6 > gpurun_out/sbv_$v.log 2>&1
done
