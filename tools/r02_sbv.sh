#!/bin/bash
# time the fused sampled forward and its diagnostic variants (variants/lib_*.so)
cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6
for f in variants/lib_*.so; do
v=$(basename $f .so); echo "== $v"
IKEA_REC_HIP_LIB=$PWD/$f timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6
done
