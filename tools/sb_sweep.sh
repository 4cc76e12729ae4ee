#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
for r in 32 64 128 256 512; do
  RG_SAMPLED_RPB=$r timeout -k 10 60 python tools/sampbench.py --prec f32x6 > gpurun_out/sbw_$r.log 2>&1
done
