#!/bin/bash
# fused head A/B on one box: pass timings of the base library vs variants (twice, interleaved)
set -o pipefail
for rep in 1 2; do
for v in base OLD; do
  if [ $v = base ]; then unset IKEA_REC_HIP_LIB; else export IKEA_REC_HIP_LIB=$PWD/variants/lib_$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/flashx.py --terms 6 --iters 3 | grep pass || exit 1
done
done
