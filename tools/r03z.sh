#!/bin/bash
# sampled-logits phase stamps (diagnostic builds: tree-equivalent, no W loads, no h DMA, coalesced W rows, neither)
set -o pipefail
for r in 1 2; do
for v in sfstamp sfnow sfnoh sfcoal sfnone; do
  echo "== $v"
  IKEA_REC_HIP_LIB=variants/lib_$v.so timeout -k 10 120 python tools/sfstamp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
done
