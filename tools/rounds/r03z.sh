#!/bin/bash
# sampled-logits phase stamps: tree-equivalent vs W planes pre-gathered (cold / warm)
set -o pipefail
for r in 1 2; do
  echo "== stamp"; IKEA_REC_HIP_LIB=variants/lib_sfstamp.so timeout -k 10 120 python tools/sfstamp.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== wp cold"; IKEA_REC_HIP_LIB=variants/lib_sfwp.so timeout -k 10 120 python tools/sfstamp.py --wp cold 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== wp warm"; IKEA_REC_HIP_LIB=variants/lib_sfwp.so timeout -k 10 120 python tools/sfstamp.py --wp warm 2>&1 | grep -v amdgpu.ids || exit 1
done
