#!/bin/bash
# round 4: stored-logit pass 1 without its stores (diagnostic build) vs shipped vs recomputing
set -o pipefail
mkdir -p gpurun_out/r06a
for cfg in "tree|" "tree|--zs" "abvar/lib_zsnostore.so|--zs" "tree|--zs" "abvar/lib_zsnostore.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass1 | sed "s#^#${cfg} #" | tee -a gpurun_out/r06a/flashx.txt || exit 1
done
