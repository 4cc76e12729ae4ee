#!/bin/bash
# round 4: pass 1 z stores after the O-part (ZS_LATE) vs in the softmax section
set -o pipefail
mkdir -p gpurun_out/r05t
for cfg in "tree|--zs" "abvar/lib_zslate.so|--zs" "tree|--zs" "abvar/lib_zslate.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#${cfg} #" | tee -a gpurun_out/r05t/flashx.txt || exit 1
done
