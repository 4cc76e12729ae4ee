#!/bin/bash
# round 4: stored-logit pass 2, VALU / MFMA interleave patterns (flashx --zs; ZIL_MODE 0 shipped, 1 none, 2 pairs, 3 front-loaded)
set -o pipefail
mkdir -p gpurun_out/r05x
for cfg in "tree|--zs" "abvar/lib_zil1.so|--zs" "abvar/lib_zil2.so|--zs" "abvar/lib_zil3.so|--zs" "tree|--zs" "abvar/lib_zil1.so|--zs" "abvar/lib_zil2.so|--zs" "abvar/lib_zil3.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass2 | sed "s#^#${cfg} #" | tee -a gpurun_out/r05x/flashx.txt || exit 1
done
