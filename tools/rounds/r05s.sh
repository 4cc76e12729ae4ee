#!/bin/bash
# round 4: stored-logit diagnostics (flashx): plain vs non-temporal z stores in pass 1; pass 2 without the
# LDS transposes (diagnostic, wrong results)
set -o pipefail
mkdir -p gpurun_out/r05s
for cfg in "tree|" "tree|--zs" "abvar/lib_zsplain.so|--zs" "abvar/lib_zsnotrans.so|--zs" "tree|--zs" "abvar/lib_zsplain.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#${cfg} #" | tee -a gpurun_out/r05s/flashx.txt || exit 1
done
