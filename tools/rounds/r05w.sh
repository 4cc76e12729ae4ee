#!/bin/bash
# round 4: stored-logit pass 2 bottleneck diagnostics (flashx --zs): without the R-plane LDS reads, without the
# z stream, without the dZ VALU (diagnostic builds, wrong results)
set -o pipefail
mkdir -p gpurun_out/r05w
for cfg in "tree|--zs" "abvar/lib_zdNOLDS.so|--zs" "abvar/lib_zdNOZ.so|--zs" "abvar/lib_zdNOVALU.so|--zs" "tree|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass2 | sed "s#^#${cfg} #" | tee -a gpurun_out/r05w/flashx.txt || exit 1
done
