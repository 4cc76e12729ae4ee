#!/bin/bash
# round 4: stored-logit pass 2 with the W-part MFMAs before the next chunk's dZ VALU in program order (ZL_WFIRST)
set -o pipefail
mkdir -p gpurun_out/r06h
for cfg in "tree|--zs" "abvar/lib_wfirst.so|--zs" "tree|--zs" "abvar/lib_wfirst.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass2 | sed "s#^#${cfg} #" | tee -a gpurun_out/r06h/flashx.txt || exit 1
done
