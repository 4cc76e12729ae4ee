#!/bin/bash
# round 4: pass 1 with chunk c-1's z stores deferred under chunk c's S-part (ZS_DEFER) vs shipped; correctness of the
# variant via the stored-logit kernel tests
set -o pipefail
mkdir -p gpurun_out/r06j
IKEA_REC_HIP_LIB=abvar/lib_zsdefer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_flash_head.py -k "stored_logit" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06j/pytest.txt 2>&1 || { tail -30 gpurun_out/r06j/pytest.txt; exit 1; }
tail -1 gpurun_out/r06j/pytest.txt
for cfg in "tree|--zs" "abvar/lib_zsdefer.so|--zs" "tree|--zs" "abvar/lib_zsdefer.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass1 | sed "s#^#${cfg} #" | tee -a gpurun_out/r06j/flashx.txt || exit 1
done
