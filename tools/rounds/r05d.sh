#!/bin/bash
# round 4: GPU suite; pass-2 item-block-outer variant (stamps + A/B); sampled-logits phase stamps (tree, SF_EARLY)
set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d/pytest.txt 2>&1
rc=$?
tail -8 gpurun_out/r05d/pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
FL2_OUT=gpurun_out/r05d/fl2_ibo.npy IKEA_REC_HIP_LIB=abvar/lib_fl2ibost.so timeout -k 10 240 python tools/fl2stamp.py 2>&1 | grep -v amdgpu.ids | head -14 | tee gpurun_out/r05d/fl2_ibo.txt || exit 1
VARIANT=abvar/lib_fl2ibo.so bash tools/ab_lib.sh 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05d/ab_ibo.txt || exit 1
for v in sfstamp sfearlyst; do
  IKEA_REC_HIP_LIB=abvar/lib_$v.so timeout -k 10 240 python tools/sfstamp.py --wp warm 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r05d/sfstamp.txt || exit 1
done
exit $rc
