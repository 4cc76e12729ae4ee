#!/bin/bash
# round 4: sampled logits with the bias store after every DMA issue (± SF_EARLY): stamps + north-star A/B; GPU suite
set -o pipefail
mkdir -p gpurun_out/r05f
for v in sfstamp sfblst sfblearlyst; do
  IKEA_REC_HIP_LIB=abvar/lib_$v.so timeout -k 10 240 python tools/sfstamp.py --wp warm 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r05f/sfstamp.txt || exit 1
done
for r in 1 2; do for v in "" abvar/lib_sfbl.so abvar/lib_sfblearly.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 240 python tools/nstime.py --reps 2 2>/dev/null | tee -a gpurun_out/r05f/nstime.txt || exit 1
done; done
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f/pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r05f/pytest.txt; exit $rc
