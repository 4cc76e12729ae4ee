#!/bin/bash
# round 4: k-outer sampled logits: correctness (sampled GPU tests on the variant), phase stamps, north-star A/B; then the GPU suite
set -o pipefail
mkdir -p gpurun_out/r05e
IKEA_REC_HIP_LIB=abvar/lib_sfkout.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sampled.py tests/test_gpu_bpr.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e/pytest_sampled_kout.txt 2>&1
rc=$?; tail -3 gpurun_out/r05e/pytest_sampled_kout.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in sfstamp sfkoutst; do
  IKEA_REC_HIP_LIB=abvar/lib_$v.so timeout -k 10 240 python tools/sfstamp.py --wp warm 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r05e/sfstamp.txt || exit 1
done
for v in "" abvar/lib_sfkout.so "" abvar/lib_sfkout.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 240 python tools/nstime.py --reps 2 2>/dev/null | tee -a gpurun_out/r05e/nstime.txt || exit 1
done
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e/pytest.txt 2>&1
rc2=$?; tail -4 gpurun_out/r05e/pytest.txt
exit $(( rc > rc2 ? rc : rc2 ))
