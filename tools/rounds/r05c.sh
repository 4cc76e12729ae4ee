#!/bin/bash
# round 4: GPU suite (top_scanned fix), pass-2 stamps tree vs 3-slot ring, flashx / bench A/B of the ring
set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c/pytest.txt 2>&1
rc=$?
tail -8 gpurun_out/r05c/pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
FL2_OUT=gpurun_out/r05c/fl2_tree.npy IKEA_REC_HIP_LIB=abvar/lib_fl2stamp.so timeout -k 10 240 python tools/fl2stamp.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05c/fl2_tree.txt || exit 1
FL2_OUT=gpurun_out/r05c/fl2_ring3.npy IKEA_REC_HIP_LIB=abvar/lib_fl2ring3st.so timeout -k 10 240 python tools/fl2stamp.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05c/fl2_ring3.txt || exit 1
VARIANT=abvar/lib_fl2ring3.so bash tools/ab_lib.sh 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05c/ab_ring3.txt || exit 1
exit $rc
