set -o pipefail
VARIANTS=${VARIANTS:-stage} bash tools/r03d.sh || exit 1
for v in ${VARIANTS:-stage}; do
  IKEA_REC_HIP_LIB=variants/lib_$v.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_sampled.py  > gpurun_out/r03d/pt_$v.log 2>&1; echo "pytest $v rc=$?"; tail -2 gpurun_out/r03d/pt_$v.log
done
