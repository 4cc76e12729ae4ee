set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
V=${VARIANT:-variants/lib_zt.so}
IKEA_REC_HIP_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampled.py > $O/pytest_variant.txt 2>&1 || { tail -30 $O/pytest_variant.txt; exit 1; }
tail -2 $O/pytest_variant.txt
for v in "" $V "" $V; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/sampbench.py --HF 128 256 --prec f32x6 --fused --planes 2>&1 | grep fused | sed "s|^|lib=${v:-tree} |" || exit 1
done
