set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_flash_head.py tests/test_gpu_sampled.py tests/test_gpu_kernels.py tests/test_gpu_eval.py > $O/pytest_a.txt 2>&1 || { tail -40 $O/pytest_a.txt; exit 1; }
tail -2 $O/pytest_a.txt
for v in "" variants/lib_old32.so "" variants/lib_old32.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 2>&1 | grep pass | sed "s|^|lib=${v:-tree} |" || exit 1
done
