set -o pipefail
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_flash_head.py tests/test_gpu_model_parity.py tests/test_gpu_supervised.py tests/test_gpu_ckpt_eval.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in "" variants/lib_ep0.so "" variants/lib_ep0.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 2>&1 | grep pass2 | sed "s|^|lib=${v:-tree} |" || exit 1
done
bash tools/pmc_head.sh
