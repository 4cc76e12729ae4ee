#!/bin/bash
# pass-2 epilogue with prefetched W / m / v (tree) vs guarded per-q loads (ep_old): flashx + C2 bench + flash tests
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_flash_head.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in "" variants/lib_ep_old.so "" variants/lib_ep_old.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 2>&1 | grep pass2 | sed "s|^|lib=${v:-tree} |" || exit 1
done
for v in "" variants/lib_ep_old.so "" variants/lib_ep_old.so; do
IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('lib=${v:-tree}', d['value'], d['ms_per_step'], d['step_ms']['median'], d['kernel_ms']['head_dw_adam'])"
done
