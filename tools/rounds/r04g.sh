#!/bin/bash
# pass 1 with the second half of the waves one O-part behind (FL_DEFER) vs tree
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
IKEA_REC_HIP_LIB=variants/lib_defer.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_flash_head.py tests/test_gpu_model_parity.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in flstamp fldefer; do IKEA_REC_HIP_LIB=variants/lib_$v.so timeout -k 10 120 python tools/flstamp.py 2>&1 | grep -E "pass1|barrier" | sed "s|^|$v |" || exit 1; done
for v in "" variants/lib_defer.so "" variants/lib_defer.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 2>&1 | grep -E "pass1" | sed "s|^|lib=${v:-tree} |" || exit 1
done
for v in "" variants/lib_defer.so "" variants/lib_defer.so; do
IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('lib=${v:-tree}', d['value'], d['ms_per_step'], d['step_ms']['median'], d['kernel_ms']['head_fwd'], d['kernel_ms']['head_dw_adam'])"
done
