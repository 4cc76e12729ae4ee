#!/bin/bash
# early loss readout (hip/hostsync.py) vs the full-step sync: trainer GPU tests, C2 / C3 / C4 same-box A/B
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_supervised.py tests/test_gpu_qlearning.py tests/test_gpu_sampled.py tests/test_gpu_ckpt_eval.py tests/test_gpu_model_parity.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for cfg in c3 c2 c4; do
for v in "" 1 "" 1; do
RG_LATE_SYNC=$v timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('$cfg late=${v:-0}', d['value'], d['ms_per_step'], d['step_ms']['median'])"
done
done
