#!/bin/bash
# eval_batch reads the screening overflow flag once at its end: eval / checkpoint-eval GPU tests, harness numbers
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_eval.py tests/test_gpu_ckpt_eval.py tests/test_gpu_model_parity.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-target > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));h=d['harness'];print('harness', h['harness_ms_per_step'], h['update_train_metrics_ms'], h['value'], 'train', d['ms_per_step'], 'eval', d['eval_heldout']['hr20'], d['eval_heldout']['ms'])"
done
