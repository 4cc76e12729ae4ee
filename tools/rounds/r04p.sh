#!/bin/bash
# Q heads' dense Adam sweeps on their own stream: Q-learning GPU tests, C4 same-box A/B (RG_ONE_Q=1: one stream), sharded C4
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qlearning.py tests/test_gpu_dist_q.py tests/test_gpu_ckpt_eval.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in "" 1 "" 1 "" 1; do
RG_ONE_Q=$v timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('c4 oneq=${v:-0}', d['value'], d['ms_per_step'], d['step_ms']['median'])"
done
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29537
for v in "" 1 "" 1; do
RG_ONE_Q=$v timeout -k 10 300 python bench.py --config c4 --force-shard --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > $O/s.json 2>/dev/null || exit 1
python -c "import json;d=json.loads(open('$O/s.json').read().strip().splitlines()[-1]);print('c4shard oneq=${v:-0}', d['value'], d['ms_per_step'], d['step_ms']['median'])"
done
