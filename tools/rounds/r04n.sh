#!/bin/bash
# trunk backward's GRU-weight path on a side stream: GPU suite, then same-box A/B (RG_ONE_STREAM=1: one stream) C2 / C4 / C3 / sharded C2
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_long_horizon.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for cfg in c2 c4 c3; do
for v in "" 1 "" 1; do
RG_ONE_STREAM=$v timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('$cfg one=${v:-0}', d['value'], d['ms_per_step'], d['step_ms']['median'])"
done
done
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535
for v in "" 1 "" 1; do
RG_ONE_STREAM=$v timeout -k 10 300 python bench.py --force-shard --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > $O/s.json 2>/dev/null || exit 1
python -c "import json;d=json.loads(open('$O/s.json').read().strip().splitlines()[-1]);print('c2shard one=${v:-0}', d['value'], d['ms_per_step'], d['step_ms']['median'])"
done
