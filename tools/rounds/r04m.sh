#!/bin/bash
# pass 2's side stream at high priority (RG_SIDE_PRIO=-1) vs default: C2 / C4 same box
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for cfg in c2 c4; do
for v in 0 -1 0 -1; do
RG_SIDE_PRIO=$v timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('$cfg prio=$v', d['value'], d['ms_per_step'], d['step_ms']['median'])"
done
done
