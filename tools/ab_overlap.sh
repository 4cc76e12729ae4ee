#!/bin/bash
# A/B: the head's pass 2 on a side stream (RG_OVERLAP_HEAD_DW=1) vs in line, C2 and C4
set -o pipefail
for cfg in ${CFGS:-c2 c4}; do
for v in 0 1 0 1; do
  RG_OVERLAP_HEAD_DW=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg overlap $v', d['value'], d['ms_per_step'], d['step_ms'])" || exit 1
done
done
