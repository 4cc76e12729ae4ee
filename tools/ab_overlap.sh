#!/bin/bash
# A/B: the head's pass 2 on a side stream under the trunk backward (RG_OVERLAP_HEAD_DW=1) vs in line
set -o pipefail
for v in 0 1 0 1; do
  RG_OVERLAP_HEAD_DW=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('overlap $v', d['value'], d['ms_per_step'], d['step_ms'])" || exit 1
done
