#!/bin/bash
# same-box A/B of two head precisions on a short bench: PA, PB (default f32x6 / f32x6d3), CFG (default c2)
set -o pipefail
for p in ${PA:-f32x6} ${PB:-f32x6d3} ${PA:-f32x6} ${PB:-f32x6d3}; do
  timeout -k 10 300 python bench.py --config ${CFG:-c2} --precision $p --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$p', d['value'], d['ms_per_step'], d['step_ms'])" || exit 1
done
