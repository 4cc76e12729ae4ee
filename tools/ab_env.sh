#!/bin/bash
# same-box A/B of an environment switch on a short bench: ENVVAR, CFG (default c2)
set -o pipefail
for v in 0 1 0 1; do
  env $ENVVAR=$v timeout -k 10 300 python bench.py --config ${CFG:-c2} --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$ENVVAR=$v', d['value'], d['ms_per_step'], d['step_ms'])" || exit 1
done
