#!/bin/bash
# same-box comparison of the in-tree library and variant libraries on a short bench:
# LIBS="abvar/lib_a.so abvar/lib_b.so", CFG (default c2), two rounds
set -o pipefail
for r in 1 2; do
  for v in "" $LIBS; do
    IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config ${CFG:-c2} --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('lib=${v:-tree}', d['value'], d['ms_per_step'], d['step_ms'])" || exit 1
  done
done
