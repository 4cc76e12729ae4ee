#!/bin/bash
# same-box A/B of a variant library (tools/build_variant.sh) against the in-tree one on a short
# bench and the fused-head microbench: VARIANT=abvar/lib_X.so, CFG (default c2)
set -o pipefail
for v in "" $VARIANT "" $VARIANT; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config ${CFG:-c2} --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('lib=${v:-tree}', d['value'], d['ms_per_step'], d['step_ms'])" || exit 1
done
for v in "" $VARIANT; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 2>&1 | grep pass | sed "s|^|lib=${v:-tree} |" || exit 1
done
