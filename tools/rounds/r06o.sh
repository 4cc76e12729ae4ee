#!/bin/bash
# round 4: same-box A/B of the AMDGPU machine-scheduler strategy for head_flash.hip
# (max-ilp, max-memory-clause) on the fused-head microbench (stored logits) and a short C2 bench
set -o pipefail
mkdir -p gpurun_out/r06o
for v in "" abvar/lib_ilp.so abvar/lib_mc.so "" abvar/lib_ilp.so abvar/lib_mc.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 --zs 2>&1 | grep pass | sed "s|^|lib=${v:-tree} |" || exit 1
done
for v in "" abvar/lib_ilp.so abvar/lib_mc.so "" abvar/lib_ilp.so abvar/lib_mc.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('lib=${v:-tree}', d['value'], d['ms_per_step'])" || exit 1
done
