#!/bin/bash
# s_setprio 1 for the second-dispatched half of the fused head's waves: barrier share, flashx, C2 step
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
for v in flstamp flprio; do IKEA_REC_HIP_LIB=variants/lib_$v.so timeout -k 10 120 python tools/flstamp.py 2>&1 | grep -E "pass1|pass2|barrier" | sed "s|^|$v |" || exit 1; done
for v in "" variants/lib_prio.so "" variants/lib_prio.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/flashx.py --terms 636 --iters 4 2>&1 | grep -E "pass1|pass2" | sed "s|^|lib=${v:-tree} |" || exit 1
done
for v in "" variants/lib_prio.so "" variants/lib_prio.so; do
IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval --no-target > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('lib=${v:-tree}', d['value'], d['ms_per_step'], d['step_ms']['median'], d['kernel_ms']['head_fwd'], d['kernel_ms']['head_dw_adam'])"
done
