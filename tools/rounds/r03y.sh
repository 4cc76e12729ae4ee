#!/bin/bash
# gather variants: standalone gatherbench and the north-star side run, same box, two rounds
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
for r in 1 2; do
  for v in "" variants/lib_f128.so variants/lib_pipe64.so variants/lib_pipe128.so variants/lib_r2f128.so; do
    IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/gatherbench.py --sweep 2>&1 | tail -1 | sed "s|^|lib=${v:-tree} |" || exit 1
  done
done
for v in "" variants/lib_f128.so variants/lib_pipe128.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval > $O/b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/b.json'));t=d['north_star_target'];print('lib=${v:-tree}', d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
done
