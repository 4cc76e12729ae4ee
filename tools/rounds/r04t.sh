#!/bin/bash
# gather workgroup shape: 4 rows / 128 in flight (tree) vs 8 rows, 8 rows / 256 in flight, 4 rows / 64; north-star side run
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
for r in 1 2; do
for v in "" variants/lib_r8.so variants/lib_r8f256.so variants/lib_f64.so; do
IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));t=d['north_star_target'];print('lib=${v:-tree}', d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
done
done
