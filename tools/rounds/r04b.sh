#!/bin/bash
# XCD mapping of the sampled logits: 4 row tiles x 8 negative tiles (tree) vs 8 x 4 per XCD
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
for v in sfstamp sfxcd42; do echo "== $v"; IKEA_REC_HIP_LIB=variants/lib_$v.so timeout -k 10 120 python tools/sfstamp.py --wp cold 2>&1 | grep -E "ingest|chunk 0|total"; done
for v in "" variants/lib_xcd42.so "" variants/lib_xcd42.so; do
IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));t=d['north_star_target'];print('lib=${v:-tree}', d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
done
