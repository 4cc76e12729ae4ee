#!/bin/bash
# north-star side run with 30 timed steps: stability over three default bench runs
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
for r in 1 2 3; do
timeout -k 10 400 python bench.py --no-cpu-baseline --no-native-side > $O/b$r.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b$r.json'));t=d['north_star_target'];print('run$r', d['value'], d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
done
