#!/bin/bash
# round 4: default bench line of the final tree (roofline with both head passes)
set -o pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 600 python bench.py > gpurun_out/r06k/bench_c2.json 2> gpurun_out/r06k/bench_c2.err || { tail -20 gpurun_out/r06k/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06k/bench_c2.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r['kernel'],r['bound'],r['frac'],r.get('both_passes'),d['north_star_target']['frac'])"
