#!/bin/bash
# short C2 and C3 benches (kernel_ms breakdowns)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/b_c2s.json 2> gpurun_out/b_c2s.err || { tail gpurun_out/b_c2s.err; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b_c3s.json 2> gpurun_out/b_c3s.err || { tail gpurun_out/b_c3s.err; exit 1; }
for f in b_c2s b_c3s; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'],d['kernel_ms']);print(d['north_star_target'])"; done
