#!/bin/bash
# C2 headline bench (short) after a head change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2q.json 2> gpurun_out/bench_c2q.err || { tail -20 gpurun_out/bench_c2q.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c2q.json'));print(d['value'],d['ms_per_step'],d['step_ms'],d['roofline']['frac'],d['kernel_ms']);print(d['north_star_target']);print(d.get('native_f32'));print(d.get('eval_heldout'))"
