#!/bin/bash
# C5 line with the round-3 step (one GPU: 5M items, d256, L<=100, B 8192, fp16 table, SMORL)
set -o pipefail
mkdir -p gpurun_out/r04s
timeout -k 10 900 python bench.py --config c5 --steps 4 --warmup 2 > gpurun_out/r04s/bench_c5.json 2> gpurun_out/r04s/bench_c5.err || { tail -20 gpurun_out/r04s/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04s/bench_c5.json'));print('c5', d['value'], d['ms_per_step'], (d.get('eval_heldout') or {}).get('ms'))"
