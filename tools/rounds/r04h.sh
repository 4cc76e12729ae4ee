#!/bin/bash
# round-3 final snapshot: GPU suite, C2/C3/C4 lines, rocprof C2/C3/C4, long-horizon test, C5 line
set -o pipefail
bash tools/gpu_snapshot.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread -m gpu tests/test_gpu_long_horizon.py > gpurun_out/snap/long.txt 2>&1; tail -1 gpurun_out/snap/long.txt
timeout -k 10 700 python bench.py --config c5 --steps 4 --warmup 2 > gpurun_out/snap/bench_c5.json 2> gpurun_out/snap/bench_c5.err || { tail -20 gpurun_out/snap/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/snap/bench_c5.json'));print('c5', d['value'], d['ms_per_step'])"
