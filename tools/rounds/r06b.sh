#!/bin/bash
# round 4: C5 line on one GPU (committed tree) and a marker-bounded step timeline of 3 C5 steps
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 900 python bench.py --config c5 --steps 4 --warmup 2 > gpurun_out/r06b/bench_c5.json 2> gpurun_out/r06b/bench_c5.err || { tail -20 gpurun_out/r06b/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06b/bench_c5.json'));r=d.get('roofline') or {};print('c5',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06b/c5prof -o c5 -- python3 tools/stepprof.py --config c5 --steps 3 --warmup 1 > gpurun_out/r06b/c5prof.log 2>&1 || { tail -20 gpurun_out/r06b/c5prof.log; exit 1; }
python3 tools/kwindow.py $(find gpurun_out/r06b/c5prof -name "c5_kernel_trace.csv" | head -1) --steps 3 --timeline gpurun_out/r06b/c5_timeline.txt > gpurun_out/r06b/c5_step_kernel_stats.csv 2> gpurun_out/r06b/c5_window.txt || exit 1
cat gpurun_out/r06b/c5_window.txt
rm -rf gpurun_out/r06b/c5prof
