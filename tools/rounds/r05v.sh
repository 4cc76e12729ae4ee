#!/bin/bash
# round 4 snapshot, part 2: default bench line (C2 with cpu_baseline / harness / native side run), C3, C4 lines
# (with their CPU baselines), rocprofv3 kernel stats of C2, C3, C4
set -o pipefail
mkdir -p gpurun_out/r05v
timeout -k 10 600 python bench.py > gpurun_out/r05v/bench_c2.json 2> gpurun_out/r05v/bench_c2.err || { tail -20 gpurun_out/r05v/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 > gpurun_out/r05v/bench_c3.json 2> gpurun_out/r05v/bench_c3.err || { tail -20 gpurun_out/r05v/bench_c3.err; exit 1; }
timeout -k 10 400 python bench.py --config c4 --steps 30 --warmup 5 > gpurun_out/r05v/bench_c4.json 2> gpurun_out/r05v/bench_c4.err || { tail -20 gpurun_out/r05v/bench_c4.err; exit 1; }
for f in c2 c3 c4; do python -c "import json;d=json.load(open('gpurun_out/r05v/bench_$f.json'));r=d.get('roofline') or {};t=d.get('north_star_target') or {};c=d.get('cpu_baseline') or {};print('$f',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'),t.get('frac'),c.get('value'),c.get('cores'))"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05v/prof_$c -o $c -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/r05v/prof_$c.log 2>&1 || { echo "rocprof $c failed"; tail gpurun_out/r05v/prof_$c.log; exit 1; }
  find gpurun_out/r05v/prof_$c -name "*kernel_trace.csv" -delete
done
echo done
