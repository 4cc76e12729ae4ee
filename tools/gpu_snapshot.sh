#!/bin/bash
# round-2 snapshot: full GPU suite, C2 / C3 / C4 bench lines, rocprofv3 kernel stats of a short C2 run
set -o pipefail
mkdir -p gpurun_out/snap
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --ignore=tests/test_gpu_long_horizon.py --timeout 300 --timeout-method thread > gpurun_out/snap/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" gpurun_out/snap/pytest_gpu.log | tail -20; tail -30 gpurun_out/snap/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/snap/pytest_gpu.log
timeout -k 10 500 python bench.py > gpurun_out/snap/bench_c2.json 2> gpurun_out/snap/bench_c2.err || { tail -20 gpurun_out/snap/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 > gpurun_out/snap/bench_c3.json 2> gpurun_out/snap/bench_c3.err || { tail -20 gpurun_out/snap/bench_c3.err; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 > gpurun_out/snap/bench_c4.json 2> gpurun_out/snap/bench_c4.err || { tail -20 gpurun_out/snap/bench_c4.err; exit 1; }
for f in c2 c3 c4; do python -c "import json;d=json.load(open('gpurun_out/snap/bench_$f.json'));print('$f',d['value'],d['ms_per_step'],d['step_ms'],(d.get('roofline') or {}).get('frac'))"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/snap/prof_c2 -o c2 -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/snap/prof_c2.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/snap/prof_c2.log; exit 1; }
echo done
# C3 / C4 kernel stats (round 3)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/snap/prof_c3 -o c3 -- python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/snap/prof_c3.log 2>&1 || { echo "rocprof c3 failed"; tail gpurun_out/snap/prof_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/snap/prof_c4 -o c4 -- python bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/snap/prof_c4.log 2>&1 || { echo "rocprof c4 failed"; tail gpurun_out/snap/prof_c4.log; exit 1; }
echo done2
