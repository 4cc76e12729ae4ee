# round-3 snapshot: full GPU suite, C2 / C3 / C4 bench lines, rocprofv3 kernel stats of a short C2 run
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | tail -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
for f in c2 c3 c4; do python -c "import json;d=json.load(open('$O/bench_$f.json'));print('$f',d['value'],d['ms_per_step'],d['step_ms'],(d.get('roofline') or {}).get('frac'),(d.get('north_star_target') or {}).get('frac'))"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > $O/prof_c2.json 2> $O/prof_c2.err || { echo "rocprof failed"; tail $O/prof_c2.err; exit 1; }
echo done
