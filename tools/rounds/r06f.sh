#!/bin/bash
# round 4 closing check after the v4 stored-logit layout: whole GPU suite, smoke, default bench line, 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r06f/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r06f/pytest_gpu.txt | tail -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06f/smoke.txt 2>&1 || { tail -20 gpurun_out/r06f/smoke.txt; exit 1; }
tail -1 gpurun_out/r06f/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r06f/bench_c2.json 2> gpurun_out/r06f/bench_c2.err || { tail -20 gpurun_out/r06f/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06f/bench_c2.json'));r=d.get('roofline') or {};t=d.get('north_star_target') or {};print('c2',d['value'],d['ms_per_step'],r.get('kernel'),r.get('bound'),r.get('frac'),t.get('frac'))"
timeout -k 10 400 python bench.py --config c4 --steps 30 --warmup 5 > gpurun_out/r06f/bench_c4.json 2> gpurun_out/r06f/bench_c4.err || { tail -20 gpurun_out/r06f/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06f/bench_c4.json'));r=d.get('roofline') or {};print('c4',d['value'],d['ms_per_step'],r.get('kernel'),r.get('bound'),r.get('frac'))"
bash tools/bench_ranks.sh > gpurun_out/r06f/ranks.txt 2>&1 || { grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/r06f/ranks.txt | tail -30; exit 1; }
grep -c '^{' gpurun_out/r06f/ranks.txt
