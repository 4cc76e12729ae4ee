#!/bin/bash
# round 4 closing check of the committed tree: whole GPU suite, smoke, default bench line, 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r06c/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r06c/pytest_gpu.txt | tail -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c/smoke.txt 2>&1 || { tail -20 gpurun_out/r06c/smoke.txt; exit 1; }
tail -1 gpurun_out/r06c/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r06c/bench_c2.json 2> gpurun_out/r06c/bench_c2.err || { tail -20 gpurun_out/r06c/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c/bench_c2.json'));r=d.get('roofline') or {};t=d.get('north_star_target') or {};print('c2',d['value'],d['ms_per_step'],r.get('kernel'),r.get('bound'),r.get('frac'),t.get('frac'))"
bash tools/bench_ranks.sh > gpurun_out/r06c/ranks.txt 2>&1 || { grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/r06c/ranks.txt | tail -30; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r06c/ranks.txt"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["workload"][:60], "| n_gpus", d["n_gpus"], "| global_batch", d["config"]["global_batch"], "|", d["value"], d["scaling"])
PY
