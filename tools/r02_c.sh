#!/bin/bash
# full GPU suite, then the C2 bench (headline, with the north-star side run) and C3
cd $GRAFT_REPO_ROOT
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac']);print(d['north_star_target'])"
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo "bench c3 failed"; tail -20 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
