#!/bin/bash
# round-2 GPU check: full GPU suite, then the C2 and C4 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
