#!/bin/bash
# round-3 closing snapshot: suite, C2/C3/C4 lines, rocprof C2/C3/C4, long-horizon, sharded RCCL 1-rank, 2-rank gloo, smoke
set -o pipefail
bash tools/gpu_snapshot.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread -m gpu tests/test_gpu_long_horizon.py > gpurun_out/snap/long.txt 2>&1; tail -1 gpurun_out/snap/long.txt
bash tools/bench_rccl1.sh || exit 1
bash tools/bench_ranks.sh > gpurun_out/ranks.txt 2>&1 || { tail -20 gpurun_out/ranks.txt; exit 1; }
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
