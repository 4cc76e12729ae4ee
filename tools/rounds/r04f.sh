#!/bin/bash
# multi-rank rehearsal after the round-3 changes: 2-rank GPU tests + bench.py's N=2 path over gloo on one GPU
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_dist_q.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/bench_ranks.sh || exit 1
