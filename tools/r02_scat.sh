#!/bin/bash
# sorted-scatter parity + timings, then a rocprofv3 kernel-trace summary of the same run
set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k scatter -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 200 python tools/scatbench.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scprof -o sc -- python tools/scatbench.py > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/scprof -name "*kernel_stats.csv" | head -1); cut -c1-160 "$f" | head -14
