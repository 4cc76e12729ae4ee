#!/bin/bash
# Default bench lines (C2 with the north-star side run, C3) and rocprofv3
# kernel-stats of both; outputs under gpurun_out/.
set -e
tag=${1:-r01e}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_${tag}_c3.json 2> gpurun_out/bench_${tag}_c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_c3 -o c3 -- python3 bench.py --config c3 --no-cpu-baseline --steps 5 > gpurun_out/prof_${tag}_c3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_c2 -o c2 -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/prof_${tag}_c2.log 2>&1
