#!/bin/bash
# rocprofv3 kernel-trace summaries of the bench workloads (C2 headline incl. the
# north-star side run, and C3), plus the plain bench lines.  Outputs under
# gpurun_out/prof_<tag>/ ; copy the *_kernel_stats.csv into profiles/.
set -e
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/bench_${tag}_c2.json 2> gpurun_out/bench_${tag}_c2.err
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_${tag}_c3.json 2> gpurun_out/bench_${tag}_c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_c2 -o c2 -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_${tag}_c2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_c3 -o c3 -- python3 bench.py --config c3 --no-cpu-baseline > gpurun_out/prof_${tag}_c3.log 2>&1
