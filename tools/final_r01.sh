#!/bin/bash
# Round-end evidence: full GPU suite, the default bench line (C2 f32x6 with
# cpu_baseline and the north-star side run), its rocprofv3 kernel stats, and
# FETCH_SIZE / WRITE_SIZE passes (separate runs) over the fused head kernels
# at C2 shapes for roofline.traffic.  Outputs under gpurun_out/.
set -e
tag=${1:-r01f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_${tag}.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_${tag}_c2.json 2> gpurun_out/bench_${tag}_c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_c2 -o c2 -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/prof_${tag}_c2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_${tag} -o f -- python3 tools/flashx.py --iters 1 --terms 6 > gpurun_out/pmcF_${tag}.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_${tag} -o w -- python3 tools/flashx.py --iters 1 --terms 6 > gpurun_out/pmcW_${tag}.log 2>&1
echo done
