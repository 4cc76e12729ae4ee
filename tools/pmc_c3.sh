#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the C3 step's
# north-star kernels (gather + sampled forward) for roofline.traffic.
set -e
tag=${1:-pmc_c3}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}F -o f -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}F.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}W -o w -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}W.log 2>&1
echo done
