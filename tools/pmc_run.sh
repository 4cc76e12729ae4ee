#!/bin/bash
# HBM traffic (rocprofv3 FETCH_SIZE and WRITE_SIZE, one counter per pass) of the kernels the
# bench line prices: the stored-logit head's two passes at C2 shapes (tools/flashx.py --zs) and
# the north-star kernels at C2 / C3 (tools/nsrun.py); tools/pmc_traffic.py turns the CSVs into
# profiles/pmc_traffic.json entries keyed with the hash of the measured sources
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/s6c/pmc
mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/head_$C -o p -- python3 tools/flashx.py --terms 636 --iters 2 --zs > $O/head_$C.log 2>&1
  for c in c2 c3; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/ns_${c}_$C -o p -- python3 tools/nsrun.py --config $c > $O/ns_${c}_$C.log 2>&1
  done
done
python3 tools/pmc_traffic.py $O > $O/summary.txt
cat $O/summary.txt
