#!/bin/bash
# round 4: rocprofv3 kernel stats of the final tree, C2 and C4 (10 steps after 2 warm-up)
set -o pipefail
mkdir -p gpurun_out/r06m
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06m/prof_$c -o $c -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/r06m/prof_$c.log 2>&1 || { echo "rocprof $c failed"; tail gpurun_out/r06m/prof_$c.log; exit 1; }
  find gpurun_out/r06m/prof_$c -name "*kernel_trace.csv" -delete
done
echo done
