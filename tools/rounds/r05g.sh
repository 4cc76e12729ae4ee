#!/bin/bash
# round 4: C5 step-only kernel profile (one GPU), then the C2 / C3 / C4 lines with their CPU baselines
set -o pipefail
mkdir -p gpurun_out/r05g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05g/c5prof -o c5 -- python3 tools/stepprof.py --config c5 --steps 3 --warmup 1 > gpurun_out/r05g/c5prof.log 2>&1 || { tail -20 gpurun_out/r05g/c5prof.log; exit 1; }
python3 tools/kwindow.py $(find gpurun_out/r05g/c5prof -name "c5_kernel_trace.csv" | head -1) --steps 3 > gpurun_out/r05g/c5_step_kernel_stats.csv 2> gpurun_out/r05g/c5_window.txt || exit 1
cat gpurun_out/r05g/c5_window.txt; head -12 gpurun_out/r05g/c5_step_kernel_stats.csv | cut -c1-160
rm -rf gpurun_out/r05g/c5prof
