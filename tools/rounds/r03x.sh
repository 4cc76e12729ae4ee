#!/bin/bash
# round-3 re-entry: gather microbench, long-horizon parity test, then the full snapshot (minus that test)
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 120 python tools/gatherbench.py > $O/gather.txt 2>&1; cat $O/gather.txt | tail -2
timeout -k 10 120 python tools/gatherbench.py --sweep > $O/gather_sweep.txt 2>&1; tail -1 $O/gather_sweep.txt
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread -m gpu tests/test_gpu_long_horizon.py > $O/long.txt 2>&1; grep -E "steps|f32|passed|failed|Error" $O/long.txt | tail -20
bash tools/gpu_snapshot.sh
