#!/bin/bash
# round 4: last full GPU suite of the final tree
set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n/pytest_gpu.txt 2>&1
rc=$?; tail -2 gpurun_out/r06n/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r06n/pytest_gpu.txt | tail -20; fi
exit $rc
