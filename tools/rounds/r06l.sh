#!/bin/bash
# round 4: Adam alignment guard: kernel + trainer tests, smoke
set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_supervised.py tests/test_gpu_qlearning.py tests/test_gpu_sampled.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06l/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r06l/pytest.txt | tail -20; tail -30 gpurun_out/r06l/pytest.txt; exit 1; }
tail -1 gpurun_out/r06l/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
