#!/bin/bash
# round 4: stored-logit trainer equivalence tests
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_head.py -k "trainer" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06d/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r06d/pytest.txt | tail -20; tail -40 gpurun_out/r06d/pytest.txt; exit 1; }
tail -1 gpurun_out/r06d/pytest.txt
