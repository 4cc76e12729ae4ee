#!/bin/bash
# fused argmax: kernel parity, Q-learning trainers, sharded Q test, then the C4 bench
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_qlearning.py tests/test_gpu_dist_q.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_amax.log 2>&1; rc=$?; tail -3 gpurun_out/t_amax.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_amax.log | head; exit $rc; }
timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || { tail gpurun_out/b_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_c4.json'));print(d['value'],d['ms_per_step'],d['kernel_ms'])"
