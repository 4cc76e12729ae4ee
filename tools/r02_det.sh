#!/bin/bash
# deterministic scatter + §8f tests (checkpoint resume, update_train_metrics, tokenizer remap), then trainers
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ckpt_eval.py tests/test_gpu_supervised.py tests/test_gpu_sampled.py tests/test_gpu_eval.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_det.log 2>&1; rc=$?; tail -25 gpurun_out/t_det.log; exit $rc
