set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sampled.log 2>&1; rc=$?; tail -5 gpurun_out/t_sampled.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/sampbench.py --HF 128 256 --prec f32x6 f32x9
