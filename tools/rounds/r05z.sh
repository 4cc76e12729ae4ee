#!/bin/bash
# round 4: stored-logit pass 2 with the one-hot term by the sorted scatter: tests (flash head, Q, sharded,
# checkpoint), flashx, C2 / C4 lines (stored logits on / off)
set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 700 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_qlearning.py tests/test_gpu_dist.py tests/test_gpu_dist_q.py tests/test_gpu_ckpt_eval.py tests/test_gpu_supervised.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05z/pytest.txt | tail -20; tail -40 gpurun_out/r05z/pytest.txt; exit 1; }
tail -1 gpurun_out/r05z/pytest.txt
for z in "" --zs; do timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#zs=${z:-no} #" | tee -a gpurun_out/r05z/flashx.txt || exit 1; done
for c in c2 c4; do for m in auto off; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-native-side --stored-logits $m > gpurun_out/r05z/b.json 2> gpurun_out/r05z/b.err || { tail -20 gpurun_out/r05z/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05z/b.json'));r=d.get('roofline') or {};print('$c','$m',d['value'],d['ms_per_step'],r.get('kernel'),r.get('bound'),r.get('frac'),d['kernel_ms'].get('head_fwd'),d['kernel_ms'].get('head_dw_adam'))" | tee -a gpurun_out/r05z/ab_bench.txt
done; done
