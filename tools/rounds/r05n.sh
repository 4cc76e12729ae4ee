#!/bin/bash
# round 4: stored-logit head (pass 1 stores z, pass 2 reads it): kernel tests + flashx A/B + C2 bench;
# atomic-free Q-head gradient tests; HF-256 sampled logits on 256-row workgroups: tests + C3 A/B
set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_head.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05n/pytest_flash.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05n/pytest_flash.txt | tail -20; tail -40 gpurun_out/r05n/pytest_flash.txt; exit 1; }
tail -1 gpurun_out/r05n/pytest_flash.txt
for z in "" --zs; do timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | sed "s/^/zs=${z:-no} /" | tee -a gpurun_out/r05n/flashx.txt || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05n/bench_c2.json 2> gpurun_out/r05n/bench_c2.err || { tail -20 gpurun_out/r05n/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05n/bench_c2.json'));print('c2',d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_qlearning.py tests/test_gpu_dist_q.py tests/test_gpu_ckpt_eval.py tests/test_gpu_sampled.py tests/test_gpu_bpr.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05n/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05n/pytest.txt | tail -20; tail -30 gpurun_out/r05n/pytest.txt; exit 1; }
tail -1 gpurun_out/r05n/pytest.txt
for v in "" abvar/lib_sfr128.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r05n/c3.json 2> gpurun_out/r05n/c3.err || { tail -20 gpurun_out/r05n/c3.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05n/c3.json'));t=d['north_star_target'];print('lib=${v:-tree}',d['value'],d['ms_per_step'],t['frac'],t['sampled_fwd_ms'],t['gather_ms'])" | tee -a gpurun_out/r05n/ab_c3.txt
done
