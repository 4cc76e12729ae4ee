#!/bin/bash
# round 4: stored logits v2 (lane-linear stores, LDS transpose, two-deep z prefetch): kernel tests, flashx A/B
# against v1 (abvar/lib_zs1.so) and the recomputing pass 2, C2 bench
set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_head.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05o/pytest_flash.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05o/pytest_flash.txt | tail -20; tail -40 gpurun_out/r05o/pytest_flash.txt; exit 1; }
tail -1 gpurun_out/r05o/pytest_flash.txt
for r in 1 2; do
for cfg in "tree|" "tree|--zs" "abvar/lib_zs1.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#${cfg} #" | tee -a gpurun_out/r05o/flashx.txt || exit 1
done; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05o/bench_c2.json 2> gpurun_out/r05o/bench_c2.err || { tail -20 gpurun_out/r05o/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05o/bench_c2.json'));r=d.get('roofline') or {};print('c2',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'),d.get('kernels_ms',''))"
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05o/bench_c4.json 2> gpurun_out/r05o/bench_c4.err || { tail -20 gpurun_out/r05o/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05o/bench_c4.json'));r=d.get('roofline') or {};print('c4',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
