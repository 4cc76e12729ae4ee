#!/bin/bash
# round 4: stored logits v3 (pass 2 software-pipelined: chunk c+1's dZ VALU woven into chunk c's W-part MFMAs):
# tests, flashx A/B (v1 / v2 libs, recomputing), C2 / C4 same-box A/B --stored-logits auto/off
set -o pipefail
mkdir -p gpurun_out/r05r
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_head.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05r/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05r/pytest.txt | tail -20; tail -40 gpurun_out/r05r/pytest.txt; exit 1; }
tail -1 gpurun_out/r05r/pytest.txt
for cfg in "tree|" "tree|--zs" "abvar/lib_zs2.so|--zs" "tree|--zs" "tree|"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#${cfg} #" | tee -a gpurun_out/r05r/flashx.txt || exit 1
done
for c in c2 c4; do for m in auto off auto off; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-native-side --stored-logits $m > gpurun_out/r05r/b.json 2> gpurun_out/r05r/b.err || { tail -20 gpurun_out/r05r/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05r/b.json'));r=d.get('roofline') or {};print('$c','$m',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'),r.get('stored_logits'))" | tee -a gpurun_out/r05r/ab_bench.txt
done; done
