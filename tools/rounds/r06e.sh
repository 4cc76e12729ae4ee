#!/bin/bash
# round 4: stored logits v4 (pass 2 DMAs the z tiles into an LDS ring, conflict-free transposed reads): flash-head
# tests, flashx A/B against v3 (registers + LDS transposes), C2 / C4 lines
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_head.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06e/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r06e/pytest.txt | tail -20; tail -40 gpurun_out/r06e/pytest.txt; exit 1; }
tail -1 gpurun_out/r06e/pytest.txt
for cfg in "tree|--zs" "abvar/lib_zs3.so|--zs" "tree|--zs" "abvar/lib_zs3.so|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#${cfg} #" | tee -a gpurun_out/r06e/flashx.txt || exit 1
done
for c in c2 c4; do for v in "" abvar/lib_zs3.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-native-side > gpurun_out/r06e/b.json 2> gpurun_out/r06e/b.err || { tail -20 gpurun_out/r06e/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06e/b.json'));r=d.get('roofline') or {};print('$c','${v:-tree}',d['value'],d['ms_per_step'],r.get('kernel'),r.get('bound'),r.get('frac'),d['kernel_ms'].get('head_fwd'),d['kernel_ms'].get('head_dw_adam'))" | tee -a gpurun_out/r06e/ab_bench.txt
done; done
