#!/bin/bash
# round 4: stored logits v2 + HF-256 sampled logits from h's planes (DMA ring): tests, flashx A/B (v1 lib,
# recomputing pass 2), C3 A/B (lib without the HF-256 planes path), C2 / C4 bench lines
set -o pipefail
mkdir -p gpurun_out/r05p
timeout -k 10 500 python -u -m pytest tests/test_gpu_flash_head.py tests/test_gpu_sampled.py tests/test_gpu_bpr.py "tests/test_gpu_kernels.py::test_gru_forward_emits_h_planes" -x -q --timeout 200 --timeout-method thread > gpurun_out/r05p/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05p/pytest.txt | tail -20; tail -40 gpurun_out/r05p/pytest.txt; exit 1; }
tail -1 gpurun_out/r05p/pytest.txt
for cfg in "tree|" "tree|--zs" "abvar/lib_zs1.so|--zs" "tree|--zs"; do
  lib=${cfg%%|*}; z=${cfg##*|}; [ "$lib" = tree ] && lib=""
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 python tools/flashx.py --terms 636 --iters 3 $z 2>/dev/null | grep pass | sed "s#^#${cfg} #" | tee -a gpurun_out/r05p/flashx.txt || exit 1
done
for v in "" abvar/lib_nohkp256.so "" abvar/lib_nohkp256.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r05p/c3.json 2> gpurun_out/r05p/c3.err || { tail -20 gpurun_out/r05p/c3.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05p/c3.json'));t=d['north_star_target'];print('lib=${v:-tree}',d['value'],d['ms_per_step'],t['frac'],t['sampled_fwd_ms'],t['gather_ms'])" | tee -a gpurun_out/r05p/ab_c3.txt
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05p/bench_c2.json 2> gpurun_out/r05p/bench_c2.err || { tail -20 gpurun_out/r05p/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05p/bench_c2.json'));r=d.get('roofline') or {};print('c2',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05p/bench_c4.json 2> gpurun_out/r05p/bench_c4.err || { tail -20 gpurun_out/r05p/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05p/bench_c4.json'));r=d.get('roofline') or {};print('c4',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
