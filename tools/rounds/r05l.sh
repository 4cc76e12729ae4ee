#!/bin/bash
# round 4: HF-256 sampled logits over 256-row workgroups (one round on 256 CUs): tests, C3 A/B against the
# 128-row build, C3 PMC traffic
set -o pipefail
mkdir -p gpurun_out/r05l
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampled.py tests/test_gpu_bpr.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05l/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05l/pytest.txt | tail -20; tail -30 gpurun_out/r05l/pytest.txt; exit 1; }
tail -2 gpurun_out/r05l/pytest.txt
for r in 1 2; do for v in "" abvar/lib_sfr128.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r05l/c3.json 2> gpurun_out/r05l/c3.err || { tail -20 gpurun_out/r05l/c3.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05l/c3.json'));t=d['north_star_target'];print('lib=${v:-tree}',d['value'],d['ms_per_step'],t['frac'],t['sampled_fwd_ms'],t['gather_ms'])" | tee -a gpurun_out/r05l/ab.txt
done; done
PMC_CONFIGS=c3 bash tools/pmc_ns.sh > gpurun_out/r05l/pmc_c3.txt 2>&1 || { tail gpurun_out/r05l/pmc_c3.txt; exit 1; }
cat gpurun_out/r05l/pmc_c3.txt
rm -rf gpurun_out/pmcns
