#!/bin/bash
# round 4 snapshot, part 1: the whole GPU suite, smoke, PMC traffic of the stored-logit head (C2 shapes) and
# of the C3 north-star kernels
set -o pipefail
mkdir -p gpurun_out/r05u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05u/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r05u/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r05u/pytest_gpu.txt | tail -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05u/smoke.txt 2>&1 || { tail -20 gpurun_out/r05u/smoke.txt; exit 1; }
tail -2 gpurun_out/r05u/smoke.txt
ZS=1 bash tools/pmc_head.sh > gpurun_out/r05u/pmc_head_zs.txt 2>&1 || { tail gpurun_out/r05u/pmc_head_zs.txt; exit 1; }
cat gpurun_out/r05u/pmc_head_zs.txt
PMC_CONFIGS=c3 bash tools/pmc_ns.sh > gpurun_out/r05u/pmc_c3.txt 2>&1 || { tail gpurun_out/r05u/pmc_c3.txt; exit 1; }
cat gpurun_out/r05u/pmc_c3.txt
rm -rf gpurun_out/hpmc gpurun_out/pmcns
