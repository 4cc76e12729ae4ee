#!/bin/bash
# round 4, first GPU call: full GPU suite, then the r05b experiments (unless the suite crashed / timed out)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05a_pytest.txt 2>&1
rc=$?
tail -15 gpurun_out/r05a_pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/rounds/r05b.sh
rc2=$?
exit $(( rc > rc2 ? rc : rc2 ))
