#!/bin/bash
# round 4: PMC traffic of the v4 stored-logit head (C2 shapes)
set -o pipefail
mkdir -p gpurun_out/r06i
ZS=1 bash tools/pmc_head.sh > gpurun_out/r06i/pmc_head_zs.txt 2>&1 || { tail gpurun_out/r06i/pmc_head_zs.txt; exit 1; }
cat gpurun_out/r06i/pmc_head_zs.txt
rm -rf gpurun_out/hpmc
