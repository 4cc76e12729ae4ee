#!/bin/bash
# SQ counters of the sampled-forward microbench (one pass, HF 128)
set -e
tag=${1:-pmc}
shift || true
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/${tag} -o pmc -- python3 tools/sampbench.py --HF 128 --iters 5 "$@" > gpurun_out/${tag}.log 2>&1
