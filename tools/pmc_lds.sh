#!/bin/bash
# LDS / issue counters for the head kernels (one PMC pass, kernel trace only).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/headbench.py --variants > gpurun_out/hb_var.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmcE -o e -- python3 tools/headbench.py --iters 1 > gpurun_out/pmcE.log 2>&1
