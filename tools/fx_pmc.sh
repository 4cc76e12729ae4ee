#!/bin/bash
# PMC stall breakdown of the fused-head kernels (microbench, f32x6, 1 iteration)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_fx1 -o a \
  -- python3 tools/flashx.py --terms 6 --iters 1 > gpurun_out/pmc_fx1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_fx2 -o b \
  -- python3 tools/flashx.py --terms 6 --iters 1 > gpurun_out/pmc_fx2.log 2>&1
