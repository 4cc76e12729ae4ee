#!/bin/bash
# PMC passes over the fused head's pass 1 / pass 2 at C2 shapes (TERMS, default 6;
# ZS=1: the stored-logit head)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out/flpmc
Z=${ZS:+--zs}
timeout -k 10 120 python tools/flashx.py --terms ${TERMS:-6} --iters 3 $Z > gpurun_out/flpmc/time.log 2>&1
P="python tools/flashx.py --terms ${TERMS:-6} --iters 1 $Z"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES -d gpurun_out/flpmc/p1 -o p1 --output-format csv -- $P > gpurun_out/flpmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA -d gpurun_out/flpmc/p2 -o p2 --output-format csv -- $P > gpurun_out/flpmc/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM -d gpurun_out/flpmc/p3 -o p3 --output-format csv -- $P > gpurun_out/flpmc/p3.log 2>&1 || echo "p3 failed"
cat gpurun_out/flpmc/time.log
python tools/pmc_summary.py gpurun_out/flpmc k_flash
