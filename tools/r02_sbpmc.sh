#!/bin/bash
# PMC pass over the fused sampled forward (sampbench, HF 128, f32x6)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out/sbpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/sbpmc/p1 -o p1 --output-format csv -- python tools/sampbench.py --HF 128 --prec f32x6 --iters 10 > gpurun_out/sbpmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA -d gpurun_out/sbpmc/p2 -o p2 --output-format csv -- python tools/sampbench.py --HF 128 --prec f32x6 --iters 10 > gpurun_out/sbpmc/p2.log 2>&1
find gpurun_out/sbpmc -name "*counter_collection*"
