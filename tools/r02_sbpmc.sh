#!/bin/bash
# PMC pass over the fused sampled forward (sampbench --fused, HF 128, f32x6)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out/sbpmc2
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES -d gpurun_out/sbpmc2/p1 -o p1 --output-format csv -- python tools/sampbench.py --HF 128 --prec f32x6 --fused --iters 10 > gpurun_out/sbpmc2/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d gpurun_out/sbpmc2/p2 -o p2 --output-format csv -- python tools/sampbench.py --HF 128 --prec f32x6 --fused --iters 10 > gpurun_out/sbpmc2/p2.log 2>&1
echo done
