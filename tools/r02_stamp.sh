#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 --parts --iters 100
IKEA_REC_HIP_LIB=$PWD/variants/lib_STAMP.so timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 --parts --stamps
