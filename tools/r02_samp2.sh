#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 60 python tools/sampbench.py --HF 128 --prec f32x6 f32x9 --parts --iters 100
