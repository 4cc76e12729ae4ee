#!/bin/bash
# Time each variants/lib_*.so with tools/headbench.py, two interleaved rounds.
cd $GRAFT_REPO_ROOT
for round in 1 2; do
  for v in "$@"; do
    echo "== $v round $round"
    IKEA_REC_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 120 python tools/headbench.py --iters 5 2>/dev/null || exit 1
  done
done
