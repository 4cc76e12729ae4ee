#!/bin/bash
# Rehearse bench.py's N-rank path on the one-GPU box: 2 ranks on cuda:0 over
# gloo (host-staged collectives), C2 and C4 (item-sharded tables), short runs.
set -o pipefail
mkdir -p gpurun_out/ranks
for cfg in c2 c4; do
  RG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config $cfg --steps 4 --warmup 2 \
    > gpurun_out/ranks/$cfg.json 2> gpurun_out/ranks/$cfg.err || { tail -30 gpurun_out/ranks/$cfg.err; exit 1; }
  cat gpurun_out/ranks/$cfg.json
done
