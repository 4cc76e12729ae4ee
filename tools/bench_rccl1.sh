#!/bin/bash
# The item-sharded (multi-GPU) step over RCCL with ONE rank (--force-shard): every
# collective of the N-rank path (all-to-all of ids / rows / row-gradients, all-gather
# of h, reduce-scatter of dH, all-reduces) runs through the nccl backend, C2 and C4.
set -o pipefail
mkdir -p gpurun_out/rccl1
for cfg in c2 c4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --config $cfg --force-shard --steps 10 --warmup 3 \
    --no-cpu-baseline > gpurun_out/rccl1/$cfg.json 2> gpurun_out/rccl1/$cfg.err || { tail -30 gpurun_out/rccl1/$cfg.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/rccl1/$cfg.json').read().strip().splitlines()[-1]);print('$cfg', d['value'], d['ms_per_step'], d['config']['parallelism'], d['loss_first_last'])"
done
