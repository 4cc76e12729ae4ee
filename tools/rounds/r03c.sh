set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_dist_q.py > gpurun_out/r03c/pt.log 2>&1 || { tail -30 gpurun_out/r03c/pt.log; exit 1; }
tail -1 gpurun_out/r03c/pt.log
for cfg in c2 c4; do
  RG_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --config $cfg --steps 4 --warmup 2 --no-eval \
    > gpurun_out/r03c/ranks_$cfg.json 2> gpurun_out/r03c/ranks_$cfg.err || { tail -30 gpurun_out/r03c/ranks_$cfg.err; exit 1; }
  cut -c1-400 gpurun_out/r03c/ranks_$cfg.json
done
for cfg in c2 c4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --config $cfg --force-shard --steps 20 --warmup 5 \
    --no-cpu-baseline --no-target > gpurun_out/r03c/rccl1_$cfg.json 2> gpurun_out/r03c/rccl1_$cfg.err || { tail -30 gpurun_out/r03c/rccl1_$cfg.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03c/rccl1_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', d['value'], d['ms_per_step'], d['step_ms'], d['config']['parallelism'])"
done
