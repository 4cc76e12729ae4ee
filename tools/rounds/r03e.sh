# C4: unsharded vs 1-rank RCCL sharded, with / without host routes and exact top-1
set -o pipefail
mkdir -p gpurun_out/r03e
run() {  # name, patches, extra
  timeout -k 10 300 python tools/bench_patched.py "$2" -- --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-target $3 > gpurun_out/r03e/$1.json 2> gpurun_out/r03e/$1.err || { tail -20 gpurun_out/r03e/$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03e/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['step_ms'])"
}
runs() {
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 tools/bench_patched.py "$2" -- --config c4 --force-shard --steps 20 --warmup 5 --no-cpu-baseline --no-target > gpurun_out/r03e/$1.json 2> gpurun_out/r03e/$1.err || { tail -20 gpurun_out/r03e/$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03e/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['step_ms'])"
}
run c4 none
run c4_merge1 merge1
runs s4 none
runs s4_noroute noroute
runs s4_merge1 merge1
run c4b none
