#!/bin/bash
# kernel trace of the item-sharded C2 step over RCCL with one rank (--force-shard) vs the plain step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04i
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i/shard -o s -- python bench.py --force-shard --steps 8 --warmup 3 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > gpurun_out/r04i/shard.log 2>&1 || { tail gpurun_out/r04i/shard.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i/plain -o p -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-native-side --no-eval --no-target --no-kernel-timing > gpurun_out/r04i/plain.log 2>&1 || { tail gpurun_out/r04i/plain.log; exit 1; }
grep -h '"metric"' gpurun_out/r04i/*.log | python -c "import sys,json;[print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
