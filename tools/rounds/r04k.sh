#!/bin/bash
# after the early loss readout: full snapshot (suite, C2/C3/C4 lines, rocprof), sharded 1-rank RCCL, 2-rank gloo rehearsal
set -o pipefail
bash tools/gpu_snapshot.sh || exit 1
bash tools/bench_rccl1.sh || exit 1
bash tools/bench_ranks.sh > gpurun_out/ranks.txt 2>&1 || { tail -20 gpurun_out/ranks.txt; exit 1; }
python -c "
import json
for c in ('c2','c4'):
    d=json.loads(open(f'gpurun_out/ranks/{c}.json').read().strip().splitlines()[-1]); print('2rank-gloo', c, d['n_gpus'], d['value'], d['ms_per_step'])"
