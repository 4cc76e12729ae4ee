#!/bin/bash
# round 4: pass-2 stream priority A/B (0 = default, -1 = high), C2 and C4
set -o pipefail
mkdir -p gpurun_out/r06g
for c in c2 c4; do for p in 0 -1 0 -1; do
  timeout -k 10 300 python tools/prio_ab.py $p --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-native-side > gpurun_out/r06g/b.json 2> gpurun_out/r06g/b.err || { tail -20 gpurun_out/r06g/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06g/b.json'));print('$c','prio $p',d['value'],d['ms_per_step'],d['kernel_ms'].get('head_fwd'),d['kernel_ms'].get('head_dw_adam'))" | tee -a gpurun_out/r06g/ab.txt
done; done
