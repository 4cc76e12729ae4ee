#!/bin/bash
# round 4: north-star A/B (SF_EARLY), pass-2 phase stamps, 2-rank gloo rehearsal (c2 sharded target, c4 global batch)
set -o pipefail
mkdir -p gpurun_out/r05b
for v in "" abvar/lib_sfearly.so "" abvar/lib_sfearly.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 240 python tools/nstime.py --reps 2 >> gpurun_out/r05b/nstime.txt 2>gpurun_out/r05b/nstime.err || { tail -20 gpurun_out/r05b/nstime.err; exit 1; }
done
cat gpurun_out/r05b/nstime.txt
IKEA_REC_HIP_LIB=abvar/lib_fl2stamp.so timeout -k 10 240 python tools/fl2stamp.py > gpurun_out/r05b/fl2stamp.txt 2>&1 || { tail -20 gpurun_out/r05b/fl2stamp.txt; exit 1; }
cat gpurun_out/r05b/fl2stamp.txt
bash tools/bench_ranks.sh > gpurun_out/r05b/ranks.txt 2>&1 || { tail -30 gpurun_out/r05b/ranks.txt; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05b/ranks.txt"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["workload"][:60], d["n_gpus"], d["config"]["global_batch"], d["value"], d["scaling"],
              json.dumps({k: d["north_star_target"].get(k) for k in ("frac", "gather_ms", "neg_exchange_ms", "sampled_fwd_ms", "ranks")} if d.get("north_star_target") else None))
PY
