#!/bin/bash
# round 4: GPU suite; sampled-logits bias-late + early A/B with more repetitions; 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i/pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r05i/pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
IKEA_REC_HIP_LIB=abvar/lib_sfblearly.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sampled.py tests/test_gpu_bpr.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05i/pytest_sampled_blearly.txt 2>&1
tail -2 gpurun_out/r05i/pytest_sampled_blearly.txt
for r in 1 2 3 4; do for v in "" abvar/lib_sfblearly.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 240 python tools/nstime.py --reps 3 2>/dev/null | tee -a gpurun_out/r05i/nstime.txt || exit 1
done; done
bash tools/bench_ranks.sh > gpurun_out/r05i/ranks.txt 2>&1 || { grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/r05i/ranks.txt | tail -30; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r05i/ranks.txt"):
    if l.startswith("{"):
        d = json.loads(l)
        ns = d.get("north_star_target") or {}
        print(d["config"]["workload"][:70], "| n_gpus", d["n_gpus"], "| global_batch", d["config"]["global_batch"], "|", d["value"], d["scaling"],
              {k: ns.get(k) for k in ("frac", "gather_ms", "neg_exchange_ms", "sampled_fwd_ms", "ranks")})
PY
exit $rc
