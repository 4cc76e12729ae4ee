#!/bin/bash
# HBM traffic of the fused head's two passes at C2 shapes (tools/flashx.py, precision code
# TERMS, default 636 = f32x6d3): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes,
# summarised per kernel as 2·FETCH_SIZE + WRITE_SIZE (KB -> bytes; MI355X_MICROARCH.md HBM section)
set -e
T=${TERMS:-636}
Z=${ZS:+--zs}   # ZS=1: the stored-logit head (pass 1 stores z, pass 2 reads it)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hpmc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/hpmc/F -o f -- python3 tools/flashx.py --terms $T --iters 1 $Z > gpurun_out/hpmc/F.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/hpmc/W -o w -- python3 tools/flashx.py --terms $T --iters 1 $Z > gpurun_out/hpmc/W.log 2>&1
python3 - <<'PY'
import csv, glob, collections
def load(pat, ctr):
    acc = collections.defaultdict(list)
    for f in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == ctr:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc
F = load("gpurun_out/hpmc/F/**/*counter_collection.csv", "FETCH_SIZE")
W = load("gpurun_out/hpmc/W/**/*counter_collection.csv", "WRITE_SIZE")
for k in sorted(F):
    if "k_flash_fwd" in k or "k_flash_dw" in k or "k_planes" in k:
        f = sum(F[k]) / len(F[k]); w = sum(W.get(k, [0])) / max(1, len(W.get(k, [0])))
        print(f"{k[:60]:60s} fetch {f*1024/1e9:7.3f} GB write {w*1024/1e9:7.3f} GB traffic(2F+W) {(2*f+w)*1024:.0f} B")
PY
