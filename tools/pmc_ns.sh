#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the north-star kernels
# (k_gather_e with the negatives + k_sampled_logits) at C2 and C3, tools/nsrun.py
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcns
for c in ${PMC_CONFIGS:-c2 c3}; do
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcns/${c}F -o f -- python3 tools/nsrun.py --config $c > gpurun_out/pmcns/${c}F.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcns/${c}W -o w -- python3 tools/nsrun.py --config $c > gpurun_out/pmcns/${c}W.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections, os
def load(pat, ctr):
    acc = collections.defaultdict(list)
    for f in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == ctr:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc
for c in os.environ.get("PMC_CONFIGS", "c2 c3").split():
    F = load(f"gpurun_out/pmcns/{c}F/**/*counter_collection.csv", "FETCH_SIZE")
    W = load(f"gpurun_out/pmcns/{c}W/**/*counter_collection.csv", "WRITE_SIZE")
    for k in sorted(F):
        if "k_gather_e" in k or "k_sampled_logits" in k:
            for f, w in list(zip(F[k], W.get(k, [0] * len(F[k]))))[-2:]:
                print(f"{c} {k[:48]:48s} n={len(F[k])} fetch {f*1024/1e6:8.2f} MB write {w*1024/1e6:8.2f} MB traffic(2F+W) {(2*f+w)*1024:.0f} B")
PY
