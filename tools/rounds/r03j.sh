set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j; mkdir -p $O
for v in tree nt; do
  lib=""; [ "$v" != tree ] && lib=variants/lib_$v.so
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sb_$v -o s -- python3 tools/sampbench.py --HF 128 256 --prec f32x6 --fused --iters 50 > $O/sb_$v.log 2>&1 || { tail $O/sb_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
for f in glob.glob(f"gpurun_out/r03j/sb_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sampled_logits" in r["Name"]:
            print(v, r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2))
PY
  IKEA_REC_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/F_$v -o f -- python3 tools/sampbench.py --HF 128 256 --prec f32x6 --fused --iters 3 > $O/F_$v.log 2>&1 || { tail $O/F_$v.log; exit 1; }
  IKEA_REC_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/W_$v -o w -- python3 tools/sampbench.py --HF 128 256 --prec f32x6 --fused --iters 3 > $O/W_$v.log 2>&1 || { tail $O/W_$v.log; exit 1; }
  python3 tools/pmc_summary.py $O/F_$v sampled_logits | grep -E "sampled|FETCH"
  python3 tools/pmc_summary.py $O/W_$v sampled_logits | grep -E "sampled|WRITE"
done
