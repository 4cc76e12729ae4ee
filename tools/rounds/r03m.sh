set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m; mkdir -p $O
for v in tree $VARIANTS; do
  lib=""; [ "$v" != tree ] && lib=variants/lib_$v.so
  for r in 1 2; do
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sb_${v}_$r -o s -- python3 tools/sampbench.py --HF 128 --prec f32x6 --fused --planes --iters 50 > $O/sb_$v.log 2>&1 || { tail $O/sb_$v.log; exit 1; }
  python3 - "$v" "$r" <<'PY'
import csv, glob, sys
v, r = sys.argv[1], sys.argv[2]
for f in glob.glob(f"gpurun_out/r03m/sb_{v}_{r}/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "sampled_logits" in row["Name"]:
            print(v, r, row["Name"][:48], "avg_us", round(float(row["AverageNs"]) / 1e3, 2), "min_us", round(float(row["MinNs"]) / 1e3, 2))
PY
  done
done
