# sampled-logits variants: kernel durations under rocprofv3 (same box), fused one-launch f32x6 at C2 shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
for v in tree $VARIANTS; do
  lib=""; [ "$v" != tree ] && lib=variants/lib_$v.so
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03d/$v -o s -- python3 tools/sampbench.py --HF 128 --prec f32x6 --fused --iters 50 > gpurun_out/r03d/$v.log 2>&1 || { tail gpurun_out/r03d/$v.log; exit 1; }
  grep "fused" gpurun_out/r03d/$v.log
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
for f in glob.glob(f"gpurun_out/r03d/{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sampled_logits" in r["Name"]:
            print(v, r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2), "min_us", round(float(r["MinNs"]) / 1e3, 2))
PY
done
