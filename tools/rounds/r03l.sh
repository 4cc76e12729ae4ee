set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_sampled.py tests/test_gpu_bpr.py > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; grep FAILED $O/pt.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sb -o s -- python3 tools/sampbench.py --HF 128 --prec f32x6 --fused --planes --iters 50 > $O/sb.log 2>&1 || { tail $O/sb.log; exit 1; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r03l/sb/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sampled_logits" in r["Name"]:
            print(r["Name"][:60], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2))
PY
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-native-side > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));t=d['north_star_target'];print('c2', d['value'], d['ms_per_step'], 'target', t['frac'], t['gather_ms'], t['sampled_fwd_ms'], t['kernel_ms'].get('gru_fwd'))"
