set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_sampled.py tests/test_gpu_bpr.py > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -le 1 ] || exit $rc
grep -E "FAILED" $O/pt.log | head
for v in tree stage; do
  lib=""; [ "$v" != tree ] && lib=variants/lib_$v.so
  IKEA_REC_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sb_$v -o s -- python3 tools/sampbench.py --HF 128 256 --prec f32x6 --fused --iters 50 > $O/sb_$v.log 2>&1 || { tail $O/sb_$v.log; exit 1; }
  grep -E "fused|HF" $O/sb_$v.log | grep -v rocprof
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
for f in glob.glob(f"gpurun_out/r03i/sb_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sampled" in r["Name"] or "head_fwd_x" in r["Name"]:
            print(v, r["Name"][:50], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2))
PY
done
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['gather_ms'], d['roofline']['sampled_fwd_ms'])"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/F -o f -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/F.log 2>&1 || { tail $O/F.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/W -o w -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/W.log 2>&1 || { tail $O/W.log; exit 1; }
python3 tools/pmc_summary.py $O/F gather sampled > $O/pmcF.txt; python3 tools/pmc_summary.py $O/W gather sampled > $O/pmcW.txt
cat $O/pmcF.txt $O/pmcW.txt | grep -E "^[a-zA-Z_ ]|FETCH|WRITE" | head -40
