# C5 kernel evidence: standalone fused head at HF 256 (B 8192, A 5M) timed + rocprofv3 kernel stats + PMC
# traffic passes, then a rocprofv3 kernel-stats summary of the C5 training step on one MI355X
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03g; mkdir -p $O
FX="tools/flashx.py --B 8192 --A 5000000 --H 256 --terms 636"
timeout -k 10 300 python3 $FX --iters 2 > $O/flashx.txt 2>&1 || { tail $O/flashx.txt; exit 1; }
cat $O/flashx.txt | grep terms
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fx_trace -o fx -- python3 $FX --iters 2 > $O/fx_trace.log 2>&1 || { tail $O/fx_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/F -o f -- python3 $FX --iters 1 > $O/F.log 2>&1 || { tail $O/F.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/W -o w -- python3 $FX --iters 1 > $O/W.log 2>&1 || { tail $O/W.log; exit 1; }
echo "pmc done"
timeout -k 10 1100 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_trace -o c5 -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-kernel-timing > $O/c5_trace.json 2> $O/c5_trace.err || { tail -20 $O/c5_trace.err; exit 1; }
echo "c5 trace done"
python3 - <<'PY'
import csv, glob
for d in ("fx_trace", "c5_trace"):
    for f in glob.glob(f"gpurun_out/r03g/{d}/**/*kernel_stats.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        print(d)
        for r in rows[:14]:
            print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:9.3f} ms tot {float(r['TotalDurationNs'])/1e6:9.2f} ms")
PY
