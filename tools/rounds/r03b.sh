set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r03b/pt.log 2>&1
rc=$?
tail -3 gpurun_out/r03b/pt.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r03b/bench_c2.json 2> gpurun_out/r03b/bench_c2.err || { tail -20 gpurun_out/r03b/bench_c2.err; exit 1; }
echo bench ok
