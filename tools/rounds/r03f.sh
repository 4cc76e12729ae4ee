set -o pipefail
mkdir -p gpurun_out/r03f
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_flash_head.py tests/test_gpu_eval.py tests/test_gpu_qlearning.py tests/test_gpu_ckpt_eval.py tests/test_gpu_dist_q.py > gpurun_out/r03f/pt.log 2>&1
rc=$?; tail -3 gpurun_out/r03f/pt.log; [ $rc -le 1 ] || exit $rc
run() {
  timeout -k 10 300 python tools/bench_patched.py "$2" -- --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-target $3 > gpurun_out/r03f/$1.json 2> gpurun_out/r03f/$1.err || { tail -20 gpurun_out/r03f/$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03f/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['step_ms'])"
}
run c4 none
run c4_merge1 merge1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03f/bench_c2.json 2> gpurun_out/r03f/bench_c2.err || { tail -20 gpurun_out/r03f/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r03f/bench_c2.json'));print(d['value'], d['ms_per_step'], d['harness'], d['north_star_target']['frac'])"
