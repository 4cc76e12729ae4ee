set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_ckpt_eval.py tests/test_gpu_sampled.py tests/test_gpu_flash_head.py tests/test_gpu_model_parity.py > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; grep FAILED $O/pt.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-native-side > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));t=d['north_star_target'];print('c2', d['value'], d['ms_per_step'], 'target', t['frac'], t['gather_ms'], t['sampled_fwd_ms'], 'harness', d['harness'])"
