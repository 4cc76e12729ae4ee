set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4', d['value'], d['ms_per_step'], d['eval_heldout'])"
timeout -k 10 900 python bench.py --config c5 --steps 4 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c5.json'));print('c5', d['value'], d['ms_per_step'], d['step_ms'], d['eval_heldout'], d['roofline'])"
grep "peak device memory\|trainer built" $O/bench_c5.err
