#!/bin/bash
# sampled head's W-side backward + dense Adam on its side stream: sampled / bpr GPU tests, C3 line x3, C2 side run
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sampled.py tests/test_gpu_bpr.py tests/test_gpu_supervised.py tests/test_gpu_long_horizon.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
timeout -k 10 300 python bench.py --config c3 --steps 50 --warmup 10 --no-cpu-baseline --no-native-side --no-eval > $O/c3.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/c3.json'));print('c3', d['value'], d['ms_per_step'], d['step_ms']['median'], d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval > $O/c2.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/c2.json'));t=d['north_star_target'];print('c2', d['value'], d['ms_per_step'], t['frac'], t['kernel_ms'])"
