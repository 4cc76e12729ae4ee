#!/bin/bash
# negatives gathered in the embedding-gather launch: sampled tests, north-star side run, C3, stamps
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sampled.py tests/test_gpu_bpr.py > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));t=d['north_star_target'];print('c2', d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
done
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-native-side --no-eval > $O/c3.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/c3.json'));t=d['north_star_target'];print('c3', d['value'], d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
IKEA_REC_HIP_LIB=variants/lib_sfstamp.so timeout -k 10 120 python tools/sfstamp.py --wp cold 2>&1 | grep -v amdgpu.ids
IKEA_REC_HIP_LIB=variants/lib_sfbar2.so timeout -k 10 120 python tools/sfstamp.py --wp cold 2>&1 | grep -v amdgpu.ids
for v in "" variants/lib_bar2.so "" variants/lib_bar2.so; do
IKEA_REC_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-native-side --no-eval > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));t=d['north_star_target'];print('lib=${v:-tree}', d['ms_per_step'], t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
done
