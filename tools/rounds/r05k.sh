#!/bin/bash
# round 4: atomic-free Q-head gradients (rest of the affected tests), C4 bench + kernel stats, C5 step timeline
set -o pipefail
mkdir -p gpurun_out/r05k
timeout -k 10 600 python -u -m pytest tests/test_gpu_qlearning.py tests/test_gpu_dist_q.py tests/test_gpu_ckpt_eval.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05k/pytest.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/r05k/pytest.txt | tail -20; tail -30 gpurun_out/r05k/pytest.txt; exit 1; }
tail -2 gpurun_out/r05k/pytest.txt
timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05k/bench_c4.json 2> gpurun_out/r05k/bench_c4.err || { tail -20 gpurun_out/r05k/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05k/bench_c4.json'));print('c4',d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05k/prof_c4 -o c4 -- python bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline --no-native-side --no-eval > gpurun_out/r05k/prof_c4.log 2>&1 || { echo "rocprof c4 failed"; tail gpurun_out/r05k/prof_c4.log; exit 1; }
find gpurun_out/r05k/prof_c4 -name "*kernel_trace.csv" -delete
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05k/c5prof -o c5 -- python3 tools/stepprof.py --config c5 --steps 3 --warmup 1 > gpurun_out/r05k/c5prof.log 2>&1 || { tail -20 gpurun_out/r05k/c5prof.log; exit 1; }
python3 tools/kwindow.py $(find gpurun_out/r05k/c5prof -name "c5_kernel_trace.csv" | head -1) --steps 3 --timeline gpurun_out/r05k/c5_timeline.txt > gpurun_out/r05k/c5_step_kernel_stats.csv 2> gpurun_out/r05k/c5_window.txt || exit 1
cat gpurun_out/r05k/c5_window.txt
rm -rf gpurun_out/r05k/c5prof
echo done
