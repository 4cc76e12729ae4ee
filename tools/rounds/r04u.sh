#!/bin/bash
# final check of the committed tree: GPU suite, smoke, default bench line
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));t=d['north_star_target'];print(d['value'], d['ms_per_step'], d['roofline']['frac'], t['frac'], d['cpu_baseline']['value'], d['harness']['value'])"
