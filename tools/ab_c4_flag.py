"""bench.py --config c4 with one qlearn module flag set (same-box A/B):

    python tools/ab_c4_flag.py FLAG VALUE [bench.py arguments]"""
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "ikea-recommender-system_amd"))
from recommenders.hip import qlearn  # noqa: E402

setattr(qlearn, sys.argv[1], bool(int(sys.argv[2])))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[3:]
spec = importlib.util.spec_from_file_location("bench_mod", sys.argv[0])
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
bench.main()
