"""bench.py with the fused head's pass-2 stream at another HIP priority (same-box
A/B of hip/engine.py PASS2_STREAM_PRIORITY):

    python tools/prio_ab.py PRIORITY [bench.py arguments]"""
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "ikea-recommender-system_amd"))
from recommenders.hip import engine  # noqa: E402

engine.PASS2_STREAM_PRIORITY = int(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
spec = importlib.util.spec_from_file_location("bench_mod", sys.argv[0])
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
bench.main()
