"""Share of pass 1's wave time spent waiting in its chunk barriers (diagnostic
build: tools/build_variant.sh flstamp head_flash.hip -DFL_STAMP), at C2 shapes:
runs tools/flashx.py in-process, then reads the per-wave counters of the last
pass-1 launch."""
import ctypes as C
import os
import runpy
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.argv = [os.path.join(HERE, "flashx.py"), "--terms", "636", "--iters", "2"]
runpy.run_path(sys.argv[0], run_name="__main__")
from recommenders.hip import load_library  # noqa: E402

lib = load_library()
n = 4096 * 2
buf = np.zeros(n, dtype=np.uint64)
assert lib.rg_fl_stamp_read(buf.ctypes.data_as(C.c_void_p), C.c_int64(n)) == 0
b = buf.reshape(-1, 2).astype(np.float64)
b = b[b[:, 1] > 0]
fr = b[:, 0] / b[:, 1]
print(f"waves {len(b)}: barrier wait / wave cycles median {np.median(fr):.3f} "
      f"(p10 {np.percentile(fr, 10):.3f}, p90 {np.percentile(fr, 90):.3f}); wave cycles median {np.median(b[:, 1]):.3e}")
