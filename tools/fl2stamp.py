"""Phase breakdown of pass 2 (k_flash_dw, the fused head's dW + Adam) at C2
shapes from a diagnostic build (tools/build_variant.sh fl2stamp
head_flash.hip -DFL2_STAMP): runs tools/flashx.py in-process, then reads the
per-wave phase cycles of the last pass-2 launch (prologue, S-part MFMA issue,
dZ VALU + split, W-part MFMA issue, barrier wait, epilogue) and the waves'
start / end times (100 MHz realtime) across the rounds of workgroups."""
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
NB, F = 4608, 8
buf = np.zeros(NB * 8 * F, dtype=np.uint64)
assert lib.rg_fl2_stamp_read(buf.ctypes.data_as(C.c_void_p), C.c_int64(buf.size)) == 0
b = buf.reshape(NB, 8, F)
live = b[:, :, 1] > 0
names = ["prologue", "S MFMA issue", "dZ VALU+split", "W MFMA issue", "barrier wait", "epilogue"]
acc = b[:, :, 2:].astype(np.float64)[live]
tot = acc.sum(1)
print(f"waves {live.sum()}  wave cycles median {np.median(tot):.4e}")
out = os.environ.get("FL2_OUT")
if out:
    np.save(out, b)
# per wave index: barrier share and S-issue share; which wave is each workgroup's slowest (least barrier wait)
accw = b[:, :, 2:].astype(np.float64)
totw = accw.sum(2)
full = live.all(1)
bw = accw[full][:, :, 4] / totw[full]
sw = accw[full][:, :, 1] / totw[full]
print("  by wave: barrier share median " + " ".join(f"{np.median(bw[:, i]):.3f}" for i in range(8)))
print("  by wave: S-issue share median " + " ".join(f"{np.median(sw[:, i]):.3f}" for i in range(8)))
slow = np.argmin(bw, axis=1)
print("  slowest wave of the workgroup (count by index): " + " ".join(str(int((slow == i).sum())) for i in range(8)))
for k, n in enumerate(names):
    fr = acc[:, k] / tot
    print(f"  {n:14s} median {np.median(fr):.3f}  p10 {np.percentile(fr, 10):.3f}  p90 {np.percentile(fr, 90):.3f}"
          f"  (median cycles {np.median(acc[:, k]):.3e})")
# workgroup spans (realtime, 100 MHz ticks -> us): start skew per round of 256
st = b[:, :, 0].astype(np.float64)
en = b[:, :, 1].astype(np.float64)
wl = live.any(1)
s0 = np.where(live, st, np.inf).min(1)[wl]
e1 = np.where(live, en, 0).max(1)[wl]
t0 = s0.min()
span = (e1 - s0) / 100.0
print(f"workgroups {wl.sum()}: span median {np.median(span):.1f} us (p10 {np.percentile(span, 10):.1f}, "
      f"p90 {np.percentile(span, 90):.1f}); kernel {((e1.max() - t0) / 100.0):.1f} us")
order = np.argsort(s0)
for r in range(0, min(len(order), 4096), 256):
    idx = order[r:r + 256]
    print(f"  round {r // 256:2d}: start {((s0[idx].min() - t0) / 100):8.1f} .. {((s0[idx].max() - t0) / 100):8.1f} us,"
          f" end {((e1[idx].min() - t0) / 100):8.1f} .. {((e1[idx].max() - t0) / 100):8.1f} us")
