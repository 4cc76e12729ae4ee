"""GPU idle time in a rocprofv3 kernel trace: the gaps between the busy
intervals of the last --last dispatches, summed by the kernel that ends each
gap (the one the GPU was waiting to start).

    python tools/gaps.py OUT/x_kernel_trace.csv [--last 1500]
"""
import argparse
import csv
from collections import Counter

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=1500)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]) for r in rows)[-a.last:]
busy_end, gaps = ev[0][1], []
for s, e, n in ev[1:]:
    if s > busy_end:
        gaps.append((s - busy_end, n))
    busy_end = max(busy_end, e)
tot = ev[-1][1] - ev[0][0]
g = sum(x for x, _ in gaps)
print(f"window {tot / 1e6:.3f} ms over {len(ev)} dispatches, idle {g / 1e6:.3f} ms ({g / tot:.3f}) in {len(gaps)} gaps")
c = Counter()
for x, n in gaps:
    c[n] += x
for n, x in c.most_common(12):
    print(f"{x / 1e3:9.1f} us before {n}")
