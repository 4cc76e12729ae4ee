"""Kernel statistics of a rocprofv3 kernel trace between the two marker
dispatches tools/stepprof.py launches (k_f32_to_f16 on one element), in
rocprofv3's stats CSV format, plus the window's wall span.

    python tools/kwindow.py TRACE.csv [--steps K] [--timeline FILE] > stats.csv

--timeline: every dispatch of the window longer than 0.5 ms (start relative to
the window, duration, name), to see which kernels overlap which."""
import argparse
import collections
import csv
import sys

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=0)
ap.add_argument("--timeline", default="")
ap.add_argument("--min-us", type=float, default=500.0, help="timeline: dispatches at least this long")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "k_f32_to_f16" in r["Kernel_Name"] and int(r["Grid_Size_X"]) <= 256]
if len(marks) < 2:
    sys.exit("kwindow: the two marker dispatches were not found")
win = rows[marks[-2] + 1:marks[-1]]
d = collections.defaultdict(list)
for r in win:
    d[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v, dtype=np.float64)
    w.writerow([k, len(v), int(v.sum()), round(v.mean(), 6), round(100 * v.sum() / tot, 2), int(v.min()), int(v.max()),
                round(v.std(), 6)])
if a.timeline:
    t0 = int(win[0]["Start_Timestamp"])
    with open(a.timeline, "w") as f:
        for r in win:
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e0 - s0 >= a.min_us * 1e3:
                f.write(f"{(s0 - t0) / 1e6:10.4f} {(e0 - s0) / 1e6:9.4f}  {r['Kernel_Name'][:110]}\n")
span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6
sys.stderr.write(f"kwindow: {len(win)} dispatches, kernel time {tot / 1e6:.2f} ms, wall span {span:.2f} ms"
                 + (f" ({span / a.steps:.2f} ms per step)" if a.steps else "") + "\n")
