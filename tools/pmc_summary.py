"""Per-kernel means of rocprofv3 --pmc CSV counters: python tools/pmc_summary.py DIR [substr ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
keys = sys.argv[2:]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        short = name.split("(")[0][-60:]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[short]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
