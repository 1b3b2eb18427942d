#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch). Usage: pmc_summary.py <dir>..."""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in acc.items():
    if "fill" in k or "copy" in k:
        continue
    print(f"== {k}  (profiled dispatch mean {sum(dur[k]) / len(dur[k]):.1f} us)")
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
