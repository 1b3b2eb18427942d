#!/usr/bin/env python3
"""The timed loop of one bench.py run from its rocprofv3 kernel trace: the `steps` trace dispatches after the
warm-up and settle frames (skip = 2 + warmup + settle frames), each one's start and end relative to the loop's
first start, its duration, and the other kernels dispatched in between.
Usage: loop_trace.py <kernel_trace.csv> <bench line json> <warmup>"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
line = json.loads(open(sys.argv[2]).read().strip().split("\n")[-1])
warm = int(sys.argv[3])
steps = line["steps"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tr = [r for r in rows if r["Kernel_Name"].startswith("sf_trace_queue")]
skip = 2 + warm + line["settle"]["frames"]
loop = tr[skip:skip + steps]
t0 = int(loop[0]["Start_Timestamp"])
t_end = max(int(r["End_Timestamp"]) for r in loop)
print(f"frame_ms {line['frame_ms']} fill {line['pipeline']['fill_ms']}: loop span {(t_end - t0) / 1e3:.1f} us")
ids = {id(r) for r in loop}
lo, hi = int(loop[0]["Start_Timestamp"]), t_end
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < lo or s > hi:
        continue
    tag = "T" if id(r) in ids else " "
    print(f"  {tag} {r['Kernel_Name'][:24]:24s} start {(s - t0) / 1e3:8.1f} end {(e - t0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f}"
          f" q{r.get('Queue_Id', r.get('Stream_Id', '?'))}")
