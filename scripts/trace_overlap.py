#!/usr/bin/env python3
"""Where a frame's time goes in a rocprofv3 kernel trace of frames in flight (scripts/share_trace.py):
per kernel the mean duration, the frame period (start-to-start of the trace kernel), how many trace
kernels run at once, and the time from a trace kernel's end to the next dispatch on its queue.
Usage: trace_overlap.py <run_kernel_trace.csv> [skip=50]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 50
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
trace = [r for r in rows if r["Kernel_Name"].startswith("sf_trace_queue")]
t0 = trace[skip]["s"] if len(trace) > skip else rows[0]["s"]
t1 = trace[-1]["e"]
sel = [r for r in rows if t0 <= r["s"] and r["e"] <= t1]
by = collections.defaultdict(list)
for r in sel:
    by[r["Kernel_Name"]].append((r["e"] - r["s"]) / 1e3)
tr = [r for r in trace if t0 <= r["s"]]
print(f"window {(t1 - t0) / 1e3:.1f} us, {len(tr)} trace dispatches: period {(t1 - t0) / 1e3 / max(1, len(tr)):.2f} us")
for k, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k[:40]:40s} n={len(d):5d} mean {sum(d) / len(d):7.2f} us  min {min(d):7.2f}  max {max(d):7.2f}")
# concurrency of trace kernels over the window (time-weighted)
ev = sorted([(r["s"], 1) for r in tr] + [(r["e"], -1) for r in tr])
acc = collections.Counter()
cur, last = 0, t0
for t, d in ev:
    acc[cur] += t - last
    cur, last = cur + d, t
tot = sum(acc.values()) or 1
print("  trace kernels running at once (time share): " +
      "  ".join(f"{k}: {v / tot * 100:.0f}%" for k, v in sorted(acc.items())))
# per queue: gap from a trace kernel's end to the next dispatch's start on the same queue
qk = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
if qk:
    perq = collections.defaultdict(list)
    for r in sel:
        perq[r[qk]].append(r)
    gaps = []
    for q, rs in perq.items():
        for a, b in zip(rs, rs[1:]):
            if a["Kernel_Name"].startswith("sf_trace_queue"):
                gaps.append((b["s"] - a["e"]) / 1e3)
    if gaps:
        gaps.sort()
        print(f"  {qk}s {len(perq)}; trace end -> next dispatch on its queue: median {gaps[len(gaps) // 2]:.2f} us, "
              f"p90 {gaps[int(len(gaps) * 0.9)]:.2f}")
