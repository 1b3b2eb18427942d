#!/usr/bin/env python3
"""Round 6: kernel-trace summary of multi-frame launches (sf_trace_frames1) -- per launch its duration, queue and the
overlap with the launch before it, grouped into loops by idle gaps. Usage: batch_trace_summary.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import Counter

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith("sf_trace_frames1")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
loops, cur, last_end = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last_end is not None and s - last_end > 200_000:   # (> 200 us idle: a new loop)
        loops.append(cur)
        cur = []
    cur.append((s, e, r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    last_end = e if last_end is None else max(last_end, e)
loops.append(cur)
for i, lp in enumerate(loops):
    if len(lp) < 8:
        continue
    span = (lp[-1][1] - lp[0][0]) / 1e3
    durs = [(e - s) / 1e3 for s, e, _, _ in lp]
    ov = [max(0, min(lp[k - 1][1], lp[k][1]) - lp[k][0]) / 1e3 for k in range(1, len(lp))]
    qs = Counter(q for _, _, q, _ in lp)
    print(f"loop {i}: {len(lp)} launches, span {span:.1f} us, {span / len(lp) / 8:.4f} ms-per-frame-equiv x1e3, "
          f"launch mean {sum(durs) / len(durs):.1f} us (min {min(durs):.1f} max {max(durs):.1f}), mean overlap with "
          f"the previous {sum(ov) / max(1, len(ov)):.1f} us, queues {dict(qs)}")
