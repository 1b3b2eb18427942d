#!/usr/bin/env python3
"""How long the heavy-first order's kernels hold their slot's queue (diagnostics): from a rocprofv3 kernel trace of a
bench.py run, every order-rebuild dispatch (sf_order_scan / sf_order_scatter, or since round 5 on large frames
sf_order_bucket_scan / sf_order_scatter_plan) -- its duration, and the trace kernel queued behind it on
the same queue: how long after the previous trace on that queue ended it could start. Prints quantiles, and the total
time the order kernels added to their queues' chains. Usage: order_stall.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["q"] = r.get("Queue_Id", r.get("Stream_Id", "?"))
rows.sort(key=lambda r: r["s"])
byq = defaultdict(list)
for r in rows:
    byq[r["q"]].append(r)
scan, scat, held = [], [], []
for q, ks in byq.items():
    for i, r in enumerate(ks):
        name = r["Kernel_Name"]
        if name.startswith("sf_order_scan") or name.startswith("sf_order_bucket_scan"):
            scan.append((r["e"] - r["s"]) / 1e3)
            # the trace before it on this queue, and the next trace after it
            prev = next((k for k in reversed(ks[:i]) if k["Kernel_Name"].startswith("sf_trace")), None)
            nxt = next((k for k in ks[i + 1:] if k["Kernel_Name"].startswith("sf_trace")), None)
            if prev is not None and nxt is not None:
                held.append((nxt["s"] - prev["e"]) / 1e3)
        elif name.startswith("sf_order_scatter"):
            scat.append((r["e"] - r["s"]) / 1e3)
gaps = []
for q, ks in byq.items():
    tr = [k for k in ks if k["Kernel_Name"].startswith("sf_trace")]
    gaps += [(b["s"] - a["e"]) / 1e3 for a, b in zip(tr, tr[1:]) if b["s"] - a["e"] < 5e6]


def qs(x):
    x = np.array(x)
    return (f"n {len(x)} median {np.median(x):.1f} p90 {np.percentile(x, 90):.1f} max {x.max():.1f} us, total {x.sum():.0f} us"
            if len(x) else "none")


print("scan (sf_order_scan / sf_order_bucket_scan) duration:        ", qs(scan))
print("scatter (sf_order_scatter / sf_order_scatter_plan) duration: ", qs(scat))
print("trace -> next trace on a queue, across a rebuild:", qs(held))
print("trace -> next trace on a queue, all:             ", qs(gaps))
