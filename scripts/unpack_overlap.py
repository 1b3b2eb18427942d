#!/usr/bin/env python3
"""How much of each slab-unpack dispatch runs while a trace kernel runs, from a rocprofv3 kernel trace (the evidence
that the multi-GPU receive side overlaps rank 0's / member 0's own trace, csrc/sf_dist.hip, csrc/sf_group.hip).
Usage: unpack_overlap.py <run_kernel_trace.csv> [unpack_prefix] [trace_prefix]
Prints, over the unpack dispatches: count, mean duration, and the mean fraction of each one's interval covered by
the union of trace-kernel intervals (1.0 = entirely beside a trace, 0.0 = serialised after it)."""
import csv
import sys

path = sys.argv[1]
up = sys.argv[2] if len(sys.argv) > 2 else "sf_slab_unpack"
tp = sys.argv[3] if len(sys.argv) > 3 else "sf_trace_queue"
rows = list(csv.DictReader(open(path)))
iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
unp = sorted(iv(r) for r in rows if r["Kernel_Name"].startswith(up))
trc = sorted(iv(r) for r in rows if r["Kernel_Name"].startswith(tp))
# union of the trace intervals
merged = []
for a, b in trc:
    if merged and a <= merged[-1][1]:
        merged[-1][1] = max(merged[-1][1], b)
    else:
        merged.append([a, b])
fr, dur = [], []
j = 0
for a, b in unp:
    cov = 0
    for m0, m1 in merged:
        if m1 <= a:
            continue
        if m0 >= b:
            break
        cov += min(b, m1) - max(a, m0)
    dur.append((b - a) / 1e3)
    fr.append(cov / max(1, b - a))
if not unp:
    sys.exit(f"no {up}* dispatches in {path}")
print(f"{up}*: {len(unp)} dispatches, mean {sum(dur) / len(dur):.1f} us; mean fraction beside a {tp}* dispatch "
      f"{sum(fr) / len(fr):.3f} (min {min(fr):.3f}, max {max(fr):.3f}); {len(trc)} trace dispatches")
