#!/usr/bin/env python3
"""Mean duration of a kernel's last N dispatches in a rocprofv3 kernel trace (the timed steps of a
bench run, after its warmup), to compare with bench.py's HIP-event roofline timing.
Usage: trace_avg.py <run_kernel_trace.csv> <kernel> <N>"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"] == sys.argv[2]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[3])
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[-n:]]
print(f"{sys.argv[2]}: {len(rows)} dispatches; last {len(d)}: mean {sum(d) / len(d):.1f} us, "
      f"min {min(d):.1f}, max {max(d):.1f}")
