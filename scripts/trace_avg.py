#!/usr/bin/env python3
"""Mean duration of a range of a kernel's dispatches in a rocprofv3 kernel trace (the timed steps of a
bench run, after its warmup), to compare with bench.py's HIP-event roofline timing.
Usage: trace_avg.py <run_kernel_trace.csv> <kernel> <N> [<skip>]
  the N dispatches after the first <skip> (default: the last N). The default bench (moving camera) runs
  1 code-object warm-up render (64x64) + 1 first render + W warmup + the settle frames (`settle.frames` of
  the bench line) + S timed + ... renders: its timed loop is skip = 2 + W + settle frames."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"] == sys.argv[2]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[3])
sel = rows[int(sys.argv[4]):int(sys.argv[4]) + n] if len(sys.argv) > 4 else rows[-n:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
where = f"dispatches {sys.argv[4]}..{int(sys.argv[4]) + len(d) - 1}" if len(sys.argv) > 4 else f"last {len(d)}"
print(f"{sys.argv[2]}: {len(rows)} dispatches; {where}: mean {sum(d) / len(d):.1f} us, "
      f"min {min(d):.1f}, max {max(d):.1f}")
