#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).
Usage: pmc_summary.py [--json OUT [--config KEY]] <dir>...
  --json also writes the means, for bench.py's roofline traffic and `valu`; --config names the bench
  configuration the passes profiled (bench.py pmc_config_key, e.g. "1920x1080 K=0.25 moving"): bench.py
  reports the counters only for that configuration."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

args = sys.argv[1:]
out_json = None
config = None
if args and args[0] == "--json":
    out_json, args = args[1], args[2:]
if args and args[0] == "--config":
    config, args = args[1], args[2:]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in args:
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
means = {}
for k, cs in acc.items():
    if "fill" in k or "copy" in k:
        continue
    means[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    means[k]["profiled_dispatch_us"] = sum(dur[k]) / len(dur[k])
    print(f"== {k}  (profiled dispatch mean {means[k]['profiled_dispatch_us']:.1f} us)")
    for c in sorted(cs):
        print(f"   {c:28s} {means[k][c]:16.1f}")
if out_json:
    # the library build the passes profiled (bench.py uses the counters only for that same build)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sphereflake-raytracer_amd"))
    import sphereflake_amd as sf  # noqa: E402
    with open(out_json, "w") as f:
        rel = sorted({os.path.relpath(d, os.getcwd()) for d in args})
        json.dump({"source": "rocprofv3 --pmc passes of scripts/prof_pmc.sh (" + ", ".join(rel) + "); "
                             "FETCH_SIZE/WRITE_SIZE in KB per dispatch", "config": config, "build": sf.build_info(),
                   "kernels": means}, f, indent=1)
