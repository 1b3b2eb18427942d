#!/usr/bin/env python3
"""Registers / spills / occupancy of the kernels from `make -C sphereflake-raytracer_amd isa`
(build/resource_usage.txt, -Rpass-analysis=kernel-resource-usage). Usage: resource_summary.py [kernel ...]"""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(REPO, "sphereflake-raytracer_amd", "build", "resource_usage.txt")
cur, out = None, {}
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        out[cur] = {}
        continue
    m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]|"
                  r"ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur:
        out[cur][m.group(1).split(" [")[0]] = int(m.group(2))
for k in sys.argv[1:] or ["sf_trace_queue1", "sf_trace_queue2", "sf_trace_queue2p", "sf_progressive_trace"]:
    print(k, out.get(k))
