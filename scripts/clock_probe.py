#!/usr/bin/env python3
"""The live shader clock under the bench's loop shapes: F slots, the moving 1080p path, chunks of `chunk` frames
each followed by a Synchronize (bench.settle's shape), for `ms` milliseconds; prints every 10th chunk's ms/frame and
the median clock of its timed trace kernels. PROBE_TORCH=1: a torch process (as the bench's).
Usage: clock_probe.py F chunk ms"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
if os.environ.get("PROBE_TORCH"):
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
import sphereflake_amd as sf  # noqa: E402
from bench import path_views  # noqa: E402

F, CHUNK, MS = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
view_at = path_views(1920, 1080, 0.25, lambda i: i)
d = sf.SphereflakeDist(0, 1920, 1080, slots=F)
for s in range(F):
    d.kernel_timing(s, True, period=1)
t0 = time.perf_counter()
k = c = 0
while (time.perf_counter() - t0) * 1e3 < MS:
    t = time.perf_counter()
    for _ in range(CHUNK):
        d.SetView(*view_at(k))
        d.RenderBands()
        k += 1
    d.Synchronize()
    dt = (time.perf_counter() - t) / CHUNK * 1e3
    if c % 10 == 0:
        clk = []
        for s in range(F):
            clk += list(d.kernel_clocks(s, n=max(1, CHUNK // F)))
        print(f"chunk {c:4d} (t={(time.perf_counter() - t0) * 1e3:7.1f} ms): {dt:.4f} ms/frame  clock {np.median(clk):.0f} MHz",
              flush=True)
    c += 1
d.close()
