#!/usr/bin/env python3
"""Steady state of the frames-in-flight loop: a fresh process renders the bench's moving 1080p path on F slots
in consecutive windows of 100 frames and prints each window's ms/frame and live shader clock, so the ramp
from the first frames to the steady rate is visible. Usage: ramp_probe.py [F=3] [windows=24]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 3
NW = int(sys.argv[2]) if len(sys.argv) > 2 else 24
W, H, K, WIN = 1920, 1080, 0.25, 100
views = [frame_camera(W, H, K, i).corners() for i in range(WIN * NW)]
d = sf.SphereflakeDist(0, W, H, slots=F)
for s in range(F):
    d.kernel_timing(s, True, period=10)
t_all = time.perf_counter()
for w in range(NW):
    t = time.perf_counter()
    for i in range(WIN):
        d.SetView(*views[w * WIN + i])
        d.RenderBands()
    d.Synchronize()
    ms = (time.perf_counter() - t) / WIN * 1e3
    clk = []
    for s in range(F):
        clk += list(d.kernel_clocks(s, n=4))
    print(f"window {w:2d} (t={(time.perf_counter() - t_all) * 1e3:7.1f} ms): {ms:.4f} ms/frame  "
          f"clock {np.median(clk) if clk else float('nan'):.0f} MHz", flush=True)
d.close()
