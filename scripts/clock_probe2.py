#!/usr/bin/env python3
"""The bench's loop sequence on one GPU, step by step, with the live clock of each timed loop: warm-up frames, a
150-ms settle in chunks of 20 (bench.settle), kernel timing switched on (first time: events + clock buffer), stats
reset, then three 200-frame loops back to back. PROBE_EARLY=1 switches timing on before the settle.
Usage: clock_probe2.py F"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
torch.cuda.set_device(0)
torch.cuda.synchronize()
import sphereflake_amd as sf  # noqa: E402
from bench import path_views, settle, slot_period  # noqa: E402

F = int(sys.argv[1])
view_at = path_views(1920, 1080, 0.25, lambda i: i)
views = [view_at(i) for i in range(220)]
d = sf.SphereflakeDist(0, 1920, 1080, slots=F)
early = bool(os.environ.get("PROBE_EARLY"))
kp = slot_period(200, F)
if early:
    for s in range(F):
        d.kernel_timing(s, True, period=kp)
t_w = time.perf_counter()
for i in range(20):
    d.SetView(*views[i])
    d.RenderBands()
settle(d, d.RenderBands, views, 20, t_w, 150.0)
t_gap = time.perf_counter()
for s in range(F):
    d.kernel_timing(s, True, period=kp)
d.Synchronize()
d.reset_stats()
gap = (time.perf_counter() - t_gap) * 1e3
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        d.SetView(*views[20 + i])
        d.RenderBands()
    d.Synchronize()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 200 * 1e3
    clk = []
    for s in range(F):
        clk += list(d.kernel_clocks(s, n=64))
        d.kernel_timing(s, True, period=kp)
    print(f"F={F} early={int(early)} gap {gap:.2f} ms  loop {rep}: {ms:.4f} ms/frame  clock {np.median(clk):.0f} MHz "
          f"(min {min(clk):.0f} max {max(clk):.0f}, {len(clk)} samples)", flush=True)
d.close()
