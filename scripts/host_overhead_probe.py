#!/usr/bin/env python3
"""Where a lone frame's host-measured latency goes (diagnostics): the same render + Synchronize timed on
(a) an 8x8 frame (one tile: the launch, the stats copy and the wake-up, almost no tracing), (b) a Synchronize with
nothing queued, (c) the 1080p config frame alone, with the trace kernel's own HIP-event duration beside it, and
(d) (c) rendered through a 3-slot SphereflakeDist as bench.py's latency leg does. Medians of N after a warm-up that
keeps the clock up. Usage: host_overhead_probe.py [N=40]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
W, H, K = 1920, 1080, 0.25


def med(x):
    return float(np.median(x)) * 1e6


def warm(s, views, ms=200.0):
    t0 = time.perf_counter()
    i = 0
    while (time.perf_counter() - t0) * 1e3 < ms:
        s.SetView(*views[i % len(views)])
        s.Render()
        i += 1
    s.Synchronize()


views = [frame_camera(W, H, K, i).corners() for i in range(40)]
with sf.Sphereflake(W, H) as big, sf.Sphereflake(8, 8) as tiny:
    tiny.SetView(*frame_camera(8, 8, K, 0).corners())
    warm(big, views)
    a, b, c, ke, rl = [], [], [], [], []
    big.kernel_timing(True)
    for i in range(N):
        warm(big, views, 5.0)   # (the GPU busy right before each sample: no idle clock drop)
        t = time.perf_counter()
        tiny.Render()
        tiny.Synchronize()
        a.append(time.perf_counter() - t)
        t = time.perf_counter()
        tiny.Synchronize()
        b.append(time.perf_counter() - t)
        warm(big, views, 5.0)
        big.SetView(*views[i % 40])
        t = time.perf_counter()
        big.Render()
        t1 = time.perf_counter()
        big.Synchronize()
        c.append(time.perf_counter() - t)
        rl.append(t1 - t)
        ke.append(float(big.kernel_timing(n=1)[-1]) * 1e-3)
    print(f"(a) 8x8 render + sync      {med(a):7.1f} us")
    print(f"(b) sync, nothing queued   {med(b):7.1f} us")
    print(f"(c) 1080p render + sync    {med(c):7.1f} us   (host enqueue {med(rl):.1f} us; trace kernel event {med(ke):.1f} us)")
d = sf.SphereflakeDist(0, W, H, slots=3)
try:
    for i in range(60):
        d.SetView(*views[i % 40])
        d.Render()
    d.Synchronize()
    lat = []
    for i in range(N):
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < 5.0:
            d.SetView(*views[i % 40])
            d.RenderBands()
        d.Synchronize()
        d.SetView(*views[i % 40])
        t = time.perf_counter()
        d.RenderBands()
        d.Synchronize()
        lat.append(time.perf_counter() - t)
    print(f"(d) dist 3 slots render + sync {med(lat):7.1f} us")
finally:
    d.close()
