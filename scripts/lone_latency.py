#!/usr/bin/env python3
"""Lone-frame latency probe (diagnostics): bench.py's latency leg alone -- a 3-slot SphereflakeDist, one 1080p frame of
the moving camera path at a time, SetView -> Render -> Synchronize timed on the host -- over `n` frames after a warm
loop, printed as median / p10 / p90 in us. Usage: lone_latency.py [n=200] [width height K]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
W, H, K = (int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080, 0.25)
views = [bench.frame_camera(W, H, K, i).corners() for i in range(64)]
with sf.SphereflakeDist(0, W, H, slots=3) as d:
    for i in range(100):   # warm: levels settled, clocks up, an order built
        d.SetView(*views[i % len(views)])
        d.Render()
    d.Synchronize()
    lat = []
    for i in range(n):
        d.SetView(*views[i % len(views)])
        t = time.perf_counter()
        d.Render()
        d.Synchronize()
        lat.append(time.perf_counter() - t)
    lat = np.array(lat) * 1e6
    print(f"lone frame {W}x{H}: median {np.median(lat):.1f} p10 {np.percentile(lat, 10):.1f} "
          f"p90 {np.percentile(lat, 90):.1f} us over {n}")
