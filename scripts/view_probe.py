#!/usr/bin/env python3
"""Per-view frame time on the bench's camera path: F slots render one fixed view of the path (frame index i)
for 200 frames, for several i, and the moving path itself, interleaved after a 300 ms settle. Shows whether the
fixed-camera figure differs from the moving one because of the view or of the loop. Usage: view_probe.py [F=3]"""
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
W, H, K, N = 1920, 1080, 0.25, 200
d = sf.SphereflakeDist(0, W, H, slots=F)
moving = [frame_camera(W, H, K, i).corners() for i in range(N)]


def loop(views):
    for i in range(30):
        d.SetView(*views[i % len(views)])
        d.RenderBands()
    d.Synchronize()
    t = time.perf_counter()
    for i in range(N):
        d.SetView(*views[i % len(views)])
        d.RenderBands()
    d.Synchronize()
    return (time.perf_counter() - t) / N * 1e3


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    loop(moving)
cases = {"moving": moving}
for i in (0, 5, 10, 15, 20, 30):
    cases[f"fixed frame {i}"] = [moving[i]]
res = {k: [] for k in cases}
for rep in range(3):
    for k, v in cases.items():
        res[k].append(loop(v))
for k, v in res.items():
    print(f"{k:16s}: ms/frame {np.round(v, 4)} median {np.median(v):.4f}")
d.close()
