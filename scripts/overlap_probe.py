#!/usr/bin/env python3
"""Frames in flight on one GPU: F contexts (each its own G-buffer, tile order and stream), frame i of the
bench's moving camera path rendered by context i % F, so frame i+1's persistent grid fills the slots frame
i's tail leaves idle. Prints ms/frame per F (interleaved repeats). Usage: overlap_probe.py [W H K]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

W, H, K = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080, 0.25)
STEPS, WARM = 200, 30
views = [frame_camera(W, H, K, i).corners() for i in range(WARM + STEPS)]
ctxs = [sf.Sphereflake(W, H) for _ in range(4)]


def run(F):
    cs = ctxs[:F]
    for i in range(WARM):
        c = cs[i % F]
        c.SetView(*views[i])
        c.Render()
    for c in cs:
        c.Synchronize()
    t = time.perf_counter()
    for i in range(STEPS):
        c = cs[i % F]
        c.SetView(*views[WARM + i])
        c.Render()
    for c in cs:
        c.Synchronize()
    return (time.perf_counter() - t) / STEPS * 1e3


res = {F: [] for F in (1, 2, 3, 4)}
for rep in range(4):
    for F in (1, 2, 3, 4):
        res[F].append(run(F))
for F, v in res.items():
    print(f"{W}x{H} K={K} F={F}: ms/frame {np.round(v, 4)} median {np.median(v):.4f} -> {W * H / np.median(v) / 1e3:.0f} Mrays/s")
for c in ctxs:
    c.close()
