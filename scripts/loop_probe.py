#!/usr/bin/env python3
"""Where the bench's timed loop loses against plain frames in flight: the same moving 1080p path, F slots,
rendered (a) by F plain contexts, (b) by sf_dist RenderBands, (c) sf_dist with the bench's kernel-timing period,
interleaved repeats. Prints ms/frame and the host's issue time per frame (the enqueue loop alone, before the
final wait): an issue time near the frame time means the loop is host-bound. Usage: loop_probe.py [W H K]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera, slot_period  # noqa: E402

W, H, K = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080, 0.25)
STEPS, WARM = 200, 30
views = [frame_camera(W, H, K, i).corners() for i in range(WARM + STEPS)]


def timed(issue, sync):
    for i in range(WARM):
        issue(i)
    sync()
    t = time.perf_counter()
    for i in range(STEPS):
        issue(WARM + i)
    t_issue = time.perf_counter() - t
    sync()
    return (time.perf_counter() - t) / STEPS * 1e3, t_issue / STEPS * 1e3


def plain(F):
    cs = [sf.Sphereflake(W, H) for _ in range(F)]

    def issue(i):
        c = cs[i % F]
        c.SetView(*views[i])
        c.Render()

    def sync():
        for c in cs:
            c.Synchronize()
    return cs, issue, sync


def dist(F, timing):
    d = sf.SphereflakeDist(0, W, H, slots=F)
    if timing:
        for s in range(F):
            d.kernel_timing(s, True, period=slot_period(STEPS, F))

    def issue(i):
        d.SetView(*views[i])
        d.RenderBands()
    return [d], issue, d.Synchronize


objs = {}
for F in (3, 4):
    objs[("plain", F)] = plain(F)
    objs[("dist", F)] = dist(F, False)
    objs[("dist+timing", F)] = dist(F, True)
res = {k: [] for k in objs}
for rep in range(4):
    for k, (_, issue, sync) in objs.items():
        res[k].append(timed(issue, sync))
for (name, F), v in res.items():
    v = np.array(v)
    print(f"{W}x{H} F={F} {name:12s}: ms/frame {np.round(v[:, 0], 4)} median {np.median(v[:, 0]):.4f}   "
          f"issue ms/frame median {np.median(v[:, 1]):.4f}")
