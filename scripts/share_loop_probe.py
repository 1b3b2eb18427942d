#!/usr/bin/env python3
"""Same loop, three front ends, for a member's 1/N share (rank 0's bands): Sphereflake contexts (one per slot),
SphereflakeDist (sf_dist_set_view + sf_dist_render_bands), and SphereflakeDist with the view set on the rendering
slot's context only. Long runs (STEPS frames after WARM), ms per frame and the host's enqueue time per frame.
Usage: share_loop_probe.py [N=8] [slots=3,4] [steps=2000]"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera, W, H, K  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
SLOTS = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "3,4").split(",")]
STEPS = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
WARM = 30
views = [frame_camera(W, H, K, i).corners() for i in range(WARM + STEPS)]


def timed(frame, sync):
    for i in range(WARM):
        frame(i)
    sync()
    t = time.perf_counter()
    for i in range(STEPS):
        frame(WARM + i)
    te = time.perf_counter()
    sync()
    t1 = time.perf_counter()
    return (t1 - t) / STEPS * 1e3, (te - t) / STEPS * 1e3


def ctxs(slots):
    cs = [sf.Sphereflake(W, H) for _ in range(slots)]

    def frame(i):
        c = cs[i % slots]
        c.SetView(*views[i])
        c.Render(band_rows=8, band_count=N, band_index=0)
    r = timed(frame, lambda: [c.Synchronize() for c in cs])
    for c in cs:
        c.close()
    return r


def dist(slots, own_slot_view):
    d = sf.SphereflakeDist(0, W, H, rank=0, nranks=N, slots=slots)
    lib = sf.lib()
    hs = [d.context(s) for s in range(slots)]

    def frame(i):
        if own_slot_view:
            v = [sf._vec3(x) for x in views[i]]
            lib.sf_set_view(hs[i % slots], *v)
        else:
            d.SetView(*views[i])
        d.RenderBands()
    r = timed(frame, d.Synchronize)
    d.close()
    return r


for slots in SLOTS:
    for name, fn in (("contexts", lambda: ctxs(slots)), ("dist", lambda: dist(slots, False)),
                     ("dist, view on the slot only", lambda: dist(slots, True))):
        ms, host = fn()
        print(f"N={N} slots={slots} {name:28s} {ms:.4f} ms/frame  host {host:.4f}", flush=True)
