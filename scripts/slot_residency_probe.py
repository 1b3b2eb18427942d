#!/usr/bin/env python3
"""Rehearsal of rank 0's receive beside its own trace (VERDICT r4 "residency hazard", csrc/sf_dist.hip): how long a
one-wave kernel on a second stream waits for a wave slot while a persistent 1080p trace grid fills every slot.
Per frame: render (trace on the context stream) and launch the stamp kernel (tests/hip/slot_probe.hip) on a second
stream either AFTER the trace launch (what sf_dist_render did through round 4) or BEFORE it; the stamp's
s_memrealtime against the trace's first and last tile start/end (tile trace, same 100 MHz clock) says where in the
trace the small kernel got its slot. Prints medians in us. Usage: slot_residency_probe.py [N=20]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, H, K = 1920, 1080, 0.25
hip = ctypes.CDLL("libamdhip64.so")
probe = ctypes.CDLL(os.path.join(REPO, "tests", "hip", "build", "libsf_slot_probe.so"))
probe.sf_probe_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
stream = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(stream)) == 0
dbuf = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(dbuf), ctypes.c_size_t(8)) == 0
host = np.zeros(1, np.uint64)


def read_stamp():
    assert hip.hipStreamSynchronize(stream) == 0
    assert hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), dbuf, ctypes.c_size_t(8), 2) == 0   # D2H
    return int(host[0])


views = [frame_camera(W, H, K, i).corners() for i in range(40)]
with sf.Sphereflake(W, H) as s:
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 0.3:
        s.SetView(*views[i % 40])
        s.Render()
        i += 1
    s.Synchronize()
    s.tile_trace(True)
    for order in ("after", "before"):
        rel_first, rel_span, span = [], [], []
        for k in range(N):
            s.SetView(*views[k % 40])
            if order == "before":
                probe.sf_probe_stamp(dbuf, stream)
            s.Render()
            if order == "after":
                probe.sf_probe_stamp(dbuf, stream)
            s.Synchronize()
            st = read_stamp()
            tt = s.tile_trace()
            m = tt[:, 1] > 0
            start, end = int(tt[m, 0].min()), int(tt[m, 1].max())
            rel_first.append((st - start) / 100.0)             # us after the trace's first tile started
            rel_span.append((st - start) / max(1, end - start))   # fraction of the trace's span
            span.append((end - start) / 100.0)
            s.tile_trace(True)
        print(f"stamp launched {order:6s} the trace: starts {np.median(rel_first):8.1f} us after the trace's first tile "
              f"({np.median(rel_span):.3f} of its {np.median(span):.1f}-us span; min {min(rel_first):.1f}, "
              f"max {max(rel_first):.1f})", flush=True)
hip.hipFree(dbuf)
hip.hipStreamDestroy(stream)
