#!/usr/bin/env python3
"""Round 6: why do loops of 8-frame launches (16 slots, a 1080p member's share over 8) alternate between ~0.0102 and
~0.0195 ms per frame? The slot phase: the dist's frame counter mod 16 decides which slots a launch takes (frames + k)
and which context leads it (c0, whose stream, queues and order the launch uses). Here each phase is set by per-frame
renders first, then 25 launches of 8 frames are timed, 4 reps. Usage: batch_phase_probe.py [phases...]"""
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

W, H, K = 1920, 1080, 0.25
views = np.array([[c for v in frame_camera(W, H, K, i).corners() for c in v] for i in range(40)], np.float32)
phases = [int(p) for p in sys.argv[1:]] or [0, 4, 1, 8]
with sf.SphereflakeDist(0, W, H, rank=0, nranks=8, slots=16) as d:
    def batches(nb):
        for b in range(nb):
            d.RenderBandsFrames(np.ascontiguousarray(views[[(b * 8 + j) % 40 for j in range(8)]]))
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        batches(10)
    d.Synchronize()
    for ph in phases:
        res = []
        for r in range(4):
            # bring the frame counter to phase ph (mod 16) with per-frame renders
            while (d.last_slot() + 1) % 16 != ph:   # (the dist's frame counter mod 16)
                v = views[ph]
                d.SetView(v[0:3], v[3:6], v[6:9], v[9:12])
                d.RenderBands()
            batches(10)   # (settle at this phase: 80 frames keep it)
            d.Synchronize()
            t = time.perf_counter()
            batches(25)
            d.Synchronize()
            res.append((time.perf_counter() - t) / 200 * 1e3)
        print(f"phase {ph:2d}: ms/frame " + " ".join(f"{x:.4f}" for x in res), flush=True)
