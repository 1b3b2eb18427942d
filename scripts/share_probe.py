#!/usr/bin/env python3
"""A multi-GPU member's share of a frame on one GPU: rank 0's interleaved 8-row bands of an N-way split
(band_count N, band_index 0), traced at `slots` frames in flight on the bench's moving camera path, for split
rules (SF_SPLIT_BUCKETS: auto = into idle wave slots only; model = the makespan model of sf_order_scan).
Prints ms per frame of the share, the N x speed-up over the whole frame and the host's enqueue time per frame
(the loop before the final synchronize). Usage: share_probe.py [W H K]"""
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
STEPS, WARM = int(os.environ.get("PROBE_STEPS", 120)), int(os.environ.get("PROBE_WARM", 30))
if os.environ.get("PROBE_TORCH"):   # A/B: the HIP runtime as a torch process has it (bench.py)
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
views = [frame_camera(W, H, K, i).corners() for i in range(WARM + STEPS)]


def run(n, slots, split):
    os.environ["SF_SPLIT_BUCKETS"] = split
    cs = [sf.Sphereflake(W, H) for _ in range(slots)]
    try:
        def frame(i):
            c = cs[i % slots]
            c.SetView(*views[i])
            c.Render(band_rows=8, band_count=n, band_index=0)
        for i in range(WARM):
            frame(i)
        for c in cs:
            c.Synchronize()
        t = time.perf_counter()
        for i in range(STEPS):
            frame(WARM + i)
        te = time.perf_counter()
        for c in cs:
            c.Synchronize()
        ENQ.append((te - t) / STEPS * 1e3)
        return (time.perf_counter() - t) / STEPS * 1e3
    finally:
        for c in cs:
            c.close()


ENQ = []
SLOTS = [int(v) for v in os.environ.get("PROBE_SLOTS", "1,3").split(",")]
SPLITS = os.environ.get("PROBE_SPLITS", "auto,model").split(",")
NS = [int(v) for v in os.environ.get("PROBE_N", "1,2,4,8").split(",")]
for slots in SLOTS:
    for split in SPLITS:
        base = None
        row = []
        for n in NS:
            ENQ.clear()
            ms = np.median([run(n, slots, split) for _ in range(2)])
            base = ms if n == 1 else base
            sp = f"{base / ms:.2f}x, " if base else ""
            row.append(f"N={n} {ms:.4f} ms ({sp}host {min(ENQ):.4f})")
        print(f"{W}x{H} K={K} slots={slots} split={split}: " + "  ".join(row), flush=True)
