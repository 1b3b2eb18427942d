#!/usr/bin/env python3
"""A multi-GPU member's share of a frame on one GPU: rank 0's interleaved 8-row bands of an N-way split
(band_count N, band_index 0), traced at `slots` frames in flight on the bench's moving camera path, for split
rules (SF_SPLIT_BUCKETS: auto = into idle wave slots only; model = the makespan model of sf_order_scan).
Prints ms per frame of the share, the N x speed-up over the whole frame and the host's enqueue time per frame
(the loop before the final synchronize). Usage: share_probe.py [W H K]

Frames in flight: PROBE_SLOTS=policy (the default) gives every N the bench's own policy (bench.frames_in_flight:
3 for a whole 1080p frame, 4 for a share that leaves most of the grid idle), so the N = 1 basis of every ratio is
the bench's best single-GPU period (round 5 quoted 1080p ratios against N = 1 at 4 in flight, a slower
basis); PROBE_SLOTS=1,3 runs every N at each of the given counts, as before. Each line names its N = 1 basis."""
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:   # (bench.HW_QUEUES, before the HIP runtime starts)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera, frames_in_flight  # noqa: E402

W, H, K = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080, 0.25)
STEPS, WARM = int(os.environ.get("PROBE_STEPS", 120)), int(os.environ.get("PROBE_WARM", 30))
SETTLE_MS = float(os.environ.get("PROBE_SETTLE_MS", 150))
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
        # settle the shader clock as bench.py does (--settle-ms): frames under load for SETTLE_MS before the timed
        # loop -- a 1080p loop of 150 frames (11 ms) otherwise runs inside the ~60-ms clock ramp
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < SETTLE_MS:
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
SLOTS_ENV = os.environ.get("PROBE_SLOTS", "policy")
SLOTS = [0] if SLOTS_ENV == "policy" else [int(v) for v in SLOTS_ENV.split(",")]
SPLITS = os.environ.get("PROBE_SPLITS", "auto").split(",")
NS = [int(v) for v in os.environ.get("PROBE_N", "1,2,4,8").split(",")]
CUS = int(os.environ.get("PROBE_CUS", 256))   # (MI355X: 256 CUs; the bench reads it from the device)
for slots in SLOTS:
    for split in SPLITS:
        base = None
        basis = "no N=1 run"
        row = []
        for n in NS:
            ENQ.clear()
            sl = slots or frames_in_flight(0, CUS, W, H, 8, n)
            ms = np.median([run(n, sl, split) for _ in range(2)])
            if n == 1:
                base = ms
                basis = f"N=1 basis {ms:.4f} ms at {sl} in flight"
            sp = f"{base / ms:.2f}x, " if base else ""
            row.append(f"N={n} {ms:.4f} ms ({sp}{sl} in flight, host {min(ENQ):.4f})")
        print(f"{W}x{H} K={K} slots={SLOTS_ENV if not slots else slots} split={split} [{basis}]: " + "  ".join(row),
              flush=True)
