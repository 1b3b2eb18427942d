#!/usr/bin/env python3
"""One multi-GPU member's share (rank 0's bands of an N-way split) rendered `frames` times at `slots` frames in
flight on one GPU -- run under rocprofv3 --kernel-trace to see where a small share's frame time goes.
Usage: share_trace.py [N=8] [slots=3] [frames=300] [W H K]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
SLOTS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
FRAMES = int(sys.argv[3]) if len(sys.argv) > 3 else 300
W, H, K = (int(sys.argv[4]), int(sys.argv[5]), float(sys.argv[6])) if len(sys.argv) > 6 else (1920, 1080, 0.25)
views = [frame_camera(W, H, K, i).corners() for i in range(FRAMES)]
cs = [sf.Sphereflake(W, H) for _ in range(SLOTS)]
for rep in range(2):
    t = time.perf_counter()
    for i in range(FRAMES):
        c = cs[i % SLOTS]
        c.SetView(*views[i])
        c.Render(band_rows=8, band_count=N, band_index=0)
    for c in cs:
        c.Synchronize()
    print(f"N={N} slots={SLOTS}: {(time.perf_counter() - t) / FRAMES * 1e3:.4f} ms per share-frame", flush=True)
for c in cs:
    c.close()
