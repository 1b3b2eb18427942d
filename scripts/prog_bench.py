#!/usr/bin/env python3
"""Frame-less (progressive) mode throughput: random 8-ray packets of one reference worker stream
(mt19937 draws + Sobol pixel choice + packet traversal + last-writer scatter), 1920x1080 K=0.25.
Prints rays/s for a few batch sizes (PROG_BATCHES, comma-separated packet counts). Diagnostics, not the bench line."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K = 1920, 1080, 0.25
with sf.Sphereflake(W, H) as s:
    s.SetCamera(sf.config_camera(W, H, K))
    for variant in ("avx", "sse"):
        s.SetVariant(variant)
        lanes = 8 if variant == "avx" else 4
        for batch in [int(b) for b in os.environ.get("PROG_BATCHES", "16384,65536,262144").split(",")]:
            s.Progressive(12345, batch, 0)
            s.Synchronize()
            reps = 5
            t = time.perf_counter()
            for r in range(reps):
                s.Progressive(12345, batch)
            s.Synchronize()
            dt = (time.perf_counter() - t) / reps
            print(f"{variant} batch {batch:7d} packets: {dt * 1e3:8.3f} ms  {batch * lanes / dt / 1e6:9.1f} Mrays/s")
