#!/usr/bin/env python3
"""Host cost of the index-slab format decision (csrc/sf_capi.hip sf_slab_bytes -> index_depth_proven, the branch and
bound over the node tree run inside sf_dist_render / sf_group_render for a view the cheap bound cannot decide and the
64-entry cache does not hold): N non-repeating views, camera scale K log-uniform over [0.05, 2.5] (near the flake and
inside its bounding ball included), each view timed once, uncached. Prints the time quantiles per call and the format
split. Usage: slab_bytes_probe.py [N=400]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
W, H = 1920, 1080
rng = np.random.default_rng(7)
times, fmt = [], []
with sf.Sphereflake(W, H) as s:
    for k in range(N):
        cam = sf.Camera(W, H)
        K = float(np.exp(rng.uniform(np.log(0.05), np.log(2.5))))
        cam.SetPosition(np.asarray(sf.DEFAULT_CAMERA_POSITION, np.float32) * np.float32(K)
                        + rng.normal(0.0, 0.15 * K, 3).astype(np.float32))
        cam.SetPitch(np.float32(sf.DEFAULT_PITCH + rng.uniform(-0.4, 0.4)))
        cam.SetYaw(np.float32(sf.DEFAULT_YAW + rng.uniform(-0.6, 0.6)))
        s.SetView(*cam.corners())
        t = time.perf_counter()
        b = s.slab_bytes()
        times.append(time.perf_counter() - t)
        fmt.append(b)
t = np.array(times) * 1e6
print(f"{N} views: sf_slab_bytes median {np.median(t):.1f} us, p90 {np.percentile(t, 90):.1f}, p99 "
      f"{np.percentile(t, 99):.1f}, max {t.max():.1f} us; 4-B format on {fmt.count(4)}, 16-B on {fmt.count(16)}",
      flush=True)
