#!/usr/bin/env python3
"""Diagnostics: the per-tile cost outside the traversal. Times the persistent trace kernel (HIP events
around it) on a 1920x1080 view turned away from the flake (every ray misses the root's bounding sphere:
ray generation, the root test, shading and the G-buffer stores only) next to the config view.
Usage: sky_probe.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K = 1920, 1080, 0.25
for name, dyaw in (("config view", 0.0), ("turned away (all sky)", np.pi)):
    with sf.Sphereflake(W, H) as s:
        cam = sf.config_camera(W, H, K)
        cam.SetYaw(np.float32(sf.DEFAULT_YAW + dyaw))
        cam.SetPitch(np.float32(-sf.DEFAULT_PITCH if dyaw else sf.DEFAULT_PITCH))
        s.SetCamera(cam)
        for _ in range(20):
            s.Render()
        s.kernel_timing(True)
        for _ in range(100):
            s.Render()
        ms = np.array(s.kernel_timing())
        s.Synchronize()
        st = s.GetMaxDepthReached()
        print(f"{name:24s} trace kernel {ms.mean() * 1e3:7.1f} us (min {ms.min() * 1e3:6.1f}), max depth {st}")
