#!/usr/bin/env python3
"""The SSAO consumer (sf_post_process) alone, for rocprofv3 kernel-trace / PMC passes: one
1920x1080 K=0.25 frame rendered once, then POST_REPS fused post passes (and POST_REPS of the 4-pass chain with
POST_MULTI=1). Prints the mean event time per pass and the tap-radius statistics of the frame (the SSAO taps sit
within `rad` = R / sqrt(|p.z|) pixels of the fragment, post_ssao.glsl:36-55)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K = 1920, 1080, 0.25
reps = int(os.environ.get("POST_REPS", "50"))
flags = sf.SF_POST_GENERAL if os.environ.get("POST_MULTI") == "1" else 0
with sf.Sphereflake(W, H) as s:
    s.SetCamera(sf.config_camera(W, H, K))
    s.Render()
    s.Synchronize()
    for _ in range(5):
        s.PostProcess(flags=flags)
    s.Synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        s.PostProcess(flags=flags)
    s.Synchronize()
    dt = (time.perf_counter() - t) / reps
    pos, nrm, _, _ = s.download()
    st = s.stats()
    R = 8.0 * st.closest
    z = np.abs(pos[..., 2])
    fg = (pos[..., :3] ** 2).sum(-1) > 0
    rad = R / np.sqrt(z[fg])
    q = np.percentile(rad, [50, 90, 99, 99.9, 100])
    print(f"post {'multipass' if flags else 'fused'}: {dt * 1e3:.4f} ms per pass (host-timed, {reps} reps); "
          f"R = {R:.4f}; tap radius px p50 {q[0]:.2f} p90 {q[1]:.2f} p99 {q[2]:.2f} p99.9 {q[3]:.2f} max {q[4]:.2f}; "
          f"foreground {fg.mean():.3f}")
