#!/usr/bin/env python3
"""Diagnostics: per-wave start/end of the frame-less trace kernel (SF_FLAGS=0x20 with the tile trace
enabled) for 2^18-packet AVX batches at 1920x1080 K=0.25: kernel span vs per-wave durations, and the
batch time with and without the per-pixel owner atomics (SF_FLAGS=0x60: wrong results, timing only)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K, B = 1920, 1080, 0.25, 1 << 18
with sf.Sphereflake(W, H) as s:
    s.SetCamera(sf.config_camera(W, H, K))
    s.Progressive(12345, B, 0)
    s.Synchronize()
    t = time.perf_counter()
    for _ in range(5):
        s.Progressive(12345, B)
    s.Synchronize()
    print(f"flags {os.environ.get('SF_FLAGS', '0')}: {(time.perf_counter() - t) / 5 * 1e3:.3f} ms per batch")
    if os.environ.get("SF_FLAGS"):
        s.tile_trace(True)
        s.Progressive(12345, B)
        s.Synchronize()
        s.tile_trace()
        waves = B // 8
        wr = s.wave_trace[:waves].astype(np.int64)
        t0 = wr[:, 0].min()
        st, en = (wr[:, 0] - t0) / 100.0, (wr[:, 1] - t0) / 100.0
        du = en - st
        print(f"  waves {waves}: span {en.max():.1f} us; wave us mean {du.mean():.2f} p50 {np.median(du):.2f} "
              f"p99 {np.percentile(du, 99):.2f} max {du.max():.2f}; ends 50% {np.percentile(en, 50):.1f} "
              f"90% {np.percentile(en, 90):.1f} 99% {np.percentile(en, 99):.1f}; last start {st.max():.1f}")
        top = np.argsort(du)[-5:]
        print(f"  heaviest waves {np.round(du[top], 1)} starting at {np.round(st[top], 1)} (wave index {top})")
