#!/usr/bin/env python3
"""Diagnostics: where a persistent trace frame's time goes at its end. Renders moving-camera frames with
per-tile timing (s_memrealtime, 10 ns ticks) and prints, per frame: the time by which 50/90/99/100 % of
the tiles had finished, how many tiles were still running at 80/90/95 % of the span, and when the 64
heaviest tiles (of this render) started and ended. Usage: tail_probe.py [W H K]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080, 0.25)

with sf.Sphereflake(W, H) as s:
    for f in range(30):
        cam = sf.config_camera(W, H, K)
        cam.SetYaw(np.float32(sf.DEFAULT_YAW + 1e-3 * (f % 20)))
        s.SetCamera(cam)
        if f == 24:
            s.tile_trace(True)
        s.Render()
        if f < 24:
            continue
        tr = s.tile_trace()
        st, en = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
        t0 = st.min()
        st, en = (st - t0) / 100.0, (en - t0) / 100.0   # us
        span = en.max()
        dur = en - st
        q = np.percentile(en, [50, 90, 99, 100])
        running = [int(((st <= x * span) & (en > x * span)).sum()) for x in (0.8, 0.9, 0.95)]
        top = np.argsort(-dur)[:64]
        print(f"span {span:7.1f} us | tiles done by 50/90/99/100 %: {q[0]:6.1f} {q[1]:6.1f} {q[2]:6.1f} {q[3]:6.1f} us"
              f" | running at 80/90/95 % of span: {running} | heaviest 64: dur {dur[top].min():5.1f}-{dur[top].max():5.1f} us,"
              f" start {st[top].min():4.1f}-{st[top].max():5.1f}, end {en[top].min():5.1f}-{en[top].max():5.1f}"
              f" | mean tile {dur.mean():5.1f} us, p99 {np.percentile(dur, 99):5.1f}")
