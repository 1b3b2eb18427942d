#!/usr/bin/env python3
"""What one frame rendered alone spends its time on: per-unit start/end of the persistent trace (SF_FLAGS=0x20,
SF_FLAG_DIAG_UNITS, with the tile trace on) for lone frames of the bench's camera path after a warm-up. Prints the
span, when 50/90/99/100 % of the work units had finished, the longest units (duration, start, part) and how many
units ran in the last 10 % of the span. Diagnostics (the trace stores perturb the timing a little).
Usage: SF_FLAGS=0x20 latency_probe.py [W H K]"""
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
with sf.Sphereflake(W, H) as s:
    views = [frame_camera(W, H, K, i).corners() for i in range(40)]
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 0.3:   # warm-up: the clock, the tile order
        s.SetView(*views[i % 40])
        s.Render()
        i += 1
    s.Synchronize()
    s.tile_trace(True)
    lat = []
    for k in range(6):
        s.SetView(*views[(i + k) % 40])
        t = time.perf_counter()
        s.Render()
        s.Synchronize()
        lat.append((time.perf_counter() - t) * 1e3)
        s.tile_trace()
        ut = s.unit_trace.copy()
        m = ut[:, 1] > 0
        u = ut[m]
        st, en = u[:, 0].astype(np.int64), u[:, 1].astype(np.int64)
        base = st.min()
        span = (en.max() - base) / 100.0
        fin = np.sort(en - base) / 100.0
        q = [fin[int(len(fin) * f) - 1] for f in (0.5, 0.9, 0.99)] + [fin[-1]]
        dur = (en - st) / 100.0
        top = np.argsort(-dur)[:5]
        late = int(((en - base) / 100.0 > 0.9 * span).sum())
        print(f"frame {k}: host {lat[-1] * 1e3:.1f} us, units {len(u)}, span {span:.1f} us; finished 50/90/99/100 %: "
              + "/".join(f"{x:.1f}" for x in q) + f" us; units ending in the last 10 %: {late}; longest: "
              + ", ".join(f"{dur[j]:.1f} us from {(st[j] - base) / 100.0:.1f} (part {int(u[j, 2]) >> 29})" for j in top),
              flush=True)
