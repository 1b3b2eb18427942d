#!/usr/bin/env python3
"""Diagnostics: trace-kernel duration (HIP events) next to the span of its tiles (first tile start ->
last tile end, s_memrealtime) in the same renders, to see how much of the kernel is launch ramp / drain
rather than tile work. Usage: span_probe.py [W H K]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080, 0.25)
MOVING = os.environ.get("SF_PROBE_MOVING") == "1"   # yaw +1 mrad per render, like bench.py's camera path
frame = [0]


class _Ctx(sf.Sphereflake):
    def Render(self, **kw):
        if MOVING:
            cam = sf.config_camera(W, H, K)
            cam.SetYaw(np.float32(sf.DEFAULT_YAW + 1e-3 * (frame[0] % 20)))
            self.SetCamera(cam)
            frame[0] += 1
        return super().Render(**kw)


with _Ctx(W, H) as s:
    s.SetCamera(sf.config_camera(W, H, K))
    for _ in range(5):
        s.Render()
    s.kernel_timing(True)
    for _ in range(5):
        s.Render()
    plain = s.kernel_timing()
    s.tile_trace(True)
    spans, kms = [], []
    for _ in range(5):
        order = s.tile_order()
        s.Render()
        tr = s.tile_trace().astype(np.int64)
        spans.append((tr[:, 1].max() - tr[:, 0].min()) / 100.0)
        dur = (tr[:, 1] - tr[:, 0]) / 100.0
        st = (tr[:, 0] - tr[:, 0].min()) / 100.0
    kms = s.kernel_timing()[-5:]
    top = np.argsort(dur)[-5:]
    print(f"{W}x{H} K={K}: kernel ms untraced {np.round(plain, 4)}")
    print(f"  traced: kernel ms {np.round(kms, 4)} tile span us {np.round(spans, 1)}")
    print(f"  last traced render: heaviest tiles us {np.round(dur[top], 1)} starting at {np.round(st[top], 2)}; "
          f"tiles still starting after 20 us: {(st > 20).sum()}; mean tile {dur.mean():.2f} us")
    if os.environ.get("SF_FLAGS"):   # SF_FLAGS=0x20: per-wave {start, end} records
        wr = s.wave_trace.astype(np.int64)
        wr = wr[wr[:, 0] > 0]
        t0 = tr[:, 0].min()
        print(f"  waves {len(wr)}: first wave start {(wr[:, 0].min() - t0) / 100:.2f} us, last wave start "
              f"{(wr[:, 0].max() - t0) / 100:.2f}, last wave end {(wr[:, 1].max() - t0) / 100:.2f} (tile times from first tile start)")
    if order is not None:   # where the last traced render's heaviest tiles sat in the order it used
        pos = np.full(len(dur), -1)
        u = order[0] & ((1 << 27) - 1)
        pos[u[::-1]] = np.arange(len(u))[::-1]
        print(f"  order positions of the 5 heaviest tiles: {pos[top]} (moving camera: {MOVING})")
    ends = np.sort((tr[:, 1] - tr[:, 0].min()) / 100.0)
    print(f"  tile ends: 50% by {ends[len(ends)//2]:.1f} us, 90% {ends[int(len(ends)*.9)]:.1f}, 99% {ends[int(len(ends)*.99)]:.1f}, "
          f"last {ends[-1]:.1f}")
