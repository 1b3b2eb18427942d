#!/usr/bin/env python3
"""Diagnostics: when do the tiles at the head of the heavy-first order start? Renders a few frames,
takes the order the next render will use (sf_get_tile_order), traces that render (sf_set_tile_trace)
and prints start times (us after the first tile start) by order position."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

W, H, K = 1920, 1080, 0.25
with sf.Sphereflake(W, H) as s:
    s.SetCamera(sf.config_camera(W, H, K))
    for _ in range(3):
        s.Render()
    s.Synchronize()
    units, _ = s.tile_order()
    s.tile_trace(True)
    s.Render()
    tr = s.tile_trace().astype(np.int64)
t0 = tr[:, 0].min()
start = (tr[:, 0] - t0) / 100.0
end = (tr[:, 1] - t0) / 100.0
tiles = units & ((1 << 27) - 1)
st = start[tiles]
for a, b in ((0, 8), (8, 64), (64, 256), (256, 1024), (1024, 4096), (4096, 7168), (7168, 8192)):
    print(f"order [{a:5d},{b:5d}): start us min {st[a:b].min():6.2f} median {np.median(st[a:b]):6.2f} max {st[a:b].max():6.2f}")
print(f"first 10 tiles by start: order positions {np.argsort(np.argsort(tiles))[np.argsort(start)[:10]]}")
dur = end - start
print(f"span {end.max():.1f} us; heaviest tile {dur.max():.1f} us starting at {start[np.argmax(dur)]:.2f}")
