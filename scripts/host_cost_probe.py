#!/usr/bin/env python3
"""Host cost per call of the per-frame API (what bounds a small multi-GPU share when the GPU is faster than
the host): SetView alone, Render of a sky-only view (cheap tiles, so the GPU keeps up), the raw ctypes
calls with prebuilt arguments, and the dist path. Prints microseconds per call."""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402

N = 4000
W, H = 1920, 1080
SKY = ([0.0, 0.0, 10.0], [-1.0, 1.0, 11.0], [1.0, 1.0, 11.0], [-1.0, -1.0, 11.0])   # rays leave the flake


def per_call(fn, n=N):
    fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t) / n * 1e6


def main():
    c = sf.Sphereflake(W, H)
    c.SetView(*SKY)
    lib = sf.lib()
    print(f"SetView (python)          {per_call(lambda: c.SetView(*SKY)):7.2f} us", flush=True)
    arrs = [(ctypes.c_float * 3)(*v) for v in SKY]
    ptrs = [ctypes.cast(a, sf._F) for a in arrs]
    print(f"sf_set_view (raw ctypes)  {per_call(lambda: lib.sf_set_view(c.ctx, *ptrs)):7.2f} us", flush=True)
    for n in (1, 8, 64):
        kw = dict(band_rows=8, band_count=n, band_index=0)
        c.Synchronize()
        t = per_call(lambda: c.Render(**kw), 2000)
        c.Synchronize()
        p = sf.render_params(**kw)
        pr = ctypes.byref(p)
        t2 = per_call(lambda: lib.sf_render(c.ctx, pr), 2000)
        c.Synchronize()
        print(f"Render 1/{n:<2} share (python) {t:7.2f} us   raw ctypes {t2:7.2f} us", flush=True)
    c.close()
    d = sf.SphereflakeDist(0, W, H, rank=0, nranks=8, slots=3)
    d.SetView(*SKY)
    d.RenderBands()
    d.Synchronize()
    print(f"dist SetView+RenderBands 1/8 {per_call(lambda: (d.SetView(*SKY), d.RenderBands()), 2000):7.2f} us",
          flush=True)
    d.Synchronize()
    d.close()


if __name__ == "__main__":
    main()
