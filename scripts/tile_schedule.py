#!/usr/bin/env python3
"""Diagnostics: record the per-tile schedule of the wave kernel (sf_set_tile_trace) for a config and
save it as .npy for offline analysis (start/end ticks at 100 MHz, XCC id, HW_ID)."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
import sphereflake_amd as sf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--K", type=float, default=0.25)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "tile_trace.npy"))
    ap.add_argument("--counts", action="store_true", help="library is a COUNTS=1 build: print event counts")
    a = ap.parse_args()
    with sf.Sphereflake(a.width, a.height) as s:
        s.SetCamera(sf.config_camera(a.width, a.height, a.K))
        s.Render()
        s.Synchronize()   # settle the adaptive LDS levels (host hint) before the traced renders
        s.tile_trace(True)
        for _ in range(a.reps):
            s.Render()
        tr = s.tile_trace()
        ph = s.phase_sums.astype(np.float64)
        ut = s.unit_trace.copy()
    if a.counts:
        names = ["nodes tested", "child iterations", "no-lane-hit iterations", "children entered", "leaf skips"]
        per = a.reps
        print("event counts per render:", ", ".join(f"{n} {ph[k] / per:.0f}" for k, n in enumerate(names)))
        print(f"  iterations/node {ph[1] / max(ph[0], 1):.2f}, miss share {ph[2] / max(ph[1], 1):.3f}, "
              f"entered/node {ph[3] / max(ph[0], 1):.2f}")
        it = max(ph[1], 1)
        print(f"  lane utilisation: active lanes/iteration {ph[5] / it:.2f} of 64, bounding-hit lanes/iteration "
              f"{ph[6] / it:.2f}; active lanes/expanded node {ph[7] / max(ph[0], 1):.2f}; inline leaf tests "
              f"{ph[8] / per:.0f} with {ph[9] / max(ph[8], 1):.2f} active lanes")
        print(f"  iterations at depth >= 4: {ph[10] / it:.3f} of all, {ph[11] / max(ph[10], 1):.2f} active lanes; "
              f"iterations with <= 32 active lanes: {ph[14] / it:.3f}; occlusion-checked entries {ph[13] / per:.0f}, "
              f"wholly culled {ph[12] / per:.0f}; waves {ph[15] / per:.0f}")
    elif ph.sum() > 0:
        # traverse_ray's stamps: 0 = back at the loop head (a child whose bounding/LOD test no lane passed, an inline
        # leaf, a culled entry), 2 = a child's bounding + LOD test that some lane passed, 4 = occlusion cull + self
        # test, 1 = push, 6 = expand (node read + child build + cone cull), 5 = pop
        names = {0: "loop head (misses, leaves, culls)", 2: "child test (some lane hit)", 4: "occlusion + self test",
                 1: "push", 6: "expand", 5: "pop", 3: "-"}
        tot = ph[0:7].sum()
        print("segment shares (stamp build, all reps):",
              ", ".join(f"{names[k]} {100 * ph[k] / tot:.1f}%" for k in (0, 2, 4, 1, 6, 5)))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.save(a.out, tr)
    if ut[:, 1].any():   # SF_FLAG_DIAG_UNITS: per work unit
        np.save(a.out.replace(".npy", "_units.npy"), ut)
        m = ut[:, 1] > 0
        u0 = ut[m, 0].min()
        du = (ut[m, 1] - ut[m, 0]) / 100.0
        print(f"units {m.sum()} span {(ut[m, 1].max() - u0) / 100.0:.1f} us; unit us mean {du.mean():.2f} "
              f"p99 {np.percentile(du, 99):.2f} max {du.max():.2f}")
    t0 = tr[:, 0].min()
    dur = (tr[:, 1] - tr[:, 0]) / 100.0   # us
    span = (tr[:, 1].max() - t0) / 100.0
    print(f"tiles {len(tr)} span {span:.1f} us; tile us mean {dur.mean():.2f} p50 {np.median(dur):.2f} "
          f"p99 {np.percentile(dur, 99):.2f} max {dur.max():.2f}")


if __name__ == "__main__":
    main()
