#!/usr/bin/env python3
"""Where a lone frame's latency goes, on one clock (diagnostics). Part 1 (run under
`rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d DIR -o run -- python3
scripts/lone_frame_timeline.py`): bench.py's latency leg -- a 3-slot SphereflakeDist, one 1080p frame at a time,
SetView + RenderBands + Synchronize -- after a 300-ms warm-up. Part 2 (`lone_frame_timeline.py --report DIR`): for
the last N frames, the HIP API calls and GPU operations of each frame relative to its first API call: when the trace
kernel started and ended, what ran after it, and when the host's wait returned. Prints medians."""
import glob
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 20


def run():
    sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
    sys.path.insert(0, REPO)
    import sphereflake_amd as sf
    from bench import frame_camera
    W, H, K = 1920, 1080, 0.25
    views = [frame_camera(W, H, K, i).corners() for i in range(40)]
    d = sf.SphereflakeDist(0, W, H, slots=3)
    try:
        t0 = time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < 0.3:
            d.SetView(*views[i % 40])
            d.RenderBands()
            i += 1
        d.Synchronize()
        lat = []
        for k in range(N):
            d.SetView(*views[k % 40])
            t = time.perf_counter()
            d.RenderBands()
            d.Synchronize()
            lat.append(time.perf_counter() - t)
        print(f"lone frames: median {np.median(lat) * 1e6:.1f} us (min {min(lat) * 1e6:.1f})", flush=True)
    finally:
        d.close()


def load(path):
    import csv
    with open(path) as f:
        return list(csv.DictReader(f))


def report(root):
    def one(pat):
        m = glob.glob(os.path.join(root, "**", pat), recursive=True)
        return load(m[0]) if m else []
    api = one("*hip_api_trace.csv")
    ker = one("*kernel_trace.csv")
    cpy = one("*memory_copy_trace.csv")
    ev = []
    for r in api:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]))
    for r in ker:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu", r["Kernel_Name"][:40]))
    for r in cpy:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", r.get("Direction", "copy")))
    ev.sort()
    traces = [e for e in ev if e[2] == "gpu" and e[3].startswith("sf_trace")]
    # a frame: from the last trace kernel's launch API call back to the SetView's first call is hard to find in
    # general; anchor each frame on its trace kernel and take the API calls between the previous frame's wait
    # return and this frame's wait return
    syncs = [e for e in ev if e[2] == "api" and e[3] in ("hipStreamSynchronize", "hipEventSynchronize",
                                                          "hipDeviceSynchronize")]
    rows = []
    for tk in traces[-N:]:
        after = [s for s in syncs if s[1] >= tk[1]]
        if not after:
            continue
        w = after[0]
        before = [s for s in syncs if s[1] < tk[0]]
        t0 = before[-1][1] if before else tk[0]
        frame = [e for e in ev if t0 < e[0] <= w[1]]
        first_api = min((e[0] for e in frame if e[2] == "api"), default=t0)
        launch = [e for e in frame if e[2] == "api" and "Launch" in e[3] and e[0] < tk[0]]
        post = [e for e in frame if e[2] in ("gpu", "copy") and e[0] >= tk[1]]
        rows.append({
            "host_calls_to_launch": (launch[-1][1] - first_api) / 1e3 if launch else np.nan,
            "launch_to_kernel_start": (tk[0] - launch[-1][1]) / 1e3 if launch else np.nan,
            "kernel": (tk[1] - tk[0]) / 1e3,
            "kernel_end_to_last_gpu_op_end": ((max(e[1] for e in post) - tk[1]) / 1e3) if post else 0.0,
            "last_gpu_op_end_to_wait_return": (w[1] - max([tk[1]] + [e[1] for e in post])) / 1e3,
            "total": (w[1] - first_api) / 1e3,
            "ops_after": ",".join(e[3] for e in post),
            "api_calls": len([e for e in frame if e[2] == "api"]),
        })
    if not rows:
        print("no frames found")
        return
    for k in rows[0]:
        if k in ("ops_after",):
            print(f"{k:34s} {rows[-1][k]}")
        else:
            print(f"{k:34s} median {np.nanmedian([r[k] for r in rows]):8.1f}  min {np.nanmin([r[k] for r in rows]):8.1f}"
                  f"  max {np.nanmax([r[k] for r in rows]):8.1f}")
    # the last frame in full
    tk = traces[-1]
    w = [s for s in syncs if s[1] >= tk[1]][0]
    before = [s for s in syncs if s[1] < tk[0]]
    t0 = before[-1][1] if before else tk[0]
    print("last frame, us from the previous wait's return:")
    for e in ev:
        if t0 < e[0] <= w[1]:
            print(f"  {(e[0] - t0) / 1e3:8.1f} .. {(e[1] - t0) / 1e3:8.1f}  {e[2]:4s} {e[3]}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
