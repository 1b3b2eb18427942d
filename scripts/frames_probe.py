#!/usr/bin/env python3
"""Multi-frame persistent trace probe (round 6): the bench's timed loop shape -- `steps` frames of the moving
camera path between device syncs -- with frames in flight on slots, one launch per frame (RenderBands) against
batches of B frames per launch (RenderBandsFrames), interleaved A/B on one box. Prints ms per frame for the
short loop (the driver's 20 steps), a long loop, and the steady period between them.
Usage: frames_probe.py [W H K] [--share N] [--reps R] [--configs "slots:B,slots:B,..."]"""
import argparse
import gc
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))

import numpy as np  # noqa: E402

import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("W", type=int, nargs="?", default=1920)
    ap.add_argument("H", type=int, nargs="?", default=1080)
    ap.add_argument("K", type=float, nargs="?", default=0.25)
    ap.add_argument("--share", type=int, default=1, help="render rank 0's bands of an N-way split")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--short", type=int, default=20)
    ap.add_argument("--long", type=int, default=200)
    ap.add_argument("--configs", default="3:1,4:4,8:4,8:8")
    ap.add_argument("--scaling", action="store_true",
                    help="N = 1, 2, 4, 8 shares, each with the bench's own policy (bench.frames_per_launch / "
                         "frames_in_flight): per-N frame periods and the ratios to N = 1 on the same basis")
    args = ap.parse_args()
    if args.scaling:
        return scaling(args)
    import torch
    dev = torch.device("cuda", 0)
    W, H, K = args.W, args.H, args.K
    views = np.array([[c for v in frame_camera(W, H, K, i).corners() for c in v] for i in range(40)], np.float32)
    cfgs = [tuple(int(x) for x in c.split(":")) for c in args.configs.split(",")]
    dists = {c: sf.SphereflakeDist(0, W, H, rank=0, nranks=args.share, slots=c[0]) for c in cfgs}

    def loop(d, B, n, start):   # (B = -1: one frame per launch through RenderBandsFrames, for SF_FRAMES_ONE=1)
        if B == -1:
            for i in range(n):
                d.RenderBandsFrames(np.ascontiguousarray(views[[(start + i) % 40]]))
            return
        if B == 1:
            for i in range(n):
                v = views[(start + i) % 40]
                d.SetView(v[0:3], v[3:6], v[6:9], v[9:12])
                d.RenderBands()
        else:
            i = 0
            while i < n:
                b = min(B, n - i)
                idx = [(start + i + j) % 40 for j in range(b)]
                d.RenderBandsFrames(np.ascontiguousarray(views[idx]))
                i += b

    host = {}

    def timed(d, B, n, start):
        torch.cuda.synchronize(dev)
        gc.disable()
        t0 = time.perf_counter()
        loop(d, B, n, start)
        th = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        gc.enable()
        host.setdefault(id(d), []).append(th / n * 1e3)
        return dt

    # warm up every configuration (clock ramp, first-render order)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for c, d in dists.items():
            loop(d, c[1], 40, 0)
    torch.cuda.synchronize(dev)
    res = {c: {"short": [], "long": []} for c in cfgs}
    for r in range(args.reps):
        for c, d in dists.items():
            loop(d, c[1], 40, 0)   # (a short settle before each measurement)
            res[c]["short"].append(timed(d, c[1], args.short, 3) / args.short * 1e3)
            loop(d, c[1], 40, 0)
            res[c]["long"].append(timed(d, c[1], args.long, 7) / args.long * 1e3)
    for c in cfgs:
        s, l_ = np.median(res[c]["short"]), np.median(res[c]["long"])
        steady = (l_ * args.long - s * args.short) / (args.long - args.short)
        print(f"{W}x{H} K={K} share 1/{args.share} slots={c[0]} batch={c[1]}: {args.short} steps "
              f"{s:.4f} ms/frame [{' '.join(f'{x:.4f}' for x in res[c]['short'])}], {args.long} steps {l_:.4f} "
              f"[{' '.join(f'{x:.4f}' for x in res[c]['long'])}], steady {steady:.4f}, "
              f"fill {(s - steady) * args.short:.4f} ms, host enqueue {min(host[id(dists[c])]):.4f} ms/frame", flush=True)
    for d in dists.values():
        d.Synchronize()
        d.close()


def scaling(args):
    """multi-GPU ratios against the best single-GPU period, on one box. Every N (rank 0's share of an
    N-way split -- the rank with the most rows) runs with the slots / frames per launch the bench would give it, and
    the ratio is quoted against N = 1 measured the same way (the bench's own policy, not a slower configuration)."""
    import torch
    import bench
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    W, H, K = args.W, args.H, args.K
    views = np.array([[c for v in frame_camera(W, H, K, i).corners() for c in v] for i in range(40)], np.float32)
    rows = {}
    for n in (1, 2, 4, 8):
        B = bench.frames_per_launch(-1, cus, W, H, 8, n)
        S = bench.frames_in_flight(0, cus, W, H, 8, n, B)
        d = sf.SphereflakeDist(0, W, H, rank=0, nranks=n, slots=S)
        iss = bench.FrameIssuer(d, d.RenderBands, B)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            iss.issue(views)
        d.Synchronize()
        res = {"short": [], "long": []}
        for r in range(args.reps):
            for key, n_f in (("short", args.short), ("long", args.long)):
                iss.issue(views)   # (settle)
                sel = np.ascontiguousarray(views[np.arange(3, 3 + n_f) % 40])
                torch.cuda.synchronize(dev)
                gc.disable()
                t0 = time.perf_counter()
                iss.issue(sel)
                torch.cuda.synchronize(dev)
                res[key].append((time.perf_counter() - t0) / n_f * 1e3)
                gc.enable()
        d.Synchronize()
        d.close()
        s_, l_ = float(np.median(res["short"])), float(np.median(res["long"]))
        steady = (l_ * args.long - s_ * args.short) / (args.long - args.short)
        rows[n] = (B, S, s_, steady)
    b1 = rows[1]
    for n, (B, S, s_, steady) in rows.items():
        print(f"{W}x{H} K={K} N={n}: frames/launch {B}, slots {S}: {args.short} steps {s_:.4f} ms/frame "
              f"({b1[2] / s_:.2f}x N=1's {b1[2]:.4f}), steady {steady:.4f} ms ({b1[3] / steady:.2f}x N=1's steady "
              f"{b1[3]:.4f})", flush=True)


if __name__ == "__main__":
    main()
