#!/usr/bin/env python3
"""A member's share of a multi-GPU frame measured through bench.py's own timed loop (dist_loop) on one GPU, in
the bench's process environment (torch initialised, same settle and timing): rank 0's bands of an N-way split
with no other ranks, for several frames-in-flight counts. Diagnostic only -- prints ms per frame of the share.
Usage: share_bench.py [slots,...] [N,...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import sphereflake_amd as sf  # noqa: E402  (bench put the package on the path)

import torch  # noqa: E402

SLOTS = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "3,4").split(",")]
NS = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
if os.environ.get("SHARE_NO_TIMING"):   # A/B: no trace-kernel events / clock probes in the loop
    sf.SphereflakeDist.kernel_timing = lambda self, slot, enable=None, n=64, period=1: None if enable is not None else []
    sf.SphereflakeDist.kernel_clocks = lambda self, slot, n=64: []
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
ctl = bench.Control(1, 0)
with sf.Sphereflake(64, 64) as warm:
    warm.SetCamera(sf.config_camera(64, 64, bench.K))
    warm.Render()
    warm.Synchronize()
for rep in range(2):
    for slots in SLOTS:
        row = []
        for n in NS:
            r = bench.dist_loop(ctl, torch, dev, bench.W, bench.H, bench.K, 200, 30, slots, 8, n, lambda i: i,
                                settle_ms=float(os.environ.get("SHARE_SETTLE_MS", bench.SETTLE_MS)))
            r["dist"].close()
            row.append(f"N={n} {r['t_step'] * 1e3:.4f} ms")
        print(f"slots={slots}: " + "  ".join(row), flush=True)
