#!/usr/bin/env python3
"""The bench's projected member-share leg (bench.py `member_shares`) alone, with its host enqueue trace: one dist_loop
per N exactly as bench.py runs it (64 timed steps + a long loop for the steady period), printing the timed and long
loops' ms per frame, the steady period the bench derives, and the host's enqueue time per frame in each loop.
Usage: member_share_probe.py [N=8] [long_steps=600] [reps=2]
PRE=main,c4,n2,n4 (comma list) runs the bench's legs before it first, as bench.py does (the 1080p N = 1 line with its
fixed-view, latency and first-render loops; the 4K loop; the N = 2 / 4 shares), to find what slows the shares there.
SLOTS=k: k frames in flight instead of the bench's policy. EXTRA_STREAMS=k first makes k torch streams, each with one tiny kernel run on it (a hardware queue each), kept alive."""
import os
import sys

os.environ.setdefault("SF_BENCH_ENQ_TRACE", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import bench  # noqa: E402  (raises the process's hardware queues before the HIP runtime starts, as the bench does)
import torch  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
LONG = int(sys.argv[2]) if len(sys.argv) > 2 else 600
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 2
W, H, K = 1920, 1080, 0.25
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
ctl = bench.Control(1, 0)
cus = torch.cuda.get_device_properties(0).multi_processor_count
sl = int(os.environ.get("SLOTS", "0") or 0) or bench.frames_in_flight(0, cus, W, H, 8, N)
extra = [torch.cuda.Stream(device=dev) for _ in range(int(os.environ.get("EXTRA_STREAMS", "0") or 0))]
for st in extra:
    with torch.cuda.stream(st):
        torch.ones(1, device=dev).add_(1)
torch.cuda.synchronize()
for pre in [p for p in os.environ.get("PRE", "").split(",") if p]:
    if pre == "main":
        r = bench.dist_loop(ctl, torch, dev, W, H, K, 200, 30, bench.frames_in_flight(0, cus, W, H, 8, 1), 8, 1,
                            lambda i: i, fixed=True, latency=True, first=True, settle_ms=bench.SETTLE_MS, long_steps=800)
    elif pre == "c4":
        r = bench.dist_loop(ctl, torch, dev, 3840, 2160, 0.22, 60, 15, bench.frames_in_flight(0, cus, 3840, 2160, 8, 1),
                            8, 1, lambda i: i, settle_ms=bench.SETTLE_MS)
    elif pre.startswith("mem"):   # memory only: a k-context dist's G-buffers' worth of hipMalloc / hipFree, no stream
        k = int(pre[3:] or 3)
        bufs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(k) for n in (W * H * 16, W * H * 16,
                                                                                       W * H * 4, W * H * 4)]
        torch.cuda.synchronize()
        del bufs
        torch.cuda.empty_cache()
        continue
    elif pre.startswith("churn"):   # churn<k>: k plain 1080p contexts made and destroyed one after the other
        for _ in range(int(pre[5:])):
            bench.sf.Sphereflake(W, H, device=0).close()
        continue
    elif pre.startswith("ctx"):   # ctx<k>[r]: k plain 1080p contexts made (and with r: each renders once), closed
        k = int(pre[3:].rstrip("r"))
        cs = [bench.sf.Sphereflake(W, H, device=0) for _ in range(k)]
        if pre.endswith("r"):
            for c in cs:
                c.SetCamera(bench.sf.config_camera(W, H, K))
                c.Render()
                c.Synchronize()
        for c in cs:
            c.close()
        continue
    elif pre == "warm":   # bench.py's first context (loads the code object), closed again
        with bench.sf.Sphereflake(64, 64, device=0) as warm:
            warm.SetCamera(bench.sf.config_camera(64, 64, K))
            warm.Render()
            warm.Synchronize()
        continue
    else:
        nn = int(pre[1:])
        r = bench.dist_loop(ctl, torch, dev, W, H, K, 64, 16, bench.frames_in_flight(0, cus, W, H, 8, nn), 8, nn,
                            lambda i: i, settle_ms=bench.SETTLE_MS, long_steps=600, timing=False)
    r["dist"].close()
    print(f"pre {pre}: {r['t_step'] * 1e3:.4f} ms/frame" + (f", clock {r['clock_mhz']:.0f}" if r.get("clock_mhz") else ""),
          flush=True)
for rep in range(REPS):
    rs = bench.dist_loop(ctl, torch, dev, W, H, K, 64, 16, sl, 8, N, lambda i: i, settle_ms=bench.SETTLE_MS,
                         long_steps=LONG, timing=os.environ.get("TIMING") == "1", batch=1)
    rs["dist"].close()
    tr = rs.get("enqueue_trace_us", [])
    parts = []
    for name, t in zip(("timed", "long"), tr):
        enq, end = np.array(t[:-1]), t[-1]
        parts.append(f"{name}: {end / len(enq) / 1e3:.5f} ms/frame, host {np.diff(enq).mean() / 1e3:.5f} ms/frame "
                     f"(max gap {np.diff(enq).max():.0f} us), enqueue ends at {enq[-1] / end:.2f} of the loop")
    p = rs["pipeline"]
    clk = f", clock {rs['clock_mhz']:.0f} / long {p['long_clock_mhz_live']}" if rs.get("clock_mhz") else ""
    print(f"N={N} slots={sl} long={LONG}: steady {p['steady_frame_ms']} ms, fill {p['fill_ms']} ms{clk}; " + "; ".join(parts),
          flush=True)
ctl.close()
