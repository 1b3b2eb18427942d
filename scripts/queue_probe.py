#!/usr/bin/env python3
"""Frames in flight vs HIP hardware queues: one sf_dist loop (moving 1080p path, F slots) in a fresh process
after a given preamble -- nothing, torch initialised on the device, a throw-away context (the bench's code-
object warm-up), or both -- to see whether the slots' streams land on shared hardware queues
(GPU_MAX_HW_QUEUES, 4 by default). Usage: queue_probe.py <preamble> <F>   (one line of output)
Driver: queue_probe.py all  (runs every case in its own child process, sequentially)"""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(pre, F):
    sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
    sys.path.insert(0, REPO)
    if "torch" in pre:
        import torch
        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
    import sphereflake_amd as sf
    from bench import frame_camera
    if "warm" in pre:
        with sf.Sphereflake(64, 64) as w:
            w.SetCamera(sf.config_camera(64, 64, 0.25))
            w.Render()
            w.Synchronize()
    W, H, K, STEPS, WARM = 1920, 1080, 0.25, 300, 30
    views = [frame_camera(W, H, K, i).corners() for i in range(WARM + STEPS)]
    d = sf.SphereflakeDist(0, W, H, slots=F)
    res = []
    for rep in range(3):
        for i in range(WARM):
            d.SetView(*views[i])
            d.RenderBands()
        d.Synchronize()
        t = time.perf_counter()
        for i in range(STEPS):
            d.SetView(*views[WARM + i])
            d.RenderBands()
        d.Synchronize()
        res.append((time.perf_counter() - t) / STEPS * 1e3)
    d.close()
    res.sort()
    print(f"pre={pre:10s} F={F} HWQ={os.environ.get('GPU_MAX_HW_QUEUES', '-'):3s} ms/frame {res[1]:.4f} "
          f"(min {res[0]:.4f} max {res[2]:.4f})", flush=True)


if __name__ == "__main__":
    if sys.argv[1] != "all":
        child(sys.argv[1], int(sys.argv[2]))
        sys.exit(0)
    rc = 0
    for hwq in (None, "8"):
        for pre in ("none", "torch", "warm", "torch+warm"):
            for F in (2, 3, 4):
                env = dict(os.environ)
                if hwq:
                    env["GPU_MAX_HW_QUEUES"] = hwq
                r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), pre, str(F)], env=env,
                                   timeout=120)
                if r.returncode != 0:
                    sys.exit(r.returncode)
