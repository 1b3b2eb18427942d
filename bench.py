#!/usr/bin/env python3
"""Benchmark: Mrays/s into the G-buffer at 1920x1080 depth 8 (BASELINE.json metric), MI355X.

A "step" is one full deterministic frame of the hot path (ray generation + sphereflake traversal +
G-buffer write, reference Sphereflake.h:86-226 / Sphereflake.cpp:149-201) over a 1920x1080 frame at
the depth-8 camera (BASELINE configs[2]: main.cpp:92-96 camera position scaled by K = 0.25). The
G-buffer stays resident in HBM (the D2H copy into the host GBuffer is timed separately and reported
as `d2h_ms`, never as `value`).

The camera MOVES: step i renders frame f = i * N + rank of a camera path (the config camera with its
yaw swept +-10 mrad around the config view at 1 mrad per frame, `frame_camera`), so the heavy-first tile
schedule always works from the costs of a different view (the reference is an interactive app whose view changes every frame,
main.cpp:304). `first_render_ms` is the first render of a fresh context (row-major tile order, no
previous costs); `fixed_camera` repeats the timed loop on one unchanging view.

Multi-GPU (`--gpus N`, launched by torch.distributed.run): one process per GPU. The frames of a
camera path are independent units, so each rank renders its own 1920x1080 depth-8 frame per step
(frame index = step * N + rank); no data-path collective, `scaling: weak`. `--mode rows` renders ONE
frame per step across N devices behind the C ABI (sf_group_*): interleaved 8-row
bands, strided peer copies into device 0's G-buffer, driven by rank 0 alone (the other ranks only join
the barriers); `scaling: strong`. `--mode rows-rccl` is the earlier per-rank variant (every rank traces
its bands, torch RCCL gather + reassembly on rank 0).

rank 0 prints ONE JSON line. `roofline` prices the dominant kernel against HBM (32 B/ray of G-buffer
stores); `cpu_baseline` times the reference's own AVX packet path (oracle/_ref,
compiled from the reference sources) on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)

import sphereflake_amd as sf  # noqa: E402
from sphereflake_amd import shard  # noqa: E402

W, H, K = 1920, 1080, 0.25          # BASELINE configs[2]
BYTES_PER_RAY = 32                  # two float4 G-buffer stores
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
TRACE_KERNEL = "sf_trace_queue2"    # the dominant kernel (persistent wave-coherent trace, 2 waves/workgroup)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--mode", choices=["frames", "rows", "rows-rccl"], default="frames")
    ap.add_argument("--kernel", choices=["wave", "ray"], default="wave")
    ap.add_argument("--width", type=int, default=W)
    ap.add_argument("--height", type=int, default=H)
    ap.add_argument("--K", type=float, default=K)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the post-process and transfer sections (profiling runs of the timed loop only)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--check", action="store_true", help="verify the frame against the oracle rows")
    return ap.parse_args()


PATH_AMPLITUDE = 10                  # camera path: yaw sweeps +-10 mrad around the config view, 1 mrad/frame


def path_yaw_offset(frame):
    """Yaw offset (rad) of frame `frame` of the camera path: a triangle wave 0, -1, ..., -10, ..., +10, ..., 0
    mrad (period 40 frames). The camera moves 1 mrad every frame yet stays within ~18 px of the BASELINE
    view, so every frame is the config's workload (same max depth, same scene content)."""
    a = PATH_AMPLITUDE
    return 1e-3 * (abs((frame + a) % (4 * a) - 2 * a) - a)


def frame_camera(width, height, k, frame):
    """Frame `frame` of the camera path: the config camera with yaw offset by path_yaw_offset(frame)."""
    cam = sf.config_camera(width, height, k)
    cam.SetYaw(np.float32(sf.DEFAULT_YAW + path_yaw_offset(frame)))
    return cam


KTIMING_PERIOD = 10                  # HIP events on every 10th timed render (fewer steps: denser, see ktiming_period)
KTIMING_MIN_SAMPLES = 8              # at least this many kernel-timing samples per timed loop
CPU_REPS = 40                        # ~1.2 s wall x 16 threads: ~20 s of CPU work


def ktiming_period(steps):
    """Every k-th timed render carries the kernel-timing events: k = 10 (an event pair costs ~7 us of stream
    time per frame, so it is sampled), or less when that would give fewer than KTIMING_MIN_SAMPLES samples."""
    return max(1, min(KTIMING_PERIOD, steps // KTIMING_MIN_SAMPLES))


BASELINE_CONFIGS = {(640, 360, 1.0): "configs[0]", (1280, 720, 0.8): "configs[1]", (1920, 1080, 0.25): "configs[2]",
                    (3840, 2160, 0.22): "configs[3]", (16384, 16384, 0.2): "configs[4]"}


def pmc_config_key(width, height, k, camera):
    """The bench configuration a committed PMC summary was profiled on (scripts/pmc_summary.py --config)."""
    return f"{width}x{height} K={k:g} {camera}"


def load_pmc(kernel, config_key, build):
    """Per-dispatch PMC means of `kernel` from profiles/pmc_traffic.json -- only when that summary was
    profiled on this very configuration AND this very library build (its `build.lib_sha256`); None otherwise:
    counters are never replayed onto another config or another build."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            j = json.load(f)
        if j.get("config") != config_key:
            return None, None
        if (j.get("build") or {}).get("lib_sha256") != build.get("lib_sha256"):
            return None, None
        return j["kernels"][kernel], j.get("source", path)
    except (OSError, KeyError, ValueError):
        return None, None


def pmc_valu(c, cus=256):
    """VALU issue of `kernel` from the committed PMC summary: wave-level VALU instructions per launch
    against the VALU issue slots of the profiled dispatch (CUs x 4 SIMDs x cycles / 2: one wave64
    VALU instruction issues over 2 cycles; cycles = GRBM_GUI_ACTIVE / 8 XCDs)."""
    if c is None:
        return None
    try:
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0
        slots = cus * 4 * cycles / 2.0
        # wavefront occupancy: SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md), summed over the
        # chip -> mean resident waves; against the gfx950 peak of 8 waves per SIMD
        waves = 4.0 * c["SQ_WAVE_CYCLES"] / cycles
        peak_waves = cus * 4 * 8
        out = {"valu_insts": round(c["SQ_INSTS_VALU"]), "salu_insts": round(c["SQ_INSTS_SALU"]),
               "issue_slots": round(slots), "valu_issue_frac": round(c["SQ_INSTS_VALU"] / slots, 4),
               "occupancy": {"mean_waves": round(waves, 1), "peak_waves": peak_waves,
                             "frac": round(waves / peak_waves, 4)},
               "clock_mhz": round(cycles / c["profiled_dispatch_us"], 1), "source": "profiles/pmc_traffic.json"}
        if "SQ_WAIT_INST_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            out["wait_inst_frac"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
            out["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        return out
    except (KeyError, ValueError, ZeroDivisionError):
        return None


def pmc_traffic(c):
    """HBM bytes per launch of the trace kernel from the committed PMC summary (scripts/prof_pmc.sh ->
    scripts/pmc_summary.py --json, separate rocprofv3 --pmc passes of this same bench command):
    WRITE_SIZE + 2 x FETCH_SIZE (gfx950 FETCH_SIZE counts half of a streaming read), KB -> bytes."""
    try:
        return (c["WRITE_SIZE"] + 2.0 * c["FETCH_SIZE"]) * 1024.0
    except (TypeError, KeyError, ValueError):
        return None


def cpu_share():
    """Host cores this process may use: the affinity mask, capped by a cgroup v2 CPU quota if one is set."""
    avail = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return avail, quota


def cpu_baseline(width, height, k, threads):
    """The reference AVX packet path (oracle/_ref/ref_bench, built from /root/reference) on host cores.
    Falls back to the oracle C restatement (per ray, 1 thread) if the reference build is absent."""
    from oracle import pyoracle
    ref = os.path.join(pyoracle.REF_DIR, "ref_bench")
    if os.path.exists(ref):
        r = pyoracle.ref_bench(width, height, k, threads, CPU_REPS)
        r1 = pyoracle.ref_bench(width, height, k, 1, 3)   # also one thread
        avail, quota = cpu_share()
        return {"value": round(r["mrays_per_s"], 3), "unit": "Mrays/s", "cores": threads, "kind": "reference",
                "cores_available": avail, "cgroup_cpu_quota": quota, "host_cores": os.cpu_count(),
                "sample": f"{CPU_REPS} full {width}x{height} K={k} frames (reference 8-ray packet footprint, 8/9 "
                          f"pixel coverage), median; reference AVX path -O3 -mavx, {threads} threads",
                "frame_ms": round(r["median_s"] * 1e3, 2),
                "single_thread": {"value": round(r1["mrays_per_s"], 3), "frame_ms": round(r1["median_s"] * 1e3, 1),
                                  "sample": "3 full frames, 1 thread"}}
    setup = {"W": width, "H": height}
    cam = sf.config_camera(width, height, k)
    o, tl, tr, bl = cam.corners()
    setup.update(origin=o, tl=tl, tr=tr, bl=bl, root=sf.root_transform(o), children=sf.child_transforms())
    rows = np.arange(0, height, 8)
    t0 = time.perf_counter()
    pyoracle.render(setup, rows=rows, threads=1)
    dt = time.perf_counter() - t0
    return {"value": round(len(rows) * width / dt / 1e6, 3), "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"every 8th row of a {width}x{height} K={k} frame, oracle C restatement, 1 thread"}


POST_BYTES_PER_PIXEL = 36   # fused pass: position + normal in (32 B), RGBA8 out (4 B)


def post_rates(ctx, torch, stream, width, height, reps=20):
    """Mean device time of sf_post_process (fused single pass with the reference thresholds, and the
    forced 4-pass chain) over `reps` launches, with HBM roofline of the fused kernel."""
    out = {}
    for name, flags in (("fused", 0), ("multipass", sf.SF_POST_GENERAL)):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        with torch.cuda.stream(stream):
            ctx.PostProcess(flags=flags, stream=stream.cuda_stream)
            for a, b in ev:
                a.record(stream)
                ctx.PostProcess(flags=flags, stream=stream.cuda_stream)
                b.record(stream)
        torch.cuda.synchronize()
        out[name + "_ms"] = round(float(np.mean([a.elapsed_time(b) for a, b in ev])), 4)
    gbs = POST_BYTES_PER_PIXEL * width * height / (out["fused_ms"] * 1e-3) / 1e9
    out["fused_roofline"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_pixel": POST_BYTES_PER_PIXEL}
    return out


def progressive_rates(width, height, k, batch=1 << 18, reps=5):
    """the frame-less mode (the reference's Initialize() worker stream: mt19937 draws,
    Sobol pixel picks, 8-ray AVX / 4-ray SSE packets with packet early-outs, last-writer scatter) on a
    fresh context with the same camera, in batches of `batch` packets continuing one stream."""
    out = {"batch_packets": batch}
    with sf.Sphereflake(width, height) as s:
        s.SetCamera(sf.config_camera(width, height, k))
        for variant, lanes in (("avx", 8), ("sse", 4)):
            s.SetVariant(variant)
            s.Progressive(12345, batch, 0)
            s.Synchronize()
            t = time.perf_counter()
            for _ in range(reps):
                s.Progressive(12345, batch)
            s.Synchronize()
            dt = (time.perf_counter() - t) / reps
            out[variant] = {"ms_per_batch": round(dt * 1e3, 4), "Mrays_per_s": round(batch * lanes / dt / 1e6, 1)}
    return out


def transfer_rates(ctx, torch, dev, stream, width, height, kernel, frames=8):
    """G-buffer D2H cost (positions + normals, 32 B/pixel). Pageable synchronous
    download (sf_download, what the reference-style GetGBuffer pays unpinned), stream-ordered copy into
    page-locked host memory (sf_download_async), and a double-buffered pipeline -- render frame i+1 into
    one device slab while slab i drains over PCIe on a copy stream -- giving the PCIe-inclusive frame
    rate an interactive viewer would see."""
    nbytes = width * height * 32
    ctx.Synchronize()
    t = time.perf_counter()
    ctx.download()
    pageable_ms = (time.perf_counter() - t) * 1e3
    g = ctx.pinned_gbuffer()
    ctx.download_async(g)
    ctx.Synchronize()
    t = time.perf_counter()
    for _ in range(frames):
        ctx.download_async(g)
    ctx.Synchronize()
    pinned_ms = (time.perf_counter() - t) * 1e3 / frames
    ctx.release_pinned()
    # double-buffered pipelines: render frame i+1 while frame i drains over PCIe on a copy stream.
    # "gbuffer": positions + normals (what the reference's PBO upload reads, 32 B/pixel);
    # "image": SSAO + blur + final on the device first (sf_post_process), RGBA8 out (4 B/pixel)
    copy = torch.cuda.Stream(device=dev)

    def pipeline(image):
        slabs = [[torch.empty((height, width, 4), dtype=torch.float32, device=dev) for _ in range(2)] for _ in range(2)]
        rgba = [torch.empty((height, width, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
        if image:
            host = [[torch.empty((height, width, 4), dtype=torch.uint8, pin_memory=True)] for _ in range(2)]
        else:
            host = [[torch.empty((height, width, 4), dtype=torch.float32, pin_memory=True) for _ in range(2)]
                    for _ in range(2)]
        done = [torch.cuda.Event() for _ in range(2)]
        drained = [torch.cuda.Event() for _ in range(2)]
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for i in range(frames + 1):
            b = i & 1
            if i < frames:
                with torch.cuda.stream(stream):
                    if i >= 2:
                        stream.wait_event(drained[b])
                    ctx.render_to(slabs[b][0].data_ptr(), slabs[b][1].data_ptr(), kernel=kernel,
                                  stream=stream.cuda_stream)
                    if image:
                        ctx.PostProcess(slabs[b][0].data_ptr(), slabs[b][1].data_ptr(), rgba[b].data_ptr(),
                                        flags=sf.SF_POST_UNIT_NORMALS, stream=stream.cuda_stream)
                    done[b].record(stream)
            if i >= 1:
                p = (i - 1) & 1
                with torch.cuda.stream(copy):
                    copy.wait_event(done[p])
                    if image:
                        host[p][0].copy_(rgba[p], non_blocking=True)
                    else:
                        host[p][0].copy_(slabs[p][0], non_blocking=True)
                        host[p][1].copy_(slabs[p][1], non_blocking=True)
                    drained[p].record(copy)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) * 1e3 / frames

    pipeline(False)   # warm the pinned pools
    pipe_ms = pipeline(False)
    pipeline(True)
    img_ms = pipeline(True)
    return {"bytes": nbytes, "pageable_ms": round(pageable_ms, 3), "pinned_ms": round(pinned_ms, 3),
            "pinned_GBps": round(nbytes / (pinned_ms * 1e-3) / 1e9, 2),
            "pipelined_frame_ms": round(pipe_ms, 3),
            "pcie_inclusive_Mrays": round(width * height / (pipe_ms * 1e-3) / 1e6, 2),
            "image_pipelined_frame_ms": round(img_ms, 3),
            "image_pcie_inclusive_Mrays": round(width * height / (img_ms * 1e-3) / 1e6, 2),
            "note": "PCIe-inclusive figures; `value` is the HBM-resident render rate"}


def run_rows(args, torch, dist, dist_on, rank, n, kernel):
    """--mode rows: ONE frame per step over N devices from one process (sf_group_*): member k traces the
    8-row bands b = k (mod N); members k > 0 ship theirs into member 0's G-buffer with strided peer copies.
    The camera moves as in frames mode (frame i of the path at step i). When fewer than N devices are
    visible (a one-GPU rehearsal) the members are N contexts on device 0, and the line says so."""
    width, height, band = args.width, args.height, args.band_rows
    visible = torch.cuda.device_count()
    devices = list(range(n)) if visible >= n else [0] * n
    views = [frame_camera(width, height, args.K, i).corners() for i in range(args.warmup + args.steps)]
    g = None
    first_ms = trace_ms = None
    if rank == 0:
        g = sf.SphereflakeGroup(devices, width, height)
        if kernel != sf.SF_KERNEL_WAVE:
            raise SystemExit("--mode rows traces with the wave kernel")
        g.SetView(*views[0])
        t = time.perf_counter()
        g.Render(band)
        g.Synchronize()
        first_ms = (time.perf_counter() - t) * 1e3
        for i in range(args.warmup):
            g.SetView(*views[i])
            g.Render(band)
        g.member_kernel_timing(0, True, period=ktiming_period(args.steps))
        g.Synchronize()
        g.reset_stats()
    if dist_on:
        dist.barrier()
    t0 = time.perf_counter()
    if rank == 0:
        for i in range(args.steps):
            g.SetView(*views[args.warmup + i])
            g.Render(band)
        g.Synchronize()
    dt = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
    if rank != 0:
        return
    st = g.stats()
    if st.overflow_tiles:
        raise RuntimeError("traversal overflowed SF_MAX_DEPTH_LIMIT")
    tk = g.member_kernel_timing(0, n=min(-(-args.steps // ktiming_period(args.steps)), 64))
    trace_ms = float(np.mean(tk)) if len(tk) else dt / args.steps * 1e3
    rays0 = sf.lib().sf_slab_rows(height, band, n, 0) * width   # member 0's rays per launch
    t_step = dt / args.steps
    value = width * height / t_step / 1e6
    achieved = BYTES_PER_RAY * rays0 / (trace_ms * 1e-3) / 1e9
    gather_bytes = sum(sf.lib().sf_slab_rows(height, band, n, k) for k in range(1, n)) * width * BYTES_PER_RAY
    same_dev = len(set(devices)) < n
    g.close()
    out = {
        "metric": "Mrays/sec into G-buffer at 1920x1080 depth-8; frame time ms",
        "value": round(value, 2), "unit": "Mrays/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (deterministic camera path: config camera, yaw swept +-10 mrad at 1 mrad per frame; "
                "no dataset)",
        "config": {"workload": f"{width}x{height} primary-ray G-buffer, camera K={args.K:g}, one frame per step "
                               f"cut into {band}-row bands over {n} members, moving camera",
                   "width": width, "height": height, "K": args.K, "max_depth": st.max_depth, "camera": "moving",
                   "devices": devices,
                   "parallelism": f"row-bands x{n} (sf_group: strided peer copies into device 0)"
                                  + (" [rehearsal: all members on device 0]" if same_dev else "")},
        "frame_ms": round(t_step * 1e3, 4),
        "first_render_ms": round(first_ms, 4),
        "gather_bytes_per_frame": gather_bytes,
        "rays_per_step": width * height, "rays_counted": int(st.rays),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": TRACE_KERNEL,
                     "kernel_ms": round(trace_ms, 4),
                     "note": "member 0's trace kernel over its bands (32 B/ray x its rays / HIP-event duration)"},
    }
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    dist_on = world > 1
    # SF_BENCH_BACKEND=gloo + local ranks folded onto the visible devices: rehearses the multi-rank
    # flow on a 1-GPU box (RCCL refuses two ranks on one GPU). The driver's runs use nccl (= RCCL).
    backend = os.environ.get("SF_BENCH_BACKEND", "nccl")
    gpu = local % max(1, torch.cuda.device_count()) if dist_on else 0
    torch.cuda.set_device(gpu)
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    if not os.path.exists(sf.LIB_PATH):
        if rank == 0:
            sf.build()
        if dist_on:
            dist.barrier()
    width, height = args.width, args.height
    n = world
    stream = torch.cuda.Stream(device=dev)
    kernel = sf.SF_KERNEL_WAVE if args.kernel == "wave" else sf.SF_KERNEL_PER_RAY

    # a tiny render on a throw-away context first: loads the code object, so that `first_render_ms`
    # below is the first render of a fresh context, not the process's first kernel launch
    t_load = time.perf_counter()
    with sf.Sphereflake(64, 64, device=dev.index) as warm:
        warm.SetCamera(sf.config_camera(64, 64, args.K))
        warm.Render()
        warm.Synchronize()
    module_load_ms = (time.perf_counter() - t_load) * 1e3
    ctx = sf.Sphereflake(width, height, device=dev.index)
    sh = stream.cuda_stream

    if args.mode == "rows":
        run_rows(args, torch, dist, dist_on, rank, max(n, args.gpus), kernel)   # N devices, one driving process
        ctx.close()
        if dist_on:
            dist.destroy_process_group()
        return
    if args.mode == "frames":
        # frame index = step * N + rank along the camera path (warmup, timed loop)
        views = [frame_camera(width, height, args.K, i * n + rank).corners() for i in range(args.warmup + args.steps)]
        rays_per_step_rank = width * height
        slab_rows = height
    else:
        cam = sf.config_camera(width, height, args.K)
        ctx.SetCamera(cam)
        slab_rows = sf.lib().sf_slab_rows(height, args.band_rows, n, rank)
        rays_per_step_rank = slab_rows * width
        slab_p = torch.empty((slab_rows, width, 4), dtype=torch.float32, device=dev)
        slab_n = torch.empty_like(slab_p)
        max_rows = shard.max_slab_rows(height, args.band_rows, n)
        send_p = torch.zeros((max_rows, width, 4), dtype=torch.float32, device=dev)
        send_n = torch.zeros_like(send_p)

    first_ms = None
    if args.mode == "frames":
        ctx.SetView(*views[0])
        # the first render of a fresh context: row-major tile order, no cost history
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record(stream)
            ctx.Render(kernel=kernel, stream=sh)
            e1.record(stream)
        torch.cuda.synchronize(dev)
        first_ms = e0.elapsed_time(e1)
    # HIP events around the dominant (trace) kernel of every KTIMING_PERIOD-th render: an event pair
    # costs ~7 us of stream time per frame, so it is sampled (SF_BENCH_KTIMING=0: off, for A/B)
    ktiming = os.environ.get("SF_BENCH_KTIMING", "1") != "0"
    kp = ktiming_period(args.steps)

    ev_s = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_e = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    # whole-render events (kernel_ms) on the same sampled steps as the trace-kernel events: every
    # event record on the stream costs GPU time between kernels (measured ~7 us per pair per frame)
    def run_step(i, timed, view=None):
        timed = timed and ktiming and i % kp == 0
        with torch.cuda.stream(stream):
            if timed:
                ev_s[i].record(stream)
            if args.mode == "frames":
                if view is not None:
                    ctx.SetView(*view)
                ctx.Render(kernel=kernel, stream=sh)
            else:
                ctx.render_to(slab_p.data_ptr(), slab_n.data_ptr(), band_rows=args.band_rows, band_count=n,
                              band_index=rank, compact=True, kernel=kernel, stream=sh)
            if timed:
                ev_e[i].record(stream)
            if args.mode == "rows-rccl" and dist_on:
                send_p[:slab_rows].copy_(slab_p)
                send_n[:slab_rows].copy_(slab_n)
                if backend == "nccl":
                    shard.gather_frame(send_p, height, args.band_rows)   # RCCL gather + reassembly on rank 0
                    shard.gather_frame(send_n, height, args.band_rows)
                else:   # gloo rehearsal: host tensors
                    shard.gather_frame(send_p.cpu(), height, args.band_rows)
                    shard.gather_frame(send_n.cpu(), height, args.band_rows)

    moving = args.mode == "frames"
    for i in range(args.warmup):
        run_step(i, False, views[i] if moving else None)
    ctx.kernel_timing(ktiming, period=kp)   # samples timed renders 0, kp, 2 kp, ...
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        run_step(i, True, views[args.warmup + i] if moving else None)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    st = ctx.stats()
    if st.overflow_tiles:
        raise RuntimeError("traversal overflowed SF_MAX_DEPTH_LIMIT")
    kern_ms = (float(np.mean([ev_s[i].elapsed_time(ev_e[i]) for i in range(0, args.steps, kp)]))
               if ktiming else dt / args.steps * 1e3)   # whole render, sampled
    nks = min(-(-args.steps // kp), 64)
    tk = ctx.kernel_timing(n=nks) if ktiming else []   # the trace kernel alone, last timed renders
    clk = ctx.kernel_clocks(n=nks) if ktiming else []  # live shader clock of the same renders
    trace_ms = float(np.mean(tk)) if len(tk) else kern_ms

    # the same loop on one unchanging view (the config camera, frame 0 of the path): extra key, never `value`
    fixed = None
    if moving:
        ctx.kernel_timing(False)
        ctx.SetView(*views[0])
        for i in range(args.warmup):
            run_step(i, False)
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier()
        tf = time.perf_counter()
        for i in range(args.steps):
            run_step(i, False)
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier()
        t_fixed = (time.perf_counter() - tf) / args.steps
        if dist_on:
            tt = torch.tensor([t_fixed], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t_fixed = float(tt[0])
        fixed = {"value": round(n * width * height / t_fixed / 1e6, 2), "frame_ms": round(t_fixed * 1e3, 4),
                 "note": "same timed loop on the unchanging config view (heavy-first order from identical frames)"}

    t_step = dt / args.steps
    if dist_on:
        tt = torch.tensor([t_step, kern_ms, trace_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step, kern_ms_max, trace_ms = float(tt[0]), float(tt[1]), float(tt[2])
    else:
        kern_ms_max = kern_ms
    total_rays = rays_per_step_rank * n if args.mode == "frames" else width * height
    value = total_rays / t_step / 1e6

    # SSAO post-process of the rendered G-buffer, timed alone on the render stream
    post = None
    if rank == 0 and args.mode == "frames" and not args.no_extras:
        post = post_rates(ctx, torch, stream, width, height)

    # D2H into the host GBuffer (PCIe-inclusive, reported separately -- never `value`)
    d2h = None
    if rank == 0 and args.mode == "frames" and not args.no_extras:
        d2h = transfer_rates(ctx, torch, dev, stream, width, height, kernel)
    prog = None
    if rank == 0 and args.mode == "frames" and not args.no_extras:
        prog = progressive_rates(width, height, args.K)

    check = None
    if args.check and rank == 0 and args.mode == "frames":
        from oracle import pyoracle
        pos, nrm, _, _ = ctx.download()
        o, tl, tr, bl = views[0]
        setup = {"W": width, "H": height, "origin": o, "tl": tl, "tr": tr, "bl": bl,
                 "root": sf.root_transform(o), "children": sf.child_transforms()}
        rows = np.linspace(0, height - 1, 12).astype(int)
        r = pyoracle.render(setup, rows=rows)
        check = bool(np.array_equal(r["pos4"].view(np.uint32), pos[rows].view(np.uint32)) and
                     np.array_equal(r["nrm4"].view(np.uint32), nrm[rows].view(np.uint32)))

    if rank == 0:
        per_launch_bytes = BYTES_PER_RAY * rays_per_step_rank
        achieved = per_launch_bytes / (trace_ms * 1e-3) / 1e9
        camera = "moving" if moving else "fixed"
        build = sf.build_info()
        pmc, _ = load_pmc(TRACE_KERNEL, pmc_config_key(width, height, args.K, camera), build)
        traffic = pmc_traffic(pmc)
        cfg_name = BASELINE_CONFIGS.get((width, height, round(args.K, 4)))
        out = {
            "metric": "Mrays/sec into G-buffer at 1920x1080 depth-8; frame time ms",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "frames" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic camera path: config camera, yaw swept +-10 mrad at 1 mrad per frame; "
                    "no dataset)"
                    if moving else "synthetic (deterministic fixed-camera frames; no dataset)",
            "config": {"workload": f"{width}x{height} primary-ray G-buffer, camera K={args.K:g} (reference max "
                                   f"depth {st.max_depth})"
                                   + (f", BASELINE {cfg_name}" if cfg_name else "")
                                   + f", {camera} camera, {args.kernel} kernel",
                       "width": width, "height": height, "K": args.K, "max_depth": st.max_depth, "camera": camera,
                       "parallelism": f"frames x{n}" if args.mode == "frames" else f"row-bands x{n} + RCCL gather (per rank)"},
            "frame_ms": round(t_step * 1e3, 4),
            "kernel_ms": round(kern_ms_max, 4),
            "first_render_ms": round(first_ms, 4) if first_ms is not None else None,
            "process_first_launch_ms": round(module_load_ms, 3),
            "fixed_camera": fixed,
            "post": post,
            "d2h": d2h,
            "frameless": prog,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": round(traffic) if traffic else None,
                         "kernel": TRACE_KERNEL, "kernel_ms": round(trace_ms, 4), "kernel_samples": len(tk),
                         "clock_mhz_live": round(float(np.median(clk)), 1) if len(clk) else None,
                         "note": "path is VALU/latency-bound (SURVEY.md §8(d), see `valu`); achieved = 32 B/ray x "
                                 "rays per launch / mean duration of the trace kernel (HIP events around it on its "
                                 "launch stream); traffic = PMC WRITE_SIZE + 2 x FETCH_SIZE per launch "
                                 "(profiles/pmc_traffic.json, only when profiled on this config, else null)"},
            "valu": pmc_valu(pmc),
            "build": build,
        }
        if check is not None:
            out["check_rows_bit_exact"] = check
        if not args.no_cpu_baseline and n == 1:
            avail, quota = cpu_share()
            thr = args.cpu_threads or (min(avail, quota) if quota else avail)
            try:
                cb = cpu_baseline(width, height, args.K, thr)
                if "value" in cb and cb["value"] > 0:
                    cb["gpu_cpu_ratio"] = round(value / cb["value"], 1)
                    if cb.get("kind") == "reference":
                        # linear extrapolation of the measured share to every host core (an estimate,
                        # labelled as such: SMT and memory bandwidth make it optimistic for the CPU)
                        allc = cb["value"] * (os.cpu_count() or thr) / thr
                        cb["all_host_cores_estimate"] = {"value": round(allc, 1), "gpu_cpu_ratio": round(value / allc, 1),
                                                         "note": "measured value x host_cores / cores (linear)"}
                out["cpu_baseline"] = cb
            except Exception as e:  # never lose the GPU number over the baseline leg
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
