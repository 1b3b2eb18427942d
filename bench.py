#!/usr/bin/env python3
"""Benchmark: Mrays/s into the G-buffer at 1920x1080 depth 8 (BASELINE.json metric), MI355X.

A "step" is one full deterministic frame of the hot path (ray generation + sphereflake traversal +
G-buffer write, reference Sphereflake.h:86-226 / Sphereflake.cpp:149-201) over a 1920x1080 frame at
the depth-8 camera (BASELINE configs[2]: main.cpp:92-96 camera position scaled by K = 0.25). The
G-buffer stays resident in HBM (the D2H copy into the host GBuffer is timed separately and reported
as `d2h`, never as `value`).

The camera MOVES: step i renders frame i of a camera path (the config camera with its yaw swept +-10 mrad
around the config view at 1 mrad per frame, `frame_camera`), so the heavy-first tile schedule always works
from the costs of a different view (the reference is an interactive app whose view changes every frame,
main.cpp:304). `first_render_ms` is the first render of a fresh context (row-major tile order, no previous
costs); `fixed_camera` repeats the timed loop on one unchanging view; `frame_latency_ms` is one frame
rendered and waited for alone.

Default mode `dist` (sf_dist_*, csrc/sf_dist.hip): `--slots` frames in flight (frame i on slot i % slots, each
slot its own context, stream and G-buffer; default 3, or 4 for a rank's share that leaves most of the persistent
grid idle -- frames_in_flight), so a frame's persistent trace grid fills the wave slots the previous frame's
heaviest tiles leave idle -- the reference's workers likewise trace continuously. Multi-GPU (`--gpus N`,
launched by torch.distributed.run, one process per GPU): ONE frame per step split over the N GPUs in interleaved
8-row bands, every rank tracing its bands into its own HBM -- the frame's G-buffer distributed over the GPUs,
`scaling: "strong"` (the frame is fixed, N GPUs share it): `value`. `gathered_on_rank0` times the same frames
assembled on rank 0 (ranks k > 0 send packed slabs, 4 or 16 B/pixel, over RCCL/xGMI; rank 0 unpacks them beside its
own bands): what a consumer on rank 0 sees, a transfer bound by the links into rank 0, reported beside `value`
as the D2H copy is. torch.distributed (gloo) is only the control plane: the RCCL ids, barriers and the max over
ranks of the timed region. `independent_frames` adds the weak-scaling figure (every rank its own frames).
`--mode frames` is that weak-scaling loop alone; `--mode rows` one frame over N devices from ONE process
(sf_group_*: strided peer copies).

rank 0 prints ONE JSON line. `roofline` prices the dominant kernel against HBM (32 B/ray of G-buffer
stores); `cpu_baseline` times the reference's own AVX packet path (oracle/_ref,
compiled from the reference sources) on this host's cores. `configs.c4` is BASELINE configs[3]
(3840x2160, K = 0.22, depth 9) on the same path.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import subprocess
import sys
import time

# Hardware queues per process (the HIP runtime's GPU_MAX_HW_QUEUES, default 4). Every frame in flight has a stream of
# its own; with plain streams on 4 queues, streams share them and one slot's kernel waits in order behind another's
# (round 6: a 1080p member's share over 8 GPUs at 8 frames in flight 0.0146 ms with 4 queues, 0.0121 with 16,
# profiles/r6/multi/queues.txt). Since the library gives each context's stream a queue of its own (sf_capi.hip,
# SF_STREAM_CUMASK), the slots no longer depend on this (0.0110-0.0112 ms at 4 or 16, profiles/r6/multi/queue_reuse/);
# it still serves the other streams of the process. Raised to 16 before the HIP runtime starts (its first call); a
# larger value already in the environment is kept.
HW_QUEUES = int(os.environ.get("SF_HW_QUEUES", "16") or 0)   # (SF_HW_QUEUES=0: leave the runtime's setting, A/B)
if HW_QUEUES > 0 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)

import sphereflake_amd as sf  # noqa: E402
from sphereflake_amd import shard  # noqa: E402

W, H, K = 1920, 1080, 0.25          # BASELINE configs[2]
BYTES_PER_RAY = 32                  # two float4 G-buffer stores
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
TRACE_KERNEL = "sf_trace_queue1"    # the dominant kernel (persistent wave-coherent trace, 1 wave per workgroup)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--settle-ms", type=float, default=SETTLE_MS,
                    help="untimed frames beyond --warmup until the GPU has been under load this long (0: off)")
    ap.add_argument("--mode", choices=["dist", "frames", "rows"], default="dist")
    ap.add_argument("--slots", type=int, default=DEFAULT_SLOTS, help="frames in flight (dist mode)")
    ap.add_argument("--batch", type=int, default=-1,
                    help="frames per multi-frame persistent launch (sf_render_frames; 1: one launch per frame; "
                         "-1: by the share, frames_per_launch)")
    ap.add_argument("--kernel", choices=["wave", "ray"], default="wave")
    ap.add_argument("--width", type=int, default=W)
    ap.add_argument("--height", type=int, default=H)
    ap.add_argument("--K", type=float, default=K)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the post-process, transfer, frame-less and c4 sections (profiling runs of the timed loop only)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-check", action="store_true",
                    help="skip the parity check of the timed frames (default: the last moving frame's oracle rows "
                         "and the fixed-camera frame's row digests against the golden fixture; a mismatch exits 5)")
    ap.add_argument("--launch-check", action="store_true",
                    help="bring the ranks up (spawning them for --gpus N > 1), agree on the world, report each rank's "
                         "device, and print the line without rendering (no GPU call: runs on a CPU-only host)")
    ap.add_argument("--long-steps", type=int, default=0,
                    help="frames of the second timed loop that measures the steady frame period and the pipeline fill "
                         "(0: max(4 x --steps, 200))")
    ap.add_argument("--rehearse", action="store_true",
                    help="dist mode with more ranks than GPUs (ranks share devices): every leg but the RCCL gather, "
                         "which RCCL refuses on a shared device")
    ap.add_argument("--gather-timeout", type=float, default=GATHER_TIMEOUT_S,
                    help="seconds the RCCL-gathered leg may take before the line is printed without it")
    return ap.parse_args()


DEFAULT_SLOTS = 0                    # frames in flight: 0 = by the share's tiles (frames_in_flight)
SLOTS_FULL, SLOTS_SHARE = 3, 4       # 1080p: 3 in flight 0.0751 ms steady, 4 0.0792 (the frame fills the grid);
                                     # a member's share over 8 GPUs: 3 0.0194 ms, 4 0.0156-0.0160, 5 0.0174-0.0232,
                                     # 6 0.020 (the process's 4 hardware queues); over 4: 0.0247 / 0.0235; over 2:
                                     # 0.0452 / 0.0459 (profiles/r4/slots/)
SHARE_GRID_FRAC = 1.5                # a share of at most this many persistent-grid waves' worth of tiles takes 4
SLOTS_TINY, TINY_GRID_FRAC = 8, 0.75  # round 6, with 16 hardware queues (HW_QUEUES): a share of at most 3/4 of the grid's
                                     # waves (every tile a wave of its own, the frame bound by its heaviest tiles' traversal)
                                     # takes 8 -- 1080p over 8 GPUs 0.0143-0.0146 -> 0.0121 ms; over 4, 4 stays best (0.0193
                                     # vs 0.0198-0.0199 at 6-8), whole frames 3 (profiles/r6/multi/queues.txt)
GRID_WAVES_PER_CU = 32               # the trace kernel's grid: 4 SIMDs x 8 waves per CU (LDS-limited occupancy)


BATCH_FULL, BATCH_SHARE = 1, 1       # frames per launch (frames_per_launch): one launch per frame -- multi-frame launches
                                     # measured slower at 1080p and for a 1/4 share (profiles/r6/frames/README.md)
BATCH_TINY = 1                       # (round 6: launches of 8 frames for a 1080p share over 8 GPUs, two in flight on 16
                                     # queues, reach 0.0100-0.0103 ms per frame in most loops but 0.019-0.025 in others --
                                     # alternating reps in one process, every rep in another -- against a stable 0.0110-0.0123
                                     # for one launch per frame at 8 in flight: not the default, profiles/r6/frames/README.md)
GROUPS_IN_FLIGHT = 2                 # multi-frame launches in flight: slots = batch x this


def frames_per_launch(requested, cus, width, height, band_rows, n):
    """Frames per multi-frame persistent launch for a loop whose rank renders rank 0's bands of an n-way split."""
    if requested >= 1:
        return min(8, requested)
    rows = sf.lib().sf_slab_rows(height, band_rows, n, 0) if n > 1 else height
    tiles = -(-width // 8) * -(-rows // 8)
    if BATCH_TINY > 1 and n > 1 and tiles <= TINY_GRID_FRAC * GRID_WAVES_PER_CU * cus \
            and int(os.environ.get("GPU_MAX_HW_QUEUES", 4)) >= BATCH_TINY * GROUPS_IN_FLIGHT:
        return BATCH_TINY
    return BATCH_SHARE if tiles <= SHARE_GRID_FRAC * GRID_WAVES_PER_CU * cus else BATCH_FULL


def frames_in_flight(requested, cus, width, height, band_rows, n, batch=1):
    """Frames in flight for a loop whose rank renders rank 0's bands of an n-way split (n = 1: whole frames).
    A share that leaves most of the persistent grid's wave slots idle is bounded by the per-frame chain
    (trace, order, host enqueue: ~55-60 us for a 1080p share over 8) over the frames that overlap, so it takes
    one frame more; frames that fill the grid are throughput-bound and a 4th frame only adds contention."""
    if requested:
        return max(batch, min(16, requested))
    if batch > 1:
        return batch * GROUPS_IN_FLIGHT
    rows = sf.lib().sf_slab_rows(height, band_rows, n, 0) if n > 1 else height
    tiles = -(-width // 8) * -(-rows // 8)
    own_queues = os.environ.get("SF_STREAM_CUMASK", "1") != "0"   # (the library's default: a queue per slot stream)
    if n > 1 and tiles <= TINY_GRID_FRAC * GRID_WAVES_PER_CU * cus \
            and (own_queues or int(os.environ.get("GPU_MAX_HW_QUEUES", 4)) >= SLOTS_TINY):
        return SLOTS_TINY   # (band shares only: a whole 640x360 frame measured 0.0186-0.0189 ms at 8 vs 0.0172 at 4)
    return SLOTS_SHARE if tiles <= SHARE_GRID_FRAC * GRID_WAVES_PER_CU * cus else SLOTS_FULL


GATHER_TIMEOUT_S = 180.0             # the RCCL-gathered leg (multi-GPU) runs last, under a watchdog

ENQ_TRACE = os.environ.get("SF_BENCH_ENQ_TRACE") == "1"   # diagnostics: per-frame enqueue times in the line
LONG_SETTLE_MS = 30.0               # before the steady-period loop (the GPU was idle only for the timed loop's readouts)
SETTLE_MS = 150.0                    # the shader clock ramps from ~2075 to ~2370 MHz over the first ~60 ms of load
                                     # (profiles/r3/ramp.txt): warm-up lasts at least this long. (Under sustained load
                                     # the chip may then give clock back -- 2134-2380 MHz across round-4 boxes and
                                     # settle lengths, profiles/r4/final: the line reports the live clock.)


class FrameIssuer:
    """Issues the frames of a loop on a dist: `batch` 1 -- SetView + one render call (one trace launch) per frame;
    `batch` B > 1 -- B frames of the camera path per multi-frame persistent launch (RenderBandsFrames, round 6):
    every frame is still its own view rendered into its own slot G-buffer, B per launch. `issue(rows)` renders the
    frames whose views are the rows of an n x 12 float32 array (made before any timed region: the camera path is
    precomputed either way); `view_rows` turns (origin, tl, tr, bl) tuples into that array."""

    def __init__(self, d, render, batch):
        self.d, self.render, self.batch = d, render, max(1, int(batch))

    @staticmethod
    def view_rows(views):
        return np.ascontiguousarray(np.array([[c for v in view for c in v] for view in views], np.float32).reshape(-1, 12))

    def issue(self, rows):
        d, b = self.d, self.batch
        if b == 1:
            for v in rows:
                d.SetView(v[0:3], v[3:6], v[6:9], v[9:12])
                self.render()
            return
        for i in range(0, len(rows), b):
            d.RenderBandsFrames(rows[i:i + b])


def settle(d, render, views, n_views, t_start, ms, issuer=None):
    """Untimed frames (cycling views[:n_views]) until `ms` have passed since t_start with the GPU under load;
    returns the number of extra frames."""
    k = 0
    d.Synchronize()
    rows = FrameIssuer.view_rows(views[:n_views]) if issuer is not None else None
    while (time.perf_counter() - t_start) * 1e3 < ms:
        if issuer is not None:
            issuer.issue(rows[np.arange(k, k + 20) % n_views])
            k += 20
        else:
            for _ in range(20):
                d.SetView(*views[k % n_views])
                render()
                k += 1
        d.Synchronize()
    return k


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
    """Every k-th timed render carries the kernel-timing events: k = 10 (sampled, to keep them off the frame
    period), or less when that would give fewer than KTIMING_MIN_SAMPLES samples. (Round 5: the driver's 20-step
    line measured the same with 11 or 5 samples, profiles/r5/order/kt_samples_ab.txt.)"""
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


def pmc_valu(c, frame_ms, clock_mhz, cus=256):
    """Issue of the trace kernel on the FRAME PERIOD: the committed PMC summary's wave-level instructions per launch
    (one launch = one frame) against the issue slots of one frame period at the live shader clock -- VALU: CUs x 4
    SIMDs x cycles / 2 (one wave64 VALU instruction issues over 2 cycles), SALU: one scalar instruction per CU per
    cycle. `lone_dispatch` keeps the PMC pass's own view: the passes serialise dispatches, so there one launch runs
    alone; its cycles are its profiled duration x the live shader clock of the bench's own renders (`clock_mhz`,
    from the kernel's s_memtime / s_memrealtime probe). (Round 4 divided GRBM_GUI_ACTIVE / 8 by the duration, which
    counts GPU-busy cycles outside the kernel and read 2521 MHz, above the gfx950 maximum of 2400.)"""
    if c is None:
        return None
    try:
        out = {"valu_insts": round(c["SQ_INSTS_VALU"]), "salu_insts": round(c["SQ_INSTS_SALU"]),
               "source": "profiles/pmc_traffic.json"}
        if frame_ms and clock_mhz:
            fcyc = frame_ms * 1e-3 * clock_mhz * 1e6
            out["frame_cycles"] = round(fcyc)
            out["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] / (cus * 4 * fcyc / 2.0), 4)
            out["salu_issue_frac"] = round(c["SQ_INSTS_SALU"] / (cus * fcyc), 4)
            out["basis"] = "per launch / issue slots of one frame period (ms_per_step) at clock_mhz_live"
        if not clock_mhz:
            return out
        cycles = c["profiled_dispatch_us"] * clock_mhz
        # wavefront occupancy: SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md), summed over the
        # chip -> mean resident waves; against the gfx950 peak of 8 waves per SIMD
        waves = 4.0 * c["SQ_WAVE_CYCLES"] / cycles
        peak_waves = cus * 4 * 8
        lone = {"dispatch_us": round(c["profiled_dispatch_us"], 2), "clock_mhz": round(clock_mhz, 1),
                "clock_basis": "clock_mhz_live of the bench's renders (the kernel's own clock probe)",
                "valu_issue_frac": round(c["SQ_INSTS_VALU"] / (cus * 4 * cycles / 2.0), 4),
                "salu_issue_frac": round(c["SQ_INSTS_SALU"] / (cus * cycles), 4),
                "occupancy": {"mean_waves": round(waves, 1), "peak_waves": peak_waves, "frac": round(waves / peak_waves, 4)}}
        if "SQ_WAIT_INST_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            lone["wait_inst_frac"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
            lone["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        out["lone_dispatch"] = lone
        return out
    except (KeyError, ValueError, ZeroDivisionError, TypeError):
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


def cpu_model(text=None):
    """(model name, vendor) of the host CPU from /proc/cpuinfo (state the CPU model) -- the
    first "model name" and "vendor_id" lines; None where absent (e.g. a non-x86 kernel's format)."""
    if text is None:
        try:
            with open("/proc/cpuinfo") as f:
                text = f.read()
        except OSError:
            return None, None
    model = vendor = None
    for line in text.splitlines():
        key, _, val = line.partition(":")
        key = key.strip()
        if key == "model name" and model is None:
            model = " ".join(val.split())
        elif key == "vendor_id" and vendor is None:
            vendor = val.strip()
        if model is not None and vendor is not None:
            break
    return model, vendor


def cpu_identity():
    """cpu_model / vendor keys of the baseline, with the parity caveat where the host is not Intel: the oracle's
    rsqrtps table was measured on Intel, AMD's rsqrtps returns other estimates, so the reference
    build's frames on such a host differ from the fixtures and its baseline there is timing-only."""
    model, vendor = cpu_model()
    out = {"cpu_model": model, "vendor": vendor}
    if vendor != "GenuineIntel":
        out["note"] = ("timing-only: not an Intel host, and x86 rsqrtps estimates differ by vendor (the fixtures "
                       "and the GPU path follow the Intel table, SURVEY.md §8(c)); parity is GPU vs committed fixtures")
    return out


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
                                  "sample": "3 full frames, 1 thread"}, **cpu_identity()}
    setup = {"W": width, "H": height}
    cam = sf.config_camera(width, height, k)
    o, tl, tr, bl = cam.corners()
    setup.update(origin=o, tl=tl, tr=tr, bl=bl, root=sf.root_transform(o), children=sf.child_transforms())
    rows = np.arange(0, height, 8)
    t0 = time.perf_counter()
    pyoracle.render(setup, rows=rows, threads=1)
    dt = time.perf_counter() - t0
    return {"value": round(len(rows) * width / dt / 1e6, 3), "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"every 8th row of a {width}x{height} K={k} frame, oracle C restatement, 1 thread",
            **cpu_identity()}


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


def progressive_rates(width, height, k, batch=1 << 18, reps=40, settle_ms=SETTLE_MS):
    """the frame-less mode (the reference's Initialize() worker stream: mt19937 draws,
    Sobol pixel picks, 8-ray AVX / 4-ray SSE packets with packet early-outs, last-writer scatter) on a
    fresh context with the same camera, in batches of `batch` packets continuing one stream. Untimed batches
    first, for at least `settle_ms` of load: the steady state of a running loop (the adaptive LDS levels follow
    the depth the finished batches reached, the next batch's draws and bins are prefetched) at the steady shader
    clock -- this leg follows the PCIe-bound transfer legs, after which the clock has dropped and ramps back over
    ~60 ms of load (profiles/r3/ramp.txt), longer than a few timed batches."""
    out = {"batch_packets": batch, "batches_timed": reps, "settle_ms": settle_ms}
    with sf.Sphereflake(width, height) as s:
        s.SetCamera(sf.config_camera(width, height, k))
        for variant, lanes in (("avx", 8), ("sse", 4)):
            s.SetVariant(variant)
            s.Progressive(12345, batch, 0)
            s.Synchronize()
            t_w = time.perf_counter()
            while (time.perf_counter() - t_w) * 1e3 < settle_ms:
                for _ in range(8):
                    s.Progressive(12345, batch)
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


def run_rows(args, torch, ctl, n, kernel):
    """--mode rows: ONE frame per step over N devices from ONE process (sf_group_*): member k traces the
    8-row bands b = k (mod N); members k > 0 ship theirs into member 0's G-buffer with strided peer copies.
    The camera moves as in the default mode. When fewer than N devices are visible (a one-GPU rehearsal) the
    members are N contexts on device 0, and the line says so. The other ranks only join the barriers."""
    width, height, band = args.width, args.height, args.band_rows
    visible = torch.cuda.device_count()
    devices = list(range(n)) if visible >= n else [0] * n
    views = [frame_camera(width, height, args.K, i).corners() for i in range(args.warmup + args.steps)]
    g = None
    kp = ktiming_period(args.steps)
    if ctl.rank == 0:
        g = sf.SphereflakeGroup(devices, width, height)
        if kernel != sf.SF_KERNEL_WAVE:
            raise SystemExit("--mode rows traces with the wave kernel")
        g.SetView(*views[0])
        t = time.perf_counter()
        g.Render(band)
        g.Synchronize()
        first_ms = (time.perf_counter() - t) * 1e3
        t_w = time.perf_counter()
        for i in range(args.warmup):
            g.SetView(*views[i])
            g.Render(band)
        settle(g, lambda: g.Render(band), views, max(1, args.warmup), t_w, args.settle_ms)
        g.member_kernel_timing(0, True, period=kp)
        g.Synchronize()
        g.reset_stats()
    ctl.barrier()
    t0 = time.perf_counter()
    if ctl.rank == 0:
        for i in range(args.steps):
            g.SetView(*views[args.warmup + i])
            g.Render(band)
        g.Synchronize()
    ctl.barrier()
    dt = time.perf_counter() - t0
    if ctl.rank != 0:
        return
    st = g.stats()
    if st.overflow_tiles:
        raise RuntimeError("traversal overflowed SF_MAX_DEPTH_LIMIT")
    tk = g.member_kernel_timing(0, n=min(-(-args.steps // kp), 64))
    trace_ms = float(np.mean(tk)) if len(tk) else dt / args.steps * 1e3
    t_step = dt / args.steps
    # member 0's G-buffer receives the whole frame (32 B/pixel) every frame period
    achieved = BYTES_PER_RAY * width * height / t_step / 1e9
    slab_bytes = g.slab_bytes()
    gather_bytes = sum(sf.lib().sf_slab_rows(height, band, n, k) for k in range(1, n)) * width * slab_bytes
    same_dev = len(set(devices)) < n
    g.close()
    out = {
        "metric": METRIC, "value": round(width * height / t_step / 1e6, 2), "unit": "Mrays/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": DATA_MOVING,
        "config": {"workload": f"{width}x{height} primary-ray G-buffer, camera K={args.K:g}, one frame per step "
                               f"cut into {band}-row bands over {n} members, moving camera",
                   "width": width, "height": height, "K": args.K, "max_depth": st.max_depth, "camera": "moving",
                   "devices": devices,
                   "parallelism": f"row-bands x{n} (sf_group: one process, strided peer copies into device 0)"
                                  + (" [rehearsal: all members on device 0]" if same_dev else "")},
        "frame_ms": round(t_step * 1e3, 4), "first_render_ms": round(first_ms, 4),
        "gather_bytes_per_frame": gather_bytes, "slab_bytes_per_pixel": slab_bytes,
        "rays_per_step": width * height, "rays_counted": int(st.rays),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": TRACE_KERNEL,
                     "kernel_event_ms": round(trace_ms, 4),
                     "basis": "member 0's G-buffer receives the frame (32 B/pixel) per frame period; kernel_event_ms = "
                              "member 0's trace kernel over its own bands (HIP events)"},
    }
    print(json.dumps(out), flush=True)


METRIC = "Mrays/sec into G-buffer at 1920x1080 depth-8; frame time ms"
DATA_MOVING = ("synthetic (deterministic camera path: config camera, yaw swept +-10 mrad at 1 mrad per frame; "
               "no dataset)")


class Control:
    """Control plane of a multi-rank run: torch.distributed over gloo (barriers, the RCCL ids, the max over
    ranks of the timed region). The frame data never goes through it: the gather is RCCL inside sf_dist."""

    def __init__(self, world, rank):
        self.world, self.rank = world, rank
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def combine_stats(self, st):
        """This rank's sf_stats combined over the ranks in place (max depth max, closest min, rays and overflow
        tiles summed) -- for a distributed G-buffer made without RCCL communicators."""
        if not self.dist:
            return st
        import torch
        t = torch.tensor([float(st.max_depth), -float(st.closest)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        u = torch.tensor([int(st.rays), int(st.overflow_tiles)], dtype=torch.int64)
        self.dist.all_reduce(u, op=self.dist.ReduceOp.SUM)
        st.max_depth, st.closest = int(t[0]), float(-t[1])
        st.rays, st.overflow_tiles = int(u[0]), int(u[1])
        return st

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


EXIT_GATHER_FAILED = 3              # the RCCL-gathered leg failed or hung (the line is printed first)
EXIT_CHECK_FAILED = 5               # a timed frame differs from the oracle / golden rows (the line is printed first)


class Watchdog:
    """Deadline for a leg that may hang (the RCCL gather on a node never seen before): past it, `on_timeout`
    runs (rank 0 prints the line with the leg marked as failed) and the process exits EXIT_GATHER_FAILED -- every
    rank arms the same deadline, so no rank is left waiting in a collective, and a hang is never a success."""

    def __init__(self, seconds, on_timeout):
        import threading
        self._done = threading.Event()
        self._fire = on_timeout
        self._t = threading.Thread(target=self._run, args=(seconds,), daemon=True)
        self._t.start()

    def _run(self, seconds):
        if not self._done.wait(seconds):
            try:
                self._fire()
            finally:
                sys.stdout.flush()
                os._exit(EXIT_GATHER_FAILED)

    def cancel(self):
        self._done.set()


def slot_period(steps, slots):
    """Kernel-timing period per slot so that every slot gives >= ceil(KTIMING_MIN_SAMPLES / slots) samples."""
    per_slot = max(1, steps // slots)
    need = -(-KTIMING_MIN_SAMPLES // slots)
    return max(1, min(KTIMING_PERIOD, per_slot // need))


PATH_PERIOD = 4 * PATH_AMPLITUDE     # the camera path repeats every 40 frames


def path_views(width, height, k, frame_of):
    """view_at(i) -> the corners of frame frame_of(i) of the camera path (40 distinct views, cached)."""
    cache = [frame_camera(width, height, k, f).corners() for f in range(PATH_PERIOD)]
    return lambda i: cache[frame_of(i) % PATH_PERIOD]


GOLDEN_OF = {(640, 360, 1.0): "c1", (1280, 720, 0.8): "c2", (1920, 1080, 0.25): "c3", (3840, 2160, 0.22): "c4",
             (16384, 16384, 0.2): "c5"}


def golden_frame(width, height, k):
    """The golden fixture of a BASELINE config (tests/golden/frame_c*.json: per-row SHA-256 digests of the reference
    frame, made by tests/golden/make_golden.py from the reference build), or None for other sizes."""
    name = GOLDEN_OF.get((width, height, round(k, 4)))
    if not name:
        return None
    with open(os.path.join(REPO, "tests", "golden", f"frame_{name}.json")) as f:
        return json.load(f)


def row_digest(pos, nrm, y):
    """Digest of one G-buffer row, as tests/sfcheck.py and make_golden.py define it."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(pos[y]).tobytes() + np.ascontiguousarray(nrm[y]).tobytes()).hexdigest()[:16]


def owned_rows(height, band_rows, nranks, rank):
    """Frame rows this rank's G-buffer holds (all of them on one rank)."""
    if nranks <= 1:
        return np.arange(height)
    return np.array([y for y0, y1 in shard.owned_bands(height, band_rows, nranks, rank) for y in range(y0, y1)], int)


def check_oracle_rows(pos, nrm, view, width, height, rows):
    """Rows `rows` of a downloaded frame against the oracle restatement (the checker, outside any timed region):
    True when position and normal are equal bit for bit."""
    from oracle import pyoracle
    o, tl, tr, bl = view
    setup = {"W": width, "H": height, "origin": o, "tl": tl, "tr": tr, "bl": bl,
             "root": sf.root_transform(o), "children": sf.child_transforms()}
    ro = pyoracle.render(setup, rows=rows)
    return bool(np.array_equal(ro["pos4"].view(np.uint32), pos[rows].view(np.uint32)) and
                np.array_equal(ro["nrm4"].view(np.uint32), nrm[rows].view(np.uint32)))


def check_golden_rows(pos, nrm, golden, rows):
    """Rows `rows` (those the fixture holds: every row_step-th) against the golden row digests; returns
    (rows checked, rows that differ)."""
    step = golden.get("row_step", 1)
    ref = golden["row_digest_gbuf"]
    checked = [int(y) for y in rows if y % step == 0 and y // step < len(ref)]
    bad = [y for y in checked if row_digest(pos, nrm, y) != ref[y // step]]
    return len(checked), bad


def dist_loop(ctl, torch, dev, width, height, k, steps, warmup, slots, band_rows, nranks, frame_of,
              fixed=False, latency=False, first=False, gather=False, settle_ms=SETTLE_MS, long_steps=0, check=False,
              batch=1, timing=True):
    """One timed loop of the sf_dist path: `steps` frames (frame_of(i) of the camera path at step i) after
    `warmup`, `slots` in flight, over `nranks` ranks (1: this GPU alone, every rank its own frames); each frame
    is every rank's bands into its own G-buffer (the distributed G-buffer), or with `gather` also assembled on
    rank 0 (RCCL). Barrier + device sync on both sides of the timed region; the time is the max over ranks.

    `long_steps` > steps: a second loop of that many frames, timed the same way from an empty pipeline, gives the
    steady frame period (the difference of the two loops per extra frame) and the pipeline fill (what the timed
    loop pays beyond steps x the period: its first frames start with no frame in flight).
    `check`: after the timed loop, its last frame's rows (this rank's bands; 12 of them) against the oracle, and
    after the fixed-view loop that frame's rows against the golden digests of the config (when one exists).
    `batch` > 1 (not with `gather`): the loops issue `batch` frames per multi-frame persistent launch (FrameIssuer);
    the one-frame latency stays one launch per frame."""
    rank = ctl.rank if nranks > 1 else 0
    ids = shard.dist_ids(slots) if nranks > 1 and gather else None
    d = sf.SphereflakeDist(dev.index, width, height, rank=rank, nranks=nranks, slots=slots, ids=ids,
                           band_rows=band_rows)
    render = d.Render if gather else d.RenderBands
    issuer = FrameIssuer(d, render, 1 if gather else batch)
    view_at = path_views(width, height, k, frame_of)
    views = [view_at(i) for i in range(warmup + steps)]
    out = {"checks": {}}
    mine = owned_rows(height, band_rows, nranks, rank) if not gather else np.arange(height)
    ctl.barrier()
    if first:   # the first render of a fresh context: row-major tile order, no cost history
        d.SetView(*views[0])
        t = time.perf_counter()
        render()
        d.Synchronize()
        out["first_render_ms"] = (time.perf_counter() - t) * 1e3
    # Kernel timing is switched on before the warm-up: the first switch-on creates each slot's events and clock
    # buffer (~5.7 ms of host calls at 3 slots), and an idle GPU gives its clock back within that gap -- a timed loop
    # started after it ran at 2200-2240 MHz instead of ~2375 (0.085 vs 0.0785 ms per frame, profiles/r4/clock/).
    # Switched on again after the settle, it only restarts the sample ring (host state, no GPU call).
    kp = slot_period(steps, slots)
    for s in range(slots if timing else 0):
        d.kernel_timing(s, True, period=kp)
    t_w = time.perf_counter()
    issuer.issue(FrameIssuer.view_rows(views[:warmup]))
    out["settle_frames"] = settle(d, render, views, max(1, warmup), t_w, settle_ms, issuer)
    for s in range(slots if timing else 0):
        d.kernel_timing(s, True, period=kp)
    d.reset_stats()

    def timed(n, view_of):
        rows = FrameIssuer.view_rows([view_of(i) for i in range(n)])   # (the camera path, made before the timing)
        torch.cuda.synchronize(dev)
        ctl.barrier()
        torch.cuda.synchronize(dev)
        # (no Python garbage collection inside the timed region: a collection pause on the host between two
        # enqueues starves a pipeline only ~3 frames deep -- one 20-step loop in six measured +0.15 ms)
        gc.disable()
        enq = [] if ENQ_TRACE else None
        try:
            t0 = time.perf_counter()
            if enq is not None or issuer.batch == 1:
                for i in range(n):
                    d.SetView(*view_of(i))
                    render()
                    if enq is not None:
                        enq.append(time.perf_counter())
            else:
                issuer.issue(rows)
            # the device synchronize waits for every stream of the process, the slots' own included; the dist's
            # Synchronize (its stats copy and error check) follows the timed region
            torch.cuda.synchronize(dev)
            ctl.barrier()
            dt = time.perf_counter() - t0
        finally:
            gc.enable()
        d.Synchronize()
        if enq is not None:   # diagnostics (SF_BENCH_ENQ_TRACE=1): host time at each frame's enqueue, and the end
            out.setdefault("enqueue_trace_us", []).append(
                [round((t - t0) * 1e6, 1) for t in enq] + [round(dt * 1e6, 1)])
        return ctl.max(dt)

    out["t_step"] = timed(steps, lambda i: views[warmup + i]) / steps
    tk, clk = [], []
    for s in range(slots if timing else 0):
        tk += list(d.kernel_timing(s, n=64))
        clk += list(d.kernel_clocks(s, n=64))
        d.kernel_timing(s, False)
    out["trace_ms"] = float(np.mean(tk)) if tk else None
    out["kernel_samples"] = len(tk)
    out["clock_mhz"] = float(np.median(clk)) if clk else None
    st = d.stats()   # (collective over the ranks with RCCL communicators; else combined over gloo)
    if nranks > 1 and ids is None:
        st = ctl.combine_stats(st)
    if st.overflow_tiles:
        raise RuntimeError("traversal overflowed SF_MAX_DEPTH_LIMIT")
    out["stats"] = st
    if check and (rank == 0 or not gather):   # the last timed frame, outside the timed region (downloaded now,
        pos, nrm = d.download_slot(d.last_slot())   # checked after the long loop: no idle GPU before that loop)
        rows = mine[np.linspace(0, len(mine) - 1, min(12, len(mine))).astype(int)] if len(mine) else mine
        moving = (pos[rows].copy(), nrm[rows].copy(), rows)
        del pos, nrm
    if long_steps > steps:
        # (a short settle first: the readouts above left the GPU idle for a few ms)
        settle(d, render, views, max(1, warmup), time.perf_counter(), LONG_SETTLE_MS, issuer)
        kpl = slot_period(long_steps, slots)
        for s in range(slots if timing else 0):   # the live clock of this loop too (the chip's clock moves between loops)
            d.kernel_timing(s, True, period=kpl)
        t_long = timed(long_steps, lambda i: view_at(warmup + steps + i))
        clk_l = []
        for s in range(slots if timing else 0):
            clk_l += list(d.kernel_clocks(s, n=64))
            d.kernel_timing(s, False)
        period = (t_long - out["t_step"] * steps) / (long_steps - steps)
        out["pipeline"] = {"steady_frame_ms": round(period * 1e3, 5),
                           "fill_ms": round((out["t_step"] - period) * steps * 1e3, 5),
                           "long_steps": long_steps, "long_frame_ms": round(t_long / long_steps * 1e3, 5),
                           "long_clock_mhz_live": round(float(np.median(clk_l)), 1) if clk_l else None}
    if check and (rank == 0 or not gather):
        p_rows, n_rows, rows = moving
        pos = np.zeros((height, width, 4), np.float32)
        nrm = np.zeros((height, width, 4), np.float32)
        pos[rows], nrm[rows] = p_rows, n_rows
        out["checks"]["moving_oracle_rows"] = {"rows": len(rows), "bit_exact":
                                               check_oracle_rows(pos, nrm, views[-1], width, height, rows)}
        del pos, nrm, moving
    if fixed:   # the same loop on one unchanging view (the config camera)
        cfg_view = frame_camera(width, height, k, 0).corners()
        d.SetView(*cfg_view)
        t_w = time.perf_counter()
        issuer.issue(FrameIssuer.view_rows([cfg_view] * warmup))
        # (the host work since the timed loop let the clock drop: settle again)
        settle(d, render, [cfg_view], 1, t_w, settle_ms, issuer)
        out["t_fixed"] = timed(steps, lambda i: cfg_view) / steps
        golden = golden_frame(width, height, k) if check else None
        if golden is not None and (rank == 0 or not gather):
            pos, nrm = d.download_slot(d.last_slot())
            n_rows, bad = check_golden_rows(pos, nrm, golden, mine)
            out["checks"]["fixed_golden_rows"] = {"fixture": f"tests/golden/frame_{golden['name']}.json",
                                                  "rows": n_rows, "rows_differing": bad[:16], "bit_exact": not bad}
            del pos, nrm
    if latency:   # one frame at a time, each waited for (rank 0's wait includes the gather of the others)
        lat = []
        for i in range(20):
            d.SetView(*views[i % len(views)])
            ctl.barrier()
            t = time.perf_counter()
            render()
            d.Synchronize()
            lat.append(time.perf_counter() - t)
        out["latency_ms"] = ctl.max(float(np.median(lat))) * 1e3
    out["dist"] = d
    return out


def checks_pass(ctl, checks):
    """Every check of every rank passed (combined over the control plane; True when there were none)."""
    ok = all(c.get("bit_exact", True) for c in checks.values())
    return ctl.max(0.0 if ok else 1.0) == 0.0


def rank_devices(ctl, gpu, launch_check=False):
    """Each rank's device as the rank sees it (index, PCI location, UUID), gathered on every rank."""
    import torch
    me = {"rank": ctl.rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": gpu}
    if not launch_check:
        p = torch.cuda.get_device_properties(gpu)
        me["name"] = getattr(p, "gcnArchName", None) or p.name
        for key in ("pci_bus_id", "pci_device_id", "pci_domain_id"):
            if hasattr(p, key):
                me[key] = int(getattr(p, key))
        if hasattr(p, "uuid"):
            me["uuid"] = str(p.uuid)
    if not ctl.dist:
        return [me]
    got = [None] * ctl.world
    ctl.dist.all_gather_object(got, me)
    return got


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args):
    """`--gpus N > 1` without a launcher: start N rank processes (torch.distributed.run, 127.0.0.1) with the same
    arguments and exit with their status. Runs before this process makes any GPU call (it makes none)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, SF_BENCH_SPAWNED="1")
    return subprocess.call(cmd, env=env)


def launch_world(args):
    """The rank layout of this run: (world, rank, local rank). `--gpus N > 1` with no launcher environment spawns the
    N ranks (this process then only waits for them); a launcher world that is not --gpus ranks is an error."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1 and args.mode != "rows":
            sys.exit(spawn_ranks(args))
        return 1, 0, 0
    world = int(env_world)
    if args.mode != "rows" and world != args.gpus:
        raise SystemExit(f"bench.py: the launcher started {world} rank(s) but --gpus is {args.gpus}: one rank per GPU, "
                         f"run with --gpus {world} (or without a launcher: --gpus N spawns the N ranks itself)")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def launch_check(args, world, rank, local):
    """--launch-check: the ranks come up and agree (no rendering, no GPU call)."""
    import torch
    ctl = Control(world, rank)
    ndev = torch.cuda.device_count()
    ranks = rank_devices(ctl, local % max(1, ndev) if world > 1 else 0, launch_check=True)
    t = ctl.max(0.0)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mrays/s", "n_gpus": world, "steps": 0,
                          "warmup": 0, "launch_check": True, "devices_visible": ndev, "ranks": ranks,
                          "spawned": os.environ.get("SF_BENCH_SPAWNED") == "1", "max_over_ranks": t}), flush=True)
    ctl.close()


def main():
    args = parse()
    world, rank, local = launch_world(args)
    if args.launch_check:
        launch_check(args, world, rank, local)
        return 0
    import torch
    n = world
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev) if world > 1 else 0
    if args.mode == "dist" and world > 1 and ndev < world and not args.rehearse:
        raise SystemExit(f"dist mode needs one GPU per rank (RCCL refuses two ranks on one device): {world} ranks, "
                         f"{ndev} GPU(s); rehearse with --rehearse (every leg but the RCCL gather)")
    torch.cuda.set_device(gpu)
    ctl = Control(world, rank)
    dev = torch.device("cuda", gpu)
    if not os.path.exists(sf.LIB_PATH):
        if rank == 0:
            sf.build()
        ctl.barrier()
    width, height = args.width, args.height
    kernel = sf.SF_KERNEL_WAVE if args.kernel == "wave" else sf.SF_KERNEL_PER_RAY
    if kernel != sf.SF_KERNEL_WAVE and args.mode == "dist":
        raise SystemExit("the per-ray kernel runs in --mode frames only")
    check = not args.no_check
    long_steps = args.long_steps or max(4 * args.steps, 200)

    # a tiny render on a throw-away context first: loads the code object, so that `first_render_ms`
    # below is the first render of a fresh context, not the process's first kernel launch
    t_load = time.perf_counter()
    with sf.Sphereflake(64, 64, device=dev.index) as warm:
        warm.SetCamera(sf.config_camera(64, 64, args.K))
        warm.Render()
        warm.Synchronize()
    module_load_ms = (time.perf_counter() - t_load) * 1e3

    if args.mode == "rows":
        run_rows(args, torch, ctl, max(n, args.gpus), kernel)
        ctl.close()
        return 0

    ranks = rank_devices(ctl, gpu)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nshare = n if args.mode == "dist" else 1
    batch = frames_per_launch(args.batch, cus, width, height, args.band_rows, nshare)
    slots = frames_in_flight(args.slots, cus, width, height, args.band_rows, nshare, batch)
    if args.mode == "dist":
        # the frame split over the ranks, each rank's bands into its own HBM (the distributed G-buffer)
        r = dist_loop(ctl, torch, dev, width, height, args.K, args.steps, args.warmup, slots, args.band_rows, n,
                      lambda i: i, fixed=True, latency=True, first=True, settle_ms=args.settle_ms,
                      long_steps=long_steps, check=check, batch=batch)
        rays_step = width * height
    else:   # frames: every rank its own frames (frame i * N + rank), one GPU each, slots in flight
        r = dist_loop(ctl, torch, dev, width, height, args.K, args.steps, args.warmup, slots, args.band_rows, 1,
                      lambda i: i * n + rank, fixed=True, latency=True, first=True, settle_ms=args.settle_ms,
                      long_steps=long_steps, check=check, batch=batch)
        rays_step = width * height * n
    d = r["dist"]
    t_step = r["t_step"]
    value = rays_step / t_step / 1e6
    st = r["stats"]
    d.close()

    # weak-scaling companion of a multi-GPU run: every rank renders its own frames (no gather)
    indep = None
    if args.mode == "dist" and n > 1:
        bi = frames_per_launch(args.batch, cus, width, height, args.band_rows, 1)
        ri = dist_loop(ctl, torch, dev, width, height, args.K, args.steps, args.warmup,
                       frames_in_flight(args.slots, cus, width, height, args.band_rows, 1, bi), args.band_rows, 1,
                       lambda i: i * n + rank, settle_ms=args.settle_ms, batch=bi)
        ri["dist"].close()
        indep = {"value": round(n * width * height / ri["t_step"] / 1e6, 2), "frame_ms": round(ri["t_step"] * 1e3, 4),
                 "scaling": "weak", "note": "every rank renders its own full frames (frame i * N + rank), no gather"}

    # BASELINE configs[3] (3840x2160, K = 0.22, depth 9) on the same path, all ranks
    c4 = None
    if not args.no_extras and (width, height, round(args.K, 4)) == (W, H, K):
        b4 = frames_per_launch(args.batch, cus, 3840, 2160, args.band_rows, nshare)
        r4 = dist_loop(ctl, torch, dev, 3840, 2160, 0.22, 60, 15,
                       frames_in_flight(args.slots, cus, 3840, 2160, args.band_rows, nshare, b4),
                       args.band_rows,
                       n if args.mode == "dist" else 1, (lambda i: i) if args.mode == "dist" else (lambda i: i * n + rank),
                       settle_ms=args.settle_ms, batch=b4)
        rays0_4 = (sf.lib().sf_slab_rows(2160, args.band_rows, n, 0) if args.mode == "dist" else 2160) * 3840
        a4 = BYTES_PER_RAY * rays0_4 / r4["t_step"] / 1e9
        c4 = {"config": "BASELINE configs[3]: 3840x2160, K=0.22", "max_depth": r4["stats"].max_depth,
              "value": round((3840 * 2160 * (n if args.mode == "frames" else 1)) / r4["t_step"] / 1e6, 2),
              "frame_ms": round(r4["t_step"] * 1e3, 4), "steps": 60, "warmup": 15,
              "roofline": {"achieved": round(a4, 2), "frac": round(a4 / HBM_PEAK_GBS, 5),
                           "basis": "32 B/ray x rank 0's rays per frame / frame period",
                           "kernel_event_ms_overlapped": round(r4["trace_ms"], 4) if r4["trace_ms"] else None,
                           "kernel_samples": r4["kernel_samples"],
                           "clock_mhz_live": round(r4["clock_mhz"], 1) if r4["clock_mhz"] else None}}
        r4["dist"].close()

    # Multi-GPU scaling projected on this one GPU (N = 1 runs only): rank 0's bands of an N-way split -- the member
    # with the most rows -- traced at the bench's own frames-in-flight policy, N = 2 / 4 / 8, each with its steady
    # period from a second loop; the speedup is against this run's own N = 1 steady period. Labelled a projection: the
    # N-GPU run itself is `bench.py --gpus N` (value = the distributed frame).
    shares = None
    SHARES_TIMING = os.environ.get("SF_BENCH_SHARES_TIMING", "0") == "1"   # (A/B: the kernel-timing events on)
    if n == 1 and args.mode == "dist" and not args.no_extras and "pipeline" in r:
        base = r["pipeline"]["steady_frame_ms"]
        shares = {"basis_steady_ms": base, "note": (
            "ONE GPU tracing rank 0's interleaved band share of an N-way split (the member with the most rows), at the "
            "bench's frames-in-flight and frames-per-launch policy, 64 timed steps + a 600-step loop for the steady period (kernel-timing events off); speedup = this "
            "run's N = 1 steady period / the share's; projected_mrays = W x H / the share's steady period. A "
            "projection of the distributed G-buffer at N GPUs, not an N-GPU run")}
        for nn in (2, 4, 8):
            bb = frames_per_launch(args.batch, cus, width, height, args.band_rows, nn)
            sl = frames_in_flight(args.slots, cus, width, height, args.band_rows, nn, bb)
            rs = dist_loop(ctl, torch, dev, width, height, args.K, 64, 16, sl, args.band_rows, nn, lambda i: i,
                           settle_ms=args.settle_ms, long_steps=600, timing=SHARES_TIMING, batch=bb)
            rs["dist"].close()
            sp = rs.get("pipeline", {}).get("steady_frame_ms") or rs["t_step"] * 1e3
            shares[f"n{nn}"] = {"slots": sl, "frames_per_launch": bb, "ms_per_step": round(rs["t_step"] * 1e3, 5),
                                "steady_ms": round(sp, 5), "speedup": round(base / sp, 3),
                                "projected_mrays": round(width * height / sp / 1e3, 1)}

    post = d2h = prog = None
    if rank == 0 and n == 1 and not args.no_extras:
        # the consumers of the G-buffer on a plain context: SSAO post-process, D2H into the
        # host GBuffer (PCIe-inclusive, never `value`, §8(f3)), the frame-less mode (§8(f1))
        stream = torch.cuda.Stream(device=dev)
        with sf.Sphereflake(width, height, device=dev.index) as ctx:
            ctx.SetCamera(sf.config_camera(width, height, args.K))
            ctx.Render()
            ctx.Synchronize()
            post = post_rates(ctx, torch, stream, width, height)
            d2h = transfer_rates(ctx, torch, dev, stream, width, height, kernel)
        prog = progressive_rates(width, height, args.K)

    checks = r["checks"]
    checks_ok = checks_pass(ctl, checks) if check else None
    out = None
    if rank == 0:
        band = args.band_rows
        rays0 = (sf.lib().sf_slab_rows(height, band, n, 0) if args.mode == "dist" else height) * width
        clock = r["clock_mhz"]
        # roofline of the frame: the G-buffer stores of rank 0's share of one frame per frame period (the timed
        # steps' period, as ms_per_step); with frames in flight no single kernel duration is a frame's
        achieved = BYTES_PER_RAY * rays0 / t_step / 1e9
        build = sf.build_info()
        pmc, _ = load_pmc(TRACE_KERNEL, pmc_config_key(width, height, args.K, "moving"), build)
        traffic = pmc_traffic(pmc) if n == 1 else None
        cfg_name = BASELINE_CONFIGS.get((width, height, round(args.K, 4)))
        if args.mode == "dist":
            par = (f"dist x{n}: one frame split in interleaved {band}-row bands, each rank's bands into its own HBM "
                   f"(distributed G-buffer; the RCCL-gathered rate is `gathered_on_rank0`); {slots} frames in flight"
                   if n > 1 else f"1 GPU, {slots} frames in flight (sf_dist slots)")
        else:
            par = f"frames x{n} (independent frames per rank, {slots} in flight each)"
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": round(traffic) if traffic else None,
                "kernel": TRACE_KERNEL,
                "basis": "32 B/ray x rank 0's rays of one frame / ms_per_step (one trace launch per frame)",
                "units_per_launch": rays0, "bytes_per_unit": BYTES_PER_RAY,
                "kernel_event_ms_overlapped": round(r["trace_ms"], 4) if r["trace_ms"] else None,
                "kernel_samples": r["kernel_samples"],
                "clock_mhz_live": round(clock, 1) if clock else None,
                "note": "path is issue-bound (SURVEY.md §8(d), see `valu`); kernel_event_ms_overlapped = mean HIP-event "
                        "duration of the trace kernel on its stream, which with frames in flight shares the GPU with the "
                        "next frames' launches and so exceeds the frame period by construction (not used above); "
                        "traffic = PMC WRITE_SIZE + 2 x FETCH_SIZE per launch (profiles/pmc_traffic.json, only for "
                        "this config and this library build, else null)"}
        if "pipeline" in r:
            roof["steady_achieved"] = round(BYTES_PER_RAY * rays0 / (r["pipeline"]["steady_frame_ms"] * 1e-3) / 1e9, 2)
            roof["steady_frac"] = round(roof["steady_achieved"] / HBM_PEAK_GBS, 5)
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"min_ms": args.settle_ms, "frames": r["settle_frames"],
                       "note": "untimed frames after --warmup until the GPU has been under load min_ms: the shader "
                               "clock ramps from ~2075 to ~2370 MHz over the first ~60 ms (profiles/r3/ramp.txt); "
                               "the clock the timed loop ran at is roofline.clock_mhz_live"},
            "ms_per_step": round(t_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.mode == "dist" else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": DATA_MOVING,
            "config": {"workload": f"{width}x{height} primary-ray G-buffer, camera K={args.K:g} (reference max "
                                   f"depth {st.max_depth})" + (f", BASELINE {cfg_name}" if cfg_name else "")
                                   + f", moving camera, {args.kernel} kernel",
                       "width": width, "height": height, "K": args.K, "max_depth": st.max_depth, "camera": "moving",
                       "slots": slots, "frames_per_launch": batch,
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4), "parallelism": par},
            "frame_ms": round(t_step * 1e3, 4),
            "frame_latency_ms": round(r["latency_ms"], 4),
            "first_render_ms": round(r["first_render_ms"], 4),
            "process_first_launch_ms": round(module_load_ms, 3),
            "fixed_camera": {"value": round(rays_step / r["t_fixed"] / 1e6, 2), "frame_ms": round(r["t_fixed"] * 1e3, 4),
                             "note": "same timed loop on the unchanging config view"},
            "rays_counted": int(st.rays),
            "roofline": roof,
            "valu": pmc_valu(pmc, t_step * 1e3, clock) if n == 1 else None,
            "build": build,
            "ranks": ranks,
        }
        if "pipeline" in r:
            out["pipeline"] = dict(r["pipeline"], note=(
                "a second loop of long_steps frames from an empty pipeline, timed like the first: steady_frame_ms = "
                "(its time - the timed loop's) / the extra frames; fill_ms = the timed loop's time beyond steps x "
                "steady_frame_ms (its first frames run with no frame in flight), so ms_per_step = steady_frame_ms + "
                "fill_ms / steps"))
        if "enqueue_trace_us" in r:
            out["enqueue_trace_us"] = r["enqueue_trace_us"]
        if check:
            out["check"] = {"bit_exact": checks_ok, **checks,
                            "note": "outside the timed region; this rank's rows (rank 0's bands on N > 1): the last "
                                    "timed moving frame against the oracle restatement, the last fixed-view frame "
                                    "against the reference-made golden row digests; all ranks combined in bit_exact"}
        if n > 1 and args.mode == "dist":
            out["independent_frames"] = indep
            if args.rehearse:
                out["config"]["parallelism"] += f" [rehearsal: {n} ranks on {ndev} GPU(s), no RCCL gather]"
        if c4 is not None:
            out["configs"] = {"c4": c4}
        if shares is not None:
            out["member_shares"] = shares
        if post is not None:
            out["post"], out["d2h"], out["frameless"] = post, d2h, prog
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

    # Last, the same frames assembled on rank 0 (RCCL gather of the packed slabs + unpack). It is the only leg
    # with a data-path collective, so it runs after every other number is in hand, under a watchdog: an RCCL
    # error, a hang past --gather-timeout or a gathered frame that differs from the golden frame prints the line
    # with the leg marked failed and exits EXIT_GATHER_FAILED.
    rc = 0 if checks_ok in (None, True) else EXIT_CHECK_FAILED
    if n > 1 and args.mode == "dist" and not args.rehearse:
        if rank == 0:
            out["gathered_on_rank0"] = {"error": f"not finished within {args.gather_timeout:g} s"}
        wd = Watchdog(args.gather_timeout, (lambda: print(json.dumps(out), flush=True)) if rank == 0 else (lambda: None))
        # (3 in flight whatever the share: rank 0 also runs a receive stream per slot, and more streams than the
        # process's 4 hardware queues put a waiting receive in front of another slot's trace)
        gathered = gather_leg(args, ctl, torch, dev, args.slots or SLOTS_FULL, n, rays_step, check)
        wd.cancel()
        if rank == 0:
            out["gathered_on_rank0"] = gathered
        failed = ctl.max(1.0 if "error" in gathered or gathered.get("check", {}).get("bit_exact") is False else 0.0)
        if failed:
            rc = EXIT_GATHER_FAILED
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctl.close()
    return rc


def gather_leg(args, ctl, torch, dev, slots, n, rays_step, check):
    """The timed frames assembled on rank 0 (sf_dist_render: RCCL grouped send/recv of the packed slabs, unpacked on
    rank 0 beside its own bands), then the config view once more, gathered, against the golden row digests."""
    width, height = args.width, args.height
    try:
        rg = dist_loop(ctl, torch, dev, width, height, args.K, args.steps, args.warmup, slots, args.band_rows, n,
                       lambda i: i, latency=True, gather=True, settle_ms=args.settle_ms)
        d = rg["dist"]
        comm = d.comm_info(0)
        slab_bytes = d.slab_bytes()
        peer_bytes = sum(sf.lib().sf_slab_rows(height, args.band_rows, n, kk) for kk in range(1, n)) * width * slab_bytes
        t = rg["t_step"]
        g = {"value": round(rays_step / t / 1e6, 2), "frame_ms": round(t * 1e3, 4),
             "frame_latency_ms": round(rg["latency_ms"], 4),
             "rccl": {"comm_count": comm[0], "rank0_user_rank": comm[1], "rank0_device": comm[2]},
             "slab_bytes_per_pixel": slab_bytes, "bytes_per_frame": peer_bytes,
             "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                          "achieved": round(BYTES_PER_RAY * rays_step / t / 1e9, 2),
                          "frac": round(BYTES_PER_RAY * rays_step / t / 1e9 / HBM_PEAK_GBS, 5),
                          "basis": "rank 0 writes the whole frame's G-buffer (32 B/pixel) per frame period",
                          "link_GBps_per_peer": round(peer_bytes / max(1, n - 1) / t / 1e9, 2)},
             "format": ("one uint32 hit index per pixel (rank 0 rebuilds centre, minT, position and normal from it)"
                        if slab_bytes == 4 else "float4 (nx, ny, nz, minT) per pixel; rank 0 rebuilds pos = dir * minT"),
             "transport": "RCCL grouped ncclSend/ncclRecv to rank 0 over xGMI, one communicator per slot; rank 0's "
                          "receive and unpack on a stream of their own beside its trace",
             "note": "every frame complete in rank 0's G-buffer (reference layout): the rate a consumer on rank 0 sees"}
        if check:
            golden = golden_frame(width, height, args.K)
            if golden is not None:
                d.SetView(*sf.config_camera(width, height, args.K).corners())
                d.Render()
                d.Synchronize()
                if ctl.rank == 0:
                    pos, nrm = d.download()
                    n_rows, bad = check_golden_rows(pos, nrm, golden, np.arange(height))
                    g["check"] = {"fixture": f"tests/golden/frame_{golden['name']}.json", "rows": n_rows,
                                  "rows_differing": bad[:16], "bit_exact": not bad}
        d.close()
        return g
    except Exception as e:   # (an RCCL error on one rank: the others fail or the watchdog ends them)
        return {"error": f"{type(e).__name__}: {e}"}


if __name__ == "__main__":
    sys.exit(main())
