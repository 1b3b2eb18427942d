"""Multi-rank host logic of the row-band path on CPU: world_size 2 and 3 over
gloo. Each rank produces the slab of the bands it owns, with the CPU oracle standing in for the
GPU (the checker only, as on the GPU box the slab comes from sf_render_to). Slabs are gathered and
reassembled on rank 0, and must equal the golden full frame bit for bit. Stats reduce as the
reference counters would."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, load_frame, load_npz
from sphereflake_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, band_rows, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import pyoracle
        fx = load_frame(name)
        W, H = fx["W"], fx["H"]
        setup = pyoracle.load_setup(name)
        rows = [y for y0, y1 in shard.owned_bands(H, band_rows, world, rank) for y in range(y0, y1)]
        assert len(rows) == shard.slab_rows(H, band_rows, world, rank)
        pad = shard.max_slab_rows(H, band_rows, world)
        slab = torch.zeros((pad, W, 4), dtype=torch.float32)
        st = {"max_depth": -1, "closest": float(np.finfo(np.float32).max), "rays": 0}
        if rows:
            r = pyoracle.render(setup, rows=rows, threads=1)
            slab[:len(rows)] = torch.from_numpy(r["pos4"])
            st = r["stats"]
        frame = shard.gather_frame(slab, H, band_rows)
        md, cl, ry = shard.reduce_stats(st["max_depth"], st["closest"], len(rows) * W)
        if rank == 0:
            ref = load_npz(name)
            assert frame.shape == (H, W, 4)
            assert np.array_equal(frame.numpy().view(np.uint32), ref["pos4"].view(np.uint32))
            assert ry == W * H
            assert md == fx["stats"]["max_depth"]
            assert np.float32(cl) == np.float32(ref["minT"].min())
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent, which fails the test
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _run(world, name, band_rows):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), name, band_rows, errq), nprocs=world,
                       start_method="spawn", join=True)
    assert errq.empty(), errq.get()


@pytest.mark.parametrize("world,name,band_rows", [(2, "t2", 8), (3, "t3", 8), (2, "t1", 16)])
def test_gloo_band_gather_reassembles_frame(world, name, band_rows):
    _run(world, name, band_rows)


@pytest.mark.parametrize("H,band,world", [(1080, 8, 8), (2160, 8, 8), (36, 16, 2), (7, 8, 3), (1, 8, 2),
                                          (16384, 64, 8)])
def test_slab_rows_mirror_c_abi(H, band, world):
    from sphereflake_amd import lib
    total = 0
    for r in range(world):
        n = shard.slab_rows(H, band, world, r)
        assert n == lib().sf_slab_rows(H, band, world, r)
        total += n
    assert total == H


def test_reassemble_inverts_banding():
    H, W, band, world = 53, 5, 8, 3
    frame = np.arange(H * W, dtype=np.int32).reshape(H, W)
    slabs = []
    for r in range(world):
        rows = [y for y0, y1 in shard.owned_bands(H, band, world, r) for y in range(y0, y1)]
        s = np.full((shard.max_slab_rows(H, band, world), W), -1, np.int32)
        s[:len(rows)] = frame[rows]
        slabs.append(s)
    assert np.array_equal(shard.reassemble(slabs, H, band), frame)


def test_band_rows_validation():
    with pytest.raises(ValueError):
        shard.owned_bands(100, 12, 2, 0)
    with pytest.raises(ValueError):
        shard.owned_bands(100, 8, 2, 2)


# ---- the one-process-per-GPU gather (sf_dist_*, csrc/sf_dist.hip): packed slabs and the RCCL id exchange

def _ray_dirs(setup):
    """Ray directions of every pixel exactly as the kernels' ray_dir (reference Sphereflake.cpp:149-150,
    162-167; SIMD_AVX.h:170-180 Normalize with the x86 rsqrtps of the C ABI's table), in float32 numpy
    (IEEE per operation, no contraction)."""
    from sphereflake_amd import lib
    W, H = setup["W"], setup["H"]
    f = np.float32
    o, tl, tr, bl = (np.asarray(setup[k], f) for k in ("origin", "tl", "tr", "bl"))
    dh, dv = tr - tl, bl - tl
    u = (np.arange(W, dtype=f) / f(W))[None, :]
    v = (np.arange(H, dtype=f) / f(H))[:, None]
    d = [((tl[c] + dh[c] * u) + dv[c] * v) - o[c] for c in range(3)]
    ln = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]
    nr = np.vectorize(lambda x: lib().sf_rsqrtps(float(x)), otypes=[f])(ln)
    sc = (f(0.5) * nr) * (f(3.0) - (ln * nr) * nr)
    return [c * sc for c in d]


@pytest.mark.parametrize("name", ["t1", "t2", "t3", "t4", "t5"])
def test_packed_slab_format_is_lossless(name):
    """A packed slab pixel is (nx, ny, nz, minT): rank 0 rebuilds the position as dir * minT
    (sf_band_unpack). On every golden pixel that equals the reference's position bit for bit -- a hit's
    position is exactly dir * t (Sphereflake.h:218-220), a miss keeps minT = FLT_MAX and writes (0,0,0,1)."""
    from oracle import pyoracle
    setup = pyoracle.load_setup(name)
    ref = load_npz(name)
    dx, dy, dz = _ray_dirs(setup)
    t = ref["minT"]
    hit = t < np.finfo(np.float32).max
    rebuilt = np.zeros_like(ref["pos4"])
    rebuilt[..., 0] = np.where(hit, dx * t, 0)
    rebuilt[..., 1] = np.where(hit, dy * t, 0)
    rebuilt[..., 2] = np.where(hit, dz * t, 0)
    rebuilt[..., 3] = 1.0
    assert np.array_equal(rebuilt.view(np.uint32), ref["pos4"].view(np.uint32))
    assert np.all(ref["nrm4"][~hit][:, :3] == 0.0)


def _index_unpack(setup, index, lut_fn):
    """numpy float32 restatement of sf_slab_unpack4 for one frame: from each pixel's heap index (9n+1+i) rebuild the
    sphere's frame down the chain from the root (Sphereflake.h:162-164, SIMD_AVX.h:59-81: column c = ((P0 b0 + P1 b1)
    + P2 b2) + P3 b3, translation column scaled by (4/3) r_p), its self test's minT (tca, d2, the near root with
    r_d^2, SIMD_AVX.h:236-270), then the position dir * minT and the normal Normalize(pos - centre)."""
    f = np.float32
    W, H = setup["W"], setup["H"]
    child = setup["children"].reshape(9, 4, 4)          # [i][column][row], glm column-major
    root = setup["root"].reshape(4, 4)
    rad = setup["radius"]
    dx, dy, dz = _ray_dirs(setup)
    pos = np.zeros((H, W, 4), np.float32)
    nrm = np.zeros((H, W, 4), np.float32)
    pos[..., 3] = nrm[..., 3] = 1.0
    for y in range(H):
        for x in range(W):
            n = int(index[y, x])
            if n == 0xffffffff:
                continue
            digits = []
            while n:
                q = (n - 1) // 9
                digits.append(n - 1 - 9 * q)
                n = q
            P = [root[c][:3].copy() for c in range(4)]
            for p, i in enumerate(reversed(digits)):
                s = f(f(4.0) / f(3.0)) * rad[p]
                out = []
                for c in range(4):
                    b = child[i][c].copy()
                    if c == 3:
                        b[:3] = b[:3] * s
                    out.append(((P[0] * b[0] + P[1] * b[1]) + P[2] * b[2]) + P[3] * b[3])
                P = out
            d = len(digits)
            cx, cy, cz = P[3]
            tca = (cx * dx[y, x] + cy * dy[y, x]) + cz * dz[y, x]
            d2 = ((cx * cx + cy * cy) + cz * cz) - tca * tca
            thc = np.sqrt(f(rad[d] * rad[d]) - d2, dtype=np.float32)
            t0, t1 = tca + thc, tca - thc
            t = t0 if t0 <= t1 else t1
            px, py, pz = dx[y, x] * t, dy[y, x] * t, dz[y, x] * t
            qx, qy, qz = px - cx, py - cy, pz - cz
            ln = (qx * qx + qy * qy) + qz * qz
            nr = f(lut_fn(float(ln)))
            sc = (f(0.5) * nr) * (f(3.0) - (ln * nr) * nr)
            pos[y, x, :3] = (px, py, pz)
            nrm[y, x, :3] = (qx * sc, qy * sc, qz * sc)
    return pos, nrm


@pytest.mark.parametrize("name", ["t1", "t2", "t3", "t4", "t5"])
def test_index_slab_format_is_lossless(name):
    """An index slab pixel is the hit's heap index alone (4 B): rank 0 rebuilds the sphere's frame, minT, position and
    normal from it (sf_slab_unpack4). On every golden pixel -- frames rendered by the reference itself -- that equals
    the reference's position and normal bit for bit."""
    from oracle import pyoracle
    from sphereflake_amd import lib
    setup = pyoracle.load_setup(name)
    ref = load_npz(name)
    assert int(ref["depth"].max()) <= 10   # (the index format's domain: heap indices below 2^32)
    pos, nrm = _index_unpack(setup, ref["index"], lambda v: lib().sf_rsqrtps(v))
    assert np.array_equal(pos.view(np.uint32), ref["pos4"].view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), ref["nrm4"].view(np.uint32))


def _ids_worker(rank, world, port, slots, errq, outq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ids = shard.dist_ids(slots)
        outq.put((rank, ids))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("world,slots", [(2, 2), (3, 3)])
def test_dist_ids_reach_every_rank(world, slots):
    """sf_dist_create needs the same RCCL unique id per slot on every rank: rank 0 makes them
    (sf_dist_unique_id) and broadcasts them; every rank must hold the identical, distinct ids."""
    ctx = mp.get_context("spawn")
    errq, outq = ctx.SimpleQueue(), ctx.SimpleQueue()
    mp.start_processes(_ids_worker, args=(world, _free_port(), slots, errq, outq), nprocs=world,
                       start_method="spawn", join=True)
    assert errq.empty(), errq.get()
    got = dict(outq.get() for _ in range(world))
    assert len(got) == world
    first = got[0]
    assert len(first) == slots * 128
    assert all(v == first for v in got.values())
    chunks = {first[k * 128:(k + 1) * 128] for k in range(slots)}
    assert len(chunks) == slots


def _stats_worker(rank, world, port, errq, outq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import bench
        import sphereflake_amd as sf
        ctl = bench.Control(world, rank)
        st = sf.sf_stats()
        st.max_depth, st.closest, st.rays, st.overflow_tiles = 5 + rank, 1.5 - 0.25 * rank, 1000 * (rank + 1), rank
        got = ctl.combine_stats(st)
        outq.put((rank, got.max_depth, float(got.closest), int(got.rays), int(got.overflow_tiles), ctl.max(rank * 0.5)))
        ctl.close()
    except BaseException as e:
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_bench_control_combines_rank_stats(world):
    """The multi-GPU bench's value leg renders without RCCL communicators, so each rank's sf_stats are combined
    over the gloo control plane (bench.Control.combine_stats): max depth max, closest min, rays and overflow tiles
    summed -- the same reduction sf_dist_get_stats does over RCCL; the timed region is the max over ranks."""
    ctx = mp.get_context("spawn")
    errq, outq = ctx.SimpleQueue(), ctx.SimpleQueue()
    mp.start_processes(_stats_worker, args=(world, _free_port(), errq, outq), nprocs=world, start_method="spawn",
                       join=True)
    assert errq.empty(), errq.get()
    got = [outq.get() for _ in range(world)]
    for _, md, cl, rays, ovf, tmax in got:
        assert md == 5 + world - 1
        assert cl == 1.5 - 0.25 * (world - 1)
        assert rays == 1000 * world * (world + 1) // 2
        assert ovf == world * (world - 1) // 2
        assert tmax == 0.5 * (world - 1)


def test_bench_watchdog_prints_line_and_exits():
    """A leg past its deadline (the RCCL gather hanging on an unseen node): the watchdog runs its callback (rank 0
    prints the line with the leg marked failed) and ends the process with EXIT_GATHER_FAILED -- a hang is never a
    success."""
    import subprocess
    import sys
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "bench.Watchdog(0.5, lambda: print('LINE', flush=True))\n"
            "time.sleep(30)\nprint('NOT REACHED')\n") % REPO
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    import bench
    assert r.returncode == bench.EXIT_GATHER_FAILED != 0, r.stderr
    assert r.stdout.strip() == "LINE"
    code2 = ("import sys, time; sys.path.insert(0, %r); import bench\n"
             "w = bench.Watchdog(1.0, lambda: print('LINE', flush=True))\nw.cancel()\ntime.sleep(1.5)\n"
             "print('DONE')\n") % REPO
    r = subprocess.run([sys.executable, "-c", code2], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "DONE", r.stderr


def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_spawns_the_ranks(n):
    """`python3 bench.py --gpus N` with no launcher starts the N rank processes itself (torch.distributed.run on
    127.0.0.1) before any GPU call: the line reports n_gpus N and every rank, each with its own local rank.
    (--launch-check stops before rendering, so this runs on the CPU.)"""
    r, line = _bench(["--gpus", str(n), "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert line is not None and line["n_gpus"] == n and line["spawned"] is True
    assert sorted(x["rank"] for x in line["ranks"]) == list(range(n))
    assert sorted(x["local_rank"] for x in line["ranks"]) == list(range(n))


def test_bench_world_mismatch_exits_nonzero():
    """A launcher world that is not --gpus ranks is refused (non-zero exit, no line): no silent 1-GPU measurement
    labelled as N, no N ranks measured as 1."""
    for world, gpus in ((3, 2), (2, 1)):
        r, line = _bench(["--gpus", str(gpus), "--launch-check"],
                         {"WORLD_SIZE": str(world), "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                          "MASTER_PORT": str(_free_port())}, timeout=120)
        assert r.returncode != 0 and line is None, (world, gpus, r.stdout)
        assert "--gpus" in r.stderr


def test_bench_one_gpu_launch_check():
    r, line = _bench(["--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 1 and line["spawned"] is False and len(line["ranks"]) == 1
