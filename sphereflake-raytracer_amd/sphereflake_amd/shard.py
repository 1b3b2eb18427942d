"""Row-band sharding of one frame across ranks.

The reference renders one image with host threads that share a G-buffer
(Sphereflake.cpp:67-74, 86-214). Here each rank (one process per GPU) renders the bands it owns into a
compact slab with ``sf_render_to(..., compact=1)`` (include/sphereflake/sf.h). Slabs travel to rank 0
in one ``torch.distributed.gather``. On ROCm the ``nccl`` backend is RCCL over xGMI; CPU tests use
``gloo``. Rank 0 then reassembles the frame. Stats combine as the reference's counters would:
max depth → max, closest → min, rays → sum (Sphereflake.h:30-58).

Band layout: band b covers rows [b*band_rows, min(H, (b+1)*band_rows)). Rank r owns the bands
b ≡ r (mod world). Interleaving balances the load, because sky rows cost ~1 node per ray and flake
rows ~150. Rank r's slab holds its bands in increasing b, packed contiguously.
"""
from __future__ import annotations

import numpy as np


def owned_bands(height: int, band_rows: int, world: int, rank: int):
    """[(y0, y1), ...] row ranges of the bands `rank` owns, in slab order."""
    if band_rows <= 0 or band_rows % 8:
        raise ValueError("band_rows must be a positive multiple of 8")
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    nb = (height + band_rows - 1) // band_rows
    return [(b * band_rows, min(height, (b + 1) * band_rows)) for b in range(rank, nb, world)]


def slab_rows(height: int, band_rows: int, world: int, rank: int) -> int:
    """Height of rank's compact slab (mirror of the C ABI's sf_slab_rows)."""
    return sum(y1 - y0 for y0, y1 in owned_bands(height, band_rows, world, rank))


def max_slab_rows(height: int, band_rows: int, world: int) -> int:
    return max(slab_rows(height, band_rows, world, r) for r in range(world))


def reassemble(slabs, height: int, band_rows: int, out=None):
    """Frame [H, W, ...] from the per-rank slabs (numpy arrays or torch tensors, rank order).
    Slabs may carry padding rows past their slab height; those are ignored."""
    world = len(slabs)
    first = slabs[0]
    shape = (height,) + tuple(first.shape[1:])
    if out is None:
        if isinstance(first, np.ndarray):
            out = np.empty(shape, first.dtype)
        else:
            import torch
            out = torch.empty(shape, dtype=first.dtype, device=first.device)
    for r, slab in enumerate(slabs):
        k = 0
        for y0, y1 in owned_bands(height, band_rows, world, r):
            out[y0:y1] = slab[k:k + (y1 - y0)]
            k += y1 - y0
    return out


def gather_frame(slab, height: int, band_rows: int, group=None, dst: int = 0):
    """Collect every rank's slab on `dst` and reassemble the frame there (None on other ranks).
    `slab` is a torch tensor [rows, W, C] already padded to max_slab_rows (all ranks the same
    shape, as torch.distributed.gather requires). Device placement follows the backend: CUDA
    tensors for nccl (RCCL), CPU tensors for gloo."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [torch.empty_like(slab) for _ in range(world)] if rank == dst else None
    dist.gather(slab, parts, dst=dst, group=group)
    if rank != dst:
        return None
    return reassemble(parts, height, band_rows)


def reduce_stats(max_depth: int, closest: float, rays: int, group=None, device=None):
    """All-reduce per-rank frame stats: (max depth, min closest, sum rays)."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else "cpu"
    md = torch.tensor([max_depth], dtype=torch.int64, device=dev)
    cl = torch.tensor([closest], dtype=torch.float32, device=dev)
    ry = torch.tensor([rays], dtype=torch.int64, device=dev)
    dist.all_reduce(md, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(cl, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(ry, op=dist.ReduceOp.SUM, group=group)
    return int(md.item()), float(cl.item()), int(ry.item())


def dist_ids(slots: int, group=None, src: int = 0) -> bytes:
    """RCCL unique ids for sf_dist_create (one per slot): made on rank `src` (sf_dist_unique_id), broadcast
    to every rank over torch.distributed (any backend), so all ranks initialise the same communicators."""
    import torch
    import torch.distributed as dist
    from . import SF_DIST_ID_BYTES, dist_unique_id
    n = slots * SF_DIST_ID_BYTES
    if dist.get_rank(group) == src:
        raw = b"".join(dist_unique_id() for _ in range(slots))
        t = torch.tensor(list(raw), dtype=torch.uint8)
    else:
        t = torch.zeros(n, dtype=torch.uint8)
    backend = dist.get_backend(group)
    if backend == "nccl":
        t = t.cuda()
    dist.broadcast(t, src=src, group=group)
    return bytes(t.cpu().tolist())
