#!/usr/bin/env python3
"""The index-slab unpack alone (csrc/sf_kernels.hip sf_slab_unpack4d / sf_slab_unpack4): members 1..N-1's 4-B
slabs of a frame rendered once, then unpacked REPS times into member 0's G-buffer with nothing else on the GPU,
timed with HIP events around the batch. Prints us per unpack and its HBM rate: 4 B read + 32 B written per unpacked
pixel (the node table's reads are cached and not counted). Usage: unpack_probe.py [W H K N REPS]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402

W, H, K, N, REPS = ((int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
                    if len(sys.argv) > 5 else (3840, 2160, 0.22, 8, 50))
band = 8
rows = [sf.lib().sf_slab_rows(H, band, N, k) for k in range(N)]
stage_rows = max(rows[1:])
stage = torch.zeros((N - 1, stage_rows, W), dtype=torch.int32, device="cuda")
with sf.Sphereflake(W, H) as s:
    s.SetCamera(sf.config_camera(W, H, K))
    assert s.slab_bytes() == 4
    s.Render(band_rows=band, band_count=N, band_index=0)
    for k in range(1, N):
        s.render_to(stage[k - 1].data_ptr(), 0, band_rows=band, band_count=N, band_index=k, compact=True, packed=2)
    s.Synchronize()
    for _ in range(5):
        s.unpack_slabs(stage.data_ptr(), 4, stage_rows, band, N, 1, N - 1)
    s.Synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # (a stream of torch's own -- its default stream is handle 0, which the C ABI reads as "the context's stream" --
    # so that the events bracket the unpacks)
    ts = torch.cuda.Stream()
    with torch.cuda.stream(ts):
        e0.record(ts)
        for _ in range(REPS):
            s.unpack_slabs(stage.data_ptr(), 4, stage_rows, band, N, 1, N - 1, stream=ts.cuda_stream)
        e1.record(ts)
    torch.cuda.synchronize()
    s.Synchronize()
    us = e0.elapsed_time(e1) * 1e3 / REPS
px = sum(rows[1:]) * W
gbs = px * 36 / (us * 1e-6) / 1e9
print(f"{W}x{H} K={K} N={N}: unpack of {px} pixels {us:.1f} us, {gbs:.0f} GB/s (36 B/pixel), {gbs / 8000:.3f} of 8 TB/s "
      f"[SF_UNPACK_V1={os.environ.get('SF_UNPACK_V1', '0')}]", flush=True)
