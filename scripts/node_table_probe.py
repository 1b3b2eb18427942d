#!/usr/bin/env python3
"""The node table's rebuild per view (sf_node_table, multi-GPU receive side) timed with its unpack (diagnostics): 4-B
slabs of N - 1 members rendered once, then REPS unpacks each after a new view (the table is rebuilt whenever the
root transform changes), bracketed by HIP events; and the same with the view fixed (the unpack alone). The difference
per rep is the table's rebuild. Usage: node_table_probe.py [W H K N REPS]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sphereflake-raytracer_amd"))
sys.path.insert(0, REPO)
import sphereflake_amd as sf  # noqa: E402
from bench import frame_camera  # noqa: E402

W, H, K, N, REPS = ((int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
                    if len(sys.argv) > 5 else (1920, 1080, 0.25, 8, 40))
band = 8
rows = [sf.lib().sf_slab_rows(H, band, N, k) for k in range(N)]
stage_rows = max(rows[1:])
stage = torch.zeros((N - 1, stage_rows, W), dtype=torch.int32, device="cuda")
cams = [frame_camera(W, H, K, i) for i in range(REPS)]
with sf.Sphereflake(W, H) as s:
    s.SetCamera(cams[0])
    s.Render(band_rows=band, band_count=N, band_index=0)
    for k in range(1, N):
        s.render_to(stage[k - 1].data_ptr(), 0, band_rows=band, band_count=N, band_index=k, compact=True, packed=2)
    s.Synchronize()
    ts = torch.cuda.Stream()
    out = {}
    for moving in (False, True, False, True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        with torch.cuda.stream(ts):
            e0.record(ts)
            for i in range(REPS):
                if moving:
                    s.SetCamera(cams[i])
                s.unpack_slabs(stage.data_ptr(), 4, stage_rows, band, N, 1, N - 1, stream=ts.cuda_stream)
            e1.record(ts)
        torch.cuda.synchronize()
        out.setdefault(moving, []).append(e0.elapsed_time(e1) * 1e3 / REPS)
    s.Synchronize()
fixed, mov = min(out[False]), min(out[True])
print(f"{W}x{H} N={N}: unpack alone {fixed:.1f} us, with the table rebuilt per view {mov:.1f} us: table {mov - fixed:.1f} us",
      flush=True)
