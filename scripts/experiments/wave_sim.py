#!/usr/bin/env python3
"""Drive wave_sim.c: the product kernel's wave-coherent traversal modelled on the CPU, its work counted per depth
(experiment, not product). Usage: wave_sim.py [setup=c3] [tile_step=1] [mode=0 ...]"""
import ctypes
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle  # noqa: E402

SO = "/tmp/wave_sim.so"
subprocess.check_call(["gcc", "-O2", "-mno-fma", "-ffp-contract=off", "-shared", "-fPIC", "-o", SO,
                       os.path.join(HERE, "wave_sim.c"), "-lm"])
L = ctypes.CDLL(SO)
NST = 32
FIELDS = ["exp", "iter", "miss", "lodnone", "occlnone", "entered", "leaf", "push", "act", "hitl"]
TAIL = ["tiles", "mismatch", "ties", "maxd"]


class Stats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_longlong * NST) for f in FIELDS] + [(f, ctypes.c_longlong) for f in TAIL] + \
               [("cone_tested", ctypes.c_longlong * NST), ("cone_culled", ctypes.c_longlong * NST),
                ("skip_exp", ctypes.c_longlong * NST), ("skip_lost", ctypes.c_longlong * NST),
                ("cache_hit", ctypes.c_longlong * NST)]


fp = ctypes.POINTER(ctypes.c_float)
up = ctypes.POINTER(ctypes.c_uint32)
L.wsim_tiles.argtypes = [ctypes.c_uint32, ctypes.c_uint32, fp, fp, fp, fp, fp, fp, up, fp, ctypes.c_uint32,
                         ctypes.c_uint32, ctypes.c_int, fp, up, ctypes.POINTER(Stats), ctypes.c_int, ctypes.c_int,
                         ctypes.POINTER(ctypes.c_double)]
L.wsim_depth8.argtypes = [ctypes.c_float, fp]


def run(name="c3", tile_step=1, mode=0, check=True, split=(0, 0)):
    s = pyoracle.load_setup(name)
    W, H = int(s["W"]), int(s["H"])
    lut = np.ascontiguousarray(pyoracle.load_lut(), np.uint32)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)
    o, tl, tr, bl, root, child = (f32(s[k]) for k in ("origin", "tl", "tr", "bl", "root", "children"))
    child = child.reshape(-1)
    d8 = np.zeros(NST * 8, np.float32)
    L.wsim_depth8(70.0, d8.ctypes.data_as(fp))
    tw, th = (W + 7) // 8, (H + 7) // 8
    trows = list(range(0, th, tile_step))
    ref_m = ref_i = None
    if check:
        rows = np.arange(H)
        ref = pyoracle.render(s, rows=rows)
        ref_m = np.ascontiguousarray(ref["minT"], np.float32)
        ref_i = np.ascontiguousarray(ref["index"], np.uint32)
    parts = [Stats() for _ in trows]
    works = [np.zeros(3 * tw) for _ in trows]

    def work(k):
        ty = trows[k]
        L.wsim_tiles(W, H, o.ctypes.data_as(fp), tl.ctypes.data_as(fp), tr.ctypes.data_as(fp), bl.ctypes.data_as(fp),
                     root.ctypes.data_as(fp), child.ctypes.data_as(fp), lut.ctypes.data_as(up), d8.ctypes.data_as(fp),
                     ty * tw, (ty + 1) * tw, mode,
                     ref_m.ctypes.data_as(fp) if check else None, ref_i.ctypes.data_as(up) if check else None,
                     ctypes.byref(parts[k]), split[0], split[1], works[k].ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(work, range(len(trows))))
    tot = {f: np.sum([np.array(getattr(p, f)[:]) for p in parts], 0) for f in FIELDS + ["cone_tested", "cone_culled", "skip_exp", "skip_lost", "cache_hit"]}
    for f in TAIL:
        tot[f] = max(getattr(p, f) for p in parts) if f == "maxd" else sum(getattr(p, f) for p in parts)
    tot["scale"] = tile_step
    tot["tile_work"] = np.concatenate(works).reshape(-1, 3)
    return tot


def report(t, label=""):
    sc = t["scale"]
    print(f"{label} tiles {t['tiles']} mismatch {t['mismatch']} ties {t['ties']} maxd {t['maxd']} (x{sc} for frame)")
    print(" d   exp     iter    miss   lodnone occlnone entered  leaf    push   act/it  cone-cull skip-exp lost")
    for d in range(NST):
        if t["exp"][d] == 0:
            continue
        it = t["iter"][d]
        print(f"{d:2d} {t['exp'][d]*sc:7d} {it*sc:8d} {t['miss'][d]*sc:7d} {t['lodnone'][d]*sc:7d} {t['occlnone'][d]*sc:7d}"
              f" {t['entered'][d]*sc:7d} {t['leaf'][d]*sc:7d} {t['push'][d]*sc:7d} {t['act'][d]/max(it,1):6.1f}"
              f"  {t['cone_culled'][d]/max(t['cone_tested'][d],1):.3f}  {t['skip_exp'][d]*sc:7d} {t['skip_lost'][d]*sc:6d}"
              f"  hit {t['cache_hit'][d]/max(t['exp'][d],1):.2f}")
    tot = lambda f: int(t[f].sum()) * sc
    print(f"all {tot('exp'):8d} {tot('iter'):8d} {tot('miss'):7d} {tot('lodnone'):7d} {tot('occlnone'):7d} {tot('entered'):7d}"
          f" {tot('leaf'):7d} {tot('push'):7d} {t['act'].sum()/max(t['iter'].sum(),1):6.1f}")


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    modes = [int(m) for m in sys.argv[3:]] or [0]
    for m in modes:
        report(run(name, step, m, check=(step == 1)), f"{name} mode {m}:")
