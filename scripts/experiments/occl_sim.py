#!/usr/bin/env python3
"""Drive occl_sim.c: plain vs occlusion-culling per-ray traversal on a BASELINE setup (CPU, experiment).
Usage: occl_sim.py [setup=c3] [row_step=4]"""
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

SO = "/tmp/occl_sim.so"
subprocess.check_call(["gcc", "-O2", "-mno-fma", "-ffp-contract=off", "-shared", "-fPIC", "-o", SO,
                       os.path.join(HERE, "occl_sim.c"), "-lm"])
L = ctypes.CDLL(SO)
fp = ctypes.POINTER(ctypes.c_float)
up = ctypes.POINTER(ctypes.c_uint32)
L.sim_rows.argtypes = [ctypes.c_uint32, ctypes.c_uint32, fp, fp, fp, fp, fp, fp, up, ctypes.c_uint32,
                       ctypes.c_uint32, ctypes.c_float, ctypes.c_int, fp, up, ctypes.POINTER(ctypes.c_longlong)]

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 4
s = pyoracle.load_setup(name)
W, H = int(s["W"]), int(s["H"])
rows = np.arange(0, H, step)
lut = np.ascontiguousarray(pyoracle.load_lut(), np.uint32)
f32 = lambda a: np.ascontiguousarray(a, np.float32)
o, tl, tr, bl, root, child = (f32(s[k]) for k in ("origin", "tl", "tr", "bl", "root", "children"))
child = child.reshape(-1)
ref = pyoracle.render(s, rows=rows)


def run(margin, mode):
    mint = np.empty((len(rows), W), np.float32)
    idx = np.empty((len(rows), W), np.uint32)
    st = np.zeros((len(rows), 4), np.int64)

    def work(k):
        y = int(rows[k])
        L.sim_rows(W, H, o.ctypes.data_as(fp), tl.ctypes.data_as(fp), tr.ctypes.data_as(fp), bl.ctypes.data_as(fp),
                   root.ctypes.data_as(fp), child.ctypes.data_as(fp), lut.ctypes.data_as(up), y, y + 1,
                   ctypes.c_float(margin), mode, mint[k].ctypes.data_as(fp), idx[k].ctypes.data_as(up),
                   st[k].ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)))
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(work, range(len(rows))))
    return mint, idx, st


m0, i0, s0 = run(-1.0, 0)
print(f"fast LOD decisions: violations {s0[:, 1].sum()}, band lanes {s0[:, 2].sum()} of {s0[:, 3].sum()} bounding hits")
same_plain = np.array_equal(m0.view(np.uint32), ref["minT"].view(np.uint32)) and np.array_equal(i0, ref["index"])
print(f"{name} {W}x{H} rows/{step}: pre-order plain == oracle: {same_plain}; max depth {s0[:, 0].max()} "
      f"(oracle {ref['stats']['max_depth']}); tests {s0[:, 1].sum()} expansions {s0[:, 2].sum()}")
for mode in ():
    for lg in (7,):
        m, i, st = run(2.0 ** -lg, mode)
        ok = np.array_equal(m.view(np.uint32), m0.view(np.uint32)) and np.array_equal(i, i0)
        print(f"  mode {mode} margin 2^-{lg}: exact {ok} max depth {st[:, 0].max()}  tests {st[:, 1].sum() / s0[:, 1].sum():.3f}"
              f"  expansions {st[:, 2].sum() / s0[:, 2].sum():.3f}  culled {st[:, 3].sum()}")

L.sim_tile_row.argtypes = [ctypes.c_uint32, ctypes.c_uint32, fp, fp, fp, fp, fp, fp, up, ctypes.c_uint32,
                           ctypes.c_float, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
trows = np.arange(0, (H + 7) // 8, max(1, step // 2))


def tiles(margin, mode):
    st = np.zeros((len(trows), 80), np.int64)

    def work(k):
        L.sim_tile_row(W, H, o.ctypes.data_as(fp), tl.ctypes.data_as(fp), tr.ctypes.data_as(fp), bl.ctypes.data_as(fp),
                       root.ctypes.data_as(fp), child.ctypes.data_as(fp), lut.ctypes.data_as(up), int(trows[k]),
                       ctypes.c_float(margin), mode, st[k].ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)))
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(work, range(len(trows))))
    return st.sum(0) if not (mode & 64) else st


t0 = tiles(-1.0, 0)
if len(sys.argv) > 3 and sys.argv[3] == "cone":
    st = tiles(3 * 2.0 ** -10, 17 | 64).sum(0)
    print("depth: children tested at unique expansions, cone-culled share; at |c| sinT > 4R: share of those children, culled share")
    for k in range(12):
        n, c = st[3 + k], st[19 + k]
        if n:
            print(f"  depth {k}: {n:9d} culled {c / n:.3f}")
    names = ["<=2", "<=4", "<=8", "<=16", "<=32", ">32"]
    tot = st[67:79].sum()
    print("unique expanded nodes by lanes that expand them (cone useful | cone useless, |c| sinT >= R):")
    for b in range(6):
        print(f"  {names[b]:>5} lanes: {st[67 + 2 * b] / tot:.3f} | {st[67 + 2 * b + 1] / tot:.3f}")
    print("by |c| sinT / r (the node's radius):")
    for k in range(16):
        wn, wc = st[35 + k], st[51 + k]
        if wn:
            print(f"  [2^{k - 8}, 2^{k - 7}): {wn:9d} children, culled {wc / wn:.3f}")
    sys.exit(0)
print(f"tiles (every {max(1, step // 2)}th tile row): wave expansions (union over the tile) {t0[0]}, per-lane {t0[1]}")
for mode, lg in ((17, 7), (17, 8.415), (17, 9)):
    t = tiles(2.0 ** -lg, mode)
    print(f"  mode {mode} margin 2^-{lg}: wave expansions {t[0] / t0[0]:.3f}  per-lane {t[1] / t0[1]:.3f}  non-ancestor ties {t[2]}")
