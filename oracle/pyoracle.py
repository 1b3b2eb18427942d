"""TEST INFRASTRUCTURE ONLY -- ctypes front-end of the CPU oracle (oracle/sf_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker. The product path (sphereflake-raytracer_amd/)
never imports it.

The oracle is a per-ray restatement of the reference hot path
(/root/reference/sphereflake/Sphereflake.h:86-226, SIMD_AVX.h:59-81,163-180,236-270,
Sphereflake.cpp:149-201). It is pinned bit-for-bit against frames rendered by the
reference itself (oracle/ref_harness.cpp): see tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(REPO, "tests", "golden")
LIB_PATH = os.path.join(HERE, "build", "libsf_oracle.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build() -> None:
    """Compile the C restatement (gcc only; no reference sources needed)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        up = ctypes.POINTER(ctypes.c_uint32)
        L.sfo_render_rows.argtypes = [ctypes.c_uint32, ctypes.c_uint32, fp, fp, fp, fp, fp, fp, up,
                                      ctypes.c_uint32, ctypes.c_uint32, fp, fp, fp, up,
                                      ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(ctypes.c_longlong), fp]
        L.sfo_render_rows.restype = ctypes.c_int
        L.sfo_rsqrtps.argtypes = [ctypes.c_float, up]
        L.sfo_rsqrtps.restype = ctypes.c_float
        L.sfo_normalize.argtypes = [fp, up]
        L.sfo_sobol_sample.argtypes = [ctypes.c_ulonglong, ctypes.c_uint, ctypes.c_uint, up]
        L.sfo_sobol_sample.restype = ctypes.c_float
        _lib = L
    return _lib


def load_lut() -> np.ndarray:
    return np.fromfile(os.path.join(GOLDEN, "rsqrtps_lut.bin"), dtype="<u4")


def hexfloats(vals) -> np.ndarray:
    return np.array([float.fromhex(v) for v in vals], dtype=np.float32)


def load_setup(name: str) -> dict:
    """Setup constants (camera corners, root, children) dumped from the reference."""
    with open(os.path.join(GOLDEN, f"setup_{name}.json")) as f:
        j = json.load(f)
    return {
        "W": j["W"], "H": j["H"], "K": float.fromhex(j["K"]),
        "children": np.stack([hexfloats(c) for c in j["children"]]),
        "root": hexfloats(j["root"]),
        "origin": hexfloats(j["origin"]), "tl": hexfloats(j["tl"]),
        "tr": hexfloats(j["tr"]), "bl": hexfloats(j["bl"]),
        "radius": hexfloats(j["radius"]),
    }


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def render(setup: dict, rows=None, threads: int | None = None, lut: np.ndarray | None = None,
           lod: float = 70.0) -> dict:
    """Per-ray oracle frame for the given rows (default: all). Returns numpy arrays
    pos4/nrm4 [n, W, 4] f32, minT [n, W] f32, index [n, W] u32, depth [n, W] i8, stats.
    lod: the LOD constant, 70 (AVX path, default) or 60 (SSE path, SIMD_SSE.h:21)."""
    L = lib()
    L.sfo_set_lod_constant.argtypes = [ctypes.c_float]
    L.sfo_set_lod_constant(ctypes.c_float(lod))
    W, H = int(setup["W"]), int(setup["H"])
    rows = np.arange(H) if rows is None else np.asarray(rows)
    n = len(rows)
    lut = load_lut() if lut is None else lut
    lut = np.ascontiguousarray(lut, dtype=np.uint32)
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    o, tl, tr, bl = f32(setup["origin"]), f32(setup["tl"]), f32(setup["tr"]), f32(setup["bl"])
    root, child = f32(setup["root"]), f32(setup["children"]).reshape(-1)
    pos = np.empty((n, W, 4), np.float32)
    nrm = np.empty((n, W, 4), np.float32)
    mint = np.empty((n, W), np.float32)
    idx = np.empty((n, W), np.uint32)
    dep = np.empty((n, W), np.int8)
    threads = threads or min(8, os.cpu_count() or 1)

    def work(k):
        y = int(rows[k])
        st = (ctypes.c_longlong * 4)()
        cl = ctypes.c_float()
        rc = L.sfo_render_rows(W, H, _fp(o), _fp(tl), _fp(tr), _fp(bl), _fp(root), _fp(child),
                               lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), y, y + 1,
                               _fp(pos[k]), _fp(nrm[k]), _fp(mint[k]),
                               idx[k].ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                               dep[k].ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), st, ctypes.byref(cl))
        assert rc == 0
        return list(st), cl.value

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(work, range(n)))
    stats = {
        "max_depth": max(r[0][0] for r in res) if res else 0,
        "hits": sum(r[0][1] for r in res),
        "nodes": sum(r[0][2] for r in res),
        "interior": sum(r[0][3] for r in res),
        "closest": min(r[1] for r in res) if res else float(np.finfo(np.float32).max),
        "rays": n * W,
    }
    return {"pos4": pos, "nrm4": nrm, "minT": mint, "index": idx, "depth": dep, "stats": stats}


def rsqrtps(x: float, lut: np.ndarray | None = None) -> float:
    lut = np.ascontiguousarray(load_lut() if lut is None else lut, dtype=np.uint32)
    return lib().sfo_rsqrtps(x, lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))


def ref_available() -> bool:
    return os.path.exists(os.path.join(REF_DIR, "ref_harness"))


def ref_render(W: int, H: int, K: float, row_step: int = 1, threads: int = 8, tmp: str = "/tmp",
               sse: bool = False) -> dict:
    """Run the reference itself (oracle/_ref/ref_harness, built from /root/reference; ref_harness_sse:
    the same sources built with __ARCH_NO_AVX). Returns pos/nrm (xyz) and minT for rows
    y % row_step == 0 plus its JSON stats."""
    path = os.path.join(tmp, f"sf_ref_{W}x{H}_{K}_{row_step}_{int(sse)}_{os.getpid()}.bin")
    out = subprocess.check_output([os.path.join(REF_DIR, "ref_harness_sse" if sse else "ref_harness"), "render",
                                   str(W), str(H), repr(K), path, str(threads), str(row_step)])
    stats = json.loads(out)
    n = (H + row_step - 1) // row_step
    a = np.fromfile(path, dtype=np.float32).reshape(n, W, 7)
    os.unlink(path)
    return {"pos": a[..., 0:3], "nrm": a[..., 3:6], "minT": a[..., 6], "stats": stats}


def ref_bench(W: int, H: int, K: float, threads: int, reps: int) -> dict:
    """Time the reference's own AVX packet path (oracle/_ref/ref_bench)."""
    out = subprocess.check_output([os.path.join(REF_DIR, "ref_bench"), "bench", str(W), str(H),
                                   repr(K), str(threads), str(reps)])
    return json.loads(out)
