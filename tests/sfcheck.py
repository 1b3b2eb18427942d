"""Digest helpers shared by the parity tests (same definitions as tests/golden/make_golden.py)."""
import hashlib

import numpy as np

FLT_MAX = float(np.finfo(np.float32).max)


def row_digests(pos4, nrm4):
    return [hashlib.sha256(np.ascontiguousarray(pos4[k]).tobytes() +
                           np.ascontiguousarray(nrm4[k]).tobytes()).hexdigest()[:16]
            for k in range(pos4.shape[0])]


def aux_digests(min_t, index):
    return [hashlib.sha256(np.ascontiguousarray(min_t[k]).tobytes() +
                           np.ascontiguousarray(index[k]).astype(np.uint32).tobytes()).hexdigest()[:16]
            for k in range(min_t.shape[0])]


def frame_digest(pos4, nrm4):
    h = hashlib.sha256()
    for k in range(pos4.shape[0]):
        h.update(np.ascontiguousarray(pos4[k]).tobytes())
        h.update(np.ascontiguousarray(nrm4[k]).tobytes())
    return h.hexdigest()


def bad_rows(expected, got):
    return [k for k, (a, b) in enumerate(zip(expected, got)) if a != b]


def samples_arrays(fx):
    """Sampled pixels of a frame fixture -> dict of numpy arrays."""
    s = fx["samples"]
    f = lambda col: np.array([float.fromhex(r[col]) for r in s], np.float32)
    return {
        "x": np.array([r[0] for r in s]), "y": np.array([r[1] for r in s]),
        "pos": np.stack([f(2), f(3), f(4)], -1), "nrm": np.stack([f(5), f(6), f(7)], -1),
        "minT": f(8), "index": np.array([r[9] for r in s], np.uint64).astype(np.uint32),
        "depth": np.array([r[10] for r in s]),
    }
