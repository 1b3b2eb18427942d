#!/usr/bin/env python3
"""Generate the committed parity fixtures under tests/golden/.

Runs ONLY in the build container, where /root/reference exists:
  1. oracle/_ref/gen_rsqrtps_lut measures x86 rsqrtps -> rsqrtps_lut.bin (+ summary json)
  2. oracle/_ref/ref_harness (the reference sources compiled with pinned IEEE flags)
     dumps setup constants and renders per-ray frames for every config
  3. the C restatement (oracle/sf_oracle.c) renders the same rows; the script
     ABORTS unless it equals the reference bit-for-bit (pos, nrm, minT) -- that
     gate is what lets the heap hit index (which the reference does not expose)
     come from the restatement
  4. writes per-row SHA-256 digests, sampled pixels, stats, tiny full frames,
     Sobol and mt19937 known answers.

Usage: python tests/golden/make_golden.py [--only NAME ...]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import pyoracle  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")

# name -> (W, H, K, row_step, n_samples). K scales the camera position of
# reference main.cpp:92-96 so the reference's own LOD rule reaches the config
# depth.
CONFIGS = {
    "c1": (640, 360, 1.0, 1, 4096),        # BASELINE configs[0]: 640x360 default depth (5)
    "c2": (1280, 720, 0.8, 1, 4096),       # configs[1]: depth 6
    "c3": (1920, 1080, 0.25, 1, 4096),     # configs[2]: depth 8 (north star)
    "c4": (3840, 2160, 0.22, 1, 4096),     # configs[3]: depth 9
    "c5": (16384, 16384, 0.2, 64, 4096),   # configs[4]: depth 10, rows y % 64 == 0
    # tiny / ragged frames, stored whole
    "t1": (64, 36, 1.0, 1, 0),
    "t2": (64, 36, 0.25, 1, 0),
    "t3": (80, 45, 0.22, 1, 0),
    "t4": (13, 7, 0.2, 1, 0),
    "t5": (1, 1, 0.25, 1, 0),
}


def hx(a) -> list:
    return [float(v).hex() for v in np.asarray(a, dtype=np.float32).reshape(-1)]


def row_digests(pos4, nrm4, mint, idx):
    g, a = [], []
    for k in range(pos4.shape[0]):
        g.append(hashlib.sha256(pos4[k].tobytes() + nrm4[k].tobytes()).hexdigest()[:16])
        a.append(hashlib.sha256(mint[k].tobytes() + idx[k].tobytes()).hexdigest()[:16])
    return g, a


def frame_digest(pos4, nrm4):
    h = hashlib.sha256()
    for k in range(pos4.shape[0]):
        h.update(pos4[k].tobytes())
        h.update(nrm4[k].tobytes())
    return h.hexdigest()


def run_json(args):
    return json.loads(subprocess.check_output(args))


def gen_lut():
    out = os.path.join(HERE, "rsqrtps_lut.bin")
    summ = run_json([os.path.join(REF, "gen_rsqrtps_lut"), out])
    assert summ["mismatches"] == 0 and summ["low_bits_violations"] == 0, summ
    with open(os.path.join(HERE, "rsqrtps_lut.json"), "w") as f:
        json.dump(summ, f, indent=1)
    print("lut:", summ)


def gen_setup(name, W, H, K):
    out = subprocess.check_output([os.path.join(REF, "ref_harness"), "setup", str(W), str(H), repr(K)])
    j = json.loads(out)
    with open(os.path.join(HERE, f"setup_{name}.json"), "w") as f:
        json.dump(j, f, indent=1)
    return pyoracle.load_setup(name)


def gen_frame(name, W, H, K, step, nsamp, sse=False):
    setup = gen_setup(name, W, H, K)
    ref = pyoracle.ref_render(W, H, K, row_step=step, threads=8, sse=sse)
    rows = np.arange(0, H, step)
    orc = pyoracle.render(setup, rows=rows, threads=8, lod=60.0 if sse else 70.0)
    # --- gate: restatement == reference, bit for bit
    for key, rk in (("pos4", "pos"), ("nrm4", "nrm")):
        a = orc[key][..., :3].view(np.uint32)
        b = np.ascontiguousarray(ref[rk]).view(np.uint32)
        bad = int((a != b).any(axis=-1).sum())
        assert bad == 0, f"{name}: oracle {key} differs from reference on {bad} pixels"
    bad = int((orc["minT"].view(np.uint32) != np.ascontiguousarray(ref["minT"]).view(np.uint32)).sum())
    assert bad == 0, f"{name}: oracle minT differs from reference on {bad} pixels"
    assert orc["stats"]["max_depth"] == ref["stats"]["max_depth"], (orc["stats"], ref["stats"])
    assert orc["stats"]["hits"] == ref["stats"]["hits"]
    # reference G-buffer layout: vec4(pos, 1), vec4(nrm, 1) (Sphereflake.cpp:186-196)
    pos4, nrm4 = orc["pos4"], orc["nrm4"]
    g, a = row_digests(pos4, nrm4, orc["minT"], orc["index"])
    fx = {
        "name": name, "W": W, "H": H, "K": float(np.float32(K)).hex(), "row_step": step,
        "variant": "sse" if sse else "avx",
        "stats": {
            "max_depth": ref["stats"]["max_depth"], "closest": ref["stats"]["closest"],
            "hits": ref["stats"]["hits"], "rays": int(len(rows) * W),
            "nodes": orc["stats"]["nodes"], "interior": orc["stats"]["interior"],
            "max_hit_index": int(orc["index"][orc["depth"] >= 0].max()) if ref["stats"]["hits"] else None,
            "max_hit_depth": int(orc["depth"].max()),
        },
        "frame_digest": frame_digest(pos4, nrm4),
        "row_digest_gbuf": g, "row_digest_aux": a,
    }
    if nsamp:
        rng = np.random.default_rng(1234)
        n = len(rows)
        # half uniformly random pixels, half random HIT pixels (the interesting ones)
        ys = rng.integers(0, n, nsamp // 2)
        xs = rng.integers(0, W, nsamp // 2)
        hit_k, hit_x = np.nonzero(orc["depth"] >= 0)
        sel = rng.integers(0, len(hit_k), nsamp - nsamp // 2) if len(hit_k) else np.zeros(0, int)
        ys = np.concatenate([ys, hit_k[sel]])
        xs = np.concatenate([xs, hit_x[sel]])
        samples = []
        for k, x in zip(ys.tolist(), xs.tolist()):
            samples.append([int(x), int(rows[k])] + hx(pos4[k, x, :3]) + hx(nrm4[k, x, :3]) +
                           hx(orc["minT"][k, x]) + [int(orc["index"][k, x]), int(orc["depth"][k, x])])
        fx["samples"] = samples
    with open(os.path.join(HERE, f"frame_{name}.json"), "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    if not nsamp:  # tiny frames: store everything
        np.savez_compressed(os.path.join(HERE, f"frame_{name}.npz"), pos4=pos4, nrm4=nrm4,
                            minT=orc["minT"], index=orc["index"], depth=orc["depth"])
    print(name, fx["stats"])


# frame-less progressive mode: name -> (W, H, K, seed, packets)
PROGRESSIVE = {
    "p1": (64, 36, 0.25, 1, 3000),          # dense: every pixel overwritten many times
    "p2": (640, 360, 1.0, 12345, 100000),
    "p3": (1920, 1080, 0.25, 777, 200000),
    "p4": (160, 90, 0.15, 4242, 6000),     # camera inside the root's bounding sphere: packets with t < 0
    "p5": (320, 180, 0.2, 99, 20000),      # ... and deeper (LOD) levels
}


def gen_progressive(name, W, H, K, seed, packets, sse=False):
    path = f"/tmp/sf_prog_{name}.bin"
    st = run_json([os.path.join(REF, "ref_harness_sse" if sse else "ref_harness"), "progressive", str(W), str(H),
                   repr(K), str(seed), str(packets), path])
    a = np.fromfile(path, dtype=np.float32)
    os.unlink(path)
    pos4 = a[: 4 * W * H].reshape(H, W, 4)
    nrm4 = a[4 * W * H:].reshape(H, W, 4)
    g = [hashlib.sha256(pos4[y].tobytes() + nrm4[y].tobytes()).hexdigest()[:16] for y in range(H)]
    fx = {"name": name, "W": W, "H": H, "K": float(np.float32(K)).hex(), "seed": seed, "packets": packets,
          "variant": "sse" if sse else "avx",
          "stats": st, "frame_digest": frame_digest(pos4, nrm4), "row_digest_gbuf": g,
          "written": int((pos4[..., 3] == 1.0).sum())}
    with open(os.path.join(HERE, f"progressive_{name}.json"), "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    print(name, st, fx["written"])


# The reference's SSE variant (__ARCH_NO_AVX: LOD constant 60, 4-lane packets,
# 2x2 frame-less footprint): same cameras as above.
SSE_CONFIGS = {
    "s1": (64, 36, 1.0, 1, 0),
    "s2": (80, 45, 0.22, 1, 0),
    "s3": (640, 360, 1.0, 1, 4096),
    "s4": (1920, 1080, 0.25, 1, 4096),
}
SSE_PROGRESSIVE = {
    "ps1": (64, 36, 0.25, 1, 3000),
    "ps2": (640, 360, 1.0, 12345, 100000),
    "ps3": (160, 90, 0.15, 4242, 6000),
    "ps4": (320, 180, 0.2, 99, 20000),
}


def gen_sobol_mt():
    j = run_json([os.path.join(REF, "ref_harness"), "sobol"])
    with open(os.path.join(HERE, "sobol.json"), "w") as f:
        json.dump(j, f, indent=0)
    j = run_json([os.path.join(REF, "ref_harness"), "mt", "12345", "256"])
    with open(os.path.join(HERE, "mt19937_seed12345.json"), "w") as f:
        json.dump(j, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all", "ref"])
    if not args.only or "lut" in args.only:
        gen_lut()
    if not args.only or "sobol" in args.only:
        gen_sobol_mt()
    for name, (W, H, K, step, nsamp) in CONFIGS.items():
        if args.only and name not in args.only:
            continue
        gen_frame(name, W, H, K, step, nsamp)
    for name, cfg in PROGRESSIVE.items():
        if args.only and name not in args.only:
            continue
        gen_progressive(name, *cfg)
    for name, (W, H, K, step, nsamp) in SSE_CONFIGS.items():
        if args.only and name not in args.only:
            continue
        gen_frame(name, W, H, K, step, nsamp, sse=True)
    for name, cfg in SSE_PROGRESSIVE.items():
        if args.only and name not in args.only:
            continue
        gen_progressive(name, *cfg, sse=True)


if __name__ == "__main__":
    main()
