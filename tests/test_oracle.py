"""CPU: the oracle (C restatement of the reference hot path) against the golden vectors the
reference itself produced (tests/golden/, made by tests/golden/make_golden.py from
oracle/ref_harness.cpp compiled from /root/reference)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_frame, load_npz
from oracle import pyoracle
from sfcheck import FLT_MAX, aux_digests, bad_rows, row_digests, samples_arrays


@pytest.mark.parametrize("name", ["t1", "t2", "t3", "t4", "t5"])
def test_tiny_frames_bit_exact(name, lut):
    fx = load_npz(name)
    S = pyoracle.load_setup(name)
    r = pyoracle.render(S, lut=lut, threads=4)
    for k in ("pos4", "nrm4", "minT", "index", "depth"):
        assert np.array_equal(np.ascontiguousarray(r[k]).view(np.uint8), np.ascontiguousarray(fx[k]).view(np.uint8)), k


def test_c1_full_frame_digests(lut):
    """BASELINE configs[0] (640x360, default camera, depth 5): the whole frame, bit for bit."""
    fx = load_frame("c1")
    S = pyoracle.load_setup("c1")
    r = pyoracle.render(S, lut=lut)
    assert bad_rows(fx["row_digest_gbuf"], row_digests(r["pos4"], r["nrm4"])) == []
    assert bad_rows(fx["row_digest_aux"], aux_digests(r["minT"], r["index"])) == []
    st = fx["stats"]
    assert r["stats"]["max_depth"] == st["max_depth"] == 5
    assert r["stats"]["hits"] == st["hits"]
    assert np.float32(r["stats"]["closest"]) == np.float32(float.fromhex(st["closest"]))
    assert r["stats"]["nodes"] == st["nodes"] and r["stats"]["interior"] == st["interior"]


@pytest.mark.parametrize("name,nrows", [("c2", 24), ("c3", 16), ("c4", 6), ("c5", 2)])
def test_large_config_rows(name, nrows, lut):
    """Row subsets of the bigger configs (depth 6..10) against the reference's row digests and sampled pixels."""
    fx = load_frame(name)
    S = pyoracle.load_setup(name)
    step = fx["row_step"]
    n = len(fx["row_digest_gbuf"])
    ks = np.linspace(0, n - 1, nrows).astype(int)
    r = pyoracle.render(S, rows=ks * step, lut=lut)
    got = row_digests(r["pos4"], r["nrm4"])
    assert [fx["row_digest_gbuf"][k] for k in ks] == got
    assert [fx["row_digest_aux"][k] for k in ks] == aux_digests(r["minT"], r["index"])


def test_samples_consistent_with_digests():
    """Sampled pixels are internally consistent (hits have finite t and index, misses are zero)."""
    for name in ("c1", "c3", "c5"):
        s = samples_arrays(load_frame(name))
        miss = s["depth"] < 0
        assert np.all(s["pos"][miss] == 0) and np.all(s["minT"][miss] == np.float32(FLT_MAX))
        assert np.all(s["index"][miss] == 0xFFFFFFFF)
        assert np.all(s["minT"][~miss] < np.float32(FLT_MAX))


def test_rsqrtps_emulation_specials(lut):
    summ = json.load(open(os.path.join(GOLDEN, "rsqrtps_lut.json")))
    assert summ["mismatches"] == 0 and summ["low_bits_violations"] == 0
    for xin, xout in summ["special"].items():
        x = np.array([int(xin, 16)], np.uint32).view(np.float32)[0]
        y = np.array([pyoracle.rsqrtps(float(x), lut)], np.float32).view(np.uint32)[0]
        assert y == int(xout, 16), (xin, hex(y), xout)


def test_rsqrtps_scaling_law(lut):
    """rsqrtps(4x) == rsqrtps(x) / 2 across the normal range (the table's defining property)."""
    rng = np.random.default_rng(0)
    xs = rng.uniform(1.0, 4.0, 200).astype(np.float32)
    for x in xs:
        y = np.float32(pyoracle.rsqrtps(float(x), lut))
        for k in (-40, -3, 1, 5, 30):
            z = np.float32(pyoracle.rsqrtps(float(np.float32(x) * np.float32(4.0) ** k), lut))
            assert z == np.float32(y * np.float32(2.0) ** (-k))


def test_sobol_known_answers():
    """Sobol::Sample (Sobol.cpp:41-55) KATs for dims 0/1 from the reference. Counters >= 2^52 run past
    the 52 entries of a dimension into the next one's in the reference (out of the supported range)."""
    import ctypes
    j = json.load(open(os.path.join(GOLDEN, "sobol.json")))
    m = np.array(j["dim0"] + j["dim1"], np.uint32)
    L = pyoracle.lib()
    for idx, dim, scr, v in j["samples"]:
        if idx >= 1 << 52:
            continue
        got = L.sfo_sobol_sample(idx, dim, scr, m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        assert np.float32(got) == np.float32(float.fromhex(v)), (idx, dim, scr)


@pytest.mark.skipif(not pyoracle.ref_available(), reason="reference build (oracle/_ref) only exists in the build container")
@pytest.mark.parametrize("W,H,K", [(96, 54, 1.0), (64, 40, 0.25), (48, 27, 0.2)])
def test_oracle_matches_reference_binary(W, H, K, lut):
    """Where the reference itself is built (oracle/_ref), the oracle equals it on fresh frames."""
    import subprocess
    S = json.loads(subprocess.check_output([os.path.join(pyoracle.REF_DIR, "ref_harness"), "setup", str(W), str(H), repr(K)]))
    setup = {k: (np.array([float.fromhex(v) for v in np.ravel(S[k])], np.float32).reshape(np.shape(S[k])) if k in
                 ("children", "root", "origin", "tl", "tr", "bl") else S[k]) for k in S}
    setup["W"], setup["H"] = W, H
    ref = pyoracle.ref_render(W, H, K)
    r = pyoracle.render(setup, lut=lut)
    assert np.array_equal(r["pos4"][..., :3].view(np.uint32), ref["pos"].view(np.uint32))
    assert np.array_equal(r["nrm4"][..., :3].view(np.uint32), ref["nrm"].view(np.uint32))
    assert np.array_equal(r["minT"].view(np.uint32), ref["minT"].view(np.uint32))
    assert r["stats"]["max_depth"] == ref["stats"]["max_depth"]


# ---- the reference's SSE variant (__ARCH_NO_AVX, LOD constant 60)

@pytest.mark.parametrize("name", ["s1", "s2"])
def test_sse_variant_tiny_frames_bit_exact(name, lut):
    fx = load_npz(name)
    r = pyoracle.render(pyoracle.load_setup(name), lut=lut, threads=4, lod=60.0)
    for k in ("pos4", "nrm4", "minT", "index", "depth"):
        assert np.array_equal(np.ascontiguousarray(r[k]).view(np.uint8), np.ascontiguousarray(fx[k]).view(np.uint8)), k


@pytest.mark.parametrize("name,nrows", [("s3", 40), ("s4", 12)])
def test_sse_variant_rows(name, nrows, lut):
    fx = load_frame(name)
    assert fx["variant"] == "sse"
    rows = np.linspace(0, fx["H"] - 1, nrows).astype(int)
    r = pyoracle.render(pyoracle.load_setup(name), rows=rows, lut=lut, lod=60.0)
    exp = [fx["row_digest_gbuf"][k] for k in rows]
    assert bad_rows(exp, row_digests(r["pos4"], r["nrm4"])) == []


def test_sse_and_avx_variants_differ():
    """The LOD constant changes the image: the same camera renders differently under 60 and 70."""
    assert load_frame("s4")["frame_digest"] != load_frame("c3")["frame_digest"]
