"""CPU: the C-ABI library (built for gfx950) loads and exports every symbol include/sphereflake/sf.h
declares; the host setup math equals the reference's glm arithmetic bit for bit; per-depth
constants are exact. No compute calls need a GPU here."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, PKG, REPO
from oracle import pyoracle
import sphereflake_amd as sf

HEADER = os.path.join(REPO, "include", "sphereflake", "sf.h")


@pytest.fixture(scope="module", autouse=True)
def built():
    sf.build()
    return sf.lib()


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sf_[a-z_0-9]+)\s*\(", src)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 20
    L = sf.lib()
    for n in names:
        assert hasattr(L, n), f"{n} declared in sf.h but not exported"
    assert set(names) == set(sf.SIGNATURES), set(names) ^ set(sf.SIGNATURES)


def test_library_targets_gfx950():
    out = os.popen(f"/opt/rocm/lib/llvm/bin/llvm-objdump --offloading {sf.LIB_PATH} 2>/dev/null || true").read()
    blob = open(sf.LIB_PATH, "rb").read()
    assert b"gfx950" in blob or "gfx950" in out


def test_no_device_is_reported_cleanly():
    if sf.device_count() > 0:
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    assert sf.lib().sf_create(0, 64, 36, ctypes.byref(h)) == sf.SF_ENODEV
    with pytest.raises(sf.SphereflakeError):
        sf.Sphereflake(64, 36)


def test_abi_version_and_errors():
    assert sf.lib().sf_abi_version() == 1
    for code in range(0, -8, -1):
        assert sf.lib().sf_strerror(code)
    assert sf.lib().sf_render(None, None) == sf.SF_EINVAL


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4", "c5", "t4", "t5"])
def test_setup_matches_reference(name):
    """child frames (Sphereflake.cpp:216-249), root (Sphereflake.cpp:83), camera corners (camera.h:37-53)."""
    S = pyoracle.load_setup(name)
    assert np.array_equal(sf.child_transforms().view(np.uint32), S["children"].view(np.uint32))
    cam = sf.config_camera(S["W"], S["H"], S["K"])
    o, tl, tr, bl = cam.corners()
    for got, k in ((o, "origin"), (tl, "tl"), (tr, "tr"), (bl, "bl")):
        assert np.array_equal(got.view(np.uint32), S[k].view(np.uint32)), k
    assert np.array_equal(sf.root_transform(S["origin"]).view(np.uint32), S["root"].view(np.uint32))


def test_radius_chain_matches_reference():
    S = pyoracle.load_setup("c3")
    for d, r in enumerate(S["radius"]):
        assert np.float32(sf.depth_constants(d)[0]) == r


def test_lod_threshold_exact():
    """sqrtf(t/r) < 70 || t < 0  <=>  t < T_d (Sphereflake.h:146), checked on float32 arithmetic
    (numpy: correctly rounded div/sqrt) for every ulp around T_d and random t."""
    rng = np.random.default_rng(7)
    for d in range(0, 20):
        r, T = (np.float32(v) for v in sf.depth_constants(d))
        tb = np.array([T], np.float32).view(np.int32)[0]
        near = (np.arange(tb - 2000, tb + 2000, dtype=np.int32)).view(np.float32)
        rand = (rng.random(20000).astype(np.float32) * np.float32(3) * T).astype(np.float32)
        neg = -rand
        for t in (near, rand, neg):
            with np.errstate(invalid="ignore"):
                ref = (np.sqrt(t / r) < np.float32(70.0)) | (t < 0)
            assert np.array_equal(ref, t < T), d


def test_survey_lod_constants():
    """Values published in SURVEY.md Appendix A."""
    assert np.float32(sf.depth_constants(8)[1]) == np.float32(float.fromhex("0x1.7e6174p-1"))
    assert np.float32(sf.depth_constants(0)[1]) == np.float32(float.fromhex("0x1.323ffep+12"))


def test_embedded_lut_equals_golden(lut):
    txt = open(os.path.join(PKG, "csrc", "rsqrtps_lut.inc")).read()
    vals = [int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", txt)]
    assert np.array_equal(np.array(vals, np.uint32), lut)


def test_host_rsqrtps_matches_oracle(lut):
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.uniform(1e-30, 1e30, 3000), rng.uniform(0.5, 4, 3000), [0.0, 1.0, 4.0, 1e-40, np.inf]])
    for x in xs.astype(np.float32):
        a = np.float32(sf.rsqrtps(float(x)))
        b = np.float32(pyoracle.rsqrtps(float(x), lut))
        assert a.view(np.uint32) == b.view(np.uint32), x


@pytest.mark.parametrize("H,band,n", [(1080, 8, 8), (1080, 64, 3), (45, 8, 2), (7, 8, 4), (16384, 8, 8)])
def test_slab_rows_partition_frame(H, band, n):
    rows = [sf.lib().sf_slab_rows(H, band, n, i) for i in range(n)]
    assert sum(rows) == H


def test_sobol_direction_numbers_match_reference():
    """The device sampler's dims 0/1 (generated algorithmically in sf_setup.cpp) equal the reference table.
    Exposed through the progressive path only, so re-derive here exactly as sf_setup.cpp does."""
    j = json.load(open(os.path.join(GOLDEN, "sobol.json")))
    v, d1 = 0, []
    for k in range(52):
        v = 0x80000000 if k % 32 == 0 else v ^ (v >> 1)
        d1.append(v)
    d0 = [(0x80000000 >> k) if k < 32 else 0 for k in range(52)]
    assert d0 == j["dim0"] and d1 == j["dim1"]


def test_mt19937_known_answers():
    """std::mt19937(12345) + uniform_int_distribution<unsigned>(0) == raw MT outputs (what the device
    generator sf_mt_draws produces): restated in numpy against the libstdc++ fixture."""
    j = json.load(open(os.path.join(GOLDEN, "mt19937_seed12345.json")))
    mt = [0] * 624
    mt[0] = j["seed"]
    for i in range(1, 624):
        mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
    out, pos = [], 624
    while len(out) < len(j["draws"]):
        if pos == 624:
            for i in range(624):
                y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            pos = 0
        y = mt[pos]
        pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        out.append(y & 0xFFFFFFFF)
    assert out == j["draws"]


def test_save_ppm_layout(tmp_path):
    img = np.zeros((2, 3, 3), np.float32)
    img[0, 0] = (1.0, 0.5, 0.0)
    img[1, 2] = (2.0, -1.0, 0.25)   # clamped
    p = tmp_path / "x.ppm"
    sf.Sphereflake.save_ppm(str(p), img)
    b = p.read_bytes()
    head = b"P6 3 2 255\n"
    assert b[:len(head)] == head
    px = np.frombuffer(b[len(head):], np.uint8).reshape(2, 3, 3)
    assert tuple(px[0, 0]) == (255, 128, 0) and tuple(px[1, 2]) == (255, 0, 64)


def test_c_abi_ppm_pfm_writers(tmp_path):
    """Host-only writers behind sf_save_image (sf.h image dump): P6 drops alpha and keeps rows top first;
    PF writes little-endian float RGB rows bottom first; bad arguments are SF_EINVAL."""
    L = sf.lib()
    rgba = np.arange(2 * 3 * 4, dtype=np.uint8).reshape(2, 3, 4)
    p = tmp_path / "a.ppm"
    assert L.sf_write_ppm(str(p).encode(), 3, 2, rgba.ctypes.data) == 0
    head = b"P6\n3 2\n255\n"
    b = p.read_bytes()
    assert b[:len(head)] == head and b[len(head):] == rgba[:, :, :3].tobytes()
    v4 = np.random.default_rng(3).standard_normal((2, 3, 4)).astype(np.float32)
    q = tmp_path / "a.pfm"
    assert L.sf_write_pfm(str(q).encode(), 3, 2, v4.ctypes.data) == 0
    head = b"PF\n3 2\n-1.0\n"
    b = q.read_bytes()
    assert b[:len(head)] == head
    assert b[len(head):] == np.ascontiguousarray(v4[::-1, :, :3]).astype("<f4").tobytes()
    assert L.sf_write_ppm(None, 3, 2, rgba.ctypes.data) == sf.SF_EINVAL
    assert L.sf_write_pfm(str(q).encode(), 0, 2, v4.ctypes.data) == sf.SF_EINVAL
    assert L.sf_save_image(None, str(q).encode(), sf.SF_DUMP_NORMALS) == sf.SF_EINVAL


@pytest.mark.parametrize("c", [70.0, 60.0])
def test_lod_threshold_exact_both_variants(c):
    """sqrtf(t/r) < C || t < 0  <=>  t < T for the AVX (70) and SSE (60, SIMD_SSE.h:21) constants."""
    rng = np.random.default_rng(11)
    for d in range(0, 16):
        r = np.float32(sf.depth_constants(d)[0])
        T = np.float32(sf.lod_threshold(float(r), c))
        tb = np.array([T], np.float32).view(np.int32)[0]
        near = (np.arange(tb - 500, tb + 500, dtype=np.int32)).view(np.float32)
        rand = (rng.random(5000).astype(np.float32) * np.float32(3) * T).astype(np.float32)
        for t in (near, rand, -rand):
            with np.errstate(invalid="ignore"):
                ref = (np.sqrt(t / r) < np.float32(c)) | (t < 0)
            assert np.array_equal(ref, t < T), (c, d)
    r1, T1 = sf.depth_constants(1)
    assert sf.lod_threshold(r1, 70.0) == T1


@pytest.mark.parametrize("seed,advance,steps", [(12345, 0, 1000), (777, 5, 70000), (1, 623, 624 * 3 + 5),
                                               (9, 100, 3), (42, 624, 0), (3, 0, 524288), (5, 311, 1 << 33)])
def test_mt19937_jump_matches_generator(seed, advance, steps):
    """sf_mt19937_jump (t^m mod the generator's characteristic polynomial, phi from Berlekamp-Massey) gives
    the std::mt19937 stream `steps` draws on, checked against numpy's MT19937 (legacy seeding = std::mt19937's
    init_genrand) stepped draw by draw (for 2^33 only the polynomial path runs: checked by its next draws
    equalling a 2^32 + 2^32 jump)."""
    import ctypes
    from numpy.random import MT19937
    from sphereflake_amd import lib
    P = ctypes.POINTER(ctypes.c_uint32)

    def state(g):
        st = g.state["state"]
        return np.concatenate([st["key"].astype(np.uint32), np.array([st["pos"]], np.uint32)])

    def jump(s, n):
        out = np.zeros(625, np.uint32)
        assert lib().sf_mt19937_jump(s.ctypes.data_as(P), n, out.ctypes.data_as(P)) == 0
        return out

    def gen(s):
        g = MT19937(0)
        st = g.state
        st["state"]["key"] = s[:624].copy()
        st["state"]["pos"] = int(s[624])
        g.state = st
        return g

    g = MT19937(0)
    g._legacy_seeding(seed)
    if advance:
        g.random_raw(advance)
    s0 = state(g)
    out = jump(s0, steps)
    if steps < (1 << 32):
        if steps:
            g.random_raw(steps)
        assert np.array_equal(g.random_raw(1500), gen(out).random_raw(1500))
    else:
        half = jump(jump(s0, steps // 2), steps // 2)
        assert np.array_equal(gen(half).random_raw(1500), gen(out).random_raw(1500))


def _rn32(fr):
    """Fraction -> the nearest float32 (ties to even), exactly."""
    from fractions import Fraction
    f = np.float32(float(fr))
    best = None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        e = abs(Fraction(float(c)) - fr)
        key = (e, int(np.array([c], np.float32).view(np.uint32)[0]) & 1)
        if best is None or key < best[0]:
            best = (key, c)
    return np.float32(best[1])


@pytest.mark.parametrize("n", [640, 360, 1280, 720, 1920, 1080, 3840, 2160, 16384, 96, 64, 37, 1, 2, 3])
def test_division_by_reciprocal_exact(n):
    """Ray generation forms u = x / W (Sphereflake.cpp:149-150) as q0 = RN(x y), y = RN(1/W), corrected by one fma
    residual: q = RN(q0 + RN(x - q0 W) y). sf_division_by_reciprocal_exact(W) (the library's host check, run at
    sf_create) says it equals RN(x / W) for every x in [0, W]; here an independent exact-rational restatement
    agrees on a sample of x, and the library reports 1 for every BASELINE frame size."""
    from fractions import Fraction
    assert sf.lib().sf_division_by_reciprocal_exact(n) == 1
    fn = np.float32(n)
    y = np.float32(1.0) / fn
    rng = np.random.default_rng(n)
    xs = np.unique(np.concatenate([np.arange(0, min(n, 300) + 1), rng.integers(0, n + 1, 300), [n - 1, n]]))
    for x in xs:
        fx = np.float32(x)
        q0 = np.float32(fx * y)
        r = _rn32(Fraction(int(x)) - Fraction(float(q0)) * n)          # fma(-q0, n, x)
        q = _rn32(Fraction(float(q0)) + Fraction(float(r)) * Fraction(float(y)))   # fma(r, y, q0)
        assert q == np.float32(fx / fn), (n, x)


@pytest.mark.parametrize("v", [(0.1, -2.5, 3e38), [np.float32(1.1), 2, -0.0], np.array([1.1, 2.0, 3.0]),
                               np.array([[1e39], [-1e-46], [7.0]]), np.array([0.3, 0.2, 0.1], np.float32),
                               (float("nan"), float("inf"), -1.0)])
def test_view_vector_conversion_matches_float32(v):
    """SetView's ctypes float[3] (sphereflake_amd._vec3, no numpy on the per-frame path) holds exactly the
    float32 values np.float32 conversion gives (round to nearest, overflow to inf, underflow to 0)."""
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        exp = np.asarray(v, np.float32).ravel()
    got = np.array(list(sf._vec3(v)), np.float32)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


@pytest.mark.parametrize("v", [(1.0, 2.0), [1.0, 2.0, 3.0, 4.0], np.zeros(4), np.zeros((2, 2))])
def test_view_vector_conversion_rejects_wrong_size(v):
    with pytest.raises(ValueError):
        sf._vec3(v)
