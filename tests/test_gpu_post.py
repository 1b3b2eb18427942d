"""GPU parity of the SSAO post-process kernels (csrc/sf_post.hip) against the numpy restatement
(oracle/post.py) -- bit-exact 8-bit images: both sides evaluate the same binary32 formulas in the
same order (no FMA contraction, correctly rounded div/sqrt), with the same texture model.
Inputs are the reference's own G-buffers (golden frames, re-rendered bit-exact on the device) and,
for the external-buffer path, golden G-buffers uploaded as torch tensors."""
import numpy as np
import pytest

from conftest import load_frame, load_npz
from oracle import post

pytestmark = pytest.mark.gpu

import sphereflake_amd as sf  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def device():
    sf.build()
    assert sf.device_count() >= 1, "no HIP device visible: GPU tests must run on an MI355X"


def _render(s, name):
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    cam = sf.config_camera(W, H, K)
    s.SetCamera(cam)
    s.Render()
    return fx, cam.corners()[0]


@pytest.mark.parametrize("flags", [0, sf.SF_POST_GENERAL])
@pytest.mark.parametrize("name", ["t1", "t2", "t3", "c1"])
def test_post_process_context_gbuffer(name, flags):
    fx = load_frame(name)
    W, H = fx["W"], fx["H"]
    with sf.Sphereflake(W, H) as s:
        _, origin = _render(s, name)
        s.PostProcess(flags=flags)
        img = s.download_image()
        pos, nrm, _, _ = s.download()
        closest = s.stats().closest
    radius = np.float32(8) * np.float32(closest)
    exp, ao, _, _ = post.post_process(pos, nrm, origin, radius)
    bad = np.argwhere(np.any(img != exp, axis=-1))
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}: {img[tuple(bad[0])]} vs {exp[tuple(bad[0])]}"


@pytest.mark.parametrize("downscale", [1, 2])
def test_post_process_external_buffers_accepting_blur(downscale):
    """Thresholds that accept blur taps (the general path's data-dependent branches), a half-size SSAO
    target, caller-owned device buffers and an explicit radius."""
    import torch
    name = "t1"
    fx = load_frame(name)
    g = load_npz(name)
    W, H = fx["W"], fx["H"]
    dev = torch.device("cuda", 0)
    pos = torch.from_numpy(np.ascontiguousarray(g["pos4"])).to(dev)
    nrm = torch.from_numpy(np.ascontiguousarray(g["nrm4"])).to(dev)
    rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
    aw, ah = W // downscale, H // downscale
    ao = torch.zeros((ah, aw), dtype=torch.uint8, device=dev)
    kw = dict(sample_radius=np.float32(3.5), normal_threshold=np.float32(0.6), depth_threshold=np.float32(0.0),
              camera_position=[0.25, -0.5, 1.0], downscale=downscale)
    with sf.Sphereflake(W, H) as s:
        s.PostProcess(pos.data_ptr(), nrm.data_ptr(), rgba.data_ptr(), ao.data_ptr(), **kw)
        s.Synchronize()
    exp, eao, ebx, _ = post.post_process(g["pos4"], g["nrm4"], kw["camera_position"], kw["sample_radius"], downscale,
                                         normal_threshold=kw["normal_threshold"], depth_threshold=kw["depth_threshold"])
    assert not np.array_equal(ebx, eao[:H, :W]) if downscale == 1 else True   # taps were accepted
    assert np.array_equal(ao.cpu().numpy(), eao)
    assert np.array_equal(rgba.cpu().numpy(), exp)


def test_fused_equals_general_full_hd():
    """Size-independent property at the bench size: the fused single-pass kernel equals the 4-pass
    chain bit for bit on a 1920x1080 frame (c3 camera)."""
    import torch
    fx = load_frame("c3")
    W, H = fx["W"], fx["H"]
    dev = torch.device("cuda", 0)
    outs = []
    with sf.Sphereflake(W, H) as s:
        _render(s, "c3")
        for flags in (0, sf.SF_POST_GENERAL):
            rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
            ao = torch.zeros((H, W), dtype=torch.uint8, device=dev)
            s.PostProcess(rgba_ptr=rgba.data_ptr(), ao_ptr=ao.data_ptr(), flags=flags)
            s.Synchronize()
            outs.append((rgba.cpu().numpy(), ao.cpu().numpy()))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][0], outs[1][0])
    assert (outs[0][0][..., :3] > 0).any()


def test_fastmath_matches_ieee_on_every_float():
    """sf_fastmath.h (the SSAO taps' square root and reciprocals): the short forms equal the IEEE operations on EVERY
    float of their ranges -- 2^32 patterns swept on the device (tests/hip/fastmath_check.hip); the bare v_rcp / v_sqrt
    are not correctly rounded, which is what the refinements are for."""
    import ctypes
    import os
    from conftest import REPO
    path = os.path.join(REPO, "tests", "hip", "build", "libsf_fastmath_check.so")
    assert os.path.exists(path), "build the test kernels first (__graft_entry__.build())"
    c = (ctypes.c_ulonglong * 6)()
    assert ctypes.CDLL(path).sf_fastmath_check(c) == 0
    bad_rcp, bad_sqrt, n_rcp, n_sqrt, bare_rcp, bare_sqrt = list(c)
    assert n_rcp == 2 * ((248 << 23) + 1) and n_sqrt == (224 << 23) + 1   # every float of both ranges (+-, and +0)
    assert bad_rcp == 0 and bad_sqrt == 0
    assert bare_rcp > 0 and bare_sqrt > 0


@pytest.mark.parametrize("flags", [0, sf.SF_POST_GENERAL])
def test_post_process_extreme_gbuffer_values(flags):
    """Tap arguments outside the short forms' ranges take the IEEE path for the whole fragment: a synthetic G-buffer
    with huge coordinates (d2 = inf), near-coincident positions (d2 below 2^-96), exact coincidences (d2 = 0), NaN and
    infinities, against the oracle."""
    import torch
    rng = np.random.default_rng(7)
    W, H = 64, 48
    pos = np.zeros((H, W, 4), np.float32)
    pos[..., :3] = rng.uniform(-2, 2, (H, W, 3)).astype(np.float32)
    pos[..., 2] = -np.abs(pos[..., 2]) - np.float32(0.5)
    pos[..., 3] = 1
    pos[8:16, 8:24, :3] = np.float32(1e20) * np.sign(pos[8:16, 8:24, :3])         # d2 overflows
    pos[20:28, 30:50, :3] = np.float32(0.75)                                         # d2 == 0 runs
    tiny = rng.uniform(0.5, 1.0, (8, 20, 3)).astype(np.float32) * np.float32(1e-15)  # d2 ~ 1e-30 < 2^-96
    tiny[..., 2] *= -1
    pos[30:38, 30:50, :3] = tiny
    pos[40, 5:9, 1] = np.nan
    pos[41, 5:9, 2] = -np.inf
    pos[40:44, 40:44, :3] = 0                                                        # background
    nrm = np.zeros((H, W, 4), np.float32)
    v = rng.normal(size=(H, W, 3)).astype(np.float32)
    nrm[..., :3] = v / np.linalg.norm(v, axis=-1, keepdims=True).astype(np.float32)
    nrm[..., 3] = 1
    dev = torch.device("cuda", 0)
    tp, tn = torch.from_numpy(pos).to(dev), torch.from_numpy(nrm).to(dev)
    rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
    ao = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    kw = dict(sample_radius=np.float32(2.5), camera_position=[0.25, -0.5, 1.0])
    with sf.Sphereflake(W, H) as s:
        s.PostProcess(tp.data_ptr(), tn.data_ptr(), rgba.data_ptr(), ao.data_ptr(), flags=flags, **kw)
        s.Synchronize()
    with np.errstate(all="ignore"):
        exp, eao, _, _ = post.post_process(pos, nrm, kw["camera_position"], kw["sample_radius"])
    assert np.array_equal(ao.cpu().numpy(), eao)
    assert np.array_equal(rgba.cpu().numpy(), exp)
