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
