"""GPU tests of the drop-in surfaces either side of the trace:
- the reference-compatible C++ class (csrc/Sphereflake.hpp) driven like the reference app drives
  SphereflakeRaytracer::Sphereflake (tests/cpp/class_drive.cpp), bit-exact against the golden frames;
- stream-ordered download into page-locked host buffers, bit-identical to the synchronous path."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, load_frame, load_npz
from sfcheck import FLT_MAX, frame_digest

pytestmark = pytest.mark.gpu

import sphereflake_amd as sf  # noqa: E402

DRIVE = os.path.join(PKG, "build", "class_drive")


@pytest.fixture(scope="module", autouse=True)
def device():
    sf.build()
    assert sf.device_count() >= 1, "no HIP device visible: GPU tests must run on an MI355X"
    assert os.path.exists(DRIVE), "class_drive not built (make -C sphereflake-raytracer_amd)"


def drive(name, tmp_path, frames=1, image=False, dump=None):
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    corners = sf.config_camera(W, H, K).corners()
    args = [DRIVE, str(W), str(H)] + [float(x).hex() for c in corners for x in c]
    out = tmp_path / f"{name}.bin"
    extra = [str(tmp_path / f"{name}.rgba")] if image else []
    extra += [str(dump)] if dump else []
    r = subprocess.run(args + [str(out), str(frames)] + extra, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    g = np.fromfile(out, np.float32).reshape(2, H, W, 4)
    lines = r.stdout.split("\n")
    if image:
        return fx, g[0], g[1], lines[0].split(), np.fromfile(tmp_path / f"{name}.rgba", np.uint8).reshape(H, W, 4)
    return fx, g[0], g[1], lines[0].split(), lines[1].split()


@pytest.mark.parametrize("name", ["t2", "t3"])
def test_cpp_class_matches_golden(name, tmp_path):
    fx, pos, nrm, st, reset = drive(name, tmp_path, frames=2)
    exp = load_npz(name)
    assert np.array_equal(pos.view(np.uint32), exp["pos4"].view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), exp["nrm4"].view(np.uint32))
    assert int(st[0]) == fx["stats"]["max_depth"]
    assert int(st[1]) == 2 * fx["W"] * fx["H"]
    assert np.float32(float.fromhex(st[2])) == np.float32(float.fromhex(fx["stats"]["closest"]))
    assert int(reset[0]) == 0 and int(reset[1]) == 0 and np.float32(float.fromhex(reset[2])) == np.float32(FLT_MAX)


def test_cpp_class_config_c1(tmp_path):
    fx, pos, nrm, st, _ = drive("c1", tmp_path)
    assert frame_digest(pos, nrm) == fx["frame_digest"]


def test_async_pinned_download_equals_sync():
    fx = load_frame("c1")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render()
        ref = s.GetGBuffer()
        g = s.pinned_gbuffer()
        s.Render()
        s.download_async(g)
        s.Synchronize()
        assert np.array_equal(g.positions.view(np.uint32), ref.positions.view(np.uint32))
        assert np.array_equal(g.normals.view(np.uint32), ref.normals.view(np.uint32))
        assert frame_digest(g.positions, g.normals) == fx["frame_digest"]
        s.release_pinned()


def test_cpp_ssao_class_matches_oracle(tmp_path):
    """Headless SSAO class (Sphereflake.hpp) driven like main.cpp:312-330, against oracle/post.py."""
    from oracle import post
    fx, pos, nrm, st, img = drive("t1", tmp_path, image=True)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    origin = sf.config_camera(W, H, K).corners()[0]
    radius = np.float32(8) * np.float32(float.fromhex(st[2]))
    exp = post.post_process(pos, nrm, origin, radius)[0]
    assert np.array_equal(img, exp)


def read_pnm(path):
    """(header tokens, payload bytes) of a binary PPM / PFM: magic, width, height, maxval/scale."""
    b = open(path, "rb").read()
    tok, i = [], 0
    while len(tok) < 4:
        while b[i:i + 1].isspace():
            i += 1
        j = i
        while not b[j:j + 1].isspace():
            j += 1
        tok.append(b[i:j].decode())
        i = j
    return tok, b[i + 1:]


def test_cpp_class_image_dumps(tmp_path):
    """sf_save_image through the C++ class (SaveImage / SSAO::SaveImage): the PPM of the composited image
    equals its RGB bytes, the PFM dumps are the G-buffer's (x, y, z) bit for bit with PFM's bottom-up rows,
    and the normal visualisation maps misses to black."""
    fx, pos, nrm, st, img = drive("t1", tmp_path, image=True, dump=tmp_path / "d")
    H, W = pos.shape[:2]
    tok, data = read_pnm(tmp_path / "d_image.ppm")
    assert tok == ["P6", str(W), str(H), "255"]
    assert np.array_equal(np.frombuffer(data, np.uint8).reshape(H, W, 3), img[:, :, :3])
    for suffix, ch in (("pos", pos), ("nrm", nrm)):
        tok, data = read_pnm(tmp_path / f"d_{suffix}.pfm")
        assert tok == ["PF", str(W), str(H), "-1.0"]
        got = np.frombuffer(data, "<f4").reshape(H, W, 3)[::-1]
        assert np.array_equal(got.view(np.uint32), np.ascontiguousarray(ch[:, :, :3]).view(np.uint32))
    tok, data = read_pnm(tmp_path / "d_normals.ppm")
    vis = np.frombuffer(data, np.uint8).reshape(H, W, 3)
    miss = np.all(nrm[:, :, :3] == 0, axis=2)
    assert miss.any() and (~miss).any()
    assert np.all(vis[miss] == 0)
    exp = (np.clip(np.float32(0.5) * nrm[:, :, :3] + np.float32(0.5), 0, 1) * np.float32(255) + np.float32(0.5))
    assert np.array_equal(vis[~miss], exp.astype(np.uint8)[~miss])


def test_renders_on_alternating_streams_stay_ordered():
    """Calls of one context on different streams run in call order (ctx_join in sf_capi.hip): view A on
    stream 1 and the c2 view on stream 2, alternated without host synchronisation, must leave exactly
    the golden c2 frame (overlapping renders would race on the per-context tile queues and interleave
    A's and c2's pixels), with the frame-less mode and a download joining in between."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")   # raw HIP streams (no torch import: it pages in for minutes on a fresh box)
    hs = [ctypes.c_void_p(), ctypes.c_void_p()]
    for h in hs:
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    cam_b = sf.config_camera(W, H, K)
    cam_a = sf.config_camera(W, H, K)
    cam_a.SetYaw(np.float32(sf.DEFAULT_YAW + 0.05))
    s1, s2 = hs[0].value, hs[1].value
    with sf.Sphereflake(W, H) as s:
        for _ in range(6):
            s.SetCamera(cam_a)
            s.Render(stream=s1)
            s.SetCamera(cam_b)
            s.Render(stream=s2)
        pos, nrm, _, _ = s.download()
        assert frame_digest(pos, nrm) == fx["frame_digest"]
        # frame-less batches on stream 1 after a render on stream 2, then a full frame on stream 2 again
        s.SetCamera(cam_a)
        s.Progressive(12345, 1 << 16, 0, stream=s1)
        s.SetCamera(cam_b)
        s.Render(stream=s2)
        pos, nrm, _, _ = s.download()
        assert frame_digest(pos, nrm) == fx["frame_digest"]
    for h in hs:
        hip.hipStreamDestroy(h)


def test_caller_stream_destroyed_after_use():
    """A caller renders on its own stream, waits for it and destroys it, then keeps using the context on
    the context stream and finally destroys the context: the context must never touch the dead stream
    (its join point is an event recorded when the call returned), and the frame stays golden."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    s = sf.Sphereflake(W, H)
    try:
        s.SetCamera(sf.config_camera(W, H, K))
        for _ in range(2):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(h)) == 0
            s.Render(stream=h.value)
            s.Progressive(7, 1000, 0, stream=h.value)
            assert hip.hipStreamSynchronize(h) == 0
            assert hip.hipStreamDestroy(h) == 0
            s.Render()                       # the context stream, after the destroyed one
            s.Synchronize()
            pos, nrm, _, _ = s.download()
            assert frame_digest(pos, nrm) == fx["frame_digest"]
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        s.Render(stream=h.value)             # the last call on a caller's stream ...
        assert hip.hipStreamSynchronize(h) == 0
        assert hip.hipStreamDestroy(h) == 0
    finally:
        s.close()                            # ... then sf_destroy
