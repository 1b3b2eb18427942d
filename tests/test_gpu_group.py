"""GPU: single-process multi-GPU rendering behind the C ABI (sf_group_*). The group
cuts the frame into interleaved bands, traces them on its members (members > 0 as packed slabs) and
copies those into member 0's stage, where they are unpacked into its G-buffer. On a one-GPU box the
members are n contexts on device 0 (own streams, same copy path); the assembled frame must equal the
golden c2/c3 frames bit for bit and the one-context render of any other view, frame after frame, also
with several frames in flight (double-buffered slabs and stages)."""
import numpy as np
import pytest

from conftest import load_frame
from sfcheck import bad_rows, frame_digest, row_digests

pytestmark = pytest.mark.gpu

import sphereflake_amd as sf  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def device():
    sf.build()
    n = sf.device_count()
    assert n >= 1, "no HIP device visible: GPU tests must run on an MI355X"
    return n


def single(W, H, cam):
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(cam)
        s.Render()
        pos, nrm, _, _ = s.download()
        return pos, nrm, s.stats()


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


@pytest.mark.parametrize("name,members,band", [("c2", 3, 8), ("c3", 2, 8), ("c3", 4, 16)])
def test_group_on_one_device_equals_golden(name, members, band):
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.SphereflakeGroup([0] * members, W, H) as g:
        assert g.size() == members
        g.SetCamera(sf.config_camera(W, H, K))
        for frame in range(2):   # the second frame reuses the slabs and overwrites the first
            g.Render(band)
            pos, nrm = g.download()
            bad = bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm))
            assert bad == [], f"frame {frame}: {len(bad)} rows differ, first {bad[:5]}"
            assert frame_digest(pos, nrm) == fx["frame_digest"]
            st = g.stats()
            e = fx["stats"]
            assert st.max_depth == e["max_depth"]
            assert np.float32(st.closest) == np.float32(float.fromhex(e["closest"]))
            assert st.overflow_tiles == 0
            if fx["row_step"] == 1:
                assert st.rays == (frame + 1) * e["rays"]   # accumulates like the reference's counter


def test_group_both_slab_formats():
    """The slab format follows the view (sf_group_slab_bytes): 4-B hit indices where every hit is provably at depth
    <= 10, 16-B normal + minT slabs where not (a camera inside the flake's bounding sphere) -- either way the group's
    frame equals a one-context render of the view bit for bit."""
    W, H = 200, 120
    far = sf.config_camera(W, H, 0.25)
    near = sf.config_camera(W, H, 0.25)
    near.SetPosition(np.asarray(sf.DEFAULT_CAMERA_POSITION, np.float32) * np.float32(0.2))   # (inside: c5's K)
    for cam, want in ((far, 4), (near, 16), (far, 4)):
        with sf.SphereflakeGroup([0] * 3, W, H) as g:
            g.SetCamera(cam)
            assert g.slab_bytes() == want
            g.Render(8)
            pos, nrm = g.download()
        rp, rn, _ = single(W, H, cam)
        assert same_bits(pos, rp) and same_bits(nrm, rn), want


def test_group_moving_views_and_ragged_last_band():
    """H = 100 with 8-row bands over 3 members: 13 bands, the last one 4 rows (partial copy). A sequence
    of views, each frame equal to the one-context render of the same view."""
    W, H = 136, 100
    with sf.SphereflakeGroup([0, 0, 0], W, H) as g:
        for yaw in (0.0, 0.01, -0.02, 0.0):
            cam = sf.config_camera(W, H, 0.25)
            cam.SetYaw(np.float32(sf.DEFAULT_YAW + yaw))
            g.SetCamera(cam)
            g.reset_stats()
            g.Render(8)
            pos, nrm = g.download()
            spos, snrm, sst = single(W, H, cam)
            assert same_bits(pos, spos) and same_bits(nrm, snrm), f"yaw {yaw}"
            st = g.stats()
            assert (st.max_depth, st.rays) == (sst.max_depth, sst.rays)
            assert np.float32(st.closest) == np.float32(sst.closest)


def test_group_more_members_than_bands():
    """4 members, 8-row bands, 24 rows: member 3 owns no band and is skipped."""
    W, H = 64, 24
    cam = sf.config_camera(W, H, 0.25)
    with sf.SphereflakeGroup([0, 0, 0, 0], W, H) as g:
        g.SetCamera(cam)
        g.Render(8)
        pos, nrm = g.download()
    spos, snrm, _ = single(W, H, cam)
    assert same_bits(pos, spos) and same_bits(nrm, snrm)


def test_group_errors():
    with pytest.raises(sf.SphereflakeError):
        sf.SphereflakeGroup([], 64, 64)
    with pytest.raises(sf.SphereflakeError):
        sf.SphereflakeGroup([0, 0], 0, 64)
    with sf.SphereflakeGroup([0, 0], 64, 64) as g:
        with pytest.raises(sf.SphereflakeError) as e:
            g.Render(8)   # no view yet
        assert e.value.code == sf.SF_ENOVIEW
        g.SetCamera(sf.config_camera(64, 64, 0.25))
        with pytest.raises(sf.SphereflakeError) as e:
            g.Render(12)   # bands must be whole 8-row tiles
        assert e.value.code == sf.SF_EINVAL
        assert g.member(0) and g.member(1) and not g.member(2)


def test_group_across_devices(device):
    if device < 2:
        pytest.skip("one HIP device visible: the peer-copy path across devices needs two")
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.SphereflakeGroup(list(range(min(device, 4))), W, H) as g:
        g.SetCamera(sf.config_camera(W, H, K))
        g.Render(8)
        pos, nrm = g.download()
    assert frame_digest(pos, nrm) == fx["frame_digest"]


def test_group_pipelined_frames_equal_single():
    """Five frames of different views issued back to back (members race ahead of member 0 by a frame:
    double-buffered slabs and stages), each captured by an asynchronous D2H queued on member 0's stream
    right after its render: every capture equals the one-context render of its view."""
    import ctypes
    W, H = 200, 120
    views = []
    for j in range(5):
        cam = sf.config_camera(W, H, 0.25)
        cam.SetYaw(np.float32(sf.DEFAULT_YAW + 0.015 * (j - 2)))
        views.append(cam)
    L = sf.lib()
    caps = [(np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)) for _ in views]
    for p, n in caps:
        for a in (p, n):
            assert L.sf_host_register(a.ctypes.data_as(ctypes.c_void_p), a.nbytes) == 0
    try:
        with sf.SphereflakeGroup([0, 0, 0], W, H) as g:
            c0 = g.member(0)
            for cam, (p, n) in zip(views, caps):
                g.SetCamera(cam)
                g.Render(8)
                assert L.sf_download_async(c0, p.ctypes.data_as(ctypes.c_void_p), n.ctypes.data_as(ctypes.c_void_p),
                                           None, None, None) == 0
            g.Synchronize()
        for j, (cam, (p, n)) in enumerate(zip(views, caps)):
            spos, snrm, _ = single(W, H, cam)
            assert same_bits(p, spos) and same_bits(n, snrm), f"frame {j}"
    finally:
        for p, n in caps:
            for a in (p, n):
                L.sf_host_unregister(a.ctypes.data_as(ctypes.c_void_p))


def test_group_band_split_change_resizes():
    """Switching the band height between frames re-sizes the slabs and stages (after draining the old ones)."""
    W, H = 96, 72
    cam = sf.config_camera(W, H, 0.25)
    spos, snrm, _ = single(W, H, cam)
    with sf.SphereflakeGroup([0, 0], W, H) as g:
        g.SetCamera(cam)
        for band in (8, 16, 8, 24):
            g.Render(band)
            pos, nrm = g.download()
            assert same_bits(pos, spos) and same_bits(nrm, snrm), band


def test_group_caller_stream_consumer_not_overwritten():
    """a consumer of member 0's frame queued on a CALLER's stream (sf_download_async on stream X) must
    finish reading before the next group frame's unpack rewrites the peer rows. The unpack stream waits only for
    the frame's start event on member 0's context stream, so that event has to follow the context's join of X
    (sfi_join before start0 in sf_group_render). Frames of 1280x720 with a D2H (~0.5 ms) that outlasts the next
    frame's trace + unpack: every capture must equal the one-context render of its own view."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    W, H = 1280, 720
    views = []
    for j in range(3):
        cam = sf.config_camera(W, H, 0.8)
        cam.SetYaw(np.float32(sf.DEFAULT_YAW + 0.02 * (j - 1)))
        views.append(cam)
    L = sf.lib()
    caps = [(np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)) for _ in views]
    for p, n in caps:
        for a in (p, n):
            assert L.sf_host_register(a.ctypes.data_as(ctypes.c_void_p), a.nbytes) == 0
    x = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(x)) == 0
    try:
        with sf.SphereflakeGroup([0, 0, 0], W, H) as g:
            c0 = g.member(0)
            for cam, (p, n) in zip(views, caps):
                g.SetCamera(cam)
                g.Render(8)
                assert L.sf_download_async(c0, p.ctypes.data_as(ctypes.c_void_p), n.ctypes.data_as(ctypes.c_void_p),
                                           None, None, x) == 0
            g.Synchronize()
            assert hip.hipStreamSynchronize(x) == 0
        for j, (cam, (p, n)) in enumerate(zip(views, caps)):
            spos, snrm, _ = single(W, H, cam)
            assert same_bits(p, spos) and same_bits(n, snrm), f"frame {j}"
    finally:
        hip.hipStreamDestroy(x)
        for p, n in caps:
            for a in (p, n):
                L.sf_host_unregister(a.ctypes.data_as(ctypes.c_void_p))
