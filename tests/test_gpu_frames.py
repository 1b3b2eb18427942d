"""GPU tests of the multi-frame persistent trace (sf_render_frames / sf_dist_render_bands_frames, kernel
sf_trace_frames1): several frames -- each a context's own view, G-buffer and stats -- in ONE launch over one set of
tile queues, the heaviest units of every frame first. Every frame must equal what a launch of its own writes
(sf_render), bit for bit in position, normal, t and heap hit index, with the same stats; the fixed config views
must match the reference-made golden digests (tests/golden), random views the oracle restatement. The reference
renders frames continuously with its worker pool (Sphereflake.cpp:67-74,112-213); the batch is that, on one grid."""
import numpy as np
import pytest

from conftest import load_frame
from sfcheck import frame_digest

pytestmark = pytest.mark.gpu

import sphereflake_amd as sf  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def device():
    sf.build()
    assert sf.device_count() >= 1, "no HIP device visible: GPU tests must run on an MI355X"


def path_views(W, H, K, n, start=0):
    from bench import frame_camera
    return [frame_camera(W, H, K, start + i).corners() for i in range(n)]


def single(W, H, view, **kw):
    with sf.Sphereflake(W, H) as s:
        s.SetView(*view)
        s.Render(emit_aux=True, **kw)
        out = s.download(aux=True)
        st = s.stats()
    return out, st


def assert_same(got, want, what):
    for a, b, name in zip(got, want, ("pos", "nrm", "minT", "index")):
        assert np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32)), (what, name)


@pytest.mark.parametrize("name,n", [("c2", 4), ("c3", 4), ("c3", 8), ("c1", 3), ("t3", 2)])
def test_frames_equal_single_launches(name, n):
    """n frames of the bench's moving camera path in one launch, twice (row-major or the order the first batch's
    costs built): each frame equals a launch of its own, and its context's stats equal that launch's."""
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    views = path_views(W, H, K, n)
    want = [single(W, H, v) for v in views]
    flakes = [sf.Sphereflake(W, H) for _ in range(n)]
    try:
        for rep in range(2):
            for f, v in zip(flakes, views):
                f.SetView(*v)
                f.reset_stats()
            sf.render_frames(flakes, emit_aux=True)
            for k, f in enumerate(flakes):
                got = f.download(aux=True)
                assert_same(got, want[k][0], (name, n, rep, k))
                st = f.stats()
                assert st.max_depth == want[k][1].max_depth, (name, rep, k)
                assert np.float32(st.closest) == np.float32(want[k][1].closest), (name, rep, k)
                assert st.rays == W * H
    finally:
        for f in flakes:
            f.close()


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_frames_fixed_view_golden(name, monkeypatch):
    """Every frame of a batch on the config view is the reference frame (golden digest); with the order rebuilt
    after every batch (SF_ORDER=1, SF_ORDER_EVERY=1) across four batches, the shared order changes under the frames."""
    monkeypatch.setenv("SF_ORDER", "1")
    monkeypatch.setenv("SF_ORDER_EVERY", "1")
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    view = sf.config_camera(W, H, K).corners()
    flakes = [sf.Sphereflake(W, H) for _ in range(4)]
    try:
        for f in flakes:
            f.SetView(*view)
        for rep in range(4):
            sf.render_frames(flakes)
        for k, f in enumerate(flakes):
            pos, nrm, _, _ = f.download()
            assert frame_digest(pos, nrm) == fx["frame_digest"], (name, k)
            assert f.stats().max_depth == fx["stats"]["max_depth"]
    finally:
        for f in flakes:
            f.close()


@pytest.mark.parametrize("n,band_count,band_index", [(4, 3, 1), (3, 8, 0), (5, 8, 7), (2, 2, 1)])
def test_frames_bands_equal_single_launches(n, band_count, band_index):
    """A rank's bands (a distributed G-buffer share) of n frames in one launch: each frame's G-buffer equals the
    banded launch of its own (the rows the rank does not own stay as the context left them: zero)."""
    fx = load_frame("c3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    views = path_views(W, H, K, n, start=5)
    kw = dict(band_rows=8, band_count=band_count, band_index=band_index)
    want = [single(W, H, v, **kw) for v in views]
    flakes = [sf.Sphereflake(W, H) for _ in range(n)]
    try:
        for f, v in zip(flakes, views):
            f.SetView(*v)
        sf.render_frames(flakes, emit_aux=True, **kw)
        for k, f in enumerate(flakes):
            assert_same(f.download(aux=True), want[k][0], (n, band_count, band_index, k))
            assert f.stats().max_depth == want[k][1].max_depth
    finally:
        for f in flakes:
            f.close()


def test_frames_forced_retrace_and_fallback(monkeypatch):
    """Every tile through the in-wave index-order re-trace (SF_FLAGS=0x400, DIAG_FORCE_RETRACE), where a re-trace
    continues the wave's own frame; and the fallback of one launch per frame (SF_LEVELS: levels not proven) --
    both equal single launches."""
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    views = path_views(W, H, K, 3, start=11)
    want = [single(W, H, v) for v in views]
    for env in ({"SF_FLAGS": "0x400"}, {"SF_LEVELS": "12"}):
        with monkeypatch.context() as m:
            for k_, v_ in env.items():
                m.setenv(k_, v_)
            flakes = [sf.Sphereflake(W, H) for _ in range(3)]
            try:
                for f, v in zip(flakes, views):
                    f.SetView(*v)
                sf.render_frames(flakes, emit_aux=True)
                sf.render_frames(flakes[::-1], emit_aux=True)   # (any context may lead)
                for k, f in enumerate(flakes):
                    assert_same(f.download(aux=True), want[k][0], (env, k))
            finally:
                for f in flakes:
                    f.close()


def test_frames_random_views_against_oracle():
    """Random views of one frame size in one batch (inside and outside the flake's bounding ball, other FOVs):
    each frame equals the oracle restatement bit for bit, and its stats the oracle's."""
    from oracle import pyoracle
    from test_gpu_random_views import random_view
    rng = np.random.default_rng(77)
    W, H = 96, 54
    views, refs = [], []
    while len(views) < 6:
        w, h, K, cam = random_view(rng, 2)   # (size index 2: 96 x 54)
        assert (w, h) == (W, H)
        o, tl, tr, bl = cam.corners()
        setup = {"W": W, "H": H, "origin": o, "tl": tl, "tr": tr, "bl": bl,
                 "root": sf.root_transform(o), "children": sf.child_transforms()}
        views.append((o, tl, tr, bl))
        refs.append(pyoracle.render(setup))
    flakes = [sf.Sphereflake(W, H) for _ in views]
    try:
        for f, v in zip(flakes, views):
            f.SetView(*v)
        sf.render_frames(flakes, emit_aux=True)
        for k, (f, ref) in enumerate(zip(flakes, refs)):
            pos, nrm, mint, idx = f.download(aux=True)
            assert np.array_equal(idx, ref["index"]), k
            assert np.array_equal(pos.view(np.uint32), ref["pos4"].view(np.uint32)), k
            assert np.array_equal(nrm.view(np.uint32), ref["nrm4"].view(np.uint32)), k
            assert np.array_equal(mint.view(np.uint32), ref["minT"].view(np.uint32)), k
            st = f.stats()
            assert st.max_depth == ref["stats"]["max_depth"], k
            assert np.float32(st.closest) == np.float32(ref["stats"]["closest"]), k
    finally:
        for f in flakes:
            f.close()


def test_frames_rejects_bad_batches():
    W, H = 64, 64
    flakes = [sf.Sphereflake(W, H) for _ in range(9)]
    other = sf.Sphereflake(32, 32)
    try:
        for f in flakes + [other]:
            f.SetCamera(sf.config_camera(f.width, f.height, 0.25))
        for batch, kw, code in (
                (flakes[:9], {}, sf.SF_EINVAL),                 # more than SF_RENDER_FRAMES_MAX
                ([flakes[0], flakes[0]], {}, sf.SF_EINVAL),     # one context twice
                ([flakes[0], other], {}, sf.SF_EINVAL),         # frame sizes differ
                (flakes[:2], {"compact": True}, sf.SF_EINVAL),
                (flakes[:2], {"kernel": sf.SF_KERNEL_PER_RAY}, sf.SF_EINVAL)):
            with pytest.raises(sf.SphereflakeError) as e:
                sf.render_frames(batch, **kw)
            assert e.value.code == code
        fresh = sf.Sphereflake(W, H)   # no view yet
        try:
            with pytest.raises(sf.SphereflakeError) as e:
                sf.render_frames([flakes[0], fresh])
            assert e.value.code == sf.SF_ENOVIEW
        finally:
            fresh.close()
    finally:
        for f in flakes + [other]:
            f.close()


@pytest.mark.parametrize("slots,n,nranks,rank", [(4, 4, 1, 0), (8, 4, 1, 0), (6, 3, 3, 2), (16, 8, 8, 0), (16, 8, 8, 7)])
def test_dist_render_bands_frames(slots, n, nranks, rank):
    """sf_dist_render_bands_frames: the next n frames of a camera path on slots (frames + k) % slots in one launch,
    three batches in a row -- each slot's G-buffer equals RenderBands of the same frame (a dist of its own)."""
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    views = path_views(W, H, K, 3 * n)
    with sf.SphereflakeDist(0, W, H, rank=rank, nranks=nranks, slots=slots) as d, \
            sf.SphereflakeDist(0, W, H, rank=rank, nranks=nranks, slots=slots) as ref:
        for b in range(3):
            d.RenderBandsFrames(views[b * n:(b + 1) * n])
            for v in views[b * n:(b + 1) * n]:
                ref.SetView(*v)
                ref.RenderBands()
        d.Synchronize()
        ref.Synchronize()
        assert d.last_slot() == ref.last_slot()
        for s in range(slots):
            p, q = d.download_slot(s)
            rp, rq = ref.download_slot(s)
            assert np.array_equal(p.view(np.uint32), rp.view(np.uint32)), s
            assert np.array_equal(q.view(np.uint32), rq.view(np.uint32)), s
        st, rst = d.stats(), ref.stats()
    assert st.rays == rst.rays and st.max_depth == rst.max_depth
    assert np.float32(st.closest) == np.float32(rst.closest)
