"""GPU parity: the gfx950 kernels, called through the C ABI, against the golden vectors the reference
AVX path produced (tests/golden/). Bar: bit-exact G-buffer (positions, normals), minT and hit-sphere
heap index; the north star's tolerance (nearest-hit sphere index exact, position/normal within
1e-5 fp32) is asserted separately on the sampled pixels."""
import numpy as np
import pytest

from conftest import load_frame, load_npz, load_progressive
from sfcheck import FLT_MAX, aux_digests, bad_rows, frame_digest, row_digests, samples_arrays

pytestmark = pytest.mark.gpu

import sphereflake_amd as sf  # noqa: E402

TOL = 1e-5   # north star: position/normal within 1e-5 fp32


@pytest.fixture(scope="module", autouse=True)
def device():
    sf.build()
    n = sf.device_count()
    assert n >= 1, "no HIP device visible: GPU tests must run on an MI355X"
    return n


def render(name, kernel=sf.SF_KERNEL_WAVE, **kw):
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render(kernel=kernel, emit_aux=True, **kw)
        pos, nrm, mint, idx = s.download(aux=True)
        st = s.stats()
    return fx, pos, nrm, mint, idx, st


def check_stats(fx, st, mint):
    e = fx["stats"]
    assert st.max_depth == e["max_depth"]
    assert np.float32(st.closest) == np.float32(float.fromhex(e["closest"]))
    if fx["row_step"] == 1:
        assert int((mint < np.float32(FLT_MAX)).sum()) == e["hits"]
        assert st.rays == e["rays"]
    assert st.overflow_tiles == 0


@pytest.mark.parametrize("kernel", [sf.SF_KERNEL_WAVE, sf.SF_KERNEL_PER_RAY])
@pytest.mark.parametrize("name", ["t1", "t2", "t3", "t4", "t5"])
def test_tiny_frames_bit_exact(name, kernel):
    exp = load_npz(name)
    fx, pos, nrm, mint, idx, st = render(name, kernel)
    for k, got in (("pos4", pos), ("nrm4", nrm), ("minT", mint), ("index", idx)):
        assert np.array_equal(np.ascontiguousarray(got).view(np.uint8), np.ascontiguousarray(exp[k]).view(np.uint8)), k
    check_stats(fx, st, mint)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4"])
def test_config_frames_bit_exact(name):
    fx, pos, nrm, mint, idx, st = render(name)
    bad = bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm))
    assert bad == [], f"{len(bad)} G-buffer rows differ, first {bad[:5]}"
    bad = bad_rows(fx["row_digest_aux"], aux_digests(mint, idx))
    assert bad == [], f"{len(bad)} minT/index rows differ, first {bad[:5]}"
    assert frame_digest(pos, nrm) == fx["frame_digest"]
    check_stats(fx, st, mint)


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_per_ray_kernel_bit_exact(name):
    fx, pos, nrm, mint, idx, st = render(name, sf.SF_KERNEL_PER_RAY)
    assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == []
    assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == []
    check_stats(fx, st, mint)


@pytest.mark.parametrize("name", ["c1", "c3"])
def test_north_star_tolerance_on_samples(name):
    """Hit-sphere index bit-exact, position/normal within 1e-5 (BASELINE.json north_star)."""
    fx, pos, nrm, mint, idx, st = render(name)
    s = samples_arrays(fx)
    y, x = s["y"], s["x"]
    assert np.array_equal(idx[y, x], s["index"])
    assert np.abs(pos[y, x, :3] - s["pos"]).max() <= TOL
    assert np.abs(nrm[y, x, :3] - s["nrm"]).max() <= TOL
    assert np.all(pos[y, x, 3] == 1.0) and np.all(nrm[y, x, 3] == 1.0)


def test_c5_rows_16384():
    """configs[4]: 16384x16384 depth 10. Rows y % 64 == 0 rendered as band shard 0 of 8 (8-row bands)
    into a compact slab in caller-owned device memory (torch), checked against the reference rows."""
    import torch
    fx = load_frame("c5")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    rows = sf.lib().sf_slab_rows(H, 8, 8, 0)
    assert rows == H // 8
    dev = torch.device("cuda:0")
    pos = torch.empty((rows, W, 4), dtype=torch.float32, device=dev)
    nrm = torch.empty_like(pos)
    mint = torch.empty((rows, W), dtype=torch.float32, device=dev)
    idx = torch.empty((rows, W), dtype=torch.int32, device=dev)
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        torch.cuda.synchronize()
        s.render_to(pos.data_ptr(), nrm.data_ptr(), mint.data_ptr(), idx.data_ptr(),
                    band_rows=8, band_count=8, band_index=0, compact=True, emit_aux=True)
        s.Synchronize()
        st = s.stats()
    sel = torch.arange(0, rows, 8, device=dev)
    p, n = pos[sel].cpu().numpy(), nrm[sel].cpu().numpy()
    m, i = mint[sel].cpu().numpy(), idx[sel].cpu().numpy().view(np.uint32)
    assert bad_rows(fx["row_digest_gbuf"], row_digests(p, n)) == []
    assert bad_rows(fx["row_digest_aux"], aux_digests(m, i)) == []
    assert st.overflow_tiles == 0
    assert st.max_depth >= fx["stats"]["max_depth"]   # the shard covers more rows than the fixture


def test_banded_shards_reassemble_full_frame():
    """Row-band sharding: 4 shards of 16-row bands, compact slabs, de-interleaved,
    equal the full frame bit for bit."""
    import torch
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    band, n = 16, 4
    full = np.zeros((H, W, 4), np.float32)
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for r in range(n):
            rows = sf.lib().sf_slab_rows(H, band, n, r)
            pos = torch.empty((rows, W, 4), dtype=torch.float32, device="cuda:0")
            nrm = torch.empty_like(pos)
            s.render_to(pos.data_ptr(), nrm.data_ptr(), band_rows=band, band_count=n, band_index=r, compact=True)
            s.Synchronize()
            slab = pos.cpu().numpy()
            k = 0
            for b in range(r, (H + band - 1) // band, n):
                y0, y1 = b * band, min(H, (b + 1) * band)
                full[y0:y1] = slab[k:k + (y1 - y0)]
                k += y1 - y0
            assert k == rows
    fx2, pos, nrm, mint, idx, st = render("c2")
    assert np.array_equal(full.view(np.uint32), pos.view(np.uint32))


def test_overflow_fixup_path():
    """Provision only 4 LDS levels: tiles needing depth > 4 are re-traced by sf_fixup_wave; the frame
    must still be exact and no tile may remain unresolved."""
    fx, pos, nrm, mint, idx, st = render("c3", max_depth=4)
    assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == []
    assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == []
    check_stats(fx, st, mint)


def test_repeat_renders_deterministic_and_stats_reset():
    fx = load_frame("t2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render()
        a = s.download()[0].copy()
        s.Render()
        b = s.download()[0]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        assert s.GetRaysPerSecond() == 2 * W * H
        s.ResetRaysPerSecond()
        assert s.GetRaysPerSecond() == 0
        assert s.GetMaxDepthReached() == fx["stats"]["max_depth"]
        s.ResetMaxDepthReached()
        assert s.GetMaxDepthReached() == 0
        s.ResetClosestSphereDistance()
        assert s.GetClosestSphereDistance() == np.float32(FLT_MAX)


def test_gbuffer_initial_state_and_errors():
    with sf.Sphereflake(16, 8) as s:
        g = s.GetGBuffer()
        assert np.all(g.positions == 0) and np.all(g.normals == 0)   # glm vec4() default
        with pytest.raises(sf.SphereflakeError) as e:
            s.Render()
        assert e.value.code == sf.SF_ENOVIEW
        s.SetCamera(sf.config_camera(16, 8, 1.0))
        with pytest.raises(sf.SphereflakeError) as e:
            s.Render(band_rows=12, band_count=2)
        assert e.value.code == sf.SF_EINVAL


@pytest.mark.parametrize("name,order", [("p1", "0"), ("p2", "0"), ("p3", "0"), ("p3", "1"), ("p4", "0"), ("p5", "0")])
def test_progressive_matches_reference_worker(name, order, monkeypatch):
    """Frame-less mode (Sphereflake.cpp:86-214): one reference worker's packet stream from mt19937(seed)
    -- Sobol pixel draws, 8-ray packets with packet-wide early-outs, sequential scatter. p3 also with the
    heavy-first bin order (SF_PROG_ORDER=1: its second, binned batch is ordered by the first's costs)."""
    monkeypatch.setenv("SF_PROG_ORDER", order)
    fx = load_progressive(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        half = fx["packets"] // 3
        s.Progressive(fx["seed"], half, counter0=0)
        s.Progressive(fx["seed"], fx["packets"] - half)           # continues the stream
        pos, nrm, _, _ = s.download()
        st = s.stats()
    bad = bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm))
    assert bad == [], f"{len(bad)} rows differ, first {bad[:5]}"
    assert st.max_depth == fx["stats"]["max_depth"]
    assert np.float32(st.closest) == np.float32(float.fromhex(fx["stats"]["closest"]))
    assert st.rays == fx["stats"]["rays"]


def test_progressive_reseed_skip_ahead():
    """A call that does not continue the stream reseeds and skips ahead: the pixels the p1 stream writes
    come out exactly as from one uninterrupted call on a fresh context."""
    fx = load_progressive("p1")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Progressive(fx["seed"] + 1, 100, counter0=0)               # unrelated stream first
        s.Progressive(fx["seed"], 1000, counter0=0)
        s.Progressive(fx["seed"] + 7, 10, counter0=5)
        s.Progressive(fx["seed"], fx["packets"] - 1000, counter0=1000)   # reseed + skip 2000 draws
        pos, nrm, _, _ = s.download()
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Progressive(fx["seed"], fx["packets"], counter0=0)
        epos, enrm, _, _ = s.download()
    assert bad_rows(fx["row_digest_gbuf"], row_digests(epos, enrm)) == []
    w = epos[..., 3] == 1.0
    assert np.array_equal(pos[w].view(np.uint32), epos[w].view(np.uint32))
    assert np.array_equal(nrm[w].view(np.uint32), enrm[w].view(np.uint32))


@pytest.mark.parametrize("calls", [
    [(0, 100000), (0, 100000)],                          # the second batch is the prefetched draws
    [(0, 100000), (0, 50000), (0, 50000)],               # size changes: prefetch undone, state restored
    [(0, 70000), (1, 10), (0, 130000)],                  # another stream in between: restore + reseed/skip
    [(0, 70000), (0, 70000), (0, 60000)],                # two prefetch hits, then a smaller batch
])
def test_progressive_draw_prefetch_paths(calls, monkeypatch):
    """Large batches prefetch the next batch's mt19937 draws on a side stream; whatever the next call
    is, the frame equals the same calls with the prefetch off (SF_PROG_PREFETCH=0), and a p3-only
    sequence equals the reference worker's p3 stream (200000 packets of mt19937(777))."""
    fx = load_progressive("p3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])

    def run():
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, K))
            done = 0
            for other, n in calls:
                if other:
                    s.Progressive(fx["seed"] + 1, n, counter0=3)
                else:
                    s.Progressive(fx["seed"], n, counter0=done)
                    done += n
            assert done == fx["packets"]
            pos, nrm, _, _ = s.download()
            return pos, nrm, s.stats()

    pos, nrm, st = run()
    monkeypatch.setenv("SF_PROG_PREFETCH", "0")
    epos, enrm, est = run()
    assert np.array_equal(pos.view(np.uint32), epos.view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), enrm.view(np.uint32))
    assert (st.max_depth, st.closest, st.rays) == (est.max_depth, est.closest, est.rays)
    if not any(other for other, _ in calls):
        assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == []
        assert st.max_depth == fx["stats"]["max_depth"]


def test_progressive_prefetched_bins_follow_the_variant(monkeypatch):
    """The next batch's binned order is prefetched with its draws for the variant of the batch that issued the
    prefetch (packet width 8 or 4); a continuing batch of the other variant bins afresh. Frames and stats equal
    the same calls with the prefetch off."""
    fx = load_progressive("p3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])

    def run():
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, K))
            done = 0
            for variant in ("avx", "sse", "sse", "avx"):
                s.SetVariant(variant)
                s.Progressive(fx["seed"], 70000, counter0=done)
                done += 70000
            pos, nrm, _, _ = s.download()
            return pos, nrm, s.stats()

    pos, nrm, st = run()
    monkeypatch.setenv("SF_PROG_PREFETCH", "0")
    epos, enrm, est = run()
    assert np.array_equal(pos.view(np.uint32), epos.view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), enrm.view(np.uint32))
    assert (st.max_depth, st.closest, st.rays) == (est.max_depth, est.closest, est.rays)


def test_repeat_renders_heavy_first_order_bit_exact(monkeypatch):
    """From the second render on, the persistent kernel takes its tiles heaviest-first (costs of the
    previous render, sf_tile_order; SF_ORDER=1: on for this full-grid frame too). The image must not depend
    on the order: renders 2 and 3 of c3 equal the golden digests, and kernel timing reports one duration per
    render."""
    monkeypatch.setenv("SF_ORDER", "1")
    fx = load_frame("c3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.kernel_timing(True)
        for k in range(3):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"render {k}"
            assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], f"render {k}"
        ms = s.kernel_timing()
        s.kernel_timing(True, period=2)     # sampled: renders 0 and 2 of the next three
        for k in range(3):
            s.Render()
        ms2 = s.kernel_timing()
        st = s.stats()
    assert len(ms) == 3 and np.all(ms > 0)
    assert len(ms2) == 2 and np.all(ms2 > 0)
    assert st.max_depth == fx["stats"]["max_depth"] and st.overflow_tiles == 0


@pytest.mark.parametrize("qpx", ["2", "4"])
def test_several_queues_per_xcd_bit_exact(monkeypatch, qpx):
    """SF_QUEUES_PER_XCD: each XCD's tickets split over several queue words (sub-queues served by disjoint
    sets of that XCD's waves). Every unit must still be traced exactly once: the c3 frame stays golden over
    repeated renders (row-major, then heavy-first)."""
    monkeypatch.setenv("SF_QUEUES_PER_XCD", qpx)
    fx = load_frame("c3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(3):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"render {k}"
            assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], f"render {k}"
        st = s.stats()
    assert st.rays == 3 * W * H and st.overflow_tiles == 0


@pytest.mark.parametrize("name,pipe", [("c1", "0"), ("c3", "1")])
def test_trace_variants_forced_bit_exact(monkeypatch, name, pipe):
    """The persistent trace has a latency variant (sf_trace_queue2p, pipelined child loop) that the host
    picks for small frames; SF_PIPE forces either. Each variant on the other's frame size: golden frame."""
    monkeypatch.setenv("SF_PIPE", pipe)
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(2):   # row-major first render, then the heavy-first order
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"render {k}"
            assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], f"render {k}"


@pytest.mark.parametrize("every", ["2", "3"])
def test_order_rebuilt_every_kth_render_bit_exact(monkeypatch, every):
    """SF_ORDER_EVERY=k: renders between two order rebuilds record tile costs without the histogram and
    keep the last order (sf_capi.hip `rebuild`). Every render still equals the golden c2 frame, the kept
    order stays a valid permutation of the tiles, and a rebuild after skipped renders gives the order of
    the costs it was built from (no histogram counts carried over from the skipped renders). (SF_ORDER=1: c2
    is not ordered by default.)"""
    monkeypatch.setenv("SF_ORDER", "1")
    monkeypatch.setenv("SF_ORDER_EVERY", every)
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    n = ((W + 7) // 8) * ((H + 7) // 8)
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(2 * int(every) + 2):
            s.Render()
            pos, nrm, _, _ = s.download()
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"render {k}"
            units, cost = s.tile_order()
            tiles = units & ((1 << 27) - 1)
            assert np.array_equal(np.unique(tiles), np.arange(n)), f"render {k}: order is not a permutation"
            if k % int(every) == 0:   # a rebuild render (0, k, 2k, ...): the order of its own costs
                assert len(units) == n   # (14 400 tiles > the persistent grid's waves: no splits)
                assert np.array_equal(units, expected_units(cost, None, 0)[0]), f"render {k}"
        st = s.stats()
    assert st.max_depth == fx["stats"]["max_depth"]


def test_camera_inside_bounding_ball_uses_fixup_levels():
    """K = 0.2 puts the camera inside the flake's bounding ball: no geometric level bound, so the
    adaptive levels and the overflow re-trace path carry the frame (c5's camera on a small frame)."""
    W, H, K = 256, 256, 0.2
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render(emit_aux=True)
        a = s.download(aux=True)
        s.Render(emit_aux=True)
        b = s.download(aux=True)
        st = s.stats()
    for x, y in zip(a, b):
        assert np.array_equal(np.ascontiguousarray(x).view(np.uint8), np.ascontiguousarray(y).view(np.uint8))
    assert st.overflow_tiles == 0


# ---- the reference's SSE variant: LOD 60, 4-lane packets, 2x2 footprint

@pytest.mark.parametrize("name", ["s1", "s2"])
def test_sse_variant_tiny_frames_bit_exact(name):
    exp = load_npz(name)
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetVariant("sse")
        assert s.GetVariant() == sf.SF_VARIANT_SSE
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render(emit_aux=True)
        pos, nrm, mint, idx = s.download(aux=True)
        st = s.stats()
    for k, got in (("pos4", pos), ("nrm4", nrm), ("minT", mint), ("index", idx)):
        assert np.array_equal(np.ascontiguousarray(got).view(np.uint8), np.ascontiguousarray(exp[k]).view(np.uint8)), k
    check_stats(fx, st, mint)


@pytest.mark.parametrize("name", ["s3", "s4"])
def test_sse_variant_config_frames_bit_exact(name):
    """Full frames, rendered twice (the second with the heavy-first tile order) after switching an AVX
    context to the SSE variant: the switch must reset every per-variant table and hint."""
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render()
        s.SetVariant("sse")
        for k in range(2):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"render {k}"
            assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], f"render {k}"
        st = s.stats()
    assert st.max_depth == fx["stats"]["max_depth"]


@pytest.mark.parametrize("name", ["ps1", "ps2", "ps3", "ps4"])
def test_sse_variant_progressive_matches_reference_worker(name):
    """Frame-less mode of the SSE build: 4-ray packets on the 2x2 footprint (Sphereflake.cpp:115-138)."""
    fx = load_progressive(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetVariant(sf.SF_VARIANT_SSE)
        s.SetCamera(sf.config_camera(W, H, K))
        half = fx["packets"] // 3
        s.Progressive(fx["seed"], half, counter0=0)
        s.Progressive(fx["seed"], fx["packets"] - half)
        pos, nrm, _, _ = s.download()
        st = s.stats()
    bad = bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm))
    assert bad == [], f"{len(bad)} rows differ, first {bad[:5]}"
    assert st.max_depth == fx["stats"]["max_depth"]
    assert np.float32(st.closest) == np.float32(float.fromhex(fx["stats"]["closest"]))
    assert st.rays == fx["stats"]["rays"]


def cost_bucket(c):
    """Host restatement of the kernels' cost_bucket (sf_kernels.hip): 2 log buckets per octave from 2^8."""
    k = (np.asarray(c | 1, np.uint32).astype(np.float32).view(np.uint32) >> 22).astype(np.int64)
    b = k - (135 << 1)
    return np.where((b >= 0) & (b < 32), b, np.where(k < (135 << 1), 0, 31))


def expected_units(cost, split_buckets, spare=0, parts=2, prio_buckets=8):
    """Host restatement of sf_order_scan + sf_order_scatter: tiles stably sorted by cost bucket, heaviest
    first; split tiles become `parts` adjacent part units (halves tile | 1 << 29, tile | 2 << 29; quarters
    tile | 3..6 << 29). split_buckets None (auto): whole buckets from the heaviest while the extra units
    fit `spare` idle waves; k: the top k occupied buckets, at most an eighth of the tiles. Bucket 0 is
    never split. Every unit carries its wave priority at bit 27 (SF_UNIT_PRIO_SHIFT): of the top
    `prio_buckets` buckets from the highest occupied one down, the lowest 3 get 1 and the ones above 2."""
    n = len(cost)
    bk = cost_bucket(cost)
    cnt = np.bincount(bk, minlength=32)
    occ = np.nonzero(cnt)[0]
    btop = int(occ[-1]) if len(occ) else 0
    pb = 32 if prio_buckets == 0 else max(0, btop - prio_buckets + 1)
    prio = lambda b: (2 if b >= pb + 3 else 1 if b >= pb else 0) << 27
    bs, nsplit = 32, 0
    if split_buckets is None:
        for b in range(31, 0, -1):
            if (nsplit + cnt[b]) * (parts - 1) > spare:
                break
            nsplit += int(cnt[b])
            bs = b
    elif split_buckets:
        nz = np.nonzero(cnt[1:])[0]
        bmax = int(nz[-1]) + 1 if len(nz) else 0
        bs = max(1, bmax - split_buckets + 1)
        nsplit = int(cnt[bs:].sum())
        while bs < 32 and 8 * nsplit > n:
            nsplit -= int(cnt[bs])
            bs += 1
    first = 3 if parts == 4 else 1
    units = []
    for t in np.lexsort((np.arange(n), -bk)):
        u = int(t) | prio(bk[t])
        if bk[t] >= bs:
            units += [u | ((first + p) << 29) for p in range(parts)]
        else:
            units.append(u)
    return np.array(units, np.uint32), nsplit


@pytest.mark.parametrize("W,H,split,parts", [(1920, 1080, None, 2), (1920, 1080, 1, 2), (1920, 1080, 3, 2),
                                             (3840, 2160, 1, 2), (100, 60, 1, 2), (100, 60, None, 2), (640, 360, None, 2),
                                             (1920, 1080, 2, 4), (640, 360, None, 4), (100, 60, None, 4)])
def test_tile_order_is_stable_heavy_first_schedule(W, H, split, parts, monkeypatch):
    """The next render's work units (sf_order_scan + sf_order_scatter) are exactly the stable sort of
    the last render's tile costs by bucket, heaviest first, with the heaviest tiles as 2 or 4 part units:
    every tile covered once (whole, or all its parts). (SF_ORDER=1: the order on whatever the frame size.)
    Three renders, each rebuilding the order (SF_ORDER_EVERY=1), so the cleared histograms are covered too, for
    orders scattered by the scan's own workgroup (<= SF_ORDER_FUSE_CHUNKS chunks) and by sf_order_scatter."""
    monkeypatch.setenv("SF_ORDER", "1")
    monkeypatch.setenv("SF_ORDER_EVERY", "1")
    monkeypatch.setenv("SF_SPLIT_BUCKETS", "auto" if split is None else str(split))
    monkeypatch.setenv("SF_SPLIT_PARTS", str(parts))
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, 0.25))
        assert s.tile_order() is None
        for _ in range(3):
            s.Render()
            check_tile_order(W, H, split, parts, *s.tile_order())


def check_tile_order(W, H, split, parts, units, cost):
    n = ((W + 7) // 8) * ((H + 7) // 8)
    if split is None:   # auto: recover the idle-wave count from the split made (<= spare < next bucket)
        n_extra = len(units) - n
        exp, nsplit = expected_units(cost, None, n_extra, parts)
    else:
        exp, nsplit = expected_units(cost, split, parts=parts)
    assert np.array_equal(units, exp)
    assert len(units) == n + nsplit * (parts - 1)
    tiles, part = units & ((1 << 27) - 1), units >> 29
    first = 3 if parts == 4 else 1
    assert np.array_equal(np.sort(tiles[(part == 0) | (part == first)]), np.arange(n, dtype=np.uint32))
    for p in range(1, parts):
        assert np.array_equal(np.sort(tiles[part == first]), np.sort(tiles[part == first + p]))
    if split is None and W * H >= 1920 * 1080:
        assert nsplit == 0   # auto: more tiles than resident waves, nothing split
    elif split is None and W * H <= 100 * 60:
        assert nsplit == np.count_nonzero(cost_bucket(cost) >= 1)   # few tiles: every splittable one
    elif W * H > 100 * 60:
        assert nsplit > 0
    # (a 100x60 frame's 104 tiles with an explicit bucket count: its top bucket may hold more than the eighth of
    # the tiles that may split -- with the one-wave kernel its costs are flat enough -- and then none is split;
    # the schedule still equals the restatement, asserted above)


@pytest.mark.parametrize("parts", [2, 4])
def test_split_render_bit_exact_and_stable(parts, monkeypatch):
    """With part units in the schedule (renders 2+: halves or quarters), c3 stays bit-exact, splitting the
    heaviest bucket and with every tile split-eligible (SF_SPLIT_BUCKETS=32: the cap of one eighth of the
    tiles applies). (SF_ORDER=1: the order -- and with it the splits -- on for this full-grid frame.)"""
    fx = load_frame("c3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    import os
    monkeypatch.setenv("SF_ORDER", "1")
    monkeypatch.setenv("SF_SPLIT_PARTS", str(parts))
    for split in ("1", "32"):
        os.environ["SF_SPLIT_BUCKETS"] = split
        try:
            with sf.Sphereflake(W, H) as s:
                s.SetCamera(sf.config_camera(W, H, K))
                for k in range(3):
                    s.Render(emit_aux=True)
                    pos, nrm, mint, idx = s.download(aux=True)
                    assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"split {split} render {k}"
                    assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], f"split {split} render {k}"
                units, _ = s.tile_order()
                st = s.stats()
            assert (units >> 29).max() == (6 if parts == 4 else 2)
            assert st.max_depth == fx["stats"]["max_depth"] and st.overflow_tiles == 0
        finally:
            del os.environ["SF_SPLIT_BUCKETS"]


def test_progressive_adaptive_levels_fixup(monkeypatch):
    """Frame-less batches provision LDS levels for the deepest level seen so far + 1; a wave that needs
    more is re-traced by sf_progressive_fixup. Moving the camera from the depth-5 view (levels 6) to the
    depth-8 view forces that path: the frame equals the same calls with SF_PROGRESSIVE_LEVELS always
    (SF_PROG_ADAPT=0), bit for bit, and nothing is left unresolved."""
    W, H = 640, 360

    def run():
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, 1.0))
            s.Progressive(5, 70000, counter0=0)
            s.Synchronize()
            s.SetCamera(sf.config_camera(W, H, 0.25))
            for _ in range(3):
                s.Progressive(5, 70000)
            s.Synchronize()
            pos, nrm, _, _ = s.download()
            return pos, nrm, s.stats()

    pos, nrm, st = run()
    monkeypatch.setenv("SF_PROG_ADAPT", "0")
    epos, enrm, est = run()
    assert np.array_equal(pos.view(np.uint32), epos.view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), enrm.view(np.uint32))
    assert (st.max_depth, st.closest) == (est.max_depth, est.closest)
    assert st.max_depth >= 8 and st.overflow_tiles == 0 and est.overflow_tiles == 0


def test_progressive_full_size_batches_binned_equal_unbinned(monkeypatch):
    """The bench / Initialize() batch shape: 1920x1080 at the depth-8 camera, batches of 2^18 packets
    (sf_packet_scan over 32 400 bins, 32 per scan thread, staged through LDS). Binning only changes the
    trace order: two such batches continuing one stream give the frame, stats and ray count of the
    same calls traced in draw order (SF_PROG_BIN=0), bit for bit. A scan that lost or duplicated a
    packet in the permutation would leave pixels of the missing packets unwritten or stale."""
    W, H, K, B = 1920, 1080, 0.25, 1 << 18

    def run():
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, K))
            s.Progressive(99, B, counter0=0)
            s.Progressive(99, B)
            s.Synchronize()
            pos, nrm, _, _ = s.download()
            return pos, nrm, s.stats()

    pos, nrm, st = run()
    monkeypatch.setenv("SF_PROG_BIN", "0")
    epos, enrm, est = run()
    assert np.array_equal(pos.view(np.uint32), epos.view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), enrm.view(np.uint32))
    assert (st.max_depth, st.closest, st.rays) == (est.max_depth, est.closest, est.rays)
    assert st.rays == 2 * 8 * B and (pos[..., 3] == 1.0).sum() > W * H // 2


@pytest.mark.parametrize("nq", ["1", "2", "4"])
def test_fewer_tile_queues_bit_exact(nq, monkeypatch):
    """The persistent grid drains one queue per XCD; a partitioned chip exposes fewer XCDs and uses
    fewer queues (SF_NQUEUES forces the count): every unit is still traced, frames equal the golden."""
    monkeypatch.setenv("SF_NQUEUES", nq)
    for name in ("c2", "c3"):
        fx = load_frame(name)
        W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, K))
            for _ in range(2):   # row-major, then the heavy-first unit order
                s.Render()
                pos, nrm, _, _ = s.download()
                assert frame_digest(pos, nrm) == fx["frame_digest"], (name, nq)


@pytest.mark.parametrize("prio", ["0", "1", "32"])
def test_raised_priority_tiles_bit_exact(prio, monkeypatch):
    """The top SF_PRIO_BUCKETS cost buckets of the last render run at raised wave priority (none / the
    top one / all): scheduling only, frames equal the golden. (SF_ORDER=1: the order on for this full grid.)"""
    monkeypatch.setenv("SF_ORDER", "1")
    monkeypatch.setenv("SF_PRIO_BUCKETS", prio)
    fx = load_frame("c3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for _ in range(3):
            s.Render()
            pos, nrm, _, _ = s.download()
            assert frame_digest(pos, nrm) == fx["frame_digest"], prio
        units, cost = s.tile_order()
    lv = (units >> 27) & 3
    assert np.array_equal(units, expected_units(cost, None, len(units) - len(cost), 4, int(prio))[0])
    if prio == "0":
        assert lv.max() == 0
    elif prio == "32":
        assert lv.min() >= 1 and lv.max() == 2
    else:
        assert 0 < np.count_nonzero(lv) < len(units)


@pytest.mark.parametrize("name,ordered", [("c1", True), ("c2", False), ("c3", True), ("c4", True)])
def test_tile_order_auto_by_frame_size(name, ordered):
    """Default tile order (sf_capi.hip order_mode -1): heavy-first for frames whose tiles fill at most half the
    persistent grid's waves (c1: 3 600 tiles for 8 192 waves) and for frames of more than twice its waves (c3, c4:
    rebuilt every 64th render, no splits), row-major between (c2: 14 400 tiles, where the order measured
    slower). Either way every render equals the golden frame."""
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(3):
            s.Render()
            pos, nrm, _, _ = s.download()
            assert frame_digest(pos, nrm) == fx["frame_digest"], (name, k)
        assert (s.tile_order() is not None) == ordered


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4"])
def test_occlusion_cull_on_off_identical(name, monkeypatch):
    """The per-ray traversal's occlusion cull (a lane skips a subtree whose fattened bounding ball starts
    beyond its nearest hit, and only where the subtree cannot pass LOD deeper than the depth already
    reached) changes neither a pixel nor a statistic: frames with the cull off (SF_FLAGS=0x100) and on are
    identical -- G-buffer, minT, hit index, max depth, closest -- and equal the golden frame."""
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    out = {}
    for flags in ("0x100", "0"):
        monkeypatch.setenv("SF_FLAGS", flags)
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, K))
            for _ in range(2):   # row-major, then heavy-first order
                s.Render(emit_aux=True)
            out[flags] = s.download(aux=True), s.stats()
    (a, sa), (b, sb) = out["0x100"], out["0"]
    for x, y in zip(a, b):
        assert np.array_equal(np.ascontiguousarray(x).view(np.uint8), np.ascontiguousarray(y).view(np.uint8))
    assert (sa.max_depth, sa.closest, sa.rays) == (sb.max_depth, sb.closest, sb.rays)
    assert frame_digest(b[0], b[1]) == fx["frame_digest"]
    assert sb.max_depth == fx["stats"]["max_depth"]


@pytest.mark.parametrize("blocks,nq", [("4", "8"), ("3", "8"), ("1", "8"), ("6", "4")])
def test_tiny_grid_many_queues_bit_exact(blocks, nq, monkeypatch):
    """A persistent grid of fewer blocks than tile queues (SF_MAX_BLOCKS below SF_NQUEUES, as a CU-masked
    stream or a partitioned chip can give): the host drops to as many queue groups as the grid has blocks,
    so every queue has waves and every unit is traced -- golden frames, first and heavy-first renders."""
    monkeypatch.setenv("SF_MAX_BLOCKS", blocks)
    monkeypatch.setenv("SF_NQUEUES", nq)
    fx = load_frame("t3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    exp = load_npz("t3")
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for _ in range(2):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            for k, got in (("pos4", pos), ("nrm4", nrm), ("minT", mint), ("index", idx)):
                assert np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                                      np.ascontiguousarray(exp[k]).view(np.uint8)), (k, blocks, nq)


@pytest.mark.parametrize("sizes", [(40000,), (16400, 70001, 5), (1 << 18, 1 << 18), (300, 50000, 624 * 40 + 7)])
def test_parallel_mt_draws_equal_sequential(sizes, monkeypatch):
    """The frame-less draws from the jump-ahead generator (K segments, each started from the stream state
    the polynomial t^(j L) mod phi jumps to; sf_mt_raw / sf_mt_jump_partial / sf_mt_segments) equal the
    single-workgroup generator's (SF_MT_PARALLEL=0) over batch sequences of assorted sizes, including
    mid-buffer starts: same frames, same stats. (Prefetch off, so every batch generates its own draws.)"""
    W, H, K = 320, 180, 0.25
    monkeypatch.setenv("SF_PROG_PREFETCH", "0")

    def run():
        with sf.Sphereflake(W, H) as s:
            s.SetCamera(sf.config_camera(W, H, K))
            c = 0
            for n in sizes:
                s.Progressive(2024, n, counter0=c)
                c += n
            s.Progressive(2024, 3000, counter0=c + 12345)   # a jump (host) into the stream
            pos, nrm, _, _ = s.download()
            return pos, nrm, s.stats()

    pos, nrm, st = run()
    monkeypatch.setenv("SF_MT_PARALLEL", "0")
    epos, enrm, est = run()
    assert np.array_equal(pos.view(np.uint32), epos.view(np.uint32))
    assert np.array_equal(nrm.view(np.uint32), enrm.view(np.uint32))
    assert (st.max_depth, st.closest, st.rays) == (est.max_depth, est.closest, est.rays)


@pytest.mark.parametrize("inline,order", [("1", ""), ("0", ""), ("1", "split")])
@pytest.mark.parametrize("flags", ["0x200", "0x400"])
@pytest.mark.parametrize("name", ["t3", "c2"])
def test_front_first_order_and_tie_fallback(name, flags, inline, order, monkeypatch):
    """Children entered in index order only (SF_FLAG_NO_FRONT_FIRST), and every tile forced through the tie
    fallback of the front-first order (SF_FLAG_DIAG_FORCE_RETRACE): with the levels proven, the tile's own wave
    re-traces it in index order at once (SF_TIE_INLINE, default; also with the heavy-first order splitting tiles into
    part units), or (SF_TIE_INLINE=0) it is queued like an overflow and sf_fixup_wave re-traces it: golden frames,
    aux channels and stats every way."""
    monkeypatch.setenv("SF_FLAGS", flags)
    monkeypatch.setenv("SF_TIE_INLINE", inline)
    if order == "split":
        monkeypatch.setenv("SF_ORDER", "1")
        monkeypatch.setenv("SF_SPLIT_BUCKETS", "model")
        monkeypatch.setenv("SF_SPLIT_PARTS", "4")
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for _ in range(3):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert frame_digest(pos, nrm) == fx["frame_digest"], flags
            if "row_digest_aux" in fx and fx.get("row_step", 1) == 1:
                assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == []
        st = s.stats()
    assert st.max_depth == fx["stats"]["max_depth"]
    assert np.float32(st.closest) == np.float32(float.fromhex(fx["stats"]["closest"]))
    assert st.overflow_tiles == 0


@pytest.mark.parametrize("order", ["0", "1"])
def test_member_share_with_and_without_order_bit_exact(order, monkeypatch):
    """A multi-GPU member's share (band 3 of an 8-way split of c2's 8-row bands) rendered four times on a fresh
    context with the heavy-first order forced on (SF_ORDER=1: the scan's own workgroup scatters the small order,
    heavy tiles split into idle wave slots) and off (the default for shares): every render's rows equal the
    whole frame's, bit for bit."""
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        s.Render()
        ref_pos, ref_nrm, _, _ = s.download()
    assert bad_rows(fx["row_digest_gbuf"], row_digests(ref_pos, ref_nrm)) == []
    monkeypatch.setenv("SF_ORDER", order)
    rows = [y for b in range(3, (H + 7) // 8, 8) for y in range(8 * b, min(8 * b + 8, H))]
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(4):
            s.Render(band_rows=8, band_count=8, band_index=3)
            pos, nrm, _, _ = s.download()
            assert np.array_equal(pos[rows].view(np.uint32), ref_pos[rows].view(np.uint32)), k
            assert np.array_equal(nrm[rows].view(np.uint32), ref_nrm[rows].view(np.uint32)), k
        # (sf_get_tile_order reports whole-frame orders only: a share's order is not readable through it)
        assert s.stats().overflow_tiles == 0


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4"])
def test_active_ray_compaction_kernel_bit_exact(name, monkeypatch):
    """The opt-in trace kernel with active-ray compaction of sparse nodes (SF_COMPACT=1, sf_trace_queue2c: the few
    rays visiting a node packed by their prefix-sum rank so one wave pass tests all its children) is a filter: the
    G-buffer, minT, hit index and stats equal the golden frame's on every render (row-major, then ordered)."""
    monkeypatch.setenv("SF_COMPACT", "1")
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(2):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], (name, k)
            if fx.get("row_step", 1) == 1:
                assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], (name, k)
        st = s.stats()
    assert st.max_depth == fx["stats"]["max_depth"] and st.overflow_tiles == 0


@pytest.mark.parametrize("name", ["t3", "t5"])
def test_row_major_halves_bit_exact(name, monkeypatch):
    """SF_HALVES=1 (SF_FLAG_HALVES, round-6 A/B): row-major frames traced as tile halves (pixel rows 0-3 / 4-7, two
    waves per tile) equal the golden frames bit for bit, twice in a row (the queues' second parity)."""
    monkeypatch.setenv("SF_HALVES", "1")
    monkeypatch.setenv("SF_ORDER", "0")
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    exp = load_npz(name)
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for _ in range(2):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            for k, got in (("pos4", pos), ("nrm4", nrm), ("minT", mint), ("index", idx)):
                assert np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                                      np.ascontiguousarray(exp[k]).view(np.uint8)), (k, name)


def test_set_setup_refuses_non_affine_child_frames():
    """The kernels fuse the 4th term of every child product (SF_AFFINE_FMA: exact only when row 3 of every unit child
    frame is 0, 0, 0, 1, as the reference's ComputeChildTransformations makes them), so sf_set_setup refuses any other
    child frames with SF_EINVAL and keeps the setup it had; the affine setup read back is accepted unchanged."""
    with sf.Sphereflake(64, 32) as s:
        child, root = s.GetSetup()
        assert np.all(child.reshape(9, 4, 4)[:, :3, 3] == 0.0) and np.all(child.reshape(9, 4, 4)[:, 3, 3] == 1.0)
        s.SetSetup(child, root)
        for col, val in ((0, 1e-30), (3, 1.0 + 2.0 ** -23), (1, -0.0 + 0.5)):
            bad = child.copy().reshape(9, 16)
            bad[4, 4 * col + 3] = val
            with pytest.raises(sf.SphereflakeError) as e:
                s.SetSetup(bad, root)
            assert e.value.code == sf.SF_EINVAL
        c2, r2 = s.GetSetup()
        assert np.array_equal(c2.view(np.uint32), child.view(np.uint32)) and np.array_equal(r2.view(np.uint32), root.view(np.uint32))
