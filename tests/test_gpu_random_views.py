"""GPU parity on seeded random views (beyond the fixed BASELINE cameras): random camera position
(scale K log-uniform over [0.12, 2.5], inside and outside the flake's bounding ball), pitch, yaw,
roll, FOV and frame sizes that are not multiples of the 8x8 tile, both reference variants (AVX LOD 70,
SSE LOD 60). Each view is rendered three times -- row-major, then heavy-first, then with the heavy-
first schedule's half units where the frame leaves idle waves -- and every render must equal the oracle
restatement (oracle/sf_oracle.c, pinned to the reference build by tests/golden) bit for bit in
position, normal, t and heap hit index. Camera setup (a1-a3) comes from the library, as in the
product path; its bit-exactness against the reference dump is tests/test_host.py's job."""
import numpy as np
import pytest

import sphereflake_amd as sf
from oracle import pyoracle

pytestmark = pytest.mark.gpu

SIZES = [(72, 40), (61, 37), (96, 54), (33, 70), (128, 72)]


def random_view(rng, k):
    W, H = SIZES[k % len(SIZES)]
    cam = sf.Camera(W, H)
    K = float(np.exp(rng.uniform(np.log(0.12), np.log(2.5))))
    cam.SetPosition(np.asarray(sf.DEFAULT_CAMERA_POSITION, np.float32) * np.float32(K)
                    + rng.normal(0.0, 0.15 * K, 3).astype(np.float32))
    cam.SetPitch(np.float32(sf.DEFAULT_PITCH + rng.uniform(-0.4, 0.4)))
    cam.SetYaw(np.float32(sf.DEFAULT_YAW + rng.uniform(-0.6, 0.6)))
    cam.SetRoll(np.float32(rng.uniform(-0.3, 0.3)))
    cam.SetFOV(float(rng.choice([45.0, 60.0, 90.0])))
    return W, H, K, cam


@pytest.mark.parametrize("variant", ["avx", "sse", "compact", "subtree", "subtree_d2"])
@pytest.mark.parametrize("seed", range(16))
def test_random_view_bit_exact(seed, variant, monkeypatch):
    """("compact": the AVX variant traced by the opt-in active-ray compaction kernel, SF_COMPACT=1 with the
    throughput variant forced, SF_PIPE=0, since these small frames would take the latency variant. "subtree":
    the AVX variant with the split tiles traced as subtree parts, SF_SPLIT_PARTS=subtree, at the default split
    depth and at depth 2 -- these frames leave idle waves, so renders 2 and 3 split their heaviest tiles.)"""
    if variant == "compact":
        monkeypatch.setenv("SF_COMPACT", "1")
        monkeypatch.setenv("SF_PIPE", "0")
        variant = "avx"
    elif variant.startswith("subtree"):
        monkeypatch.setenv("SF_SPLIT_PARTS", "subtree")
        if variant == "subtree_d2":
            monkeypatch.setenv("SF_SPLIT_DEPTH", "2")
        variant = "avx"
    rng = np.random.default_rng(1000 + seed)
    W, H, K, cam = random_view(rng, seed)
    o, tl, tr, bl = cam.corners()
    setup = {"W": W, "H": H, "origin": o, "tl": tl, "tr": tr, "bl": bl,
             "root": sf.root_transform(o), "children": sf.child_transforms()}
    ref = pyoracle.render(setup, lod=70.0 if variant == "avx" else 60.0)
    with sf.Sphereflake(W, H) as s:
        s.SetVariant(variant)
        s.SetView(o, tl, tr, bl)
        for k in range(3):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            what = f"seed {seed} {variant} {W}x{H} K={K:.3f} render {k}"
            assert np.array_equal(idx, ref["index"]), what
            assert np.array_equal(pos.view(np.uint32), ref["pos4"].view(np.uint32)), what
            assert np.array_equal(nrm.view(np.uint32), ref["nrm4"].view(np.uint32)), what
            assert np.array_equal(mint.view(np.uint32), ref["minT"].view(np.uint32)), what
        st = s.stats()
    assert st.max_depth == ref["stats"]["max_depth"]
    assert np.float32(st.closest) == np.float32(ref["stats"]["closest"])


@pytest.mark.parametrize("seed", range(16))
def test_random_view_band_slabs_bit_exact(seed):
    """The multi-GPU slab formats on random views (camera scale 0.12-2.5: inside and outside the flake's bounding
    ball, where the index format's depth proof succeeds or falls back): member 0's bands in place, members 1-2 as
    slabs of the format sf_slab_bytes picks for the view, unpacked beside them -- the frame equals the oracle bit for
    bit. When the view allows 4-B slabs the 16-B form is unpacked too."""
    import torch
    rng = np.random.default_rng(1000 + seed)
    W, H, K, cam = random_view(rng, seed)
    o, tl, tr, bl = cam.corners()
    setup = {"W": W, "H": H, "origin": o, "tl": tl, "tr": tr, "bl": bl,
             "root": sf.root_transform(o), "children": sf.child_transforms()}
    ref = pyoracle.render(setup)
    n, band = 3, 8
    sr = max(sf.lib().sf_slab_rows(H, band, n, k) for k in range(1, n))
    with sf.Sphereflake(W, H) as s:
        s.SetView(o, tl, tr, bl)
        fmts = [4, 16] if s.slab_bytes() == 4 else [16]
        for bpp in fmts:
            stage = torch.full((n - 1, sr, W, bpp // 4), float("nan"), dtype=torch.float32, device="cuda")
            s.Render(band_rows=band, band_count=n, band_index=0)
            for k in range(1, n):
                s.render_to(stage[k - 1].data_ptr(), 0, band_rows=band, band_count=n, band_index=k, compact=True,
                            packed=sf.SF_PACKED_INDEX if bpp == 4 else sf.SF_PACKED_NORMAL)
            s.unpack_slabs(stage.data_ptr(), bpp, sr, band, n, 1, n - 1)
            pos, nrm, _, _ = s.download()
            what = f"seed {seed} {W}x{H} K={K:.3f} slab {bpp} B"
            assert np.array_equal(pos.view(np.uint32), ref["pos4"].view(np.uint32)), what
            assert np.array_equal(nrm.view(np.uint32), ref["nrm4"].view(np.uint32)), what
