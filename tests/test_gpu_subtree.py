"""GPU parity of subtree-split tiles (SF_SPLIT_PARTS=subtree, SF_FLAG_SUBTREE; csrc/sf_kernels.hip trace_tile): the
heaviest tiles of the unit order are traced as 4 part units, each tracing the whole 8x8 tile but entering, of the
nodes at the split depth, only those whose heap index is its part mod 4; the part that finishes last merges the four
per-pixel results (nearest sphere; the reference's ancestor rule on an exact tie, else the index-order re-trace) and
writes the tile. Schedules only: every frame must equal the reference-made golden frame (or the oracle restatement)
bit for bit, with the reference's stats."""
import numpy as np
import pytest

from conftest import load_frame
from sfcheck import aux_digests, bad_rows, row_digests

import sphereflake_amd as sf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device():
    sf.build()
    assert sf.device_count() >= 1, "no HIP device visible: GPU tests must run on an MI355X"


def subtree_env(monkeypatch, buckets="32", depth=None, flags=None):
    monkeypatch.setenv("SF_ORDER", "1")
    monkeypatch.setenv("SF_ORDER_EVERY", "1")
    monkeypatch.setenv("SF_SPLIT_PARTS", "subtree")
    monkeypatch.setenv("SF_SPLIT_BUCKETS", buckets)
    if depth is not None:
        monkeypatch.setenv("SF_SPLIT_DEPTH", str(depth))
    if flags is not None:
        monkeypatch.setenv("SF_FLAGS", hex(flags))


@pytest.mark.parametrize("depth", [None, 1, 3])
@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4"])
def test_subtree_split_config_frames_bit_exact(name, depth, monkeypatch):
    """Every BASELINE view with the top cost buckets split (SF_SPLIT_BUCKETS=32: at most an eighth of the tiles, and
    at most SF_SPLIT_CAP -- 4K's eighth is above it), at the default split depth (the view's deepest LOD-passable
    depth - 2) and at depths 1 and 3; renders 2 and 3 trace the split units."""
    subtree_env(monkeypatch, depth=depth)
    fx = load_frame(name)
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(3):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            what = f"{name} depth {depth} render {k}"
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], what
            assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], what
        units, _ = s.tile_order()
        st = s.stats()
    parts = units >> 29
    assert parts.max() == 6 and np.count_nonzero(parts == 3) <= 4096
    assert st.max_depth == fx["stats"]["max_depth"] and st.overflow_tiles == 0


def test_subtree_split_forced_retrace_bit_exact(monkeypatch):
    """Every tile flagged as if a tie had been seen (SF_FLAG_DIAG_FORCE_RETRACE): a split tile's merged flag sends
    the whole tile to its index-order re-trace by the merging wave, and the frame stays exact."""
    subtree_env(monkeypatch, flags=0x400)
    fx = load_frame("c2")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        for k in range(3):
            s.Render(emit_aux=True)
            pos, nrm, mint, idx = s.download(aux=True)
            assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == [], f"render {k}"
            assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == [], f"render {k}"


@pytest.mark.parametrize("buckets", ["auto", "model"])
def test_subtree_split_band_shares_bit_exact(buckets, monkeypatch):
    """A 1080p frame as 8 band shares (a member's share of an 8-GPU frame: half the persistent grid's waves, where
    `auto` splits into the idle slots) rendered into one context, each share three times: the assembled frame
    equals the golden frame."""
    subtree_env(monkeypatch, buckets=buckets)
    fx = load_frame("c3")
    W, H, K = fx["W"], fx["H"], float.fromhex(fx["K"])
    with sf.Sphereflake(W, H) as s:
        s.SetCamera(sf.config_camera(W, H, K))
        split = 0
        for k in range(8):
            for _ in range(3):
                s.Render(band_rows=8, band_count=8, band_index=k, emit_aux=True)
                units, _ = s.tile_order()
                split = max(split, np.count_nonzero((units >> 29) == 3))
        pos, nrm, mint, idx = s.download(aux=True)
    assert bad_rows(fx["row_digest_gbuf"], row_digests(pos, nrm)) == []
    assert bad_rows(fx["row_digest_aux"], aux_digests(mint, idx)) == []
    assert split > 0
