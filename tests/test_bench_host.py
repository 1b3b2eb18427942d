"""Host logic of bench.py on the CPU: the parity check of the timed frames (golden row digests, the rows a rank
owns), the roofline/issue arithmetic on the frame period, and the rank launcher's world check."""
import numpy as np
import pytest

from conftest import REPO, load_frame, load_npz

import bench


@pytest.mark.parametrize("name", ["t1", "t2", "t3"])
def test_golden_row_check_accepts_reference_frame_and_flags_a_bit(name):
    """check_golden_rows: the reference-rendered frame passes every row; one flipped mantissa bit in one pixel is
    reported as that row (the bench exits 5 on it)."""
    fx = load_frame(name)
    ref = load_npz(name)
    pos, nrm = ref["pos4"].copy(), ref["nrm4"].copy()
    H = pos.shape[0]
    n, bad = bench.check_golden_rows(pos, nrm, fx, np.arange(H))
    assert n == H and bad == []
    y = H // 2
    nrm.view(np.uint32)[y, 3, 1] ^= 1
    n, bad = bench.check_golden_rows(pos, nrm, fx, np.arange(H))
    assert bad == [y]


def test_golden_row_check_respects_row_step_and_ownership():
    """Only the rows the fixture holds (every row_step-th) and the rows this rank owns are checked."""
    fx = load_frame("t3")
    ref = load_npz("t3")
    H = ref["pos4"].shape[0]
    fx2 = dict(fx, row_step=2, row_digest_gbuf=fx["row_digest_gbuf"][::2])
    rows = bench.owned_rows(H, 8, 3, 1)
    n, bad = bench.check_golden_rows(ref["pos4"], ref["nrm4"], fx2, rows)
    assert bad == [] and n == len([y for y in rows if y % 2 == 0])


@pytest.mark.parametrize("H,band,world", [(1080, 8, 8), (45, 8, 3), (7, 8, 2)])
def test_owned_rows_partition_the_frame(H, band, world):
    rows = np.concatenate([bench.owned_rows(H, band, world, r) for r in range(world)])
    assert np.array_equal(np.sort(rows), np.arange(H))
    assert np.array_equal(bench.owned_rows(H, band, 1, 0), np.arange(H))


def test_issue_fractions_on_the_frame_period():
    """pmc_valu prices the PMC instruction counts on one frame period at the live clock: VALU over 1024 SIMDs x
    cycles / 2, SALU over 256 CUs x cycles; the lone-dispatch view stays separate."""
    c = {"SQ_INSTS_VALU": 59.5e6, "SQ_INSTS_SALU": 33.0e6, "GRBM_GUI_ACTIVE": 8 * 300000.0, "SQ_WAVE_CYCLES": 3.5e8,
         "profiled_dispatch_us": 130.0, "SQ_WAIT_INST_ANY": 1.35e8, "SQ_WAIT_ANY": 1.0e8}
    v = bench.pmc_valu(c, 0.078, 2370.0)
    fc = 0.078e-3 * 2370e6
    assert v["frame_cycles"] == round(fc)
    assert abs(v["valu_issue_frac"] - 59.5e6 / (1024 * fc / 2)) < 1e-4
    assert abs(v["salu_issue_frac"] - 33.0e6 / (256 * fc)) < 1e-4
    # the lone dispatch's cycles: its duration at the live clock (never a clock above the gfx950 maximum)
    lc = 130.0 * 2370.0
    assert v["lone_dispatch"]["clock_mhz"] == 2370.0
    assert v["lone_dispatch"]["valu_issue_frac"] == round(59.5e6 / (1024 * lc / 2), 4)
    assert v["lone_dispatch"]["occupancy"]["mean_waves"] == round(4.0 * 3.5e8 / lc, 1)
    assert bench.pmc_valu(None, 0.078, 2370.0) is None


@pytest.mark.parametrize("w,h,n,want", [(1920, 1080, 1, 3), (1920, 1080, 2, 3), (1920, 1080, 4, 4), (1920, 1080, 8, 8),
                                        (640, 360, 1, 4), (1280, 720, 1, 3), (3840, 2160, 8, 3), (3840, 2160, 1, 3)])
def test_frames_in_flight_by_share(w, h, n, want, monkeypatch):
    """8 frames in flight where rank 0's band share of 8x8 tiles is at most 3/4 of a persistent grid (256 CUs x 32
    waves) and the slot streams have hardware queues of their own (the library's default; else the process needs the
    16 shared queues bench.py gives it), 4 up to 1.5 grids (and for small whole
    frames), else 3; an explicit --slots wins
    (clamped to batch..16). With multi-frame launches of B frames (round 6), B x GROUPS_IN_FLIGHT slots, and never
    fewer slots than one launch's frames."""
    assert int(bench.os.environ["GPU_MAX_HW_QUEUES"]) >= bench.HW_QUEUES   # (raised at import, before any HIP call)
    assert bench.frames_in_flight(0, 256, w, h, 8, n) == want
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")   # (the slot streams have queues of their own: 4 shared ones do)
    assert bench.frames_in_flight(0, 256, w, h, 8, n) == want
    monkeypatch.setenv("SF_STREAM_CUMASK", "0")    # (plain streams on HIP's 4 shared queues: 4 for small shares)
    assert bench.frames_in_flight(0, 256, w, h, 8, n) == (4 if want == 8 else want)
    monkeypatch.delenv("SF_STREAM_CUMASK")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", str(bench.HW_QUEUES))
    assert bench.frames_in_flight(5, 256, w, h, 8, n) == 5
    assert bench.frames_in_flight(99, 256, w, h, 8, n) == 16
    assert bench.frames_in_flight(0, 256, w, h, 8, n, batch=4) == 4 * bench.GROUPS_IN_FLIGHT
    assert bench.frames_in_flight(2, 256, w, h, 8, n, batch=4) == 4
    assert bench.frames_per_launch(3, 256, w, h, 8, n) == 3
    # one frame per launch (the multi-frame launch is opt-in: --batch)
    assert bench.frames_per_launch(0, 256, w, h, 8, n) == (bench.BATCH_TINY if want == 8 else 1) == 1
    assert bench.frames_in_flight(0, 256, w, h, 8, n, batch=8) == 16


def test_cpu_model_and_vendor_parsed():
    """the CPU baseline states the CPU model; the vendor decides whether its frames can match the
    Intel-measured rsqrtps fixtures (AMD hosts: timing-only)."""
    amd = ("processor\t: 0\nvendor_id\t: AuthenticAMD\ncpu family\t: 26\n"
           "model name\t: AMD EPYC 9575F 64-Core Processor\nflags\t\t: fpu avx2\n\nprocessor\t: 1\n"
           "vendor_id\t: AuthenticAMD\nmodel name\t: AMD EPYC 9575F 64-Core Processor\n")
    assert bench.cpu_model(amd) == ("AMD EPYC 9575F 64-Core Processor", "AuthenticAMD")
    intel = "vendor_id\t: GenuineIntel\nmodel name\t: Intel(R) Xeon(R)   Platinum 8480+\n"
    assert bench.cpu_model(intel) == ("Intel(R) Xeon(R) Platinum 8480+", "GenuineIntel")
    assert bench.cpu_model("processor : 0\n") == (None, None)
    ident = bench.cpu_identity()   # this host's /proc/cpuinfo
    assert set(ident) >= {"cpu_model", "vendor"}
    assert ("note" in ident) == (ident["vendor"] != "GenuineIntel")
