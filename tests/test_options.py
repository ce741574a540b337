"""The bench's own batch path and every entropy-stage variant (C ABI,
include/mijpeg.h), against the oracle (oracle/cpu_ref.c, the restatement of
/root/reference/main/encoder.c, pinned by tests/test_oracle.py).

A config-3-sized batch takes paths no small batch reaches (mij_api.hip
ent_args / run_entropy): 48 JFIF-assembly slots per frame at >= 43 frames
and Q <= 60, the AC tables built beside the segment DCs (k_segdc_actab) plus
DC-only tables at >= 16 frames, and the histogram / pack-state fills the
next encode skips after them.  bench.py verifies its own run; these tests
pin the same paths in the GPU suite, at frame counts that move across the
thresholds in both directions.  Then every MIJ_OPT_* setting other than the
default, which the bench never runs, must give the same bytes."""
import numpy as np
import pytest

import mijpeg
import oracle as O
import recipes

pytestmark = pytest.mark.gpu

W, H = 512, 256


def _frames(n, seed0=0, noise_every=0):
    out = []
    for i in range(n):
        if noise_every and i % noise_every == noise_every - 1:
            out.append(recipes.noise(H, W, 500 + seed0 + i))
        else:
            out.append(recipes.config3_frame(seed0 + i, H, W))
    return np.stack(out)


def _check(b, frames, n, q, want=None):
    for i in range(n):
        ref = want[i] if want is not None else O.cref_encode(frames[i], q)
        got = b.output(i)
        assert got == ref, f"frame {i} of {n} (q{q}): {len(got)} vs {len(ref)} bytes"


def test_bench_sized_batch_frame_counts_across_thresholds():
    """48 config-3 frames + 2 noise frames at Q=50, encoded 50, 17, 50, 5,
    50, 16, 15 frames in turn: the 48-slot emit (>= 43 frames), the AC
    tables beside the segment DCs (>= 16) and the histogram fills skipped
    after them each run after the others; every output is the oracle's."""
    n = 50
    frames = np.concatenate([_frames(48), np.stack([recipes.noise(H, W, 900), recipes.noise(H, W, 901)])])
    want = [O.cref_encode(f) for f in frames]
    b = mijpeg.Batch(W, H, n)
    b.upload(frames)
    for k in (50, 17, 50, 5, 50, 16, 15):
        b.encode(k)
        _check(b, frames, k, 50, want)
    b.close()


def test_high_quality_batch_wide_pack_window():
    """>= 16 frames at Q=90: the wide pack window (Q >= 85), the AC tables
    beside the segment DCs, and the cooperative FP64 replays of a high-Q K1,
    twice in a row (the second encode skips the fills)."""
    n, q = 20, 90
    frames = _frames(n, seed0=60, noise_every=7)
    want = [O.cref_encode(f, q) for f in frames]
    b = mijpeg.Batch(W, H, n, q)
    assert b.geometry()["pack_window_words"] > mijpeg.Batch(64, 64, 1, 50).geometry()["pack_window_words"]
    b.upload(frames)
    for k in (n, 18):
        b.encode(k)
        _check(b, frames, k, q, want)
    assert b.replays() > 0
    b.close()


def test_band_analyze_then_fewer_frames_encode():
    """An encode leaves its counts zeroed and the next encode skips the fill
    for those frames; a band call in between writes the counts (K1 through
    mij_band_analyze, not ent_args), so an encode of no more frames than the
    first must still zero them (encode(3), band_analyze(2),
    encode(2) used to add the band's counts onto the tables)."""
    w, h = 320, 160
    frames = np.stack([recipes.config3_frame(i + 40, h, w) for i in range(3)])
    want = [O.cref_encode(f) for f in frames]
    b = mijpeg.Batch(w, h, 3)
    b.upload(frames)
    b.encode(3)
    _check(b, frames, 3, 50, want)
    b.band_analyze(2)
    b.encode(2)
    _check(b, frames, 2, 50, want)
    b.encode(3)
    _check(b, frames, 3, 50, want)
    b.close()


# (option, value, quality, frames): every non-default setting
CASES = [
    ("seam", 0, 50, 20),
    ("seam", 0, 90, 4),
    ("ff_pack", 0, 50, 20),
    ("ff_pack", 0, 90, 4),
    ("actab", 0, 50, 20),
    ("segdc_fused", 1, 50, 20),
    ("segdc_fused", 1, 75, 3),
    ("pack_wide", 1, 50, 20),
    ("pack_wide", 0, 90, 20),
    ("emit_slots", 8, 50, 20),
    ("emit_slots", 512, 90, 3),
    ("pack_segs", 0, 50, 20),  # 32-segment groups throughout
    ("pack_segs", 5, 50, 20),  # 64 / 64
    ("pack_segs", 15, 50, 20),  # 256-segment groups throughout
    ("pack_segs", 15, 90, 4),  # (groups past the window: the window-by-window path)
    ("pack_segs", 10, 75, 6),  # 128 / 128
]


@pytest.mark.parametrize("opt,value,q,n", CASES)
def test_option_same_bytes(opt, value, q, n):
    frames = _frames(n, seed0=100 + n, noise_every=5)
    b = mijpeg.Batch(W, H, n, q)
    b.set_option(opt, value)
    assert b.get_option(opt) == value
    b.upload(frames)
    want = [O.cref_encode(f, q) for f in frames]
    for k in (n, max(1, n - 3)):  # twice: the second encode skips the fills
        b.encode(k)
        _check(b, frames, k, q, want)
    b.close()


def test_overlap_low_priority_same_bytes():
    n = 6
    frames = _frames(n, seed0=300, noise_every=3)
    b = mijpeg.Batch(W, H, n)
    b.set_option("overlap_prio", 0)
    b.set_overlap(3)
    with pytest.raises(mijpeg.MijError, match="overlap stream exists"):
        b.set_option("overlap_prio", 1)
    b.upload(frames)
    b.encode(n)
    _check(b, frames, n, 50)
    b.close()


def test_option_validation():
    b = mijpeg.Batch(64, 64, 1)
    for opt, bad in (("seam", 2), ("pack_wide", 3), ("emit_slots", -1), ("pack_segs", 16), ("pack_segs", -2)):
        with pytest.raises(mijpeg.MijError, match="out of range"):
            b.set_option(opt, bad)
    with pytest.raises(mijpeg.MijError, match="unknown option"):
        mijpeg._check(b.lib.mij_batch_set_option(b.h_, 99, 0), "set_option")
    b.close()


def test_stale_pack_ticket_fails_the_frame_instead_of_hanging():
    """Every device-side wait is bounded (mij_internal.h SPIN_TICKS).  A
    stale pack ticket (mij_test_stale_ticket, csrc/mij_testing.h -- a
    test-only entry point, not the public option enum: frame 0's luma ticket starts at
    1, so pack group 0 never runs and group 1's look-back waits for a
    publication that never comes) fails frame 0 with MIJ_EHANG within the
    bound, the other frames stay byte-exact, and the next encode of the same
    batch is whole again."""
    import time
    frames = _frames(3)
    want = [O.cref_encode(f) for f in frames]
    b = mijpeg.Batch(W, H, 3)
    b.upload(frames)
    import ctypes as C
    arm = b.lib.mij_test_stale_ticket
    arm.argtypes, arm.restype = [C.c_void_p, C.c_int], C.c_int
    assert arm(b.h_, 1) == 0
    t0 = time.time()
    b.encode(3)
    b.sync()
    assert time.time() - t0 < 10.0, "the bounded wait (2 s without progress) should end the wait"
    with pytest.raises(mijpeg.MijError, match="outlasted its bound"):
        b.output(0)
    assert b.lib.mij_last_error() == 9  # MIJ_EHANG
    for i in (1, 2):
        assert b.output(i) == want[i]
    assert arm(b.h_, 0) == 0  # consumed by that encode
    b.encode(3)
    _check(b, frames, 3, 50, want)
    b.close()


def test_reserved_option_slot_is_not_settable():
    """Option slot 7 is the test suite's fault hook: the public option calls
    refuse it (include/mijpeg.h marks it reserved)."""
    b = mijpeg.Batch(W, H, 1)
    try:
        assert b.lib.mij_batch_set_option(b.h_, 7, 1) != 0
        assert b.lib.mij_batch_get_option(b.h_, 7) == -2
    finally:
        b.close()


def test_get_option_error_raises():
    b = mijpeg.Batch(W, H, 1)
    h = b.h_
    b.h_ = None  # a null handle: mij_batch_get_option returns -2 and sets the error
    try:
        with pytest.raises(mijpeg.MijError):
            b.get_option("seam")
    finally:
        b.h_ = h
        b.close()
