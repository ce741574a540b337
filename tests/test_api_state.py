"""Batch state across calls (C ABI, include/mijpeg.h): region sizes that
survive partial uploads, scan buffers left dirty by the band and assembly
paths, and the assembler's refusal of pipeline entry points.  Each case ends
in an encode whose bytes must equal the oracle's (oracle/cpu_ref.c, the
restatement of /root/reference/main/encoder.c)."""
import numpy as np
import pytest

import mijpeg
import oracle as O
import recipes

pytestmark = pytest.mark.gpu


def test_partial_upload_keeps_other_region_sizes():
    """set_frame_dims, then upload(first=1): slot 1 is a canvas frame again,
    slots 0 and 2 keep their region sizes (no silent full-canvas JPEGs)."""
    W, H = 256, 128
    frames = np.stack([recipes.config3_frame(i, H, W) for i in range(3)])
    b = mijpeg.Batch(W, H, 3)
    b.upload(frames)
    dims = [(128, 64), (64, 32), (48, 96)]
    b.set_frame_dims(dims)
    new1 = recipes.noise(H, W, 11)
    b.upload(new1, first=1)
    assert b.fdims == [(128, 64), (W, H), (48, 96)]
    b.encode(3)
    assert b.output(0) == O.cref_encode(frames[0], region=(0, 0, 128, 64))
    assert b.output(1) == O.cref_encode(new1)
    assert b.output(2) == O.cref_encode(frames[2], region=(0, 0, 48, 96))
    # every slot canvas-sized again: a plain batch
    b.upload(frames[[0, 2]][:1], first=0)
    b.upload(frames[2], first=2)
    assert b.fdims is None
    b.encode(3)
    for i, f in enumerate([frames[0], new1, frames[2]]):
        assert b.output(i) == O.cref_encode(f)
    b.close()


def test_band_words_of_fewer_frames_than_packed_then_encode():
    """mij_band_pack over 2 frames, mij_band_words_all over only the first:
    frame 1's band words stay in its scan buffers, so the next encode must
    clear them before the band packing ORs its edge words in."""
    W, H, n = 256, 64, 2
    frames = np.stack([recipes.config3_frame(i, H, W) for i in range(n)])
    b = mijpeg.Batch(W, H, n)
    b.upload(frames)
    b.band_analyze(n)
    hist = b.band_histograms(n, np.zeros((n, 3), np.int16))
    b.band_tables(n, hist)
    nw = b.band_pack(n, np.full((n, 3), 5, np.uint64))  # a non-zero in-word start offset
    assert int(nw[1].sum()) > 0
    b.band_words_all(1, cap_words=int(nw[0].sum()) + 64)
    b.encode(n)
    for i in range(n):
        assert b.output(i) == O.cref_encode(frames[i]), f"frame {i}"
    b.close()


def test_assemble_without_end_then_encode():
    """mij_assemble_begin + words OR-ed into a normal batch's scan buffers,
    mij_assemble_end skipped: the next encode starts from zeroed buffers."""
    W, H = 256, 64
    fr = recipes.config3_frame(3, H, W)
    b = mijpeg.Batch(W, H, 1)
    b.upload(fr)
    b.encode(1)
    want = O.cref_encode(fr)
    assert b.output(0) == want
    hist = np.zeros((1, 4, 257), np.uint32)
    hist[0, :, 0] = 1
    hist[0, 1, 0xF0] = 1
    hist[0, 3, 0xF0] = 1
    b.assemble_begin(1, hist)
    b.assemble_words(0, 0, 3, np.full(40, 0xA5A5A5A5, np.uint32))
    b.encode(1)
    assert b.output(0) == want
    b.close()


def test_assembler_refuses_pipeline_entry_points():
    """An assembler has no input, coefficient or token buffers: every entry
    point that would run the encoder fails with MIJ_EINVAL, not a fault."""
    a = mijpeg.Batch(256, 64, 2, assembler=True)
    fr = recipes.config3_frame(0, 64, 256)
    calls = [lambda: a.encode(1), lambda: a.coefs(0), lambda: a.upload(fr),
             lambda: a.upload_regions(fr, [(0, 0, 64, 32)]), lambda: a.set_rgb(True),
             lambda: a.set_split(True), lambda: a.set_overlap(2),
             lambda: mijpeg._check(a.lib.mij_batch_keep_coefs(a.h_, 1), "keep_coefs")]
    for c in calls:
        with pytest.raises(mijpeg.MijError, match="an assembler only assembles"):
            c()
    a.close()


def test_repeated_encodes_growing_and_shrinking_frame_counts():
    """The encode path leaves the counts it read (and k_pack_flat's look-back
    state) zeroed, and the next encode skips those fills only for the frames
    known clean: 1 frame, then 3 (two never zeroed), then 3 again, then 2,
    a band call in between (which writes the counts) and 3 again -- every
    output the oracle's bytes."""
    W, H = 320, 160
    frames = np.stack([recipes.config3_frame(i + 20, H, W) for i in range(3)])
    want = [O.cref_encode(f) for f in frames]
    b = mijpeg.Batch(W, H, 3)
    b.upload(frames)
    for n in (1, 3, 3, 2):
        b.encode(n)
        assert [b.output(i) for i in range(n)] == want[:n], n
    b.band_analyze(2)
    b.encode(3)
    assert [b.output(i) for i in range(3)] == want
    # the skip path after a band call: encode(3) leaves 3 frames' counts
    # zeroed, band_analyze writes counts again, encode(2 <= 3) must refill
    b.band_analyze(2)
    b.encode(2)
    assert [b.output(i) for i in range(2)] == want[:2]
    b.close()
