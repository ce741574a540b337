"""Round-trip verifier: the reference has no
decoder (its output was checked with libjpeg only).  mij_decoder entropy-
decodes the JFIF streams of encoder.c:549-644's shape on the GPU back into
the encoder's coefficient planes (zigzag order, DC as the coded difference),
so decode(jpg) must equal rgb_to_dct(frame) bit for bit:

* on the committed reference fixtures: the reference's own coefficient
  dumps (tests/golden/sample_64x64.coefs.npz, manifest coef_sha256);
* at full size (config 3, 3840x2160) as a size-independent property:
  decode(GPU encode(x)) == the GPU encoder's kept coefficient planes.
"""
import hashlib

import numpy as np
import pytest

import mijpeg
import oracle as O
import recipes
from test_oracle import case_input


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_decoder_validates_before_device_use():
    lib = mijpeg.load()
    assert not lib.mij_decoder_create(0, 24, 16, 1)
    assert lib.mij_last_error() == 1


@pytest.mark.gpu
def test_decode_reference_golden_64x64():
    jpg = open(f"{recipes.GOLDEN}/sample_64x64.jpg", "rb").read()
    z = np.load(f"{recipes.GOLDEN}/sample_64x64.coefs.npz")
    d = mijpeg.Decoder(64, 64, 1)
    try:
        d.decode([jpg])
        w, h, dqt = d.info(0)
        assert (w, h) == (64, 64)
        Y, Cb, Cr = d.coefs(0)
        assert (Y == z["Y"]).all() and (Cb == z["Cb"]).all() and (Cr == z["Cr"]).all()
    finally:
        d.close()


@pytest.mark.gpu
def test_decode_manifest_cases(manifest):
    """Every small golden case: decode(oracle jpg whose sha the reference
    pinned) has the reference's coefficient sha256 (the oracle's planes for
    cases whose manifest entry holds only the jpg sha)."""
    cases = [(k, e) for k, e in sorted(manifest.items())
             if e["frame"][0] * e["frame"][1] <= 1920 * 1280 and e["quality"] == 50]
    streams, want = [], []
    for name, ent in cases:
        bgr = case_input(name, ent)
        region = tuple(ent["region"])
        Y, Cb, Cr, _, jpg = O.cref_stages(bgr, 50, region)
        assert sha(jpg) == ent["jpg_sha256"], name
        streams.append(jpg)
        # the reference's coefficient dump where the manifest holds one
        want.append(ent.get("coef_sha256", [sha(Y), sha(Cb), sha(Cr)]))
    mw = max(e["region"][2] for _, e in cases)
    mh = max(e["region"][3] for _, e in cases)
    d = mijpeg.Decoder(mw, mh, len(streams))
    try:
        d.decode(streams)
        for i, (name, _) in enumerate(cases):
            Y, Cb, Cr = d.coefs(i)
            assert [sha(Y), sha(Cb), sha(Cr)] == want[i], name
    finally:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("quality", [50, 75, 90, 100, 10])
def test_decode_quality_sweep_and_long_codes(quality):
    """Q sweep (original.c:504-509) on natural and uniform-noise content (the
    noise needs AC codes longer than the 9-bit lookahead)."""
    frames = [recipes.noise(), recipes.gradients(), recipes.checkerboards(64, 128)]
    streams, want = [], []
    for f in frames:
        Y, Cb, Cr, _, jpg = O.cref_stages(f, quality)
        streams.append(jpg)
        want.append((Y, Cb, Cr))
    d = mijpeg.Decoder(256, 128, len(frames))
    try:
        d.decode(streams)
        lq, cq = O.quality_tables(quality)
        for i in range(len(frames)):
            got = d.coefs(i)
            for g, w in zip(got, want[i]):
                assert (g == w).all()
        _, _, dqt = d.info(0)
        assert dqt.size == 128
    finally:
        d.close()


@pytest.mark.gpu
def test_repeated_encodes_same_bytes_small_batch():
    """The same two-frame batch (config-3 frame + uniform noise, the
    small-batch paths: seam fixes inside k_emit_scan, DC tables inside the
    segment-DC launch) encoded 12 times: identical JFIF bytes every time, and
    each decodes to the encoder's own coefficients.  (Round 6: a missing
    barrier between the seam fixes and the chunk-count reads made the noise
    frame's bytes differ in about a third of the repetitions.)"""
    frames = np.stack([recipes.config3_frame(0), recipes.config3_uniform(1)])
    b = mijpeg.Batch(3840, 2160, 2, 50, keep_coefs=True)
    d = mijpeg.Decoder(3840, 2160, 2)
    try:
        b.upload(frames)
        first = None
        for _ in range(12):
            b.encode(2)
            streams = [b.output(i) for i in range(2)]
            shas = [hashlib.sha256(x).hexdigest() for x in streams]
            if first is None:
                first = shas
                d.decode(streams)
                for i in range(2):
                    for g, w in zip(d.coefs(i), b.coefs(i, diffed=True)):
                        assert (g == w).all()
            assert shas == first
    finally:
        b.close()
        d.close()


@pytest.mark.gpu
def test_round_trip_config3_full_size():
    """decode(GPU encode) == the GPU encoder's own coefficients, 3840x2160."""
    frames = np.stack([recipes.config3_frame(0), recipes.config3_uniform(1)])
    b = mijpeg.Batch(3840, 2160, 2, 50, keep_coefs=True)
    d = mijpeg.Decoder(3840, 2160, 2)
    try:
        b.upload(frames)
        b.encode(2)
        streams = [b.output(i) for i in range(2)]
        d.decode(streams)
        for i in range(2):
            for g, w in zip(d.coefs(i), b.coefs(i, diffed=True)):
                assert (g == w).all()
    finally:
        b.close()
        d.close()


@pytest.mark.gpu
def test_corrupt_streams_rejected():
    jpg = bytearray(open(f"{recipes.GOLDEN}/sample_64x64.jpg", "rb").read())
    d = mijpeg.Decoder(64, 64, 1)
    try:
        with pytest.raises(mijpeg.MijError):
            d.decode([bytes(jpg[:200])])           # cut inside the headers
        bad = bytes(jpg[:330]) + bytes(jpg[-2:])   # first scan cut short
        with pytest.raises(mijpeg.MijError):
            d.decode([bad])
        prog = bytearray(jpg)
        prog[293 + 1] = 0xC2                       # SOF2: progressive
        with pytest.raises(mijpeg.MijError):
            d.decode([bytes(prog)])
        d.decode([bytes(jpg)])                     # and still usable afterwards
    finally:
        d.close()


@pytest.mark.gpu
def test_round_trip_region_batch_and_config4():
    """Streams of different sizes in one decode: the JFIFs of a region batch
    (per-region SOF0 sizes) and one 7680x4320 config-4 frame."""
    frame = np.ascontiguousarray(recipes.config3_frame(3, 1080, 1920))
    regions = [(0, 0, 16, 16), (32, 48, 320, 240), (1904 - 512, 1064 - 256, 512, 256),
               (7, 5, 1008, 64), (600, 400, 48, 1024 - 400 + 16)]
    regions = [r for r in regions if r[0] + r[2] <= 1920 and r[1] + r[3] <= 1080]
    cw, ch = max(r[2] for r in regions), max(r[3] for r in regions)
    b = mijpeg.Batch(cw, ch, len(regions), 50, keep_coefs=True)
    big = np.ascontiguousarray(recipes.config4_frame(0))
    b4 = mijpeg.Batch(7680, 4320, 1, 50, keep_coefs=True)
    d = mijpeg.Decoder(7680, 4320, len(regions) + 1)
    try:
        b.upload_regions(frame, regions)
        b.encode(len(regions))
        b4.upload(big[None])
        b4.encode(1)
        streams = [b.output(i) for i in range(len(regions))] + [b4.output(0)]
        d.decode(streams)
        for i, r in enumerate(regions):
            assert d.info(i)[:2] == (r[2], r[3])
            for g, w in zip(d.coefs(i), b.coefs(i, diffed=True)):
                assert (g == w).all(), r
        for g, w in zip(d.coefs(len(regions)), b4.coefs(0, diffed=True)):
            assert (g == w).all()
    finally:
        b.close()
        b4.close()
        d.close()


@pytest.mark.gpu
def test_decode_badly_synchronising_stream():
    """Q=100 uniform noise: blocks of ~1000 bits, longer than a chunk, so
    chunks rarely self-synchronise -- many passes, still bit-exact."""
    f = np.random.default_rng(5).integers(0, 256, (256, 512, 3), dtype=np.uint8)
    Y, Cb, Cr, _, jpg = O.cref_stages(f, 100)
    d = mijpeg.Decoder(512, 256, 1)
    try:
        d.decode([jpg])
        for g, w in zip(d.coefs(0), (Y, Cb, Cr)):
            assert (g == w).all()
    finally:
        d.close()
