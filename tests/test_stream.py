"""PPM ingest (mij_ppm_header / mij_ppm_read: the acceptance rules of the
reference's reader, utils/original.c:294-365) and the streaming encoder
(mij_stream_*: PPM files or RGB frames -> .jpg through two device batches in
ping-pong).  The reader tests run on the CPU (host code of libmijpeg.so, no
device call); the stream tests are GPU tests and compare every output with
the golden vectors or the oracle."""
import hashlib
import os
import tempfile

import numpy as np
import pytest

import mijpeg
import oracle as O
import ppm
import recipes


def sha(b) -> str:
    return hashlib.sha256(b).hexdigest()


def write(d, name, data: bytes) -> str:
    path = os.path.join(d, name)
    with open(path, "wb") as f:
        f.write(data)
    return path


def rejects(path, code):
    with pytest.raises(mijpeg.MijError) as e:
        mijpeg.ppm_header(path)
    assert f"({code})" in str(e.value)


# ---------------------------------------------------------------------------
# reader rules (CPU)
# ---------------------------------------------------------------------------

def test_ppm_reader_accepts_reference_layouts():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (32, 48, 3), dtype=np.uint8)
    img[0, 0, 0] = 0x20
    with tempfile.TemporaryDirectory() as d:
        plain = write(d, "a.ppm", ppm.ppm_bytes(img))
        # a whitespace first pixel byte: "%d\n" (original.c:330) swallows it,
        # so the reference's length check rejects the file
        rejects(plain, 6)
        img[0, 0, 0] = 7
        plain = write(d, "a.ppm", ppm.ppm_bytes(img))
        w, h, off = mijpeg.ppm_header(plain)
        assert (w, h, off) == (48, 32, len(b"P6\n48 32\n255\n"))
        assert (mijpeg.ppm_read(plain) == img).all()
        assert (mijpeg.ppm_read(plain, to_bgr=True) == img[..., ::-1]).all()
        # comment lines between the magic and the size (original.c:303-316)
        com = write(d, "c.ppm", b"P6\n# one\n#two\n48 32\n255\n" + img.tobytes())
        assert (mijpeg.ppm_read(com) == img).all()


def test_ppm_reader_rejections():
    px = bytes(16 * 32 * 3)
    cases = [
        (b"P3\n32 16\n255\n" + px, 6),               # magic (:296-300)
        (b"P6 32 16\n255\n" + px, 6),                # no newline after the magic (:302-303)
        (b"P6\n30 16\n255\n" + bytes(30 * 16 * 3), 6),  # not a multiple of 16 (:324-328)
        (b"P6\n32 16\n65535\n" + px + px, 6),         # depth (:333-337)
        (b"P6\n32 16\n255\n" + px[:-1], 6),           # short pixel data (:339-344)
        (b"P6\n32 16\n255\n" + px + b"\0", 6),        # trailing bytes
        (b"P6\nsize\n255\n" + px, 6),                 # unparsable size
        (b"P6\n# only a comment", 6),                 # EOF inside the header
    ]
    with tempfile.TemporaryDirectory() as d:
        for i, (data, code) in enumerate(cases):
            rejects(write(d, f"bad{i}.ppm", data), code)
        rejects(os.path.join(d, "missing.ppm"), 7)


def test_ppm_reader_matches_golden_sample():
    with tempfile.TemporaryDirectory() as d:
        rgb = recipes.sample("sample_640x640")
        path = write(d, "s.ppm", ppm.ppm_bytes(rgb))
        assert (mijpeg.ppm_read(path) == rgb).all()
    gold = os.path.join(recipes.GOLDEN, "sample_64x64.ppm")
    assert (mijpeg.ppm_read(gold) == recipes.sample("sample_64x64")).all()


def test_stream_create_validates_before_device_use():
    lib = mijpeg.load()
    assert not lib.mij_stream_create(0, 30, 16, 1, 50, 1)
    assert lib.mij_last_error() == 1
    assert not lib.mij_stream_create(0, 32, 16, 0, 50, 1)
    assert not lib.mij_stream_create(0, 32, 16, 1, 101, 1)


# ---------------------------------------------------------------------------
# streaming encoder (GPU)
# ---------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
def test_batch_rgb_input_same_bytes_as_bgr(split):
    """K1 reading R, G, B (PPM order) gives the bytes of the B, G, R path."""
    rgb = np.stack([recipes.sample("sample_640x640"), recipes.sample("sample_640x640_diffs")])
    b = mijpeg.Batch(640, 640, 2)
    b.set_split(split)
    b.set_rgb(True)
    b.upload(rgb)
    b.encode(2)
    for i in range(2):
        assert b.output(i) == O.cref_encode(ppm.rgb_to_bgr(rgb[i]))
    b.close()


@pytest.mark.gpu
def test_stream_files_match_golden(manifest):
    """PPM files -> .jpg files; a ragged last chunk (5 files, chunk 2)."""
    names = ["sample_640x640", "sample_640x640_diffs", "sample_640x640",
             "sample_640x640_diffs", "sample_640x640"]
    with tempfile.TemporaryDirectory() as d:
        ins, outs = [], []
        for i, n in enumerate(names):
            ins.append(write(d, f"in{i}.ppm", ppm.ppm_bytes(recipes.sample(n))))
            outs.append(os.path.join(d, f"out{i}.jpg"))
        s = mijpeg.Stream(640, 640, chunk=2, threads=4)
        s.encode_files(ins, outs)
        for n, o in zip(names, outs):
            assert sha(open(o, "rb").read()) == manifest[n]["jpg_sha256"]
        st = s.stats()
        assert st["frames"] == 5 and st["bytes_in"] == 5 * 640 * 640 * 3
        assert st["bytes_out"] == sum(os.path.getsize(o) for o in outs)
        s.close()


@pytest.mark.gpu
def test_stream_frames_vs_oracle_and_errors():
    rng = np.random.default_rng(9)
    frames = [rng.integers(0, 256, (96, 160, 3), dtype=np.uint8),
              np.zeros((96, 160, 3), np.uint8),
              recipes.near_gray(96, 160, 4)[..., ::-1],
              recipes.config3_frame(2, 96, 160)[..., ::-1]]
    s = mijpeg.Stream(160, 96, chunk=3, quality=75)
    got = s.encode_frames(frames)
    for f, g in zip(frames, got):
        assert g == O.cref_encode(ppm.rgb_to_bgr(f), 75)
    # a file of another geometry stops the stream at its index
    with tempfile.TemporaryDirectory() as d:
        ok = write(d, "ok.ppm", ppm.ppm_bytes(frames[0]))
        bad = write(d, "bad.ppm", ppm.ppm_bytes(np.zeros((32, 32, 3), np.uint8)))
        with pytest.raises(mijpeg.MijError, match="file 1"):
            s.encode_files([ok, bad, ok], [os.path.join(d, f"o{i}.jpg") for i in range(3)])
    s.close()
