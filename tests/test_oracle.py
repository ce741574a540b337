"""CPU tests: the oracle (oracle/cpu_ref.c, a restatement of the reference's
main/encoder.c) against the golden vectors generated from the reference
itself (tests/golden/, oracle/gen_golden.py), plus direct comparisons with
the compiled reference where oracle/_ref exists."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
import ppm
import recipes

GOLD = recipes.GOLDEN


def sha(b) -> str:
    if isinstance(b, np.ndarray):
        b = b.tobytes()
    return hashlib.sha256(b).hexdigest()


def case_input(name, ent):
    src = ent["input"]
    if src in ("sample_64x64", "sample_640x640", "sample_640x640_diffs"):
        return ppm.rgb_to_bgr(recipes.sample(src))
    if src == "standin_1920x1280":
        return ppm.rgb_to_bgr(recipes.standin_1920x1280_rgb())
    if src == "sample_640x640[:240,:320]":
        return ppm.rgb_to_bgr(recipes.sample("sample_640x640")[:240, :320])
    if src.startswith("recipes."):
        fn = src[len("recipes."):].split("(")[0]
        arg = src.split("(")[1].rstrip(")")
        f = getattr(recipes, fn)
        return np.ascontiguousarray(f(int(arg)) if arg else f())
    raise KeyError(src)


SMALL = ["sample_64x64", "sample_640x640", "sample_640x640_diffs", "region_0", "region_1",
         "region_2", "region_3", "region_4", "gray_levels", "flat_colours", "gradients",
         "checkerboards", "noise", "near_gray"]


@pytest.mark.parametrize("name", SMALL)
def test_oracle_matches_reference_golden(manifest, name):
    ent = manifest[name]
    bgr = case_input(name, ent)
    region = tuple(ent["region"])
    Y, Cb, Cr, _, jpg = O.cref_stages(bgr, ent["quality"], region)
    assert len(jpg) == ent["jpg_len"]
    assert sha(jpg) == ent["jpg_sha256"]
    assert [sha(Y), sha(Cb), sha(Cr)] == ent["coef_sha256"]


def test_oracle_standin_1920x1280(manifest):
    ent = manifest["standin_1920x1280"]
    jpg = O.cref_encode(case_input("standin_1920x1280", ent))
    assert sha(jpg) == ent["jpg_sha256"] and len(jpg) == 237044


@pytest.mark.parametrize("name", ["sample_640x640_q10", "sample_640x640_q75",
                                  "sample_640x640_q90", "sample_640x640_q100",
                                  "sample_64x64_q75", "sample_64x64_q90"])
def test_oracle_quality_sweep(manifest, name):
    ent = manifest[name]
    bgr = ppm.rgb_to_bgr(recipes.sample(ent["input"]))
    jpg = O.cref_encode(bgr, ent["quality"])
    assert sha(jpg) == ent["jpg_sha256"]


def test_sample_64x64_full_intermediates():
    bgr = ppm.rgb_to_bgr(recipes.sample("sample_64x64"))
    Y, Cb, Cr, tabs, jpg = O.cref_stages(bgr)
    gold = np.load(os.path.join(GOLD, "sample_64x64.coefs.npz"))
    assert (Y == gold["Y"]).all() and (Cb == gold["Cb"]).all() and (Cr == gold["Cr"]).all()
    with open(os.path.join(GOLD, "sample_64x64.tables.json")) as f:
        gt = json.load(f)
    for t, g in zip(tabs, gt):
        for field, _ in O.Huff._fields_:
            assert list(getattr(t, field)) == g[field], field
    with open(os.path.join(GOLD, "sample_64x64.jpg"), "rb") as f:
        assert f.read() == jpg


def test_marker_layout_64x64():
    """SOI 0, APP0 2, DQT 20/89, DHT 158.., SOF0 293, SOS .., EOI."""
    with open(os.path.join(GOLD, "sample_64x64.jpg"), "rb") as f:
        b = f.read()
    pos = [i for i in range(len(b) - 1) if b[i] == 0xFF and b[i + 1] in
           (0xD8, 0xE0, 0xDB, 0xC4, 0xC0, 0xDA, 0xD9)]
    assert pos[:9] == [0, 2, 20, 89, 158, 187, 229, 257, 293]
    assert b[-2:] == b"\xff\xd9" and len(b) == 566


def test_cos_table_matches_reference():
    with open(os.path.join(GOLD, "cos_table.json")) as f:
        gold = np.array(json.load(f), np.int64)
    assert (O.cos_bits_cref() == gold).all()


def test_colour_exceptions_exhaustive():
    """Every exception triple in the golden set truncates one below the exact
    integer in the oracle, and the counts match SURVEY §0 (3464/942/2706)."""
    ex = np.load(os.path.join(GOLD, "colour_exceptions.npz"))
    assert [len(ex[k]) for k in ("Y", "Cb", "Cr")] == [3464, 942, 2706]
    lib = O.cref()
    out = np.zeros(3, np.uint8)
    import ctypes
    for ch, key in enumerate(("Y", "Cb", "Cr")):
        for r, g, b in ex[key][::37].astype(np.int64):
            lib.cref_pixel_ycc(ctypes.c_uint8(b), ctypes.c_uint8(g), ctypes.c_uint8(r),
                               out.ctypes.data)
            exact = [(299 * r + 587 * g + 114 * b) // 1000,
                     (128_000_000 - 168736 * r - 331264 * g + 500000 * b) // 1_000_000,
                     (128_000_000 + 500000 * r - 418688 * g - 81312 * b) // 1_000_000][ch]
            assert out[ch] == exact - 1


def test_ppm_parser_rules():
    good = ppm.ppm_bytes(np.zeros((16, 32, 3), np.uint8))
    assert ppm.parse_ppm(good).shape == (16, 32, 3)
    with_comment = b"P6\n# made by a test\n32 16\n255\n" + bytes(16 * 32 * 3)
    assert ppm.parse_ppm(with_comment).shape == (16, 32, 3)
    with pytest.raises(ValueError):
        ppm.parse_ppm(b"P6\n30 16\n255\n" + bytes(30 * 16 * 3))
    with pytest.raises(ValueError):
        ppm.parse_ppm(b"P6\n32 16\n65535\n" + bytes(16 * 32 * 6))


def test_oracle_rejects_bad_dims():
    with pytest.raises(ValueError):
        O.cref_encode(np.zeros((16, 24, 3), np.uint8))


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built here")
@pytest.mark.parametrize("seed", range(12))
def test_oracle_vs_compiled_reference_random(seed):
    rng = np.random.default_rng(100 + seed)
    W, H = 16 * int(rng.integers(1, 10)), 16 * int(rng.integers(1, 10))
    kind = seed % 4
    if kind == 0:
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    elif kind == 1:
        img = np.repeat(rng.integers(0, 256, (H, W, 1), dtype=np.uint8), 3, axis=2)
    elif kind == 2:
        img = np.full((H, W, 3), rng.integers(0, 256, 3), np.uint8)
    else:
        img = recipes.near_gray(H, W, seed)
    frame = rng.integers(0, 256, (H + 32, W + 48, 3), dtype=np.uint8)
    ox, oy = int(rng.integers(0, 49)), int(rng.integers(0, 33))
    frame[oy:oy + H, ox:ox + W] = img
    a = O.ref_stages(frame, (ox, oy, W, H))
    b = O.cref_stages(frame, 50, (ox, oy, W, H))
    assert a[4] == b[4]
    for x, y in zip(a[:3], b[:3]):
        assert (x == y).all()
    for x, y in zip(a[3], b[3]):
        assert bytes(x) == bytes(y)
