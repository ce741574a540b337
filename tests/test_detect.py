"""Change detector: reference main/brain.c,
caller main.c:136-163 -- subsample the frame 4x4, compare it with the stored
subsampled frame, join the differing runs into at most 100 areas, store.

CPU tests pin the C restatement (oracle/cpu_ref.c) to the committed golden
vectors (tests/golden/detect.json, generated from the unmodified reference
by oracle/gen_detect_golden.py) and, where it was built, to the reference
itself on fresh scenes.  GPU tests compare the HIP detector (k_detect + host
joining, csrc/mij_detect.hip) and the drop-in brain.h entry points with the
golden vectors and the oracle; bit-exact (integer work)."""
import hashlib
import json
import os

import numpy as np
import pytest

import mijpeg
import oracle as O
import ppm
import recipes

with open(os.path.join(recipes.GOLDEN, "detect.json")) as f:
    GOLD = json.load(f)["cases"]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def scene(c):
    if "recipe" in c:
        seed, w, h, kind = c["recipe"]
        return recipes.detect_scene(seed, w, h, kind)
    a = ppm.rgb_to_bgr(recipes.sample("sample_640x640"))
    b = ppm.rgb_to_bgr(recipes.sample("sample_640x640_diffs"))
    return (a, b) if c["images"] == "sample_640x640->diffs" else (b, a)


def case_id(c):
    return "-".join(map(str, c["recipe"])) if "recipe" in c else c["images"]


def numpy_mask(sub, saved):
    """brain.c:184-195 evaluated in FP64 as the reference writes it."""
    a = sub.astype(np.float64)
    b = saved.astype(np.float64)
    cR = (a[..., 0] + b[..., 0]) / 2
    d = a - b
    r = np.trunc(d[..., 0] ** 2 * (2 + cR / 256))
    g = d[..., 1] ** 2 * 4
    bb = np.trunc(d[..., 2] ** 2 * (2 + (255 - cR) / 256))
    return (r + g + bb) > 600


# ---------------------------------------------------------------- CPU -------

@pytest.mark.parametrize("c", GOLD, ids=case_id)
def test_oracle_matches_reference_golden(c):
    stored, cur = scene(c)
    if c["w"] * c["h"] > 1920 * 1080:
        pytest.skip("large case: checked on the GPU run")
    s0, s1 = O.cref_subsample(stored), O.cref_subsample(cur)
    assert sha(s0) == c["sub_stored_sha256"] and sha(s1) == c["sub_current_sha256"]
    n, areas = O.cref_compare(s1, s0, c["w"], c["h"])
    assert (n, [list(a) for a in areas]) == (c["count"], c["areas"])


def test_golden_covers_the_reference_paths():
    counts = [c["count"] for c in GOLD]
    assert 0 in counts and 100 in counts and any(1 < n < 100 for n in counts)
    # the 100-area overflow that returns un-enlarged areas (brain.c:167)
    assert any(c["count"] == 100 and any(a[2] < a[0] + 16 for a in c["areas"]) for c in GOLD)


@pytest.mark.skipif(not O.ref_brain_available(), reason="reference build absent (GPU box)")
def test_oracle_matches_reference_on_fresh_scenes():
    for seed in range(40):
        kind = ["objects", "many", "edge", "grid", "noise"][seed % 5]
        w, h = [(320, 240), (160, 128), (480, 272)][seed % 3]
        stored, cur = recipes.detect_scene(1000 + seed, w, h, kind)
        s0, s1 = O.ref_subsample(stored), O.ref_subsample(cur)
        assert (O.cref_subsample(stored) == s0).all()
        assert O.cref_compare(s1, s0, w, h) == O.ref_compare(s1, s0, w, h), (seed, kind)


def test_integer_distance_equals_fp64_form():
    """The integer form used by the kernel and the oracle equals the
    reference's FP64 expression over all channel pairs that matter."""
    a = np.arange(256)
    A, B = np.meshgrid(a, a, indexing="ij")
    d2 = (A - B) ** 2
    s = A + B
    r_int = (d2 * (1024 + s)) >> 9
    b_int = (d2 * (1534 - s)) >> 9
    cR = s / 2
    assert (r_int == np.trunc(d2 * (2 + cR / 256))).all()
    assert (b_int == np.trunc(d2 * (2 + (255 - cR) / 256))).all()


# ---------------------------------------------------------------- GPU -------

@pytest.mark.gpu
@pytest.mark.parametrize("c", GOLD, ids=case_id)
def test_detector_step_matches_golden(c):
    stored, cur = scene(c)
    d = mijpeg.Detector(c["w"], c["h"])
    try:
        d.subsample(d.upload(stored))
        d.store()
        n, areas = d.step(d.upload(cur))
        assert sha(d.plane(1)) == c["sub_stored_sha256"]
        assert sha(d.plane(0)) == c["sub_current_sha256"]
        assert (n, [list(a) for a in areas]) == (c["count"], c["areas"])
        assert (d.mask() == numpy_mask(d.plane(0), d.plane(1))).all()
    finally:
        d.close()


@pytest.mark.gpu
def test_detector_sequence_matches_oracle():
    """main.c:136-163 loop over a moving-object sequence: step, store."""
    W, H = 640, 480
    frames = [recipes.detect_scene(300 + i, W, H, "objects")[1] for i in range(6)]
    d = mijpeg.Detector(W, H)
    saved = np.zeros((H // 4, W // 4, 3), np.uint8)  # main.c:33 static
    try:
        for f in frames:
            sub = O.cref_subsample(f)
            want = O.cref_compare(sub, saved, W, H)
            assert d.step(d.upload(f)) == want
            d.store()
            saved = sub
    finally:
        d.close()


@pytest.mark.gpu
def test_detector_reads_pitched_device_frames():
    W, H = 320, 240
    stored, cur = recipes.detect_scene(7, W, H, "objects")
    pitch = 3 * W + 64
    d = mijpeg.Detector(W, H)
    try:
        padded = np.zeros((H, pitch), np.uint8)
        padded[:, :3 * W] = stored.reshape(H, 3 * W)
        padded[:, 3 * W:] = 255  # padding must not be read
        d.subsample(d.upload(padded, pitch), pitch)
        d.store()
        padded[:, :3 * W] = cur.reshape(H, 3 * W)
        got = d.step(d.upload(padded, pitch), pitch)
        s0, s1 = O.cref_subsample(stored), O.cref_subsample(cur)
        assert got == O.cref_compare(s1, s0, W, H)
        # compare() on planes already on the device (brain.c:104 on sub/saved)
        d.set_plane(0, s1)
        d.set_plane(1, s0)
        assert d.compare() == got
    finally:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("c", [g for g in GOLD if g["w"] * g["h"] <= 640 * 640], ids=case_id)
def test_drop_in_entry_points(c):
    stored, cur = scene(c)
    s0 = mijpeg.drop_in_subsample(stored)
    s1 = mijpeg.drop_in_subsample(cur)
    assert sha(s0) == c["sub_stored_sha256"] and sha(s1) == c["sub_current_sha256"]
    n, areas = mijpeg.drop_in_compare(s1, s0, c["w"], c["h"])
    assert (n, [list(a) for a in areas]) == (c["count"], c["areas"])


@pytest.mark.gpu
def test_detect_then_encode_regions():
    """The reference's loop body end to end: detected areas of a frame are
    encoded each to its own JPEG (main.c:142-155), bytes = the oracle's."""
    W, H = 640, 480
    stored, cur = recipes.detect_scene(11, W, H, "objects")
    d = mijpeg.Detector(W, H)
    try:
        d.subsample(d.upload(stored))
        d.store()
        ptr = d.upload(cur)
        n, areas = d.step(ptr)
        assert n > 0
        cw = max(a[2] for a in areas)
        ch = max(a[3] for a in areas)
        b = mijpeg.Batch(cw, ch, n)
        try:
            b.gather_regions(ptr, 3 * W, W, H, areas)
            b.encode(n)
            for i, a in enumerate(areas):
                assert b.output(i) == O.cref_encode(cur, 50, a), a
        finally:
            b.close()
    finally:
        d.close()


@pytest.mark.gpu
def test_enlarge_adjust_drop_in():
    for a in [(0, 0, 0, 0), (5, 7, 20, 9), (70, 50, 79, 59), (0, 0, 79, 59), (78, 1, 79, 3)]:
        want = O.cref_area_adjust(a, 320, 240)
        assert mijpeg.drop_in_enlarge_adjust(a, 320, 240) == want


@pytest.mark.gpu
def test_detector_config4_frame():
    """7680x4320 (config 4 size) against the oracle: planes, mask, areas."""
    W, H = 7680, 4320
    stored, cur = recipes.detect_scene(400, W, H, "objects")
    d = mijpeg.Detector(W, H)
    try:
        d.subsample(d.upload(stored))
        d.store()
        got = d.step(d.upload(cur))
        s0, s1 = O.cref_subsample(stored), O.cref_subsample(cur)
        assert (d.plane(0) == s1).all() and (d.plane(1) == s0).all()
        assert (d.mask() == numpy_mask(s1, s0)).all()
        assert got == O.cref_compare(s1, s0, W, H)
    finally:
        d.close()
