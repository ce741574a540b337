"""GPU parity tests: the HIP path through the C ABI (libmijpeg.so) against
(a) the golden vectors generated from the reference itself and (b) the CPU
oracle on seeded inputs.  Integer/byte work: bit-exact everywhere."""
import hashlib
import io
import os
import subprocess
import tempfile

import numpy as np
import pytest

import mijpeg
import oracle as O
import ppm
import recipes
from test_oracle import SMALL, case_input

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sha(b) -> str:
    if isinstance(b, np.ndarray):
        b = b.tobytes()
    return hashlib.sha256(b).hexdigest()


def first_diff(a: bytes, b: bytes) -> int:
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return i
    return n


# ---------------------------------------------------------------------------
# hardware/lowering checks the kernels rely on
# ---------------------------------------------------------------------------

def test_mfma_i8_operand_layout():
    """v_mfma_i32_16x16x64_i8: lane l of A holds row l&15, k-group l>>4;
    B likewise for columns; D lane l reg r = row 4(l>>4)+r, col l&15."""
    rng = np.random.default_rng(5)
    A = rng.integers(-128, 128, (64, 16), dtype=np.int8)
    B = rng.integers(-128, 128, (64, 16), dtype=np.int8)
    D = mijpeg.probe_mfma(A, B)
    M = np.zeros((16, 64), np.int64)
    N = np.zeros((64, 16), np.int64)
    for lane in range(64):
        kg = lane >> 4
        M[lane & 15, 16 * kg:16 * kg + 16] = A[lane]
        N[16 * kg:16 * kg + 16, lane & 15] = B[lane]
    ref = M @ N
    for lane in range(64):
        for r in range(4):
            assert D[lane, r] == ref[4 * (lane >> 4) + r, lane & 15]


def test_colour_exception_bitmaps_match_reference_set():
    lut = mijpeg.colour_lut()
    ex = np.load(os.path.join(recipes.GOLDEN, "colour_exceptions.npz"))
    want = np.zeros((3, 32768), bool)
    for ch, key in enumerate(("Y", "Cb", "Cr")):
        t = ex[key].astype(np.int64)
        r, g, b = t[:, 0], t[:, 1], t[:, 2]
        # integer points need equal parities, so each table is indexed by 15 bits
        assert (((r ^ g) & 1) == 0).all() and (ch == 0 or (((b ^ g) & 1) == 0).all())
        idx = [(r << 7) | (g >> 1), (g << 7) | (b >> 1), (g << 7) | (r >> 1)][ch]
        want[ch, idx] = True
    got = np.unpackbits(lut.view(np.uint8).reshape(3, -1), axis=1, bitorder="little").astype(bool)
    assert (got == want).all()


# ---------------------------------------------------------------------------
# golden cases (expected outputs produced by the reference build)
# ---------------------------------------------------------------------------

FULL_FRAME = ["sample_64x64", "sample_640x640", "sample_640x640_diffs", "gray_levels",
              "flat_colours", "gradients", "checkerboards", "noise", "near_gray"]


@pytest.mark.parametrize("name", FULL_FRAME)
def test_batch_matches_reference_golden(manifest, name):
    ent = manifest[name]
    bgr = case_input(name, ent)
    H, W = bgr.shape[:2]
    b = mijpeg.Batch(W, H, 1, ent["quality"], keep_coefs=True)
    b.upload(bgr)
    b.encode(1)
    jpg = b.output(0)
    if sha(jpg) != ent["jpg_sha256"]:
        ref = O.cref_encode(bgr)
        pytest.fail(f"{name}: {len(jpg)} vs {len(ref)} bytes, first diff at {first_diff(jpg, ref)}")
    Y, Cb, Cr = b.coefs(0, diffed=True)
    assert [sha(Y), sha(Cb), sha(Cr)] == ent["coef_sha256"]
    b.close()


def test_standin_1920x1280_bit_exact_gate(manifest):
    ent = manifest["standin_1920x1280"]
    bgr = case_input("standin_1920x1280", ent)
    b = mijpeg.Batch(1920, 1280, 1, keep_coefs=True)
    b.upload(bgr)
    b.encode(1)
    jpg = b.output(0)
    assert len(jpg) == ent["jpg_len"] == 237044
    assert sha(jpg) == ent["jpg_sha256"]
    Y, Cb, Cr = b.coefs(0)
    assert [sha(Y), sha(Cb), sha(Cr)] == ent["coef_sha256"]
    b.close()


@pytest.mark.parametrize("name", ["region_0", "region_1", "region_2", "region_3", "region_4"])
def test_drop_in_three_calls_on_regions(manifest, name):
    """main.c:144-152 call sequence on a 320-stride frame (define.h:3)."""
    ent = manifest[name]
    frame = case_input(name, ent)
    region = tuple(ent["region"])
    Y, Cb, Cr = mijpeg.rgb_to_dct(frame, region)
    assert [sha(Y), sha(Cb), sha(Cr)] == ent["coef_sha256"]
    tabs = mijpeg.init_huffman(Y, Cb, Cr, region)
    _, _, _, ref_tabs, _ = O.cref_stages(frame, 50, region)
    for t, r in zip(tabs, ref_tabs):
        assert bytes(t) == bytes(r)
    jpg = mijpeg.write_jpg(Y, Cb, Cr, region, tabs)
    assert sha(jpg) == ent["jpg_sha256"]
    assert mijpeg.encode(frame, 50, region) == jpg


def test_tables_struct_parity_640(manifest):
    bgr = case_input("sample_640x640", manifest["sample_640x640"])
    b = mijpeg.Batch(640, 640, 1)
    b.upload(bgr)
    b.encode(1)
    got = b.tables(0)
    _, _, _, ref, _ = O.cref_stages(bgr)
    for field, _ in mijpeg.Huff._fields_:
        for t in range(4):
            assert list(getattr(got[t], field)) == list(getattr(ref[t], field)), (t, field)
    b.close()


@pytest.mark.parametrize("q", [10, 75, 90, 100])
def test_quality_sweep_matches_original_c(manifest, q):
    ent = manifest[f"sample_640x640_q{q}"]
    bgr = ppm.rgb_to_bgr(recipes.sample("sample_640x640"))
    b = mijpeg.Batch(640, 640, 1, q)
    b.upload(bgr)
    b.encode(1)
    assert sha(b.output(0)) == ent["jpg_sha256"]
    b.close()


@pytest.mark.parametrize("split", [False, True])
def test_config5_frame_size_q75_q90_match_original_c(manifest, split):
    """Config 5 at frame size: config-3 frames at Q=75 and Q=90 (thousands
    of FP64 replays per frame) against the reference's own bytes
    (utils/original.c + set_quality, oracle/gen_golden.py), both pipelines."""
    for f, q in ((0, 75), (1, 90)):
        ent = manifest[f"config3_frame{f}_q{q}"]
        b = mijpeg.Batch(3840, 2160, 1, q)
        b.set_split(split)
        b.upload(recipes.config3_frame(f))
        b.encode(1)
        got = b.output(0)
        assert len(got) == ent["jpg_len"] and sha(got) == ent["jpg_sha256"], (f, q, split)
        assert b.replays() > 1000
        b.close()


def test_config3_batch_frames(manifest):
    """3840x2160 batch (config 3 shape): two natural frames + one uniform
    high-entropy frame, one launch sequence."""
    frames = np.stack([recipes.config3_frame(0), recipes.config3_frame(1),
                       recipes.config3_uniform(0)])
    b = mijpeg.Batch(3840, 2160, 3)
    b.upload(frames)
    b.encode(3)
    for i, name in enumerate(["config3_frame0", "config3_frame1", "config3_uniform0"]):
        assert sha(b.output(i)) == manifest[name]["jpg_sha256"], name
    b.close()


# ---------------------------------------------------------------------------
# seeded inputs against the oracle
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("seed", range(10))
def test_random_shapes_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    W = 16 * int(rng.integers(1, 40))   # includes widths that are not tile multiples
    H = 16 * int(rng.integers(1, 12))
    kind = seed % 5
    if kind == 0:
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    elif kind == 1:
        img = np.repeat(rng.integers(0, 256, (H, W, 1), dtype=np.uint8), 3, axis=2)
    elif kind == 2:
        img = recipes.near_gray(H, W, seed)
    elif kind == 3:
        big = np.tile(recipes.sample("sample_640x640"), (2, 2, 1))
        img = ppm.rgb_to_bgr(big[:H, :W])
    else:
        base = rng.integers(0, 256, (H // 16, W // 16, 3), dtype=np.uint8)
        img = np.kron(base, np.ones((16, 16, 1), np.uint8))
    q = [50, 75, 90, 25, 100][seed % 5]
    b = mijpeg.Batch(W, H, 1, q)
    b.upload(img)
    b.encode(1)
    got = b.output(0)
    ref = O.cref_encode(img, q)
    assert got == ref, f"{W}x{H} q{q}: first diff {first_diff(got, ref)}"
    b.close()


def test_short_last_pack_group_seams():
    """432x304: 513 chroma blocks, so each chroma scan's last pack group is one
    segment of a single block.  Mostly flat frames make that group a few bits
    long: it starts inside the word where the group before it ends and often
    ends there too (seam mode: the word is the previous group's store OR-ed
    with both groups' seams, and the pad byte comes from it)."""
    W, H, n = 432, 304, 8
    rng = np.random.default_rng(432)
    frames = np.empty((n, H, W, 3), np.uint8)
    for i in range(n):
        frames[i] = rng.integers(0, 256, 3, dtype=np.uint8)
        k = int(rng.integers(1, 40))  # a few busy 16x16 blocks in the first MCU row
        for x in rng.choice(W // 16, size=min(k, W // 16), replace=False):
            frames[i, :16, 16 * x:16 * x + 16] = rng.integers(0, 256, (16, 16, 3), dtype=np.uint8)
        frames[i, -16:, -16:] = rng.integers(0, 256, 3, dtype=np.uint8)  # a last block of its own colour
    b = mijpeg.Batch(W, H, n, 50)
    b.upload(frames)
    b.encode(n)
    for i in range(n):
        ref = O.cref_encode(frames[i], 50)
        got = b.output(i)
        assert got == ref, f"frame {i}: first diff {first_diff(got, ref)}"
    b.close()


def test_multi_frame_batch_independent_tables():
    rng = np.random.default_rng(11)
    frames = np.stack([rng.integers(0, 256, (64, 96, 3), dtype=np.uint8),
                       np.zeros((64, 96, 3), np.uint8),
                       recipes.near_gray(64, 96, 2)])
    b = mijpeg.Batch(96, 64, 3)
    b.upload(frames)
    b.encode(3)
    for i in range(3):
        assert b.output(i) == O.cref_encode(frames[i])
    b.close()


def test_dct_tolerance_and_replays_on_extremes():
    """Checkerboards maximise |coefficient| and the accumulation bound; flat
    even-offset blocks put DC exactly on integers; all must stay exact."""
    for img in (recipes.checkerboards(), recipes.gray_levels(), recipes.flat_colours(3)):
        H, W = img.shape[:2]
        b = mijpeg.Batch(W, H, 1, 100)
        b.upload(img)
        b.encode(1)
        assert b.output(0) == O.cref_encode(img, 100)
        b.close()


# ---------------------------------------------------------------------------
# size-independent properties at full size
# ---------------------------------------------------------------------------

def test_decodes_with_libjpeg_psnr():
    PIL = pytest.importorskip("PIL.Image")
    rgb = recipes.sample("sample_640x640")
    b = mijpeg.Batch(640, 640, 1)
    b.upload(ppm.rgb_to_bgr(rgb))
    b.encode(1)
    img = np.asarray(PIL.open(io.BytesIO(b.output(0))).convert("RGB"), np.float64)
    mse = ((img - rgb) ** 2).mean()
    psnr = 10 * np.log10(255 ** 2 / mse)
    assert psnr > 24.0  # survey: 25.31 dB via PIL on the reference output
    b.close()


def test_c_host_tool_three_call_and_fused():
    pkg = os.path.dirname(mijpeg.LIB_PATH)
    tool = os.path.join(pkg, "host", "encode_ppm")
    if not os.path.exists(tool):
        subprocess.check_call(["make", "-s", "-C", pkg, "host/encode_ppm"])
    src = os.path.join(recipes.GOLDEN, "sample_64x64.ppm")
    gold = open(os.path.join(recipes.GOLDEN, "sample_64x64.jpg"), "rb").read()
    with tempfile.TemporaryDirectory() as d:
        for extra in ([], ["--fused"]):
            out = os.path.join(d, "o.jpg")
            subprocess.check_call([tool, src, out, "50"] + extra, stdout=subprocess.DEVNULL)
            assert open(out, "rb").read() == gold


@pytest.mark.parametrize("split", [True, False])
def test_split_and_fused_pipelines_same_bytes(split):
    """split (K1 -> coefficient planes -> tokenize pass) and fused (K1 emits
    tokens) give the reference's JFIF."""
    frames = np.stack([recipes.config3_frame(0, 544, 960), recipes.noise(544, 960, 3)])
    b = mijpeg.Batch(960, 544, 2)
    b.set_split(split)
    b.upload(frames)
    b.encode(2)
    for i in range(2):
        assert b.output(i) == O.cref_encode(frames[i])
    b.close()


def test_fused_pipeline_keep_coefs_golden(manifest):
    ent = manifest["sample_640x640"]
    bgr = case_input("sample_640x640", ent)
    b = mijpeg.Batch(640, 640, 1, keep_coefs=True)
    b.set_split(False)
    b.upload(bgr)
    b.encode(1)
    assert sha(b.output(0)) == ent["jpg_sha256"]
    Y, Cb, Cr = b.coefs(0, diffed=True)
    assert [sha(Y), sha(Cb), sha(Cr)] == ent["coef_sha256"]
    b.close()


def _luma_group_bits(Y, tabs, W, H, group, tiles_x):
    """Exact bits of luma pack group `group` (PACK_SEGS = 64 segments; a
    segment is 16 blocks of one block row inside one 128-px tile column),
    from the oracle's differenced coefficients and tables (encoder.c:434-502)."""
    dc, ac = tabs[0], tabs[1]
    bw, bh = W // 8, H // 8
    Yb = Y.reshape(bh * bw, 64)
    bits = 0
    for s in range(64 * group, min(64 * (group + 1), bh * tiles_x)):
        r, tx = divmod(s, tiles_x)
        for bx in range(16 * tx, min(16 * tx + 16, bw)):
            blk = Yb[r * bw + bx]
            d = int(blk[0])
            c = abs(d).bit_length()
            bits += dc.sym_code_len[c] + c
            nz = np.flatnonzero(blk[1:]) + 1
            prev = 0
            for z in nz:
                run = int(z) - prev - 1
                c = abs(int(blk[z])).bit_length()
                bits += (run >> 4) * ac.sym_code_len[0xF0] + ac.sym_code_len[((run & 15) << 4) | c] + c
                prev = int(z)
            if blk[63] == 0:
                bits += ac.sym_code_len[0x00]
    return bits


@pytest.mark.parametrize("q", [50, 100])
def test_pack_window_paths_in_one_scan(q):
    """k_pack_flat's two placement paths in one scan (both at Q=100, the
    single-window one alone at Q=50): a pack group whose bits fit one LDS
    window (4096 words; the 6144-word variant at Q >= 85) is placed relative to its own
    first bit and stored after the look-back; a wider one (noise rows: its
    bits are asserted to exceed the window) takes the look-back first and is
    packed window by window at absolute offsets (put_bits64_win, tokens
    reloaded per window).  Natural and flat rows follow in the same scan, so
    the seams between both kinds of groups land in one bitstream."""
    rng = np.random.default_rng(q)
    W, H = 1920, 96
    nat = ppm.rgb_to_bgr(np.tile(recipes.sample("sample_640x640"), (1, 3, 1))[:32, :W])
    img = np.concatenate([rng.integers(0, 256, (32, W, 3), dtype=np.uint8), nat,
                          np.full((32, W, 3), 77, np.uint8)])
    frames = np.stack([img, img[::-1].copy()])
    # frame 0's first luma group (noise) is wider than one window at Q=100
    # (516k bits) and fits one at Q=50 (124k); frame 1's first (flat) fits
    b = mijpeg.Batch(W, H, 2, q)
    # the library's window at this quality (mij_batch_geometry: ent_args'
    # pack_wide choice, whatever window sizes it was built with)
    window = b.geometry()["pack_window_words"] * 32
    Y, _, _, tabs, _ = O.cref_stages(frames[0], q)
    wide = _luma_group_bits(Y, tabs, W, H, 0, (W + 127) // 128) > window
    assert wide == (q == 100)
    Y1, _, _, tabs1, _ = O.cref_stages(frames[1], q)
    assert _luma_group_bits(Y1, tabs1, W, H, 0, (W + 127) // 128) < window
    b.upload(frames)
    b.encode(2)
    for i in range(2):
        got, ref = b.output(i), O.cref_encode(frames[i], q)
        assert got == ref, f"frame {i} q{q}: first diff {first_diff(got, ref)}"
    b.close()


@pytest.mark.parametrize("nsub", [2, 3])
def test_overlapped_sub_batches_same_bytes(nsub):
    """mij_batch_set_overlap: sub-batches whose entropy stages run on a second
    stream beside the next sub-batch's K1 give the reference's JFIF, also
    when the frame count does not divide evenly, and across repeated encodes."""
    frames = np.stack([recipes.config3_frame(i, 272, 480) for i in range(4)] + [recipes.noise(272, 480, 5)])
    b = mijpeg.Batch(480, 272, 5)
    b.set_overlap(nsub)
    b.upload(frames)
    for _ in range(2):
        b.encode(5)
        for i in range(5):
            assert b.output(i) == O.cref_encode(frames[i])
    b.close()


@pytest.mark.parametrize("q", [75, 90])
@pytest.mark.parametrize("split", [False, True])
def test_high_quality_replays_both_pipelines(q, split):
    """At high Q most N-tiles carry a straddling coefficient (~10^4 FP64
    replays per 4K frame at Q=90): the in-place replays of the fused K1 and
    k_fix_blocks of the split pipeline both give the reference's bytes, and
    the replay counter counts them."""
    frames = np.stack([recipes.config3_frame(i, 256, 512) for i in range(3)])
    b = mijpeg.Batch(512, 256, 3, q)
    b.set_split(split)
    b.upload(frames)
    b.encode(3)
    for i in range(3):
        assert b.output(i) == O.cref_encode(frames[i], q)
    assert b.replays() > 0
    b.close()


@pytest.mark.parametrize("W", [144, 160, 176, 192, 208, 224, 240])
def test_coefficient_k1_partial_last_tile(W):
    """The coefficient K1 stores whole block lines by trading chunks between
    lanes b and b^8; in the last 128-px tile of a row only some block
    columns exist (here 2..14 luma, 1..7 chroma), so the second store's lanes
    fall back to repeating their first.  Split pipeline (coefficient planes
    -> tokenize) against the reference's bytes, natural and noise content."""
    H = 48
    frames = np.stack([recipes.config3_frame(1, H, W), recipes.noise(H, W, W)])
    b = mijpeg.Batch(W, H, 2)
    b.set_split(True)
    b.upload(frames)
    b.encode(2)
    for i in range(2):
        got, ref = b.output(i), O.cref_encode(frames[i])
        assert got == ref, f"W={W} frame {i}: first diff {first_diff(got, ref)}"
    b.close()
