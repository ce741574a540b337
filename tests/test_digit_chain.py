"""The K1 MFMA digit chain's pair shifts (DESIGN.md §3 'DCT on MFMA', §5.2
'Pair shifts'): K1 shifts the int32 accumulators of rows z | z + 1 (z even)
as one 64-bit value between the three base-128 digits, with a bias of 2^17
on the low element from the first digit's C input.  That is exact only if
the low element stays in [0, 2^25) before each 7-bit shift, for every row of
fill_tables' digit matrix (mij_api.hip fill_tables, restated here as in
tests/tau_check.c) and every block of pixels.  CPU only."""
import math

import numpy as np

K_ZZ = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,
        7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
        39, 46, 53, 60, 61, 54, 47, 55, 62, 63]
BIAS = 1 << 17


def digits():
    """[3][64 z][64 pixels] int8 digits, top first (fill_tables' dig[0..2])."""
    cosd = [math.cos((2 * (i // 8) + 1) * (i % 8) * math.pi / 16) for i in range(64)]
    d = np.zeros((3, 64, 64), dtype=np.int64)
    for z in range(64):
        rz = K_ZZ[z]
        v, u = rz >> 3, rz & 7
        for p in range(64):
            if z == 0:
                d[2, z, p] = 1  # DC row: the exact pixel sum in the last digit
                continue
            k = cosd[(p >> 3) * 8 + v] * cosd[(p & 7) * 8 + u]
            if u == 0:
                k *= math.sqrt(0.5)
            if v == 0:
                k *= math.sqrt(0.5)
            w = int(np.rint(k * 524288.0))  # llround (no ties at these values)
            d0 = ((w + 64) & 127) - 64
            w1 = (w - d0) >> 7
            d1 = ((w1 + 64) & 127) - 64
            d2 = (w1 - d1) >> 7
            assert (d2 << 14) + (d1 << 7) + d0 == w and -128 <= d2 <= 127
            d[0, z, p], d[1, z, p], d[2, z, p] = d2, d1, d0
    return d


def extremes(w):
    """min and max of sum w * x over x in [-128, 127]^64."""
    return int(np.where(w > 0, -128 * w, 127 * w).sum()), int(np.where(w > 0, 127 * w, -128 * w).sum())


def test_partial_sums_keep_the_low_element_in_range():
    d = digits()
    for z in range(0, 64, 2):  # the low element of each pair
        lo1, hi1 = extremes(d[0, z])
        lo2, hi2 = extremes(d[0, z] * 128 + d[1, z])
        assert 0 <= lo1 + BIAS and hi1 + BIAS < 1 << 25, z
        assert 0 <= lo2 + (BIAS << 7) and hi2 + (BIAS << 7) < 1 << 25, z


def _u32(a):
    return a & 0xFFFFFFFF


def test_pair_shift_chain_equals_the_plain_chain():
    d = digits()
    rng = np.random.default_rng(7)
    blocks = [rng.integers(-128, 128, 64), np.full(64, -128), np.full(64, 127)]
    # the extreme pattern of every row (the worst case of its partial sums)
    for z in range(64):
        w = d[0, z] * 128 + d[1, z]
        blocks.append(np.where(w > 0, 127, -128))
        blocks.append(np.where(w > 0, -128, 127))
    for x in blocks:
        x = np.asarray(x, dtype=np.int64)
        D = [d[k] @ x for k in range(3)]  # per-digit sums, [64 z]
        plain = _u32(_u32(_u32(D[0] << 7) + D[1]) << 7) + D[2]
        bias = np.where(np.arange(64) % 2 == 0, BIAS, 0)
        acc = _u32(D[0] + bias)
        for k in (1, 2):
            lo, hi = acc[0::2].astype(np.uint64), acc[1::2].astype(np.uint64)
            assert (lo < 1 << 25).all()  # no bit of the low element crosses
            pair = ((hi << np.uint64(32)) | lo) << np.uint64(7)  # wraps mod 2^64
            acc = np.empty_like(acc)
            acc[0::2] = (pair & np.uint64(0xFFFFFFFF)).astype(np.int64)
            acc[1::2] = (pair >> np.uint64(32)).astype(np.int64)
            acc = _u32(acc + D[k])
        acc[0::2] ^= 0x80000000
        assert (_u32(acc) == _u32(plain)).all()
        n = np.where(plain >= 1 << 31, plain - (1 << 32), plain)
        assert (n == d[0] @ x * 16384 + d[1] @ x * 128 + d[2] @ x).all()
