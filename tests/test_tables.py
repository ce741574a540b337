"""GPU: k_tables (the optimized Huffman tables, /root/reference/main/encoder.c:180-301)
against the oracle (oracle/cpu_ref.c build_table, pinned to the reference
build by the golden table dumps) on synthetic histograms rich in ties -- the
selection's tie rule (the <= scan of :196-206 picks the highest index), the
16-bit limit loop (:239-259) and the sentinel quirk (:277) decide every
field of the huff_code struct, including sym_freq's merged counts and the
`next` chains.  Histograms are uploaded through mij_batch_build_tables (k_tables alone)."""
import numpy as np
import pytest

import mijpeg
import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ["sym_freq", "code_len", "next", "code_len_freq", "sym_sorted", "sym_code_len", "sym_code"]


def fib_hist(n):
    """counts 1, 1, 2, 3, 5, ... on n symbols: code lengths up to n - 1"""
    h = np.zeros(256, np.uint32)
    a, b = 1, 1
    for s in range(n):
        h[s * 7 % 256] = a
        a, b = b, a + b
    return h


def cases():
    rng = np.random.default_rng(2024)
    out = []
    out.append(("random 0..3", rng.integers(0, 4, 256)))
    live = np.arange(256) < 254  # at most 254 coded symbols (the sentinel of :277 needs a free slot)
    out.append(("all ones", live * 1))
    out.append(("all equal 1000", live * 1000))
    out.append(("two symbols", np.where(np.arange(256) < 2, 5, 0)))
    out.append(("one symbol", np.where(np.arange(256) == 17, 9, 0)))
    out.append(("dc-like 12", np.where(np.arange(256) < 12, rng.integers(1, 50, 256), 0)))
    out.append(("pairs", live * np.repeat(rng.integers(1, 20, 128), 2)))
    out.append(("power law", live * (1e6 / (1 + np.arange(256)) ** 1.5).astype(np.int64)))
    out.append(("large counts", live * rng.integers(1 << 21, 1 << 22, 256)))
    # counts of 2^23 and more: the 64-bit leaf sort and the wide merge keys
    # (the whole table's count kept below 2^31, as the reference's int sums need)
    out.append(("counts above 2^23", live * rng.integers(1 << 23, 1 << 24, 256) * (rng.random(256) < 0.15)))
    out.append(("one count above 2^23", np.where(np.arange(256) == 3, (1 << 24) + 5, live * rng.integers(0, 9, 256))))
    out.append(("ac-like 162", np.where((np.arange(256) & 15) <= 10, rng.integers(0, 300, 256), 0)))
    out.append(("sparse ties", np.where(rng.random(256) < 0.2, rng.integers(1, 4, 256), 0)))
    out.append(("fibonacci 30", fib_hist(30)))
    out.append(("fibonacci 45 (limit loop: lengths to 24)", fib_hist(45)))
    for k in range(4):  # more random tie-rich mixes
        v = live * rng.integers(0, 6, 256) * rng.integers(0, 2, 256) * (1 + (rng.random(256) < 0.1) * 37)
        out.append((f"mixed {k}", v))
    return [(n, np.asarray(h, np.uint32)) for n, h in out]


def test_tables_match_oracle_on_tie_rich_histograms():
    cs = cases()
    n = len(cs)
    hist = np.zeros((n, 4, 257), np.uint32)
    for f, (_, h) in enumerate(cs):
        for t in range(4):  # four tables per frame: the case and three rotations of it
            hist[f, t, :256] = np.roll(h, 37 * t)
    b = mijpeg.Batch(16, 16, n)
    b.build_tables(n, hist)
    for f, (name, _) in enumerate(cs):
        got = b.tables(f)
        for t in range(4):
            rc, want = O.cref_build_table(hist[f, t, :256])
            assert rc == 0, name
            for fld in FIELDS:
                assert list(getattr(got[t], fld)) == list(getattr(want, fld)), (name, t, fld)
    b.close()


def test_table_failure_matches_oracle():
    """All 256 symbols coded: the reference's sentinel write (:277) would land
    on a live sym_sorted entry (undefined): the oracle refuses the counts and
    so does the library (MIJ_ETABLE), naming that frame."""
    bad = np.ones(256, np.uint32)
    rc, _ = O.cref_build_table(bad)
    assert rc != 0
    hist = np.zeros((2, 4, 257), np.uint32)
    hist[0, :, :10] = 3
    hist[1, :, :256] = bad
    b = mijpeg.Batch(16, 16, 2)
    with pytest.raises(mijpeg.MijError, match="frame 1"):
        b.build_tables(2, hist)
    b.close()


def test_tables_match_oracle_on_random_histograms():
    """Randomised shapes for the merge loop's forms (the scalar short form,
    its window reloads, and the general loop it leaves for on an insert or a
    merged queue longer than its window): power laws of random slope, flat
    and near-flat counts, few and many symbols, heavy ties -- 256 tables
    against the oracle, every field."""
    rng = np.random.default_rng(77)
    n = 64
    hist = np.zeros((n, 4, 257), np.uint32)
    for f in range(n):
        for t in range(4):
            k = int(rng.integers(2, 254))  # coded symbols
            kind = (4 * f + t) % 5
            if kind == 0:  # power law
                v = (rng.integers(1000, 200000) / (1 + np.arange(k)) ** rng.uniform(0.5, 2.5)).astype(np.int64) + 1
            elif kind == 1:  # flat
                v = np.full(k, int(rng.integers(1, 50)))
            elif kind == 2:  # near-flat
                v = rng.integers(100, 104, k)
            elif kind == 3:  # heavy ties from a small alphabet of counts
                v = rng.choice(np.array([1, 2, 3, 5, 8]), k)
            else:  # wide spread
                v = rng.integers(1, 1 << int(rng.integers(2, 20)), k)
            h = np.zeros(256, np.int64)
            h[rng.permutation(256)[:k]] = v
            hist[f, t, :256] = h.astype(np.uint32)
    b = mijpeg.Batch(16, 16, n)
    b.build_tables(n, hist)
    for f in range(n):
        got = b.tables(f)
        for t in range(4):
            rc, want = O.cref_build_table(hist[f, t, :256])
            assert rc == 0, (f, t)
            for fld in FIELDS:
                assert list(getattr(got[t], fld)) == list(getattr(want, fld)), (f, t, fld)
    b.close()
