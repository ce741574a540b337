"""Multi-process (world_size 2, gloo, CPU) coverage of the frame-parallel
path: the shard partition, the timing/unit reduction bench.py reports, and
that per-rank shards encoded independently reassemble into the single-process
result (the encode itself is the CPU oracle here -- the GPU encode of a shard
is the same library call the -m gpu tests cover)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import sharding


def test_frame_range_partitions_exactly():
    for n in (0, 1, 7, 8, 9, 255, 256, 1000):
        for world in (1, 2, 3, 4, 8):
            got = [list(sharding.frame_range(n, world, r)) for r in range(world)]
            flat = [i for g in got for i in g]
            assert flat == list(range(n))
            sizes = [len(g) for g in got]
            assert max(sizes) - min(sizes) <= (1 if n else 0)


def test_frame_range_rejects_bad_args():
    for args in ((4, 0, 0), (4, 2, 2), (4, 2, -1), (-1, 2, 0)):
        with pytest.raises(ValueError):
            sharding.frame_range(*args)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, frames, q, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        mine = sharding.frame_range(len(frames), world, rank)
        blobs = [O.cref_encode(frames[i], q) for i in mine]
        # rank-dependent fake timings: the reduction must report the max
        el, units = sharding.reduce_timing(0.5 + rank, len(mine) * 64 * 48, dist, "cpu")
        gathered = [None] * world
        dist.all_gather_object(gathered, blobs)
        if rank == 0:
            out.put((el, units, [b for g in gathered for b in g]))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_encode_matches_single_process():
    rng = np.random.default_rng(3)
    frames = [rng.integers(0, 256, (48, 64, 3), dtype=np.uint8) for _ in range(5)]
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, frames, 50, out)) for r in range(2)]
    for p in procs:
        p.start()
    el, units, blobs = out.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle as O
    assert el == 1.5
    assert units == 5 * 64 * 48
    assert blobs == [O.cref_encode(f, 50) for f in frames]


def test_band_rows_tile_the_frame():
    for H, world in ((4320, 8), (4320, 7), (64, 4), (2160, 3), (16, 1)):
        rows = [sharding.band_rows(H, world, r) for r in range(world)]
        assert rows[0][0] == 0
        for (a0, an), (b0, _) in zip(rows, rows[1:]):
            assert a0 + an == b0 and an % 16 == 0 and an > 0
        assert rows[-1][0] + rows[-1][1] == H
    with pytest.raises(ValueError):
        sharding.band_rows(48, 4, 0)   # 3 MCU rows for 4 bands
    with pytest.raises(ValueError):
        sharding.band_rows(40, 2, 0)   # not whole MCU rows


def _xch_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        x = sharding.TorchExchange(dist, "cpu")
        g = x.all_gather(np.full((2, 3), rank + 1, np.int16))
        b = x.all_gather(np.full((2, 3), (1 << 40) + rank, np.uint64))
        s = x.all_reduce_sum(np.full((2, 4, 257), rank + 1, np.uint32))
        buf = x.words_buffer(5)
        buf.copy_(torch.arange(5, dtype=torch.int32) + 10 * rank)
        got = x.gather_words(buf)
        if rank == 0:
            out.put(([a.tolist() for a in g], [a.tolist() for a in b], str(b[0].dtype), int(s.sum()),
                     str(s.dtype), got.tolist()))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_torch_exchange_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xch_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    g, b, bdt, total, sdt, words = out.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert g == [[[1] * 3] * 2, [[2] * 3] * 2]
    assert b == [[[(1 << 40)] * 3] * 2, [[(1 << 40) + 1] * 3] * 2] and bdt == "uint64"
    assert total == (1 + 2) * 2 * 4 * 257 and sdt == "uint32"
    assert words == [[0, 1, 2, 3, 4], [10, 11, 12, 13, 14]]


def test_band_pieces_table_reassembles_scans():
    """sharding.band_pieces: the word counts follow from the bit counts, and
    OR-ing the pieces of a gathered [world, maxw] buffer at their first words
    rebuilds each scan's bit string (a CPU model of mij_assemble_pieces)."""
    rng = np.random.default_rng(5)
    world, n = 4, 3
    bits = rng.integers(0, 300, (world, n, 3)).astype(np.uint64)
    bits[1, 0, 2] = 0  # an empty band share
    off = np.concatenate([np.zeros((1, n, 3), np.uint64), np.cumsum(bits, axis=0)[:-1]])
    allnw, maxw, pieces = sharding.band_pieces(bits, off)
    # every band share as a bit string placed at its global offset
    streams = {(f, c): rng.integers(0, 2, int(bits[:, f, c].sum())) for f in range(n) for c in range(3)}
    gathered = np.zeros((world, maxw), np.uint32)
    for r in range(world):
        w = []
        for f in range(n):
            for c in range(3):
                o, b = int(off[r, f, c]), int(bits[r, f, c])
                nw = int(allnw[r, f, c])
                assert nw == (o % 32 + b + 31) // 32
                piece = np.zeros(nw * 32, np.uint8)
                piece[o % 32:o % 32 + b] = streams[(f, c)][o:o + b]
                w.append(np.packbits(piece).view(">u4").astype(np.uint32))
        row = np.concatenate(w) if w else np.zeros(0, np.uint32)
        gathered[r, :row.size] = row
    scans = {k: np.zeros((v.size + 31) // 32 + 1, np.uint32) for k, v in streams.items()}
    flat = gathered.reshape(-1)
    for fc, first, src, cnt in pieces.tolist():
        scans[(fc // 3, fc % 3)][first:first + cnt] |= flat[src:src + cnt]
    for k, v in streams.items():
        bitsout = np.unpackbits(scans[k].astype(">u4").view(np.uint8))[:v.size]
        assert np.array_equal(bitsout, v), k
