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
        x = sharding.TorchExchange(dist, "cpu")
        g = x.all_gather(np.full((2, 3), rank + 1, np.int16))
        s = x.all_reduce_sum(np.full((2, 4, 257), rank + 1, np.uint32))
        if rank == 0:
            buf = x.words_buffer(5)
            x.recv_from(buf, 1)
            out.put(([a.tolist() for a in g], int(s.sum()), buf.tolist()))
        else:
            import torch
            x.send_to_root(torch.arange(5, dtype=torch.int32))
    finally:
        dist.destroy_process_group()


def test_torch_exchange_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xch_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    g, total, words = out.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert g == [[[1] * 3] * 2, [[2] * 3] * 2]
    assert total == (1 + 2) * 2 * 4 * 257
    assert words == [0, 1, 2, 3, 4]
