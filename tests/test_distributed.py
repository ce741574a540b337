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
