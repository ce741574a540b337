"""Frame-parallel sharding across GPUs (one process per GPU).

The encode path shards by frame: every frame is an independent JFIF stream
with its own Huffman tables (reference main/encoder.c builds tables per
image, :193-298), so ranks never exchange data on the data path.  The only
collectives are control-plane ones: a barrier around timed regions and a
MAX / SUM reduction of the per-rank timings and unit counts (bench.py).

Strong scaling (a fixed list of frames spread over the ranks) uses
`frame_range`; weak scaling (each rank its own fixed batch, bench.py's
default) needs no partition at all.
"""
from __future__ import annotations


def frame_range(n_frames: int, world: int, rank: int) -> range:
    """Contiguous, balanced block of frame indices owned by `rank`.

    The first n_frames % world ranks take one extra frame; the blocks cover
    0..n_frames-1 exactly once, in order, so concatenating the ranks' outputs
    rank by rank restores the input order."""
    if world < 1 or not 0 <= rank < world or n_frames < 0:
        raise ValueError(f"bad shard request: n={n_frames} world={world} rank={rank}")
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def reduce_timing(elapsed_s: float, units: int, dist=None, device=None):
    """(max elapsed over ranks, sum of units over ranks).

    `dist` is torch.distributed (or None for a single process); `device` the
    tensor device the backend needs ("cuda:<local>" for nccl/RCCL, cpu for
    gloo)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(elapsed_s), int(units)
    import torch
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    u = torch.tensor([int(units)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), int(u.item())
