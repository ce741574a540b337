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


# ---------------------------------------------------------------------------
# one large frame over several ranks
# ---------------------------------------------------------------------------

def band_rows(height: int, world: int, rank: int):
    """(first row, rows) of rank's band: a contiguous, balanced block of MCU
    rows (16 pixel rows each).  Bands in rank order tile the frame, so every
    component's blocks of a band are one contiguous range of its scan."""
    if height % 16 or height // 16 < world:
        raise ValueError(f"cannot split {height} rows into {world} bands of whole MCU rows")
    r = frame_range(height // 16, world, rank)
    return 16 * r.start, 16 * len(r)


class TorchExchange:
    """The four exchanges of a banded encode over torch.distributed: small
    all-gathers / one all-reduce, plus point-to-point transfer of the packed
    words to the root.  `device` is "cuda:<local>" for nccl (RCCL over xGMI)
    or "cpu" for gloo."""

    def __init__(self, dist, device="cpu"):
        import torch
        self.torch, self.dist, self.device = torch, dist, device
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()

    def all_gather(self, arr):
        import numpy as np
        t = self.torch.from_numpy(np.ascontiguousarray(arr).astype(np.int64)).to(self.device)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.cpu().numpy() for o in out]

    def all_reduce_sum(self, arr):
        import numpy as np
        t = self.torch.from_numpy(np.ascontiguousarray(arr).astype(np.int64)).to(self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.cpu().numpy()

    def words_buffer(self, nwords: int):
        # empty, not zeros: a fill kernel on torch's stream could race with the
        # library's copy into the buffer on its own stream
        return self.torch.empty(max(int(nwords), 1), dtype=self.torch.int32, device=self.device)

    def send_to_root(self, buf):
        self.dist.send(buf, dst=0)

    def recv_from(self, buf, src: int):
        self.dist.recv(buf, src=src)


class LocalExchange:
    """world = 1: the exchanges of encode_banded degenerate to identities."""
    world, rank, device = 1, 0, "cpu"

    def __init__(self):
        import torch
        self.torch = torch

    def all_gather(self, arr):
        import numpy as np
        return [np.ascontiguousarray(arr).astype(np.int64)]

    def all_reduce_sum(self, arr):
        import numpy as np
        return np.ascontiguousarray(arr).astype(np.int64)

    def words_buffer(self, nwords: int):
        return self.torch.empty(max(int(nwords), 1), dtype=self.torch.int32)


def encode_banded(band, n: int, xch, frame_batch=None):
    """This rank's share of encoding n frames split into xch.world bands.

    `band` is a mijpeg.Batch of width x band rows holding this rank's bands of
    the n frames; `frame_batch` (root only) a Batch of the whole frame that
    receives the assembled JFIF streams (read them with frame_batch.output).
    Returns the per-frame, per-scan total bits.  The exchanges follow
    include/mijpeg.h: last DCs (all-gather), histograms (all-reduce), bits
    (all-gather), packed words (to the root)."""
    import numpy as np
    rank, world = xch.rank, xch.world
    last = band.band_analyze(n)                                    # [n, 3]
    lasts = xch.all_gather(last)
    prev = np.zeros((n, 3), np.int16) if rank == 0 else lasts[rank - 1].astype(np.int16)
    hist = band.band_histograms(n, prev)                           # [n, 4, 257]
    ghist = xch.all_reduce_sum(hist).astype(np.uint32)
    bits = band.band_tables(n, ghist)                              # [n, 3]
    allbits = np.stack(xch.all_gather(bits)).astype(np.uint64)    # [world, n, 3]
    offset = allbits[:rank].sum(axis=0) if rank else np.zeros((n, 3), np.uint64)
    total = allbits.sum(axis=0)
    nw = band.band_pack(n, offset).astype(np.int64)                # [n, 3]
    allnw = np.stack(xch.all_gather(nw))                           # [world, n, 3]
    alloff = np.concatenate([np.zeros((1, n, 3), np.uint64), np.cumsum(allbits, axis=0)[:-1]])
    on_dev = str(xch.device).startswith("cuda")

    def flat_words(r_nw):
        starts = np.concatenate([[0], np.cumsum(r_nw.reshape(-1))])
        return starts

    my_starts = flat_words(nw)
    buf = xch.words_buffer(my_starts[-1])
    for f in range(n):
        for c in range(3):
            k = f * 3 + c
            cnt = int(nw[f, c])
            if not cnt:
                continue
            if on_dev:
                band.band_words(f, c, cnt, dst_dev_ptr=buf.data_ptr() + 4 * int(my_starts[k]))
            else:
                buf[int(my_starts[k]):int(my_starts[k]) + cnt] = xch.torch.from_numpy(
                    band.band_words(f, c, cnt).view(np.int32))
    if rank != 0:
        xch.send_to_root(buf)
        return total
    frame_batch.assemble_begin(n, ghist)
    for r in range(world):
        starts = flat_words(allnw[r])
        if r == 0:
            rbuf = buf
        else:
            rbuf = xch.words_buffer(starts[-1])
            xch.recv_from(rbuf, r)
        if on_dev:
            xch.torch.cuda.synchronize(xch.device)
        for f in range(n):
            for c in range(3):
                k = f * 3 + c
                cnt = int(allnw[r][f, c])
                if not cnt:
                    continue
                first_word = int(alloff[r][f, c]) >> 5
                if on_dev:
                    frame_batch.assemble_words(f, c, first_word, src_dev_ptr=rbuf.data_ptr() + 4 * int(starts[k]),
                                               nwords=cnt)
                else:
                    frame_batch.assemble_words(f, c, first_word,
                                               rbuf[int(starts[k]):int(starts[k]) + cnt].numpy().view(np.uint32))
    frame_batch.assemble_end(n, total)
    return total
