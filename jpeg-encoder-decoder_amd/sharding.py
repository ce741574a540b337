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

import os


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


def gather_ints(values, dist=None, device=None):
    """Every rank's list of ints (same length on every rank), in rank order:
    [[rank 0's values], [rank 1's], ...].  One all-gather; a single process
    returns [values]."""
    vals = [int(v) for v in values]
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [vals]
    import torch
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[int(x) for x in o.cpu().tolist()] for o in out]


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
    """The exchanges of a banded encode over torch.distributed: three small
    collectives (all-gather of the last DCs, all-reduce of the histograms,
    all-gather of the bit counts) and one gather of every rank's packed words
    to the root.  `device` is "cuda:<local>" for nccl (RCCL over xGMI: the
    words never leave HBM) or "cpu" for gloo."""

    def __init__(self, dist, device="cpu"):
        import torch
        self.torch, self.dist, self.device = torch, dist, device
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.on_dev = str(device).startswith("cuda")

    def _tensor(self, arr):
        # int16 / uint32 / uint64 counts travel as int32 / int32 / int64 (same bits)
        import numpy as np
        a = np.ascontiguousarray(arr)
        view = {np.dtype(np.int16): np.int32, np.dtype(np.uint32): np.int32,
                np.dtype(np.uint64): np.int64}.get(a.dtype)
        a = a.astype(np.int32) if a.dtype == np.int16 else (a.view(view) if view else a)
        return self.torch.from_numpy(a).to(self.device)

    def all_gather(self, arr):
        import numpy as np
        t = self._tensor(arr)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        dt = np.asarray(arr).dtype
        res = [o.cpu().numpy() for o in out]
        return [r.astype(dt) if dt == np.int16 else r.view(dt) for r in res]

    def all_reduce_sum(self, arr):
        import numpy as np
        t = self._tensor(arr)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.cpu().numpy().view(np.asarray(arr).dtype)

    def words_buffer(self, nwords: int):
        # empty, not zeros: a fill kernel on torch's stream could race with the
        # library's copy into the buffer on its own stream
        t = self.torch.empty(max(int(nwords), 1), dtype=self.torch.int32, device=self.device)
        if self.on_dev:  # the block is free on torch's stream order; the library writes on its own
            self.torch.cuda.current_stream(self.device).synchronize()
        return t

    def gather_words(self, buf):
        """Every rank's equally sized word buffer to the root: [world, n] there,
        None elsewhere."""
        out = None
        if self.rank == 0:
            out = self.torch.empty((self.world, buf.numel()), dtype=buf.dtype, device=buf.device)
            self.dist.gather(buf, gather_list=list(out.unbind(0)), dst=0)
            if self.on_dev:  # the library reads it on its own stream
                self.torch.cuda.synchronize(self.device)
        else:
            self.dist.gather(buf, dst=0)
        return out


class LocalExchange:
    """world = 1: the exchanges of encode_banded degenerate to identities.
    device "cuda:<n>" keeps the word buffer in HBM (torch's HIP runtime must
    then have been initialised before the library's, as bench.py does)."""
    world, rank = 1, 0

    def __init__(self, device="cpu"):
        import torch
        self.torch, self.device = torch, device
        self.on_dev = str(device).startswith("cuda")

    def all_gather(self, arr):
        import numpy as np
        return [np.ascontiguousarray(arr)]

    def all_reduce_sum(self, arr):
        import numpy as np
        return np.ascontiguousarray(arr)

    def words_buffer(self, nwords: int):
        t = self.torch.empty(max(int(nwords), 1), dtype=self.torch.int32, device=self.device)
        if self.on_dev:
            self.torch.cuda.current_stream(self.device).synchronize()
        return t

    def gather_words(self, buf):
        return buf.reshape(1, -1)


def band_pieces(allbits, alloff):
    """Word counts of every (rank, frame, scan) band share -- they follow from
    the bit counts, so they need no exchange of their own -- and the
    assemble_pieces table for a [world, maxw] gathered buffer whose rank-r row
    holds that rank's words in (frame, scan) order: rows {frame * 3 + scan,
    first word in the scan, first source word, words}."""
    import numpy as np
    world, n = allbits.shape[:2]
    allnw = ((alloff & np.uint64(31)) + allbits + np.uint64(31)) >> np.uint64(5)   # [world, n, 3]
    flat = allnw.reshape(world, n * 3)
    starts = np.concatenate([np.zeros((world, 1), np.uint64), np.cumsum(flat, axis=1)[:, :-1]], axis=1)
    maxw = int(flat.sum(axis=1).max()) if world else 0
    r, k = np.nonzero(flat)
    pieces = np.stack([k.astype(np.uint64), alloff.reshape(world, n * 3)[r, k] >> np.uint64(5),
                       r.astype(np.uint64) * np.uint64(max(maxw, 1)) + starts[r, k], flat[r, k]], axis=1)
    return allnw, maxw, pieces.astype(np.uint64)


def encode_banded(band, n: int, xch, frame_batch=None):
    """This rank's share of encoding n frames split into xch.world bands.

    `band` is a mijpeg.Batch of width x band rows holding this rank's bands of
    the n frames; `frame_batch` (root only) a Batch of the whole frame -- an
    assembler (mijpeg.Batch(..., assembler=True)) is enough -- that receives
    the assembled JFIF streams (read them with frame_batch.output).  Returns
    the per-frame, per-scan total bits.  The exchanges follow
    include/mijpeg.h: last DCs (all-gather), histograms (all-reduce), bits
    (all-gather), then every rank's packed words in one buffer (one library
    copy), gathered to the root in one collective and OR-ed into the scans in
    one launch."""
    import numpy as np
    rank, world = xch.rank, xch.world
    last = band.band_analyze(n)                                    # [n, 3] int16
    lasts = xch.all_gather(last)
    prev = np.zeros((n, 3), np.int16) if rank == 0 else lasts[rank - 1]
    hist = band.band_histograms(n, prev)                           # [n, 4, 257] uint32
    ghist = xch.all_reduce_sum(hist)
    bits = band.band_tables(n, ghist)                              # [n, 3] uint64
    allbits = np.stack(xch.all_gather(bits))                       # [world, n, 3]
    alloff = np.concatenate([np.zeros((1, n, 3), np.uint64), np.cumsum(allbits, axis=0)[:-1]])
    total = allbits.sum(axis=0)
    nw = band.band_pack(n, alloff[rank])                           # [n, 3]
    allnw, maxw, pieces = band_pieces(allbits, alloff)
    if not np.array_equal(allnw[rank], nw):
        raise RuntimeError("band word counts differ from the ones the bit counts imply")
    buf = xch.words_buffer(maxw)
    if xch.on_dev:
        band.band_words_all(n, dst_dev_ptr=buf.data_ptr(), cap_words=buf.numel())
    else:
        band.band_words_all(n, dst=buf.numpy())
    gathered = xch.gather_words(buf)
    if rank != 0:
        return total
    frame_batch.assemble_begin(n, ghist)
    if xch.on_dev:
        frame_batch.assemble_pieces(pieces, src_dev_ptr=gathered.data_ptr(), src_words=gathered.numel())
    else:
        frame_batch.assemble_pieces(pieces, src=gathered.numpy())
    frame_batch.assemble_end(n, total)
    return total


# ---------------------------------------------------------------------------
# the band protocol device-resident (include/mijpeg.h mij_band_*_async):
# every exchanged value stays in HBM, every library call and collective is
# enqueued on the band batch's own HIP stream; one host read per step (the
# largest band's word count, to size the gather)
# ---------------------------------------------------------------------------

class DeviceExchange:
    """Collectives on device tensors for encode_banded_dev: torch.distributed
    (nccl = RCCL over xGMI) with the current stream set to the band batch's
    stream, or the identities of one rank (dist None).  Every result is a
    device tensor; nothing is copied to the host."""

    def __init__(self, dist=None, device="cuda:0"):
        import torch
        self.torch, self.dist, self.device = torch, dist, device
        self.world = dist.get_world_size() if dist is not None else 1
        self.rank = dist.get_rank() if dist is not None else 0

    def all_gather(self, t):
        """[world, *t.shape] (t's bytes, any dtype)"""
        if self.world == 1:
            return t.unsqueeze(0)
        out = self.torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(out, t.contiguous())
        return out

    def all_reduce_sum(self, t):
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t

    def host_buffer(self, n: int):
        """a pinned host int64 buffer of n values, reused (a step reads it
        before the next step writes it)"""
        hb = getattr(self, "_hbuf", None)
        if hb is None or hb.numel() < n:
            hb = self._hbuf = self.torch.empty(n, dtype=self.torch.int64, pin_memory=True)
        return hb[:n]

    def gather(self, buf):
        """every rank's equally sized buffer to the root: [world, n] there"""
        if self.world == 1:
            return buf.reshape(1, -1)
        if self.rank == 0:
            out = self.torch.empty((self.world, buf.numel()), dtype=buf.dtype, device=buf.device)
            self.dist.gather(buf, gather_list=list(out.unbind(0)), dst=0)
            return out
        self.dist.gather(buf, dst=0)
        return None


class StagedExchange(DeviceExchange):
    """DeviceExchange's collectives over a host backend (gloo): each one
    copies its device tensor to the host on the current stream (the band
    batch's stream inside encode_banded_dev, so the copy waits for the
    library's kernels), runs the gloo collective there and copies the result
    back to the device on the same stream.  encode_banded_dev then runs with
    world > 1 on one GPU -- several processes sharing it -- with exactly the
    indexing the RCCL run uses (the prefix bands' last DCs, the bounds, the
    [world, 3n + 1] bits, the gathered [world, stride] words)."""

    def __init__(self, dist, device="cuda:0"):
        super().__init__(dist, device)
        if dist is None:
            raise ValueError("StagedExchange needs a process group")

    def _to_host(self, t):
        return t.contiguous().cpu()  # blocking copy: waits for the current stream

    def all_gather(self, t):
        h = self._to_host(t)
        out = self.torch.empty((self.world,) + tuple(h.shape), dtype=h.dtype)
        self.dist.all_gather(list(out.unbind(0)), h)
        return out.to(t.device)

    def all_reduce_sum(self, t):
        h = self._to_host(t)
        self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM)
        t.copy_(h)
        return t

    def gather(self, buf):
        h = self._to_host(buf)
        if self.rank == 0:
            out = self.torch.empty((self.world, h.numel()), dtype=h.dtype)
            self.dist.gather(h, gather_list=list(out.unbind(0)), dst=0)
            return out.to(buf.device)
        self.dist.gather(h, dst=0)
        return None


# MIJ_HOST_READ=default: the host reads' copies on torch's default stream
# (rounds 4-6, kept for A/B) instead of the band batch's stream
_HOST_READ_DEFAULT = os.environ.get("MIJ_HOST_READ", "batch") == "default"
# MIJ_ASSEMBLE_STREAM=own: the root's assembly on the assembler's own stream
# behind cross-queue waits (rounds 4-6, kept for A/B)
_ASSEMBLE_OWN_STREAM = os.environ.get("MIJ_ASSEMBLE_STREAM", "band") == "own"


def _to_host(band, s, h, d_src, dev):
    """d_src (int64, on the band stream) -> the pinned host tensor h; returns
    the event to wait on.  The copy is the library's, on the band stream right
    after the collective that produced d_src, so it runs before the packing
    launched next (a copy on another stream waits for a free slot behind the
    packing's workgroups: 40 us on config 4), and torch's pinned allocator
    records no event of the library's stream."""
    import torch
    if _HOST_READ_DEFAULT:
        # (on torch's own stream: the host allocator keeps an event of the
        # copy's stream, and the library's stream may be gone before that
        # event is released)
        d = torch.cuda.default_stream(dev)
        d.wait_stream(s)
        with torch.cuda.stream(d):
            h.copy_(d_src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(d)
        return ev
    band.copy_to_host_async(h.data_ptr(), d_src.data_ptr(), 8 * d_src.numel())
    ev = torch.cuda.Event()
    ev.record(s)
    return ev


def encode_banded_dev(band, n: int, xch, frame_batch=None, events=None, emit: str = "root"):
    """encode_banded with the device-resident protocol: the last DCs (int16
    [n, 4], gathered as int32 pairs), the histograms (summed in place), the
    bit counts (gathered) and the packed words (gathered to the root) never
    leave HBM -- only the bands' word bounds (one int64 per rank) come to the
    host, to size the word exchange; the library calls and the collectives all
    run on the band batch's stream.  Every band packs from bit 0, so the bands pack at once;
    the root shifts each band's words to its bit position while assembling.
    The root's frame_batch (an assembler) builds its tables on its own stream
    while the bands pack, then assembles.  `events`: optional list that
    receives (name, torch.cuda.Event) pairs recorded on the band stream after
    each phase.  Returns nothing; read the frames from frame_batch.output().

    emit="bands" distributes the JFIF byte emission: once the bit counts are
    gathered every band knows where its scans start, stuffs the bytes of the
    final scans that lie wholly inside it (mij_band_stuff_async) and sends
    those, with a record of its few edge bits per scan, to the root, which
    writes the headers, the seam bytes between bands, the pads and EOI and
    copies the stuffed bytes into place (mij_assemble_stuffed_async) -- the
    root's share of the byte work no longer grows with the frame.  The price is
    a second host read (the stuffed sizes, to size the gather exactly).
    emit="root": the bands' packed words go to the root, which shifts them
    into place and emits the whole frame (mij_assemble_async)."""
    if emit not in ("root", "bands"):
        raise ValueError(f"emit must be 'root' or 'bands', not {emit!r}")
    torch = xch.torch
    rank, world = xch.rank, xch.world
    dev = xch.device
    s = torch.cuda.ExternalStream(band.stream_ptr(), device=dev)
    a = torch.cuda.ExternalStream(frame_batch.stream_ptr(), device=dev) if rank == 0 else None

    def mark(name):
        if events is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            events.append((name, e))

    with torch.cuda.stream(s):
        mark("start")
        last = torch.empty((n, 4), dtype=torch.int16, device=dev)
        band.band_analyze_async(n, last.data_ptr())
        mark("analyze")
        prev = 0                                                  # band 0: zeros
        if world > 1:
            lasts = xch.all_gather(last.view(torch.int32))       # [world, n, 2] = int16 [world, n, 4]
            if rank:
                prev = lasts[rank - 1].contiguous().view(torch.int16)
        hist = torch.empty((n, 4, 257), dtype=torch.int32, device=dev)
        band.band_histograms_async(n, prev if isinstance(prev, int) else prev.data_ptr(), hist.data_ptr())
        xch.all_reduce_sum(hist)
        mark("histograms")
        if a is not None:
            a.wait_stream(s)
            with torch.cuda.stream(a):
                frame_batch.assemble_tables_async(n, hist.data_ptr())
        # the bands' word bounds reach the host while the bands pack: no step
        # waits for the packing before the word exchange is issued
        bound = torch.empty(1, dtype=torch.int64, device=dev)
        band.band_tables_async(n, hist.data_ptr(), bound.data_ptr())
        bounds = xch.all_gather(bound)                            # [world, 1]
        h_bounds = xch.host_buffer(world)
        ready = _to_host(band, s, h_bounds, bounds.view(-1), dev)
        bits = torch.empty(3 * n + 1, dtype=torch.int64, device=dev)
        band.band_pack_async(n, bits.data_ptr())
        allbits = xch.all_gather(bits).contiguous()               # [world, 3n + 1]
        mark("pack")
        ready.synchronize()
        if emit == "bands":
            # the stuffed bytes of a band <= 2x its whole bytes <= 8 x its word bound
            cap = 8 * max(1, int(h_bounds.max()))
            sbuf = torch.empty(cap + 48, dtype=torch.uint8, device=dev)
            rec = torch.empty(n * 3 * 4, dtype=torch.int64, device=dev)
            tot = torch.empty(1, dtype=torch.int64, device=dev)
            band.band_stuff_async(n, allbits.data_ptr(), world, rank, rec.data_ptr(), tot.data_ptr(),
                                  sbuf.data_ptr(), cap)
            allrec = xch.all_gather(rec).contiguous()             # [world, n*3*4]
            tots = xch.all_gather(tot)                           # [world, 1]
            h_tot = xch.host_buffer(2 * world)[world:]
            _to_host(band, s, h_tot, tots.view(-1), dev).synchronize()
            if int(h_tot.max()) > cap:  # (every rank sees the same totals: all raise)
                raise RuntimeError(f"band stuffing: {int(h_tot.max())} stuffed bytes exceed the "
                                   f"{cap}-byte buffer the word bound gave")
            # exact gather size (+16: the root's word copies read one word past)
            stride = (int(h_tot.max()) + 31) & ~15
            gathered = xch.gather(sbuf[:stride])
            mark("stuff")
            if a is None:
                return
        else:
            stride = max(1, int(h_bounds.max()))
            buf = torch.empty(stride, dtype=torch.int32, device=dev)
            band.band_words_async(n, buf.data_ptr(), stride)
            gathered = xch.gather(buf)
            mark("words")
            if a is None:
                return
    # the assembly runs on the band stream itself (after the root's tables on
    # its own stream: mij_batch_set_stream orders the switch), so the word
    # move, the assembly and the next step's K1 follow each other in one
    # queue -- a cross-queue wait costs ~13 us each way on config 4
    # (profiles/r06/probe/c4_trace/); the tensors it reads are freed on that
    # stream too
    if _ASSEMBLE_OWN_STREAM:
        a.wait_stream(s)
        with torch.cuda.stream(a):
            _assemble(frame_batch, emit, n, allbits, allrec if emit == "bands" else None, world, gathered, stride)
        s.wait_stream(a)
    else:
        frame_batch.set_stream(band.stream_ptr())
        try:
            _assemble(frame_batch, emit, n, allbits, allrec if emit == "bands" else None, world, gathered, stride)
        finally:
            frame_batch.set_stream(0)
    mark("assemble")


def _assemble(frame_batch, emit, n, allbits, allrec, world, gathered, stride):
    if emit == "bands":
        frame_batch.assemble_stuffed_async(n, allrec.data_ptr(), world, gathered.data_ptr(), stride)
    else:
        frame_batch.assemble_async(n, allbits.data_ptr(), world, gathered.data_ptr(), stride)
