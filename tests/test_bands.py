"""One large frame split into MCU-row bands:
each band is encoded by the library as its own frame, the bands exchange
their last DCs, histograms, bit counts and packed words, and one side
assembles the JFIF.  The result must be the reference's bytes for the whole
frame.  GPU tests drive the bands in one process (the exchanges done in
Python) and over two processes with torch.distributed (gloo, both ranks on
GPU 0)."""
import os
import socket

import numpy as np
import pytest

import sharding

pytestmark = pytest.mark.gpu


def encode_banded_local(frames: np.ndarray, world: int, quality: int = 50, per_scan: bool = False):
    """All bands of n frames in one process; mirrors sharding.encode_banded
    (per_scan: the per-(frame, scan) calls mij_band_words / mij_assemble_words
    on a full batch instead of the one-call exchange on an assembler)."""
    import mijpeg
    n, H, W = frames.shape[:3]
    bands = []
    for r in range(world):
        r0, rows = sharding.band_rows(H, world, r)
        b = mijpeg.Batch(W, rows, n, quality)
        b.upload(np.ascontiguousarray(frames[:, r0:r0 + rows]))
        bands.append(b)
    lasts = [b.band_analyze(n) for b in bands]
    hists = [b.band_histograms(n, np.zeros((n, 3), np.int16) if r == 0 else lasts[r - 1])
             for r, b in enumerate(bands)]
    ghist = np.sum(np.stack(hists).astype(np.int64), axis=0).astype(np.uint32)
    bits = np.stack([b.band_tables(n, ghist) for b in bands]).astype(np.uint64)
    offs = np.concatenate([np.zeros((1, n, 3), np.uint64), np.cumsum(bits, axis=0)[:-1]])
    full = mijpeg.Batch(W, H, n, quality, assembler=not per_scan)
    full.assemble_begin(n, ghist)
    if per_scan:
        for r, b in enumerate(bands):
            nw = b.band_pack(n, offs[r])
            for f in range(n):
                for c in range(3):
                    words = b.band_words(f, c, int(nw[f, c]))
                    full.assemble_words(f, c, int(offs[r][f, c]) >> 5, words)
    else:
        allnw, maxw, pieces = sharding.band_pieces(bits, offs)
        gathered = np.zeros((world, max(maxw, 1)), np.uint32)
        for r, b in enumerate(bands):
            assert np.array_equal(b.band_pack(n, offs[r]), allnw[r])
            b.band_words_all(n, dst=gathered[r])
        full.assemble_pieces(pieces, src=gathered)
    full.assemble_end(n, bits.sum(axis=0))
    out = [full.output(f) for f in range(n)]
    for b in bands:
        b.close()
    full.close()
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_bands_match_reference(world):
    import oracle as O
    import recipes
    frames = np.stack([recipes.config3_frame(0, 320, 480), recipes.noise(320, 480, 7)])
    got = encode_banded_local(frames, world)
    for f in range(2):
        assert got[f] == O.cref_encode(frames[f]), f"world {world} frame {f}"


def test_bands_one_mcu_row_each_and_quality():
    import oracle as O
    import recipes
    frame = recipes.config3_frame(3, 64, 640)[None]  # 4 MCU rows -> 4 one-row bands
    assert encode_banded_local(frame, 4, 75)[0] == O.cref_encode(frame[0], 75)
    assert encode_banded_local(frame, 4, 75, per_scan=True)[0] == O.cref_encode(frame[0], 75)


def test_bands_config4_shape_two_bands():
    """A 7680x4320 frame (config-4 shape) in two bands == the one-frame encode."""
    import mijpeg
    import recipes
    frame = recipes.config4_frame(0)[None]
    got = encode_banded_local(frame, 2)[0]
    b = mijpeg.Batch(7680, 4320, 1)
    b.upload(frame)
    b.encode(1)
    assert got == b.output(0)
    b.close()


def _sha(b: bytes) -> str:
    import hashlib
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("f", [0, 1])
def test_config4_frames_match_reference_goldens(f, manifest):
    """SURVEY §8(d) config 4 at full size: the 7680x4320 frames encoded whole
    and in 2, 4 and 8 MCU-row bands give the reference's bytes (sha256 of the
    reference build's output, tests/golden/manifest.json, oracle/gen_golden.py)."""
    import mijpeg
    import recipes
    want = manifest[f"config4_frame{f}"]
    frame = recipes.config4_frame(f)[None]
    b = mijpeg.Batch(7680, 4320, 1)
    b.upload(frame)
    b.encode(1)
    got = b.output(0)
    b.close()
    assert (len(got), _sha(got)) == (want["jpg_len"], want["jpg_sha256"])
    for world in (2, 4, 8):
        got = encode_banded_local(frame, world)[0]
        assert (len(got), _sha(got)) == (want["jpg_len"], want["jpg_sha256"]), f"{world} bands"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import mijpeg
    import recipes
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = np.stack([recipes.config3_frame(1, 320, 480), recipes.noise(320, 480, 9)])
        H, W = frames.shape[1:3]
        r0, rows = sharding.band_rows(H, world, rank)
        band = mijpeg.Batch(W, rows, 2)
        band.upload(np.ascontiguousarray(frames[:, r0:r0 + rows]))
        full = mijpeg.Batch(W, H, 2, assembler=True) if rank == 0 else None
        sharding.encode_banded(band, 2, sharding.TorchExchange(dist, "cpu"), full)
        if rank == 0:
            q.put([full.output(f) for f in range(2)])
    finally:
        dist.destroy_process_group()


def test_two_process_banded_encode_gloo():
    import multiprocessing as mp
    import oracle as O
    import recipes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    frames = [recipes.config3_frame(1, 320, 480), recipes.noise(320, 480, 9)]
    assert outs == [O.cref_encode(f) for f in frames]


def _rank_full(rank, world, port, q):
    """One rank of a two-process gloo band encode of config-4 frame 0 at full
    size (7680x4320): its band only, host exchanges over gloo; rank 0
    assembles and reports (length, sha256)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import hashlib
    import torch.distributed as dist
    import mijpeg
    import recipes
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frame = recipes.config4_frame(0)[None]
        H, W = frame.shape[1:3]
        r0, rows = sharding.band_rows(H, world, rank)
        band = mijpeg.Batch(W, rows, 1)
        band.upload(np.ascontiguousarray(frame[:, r0:r0 + rows]))
        full = mijpeg.Batch(W, H, 1, assembler=True) if rank == 0 else None
        sharding.encode_banded(band, 1, sharding.TorchExchange(dist, "cpu"), full)
        if rank == 0:
            out = full.output(0)
            q.put((len(out), hashlib.sha256(out).hexdigest()))
            full.close()
        band.close()
    finally:
        dist.destroy_process_group()


def test_two_process_banded_encode_gloo_full_size(manifest):
    """SURVEY §8(e) rehearsal at config 4's size: two processes, one band
    each, gloo exchanges; the assembled frame is the reference's bytes for
    config4_frame0 (tests/golden/manifest.json)."""
    import multiprocessing as mp
    want = manifest["config4_frame0"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_full, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == (want["jpg_len"], want["jpg_sha256"])


def _nccl_rank(port, q):
    # torch's HIP runtime first (as bench.py's dist_setup does): the bundled
    # runtime of torch does not initialise after the library's in one process
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    import mijpeg
    import recipes
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        frames = np.stack([recipes.config3_frame(2, 320, 480), recipes.noise(320, 480, 4)])
        band = mijpeg.Batch(480, 320, 2)
        band.upload(frames)
        full = mijpeg.Batch(480, 320, 2, assembler=True)
        xch = sharding.TorchExchange(dist, "cuda:0")
        outs = []
        for _ in range(2):  # a second step reuses torch's freed blocks
            sharding.encode_banded(band, 2, xch, full)
            outs.append([full.output(f) for f in range(2)])
        try:
            full.encode(1)
            rejected = False
        except mijpeg.MijError:
            rejected = True
        band.close()
        full.close()
        q.put((outs, rejected))
    finally:
        dist.destroy_process_group()


def test_one_rank_nccl_exchange_device_branch():
    """encode_banded over a one-rank nccl (RCCL) process group: the device
    branch -- band words copied into a device tensor in one call, gathered by
    RCCL, OR-ed into an assembler's scans from device memory in one launch --
    against the reference, in a fresh process."""
    import multiprocessing as mp
    import oracle as O
    import recipes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_rank, args=(_free_port(), q))
    p.start()
    outs, rejected = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    want = [O.cref_encode(recipes.config3_frame(2, 320, 480)), O.cref_encode(recipes.noise(320, 480, 4))]
    assert outs == [want, want]
    assert rejected, "an assembler batch must refuse to encode"


def _fp_rank(rank, world, port, q):
    """frame-parallel config-3 path on GPU 0: this rank's shard of the frames
    through the HIP library, the timing reduction, the blobs to rank 0"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import mijpeg
    import recipes
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = [recipes.config3_frame(f, 160, 256) for f in range(5)]
        mine = sharding.frame_range(len(frames), world, rank)
        b = mijpeg.Batch(256, 160, len(mine))
        b.upload(np.stack([frames[i] for i in mine]))
        b.encode(len(mine))
        blobs = [b.output(i) for i in range(len(mine))]
        b.close()
        el, units = sharding.reduce_timing(1.0 + rank, len(mine), dist, "cpu")
        got = [None] * world
        dist.all_gather_object(got, blobs)
        if rank == 0:
            q.put((el, units, [x for g in got for x in g]))
    finally:
        dist.destroy_process_group()


def test_two_process_frame_parallel_hip_gloo():
    import multiprocessing as mp
    import oracle as O
    import recipes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fp_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    el, units, blobs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert (el, units) == (2.0, 5)
    assert blobs == [O.cref_encode(recipes.config3_frame(f, 160, 256)) for f in range(5)]


# ---------------------------------------------------------------------------
# the device-resident protocol (mij_band_*_async, sharding.encode_banded_dev)
# ---------------------------------------------------------------------------

def _dev_bands(port, q):
    """In a fresh process (torch's HIP runtime first): W bands of the same
    frames in one process through the async calls, the exchanges done with
    torch ops on device tensors (full syncs between the steps), for W = 1..4;
    then encode_banded_dev itself over a one-rank nccl group (ExternalStream
    on the band batch's stream, RCCL collectives) twice in a row."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    import mijpeg
    import recipes
    dev = "cuda:0"
    frames = np.stack([recipes.config3_frame(5, 320, 480), recipes.noise(320, 480, 9),
                       recipes.config3_frame(6, 320, 480)])
    n, H, W = frames.shape[:3]
    res = {}

    def protocol(world, shrink=0, emit="root"):
        bands = []
        for r in range(world):
            r0, rows = sharding.band_rows(H, world, r)
            b = mijpeg.Batch(W, rows, n)
            b.upload(np.ascontiguousarray(frames[:, r0:r0 + rows]))
            bands.append(b)
        last = [torch.empty((n, 4), dtype=torch.int16, device=dev) for _ in bands]
        for b, l in zip(bands, last):
            b.band_analyze_async(n, l.data_ptr())
            b.sync()
        hist = [torch.empty((n, 4, 257), dtype=torch.int32, device=dev) for _ in bands]
        for r, b in enumerate(bands):
            b.band_histograms_async(n, 0 if r == 0 else last[r - 1].data_ptr(), hist[r].data_ptr())
            b.sync()
        ghist = torch.stack(hist).sum(0, dtype=torch.int32).contiguous()
        torch.cuda.synchronize()
        full = mijpeg.Batch(W, H, n, assembler=True)
        full.assemble_tables_async(n, ghist.data_ptr())
        bound = [torch.empty(1, dtype=torch.int64, device=dev) for _ in bands]
        bits = [torch.empty(3 * n + 1, dtype=torch.int64, device=dev) for _ in bands]
        for b, d, t in zip(bands, bound, bits):
            b.band_tables_async(n, ghist.data_ptr(), d.data_ptr())
            b.band_pack_async(n, t.data_ptr())
            b.sync()
        allbits = torch.stack(bits).contiguous()
        # the bounds hold (at most 3 words per frame above the words)
        for d, t in zip(bound, bits):
            assert 0 <= int(d) - int(t[3 * n]) <= 3 * n
        if emit == "bands":  # distributed emission: each band stuffs its interiors
            cap = 8 * int(torch.cat(bound).max())
            bufs = [torch.zeros(cap + 48, dtype=torch.uint8, device=dev) for _ in bands]
            recs = [torch.empty(n * 3 * 4, dtype=torch.int64, device=dev) for _ in bands]
            tots = [torch.empty(1, dtype=torch.int64, device=dev) for _ in bands]
            torch.cuda.synchronize()
            for r, b in enumerate(bands):
                b.band_stuff_async(n, allbits.data_ptr(), world, r, recs[r].data_ptr(), tots[r].data_ptr(),
                                   bufs[r].data_ptr(), cap)
                b.sync()
            stride = (int(torch.cat(tots).max()) + 31) & ~15
            gathered = torch.stack([x[:stride] for x in bufs]).contiguous()
            allrec = torch.stack(recs).contiguous()
            # every band's words are consumed: zero again for the next pack
            full.assemble_stuffed_async(n, allrec.data_ptr(), world, gathered.data_ptr(), stride)
            full.sync()
        else:
            stride = int(torch.cat(bound).max()) - shrink
            gathered = torch.zeros((world, stride), dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            for r, b in enumerate(bands):
                b.band_words_async(n, gathered[r].data_ptr(), stride)
                b.sync()
            full.assemble_async(n, allbits.data_ptr(), world, gathered.data_ptr(), stride)
            full.sync()
        out = []
        for f in range(n):
            try:
                out.append(full.output(f))
            except mijpeg.MijError as e:
                out.append(str(e))
        # the band batches encode whole frames correctly afterwards
        bands[-1].encode(n)
        after = bands[-1].output(0)
        for b in bands:
            b.close()
        full.close()
        return out, after

    for world in (1, 2, 3, 4):
        res[world], res[(world, "after")] = protocol(world)
    # distributed emission, up to one MCU row per band (20 bands of 16 rows:
    # seam bytes between most bands, bands of a few bits per chroma scan)
    for world in (1, 2, 3, 4, 7, 20):
        res[(world, "bands")], res[(world, "bands_after")] = protocol(world, emit="bands")
    # a word buffer shorter than a band's words: every frame fails, nothing
    # is written past the buffer
    res["short"], _ = protocol(2, shrink=4000)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        band = mijpeg.Batch(W, H, n)
        band.upload(frames)
        full = mijpeg.Batch(W, H, n, assembler=True)
        xch = sharding.DeviceExchange(dist, dev)
        outs = []
        for _ in range(2):
            ev = []
            sharding.encode_banded_dev(band, n, xch, full, events=ev)
            full.sync()
            outs.append([full.output(f) for f in range(n)])
        res["nccl"] = outs
        res["phases"] = [name for name, _ in ev]
        band.close()
        full.close()
    finally:
        dist.destroy_process_group()
    q.put(res)


def test_device_resident_band_protocol():
    """mij_band_*_async for 1-4 bands in one process and encode_banded_dev
    over a one-rank nccl group: the reference's bytes for whole frames
    (/root/reference/main/encoder.c through the oracle), with every exchanged
    value kept in device memory."""
    import multiprocessing as mp
    import oracle as O
    import recipes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_dev_bands, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=600)
    p.join(timeout=120)
    assert p.exitcode == 0
    frames = [recipes.config3_frame(5, 320, 480), recipes.noise(320, 480, 9), recipes.config3_frame(6, 320, 480)]
    want = [O.cref_encode(f) for f in frames]
    for world in (1, 2, 3, 4):
        assert res[world] == want, f"{world} bands"
        # a band batch left by the protocol encodes its own rows correctly
        r0, rows = sharding.band_rows(320, world, world - 1)
        assert res[(world, "after")] == O.cref_encode(np.ascontiguousarray(frames[0][r0:r0 + rows]))
    for world in (1, 2, 3, 4, 7, 20):
        assert res[(world, "bands")] == want, f"{world} bands, distributed emission"
        r0, rows = sharding.band_rows(320, world, world - 1)
        assert res[(world, "bands_after")] == O.cref_encode(np.ascontiguousarray(frames[0][r0:r0 + rows]))
    assert all(isinstance(o, str) for o in res["short"]), res["short"]
    assert res["nccl"] == [want, want]
    assert res["phases"] == ["start", "analyze", "histograms", "pack", "words", "assemble"]


# ---------------------------------------------------------------------------
# encode_banded_dev with world > 1: several processes share GPU 0, the
# collectives of the device protocol staged through host memory over gloo
# (sharding.StagedExchange) -- the indexing the RCCL run uses at N > 1
# (the previous band's last DCs, the word bounds, the [world, 3n + 1] bits,
# the gathered [world, stride] words) runs exactly as there
# ---------------------------------------------------------------------------

def _staged_rank(rank, world, port, q, spec, emit="root"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import hashlib
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)  # torch's HIP runtime before the library's
    import mijpeg
    import recipes
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        W, H, kind = spec
        if kind == "small":
            frames = np.stack([recipes.config3_frame(7, H, W), recipes.noise(H, W, 12),
                               recipes.config3_frame(8, H, W)])
        else:
            frames = recipes.config4_frame(0)[None]
        n = frames.shape[0]
        r0, rows = sharding.band_rows(H, world, rank)
        band = mijpeg.Batch(W, rows, n)
        band.upload(np.ascontiguousarray(frames[:, r0:r0 + rows]))
        full = mijpeg.Batch(W, H, n, assembler=True) if rank == 0 else None
        xch = sharding.StagedExchange(dist, "cuda:0")
        outs = []
        for _ in range(2):  # twice: the second step reuses every buffer
            sharding.encode_banded_dev(band, n, xch, full, emit=emit)
            band.sync()
            if full is not None:
                full.sync()
                got = [full.output(f) for f in range(n)]
                outs.append(got if kind == "small" else
                            [(len(g), hashlib.sha256(g).hexdigest()) for g in got])
            dist.barrier()
        band.close()
        if full is not None:
            full.close()
            q.put(outs)
    finally:
        dist.destroy_process_group()


def _run_staged(world, spec, emit="root"):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_staged_rank, args=(r, world, port, q, spec, emit)) for r in range(world)]
    for p in procs:
        p.start()
    # poll: a rank that fails leaves the others blocked in a collective, so
    # stop at the first non-zero exit instead of waiting out the queue
    import queue
    import time
    t_end = time.time() + 150
    outs = None
    while outs is None:
        try:
            outs = q.get(timeout=2)
        except queue.Empty:
            bad = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if bad or time.time() > t_end:
                for p in procs:
                    p.kill()
                raise AssertionError(f"staged ranks failed (exit codes {[p.exitcode for p in procs]})")
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return outs


@pytest.mark.parametrize("emit", ["root", "bands"])
@pytest.mark.parametrize("world", [2, 3])
def test_device_protocol_multi_rank_staged(world, emit):
    """encode_banded_dev over 2 and 3 ranks (processes on one GPU, gloo
    collectives staged through host memory): each band's first DC predicted
    from the previous rank's last DC, histograms summed, every band packed
    from bit 0 and shifted into place by the root -- the reference's bytes,
    twice in a row."""
    import oracle as O
    import recipes
    W, H = 480, 320
    outs = _run_staged(world, (W, H, "small"), emit)
    want = [O.cref_encode(recipes.config3_frame(7, H, W)), O.cref_encode(recipes.noise(H, W, 12)),
            O.cref_encode(recipes.config3_frame(8, H, W))]
    assert outs == [want, want]


@pytest.mark.parametrize("emit", ["root", "bands"])
def test_device_protocol_two_ranks_full_size(manifest, emit):
    """The same at config 4's size: 7680x4320 frame 0 in two bands, against
    the reference build's sha256 (tests/golden/manifest.json), with the
    root's emission and with the distributed one."""
    want = manifest["config4_frame0"]
    outs = _run_staged(2, (7680, 4320, "full"), emit)
    assert outs == [[(want["jpg_len"], want["jpg_sha256"])]] * 2
