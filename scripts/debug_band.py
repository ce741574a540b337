"""debug: the device-resident band protocol exactly as tests/test_bands.py
drives it (worlds in argv order, one process), then the host protocol's
intermediate values for comparison."""
import os, sys
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "jpeg-encoder-decoder_amd"), os.path.join(R, "tests"), os.path.join(R, "oracle")]
import numpy as np
import torch
import mijpeg, sharding, recipes
import oracle as O
torch.cuda.set_device(0)
frames = np.stack([recipes.config3_frame(5, 320, 480), recipes.noise(320, 480, 9), recipes.config3_frame(6, 320, 480)])
n, H, W = frames.shape[:3]
want = [O.cref_encode(f) for f in frames]
dev = "cuda:0"
for world in [int(a) for a in sys.argv[1:]]:
    bands = []
    for r in range(world):
        r0, rows = sharding.band_rows(H, world, r)
        b = mijpeg.Batch(W, rows, n); b.upload(np.ascontiguousarray(frames[:, r0:r0 + rows])); bands.append(b)
    last = [torch.empty((n, 4), dtype=torch.int16, device=dev) for _ in bands]
    for b, l in zip(bands, last):
        b.band_analyze_async(n, l.data_ptr()); b.sync()
    hist = [torch.empty((n, 4, 257), dtype=torch.int32, device=dev) for _ in bands]
    zero = torch.zeros((n, 4), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()  # (torch zeroes it on its own stream)
    for r, b in enumerate(bands):
        b.band_histograms_async(n, (zero if r == 0 else last[r - 1]).data_ptr(), hist[r].data_ptr()); b.sync()
    ghist = torch.stack(hist).sum(0, dtype=torch.int32).contiguous(); torch.cuda.synchronize()
    bits = [torch.empty((n, 3), dtype=torch.int64, device=dev) for _ in bands]
    for b, t in zip(bands, bits):
        b.band_tables_async(n, ghist.data_ptr(), t.data_ptr()); b.sync()
    allbits = torch.stack(bits).contiguous(); torch.cuda.synchronize()
    nw = [torch.empty(1, dtype=torch.int64, device=dev) for _ in bands]
    for r, b in enumerate(bands):
        b.band_pack_async(n, allbits.data_ptr(), world, r, nw[r].data_ptr()); b.sync()
    stride = max(int(x.item()) for x in nw)
    g = torch.zeros((world, stride), dtype=torch.int32, device=dev); torch.cuda.synchronize()
    for r, b in enumerate(bands):
        b.band_words_async(n, g[r].data_ptr()); b.sync()
    full = mijpeg.Batch(W, H, n, assembler=True)
    full.assemble_async(n, ghist.data_ptr(), allbits.data_ptr(), world, g.data_ptr(), stride); full.sync()
    out = [full.output(f) for f in range(n)]
    ok = [o == w for o, w in zip(out, want)]
    print(world, "dev ok", ok, [len(o) for o in out], [len(w) for w in want], flush=True)
    if not all(ok):
        hb = []
        for r in range(world):
            r0, rows = sharding.band_rows(H, world, r)
            b = mijpeg.Batch(W, rows, n); b.upload(np.ascontiguousarray(frames[:, r0:r0 + rows])); hb.append(b)
        hl = [b.band_analyze(n) for b in hb]
        hh = [b.band_histograms(n, np.zeros((n, 3), np.int16) if r == 0 else hl[r - 1]) for r, b in enumerate(hb)]
        hg = np.sum(np.stack(hh).astype(np.int64), axis=0).astype(np.uint32)
        hbits = np.stack([b.band_tables(n, hg) for b in hb]).astype(np.uint64)
        offs = np.concatenate([np.zeros((1, n, 3), np.uint64), np.cumsum(hbits, axis=0)[:-1]])
        hnw = [b.band_pack(n, offs[r]) for r, b in enumerate(hb)]
        hw = []
        for r, b in enumerate(hb):
            tot = int(np.sum(hnw[r])); d = np.zeros(max(tot, 1), np.uint32); b.band_words_all(n, dst=d); hw.append(d[:tot])
        for r in range(world):
            print("last", r, np.array_equal(last[r].cpu().numpy()[:, :3], hl[r]))
            print("hist", r, np.array_equal(hist[r].cpu().numpy().view(np.uint32), hh[r].reshape(n, 4, 257)))
            print("bits", r, bits[r].cpu().numpy().tolist(), hbits[r].tolist())
            print("nw", r, int(nw[r].item()), int(np.sum(hnw[r])), hnw[r].tolist())
            gn = g.cpu().numpy().view(np.uint32)
            k = len(hw[r]); eq = np.array_equal(gn[r, :k], hw[r])
            print("words", r, eq, "" if eq else np.nonzero(gn[r, :k] != hw[r])[0][:10])
        for b in hb:
            b.close()
    bands[-1].encode(n)
    for b in bands:
        b.close()
    full.close()
