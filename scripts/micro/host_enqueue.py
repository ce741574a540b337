"""Is a one-frame encode step bound by the host's launch submissions?
Times N back-to-back encode(1) calls without a sync (the enqueue cost alone)
and with the final sync (the step), for a 1920x1280 frame.  Usage:
python3 scripts/micro/host_enqueue.py [N]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jpeg-encoder-decoder_amd"))
import numpy as np
import mijpeg

N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
W, H = 1920, 1280
rng = np.random.default_rng(0)
frame = (rng.integers(0, 256, (H, W, 3), dtype=np.uint8) // 4 + np.arange(W, dtype=np.uint8)[None, :, None] // 8)
b = mijpeg.Batch(W, H, 1, 50, device=0)
b.set_timing(False)
b.upload(frame, first=0)
for _ in range(20):
    b.encode(1)
b.sync()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(N):
        b.encode(1)
    t1 = time.perf_counter()
    b.sync()
    t2 = time.perf_counter()
    print(f"enqueue {1e6 * (t1 - t0) / N:.1f} us/step, step {1e6 * (t2 - t0) / N:.1f} us/step", flush=True)
