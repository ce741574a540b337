"""scripts/stress_repeat.py -- determinism check across the batch-size
paths: each case encodes the same batch N times and compares every
repetition's JFIF bytes with the first (small batches: seam fixes inside
k_emit_scan, DC tables inside the segment-DC launch, one K1 workgroup per
CU; large: k_seam_fix, the DC-table launch, the wide pack window at Q=90).
python3 scripts/stress_repeat.py [N]"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "jpeg-encoder-decoder_amd"))
import mijpeg  # noqa: E402
import recipes  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
f4k = [recipes.config3_frame(i) for i in range(4)] + [recipes.config3_uniform(i) for i in range(2)]
small = recipes.standin_1920x1280_rgb()[:, :, ::-1].copy()
cases = [
    ("1 x 1920x1280 Q=50", 1920, 1280, 50, [small]),
    ("4 x 4K Q=50 (2 noise)", 3840, 2160, 50, [f4k[0], f4k[4], f4k[1], f4k[5]]),
    ("16 x 4K Q=50", 3840, 2160, 50, [f4k[i % 6] for i in range(16)]),
    ("16 x 4K Q=90", 3840, 2160, 90, [f4k[i % 6] for i in range(16)]),
    ("96 x 4K Q=50", 3840, 2160, 50, [f4k[i % 6] for i in range(96)]),
]
bad = 0
for name, w, h, q, frames in cases:
    b = mijpeg.Batch(w, h, len(frames), q)
    try:
        b.upload(np.stack(frames))
        ref = None
        nb = 0
        for _ in range(n):
            b.encode(len(frames))
            hs = [hashlib.sha256(b.output(i)).hexdigest()[:16] for i in range(len(frames))]
            if ref is None:
                ref = hs
            elif hs != ref:
                nb += 1
        print(f"{name}: {n} encodes, {nb} differ", flush=True)
        bad += nb
    finally:
        b.close()
sys.exit(1 if bad else 0)
