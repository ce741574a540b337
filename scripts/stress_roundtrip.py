"""scripts/stress_roundtrip.py -- repeat tests/test_decode.py's full-size
round trip (decode(GPU encode) == the encoder's own coefficients on a
config-3 frame and a uniform-noise frame) N times in one process, and
compare every repetition's JFIF bytes with the first; prints mismatches.
python3 scripts/stress_roundtrip.py [N]"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "jpeg-encoder-decoder_amd"))
import mijpeg  # noqa: E402
import recipes  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
frames = np.stack([recipes.config3_frame(0), recipes.config3_uniform(1)])
b = mijpeg.Batch(3840, 2160, 2, 50, keep_coefs=True)
d = mijpeg.Decoder(3840, 2160, 2)
ref = None
bad = 0
try:
    b.upload(frames)
    for it in range(n):
        b.encode(2)
        streams = [b.output(i) for i in range(2)]
        h = [hashlib.sha256(s).hexdigest()[:16] for s in streams]
        if ref is None:
            ref = h
        d.decode(streams)
        ok = all((g == w).all() for i in range(2) for g, w in zip(d.coefs(i), b.coefs(i, diffed=True)))
        if h != ref or not ok:
            bad += 1
            print(f"iteration {it}: sha {h} (first {ref}), round trip {'ok' if ok else 'MISMATCH'}", flush=True)
    print(f"{n} iterations, {bad} bad", flush=True)
finally:
    b.close()
    d.close()
sys.exit(1 if bad else 0)
