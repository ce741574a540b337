"""Debug: encode a config-3 batch and list every slot that differs from the oracle."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, p) for p in ("jpeg-encoder-decoder_amd", "oracle", "tests")]
import numpy as np, mijpeg, oracle as O, recipes
F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
D = int(sys.argv[2]) if len(sys.argv) > 2 else 16
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
frames = [recipes.config3_frame(f) for f in range(D)]
want = [O.cref_encode(fr) for fr in frames]
b = mijpeg.Batch(3840, 2160, F, 50)
for i in range(F):
    b.upload(frames[i % D], first=i)
for r in range(reps):
    b.encode(F)
    b.sync()
    bad = []
    for i in range(F):
        g, w = b.output(i), want[i % D]
        if g != w:
            n = min(len(g), len(w))
            fd = next((k for k in range(n) if g[k] != w[k]), n)
            bad.append((i, len(g), len(w), fd))
    print(f"rep {r}: {len(bad)} bad", bad[:12], flush=True)
