"""Offline count (not a test): where the token K1's luma hazards fall on a
config-3 frame -- coefficients whose fast-path interval [N' - E, N' + E]
straddles a truncation boundary (the integer rule) and go to
the FP64 replay.  Restates fill_tables' prescaled rows (mij_api.hip) in numpy;
the luma plane uses the FP64 colour formula without the exception table (a
count, not a parity check).  DESIGN.md §7 quotes its output: at Q=90, 88% of
the hazards sit at (u, v) in {(0,4), (4,0), (4,4)}, the positions whose DCT
weights are all +-1/2 (cos(pi/4)^2, or cos(pi/4) times the 1/sqrt(2) of
frequency 0): F = S / 8 for an integer S, so F / q is either an exact
integer there -- where only the reference's FP64 rounding decides, at any
precision of N' -- or at least 1 / (8 q) away from one.
python3 tests/hazard_positions.py [Q ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle as O  # noqa: E402
import recipes  # noqa: E402

ZZ = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,
      7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
      39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


def luma_blocks(f: int = 0) -> np.ndarray:
    bgr = recipes.config3_frame(f).astype(np.float64)
    y = np.floor(0.299 * bgr[..., 2] + 0.587 * bgr[..., 1] + 0.114 * bgr[..., 0]).astype(np.int64)
    h, w = y.shape
    return y.reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64) - 128


def hazards(X: np.ndarray, q: int) -> np.ndarray:
    lq = np.asarray(O.quality_tables(q)[0]).reshape(-1)
    qz = np.array([lq[ZZ[z]] for z in range(64)])
    sg = []
    for g in range(4):
        qmin = min(int(qz[z]) for z in range(16 * g, 16 * g + 16) if z)
        s = 0
        while (2 << s) <= qmin:
            s += 1
        sg.append(s)
    cosd = np.array([np.cos((2 * (i // 8) + 1) * (i % 8) * np.pi / 16) for i in range(64)])
    Wm = np.zeros((64, 64), np.int64)
    for z in range(1, 64):
        v, u = ZZ[z] >> 3, ZZ[z] & 7
        for p in range(64):
            k = cosd[(p >> 3) * 8 + v] * cosd[(p & 7) * 8 + u]
            k *= np.sqrt(0.5) if u == 0 else 1.0
            k *= np.sqrt(0.5) if v == 0 else 1.0
            Wm[z, p] = int(np.round(k * 2.0 ** (19 + sg[z >> 4]) / qz[z]))
    N = X @ Wm.T
    E = (np.abs(X).sum(1) >> 1) + 1
    kq = np.array([21 + sg[z >> 4] for z in range(64)])
    a = np.where(N < 0, -N - 1, N)
    hz = ((a + E[:, None] + 1) >> kq) != (np.maximum(a - E[:, None], 0) >> kq)
    hz[:, 0] = False
    return hz


if __name__ == "__main__":
    X = luma_blocks(0)
    for q in [int(a) for a in sys.argv[1:]] or [50, 90]:
        cnt = hazards(X, q).sum(0)
        tot = int(cnt.sum())
        rat = sum(int(cnt[z]) for z in range(64) if (ZZ[z] & 3) == 0 and (ZZ[z] >> 3) & 3 == 0)
        top = ", ".join(f"(u,v)=({ZZ[z] & 7},{ZZ[z] >> 3}): {int(cnt[z])}" for z in np.argsort(-cnt)[:4])
        print(f"Q={q} luma hazards, config-3 frame 0: {tot}; at u, v in {{0, 4}}: {rat} ({rat / max(tot, 1):.0%}); {top}")
