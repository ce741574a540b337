"""Offline count (not a test): iterations of the token K1's AC-token loop per
luma N-tile for the wave's busiest lane, on the oracle's coefficients of a
config-3 frame (16 consecutive blocks per N-tile), for the current lane
partition (lane (g, b): zigzag positions z = g mod 4 of block b, the low and
the high 32 positions in two loops) against a perfectly balanced split and a
block-aligned contiguous split (lanes per block proportional to its tokens).
DESIGN.md §7 quotes its output.  python3 tests/acloop_sim.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle as O  # noqa: E402
import recipes  # noqa: E402

W, H = 3840, 2160


def counts(P):
    B = P.reshape(-1, 64)
    nz = B != 0
    nz[:, 0] = False  # the DC is not an AC token
    nt = B.shape[0] // 16
    nzt = nz[: nt * 16].reshape(nt, 16, 64)
    nac = nzt.sum(2)
    T = nac.sum(1)
    z = np.arange(64)
    lo = np.stack([(nzt[:, :, :32] & (z[:32] % 4 == g)).sum(2) for g in range(4)], 2).max((1, 2))
    hi = np.stack([(nzt[:, :, 32:] & (z[32:] % 4 == g)).sum(2) for g in range(4)], 2).max((1, 2))
    ideal = -(-T // 64)
    qa = np.maximum(ideal, 1)  # smallest q with sum ceil(nac / q) <= 64
    for _ in range(64):
        bad = (-(-nac // qa[:, None])).sum(1) > 64
        if not bad.any():
            break
        qa = qa + bad
    qa = np.where(T == 0, 0, qa)
    return T.mean(), (lo + hi).mean(), ideal.mean(), qa.mean()


if __name__ == "__main__":
    for q in (50, 90):
        Y = O.cref_stages(recipes.config3_frame(0, H, W), q)[0]
        t, cur, ideal, blk = counts(Y)
        print(f"Q={q} luma: {t:.1f} AC tokens per N-tile; busiest-lane iterations: current {cur:.2f}, "
              f"balanced {ideal:.2f}, block-aligned contiguous {blk:.2f}")
