"""Deterministic synthetic frames shared by the tests, the golden-fixture
generator (oracle/gen_golden.py) and bench.py.  All frames are BGR888
(the reference's input convention, encoder.c:133) as HxWx3 uint8 arrays.

Recipes follow SURVEY.md §8(d):
  * stand-in 1920x1280: sample_640x640 tiled 3 wide x 2 high (the real
    images/sample_1920x1280.ppm is missing from the reference mount);
  * config 3 frame f: top-left 2160x3840 crop of tile(sample_640x640, 4x6),
    rolled by (17f, 29f) px, plus default_rng(f).integers(-4, 5) noise;
  * config 3 high-entropy variant: default_rng(1000+f).integers(0, 256).
"""
from __future__ import annotations

import os

import numpy as np

from ppm import read_ppm, rgb_to_bgr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_cache: dict = {}


def sample(name: str) -> np.ndarray:
    """RGB array of a committed reference image (tests/golden/*.ppm[.gz])."""
    if name not in _cache:
        for suffix in (".ppm", ".ppm.gz"):
            p = os.path.join(GOLDEN, name + suffix)
            if os.path.exists(p):
                _cache[name] = read_ppm(p)
                break
        else:
            raise FileNotFoundError(name)
    return _cache[name]


def standin_1920x1280_rgb() -> np.ndarray:
    return np.tile(sample("sample_640x640"), (2, 3, 1))


def config3_frame(f: int, h: int = 2160, w: int = 3840) -> np.ndarray:
    """BGR natural-statistics frame f of the 3840x2160 batch."""
    base = np.tile(sample("sample_640x640"), (4, 6, 1))[:h, :w]
    base = np.roll(base, (17 * f, 29 * f), axis=(0, 1)).astype(np.int16)
    noise = np.random.default_rng(f).integers(-4, 5, size=base.shape, dtype=np.int16)
    return rgb_to_bgr(np.clip(base + noise, 0, 255).astype(np.uint8))


def config3_uniform(f: int, h: int = 2160, w: int = 3840) -> np.ndarray:
    rng = np.random.default_rng(1000 + f)
    return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def config4_frame(f: int, h: int = 4320, w: int = 7680) -> np.ndarray:
    """7680x4320 stream frame: the config-3 recipe with tile(7 x 12)."""
    base = np.tile(sample("sample_640x640"), (7, 12, 1))[:h, :w]
    base = np.roll(base, (17 * f, 29 * f), axis=(0, 1)).astype(np.int16)
    noise = np.random.default_rng(f).integers(-4, 5, size=base.shape, dtype=np.int16)
    return rgb_to_bgr(np.clip(base + noise, 0, 255).astype(np.uint8))


# ---- adversarial exactness suite ----------------------

def gray_levels() -> np.ndarray:
    """256x256 frame: MCU i (raster) is flat gray level i (all 256 levels)."""
    lv = np.arange(256, dtype=np.uint8).reshape(16, 16)
    g = np.kron(lv, np.ones((16, 16), np.uint8))
    return np.repeat(g[..., None], 3, axis=2)


def flat_colours(seed: int = 1, mcus: int = 16) -> np.ndarray:
    rng = np.random.default_rng(seed)
    c = rng.integers(0, 256, size=(mcus, mcus, 3), dtype=np.uint8)
    return np.kron(c, np.ones((16, 16, 1), np.uint8))


def gradients(h: int = 128, w: int = 256) -> np.ndarray:
    yy, xx = np.mgrid[0:h, 0:w]
    b = (xx * 2) % 256
    g = (yy * 4 + xx) % 256
    r = (xx * 8 + yy * 8) % 256
    return np.stack([b, g, r], -1).astype(np.uint8)


def checkerboards(h: int = 64, w: int = 128) -> np.ndarray:
    """Extreme +-128 patterns: maximise |DCT| and the accumulation bound."""
    yy, xx = np.mgrid[0:h, 0:w]
    out = np.zeros((h, w, 3), np.uint8)
    out[..., 0] = np.where((xx + yy) % 2, 255, 0)
    out[..., 1] = np.where((xx // 2 + yy // 3) % 2, 255, 0)
    out[..., 2] = np.where(((xx * 3) // 5 + yy) % 2, 0, 255)
    return out


def noise(h: int = 128, w: int = 256, seed: int = 7) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def near_gray(h: int = 128, w: int = 256, seed: int = 3) -> np.ndarray:
    """Pixels with R==G, B==G or all equal -- the colour-exception lattice."""
    rng = np.random.default_rng(seed)
    g = rng.integers(0, 256, size=(h, w), dtype=np.int16)
    d = rng.integers(-40, 41, size=(h, w), dtype=np.int16)
    sel = rng.integers(0, 3, size=(h, w))
    b = np.where(sel == 0, g, np.clip(g + d, 0, 255))
    r = np.where(sel == 1, g, np.clip(g - d, 0, 255))
    r = np.where(sel == 2, g, r)
    b = np.where(sel == 2, g, b)
    return np.stack([b, g, r], -1).astype(np.uint8)


ADVERSARIAL = {
    "gray_levels": gray_levels,
    "flat_colours": flat_colours,
    "gradients": gradients,
    "checkerboards": checkerboards,
    "noise": noise,
    "near_gray": near_gray,
}


def detect_scene(seed: int, w: int = 320, h: int = 240, kind: str = "objects"):
    """(stored, current) BGR frame pair for the change detector (brain.c).

    kinds: "objects" -- a smooth background with a few solid/noisy rectangles
    pasted into the current frame; "many" -- hundreds of small patches (the
    100-area overflow path of brain.c:156-168); "noise" -- the whole current
    frame perturbed by +-30; "same" -- identical frames; "edge" -- patches
    touching the right and bottom edges (runs left open at a row end);
    "grid" -- a regular grid of small separated patches (> 100 areas)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)),
                     ((xx + yy) * 127 // max(w + h - 2, 1))], axis=-1).astype(np.uint8)
    base = np.clip(base.astype(int) + rng.integers(-3, 4, base.shape), 0, 255).astype(np.uint8)
    cur = base.copy()
    if kind == "same":
        return base, cur
    if kind == "noise":
        cur = np.clip(cur.astype(int) + rng.integers(-30, 31, cur.shape), 0, 255).astype(np.uint8)
        return base, cur
    if kind == "grid":  # separated 8x8 patches every 24 px: > 100 areas
        for y in range(8, h - 16, 24):
            for x in range(8, w - 16, 24):
                cur[y:y + 8, x:x + 8] = rng.integers(0, 256, 3)
        return base, cur
    n = {"objects": int(rng.integers(1, 12)), "many": 400, "edge": 6}[kind]
    big = {"objects": 0.12, "many": 0.03, "edge": 0.3}[kind]
    for _ in range(n):
        rw = int(rng.integers(2, max(3, int(w * big) + 3)))
        rh = int(rng.integers(2, max(3, int(h * big) + 3)))
        if kind == "edge":
            x, y = (w - rw, int(rng.integers(0, h - rh))) if rng.random() < 0.5 else \
                   (int(rng.integers(0, w - rw)), h - rh)
        else:
            x, y = int(rng.integers(0, w - rw)), int(rng.integers(0, h - rh))
        if rng.random() < 0.6:
            cur[y:y + rh, x:x + rw] = rng.integers(0, 256, 3)
        else:
            cur[y:y + rh, x:x + rw] = rng.integers(0, 256, (rh, rw, 3))
    return base, cur


# (seed, w, h, kind) of the committed detector fixtures (tests/golden/detect.json)
DETECT_CASES = [(s, 320, 240, "objects") for s in range(12)] + \
    [(100 + s, 320, 240, k) for s, k in enumerate(["many", "many", "noise", "same", "edge", "edge"])] + \
    [(200, 64, 64, "objects"), (201, 640, 480, "objects"), (202, 1920, 1080, "objects"),
     (203, 1920, 1080, "many"), (204, 3840, 2160, "objects"), (205, 336, 208, "edge"),
     (206, 320, 240, "grid"), (207, 640, 480, "grid"), (208, 1280, 720, "noise")]
