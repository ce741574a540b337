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
