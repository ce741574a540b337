"""Minimal P6 PPM helpers for the tests (mirrors original.c:294-365 checks)."""
import gzip

import numpy as np


def parse_ppm(data: bytes) -> np.ndarray:
    """Return an HxWx3 RGB uint8 array.  Accepts '#' comment lines like
    original.c:303-316; requires depth 255 and W, H multiples of 16."""
    if data[:2] != b"P6":
        raise ValueError("not a P6 PPM")
    pos = 2
    fields = []
    while len(fields) < 3:
        while data[pos:pos + 1].isspace():
            pos += 1
        if data[pos:pos + 1] == b"#":
            pos = data.index(b"\n", pos) + 1
            continue
        end = pos
        while not data[end:end + 1].isspace():
            end += 1
        fields.append(int(data[pos:end]))
        pos = end
    pos += 1  # single whitespace after depth
    w, h, depth = fields
    if depth != 255:
        raise ValueError("only depth 255 is supported")
    if w % 16 or h % 16:
        raise ValueError("dimensions must be multiples of 16")
    px = np.frombuffer(data, np.uint8, count=w * h * 3, offset=pos)
    return px.reshape(h, w, 3).copy()


def read_ppm(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith(".gz"):
        data = gzip.decompress(data)
    return parse_ppm(data)


def ppm_bytes(rgb: np.ndarray) -> bytes:
    h, w = rgb.shape[:2]
    return b"P6\n%d %d\n255\n" % (w, h) + np.ascontiguousarray(rgb, np.uint8).tobytes()


def rgb_to_bgr(rgb: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(rgb[..., ::-1])
