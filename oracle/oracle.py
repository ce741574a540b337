"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the two CPU checkers:
  * ``libcref.so``  -- the plain-C restatement (oracle/cpu_ref.c), and
  * ``_ref/libref_encoder.so`` -- the unmodified reference main/encoder.c
    compiled by oracle/Makefile (present only where it was built).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (jpeg-encoder-decoder_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CREF_SO = os.path.join(HERE, "libcref.so")
REF_SO = os.path.join(HERE, "_ref", "libref_encoder.so")
REF_QUALITY = os.path.join(HERE, "_ref", "ref_quality")
REF_BRAIN_SO = os.path.join(HERE, "_ref", "libref_brain.so")


class Huff(C.Structure):
    """Layout of huff_code (reference include/structs.h:5-13)."""
    _fields_ = [
        ("sym_freq", C.c_int * 257),
        ("code_len", C.c_int * 257),
        ("next", C.c_int * 257),
        ("code_len_freq", C.c_int * 32),
        ("sym_sorted", C.c_int * 256),
        ("sym_code_len", C.c_int * 256),
        ("sym_code", C.c_int * 256),
    ]


class Area(C.Structure):
    _fields_ = [("x", C.c_int), ("y", C.c_int), ("w", C.c_int), ("h", C.c_int)]


def build(force: bool = False) -> None:
    """Compile the checkers (libcref.so always; _ref when /root/reference exists)."""
    if force or not os.path.exists(CREF_SO) or (
            os.path.getmtime(CREF_SO) < os.path.getmtime(os.path.join(HERE, "cpu_ref.c"))):
        subprocess.check_call(["make", "-s", "-C", HERE, "libcref.so"])
    if os.path.isdir("/root/reference"):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


_cref = None
_ref = None


def cref() -> C.CDLL:
    global _cref
    if _cref is None:
        build()
        lib = C.CDLL(CREF_SO)
        p = C.c_void_p
        lib.cref_encode.restype = C.c_size_t
        lib.cref_encode.argtypes = [p, C.c_int, Area, C.c_int, p, C.c_size_t]
        lib.cref_rgb_to_dct.argtypes = [p, C.c_int, p, p, p, Area, p, p]
        lib.cref_init_huffman.restype = C.c_int
        lib.cref_init_huffman.argtypes = [p, p, p, Area, p, p]
        lib.cref_build_table.restype = C.c_int
        lib.cref_build_table.argtypes = [p, p]
        lib.cref_write_jpg.restype = C.c_size_t
        lib.cref_write_jpg.argtypes = [p, p, p, p, Area, p, p, p, p]
        lib.cref_quality_tables.argtypes = [C.c_int, p, p]
        lib.cref_dct_block_f64.argtypes = [p, C.c_int, p]
        lib.cref_pixel_ycc.argtypes = [C.c_uint8, C.c_uint8, C.c_uint8, p]
        lib.cref_cos_bits.argtypes = [p]
        lib.cref_max_jpg_bytes.restype = C.c_size_t
        lib.cref_max_jpg_bytes.argtypes = [C.c_int, C.c_int]
        lib.cref_subsample.argtypes = [p, C.c_int, C.c_int, p]
        lib.cref_compare.restype = C.c_int
        lib.cref_compare.argtypes = [p, p, C.c_int, C.c_int, p]
        lib.cref_enlarge_adjust.argtypes = [p, C.c_int, C.c_int]
        _cref = lib
    return _cref


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref() -> C.CDLL:
    global _ref
    if _ref is None:
        lib = C.CDLL(REF_SO)
        p = C.c_void_p
        lib.ref_encode.restype = C.c_size_t
        lib.ref_encode.argtypes = [p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   p, p, p, p, p]
        lib.ref_stage_dct.argtypes = [p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      p, p, p]
        lib.ref_cos_bits.argtypes = [p]
        lib.ref_encode_file.restype = C.c_size_t
        lib.ref_encode_file.argtypes = [C.c_char_p, C.c_char_p, p, C.c_size_t, p, p, p, p]
        lib.ref_huff_size.restype = C.c_size_t
        _ref = lib
    return _ref


_file_bufs = {}


def ref_encode_file(ppm_path: str, jpg_path: str, max_px: int = 3840 * 2160) -> int:
    """The reference encoder.c on a file (oracle/_ref ref_encode_file): PPM
    read + RGB->BGR + rgb_to_dct + init_huffman + write_jpg into jpg_path.
    Returns the .jpg size (0: unreadable file).  Buffers are kept per size,
    as main.c keeps its buffers static."""
    lib = ref()
    bufs = _file_bufs.get(max_px)
    if bufs is None:
        bufs = (np.zeros(max_px * 3, np.uint8), np.zeros(max_px, np.int16), np.zeros(max_px // 4, np.int16),
                np.zeros(max_px // 4, np.int16), np.zeros(max_jpg_bytes(16, max_px // 16), np.uint8))
        _file_bufs[max_px] = bufs
    bgr, Y, Cb, Cr, jpg = bufs
    return int(lib.ref_encode_file(ppm_path.encode(), jpg_path.encode(), _ptr(bgr), bgr.size, _ptr(Y),
                                   _ptr(Cb), _ptr(Cr), _ptr(jpg)))


_ref_brain = None


def ref_brain_available() -> bool:
    return os.path.exists(REF_BRAIN_SO)


def ref_brain() -> C.CDLL:
    """The unmodified reference main/brain.c (oracle/_ref/libref_brain.so)."""
    global _ref_brain
    if _ref_brain is None:
        lib = C.CDLL(REF_BRAIN_SO)
        p = C.c_void_p
        lib.ref_subsample.restype = C.c_int
        lib.ref_subsample.argtypes = [p, C.c_int, C.c_int, p]
        lib.ref_compare.restype = C.c_int
        lib.ref_compare.argtypes = [p, p, C.c_int, C.c_int, p]
        lib.ref_enlarge_adjust.argtypes = [p, C.c_int, C.c_int]
        _ref_brain = lib
    return _ref_brain


def _areas(outs, n):
    return [(a.x, a.y, a.w, a.h) for a in outs[:max(0, min(n, 100))]]


def cref_subsample(bgr: np.ndarray) -> np.ndarray:
    """brain.c:16-45 restated: (H/4, W/4, 3) RGB plane of a BGR frame."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    sub = np.zeros((H // 4, W // 4, 3), np.uint8)
    cref().cref_subsample(_ptr(bgr), W, H, _ptr(sub))
    return sub


def cref_compare(sub: np.ndarray, saved: np.ndarray, W: int, H: int):
    """brain.c:104-233 restated: (count, [areas]) for two subsampled planes."""
    sub = np.ascontiguousarray(sub, dtype=np.uint8)
    saved = np.ascontiguousarray(saved, dtype=np.uint8)
    outs = (Area * 100)()
    n = cref().cref_compare(_ptr(sub), _ptr(saved), W, H, outs)
    return n, _areas(outs, n)


def cref_area_adjust(area, W: int, H: int):
    """brain.c:240-261 restated."""
    a = Area(*area)
    cref().cref_enlarge_adjust(C.byref(a), W, H)
    return (a.x, a.y, a.w, a.h)


def ref_subsample(bgr: np.ndarray) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    sub = np.zeros((H // 4, W // 4, 3), np.uint8)
    if ref_brain().ref_subsample(_ptr(bgr), W, H, _ptr(sub)):
        raise OSError("ref_subsample failed")
    return sub


def ref_compare(sub: np.ndarray, saved: np.ndarray, W: int, H: int):
    sub = np.ascontiguousarray(sub, dtype=np.uint8)
    saved = np.ascontiguousarray(saved, dtype=np.uint8)
    outs = (Area * 100)()
    n = ref_brain().ref_compare(_ptr(sub), _ptr(saved), W, H, outs)
    return n, _areas(outs, n)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def max_jpg_bytes(w: int, h: int) -> int:
    return int(cref().cref_max_jpg_bytes(w, h))


def quality_tables(q: int):
    lq = np.zeros(64, np.int32)
    cq = np.zeros(64, np.int32)
    cref().cref_quality_tables(q, _ptr(lq), _ptr(cq))
    return lq, cq


def cref_encode(bgr: np.ndarray, quality: int = 50, region=None) -> bytes:
    """Encode an HxWx3 BGR uint8 frame (or `region`=(x,y,w,h) of it)."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    x, y, w, h = region if region else (0, 0, W, H)
    cap = max_jpg_bytes(w, h)
    out = np.zeros(cap, np.uint8)
    n = cref().cref_encode(_ptr(bgr), W, Area(x, y, w, h), quality, _ptr(out), cap)
    if n == 0:
        raise ValueError("cref_encode rejected the input")
    return out[:n].tobytes()


def cref_build_table(freq: np.ndarray):
    """(rc, Huff) of one table built from counts of symbols 0..255
    (encoder.c:180-301; sym_freq[256] = 1 as :367 sets it)."""
    f = np.ascontiguousarray(freq, np.uint32).reshape(256)
    h = Huff()
    rc = cref().cref_build_table(_ptr(f), C.addressof(h))
    return rc, h


def cref_stages(bgr: np.ndarray, quality: int = 50, region=None):
    """(Y, Cb, Cr coefficient planes after DC-diff, [4 Huff], jpg bytes)."""
    lib = cref()
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    x, y, w, h = region if region else (0, 0, W, H)
    lq, cq = quality_tables(quality)
    Y = np.zeros(w * h, np.int16)
    Cb = np.zeros(w * h // 4, np.int16)
    Cr = np.zeros(w * h // 4, np.int16)
    a = Area(x, y, w, h)
    lib.cref_rgb_to_dct(_ptr(bgr), W, _ptr(Y), _ptr(Cb), _ptr(Cr), a, _ptr(lq), _ptr(cq))
    tabs = (Huff * 4)()
    rc = lib.cref_init_huffman(_ptr(Y), _ptr(Cb), _ptr(Cr), a, C.addressof(tabs),
                               C.addressof(tabs) + 2 * C.sizeof(Huff))
    if rc:
        raise ValueError("table construction failed")
    out = np.zeros(max_jpg_bytes(w, h), np.uint8)
    n = lib.cref_write_jpg(_ptr(out), _ptr(Y), _ptr(Cb), _ptr(Cr), a, C.addressof(tabs),
                           C.addressof(tabs) + 2 * C.sizeof(Huff), _ptr(lq), _ptr(cq))
    return Y, Cb, Cr, list(tabs), out[:n].tobytes()


def ref_stages(bgr: np.ndarray, region=None):
    """Same as cref_stages(quality=50) but through the compiled reference."""
    lib = ref()
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    x, y, w, h = region if region else (0, 0, W, H)
    Y = np.zeros(w * h, np.int16)
    Cb = np.zeros(w * h // 4, np.int16)
    Cr = np.zeros(w * h // 4, np.int16)
    tabs = (Huff * 4)()
    out = np.zeros(max_jpg_bytes(w, h), np.uint8)
    n = lib.ref_encode(_ptr(bgr), W, x, y, w, h, _ptr(Y), _ptr(Cb), _ptr(Cr),
                       C.addressof(tabs), _ptr(out))
    return Y, Cb, Cr, list(tabs), out[:n].tobytes()


def ref_quality_encode(rgb_ppm_path: str, quality: int, workdir: str) -> bytes:
    """Q-sweep through the unmodified upstream original.c (set_quality)."""
    os.makedirs(os.path.join(workdir, "hisParts"), exist_ok=True)
    subprocess.check_call([REF_QUALITY, os.path.abspath(rgb_ppm_path), str(quality)],
                          cwd=workdir, stdout=subprocess.DEVNULL)
    with open(os.path.join(workdir, "out.jpg"), "rb") as f:
        return f.read()


def dct_block_f64(block: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(block, dtype=np.uint8).reshape(64)
    out = np.zeros(64, np.float64)
    cref().cref_dct_block_f64(_ptr(b), 8, _ptr(out))
    return out


def cos_bits_cref() -> np.ndarray:
    out = np.zeros(64, np.int64)
    cref().cref_cos_bits(_ptr(out))
    return out


def cos_bits_ref() -> np.ndarray:
    out = np.zeros(64, np.int64)
    ref().ref_cos_bits(_ptr(out))
    return out
