"""ctypes binding of libmijpeg.so (include/mijpeg.h) for tests and bench.py.

The product is the C ABI; this module only marshals numpy buffers across it.
There is deliberately no CPU fallback: if the HIP library is missing or no
GPU is visible, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MIJ_LIB: alternative build of the same library (A/B timing runs, scripts/ab.sh)
LIB_PATH = os.environ.get("MIJ_LIB") or os.path.join(HERE, "libmijpeg.so")

EXPORTS = [
    # drop-in (reference include/encoder.h:10-12)
    "rgb_to_dct", "init_huffman", "write_jpg",
    # extensions
    "mij_set_input_stride", "mij_set_quality", "mij_last_error", "mij_strerror", "mij_last_message",
    "mij_max_jpg_bytes", "mij_encode",
    "mij_batch_create", "mij_batch_destroy", "mij_batch_upload", "mij_batch_set_input",
    "mij_batch_encode", "mij_batch_keep_coefs", "mij_batch_set_split", "mij_batch_set_overlap", "mij_batch_set_option", "mij_batch_get_option", "mij_batch_dct", "mij_batch_pattern_floor", "mij_batch_sync", "mij_batch_output",
    "mij_batch_lengths", "mij_batch_coefs", "mij_batch_tables", "mij_batch_set_timing",
    "mij_batch_stage_ms", "mij_batch_stage_history", "mij_batch_token_count", "mij_batch_geometry", "mij_batch_replays", "mij_batch_stream", "mij_batch_set_stream", "mij_batch_audit", "mij_batch_build_tables",
    "mij_band_analyze", "mij_band_histograms", "mij_band_tables", "mij_band_pack", "mij_band_words",
    "mij_assemble_begin", "mij_assemble_words", "mij_assemble_end",
    "mij_band_words_all", "mij_assemble_pieces", "mij_assembler_create",
    "mij_band_analyze_async", "mij_band_histograms_async", "mij_band_tables_async", "mij_band_pack_async",
    "mij_band_words_async", "mij_assemble_tables_async", "mij_assemble_async",
    "mij_band_stuff_async", "mij_assemble_stuffed_async", "mij_copy_to_host_async",
    "mij_probe_mfma", "mij_colour_lut", "mij_build_target",
    # change detector (reference include/brain.h:7-10 drop-in + extensions)
    "subsample", "store", "compare", "enlargeAdjust", "mij_set_frame_height",
    "mij_decoder_create", "mij_decoder_destroy", "mij_decoder_decode", "mij_decoder_info",
    "mij_decoder_coefs", "mij_decoder_device_coefs", "mij_decoder_passes",
    "mij_detector_create", "mij_detector_destroy", "mij_detector_subsample", "mij_detector_compare",
    "mij_detector_step", "mij_detector_launch", "mij_detector_store", "mij_detector_upload", "mij_detector_get_plane",
    "mij_detector_set_plane", "mij_detector_mask", "mij_detector_stream",
    "mij_batch_set_rgb", "mij_ppm_header", "mij_ppm_read",
    "mij_stream_create", "mij_stream_destroy", "mij_stream_encode_files",
    "mij_stream_encode_frames", "mij_stream_stats",
    "mij_batch_set_frame_dims", "mij_batch_gather_regions", "mij_batch_upload_regions",
    "mij_encode_regions",
]


class Huff(C.Structure):
    """huff_code (reference include/structs.h:5-13)."""
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
    """area_t (reference include/structs.h:15-18)."""
    _fields_ = [("x", C.c_int), ("y", C.c_int), ("w", C.c_int), ("h", C.c_int)]


class MijError(RuntimeError):
    pass


# mij_batch_set_option (include/mijpeg.h: MIJ_OPT_*)
OPTIONS = {"seam": 0, "ff_pack": 1, "actab": 2, "segdc_fused": 3, "pack_wide": 4, "emit_slots": 5,
           "overlap_prio": 6, "pack_segs": 8}


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MijError(f"{LIB_PATH} missing: build it with `make -C {HERE}` "
                       "(there is no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    p, i, sz = C.c_void_p, C.c_int, C.c_size_t
    lib.rgb_to_dct.argtypes = [p, p, p, p, Area]
    lib.rgb_to_dct.restype = None
    lib.init_huffman.argtypes = [p, p, p, Area, p, p]
    lib.init_huffman.restype = None
    lib.write_jpg.argtypes = [p, p, p, p, p, Area, p, p]
    lib.write_jpg.restype = sz
    lib.mij_set_input_stride.argtypes = [i]
    lib.mij_set_quality.argtypes = [i]
    lib.mij_last_error.restype = i
    lib.mij_strerror.restype = C.c_char_p
    lib.mij_strerror.argtypes = [i]
    lib.mij_last_message.restype = C.c_char_p
    lib.mij_last_message.argtypes = []
    lib.mij_max_jpg_bytes.restype = sz
    lib.mij_max_jpg_bytes.argtypes = [i, i]
    lib.mij_encode.argtypes = [p, i, Area, i, p, sz, C.POINTER(sz)]
    lib.mij_batch_create.restype = p
    lib.mij_batch_create.argtypes = [i, i, i, i, i]
    lib.mij_batch_destroy.argtypes = [p]
    lib.mij_batch_destroy.restype = None
    lib.mij_batch_upload.argtypes = [p, p, i, i]
    lib.mij_batch_set_input.argtypes = [p, p, C.c_longlong, i]
    lib.mij_batch_encode.argtypes = [p, i]
    lib.mij_batch_keep_coefs.argtypes = [p, i]
    lib.mij_batch_set_split.argtypes = [p, i]
    lib.mij_batch_set_overlap.argtypes = [p, i]
    lib.mij_batch_set_option.argtypes = [p, i, i]
    lib.mij_batch_get_option.argtypes = [p, i]
    lib.mij_batch_dct.argtypes = [p, i]
    lib.mij_batch_pattern_floor.argtypes = [p, i]
    lib.mij_batch_audit.argtypes = [p, i, p]
    lib.mij_band_analyze_async.argtypes = [p, i, p]
    lib.mij_band_histograms_async.argtypes = [p, i, p, p]
    lib.mij_band_tables_async.argtypes = [p, i, p, p]
    lib.mij_band_pack_async.argtypes = [p, i, p]
    lib.mij_band_words_async.argtypes = [p, i, p, sz]
    lib.mij_assemble_tables_async.argtypes = [p, i, p]
    lib.mij_assemble_async.argtypes = [p, i, p, i, p, sz]
    lib.mij_band_stuff_async.argtypes = [p, i, p, i, i, p, p, p, sz]
    lib.mij_assemble_stuffed_async.argtypes = [p, i, p, i, p, sz]
    lib.mij_copy_to_host_async.argtypes = [p, p, p, sz]
    lib.mij_batch_build_tables.argtypes = [p, i, p]
    lib.mij_batch_sync.argtypes = [p]
    lib.mij_batch_output.argtypes = [p, i, p, sz, C.POINTER(sz)]
    lib.mij_batch_lengths.argtypes = [p, C.POINTER(sz), i]
    lib.mij_batch_coefs.argtypes = [p, i, p, p, p, i]
    lib.mij_batch_tables.argtypes = [p, i, p]
    lib.mij_batch_set_timing.argtypes = [p, i]
    lib.mij_batch_stage_ms.argtypes = [p, p, i]
    lib.mij_batch_stage_history.argtypes = [p, p, i]
    lib.mij_batch_token_count.restype = C.c_ulonglong
    lib.mij_batch_token_count.argtypes = [p, i]
    lib.mij_batch_geometry.argtypes = [p, p, i]
    lib.mij_batch_replays.restype = C.c_ulonglong
    lib.mij_batch_replays.argtypes = [p]
    lib.mij_batch_stream.restype = p
    lib.mij_batch_stream.argtypes = [p]
    lib.mij_batch_set_stream.argtypes = [p, p]
    u64 = C.c_ulonglong
    lib.mij_band_analyze.argtypes = [p, i, p]
    lib.mij_band_histograms.argtypes = [p, i, p, p]
    lib.mij_band_tables.argtypes = [p, i, p, p]
    lib.mij_band_pack.argtypes = [p, i, p, p]
    lib.mij_band_words.argtypes = [p, i, i, p, C.c_size_t, i]
    lib.mij_assemble_begin.argtypes = [p, i, p]
    lib.mij_assemble_words.argtypes = [p, i, i, u64, p, C.c_size_t, i]
    lib.mij_assemble_end.argtypes = [p, i, p]
    lib.mij_band_words_all.argtypes = [p, i, p, C.c_size_t, i]
    lib.mij_assemble_pieces.argtypes = [p, p, C.c_size_t, i, p, i]
    lib.mij_assembler_create.restype = p
    lib.mij_assembler_create.argtypes = [i, i, i, i, i]
    lib.mij_probe_mfma.argtypes = [p, p, p]
    lib.mij_colour_lut.argtypes = [p]
    lib.mij_build_target.restype = C.c_char_p
    lib.mij_batch_set_rgb.argtypes = [p, i]
    lib.mij_ppm_header.argtypes = [C.c_char_p, C.POINTER(i), C.POINTER(i), C.POINTER(C.c_longlong)]
    lib.mij_ppm_read.argtypes = [C.c_char_p, p, sz, i, i]
    lib.mij_stream_create.restype = p
    lib.mij_stream_create.argtypes = [i, i, i, i, i, i]
    lib.mij_stream_destroy.argtypes = [p]
    lib.mij_stream_destroy.restype = None
    lib.mij_stream_encode_files.argtypes = [p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), i,
                                            C.POINTER(i)]
    lib.mij_stream_encode_frames.argtypes = [p, C.POINTER(p), i, C.POINTER(p), C.POINTER(sz),
                                             C.POINTER(sz)]
    lib.mij_stream_stats.argtypes = [p, p, i]
    try:
        lib.mij_detector_create.restype = p
        lib.mij_detector_create.argtypes = [i, i, i]
        lib.mij_detector_destroy.argtypes = [p]
        lib.mij_detector_subsample.argtypes = [p, p, C.c_longlong]
        lib.mij_detector_compare.argtypes = [p, p, C.POINTER(i)]
        lib.mij_detector_step.argtypes = [p, p, C.c_longlong, p, C.POINTER(i)]
        lib.mij_detector_store.argtypes = [p]
        lib.mij_detector_launch.argtypes = [p, p, C.c_longlong]
        lib.mij_detector_upload.argtypes = [p, p, C.c_longlong, C.POINTER(p)]
        lib.mij_detector_get_plane.argtypes = [p, i, p]
        lib.mij_detector_set_plane.argtypes = [p, i, p]
        lib.mij_detector_mask.argtypes = [p, p, sz, C.POINTER(i)]
        lib.mij_detector_stream.restype = p
        lib.mij_detector_stream.argtypes = [p]
        lib.mij_set_frame_height.argtypes = [i]
        lib.mij_decoder_create.restype = p
        lib.mij_decoder_create.argtypes = [i, i, i, i]
        lib.mij_decoder_destroy.argtypes = [p]
        lib.mij_decoder_decode.argtypes = [p, C.POINTER(p), C.POINTER(sz), i]
        lib.mij_decoder_info.argtypes = [p, i, C.POINTER(i), C.POINTER(i), p]
        lib.mij_decoder_coefs.argtypes = [p, i, p, p, p]
        lib.mij_decoder_device_coefs.restype = p
        lib.mij_decoder_device_coefs.argtypes = [p, i]
        lib.mij_decoder_passes.argtypes = [p]
        lib.subsample.restype = None
        lib.subsample.argtypes = [p, p, p]
        lib.store.restype = None
        lib.store.argtypes = [p, p]
        lib.compare.restype = C.c_uint8
        lib.compare.argtypes = [p, p, p, p]
        lib.enlargeAdjust.restype = None
        lib.enlargeAdjust.argtypes = [p]
        lib.mij_batch_set_frame_dims.argtypes = [p, p, i]
        lib.mij_batch_gather_regions.argtypes = [p, p, C.c_longlong, i, i, p, i]
        lib.mij_batch_upload_regions.argtypes = [p, p, i, i, p, i]
        lib.mij_encode_regions.argtypes = [p, i, i, p, i, i, p, sz, p]
    except AttributeError:
        if not os.environ.get("MIJ_LIB"):  # older builds only in A/B timing runs
            raise
    _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        lib = load()
        raise MijError(f"{what}: {lib.mij_strerror(rc).decode()} ({rc}): "
                       f"{lib.mij_last_message().decode(errors='replace')}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def max_jpg_bytes(w: int, h: int) -> int:
    return int(load().mij_max_jpg_bytes(w, h))


# ---- drop-in three-call path (main.c:144-152 call sequence) -----------------

def set_input_stride(px: int) -> None:
    _check(load().mij_set_input_stride(px), "mij_set_input_stride")


def set_quality(q: int) -> None:
    _check(load().mij_set_quality(q), "mij_set_quality")


def rgb_to_dct(frame_bgr: np.ndarray, region):
    """encoder.h:10 on a BGR frame; returns (Y, Cb, Cr) int16 planes."""
    lib = load()
    frame_bgr = np.ascontiguousarray(frame_bgr, np.uint8)
    x, y, w, h = region
    set_input_stride(frame_bgr.shape[1])
    Y = np.zeros(w * h, np.int16)
    Cb = np.zeros(w * h // 4, np.int16)
    Cr = np.zeros(w * h // 4, np.int16)
    lib.rgb_to_dct(_ptr(frame_bgr), _ptr(Y), _ptr(Cb), _ptr(Cr), Area(x, y, w, h))
    _check(lib.mij_last_error(), "rgb_to_dct")
    return Y, Cb, Cr


def init_huffman(Y, Cb, Cr, region):
    lib = load()
    x, y, w, h = region
    t = (Huff * 4)()
    lib.init_huffman(_ptr(Y), _ptr(Cb), _ptr(Cr), Area(x, y, w, h), C.addressof(t),
                     C.addressof(t) + 2 * C.sizeof(Huff))
    _check(lib.mij_last_error(), "init_huffman")
    return list(t)


def write_jpg(Y, Cb, Cr, region, tables) -> bytes:
    lib = load()
    x, y, w, h = region
    t = (Huff * 4)(*tables)
    out = np.zeros(max_jpg_bytes(w, h), np.uint8)
    n = lib.write_jpg(None, _ptr(out), _ptr(Y), _ptr(Cb), _ptr(Cr), Area(x, y, w, h),
                      C.addressof(t), C.addressof(t) + 2 * C.sizeof(Huff))
    _check(lib.mij_last_error(), "write_jpg")
    return out[:n].tobytes()


def _areas(regions):
    arr = (Area * len(regions))(*[Area(*map(int, r)) for r in regions])
    return arr


def encode_regions(frame_bgr: np.ndarray, regions, quality: int = 50) -> list:
    """mij_encode_regions: every (x, y, w, h) region of a BGR frame to its own
    JPEG in one launch sequence (main.c:142-155)."""
    lib = load()
    frame_bgr = np.ascontiguousarray(frame_bgr, np.uint8)
    H, W = frame_bgr.shape[:2]
    cap = sum(max_jpg_bytes(r[2], r[3]) for r in regions)
    out = np.zeros(max(cap, 1), np.uint8)
    lens = (C.c_size_t * len(regions))()
    _check(lib.mij_encode_regions(_ptr(frame_bgr), W, H, _areas(regions), len(regions), quality,
                                  _ptr(out), out.size, lens), "mij_encode_regions")
    res, off = [], 0
    for n in lens:
        res.append(out[off:off + n].tobytes())
        off += n
    return res


def encode(frame_bgr: np.ndarray, quality: int = 50, region=None) -> bytes:
    """mij_encode: whole path host->host."""
    lib = load()
    frame_bgr = np.ascontiguousarray(frame_bgr, np.uint8)
    H, W = frame_bgr.shape[:2]
    x, y, w, h = region if region else (0, 0, W, H)
    cap = max_jpg_bytes(w, h)
    out = np.zeros(cap, np.uint8)
    n = C.c_size_t(0)
    _check(lib.mij_encode(_ptr(frame_bgr), W, Area(x, y, w, h), quality, _ptr(out), cap,
                          C.byref(n)), "mij_encode")
    return out[:n.value].tobytes()


# ---- device-resident batch ---------------------------------------------------

class Batch:
    STAGES = ["k1_colour_dct_quant", "fix", "tokenize", "stats", "tables", "pack", "emit", "total"]

    def __init__(self, w: int, h: int, max_frames: int, quality: int = 50, device: int = 0,
                 keep_coefs: bool = False, assembler: bool = False):
        """assembler=True: mij_assembler_create -- a batch that only assembles
        whole frames from band words (no input, coefficient or token buffers)."""
        self.lib = load()
        self.w, self.h, self.max_frames = w, h, max_frames
        create = self.lib.mij_assembler_create if assembler else self.lib.mij_batch_create
        self.h_ = create(device, w, h, max_frames, quality)
        self.fdims = None  # per-frame (w, h) of a region batch
        if not self.h_:
            raise MijError(f"{'mij_assembler_create' if assembler else 'mij_batch_create'} failed: "
                           f"{self.lib.mij_strerror(self.lib.mij_last_error()).decode()}")
        if keep_coefs:
            _check(self.lib.mij_batch_keep_coefs(self.h_, 1), "keep_coefs")

    def close(self) -> None:
        if self.h_:
            self.lib.mij_batch_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_split(self, on: bool) -> None:
        _check(self.lib.mij_batch_set_split(self.h_, int(on)), "set_split")

    def set_overlap(self, nsub: int) -> None:
        """fused pipeline in nsub sub-batches, entropy of one beside K1 of the next"""
        _check(self.lib.mij_batch_set_overlap(self.h_, int(nsub)), "set_overlap")

    def set_option(self, name: str, value: int) -> None:
        """entropy-stage variant (include/mijpeg.h MIJ_OPT_*; same bytes)"""
        _check(self.lib.mij_batch_set_option(self.h_, OPTIONS[name], int(value)), f"set_option({name})")

    def get_option(self, name: str) -> int:
        v = int(self.lib.mij_batch_get_option(self.h_, OPTIONS[name]))
        if v == -2:  # mij_batch_get_option's error value (the error is set)
            _check(self.lib.mij_last_error() or 1, "get_option")
        return v

    def set_rgb(self, on: bool) -> None:
        """frames in R, G, B byte order (PPM) instead of the encoder's B, G, R"""
        _check(self.lib.mij_batch_set_rgb(self.h_, int(on)), "set_rgb")

    def set_frame_dims(self, dims) -> None:
        """per-frame (w, h) of a region batch; None restores the batch geometry"""
        if dims is None:
            _check(self.lib.mij_batch_set_frame_dims(self.h_, None, 0), "set_frame_dims")
            self.fdims = None
            return
        wh = np.ascontiguousarray(np.asarray(dims, np.int32).reshape(-1, 2))
        _check(self.lib.mij_batch_set_frame_dims(self.h_, _ptr(wh), wh.shape[0]), "set_frame_dims")
        self.fdims = [tuple(map(int, d)) for d in wh]

    def upload_regions(self, frame_bgr: np.ndarray, regions) -> None:
        frame_bgr = np.ascontiguousarray(frame_bgr, np.uint8)
        H, W = frame_bgr.shape[:2]
        _check(self.lib.mij_batch_upload_regions(self.h_, _ptr(frame_bgr), W, H, _areas(regions),
                                                 len(regions)), "upload_regions")
        self.fdims = [(int(r[2]), int(r[3])) for r in regions]

    def gather_regions(self, dev_ptr: int, pitch: int, frame_w: int, frame_h: int, regions) -> None:
        _check(self.lib.mij_batch_gather_regions(self.h_, dev_ptr, pitch, frame_w, frame_h,
                                                 _areas(regions), len(regions)), "gather_regions")
        self.fdims = [(int(r[2]), int(r[3])) for r in regions]

    def upload(self, frames_bgr: np.ndarray, first: int = 0) -> None:
        frames_bgr = np.ascontiguousarray(frames_bgr, np.uint8)
        n = frames_bgr.shape[0] if frames_bgr.ndim == 4 else 1
        _check(self.lib.mij_batch_upload(self.h_, _ptr(frames_bgr), first, n), "upload")
        # full frames: the uploaded slots are canvas-sized again, the others
        # keep their region sizes (as the library does)
        if self.fdims is not None:
            dims = list(self.fdims) + [(self.w, self.h)] * max(0, self.max_frames - len(self.fdims))
            dims[first:first + n] = [(self.w, self.h)] * n
            self.fdims = None if all(d == (self.w, self.h) for d in dims) else dims

    def set_input(self, dev_ptr: int, frame_stride: int, pitch: int) -> None:
        _check(self.lib.mij_batch_set_input(self.h_, dev_ptr, frame_stride, pitch), "set_input")
        self.fdims = None

    def encode(self, n: int) -> None:
        _check(self.lib.mij_batch_encode(self.h_, n), "encode")

    def dct(self, n: int) -> None:
        _check(self.lib.mij_batch_dct(self.h_, n), "dct")

    def pattern_floor(self, n: int) -> None:
        """measurement only: K1's memory traffic without its arithmetic
        (mij_batch_pattern_floor); leaves garbage in the coefficient planes"""
        _check(self.lib.mij_batch_pattern_floor(self.h_, n), "pattern_floor")

    def sync(self) -> None:
        _check(self.lib.mij_batch_sync(self.h_), "sync")

    def output(self, frame: int) -> bytes:
        n = C.c_size_t(0)
        _check(self.lib.mij_batch_output(self.h_, frame, None, 0, C.byref(n)), "output")
        buf = np.zeros(max(n.value, 1), np.uint8)
        _check(self.lib.mij_batch_output(self.h_, frame, _ptr(buf), buf.size, C.byref(n)),
               "output")
        return buf[:n.value].tobytes()

    def lengths(self, n: int) -> np.ndarray:
        arr = (C.c_size_t * n)()
        _check(self.lib.mij_batch_lengths(self.h_, arr, n), "lengths")
        return np.array(arr[:], np.int64)

    def coefs(self, frame: int, diffed: bool = True):
        w, h = self.fdims[frame] if self.fdims and frame < len(self.fdims) else (self.w, self.h)
        Y = np.zeros(w * h, np.int16)
        Cb = np.zeros(w * h // 4, np.int16)
        Cr = np.zeros(w * h // 4, np.int16)
        _check(self.lib.mij_batch_coefs(self.h_, frame, _ptr(Y), _ptr(Cb), _ptr(Cr),
                                        int(diffed)), "coefs")
        return Y, Cb, Cr

    def tables(self, frame: int):
        t = (Huff * 4)()
        _check(self.lib.mij_batch_tables(self.h_, frame, C.addressof(t)), "tables")
        return list(t)

    def set_timing(self, on: bool) -> None:
        _check(self.lib.mij_batch_set_timing(self.h_, int(on)), "set_timing")

    def stage_ms(self) -> dict:
        ms = np.zeros(len(self.STAGES), np.float32)
        _check(self.lib.mij_batch_stage_ms(self.h_, _ptr(ms), len(ms)), "stage_ms")
        return dict(zip(self.STAGES, [float(v) for v in ms]))

    def stage_history(self, steps: int) -> list:
        ms = np.zeros((steps, len(self.STAGES)), np.float32)
        n = self.lib.mij_batch_stage_history(self.h_, _ptr(ms), steps)
        if n < 0:
            _check(self.lib.mij_last_error(), "stage_history")
        return [dict(zip(self.STAGES, [float(v) for v in row])) for row in ms[:n]]

    def token_count(self, n: int) -> int:
        return int(self.lib.mij_batch_token_count(self.h_, n))

    def geometry(self) -> dict:
        keys = ["w", "h", "nblk", "nseg", "tiles_per_frame", "pack_window_words"]
        g = np.zeros(len(keys), np.int64)
        _check(self.lib.mij_batch_geometry(self.h_, _ptr(g), len(keys)), "geometry")
        return dict(zip(keys, [int(v) for v in g]))

    def audit(self, n: int) -> np.ndarray:
        """K1's fast-path keep/replay decisions (mij_batch_audit): uint64 per
        block [n, nblk], bit z = zigzag coefficient z was replayed in FP64."""
        nblk = self.geometry()["nblk"]
        m = np.zeros((n, nblk, 4), np.uint16)
        _check(self.lib.mij_batch_audit(self.h_, n, _ptr(m)), "audit")
        m = m.astype(np.uint64)
        return m[..., 0] | (m[..., 1] << np.uint64(16)) | (m[..., 2] << np.uint64(32)) | (m[..., 3] << np.uint64(48))

    def build_tables(self, n: int, hist: np.ndarray) -> None:
        """the four tables of frames 0..n-1 from given counts [n, 4, 257]
        (mij_batch_build_tables; read them with tables())"""
        h = np.ascontiguousarray(hist, np.uint32).reshape(n, 4, 257)
        _check(self.lib.mij_batch_build_tables(self.h_, n, _ptr(h)), "build_tables")

    def replays(self) -> int:
        return int(self.lib.mij_batch_replays(self.h_))

    # ---- one large frame over several ranks (include/mijpeg.h, sharding.py) ----
    def band_analyze(self, n: int) -> np.ndarray:
        last = np.zeros((n, 3), np.int16)
        _check(self.lib.mij_band_analyze(self.h_, n, _ptr(last)), "band_analyze")
        return last

    def band_histograms(self, n: int, prev_dc: np.ndarray) -> np.ndarray:
        prev = np.ascontiguousarray(prev_dc, np.int16).reshape(n, 3)
        hist = np.zeros((n, 4, 257), np.uint32)
        _check(self.lib.mij_band_histograms(self.h_, n, _ptr(prev), _ptr(hist)), "band_histograms")
        return hist

    def band_tables(self, n: int, hist: np.ndarray) -> np.ndarray:
        h = np.ascontiguousarray(hist, np.uint32).reshape(n, 4, 257)
        bits = np.zeros((n, 3), np.uint64)
        _check(self.lib.mij_band_tables(self.h_, n, _ptr(h), _ptr(bits)), "band_tables")
        return bits

    def band_pack(self, n: int, bit_offset: np.ndarray) -> np.ndarray:
        off = np.ascontiguousarray(bit_offset, np.uint64).reshape(n, 3)
        nw = np.zeros((n, 3), np.uint64)
        _check(self.lib.mij_band_pack(self.h_, n, _ptr(off), _ptr(nw)), "band_pack")
        return nw

    def band_words(self, frame: int, comp: int, nwords: int, dst_dev_ptr: int = 0):
        """Packed words of one band scan: into host memory (returned array), or
        into device memory at dst_dev_ptr (returns None)."""
        if dst_dev_ptr:
            _check(self.lib.mij_band_words(self.h_, frame, comp, dst_dev_ptr, nwords, 1), "band_words")
            return None
        out = np.zeros(max(nwords, 1), np.uint32)
        _check(self.lib.mij_band_words(self.h_, frame, comp, _ptr(out), nwords, 0), "band_words")
        return out[:nwords]

    def band_words_all(self, n: int, dst=None, dst_dev_ptr: int = 0, cap_words: int = 0):
        """Every scan's band words of frames 0..n-1 in (frame, comp) order, one
        call: into device memory at dst_dev_ptr (cap_words words), into the
        host array dst, or into a returned host array."""
        if dst_dev_ptr:
            _check(self.lib.mij_band_words_all(self.h_, n, dst_dev_ptr, cap_words, 1), "band_words_all")
            return None
        if dst is None:
            dst = np.zeros(max(cap_words, 1), np.uint32)
        _check(self.lib.mij_band_words_all(self.h_, n, _ptr(dst), dst.size, 0), "band_words_all")
        return dst

    def assemble_pieces(self, pieces: np.ndarray, src=None, src_dev_ptr: int = 0, src_words: int = 0) -> None:
        """OR pieces {frame*3+comp, first word, first src word, words} of one
        source buffer (device pointer or host array) into the scans."""
        pc = np.ascontiguousarray(pieces, np.uint64).reshape(-1, 4)
        if src_dev_ptr:
            _check(self.lib.mij_assemble_pieces(self.h_, src_dev_ptr, src_words, 1, _ptr(pc), pc.shape[0]),
                   "assemble_pieces")
        else:
            w = np.ascontiguousarray(src).view(np.uint32).reshape(-1)
            _check(self.lib.mij_assemble_pieces(self.h_, _ptr(w), w.size, 0, _ptr(pc), pc.shape[0]),
                   "assemble_pieces")

    # ---- the device-resident band protocol (all pointers device memory) ----
    def stream_ptr(self) -> int:
        """the batch's HIP stream (hipStream_t), for torch.cuda.ExternalStream"""
        return int(self.lib.mij_batch_stream(self.h_) or 0)

    def set_stream(self, stream_ptr: int) -> None:
        """enqueue on another HIP stream from now on (0: the batch's own);
        ordered after the work enqueued before (mij_batch_set_stream)"""
        _check(self.lib.mij_batch_set_stream(self.h_, stream_ptr or None), "set_stream")

    def band_analyze_async(self, n: int, d_last: int) -> None:
        _check(self.lib.mij_band_analyze_async(self.h_, n, d_last), "band_analyze_async")

    def band_histograms_async(self, n: int, d_prev: int, d_hist: int) -> None:
        _check(self.lib.mij_band_histograms_async(self.h_, n, d_prev, d_hist), "band_histograms_async")

    def band_tables_async(self, n: int, d_ghist: int, d_bound: int) -> None:
        """tables from the summed histograms; an upper bound of the band's
        words -> d_bound (uint64 [1] device buffer)"""
        _check(self.lib.mij_band_tables_async(self.h_, n, d_ghist, d_bound), "band_tables_async")

    def band_pack_async(self, n: int, d_bits: int) -> None:
        """the band packed from bit 0; d_bits: uint64 [3n + 1] device buffer
        (bits per scan, then the word count)"""
        _check(self.lib.mij_band_pack_async(self.h_, n, d_bits), "band_pack_async")

    def band_words_async(self, n: int, d_dst: int, cap_words: int) -> None:
        _check(self.lib.mij_band_words_async(self.h_, n, d_dst, cap_words), "band_words_async")

    def assemble_tables_async(self, n: int, d_ghist: int) -> None:
        _check(self.lib.mij_assemble_tables_async(self.h_, n, d_ghist), "assemble_tables_async")

    def assemble_async(self, n: int, d_allbits: int, world: int, d_src: int, stride_words: int) -> None:
        _check(self.lib.mij_assemble_async(self.h_, n, d_allbits, world, d_src, stride_words), "assemble_async")

    def band_stuff_async(self, n: int, d_allbits: int, world: int, rank: int, d_rec: int, d_total: int,
                         d_dst: int, cap: int) -> None:
        """distributed emission: this band's whole bytes of the final scans,
        stuffed, into d_dst; records [n, 3, 4] u64 and the total to d_rec / d_total"""
        _check(self.lib.mij_band_stuff_async(self.h_, n, d_allbits, world, rank, d_rec, d_total, d_dst, cap),
               "band_stuff_async")

    def copy_to_host_async(self, h_dst: int, d_src: int, nbytes: int) -> None:
        """device -> pinned host bytes on the batch's stream"""
        _check(self.lib.mij_copy_to_host_async(self.h_, h_dst, d_src, nbytes), "copy_to_host_async")

    def assemble_stuffed_async(self, n: int, d_allrec: int, world: int, d_src: int, stride: int) -> None:
        _check(self.lib.mij_assemble_stuffed_async(self.h_, n, d_allrec, world, d_src, stride),
               "assemble_stuffed_async")

    def assemble_begin(self, n: int, hist: np.ndarray) -> None:
        h = np.ascontiguousarray(hist, np.uint32).reshape(n, 4, 257)
        _check(self.lib.mij_assemble_begin(self.h_, n, _ptr(h)), "assemble_begin")

    def assemble_words(self, frame: int, comp: int, first_word: int, words=None,
                       src_dev_ptr: int = 0, nwords: int = 0) -> None:
        if src_dev_ptr:
            _check(self.lib.mij_assemble_words(self.h_, frame, comp, first_word, src_dev_ptr,
                                               nwords, 1), "assemble_words")
        else:
            w = np.ascontiguousarray(words, np.uint32)
            _check(self.lib.mij_assemble_words(self.h_, frame, comp, first_word, _ptr(w), w.size, 0),
                   "assemble_words")

    def assemble_end(self, n: int, total_bits: np.ndarray) -> None:
        t = np.ascontiguousarray(total_bits, np.uint64).reshape(n, 3)
        _check(self.lib.mij_assemble_end(self.h_, n, _ptr(t)), "assemble_end")


# ---- PPM ingest (utils/original.c:294-365 rules) and the streaming encoder ----

def ppm_header(path: str):
    """(width, height, pixel data offset) of a P6 file; raises MijError with
    the reference reader's message class (MIJ_EPPM / MIJ_EIO) otherwise."""
    w, h, off = C.c_int(0), C.c_int(0), C.c_longlong(0)
    _check(load().mij_ppm_header(path.encode(), C.byref(w), C.byref(h), C.byref(off)),
           f"ppm_header({path})")
    return w.value, h.value, off.value


def ppm_read(path: str, to_bgr: bool = False) -> np.ndarray:
    w, h, _ = ppm_header(path)
    out = np.zeros((h, w, 3), np.uint8)
    _check(load().mij_ppm_read(path.encode(), _ptr(out), out.nbytes, 3 * w, int(to_bgr)),
           f"ppm_read({path})")
    return out


class Stream:
    """mij_stream: PPM files / RGB frames -> JPEG through two device batches
    in ping-pong (include/mijpeg.h)."""
    STATS = ["wall_s", "read_s", "write_s", "gpu_s", "frames", "bytes_in", "bytes_out"]

    def __init__(self, w: int, h: int, chunk: int, quality: int = 50, device: int = 0,
                 threads: int = 0):
        self.lib = load()
        self.w, self.h = w, h
        self.h_ = self.lib.mij_stream_create(device, w, h, chunk, quality, threads)
        if not self.h_:
            raise MijError(f"mij_stream_create failed: "
                           f"{self.lib.mij_strerror(self.lib.mij_last_error()).decode()}")

    def close(self) -> None:
        if self.h_:
            self.lib.mij_stream_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode_files(self, ins, outs) -> None:
        n = len(ins)
        a = (C.c_char_p * n)(*[s.encode() for s in ins])
        b = (C.c_char_p * n)(*[s.encode() for s in outs])
        failed = C.c_int(-1)
        rc = self.lib.mij_stream_encode_files(self.h_, a, b, n, C.byref(failed))
        if rc:
            raise MijError(f"stream_encode_files: {self.lib.mij_strerror(rc).decode()} ({rc}), "
                           f"file {failed.value}")

    def encode_frames(self, frames_rgb) -> list:
        n = len(frames_rgb)
        frames = [np.ascontiguousarray(f, np.uint8) for f in frames_rgb]
        cap = max_jpg_bytes(self.w, self.h)
        outs = [np.zeros(cap, np.uint8) for _ in range(n)]
        ins = (C.c_void_p * n)(*[_ptr(f) for f in frames])
        ops = (C.c_void_p * n)(*[_ptr(o) for o in outs])
        caps = (C.c_size_t * n)(*([cap] * n))
        lens = (C.c_size_t * n)()
        _check(self.lib.mij_stream_encode_frames(self.h_, ins, n, ops, caps, lens), "stream_encode_frames")
        return [o[:lens[i]].tobytes() for i, o in enumerate(outs)]

    def stats(self) -> dict:
        v = np.zeros(len(self.STATS), np.float64)
        _check(self.lib.mij_stream_stats(self.h_, _ptr(v), len(v)), "stream_stats")
        return dict(zip(self.STATS, [float(x) for x in v]))


def probe_mfma(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    A = np.ascontiguousarray(A, np.int8).reshape(64, 16)
    B = np.ascontiguousarray(B, np.int8).reshape(64, 16)
    D = np.zeros((64, 4), np.int32)
    _check(load().mij_probe_mfma(_ptr(A), _ptr(B), _ptr(D)), "probe_mfma")
    return D


def colour_lut() -> np.ndarray:
    out = np.zeros(3 * 1024, np.uint32)
    _check(load().mij_colour_lut(_ptr(out)), "colour_lut")
    return out.reshape(3, 1024)


# ---- change detector (reference main/brain.c) ------

class Pair(C.Structure):
    """pair_t, reference include/structs.h:20-22."""
    _fields_ = [("beg", C.c_int), ("end", C.c_int), ("row", C.c_int), ("done", C.c_int)]


def _area_list(outs, n: int) -> list:
    return [(a.x, a.y, a.w, a.h) for a in outs[:max(0, min(n, 100))]]


class Detector:
    """Device-resident change detector over frames of w x h BGR pixels.

    step(frame) = the reference's subsample + compare (main.c:140-143) in one
    kernel launch plus the host-side area joining; store() = main.c:161.
    Returns (count, areas) with the count the reference's compare returns."""

    def __init__(self, w: int, h: int, device: int = 0):
        self.lib = load()
        self.w, self.h = w, h
        self.h_ = self.lib.mij_detector_create(device, w, h)
        if not self.h_:
            raise MijError("mij_detector_create failed: "
                           f"{self.lib.mij_strerror(self.lib.mij_last_error()).decode()}")
        self._outs = (Area * 100)()

    def close(self) -> None:
        if self.h_:
            self.lib.mij_detector_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, frame_bgr: np.ndarray, pitch: int = 0) -> int:
        """Copies a host frame ((h, w, 3), or (h, pitch) bytes rows) to the
        detector's frame buffer; returns its device address."""
        f = np.ascontiguousarray(frame_bgr, np.uint8)
        if pitch:
            assert f.shape == (self.h, pitch), f.shape
        else:
            assert f.shape == (self.h, self.w, 3), f.shape
        ptr = C.c_void_p()
        _check(self.lib.mij_detector_upload(self.h_, _ptr(f), pitch, C.byref(ptr)), "detector_upload")
        return ptr.value

    def subsample(self, dev_ptr: int, pitch: int | None = None) -> None:
        _check(self.lib.mij_detector_subsample(self.h_, dev_ptr, pitch or 3 * self.w),
               "detector_subsample")

    def compare(self):
        n = C.c_int()
        _check(self.lib.mij_detector_compare(self.h_, self._outs, C.byref(n)), "detector_compare")
        return n.value, _area_list(self._outs, n.value)

    def step(self, dev_ptr: int, pitch: int | None = None):
        n = C.c_int()
        _check(self.lib.mij_detector_step(self.h_, dev_ptr, pitch or 3 * self.w, self._outs,
                                          C.byref(n)), "detector_step")
        return n.value, _area_list(self._outs, n.value)

    def launch(self, dev_ptr: int, pitch: int | None = None) -> None:
        """The step's kernel alone, asynchronous (timing)."""
        _check(self.lib.mij_detector_launch(self.h_, dev_ptr, pitch or 3 * self.w), "detector_launch")

    def stream(self) -> int:
        return int(self.lib.mij_detector_stream(self.h_) or 0)

    def store(self) -> None:
        _check(self.lib.mij_detector_store(self.h_), "detector_store")

    def plane(self, which: int = 0) -> np.ndarray:
        out = np.zeros((self.h // 4, self.w // 4, 3), np.uint8)
        _check(self.lib.mij_detector_get_plane(self.h_, which, _ptr(out)), "detector_get_plane")
        return out

    def set_plane(self, which: int, rgb: np.ndarray) -> None:
        rgb = np.ascontiguousarray(rgb, np.uint8)
        assert rgb.shape == (self.h // 4, self.w // 4, 3), rgb.shape
        _check(self.lib.mij_detector_set_plane(self.h_, which, _ptr(rgb)), "detector_set_plane")

    def mask(self) -> np.ndarray:
        """Bit mask of the last compare as a bool array (h/4, w/4)."""
        words = C.c_int()
        _check(self.lib.mij_detector_mask(self.h_, None, 0, C.byref(words)), "detector_mask")
        m = np.zeros((self.h // 4, words.value), np.uint64)
        _check(self.lib.mij_detector_mask(self.h_, _ptr(m), m.size, C.byref(words)), "detector_mask")
        bits = np.unpackbits(m.view(np.uint8).reshape(self.h // 4, -1), axis=1, bitorder="little")
        return bits[:, :self.w // 4].astype(bool)


def drop_in_subsample(frame_bgr: np.ndarray) -> np.ndarray:
    """brain.h:7 subsample() through the drop-in entry point (f = NULL)."""
    lib = load()
    f = np.ascontiguousarray(frame_bgr, np.uint8)
    H, W = f.shape[:2]
    _check(lib.mij_set_input_stride(W), "set_input_stride")
    _check(lib.mij_set_frame_height(H), "set_frame_height")
    out = np.zeros((H // 4, W // 4, 3), np.uint8)
    lib.subsample(None, _ptr(f), _ptr(out))
    _check(lib.mij_last_error(), "subsample")
    return out


def drop_in_compare(sub: np.ndarray, saved: np.ndarray, W: int, H: int):
    """brain.h:9 compare() through the drop-in entry point."""
    lib = load()
    _check(lib.mij_set_input_stride(W), "set_input_stride")
    _check(lib.mij_set_frame_height(H), "set_frame_height")
    sub = np.ascontiguousarray(sub, np.uint8)
    saved = np.ascontiguousarray(saved, np.uint8)
    outs = (Area * 100)()
    diffs = (Pair * (2 * (W // 8)))()
    n = lib.compare(_ptr(sub), _ptr(saved), outs, diffs)
    _check(lib.mij_last_error(), "compare")
    return int(n), _area_list(outs, int(n))


def drop_in_enlarge_adjust(area, W: int, H: int):
    lib = load()
    _check(lib.mij_set_input_stride(W), "set_input_stride")
    _check(lib.mij_set_frame_height(H), "set_frame_height")
    a = Area(*area)
    lib.enlargeAdjust(C.byref(a))
    return (a.x, a.y, a.w, a.h)


# ---- round-trip verifier ---------------------------

class Decoder:
    """Baseline JFIF streams (the shape encoder.c:549-644 writes) -> the
    encoder's coefficient planes, entropy-decoded on the GPU."""

    def __init__(self, max_w: int, max_h: int, max_frames: int, device: int = 0):
        self.lib = load()
        self.h_ = self.lib.mij_decoder_create(device, max_w, max_h, max_frames)
        if not self.h_:
            raise MijError("mij_decoder_create failed: "
                           f"{self.lib.mij_strerror(self.lib.mij_last_error()).decode()}")

    def close(self) -> None:
        if self.h_:
            self.lib.mij_decoder_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, streams) -> None:
        n = len(streams)
        bufs = [np.frombuffer(s, np.uint8) for s in streams]
        ptrs = (C.c_void_p * n)(*[_ptr(b) for b in bufs])
        lens = (C.c_size_t * n)(*[len(s) for s in streams])
        _check(self.lib.mij_decoder_decode(self.h_, ptrs, lens, n), "decoder_decode")

    def passes(self) -> int:
        return int(self.lib.mij_decoder_passes(self.h_))

    def info(self, frame: int):
        w, h = C.c_int(), C.c_int()
        dqt = np.zeros(128, np.uint8)
        _check(self.lib.mij_decoder_info(self.h_, frame, C.byref(w), C.byref(h), _ptr(dqt)), "decoder_info")
        return w.value, h.value, dqt

    def coefs(self, frame: int):
        w, h, _ = self.info(frame)
        Y = np.zeros(w * h, np.int16)
        Cb = np.zeros(w * h // 4, np.int16)
        Cr = np.zeros(w * h // 4, np.int16)
        _check(self.lib.mij_decoder_coefs(self.h_, frame, _ptr(Y), _ptr(Cb), _ptr(Cr)), "decoder_coefs")
        return Y, Cb, Cr
