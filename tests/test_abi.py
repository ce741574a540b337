"""CPU tests of the C-ABI boundary: the library builds for gfx950, loads, and
exports every function include/mijpeg.h declares with the reference's
signatures (encoder.h:10-12) and struct layouts (structs.h:5-18).  No GPU
compute is attempted here."""
import ctypes as C
import os
import re
import subprocess

import pytest

import mijpeg

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mijpeg.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", src)
    return sorted(set(n for n in names if n not in ("sizeof",)))


def test_header_declares_reference_entry_points():
    names = declared_functions()
    for fn in ("rgb_to_dct", "init_huffman", "write_jpg"):
        assert fn in names
    src = open(HEADER).read()
    # exact reference prototypes (encoder.h:10-12), modulo whitespace
    norm = re.sub(r"\s+", " ", src)
    assert "void rgb_to_dct(uint8_t *in, int16_t *Y, int16_t *Cb, int16_t *Cr, area_t dims);" in norm
    assert ("void init_huffman(int16_t *Y, int16_t *Cb, int16_t *Cr, area_t dims, "
            "huff_code Luma[2], huff_code Chroma[2]);") in norm
    assert ("size_t write_jpg(FILE *f, uint8_t *jpg, int16_t *Y, int16_t *Cb, int16_t *Cr, "
            "area_t dims, huff_code Luma[2], huff_code Chroma[2]);") in norm


def test_library_exports_every_declared_symbol():
    lib = mijpeg.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared_functions()) <= set(mijpeg.EXPORTS)


def test_code_object_targets_gfx950():
    blob = open(mijpeg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle of the code object
    assert mijpeg.load().mij_build_target() == b"gfx950"


def test_struct_layouts():
    assert C.sizeof(mijpeg.Huff) == 6284
    assert mijpeg.Huff.sym_sorted.offset + 256 * 4 == mijpeg.Huff.sym_code_len.offset
    assert C.sizeof(mijpeg.Area) == 16


def test_max_jpg_bytes_bounds():
    assert mijpeg.max_jpg_bytes(64, 64) >= 566
    assert mijpeg.max_jpg_bytes(15, 16) == 0
    assert mijpeg.max_jpg_bytes(0, 16) == 0


def test_validation_precedes_device_use():
    lib = mijpeg.load()
    assert lib.mij_set_quality(0) == 1 and lib.mij_set_quality(101) == 1
    assert lib.mij_set_input_stride(3) == 1
    assert not lib.mij_batch_create(0, 30, 16, 1, 50)
    assert lib.mij_last_error() == 1
    # the failure's text names what was wrong (mij_last_message)
    assert b"bad geometry 30x16" in lib.mij_last_message()


def test_c_host_builds():
    pkg = os.path.dirname(mijpeg.LIB_PATH)
    subprocess.check_call(["make", "-s", "-C", pkg, "host/encode_ppm"])
    assert os.access(os.path.join(pkg, "host", "encode_ppm"), os.X_OK)


MAIN_LOOP_C = r"""
/* main.c:25-37 buffers and :136-163 loop body, as the reference writes them,
 * compiled against mijpeg.h in place of brain.h / encoder.h / structs.h */
#include "mijpeg.h"
#define WIDTH 320
#define HEIGHT 240
#define PIX_LEN WIDTH*HEIGHT
static uint8_t raw[3*PIX_LEN], sub[3*PIX_LEN/16], saved[3*PIX_LEN/16], jpg[3*PIX_LEN];
static int16_t ordered_dct_Y[PIX_LEN], ordered_dct_Cb[PIX_LEN/4], ordered_dct_Cr[PIX_LEN/4];
static area_t diffDims[100];
static pair_t differences[2][WIDTH/8];
static huff_code Luma[2], Chroma[2];
int main(void) {
  subsample(NULL, raw, sub);
  store(sub, saved);
  int different = compare(sub, saved, diffDims, differences);
  for (int i = 0; i < different; i++) {
    enlargeAdjust(&diffDims[i]);
    rgb_to_dct(raw, ordered_dct_Y, ordered_dct_Cb, ordered_dct_Cr, diffDims[i]);
    init_huffman(ordered_dct_Y, ordered_dct_Cb, ordered_dct_Cr, diffDims[i], Luma, Chroma);
    FILE *f = fopen("/dev/null", "w");
    (void)write_jpg(f, jpg, ordered_dct_Y, ordered_dct_Cb, ordered_dct_Cr, diffDims[i], Luma, Chroma);
    fclose(f);
  }
  return 0;
}
"""


def test_reference_main_loop_compiles_and_links(tmp_path):
    """The reference's caller (brain.h + encoder.h calls with its own buffer
    types, main.c:25-37/136-163) compiles warning-free against mijpeg.h and
    links against libmijpeg.so (nothing is run: no GPU here)."""
    src = tmp_path / "main_loop.c"
    src.write_text(MAIN_LOOP_C)
    pkg = os.path.dirname(mijpeg.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                           str(src), "-L", pkg, "-lmijpeg", "-o", str(tmp_path / "main_loop")])


def test_division_magic(tmp_path):
    """K1 computes (frame, tile row, tile column) of a tile index with a
    multiply-high by a host-built magic number (mij_divmagic.h): checked
    against integer division over every divisor < 4096 and 2000 random ones."""
    exe = str(tmp_path / "div_check")
    subprocess.check_call(["g++", "-O2", "-I" + os.path.join(REPO, "jpeg-encoder-decoder_amd", "csrc"),
                           "-o", exe, os.path.join(REPO, "tests", "div_check.cpp")])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")


def test_fault_hook_is_not_public_abi():
    """The stale-ticket fault injection is a test-only entry point
    (csrc/mij_testing.h): exported for the GPU tests, absent from the public
    header and from the option enum."""
    src = open(HEADER).read()
    assert "FAULT" not in src and "mij_test_" not in src
    assert "fault_ticket" not in mijpeg.OPTIONS
    assert hasattr(mijpeg.load(), "mij_test_stale_ticket")
