/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 * Thin C wrapper linked with the unmodified reference main/encoder.c into
 * oracle/_ref/libref_encoder.so.  It reproduces the caller contract of
 * main.c:144-152 (rgb_to_dct -> init_huffman -> write_jpg) on a caller-given
 * BGR frame with a runtime stride (see ref_shim.h).
 */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "encoder.h"

int ref_stride = 320;
extern const int64_t lookup_table[];

void ref_cos_bits(int64_t out[64]) { memcpy(out, lookup_table, 64 * sizeof(int64_t)); }

size_t ref_huff_size(void) { return sizeof(huff_code); }

/* Runs the three entry points; coefficient planes and tables are returned
 * through the caller's buffers so they can be compared field by field. */
size_t ref_encode(const uint8_t *bgr, int stride_px, int x, int y, int w, int h,
                  int16_t *Y, int16_t *Cb, int16_t *Cr, huff_code tables[4],
                  uint8_t *jpg) {
    area_t d = {x, y, w, h};
    ref_stride = stride_px;
    rgb_to_dct((uint8_t *)bgr, Y, Cb, Cr, d);
    init_huffman(Y, Cb, Cr, d, tables, tables + 2);
    FILE *f = fopen("/dev/null", "w");
    if (!f) return 0;
    size_t n = write_jpg(f, jpg, Y, Cb, Cr, d, tables, tables + 2);
    fclose(f);
    return n;
}

/* Stage-split variant for the CPU-baseline timing (same calls). */
void ref_stage_dct(const uint8_t *bgr, int stride_px, int x, int y, int w, int h,
                   int16_t *Y, int16_t *Cb, int16_t *Cr) {
    area_t d = {x, y, w, h};
    ref_stride = stride_px;
    rgb_to_dct((uint8_t *)bgr, Y, Cb, Cr, d);
}
