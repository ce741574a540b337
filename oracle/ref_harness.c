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

/* The reference's caller shape on a file (main.c:131-155 with the camera
 * replaced by a PPM file): read a binary P6 file (RGB, depth 255, w and h
 * multiples of 16), swap it to the encoder's B, G, R (brain.c:25-42), run
 * the three entry points and let write_jpg write the .jpg file itself
 * (fputc per byte, as on the SD card).  Used as the host-fed stream's CPU
 * baseline (bench.py --workload stream).  Returns the .jpg size, 0 on error.
 * Scratch buffers are the caller's (main.c keeps them static). */
static int ppm_int(FILE *f, int *v) {
    int c = fgetc(f);
    for (;;) { /* whitespace and '#' comments between header fields */
        while (c == ' ' || c == '\t' || c == '\n' || c == '\r') c = fgetc(f);
        if (c != '#') break;
        while (c != '\n' && c != EOF) c = fgetc(f);
    }
    if (c < '0' || c > '9') return -1;
    *v = 0;
    while (c >= '0' && c <= '9') { *v = *v * 10 + (c - '0'); c = fgetc(f); }
    return 0; /* the single whitespace byte after the field is consumed */
}

size_t ref_encode_file(const char *ppm_path, const char *jpg_path, uint8_t *bgr, size_t bgr_cap,
                       int16_t *Y, int16_t *Cb, int16_t *Cr, uint8_t *jpg) {
    FILE *f = fopen(ppm_path, "rb");
    if (!f) return 0;
    int w, h, depth;
    if (fgetc(f) != 'P' || fgetc(f) != '6' || ppm_int(f, &w) || ppm_int(f, &h) || ppm_int(f, &depth) ||
        depth != 255 || w <= 0 || h <= 0 || (w % 16) || (h % 16) || (size_t)w * h * 3 > bgr_cap) {
        fclose(f);
        return 0;
    }
    const size_t n = (size_t)w * h * 3;
    if (fread(bgr, 1, n, f) != n) {
        fclose(f);
        return 0;
    }
    fclose(f);
    for (size_t i = 0; i < n; i += 3) { /* R, G, B -> B, G, R */
        const uint8_t t = bgr[i];
        bgr[i] = bgr[i + 2];
        bgr[i + 2] = t;
    }
    huff_code tables[4];
    area_t d = {0, 0, w, h};
    ref_stride = w;
    rgb_to_dct(bgr, Y, Cb, Cr, d);
    init_huffman(Y, Cb, Cr, d, tables, tables + 2);
    FILE *o = fopen(jpg_path, "wb");
    if (!o) return 0;
    const size_t len = write_jpg(o, jpg, Y, Cb, Cr, d, tables, tables + 2);
    fclose(o);
    return len;
}
