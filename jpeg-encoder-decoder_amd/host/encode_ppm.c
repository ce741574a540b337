/*
 * encode_ppm.c -- C host for libmijpeg.so.
 *
 * Reproduces the reference caller's sequence (main.c:144-152:
 * rgb_to_dct -> init_huffman -> write_jpg on caller-owned buffers) on a PPM
 * file, with the PPM checks of utils/original.c:294-365 (P6, '#' comments,
 * depth 255, width/height multiples of 16).  The PPM is RGB; the encoder's
 * input convention is BGR888 (encoder.c:133), so channels are swapped on load.
 *
 *   encode_ppm <in.ppm> <out.jpg> [quality] [x y w h] [--fused]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mijpeg.h"

static uint8_t *read_ppm_bgr(const char *path, int *w, int *h) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); return NULL; }
    char magic[3] = {0};
    if (fread(magic, 1, 2, f) != 2 || strcmp(magic, "P6")) {
        fprintf(stderr, "%s: not a P6 PPM\n", path);
        fclose(f);
        return NULL;
    }
    int vals[3], n = 0;
    while (n < 3) {
        int c = fgetc(f);
        if (c == EOF) break;
        if (c == '#') { while (c != '\n' && c != EOF) c = fgetc(f); continue; }
        if (c == ' ' || c == '\t' || c == '\n' || c == '\r') continue;
        ungetc(c, f);
        if (fscanf(f, "%d", &vals[n]) != 1) break;
        n++;
    }
    fgetc(f); /* single whitespace after the depth */
    if (n != 3 || vals[2] != 255 || vals[0] % 16 || vals[1] % 16 || vals[0] <= 0 || vals[1] <= 0) {
        fprintf(stderr, "%s: need depth 255 and dimensions multiple of 16\n", path);
        fclose(f);
        return NULL;
    }
    *w = vals[0];
    *h = vals[1];
    size_t np = (size_t)*w * *h;
    uint8_t *px = malloc(np * 3);
    if (!px || fread(px, 3, np, f) != np) {
        fprintf(stderr, "%s: truncated pixel data\n", path);
        free(px);
        fclose(f);
        return NULL;
    }
    fclose(f);
    for (size_t i = 0; i < np; i++) { uint8_t t = px[3 * i]; px[3 * i] = px[3 * i + 2]; px[3 * i + 2] = t; }
    return px;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <in.ppm> <out.jpg> [quality] [x y w h] [--fused]\n", argv[0]);
        return 2;
    }
    int fused = 0;
    if (!strcmp(argv[argc - 1], "--fused")) { fused = 1; argc--; }
    int W, H;
    uint8_t *raw = read_ppm_bgr(argv[1], &W, &H);
    if (!raw) return 1;
    int quality = argc > 3 ? atoi(argv[3]) : 50;
    area_t dims = {0, 0, W, H};
    if (argc > 7) { dims.x = atoi(argv[4]); dims.y = atoi(argv[5]); dims.w = atoi(argv[6]); dims.h = atoi(argv[7]); }
    size_t cap = mij_max_jpg_bytes(dims.w, dims.h);
    uint8_t *jpg = malloc(cap ? cap : 1);
    size_t size = 0;
    if (fused) {
        if (mij_encode(raw, W, dims, quality, jpg, cap, &size) != MIJ_OK) return 1;
        FILE *f = fopen(argv[2], "wb");
        if (!f || fwrite(jpg, 1, size, f) != size) { perror(argv[2]); return 1; }
        fclose(f);
    } else {
        /* caller-owned buffers as in main.c:25-37 */
        int16_t *Y = malloc(sizeof(int16_t) * dims.w * dims.h);
        int16_t *Cb = malloc(sizeof(int16_t) * dims.w * dims.h / 4);
        int16_t *Cr = malloc(sizeof(int16_t) * dims.w * dims.h / 4);
        huff_code Luma[2], Chroma[2];
        mij_set_input_stride(W); /* define.h:3 WIDTH, now a runtime value */
        if (mij_set_quality(quality) != MIJ_OK) return 1;
        rgb_to_dct(raw, Y, Cb, Cr, dims);
        if (mij_last_error()) return 1;
        init_huffman(Y, Cb, Cr, dims, Luma, Chroma);
        if (mij_last_error()) return 1;
        FILE *f = fopen(argv[2], "wb");
        if (!f) { perror(argv[2]); return 1; }
        size = write_jpg(f, jpg, Y, Cb, Cr, dims, Luma, Chroma);
        fclose(f);
        if (!size) return 1;
        free(Y); free(Cb); free(Cr);
    }
    printf("%s: %dx%d region (%d,%d %dx%d) Q=%d -> %zu bytes\n", argv[2], W, H, dims.x, dims.y,
           dims.w, dims.h, quality, size);
    free(raw);
    free(jpg);
    return 0;
}
