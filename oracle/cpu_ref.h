/*
 * oracle/cpu_ref.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference JPEG block-encode path
 * (MattiaDallaCosta/JPEG-encoder-decoder, main/encoder.c), written from the
 * behaviour documented in SURVEY.md §8(a).  It is the checker that the HIP
 * product path in jpeg-encoder-decoder_amd/ is compared against; nothing in the
 * product links or calls it.  Pinned against the compiled reference
 * (oracle/_ref, built by oracle/Makefile from /root/reference sources) and the
 * committed golden fixtures in tests/golden/.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field order as the reference's huff_code (include/structs.h:5-13);
 * the order matters for the sentinel aliasing in encoder.c:277. */
typedef struct {
    int sym_freq[257];
    int code_len[257];
    int next[257];
    int code_len_freq[32];
    int sym_sorted[256];
    int sym_code_len[256];
    int sym_code[256];
} cref_huff;

typedef struct { int x, y, w, h; } cref_area;   /* structs.h:15-18 */

/* original.c:504-509 quality scaling; quality 50 reproduces encoder.c:18-36. */
void cref_quality_tables(int quality, int luma_q[64], int chroma_q[64]);

/* encoder.c:158-178 (+121-150, 81-112, 65-70).  `stride_px` replaces the
 * compile-time WIDTH of define.h:3. */
void cref_rgb_to_dct(const uint8_t *bgr, int stride_px, int16_t *Y, int16_t *Cb,
                     int16_t *Cr, cref_area d, const int luma_q[64],
                     const int chroma_q[64]);

/* encoder.c:360-381 (+180-358). */
int cref_init_huffman(const int16_t *Y, const int16_t *Cb, const int16_t *Cr,
                      cref_area d, cref_huff luma[2], cref_huff chroma[2]);

/* encoder.c:180-301 for one histogram of symbols 0..255 (+ the reserved
 * sym_freq[256] = 1 of :367).  0 on success. */
int cref_build_table(const uint32_t freq[256], cref_huff *hc);

/* encoder.c:549-644 (+383-532).  Writes into jpg, returns byte count. */
size_t cref_write_jpg(uint8_t *jpg, const int16_t *Y, const int16_t *Cb,
                      const int16_t *Cr, cref_area d, const cref_huff luma[2],
                      const cref_huff chroma[2], const int luma_q[64],
                      const int chroma_q[64]);

/* Whole path: rgb_to_dct -> init_huffman -> write_jpg (main.c:144-152).
 * Returns bytes written to jpg (capacity cap) or 0 on error. */
size_t cref_encode(const uint8_t *bgr, int stride_px, cref_area d, int quality,
                   uint8_t *jpg, size_t cap);

/* Un-quantized, un-zigzagged FP64 DCT value of one 8x8 block exactly as
 * encoder.c:87-106 computes it (for tolerance studies). */
void cref_dct_block_f64(const uint8_t *pix, int gap, double out[64]);

/* Colour conversion of one BGR pixel exactly as encoder.c:133-135. */
void cref_pixel_ycc(uint8_t b, uint8_t g, uint8_t r, uint8_t out[3]);

/* The 64 cosines of encoder.c:8-16 (as raw IEEE-754 bit patterns). */
void cref_cos_bits(int64_t out[64]);

/* Number of worst-case bytes a frame of w*h pixels can need. */
size_t cref_max_jpg_bytes(int w, int h);

/* ---- change detector (main/brain.c) ------------------------------------ */

typedef struct { int beg, end, row, done; } cref_run;   /* structs.h:20-22 pair_t */

/* brain.c:16-45: 4x4 box average of a w x h BGR frame (stride w) into a
 * (w/4) x (h/4) RGB plane (sub[3i] = R average). */
void cref_subsample(const uint8_t *bgr, int w, int h, uint8_t *sub);

/* brain.c:104-233 (+64-102, 240-261): compares two (w/4) x (h/4) RGB planes
 * and writes up to 100 areas into outs (100 entries); returns the count the
 * reference returns (its uint8_t). */
int cref_compare(const uint8_t *sub, const uint8_t *saved, int w, int h, cref_area outs[100]);

/* brain.c:240-261 for a w x h frame. */
void cref_enlarge_adjust(cref_area *a, int w, int h);

#ifdef __cplusplus
}
#endif
