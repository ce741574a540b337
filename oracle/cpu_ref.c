/*
 * oracle/cpu_ref.c -- TEST INFRASTRUCTURE ONLY (see cpu_ref.h).
 *
 * A plain-C restatement of the reference encoder's arithmetic, written from
 * SURVEY.md §8(a) and cited line by line against
 * MattiaDallaCosta/JPEG-encoder-decoder main/encoder.c.  Every floating-point
 * expression keeps the reference's evaluation order, in IEEE double with no
 * FMA contraction (build with -ffp-contract=off), because the output depends
 * on FP64 last-ulp rounding (encoder.c:108, :133-135).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 */
#include "cpu_ref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- constant tables ---------------------------------------------------- */

/* encoder.c:18-26 */
static const int k_luma_q[64] = {
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
/* encoder.c:28-36 */
static const int k_chroma_q[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
/* encoder.c:38-46: zigzag position -> raster index inside the 8x8 block */
static const int k_zigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* encoder.c:8-16 stores cos((2t+1) f pi / 16) as bit patterns; they were
 * produced by utils/lookup.c:10 with exactly this expression. */
static double g_cos[64];
static int g_cos_ready = 0;
static void init_cos(void) {
    if (g_cos_ready) return;
    for (int i = 0; i < 64; i++)
        g_cos[i] = cos((double)(2 * (i / 8) + 1) * (i % 8) * M_PI / 16);
    g_cos_ready = 1;
}

void cref_cos_bits(int64_t out[64]) {
    init_cos();
    memcpy(out, g_cos, sizeof(g_cos));
}

/* original.c:504-509: q' = (int) CLIP((100-Q)/50.0 * q, 1, 255) */
void cref_quality_tables(int quality, int luma_q[64], int chroma_q[64]) {
    for (int i = 0; i < 64; i++) {
        double l = (100 - quality) / 50.0 * k_luma_q[i];
        double c = (100 - quality) / 50.0 * k_chroma_q[i];
        l = l < 1 ? 1 : l; l = l > 255 ? 255 : l;
        c = c < 1 ? 1 : c; c = c > 255 ? 255 : c;
        luma_q[i] = (int)l;
        chroma_q[i] = (int)c;
    }
}

/* ---- colour conversion: encoder.c:133-135 ------------------------------ */

void cref_pixel_ycc(uint8_t b, uint8_t g, uint8_t r, uint8_t out[3]) {
    /* left-to-right double evaluation, then truncation to uint8_t */
    double y = 0.299 * r + 0.587 * g + 0.114 * b;
    double cb = 128 - 0.168736 * r - 0.331264 * g + 0.5 * b;
    double cr = 128 + 0.5 * r - 0.418688 * g - 0.081312 * b;
    out[0] = (uint8_t)(int)y;
    out[1] = (uint8_t)(int)cb;
    out[2] = (uint8_t)(int)cr;
}

/* ---- DCT: encoder.c:81-112 --------------------------------------------- */

void cref_dct_block_f64(const uint8_t *pix, int gap, double out[64]) {
    init_cos();
    double col[64]; /* col[x*8 + v]: 1-D transform down column x (:87-94) */
    for (int x = 0; x < 8; x++)
        for (int v = 0; v < 8; v++) {
            double acc = 0;
            for (int y = 0; y < 8; y++)
                acc += (pix[y * gap + x] - 128) * g_cos[y * 8 + v];
            col[x * 8 + v] = acc;
        }
    for (int v = 0; v < 8; v++)          /* :98-106, output raster [v][u] */
        for (int u = 0; u < 8; u++) {
            double f = 0;
            for (int x = 0; x < 8; x++) f += col[x * 8 + v] * g_cos[x * 8 + u];
            if (u == 0) f *= M_SQRT1_2;
            if (v == 0) f *= M_SQRT1_2;
            f /= 4;
            out[v * 8 + u] = f;
        }
}

static void dct_quant_zigzag(const uint8_t *pix, int gap, int16_t *dst,
                             const int q[64]) {
    double f[64];
    int16_t raster[64];
    cref_dct_block_f64(pix, gap, f);
    for (int k = 0; k < 64; k++) {
        int16_t t = (int16_t)(int)(f[k] / q[k]); /* :108 trunc */
        raster[k] = t < -2048 ? -2048 : (t > 2047 ? 2047 : t); /* :109 */
    }
    for (int i = 0; i < 64; i++) dst[i] = raster[k_zigzag[i]]; /* :65-70 */
}

/* ---- per-MCU driver: encoder.c:121-150, frame driver :158-178 ---------- */

static void mcu(const uint8_t *bgr, int stride, int16_t *Y, int16_t *Cb,
                int16_t *Cr, int mx, int my, cref_area d, const int *lq,
                const int *cq) {
    uint8_t luma[256], cbf[256], crf[256], cbs[64], crs[64];
    for (int l = 0; l < 16; l++)
        for (int r = 0; r < 16; r++) {
            size_t idx = 3 * ((size_t)(my * 16 + d.y + l) * stride + mx * 16 +
                              d.x + r);
            uint8_t o[3];
            cref_pixel_ycc(bgr[idx], bgr[idx + 1], bgr[idx + 2], o);
            luma[l * 16 + r] = o[0];
            cbf[l * 16 + r] = o[1];
            crf[l * 16 + r] = o[2];
        }
    /* :136-138 -- integer floor average of each 2x2 */
    for (int l = 0; l < 8; l++)
        for (int r = 0; r < 8; r++) {
            int a = (2 * l) * 16 + 2 * r;
            cbs[l * 8 + r] = (cbf[a] + cbf[a + 1] + cbf[a + 16] + cbf[a + 17]) / 4;
            crs[l * 8 + r] = (crf[a] + crf[a + 1] + crf[a + 16] + crf[a + 17]) / 4;
        }
    int bw = d.w / 8; /* luma blocks per row, :144 */
    for (int iv = 0; iv < 2; iv++)
        for (int ih = 0; ih < 2; ih++)
            dct_quant_zigzag(luma + iv * 128 + ih * 8, 16,
                             Y + ((size_t)(my * 2 + iv) * bw + mx * 2 + ih) * 64, lq);
    size_t c = ((size_t)my * (d.w / 16) + mx) * 64; /* :125 */
    dct_quant_zigzag(cbs, 8, Cb + c, cq);
    dct_quant_zigzag(crs, 8, Cr + c, cq);
}

void cref_rgb_to_dct(const uint8_t *bgr, int stride_px, int16_t *Y, int16_t *Cb,
                     int16_t *Cr, cref_area d, const int luma_q[64],
                     const int chroma_q[64]) {
    int mw = d.w / 16, mh = d.h / 16;
    for (int my = 0; my < mh; my++)
        for (int mx = 0; mx < mw; mx++)
            mcu(bgr, stride_px, Y, Cb, Cr, mx, my, d, luma_q, chroma_q);
    /* :168-177 DC differencing along block-raster order, per component */
    int nY = d.w * d.h / 64, nC = d.w * d.h / 256;
    int16_t prev = 0;
    for (int i = 0; i < nY; i++) {
        int16_t dc = Y[(size_t)i * 64];
        Y[(size_t)i * 64] = (int16_t)(dc - prev);
        prev = dc;
    }
    int16_t *planes[2] = {Cb, Cr};
    for (int p = 0; p < 2; p++) {
        prev = 0;
        for (int i = 0; i < nC; i++) {
            int16_t dc = planes[p][(size_t)i * 64];
            planes[p][(size_t)i * 64] = (int16_t)(dc - prev);
            prev = dc;
        }
    }
}

/* ---- symbol statistics: encoder.c:303-358 ------------------------------ */

static int magnitude_class(int v) { /* :303-313 */
    v = v < 0 ? -v : v;
    int c = 0;
    while (v > 0) { v >>= 1; c++; }
    return c;
}

/* Walks one block's AC run/size symbols in the order encoder.c:321-358 and
 * :462-502 visit them; emit(sym, value, ctx) is called for every symbol
 * (value only meaningful for run/size symbols). */
typedef void (*sym_fn)(int sym, int value, void *ctx);
static void walk_ac(const int16_t *blk, sym_fn emit, void *ctx) {
    int last = 63;
    while (last > 0 && blk[last] == 0) last--;
    int zeros = 0;
    for (int k = 1; k <= last; k++) {
        if (blk[k] == 0) {
            if (++zeros == 16) { emit(0xF0, 0, ctx); zeros = 0; } /* ZRL */
            continue;
        }
        emit(((zeros << 4) & 0xF0) | (magnitude_class(blk[k]) & 0x0F), blk[k], ctx);
        zeros = 0;
    }
    if (last < 63) emit(0x00, 0, ctx); /* EOB */
}

static void count_sym(int sym, int value, void *ctx) {
    (void)value;
    ((int *)ctx)[sym]++;
}

/* ---- Huffman table construction: encoder.c:180-301 --------------------- */

static int build_table(cref_huff *hc) {
    for (int i = 0; i < 257; i++) { hc->code_len[i] = 0; hc->next[i] = -1; }
    for (;;) { /* :190-228 */
        /* v1: least frequency, ties to the highest index; v2: next least */
        int v1 = -1, v2 = -1;
        for (int i = 0; i < 257; i++) {
            int f = hc->sym_freq[i];
            if (!f) continue;
            if (v1 < 0 || f <= hc->sym_freq[v1]) { v2 = v1; v1 = i; }
            else if (v2 < 0 || f <= hc->sym_freq[v2]) v2 = i;
        }
        if (v2 < 0) break;
        hc->sym_freq[v1] += hc->sym_freq[v2];
        hc->sym_freq[v2] = 0;
        int s = v1;
        for (;;) { hc->code_len[s]++; if (hc->next[s] < 0) break; s = hc->next[s]; }
        hc->next[s] = v2;
        for (s = v2;; s = hc->next[s]) { hc->code_len[s]++; if (hc->next[s] < 0) break; }
    }
    int *clf = hc->code_len_freq;
    for (int i = 0; i < 32; i++) clf[i] = 0;
    for (int i = 0; i < 257; i++) {
        if (hc->code_len[i] >= 32) return -1; /* reference indexes past clf[31] (UB) */
        if (hc->code_len[i]) clf[hc->code_len[i]]++;
    }
    int n_live = 0;
    for (int i = 1; i < 32; i++) n_live += clf[i];
    if (n_live < 2) return -2; /* no real symbol: reference walks off clf[0] */
    /* :239-259 limit to 16 bits (JPEG Annex K.3 adjust) */
    int i = 31;
    for (;;) {
        if (clf[i] > 0) {
            int j = i - 1;
            do { j--; } while (clf[j] <= 0);
            clf[i] -= 2;
            clf[i - 1]++;
            clf[j + 1] += 2;
            clf[j]--;
            continue;
        }
        i--;
        if (i != 16) continue;
        while (clf[i] == 0) i--;
        clf[i]--; /* drop the reserved all-ones code point */
        break;
    }
    /* :262-268 symbols 0..255 ordered by (unlimited) code length, then value */
    for (int k = 0; k < 256; k++) hc->sym_sorted[k] = -1;
    int n = 0;
    for (int len = 1; len < 32; len++)
        for (int s = 0; s < 256; s++)
            if (hc->code_len[s] == len) hc->sym_sorted[n++] = s;
    /* :271-277 limited lengths in that order.  The reference then stores a 0
     * through sym_sorted[n] == -1, i.e. into sym_code_len[-1], which is the
     * last element of sym_sorted in the struct (structs.h:10-11): that
     * sentinel is what terminates :285-300.  Restated explicitly here. */
    for (int k = 0; k < 256; k++) hc->sym_code_len[k] = 0;
    int k = 0;
    for (int len = 1; len <= 16; len++)
        for (int c = 0; c < clf[len]; c++) hc->sym_code_len[hc->sym_sorted[k++]] = len;
    if (k >= 255) return -3; /* sentinel would alias a live entry */
    hc->sym_sorted[255] = 0;
    /* :280-300 canonical code assignment */
    for (int s = 0; s < 256; s++) hc->sym_code[s] = -1;
    int code = 0;
    for (int m = 0; m < k; m++) {
        int s = hc->sym_sorted[m];
        if (m > 0) {
            int prev_len = hc->sym_code_len[hc->sym_sorted[m - 1]];
            code <<= (hc->sym_code_len[s] - prev_len);
        }
        hc->sym_code[s] = code++;
    }
    return 0;
}

/* One table from a histogram of symbols 0..255 (encoder.c:180-301, with the
 * reserved count sym_freq[256] = 1 of :367); 0, or the error of build_table. */
int cref_build_table(const uint32_t freq[256], cref_huff *hc) {
    for (int i = 0; i < 256; i++) hc->sym_freq[i] = (int)freq[i];
    hc->sym_freq[256] = 1;
    return build_table(hc);
}

int cref_init_huffman(const int16_t *Y, const int16_t *Cb, const int16_t *Cr,
                      cref_area d, cref_huff luma[2], cref_huff chroma[2]) {
    cref_huff *t[4] = {&luma[0], &luma[1], &chroma[0], &chroma[1]};
    for (int j = 0; j < 4; j++) {
        memset(t[j]->sym_freq, 0, sizeof(t[j]->sym_freq));
        t[j]->sym_freq[256] = 1; /* :367 reserved code point */
    }
    size_t nY = (size_t)d.w * d.h / 64, nC = nY / 4;
    const int16_t *plane[3] = {Y, Cb, Cr};
    size_t nb[3] = {nY, nC, nC};
    for (int p = 0; p < 3; p++) {
        cref_huff *dc = p ? &chroma[0] : &luma[0];
        cref_huff *ac = p ? &chroma[1] : &luma[1];
        for (size_t b = 0; b < nb[p]; b++) {
            const int16_t *blk = plane[p] + b * 64;
            dc->sym_freq[magnitude_class(blk[0])]++; /* :315-319 */
            walk_ac(blk, count_sym, ac->sym_freq);   /* :321-358 */
        }
    }
    for (int j = 0; j < 4; j++) /* :377-380 */
        if (build_table(t[j])) return -1;
    return 0;
}

/* ---- bitstream: encoder.c:383-502 -------------------------------------- */

typedef struct {
    uint8_t *out;
    size_t n;
    uint32_t acc; /* pending bits, right-aligned */
    int nacc;
    const cref_huff *ac;
} bitw;

static void put_bits(bitw *w, uint32_t v, int len) { /* :385-423 */
    for (int i = len - 1; i >= 0; i--) {
        w->acc = (w->acc << 1) | ((v >> i) & 1);
        if (++w->nacc == 8) {
            uint8_t byte = (uint8_t)w->acc;
            w->out[w->n++] = byte;
            if (byte == 0xFF) w->out[w->n++] = 0x00; /* :405-408 stuffing */
            w->acc = 0;
            w->nacc = 0;
        }
    }
}

static void put_value(bitw *w, int v, int cls) { /* :442-444, :456-458 */
    uint32_t id = (uint32_t)(v < 0 ? -v : v);
    if (v < 0) id = ~id;
    put_bits(w, id & ((1u << cls) - 1), cls);
}

static void emit_ac(int sym, int value, void *ctx) {
    bitw *w = (bitw *)ctx;
    put_bits(w, (uint32_t)w->ac->sym_code[sym], w->ac->sym_code_len[sym]);
    if (sym != 0x00 && sym != 0xF0) put_value(w, value, sym & 0x0F);
}

/* :425-432 pad: OR 1-bits into the free low bits; a full 0xFF byte is still
 * written when the scan ended on a byte boundary, and the pad is never
 * stuffed. */
static void pad_scan(bitw *w) {
    int free_bits = 8 - w->nacc;
    uint8_t byte = (uint8_t)((w->acc << free_bits) | ((1u << free_bits) - 1));
    w->out[w->n++] = byte;
    w->acc = 0;
    w->nacc = 0;
}

static void scan(bitw *w, const int16_t *plane, size_t nblocks,
                 const cref_huff *dc, const cref_huff *ac) { /* :462-502 */
    w->ac = ac;
    for (size_t b = 0; b < nblocks; b++) {
        const int16_t *blk = plane + b * 64;
        int cls = magnitude_class(blk[0]);
        put_bits(w, (uint32_t)dc->sym_code[cls], dc->sym_code_len[cls]);
        put_value(w, blk[0], cls);
        walk_ac(blk, emit_ac, w);
    }
    pad_scan(w);
}

static void put(bitw *w, int byte) { w->out[w->n++] = (uint8_t)byte; }

static void dht(bitw *w, const cref_huff *h, int tc_th) { /* :504-532 */
    int n = 0;
    for (int i = 1; i <= 16; i++) n += h->code_len_freq[i];
    int len = 19 + n;
    put(w, 0xFF); put(w, 0xC4);
    put(w, len >> 8); put(w, len & 0xFF);
    put(w, tc_th);
    for (int i = 1; i <= 16; i++) put(w, h->code_len_freq[i]);
    for (int i = 0; i < n; i++) put(w, h->sym_sorted[i]);
}

size_t cref_write_jpg(uint8_t *jpg, const int16_t *Y, const int16_t *Cb,
                      const int16_t *Cr, cref_area d, const cref_huff luma[2],
                      const cref_huff chroma[2], const int luma_q[64],
                      const int chroma_q[64]) {
    static const uint8_t app0[20] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 0x4A,
                                     0x46, 0x49, 0x46, 0x00, 0x01, 0x01, 0x00,
                                     0x00, 0x48, 0x00, 0x48, 0x00, 0x00}; /* :534 */
    bitw w = {jpg, 0, 0, 0, NULL};
    for (int i = 0; i < 20; i++) put(&w, app0[i]);
    for (int t = 0; t < 2; t++) { /* :558-582 DQT id 0 then id 1, zigzag order */
        const int *q = t ? chroma_q : luma_q;
        put(&w, 0xFF); put(&w, 0xDB); put(&w, 0x00); put(&w, 0x43); put(&w, t);
        for (int i = 0; i < 64; i++) put(&w, q[k_zigzag[i]]);
    }
    dht(&w, &luma[0], 0x00); /* :584-587 */
    dht(&w, &luma[1], 0x10);
    dht(&w, &chroma[0], 0x01);
    dht(&w, &chroma[1], 0x11);
    /* :589-603, :536 SOF0, 3 components, Y 2x2, Cb/Cr 1x1 */
    put(&w, 0xFF); put(&w, 0xC0); put(&w, 0x00); put(&w, 0x11); put(&w, 0x08);
    put(&w, (d.h >> 8) & 0xFF); put(&w, d.h & 0xFF);
    put(&w, (d.w >> 8) & 0xFF); put(&w, d.w & 0xFF);
    put(&w, 0x03);
    put(&w, 0x01); put(&w, 0x22); put(&w, 0x00);
    put(&w, 0x02); put(&w, 0x11); put(&w, 0x01);
    put(&w, 0x03); put(&w, 0x11); put(&w, 0x01);
    /* :605-635 three non-interleaved scans, :537 SOS layout */
    size_t nY = (size_t)d.w * d.h / 64;
    const int16_t *plane[3] = {Y, Cb, Cr};
    size_t nb[3] = {nY, nY / 4, nY / 4};
    for (int c = 0; c < 3; c++) {
        int td_ta = c ? 0x11 : 0x00;
        put(&w, 0xFF); put(&w, 0xDA); put(&w, 0x00); put(&w, 0x08); put(&w, 0x01);
        put(&w, c + 1); put(&w, td_ta); put(&w, 0x00); put(&w, 0x3F); put(&w, 0x00);
        scan(&w, plane[c], nb[c], c ? &chroma[0] : &luma[0], c ? &chroma[1] : &luma[1]);
    }
    put(&w, 0xFF); put(&w, 0xD9); /* :637-641 */
    return w.n;
}

size_t cref_max_jpg_bytes(int w, int h) {
    /* per block <= 28 DC bits + 63*27 AC bits = 1729 bits -> 217 bytes,
     * doubled for worst-case stuffing; plus headers and 3 pad bytes */
    size_t blocks = (size_t)w * h / 64 + (size_t)w * h / 128;
    return blocks * 434 + 4096;
}

size_t cref_encode(const uint8_t *bgr, int stride_px, cref_area d, int quality,
                   uint8_t *jpg, size_t cap) {
    if (d.w <= 0 || d.h <= 0 || d.w % 16 || d.h % 16) return 0;
    if (cap < cref_max_jpg_bytes(d.w, d.h)) return 0;
    int lq[64], cq[64];
    cref_quality_tables(quality, lq, cq);
    size_t nY = (size_t)d.w * d.h;
    int16_t *Y = (int16_t *)malloc(nY * 2), *Cb = (int16_t *)malloc(nY / 2),
            *Cr = (int16_t *)malloc(nY / 2);
    cref_huff *t = (cref_huff *)malloc(4 * sizeof(cref_huff));
    size_t n = 0;
    if (Y && Cb && Cr && t) {
        cref_rgb_to_dct(bgr, stride_px, Y, Cb, Cr, d, lq, cq);
        if (cref_init_huffman(Y, Cb, Cr, d, t, t + 2) == 0)
            n = cref_write_jpg(jpg, Y, Cb, Cr, d, t, t + 2, lq, cq);
    }
    free(Y); free(Cb); free(Cr); free(t);
    return n;
}

/* ======================================================================== */
/* Change detector: main/brain.c                                            */
/* ======================================================================== */

/* brain.c:16-45.  Sums of 16 bytes (uint16 in the reference) floored by 16;
 * the output is R, G, B (R = in[+2] of the BGR input). */
void cref_subsample(const uint8_t *bgr, int w, int h, uint8_t *sub) {
    int sw = w / 4, sh = h / 4;
    for (int sy = 0; sy < sh; sy++)
        for (int sx = 0; sx < sw; sx++)
            for (int c = 0; c < 3; c++) {
                unsigned acc = 0;
                for (int r = 0; r < 4; r++)
                    for (int k = 0; k < 4; k++)
                        acc += bgr[3 * ((size_t)(4 * sy + r) * w + 4 * sx + k) + (2 - c)];
                sub[3 * ((size_t)sy * sw + sx) + c] = (uint8_t)(acc / 16);
            }
}

/* brain.c:184-195: the weighted colour distance is evaluated in FP64 in the
 * reference; every intermediate is an exact dyadic rational there
 * (d^2 * (2 + cR/256) with cR = (a+b)/2), so the integer form below is the
 * same value: floor(d^2 (1024+s) / 512), 4 d^2, floor(d^2 (1534-s) / 512),
 * s = a_R + b_R.  The deltas go through uint32 (two's complement squares). */
static int cref_pixel_differs(const uint8_t *a, const uint8_t *b) {
    uint32_t s = (uint32_t)a[0] + b[0];
    uint32_t dr = (uint32_t)((int)a[0] - (int)b[0]);
    uint32_t dg = (uint32_t)((int)a[1] - (int)b[1]);
    uint32_t db = (uint32_t)((int)a[2] - (int)b[2]);
    dr *= dr; dg *= dg; db *= db;
    uint32_t t = (uint32_t)(((uint64_t)dr * (1024 + s)) >> 9) + 4 * dg +
                 (uint32_t)(((uint64_t)db * (1534 - s)) >> 9);
    return t > 600;
}

static int cref_invalid(const cref_area *a) { return a->x < 0 || a->y < 0 || a->w < 0 || a->h < 0; }

/* brain.c:86-102 (areas as x0, y0, x1, y1 during the scan) */
static void cref_sum_areas(cref_area *a, cref_area b) {
    if (cref_invalid(a) && cref_invalid(&b)) {
        a->x = a->y = a->w = a->h = -1;
    } else if (cref_invalid(a)) {
        *a = b;
    } else if (!cref_invalid(&b)) {
        if (b.x < a->x) a->x = b.x;
        if (b.y < a->y) a->y = b.y;
        if (b.w > a->w) a->w = b.w;
        if (b.h > a->h) a->h = b.h;
    }
}

/* brain.c:64-74 */
static int cref_overlap(cref_area a, cref_area b) {
    return !(a.x > b.w + 1 || a.w + 1 < b.x) && !(a.y > b.h + 1 || a.h + 1 < b.y);
}
static int cref_overlap2(cref_area a, cref_area b) {
    return !(a.x > b.x + b.w + 2 || a.x + a.w + 2 < b.x) &&
           !(a.y > b.y + b.h + 2 || a.y + a.h + 2 < b.y);
}

/* brain.c:240-261 */
void cref_enlarge_adjust(cref_area *a, int w, int h) {
    a->w = (a->w - a->x + 1) * 4;
    a->h = (a->h - a->y + 1) * 4;
    a->x *= 4;
    a->y *= 4;
    a->x -= (16 - a->w % 16) / 2;
    a->y -= (16 - a->h % 16) / 2;
    if (a->w % 16) a->w += 16 - a->w % 16;
    if (a->h % 16) a->h += 16 - a->h % 16;
    if (a->w > w) a->w = w;
    if (a->h > h) a->h = h;
    if (a->x + a->w > w) a->x -= a->x + a->w - w;
    if (a->y + a->h > h) a->y -= a->y + a->h - h;
    if (a->x < 0) a->x = 0;
    if (a->y < 0) a->y = 0;
}

/* brain.c:104-233.  Runs of differing pixels are collected per sub-row into
 * one of two alternating lists; when a sub-row starts, the runs of the row
 * before it are joined to the runs of the row before that (8-adjacency)
 * into areas.  Kept as the reference has it: a run still open at the end of
 * a row is dropped, the last row is never joined, the 100-area overflow
 * compaction leaves run labels stale, and sumAreas after enlargeAdjust takes
 * the larger width/height rather than the union. */
int cref_compare(const uint8_t *sub, const uint8_t *saved, int w, int h, cref_area outs[100]) {
    int sw = w / 4, sh = h / 4, cap = w / 8;
    cref_run *lists = malloc(sizeof(cref_run) * 2 * (size_t)cap);
    cref_run *L[2] = {lists, lists + cap};
    int n = 0, cur = 0, ncur = 0, nprev = 0, open = 0;
    for (int i = 0; i < 100; i++) outs[i].x = outs[i].y = outs[i].w = outs[i].h = -1;
    for (int i = 0; i < 2 * cap; i++) lists[i].beg = lists[i].end = lists[i].row = lists[i].done = -1;
    for (int y = 0; y < sh; y++) {
        /* :124-181 join the finished row's runs (L[cur]) to L[!cur] */
        cref_run *rk = L[cur], *rz = L[!cur];
        for (int k = 0; k < ncur; k++) {
            int joined = 0;
            for (int z = 0; z < nprev; z++) {
                if (rk[k].end < rz[z].beg - 1 || rk[k].beg > rz[z].end + 1) continue;
                joined = 1;
                if (rk[k].done >= 0) {
                    int lo = rz[z].done < rk[k].done ? rz[z].done : rk[k].done;
                    int hi = rz[z].done < rk[k].done ? rk[k].done : rz[z].done;
                    if (lo == hi) continue;
                    cref_sum_areas(&outs[lo], outs[hi]);
                    n--;
                    if (hi < n) outs[hi] = outs[n];
                    rk[k].done = rz[z].done = lo;
                    for (int a = 0; a < k; a++) {
                        if (rk[a].done == hi) rk[a].done = lo;
                        if (rk[a].done == n) rk[a].done = hi;
                    }
                    for (int a = z + 1; a < nprev; a++) {
                        if (rz[a].done == hi) rz[a].done = lo;
                        if (rz[a].done == n) rz[a].done = hi;
                    }
                } else {
                    rk[k].done = rz[z].done;
                    cref_area seg = {rk[k].beg, rk[k].row, rk[k].end, rk[k].row};
                    cref_sum_areas(&outs[rz[z].done], seg);
                }
            }
            if (!joined) {
                if (n > 99) { /* :156-168 */
                    for (int i = 0; i < n; i++)
                        for (int j = i + 1; j < n; j++)
                            if (cref_overlap(outs[i], outs[j])) {
                                cref_sum_areas(&outs[i], outs[j]);
                                n--;
                                outs[j] = outs[n];
                            }
                    if (n > 99) { free(lists); return n; }
                }
                rk[k].done = n;
                cref_area seg = {rk[k].beg, rk[k].row, rk[k].end, rk[k].row};
                outs[n++] = seg;
            }
        }
        cur = !cur;
        open = 0;
        nprev = ncur;
        ncur = 0;
        /* :184-210 scan row y into L[cur] */
        for (int x = 0; x < sw; x++) {
            size_t o = 3 * ((size_t)y * sw + x);
            if (cref_pixel_differs(sub + o, saved + o)) {
                if (!open) {
                    open = 1;
                    L[cur][ncur].beg = x;
                    L[cur][ncur].row = y;
                    L[cur][ncur].done = -1;
                }
                L[cur][ncur].end = x;
            } else if (open) {
                open = 0;
                ncur++;
            }
        }
    }
    free(lists);
    /* :212-232 */
    for (int i = 0; i < n; i++) cref_enlarge_adjust(&outs[i], w, h);
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++)
            if (cref_overlap2(outs[i], outs[j])) {
                cref_sum_areas(&outs[i], outs[j]);
                n--;
                outs[j] = outs[n];
                j--;
            }
    for (int i = 0; i < n;) {
        if (outs[i].w < 32 && outs[i].h < 24) {
            n--;
            if (i < n) outs[i] = outs[n];
            outs[n].x = outs[n].y = outs[n].w = outs[n].h = -1;
        } else {
            i++;
        }
    }
    return n;
}
