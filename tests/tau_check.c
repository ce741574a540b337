/*
 * tests/tau_check.c -- TEST INFRASTRUCTURE: machine check of K1's fast-path
 * decision rule against the reference's FP64 DCT.
 *
 * K1 (jpeg-encoder-decoder_amd/csrc/mij_kernels.hip, k_mcu_dct) computes each
 * AC coefficient as the exact integer N = sum_k W[z][k] * (p_k - 128), with
 * W = llround(C C s_u s_v * 2^19) split into three base-128 int8 digits
 * (fill_tables, mij_api.hip), and quantises it in fp32:
 *     fac = (float)(1 / (2^21 q)),  lc = fmaf(L1, 0.72f, 80.0f),
 *     tv  = fmaf(fac, lc, 1e-6f),  lo = fmaf(N, fac, -tv),  hi = fmaf(N, fac, tv)
 * and keeps trunc(lo) when trunc(lo) == trunc(hi); otherwise it replays the
 * coefficient in FP64 the reference's way.  This program restates those
 * steps bit for bit (C fmaf is the correctly rounded fused multiply-add the
 * GPU's v_fma_f32 / v_pk_fma_f32 perform) and checks, over generated blocks
 * and EVERY quantiser value q that some quality 1..100 produces at that
 * zigzag position of either table (original.c:504-509), that a kept value
 * always equals the reference's (int)(F / q) clipped to [-2048, 2047]
 * (encoder.c:108-109), F from the oracle's cref_dct_block_f64 (the pinned
 * FP64 restatement of encoder.c:81-106).
 *
 *   tau_check <nblocks> <seed> <threads>
 * prints one JSON line: blocks, checks, kept, hazards, misses, worst ratio of
 * |N - 2^21 F| to the bound L1/2 + 64 the tau formula assumes.
 * Exit status 1 if any kept value differs from the reference.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/cpu_ref.h"

static const int k_zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

static int64_t W[64][64];      /* [zigzag z][pixel k], the digits' value */
static int qset[64][256];      /* distinct q per zigzag position over Q = 1..100, both tables */
static int nq[64];
static float qfac[256];        /* (float)(1 / (2^21 q)) as fill_tables stores it */
static double qinv[256];       /* 1 / q, the fast screen of the reference's f / q */
static double basis[8][8];     /* cos((2x+1) u pi / 16), the generators' inverse DCT */

static void build_tables(void) {
    double cosd[64];
    for (int i = 0; i < 64; i++) cosd[i] = cos((double)(2 * (i / 8) + 1) * (i % 8) * M_PI / 16);
    for (int z = 1; z < 64; z++) {
        const int rz = k_zz[z], v = rz >> 3, u = rz & 7;
        for (int p = 0; p < 64; p++) {
            const int y = p >> 3, x = p & 7;
            double k = cosd[y * 8 + v] * cosd[x * 8 + u];
            if (u == 0) k *= M_SQRT1_2;
            if (v == 0) k *= M_SQRT1_2;
            const long long w = llround(k * 524288.0);
            /* the base-128 digits of fill_tables recombine to w exactly */
            const long long d0 = ((w + 64) & 127) - 64, w1 = (w - d0) >> 7;
            const long long d1 = ((w1 + 64) & 127) - 64, d2 = (w1 - d1) >> 7;
            if (d2 < -128 || d2 > 127 || ((d2 << 14) + (d1 << 7) + d0) != w) {
                fprintf(stderr, "digit split fails at z=%d p=%d\n", z, p);
                exit(2);
            }
            W[z][p] = w;
        }
    }
    for (int x = 0; x < 8; x++)
        for (int u = 0; u < 8; u++) basis[x][u] = cos((2 * x + 1) * u * M_PI / 16);
    for (int q = 1; q < 256; q++) {
        qfac[q] = (float)(1.0 / (2097152.0 * q));
        qinv[q] = 1.0 / q;
    }
    static unsigned char seen[64][256];
    for (int Q = 1; Q <= 100; Q++) {
        int lq[64], cq[64];
        cref_quality_tables(Q, lq, cq);
        for (int z = 1; z < 64; z++)
            for (int t = 0; t < 2; t++) {
                const int q = t ? cq[k_zz[z]] : lq[k_zz[z]];
                if (!seen[z][q]) {
                    seen[z][q] = 1;
                    qset[z][nq[z]++] = q;
                }
            }
    }
}

/* xorshift64* */
static inline uint64_t rnd(uint64_t *s) {
    uint64_t x = *s;
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    *s = x;
    return x * 0x2545F4914F6CDD1DULL;
}
static inline int clamp255(double v) { return v < 0 ? 0 : (v > 255 ? 255 : (int)lrint(v)); }

/* Block generators: random, flat (+ one-pixel bumps), checkerboards, ramps,
 * near-flat noise, 0/255 extremes, DCT basis patterns, and "targeted" blocks
 * synthesised from integer multiples of a quantiser (their coefficients sit
 * on or near truncation boundaries, the case the rule must get right). */
static void gen_block(uint64_t *s, uint8_t px[64]) {
    const int kind = (int)(rnd(s) % 9);
    switch (kind) {
    case 0:
        for (int i = 0; i < 64; i++) px[i] = (uint8_t)rnd(s);
        break;
    case 1: {
        const int v = (int)(rnd(s) & 255);
        for (int i = 0; i < 64; i++) px[i] = (uint8_t)v;
        const int nb = (int)(rnd(s) % 3);
        for (int b = 0; b < nb; b++) px[rnd(s) & 63] = (uint8_t)(v + (int)(rnd(s) % 5) - 2);
        break;
    }
    case 2: {
        const int a = (int)(rnd(s) % 128), m = 128 + (int)(rnd(s) % 3) - 1, ph = (int)(rnd(s) & 3);
        for (int i = 0; i < 64; i++) {
            const int y = i >> 3, x = i & 7;
            const int sgn = (ph & 1 ? (x ^ y) : (ph & 2 ? x : y)) & 1;
            px[i] = (uint8_t)clamp255(m + (sgn ? a : -a));
        }
        break;
    }
    case 3: {
        const double gx = ((double)(rnd(s) % 2001) - 1000) / 100.0, gy = ((double)(rnd(s) % 2001) - 1000) / 100.0;
        const double c = (double)(rnd(s) & 255);
        for (int i = 0; i < 64; i++) px[i] = (uint8_t)clamp255(c + gx * ((i & 7) - 3.5) + gy * ((i >> 3) - 3.5));
        break;
    }
    case 4: {
        const int m = (int)(rnd(s) & 255), k = 1 + (int)(rnd(s) % 4);
        for (int i = 0; i < 64; i++) px[i] = (uint8_t)clamp255(m + (int)(rnd(s) % (2 * k + 1)) - k);
        break;
    }
    case 5:
        for (int i = 0; i < 64; i++) px[i] = (rnd(s) & 1) ? 255 : 0;
        break;
    case 6: {
        const int u = (int)(rnd(s) & 7), v = (int)(rnd(s) & 7);
        const double a = (double)(rnd(s) % 128);
        for (int i = 0; i < 64; i++) {
            const int y = i >> 3, x = i & 7;
            px[i] = (uint8_t)clamp255(128 + a * basis[x][u] * basis[y][v]);
        }
        break;
    }
    default: {
        /* inverse DCT of a few coefficients at integer multiples of q: the
         * forward FP64 DCT of the rounded pixels lands near those multiples */
        double F[64];
        memset(F, 0, sizeof(F));
        const int nc = 1 + (int)(rnd(s) % 4);
        const int q = 1 + (int)(rnd(s) % 40);
        F[0] = ((double)(rnd(s) % 512) - 256);
        for (int c = 0; c < nc; c++) {
            const int rz = (int)(rnd(s) % 63) + 1;
            F[rz] = q * (((double)(rnd(s) % 21) - 10)) + ((double)(rnd(s) % 3) - 1) * 0.5 / 64;
        }
        for (int i = 0; i < 64; i++) {
            const int y = i >> 3, x = i & 7;
            double acc = 0;
            for (int v = 0; v < 8; v++)
                for (int u = 0; u < 8; u++) {
                    const double cu = u ? 1 : M_SQRT1_2, cv = v ? 1 : M_SQRT1_2;
                    acc += cu * cv * F[v * 8 + u] * basis[x][u] * basis[y][v];
                }
            px[i] = (uint8_t)clamp255(128 + acc / 4);
        }
        break;
    }
    }
}

typedef struct {
    long long blocks, seed;
    long long checks, kept, hazards, misses;
    double worst;
    int first_miss_z, first_miss_q;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    uint64_t s = 0x9E3779B97F4A7C15ULL ^ ((uint64_t)j->seed * 0xD1B54A32D192ED03ULL);
    if (!s) s = 1;
    uint8_t px[64];
    double F[64];
    for (long long b = 0; b < j->blocks; b++) {
        gen_block(&s, px);
        cref_dct_block_f64(px, 8, F);
        int X[64], L1 = 0;
        for (int k = 0; k < 64; k++) {
            X[k] = px[k] - 128;
            L1 += X[k] < 0 ? -X[k] : X[k];
        }
        const float lc = fmaf((float)L1, 0.72f, 80.0f);
        for (int z = 1; z < 64; z++) {
            int64_t N = 0;
            for (int k = 0; k < 64; k++) N += W[z][k] * X[k];
            const double f = F[k_zz[z]];
            const double r = fabs((double)N - 2097152.0 * f) / (0.5 * L1 + 64.0);
            if (r > j->worst) j->worst = r;
            const float nf = (float)(int32_t)N;
            /* branch-free over the q values (vectorises); the reference's
             * (int)(f / q) is formed as trunc(f * (1/q)) and recomputed with
             * the true division below wherever f / q is near an integer */
            const int n = nq[z];
            const int *qs = qset[z];
            int hz = 0, bad = 0, near = 0;
            for (int i = 0; i < n; i++) {
                const int q = qs[i];
                const float fa = qfac[q];
                const float tv = fmaf(fa, lc, 1.0e-6f);
                const int lo = (int)fmaf(nf, fa, -tv), hi = (int)fmaf(nf, fa, tv);
                const double t = f * qinv[q];
                const double tr = trunc(t);
                const double d = fabs(t - tr);
                near |= (d < 1e-9) | (d > 1.0 - 1e-9);
                hz += lo != hi;
                bad += (lo == hi) & (lo != (int)tr);
            }
            j->checks += n;
            j->hazards += hz;
            j->kept += n - hz;
            if (bad || near) {  /* exact reference semantics, one q at a time */
                bad = 0;
                for (int i = 0; i < n; i++) {
                    const int q = qs[i];
                    const float fa = qfac[q];
                    const float tv = fmaf(fa, lc, 1.0e-6f);
                    const int lo = (int)fmaf(nf, fa, -tv), hi = (int)fmaf(nf, fa, tv);
                    if (lo != hi) continue;
                    int ref = (int)(int16_t)(int)(f / q); /* encoder.c:108 */
                    ref = ref < -2048 ? -2048 : (ref > 2047 ? 2047 : ref);
                    if (lo != ref) {
                        if (!j->misses && !bad) {
                            j->first_miss_z = z;
                            j->first_miss_q = q;
                        }
                        bad++;
                    }
                }
                j->misses += bad;
            }
        }
    }
    return NULL;
}

/* tau_check dump <nblocks> <seed> <Q> <out>: the generated blocks and, for
 * each, the rule's decision at every AC position under the LUMA table of
 * quality Q, for tests/test_tau_kernel.py to compare with K1's own decisions
 * (mij_batch_audit).  Writes <out>.px (nblocks x 64 bytes, row-major) and
 * <out>.mask (nblocks uint64, bit z = zigzag coefficient z straddles a
 * truncation boundary, i.e. trunc(lo) != trunc(hi)). */
static int dump(long long nblocks, long long seed, int Q, const char *out) {
    int lq[64], cq[64];
    cref_quality_tables(Q, lq, cq);
    char path[4096];
    snprintf(path, sizeof path, "%s.px", out);
    FILE *fp = fopen(path, "wb");
    snprintf(path, sizeof path, "%s.mask", out);
    FILE *fm = fopen(path, "wb");
    if (!fp || !fm) return 2;
    uint64_t st = 0x9E3779B97F4A7C15ULL ^ ((uint64_t)seed * 0xD1B54A32D192ED03ULL);
    if (!st) st = 1;
    uint8_t px[64];
    for (long long b = 0; b < nblocks; b++) {
        gen_block(&st, px);
        int X[64], L1 = 0;
        for (int k = 0; k < 64; k++) {
            X[k] = px[k] - 128;
            L1 += X[k] < 0 ? -X[k] : X[k];
        }
        const float lc = fmaf((float)L1, 0.72f, 80.0f);
        uint64_t m = 0;
        for (int z = 1; z < 64; z++) {
            int64_t N = 0;
            for (int k = 0; k < 64; k++) N += W[z][k] * X[k];
            const float nf = (float)(int32_t)N;
            const float fa = qfac[lq[k_zz[z]]];
            const float tv = fmaf(fa, lc, 1.0e-6f);
            if ((int)fmaf(nf, fa, -tv) != (int)fmaf(nf, fa, tv)) m |= 1ull << z;
        }
        fwrite(px, 1, 64, fp);
        fwrite(&m, 8, 1, fm);
    }
    fclose(fp);
    fclose(fm);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 5 && !strcmp(argv[1], "dump")) {
        build_tables();
        return dump(atoll(argv[2]), atoll(argv[3]), atoi(argv[4]), argv[5]);
    }
    const long long nblocks = argc > 1 ? atoll(argv[1]) : 100000;
    const long long seed = argc > 2 ? atoll(argv[2]) : 1;
    int nth = argc > 3 ? atoi(argv[3]) : 1;
    if (nth < 1) nth = 1;
    if (nth > 64) nth = 64;
    build_tables();
    pthread_t th[64];
    job_t jobs[64];
    for (int t = 0; t < nth; t++) {
        memset(&jobs[t], 0, sizeof(job_t));
        jobs[t].blocks = nblocks / nth + (t < nblocks % nth);
        jobs[t].seed = seed * 1000003LL + t;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    job_t tot;
    memset(&tot, 0, sizeof(tot));
    tot.first_miss_z = tot.first_miss_q = -1;
    for (int t = 0; t < nth; t++) {
        pthread_join(th[t], NULL);
        tot.blocks += jobs[t].blocks;
        tot.checks += jobs[t].checks;
        tot.kept += jobs[t].kept;
        tot.hazards += jobs[t].hazards;
        if (jobs[t].misses && tot.first_miss_z < 0) {
            tot.first_miss_z = jobs[t].first_miss_z;
            tot.first_miss_q = jobs[t].first_miss_q;
        }
        tot.misses += jobs[t].misses;
        if (jobs[t].worst > tot.worst) tot.worst = jobs[t].worst;
    }
    int nqt = 0;
    for (int z = 1; z < 64; z++) nqt += nq[z];
    printf("{\"blocks\": %lld, \"seed\": %lld, \"q_values_per_block\": %d, \"checks\": %lld, \"kept\": %lld, "
           "\"hazards\": %lld, \"misses\": %lld, \"first_miss_z\": %d, \"first_miss_q\": %d, "
           "\"worst_err_over_bound\": %.6f}\n",
           tot.blocks, seed, nqt, tot.checks, tot.kept, tot.hazards, tot.misses, tot.first_miss_z,
           tot.first_miss_q, tot.worst);
    return tot.misses ? 1 : 0;
}
