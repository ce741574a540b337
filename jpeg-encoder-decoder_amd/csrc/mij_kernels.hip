// mij_kernels.hip -- gfx950 (CDNA4) kernels of the MI355X JPEG block-encode
// path.  Reference: MattiaDallaCosta/JPEG-encoder-decoder main/encoder.c.
//
//   k_colour_lut   colour-exception bitmaps (encoder.c:133-135 in FP64)
//   k_mcu_dct      K1: BGR -> YCbCr -> 4:2:0 -> DCT (i8 MFMA, exact integer)
//                  -> quantize/trunc (+FP64 replay near boundaries) -> zigzag
//                  (encoder.c:121-150, :81-112, :65-70)
//   k_dc_diff      DC differencing into the coefficient planes (:168-177)
//   k_tokens       per-block symbol lists + histograms (:315-358, :462-502)
//   k_tables       optimized Huffman tables, wave-parallel (:180-301)
//   k_ehuf_struct  code tables from caller-owned huff_code structs
//   k_bits         bits per block
//   k_scan         per-scan offsets of each chunk
//   k_pack         bit packing of each chunk in LDS (:434-502)
//   k_emit         JFIF assembly + 0xFF stuffing + pad quirks (:383-432,
//                  :504-644)
//
// Compiled with -ffp-contract=off: every FP64 operation that has to match the
// reference is written with explicit __dmul_rn/__dadd_rn in the reference's
// evaluation order; fp32 FMAs are explicit fmaf() calls.
#include "mij_internal.h"

namespace mij {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__constant__ int c_zigzag[64] = {  // encoder.c:38-46
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

#define SQRT1_2 0.70710678118654752440  // <math.h> M_SQRT1_2

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int mag_class(int v) {  // encoder.c:303-313
  v = v < 0 ? -v : v;
  return 32 - __clz(v);
}

// ===========================================================================
// Colour-exception bitmaps.  Exact-integer colour values for which the FP64
// expression of encoder.c:133-135 lands one ulp-ish below the integer, so the
// uint8_t truncation yields value-1.  Y indexed by (R,G) (the B of an integer
// point is unique), Cb by (G,B) with R==G, Cr by (G,R) with B==G.
// ===========================================================================
__global__ void k_colour_lut(uint32_t *lut /* [3][2048] */) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;  // 0 .. 65535
  if (i >= 65536) return;
  int hi = i >> 8, lo = i & 255;
  bool ey = false, ecb = false, ecr = false;
  {  // Y: (R,G) = (hi,lo)
    int R = hi, G = lo;
    for (int B = 0; B < 256; B++) {
      int n = 299 * R + 587 * G + 114 * B;
      if (n % 1000) continue;
      double y = __dadd_rn(__dadd_rn(__dmul_rn(0.299, (double)R), __dmul_rn(0.587, (double)G)),
                           __dmul_rn(0.114, (double)B));
      ey = (int)y != n / 1000;
    }
  }
  {  // Cb: (G,B) = (hi,lo), R = G
    int G = hi, B = lo, R = G;
    long long n = 128000000LL - 168736LL * R - 331264LL * G + 500000LL * B;
    if (n % 1000000 == 0) {
      double cb = __dadd_rn(__dadd_rn(__dadd_rn(128.0, -__dmul_rn(0.168736, (double)R)),
                                      -__dmul_rn(0.331264, (double)G)),
                            __dmul_rn(0.5, (double)B));
      ecb = (int)cb != (int)(n / 1000000);
    }
  }
  {  // Cr: (G,R) = (hi,lo), B = G
    int G = hi, R = lo, B = G;
    long long n = 128000000LL + 500000LL * R - 418688LL * G - 81312LL * B;
    if (n % 1000000 == 0) {
      double cr = __dadd_rn(__dadd_rn(__dadd_rn(128.0, __dmul_rn(0.5, (double)R)),
                                      -__dmul_rn(0.418688, (double)G)),
                            -__dmul_rn(0.081312, (double)B));
      ecr = (int)cr != (int)(n / 1000000);
    }
  }
  if (ey) atomicOr(&lut[0 * 2048 + (i >> 5)], 1u << (i & 31));
  if (ecb) atomicOr(&lut[1 * 2048 + (i >> 5)], 1u << (i & 31));
  if (ecr) atomicOr(&lut[2 * 2048 + (i >> 5)], 1u << (i & 31));
}

// ===========================================================================
// K1 helpers
// ===========================================================================

// encoder.c:133-135 bit-exactly.  The fp32 forms below carry an error
// < 2e-5 (Y) / 1e-5 (Cb, Cr), while a non-integer exact value is >= 1e-3 (Y)
// or >= 3.2e-5 (Cb/Cr, proof in DESIGN.md) away from the next integer, so the
// truncation is exact everywhere except at exact-integer points, where the
// precomputed bitmaps say whether the FP64 reference lands one below.
__device__ __forceinline__ void pixel_ycc(uint32_t B, uint32_t G, uint32_t R,
                                          const uint32_t *__restrict__ lut,
                                          int &y, int &cb, int &cr) {
  float fb = (float)B, fg = (float)G, fr = (float)R;
  float dr = fr - fg, db = fb - fg;
  float yf = fmaf(0.114f, db, fmaf(0.299f, dr, fg)) + 0.0005f;
  y = (int)yf;
  cb = (int)fmaf(-0.168736f, dr, fmaf(0.5f, db, 128.0f));
  cr = (int)fmaf(-0.081312f, db, fmaf(0.5f, dr, 128.0f));
  if (yf - (float)y < 0.001f) {
    uint32_t i = (R << 8) | G;
    y -= (lut[i >> 5] >> (i & 31)) & 1;
  }
  if (dr == 0.0f) {
    uint32_t i = (G << 8) | B;
    cb -= (lut[2048 + (i >> 5)] >> (i & 31)) & 1;
  }
  if (db == 0.0f) {
    uint32_t i = (G << 8) | R;
    cr -= (lut[4096 + (i >> 5)] >> (i & 31)) & 1;
  }
}

// DC of one block exactly as encoder.c:87-109: the cosines of frequency 0
// are exactly 1.0, so both passes are exact integer sums S; what remains is
// fl(fl(fl(S*r)*r)/4) / q with r = M_SQRT1_2, then truncation.
__device__ __forceinline__ int dc_exact(int S, int q) {
  double f = __dmul_rn(__dmul_rn((double)S, SQRT1_2), SQRT1_2);
  f = __dmul_rn(f, 0.25);
  int t = (int)__ddiv_rn(f, (double)q);
  return t < -2048 ? -2048 : (t > 2047 ? 2047 : t);
}

// One AC coefficient replayed exactly as encoder.c:87-109 computes it
// (column pass summed from 0 in y order, row pass in x order, FP64, no FMA).
__device__ __noinline__ int ac_exact(const uint8_t *blk, int z, int q,
                                     const double *__restrict__ C) {
  int rz = c_zigzag[z];
  int v = rz >> 3, u = rz & 7;
  double freq = 0.0;
  for (int x = 0; x < 8; x++) {
    double inner = 0.0;
    for (int y = 0; y < 8; y++)
      inner = __dadd_rn(inner, __dmul_rn((double)((int)blk[y * 8 + x] - 128), C[y * 8 + v]));
    freq = __dadd_rn(freq, __dmul_rn(inner, C[x * 8 + u]));
  }
  if (u == 0) freq = __dmul_rn(freq, SQRT1_2);
  if (v == 0) freq = __dmul_rn(freq, SQRT1_2);
  freq = __dmul_rn(freq, 0.25);
  int t = (int)__ddiv_rn(freq, (double)q);
  return t < -2048 ? -2048 : (t > 2047 ? 2047 : t);
}

// ===========================================================================
// K1: fused colour conversion + 4:2:0 + DCT + quantization + zigzag.
//
// Persistent grid; each wave owns one 128x16 tile at a time:
//   1. 64 lanes load the tile's 16 rows of BGR888 (12 B = 4 px per lane and
//      row, coalesced), convert two 4x1 pixel runs (a 4x2 patch) per step,
//      average the two 2x2 chroma quads, and stage Y/Cb/Cr bytes in LDS in
//      block-major order (64 px per 8x8 block, LDS_BLK stride).
//   2. three MFMA N-tiles of 16 blocks (Y block row 0, Y block row 1,
//      Cb|Cr): v_mfma_i32_16x16x64_i8 with B = the blocks' pixels - 128
//      (exact int8) and A = the 64x64 DCT matrix (rows in zigzag order,
//      cos*cos*scale * 2^19 rounded) split into three base-128 digits.  The
//      int32 sum N is exact; N / 2^21 is the un-quantized coefficient to
//      within 0.002, and the DC row holds the exact pixel sum.
//   3. quantize with trunc; a coefficient whose +-tau interval straddles a
//      truncation boundary is recomputed in FP64 exactly like the reference.
//   4. lane (g, b) owns zigzag coefficients 16g..16g+15 of block b: two
//      16-byte stores per lane.
// ===========================================================================
__global__ __launch_bounds__(256) void k_mcu_dct(K1Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_tile[K1_WAVES][LDS_WAVE];
  __shared__ uint32_t s_lut[3 * 2048];
  __shared__ __attribute__((aligned(16))) float s_fac[2][64];
  __shared__ __attribute__((aligned(16))) float s_tau[2][64];

  const Tables *__restrict__ T = a.tab;
  for (int i = threadIdx.x; i < 3 * 2048; i += 256) s_lut[i] = (&T->lut[0][0])[i];
  for (int i = threadIdx.x; i < 128; i += 256) {
    s_fac[i >> 6][i & 63] = T->qfac[i >> 6][i & 63];
    s_tau[i >> 6][i & 63] = T->qtau[i >> 6][i & 63];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t *L = s_tile[wave];
  const int g = lane >> 4, bcol = lane & 15;
  const int q_dc[2] = {T->qint[0][0], T->qint[1][0]};

  v4i A[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    int4 t = T->mfma_a[i * 64 + lane];
    A[i] = v4i{t.x, t.y, t.z, t.w};
  }

  const Geom G = a.g;
  const int bw = G.w >> 3, mw = G.w >> 4;
  const long long ntiles = (long long)a.nframes * G.tiles_per_frame;
  const int c4 = lane & 31, pr = lane >> 5;

  for (long long t = (long long)blockIdx.x * K1_WAVES + wave; t < ntiles;
       t += (long long)gridDim.x * K1_WAVES) {
    const int f = (int)(t / G.tiles_per_frame);
    const int rem = (int)(t - (long long)f * G.tiles_per_frame);
    const int ty = rem / G.tiles_x, tx = rem - ty * G.tiles_x;
    const int valid_px = min(TILE_W, G.w - tx * TILE_W);
    const uint8_t *src = a.in + (long long)f * a.in_fs + (long long)(ty * TILE_H) * a.pitch +
                         tx * TILE_W * 3;

    // ---- 1. load + colour convert + subsample + stage --------------------
    const bool colv = 4 * c4 < valid_px;
    uint32_t d[4][2][3];
#pragma unroll
    for (int it = 0; it < 4; it++)
#pragma unroll
      for (int dy = 0; dy < 2; dy++) {
        const int row = 2 * (2 * it + pr) + dy;
        if (colv) {
          const uint32_t *p = (const uint32_t *)(src + (long long)row * a.pitch + 12 * c4);
          d[it][dy][0] = __builtin_nontemporal_load(p);
          d[it][dy][1] = __builtin_nontemporal_load(p + 1);
          d[it][dy][2] = __builtin_nontemporal_load(p + 2);
        } else {
          d[it][dy][0] = d[it][dy][1] = d[it][dy][2] = 0;
        }
      }
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int rp = 2 * it + pr;  // row pair 0..7 == chroma row
      int cbs[2][4], crs[2][4];
#pragma unroll
      for (int dy = 0; dy < 2; dy++) {
        const uint32_t w0 = d[it][dy][0], w1 = d[it][dy][1], w2 = d[it][dy][2];
        int y0, y1, y2, y3;
        pixel_ycc(w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255, s_lut, y0, cbs[dy][0], crs[dy][0]);
        pixel_ycc(w0 >> 24, w1 & 255, (w1 >> 8) & 255, s_lut, y1, cbs[dy][1], crs[dy][1]);
        pixel_ycc((w1 >> 16) & 255, w1 >> 24, w2 & 255, s_lut, y2, cbs[dy][2], crs[dy][2]);
        pixel_ycc((w2 >> 8) & 255, (w2 >> 16) & 255, w2 >> 24, s_lut, y3, cbs[dy][3], crs[dy][3]);
        const int yrow = 2 * rp + dy;  // 0..15
        const int by = yrow >> 3, bx = c4 >> 1;
        uint32_t packed = (uint32_t)y0 | ((uint32_t)y1 << 8) | ((uint32_t)y2 << 16) |
                          ((uint32_t)y3 << 24);
        *(uint32_t *)(L + (by * 16 + bx) * LDS_BLK + (yrow & 7) * 8 + (c4 & 1) * 4) = packed;
      }
      // encoder.c:137-138 -- floor((a+b+c+d)/4) of the truncated values
      const uint32_t cb0 = (uint32_t)(cbs[0][0] + cbs[0][1] + cbs[1][0] + cbs[1][1]) >> 2;
      const uint32_t cb1 = (uint32_t)(cbs[0][2] + cbs[0][3] + cbs[1][2] + cbs[1][3]) >> 2;
      const uint32_t cr0 = (uint32_t)(crs[0][0] + crs[0][1] + crs[1][0] + crs[1][1]) >> 2;
      const uint32_t cr1 = (uint32_t)(crs[0][2] + crs[0][3] + crs[1][2] + crs[1][3]) >> 2;
      const int cblk = c4 >> 2, ccol = (2 * c4) & 7;
      uint8_t *C0 = L + (32 + cblk) * LDS_BLK + rp * 8 + ccol;
      *(uint16_t *)C0 = (uint16_t)(cb0 | (cb1 << 8));
      *(uint16_t *)(C0 + 8 * LDS_BLK) = (uint16_t)(cr0 | (cr1 << 8));
    }
    wave_lds_sync();

    // ---- 2-4. DCT on MFMA, quantize, store -------------------------------
#pragma unroll 1
    for (int nt = 0; nt < 3; nt++) {
      const int comp = nt == 2 ? 1 : 0;
      const uint8_t *Pb = L + (nt * 16 + bcol) * LDS_BLK;
      v4i Bf = *(const v4i *)(Pb + 16 * g);
      Bf ^= (int)0x80808080;  // pixel - 128 as int8

      bool valid;
      long long blk;  // block index inside the frame's coefficient space
      if (nt < 2) {
        const int bx = tx * 16 + bcol;
        valid = bx < bw;
        blk = (long long)(2 * ty + nt) * bw + bx;
      } else {
        const int mx = tx * 8 + (bcol & 7);
        valid = mx < mw;
        blk = (long long)G.nY + (bcol >= 8 ? G.nC : 0) + (long long)ty * mw + mx;
      }

      int out[16];
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const v4i zero = {0, 0, 0, 0};
        v4i a2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[3 * m + 0], Bf, zero, 0, 0, 0);
        v4i a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[3 * m + 1], Bf, zero, 0, 0, 0);
        v4i a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[3 * m + 2], Bf, zero, 0, 0, 0);
        const float4 fac = *(const float4 *)&s_fac[comp][16 * g + 4 * m];
        const float4 tau = *(const float4 *)&s_tau[comp][16 * g + 4 * m];
        const float fa[4] = {fac.x, fac.y, fac.z, fac.w};
        const float ta[4] = {tau.x, tau.y, tau.z, tau.w};
        int haz = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int N = (a2[r] << 14) + (a1[r] << 7) + a0[r];
          const float nf = (float)N;
          const int lo = (int)fmaf(nf, fa[r], -ta[r]);
          const int hi = (int)fmaf(nf, fa[r], ta[r]);
          out[4 * m + r] = lo;
          haz |= (lo != hi) << r;
        }
        if (m == 0) {  // DC: the DC row of A is all-ones in digit 0 -> exact sum
          const int dcq = dc_exact(a0[0], q_dc[comp]);
          if (g == 0) {
            out[0] = dcq;
            haz &= ~1;
          }
        }
        if (__ballot(haz != 0)) {
          int nrep = 0;
#pragma unroll
          for (int r = 0; r < 4; r++)
            if ((haz >> r) & 1) {
              out[4 * m + r] = ac_exact(Pb, 16 * g + 4 * m + r, T->qint[comp][16 * g + 4 * m + r],
                                        T->cosd);
              nrep++;
            }
          if (nrep) atomicAdd(a.replays, (unsigned)nrep);
        }
      }
      if (valid) {
        int16_t *dst = a.coef + (long long)f * G.coef_fs + blk * 64 + 16 * g;
        u4v s0, s1;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          s0[k] = (uint32_t)(uint16_t)out[2 * k] | ((uint32_t)out[2 * k + 1] << 16);
          s1[k] = (uint32_t)(uint16_t)out[8 + 2 * k] | ((uint32_t)out[9 + 2 * k] << 16);
        }
        __builtin_nontemporal_store(s0, (u4v *)dst);
        __builtin_nontemporal_store(s1, (u4v *)(dst + 8));
        if (g == 0) a.dc[(long long)f * G.nblk + blk] = (int16_t)out[0];
      }
    }
    wave_lds_sync();
  }
}

// ===========================================================================
// DC differencing in place (encoder.c:168-177), for the drop-in rgb_to_dct
// whose caller expects differenced DCs in the planes.
// ===========================================================================
__global__ void k_dc_diff(int16_t *coef, const int16_t *dc, Geom G, int nframes) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)nframes * G.nblk;
  if (i >= total) return;
  const int f = (int)(i / G.nblk);
  const int j = (int)(i - (long long)f * G.nblk);
  const bool first = j == 0 || j == G.nY || j == G.nY + G.nC;
  const int16_t prev = first ? 0 : dc[i - 1];
  coef[(long long)f * G.coef_fs + (long long)j * 64] = (int16_t)(dc[i] - prev);
}

// ===========================================================================
// Entropy helpers
// ===========================================================================
struct Chunk {
  int f, comp, first, n, cstart;  // first block (frame-relative), count, comp start
};

__device__ __forceinline__ Chunk chunk_of(const Geom &G, int q) {
  Chunk c;
  c.f = q / G.cpf;
  int r = q - c.f * G.cpf;
  if (r < G.cy) {
    c.comp = 0;
    c.cstart = 0;
    c.first = r * CHUNK;
    c.n = min(CHUNK, G.nY - c.first);
  } else {
    r -= G.cy;
    c.comp = 1 + (r >= G.cc);
    if (r >= G.cc) r -= G.cc;
    c.cstart = c.comp == 1 ? G.nY : G.nY + G.nC;
    c.first = c.cstart + r * CHUNK;
    c.n = min(CHUNK, G.nC - r * CHUNK);
  }
  return c;
}

// Magnitude bits of a value of class cls (encoder.c:442-444 / :456-458:
// negative values are written as ~|v|, i.e. the low cls bits of v-1).
__device__ __forceinline__ uint32_t mag_bits(int v, int cls) {
  uint32_t id = (uint32_t)(v < 0 ? -v : v);
  if (v < 0) id = ~id;
  return id & ((1u << cls) - 1u);
}

// ===========================================================================
// k_tokens: coefficient planes -> per-block symbol lists + histograms.
//
// Token = symbol (bits 0-7) | ZRL count before it (bits 8-9) | magnitude
// bits (16-27).  Block slot: token 0 = DC difference (symbol = its class,
// encoder.c:434-446), tokens 1..n = the AC run/size symbols in zigzag order
// exactly as encoder.c:321-358 / :462-502 visit them (a nonzero at zigzag k
// after r zeros emits r/16 ZRLs, then ((r%16)<<4)|class); hdr = n | EOB<<7
// (EOB unless coefficient 63 is nonzero).  Histograms: DC classes and AC
// symbols per table (:315-319, :321-358), ZRLs and EOBs included.
//
// One workgroup per chunk; lane (g, b) of a wave holds zigzag coefficients
// 16g..16g+15 of block b, so a wave covers 16 blocks per iteration and the
// 64-bit nonzero mask of a block is assembled from its 4 lanes.
// ===========================================================================
__global__ __launch_bounds__(256) void k_tokens(EntArgs a) {
  __shared__ uint32_t h[2][257];
  __shared__ __attribute__((aligned(16))) int16_t s_coef[4][64][16];
  const Chunk c = chunk_of(a.g, blockIdx.x);
  for (int i = threadIdx.x; i < 2 * 257; i += 256) h[i / 257][i % 257] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, bcol = lane & 15;
  const long long fb = (long long)c.f * a.g.nblk;
  for (int base = wave * 16; base < c.n; base += 64) {
    const int i = base + bcol;
    const bool v = i < c.n;
    const int j = c.first + i;
    u4v w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0};
    if (v) {
      const int16_t *blk = a.coef + (long long)c.f * a.g.coef_fs + (long long)j * 64 + 16 * g;
      w0 = *(const u4v *)blk;
      w1 = *(const u4v *)(blk + 8);
    }
    *(u4v *)&s_coef[wave][lane][0] = w0;
    *(u4v *)&s_coef[wave][lane][8] = w1;
    uint32_t m16 = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t wd = k < 4 ? w0[k] : w1[k - 4];
      m16 |= ((wd & 0xFFFFu) != 0u ? 1u : 0u) << (2 * k);
      m16 |= ((wd >> 16) != 0u ? 1u : 0u) << (2 * k + 1);
    }
    if (g == 0) m16 &= ~1u;  // the DC is not part of the AC run structure
    unsigned long long M = (unsigned long long)m16 << (16 * g);
    M |= __shfl_xor(M, 16);
    M |= __shfl_xor(M, 32);
    uint32_t *tok = a.tok + (fb + j) * 64;
    if (g == 0 && v) {
      const int dc = (int16_t)(w0[0] & 0xFFFFu);
      const int diff =
          a.dc_mode ? dc : dc - (j == c.cstart ? 0 : (int)a.dc[fb + j - 1]);  // :168-177
      const int cls = mag_class(diff);
      tok[0] = (uint32_t)cls | (mag_bits(diff, cls) << 16);
      atomicAdd(&h[0][cls], 1u);
      const int eob = !((M >> 63) & 1ull);
      a.hdr[fb + j] = (uint8_t)(__popcll(M) | (eob << 7));
      if (eob) atomicAdd(&h[1][0x00], 1u);
    }
    wave_lds_sync();
    uint32_t mm = v ? m16 : 0u;
    while (mm) {
      const int k = __ffs(mm) - 1;
      mm &= mm - 1u;
      const int z = 16 * g + k;
      const int cz = s_coef[wave][lane][k];
      const unsigned long long before = M & ((1ull << z) - 1ull);
      const int run = z - (63 - __clzll(before | 1ull)) - 1;
      const int cls = mag_class(cz);
      const int sym = ((run & 15) << 4) | cls;
      tok[1 + __popcll(before)] = (uint32_t)sym | ((uint32_t)(run >> 4) << 8) |
                                  (mag_bits(cz, cls) << 16);
      atomicAdd(&h[1][sym], 1u);
      if (run >= 16) atomicAdd(&h[1][0xF0], (unsigned)(run >> 4));
    }
    wave_lds_sync();
  }
  __syncthreads();
  uint32_t *gh = a.hist + ((long long)c.f * 4 + (c.comp ? 2 : 0)) * 257;
  for (int i = threadIdx.x; i < 2 * 257; i += 256) {
    const uint32_t hv = h[i / 257][i % 257];
    if (hv) atomicAdd(&gh[i], hv);
  }
}


// ===========================================================================
// k_tables: the four optimized Huffman tables of a frame (encoder.c:180-301),
// one wave per table.  The reference's O(n^2) selection loop is restated as a
// wave reduction: v1 = least frequency with ties to the highest index, v2 =
// the next (exactly what the <= scan of :196-206 selects), merged chains are
// tracked by root label (code_len += 1 for both chains, :213-227) and the
// `next` links are kept so the whole huff_code struct matches.
// ===========================================================================
struct TabScratch {
  int next[257];
  int tail[257];
  int sorted[256];
  int clf[32];       // code_len_freq (all 257 symbols), then limited
  int cnt[32];       // symbols 0..255 per unlimited length
  int base[32];
  int cum[18];       // cumulative limited counts
  int first_code[18];
  int slen[256];
  int scode[256];
  int n;
  int err;
};

__device__ __forceinline__ void top2(unsigned long long &k1, unsigned long long &k2,
                                     unsigned long long o1, unsigned long long o2) {
  // merge sorted pairs (k1<=k2) and (o1<=o2) keeping the two smallest
  const unsigned long long lo = k1 < o1 ? k1 : o1;
  const unsigned long long hi = k1 < o1 ? o1 : k1;
  const unsigned long long m2 = k2 < o2 ? k2 : o2;
  k1 = lo;
  k2 = hi < m2 ? hi : m2;
}

__device__ void build_table_wave(const uint32_t *hist, HuffCode *hc, uint32_t *ehuf,
                                 TabScratch *S, int lane, int *err) {
  uint32_t f[5];
  int cl[5], gr[5];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int s = lane + 64 * i;
    f[i] = s < 256 ? hist[s] : (s == 256 ? 1u : 0u);  // :364-367
    cl[i] = 0;
    gr[i] = s;
    if (s < 257) {
      S->next[s] = -1;
      S->tail[s] = s;
    }
  }
  if (lane < 32) { S->clf[lane] = 0; S->cnt[lane] = 0; }
  wave_lds_sync();
  for (;;) {
    unsigned long long k1 = ~0ull, k2 = ~0ull;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int s = lane + 64 * i;
      if (s < 257 && f[i]) {
        const unsigned long long key = ((unsigned long long)f[i] << 9) | (unsigned)(256 - s);
        top2(k1, k2, key, ~0ull);
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const unsigned long long o1 = __shfl_xor(k1, off);
      const unsigned long long o2 = __shfl_xor(k2, off);
      top2(k1, k2, o1, o2);
    }
    if (k2 == ~0ull) break;
    const int v1 = 256 - (int)(k1 & 511), v2 = 256 - (int)(k2 & 511);
    const uint32_t fs = (uint32_t)(k1 >> 9) + (uint32_t)(k2 >> 9);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int s = lane + 64 * i;
      if (s == v1) f[i] = fs;
      if (s == v2) f[i] = 0;
      if (gr[i] == v1 || gr[i] == v2) {
        cl[i]++;
        gr[i] = v1;
      }
    }
    if (lane == 0) {
      const int t1 = S->tail[v1];
      S->next[t1] = v2;
      S->tail[v1] = S->tail[v2];
    }
    wave_lds_sync();
  }
  wave_lds_sync();
  int bad = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int s = lane + 64 * i;
    if (s < 257) {
      hc->sym_freq[s] = (int)f[i];
      hc->code_len[s] = cl[i];
      hc->next[s] = S->next[s];
      if (cl[i] >= 32) bad = 1;  // the reference indexes code_len_freq out of bounds
      else if (cl[i]) {
        atomicAdd(&S->clf[cl[i]], 1);
        if (s < 256) atomicAdd(&S->cnt[cl[i]], 1);
      }
    }
  }
  if (__ballot(bad)) {
    if (lane == 0) *err = 1;
    return;
  }
  wave_lds_sync();
  if (lane == 0) {
    int *clf = S->clf;
    int nl = 0;
    for (int i = 1; i < 32; i++) nl += clf[i];
    S->err = nl < 2;
    if (!S->err) {
      // :239-259 limit to 16 bits
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
        clf[i]--;
        break;
      }
      int acc = 0;
      for (int L = 0; L < 32; L++) { S->base[L] = acc; acc += S->cnt[L]; }
      S->n = acc;  // symbols 0..255 with a code
      S->cum[0] = 0;
      for (int L = 1; L <= 16; L++) S->cum[L] = S->cum[L - 1] + clf[L];
      // :280-300 canonical codes
      int code = 0, started = 0;
      for (int L = 1; L <= 16; L++) {
        if (started) code <<= 1;
        S->first_code[L] = code;
        if (clf[L]) started = 1;
        code += clf[L];
      }
      if (S->cum[16] != S->n || S->n >= 255) S->err = 1;
    }
  }
  wave_lds_sync();
  if (S->err) {
    if (lane == 0) *err = 1;
    return;
  }
  // :262-268 order symbols 0..255 by (unlimited length, value)
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int s = lane + 64 * i;
    for (int L = 1; L < 32; L++) {
      const unsigned long long m = __ballot(cl[i] == L);
      if (!m) continue;
      if (cl[i] == L) {
        const int pos = S->base[L] + __popcll(m & ((1ull << lane) - 1ull));
        S->sorted[pos] = s;
      }
      if (lane == 0) S->base[L] += __popcll(m);
      wave_lds_sync();
    }
  }
  wave_lds_sync();
  const int n = S->n;
  // every output address is written exactly once, from LDS staging
  for (int k = lane; k < 256; k += 64) {
    S->slen[k] = 0;
    S->scode[k] = -1;
  }
  wave_lds_sync();
  for (int k = lane; k < n; k += 64) {  // :271-276 and :280-300
    int L = 1;
    while (S->cum[L] <= k) L++;
    const int s = S->sorted[k];
    S->slen[s] = L;
    S->scode[s] = S->first_code[L] + (k - S->cum[L - 1]);
  }
  wave_lds_sync();
  if (lane < 32) hc->code_len_freq[lane] = S->clf[lane];
  for (int k = lane; k < 256; k += 64) {
    // sym_sorted: -1 past the end, except that the sentinel write of :277
    // lands in sym_sorted[255] (it aliases sym_code_len[-1], structs.h:10-11)
    hc->sym_sorted[k] = k < n ? S->sorted[k] : (k == 255 ? 0 : -1);
    const int L = S->slen[k];
    hc->sym_code_len[k] = L;
    hc->sym_code[k] = S->scode[k];
    ehuf[k] = L ? ((uint32_t)L << 16) | (uint32_t)S->scode[k] : 0u;
  }
}

__global__ __launch_bounds__(256) void k_tables(EntArgs a) {
  __shared__ TabScratch S[4];
  const int f = blockIdx.x, t = threadIdx.x >> 6, lane = threadIdx.x & 63;
  build_table_wave(a.hist + ((long long)f * 4 + t) * 257, (HuffCode *)a.hc + (long long)f * 4 + t,
                   (uint32_t *)a.ehuf + ((long long)f * 4 + t) * 256, &S[t], lane, a.err + f);
}

// code tables from caller-owned huff_code structs (drop-in write_jpg)
__global__ void k_ehuf_struct(const HuffCode *hc, uint32_t *ehuf) {
  const int t = blockIdx.x;
  for (int s = threadIdx.x; s < 256; s += blockDim.x) {
    const int L = hc[t].sym_code_len[s];
    ehuf[t * 256 + s] = L > 0 ? ((uint32_t)L << 16) | ((uint32_t)hc[t].sym_code[s] & 0xFFFFu) : 0u;
  }
}

// ===========================================================================
// k_bits: bits of every block from its tokens and the frame's code lengths;
// chunk totals.  One thread per block.
// ===========================================================================
__global__ __launch_bounds__(256) void k_bits(EntArgs a) {
  __shared__ uint32_t tab[2][256];
  __shared__ uint32_t wsum[4];
  const Chunk c = chunk_of(a.g, blockIdx.x);
  const uint32_t *et = a.ehuf + ((long long)c.f * 4 + (c.comp ? 2 : 0)) * 256;
  for (int i = threadIdx.x; i < 512; i += 256) tab[i >> 8][i & 255] = et[i];
  __syncthreads();
  const int t = threadIdx.x;
  uint32_t bits = 0;
  if (t < c.n) {
    const long long gb = (long long)c.f * a.g.nblk + c.first + t;
    const uint32_t *tok = a.tok + gb * 64;
    const int hd = a.hdr[gb];
    const int n = hd & 63;
    const int dcls = (int)(tok[0] & 255u);
    bits = (tab[0][dcls] >> 16) + (uint32_t)dcls;
    const uint32_t lz = tab[1][0xF0] >> 16;
    for (int i = 1; i <= n; i++) {
      const uint32_t tk = tok[i];
      const uint32_t sym = tk & 255u;
      bits += (tab[1][sym] >> 16) + (sym & 15u) + ((tk >> 8) & 3u) * lz;
    }
    if (hd & 128) bits += tab[1][0x00] >> 16;
    a.bits[gb] = bits;
  }
  uint32_t x = bits;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
  if ((t & 63) == 0) wsum[t >> 6] = x;
  __syncthreads();
  if (t == 0) a.chunk_bits[blockIdx.x] = (unsigned long long)wsum[0] + wsum[1] + wsum[2] + wsum[3];
}


// ===========================================================================
// k_scan: per scan (frame, component) exclusive scan of chunk bit totals;
// zeroes the words a chunk shares with a neighbour (they are OR-combined).
// One wave per scan.
// ===========================================================================
__global__ void k_scan(EntArgs a) {
  const int sid = blockIdx.x;  // frame * 3 + comp
  const int f = sid / 3, comp = sid - f * 3;
  const int lane = threadIdx.x;
  const int q0 = f * a.g.cpf + (comp == 0 ? 0 : a.g.cy + (comp - 1) * a.g.cc);
  const int nq = comp == 0 ? a.g.cy : a.g.cc;
  uint32_t *raw = a.raw + (long long)f * a.g.raw_fs +
                  (comp == 0 ? 0 : a.g.raw_words[0] + (comp == 2 ? a.g.raw_words[1] : 0));
  unsigned long long carry = 0;
  for (int base = 0; base < nq; base += 64) {
    const int i = base + lane;
    const unsigned long long v = i < nq ? a.chunk_bits[q0 + i] : 0ull;
    unsigned long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    const unsigned long long excl = carry + x - v;
    if (i < nq) {
      a.chunk_off[q0 + i] = excl;
      raw[excl >> 5] = 0;
      raw[(excl + v - 1) >> 5] = 0;
    }
    carry += __shfl(x, 63);
  }
  if (lane == 0) a.scan_bits[sid] = carry;
}

// ===========================================================================
// k_pack: bit-pack one chunk into LDS, then store it.  Thread t writes block
// t's tokens at the block's offset (chunk offset + exclusive scan of block
// bits); pieces are OR-ed into LDS words in big-endian bit order.  Interior
// words are stored plainly, the two words shared with neighbouring chunks
// atomically (k_scan zeroed them).
// ===========================================================================
__device__ __forceinline__ void put_bits(uint32_t *buf, uint32_t pos, uint32_t val, int len) {
  // len in 1..28, val < 2^len
  const uint32_t w = pos >> 5;
  const int sh = 32 - (int)(pos & 31) - len;
  if (sh >= 0) {
    atomicOr(&buf[w], val << sh);
  } else {
    atomicOr(&buf[w], val >> (-sh));
    atomicOr(&buf[w + 1], val << (32 + sh));
  }
}

__global__ __launch_bounds__(256) void k_pack(EntArgs a) {
  __shared__ uint32_t buf[CHUNK_WORDS];
  __shared__ uint32_t tab[2][256];
  __shared__ uint32_t wsum[4];
  const Chunk c = chunk_of(a.g, blockIdx.x);
  const uint32_t *et = a.ehuf + ((long long)c.f * 4 + (c.comp ? 2 : 0)) * 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 512; i += 256) tab[i >> 8][i & 255] = et[i];
  const long long gb = (long long)c.f * a.g.nblk + c.first + tid;
  const uint32_t mybits = tid < c.n ? a.bits[gb] : 0u;
  uint32_t x = mybits;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < wave; w++) wbase += wsum[w];
  const uint32_t chunk_bits = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const unsigned long long base = a.chunk_off[blockIdx.x];
  const uint32_t bit0 = (uint32_t)(base & 31);
  const uint32_t nw = (bit0 + chunk_bits + 31) >> 5;
  for (uint32_t i = tid; i < nw; i += 256) buf[i] = 0;
  __syncthreads();
  if (tid < c.n) {
    uint32_t pos = bit0 + wbase + x - mybits;
    const uint32_t *tok = a.tok + gb * 64;
    const int hd = a.hdr[gb];
    const int n = hd & 63;
    uint32_t tk = tok[0];
    int cls = (int)(tk & 255u);
    uint32_t e = tab[0][cls];
    int L = (int)(e >> 16);
    put_bits(buf, pos, ((e & 0xFFFFu) << cls) | (tk >> 16), L + cls);  // :434-446
    pos += L + cls;
    const uint32_t zrl = tab[1][0xF0];
    const int Lz = (int)(zrl >> 16);
    for (int i = 1; i <= n; i++) {
      tk = tok[i];
      for (uint32_t k = (tk >> 8) & 3u; k; k--) {  // :490-494 ZRL
        put_bits(buf, pos, zrl & 0xFFFFu, Lz);
        pos += Lz;
      }
      const uint32_t sym = tk & 255u;
      cls = (int)(sym & 15u);
      e = tab[1][sym];
      L = (int)(e >> 16);
      put_bits(buf, pos, ((e & 0xFFFFu) << cls) | (tk >> 16), L + cls);  // :448-460
      pos += L + cls;
    }
    if (hd & 128) {  // :479-484 EOB
      e = tab[1][0x00];
      put_bits(buf, pos, e & 0xFFFFu, (int)(e >> 16));
    }
  }
  __syncthreads();
  uint32_t *raw = a.raw + (long long)c.f * a.g.raw_fs +
                  (c.comp == 0 ? 0 : a.g.raw_words[0] + (c.comp == 2 ? a.g.raw_words[1] : 0)) +
                  (base >> 5);
  for (uint32_t i = tid; i < nw; i += 256) {
    if (i == 0 || i == nw - 1) atomicOr(&raw[i], buf[i]);
    else raw[i] = buf[i];
  }
}


// ===========================================================================
// k_emit: one workgroup per frame assembles the JFIF stream (encoder.c
// :549-644): SOI/APP0, DQT x2, DHT x4, SOF0, then per component SOS + the
// scan bytes with 0xFF 0x00 stuffing (:405-408) + the pad byte of
// fill_last_byte (:425-432: 1-bits OR-ed into the free low bits, a whole 0xFF
// when the scan ended byte-aligned, never stuffed), then EOI.
// ===========================================================================
__global__ __launch_bounds__(256) void k_emit(EntArgs a) {
  __shared__ uint32_t s_ff[256];
  __shared__ unsigned long long s_pos;
  const int f = blockIdx.x, tid = threadIdx.x;
  if (a.err[f]) {
    if (tid == 0) a.out_len[f] = 0;
    return;
  }
  uint8_t *out = a.out + (long long)f * a.g.out_cap;
  const HuffCode *hc = a.hc + (long long)f * 4;
  if (tid == 0) {
    unsigned long long p = 0;
    const uint8_t app0[20] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 0x4A, 0x46, 0x49, 0x46,
                              0x00, 0x01, 0x01, 0x00, 0x00, 0x48, 0x00, 0x48, 0x00, 0x00};
    for (int i = 0; i < 20; i++) out[p++] = app0[i];
    for (int t = 0; t < 2; t++) {
      out[p++] = 0xFF; out[p++] = 0xDB; out[p++] = 0x00; out[p++] = 0x43; out[p++] = (uint8_t)t;
      for (int i = 0; i < 64; i++) out[p++] = (uint8_t)a.tab->dqt[t][i];
    }
    const int tcth[4] = {0x00, 0x10, 0x01, 0x11};
    for (int t = 0; t < 4; t++) {
      int n = 0;
      for (int i = 1; i <= 16; i++) n += hc[t].code_len_freq[i];
      const int len = 19 + n;
      out[p++] = 0xFF; out[p++] = 0xC4;
      out[p++] = (uint8_t)(len >> 8); out[p++] = (uint8_t)len;
      out[p++] = (uint8_t)tcth[t];
      for (int i = 1; i <= 16; i++) out[p++] = (uint8_t)hc[t].code_len_freq[i];
      for (int i = 0; i < n; i++) out[p++] = (uint8_t)hc[t].sym_sorted[i];
    }
    const int W = a.g.w, H = a.g.h;
    const uint8_t sof[19] = {0xFF, 0xC0, 0x00, 0x11, 0x08, (uint8_t)(H >> 8), (uint8_t)H,
                             (uint8_t)(W >> 8), (uint8_t)W, 0x03, 0x01, 0x22, 0x00,
                             0x02, 0x11, 0x01, 0x03, 0x11, 0x01};
    for (int i = 0; i < 19; i++) out[p++] = sof[i];
    s_pos = p;
  }
  __syncthreads();
  for (int comp = 0; comp < 3; comp++) {
    if (tid == 0) {
      unsigned long long p = s_pos;
      const uint8_t sos[10] = {0xFF, 0xDA, 0x00, 0x08, 0x01, (uint8_t)(comp + 1),
                               (uint8_t)(comp ? 0x11 : 0x00), 0x00, 0x3F, 0x00};
      for (int i = 0; i < 10; i++) out[p++] = sos[i];
      s_pos = p;
    }
    __syncthreads();
    const uint32_t *raw = a.raw + (long long)f * a.g.raw_fs +
                          (comp == 0 ? 0 : a.g.raw_words[0] + (comp == 2 ? a.g.raw_words[1] : 0));
    const unsigned long long nbits = a.scan_bits[f * 3 + comp];
    const unsigned long long nbytes = nbits >> 3;
    unsigned long long pos = s_pos;
    for (unsigned long long b0 = 0; b0 < nbytes; b0 += 256 * 16) {
      const unsigned long long mb = b0 + (unsigned long long)tid * 16;
      uint32_t w4[4] = {0, 0, 0, 0};
      int cnt = 0;
      if (mb < nbytes) {
        const uint4 v = *(const uint4 *)(raw + (mb >> 2));
        w4[0] = v.x; w4[1] = v.y; w4[2] = v.z; w4[3] = v.w;
        const int lim = (int)min(16ull, nbytes - mb);
        for (int k = 0; k < lim; k++) cnt += ((w4[k >> 2] >> (24 - 8 * (k & 3))) & 255u) == 255u;
      }
      // workgroup exclusive scan of the 0xFF counts
      int xs = cnt;
      const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(xs, off);
        if (lane >= off) xs += y;
      }
      if (lane == 63) s_ff[wave] = (uint32_t)xs;
      __syncthreads();
      int wb = 0, tot = 0;
      for (int w = 0; w < 4; w++) { if (w < wave) wb += (int)s_ff[w]; tot += (int)s_ff[w]; }
      if (mb < nbytes) {
        unsigned long long o = pos + (unsigned long long)tid * 16 + (unsigned long long)(wb + xs - cnt);
        const int lim = (int)min(16ull, nbytes - mb);
        for (int k = 0; k < lim; k++) {
          const uint8_t byte = (uint8_t)(w4[k >> 2] >> (24 - 8 * (k & 3)));
          out[o++] = byte;
          if (byte == 0xFF) out[o++] = 0x00;
        }
      }
      const unsigned long long step = min(256ull * 16, nbytes - b0);
      pos += step + (unsigned long long)tot;
      __syncthreads();
    }
    if (tid == 0) {
      const int r = (int)(nbits & 7);
      uint8_t pad = 0xFF;
      if (r) {
        const uint8_t part = (uint8_t)(raw[nbytes >> 2] >> (24 - 8 * (nbytes & 3)));
        pad = (uint8_t)(part | ((1u << (8 - r)) - 1u));
      }
      out[pos++] = pad;
      s_pos = pos;
    }
    __syncthreads();
  }
  if (tid == 0) {
    unsigned long long p = s_pos;
    out[p++] = 0xFF;
    out[p++] = 0xD9;
    a.out_len[f] = p;
  }
}

// ---- tiny self-test used by the test-suite: exact i8 MFMA layout check ----
__global__ void k_mfma_probe(const int4 *A, const int4 *B, int4 *D) {
  const int lane = threadIdx.x;
  const int4 a4 = A[lane], b4 = B[lane];
  const v4i a = {a4.x, a4.y, a4.z, a4.w}, b = {b4.x, b4.y, b4.z, b4.w};
  const v4i z = {0, 0, 0, 0};
  const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, z, 0, 0, 0);
  D[lane] = int4{d[0], d[1], d[2], d[3]};
}

// ===========================================================================
// host-side launch wrappers (kernels are launched only through these)
// ===========================================================================
static int g_k1_blocks_per_cu = -1;

int k1_grid(int device, long long ntiles) {
  if (g_k1_blocks_per_cu < 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_mcu_dct, 256, 0) != hipSuccess || nb < 1)
      nb = 1;
    g_k1_blocks_per_cu = nb;
  }
  hipDeviceProp_t prop;
  int cus = 256;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus = prop.multiProcessorCount;
  long long want = (ntiles + K1_WAVES - 1) / K1_WAVES;
  long long cap = (long long)cus * g_k1_blocks_per_cu;
  return (int)(want < cap ? want : cap);
}

hipError_t launch_colour_lut(uint32_t *lut, hipStream_t s) {
  hipLaunchKernelGGL(k_colour_lut, dim3(256), dim3(256), 0, s, lut);
  return hipGetLastError();
}
hipError_t launch_k1(const K1Args &a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_mcu_dct, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_dc_diff(int16_t *coef, const int16_t *dc, const Geom &g, int nframes,
                          hipStream_t s) {
  long long n = (long long)nframes * g.nblk;
  hipLaunchKernelGGL(k_dc_diff, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, coef, dc, g,
                     nframes);
  return hipGetLastError();
}
hipError_t launch_stats(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_tokens, dim3(a.nframes * a.g.cpf), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_tables(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_tables, dim3(a.nframes), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_ehuf_struct(const HuffCode *hc, uint32_t *ehuf, hipStream_t s) {
  hipLaunchKernelGGL(k_ehuf_struct, dim3(4), dim3(256), 0, s, hc, ehuf);
  return hipGetLastError();
}
hipError_t launch_bits(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_bits, dim3(a.nframes * a.g.cpf), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_scan(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_scan, dim3(a.nframes * 3), dim3(64), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_pack(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_pack, dim3(a.nframes * a.g.cpf), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_emit(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_emit, dim3(a.nframes), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_mfma_probe(const int4 *A, const int4 *B, int4 *D, hipStream_t s) {
  hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, s, A, B, D);
  return hipGetLastError();
}

}  // namespace mij
