// mij_kernels.hip -- gfx950 (CDNA4) kernels of the MI355X JPEG block-encode
// path.  Reference: MattiaDallaCosta/JPEG-encoder-decoder main/encoder.c.
//
//   k_colour_lut   colour-exception bitmaps (encoder.c:133-135 in FP64)
//   k_mcu_dct      K1: BGR -> YCbCr -> 4:2:0 -> DCT (i8 MFMA, exact integer)
//                  -> quantize/trunc (+FP64 replay near boundaries) -> zigzag
//                  (encoder.c:121-150, :81-112, :65-70)
//   k_dc_diff      DC differencing into the coefficient planes (:168-177)
//                  and (token mode) per-segment symbol streams + histograms
//                  (:315-358, :462-502)
//   k_seg_dc       DC token of each segment's first block (:168-177)
//   k_tables       optimized Huffman tables, wave-parallel (:180-301)
//   k_ehuf_struct  code tables from caller-owned huff_code structs
//   k_seg_bits     bits per segment
//   k_scan         per-scan offsets of each segment
//   k_pack_flat    segment bits + look-back offsets + bit packing (:434-502)
//   k_emit         JFIF assembly + 0xFF stuffing + pad quirks (:383-432,
//                  :504-644)
//
// Compiled with -ffp-contract=off: every FP64 operation that has to match the
// reference is written with explicit __dmul_rn/__dadd_rn in the reference's
// evaluation order; fp32 FMAs are explicit fmaf() calls.
#include <stdlib.h>

#include "mij_internal.h"

namespace mij {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

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

// DPP row_shr:n with zero fill (lanes below n in their 16-lane row read 0)
template <int N>
__device__ __forceinline__ uint32_t row_shr0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + N, 0xF, 0xF, true);
}
// inclusive prefix sum inside each 16-lane row
__device__ __forceinline__ uint32_t row_scan16(uint32_t x) {
  x += row_shr0<1>(x);
  x += row_shr0<2>(x);
  x += row_shr0<4>(x);
  x += row_shr0<8>(x);
  return x;
}
// lane 15 of each 16-lane row, broadcast to the row (DPP row_newbcast:15)
__device__ __forceinline__ uint32_t row_last(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x15F, 0xF, 0xF, false);
}
// inclusive prefix sum over the wave (row scans + row_bcast:15 / row_bcast:31)
__device__ __forceinline__ uint32_t wave_scan64(uint32_t x) {
  x = row_scan16(x);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return x;
}

__device__ __forceinline__ int mag_class(int v) {  // encoder.c:303-313
  v = v < 0 ? -v : v;
  return 32 - __clz(v);
}

// Magnitude bits of a value of class cls (encoder.c:442-444 / :456-458:
// negative values are written as ~|v|, i.e. the low cls bits of v-1).
__device__ __forceinline__ uint32_t mag_bits(int v, int cls) {
  uint32_t id = (uint32_t)(v < 0 ? -v : v);
  if (v < 0) id = ~id;
  return id & ((1u << cls) - 1u);
}

// ===========================================================================
// Colour-exception bitmaps.  Exact-integer colour values for which the FP64
// expression of encoder.c:133-135 lands one ulp-ish below the integer, so the
// uint8_t truncation yields value-1.  Y indexed by (R,G) (the B of an integer
// point is unique), Cb by (G,B) with R==G, Cr by (G,R) with B==G.
// ===========================================================================
__global__ void k_colour_lut(uint32_t *lut /* [3][LUT_WORDS] */) {
  // An exact-integer colour value needs equal parities: Y: 299R+587G+114B
  // == 0 (mod 1000) forces R == G (mod 2); Cb needs R == G and B == G (mod
  // 2); Cr needs B == G and R == G (mod 2).  So each table has 2^15 entries:
  // Y by (R, G>>1), Cb by (G, B>>1), Cr by (G, R>>1).
  int i = blockIdx.x * blockDim.x + threadIdx.x;  // 0 .. 32767
  if (i >= 32768) return;
  const int hi = i >> 7, lo = i & 127;
  bool ey = false, ecb = false, ecr = false;
  {  // Y: R = hi, G = 2*lo + (R & 1)
    const int R = hi, G = 2 * lo + (R & 1);
    for (int B = 0; B < 256; B++) {
      const int n = 299 * R + 587 * G + 114 * B;
      if (n % 1000) continue;
      const double y = __dadd_rn(__dadd_rn(__dmul_rn(0.299, (double)R), __dmul_rn(0.587, (double)G)),
                                 __dmul_rn(0.114, (double)B));
      ey = (int)y != n / 1000;
    }
  }
  {  // Cb: G = hi, B = 2*lo + (G & 1), R = G
    const int G = hi, B = 2 * lo + (G & 1), R = G;
    const long long n = 128000000LL - 168736LL * R - 331264LL * G + 500000LL * B;
    if (n % 1000000 == 0) {
      const double cb = __dadd_rn(__dadd_rn(__dadd_rn(128.0, -__dmul_rn(0.168736, (double)R)),
                                            -__dmul_rn(0.331264, (double)G)),
                                  __dmul_rn(0.5, (double)B));
      ecb = (int)cb != (int)(n / 1000000);
    }
  }
  {  // Cr: G = hi, R = 2*lo + (G & 1), B = G
    const int G = hi, R = 2 * lo + (G & 1), B = G;
    const long long n = 128000000LL + 500000LL * R - 418688LL * G - 81312LL * B;
    if (n % 1000000 == 0) {
      const double cr = __dadd_rn(__dadd_rn(__dadd_rn(128.0, __dmul_rn(0.5, (double)R)),
                                            -__dmul_rn(0.418688, (double)G)),
                                  -__dmul_rn(0.081312, (double)B));
      ecr = (int)cr != (int)(n / 1000000);
    }
  }
  if (ey) atomicOr(&lut[0 * LUT_WORDS + (i >> 5)], 1u << (i & 31));
  if (ecb) atomicOr(&lut[1 * LUT_WORDS + (i >> 5)], 1u << (i & 31));
  if (ecr) atomicOr(&lut[2 * LUT_WORDS + (i >> 5)], 1u << (i & 31));
}

// ===========================================================================
// K1 helpers
// ===========================================================================

// DC of one block exactly as encoder.c:87-109: the cosines of frequency 0
// are exactly 1.0, so both passes are exact integer sums S; what remains is
// fl(fl(fl(S*r)*r)/4) / q with r = M_SQRT1_2, then truncation.
__device__ __forceinline__ int dc_exact(int S, int q) {
  double f = __dmul_rn(__dmul_rn((double)S, SQRT1_2), SQRT1_2);
  f = __dmul_rn(f, 0.25);
  int t = (int)__ddiv_rn(f, (double)q);
  return t < -2048 ? -2048 : (t > 2047 ? 2047 : t);
}

// DC fast path: the reference's FP64 DC (dc_exact) equals trunc(S / 8q) with
// the sign of S, except possibly when |S| is a multiple of 8q (then its FP64
// roundings decide between K and K-1).  k = trunc(|S|*fl(1/8q) + 2e-4) is
// floor(|S|/8q) exactly: the fp32 error is < 1.2e-4 and a non-integer |S|/8q
// is >= 1/2040 from an integer.  `tie` flags the |S| = K*8q (K > 0) case.
__device__ __forceinline__ int dc_fast(int S, int q8, float inv8q, bool &tie) {
  const int s = S >> 31;
  const int a = (S ^ s) - s;
  const int k = (int)fmaf((float)a, inv8q, 2e-4f);
  tie = a != 0 && k * q8 == a;
  return (k ^ s) - s;
}

// DC at a tie |S| = K * 8q: the FP64 chain of dc_exact lands on K or K - 1
// depending only on K and q; Tables::dctie holds "K - 1" bits per K, built on
// the host with the reference's double operations (mij_api.hip fill_tables).
// d = the fast-path value (+-K).
__device__ __forceinline__ int dc_tie(int d, const uint32_t *bits) {
  const int s = d >> 31;
  int k = (d ^ s) - s;
  k -= (int)((bits[k >> 5] >> (k & 31)) & 1u);
  return (k ^ s) - s;
}

// ===========================================================================
// K1: fused colour conversion + 4:2:0 + DCT + quantization + zigzag.
//
// Persistent grid; workgroup w owns a contiguous range of 128x16 tiles and
// its 4 waves take every 4th tile of it.  Per tile a wave:
//   1. the tile's 16 rows of BGR888 arrive in LDS by LDS-DMA, issued while
//      the previous tile was in its DCT phase; each lane reads 12 B = 4 px
//      per row, converts a 4x2 patch per step, averages the
//      two 2x2 chroma quads, and stages Y/Cb/Cr bytes in LDS in block-major
//      order (64 px per 8x8 block, LDS_BLK stride).
//   2. three MFMA N-tiles of 16 blocks (Y block row 0, Y block row 1,
//      Cb|Cr): v_mfma_i32_16x16x64_i8 with B = the blocks' pixels - 128
//      (exact int8) and A = the 64x64 DCT matrix (rows in zigzag order,
//      cos*cos*scale * 2^19 rounded) split into three base-128 digits, read
//      from LDS.  The int32 sum N is exact; N / 2^21 is the un-quantized
//      coefficient to within 0.002, and the DC row holds the
//      exact pixel sum.
//   3. quantize with trunc; a coefficient whose +-tau interval straddles a
//      truncation boundary is recomputed in FP64 exactly like the reference.
//   4. lane (g, b) owns zigzag coefficients 16g..16g+15 of block b: two
//      16-byte stores per lane.
// ===========================================================================
struct TilePos {
  int f, tx, ty, valid_px;
};

__device__ __forceinline__ TilePos tile_pos(const Geom &G, int t) {
  TilePos p;
  p.f = (int)div_by((uint32_t)t, G.tpf_m, G.tpf_s);
  const int rem = t - p.f * G.tiles_per_frame;
  p.ty = (int)div_by((uint32_t)rem, G.tx_m, G.tx_s);
  p.tx = rem - p.ty * G.tiles_x;
  p.valid_px = min(TILE_W, G.w - p.tx * TILE_W);
  return p;
}

// region batches: the tile inside its frame's own size (valid_px), and
// whether it holds any of the frame (the canvas tiles outside are skipped)
__device__ __forceinline__ TilePos tile_pos_r(const Geom &G, const int2 *fd, int t, bool &ok) {
  TilePos p = tile_pos(G, t);
  const FGeom fg = frame_geom(G, fd, p.f);
  p.valid_px = min(TILE_W, fg.w - p.tx * TILE_W);
  ok = p.tx < fg.tiles_x && p.ty < fg.rows;
  return p;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void global_void_t;
constexpr int TILE_RAW = TILE_W * 3 * TILE_H;  // 6144 B of BGR888 per tile

// Streams a tile's 16 rows x 384 B into LDS with global_load_lds_dwordx4 (no
// VGPRs for the data): instruction k moves rows 2k and 2k+1 = LDS bytes
// [768k, 768k + 768); lane i < 48 moves the 16 B at row 2k + i / 24, column
// 16 * (i % 24).  One per-lane offset serves all eight instructions (DmaOff,
// one VGPR for the kernel); instruction k's scalar base is the tile's base +
// 2k rows (an SGPR pair each, SALU adds) and its LDS base m0 = base + 768k.
// (Eight per-lane offsets, one per instruction, held eight VGPRs for the
// whole kernel: at 168 the coefficient variant spilled one pair, and the
// reload before every tile's DMA waited, vmcnt(0), for the previous tile's
// coefficient stores.)
constexpr int DMA_K = TILE_H / 2;
struct DmaOff {
  uint32_t v;
};
__device__ __forceinline__ DmaOff dma_offsets(int pitch, int lane) {
  const int l = lane < 48 ? lane : 0;
  return DmaOff{(uint32_t)((l / 24) * pitch + (l % 24) * 16)};
}
template <int K>
__device__ __forceinline__ void dma_one(uint32_t off, uint32_t lds, const uint8_t *src) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, %2 nt" : : "v"(off), "s"(lds), "s"(src)
               : "memory", "m0");
}
__device__ __forceinline__ void issue_tile_dma(const K1Args &a, const TilePos &p, int lane, uint8_t *raw,
                                               const DmaOff &off) {
  const uint64_t srcv = (uint64_t)(uintptr_t)(a.in + (long long)p.f * a.in_fs +
                                              (long long)(p.ty * TILE_H) * a.pitch + p.tx * TILE_W * 3);
  // (wave-uniform; readfirstlane keeps it in SGPRs for the "s" operand)
  // (readfirstlane returns int: widen through uint32_t, never sign-extend)
  const uint32_t src_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(srcv >> 32));
  const uint32_t src_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)srcv);
  const uint8_t *src = (const uint8_t *)(uintptr_t)(((uint64_t)src_hi << 32) | (uint64_t)src_lo);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t *)raw);
  const long long step = 2LL * a.pitch;  // kernel argument: an SGPR
  // right frame edge: only the valid columns
  const bool on = lane < 48 && (p.valid_px == TILE_W || (lane % 24) * 16 < p.valid_px * 3);
  // issued as asm so the compiler does not tie the next LDS read of `raw` to
  // vmcnt(0) -- that wait would also drain the previous tile's coefficient
  // stores; K1 waits for the DMA itself (dma_wait) before its first store,
  // when the DMA has long landed
  if (on) {
    dma_one<0>(off.v, lds0, src);
    dma_one<1>(off.v, lds0 + 768, src + step);
    dma_one<2>(off.v, lds0 + 1536, src + 2 * step);
    dma_one<3>(off.v, lds0 + 2304, src + 3 * step);
    dma_one<4>(off.v, lds0 + 3072, src + 4 * step);
    dma_one<5>(off.v, lds0 + 3840, src + 5 * step);
    dma_one<6>(off.v, lds0 + 4608, src + 6 * step);
    dma_one<7>(off.v, lds0 + 5376, src + 7 * step);
  }
}
static_assert(DMA_K == 8 && TILE_W * 3 * 2 == 768, "issue_tile_dma: 8 instructions of 2 rows x 384 B");

// all of this wave's outstanding vector-memory operations (the tile DMA above
// included) have completed; VMEM operations retire in issue order
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// the tile DMA has landed once at most the wave's 6 youngest VMEM operations
// are outstanding: the coefficient variant issues 9 stores per tile (2
// coefficient + 1 raw-DC store per N-tile) after it, so the previous tile's
// stores stay in flight across the wait
__device__ __forceinline__ void dma_wait_behind_stores() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }

// byte N of w as float (v_cvt_f32_ubyteN); asm keeps the compiler from
// rewriting fsub(cvt(a), cvt(b)) into cvt(sub(a, b)), which costs two slow
// conversions instead of one
template <int N>
__device__ __forceinline__ float ubyte_f32(uint32_t w) {
  float r;
  if constexpr (N == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(w));
  else if constexpr (N == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(w));
  else if constexpr (N == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(w));
  else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(w));
  return r;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// low 16 bits of lo | low 16 bits of hi << 16 (one v_perm_b32)
__device__ __forceinline__ uint32_t pack_i16x2(int lo, int hi) {
  return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}

// a + k in both halves (v_pk_add_f32 with k in an SGPR): the compiler would
// otherwise split a packed add of a non-inline constant into two VALU adds
__device__ __forceinline__ f2v pk_add_k(f2v a, float k) {
  f2v r;
  const unsigned long long kk = __float_as_uint(k);
  asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "s"(kk));
  return r;
}

// Chroma in "magic" form: x + 1.5*2^23 rounds x to an integer held in the low
// mantissa bits, so bits(x + MAGIC) - MAGIC_BITS = round(x) and four such bit
// patterns add as integers.  The chroma expressions carry a -0.5 + 2^-16
// bias (CH_BIAS = 128 - 0.5 + 2^-16), which turns the rounding into the
// floor of the exact value.
constexpr float CH_BIAS = 127.5f + 0x1p-16f;
constexpr float MAGIC = 12582912.0f;  // 1.5 * 2^23
constexpr uint32_t MAGIC_BITS = 0x4B400000u;

// Colour conversion of 4 pixels (12 bytes) of one row, encoder.c:133-135.
// fp32 forms (error < 2e-5 Y, < 1e-5 Cb/Cr) give the floor
// of the exact value; the FP64 reference differs from it only at
// exact-integer values, which need equal parities and R == G (Cb) or B == G
// (Cr), or fract(Y) ~ 0: there the device-built bitmaps say whether the
// reference lands one below.  This is the common path: it only flags a
// 4-pixel run that holds such a point (a product of the R-G and B-G
// differences, a min of the Y fractions); the bitmap corrections are
// applied by y_fix / chroma_fix to the values already staged in LDS, so the
// common path carries no merge copies.
// Y in magic form too (round 5): fl(Y + 1.5 * 2^13) rounds Y to a multiple
// of 2^-10, so its bits are 0x46400000 + round(1024 Y); with the fp32 chain
// within 2e-5 of the exact value, floor(Y) is bits 10-17 and an integer Y
// is exactly "low 10 bits zero" (non-integers are >= 1e-3 away: their low
// bits lie in [1, 1023]).  tests/colour_check.c checks both over all 2^24
// colours.  This replaced a +0.0005 bias, a truncating conversion and a
// fract per pixel (two slow-class VALU ops) by one fast shift and one AND.
// Outputs: yb = Y in magic form, cbm/crm = chroma in magic form, pd = 0 when
// the run holds a possible Cb/Cr exception, cy = it holds a possible Y one.
constexpr float YMAGIC = 12288.0f;  // 1.5 * 2^13
struct Run4 {
  uint32_t yb[4];
  uint32_t cbm[4], crm[4];
  float pd;  // product of the run's R-G and B-G differences (0: a possible Cb/Cr exception)
  bool cy;
};

template <bool RGB>
__device__ __forceinline__ void convert4(uint32_t w0, uint32_t w1, uint32_t w2, Run4 &o) {
  // BGR of pixel p: w0 = B0 G0 R0 B1, w1 = G1 R1 B2 G2, w2 = R2 B3 G3 R3
  // (RGB input -- PPM order -- swaps the first and third byte of each pixel)
  const f2v f0[2] = {{ubyte_f32<0>(w0), ubyte_f32<3>(w0)}, {ubyte_f32<2>(w1), ubyte_f32<1>(w2)}};
  const f2v fg[2] = {{ubyte_f32<1>(w0), ubyte_f32<0>(w1)}, {ubyte_f32<3>(w1), ubyte_f32<2>(w2)}};
  const f2v f2[2] = {{ubyte_f32<2>(w0), ubyte_f32<1>(w1)}, {ubyte_f32<0>(w2), ubyte_f32<3>(w2)}};
  const f2v(&fb)[2] = RGB ? f2 : f0;
  const f2v(&fr)[2] = RGB ? f0 : f2;
  f2v dr[2], db[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    dr[h] = fr[h] - fg[h];
    db[h] = fb[h] - fg[h];
    const f2v yf = pk_add_k(__builtin_elementwise_fma((f2v)0.114f, db[h],
                                                      __builtin_elementwise_fma((f2v)0.299f, dr[h], fg[h])),
                            YMAGIC);
    const f2v cb = pk_add_k(__builtin_elementwise_fma((f2v)-0.168736f, dr[h],
                                                      __builtin_elementwise_fma((f2v)0.5f, db[h], (f2v)CH_BIAS)),
                            MAGIC);
    const f2v cr = pk_add_k(__builtin_elementwise_fma((f2v)-0.081312f, db[h],
                                                      __builtin_elementwise_fma((f2v)0.5f, dr[h], (f2v)CH_BIAS)),
                            MAGIC);
#pragma unroll
    for (int e = 0; e < 2; e++) {
      // (element copies first: __builtin_bit_cast of a vector element
      // subscript yields element 0 with this compiler)
      const float ye = yf[e], cbe = cb[e], cre = cr[e];
      o.yb[2 * h + e] = __float_as_uint(ye);
      o.cbm[2 * h + e] = __float_as_uint(cbe);
      o.crm[2 * h + e] = __float_as_uint(cre);
    }
  }
  // some pixel has R == G or B == G: the product of the 8 (exact, integer)
  // differences is 0; colour_stage multiplies the two rows' products (16
  // nonzero integer factors: |product| <= 255^16 < 2^128, no overflow, and
  // >= 1, no underflow) and tests once per run pair
  const f2v pd = (dr[0] * db[0]) * (dr[1] * db[1]);
  o.pd = pd[0] * pd[1];
  // some pixel has an exact-integer Y: the low 10 bits of its magic form are 0
  const uint32_t m01 = min(o.yb[0] & 0x3FFu, o.yb[1] & 0x3FFu), m23 = min(o.yb[2] & 0x3FFu, o.yb[3] & 0x3FFu);
  o.cy = min(m01, m23) == 0u;
}

// The reference's colour expressions in FP64, operation for operation
// (encoder.c:133-135: left to right, no contraction), truncated to uint8_t
// (k_fix_blocks' recomputation of listed blocks).
__device__ __forceinline__ int y_f64(uint32_t R, uint32_t G, uint32_t B) {
  const double y = __dadd_rn(__dadd_rn(__dmul_rn(0.299, (double)R), __dmul_rn(0.587, (double)G)),
                             __dmul_rn(0.114, (double)B));
  return (int)(uint8_t)(int)y;
}
__device__ __forceinline__ int cb_f64(uint32_t R, uint32_t G, uint32_t B) {
  const double v = __dadd_rn(__dadd_rn(__dadd_rn(128.0, -__dmul_rn(0.168736, (double)R)),
                                       -__dmul_rn(0.331264, (double)G)),
                             __dmul_rn(0.5, (double)B));
  return (int)(uint8_t)(int)v;
}
__device__ __forceinline__ int cr_f64(uint32_t R, uint32_t G, uint32_t B) {
  const double v = __dadd_rn(__dadd_rn(__dadd_rn(128.0, __dmul_rn(0.5, (double)R)),
                                       -__dmul_rn(0.418688, (double)G)),
                             -__dmul_rn(0.081312, (double)B));
  return (int)(uint8_t)(int)v;
}

// Rare path: the Y corrections of a run as a packed byte-wise subtrahend.
// Only the pixel slots that hold an exact-integer Y in some lane pay for a
// bitmap read (one wave-uniform branch per slot), and the read walks the
// lanes that need it with scalar loads: a vector load's s_waitcnt vmcnt(0)
// would also wait for every token store still in flight.  (Measured and
// dropped, round 5: the flagged lanes evaluating the reference's FP64
// expression (y_f64) instead of the walk -- token K1 2.96 -> 3.01 ms at Q=50,
// 4.56 -> 4.63 at Q=90: more code and SGPR spills in the colour stage.)
// (GLOBAL_LUT false: the bitmap is in LDS, read per lane)
template <bool RGB, bool GLOBAL_LUT>
__device__ __forceinline__ uint32_t y_fix(uint32_t w0, uint32_t w1, uint32_t w2, const uint32_t (&yb)[4],
                                          const uint32_t *__restrict__ lut, int lane) {
  const uint32_t Gv[4] = {(w0 >> 8) & 255, w1 & 255, w1 >> 24, (w2 >> 16) & 255};
  const uint32_t B0[4] = {w0 & 255, w0 >> 24, (w1 >> 16) & 255, (w2 >> 8) & 255};
  const uint32_t R0[4] = {(w0 >> 16) & 255, (w1 >> 8) & 255, w2 & 255, w2 >> 24};
  const uint32_t(&Rv)[4] = RGB ? B0 : R0;
  typedef __attribute__((address_space(4))) const uint32_t cu32;  // uniform address: s_load
  cu32 *slut = (cu32 *)lut;
  uint32_t corr = 0;
#pragma unroll
  for (int p = 0; p < 4; p++) {
    const bool ey = (yb[p] & 0x3FFu) == 0u;
    unsigned long long m = __ballot(ey);
    if (m && !GLOBAL_LUT) {
      const uint32_t i = (Rv[p] << 7) | (Gv[p] >> 1);  // integer Y needs R == G (mod 2)
      const uint32_t bit = (lut[i >> 5] >> (i & 31)) & 1u;
      corr |= (ey ? bit : 0u) << (8 * p);
    } else if (m) {
      const uint32_t i = (Rv[p] << 7) | (Gv[p] >> 1);
      do {
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const uint32_t il = (uint32_t)__builtin_amdgcn_readlane((int)i, l);
        const uint32_t bit = (slut[il >> 5] >> (il & 31)) & 1u;
        if (lane == l) corr |= bit << (8 * p);
      } while (m);
    }
  }
  return corr;
}

// Rare path: Cb / Cr corrections (0/1 per pixel) of a run.  GLOBAL_LUT:
// per pixel slot, only the lanes with an exact-integer candidate read the
// bitmap, by scalar loads (as y_fix).
template <bool RGB, bool GLOBAL_LUT>
__device__ __forceinline__ void chroma_fix(uint32_t w0, uint32_t w1, uint32_t w2,
                                           const uint32_t *__restrict__ lut, uint32_t (&cbc)[4],
                                           uint32_t (&crc)[4], int lane) {
  const uint32_t B0[4] = {w0 & 255, w0 >> 24, (w1 >> 16) & 255, (w2 >> 8) & 255};
  const uint32_t Gv[4] = {(w0 >> 8) & 255, w1 & 255, w1 >> 24, (w2 >> 16) & 255};
  const uint32_t R0[4] = {(w0 >> 16) & 255, (w1 >> 8) & 255, w2 & 255, w2 >> 24};
  const uint32_t(&Bv)[4] = RGB ? R0 : B0;
  const uint32_t(&Rv)[4] = RGB ? B0 : R0;
  typedef __attribute__((address_space(4))) const uint32_t cu32;
  cu32 *slut = (cu32 *)lut;
#pragma unroll
  for (int p = 0; p < 4; p++) {
    // bit (G<<7 | B>>1) of the Cb table; valid when R == G and B == G (mod 2)
    const bool eb = Rv[p] == Gv[p] && !((Bv[p] ^ Gv[p]) & 1);
    const bool er = Bv[p] == Gv[p] && !((Rv[p] ^ Gv[p]) & 1);
    if (!GLOBAL_LUT) {
      const uint32_t wb = lut[LUT_WORDS + ((Gv[p] << 2) | (Bv[p] >> 6))];
      const uint32_t wr = lut[2 * LUT_WORDS + ((Gv[p] << 2) | (Rv[p] >> 6))];
      cbc[p] = (wb >> ((Bv[p] >> 1) & 31)) & (uint32_t)eb;
      crc[p] = (wr >> ((Rv[p] >> 1) & 31)) & (uint32_t)er;
      continue;
    }
    cbc[p] = crc[p] = 0;
    for (int t = 0; t < 2; t++) {
      unsigned long long m = __ballot(t ? er : eb);
      if (!m) continue;
      const uint32_t i = (Gv[p] << 7) | ((t ? Rv[p] : Bv[p]) >> 1);
      do {
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const uint32_t il = (uint32_t)__builtin_amdgcn_readlane((int)i, l);
        const uint32_t bit = (slut[(1 + t) * LUT_WORDS + (il >> 5)] >> (il & 31)) & 1u;
        if (lane == l) (t ? crc[p] : cbc[p]) = bit;
      } while (m);
    }
  }
}

// the four floor(Y) bytes of a run (bits 10-17 of the magic forms): fast
// right shifts, then two byte permutes and an OR
__device__ __forceinline__ uint32_t pack_y(const uint32_t (&yb)[4]) {
  const uint32_t s0 = yb[0] >> 10, s1 = yb[1] >> 10, s2 = yb[2] >> 10, s3 = yb[3] >> 10;
  return __builtin_amdgcn_perm(s1, s0, 0x0c0c0400u) | __builtin_amdgcn_perm(s3, s2, 0x04000c0cu);
}

// encoder.c:137-138 -- floor((a+b+c+d)/4) of the truncated values of the
// chroma quads (q = 0: pixels 0,1 of both rows; q = 1: pixels 2,3), from the
// magic forms (sum - 4 * MAGIC_BITS is the integer sum) minus corrections c
__device__ __forceinline__ uint32_t chroma_pair(const uint32_t (&r0)[4], const uint32_t (&r1)[4],
                                                uint32_t c0, uint32_t c1) {
  const uint32_t s0 = (r0[0] + r0[1] + r1[0] + r1[1] - 4u * MAGIC_BITS - c0) >> 2;
  const uint32_t s1 = (r0[2] + r0[3] + r1[2] + r1[3] - 4u * MAGIC_BITS - c1) >> 2;
  return s0 | (s1 << 8);
}

template <bool RGB, bool GLOBAL_LUT>
__device__ __forceinline__ void colour_stage(const uint8_t *raw, uint8_t *L, int c4, int pr,
                                             const uint32_t *__restrict__ lut, bool use_lut) {
  // all 8 row pieces of this lane up front: the exception branches below
  // split the code into many blocks the scheduler cannot hoist loads across
  uint32_t w[4][2][3];
#pragma unroll
  for (int it = 0; it < 4; it++)
#pragma unroll
    for (int dy = 0; dy < 2; dy++) {
      const uint32_t *rw = (const uint32_t *)(raw + (4 * it + 2 * pr + dy) * (TILE_W * 3) + 12 * c4);
#pragma unroll
      for (int k = 0; k < 3; k++) w[it][dy][k] = rw[k];
    }
#pragma unroll
  for (int it = 0; it < 4; it++) {
    const int rp = 2 * it + pr;  // row pair 0..7 == chroma row
    Run4 r[2];
    uint32_t py[2];
    uint32_t *Yd[2];
#pragma unroll
    for (int dy = 0; dy < 2; dy++) {
      convert4<RGB>(w[it][dy][0], w[it][dy][1], w[it][dy][2], r[dy]);
      const int yrow = 2 * rp + dy;  // 0..15
      const int by = yrow >> 3, bx = c4 >> 1;
      Yd[dy] = (uint32_t *)(L + (by * 16 + bx) * LDS_BLK + (yrow & 7) * 8 + (c4 & 1) * 4);
      py[dy] = pack_y(r[dy].yb);
      *Yd[dy] = py[dy];
    }
    uint8_t *C0 = L + (32 + (c4 >> 2)) * LDS_BLK + rp * 8 + ((2 * c4) & 7);
    *(uint16_t *)C0 = (uint16_t)chroma_pair(r[0].cbm, r[1].cbm, 0, 0);
    *(uint16_t *)(C0 + 8 * LDS_BLK) = (uint16_t)chroma_pair(r[0].crm, r[1].crm, 0, 0);
    if (!use_lut) continue;
    // rare paths: rewrite the staged values of runs with exceptions
#pragma unroll
    for (int dy = 0; dy < 2; dy++)
      if (__ballot(r[dy].cy)) {
        const uint32_t corr = y_fix<RGB, GLOBAL_LUT>(w[it][dy][0], w[it][dy][1], w[it][dy][2], r[dy].yb, lut,
                                                     c4 | (pr << 5));
        if (corr) *Yd[dy] = py[dy] - corr;  // no borrows: a corrected Y is >= 1
      }
    if (__ballot(r[0].pd * r[1].pd == 0.0f)) {
      uint32_t cbc[2][4], crc[2][4];
#pragma unroll
      for (int dy = 0; dy < 2; dy++)
        chroma_fix<RGB, GLOBAL_LUT>(w[it][dy][0], w[it][dy][1], w[it][dy][2], lut, cbc[dy], crc[dy], c4 | (pr << 5));
      const uint32_t nb0 = cbc[0][0] + cbc[0][1] + cbc[1][0] + cbc[1][1];
      const uint32_t nb1 = cbc[0][2] + cbc[0][3] + cbc[1][2] + cbc[1][3];
      const uint32_t nr0 = crc[0][0] + crc[0][1] + crc[1][0] + crc[1][1];
      const uint32_t nr1 = crc[0][2] + crc[0][3] + crc[1][2] + crc[1][3];
      if (nb0 | nb1) *(uint16_t *)C0 = (uint16_t)chroma_pair(r[0].cbm, r[1].cbm, nb0, nb1);
      if (nr0 | nr1) *(uint16_t *)(C0 + 8 * LDS_BLK) = (uint16_t)chroma_pair(r[0].crm, r[1].crm, nr0, nr1);
    }
  }
}

// Token of the per-segment streams: symbol (bits 0-7) | ZRL count before it
// (bits 8-9) | TOK_AC for the AC table (bit 10) | magnitude bits (16-27).
// Bit length = code length + (symbol & 15) + ZRLs * ZRL code length for
// every token kind (DC: symbol = class <= 11; EOB: symbol 0x00).
constexpr uint32_t TOK_AC = 1u << 10;
// the padding token after a segment's last one (AC symbol 0xFF, which no
// token carries: magnitudes stop at class 11): the packing's code table holds
// 0 for it -- no bits, no ZRLs
constexpr uint32_t LB_NOTOK = TOK_AC | 0xFFu;

// One N-tile of coefficients -> compacted token stream of its segment(s).
// o[k] = zigzag coefficient 16g+k of block bcol (DC raw in o[0] of g == 0,
// or the DC difference when dc_diffed).  Every lane of the wave calls this.
// Tokens of a block, in bitstream order (encoder.c:462-502): its DC
// difference (:434-446), the AC run/size symbols (:448-460, ZRLs folded in,
// :490-494), then EOB unless coefficient 63 is nonzero (:479-484).  The DC of
// a segment's first block depends on the previous segment: with first_pred
// the caller supplies that block's predecessor DC (pred0), otherwise (token
// variant fed from pixels) it is left for k_seg_dc.
// token i of a frame's streams: a wave-uniform frame base and a 32-bit byte
// offset, so the store takes the SGPR-base form instead of a 64-bit address
// add per token (A/B on config 3, 3 rounds: K1 3.280 -> 3.262 ms,
// profiles/r03/probe/k1_tokoff_ab.txt)
__device__ __forceinline__ uint32_t &tok_at(uint32_t *base, uint32_t i) {
  return *(uint32_t *)((char *)base + (i << 2));
}
__device__ __forceinline__ void emit_tokens(const int (&o)[16], int lane, int g, int bcol,
                                            bool valid, bool chroma, bool dc_diffed,
                                            bool first_pred, int pred0,
                                            uint32_t *segtok, uint32_t segoff, uint32_t *tok0, uint32_t *segcnt, uint32_t *hDC,
                                            uint32_t *hAC, int16_t (*st)[16], int kflags = 0, bool acz = false) {
  // acz (a compile-time constant where it is set): every AC coefficient of
  // the N-tile is zero -- no staging, no masks, no AC tokens; each block is
  // its DC token and EOB
  uint32_t Mlo = 0, Mhi = 0;
  const int zsw = 8 * (bcol & 7);
  if (!acz) {
  u4v c0, c1;
#pragma unroll
  for (int k = 0; k < 4; k++) {  // one v_perm per pair
    c0[k] = pack_i16x2(o[2 * k], o[2 * k + 1]);
    c1[k] = pack_i16x2(o[8 + 2 * k], o[9 + 2 * k]);
  }
  // staged block-major (block b's 64 coefficients in zigzag order at st +
  // 64 b), its 16-byte chunks XOR-swizzled by b & 7 (coefficient z at
  // 64 b + (z ^ 8 (b & 7))): the 8 lanes of a ds_write_b128 group store to 8
  // different bank quads instead of one (blocks are 128 B = 32 banks apart:
  // 8-way conflicts), and the AC loop's reads of one z spread over the banks
  int16_t *stb = &st[0][0] + 64 * bcol;
  *(u4v *)(stb + ((16 * g) ^ zsw)) = c0;
  *(u4v *)(stb + ((16 * g + 8) ^ zsw)) = c1;
  // nonzero mask: min(half, 1) per packed int16 pair puts coefficient 2k's
  // flag at bit 2k and 2k+1's at bit 16+2k
  // (v_pk_min_u16 in asm: the compiler rewrites min(h, 1) into compares and
  // selects, three times the instructions)
  // (the flags gathered by a v_lshl_or chain: left to itself the compiler
  // emits a separate shift per word and v_or3 trees, ~1.5x the cycles)
  uint32_t pm;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(pm) : "v"(c0[0]));
#pragma unroll
  for (int k = 1; k < 8; k++) {
    const uint32_t w = k < 4 ? c0[k] : c1[k - 4];
    uint32_t h;
    asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(h) : "v"(w));
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(pm) : "v"(h), "i"(2 * k), "v"(pm));
  }
  uint32_t m16 = (pm & 0x5555u) | ((pm >> 15) & 0xAAAAu);
  if (g == 0) m16 &= ~1u;  // the DC is not part of the AC run structure
  // the block's 64-bit mask: rows 0|1 form the low word, rows 2|3 the high
  uint32_t h = m16 << (16 * (g & 1));
  const auto r16 = __builtin_amdgcn_permlane16_swap(h, h, false, false);
  h = r16[0] | r16[1];
  const auto r32 = __builtin_amdgcn_permlane32_swap(h, h, false, false);
  Mlo = r32[0];
  Mhi = r32[1];
  }
  const int eob = !(Mhi >> 31);
  const int n = valid ? 1 + __popc(Mlo) + __popc(Mhi) + eob : 0;
  // token offsets of the blocks inside their segment (chroma rows hold two
  // 8-block segments: Cb | Cr; a luma row is one 16-block segment, where the
  // zero fill of row_shr already stops the scan at the row start)
  const int pos = chroma ? (bcol & 7) : bcol;
  // (chroma: the row's scan minus, in the Cr half, the Cb half's total --
  // DPP row_newbcast:7 -- where three masked half-row steps cost twice the
  // cycles with their lane-mask selects)
  uint32_t incl = row_scan16((uint32_t)n);
  if (chroma)
    incl -= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x157, 0xF, 0xF, false) & (0u - (uint32_t)(bcol >> 3));
  const int base = (int)incl - n;
  const int dc0 = o[0];
  const int prev = (int)row_shr0<1>((uint32_t)dc0);
  wave_lds_sync();
  if (pos == (chroma ? 7 : 15)) {
    if (g == 0) *segcnt = incl;
    // the segment's token count padded to a multiple of 4 with LB_NOTOK
    // (k_pack_flat decodes 4-token chunks: a lane's slots are then all
    // tokens or all padding, and no token needs a mask); the last block's
    // lanes g < pads write one slot each (all four hold the same incl), where
    // a loop in one lane cost the wave a dozen instructions per pad
    if ((uint32_t)g < ((0u - incl) & 3u)) tok_at(segtok, segoff + incl + (uint32_t)g) = LB_NOTOK;
  }
  if (g == 0) {
    if (valid) {
      if (dc_diffed || pos != 0 || first_pred) {
        const int diff = dc_diffed ? dc0 : dc0 - (pos != 0 ? prev : pred0);  // :168-177
        const int cls = mag_class(diff);
        // a segment's first token lives in the dense tok0 array (one word per
        // segment: written there it is a whole-line store, not a lone word)
        const uint32_t tk = (uint32_t)cls | (mag_bits(diff, cls) << 16);
        if (pos == 0) *tok0 = tk;
        else tok_at(segtok, segoff + base) = tk;
        atomicAdd(&hDC[cls], 1u);
      }
      if (eob) tok_at(segtok, segoff + base + n - 1) = TOK_AC;
    }
  }
  {  // one histogram update for all of the wave's EOBs
    const unsigned long long eobs = __ballot(g == 0 && valid && eob);
    if (lane == 0 && eobs) atomicAdd(&hAC[0x00], (unsigned)__popcll(eobs));
  }
  // (Measured and dropped: reading the next set bit's coefficient one
  // iteration ahead, 3.43 -> 3.49 ms -- the other waves already hide the LDS
  // round trip, the prefetch adds VALU; ZRL counts summed per N-tile instead
  // of the conditional atomic, 3.48.)
  // AC tokens (encoder.c:448-460, ZRLs :490-494): lane (g, b) takes the
  // zigzag positions z == g (mod 4) of block b, those below 32 first, then
  // the rest, so the mask work is 32-bit: a token's index in the segment is
  // base + 1 + the block's set bits below z, its run the distance to the
  // highest of them (the DC at z = 0 when there is none).  Token word:
  // (run << 4 | cls) is sym | ZRLs << 8 (run <= 62).
  if (!acz && valid && !(kflags & K1F_NO_ACLOOP)) {
    const int16_t *sl = &st[0][0] + 64 * bcol;
    // token of AC coefficient z; rank: the set bits of the block's mask below
    // z with the DC position counted (the token's index is base + rank); zp:
    // 63 - the previous set bit (0 for the first: the DC position)
    auto token = [&](int z, int rank, int zp) {
      const int cz = sl[z ^ zsw];
      // m = cz, or ~|cz| when negative (its low cls bits are the magnitude
      // bits, encoder.c:456-458); its leading sign bits (v_ffbh_i32) are
      // clz(|cz|), so cls = 32 - ffbh_i32(m) (cz != 0: m is neither 0 nor -1;
      // no builtin: __builtin_clrsb lowers to four instructions)
      const int m = cz + (cz >> 31);
      uint32_t lead;
      asm("v_ffbh_i32 %0, %1" : "=v"(lead) : "v"(m));
      const uint32_t cls = 32u - lead;
      const uint32_t mag = __builtin_amdgcn_ubfe((uint32_t)m, 0u, cls);
      // run + 64 = z + zp (one add) shifted by 4 is TOK_AC | run << 4 (run <=
      // 62): the symbol word in one v_lshl_add (cls < 16), the token in one
      // v_lshl_or
      const uint32_t runp = (uint32_t)(z + zp);
      const uint32_t t = (runp << 4) + cls;
      if (!(kflags & K1F_NO_TOKSTORE)) tok_at(segtok, segoff + (uint32_t)(base + rank)) = t | (mag << 16);
      if (!(kflags & K1F_NO_HIST)) {
        atomicAdd(&hAC[t & 255u], 1u);
        if (runp >= 80u) atomicAdd(&hAC[0xF0], (runp - 64u) >> 4);
      }
    };
    const uint32_t cm = 0x11111111u << g;
    const int rank_lo = __popc(Mlo), zp_lo = 31 - __clz((int)(Mlo | 1u));
    // (Measured and dropped: one loop over both 32-bit halves, the wave
    // running max(lo + hi) iterations instead of max(lo) + max(hi) at a few
    // selects per iteration: 3.39 -> 3.49 ms.)
    // The DC position (bit 0) counted as set below every AC token of the low
    // half: the set bits below z then always include one (the run's start is
    // their highest, 0 for the first token) and their count is the token's
    // index past the block's DC token
    const uint32_t M1 = Mlo | 1u;
    for (uint32_t m = Mlo & cm; m; m &= m - 1u) {
      const int z = __builtin_ctz(m);
      const uint32_t bef = __builtin_amdgcn_ubfe(M1, 0u, (uint32_t)z);  // bits below z: one v_bfe
      uint32_t lz;  // (bef != 0: no zero check)
      asm("v_ffbh_u32 %0, %1" : "=v"(lz) : "v"(bef));
      token(z, __popc(bef), 32 + (int)lz);
    }
    const int rank_lo1 = rank_lo + 1;
    for (uint32_t m = Mhi & cm; m; m &= m - 1u) {
      const int zz = __builtin_ctz(m);
      const uint32_t bef = __builtin_amdgcn_ubfe(Mhi, 0u, (uint32_t)zz);
      // v_ffbh_u32 of 0 is ~0u: the min picks 63 - zp_lo exactly when no
      // bit of the high half lies below zz (no compare and select)
      uint32_t lz;
      asm("v_ffbh_u32 %0, %1" : "=v"(lz) : "v"(bef));
      token(32 + zz, rank_lo1 + __popc(bef), (int)min(lz, (uint32_t)(63 - zp_lo)));
    }
  }
  wave_lds_sync();
}

// K1 modes
constexpr int K1M_COEF_OUT = 1;  // write zigzag coefficient planes
constexpr int K1M_TOK_OUT = 2;   // write per-segment token streams + histograms
constexpr int K1M_COEF_IN = 4;   // read coefficient planes (DC differences) instead of pixels
constexpr int K1M_RGB = 8;       // pixels in RGB order (PPM) instead of BGR (encoder.c:133)
constexpr int K1M_REGIONS = 16;  // per-frame image sizes inside the canvas (region batches)
constexpr int K1M_AUDIT = 32;    // coefficient variant + every block's straddle decisions (tests)
// measurement only (mij_batch_pattern_floor): the coefficient variant's
// memory traffic -- persistent grid, tile claims, LDS-DMA one tile ahead,
// whole-line coefficient stores and raw DCs -- with no colour, DCT or
// quantisation: its launch time is the floor of K1's access pattern on the
// box it runs on (bench.py reports K1 beside it)
constexpr int K1M_FLOOR = 64;
constexpr int k1_base(int mode) { return mode & ~(K1M_RGB | K1M_REGIONS | K1M_AUDIT | K1M_FLOOR); }

// Waves per workgroup: the coefficient-only variant runs one 12-wave
// workgroup per CU (3 waves per SIMD: 120 KB of per-wave tile buffers + the
// shared tables fit the 160 KB LDS, <= 168 VGPRs); the token variants carry
// per-wave token staging and run 4-wave workgroups, two per CU.
template <int MODE>
constexpr bool k1_wide() { return k1_base(MODE) == K1M_COEF_OUT || k1_base(MODE) == K1M_TOK_OUT; }
template <int MODE>
constexpr int k1_waves() {
  return k1_wide<MODE>() ? 12 : 4;
}

template <int MODE>
__global__ __launch_bounds__(64 * k1_waves<MODE>(), k1_wide<MODE>() ? 1 : 2) void k_mcu_dct(K1Args a) {
  constexpr bool PIX = !(MODE & K1M_COEF_IN);
  constexpr bool TOK = MODE & K1M_TOK_OUT;
  constexpr int NW = k1_waves<MODE>();
  constexpr int NT = 64 * NW;  // threads per workgroup
  // coefficient variant: FP64 replays are deferred to k_fix_blocks; the
  // token variants replay in place (their tokens are emitted here)
  constexpr bool DEFER = k1_base(MODE) == K1M_COEF_OUT;
  constexpr bool RGB = MODE & K1M_RGB;
  // region batches only: the frame sizes (compile-time null otherwise, so
  // the per-tile geometry folds to the batch's)
  constexpr bool REG = MODE & K1M_REGIONS;
  // audit (tests only): per block the 64 keep/replay decisions of the fast
  // path, exported so they can be compared with tests/tau_check.c's model
  constexpr bool AUDIT = MODE & K1M_AUDIT;
  constexpr bool FLOOR = MODE & K1M_FLOOR;
  const int2 *const fdims = REG ? a.fdims : nullptr;
  __shared__ __attribute__((aligned(16))) uint8_t s_raw[PIX ? NW : 1][TILE_RAW];
  __shared__ __attribute__((aligned(16))) uint8_t s_tile[PIX ? NW : 1][LDS_WAVE];
  __shared__ __attribute__((aligned(16))) int4 s_A[PIX ? 12 * 64 : 1];
  __shared__ __attribute__((aligned(16))) float s_fac[2][64];
  __shared__ float s_inv8q[2];
  __shared__ uint32_t s_dctie[2][DCTIE_WORDS];
  // colour-exception bitmaps: in LDS for the coefficient variant; the wide
  // token variant reads them from global memory (rare path, L1/L2 hits) to
  // fit its token staging into the 160 KB
  constexpr bool LUT_LDS = PIX && !(TOK && NW >= 8);
  __shared__ uint32_t s_lut[LUT_LDS ? 3 * LUT_WORDS : 1];
  __shared__ double s_cos[64];
  __shared__ uint8_t s_zz[64];
  __shared__ int s_qint[2][64];
  __shared__ __attribute__((aligned(16))) int s_czl[PIX ? 64 : 1];  // chroma all-AC-zero limits
  __shared__ __attribute__((aligned(16))) int16_t s_st[TOK ? NW : 1][64][16];  // token staging
  // per-frame histograms of this workgroup: [frame slot][luma, chroma][copy][symbol];
  // the tokenize pass keeps HREP copies (by block) to spread same-symbol atomics
  constexpr int HREP = PIX ? 1 : 4;
  __shared__ uint32_t s_hac[TOK ? 2 : 1][2][HREP][256];
  __shared__ uint32_t s_hdc[TOK ? 2 : 1][2][HREP][16];
  // next unclaimed tile of this workgroup's range: waves claim tiles
  // dynamically, so waves the SIMD arbiter favours do more of them and the
  // workgroup's waves finish together (static round-robin left the youngest
  // wave of each SIMD running alone for the last third of the launch)
  __shared__ int s_next;

  const Tables *__restrict__ T = a.tab;
  // diagnostic switches exist only in the MIJ_K1_DIAG build (make diag): in
  // the product kernel they fold away at compile time
#ifdef MIJ_K1_DIAG
  const int kflags = a.flags;
#else
  constexpr int kflags = 0;
#endif
  if (threadIdx.x < 64) {
    s_cos[threadIdx.x] = T->cosd[threadIdx.x];
    s_zz[threadIdx.x] = (uint8_t)c_zigzag[threadIdx.x];
  }
  if (TOK) {
    for (int i = threadIdx.x; i < 2 * 2 * HREP * 256; i += NT) (&s_hac[0][0][0][0])[i] = 0;
    for (int i = threadIdx.x; i < 2 * 2 * HREP * 16; i += NT) (&s_hdc[0][0][0][0])[i] = 0;
  }
  if (threadIdx.x < 128) s_qint[threadIdx.x >> 6][threadIdx.x & 63] = T->qint[threadIdx.x >> 6][threadIdx.x & 63];
  if (threadIdx.x < 2) s_inv8q[threadIdx.x] = 1.0f / (float)(8 * T->qint[threadIdx.x][0]);
  if (PIX && threadIdx.x < 64) s_czl[threadIdx.x] = T->czl[threadIdx.x];
  if (threadIdx.x < 2 * DCTIE_WORDS) (&s_dctie[0][0])[threadIdx.x] = (&T->dctie[0][0])[threadIdx.x];
  if (PIX) {
    for (int i = threadIdx.x; i < 12 * 64; i += NT) s_A[i] = T->mfma_a[i];
    if (LUT_LDS)
      for (int i = threadIdx.x; i < 3 * LUT_WORDS; i += NT) s_lut[i] = (&T->lut[0][0])[i];
  }
  const uint32_t *__restrict__ lut = LUT_LDS ? (const uint32_t *)s_lut : &T->lut[0][0];
  for (int i = threadIdx.x; i < 128; i += NT) {
    s_fac[i >> 6][i & 63] = T->qfac[i >> 6][i & 63];
  }
  if (threadIdx.x == 0) s_next = (int)blockIdx.x * a.per_wg + NW;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < a.nerr_zero; i += NT) a.err_zero[i] = 0;
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: tile math on SALU
  uint8_t *L = s_tile[PIX ? wave : 0];
  const int g = lane >> 4, bcol = lane & 15;
  const int c4 = lane & 31, pr = lane >> 5;
  const uint32_t kq = (uint32_t)T->kq[g];  // luma shift of this lane's zigzag group
  const int q_dc[2] = {T->qint[0][0], T->qint[1][0]};
  const bool cz_on = PIX && !AUDIT && T->cz_on;  // wave-uniform
  const Geom &G = a.g;
  const int bw = G.w >> 3, mw = G.w >> 4;
  const int ntiles = a.nframes * G.tiles_per_frame;
  const int t0 = (int)blockIdx.x * a.per_wg;  // per_wg <= tiles_per_frame:
  const int f0 = t0 / G.tiles_per_frame;      // a workgroup spans <= 2 frames
  const int tend = min(ntiles, t0 + a.per_wg);
  int t = t0 + wave;
  // region batches: a tile holds pixels of its frame, or the wave claims the
  // next one (the canvas tiles outside a frame are skipped)
  auto skip_outside = [&](int &tt) {
    bool ok;
    while (tt < tend && (tile_pos_r(G, fdims, tt, ok), !ok)) {
      int v = 0;
      if (lane == 0) v = atomicAdd(&s_next, 1);
      tt = __builtin_amdgcn_readfirstlane(v);
    }
  };
  auto tpos = [&](int tt) {
    bool ok;
    return REG ? tile_pos_r(G, fdims, tt, ok) : tile_pos(G, tt);
  };
  if (REG) skip_outside(t);
#ifdef MIJ_K1_DIAG
  const unsigned long long w_t0 = __builtin_amdgcn_s_memrealtime();
  int w_ntiles = 0;
  // per-phase wall time of this wave (s_memtime, shader clock), summed over
  // its tiles: [0] DMA wait, [1] colour, [2] next-DMA issue, [3] DCT +
  // quantise per N-tile, [4] store / emit per N-tile
  unsigned long long ph[5] = {0, 0, 0, 0, 0}, tph = __builtin_amdgcn_s_memtime();
#define K1_PHASE(k)                                                  \
  do {                                                               \
    const unsigned long long tn_ = __builtin_amdgcn_s_memtime();     \
    ph[k] += tn_ - tph;                                              \
    tph = tn_;                                                       \
  } while (0)
#else
#define K1_PHASE(k)
#endif
  // coefficients this lane replayed in FP64 (or listed for k_fix_blocks):
  // summed over the wave and added once at the end (an atomic per replaying
  // lane on the one counter cost 12 ms per launch at Q=90, where 2.7 M
  // coefficients are replayed: 17.5 -> 5.3 ms)
  uint32_t nrep = 0;
  if (t < tend) {
    uint8_t *raw = s_raw[PIX ? wave : 0];
    TilePos p = tpos(t);
    const DmaOff doff = dma_offsets(a.pitch, lane);
    if (PIX) issue_tile_dma(a, p, lane, raw, doff);
    // coefficient input: the three N-tiles' 32 B per lane of a tile
    auto load_coefs = [&](const TilePos &pp, u4v (&dst)[PIX ? 1 : 3][2]) {
#pragma unroll
      for (int nt = 0; nt < 3; nt++) {
        bool valid;
        long long blk;
        const FGeom fg = frame_geom(G, fdims, pp.f);  // REG only
        const int bwf = REG ? fg.bw : bw, mwf = REG ? fg.mw : mw;
        const int nYf = REG ? fg.nY : G.nY, nCf = REG ? fg.nC : G.nC;
        if (nt < 2) {
          const int bx = pp.tx * 16 + bcol;
          valid = bx < bwf;
          blk = (long long)(2 * pp.ty + nt) * bwf + bx;
        } else {
          const int mx = pp.tx * 8 + (bcol & 7);
          valid = mx < mwf;
          blk = nYf + (bcol >= 8 ? nCf : 0) + (long long)pp.ty * mwf + mx;
        }
        dst[PIX ? 0 : nt][0] = dst[PIX ? 0 : nt][1] = u4v{0, 0, 0, 0};
        if (valid) {
          const int16_t *src = a.coef + (long long)pp.f * G.coef_fs + blk * 64 + 16 * g;
          dst[PIX ? 0 : nt][0] = *(const u4v *)src;
          dst[PIX ? 0 : nt][1] = *(const u4v *)(src + 8);
        }
      }
    };
    u4v cnext[PIX ? 1 : 3][2];
    if (!PIX) load_coefs(p, cnext);
    bool first = true;
    for (;;) {
      TilePos pn = p;
      // claim the wave's next tile now: the LDS atomic's result is needed only
      // after the colour stage, when the next tile's DMA goes out
      int tn = 0;
      if (lane == 0) tn = atomicAdd(&s_next, 1);
      tn = __builtin_amdgcn_readfirstlane(tn);
      uint32_t fl_w = 0;  // FLOOR: one word of the tile, so the stores depend on its DMA
      if (PIX) {
        // ---- 1. colour convert + subsample + stage.  Wait for this tile's
        // DMA: the coefficient variant leaves the previous tile's stores in
        // flight (counted wait); the token variants waited before their first
        // store of the previous tile; the first tile and the diagnostic
        // variants without stores drain everything.
        K1_PHASE(3);
        if (first || (kflags & (K1F_NO_DCT | K1F_NO_STORE)))
          dma_wait();
        else if (DEFER)
          dma_wait_behind_stores();
        K1_PHASE(0);
        if (!(kflags & K1F_NO_COLOUR) && !FLOOR) colour_stage<RGB, !LUT_LDS>(raw, L, c4, pr, lut, !(kflags & K1F_NO_LUT));
        if (FLOOR) fl_w = ((const uint32_t *)raw)[lane];
        wave_lds_sync();
        K1_PHASE(1);
        // ---- stream the wave's next tile into the freed raw buffer -----------
        if (REG) skip_outside(tn);
        if (tn < tend) {
          pn = tpos(tn);
          issue_tile_dma(a, pn, lane, raw, doff);
        }
        K1_PHASE(2);
      } else {
        if (REG) skip_outside(tn);
        if (tn < tend) pn = tpos(tn);
      }

      // ---- 2. DCT on MFMA, one 16-block N-tile at a time ----------------------
      // N = ((D2.X << 7) + D1.X << 7) + D0.X, accumulated in place: each
      // digit's MFMA takes the shifted partial sum as its C input.  The four
      // M-tile chains of an N-tile are issued digit by digit, so no MFMA waits
      // on its predecessor's result; the N-tile's quantisation and stores
      // follow before the next N-tile's MFMAs (16 accumulator VGPRs live).
      const bool do_dct = !(kflags & K1F_NO_DCT);
      // digit d of the chain for the four M-tiles (B operand Bf)
      auto dct_digit = [&](const int d, v4i (&acc)[4], const v4i Bf) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
          const int4 F = s_A[(3 * m + d) * 64 + lane];
#ifdef MIJ_K1_DIAG
          if (kflags & K1F_EXTRA_LDS) {  // diagnostics: a second, unused read of the fragment
            v4i dummy;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(dummy) : "v"((uint32_t)(uintptr_t)(lds_void_t *)&s_A[(3 * m + d) * 64 + lane]) : "memory");
          }
#endif
          const v4i Fv = {F.x, F.y, F.z, F.w};
          // The digit shifts two accumulators at a time (v_lshlrev_b64 of
          // the pairs r = 0|1 and 2|3): the low element of a pair carries a
          // bias of 2^17 from the first digit on, which keeps it inside
          // [0, 2^25) before each shift (the partial sums stay within
          // +-2^17 and +-16,711,680), so no bit crosses
          // into its partner; N = the low element ^ 2^31 at the end.
          v4i c;
          if (d == 0) {
            c = v4i{1 << 17, 0, 1 << 17, 0};
          } else {
            // (the accumulator as two 64-bit values: the compiler's own
            // v_lshlrev_b64 on the register pairs, with its MFMA-read wait
            // states; inline asm here read stale results)
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            c = __builtin_bit_cast(v4i, __builtin_bit_cast(u64x2, acc[m]) << 7);
          }
          acc[m] = (kflags & K1F_NO_MFMA) ? c + Fv + Bf
                                          : __builtin_amdgcn_mfma_i32_16x16x64_i8(Fv, Bf, c, 0, 0, 0);
        }
        if (d == 2) {
#pragma unroll
          for (int m = 0; m < 4; m++) {
            acc[m][0] ^= (int)0x80000000u;
            acc[m][2] ^= (int)0x80000000u;
          }
        }
      };
      // N-tile nt: the error bound of its N (lanes of a block: its L1) and
      // the three digits
      auto dct_ntile = [&](const int nt, v4i (&acc)[4], uint32_t &lc) {
        const v4i Bp = *(const v4i *)(L + (nt * 16 + bcol) * LDS_BLK + 16 * g);
        // L1 = sum |pixel - 128| of the block bounds the integer DCT's
        // rounding error: |N - 2^19 sum K X| <= sum |W - 2^19 K| |X| <= L1 / 2
        uint32_t l1 = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) l1 = __builtin_amdgcn_sad_u8((uint32_t)Bp[k], 0x80808080u, l1);
        const auto r16 = __builtin_amdgcn_permlane16_swap(l1, l1, false, false);
        l1 = r16[0] + r16[1];
        const auto r32 = __builtin_amdgcn_permlane32_swap(l1, l1, false, false);
        const uint32_t L1 = r32[0] + r32[1];
        if (nt < 2) {
          // luma, integer rule: E = floor(L1 / 2) + 1 >= L1 / 2 + the
          // reference's own FP64 rounding (< 1e-3 in N' units), an integer
          lc = (L1 >> 1) + 1u;
        } else {
          // chroma, fp32 rule: 1.25 * (L1/2 + 64) for the integer DCT and
          // float(N'), + 0.095 L1 for the fp32 roundings of t -+ tau (<= 1.8e-7
          // |N'| with |N'| <= 2^19 L1)
          // (the float's bits: lc is a uint32_t, so no float value ever
          // holds the luma bound's integer bits)
          lc = __float_as_uint(fmaf((float)L1, 0.72f, 80.0f));
        }
        const v4i Bf = Bp ^ (int)0x80808080;  // pixel - 128 as int8
#pragma unroll
        for (int d = 0; d < 3; d++) dct_digit(d, acc, Bf);
      };

      // coefficient input: this tile's planes were loaded one tile ahead;
      // the next tile's loads go out now, in flight during this tile's work
      u4v pre[PIX ? 1 : 3][2];
      if (!PIX) {
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
          pre[PIX ? 0 : nt][0] = cnext[PIX ? 0 : nt][0];
          pre[PIX ? 0 : nt][1] = cnext[PIX ? 0 : nt][1];
        }
        if (tn < tend) load_coefs(pn, cnext);
      }

      // ---- 3-4. quantize, replay, store, emit -----------------------------------
      // block (index inside the frame's coefficient space) of this lane's
      // column in N-tile nt; false for columns beyond the frame edge
      auto block_at = [&](const int nt, const int col, int &blk) -> bool {
        const FGeom fg = frame_geom(G, fdims, p.f);  // REG only
        const int bwf = REG ? fg.bw : bw, mwf = REG ? fg.mw : mw;
        const int nYf = REG ? fg.nY : G.nY, nCf = REG ? fg.nC : G.nC;
        if (nt < 2) {
          const int bx = p.tx * 16 + col;
          blk = (2 * p.ty + nt) * bwf + bx;
          return bx < bwf;
        }
        const int mx = p.tx * 8 + (col & 7);
        blk = nYf + (col >= 8 ? nCf : 0) + p.ty * mwf + mx;
        return mx < mwf;
      };
      auto block_of = [&](const int nt, int &blk) -> bool { return block_at(nt, bcol, blk); };
      auto finish = [&](const int nt, int (&o)[16], bool acz) {
        const int comp = nt == 2 ? 1 : 0;
        int blk;
        const bool valid = block_of(nt, blk);
        // segment index inside the frame
        const int seg = nt < 2 ? (2 * p.ty + nt) * G.tiles_x + p.tx
                               : G.nsy + (bcol >= 8 ? G.nsc : 0) + p.ty * G.tiles_x + p.tx;
        if (!PIX) {  // coefficients from memory (drop-in write_jpg / init_huffman)
          const u4v c0 = pre[PIX ? 0 : nt][0], c1 = pre[PIX ? 0 : nt][1];
#pragma unroll
          for (int k = 0; k < 4; k++) {
            o[2 * k] = (int16_t)(c0[k] & 0xFFFFu);
            o[2 * k + 1] = (int16_t)(c0[k] >> 16);
            o[8 + 2 * k] = (int16_t)(c1[k] & 0xFFFFu);
            o[9 + 2 * k] = (int16_t)(c1[k] >> 16);
          }
        }
        if ((MODE & K1M_COEF_OUT) && !(kflags & K1F_NO_STORE)) {
          u4v s0, s1;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            s0[k] = pack_i16x2(o[2 * k], o[2 * k + 1]);
            s1[k] = pack_i16x2(o[8 + 2 * k], o[9 + 2 * k]);
          }
          int16_t *const fcoef = a.coef + (long long)p.f * G.coef_fs;
          if (kflags & (K1F_LINEAR_STORE | K1F_PLAIN_STORE)) {
            int16_t *dst = fcoef + (long long)blk * 64 + 16 * g;
            if (!valid) {
            } else if (kflags & K1F_LINEAR_STORE) {  // diagnostics: timing of fully contiguous stores
              const long long b0 = nt < 2 ? blk - bcol : G.nY + (long long)p.ty * mw + p.tx * 8;
              int16_t *lin = fcoef + b0 * 64 + 8 * lane;
              __builtin_nontemporal_store(s0, (u4v *)lin);
              __builtin_nontemporal_store(s1, (u4v *)(lin + 512));
            } else {  // diagnostics: the lane-owned halves with the default cache policy
              *(u4v *)dst = s0;
              *(u4v *)(dst + 8) = s1;
            }
          } else {
            // Whole block lines per store instruction.  Lane (g, b) holds
            // chunks (b, 2g) = s0 and (b, 2g+1) = s1 of the 16-byte chunks of
            // its block; stored as they are, each instruction would cover one
            // half of every block's 128-byte line (written in two partial
            // halves: 1.16x write traffic).  Lanes b and b^8 (one DPP row
            // rotate by 8) trade: the first store writes blocks 0-7 whole
            // (b < 8 its own s0, b >= 8 the s1 of block b-8), the second
            // blocks 8-15 (b < 8 the s0 of block b+8, b >= 8 its own s1).
            // Blocks 0-7 and 8-15 are each 1 KB contiguous (a luma block row
            // of the tile; the tile's Cb and Cr blocks).
            u4v d1, d2;
#pragma unroll
            for (int k = 0; k < 4; k++) {
              d1[k] = (uint32_t)__builtin_amdgcn_update_dpp((int)s0[k], (int)s1[k], 0x128, 0xF, 0xC, false);
              d2[k] = (uint32_t)__builtin_amdgcn_update_dpp((int)s1[k], (int)s0[k], 0x128, 0xF, 0x3, false);
            }
            const int off = 16 * g + 8 * (bcol >> 3);
            int b1, b2;
            const bool v1 = block_at(nt, bcol & 7, b1), v2 = block_at(nt, bcol | 8, b2);
            // The DEFER variant's counted DMA wait needs both store
            // instructions issued on every N-tile: column 0's lanes are always
            // valid for the first, and a lane whose second block lies beyond
            // the frame edge repeats its first store (same bytes, same
            // address) instead of dropping out, so the second never runs on
            // an empty exec mask either.
            int16_t *const p1 = fcoef + (long long)b1 * 64 + off;
            if (v1) __builtin_nontemporal_store(d1, (u4v *)p1);
            if (v1 || v2) __builtin_nontemporal_store(v2 ? d2 : d1, (u4v *)(v2 ? fcoef + (long long)b2 * 64 + off : p1));
          }
        }
        if (PIX && valid && g == 0) a.dc[(long long)p.f * G.nblk + blk] = (int16_t)o[0];
        if (TOK && !(kflags & K1F_NO_EMIT)) {
          const long long fs = (long long)p.f * G.nseg + seg;
          const int slot = p.f - f0;
          // the coefficient-input variant predicts a segment's first DC from the
          // raw DC K1 stored for the block before it (0 at a component start,
          // or the band predictor), unless k_seg_dc runs (seg_dc_inline == 0)
          int pred0 = 0;
          const bool first_pred = !PIX && a.seg_dc_inline;
          if (first_pred && valid && g == 0 && (comp == 1 ? (bcol & 7) : bcol) == 0) {
            const FGeom fg = frame_geom(G, fdims, p.f);  // REG only
            const int nYf = REG ? fg.nY : G.nY, nCf = REG ? fg.nC : G.nC;
            const int cstart = comp == 0 ? 0 : (bcol >= 8 ? nYf + nCf : nYf);
            pred0 = blk == cstart ? (a.dc_pred ? (int)a.dc_pred[p.f * 4 + (comp == 0 ? 0 : (bcol >= 8 ? 2 : 1))] : 0)
                                  : (int)a.dc[(long long)p.f * G.nblk + blk - 1];
          }
          emit_tokens(o, lane, g, bcol, valid, comp == 1, !PIX && a.dc_diffed, first_pred, pred0,
                      a.tok + (long long)p.f * G.nseg * SEG_TOK, (uint32_t)seg * SEG_TOK, a.tok0 + fs,
                      a.seg_ntok + fs, s_hdc[TOK ? slot : 0][comp][bcol & (HREP - 1)],
                      s_hac[TOK ? slot : 0][comp][bcol & (HREP - 1)],
                      s_st[TOK ? wave : 0], kflags, acz);
        }
      };
      if (FLOOR) {
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
          int o[16];
#pragma unroll
          for (int k = 0; k < 16; k++) o[k] = (int)(fl_w >> k) & 0xFF;
          finish(nt, o, false);
        }
      } else if (PIX && do_dct) {
        // token variants: N-tile nt + 1's MFMA chain is issued before N-tile
        // nt is quantised, so the wave's own quantisation covers the chain's
        // latency (two accumulator sets live; measured: token K1 3.504 ->
        // 3.441 and 3.514 -> 3.459 ms, two A/B rounds on one box; the
        // coefficient variant spills at 168 VGPRs with it, 3.12 -> 3.18)
        constexpr bool PIPE = TOK;
        v4i accs[PIPE ? 2 : 1][4];
        uint32_t lcs[PIPE ? 2 : 1];  // per block: error bound of N (luma: integer E; chroma: fp32 bits)
        if (PIPE) dct_ntile(0, accs[0], lcs[0]);
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
          const int comp = nt == 2 ? 1 : 0;
          const int cur = PIPE ? (nt & 1) : 0;
          if (!PIPE) {
            dct_ntile(nt, accs[0], lcs[0]);
          } else if (nt + 1 < 3) {
            dct_ntile(nt + 1, accs[PIPE ? (cur ^ 1) : 0], lcs[PIPE ? (cur ^ 1) : 0]);
          }
          v4i(&acc)[4] = accs[cur];
          const uint32_t lcb = lcs[cur];
          int o[16];
          // Chroma N-tile: when |N| < L_z (Tables::czl) for every AC
          // coefficient of every lane, all of them quantise to 0 (the
          // reference's |F/q| < 1: DESIGN.md §5.2) -- common at Q <= 75, where
          // the chroma quantisers are large.  Then the N-tile is its DC
          // coefficients alone: no quantisation or replay, and in the token
          // variants no staging or AC tokens (the coefficient variants store
          // the zeros).  (Not in the audit variant, whose decisions the tests
          // compare with tests/tau_check.c's model coefficient by coefficient.)
          if constexpr (!AUDIT) {
            if (nt == 2 && cz_on) {
              // |N| < L_z for coefficient z: N + L and N - L both in range,
              // i.e. (N - L) negative and (N + L) not; the sign bit of the
              // AND of (N - L) & ~(N + L) over the lane's 16 is set iff all are
              const int4 *czl = (const int4 *)&s_czl[16 * g];
              uint32_t all = ~0u;
#pragma unroll
              for (int m = 0; m < 4; m++) {
                const int4 Lq = czl[m];
                const int Lv[4] = {Lq.x, Lq.y, Lq.z, Lq.w};
#pragma unroll
                for (int r = 0; r < 4; r++) {
                  const uint32_t lo = (uint32_t)acc[m][r] - (uint32_t)Lv[r], hi = (uint32_t)acc[m][r] + (uint32_t)Lv[r];
                  all &= lo & ~hi;
                }
              }
              if (!__ballot((int)all >= 0)) {
#pragma unroll
                for (int k = 0; k < 16; k++) o[k] = 0;
                bool tie;
                const int dcv = dc_fast(acc[0][0], 8 * q_dc[comp], s_inv8q[comp], tie);
                if (g == 0) o[0] = dcv;
                if (__ballot(tie && g == 0))
                  if (g == 0 && tie) o[0] = dc_tie(dcv, s_dctie[comp]);
                K1_PHASE(3);
                finish(nt, o, true);
                K1_PHASE(4);
                continue;
              }
            }
          }
          // Luma: N' = 2^k t to within E (the A rows carry
          // 2^s_g / q_z, k = 21 + s_g per lane group).  With a = |N'| (one's
          // complement for negatives, so a in [|N'| - 1, |N'|]), hi = a + E + 1
          // and lo = max(a - E, 0) (v_sub_u32 clamp), every multiple m 2^k, m
          // >= 1, of [|N'| - E, |N'| + E] separates hi >> k from lo >> k; when
          // none does, |trunc(t)| = hi >> k, and the signed value is ((hi ^ s)
          // >> k) - s (floor((-x - 1) / 2^k) = -floor(x / 2^k) - 1).  The
          // lane's hazard: some bit >= k set in the OR of (hi ^ lo).  All ops
          // but the xor-add issue at the fast VALU rate
          // (profiles/r05/probe/valu_rate6.txt).  Chroma keeps the fp32 rule:
          // trunc(t - tau) is the output, and the lane's sums of trunc(t -
          // tau) and trunc(t + tau) differ iff some coefficient straddles.
          uint32_t hz;
          // per M-tile: luma, the OR of (hi ^ lo) of its 4 coefficients;
          // chroma, [0] and [1] the sums of trunc(t - tau) and trunc(t + tau)
          // over M-tiles 0-1, [2] and [3] over M-tiles 2-3
          uint32_t xq[4] = {0u, 0u, 0u, 0u};
          auto lquant = [&](int n, uint32_t E1, uint32_t EE, uint32_t kq, uint32_t &x) -> int {
            const int sgn = n >> 31;
            uint32_t hi;
            asm("v_xad_u32 %0, %1, %2, %3" : "=v"(hi) : "v"(n), "v"(sgn), "v"(E1));
            uint32_t lo;
            asm("v_sub_u32_e64 %0, %1, %2 clamp" : "=v"(lo) : "v"(hi), "v"(EE));
            x = __builtin_amdgcn_bitop3_b32(x, hi, lo, 0xF6);  // x | (hi ^ lo)
            // without a hazard hi >> k == lo >> k, and |N'| lies between them:
            // the truncation is (N' >> k) - sgn (floor, +1 for negatives),
            // two fast ops (tests/tau_check.c restates this form)
            return (n >> kq) - sgn;
          };
          if (kflags & K1F_NO_QUANT) {
#pragma unroll
            for (int k = 0; k < 16; k++) o[k] = acc[k >> 2][k & 3];
            hz = 0;
          } else if (nt < 2) {
            const uint32_t E = lcb;
            const uint32_t E1 = E + 1u, EE = 2u * E + 1u;  // hi - EE = a - E
            // one OR per M-tile (4 coefficients): the rare path recomputes only
            // the M-tiles some lane flags
#pragma unroll
            for (int k = 0; k < 16; k++) o[k] = lquant(acc[k >> 2][k & 3], E1, EE, kq, xq[k >> 2]);
            hz = (xq[0] | xq[1] | xq[2] | xq[3]) >> kq;  // nonzero iff a hazard
          } else {
            int slo = 0, shi = 0;
#pragma unroll
            for (int m = 0; m < 4; m++) {
              const float4 fac = *(const float4 *)&s_fac[comp][16 * g + 4 * m];
              const float lc = __uint_as_float(lcb);
              const f2v lc2 = {lc, lc};
#pragma unroll
              for (int h = 0; h < 2; h++) {
                const f2v fa = h ? f2v{fac.z, fac.w} : f2v{fac.x, fac.y};
                const f2v nf = {(float)acc[m][2 * h], (float)acc[m][2 * h + 1]};
                // tau = fac * lc + 1e-6, packed over two coefficients
                const f2v tv = __builtin_elementwise_fma(fa, lc2, (f2v)1.0e-6f);
                const f2v lo = __builtin_elementwise_fma(nf, fa, -tv);
                const f2v hi = __builtin_elementwise_fma(nf, fa, tv);
                const float lo0 = lo[0], lo1 = lo[1], hi0 = hi[0], hi1 = hi[1];
                const int l0 = (int)lo0, l1 = (int)lo1;
                o[4 * m + 2 * h] = l0;
                o[4 * m + 2 * h + 1] = l1;
                slo += l0 + l1;
                shi += (int)hi0 + (int)hi1;
              }
              if (m == 1) {
                xq[0] = (uint32_t)slo;
                xq[1] = (uint32_t)shi;
              }
            }
            xq[2] = (uint32_t)slo;
            xq[3] = (uint32_t)shi;
            hz = (uint32_t)(slo ^ shi);  // nonzero iff a hazard
          }
          // the lane's straddling coefficients, one bit each (same arithmetic
          // as above, coefficient by coefficient), in the M-tiles `need` flags
          // for some lane of the wave (a wave-uniform branch per M-tile: a
          // hazard usually sits in one of them, where recomputing all 16
          // coefficients cost the wave ~100 instructions per rare-path entry)
          auto straddle_mask = [&](uint32_t need) {
            uint32_t mm = 0;
#pragma unroll
            for (int m = 0; m < 4; m++) {
              if (!__ballot((need >> m) & 1u)) continue;
#pragma unroll
              for (int r = 0; r < 4; r++) {
                const int k = 4 * m + r;
                if (nt < 2) {
                  const uint32_t E = lcb;
                  uint32_t x = 0;
                  (void)lquant(acc[m][r], E + 1u, 2u * E + 1u, kq, x);
                  mm |= (uint32_t)((x >> kq) != 0) << k;
                } else {
                  const float nf = (float)acc[m][r];
                  const float fa = s_fac[comp][16 * g + k];
                  const float tv = fmaf(fa, __uint_as_float(lcb), 1.0e-6f);
                  mm |= (uint32_t)((int)fmaf(nf, fa, -tv) != (int)fmaf(nf, fa, tv)) << k;
                }
              }
            }
            return mm;
          };
          // the M-tiles with a hazard in this lane
          auto need_mtiles = [&]() -> uint32_t {
            if (nt < 2) {
              uint32_t nd = 0;
#pragma unroll
              for (int m = 0; m < 4; m++) nd |= (uint32_t)((xq[m] >> kq) != 0u) << m;
              return nd;
            }
            const uint32_t d01 = xq[0] != xq[1], d23 = (xq[2] - xq[0]) != (xq[3] - xq[1]);
            return d01 * 3u + d23 * 12u;
          };
          if constexpr (AUDIT) {
            int blk;
            if (block_of(nt, blk)) a.audit[((long long)p.f * G.nblk + blk) * 4 + g] = (uint16_t)straddle_mask(0xFu);
          }
          {  // z = 0: exact from the pixel sum (fac = 0 above)
            bool tie;
            const int dcv = dc_fast(acc[0][0], 8 * q_dc[comp], s_inv8q[comp], tie);
            if (g == 0) o[0] = dcv;
            if (__ballot(tie && g == 0))
              if (g == 0 && tie) o[0] = dc_tie(dcv, s_dctie[comp]);
          }
          if constexpr (DEFER) {
            // blocks with a straddling coefficient: the N-tile's 16-bit mask
            // goes to the fix masks (one plain store, no returning atomic: a
            // returning one waits, vmcnt(0), for the next tile's DMA and every
            // store in flight); k_fix_blocks recomputes them in FP64 after
            // this kernel
            const unsigned long long need = __ballot(hz != 0);
            if (need && !(kflags & K1F_NO_REPLAY)) {
              int blk;
              const bool valid = block_of(nt, blk);
              const unsigned long long vm = __ballot(valid);
              const uint32_t m16 = (uint32_t)((need | need >> 16 | need >> 32 | need >> 48) & vm) & 0xFFFFu;
              if (m16 && lane == 0) {
                a.fix_mask[(long long)t * 3 + nt] = (uint16_t)m16;
                nrep += (uint32_t)__popc(m16);
              }
            }
          }
          if (!DEFER && __ballot(hz != 0) && !(kflags & K1F_NO_REPLAY)) {
            // rare path: find the straddling coefficients (same arithmetic) and
            // recompute them in FP64 exactly as encoder.c:87-109
            const uint32_t mm = straddle_mask(need_mtiles());
            if (!(kflags & K1F_COUNT_LUMA) || nt < 2)
              nrep += (kflags & K1F_COUNT_PASSES) ? (uint32_t)(lane == 0) : (uint32_t)__popc(mm);
            if constexpr (TOK) {
              // The wave's straddles listed (lane << 4 | k, in the wave's
              // token staging, free until this N-tile's tokens) and replayed
              // 8 at a time: lane x of an 8-lane group sums column x of its
              // block (the reference's inner loop, y order), the group's 8
              // column sums meet by shuffles and every lane of it folds them
              // in x order.  The FP64 operations are encoder.c:87-109's, in its order
              // a lane with several straddles no longer replays them one
              // after another while the wave waits.
              const int c = __popc(mm);
              const int incl = (int)wave_scan64((uint32_t)c);
              const int T = __builtin_amdgcn_readlane(incl, 63);
              const int base = incl - c;
              uint16_t *lst = (uint16_t *)&s_st[wave][0][0];
              int *res = (int *)((uint8_t *)&s_st[wave][0][0] + 256);
              for (int c0 = 0; c0 < T; c0 += 64) {
                {
                  uint32_t m2 = mm;
                  for (int idx = base; m2; idx++) {
                    const int k = __ffs(m2) - 1;
                    m2 &= m2 - 1u;
                    if (idx >= c0 && idx < c0 + 64) lst[idx - c0] = (uint16_t)(lane << 4 | k);
                  }
                }
                wave_lds_sync();
                const int nch = min(T - c0, 64);
                for (int r = 0; r < nch && !(kflags & K1F_REPLAY_NO_FP64); r += 8) {
                  const int j = r + (lane >> 3), x = lane & 7;
                  const int e = lst[j < nch ? j : 0];
                  const int ol = e >> 4, k = e & 15;
                  const int z = 16 * (ol >> 4) + k;
                  const int rz = s_zz[z], v = rz >> 3, u = rz & 7;
                  const uint8_t *Pb = L + (nt * 16 + (ol & 15)) * LDS_BLK;
                  double in = 0.0;
#pragma unroll
                  for (int y = 0; y < 8; y++)
                    in = __dadd_rn(in, __dmul_rn((double)((int)Pb[y * 8 + x] - 128), s_cos[y * 8 + v]));
                  double freq = 0.0;
#pragma unroll
                  for (int xx = 0; xx < 8; xx++)
                    freq = __dadd_rn(freq, __dmul_rn(__shfl(in, (lane & ~7) + xx), s_cos[xx * 8 + u]));
                  if (u == 0) freq = __dmul_rn(freq, SQRT1_2);
                  if (v == 0) freq = __dmul_rn(freq, SQRT1_2);
                  freq = __dmul_rn(freq, 0.25);
                  int tq = (int)__ddiv_rn(freq, (double)s_qint[comp][z]);
                  tq = tq < -2048 ? -2048 : (tq > 2047 ? 2047 : tq);
                  if (x == 0 && j < nch) res[j] = tq;
                }
                wave_lds_sync();
                {
                  // (Measured and dropped, round 5: per slot some lane replayed
                  // a wave-uniform branch, or a wave-uniform walk of the list
                  // writing o[k] by scalar index -- both no faster at Q=50 and
                  // 0.3-0.5% slower at Q=90 than this per-lane select chain,
                  // the first with three times the SGPR spills.)
                  uint32_t m2 = mm;
                  for (int idx = base; m2; idx++) {
                    const int k = __ffs(m2) - 1;
                    m2 &= m2 - 1u;
                    if (idx >= c0 && idx < c0 + 64) {
                      const int v = res[idx - c0];
#pragma unroll
                      for (int jj = 0; jj < 16; jj++) o[jj] = jj == k ? v : o[jj];
                    }
                  }
                }
                wave_lds_sync();
              }
            }
          }
          // token variants: the next tile's DMA has landed before the first
          // store (their VMEM count per tile varies; waiting before N-tile
          // 0, 1 or 2 measured equal, 3.36-3.39 ms)
          if (nt == 0 && !DEFER && !(kflags & K1F_NO_DMAWAIT)) dma_wait();
          K1_PHASE(3);
          finish(nt, o, false);
          K1_PHASE(4);
        }
      } else if (!PIX) {
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
          int o[16];
          finish(nt, o, false);
        }
      }
      if (PIX) wave_lds_sync();
#ifdef MIJ_K1_DIAG
      w_ntiles++;
#endif
      if (tn >= tend) break;
      p = pn;
      t = tn;
      first = false;
    }
  }
  if (__ballot(nrep != 0)) {
    const uint32_t tot = wave_scan64(nrep);
    if (lane == 63) atomicAdd(a.replays, tot);
  }
#ifdef MIJ_K1_DIAG
  if (a.wtime && lane == 0) {
    unsigned long long *w = a.wtime + K1_WTIME_WORDS * ((long long)blockIdx.x * NW + wave);
    w[0] = w_t0;
    w[1] = __builtin_amdgcn_s_memrealtime();
    w[2] = (unsigned long long)w_ntiles;
    for (int k = 0; k < 5; k++) w[3 + k] = ph[k];
  }
#endif
  if (TOK) {  // per-frame histograms of this workgroup
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * 2 * 256; i += NT) {
      const int slot = i >> 9, tb = (i >> 8) & 1, sym = i & 255;
      uint32_t v = 0;
#pragma unroll
      for (int c = 0; c < HREP; c++) v += s_hac[slot][tb][c][sym];
      if (v && f0 + slot < a.nframes)
        atomicAdd(&a.hist[((long long)(f0 + slot) * 4 + (tb ? 3 : 1)) * 257 + sym], v);
    }
    if (threadIdx.x < 64) {
      const int slot = threadIdx.x >> 5, tb = (threadIdx.x >> 4) & 1, sym = threadIdx.x & 15;
      uint32_t v = 0;
#pragma unroll
      for (int c = 0; c < HREP; c++) v += s_hdc[slot][tb][c][sym];
      if (v && f0 + slot < a.nframes)
        atomicAdd(&a.hist[((long long)(f0 + slot) * 4 + (tb ? 2 : 0)) * 257 + sym], v);
    }
  }
}


// ===========================================================================
// k_fix_blocks: the blocks K1 listed (a coefficient whose fast-path error
// interval straddles a truncation boundary, or a DC tie) recomputed exactly
// as the reference computes them: colour conversion in FP64 with uint8_t
// truncation (encoder.c:133-135), 4:2:0 integer averages (:137-138), the
// FP64 DCT, quantisation, clip and zigzag (:81-112, :65-70).  One wave per
// listed block: lane l stages pixel (l & 7, l >> 3), then computes zigzag
// coefficient l.  Persistent grid over the device-side list length.
// ===========================================================================
// px = B, G, R (ib = 0, ir = 2) or R, G, B (ib = 2, ir = 0)
__device__ __forceinline__ int y_ref(const uint8_t *px, int ib, int ir) { return y_f64(px[ir], px[1], px[ib]); }
__device__ __forceinline__ int cb_ref(const uint8_t *px, int ib, int ir) { return cb_f64(px[ir], px[1], px[ib]); }
__device__ __forceinline__ int cr_ref(const uint8_t *px, int ib, int ir) { return cr_f64(px[ir], px[1], px[ib]); }

// The blocks come from K1's per-N-tile fix masks (K1Args::fix_mask): each
// wave scans 64 masks per step, takes the nonzero ones in turn, zeroes them
// and recomputes their blocks one after another.
__global__ __launch_bounds__(256) void k_fix_blocks(K1Args a) {
  __shared__ __attribute__((aligned(8))) uint8_t s_px[4][64];
  __shared__ double s_inner[4][64];
  __shared__ double s_cos[64];
  __shared__ int s_q[2][64];
  const Tables *__restrict__ T = a.tab;
  if (threadIdx.x < 64) s_cos[threadIdx.x] = T->cosd[threadIdx.x];
  if (threadIdx.x < 128) s_q[threadIdx.x >> 6][threadIdx.x & 63] = T->qint[threadIdx.x >> 6][threadIdx.x & 63];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Geom G = a.g;
  const int x = lane & 7, y = lane >> 3;
  // lane z's output coefficient: zigzag z = frequency (v, u) (encoder.c:38-46)
  const int rz = c_zigzag[lane], v = rz >> 3, u = rz & 7;
  const int ib = a.rgb ? 2 : 0, ir = 2 - ib;
  const long long nmask = (long long)a.nframes * G.tiles_per_frame * 3;
  for (long long base = ((long long)blockIdx.x * 4 + wave) * 64; base < nmask; base += (long long)gridDim.x * 4 * 64) {
    const long long e = base + lane;
    const uint32_t mk = e < nmask ? a.fix_mask[e] : 0u;
    unsigned long long any = __ballot(mk != 0);
    if (mk) a.fix_mask[e] = 0;  // consumed: all zero again for the next K1
    while (any) {
      const int l = __ffsll((long long)any) - 1;
      any &= any - 1ull;
      uint32_t mm = (uint32_t)__builtin_amdgcn_readlane((int)mk, l);
      const int tg = (int)((base + l) / 3), nt = (int)(base + l - 3LL * tg);  // global tile, N-tile
      const int f = tg / G.tiles_per_frame, rem = tg - f * G.tiles_per_frame;
      const int ty = rem / G.tiles_x, tx = rem - ty * G.tiles_x;
      const uint8_t *img = a.in + (long long)f * a.in_fs;
      const FGeom fg = frame_geom(G, a.fdims, f);
      const int bw = fg.bw, mw = fg.mw;
      while (mm) {
        const int bb = __ffs(mm) - 1;
        mm &= mm - 1u;
        // the block of column bb of N-tile nt (K1's block_at)
        const int blk = nt < 2 ? (2 * ty + nt) * bw + tx * 16 + bb
                               : fg.nY + (bb >= 8 ? fg.nC : 0) + ty * mw + tx * 8 + (bb & 7);
        int pv, comp;
        if (nt < 2) {  // lane = pixel (x, y) of the block
          comp = 0;
          const int bx = tx * 16 + bb, by = 2 * ty + nt;
          pv = y_ref(img + (long long)(8 * by + y) * a.pitch + (8 * bx + x) * 3, ib, ir);
        } else {
          comp = 1;
          const int cr = bb >= 8, mx = tx * 8 + (bb & 7), my = ty;
          const uint8_t *q = img + (long long)(16 * my + 2 * y) * a.pitch + (16 * mx + 2 * x) * 3;
          int sum = 0;
          for (int dy = 0; dy < 2; dy++)
            for (int dx = 0; dx < 2; dx++) {
              const uint8_t *px = q + (long long)dy * a.pitch + dx * 3;
              sum += cr ? cr_ref(px, ib, ir) : cb_ref(px, ib, ir);
            }
          pv = sum / 4;
        }
        s_px[wave][lane] = (uint8_t)pv;
        wave_lds_sync();
        {  // column pass, lane = (x_t = lane >> 3, y_f = lane & 7), summed from 0 in y_t order
          const int xt = lane >> 3, yf = lane & 7;
          double in = 0.0;
          for (int yt = 0; yt < 8; yt++)
            in = __dadd_rn(in, __dmul_rn((double)((int)s_px[wave][yt * 8 + xt] - 128), s_cos[yt * 8 + yf]));
          s_inner[wave][xt * 8 + yf] = in;
        }
        wave_lds_sync();
        // row pass for frequency (v, u), summed from 0 in x_t order, then the
        // 1/sqrt2 factors (u first), /4, quantisation, clip
        double freq = 0.0;
        for (int xt = 0; xt < 8; xt++) freq = __dadd_rn(freq, __dmul_rn(s_inner[wave][xt * 8 + v], s_cos[xt * 8 + u]));
        if (u == 0) freq = __dmul_rn(freq, SQRT1_2);
        if (v == 0) freq = __dmul_rn(freq, SQRT1_2);
        freq = __dmul_rn(freq, 0.25);
        int o = (int)__ddiv_rn(freq, (double)s_q[comp][lane]);
        o = o < -2048 ? -2048 : (o > 2047 ? 2047 : o);
        a.coef[(long long)f * G.coef_fs + (long long)blk * 64 + lane] = (int16_t)o;
        if (lane == 0) a.dc[(long long)f * G.nblk + blk] = (int16_t)o;
        wave_lds_sync();
      }
    }
  }
}

// ===========================================================================
// DC differencing in place (encoder.c:168-177), for the drop-in rgb_to_dct
// whose caller expects differenced DCs in the planes.
// ===========================================================================
__global__ void k_dc_diff(int16_t *coef, const int16_t *dc, Geom G, int nframes, const int2 *fd) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)nframes * G.nblk;
  if (i >= total) return;
  const int f = (int)(i / G.nblk);
  const int j = (int)(i - (long long)f * G.nblk);
  const FGeom fg = frame_geom(G, fd, f);
  if (j >= fg.nY + 2 * fg.nC) return;
  const bool first = j == 0 || j == fg.nY || j == fg.nY + fg.nC;
  const int16_t prev = first ? 0 : dc[i - 1];
  coef[(long long)f * G.coef_fs + (long long)j * 64] = (int16_t)(dc[i] - prev);
}

// ===========================================================================
// Segments.  Segment s of a frame = the blocks of one K1 N-tile row run:
//   Y  s in [0, nsy):           block row s / tiles_x, tile column s % tiles_x
//   Cb s in [nsy, nsy+nsc):     MCU row, tile column (8 blocks)
//   Cr s in [nsy+nsc, nseg):    likewise
// so each scan's segments are contiguous and in scan order.
// ===========================================================================
// (fg: the frame's image; returns false for a canvas segment outside it)
__device__ __forceinline__ bool seg_info(const Geom &G, const FGeom &fg, int s, int &comp, int &first,
                                         int &cstart, int &local) {
  if (s < G.nsy) {
    comp = 0;
    local = s;
    cstart = 0;
    const int r = (int)div_by((uint32_t)s, G.tx_m, G.tx_s), tx = s - r * G.tiles_x;
    first = r * fg.bw + tx * 16;
    return r < 2 * fg.rows && tx < fg.tiles_x;
  }
  const int c = s - G.nsy;
  comp = 1 + (c >= G.nsc);
  local = comp == 1 ? c : c - G.nsc;
  cstart = comp == 1 ? fg.nY : fg.nY + fg.nC;
  const int r = (int)div_by((uint32_t)local, G.tx_m, G.tx_s), tx = local - r * G.tiles_x;
  first = cstart + r * fg.mw + tx * 8;
  return r < fg.rows && tx < fg.tiles_x;
}

// ===========================================================================
// k_seg_dc: DC difference of every segment's first block (its predecessor
// lies in another segment, encoder.c:168-177): token 0 of the segment and
// the DC class histogram h[luma, chroma][class] (LDS).  One thread per
// segment; k_tables runs the same per-segment step in its DC-table waves.
// ===========================================================================
// (split in two so that callers can have several segments' loads in flight)
struct SegDc {
  int comp, dc, pred;
  bool ok;
};
constexpr int SEGDC_U = 32;  // segments in flight per lane in k_tables' DC waves
__device__ __forceinline__ SegDc seg_dc_load(const EntArgs &a, const FGeom &fg, int f, int s) {
  SegDc r;
  int first, cstart, local;
  r.ok = seg_info(a.g, fg, s, r.comp, first, cstart, local);
  r.dc = r.pred = 0;
  if (r.ok) {
    const long long fb = (long long)f * a.g.nblk;
    // a component's first block is predicted from 0 (encoder.c:168-177), or
    // from the previous band's last DC when the frame is split into bands
    r.pred = first == cstart ? (a.dc_pred ? (int)a.dc_pred[f * 4 + r.comp] : 0) : (int)a.dc[fb + first - 1];
    r.dc = (int)a.dc[fb + first];
  }
  return r;
}
// The class counts go to hs[(luma ? 0 : 16) + class][lane & 31]: 32 copies
// of every counter, so a wave's 64 atomics meet at most in pairs (one
// counter per class took every lane of a wave with the same class in turn).
__device__ __forceinline__ void seg_dc_store(const EntArgs &a, int f, int s, const SegDc &r, uint32_t *hs, int lane) {
  if (!r.ok) return;
  const int diff = r.dc - r.pred;
  const int cls = mag_class(diff);
#ifdef MIJ_K1_DIAG
  if (!(a.seg_dc & 2))
#endif
  a.tok0[(long long)f * a.g.nseg + s] = (uint32_t)cls | (mag_bits(diff, cls) << 16);
  atomicAdd(&hs[((r.comp ? 16 : 0) + cls) * 32 + (lane & 31)], 1u);
}

constexpr int SEGDC_WG = 256;
// (64-thread workgroups fit beside a running 10-wave K1 -- 256-thread ones
// wait for it to end; profiles/r03/overlap_trace.txt; the 12-wave K1 leaves
// room for neither)
// one workgroup's share (workgroup b of the launch's segment DCs; hs: 32 x
// 32 words of LDS)
__device__ __forceinline__ void seg_dc_block(const EntArgs &a, int b, uint32_t *hs) {
  const int per = (a.g.nseg + SEGDC_WG - 1) / SEGDC_WG;
  const int f = b / per;
  const int s = (b - f * per) * SEGDC_WG + threadIdx.x;
  for (int i = threadIdx.x; i < 32 * 32; i += SEGDC_WG) hs[i] = 0;
  __syncthreads();
  if (s < a.g.nseg) seg_dc_store(a, f, s, seg_dc_load(a, frame_geom(a.g, a.fdims, f), f, s), hs, threadIdx.x & 63);
  __syncthreads();
  if (threadIdx.x < 32) {
    uint32_t v = 0;
    for (int c = 0; c < 32; c++) v += hs[threadIdx.x * 32 + ((c + threadIdx.x) & 31)];
    if (v) {
      if (a.dc_last) {
        // (returning: the wave waits until the add is performed -- device-wide
        // atomics meet at one coherence point -- before the block's arrival
        // is counted; no cache-writeback fence)
        const uint32_t old = atomicAdd(&a.dcx[(long long)f * 64 + threadIdx.x], v);
        asm volatile("" ::"v"(old));
      } else {
        atomicAdd(&a.hist[((long long)f * 4 + (threadIdx.x >= 16 ? 2 : 0)) * 257 + (threadIdx.x & 15)], v);
      }
    }
  }
}

__global__ __launch_bounds__(SEGDC_WG) void k_seg_dc(EntArgs a) {
  __shared__ uint32_t hs[32 * 32];
  seg_dc_block(a, blockIdx.x, hs);
}


// ===========================================================================
// k_tables / k_tables_1w: the four optimized Huffman tables of a frame
// (encoder.c:180-301), one wave per table (build_table_wave2 below).
// ===========================================================================
template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
  return ((unsigned long long)hi << 32) | lo;
}
// permlane16/32 swap of a 64-bit value: (a, b) = one lane's own value and its
// partner's (a in the odd rows / upper half, b in the others)
template <int W>
__device__ __forceinline__ void swap_u64(unsigned long long x, unsigned long long &a, unsigned long long &b) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if constexpr (W == 16) {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a = ((unsigned long long)rh[0] << 32) | rl[0];
    b = ((unsigned long long)rh[1] << 32) | rl[1];
  } else {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = ((unsigned long long)rh[0] << 32) | rl[0];
    b = ((unsigned long long)rh[1] << 32) | rl[1];
  }
}

// (MIJ_K1_DIAG build, MIJ_TAB_TIME: tm != null gets the wave's phase clocks)
#ifdef MIJ_K1_DIAG
#define TAB_T(k) do { if (tm && lane == 0) tm[k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define TAB_T(k) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// build_table_wave2: init_huff_table restated so that no phase is a
// lane-serial LDS chain.
//  - leaves sorted by a register bitonic network (DPP / permlane partners, no
//    LDS round trips);
//  - the two-queue merge runs on uniform values read with v_readlane from
//    64-entry register windows of the queues; a key carries its node's id and
//    leaf count, so lane 0 only writes (the new queue entry and the two
//    children's parent links, no dependent reads);
//  - code lengths (leaf depths) and the chain order of :223-226 (a leaf's
//    place = the leaves of the left subtrees it hangs right of) by pointer
//    jumping over the merge tree;
//  - counts, the 16-bit limit loop (:239-259), the symbol order (:262-268) and
//    the canonical codes (:280-300) on per-lane length vectors with ballots
//    and readlane.
// Key: freq << 32 | (256 - label) << 19 | leaves << 10 | node; (freq, label)
// order the entries (labels of live entries are distinct), the low bits ride
// along.  Nodes: leaf = its queue slot (0 = symbol 256), merge j = nl + j.
// ---------------------------------------------------------------------------
struct TabScratch2 {
  union {
    struct {
      unsigned long long ql[257 + 64];  // sorted leaves, ~0 past the end
      unsigned long long qm[256 + 64];  // merged nodes in queue order
    };
    struct {  // after the merges
      int sorted[256];
      int slen[256];
      int scode[256];
    };
  };
  int rec[256];  // narrow merge loop: per merge c1 | c2 << 10 | leaves(c1) << 20
  int par[514];  // node -> parent (0xFFFF: root), then pointer-jumping state
  int dep[514];
  int off[514];
  int scl[257];  // symbol -> code length (unlimited)
  int spos[257];  // symbol -> place in the chain
  int seq[257];   // chain order -> symbol
};

// a uniform int the compiler cannot follow (keeps it from strength-reducing
// rare-path LDS addresses into per-iteration VALU adds)
__device__ __forceinline__ int opq(int x) {
  asm volatile("" : "+s"(x));
  return x;
}
// v_writelane: v with lane idx (uniform) set to x (uniform)
__device__ __forceinline__ uint32_t wl32(uint32_t v, uint32_t x, int idx) {
  // (two scalar operands: the lane select goes through m0, gfx9's one-SGPR constant bus)
  asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "s"(idx) : "m0");
  return v;
}
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int idx) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, idx);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), idx);
  return ((unsigned long long)hi << 32) | lo;
}
// the value of lane ^ J (J < 64)
template <int J>
__device__ __forceinline__ unsigned long long xor_fetch(unsigned long long x, int lane) {
  if constexpr (J == 1) return dpp_u64<0xB1>(x);  // quad_perm [1,0,3,2]
  else if constexpr (J == 2) return dpp_u64<0x4E>(x);  // quad_perm [2,3,0,1]
  else if constexpr (J == 4) {
    const unsigned long long up = dpp_u64<0x12C>(x), dn = dpp_u64<0x124>(x);  // row_ror:12 (lane+4), :4 (lane-4)
    return (lane & 4) ? dn : up;
  } else if constexpr (J == 8) return dpp_u64<0x128>(x);  // row_ror:8
  else {
    unsigned long long a, b;
    swap_u64<J>(x, a, b);
    return (lane & J) ? a : b;
  }
}
// the value of lane ^ (K - 1) (K <= 64)
template <int K>
__device__ __forceinline__ unsigned long long flip_fetch(unsigned long long x, int lane) {
  if constexpr (K == 2) return dpp_u64<0xB1>(x);
  else if constexpr (K == 4) return dpp_u64<0x1B>(x);  // quad_perm [3,2,1,0]
  else if constexpr (K == 8) return dpp_u64<0x141>(x);  // row_half_mirror
  else if constexpr (K == 16) return dpp_u64<0x140>(x);  // row_mirror
  else if constexpr (K == 32) return dpp_u64<0x140>(xor_fetch<16>(x, lane));
  else return flip_fetch<32>(xor_fetch<32>(x, lane), lane);
}
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a < b ? b : a; }

// 32-bit partners for the narrow-key sort
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
template <int J>
__device__ __forceinline__ uint32_t xor_fetch32(uint32_t x, int lane) {
  if constexpr (J == 1) return dpp32<0xB1>(x);
  else if constexpr (J == 2) return dpp32<0x4E>(x);
  else if constexpr (J == 4) {
    // (both moves with every lane active: a DPP under a lane branch reads 0
    // from the inactive lanes)
    const uint32_t up = dpp32<0x12C>(x), dn = dpp32<0x124>(x);
    return (lane & 4) ? dn : up;
  }
  else if constexpr (J == 8) return dpp32<0x128>(x);
  else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (lane & 32) ? r[0] : r[1];
  }
}
template <int K>
__device__ __forceinline__ uint32_t flip_fetch32(uint32_t x, int lane) {
  if constexpr (K == 2) return dpp32<0xB1>(x);
  else if constexpr (K == 4) return dpp32<0x1B>(x);
  else if constexpr (K == 8) return dpp32<0x141>(x);
  else if constexpr (K == 16) return dpp32<0x140>(x);
  else if constexpr (K == 32) return dpp32<0x140>(xor_fetch32<16>(x, lane));
  else return flip_fetch32<32>(xor_fetch32<32>(x, lane), lane);
}
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a < b ? b : a; }
template <int J>
__device__ __forceinline__ void bsort_half32(uint32_t (&k)[4], int lane) {
  if constexpr (J >= 64) {
    constexpr int R = J / 64;
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (!(r & R)) {
        const uint32_t x = k[r], y = k[r | R];
        k[r] = umin32(x, y);
        k[r | R] = umax32(x, y);
      }
  } else {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t p = xor_fetch32<J>(k[r], lane);
      k[r] = (lane & J) ? umax32(k[r], p) : umin32(k[r], p);
    }
  }
  if constexpr (J > 1) bsort_half32<J / 2>(k, lane);
}
template <int K>
__device__ __forceinline__ void bsort_level32(uint32_t (&k)[4], int lane) {
  if constexpr (K <= 64) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t p = flip_fetch32<K>(k[r], lane);
      k[r] = (lane & (K / 2)) ? umax32(k[r], p) : umin32(k[r], p);
    }
  } else {
    constexpr int X = K / 64 - 1;
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (r < (r ^ X)) {
        const int q = r ^ X;
        const uint32_t mr = flip_fetch32<64>(k[r], lane), mq = flip_fetch32<64>(k[q], lane);
        k[r] = umin32(k[r], mq);
        k[q] = umax32(k[q], mr);
      }
  }
  if constexpr (K >= 4) bsort_half32<K / 4>(k, lane);
  if constexpr (K < 256) bsort_level32<K * 2>(k, lane);
}

// ascending bitonic sort of 256 keys, element e = lane + 64 r in k[r]
template <int J>
__device__ __forceinline__ void bsort_half(unsigned long long (&k)[4], int lane) {
  if constexpr (J >= 64) {
    constexpr int R = J / 64;
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (!(r & R)) {
        const unsigned long long x = k[r], y = k[r | R];
        k[r] = umin64(x, y);
        k[r | R] = umax64(x, y);
      }
  } else {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned long long p = xor_fetch<J>(k[r], lane);
      k[r] = (lane & J) ? umax64(k[r], p) : umin64(k[r], p);
    }
  }
  if constexpr (J > 1) bsort_half<J / 2>(k, lane);
}
template <int K>
__device__ __forceinline__ void bsort_level(unsigned long long (&k)[4], int lane) {
  if constexpr (K <= 64) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned long long p = flip_fetch<K>(k[r], lane);
      k[r] = (lane & (K / 2)) ? umax64(k[r], p) : umin64(k[r], p);
    }
  } else {
    // partner e ^ (K - 1): register r ^ (K / 64 - 1), lane ^ 63
    constexpr int X = K / 64 - 1;
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (r < (r ^ X)) {
        const int q = r ^ X;
        const unsigned long long mr = flip_fetch<64>(k[r], lane), mq = flip_fetch<64>(k[q], lane);
        k[r] = umin64(k[r], mq);
        k[q] = umax64(k[q], mr);
      }
  }
  if constexpr (K >= 4) bsort_half<K / 4>(k, lane);
  if constexpr (K < 256) bsort_level<K * 2>(k, lane);
}

__device__ __forceinline__ void build_table_wave2(const uint32_t *hist, const uint32_t *extra, HuffCode *hc, uint32_t *ehuf,
                                  TabScratch2 *S, int lane, int *err, unsigned long long *tm = nullptr) {
  TAB_T(0);
  uint32_t f[5];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int s = lane + 64 * i;
    f[i] = s < 256 ? hist[s] : (s == 256 ? 1u : 0u);  // :364-367
    if (extra && i == 0 && lane < 16) f[i] += extra[lane];
    if (s < 257) S->scl[s] = 0;
  }
  TAB_T(1);
  // leaves: symbols 0..255 with a count, ascending; symbol 256 (count 1, the
  // highest index) is the least key of all and heads the queue
  unsigned long long k[4];
  bool wide = false;
#pragma unroll
  for (int r = 0; r < 4; r++) wide |= f[r] >= (1u << 23);
  if (__ballot(wide)) {
#pragma unroll
    for (int r = 0; r < 4; r++)
      k[r] = f[r] ? ((unsigned long long)f[r] << 32) | ((unsigned long long)(256 - (lane + 64 * r)) << 19) | (1ull << 10)
                  : ~0ull;
    bsort_level<2>(k, lane);
  } else {
    // counts below 2^23 (every frame up to 8K at Q=50): the same order on
    // 32-bit keys (count << 9 | 256 - symbol), half the partner moves
    uint32_t k32[4];
#pragma unroll
    for (int r = 0; r < 4; r++) k32[r] = f[r] ? (f[r] << 9) | (uint32_t)(256 - (lane + 64 * r)) : ~0u;
    bsort_level32<2>(k32, lane);
#pragma unroll
    for (int r = 0; r < 4; r++)
      k[r] = k32[r] == ~0u ? ~0ull
                           : ((unsigned long long)(k32[r] >> 9) << 32) | ((unsigned long long)(k32[r] & 511) << 19) |
                                 (1ull << 10);
  }
  int nl = 1;
#pragma unroll
  for (int r = 0; r < 4; r++) nl += __popcll(__ballot(f[r] != 0));
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int q = 1 + lane + 64 * r;
    S->ql[q] = k[r] == ~0ull ? ~0ull : k[r] | (unsigned)q;
  }
  if (lane == 0) S->ql[0] = (1ull << 32) | (1ull << 10);
  S->ql[257 + lane] = ~0ull;
#pragma unroll
  for (int i = 0; i < 5; i++)
    if (lane + 64 * i < 320) S->qm[lane + 64 * i] = ~0ull;
  wave_lds_sync();
  TAB_T(2);
  // the merges (encoder.c:196-226) on uniform values; v1 = the least key, v2
  // the next; K = the merged node, queued at its key's place.  Narrow keys
  // when the table's whole count is below 2^23 (every frame up to ~4K at
  // Q=50): count << 9 | (256 - label) in one 32-bit word, leaves << 10 |
  // node beside it, one scalar compare per decision; the merge records stay
  // in a register (one lane per merge) and go to LDS 64 at a time.
  uint32_t fsum = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) fsum += f[r];
  const uint32_t total_count = __builtin_amdgcn_readlane((int)wave_scan64(fsum), 63) + 1u;
  int root_label = 256;
  uint32_t total = 1;
  bool narrow_done = false;
  if (total_count < (1u << 23)) {
    // Short form (every table whose merged nodes queue in creation order, i.e.
    // no insert below): the loop carries only what decides the merges -- the
    // narrow keys of the four queue heads and the leaf counts of the merged
    // ones -- and records per merge which heads it took (2 bits) and v1's
    // leaf count.  The queue places, hence the node ids (leaf = its place,
    // merge j = nl + j), follow after the loop from a prefix sum of the taken
    // leaves: each merge takes two heads, so mh = 2 step - lh.  New entries
    // go into the merged-key window by v_writelane (to LDS only past it); an
    // insert abandons this form for the general loop below.
    int lw = 0, mw = 0, lh = 0, mh = 0, step = 0;
    uint32_t wlk, wmk = ~0u, wms = 0, rec = 0, mlast = 0;
    {
      const unsigned long long v = S->ql[lane];
      wlk = ((uint32_t)(v >> 32) << 9) | ((uint32_t)v >> 19);
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    const int nsteps = nl - 1;
    bool ok = true;
    while (step < nsteps) {
      if (lh - lw > 30) {  // (early reloads: the runs below stay long)
        lw = lh;
        const unsigned long long v = S->ql[lw + lane];
        wlk = ((uint32_t)(v >> 32) << 9) | ((uint32_t)v >> 19);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      }
      if (mh - mw > 30 || step - mw >= 48) {
        // the window's entries to LDS, then the window from the merged head
        // (also when the appended entries near its end: a queue of up to 63
        // merged nodes stays in this form)
        if (mw + lane < step) S->qm[mw + lane] = ((unsigned long long)wms << 32) | wmk;
        wave_lds_sync();
        mw = mh;
        const unsigned long long v = S->qm[mw + lane];
        wmk = (uint32_t)v;
        wms = (uint32_t)(v >> 32);
        __builtin_amdgcn_s_waitcnt(0xC07F);
      }
      // merges the windows hold: the heads' readlanes in range (two heads
      // taken per merge), each new entry in the merged window, the records in
      // one 64-lane row
      int bud = nsteps - step;
      bud = min(bud, (63 - (lh - lw)) >> 1);
      bud = min(bud, (63 - (mh - mw)) >> 1);
      bud = min(bud, 64 - (step - mw));
      bud = min(bud, 64 - (step & 63));
      if (bud < 1) {  // more than a window of merged nodes queued: the general loop
        ok = false;
        break;
      }
      uint32_t il = lh - lw, im = mh - mw, mwl = step - mw, rl = step & 63, st = step;
      // (the budget's min may land in a VGPR: its end made scalar for the asm)
      const uint32_t send = (uint32_t)__builtin_amdgcn_readfirstlane(step + bud);
      uint32_t flag, K, sz, t1, t2, t3, t4, t5;
      // One merge per pass, all scalar but the readlanes and writelanes:
      //   a, b = leaf heads; c, d = merged heads (sc, sd their leaf counts)
      //   ac = a < c; k1 = min; x = ac ? b : a; y = ac ? c : d; bx = x < y
      //   K = k1 + (k2 & ~511) (counts add, v1's label stays)
      //   rec lane (step & 63) = ac | bx << 1 | leaves(v1) << 2
      // An entry below the last appended key (a possible insert) leaves the
      // loop before its append (flag = 1).  (s_nop 4 first: the operands may
      // come from VALU writes just before.)
      asm volatile(
          "s_nop 4\n"
          "1:\n\t"
          "s_add_u32 %[t5], %[il], 1\n\t"
          "s_add_u32 %[t4], %[im], 1\n\t"
          "v_readlane_b32 %[K], %[wlk], %[il]\n\t"
          "v_readlane_b32 %[t1], %[wlk], %[t5]\n\t"
          "v_readlane_b32 %[t2], %[wmk], %[im]\n\t"
          "v_readlane_b32 %[t3], %[wmk], %[t4]\n\t"
          "v_readlane_b32 %[sz], %[wms], %[im]\n\t"
          "v_readlane_b32 %[t4], %[wms], %[t4]\n\t"
          // K = a, t1 = b, t2 = c, t3 = d, sz = sc, t4 = sd
          "s_cmp_lt_u32 %[K], %[t2]\n\t"
          "s_cselect_b32 %[t5], %[K], %[t2]\n\t"   // t5 = k1
          "s_cselect_b32 %[K], %[t1], %[K]\n\t"    // K = x
          "s_cselect_b32 %[t1], %[t2], %[t3]\n\t"  // t1 = y
          "s_cselect_b32 %[t2], 1, %[sz]\n\t"      // t2 = s1
          "s_cselect_b32 %[t3], %[sz], %[t4]\n\t"  // t3 = sy
          "s_cselect_b32 %[t4], 1, 0\n\t"          // t4 = ac
          "s_cmp_lt_u32 %[K], %[t1]\n\t"
          "s_cselect_b32 %[K], %[K], %[t1]\n\t"    // K = k2
          "s_cselect_b32 %[t3], 1, %[t3]\n\t"      // t3 = s2
          "s_cselect_b32 %[t1], 1, 0\n\t"          // t1 = bx
          "s_and_b32 %[K], %[K], 0xfffffe00\n\t"
          "s_add_u32 %[K], %[K], %[t5]\n\t"        // K
          "s_add_u32 %[sz], %[t2], %[t3]\n\t"      // sz = s1 + s2
          "s_add_u32 %[t3], %[t4], %[t1]\n\t"      // t3 = leaves taken
          "s_lshl1_add_u32 %[t1], %[t1], %[t4]\n\t"
          "s_lshl2_add_u32 %[t1], %[t2], %[t1]\n\t"  // record
          "s_mov_b32 m0, %[rl]\n\t"
          "v_writelane_b32 %[rec], %[t1], m0\n\t"
          "s_add_u32 %[il], %[il], %[t3]\n\t"
          "s_sub_u32 %[im], %[im], %[t3]\n\t"
          "s_add_u32 %[im], %[im], 2\n\t"
          "s_cmp_gt_u32 %[ml], %[K]\n\t"
          "s_cbranch_scc1 2f\n\t"
          "s_mov_b32 m0, %[mwl]\n\t"
          "v_writelane_b32 %[wmk], %[K], m0\n\t"
          "v_writelane_b32 %[wms], %[sz], m0\n\t"
          "s_mov_b32 %[ml], %[K]\n\t"
          "s_add_u32 %[mwl], %[mwl], 1\n\t"
          "s_add_u32 %[rl], %[rl], 1\n\t"
          "s_add_u32 %[st], %[st], 1\n\t"
          "s_cmp_lg_u32 %[st], %[send]\n\t"
          "s_cbranch_scc1 1b\n\t"
          "s_mov_b32 %[flag], 0\n\t"
          "s_branch 3f\n"
          "2:\n\t"
          "s_mov_b32 %[flag], 1\n"
          "3:"
          : [il] "+s"(il), [im] "+s"(im), [mwl] "+s"(mwl), [rl] "+s"(rl), [st] "+s"(st), [ml] "+s"(mlast),
            [rec] "+v"(rec), [wmk] "+v"(wmk), [wms] "+v"(wms), [flag] "=&s"(flag), [K] "=&s"(K), [sz] "=&s"(sz),
            [t1] "=&s"(t1), [t2] "=&s"(t2), [t3] "=&s"(t3), [t4] "=&s"(t4), [t5] "=&s"(t5)
          : [wlk] "v"(wlk), [send] "s"(send)
          : "m0", "scc");
      step = (int)st;
      lh = lw + (int)il;
      mh = mw + (int)im;
      if (flag) {
        if (step > mh) {  // an equal-count node with a smaller key is queued: the general loop
          ok = false;
          break;
        }
        wmk = wl32(wmk, K, step - mw);  // (step - mw < 64: the budget)
        wms = wl32(wms, sz, step - mw);
        mlast = K;
        step++;
      }
      if ((step & 63) == 0) S->rec[step - 64 + lane] = (int)rec;
    }
    const uint32_t klast = mlast;
    if (ok) {
      {
        const int b0 = nsteps & ~63;
        if (b0 + lane < nsteps) S->rec[b0 + lane] = (int)rec;
      }
      wave_lds_sync();
      // the merges' children: leaf places by a prefix sum of the leaves taken
      int carry = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int j = lane + 64 * i;
        const uint32_t r = j < nsteps ? (uint32_t)S->rec[j] : 0u;
        const int e = (int)(r & 1u) + (int)((r >> 1) & 1u);
        const int incl = (int)wave_scan64((uint32_t)e);
        const int lb = carry + incl - e, mb = 2 * j - lb;
        carry += __builtin_amdgcn_readlane(incl, 63);
        if (j < nsteps) {
          const bool ac = r & 1u, bx = r & 2u;
          const int c1 = ac ? lb : nl + mb;
          const int c2 = bx ? (ac ? lb + 1 : lb) : (ac ? nl + mb : nl + mb + 1), node = nl + j;
          S->par[c1] = node;
          S->par[c2] = node;
          S->off[c1] = 0;
          S->off[c2] = (int)(r >> 2);  // v2's chain follows v1's (:223-226)
        }
      }
      if (nsteps > 0) {
        root_label = 256 - (int)(klast & 511u);
        total = klast >> 9;
      }
      narrow_done = true;
    } else {
#pragma unroll
      for (int i = 0; i < 5; i++)
        if (lane + 64 * i < 320) S->qm[lane + 64 * i] = ~0ull;
      wave_lds_sync();
    }
  }
  if (total_count < (1u << 23) && !narrow_done) {
    int lw = 0, mw = 0, lh = 0, mh = 0, mt = 0;
    uint32_t wlk, wla, wmk = ~0u, wma = ~0u, rec = 0;
    auto split = [](unsigned long long v, uint32_t &key, uint32_t &aux) {
      key = ((uint32_t)(v >> 32) << 9) | ((uint32_t)v >> 19);
      aux = (uint32_t)v & 0x7FFFFu;
    };
    split(S->ql[lane], wlk, wla);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    uint32_t mlast = 0;  // the last appended key
    const int nsteps = nl - 1;
    for (int step = 0; step < nsteps; step++) {
      if (lh + 1 - lw > 63) {
        lw = lh;
        split(S->ql[lw + lane], wlk, wla);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      }
      if (mh + 1 - mw > 63) {
        mw = mh;
        split(S->qm[mw + lane], wmk, wma);
        __builtin_amdgcn_s_waitcnt(0xC07F);
      }
      const int il = lh - lw, im = mh - mw;
      const uint32_t ak = __builtin_amdgcn_readlane(wlk, il), bk = __builtin_amdgcn_readlane(wlk, il + 1);
      const uint32_t ck = __builtin_amdgcn_readlane(wmk, im), dk = __builtin_amdgcn_readlane(wmk, im + 1);
      const uint32_t aa = __builtin_amdgcn_readlane(wla, il), ba = __builtin_amdgcn_readlane(wla, il + 1);
      const uint32_t ca = __builtin_amdgcn_readlane(wma, im), da = __builtin_amdgcn_readlane(wma, im + 1);
      const bool ac = ak < ck;
      const uint32_t k1 = ac ? ak : ck, k1a = ac ? aa : ca;
      const uint32_t x = ac ? bk : ak, xa = ac ? ba : aa, y = ac ? ck : dk, ya = ac ? ca : da;
      const bool bx = x < y;
      const uint32_t k2 = bx ? x : y, k2a = bx ? xa : ya;
      const int dlh = ac ? (bx ? 2 : 1) : (bx ? 1 : 0);
      lh += dlh;
      mh += 2 - dlh;
      const uint32_t lab1 = k1 & 511u;  // 256 - v1
      const uint32_t fs = (k1 >> 9) + (k2 >> 9);
      const uint32_t sz1 = k1a >> 10, node = (uint32_t)(nl + step);
      const uint32_t K = (fs << 9) | lab1, Ka = ((sz1 + (k2a >> 10)) << 10) | node;
      // v2's chain follows v1's (:223-226): the merge's record
      if (lane == (step & 63)) rec = (k1a & 1023u) | ((k2a & 1023u) << 10) | (sz1 << 20);
      if ((step & 63) == 63) S->rec[step - 63 + lane] = (int)rec;
      const unsigned long long K64 = ((unsigned long long)fs << 32) | (lab1 << 19) | Ka;
      if (mt > mh && mlast > K) {
        // (rare) an equal-count node with a smaller key is queued: insert
        int pos = mt;
        wave_lds_sync();
        while (pos > mh && S->qm[pos - 1] > K64) {
          if (lane == 0) S->qm[pos] = S->qm[pos - 1];
          wave_lds_sync();
          pos--;
        }
        if (lane == 0) S->qm[pos] = K64;
        wave_lds_sync();
        mw = mh;
        split(S->qm[mw + lane], wmk, wma);
        __builtin_amdgcn_s_waitcnt(0xC07F);
      } else {
        if (lane == 0) S->qm[mt] = K64;
        if (lane == mt - mw) {
          wmk = K;
          wma = Ka;
        }
        mlast = K;
      }
      mt++;
      root_label = 256 - (int)lab1;
      total = fs;
    }
    // the last partial row of records, then the tree from all of them
    {
      const int b0 = nsteps & ~63;
      if (b0 + lane < nsteps) S->rec[b0 + lane] = (int)rec;
    }
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int j = lane + 64 * i;
      if (j < nsteps) {
        const uint32_t r = (uint32_t)S->rec[j];
        const int c1 = (int)(r & 1023u), c2 = (int)((r >> 10) & 1023u), node = nl + j;
        S->par[c1] = node;
        S->par[c2] = node;
        S->off[c1] = 0;
        S->off[c2] = (int)(r >> 20);
      }
    }
  } else if (total_count >= (1u << 23)) {
    // the merges (encoder.c:196-226) on uniform values; v1 = the least key, v2
    // the next; K = the merged node, queued at its key's place
    // (keys as two 32-bit words -- freq, then label | leaves | node -- so the
    // uniform compares stay on the scalar unit)
    int lw = 0, mw = 0, lh = 0, mh = 0, mt = 0;
    uint32_t wlh, wll, wmh = ~0u, wml = ~0u;
    {
      const unsigned long long v = S->ql[lane];
      wlh = (uint32_t)(v >> 32);
      wll = (uint32_t)v;
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    uint32_t mlh = 0, mll = 0;  // the last appended key
    for (int step = 0; step + 1 < nl; step++) {
      // (window reloads wait for their loads inside the branch, so the common
      // path never waits for lane 0's queue and tree stores)
      if (lh + 1 - lw > 63) {
        lw = lh;
        const unsigned long long v = S->ql[lw + lane];
        wlh = (uint32_t)(v >> 32);
        wll = (uint32_t)v;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      }
      if (mh + 1 - mw > 63) {
        mw = mh;
        const unsigned long long v = S->qm[mw + lane];
        wmh = (uint32_t)(v >> 32);
        wml = (uint32_t)v;
        __builtin_amdgcn_s_waitcnt(0xC07F);
      }
      const int il = lh - lw, im = mh - mw;
      const uint32_t ah = __builtin_amdgcn_readlane(wlh, il), al = __builtin_amdgcn_readlane(wll, il);
      const uint32_t bh = __builtin_amdgcn_readlane(wlh, il + 1), bl = __builtin_amdgcn_readlane(wll, il + 1);
      const uint32_t ch = __builtin_amdgcn_readlane(wmh, im), cl0 = __builtin_amdgcn_readlane(wml, im);
      const uint32_t dh = __builtin_amdgcn_readlane(wmh, im + 1), dl = __builtin_amdgcn_readlane(wml, im + 1);
      const bool ac = ah < ch || (ah == ch && al < cl0);
      const uint32_t k1h = ac ? ah : ch, k1l = ac ? al : cl0;
      const uint32_t xh = ac ? bh : ah, xl = ac ? bl : al, yh = ac ? ch : dh, yl = ac ? cl0 : dl;
      const bool bx = xh < yh || (xh == yh && xl < yl);
      const uint32_t k2h = bx ? xh : yh, k2l = bx ? xl : yl;
      const int dlh = ac ? (bx ? 2 : 1) : (bx ? 1 : 0);
      lh += dlh;
      mh += 2 - dlh;
      const int lab1 = (int)(k1l >> 19);  // 256 - v1
      const uint32_t fs = k1h + k2h;
      const int sz1 = (int)((k1l >> 10) & 511), sz2 = (int)((k2l >> 10) & 511);
      const int c1 = (int)(k1l & 1023), c2 = (int)(k2l & 1023), node = nl + step;
      const uint32_t Kh = fs, Kl = ((uint32_t)lab1 << 19) | ((uint32_t)(sz1 + sz2) << 10) | (uint32_t)node;
      if (lane == 0) {
        S->par[c1] = node;
        S->par[c2] = node;
        S->off[c1] = 0;
        S->off[c2] = sz1;  // v2's chain follows v1's (:223-226)
      }
      const unsigned long long K = ((unsigned long long)Kh << 32) | Kl;
      if (mt > mh && (mlh > Kh || (mlh == Kh && mll > Kl))) {
        // (rare) an equal-count node with a smaller key is queued: insert
        int pos = mt;
        wave_lds_sync();
        while (pos > mh && S->qm[pos - 1] > K) {
          if (lane == 0) S->qm[pos] = S->qm[pos - 1];
          wave_lds_sync();
          pos--;
        }
        if (lane == 0) S->qm[pos] = K;
        wave_lds_sync();
        mw = mh;
        const unsigned long long v = S->qm[mw + lane];
        wmh = (uint32_t)(v >> 32);
        wml = (uint32_t)v;
        __builtin_amdgcn_s_waitcnt(0xC07F);
      } else {
        if (lane == 0) S->qm[mt] = K;
        if (lane == mt - mw) {
          wmh = Kh;
          wml = Kl;
        }
        mlh = Kh;
        mll = Kl;
      }
      mt++;
      root_label = 256 - lab1;
      total = fs;
    }
  }
  const int nn = 2 * nl - 1, root = nn - 1;
  if (lane == 0) {
    S->par[root] = 0xFFFF;
    S->off[root] = 0;
  }
  wave_lds_sync();
  TAB_T(3);
  // depth and chain place of every merged node (nodes nl..nn-1, parents among
  // them): pointer jumping to the root; then each leaf from its parent's
  {
    const int ni = nn - nl;  // merged nodes (<= 256)
    int pp[4], dd[4], oo[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int nd = nl + lane + 64 * i;
      pp[i] = 0xFFFF;
      dd[i] = 0;
      oo[i] = 0;
      if (64 * i < ni && nd < nn) {
        pp[i] = S->par[nd];
        oo[i] = S->off[nd];
        dd[i] = pp[i] != 0xFFFF;
        S->dep[nd] = dd[i];
      }
    }
    wave_lds_sync();
    for (int round = 0; round < 10; round++) {
      bool more = false;
#pragma unroll
      for (int i = 0; i < 4; i++) more |= pp[i] != 0xFFFF;
      if (!__ballot(more)) break;
      int nd2[4], no2[4], np2[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        nd2[i] = dd[i];
        no2[i] = oo[i];
        np2[i] = pp[i];
        if (64 * i < ni && pp[i] != 0xFFFF) {
          nd2[i] += S->dep[pp[i]];
          no2[i] += S->off[pp[i]];
          np2[i] = S->par[pp[i]];
        }
      }
      wave_lds_sync();
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int nd = nl + lane + 64 * i;
        dd[i] = nd2[i];
        oo[i] = no2[i];
        pp[i] = np2[i];
        if (64 * i < ni && nd < nn) {
          S->dep[nd] = dd[i];
          S->off[nd] = oo[i];
          S->par[nd] = pp[i];
        }
      }
      wave_lds_sync();
    }
    // leaves (nodes 0..nl-1): one edge to the parent plus the parent's path;
    // their symbols' lengths and chain places
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int q = lane + 64 * i;
      if (q < nl && nl > 1) {
        const int pq = S->par[q];
        const int d = 1 + S->dep[pq], o = S->off[q] + S->off[pq];
        const int sy = 256 - (int)((S->ql[q] >> 19) & 511);
        S->scl[sy] = d;
        S->spos[sy] = o;
        S->seq[o] = sy;
      }
    }
  }
  wave_lds_sync();
  TAB_T(4);
  int cl[5];
  int bad = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int s = lane + 64 * i;
    cl[i] = 0;
    if (s < 257) {
      cl[i] = S->scl[s];
      const bool in = cl[i] > 0;
      const int nx = in && S->spos[s] + 1 < nl ? S->seq[S->spos[s] + 1] : -1;
      hc->sym_freq[s] = in ? (s == root_label ? (int)total : 0) : (int)f[i];  // :221-222
      hc->code_len[s] = cl[i];
      hc->next[s] = nx;
      if (cl[i] >= 32) bad = 1;  // the reference indexes code_len_freq out of bounds
    }
  }
  if (__ballot(bad)) {
    if (lane == 0) *err = FERR_TABLE;
    return;
  }
  // code_len_freq (all 257 symbols) and counts of 0..255, length L in lane L;
  // the nl leaves (nl - 1 of them symbols 0..255) are all counted by the
  // longest length
  // (by LDS atomics into the merge records' words, free by now: a ballot
  // per length and register cost ~20 instructions per length)
  const int nlc = nl > 1 ? nl : 0;
  if (lane < 32) S->rec[lane] = 0;
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < 5; i++)
    if (cl[i] > 0 && (i < 4 || lane == 0)) atomicAdd(&S->rec[cl[i]], 1);
  wave_lds_sync();
  int clf = lane < 32 ? S->rec[lane] : 0;
  const int l256 = __builtin_amdgcn_readfirstlane(cl[4]);  // symbol 256's length (lane 0)
  const int cnt = clf - (l256 > 0 && lane == l256 ? 1 : 0);  // symbols 0..255
  const unsigned long long lens = __ballot(clf > 0);
  const int maxl = lens ? 63 - __clzll(lens) : 0;
  bool fail = nlc < 2;
  if (!fail) {
    // :239-259 limit to 16 bits (the lengths above the longest are empty:
    // the walk down from 31 starts there)
    int i = max(maxl, 17);
    for (int guard = 0; guard < 4096; guard++) {
      if (__builtin_amdgcn_readlane(clf, i) > 0) {
        const unsigned long long m = __ballot(clf > 0) & ((1ull << (i - 1)) - 1ull);
        if (!m) {
          fail = true;
          break;
        }
        const int j = 63 - __clzll(m);
        clf += (lane == i ? -2 : 0) + (lane == i - 1 ? 1 : 0) + (lane == j + 1 ? 2 : 0) + (lane == j ? -1 : 0);
        continue;
      }
      i--;
      if (i != 16) continue;
      const unsigned long long m = __ballot(clf != 0) & ((1ull << 17) - 1ull);
      i = 63 - __clzll(m);
      clf -= lane == i ? 1 : 0;
      break;
    }
  }
  const int cum = (int)wave_scan64((uint32_t)(lane <= 16 ? clf : 0));
  const int basev = (int)wave_scan64((uint32_t)cnt) - cnt;
  const int n = nlc ? nlc - 1 : 0;  // symbols 0..255 with a code
  if (!fail && (__builtin_amdgcn_readlane(cum, 16) != n || n >= 255)) fail = true;
  if (fail) {
    if (lane == 0) *err = FERR_TABLE;
    return;
  }
  // :280-300 canonical first codes, length L in lane L
  int fc = 0;
  {
    int code = 0, started = 0;
    for (int L = 1; L <= 16; L++) {
      if (started) code <<= 1;
      if (lane == L) fc = code;
      const int cL = __builtin_amdgcn_readlane(clf, L);
      if (cL) started = 1;
      code += cL;
    }
  }
  TAB_T(5);
  // :262-268 order symbols 0..255 by (unlimited length, value)
  {
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int L = 1; L <= maxl; L++) {
      int at = __builtin_amdgcn_readlane(basev, L);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const unsigned long long m = __ballot(cl[r] == L);
        if (cl[r] == L) S->sorted[at + __popcll(m & lt)] = lane + 64 * r;
        at += __popcll(m);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    S->slen[lane + 64 * r] = 0;
    S->scode[lane + 64 * r] = -1;
  }
  wave_lds_sync();
  TAB_T(6);
#pragma unroll
  for (int r = 0; r < 4; r++) {  // :271-276 and :280-300
    const int kk = lane + 64 * r;
    int L = 1;
    for (int l = 1; l <= 16; l++) L += __builtin_amdgcn_readlane(cum, l) <= kk ? 1 : 0;
    L = min(L, 16);
    // (lane reads with every lane active: an inactive source lane reads 0)
    const int code = __shfl(fc, L) + (kk - __shfl(cum, L - 1));
    if (kk < n) {
      const int sy = S->sorted[kk];
      S->slen[sy] = L;
      S->scode[sy] = code;
    }
  }
  wave_lds_sync();
  if (lane < 32) hc->code_len_freq[lane] = clf;
  for (int kk = lane; kk < 256; kk += 64) {
    // sym_sorted: -1 past the end, except that the sentinel write of :277
    // lands in sym_sorted[255] (it aliases sym_code_len[-1], structs.h:10-11)
    hc->sym_sorted[kk] = kk < n ? S->sorted[kk] : (kk == 255 ? 0 : -1);
    const int L = S->slen[kk];
    hc->sym_code_len[kk] = L;
    hc->sym_code[kk] = S->scode[kk];
    ehuf[kk] = L ? ((uint32_t)L << 16) | (uint32_t)S->scode[kk] : 0u;
  }
  TAB_T(7);
}

// With a.seg_dc the DC-table waves (0, 2) first compute the segments' first
// DC tokens and class counts (k_seg_dc's step; half of the frame's segments
// each, 32 segments in flight per lane) while the AC-table waves, the long
// pole (~160 symbols to merge against <= 12), already build theirs.
__global__ __launch_bounds__(256) void k_tables(EntArgs a) {
  __shared__ TabScratch2 S[4];
  __shared__ uint32_t h[2][16];
  __shared__ uint32_t hs[32 * 32];  // seg_dc_store's spread counters
  __shared__ int s_done;
  const int f = blockIdx.x, t = threadIdx.x >> 6, lane = threadIdx.x & 63;
#ifdef MIJ_K1_DIAG
  if (a.dbg && lane == 0) a.dbg[((long long)f * 4 + t) * 10 + 8] = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t *extra = nullptr;
  if (a.seg_dc) {
    for (int i = threadIdx.x; i < 32 * 32; i += 256) hs[i] = 0;
    if (threadIdx.x == 0) s_done = 0;
  }
  __syncthreads();
  if (a.seg_dc && !(t & 1)) {
    const FGeom fg = frame_geom(a.g, a.fdims, f);
    const int half = (a.g.nseg + 1) / 2;
    const int sb = t == 0 ? 0 : half, se = t == 0 ? half : a.g.nseg;
    constexpr int U = SEGDC_U;  // segments in flight per lane
    for (int s0 = sb + lane; s0 < se; s0 += 64 * U) {
      SegDc r[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int s = s0 + 64 * u;
        r[u] = s < se ? seg_dc_load(a, fg, f, s) : SegDc{0, 0, 0, false};
      }
#pragma unroll
      for (int u = 0; u < U; u++) seg_dc_store(a, f, s0 + 64 * u, r[u], hs, lane);
    }
#ifdef MIJ_K1_DIAG
    if (a.dbg && lane == 0) a.dbg[((long long)f * 4 + t) * 10 + 9] = __builtin_amdgcn_s_memtime();
#endif
    // both DC waves' counts are in before either builds its table
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) atomicAdd(&s_done, 1);
    // (the other DC wave of this workgroup; bounded like every device wait)
    const unsigned long long t_wait = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&s_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 2) {
      if (__builtin_amdgcn_s_memrealtime() - t_wait > SPIN_TICKS) {
        if (lane == 0) a.err[f] = FERR_SPIN;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // this wave's component: the 32 copies of its 16 counters summed
    if (lane < 16) {
      const int key = (t >> 1) * 16 + lane;
      uint32_t v = 0;
      for (int c = 0; c < 32; c++) v += hs[key * 32 + ((c + lane) & 31)];
      h[t >> 1][lane] = v;
    }
    wave_lds_sync();
    extra = h[t >> 1];
  }
  build_table_wave2(a.hist + ((long long)f * 4 + t) * 257, extra, (HuffCode *)a.hc + (long long)f * 4 + t,
                   (uint32_t *)a.ehuf + ((long long)f * 4 + t) * 256, &S[t], lane, a.err + f,
                   a.dbg ? a.dbg + ((long long)f * 4 + t) * 10 : nullptr);
}

// The same tables one wave (workgroup) per table when the segment DCs ran on
// their own (k_seg_dc): 14 KB of LDS per workgroup instead of 61 KB, so the
// tables of one sub-batch fit beside the next sub-batch's K1 (overlap path).
// (EntArgs::tab_dc_only: the two DC tables of each frame only, k_segdc_actab
// built the AC tables)
__global__ __launch_bounds__(64) void k_tables_1w(EntArgs a) {
  __shared__ TabScratch2 S;
  const int nt = a.tab_dc_only ? 2 : 4, lane = threadIdx.x;
  const int f = blockIdx.x / nt, idx = blockIdx.x - f * nt, t = a.tab_dc_only ? 2 * idx : idx;
  if (a.zero_pack) {  // (k_pack_flat runs next: its state, zeroed here instead of two fills)
    const long long st = pack_stride(a.g);
    for (long long i = 64 * idx + lane; i < st; i += 64 * nt) a.pack_state[f * st + i] = 0;
    if (t == 0 && lane < 3) a.pack_ticket[f * 3 + lane] = 0;
  }
#ifdef MIJ_K1_DIAG
  if (a.dbg && lane == 0) a.dbg[((long long)f * 4 + t) * 10 + 8] = __builtin_amdgcn_s_memtime();
#endif
  build_table_wave2(a.hist + ((long long)f * 4 + t) * 257, nullptr, (HuffCode *)a.hc + (long long)f * 4 + t,
                    (uint32_t *)a.ehuf + ((long long)f * 4 + t) * 256, &S, lane, a.err + f,
                    a.dbg ? a.dbg + ((long long)f * 4 + t) * 10 : nullptr);
  if (a.zero_pack)  // the counts are read: left zeroed for the next K1 (no fill before it)
    for (int i = lane; i < 257; i += 64) a.hist[((long long)f * 4 + t) * 257 + i] = 0;
}

// The segment-first DCs (k_seg_dc) and, in the first 2 x nframes
// workgroups, the frames' two AC tables, which do not depend on them: the
// luma AC table's merge (the long pole of the table stage) runs beside the
// segment DCs, and k_tables_1w builds only the DC tables after
// (EntArgs::tab_dc_only).  One wave of an AC workgroup works.
// DC_LAST (EntArgs::dc_last, small batches): the segment-DC workgroups
// count their classes into dcx and the last of a frame's to arrive builds
// the frame's two DC tables, two waves at once, while the AC tables' waves
// are still merging; its other two waves zero the frame's pack state -- so
// the table stage is one launch whose length is the luma AC table's.  (Not
// on large batches: a frame's DC tables then wait for its own segment DCs,
// dispatched frame after frame, where k_tables_1w builds all of them at once
// after the launch; config 3: 0.052 -> 0.10 ms.)
template <bool DC_LAST>
__global__ __launch_bounds__(SEGDC_WG) void k_segdc_actab(EntArgs a) {
  __shared__ TabScratch2 S[DC_LAST ? 2 : 1];
  __shared__ uint32_t hs[32 * 32];
  __shared__ uint32_t s_x[32];
  __shared__ int s_last;
  const int nac = 2 * a.nframes;
  if ((int)blockIdx.x >= nac) {
    const int b = (int)blockIdx.x - nac;
    seg_dc_block(a, b, hs);
    if (!DC_LAST) return;
    const int per = (a.g.nseg + SEGDC_WG - 1) / SEGDC_WG, f = b / per;
    uint32_t *dcx = a.dcx + (long long)f * 64;
    // Arrival after the block's counts are performed (seg_dc_block waited for
    // its returning adds); the last arrival's own atomics then find every
    // count (a device-scope fence here -- an L2 writeback per block -- cost
    // 1.6 ms per config-3 launch)
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&dcx[32], 1u) == (unsigned)(per - 1);
    __syncthreads();
    if (!s_last) return;
    // the counts read and reset by one atomic each (left zeroed for the next launch)
    if (threadIdx.x < 33) {
      const uint32_t v = atomicExch(&dcx[threadIdx.x], 0u);
      if (threadIdx.x < 32) s_x[threadIdx.x] = v;
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < 2) {
      const int t = 2 * w;  // luma DC, chroma DC
      build_table_wave2(a.hist + ((long long)f * 4 + t) * 257, &s_x[16 * w], (HuffCode *)a.hc + (long long)f * 4 + t,
                        (uint32_t *)a.ehuf + ((long long)f * 4 + t) * 256, &S[DC_LAST ? w : 0], lane, a.err + f,
                        nullptr);
      if (a.zero_pack)  // the counts are read: left zeroed for the next K1
        for (int i = lane; i < 257; i += 64) a.hist[((long long)f * 4 + t) * 257 + i] = 0;
    } else if (a.zero_pack) {  // k_pack_flat runs next: its look-back words and tickets zeroed
      const long long st = pack_stride(a.g);
      for (long long i = threadIdx.x - 128; i < st; i += 128) a.pack_state[f * st + i] = 0;
      if (threadIdx.x - 128 < 3) a.pack_ticket[f * 3 + threadIdx.x - 128] = 0;
    }
    return;
  }
  if (threadIdx.x >= 64) return;
  const int f = blockIdx.x >> 1, t = 1 + 2 * (blockIdx.x & 1), lane = threadIdx.x;
  build_table_wave2(a.hist + ((long long)f * 4 + t) * 257, nullptr, (HuffCode *)a.hc + (long long)f * 4 + t,
                    (uint32_t *)a.ehuf + ((long long)f * 4 + t) * 256, &S[0], lane, a.err + f, nullptr);
  if (a.zero_pack)  // the counts are read: left zeroed for the next K1
    for (int i = lane; i < 257; i += 64) a.hist[((long long)f * 4 + t) * 257 + i] = 0;
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
// k_seg_bits: bits of every segment with the frame's tables.  One wave per
// segment, lanes over its tokens; a workgroup covers SEG_PER_WG segments of
// one frame.
// ===========================================================================
__device__ __forceinline__ uint32_t tok_bits(uint32_t tk, const uint32_t (*tab)[256], int chroma) {
  const int t = (chroma ? 2 : 0) + ((tk & TOK_AC) ? 1 : 0);
  const uint32_t sym = tk & 255u;
  return (tab[t][sym] >> 16) + (sym & 15u) + ((tk >> 8) & 3u) * (tab[t][0xF0] >> 16);
}

__global__ __launch_bounds__(256) void k_seg_bits(EntArgs a) {
  __shared__ uint32_t tab[4][256];
  const int per = (a.g.nseg + SEG_PER_WG - 1) / SEG_PER_WG;
  const int f = blockIdx.x / per;
  const int s0 = (blockIdx.x - f * per) * SEG_PER_WG;
  for (int i = threadIdx.x; i < 1024; i += 256) tab[i >> 8][i & 255] = a.ehuf[(long long)f * 1024 + i];
  __syncthreads();
  // 16 lanes per segment, 16 segments in flight per workgroup
  const int sub = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int send = min(s0 + SEG_PER_WG, a.g.nseg);
  for (int s = s0 + grp; s < send; s += 16) {
    const long long fs = (long long)f * a.g.nseg + s;
    const int n = min((int)a.seg_ntok[fs], SEG_TOK);
    const uint32_t *tk = a.tok + fs * SEG_TOK;
    const uint32_t tz = a.tok0[fs];  // token 0
    const int chroma = s >= a.g.nsy;
    uint32_t b = 0;
    // four loads in flight per lane before any is used (latency-bound loop)
    for (int i0 = 0; i0 < n; i0 += 64) {
      uint32_t t[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int i = i0 + 16 * u + sub;
        t[u] = i < n ? (i ? tk[i] : tz) : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (i0 + 16 * u + sub < n) b += tok_bits(t[u], tab, chroma);
    }
    b = row_scan16(b);
    if (sub == 15) a.seg_bits[fs] = b;
  }
}

// ===========================================================================
// k_scan: per scan (frame, component) exclusive scan of segment bits; zeroes
// the first/last word of every pack group (shared with neighbour groups and
// OR-combined by the band packing).  One wave per scan.
// ===========================================================================
__global__ void k_scan(EntArgs a) {
  const int sid = blockIdx.x;  // frame * 3 + comp
  const int f = sid / 3, comp = sid - f * 3;
  const int lane = threadIdx.x;
  const int sbase = comp == 0 ? 0 : a.g.nsy + (comp - 1) * a.g.nsc;
  const int ns = comp == 0 ? a.g.nsy : a.g.nsc;
  const long long f0 = (long long)f * a.g.nseg + sbase;
  uint32_t *raw = a.raw + (long long)f * a.g.raw_fs +
                  (comp == 0 ? 0 : a.g.raw_words[0] + (comp == 2 ? a.g.raw_words[1] : 0));
  unsigned long long carry = a.bit_base ? a.bit_base[f * 4 + comp] : 0u;  // band: start bit in word 0
  for (int base = 0; base < ns; base += 64) {
    const int i = base + lane;
    const unsigned long long v = i < ns ? a.seg_bits[f0 + i] : 0ull;
    unsigned long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    const unsigned long long excl = carry + x - v;
    if (i < ns) {
      a.seg_off[f0 + i] = excl;
      // (bits past the scan buffer: tokens that no K1 wrote -- flag the frame,
      // never write out of bounds)
      const unsigned long long wl = excl >> 5, wh = (excl + v - 1) >> 5;
      if (wh >= (unsigned long long)a.g.raw_words[comp]) {
        a.err[f] = FERR_OVERFLOW;
      } else {
        const int gsz = PACK_SEGS << a.pack_ls[comp != 0];  // (the pack groups' first / last words)
        if (i % gsz == 0) raw[wl] = 0;
        if (i % gsz == gsz - 1 || i == ns - 1) raw[wh] = 0;
      }
    }
    carry += __shfl(x, 63);
  }
  if (lane == 0) a.scan_bits[sid] = carry;
}

// ===========================================================================
// Bit placement helpers of k_pack_flat's token-by-token and window paths
// (big-endian bit order).
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

// the part of a piece that falls inside the LDS window [lo_bit, hi_bit)
__device__ __forceinline__ void put_bits_window(uint32_t *buf, uint32_t pos, uint32_t lo_bit,
                                                uint32_t hi_bit, uint32_t val, int len) {
  const uint32_t w = pos >> 5, wl = lo_bit >> 5, wh = hi_bit >> 5;
  const int sh = 32 - (int)(pos & 31) - len;
  if (sh >= 0) {
    if (w >= wl && w < wh) atomicOr(&buf[w - wl], val << sh);
  } else {
    if (w >= wl && w < wh) atomicOr(&buf[w - wl], val >> (-sh));
    if (w + 1 >= wl && w + 1 < wh) atomicOr(&buf[w + 1 - wl], val << (32 + sh));
  }
}

// Pack groups' look-back words (EntArgs::pack_state, one per group of
// 32 << pack_ls segments of one scan): flag << 62 | bits, flag 1 = the group's
// own bit count (aggregate), 2 = the inclusive prefix of its scan.
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1;

// The packing's code table: per [DC | AC][symbol] the Huffman code already
// shifted left by the symbol's magnitude bit count (cls = symbol & 15,
// encoder.c:434-460) in bits 0-26 and the total length code length + cls in
// bits 27-31 (<= 16 + 11 = 27 bits: magnitudes stop at class 11 after
// encoder.c:109's clip), so a token's code is one table read and one OR;
// symbols without a code read 0.  A token slot past the end of its segment
// is LB_NOTOK (K1 pads every segment to a multiple of 4 tokens with it),
// whose entry is 0: no bits, no ZRLs, nothing to mask in its decode.
constexpr uint32_t LB_CODE = (1u << 27) - 1u;
__device__ __forceinline__ uint32_t lb_tab_entry(uint32_t e, uint32_t sym) {
  const uint32_t cls = sym & 15u;
  return e ? ((e & 0xFFFFu) << cls) | (((e >> 16) + cls) << 27) : 0u;
}
// bits of a token (encoder.c:434-460, ZRLs :490-494 apart): code (with the
// magnitude bits) into `code`, its length returned
__device__ __forceinline__ uint32_t lb_tok_code(const uint32_t *tab, uint32_t t, uint32_t &code) {
  const uint32_t e = tab[((t >> 2) & 256u) | (t & 255u)];  // TOK_AC (bit 10) selects the AC table
  code = (e & LB_CODE) | (t >> 16);
  return e >> 27;
}
// its length alone
__device__ __forceinline__ uint32_t lb_tok_len(const uint32_t *tab, uint32_t t) {
  return tab[((t >> 2) & 256u) | (t & 255u)] >> 27;
}

// OR `len` (1..64) bits, left-aligned in v, into the big-endian word buffer at
// bit pos (pos + len within the buffer)
__device__ __forceinline__ void put_bits64(uint32_t *buf, uint32_t pos, unsigned long long v, uint32_t len) {
  const uint32_t w = pos >> 5, off = pos & 31u;
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  atomicOr(&buf[w], hi >> off);
  if (off + len > 32) atomicOr(&buf[w + 1], __builtin_amdgcn_alignbit(hi, lo, off));
  if (off + len > 64) atomicOr(&buf[w + 2], __builtin_amdgcn_alignbit(lo, 0u, off));
}

// put_bits64 into the window [lo_bit, hi_bit) of the group's bits only
// (buf holds the window's words)
__device__ __forceinline__ void put_bits64_win(uint32_t *buf, uint32_t pos, unsigned long long v, uint32_t len,
                                               uint32_t lo_bit, uint32_t hi_bit) {
  if (pos + len <= lo_bit || pos >= hi_bit) return;
  const uint32_t w = pos >> 5, off = pos & 31u, wl = lo_bit >> 5, wh = hi_bit >> 5;
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  if (w >= wl && w < wh) atomicOr(&buf[w - wl], hi >> off);
  if (off + len > 32 && w + 1 >= wl && w + 1 < wh) atomicOr(&buf[w + 1 - wl], __builtin_amdgcn_alignbit(hi, lo, off));
  if (off + len > 64 && w + 2 >= wl && w + 2 < wh) atomicOr(&buf[w + 2 - wl], __builtin_amdgcn_alignbit(lo, 0u, off));
}

// 0xFF bytes among the first `lim` (0..4) bytes of a big-endian stream word
__device__ __forceinline__ int ff_bytes(uint32_t w, int lim) {
  const uint32_t x = ~w;
  const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 per zero byte of x
  const uint32_t keep = lim >= 4 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (8 * lim));
  return __popc(t & keep);
}

// ff_pack: the 0xFF bytes of stream word W (bytes past the scan's whole bytes
// nb do not count: the pad byte is written apart, never stuffed)
__device__ __forceinline__ int ff_word(uint32_t v, uint32_t W, uint32_t nb) {
  const uint32_t b = 4 * W;
  return b >= nb ? 0 : ff_bytes(v, (int)min(nb - b, 4u));
}
constexpr int EMIT_CW = EMIT_CH / 4;  // stream words per emit chunk


// ===========================================================================
// k_pack_flat: segment bits, scan offsets and bit packing in one pass
// (encoder.c:434-502).  Each workgroup takes the next pack group of 32 << ls
// segments of one scan (a per-scan ticket keeps groups claimed in scan order,
// so a look-back only waits on groups that have started).  A pack group's
// bitstream is its segments' token strings back to back, and K1 pads every
// segment to a multiple of 4 tokens (LB_NOTOK, no bits), so the group is a
// list of 4-token chunks, each inside one segment slot and 16-byte aligned.
// Every thread takes K consecutive chunks per round (the first's segment by binary
// search of the chunk counts' prefix), merges each chunk's 4 tokens into one
// bit string, and a workgroup scan of the string lengths places them in the
// LDS window relative to the group's first bit -- every token is read and
// decoded once, and no lane idles on a short segment.  The next round's
// chunks are loaded while a round is placed.  The group's aggregate goes out
// as soon as the last round's scan has it; then the decoupled look-back over
// the groups before it finds its start bit (by then they have usually
// published; the wait is bounded, MIJ_SPIN_LIMIT) and the window is stored
// shifted into place.  A group whose bits outgrow the window (near
// worst-case entropy) takes its start bit and sweeps its chunks again once
// per window, at absolute offsets.
//
// Seam mode (EntArgs::seam, the frame encodes): a group stores every word it
// reaches the end of plainly; its first word, when the group before it ends
// inside that word, goes to seam[] for k_seam_fix -- the scan buffers may
// hold anything when the kernel starts, and no word is written twice (A/B,
// config 3: 0.72 ms against 0.80 for the OR-onto-zero form, which the band
// paths keep: there the buffers are all-zero on entry and a group ORs its
// first and last word, which it may share with a neighbour).
//
// Tuning (profiles/r04): 2 chunks per thread per round at 8
// workgroups per CU (1 chunk: 0.65-0.69 ms, 3 chunks at occupancy 7:
// 1.51-1.57); the wide window (PACK_WIDE_WORDS, high quality) runs 6
// workgroups per CU by its LDS.
// ===========================================================================
constexpr int PF_THREADS = 256, PF_WAVES = PF_THREADS / 64;
constexpr int PF_K = 2, PF_OCC = 8, PF_OCC_WIDE = 6;
// Round 6: a thread's chunks of a round are consecutive in the stream (chunks
// K tid .. K tid + K - 1 of the round), so one segment search and one wave
// scan serve all K of them (round 5: chunks tid + 256 k, a search and a scan
// each).  PF_K_WIDE: chunks per thread for the wide window (high quality),
// whose LDS holds it at 6 workgroups per CU; measured at Q=90 (one box,
// three rounds): 2 chunks 1.238-1.244 ms, 3 chunks 1.265-1.267 (no spills,
// fewer rounds per group, but longer rounds), 4 chunks spill 13 VGPRs.
#ifndef PF_K_WIDE
#define PF_K_WIDE 2
#endif
template <int PW>
constexpr int pf_k() { return PW > PACK_WORDS ? PF_K_WIDE : PF_K; }
template <int PW>
constexpr int pf_occ() { return PW > PACK_WORDS ? PF_OCC_WIDE : PF_OCC; }
static_assert(PACK_SEGS_MAX == PF_THREADS, "k_pack_flat: a thread per segment of the widest group");
template <int PW, bool FF>
__global__ __launch_bounds__(PF_THREADS, pf_occ<PW>()) void k_pack_flat(EntArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[PW];
  __shared__ uint32_t tab[2 * 256];
  __shared__ uint32_t s_cp[PACK_SEGS_MAX + 1];  // exclusive prefix of the segments' chunks; [MAX]: all
  __shared__ uint32_t s_wt[PF_WAVES];
  // the first pass's bit offset at every round start (the windowed path
  // starts a window's sweep at the round it begins in), and the first bit it
  // could not place
  constexpr int K = pf_k<PW>();  // chunks per thread and round
  constexpr int PF_ROUNDS = (PACK_SEGS_MAX * (SEG_TOK / 4) + K * PF_THREADS - 1) / (K * PF_THREADS);
  __shared__ uint32_t s_run[PF_ROUNDS + 1];
  __shared__ uint32_t s_p1;
  __shared__ uint32_t s_ws[2][PF_WAVES];  // a round's bits per wave (two rounds in turn)
  __shared__ unsigned long long s_prefix;
  __shared__ int s_ticket;
  __shared__ uint32_t s_over;
  __shared__ bool s_hung;
  constexpr int FFN = PW / EMIT_CW + 2;
  __shared__ uint32_t s_ff[FFN];
  __shared__ uint32_t s_ffnb;
#ifdef MIJ_K1_DIAG
  // per-group phase stamps (MIJ_PACK_TIME): start, chunk counts ready, sweep
  // done, look-back done, end; [5] ticket and code table in
  unsigned long long pst[6];
  pst[0] = __builtin_amdgcn_s_memrealtime();
#define PF_STAMP(k) pst[k] = __builtin_amdgcn_s_memrealtime()
#else
#define PF_STAMP(k)
#endif
  const Geom &G = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (FF && tid < FFN) s_ff[tid] = 0;
  if (tid == 0) {
    s_over = 0;
    s_hung = false;
    s_p1 = ~0u;
    s_run[0] = 0;
  }
  const PackGrid P = pack_grid(a);
  const int gy = P.gy, gc = P.gc, gpf = P.gpf;
  // the scan from the workgroup's index, the group inside it from the scan's
  // ticket (groups claimed in scan order)
  const int f = blockIdx.x / gpf, bq = blockIdx.x - f * gpf;
  const int comp = bq < gy ? 0 : (bq < gy + gc ? 1 : 2);
  const int sbase = comp == 0 ? 0 : (comp == 1 ? G.nsy : G.nsy + G.nsc), ns = comp == 0 ? G.nsy : G.nsc;
  const int gscan0 = f * P.stride + (comp == 0 ? 0 : gy + (comp == 2 ? gc : 0));
  const int pseg = PACK_SEGS << a.pack_ls[comp != 0];  // the group's segments (32 to 256)
  const int nq = comp == 0 ? gy : gc;
  // Every load of the prologue goes out before the ticket's atomic, so one
  // memory latency covers them all (in program order each waited for the
  // one before): the code table, the ZRL code, and the group's segment
  // counts for the group this workgroup's dispatch place names -- the scan's
  // groups are dispatched in order, so the ticket usually equals it, and
  // otherwise the counts are loaded again after it.
  const int chroma = comp != 0;
  const uint32_t *eh = a.ehuf + (long long)f * 1024 + (chroma ? 512 : 0);
  static_assert(2 * PF_THREADS == 512, "k_pack_flat: two code-table entries per thread");
  const uint32_t e0 = eh[tid], e1 = eh[256 + tid], zac = eh[256 + 0xF0];
  const int qg = bq - (comp == 0 ? 0 : (comp == 1 ? gy : gy + gc));
  auto seg_count = [&](int qq) -> uint32_t {
    const int s0q = qq * pseg, nsq = min(ns, s0q + pseg) - s0q;
    return tid < nsq ? a.seg_ntok[(long long)f * G.nseg + sbase + s0q + tid] : 0u;
  };
  const uint32_t nt_guess = seg_count(qg);
  if (tid == 0) s_ticket = (int)atomicAdd(&a.pack_ticket[f * 3 + comp], 1u);
  tab[tid] = lb_tab_entry(e0, (uint32_t)tid);
  tab[256 + tid] = lb_tab_entry(e1, (uint32_t)tid);
  // the ZRL code (AC symbol 0xF0: cls 0, so the entry is code / length)
  const uint32_t Lz = zac >> 16, zcode = zac & 0xFFFFu;
  __syncthreads();
  PF_STAMP(5);
  const int q = s_ticket;
  // a ticket past the scan's groups (the ticket word was not reset, or was
  // overwritten): nothing of it belongs to this launch -- flag the frame and
  // leave the other scans' look-back words alone
  if (q < 0 || q >= nq) {
    if (tid == 0) a.err[f] = FERR_SPIN;
    return;
  }
  const int gid = gscan0 + q;
  const int s0 = q * pseg, nsg = min(ns, s0 + pseg) - s0;
  const long long fs0 = (long long)f * G.nseg + sbase + s0;  // the group's first segment
  {  // chunks per segment (K1 padded each to a multiple of 4 tokens), a thread per segment
    const uint32_t nt = min(q == qg ? nt_guess : seg_count(q), (uint32_t)SEG_TOK);
    const uint32_t ch = (nt + 3u) >> 2;
    const uint32_t incl = wave_scan64(ch);
    if (lane == 63) s_wt[wave] = incl;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < PF_WAVES; w++) {
      const uint32_t v = s_wt[w];
      tot += v;
      before += w < wave ? v : 0u;
    }
    s_cp[tid] = tid < nsg ? before + incl - ch : 0xFFFFFFFFu;  // (no chunk maps past the group)
    if (tid == 0) s_cp[PACK_SEGS_MAX] = tot;
  }
  __syncthreads();
  const uint32_t C = s_cp[PACK_SEGS_MAX];
  PF_STAMP(1);
  // The window is zeroed as far as the group can need it at <= 96 bits per
  // chunk (3C + 2 words: a chroma group of ~256 chunks zeroes ~770 words, not
  // the whole window; config-3 luma groups run ~20 bits per chunk at Q=50,
  // ~70 at Q=90); a chunk that would place past it takes the
  // window-by-window path, which zeroes its own windows.  16-byte stores;
  // the sweep's first barrier orders them before any placement.
  const uint32_t wz = min((uint32_t)PW, (3u * C + 2u + 3u) & ~3u);
  for (uint32_t i = 4u * tid; i < wz; i += 4u * PF_THREADS) *(u4v *)&buf[i] = u4v{0u, 0u, 0u, 0u};
  const uint32_t *tokg = a.tok + fs0 * SEG_TOK;
  // chunk c's 4 tokens (c < C): its segment s is the last with s_cp[s] <= c
  auto chunk_seg = [&](uint32_t c) -> int {
    int s = 0;
#pragma unroll
    for (int step = PACK_SEGS_MAX / 2; step; step >>= 1)  // (entries past the group read ~0)
      if (s_cp[s + step] <= c) s += step;
    return s;
  };
  auto chunk_at = [&](uint32_t c, int s, u4v &t) {
    const uint32_t o = 4u * (c - s_cp[s]);
    t = *(const u4v *)(tokg + (long long)s * SEG_TOK + o);
    if (o == 0) t[0] = a.tok0[fs0 + s];  // token 0 of a segment (dense array)
  };
  auto chunk_load = [&](uint32_t c, u4v &t) {
    t = u4v{0u, 0u, 0u, 0u};
    if (c >= C) return;
    chunk_at(c, chunk_seg(c), t);
  };
  // a thread's K chunks of a round are consecutive (c .. c + K - 1): one
  // search for the first, and each next chunk's segment is the one before or
  // a later one (later than the next only past empty segments: region batches)
  auto run_load = [&](uint32_t c, u4v (&t)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) t[k] = u4v{0u, 0u, 0u, 0u};
    if (c >= C) return;
    int s = chunk_seg(c);
    chunk_at(c, s, t[0]);
#pragma unroll
    for (int k = 1; k < K; k++) {
      if (c + k >= C) break;
      while (s_cp[s + 1] <= c + k) s++;
      chunk_at(c + k, s, t[k]);
    }
  };
  // a chunk's bits: per token the code (magnitude bits included) and its
  // ZRLs (encoder.c:490-494); merged into one left-growing string when they
  // fit 64 bits
  auto decode = [&](const u4v &t, uint32_t (&L)[4], uint32_t (&code)[4], uint32_t (&nzr)[4]) -> uint32_t {
    uint32_t nb = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      L[e] = lb_tok_code(tab, t[e], code[e]);
      nzr[e] = (t[e] >> 8) & 3u;
      nb += L[e] + nzr[e] * Lz;
    }
    return nb;
  };
  // one sweep over the group's chunks: positions relative to the group's
  // first bit (+ boff); whole: every bit into the window (a chunk past it
  // sets the overflow flag and is left out), else only the bits inside
  // [lo_bit, hi_bit), from the round that window starts in to the round that
  // passes its end.  A round takes K chunks per thread (chunks c0 + K tid +
  // k), all loaded at once, and needs one barrier; with `publish` the
  // group's aggregate goes out as soon as the last round's scan has it,
  // before that round is placed.
  // chunk k of this thread in a round, relative to the round's first chunk
  auto chunk_of = [&](int k) -> uint32_t { return (uint32_t)(K * tid + k); };
  auto sweep = [&](bool whole, uint32_t boff, uint32_t lo_bit, uint32_t hi_bit, bool publish) -> uint32_t {
    const uint32_t lim = (wz - 1) * 32;  // the zeroed words, one spare for the shifted store
    uint32_t r0 = 0;
    if (!whole) {  // the last round starting at or before lo_bit (s_run from the whole pass)
      const uint32_t nr = (C + K * PF_THREADS - 1) / (K * PF_THREADS);
#pragma unroll
      for (uint32_t step = 128; step; step >>= 1)
        if (r0 + step < nr && boff + s_run[r0 + step] <= lo_bit) r0 += step;
    }
    uint32_t run = boff + s_run[r0];
    bool over = false;
    u4v tn[K];  // the next round's chunks, loaded while a round is placed
    run_load(r0 * K * PF_THREADS + chunk_of(0), tn);
    for (uint32_t c0 = r0 * K * PF_THREADS, r = r0; c0 < C && (whole || run < hi_bit);
         c0 += K * PF_THREADS, r++) {
      u4v t[K];
#pragma unroll
      for (int k = 0; k < K; k++) t[k] = tn[k];
      if (c0 + K * PF_THREADS < C) run_load(c0 + K * PF_THREADS + chunk_of(0), tn);
      uint32_t nb[K], tot_t = 0;
      unsigned long long acc[K];
#pragma unroll
      for (int k = 0; k < K; k++) {
        uint32_t L[4], code[4], nzr[4];
        nb[k] = decode(t[k], L, code, nzr);  // (a chunk past the group: zero tokens, no bits)
        if (c0 + chunk_of(k) >= C) nb[k] = 0;
        acc[k] = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
          for (uint32_t z = nzr[e]; z; z--) acc[k] = (acc[k] << Lz) | zcode;
          acc[k] = (acc[k] << L[e]) | code[e];
        }
        tot_t += nb[k];
      }
      // one scan of the thread's bits: its K chunks are consecutive in the stream
      const uint32_t x = wave_scan64(tot_t);
      if (lane == 63) s_ws[r & 1][wave] = x;
      __syncthreads();
      uint32_t pos[K];
      {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < PF_WAVES; w++) {
          const uint32_t v = s_ws[r & 1][w];
          tot += v;
          before += w < wave ? v : 0u;
        }
        pos[0] = run + before + x - tot_t;
#pragma unroll
        for (int k = 1; k < K; k++) pos[k] = pos[k - 1] + nb[k - 1];
        run += tot;
      }
      if (publish && c0 + K * PF_THREADS >= C && tid == 0 && q > 0)
        __hip_atomic_store(&a.pack_state[gid], LB_AGG | (run - boff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (whole && tid == 0) s_run[r + 1] = run;  // (read after the look-back's barrier)
#pragma unroll
      for (int k = 0; k < K; k++) {
        const uint32_t n = nb[k], p0 = pos[k];
        if (!n) continue;
        if (whole && p0 + n > lim) {
          over = true;
          atomicMin(&s_p1, p0);
        } else if (n <= 64) {
          if (whole) put_bits64(buf, p0, acc[k] << (64 - n), n);
          else put_bits64_win(buf, p0, acc[k] << (64 - n), n, lo_bit, hi_bit);
        } else {  // more than 64 bits (rare): the chunk again, token by token
          u4v tt;
          chunk_load(c0 + chunk_of(k), tt);
          uint32_t L[4], code[4], nzr[4];
          decode(tt, L, code, nzr);
          uint32_t p = p0;
          for (int e = 0; e < 4; e++) {
            for (uint32_t z = nzr[e]; z; z--) {
              if (whole) put_bits(buf, p, zcode, (int)Lz);
              else if (p < hi_bit && p + Lz > lo_bit) put_bits_window(buf, p, lo_bit, hi_bit, zcode, (int)Lz);
              p += Lz;
            }
            if (L[e]) {
              if (whole) put_bits(buf, p, code[e], (int)L[e]);
              else if (p < hi_bit && p + L[e] > lo_bit) put_bits_window(buf, p, lo_bit, hi_bit, code[e], (int)L[e]);
            }
            p += L[e];
          }
        }
      }
    }
    if (whole && __ballot(over) && lane == 0) s_over = 1;
    return run - boff;
  };
  // (the group's aggregate goes out inside the sweep; an empty group's here)
  const uint32_t gbits = sweep(true, 0u, 0u, 0u, true);
  PF_STAMP(2);
  if (C == 0 && tid == 0 && q > 0)
    __hip_atomic_store(&a.pack_state[gid], LB_AGG | 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // its start bit by decoupled look-back over the groups before it (wave 0;
  // publishes the inclusive prefix)
  if (wave == 0) {
    const unsigned long long base = a.bit_base ? a.bit_base[f * 4 + comp] : 0u;
    unsigned long long *stt = a.pack_state;
    unsigned long long prefix = base;
    bool hung = false;
    if (q > 0) {
      prefix = 0;
      long long j = gid - 1;
      // the bound counts from the last progress seen (a predecessor's
      // state word changing, or the window moving back), so a long but
      // live wait -- a predecessor slowed by time-slicing -- never trips it
      unsigned long long t_wait = __builtin_amdgcn_s_memrealtime();
      unsigned long long seen = ~0ull;
      while (true) {
        const long long jj = j - lane;
        unsigned long long sv = jj >= gscan0 ? __hip_atomic_load(&stt[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                             : (LB_INC | base);
        const unsigned long long m2 = __ballot((sv >> 62) == 2), m0 = __ballot((sv >> 62) == 0);
        const unsigned long long upto = m2 ? (m2 & (~m2 + 1)) : 0ull;  // lowest inclusive lane
        if (m0 & (upto ? upto - 1 : ~0ull)) {  // a group before it has not published yet
          // (groups publish in claim order, so this wait is short; one that
          // outlasts SPIN_TICKS without progress means a lost publication:
          // the frame fails instead of the launch hanging)
          const unsigned long long now = __builtin_amdgcn_s_memrealtime();
          if (m0 != seen) {
            seen = m0;
            t_wait = now;
          } else if (now - t_wait > SPIN_TICKS) {
            hung = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        seen = ~0ull;
        t_wait = __builtin_amdgcn_s_memrealtime();
        const int kk = upto ? __ffsll((long long)m2) - 1 : 63;
        unsigned long long add = lane <= kk ? (sv & LB_VAL) : 0ull;
        for (int off = 32; off; off >>= 1) add += __shfl_xor(add, off);
        prefix += add;
        if (upto) break;
        j -= 64;
      }
    }
    if (lane == 0) {
      // (a timed-out group still publishes, so the groups after it do not
      // wait out the bound as well; the frame is failed)
      __hip_atomic_store(&stt[gid], LB_INC | (prefix + gbits), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (q == nq - 1) a.scan_bits[f * 3 + comp] = prefix + gbits;
      s_prefix = prefix;
      if (FF) s_ffnb = q == nq - 1 ? (uint32_t)((prefix + gbits) >> 3) : ~0u;
      if (hung) a.err[f] = FERR_SPIN;
      s_hung = hung;
    }
  }
  __syncthreads();
  PF_STAMP(3);
  if (s_hung) return;  // (its start bit is unknown: nothing is stored)
  uint32_t *raw_scan = a.raw + (long long)f * G.raw_fs +
                       (comp == 0 ? 0 : G.raw_words[0] + (comp == 2 ? G.raw_words[1] : 0));
  const unsigned long long prefix = s_prefix;
  // the group's words in the scan: [first, first + n)
  uint32_t n = (uint32_t)(((prefix & 31) + gbits + 31) >> 5);
  if ((prefix >> 5) + n + 1 > (unsigned long long)G.raw_words[comp]) {  // cannot happen for valid tokens;
    if (tid == 0) a.err[f] = FERR_OVERFLOW;                              // never write out of bounds
    n = 0;
  }
  const unsigned long long gw = prefix >> 5;
  uint32_t *raw = raw_scan + gw;
  auto ff_add = [&](uint32_t v, uint32_t W, uint32_t c0) {
    const int c = ff_word(v, W, s_ffnb);
    if (c) atomicAdd(&s_ff[W / EMIT_CW - c0], (uint32_t)c);
  };
  auto ff_flush = [&](uint32_t w_first) {
    __syncthreads();
    if (FF && tid < FFN && s_ff[tid]) {  // the window's chunk counts out, zeroed for the next
      atomicAdd(&a.ffc[(long long)(f * 3 + comp) * emit_chunks(G) + w_first / EMIT_CW + tid], s_ff[tid]);
      s_ff[tid] = 0;
    }
  };
  if (!s_over) {
    // the window shifted into place: the edge words may be shared with the
    // neighbouring groups -- OR (onto zero), or in seam mode (EntArgs::seam)
    // the first word to the side
    const uint32_t sh = (uint32_t)(prefix & 31);
    const uint32_t c0 = (uint32_t)gw / EMIT_CW;
    for (uint32_t i = tid; i < n; i += PF_THREADS) {
      const uint32_t v = __builtin_amdgcn_alignbit(i ? buf[i - 1] : 0u, buf[i], sh);
      if (FF || a.seam) {
        if (i == 0 && sh) {
          a.seam[gid] = v;
        } else {
          raw[i] = v;
          if (FF) ff_add(v, (uint32_t)gw + i, c0);
        }
      } else if (i == 0 || i == n - 1) atomicOr(&raw[i], v);
      else raw[i] = v;
    }
    ff_flush((uint32_t)gw);
#ifdef MIJ_K1_DIAG
    PF_STAMP(4);
    if (a.dbg && tid == 0)
      for (int k = 0; k < 6; k++) a.dbg[(long long)gid * 6 + k] = pst[k];
#endif
    return;
  }
  // wider than the window: the words the first pass completed (every bit
  // before the first chunk it left out), then window by window from there at
  // offsets from the group's first word (boff = its first bit inside that
  // word), each window's sweep from the round it begins in
  const uint32_t boff = (uint32_t)(prefix & 31);
  const uint32_t k1 = min(n, (uint32_t)(((unsigned long long)s_p1 + boff) >> 5));
  {
    const uint32_t c0 = (uint32_t)gw / EMIT_CW;
    for (uint32_t i = tid; i < k1; i += PF_THREADS) {
      const uint32_t v = __builtin_amdgcn_alignbit(i ? buf[i - 1] : 0u, buf[i], boff);
      if (FF || a.seam) {
        if (i == 0 && boff) {
          a.seam[gid] = v;
        } else {
          raw[i] = v;
          if (FF) ff_add(v, (uint32_t)gw + i, c0);
        }
      } else if (i == 0) atomicOr(&raw[i], v);
      else raw[i] = v;
    }
    ff_flush((uint32_t)gw);
  }
  for (uint32_t w0 = k1; w0 < n; w0 += PW) {
    const uint32_t wn = min((uint32_t)PW, n - w0);
    __syncthreads();
    for (uint32_t i = tid; i < wn; i += PF_THREADS) buf[i] = 0;
    __syncthreads();
    sweep(false, boff, w0 * 32, (w0 + wn) * 32, false);
    __syncthreads();
    const uint32_t c0 = ((uint32_t)gw + w0) / EMIT_CW;
    for (uint32_t i = tid; i < wn; i += PF_THREADS) {
      const uint32_t wi = w0 + i;
      if (FF || a.seam) {
        if (wi == 0 && boff) {
          a.seam[gid] = buf[i];
        } else {
          raw[wi] = buf[i];
          if (FF) ff_add(buf[i], (uint32_t)gw + wi, c0);
        }
      } else if (wi == 0 || wi == n - 1) atomicOr(&raw[wi], buf[i]);
      else raw[wi] = buf[i];
    }
    ff_flush((uint32_t)gw + w0);
  }
}

// k_seam_fix (seam mode, EntArgs::seam): k_pack_flat stored every scan word
// whole, each by the one group that reaches its end, and left a group's first
// word, when the group before it ends inside that word, in seam[]; this ORs
// those words in (one thread per group; atomics only because the last, short
// group of a scan may start inside the same word as the one before it).
// Nothing then needs zeroed scan buffers: no OR-ing onto zero in the packing,
// no zeroing in k_emit_write.
// One group's seam word (frame f, group bq of the frame's gpf).
__device__ __forceinline__ void seam_fix_group(const EntArgs &a, const PackGrid &P, int f, int bq) {
  const Geom &G = a.g;
  const int gy = P.gy, gc = P.gc;
  const long long g = (long long)f * P.stride + bq;  // the group's look-back word
  const int comp = bq < gy ? 0 : (bq < gy + gc ? 1 : 2);
  const int q = bq - (comp == 0 ? 0 : (comp == 1 ? gy : gy + gc));
  if (q == 0) return;
  const unsigned long long start = a.pack_state[g - 1] & LB_VAL;  // the group's first bit
  if (!(start & 31)) return;
  uint32_t *raw = a.raw + (long long)f * G.raw_fs + (comp == 0 ? 0 : G.raw_words[0] + (comp == 2 ? G.raw_words[1] : 0));
  const uint32_t sv = a.seam[g], old = atomicOr(&raw[start >> 5], sv);
  if (a.ff_pack) {  // the 0xFF bytes the OR adds (an OR never removes one, so the adds telescope)
    const uint32_t W = (uint32_t)(start >> 5), nb = (uint32_t)(a.scan_bits[f * 3 + comp] >> 3);
    const int d = ff_word(old | sv, W, nb) - ff_word(old, W, nb);
    if (d) atomicAdd(&a.ffc[(long long)(f * 3 + comp) * emit_chunks(G) + W / EMIT_CW], (uint32_t)d);
  }
}

// Its own launch unless k_emit_scan does it (EntArgs::seam_in_scan: small
// batches with the packing's 0xFF counts, one launch fewer per encode).
__global__ __launch_bounds__(256) void k_seam_fix(EntArgs a) {
  const PackGrid P = pack_grid(a);
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)a.nframes * P.gpf) return;
  const int f = (int)(t / P.gpf), bq = (int)(t - (long long)f * P.gpf);
  if (a.err[f]) return;  // (a failed frame is dropped by the assembly)
  seam_fix_group(a, P, f, bq);
}

// ===========================================================================
// JFIF assembly (encoder.c:549-644): SOI/APP0, DQT x2, DHT x4, SOF0, then per
// component SOS + the scan bytes with 0xFF 0x00 stuffing (:405-408) + the pad
// byte of fill_last_byte (:425-432: 1-bits OR-ed into the free low bits, a
// whole 0xFF when the scan ended byte-aligned, never stuffed), then EOI.
//
// Each scan is cut into EMIT_CH-byte chunks.  k_emit_count counts the 0xFF
// bytes of every chunk; k_emit_write then knows every chunk's output offset
// (header + earlier scans + earlier chunks' stuffing) and writes the chunks
// independently: the stuffed bytes are laid out in LDS and leave in
// coalesced stores.  Workgroup (frame, j) takes chunks j, j + a.emit_slots, ..
// of the frame's chunk list (scan 0's, then 1's, then 2's), so the luma
// scan's chunks do not all queue behind a third of the workgroups.
// ===========================================================================
__device__ __forceinline__ bool emit_frame_ok(const EntArgs &a, int f) {
  unsigned long long need = 1024;  // headers, markers, pads
  for (int c = 0; c < 3; c++) need += 2 * (a.scan_bits[f * 3 + c] >> 3) + 2;
  return !a.err[f] && need <= (unsigned long long)a.g.out_cap &&
         a.scan_bits[f * 3 + 0] <= 32ull * a.g.raw_words[0] &&
         a.scan_bits[f * 3 + 1] <= 32ull * a.g.raw_words[1] &&
         a.scan_bits[f * 3 + 2] <= 32ull * a.g.raw_words[2];
}

__device__ __forceinline__ const uint32_t *scan_raw(const EntArgs &a, int f, int comp) {
  return a.raw + (long long)f * a.g.raw_fs +
         (comp == 0 ? 0 : a.g.raw_words[0] + (comp == 2 ? a.g.raw_words[1] : 0));
}


__device__ __forceinline__ int block_sum256(int v, int *red) {
  for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const int t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(256) void k_emit_count(EntArgs a) {
  __shared__ int red[4];
  const int slot = blockIdx.x % a.emit_slots, f = blockIdx.x / a.emit_slots;
  long long nch[3];
  unsigned long long nbs[3];
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    nbs[comp] = a.scan_bits[f * 3 + comp] >> 3;
    nch[comp] = nbs[comp] > 4ull * a.g.raw_words[comp] ? 0 : (long long)((nbs[comp] + EMIT_CH - 1) / EMIT_CH);
  }  // (a scan past its buffer: k_emit_write drops the frame)
  // the frame's chunks, scan after scan, dealt round-robin to its workgroups
  for (long long i = slot; i < nch[0] + nch[1] + nch[2]; i += a.emit_slots) {
    const int comp = i < nch[0] ? 0 : (i < nch[0] + nch[1] ? 1 : 2);
    const long long c = i - (comp == 0 ? 0 : (comp == 1 ? nch[0] : nch[0] + nch[1]));
    const unsigned long long nbytes = nbs[comp];
    const uint32_t *raw = scan_raw(a, f, comp);
    const unsigned long long b0 = (unsigned long long)c * EMIT_CH + threadIdx.x * (EMIT_CH / 256);
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < EMIT_CH / 4096; k++) {
      const unsigned long long mb = b0 + 16 * k;
      if (mb < nbytes) {
        const uint4 v = *(const uint4 *)(raw + (mb >> 2));
        const long long rem = (long long)(nbytes - mb);
        cnt += ff_bytes(v.x, (int)min(rem, 4ll)) + ff_bytes(v.y, (int)max(0ll, min(rem - 4, 4ll))) +
               ff_bytes(v.z, (int)max(0ll, min(rem - 8, 4ll))) + ff_bytes(v.w, (int)max(0ll, min(rem - 12, 4ll)));
      }
    }
    const int tot = block_sum256(cnt, red);
    if (threadIdx.x == 0) a.ffc[(long long)(f * 3 + comp) * emit_chunks(a.g) + c] = (uint32_t)tot;
  }
}

// Frame headers (encoder.c:549-600) into out[0, hlen); returns hlen.  Called
// by a whole workgroup (s_n: 4 ints of LDS; one barrier inside).
__device__ __forceinline__ int emit_headers(const EntArgs &a, int f, uint8_t *out, int *s_n) {
  const int tid = threadIdx.x;
  const HuffCode *hc = a.hc + (long long)f * 4;
  // headers, one byte per thread (a single thread's byte loop is a chain of
  // dependent loads and stores: 40 us per launch): APP0 20 + DQT 2 x 69 +
  // DHT 4 x (21 + n_t) + SOF0 19
  {
    int hn = tid < 64 ? hc[tid >> 4].code_len_freq[1 + (tid & 15)] : 0;
    for (int o = 8; o; o >>= 1) hn += __shfl_xor(hn, o);  // sums over 16 lanes
    if (tid < 64 && (tid & 15) == 0) s_n[tid >> 4] = hn;
  }
  __syncthreads();
  int doff[5];  // DHT t starts at doff[t]; SOF0 at doff[4]
  doff[0] = 20 + 2 * 69;
  for (int t = 0; t < 4; t++) doff[t + 1] = doff[t] + 21 + s_n[t];
  const int hlen = doff[4] + 19;
  {
    const FGeom fg = frame_geom(a.g, a.fdims, f);
    const int W = fg.w, H = fg.h;
    auto hbyte = [&](int i) -> uint8_t {
      if (i < 20) {
        const uint8_t app0[20] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 0x4A, 0x46, 0x49, 0x46,
                                  0x00, 0x01, 0x01, 0x00, 0x00, 0x48, 0x00, 0x48, 0x00, 0x00};
        return app0[i];
      }
      if (i < doff[0]) {  // DQT (encoder.c:559-571)
        const int t = (i - 20) / 69, k = (i - 20) - 69 * t;
        const uint8_t m[5] = {0xFF, 0xDB, 0x00, 0x43, (uint8_t)t};
        return k < 5 ? m[k] : (uint8_t)a.tab->dqt[t][k - 5];
      }
      if (i < doff[4]) {  // DHT (encoder.c:504-532)
        const int t = i >= doff[3] ? 3 : i >= doff[2] ? 2 : i >= doff[1] ? 1 : 0;
        const int k = i - doff[t], len = 19 + s_n[t];
        const uint8_t m[5] = {0xFF, 0xC4, (uint8_t)(len >> 8), (uint8_t)len, (uint8_t)((t & 1) << 4 | (t >> 1))};
        return k < 5 ? m[k] : k < 21 ? (uint8_t)hc[t].code_len_freq[k - 4] : (uint8_t)hc[t].sym_sorted[k - 21];
      }
      // SOF0 (encoder.c:573-600)
      const uint8_t sof[19] = {0xFF, 0xC0, 0x00, 0x11, 0x08, (uint8_t)(H >> 8), (uint8_t)H,
                               (uint8_t)(W >> 8), (uint8_t)W, 0x03, 0x01, 0x22, 0x00,
                               0x02, 0x11, 0x01, 0x03, 0x11, 0x01};
      return sof[i - doff[4]];
    };
    // a thread's first HB bytes all computed before any is stored: their
    // loads then go out together instead of each waiting behind the store
    // before it (hlen = 261 + the four tables' symbols: <= 768 whenever the
    // tables hold <= 507 symbols in all -- 2 x 162 AC + 2 x 12 DC at most in
    // practice; the loop after covers the rest)
    constexpr int HB = 3;
    uint8_t hv[HB];
#pragma unroll
    for (int hb = 0; hb < HB; hb++) hv[hb] = tid + 256 * hb < hlen ? hbyte(tid + 256 * hb) : (uint8_t)0;
#pragma unroll
    for (int hb = 0; hb < HB; hb++)
      if (tid + 256 * hb < hlen) out[tid + 256 * hb] = hv[hb];
    for (int i = tid + 256 * HB; i < hlen; i += 256) out[i] = hbyte(i);
  }
  return hlen;
}

// k_emit_scan: one workgroup per frame.  Headers (encoder.c:549-600), the
// SOS of each scan, the output offset of every chunk (exclusive scan of the
// 0xFF counts), the pad bytes (:425-432), EOI and the frame's length.
__global__ __launch_bounds__(256) void k_emit_scan(EntArgs a) {
  __shared__ int red[3][4];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (!emit_frame_ok(a, f)) {
    if (tid == 0) a.out_len[f] = 0;
    return;
  }
  uint8_t *out = a.out + (long long)f * a.g.out_cap;
  const long long nchmax = emit_chunks(a.g);
  // the scans' bit counts, once (the byte stores below may alias them for
  // the compiler, which would load them again after each)
  unsigned long long nbits[3];
  long long nch[3];
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    nbits[comp] = a.scan_bits[f * 3 + comp];
    nch[comp] = (long long)(((nbits[comp] >> 3) + EMIT_CH - 1) / EMIT_CH);
  }
  // seam mode with the packing's 0xFF counts: the frame's seam words first
  // (their OR-s and count adds land in L2; the counts and the pad words below
  // are read past this CU's L1, which may hold lines of a neighbouring frame)
  // (one device fence per frame here: at most 15 frames take this path; the
  // counts and pad words are then read past this CU's L1.  Reading them back
  // by atomics instead, without the fence, measured 0.9 us slower on four
  // frames, equal on one)
  const bool seams = a.seam && a.ff_pack && a.seam_in_scan;
  if (seams) {
    const PackGrid P = pack_grid(a);
    for (int bq = tid; bq < P.gpf; bq += 256) seam_fix_group(a, P, f, bq);
    __threadfence();
    // every thread's fixes in before any thread reads a count or pad word
    // (the loads below come before the headers' barrier)
    __syncthreads();
  }
  auto count_at = [&](int comp, long long c) -> int {
    const uint32_t *cnt = a.ffc + (long long)(f * 3 + comp) * nchmax;
    return c < nch[comp] ? (int)(seams ? __hip_atomic_load(cnt + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : cnt[c])
                         : 0;
  };
  // the loads the offsets and pads need, all issued before the headers'
  // (one memory latency for all of them): the first 256 chunk counts of each
  // scan and the words holding the pad bytes' bits
  int v0[3];
  uint32_t padw[3] = {0u, 0u, 0u};
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    v0[comp] = count_at(comp, tid);
    const unsigned long long nbytes = nbits[comp] >> 3;
    if (tid == 0 && (nbits[comp] & 7)) {
      const uint32_t *raw = scan_raw(a, f, comp);
      padw[comp] = seams ? __hip_atomic_load(raw + (nbytes >> 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : raw[nbytes >> 2];
    }
  }
  __shared__ int s_n[4];
  const int hlen = emit_headers(a, f, out, s_n);
  // the three scans' first rounds of offsets in one pass (one barrier)
  int incl0[3];
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    incl0[comp] = (int)wave_scan64((uint32_t)v0[comp]);
    if (lane == 63) red[comp][wave] = incl0[comp];
  }
  __syncthreads();
  unsigned long long pos = (unsigned long long)hlen;
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    if (tid == 0) {  // SOS (encoder.c:601-620)
      const uint8_t sos[10] = {0xFF, 0xDA, 0x00, 0x08, 0x01, (uint8_t)(comp + 1),
                               (uint8_t)(comp ? 0x11 : 0x00), 0x00, 0x3F, 0x00};
      for (int i = 0; i < 10; i++) out[pos + i] = sos[i];
    }
    pos += 10;
    const unsigned long long nbytes = nbits[comp] >> 3;
    uint32_t *off = a.choff + (long long)(f * 3 + comp) * nchmax;
    unsigned long long carry = 0;  // 0xFF bytes of the earlier chunks
    {
      int wb = 0, tot = 0;
      for (int q = 0; q < 4; q++) {
        if (q < wave) wb += red[comp][q];
        tot += red[comp][q];
      }
      if (tid < nch[comp]) off[tid] = (uint32_t)(pos + (unsigned long long)tid * EMIT_CH + wb + incl0[comp] - v0[comp]);
      carry = tot;
    }
    for (long long c0 = 256; c0 < nch[comp]; c0 += 256) {  // (scans of more than 256 chunks: 2 MB)
      const long long c = c0 + tid;
      const int v = count_at(comp, c);
      const int incl = (int)wave_scan64((uint32_t)v);
      __syncthreads();  // (red: the pass before has read it)
      if (lane == 63) red[comp][wave] = incl;
      __syncthreads();
      int wb = 0, tot = 0;
      for (int q = 0; q < 4; q++) {
        if (q < wave) wb += red[comp][q];
        tot += red[comp][q];
      }
      if (c < nch[comp]) off[c] = (uint32_t)(pos + (unsigned long long)c * EMIT_CH + carry + wb + incl - v);
      carry += tot;
    }
    pos += nbytes + carry;
    if (tid == 0) {  // the pad byte of fill_last_byte, never stuffed
      const int r = (int)(nbits[comp] & 7);
      uint8_t pad = 0xFF;
      if (r) {
        const uint8_t part = (uint8_t)(padw[comp] >> (24 - 8 * (nbytes & 3)));
        pad = (uint8_t)(part | ((1u << (8 - r)) - 1u));
      }
      out[pos] = pad;
    }
    pos += 1;
  }
  if (tid == 0) {
    out[pos] = 0xFF;
    out[pos + 1] = 0xD9;
    a.out_len[f] = pos + 2;
  }
}

// The stuffed bytes (encoder.c:403-408: 0x00 after every 0xFF) of chunk
// [cb, cb + EMIT_CH) of a byte stream nbytes long whose big-endian word w is
// word(w), written at out + o0; tot = the chunk's 0xFF bytes, both from
// meta(o0, tot), called after the words' loads are issued (its own loads then
// share their wait instead of preceding them).  after_load(w) runs once per
// loaded word, after the load (k_emit_write zeroes the scan word there).
// Called by a whole 256-thread workgroup; s_out: 2 * EMIT_CH bytes, red: 4
// ints of LDS.  DIRECT: every word's bytes go straight to out (a word without
// 0xFF bytes by one unaligned dword store, the rest byte by byte); s_out is
// not used.
template <bool DIRECT = false, class WordFn, class AfterFn, class MetaFn>
__device__ __forceinline__ void stuff_chunk(const WordFn &word, const AfterFn &after_load, const MetaFn &meta,
                                            unsigned long long nbytes, unsigned long long cb, uint8_t *out,
                                            uint8_t *s_out, int *red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int WPW = EMIT_CH / 16;  // stream words per wave
  // Stuffed bytes into LDS, chunk-relative.  Wave v takes stream words
  // [WPW v, WPW v + WPW) of the chunk, lane l word 64 k + l of it in round
  // k: consecutive lanes write consecutive bytes (no LDS bank conflicts).
  // All of the lane's words are loaded at once; a word's offset is 4 w +
  // the 0xFF bytes before it (wave totals through LDS, a wave scan per round).
  const unsigned long long wb0 = cb + (unsigned long long)wave * (4 * WPW);
  uint32_t wds[WPW / 64];
  int lims[WPW / 64], cfs[WPW / 64];
  int wcnt = 0;
#pragma unroll
  for (int k = 0; k < WPW / 64; k++) {
    const unsigned long long mb = wb0 + 4ull * (64 * k + lane);
    lims[k] = mb < nbytes ? (int)min(nbytes - mb, 4ull) : 0;
    wds[k] = lims[k] ? word(mb >> 2) : 0u;
  }
  unsigned long long o0;
  int tot;
  meta(o0, tot);
#pragma unroll
  for (int k = 0; k < WPW / 64; k++) {  // (kept: the layout pass below needs them again)
    cfs[k] = lims[k] ? ff_bytes(wds[k], lims[k]) : 0;
    wcnt += cfs[k];
  }
#pragma unroll
  for (int k = 0; k < WPW / 64; k++)
    if (lims[k]) after_load((wb0 + 4ull * (64 * k + lane)) >> 2);
  for (int off = 32; off; off >>= 1) wcnt += __shfl_xor(wcnt, off);
  if (lane == 0) red[wave] = wcnt;
  __syncthreads();
  int carry = wave * 4 * WPW;
  for (int q = 0; q < wave; q++) carry += red[q];
#pragma unroll
  for (int k = 0; k < WPW / 64; k++) {
    const int lim = lims[k];
    const uint32_t wd = wds[k];
    const int cf = cfs[k];
    const int incl = (int)wave_scan64((uint32_t)(lim + cf));
    int op = carry + incl - (lim + cf);
    carry += __shfl(incl, 63);
    if (DIRECT) {
      uint8_t *d = out + o0;
      if (cf == 0 && lim == 4) {
        *(uint32_t *)(d + op) = __builtin_bswap32(wd);  // (unaligned: the hardware's unaligned mode)
      } else {
        for (int j = 0; j < lim; j++) {
          const uint8_t byte = (uint8_t)(wd >> (24 - 8 * j));
          d[op++] = byte;
          if (byte == 0xFF) d[op++] = 0x00;
        }
      }
    } else if (cf == 0) {
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (j < lim) s_out[op + j] = (uint8_t)(wd >> (24 - 8 * j));
    } else {
      for (int j = 0; j < lim; j++) {
        const uint8_t byte = (uint8_t)(wd >> (24 - 8 * j));
        s_out[op++] = byte;
        if (byte == 0xFF) s_out[op++] = 0x00;
      }
    }
  }
  __syncthreads();  // (DIRECT: before the next chunk's wave totals overwrite red)
  if (DIRECT) return;
  // copy out: head bytes up to a 4-byte boundary, whole words (re-aligned
  // from LDS words with v_alignbyte), tail bytes; every byte of
  // [o0, o0 + clen) belongs to this chunk alone
  const int clen = (int)min((unsigned long long)EMIT_CH, nbytes - cb) + tot;
  const int head = min(clen, (int)((4 - (o0 & 3)) & 3));
  const int nwd = (clen - head) >> 2;
  if (tid < head) out[o0 + tid] = s_out[tid];
  const int tl = clen - head - 4 * nwd;
  if (tid < tl) out[o0 + head + 4 * nwd + tid] = s_out[head + 4 * nwd + tid];
  const uint32_t *s32 = (const uint32_t *)s_out;
  uint32_t *d32 = (uint32_t *)(out + o0 + head);
  const int sh = head & 3;  // LDS byte offset of output word j = head + 4j
  for (int j = tid; j < nwd; j += 256) {
    const int m = (head >> 2) + j;
    const uint32_t lo = s32[m];
    d32[j] = sh ? __builtin_amdgcn_alignbyte(s32[m + 1], lo, sh) : lo;
  }
  __syncthreads();
}

// k_emit_write: the stuffed bytes of every chunk at the offset k_emit_scan gave.
__global__ __launch_bounds__(256) void k_emit_write(EntArgs a) {
  // (no LDS staging: each word's bytes go straight to the output, round 6:
  // emit 0.142 -> 0.111 ms at Q=50, 0.390 -> 0.315 at Q=90)
  constexpr bool DIRECT = true;
  uint8_t *s_out = nullptr;
  __shared__ int red[4];
  const int slot = blockIdx.x % a.emit_slots, f = blockIdx.x / a.emit_slots;
  const int tid = threadIdx.x;
  // every scan-buffer word read here is zeroed after use: the band packing needs
  // all-zero buffers (a failed frame's buffers are cleared whole) -- except
  // in seam mode, where k_pack_flat stores whole words and nothing is zeroed
  const bool zero = a.seam == nullptr;
  if (!emit_frame_ok(a, f)) {
    uint32_t *rawf = a.raw + (long long)f * a.g.raw_fs;
    if (zero)
      for (long long i = (long long)slot * 256 + tid; i < a.g.raw_fs; i += (long long)a.emit_slots * 256) rawf[i] = 0;
    // the chunk counts left zeroed (ff_pack adds to them)
    for (long long i = (long long)slot * 256 + tid; i < 3 * emit_chunks(a.g); i += (long long)a.emit_slots * 256)
      a.ffc[(long long)f * 3 * emit_chunks(a.g) + i] = 0;
    return;
  }
  uint8_t *out = a.out + (long long)f * a.g.out_cap;
  const long long nchmax = emit_chunks(a.g);
  long long nch[3];
  unsigned long long nbs[3];  // (kept: the stores below may alias scan_bits for the compiler)
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    const unsigned long long nbits = a.scan_bits[f * 3 + comp], nbytes = nbits >> 3;
    nbs[comp] = nbytes;
    nch[comp] = (long long)((nbytes + EMIT_CH - 1) / EMIT_CH);
    if (zero && slot == 0 && tid < 2) {  // words past the last whole byte (the pad byte's bits)
      const unsigned long long w = ((nbytes + 3) >> 2) + tid;
      if (w < ((nbits + 31) >> 5)) ((uint32_t *)scan_raw(a, f, comp))[w] = 0;
    }
  }
  // the frame's chunks, scan after scan, dealt round-robin to its workgroups
  for (long long i = slot; i < nch[0] + nch[1] + nch[2]; i += a.emit_slots) {
    const int comp = i < nch[0] ? 0 : (i < nch[0] + nch[1] ? 1 : 2);
    const long long c = i - (comp == 0 ? 0 : (comp == 1 ? nch[0] : nch[0] + nch[1]));
    const unsigned long long nbytes = comp == 0 ? nbs[0] : (comp == 1 ? nbs[1] : nbs[2]);
    uint32_t *raw = (uint32_t *)scan_raw(a, f, comp);
    const long long ci = (long long)(f * 3 + comp) * nchmax + c;
    stuff_chunk<DIRECT>([&](unsigned long long w) { return raw[w]; },
                [&](unsigned long long w) {
                  if (zero) raw[w] = 0u;
                },
                [&](unsigned long long &o0, int &tot) {
                  tot = (int)a.ffc[ci];
                  o0 = a.choff[ci];
                },
                nbytes, (unsigned long long)c * EMIT_CH, out, s_out, red);
    if (tid == 0) a.ffc[ci] = 0;  // read: left zeroed (ff_pack adds)
  }
}

// ===========================================================================
// Distributed JFIF emission of one large frame in bands (config 4, SURVEY.md
// §8(e)).  After every band packed its scans from bit 0 and the bands' bit
// counts were all-gathered, band r knows where each of its scans starts in
// the frame's scan: bit B = the bits of bands 0..r-1 (encoder.c:462-502's
// running bit position).  The final stream's bytes that lie wholly inside
// the band (its "interior", from the first byte boundary at or after B) are
// stuffed here, on the band's own GPU (k_emit_count on the band's words read
// shifted by the head, k_band_stuff_scan, k_band_write); the bits before
// that boundary (the head, <= 7, completing the byte the previous band
// started) and after the last whole interior byte (the tail) go to the root
// in a per-scan record.  The root then only writes headers, the seam bytes
// (previous tail | head, stuffed when 0xFF), the pads and EOI, and copies the
// bands' stuffed interiors into place (k_band_join, k_copy_bytes).
// Record per (frame, scan), four u64: stuffed interior bytes; bits; head
// bits << 8 | head count; tail bits << 8 | tail count.
// ===========================================================================
constexpr int BREC = 4;

// per (frame, scan): the band's start offset and head/tail, the interior's
// byte count into scan_bits (as bits, for k_emit_count and the writer) and
// the head shift into bit_base; one thread per scan
__global__ void k_band_stuff_prep(EntArgs a, const unsigned long long *allbits, int world, int rank,
                                  unsigned long long *rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // f * 3 + comp
  if (i >= 3 * a.nframes) return;
  const int f = i / 3, comp = i - 3 * f;
  unsigned long long B = 0;
  for (int r = 0; r < rank; r++) B += allbits[(long long)r * (3 * a.nframes + 1) + i];
  const unsigned long long bits = allbits[(long long)rank * (3 * a.nframes + 1) + i];
  const uint32_t *raw = scan_raw(a, f, comp);
  const uint32_t h0 = (uint32_t)((8 - (B & 7)) & 7);
  const uint32_t h = bits < h0 ? (uint32_t)bits : h0;  // head: completes the byte before
  const unsigned long long ni = (bits - h) >> 3;        // whole bytes after the head
  const uint32_t t = (uint32_t)((bits - h) & 7);        // tail bits
  // bit j of the band's stream (big-endian words)
  auto bits_at = [&](unsigned long long j, uint32_t n) -> uint32_t {  // n <= 8, j + n <= bits
    if (!n) return 0u;
    const unsigned long long w = j >> 5;
    const uint32_t o = (uint32_t)(j & 31);
    const uint64_t two = ((uint64_t)raw[w] << 32) | (o + n > 32 ? raw[w + 1] : 0u);
    return (uint32_t)(two >> (64 - o - n)) & ((1u << n) - 1u);
  };
  unsigned long long *rc = rec + (long long)i * BREC;
  rc[1] = bits;
  rc[2] = ((unsigned long long)bits_at(0, h) << 8) | h;
  rc[3] = ((unsigned long long)bits_at(h + 8 * ni, t) << 8) | t;
  a.scan_bits[i] = 8 * ni;
  const_cast<uint32_t *>(a.bit_base)[f * 4 + comp] = h;
}

// the band's interiors in (frame, scan) order into dst: every chunk's output
// offset inside its scan (an exclusive scan of the 0xFF counts; 32 bits: a
// scan's stuffed bytes stay below a frame's out_cap) and every scan's first
// byte in dst (scan_base, 64 bits: the band's buffer holds all n frames'
// scans), the stuffed bytes per scan into rec[0] and the band's total into
// *total; one workgroup
__global__ __launch_bounds__(256) void k_band_stuff_scan(EntArgs a, unsigned long long *rec,
                                                         unsigned long long *total) {
  __shared__ int red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long nchmax = emit_chunks(a.g);
  unsigned long long pos = 0;
  for (int i = 0; i < 3 * a.nframes; i++) {
    const unsigned long long nbytes = a.scan_bits[i] >> 3;
    const long long nch = (long long)((nbytes + EMIT_CH - 1) / EMIT_CH);
    const uint32_t *cnt = a.ffc + (long long)i * nchmax;
    uint32_t *off = a.choff + (long long)i * nchmax;
    unsigned long long carry = 0;
    for (long long c0 = 0; c0 < nch; c0 += 256) {
      const long long c = c0 + tid;
      const int v = c < nch ? (int)cnt[c] : 0;
      const int incl = (int)wave_scan64((uint32_t)v);
      if (lane == 63) red[wave] = incl;
      __syncthreads();
      int wb = 0, tot = 0;
      for (int q = 0; q < 4; q++) {
        if (q < wave) wb += red[q];
        tot += red[q];
      }
      __syncthreads();
      if (c < nch) off[c] = (uint32_t)((unsigned long long)c * EMIT_CH + carry + wb + incl - v);
      carry += tot;
    }
    if (tid == 0) {
      rec[(long long)i * BREC] = nbytes + carry;
      a.scan_base[i] = pos;
    }
    pos += nbytes + carry;
  }
  if (tid == 0) *total = pos;
}

// the band's word w of scan (f, comp) read shifted left by its head
__device__ __forceinline__ uint32_t shifted_word(const uint32_t *raw, unsigned long long w, uint32_t h) {
  return h ? __builtin_amdgcn_alignbit(raw[w], raw[w + 1], 32 - h) : raw[w];
}

// k_emit_count on the shifted interiors
__global__ __launch_bounds__(256) void k_band_count_ff(EntArgs a) {
  __shared__ int red[4];
  const int slot = blockIdx.x % a.emit_slots, f = blockIdx.x / a.emit_slots;
  long long nch[3];
  unsigned long long nbs[3];
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    nbs[comp] = a.scan_bits[f * 3 + comp] >> 3;
    nch[comp] = (long long)((nbs[comp] + EMIT_CH - 1) / EMIT_CH);
  }
  for (long long i = slot; i < nch[0] + nch[1] + nch[2]; i += a.emit_slots) {
    const int comp = i < nch[0] ? 0 : (i < nch[0] + nch[1] ? 1 : 2);
    const long long c = i - (comp == 0 ? 0 : (comp == 1 ? nch[0] : nch[0] + nch[1]));
    const unsigned long long nbytes = nbs[comp];
    const uint32_t *raw = scan_raw(a, f, comp);
    const uint32_t h = a.bit_base[f * 4 + comp];
    const unsigned long long b0 = (unsigned long long)c * EMIT_CH + threadIdx.x * (EMIT_CH / 256);
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < EMIT_CH / 1024; k++) {
      const unsigned long long mb = b0 + 4 * k;
      if (mb < nbytes) cnt += ff_bytes(shifted_word(raw, mb >> 2, h), (int)min(nbytes - mb, 4ull));
    }
    const int tot = block_sum256(cnt, red);
    if (threadIdx.x == 0) a.ffc[(long long)(f * 3 + comp) * emit_chunks(a.g) + c] = (uint32_t)tot;
  }
}

// the stuffed interiors at the offsets k_band_stuff_scan gave (dst: the
// band's buffer, cap bytes: a chunk that would end past it is not written,
// and the counts say so to the caller via the total)
__global__ __launch_bounds__(256) void k_band_write(EntArgs a, uint8_t *dst, unsigned long long cap) {
  uint8_t *s_out = nullptr;  // (stuff_chunk<true>: straight to dst, as k_emit_write)
  __shared__ int red[4];
  const int slot = blockIdx.x % a.emit_slots, f = blockIdx.x / a.emit_slots;
  const long long nchmax = emit_chunks(a.g);
  long long nch[3];
#pragma unroll
  for (int comp = 0; comp < 3; comp++) nch[comp] = (long long)(((a.scan_bits[f * 3 + comp] >> 3) + EMIT_CH - 1) / EMIT_CH);
  for (long long i = slot; i < nch[0] + nch[1] + nch[2]; i += a.emit_slots) {
    const int comp = i < nch[0] ? 0 : (i < nch[0] + nch[1] ? 1 : 2);
    const long long c = i - (comp == 0 ? 0 : (comp == 1 ? nch[0] : nch[0] + nch[1]));
    const unsigned long long nbytes = a.scan_bits[f * 3 + comp] >> 3;
    const uint32_t *raw = scan_raw(a, f, comp);
    const uint32_t h = a.bit_base[f * 4 + comp];
    const long long ci = (long long)(f * 3 + comp) * nchmax + c;
    const int tot = (int)a.ffc[ci];
    const unsigned long long o0 = a.scan_base[f * 3 + comp] + a.choff[ci];
    const unsigned long long clen = min((unsigned long long)EMIT_CH, nbytes - (unsigned long long)c * EMIT_CH) + tot;
    if (o0 + clen <= cap)  // (workgroup-uniform)
      stuff_chunk<true>([&](unsigned long long w) { return shifted_word(raw, w, h); }, [](unsigned long long) {},
                  [&](unsigned long long &o, int &t) {
                    o = o0;
                    t = tot;
                  },
                  nbytes, (unsigned long long)c * EMIT_CH, dst, s_out, red);
    if (threadIdx.x == 0) a.ffc[ci] = 0;  // left zeroed for the next count
  }
}

// the band's scan words zeroed again (the band packing ORs onto zero):
// the words of its bits only
__global__ void k_band_zero(EntArgs a, const unsigned long long *rec) {
  const int i = blockIdx.y;  // f * 3 + comp
  const int f = i / 3, comp = i - 3 * f;
  uint32_t *raw = (uint32_t *)scan_raw(a, f, comp);
  const unsigned long long nw = (rec[(long long)i * BREC + 1] + 31) >> 5;
  for (unsigned long long w = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; w < nw;
       w += (unsigned long long)gridDim.x * blockDim.x)
    raw[w] = 0u;
}

// root: frame f from every band's records allrec[world][n][3][BREC] and
// stuffed interiors src[world][stride]: headers, per scan the SOS, the seam
// bytes between the bands (the pending bits of the bands before, completed
// by the next band's head: encoder.c:385-415, stuffed when 0xFF), the pad
// (:425-432) and EOI; the interiors' copies go to the piece table
// pieces[f][world][3] = {src offset, dst offset, bytes} for k_copy_bytes.
// One workgroup per frame.
__global__ __launch_bounds__(256) void k_band_join(EntArgs a, const unsigned long long *allrec, int world,
                                                   unsigned long long stride, unsigned long long *pieces) {
  const int f = blockIdx.x, tid = threadIdx.x;
  const int n = a.nframes;
  uint8_t *out = a.out + (long long)f * a.g.out_cap;
  __shared__ int s_n[4];
  __shared__ int s_bad;
  if (tid == 0) {
    // the frame fits its output (headers, markers and pads within 1024 B)
    unsigned long long need = 1024;
    for (int r = 0; r < world; r++)
      for (int c = 0; c < 3; c++) need += 2 * allrec[(((long long)r * n + f) * 3 + c) * BREC] + 4;
    s_bad = a.err[f] || need > (unsigned long long)a.g.out_cap;
    for (int r = 0; r < world && !s_bad; r++) {  // every band's interiors inside its stride
      unsigned long long end = 0;
      for (int i = 0; i < 3 * n; i++) end += allrec[((long long)r * n * 3 + i) * BREC];
      s_bad = end > stride;
    }
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) {
      a.out_len[f] = 0;
      a.err[f] = a.err[f] ? a.err[f] : FERR_ASSEMBLY;
      for (int r = 0; r < world; r++)
        for (int c = 0; c < 3; c++) pieces[(((long long)f * world + r) * 3 + c) * 3 + 2] = 0;
    }
    return;
  }
  const int hlen = emit_headers(a, f, out, s_n);
  if (tid != 0) return;
  unsigned long long pos = (unsigned long long)hlen;
  for (int c = 0; c < 3; c++) {
    const uint8_t sos[10] = {0xFF, 0xDA, 0x00, 0x08, 0x01, (uint8_t)(c + 1), (uint8_t)(c ? 0x11 : 0x00), 0x00, 0x3F, 0x00};
    for (int i = 0; i < 10; i++) out[pos + i] = sos[i];
    pos += 10;
    uint32_t pend = 0, np = 0;  // bits of the byte being filled (np < 8)
    unsigned long long total_bits = 0;
    for (int r = 0; r < world; r++) {
      const unsigned long long *rc = allrec + (((long long)r * n + f) * 3 + c) * BREC;
      // this band's interiors start in its buffer after those of the earlier scans
      unsigned long long so = 0;
      for (int i = 0; i < f * 3 + c; i++) so += allrec[((long long)r * n * 3 + i) * BREC];
      const uint32_t h = (uint32_t)(rc[2] & 255), hv = (uint32_t)(rc[2] >> 8);
      const uint32_t t = (uint32_t)(rc[3] & 255), tv = (uint32_t)(rc[3] >> 8);
      total_bits += rc[1];
      pend = (pend << h) | hv;
      np += h;
      if (np == 8) {  // a seam byte completed
        out[pos++] = (uint8_t)pend;
        if ((pend & 255) == 0xFF) out[pos++] = 0x00;
        pend = np = 0;
      }
      unsigned long long *pc = pieces + (((long long)f * world + r) * 3 + c) * 3;
      pc[0] = (unsigned long long)r * stride + so;
      pc[1] = (unsigned long long)f * a.g.out_cap + pos;
      pc[2] = rc[0];
      pos += rc[0];
      // the tail (t > 0 only after the head reached a byte boundary: pend
      // is empty then) starts the next byte
      pend = (pend << t) | tv;
      np += t;
    }
    a.scan_bits[f * 3 + c] = total_bits;
    // fill_last_byte (:425-432): the free low bits set, never stuffed; a
    // whole 0xFF when the scan ended on a byte boundary
    out[pos++] = np ? (uint8_t)((pend << (8 - np)) | ((1u << (8 - np)) - 1u)) : (uint8_t)0xFF;
  }
  out[pos] = 0xFF;
  out[pos + 1] = 0xD9;
  a.out_len[f] = pos + 2;
}

// byte copies of the piece table {src offset, dst offset, bytes} (blockIdx.y
// = piece; destination words whole, sources re-aligned with v_alignbyte)
__global__ __launch_bounds__(256) void k_copy_bytes(uint8_t *dst, const uint8_t *src, const unsigned long long *pieces) {
  const unsigned long long *pc = pieces + 3 * (long long)blockIdx.y;
  const unsigned long long so = pc[0], dof = pc[1], n = pc[2];
  if (!n) return;
  const unsigned long long G = (unsigned long long)gridDim.x * blockDim.x;
  const unsigned long long t0 = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  // head bytes up to the destination's word boundary, then whole words
  const unsigned long long head = min(n, (4 - (dof & 3)) & 3);
  if (t0 < head) dst[dof + t0] = src[so + t0];
  const unsigned long long nw = (n - head) >> 2, s1 = so + head;
  const uint32_t *sw = (const uint32_t *)(src + (s1 & ~3ull));
  const uint32_t sh = (uint32_t)(s1 & 3);
  uint32_t *dw = (uint32_t *)(dst + dof + head);
  for (unsigned long long j = t0; j < nw; j += G) {
    const uint32_t lo = sw[j];
    dw[j] = sh ? __builtin_amdgcn_alignbyte(sw[j + 1], lo, sh) : lo;
  }
  const unsigned long long tl = n - head - 4 * nw;
  if (t0 < tl) dst[dof + head + 4 * nw + t0] = src[so + head + 4 * nw + t0];
}

// ---- region batches: each region (x, y, w, h) of one frame into its slot ---
// (the top-left w x h of the slot, rows `pitch` bytes apart), as main.c:142-152
// hands every region of a frame to rgb_to_dct(raw, .., dims[i]).  Workgroup
// (row, region) copies one row of the region; rows beyond a region idle.
__global__ __launch_bounds__(256) void k_gather_regions(uint8_t *dst, long long slot_bytes, int pitch,
                                                        const uint8_t *src, long long src_pitch,
                                                        const int4 *regions) {
  const int4 r = regions[blockIdx.y];  // x, y, w, h
  const int row = blockIdx.x;
  if (row >= r.w) return;
  const uint8_t *s = src + (long long)(r.y + row) * src_pitch + (long long)r.x * 3;
  uint8_t *d = dst + (long long)blockIdx.y * slot_bytes + (long long)row * pitch;
  for (int i = threadIdx.x; i < r.z * 3; i += 256) d[i] = s[i];
}

// ---- band assembly: OR a band's packed words into the frame's scan buffer ----
__global__ void k_or_words(uint32_t *dst, const uint32_t *src, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] |= src[i];
}

// All bands' pieces of all scans in one launch (mij_assemble_pieces): piece
// y = {frame * 3 + comp, first word in the scan, first source word, words};
// blockIdx.x strides over the piece's words
__global__ void k_or_pieces(uint32_t *raw, long long raw_fs, long long rw0, long long rw1,
                            const uint32_t *src, const unsigned long long *pieces) {
  const unsigned long long *pc = pieces + 4 * (long long)blockIdx.y;
  const long long fc = (long long)pc[0], n = (long long)pc[3];
  const long long f = fc / 3, c = fc - 3 * f;
  uint32_t *dst = raw + f * raw_fs + (c == 0 ? 0 : rw0 + (c == 2 ? rw1 : 0)) + (long long)pc[1];
  const uint32_t *sp = src + (long long)pc[2];
  // neighbouring bands share at most their boundary word, and their pieces
  // run concurrently: the first and last word of a piece are OR-ed atomically
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    if (i == 0 || i == n - 1) atomicOr(&dst[i], sp[i]);
    else dst[i] |= sp[i];
  }
}

// Band words out of the scan buffers, zeroed behind them (the band packing needs
// all-zero buffers): piece blockIdx.y = {frame * 3 + scan, words, first
// destination word}, from the start of the scan.
__global__ void k_move_pieces(uint32_t *raw, long long raw_fs, long long rw0, long long rw1,
                              uint32_t *dst, const unsigned long long *pieces, long long cap) {
  const unsigned long long *pc = pieces + 3 * (long long)blockIdx.y;
  const long long fc = (long long)pc[0], n = (long long)pc[1], d0 = (long long)pc[2];
  const long long f = fc / 3, c = fc - 3 * f;
  uint32_t *src = raw + f * raw_fs + (c == 0 ? 0 : rw0 + (c == 2 ? rw1 : 0));
  // four words per thread per round, loads first (a round costs one memory
  // latency, not four)
  const long long G = (long long)gridDim.x * blockDim.x;
  for (long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += 4 * G) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = i0 + u * G < n ? src[i0 + u * G] : 0u;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const long long i = i0 + u * G;
      if (i < n) {
        if (d0 + i < cap) dst[d0 + i] = v[u];  // (past the destination: dropped, still zeroed)
        src[i] = 0u;
      }
    }
  }
}
// ---- one large frame in bands, device-resident control (mij_band_*_async):
// the small per-frame values the bands exchange stay in HBM and these kernels
// turn them into the next step's arguments, so no step waits for the host.
// One thread per frame (n <= a batch's frames).

// the last raw DC of every component of frames 0..n-1 (the next band's
// predictors, encoder.c:168-177) -> last[f * 4 + c]
__global__ void k_band_last(const int16_t *dc, Geom g, int n, int16_t *last) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const long long fb = (long long)f * g.nblk;
  last[f * 4 + 0] = dc[fb + g.nY - 1];
  last[f * 4 + 1] = dc[fb + g.nY + g.nC - 1];
  last[f * 4 + 2] = dc[fb + g.nY + 2LL * g.nC - 1];
  last[f * 4 + 3] = 0;
}

// a band packed from bit 0 of every scan: its bits per scan (the pack's scan
// totals) -> bits[f * 3 + c], its word count -> bits[3n], and the (frame,
// scan)-ordered move table {frame * 3 + scan, words, first destination word}
// -> pieces
__global__ void k_band_count(const unsigned long long *scan_bits, int n, unsigned long long *pieces,
                             unsigned long long *bits) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned long long at = 0;
  for (int i = 0; i < 3 * n; i++) {
    const unsigned long long b = scan_bits[i], nw = (b + 31) >> 5;
    bits[i] = b;
    unsigned long long *pc = pieces + 3 * i;
    pc[0] = (unsigned long long)i;
    pc[1] = nw;
    pc[2] = at;
    at += nw;
  }
  bits[3 * n] = at;
}

// the root's assembly table from allbits[world][3n + 1] (k_band_count's
// output of every band) for a gathered buffer whose band-r row (stride words)
// holds that band's words in (frame, scan) order: piece (r, f, c) = {frame * 3
// + scan, first bit in the scan (the sum of the earlier bands' bits, encoder.c
// :462-502's running bit position), first source word, bits}; the scans'
// total bits -> scan_bits[f * 3 + c]
__global__ void k_band_assembly(const unsigned long long *allbits, int world, int n, unsigned long long stride,
                                unsigned long long *pieces, unsigned long long *scan_bits, int *over) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int i = 0; i < 3 * n; i++) scan_bits[i] = 0;
  bool overflow = false;
  for (int r = 0; r < world; r++) {
    const unsigned long long *rb = allbits + (long long)r * (3 * n + 1);
    unsigned long long at = 0;
    for (int i = 0; i < 3 * n; i++) {
      const unsigned long long off = scan_bits[i], bits = rb[i];
      unsigned long long *pc = pieces + 4 * ((long long)r * 3 * n + i);
      pc[0] = (unsigned long long)i;
      pc[1] = off;
      pc[2] = (unsigned long long)r * stride + at;
      pc[3] = bits;
      at += (bits + 31) >> 5;
      scan_bits[i] = off + bits;
    }
    overflow |= at > stride;
  }
  // a band's words beyond its row (the gather dropped them): fail the frames
  // and give every piece 0 bits, so k_or_shift_pieces reads and writes
  // nothing (its source offsets would run past the band's row, and for the
  // last band past the gathered buffer)
  if (overflow) {
    for (int f = 0; f < n; f++) over[f] = 1;
    for (long long k = 0; k < (long long)world * 3 * n; k++) pieces[4 * k + 3] = 0;
  }
}

// An upper bound of a band's words before it packs: its bits per frame are
// exactly the sum over its tokens of code length + magnitude bits (the low
// nibble of the symbol, encoder.c:385-423), i.e. its own histograms
// (hist[f][t][sym]) weighted by the tables' code lengths (ehuf, len << 16 |
// code); the three scans' words round up at most 3 words more.  A wave per
// frame; the workgroups' sums meet in acc = {sum, arrivals}, which the last
// workgroup to arrive reads, writes to bound[0] and leaves zeroed.  The
// histograms are left zeroed (each count by the lane that read it) for the
// band's next K1, which adds onto them.
__global__ __launch_bounds__(256) void k_band_bound(uint32_t *hist, const uint32_t *ehuf, int n,
                                                    unsigned long long *acc, unsigned long long *bound,
                                                    unsigned long long *pack_state, long long nstate,
                                                    unsigned *pack_ticket) {
  __shared__ unsigned long long s_w[4];
  // (the packing's look-back words and tickets zeroed here, saving two fills
  // on the band stream's critical path)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nstate; i += (long long)gridDim.x * 256)
    pack_state[i] = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < 3 * n; i += gridDim.x * 256) pack_ticket[i] = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, f = blockIdx.x * 4 + w;
  unsigned long long words = 0;
  if (f < n) {
    unsigned long long b = 0;
    for (int t = 0; t < 4; t++) {
      uint32_t *h = hist + ((long long)f * 4 + t) * 257;
      const uint32_t *e = ehuf + ((long long)f * 4 + t) * 256;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int s = 64 * k + lane;
        b += (unsigned long long)h[s] * ((e[s] >> 16) + (s & 15));
        h[s] = 0u;
      }
      if (lane == 0) h[256] = 0u;
    }
    for (int off = 32; off; off >>= 1) b += __shfl_xor(b, off);
    words = (b + 31) / 32 + 3;
  }
  if (lane == 0) s_w[w] = words;
  __syncthreads();
  if (threadIdx.x == 0) {
    // (the sum's add returns before the arrival is counted, and the last
    // arrival reads it by an atomic: both at the point where device-wide
    // atomics meet, so no cache-writeback fence is needed)
    const unsigned long long old = atomicAdd(&acc[0], s_w[0] + s_w[1] + s_w[2] + s_w[3]);
    asm volatile("" ::"v"(old));
    if (atomicAdd(&acc[1], 1ull) == gridDim.x - 1) {
      bound[0] = atomicExch(&acc[0], 0ull);
      atomicExch(&acc[1], 0ull);
    }
  }
}

// Every band's words OR-ed into the scans at their bit positions (one launch,
// piece blockIdx.y = {frame * 3 + scan, first bit in the scan, first source
// word, bits}): a band packed from bit 0 lands shifted right by its start
// bit's in-word offset (big-endian bit order), so scan word j of the piece
// takes the low bits of source word j - 1 and the high bits of word j.
// Neighbouring bands share at most their boundary word and run concurrently:
// a piece's first and last scan words are OR-ed atomically.
__global__ void k_or_shift_pieces(uint32_t *raw, long long raw_fs, long long rw0, long long rw1,
                                  const uint32_t *src, const unsigned long long *pieces) {
  const unsigned long long *pc = pieces + 4 * (long long)blockIdx.y;
  const long long fc = (long long)pc[0], bits = (long long)pc[3];
  if (!bits) return;
  const long long f = fc / 3, c = fc - 3 * f;
  const int sh = (int)(pc[1] & 31);
  const long long nsrc = (bits + 31) >> 5, ndst = (sh + bits + 31) >> 5;
  uint32_t *dst = raw + f * raw_fs + (c == 0 ? 0 : rw0 + (c == 2 ? rw1 : 0)) + (long long)(pc[1] >> 5);
  const uint32_t *sp = src + (long long)pc[2];
  const long long G = (long long)gridDim.x * blockDim.x;
  for (long long j0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; j0 < ndst; j0 += 4 * G) {
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const long long j = j0 + u * G;
      hi[u] = j < nsrc ? sp[j] : 0u;
      lo[u] = j > 0 && j <= nsrc ? sp[j - 1] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const long long j = j0 + u * G;
      if (j < ndst) {
        uint32_t v = hi[u] >> sh;
        if (sh) v |= lo[u] << (32 - sh);
        if (j == 0 || j == ndst - 1) atomicOr(&dst[j], v);
        else dst[j] = v;
      }
    }
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
template <int MODE>
static int k1_blocks_per_cu() {
  static int nb = -1;
  if (nb < 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_mcu_dct<MODE>, 64 * k1_waves<MODE>(), 0) != hipSuccess ||
        nb < 1)
      nb = 1;
  }
  return nb;
}

// persistent grid for a K1 variant: at most (resident blocks per CU) x CUs
int k1_grid(int device, long long ntiles, int mode) {
  int per_cu = 1, nw = 4;
  switch (mode) {
    case K1M_COEF_OUT:
    case K1M_COEF_OUT | K1M_FLOOR:  // (the grid of the variant it stands for)
      per_cu = k1_blocks_per_cu<K1M_COEF_OUT>();
      nw = k1_waves<K1M_COEF_OUT>();
      break;
    case K1M_TOK_OUT:
      per_cu = k1_blocks_per_cu<K1M_TOK_OUT>();
      nw = k1_waves<K1M_TOK_OUT>();
      break;
    case K1M_COEF_OUT | K1M_TOK_OUT: per_cu = k1_blocks_per_cu<K1M_COEF_OUT | K1M_TOK_OUT>(); break;
    default: per_cu = k1_blocks_per_cu<K1M_COEF_IN | K1M_TOK_OUT>(); break;
  }
  static int cus = -1;
  if (cus < 0) {
    hipDeviceProp_t prop;
    cus = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  // MIJ_K1_GRID_MULT (diag build, A/B timing): workgroups per resident slot
#ifdef MIJ_K1_DIAG
  static const int mult = getenv("MIJ_K1_GRID_MULT") ? atoi(getenv("MIJ_K1_GRID_MULT")) : 1;
#else
  constexpr int mult = 1;
#endif
  long long want = (ntiles + nw - 1) / nw;
  long long cap = (long long)cus * per_cu * (mult > 0 ? mult : 1);
  // too few tiles to give every wave of a full grid one (a single 1920x1280
  // frame: 1,200 tiles): spread them over every CU's workgroup slot instead
  // of filling a few CUs' waves -- a tile's time is then its own wave's
  // issue, not three waves' sharing one SIMD
  if (want < cap) want = ntiles < cap ? ntiles : cap;
  return (int)(want < cap ? want : cap);
}

hipError_t launch_fix_blocks(const K1Args &a, hipStream_t s) {
  // a persistent grid over the fix masks: 64 masks per wave step
  const long long steps = ((long long)a.nframes * a.g.tiles_per_frame * 3 + 255) / 256;
  hipLaunchKernelGGL(k_fix_blocks, dim3((unsigned)(steps < 4096 ? steps : 4096)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_colour_lut(uint32_t *lut, hipStream_t s) {
  hipLaunchKernelGGL(k_colour_lut, dim3(128), dim3(256), 0, s, lut);
  return hipGetLastError();
}
// mode: K1M_* bits (see k_mcu_dct)
template <int MODE>
static void launch_k1_mode(const K1Args &a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((k_mcu_dct<MODE>), dim3(grid), dim3(64 * k1_waves<MODE>()), 0, s, a);
}
// diagnostics: an empty kernel (dispatch-gap probes, MIJ_NOP_AFTER_K1 in the diag build)
hipError_t launch_k1(const K1Args &a, int grid, int mode, hipStream_t s) {
  if (a.rgb && a.fdims) return hipErrorInvalidValue;  // not instantiated (the API refuses it)
  switch (mode) {
    case K1M_COEF_OUT:
      if (a.audit) {
        if (a.rgb || a.fdims) return hipErrorInvalidValue;  // tests audit plain B, G, R batches
        launch_k1_mode<K1M_COEF_OUT | K1M_AUDIT>(a, grid, s);
      } else if (a.rgb) launch_k1_mode<K1M_COEF_OUT | K1M_RGB>(a, grid, s);
      else if (a.fdims) launch_k1_mode<K1M_COEF_OUT | K1M_REGIONS>(a, grid, s);
      else launch_k1_mode<K1M_COEF_OUT>(a, grid, s);
      break;
    case K1M_COEF_OUT | K1M_FLOOR:
      if (a.rgb || a.fdims) return hipErrorInvalidValue;  // (plain B, G, R batches only)
      launch_k1_mode<K1M_COEF_OUT | K1M_FLOOR>(a, grid, s);
      break;
    case K1M_TOK_OUT:
      if (a.rgb) launch_k1_mode<K1M_TOK_OUT | K1M_RGB>(a, grid, s);
      else if (a.fdims) launch_k1_mode<K1M_TOK_OUT | K1M_REGIONS>(a, grid, s);
      else launch_k1_mode<K1M_TOK_OUT>(a, grid, s);
      break;
    case K1M_COEF_OUT | K1M_TOK_OUT:
      if (a.rgb) launch_k1_mode<K1M_COEF_OUT | K1M_TOK_OUT | K1M_RGB>(a, grid, s);
      else if (a.fdims) launch_k1_mode<K1M_COEF_OUT | K1M_TOK_OUT | K1M_REGIONS>(a, grid, s);
      else launch_k1_mode<K1M_COEF_OUT | K1M_TOK_OUT>(a, grid, s);
      break;
    case K1M_COEF_IN | K1M_TOK_OUT:
      if (a.fdims) launch_k1_mode<K1M_COEF_IN | K1M_TOK_OUT | K1M_REGIONS>(a, grid, s);
      else launch_k1_mode<K1M_COEF_IN | K1M_TOK_OUT>(a, grid, s);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_seg_dc(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_dc, dim3(a.nframes * ((a.g.nseg + SEGDC_WG - 1) / SEGDC_WG)), dim3(SEGDC_WG),
                     0, s, a);
  return hipGetLastError();
}
hipError_t launch_dc_diff(int16_t *coef, const int16_t *dc, const Geom &g, int nframes,
                          const int2 *fd, hipStream_t s) {
  long long n = (long long)nframes * g.nblk;
  hipLaunchKernelGGL(k_dc_diff, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, coef, dc, g,
                     nframes, fd);
  return hipGetLastError();
}
hipError_t launch_segdc_actab(const EntArgs &a, hipStream_t s) {
  const dim3 grid(a.nframes * (2 + (a.g.nseg + SEGDC_WG - 1) / SEGDC_WG));
  if (a.dc_last) hipLaunchKernelGGL(k_segdc_actab<true>, grid, dim3(SEGDC_WG), 0, s, a);
  else hipLaunchKernelGGL(k_segdc_actab<false>, grid, dim3(SEGDC_WG), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_tables(const EntArgs &a, hipStream_t s) {
  if (!a.seg_dc) {
    hipLaunchKernelGGL(k_tables_1w, dim3(a.nframes * (a.tab_dc_only ? 2 : 4)), dim3(64), 0, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_tables, dim3(a.nframes), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_ehuf_struct(const HuffCode *hc, uint32_t *ehuf, hipStream_t s) {
  hipLaunchKernelGGL(k_ehuf_struct, dim3(4), dim3(256), 0, s, hc, ehuf);
  return hipGetLastError();
}
hipError_t launch_bits(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_bits, dim3(a.nframes * ((a.g.nseg + SEG_PER_WG - 1) / SEG_PER_WG)),
                     dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_scan(const EntArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_scan, dim3(a.nframes * 3), dim3(64), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_or_words(uint32_t *dst, const uint32_t *src, long long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_or_words, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

hipError_t launch_or_pieces(uint32_t *raw, const Geom &g, const uint32_t *src,
                            const unsigned long long *d_pieces, int npieces, long long max_words, hipStream_t s) {
  if (npieces <= 0 || max_words <= 0) return hipSuccess;
  const long long chunks = (max_words + 1023) / 1024;
  hipLaunchKernelGGL(k_or_pieces, dim3((unsigned)(chunks < 64 ? chunks : 64), (unsigned)npieces), dim3(256), 0, s,
                     raw, g.raw_fs, g.raw_words[0], g.raw_words[1], src, d_pieces);
  return hipGetLastError();
}

hipError_t launch_move_pieces(uint32_t *raw, const Geom &g, uint32_t *dst,
                              const unsigned long long *d_pieces, int npieces, long long max_words, long long cap,
                              hipStream_t s) {
  if (npieces <= 0 || max_words <= 0) return hipSuccess;
  const long long chunks = (max_words + 1023) / 1024;
  hipLaunchKernelGGL(k_move_pieces, dim3((unsigned)(chunks < 256 ? chunks : 256), (unsigned)npieces), dim3(256), 0, s,
                     raw, g.raw_fs, g.raw_words[0], g.raw_words[1], dst, d_pieces, cap);
  return hipGetLastError();
}

hipError_t launch_band_last(const int16_t *dc, const Geom &g, int n, int16_t *last, hipStream_t s) {
  hipLaunchKernelGGL(k_band_last, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, dc, g, n, last);
  return hipGetLastError();
}
hipError_t launch_band_bound(const EntArgs &a, unsigned long long *acc, unsigned long long *bound, hipStream_t s) {
  const int n = a.nframes;
  const long long nstate = (long long)n * pack_stride(a.g);
  const unsigned grid = (unsigned)std::max((n + 3) / 4, (int)std::min<long long>((nstate + 255) / 256, 64));
  hipLaunchKernelGGL(k_band_bound, dim3(grid), dim3(256), 0, s, a.hist, a.ehuf, n, acc, bound, a.pack_state, nstate,
                     a.pack_ticket);
  return hipGetLastError();
}
hipError_t launch_band_count(const unsigned long long *scan_bits, int n, unsigned long long *pieces,
                             unsigned long long *bits, hipStream_t s) {
  hipLaunchKernelGGL(k_band_count, dim3(1), dim3(64), 0, s, scan_bits, n, pieces, bits);
  return hipGetLastError();
}
hipError_t launch_band_assembly(const unsigned long long *allbits, int world, int n, unsigned long long stride,
                                unsigned long long *pieces, unsigned long long *scan_bits, int *over, hipStream_t s) {
  hipLaunchKernelGGL(k_band_assembly, dim3(1), dim3(64), 0, s, allbits, world, n, stride, pieces, scan_bits, over);
  return hipGetLastError();
}
hipError_t launch_or_shift_pieces(uint32_t *raw, const Geom &g, const uint32_t *src,
                                  const unsigned long long *d_pieces, int npieces, long long max_words, hipStream_t s) {
  if (npieces <= 0 || max_words <= 0) return hipSuccess;
  const long long chunks = (max_words + 1 + 1023) / 1024;
  hipLaunchKernelGGL(k_or_shift_pieces, dim3((unsigned)(chunks < 256 ? chunks : 256), (unsigned)npieces), dim3(256), 0,
                     s, raw, g.raw_fs, g.raw_words[0], g.raw_words[1], src, d_pieces);
  return hipGetLastError();
}

hipError_t launch_pack(const EntArgs &a, hipStream_t s, bool state_zeroed) {
  const long long groups = (long long)a.nframes * pack_grid(a).gpf;
  if (!state_zeroed) {
    hipError_t e = hipMemsetAsync(a.pack_state, 0, sizeof(unsigned long long) * a.nframes * pack_stride(a.g), s);
    if (e == hipSuccess) e = hipMemsetAsync(a.pack_ticket, 0, sizeof(unsigned) * 3 * a.nframes, s);
    if (e != hipSuccess) return e;
  }
  const bool ff = a.ff_pack && a.seam;
  if (a.pack_wide && ff) hipLaunchKernelGGL((k_pack_flat<PACK_WIDE_WORDS, true>), dim3((unsigned)groups), dim3(PF_THREADS), 0, s, a);
  else if (a.pack_wide) hipLaunchKernelGGL((k_pack_flat<PACK_WIDE_WORDS, false>), dim3((unsigned)groups), dim3(PF_THREADS), 0, s, a);
  else if (ff) hipLaunchKernelGGL((k_pack_flat<PACK_WORDS, true>), dim3((unsigned)groups), dim3(PF_THREADS), 0, s, a);
  else hipLaunchKernelGGL((k_pack_flat<PACK_WORDS, false>), dim3((unsigned)groups), dim3(PF_THREADS), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_seam_fix(const EntArgs &a, hipStream_t s) {
  const long long n = (long long)a.nframes * pack_grid(a).gpf;
  hipLaunchKernelGGL(k_seam_fix, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_emit(const EntArgs &a0, hipStream_t s) {
  EntArgs a = a0;
  if (a.emit_slots < 1) a.emit_slots = EMIT_SLOTS;
  if (!a.ff_pack)  // (ff_pack: the packing counted the 0xFF bytes)
    hipLaunchKernelGGL(k_emit_count, dim3(a.nframes * a.emit_slots), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_emit_scan, dim3(a.nframes), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_emit_write, dim3(a.nframes * a.emit_slots), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_band_stuff(const EntArgs &a0, const unsigned long long *allbits, int world, int rank,
                             unsigned long long *rec, unsigned long long *total, uint8_t *dst, unsigned long long cap,
                             hipStream_t s) {
  EntArgs a = a0;
  if (a.emit_slots < 1) a.emit_slots = EMIT_SLOTS;
  const int ns = 3 * a.nframes;
  hipLaunchKernelGGL(k_band_stuff_prep, dim3((ns + 63) / 64), dim3(64), 0, s, a, allbits, world, rank, rec);
  hipLaunchKernelGGL(k_band_count_ff, dim3(a.nframes * a.emit_slots), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_band_stuff_scan, dim3(1), dim3(256), 0, s, a, rec, total);
  hipLaunchKernelGGL(k_band_write, dim3(a.nframes * a.emit_slots), dim3(256), 0, s, a, dst, cap);
  hipLaunchKernelGGL(k_band_zero, dim3(64, ns), dim3(256), 0, s, a, rec);
  return hipGetLastError();
}
hipError_t launch_band_join(const EntArgs &a, const unsigned long long *allrec, int world, unsigned long long stride,
                            unsigned long long *pieces, const uint8_t *src, hipStream_t s) {
  hipLaunchKernelGGL(k_band_join, dim3(a.nframes), dim3(256), 0, s, a, allrec, world, stride, pieces);
  hipLaunchKernelGGL(k_copy_bytes, dim3(64, a.nframes * world * 3), dim3(256), 0, s, a.out, src,
                     (const unsigned long long *)pieces);
  return hipGetLastError();
}
hipError_t launch_gather_regions(uint8_t *dst, long long slot_bytes, int pitch, const uint8_t *src,
                                 long long src_pitch, const int4 *regions, int n, int max_h,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_gather_regions, dim3(max_h, n), dim3(256), 0, s, dst, slot_bytes, pitch, src,
                     src_pitch, regions);
  return hipGetLastError();
}
hipError_t launch_mfma_probe(const int4 *A, const int4 *B, int4 *D, hipStream_t s) {
  hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, s, A, B, D);
  return hipGetLastError();
}

}  // namespace mij
