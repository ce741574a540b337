// mij_internal.h -- shared definitions between the gfx950 kernels
// (mij_kernels.hip) and the host runtime (mij_api.hip).  Not a public header:
// the C ABI lives in include/mijpeg.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "mij_divmagic.h"

namespace mij {

// ---- tiling of the fused colour+DCT kernel (K1) ---------------------------
// One wave owns a 128x16-pixel tile = 8 MCUs = 32 Y blocks (two block rows of
// 16) + 8 Cb + 8 Cr blocks: exactly three 16-block MFMA N-tiles.
constexpr int TILE_W = 128;
constexpr int TILE_H = 16;
constexpr int LDS_BLK = 80;          // bytes per staged 8x8 block (64 + pad)
constexpr int LDS_WAVE = 48 * LDS_BLK;  // 32 Y + 16 chroma blocks per wave
constexpr int LUT_WORDS = 1024;      // 2^15 bits per colour-exception table
constexpr int DCTIE_WORDS = 33;      // DC tie bits for K = 0..1055 (|S| <= 8192 -> K <= 1024)

// ---- per-frame device error codes (EntArgs::err) ---------------------------
constexpr int FERR_TABLE = 1;     // Huffman construction outside the reference's defined behaviour
constexpr int FERR_OVERFLOW = 2;  // bits past a scan buffer (tokens no K1 wrote): nothing written
constexpr int FERR_ASSEMBLY = 3;  // band assembly: a piece outside its buffer
// option slot 7 (reserved in include/mijpeg.h): the test suite's stale-ticket
// fault, armed only through mij_test_stale_ticket (csrc/mij_testing.h)
constexpr int OPT_TEST_FAULT_TICKET = 7;
constexpr int FERR_SPIN = 4;      // a device-side wait outlasted SPIN_TICKS, or a stale pack ticket
// bound of every device-side wait without progress (s_memrealtime ticks,
// 100 MHz: 2 s); the waits are microseconds long when the state they wait on
// is intact, and the bound is long enough for a queue switched out under
// multi-process time-slicing (the pack look-back restarts it whenever a
// predecessor's state word changes)
constexpr unsigned long long SPIN_TICKS = 200000000ull;

// ---- entropy stage: segments ---------------------------------------------
// A segment is the run of blocks one K1 N-tile covers in a component's scan
// order: 16 luma blocks of a block row, or 8 Cb / 8 Cr blocks of an MCU row.
// K1 writes each segment's tokens compacted into a slot of SEG_TOK tokens;
// k_pack packs PACK_SEGS consecutive segments of a scan per workgroup.
constexpr int MAX_BLOCK_TOK = 65;                 // DC + 63 AC + EOB
constexpr int SEG_TOK = 16 * MAX_BLOCK_TOK;       // 1040 tokens per segment slot
constexpr int SEG_PER_WG = 64;                    // k_seg_bits segments per workgroup
constexpr int PACK_SEGS = 32;          // segments per k_pack workgroup at pack_ls 0
constexpr int PACK_LS_MAX = 3;         // pack groups of 32 << ls segments, ls <= 3
constexpr int PACK_SEGS_MAX = PACK_SEGS << PACK_LS_MAX;
constexpr int MAX_BLOCK_BITS = 1729;              // 28 DC + 63 * 27 AC bits
// k_pack assembles a group in LDS windows of PACK_WORDS words; a group wider
// than one window (only near worst-case entropy) is packed in several passes.
constexpr int PACK_WORDS = 4096;
// the window of the high-quality variant (EntArgs::pack_wide, Q >= 85)
constexpr int PACK_WIDE_WORDS = 5888;  // (6 workgroups per CU by LDS)
static_assert(PACK_WIDE_WORDS > PACK_WORDS, "the wide pack window must be wider than the default one");
constexpr int PACK_WIDE_MIN_Q = 85;  // qualities from which the wide window is launched
// JFIF assembly: scans are written in EMIT_CH-byte chunks by EntArgs::
// emit_slots workgroups per frame, EMIT_SLOTS when unset (round 2's A/B per scan on config 3,
// emit = count + scan + write: 8 slots 0.260 ms, 16 0.232, 32 0.243,
// 64 0.247, 128 0.269, 256 0.321; profiles/r02/emit_slots_ab.txt).  Round 3
// (seam mode, chunks dealt over the frame's scans, profiles/r03/seam/
// emit_ab.txt): 8 KB chunks 0.190 ms at Q=50 and 0.549 at Q=90 against
// 0.210 / 0.639 with 4 KB; 16 KB chunks 0.29 / 0.80.
constexpr int EMIT_CH = 8192;
constexpr int EMIT_SLOTS = 192;

// Layout-identical to the reference huff_code (include/structs.h:5-13).
struct HuffCode {
  int sym_freq[257];
  int code_len[257];
  int next[257];
  int code_len_freq[32];
  int sym_sorted[256];
  int sym_code_len[256];
  int sym_code[256];
};
static_assert(sizeof(HuffCode) == 6284, "huff_code layout");

// Geometry of one frame (region) as the kernels see it.
struct Geom {
  int w, h;             // multiples of 16
  int nY, nC, nblk;     // 8x8 blocks: luma, per chroma plane, total
  int tiles_x, tiles_per_frame;
  int nsy, nsc, nseg;   // segments: luma, per chroma plane, per frame
  long long coef_fs;    // coefficient elements per frame = nblk * 64
  long long raw_words[3];   // raw bit-buffer capacity per component (words)
  long long raw_fs;         // words per frame
  long long out_cap;        // output bytes per frame
  // n / tiles_per_frame and n / tiles_x for 0 <= n < 2^31 as
  // (umulhi(n, m) + n) >> s (K1's per-tile position on the scalar unit)
  uint32_t tpf_m, tpf_s, tx_m, tx_s;
};



// The image of frame f of a batch.  Buffers are laid out for the batch
// geometry G (the "canvas"); a region batch (mij_batch_set_frame_dims) holds
// smaller frames, each w x h at the top-left of its canvas slot: its blocks
// are numbered in its own raster order (per-frame bw, nY, nC), its tiles and
// segments keep the canvas numbering (tiles / segments outside the frame are
// skipped and hold no tokens).  fd == nullptr: every frame is the canvas.
struct FGeom {
  int w, h, bw, mw, nY, nC, tiles_x, rows;  // rows = MCU rows = tile rows
};
__host__ __device__ inline FGeom frame_geom(const Geom &G, const int2 *fd, int f) {
  FGeom r;
  if (!fd) {  // the canvas: the Geom fields themselves (kernel arguments the
              // compiler can reload instead of keeping them in registers)
    r.w = G.w;
    r.h = G.h;
    r.bw = G.w >> 3;
    r.mw = G.w >> 4;
    r.nY = G.nY;
    r.nC = G.nC;
    r.tiles_x = G.tiles_x;
    r.rows = G.h / TILE_H;
    return r;
  }
#ifdef __HIP_DEVICE_COMPILE__
  // f is wave-uniform wherever this is called: keep the sizes in SGPRs
  const int w = __builtin_amdgcn_readfirstlane(fd[f].x), h = __builtin_amdgcn_readfirstlane(fd[f].y);
#else
  const int w = fd[f].x, h = fd[f].y;
#endif
  r.w = w;
  r.h = h;
  r.bw = w >> 3;
  r.mw = w >> 4;
  r.nY = (w >> 3) * (h >> 3);
  r.nC = (w >> 4) * (h >> 4);
  r.tiles_x = (w + TILE_W - 1) / TILE_W;
  r.rows = h / TILE_H;
  return r;
}

// Device-resident constant tables for one quality setting.
struct Tables {
  int4 mfma_a[12 * 64];   // A fragments: 4 M-tiles x 3 digits x 64 lanes
  // K1's quantisation: the A rows are prescaled for the
  // luma table, row z by 2^s_g / q_z with s_g = floor(log2(the smallest luma
  // AC quantiser of zigzag group g = z / 16)), so a luma N' is 2^(21 + s_g)
  // t to within L1 / 2 and truncates by a shift (kq[g] = 21 + s_g); chroma
  // keeps an fp32 factor: qfac[1][z] = q_luma(z) / (2^(21 + s_g) q_chroma(z))
  float qfac[2][64];      // zigzag order; [0]: unused (luma is integer), [1]: chroma factor
  int kq[4];              // luma shift per zigzag group of 16
  int qint[2][64];        // zigzag order: integer quantizer
  int dqt[2][64];         // zigzag order: DQT bytes
  double cosd[64];        // encoder.c:8-16 constants
  uint32_t lut[3][1024];  // colour-exception bitmaps (Y by R,G/2; Cb by G,B/2; Cr by G,R/2)
  uint32_t dctie[2][DCTIE_WORDS];  // bit K: the reference's DC at |S| = 8qK is K - 1
  // K1's chroma all-AC-zero test: per zigzag z the limit L_z = (1 - 2e-6) /
  // qfac[1][z] - 6000 under which |N'| means the reference's |F/q| < 1 (z = 0,
  // the DC, never fails: 2^30); cz_on = 0 where all-zero chroma N-tiles are
  // too rare to pay for the test (Q > 75)
  int czl[64];
  int cz_on;
};

struct K1Args {
  const uint8_t *in;        // origin of frame 0's region, 4-byte aligned
  long long in_fs;          // bytes between frames
  int pitch;                // bytes per input row (multiple of 4)
  int nframes;
  Geom g;
  int16_t *coef;            // per frame: Y[nY*64] Cb[nC*64] Cr[nC*64], zigzag
  int16_t *dc;              // per frame: raw (un-differenced) DC per block
  const Tables *tab;
  unsigned int *replays;    // count of coefficients replayed in FP64
  int flags;                // diagnostics only (MIJ_K1_FLAGS): K1F_* bits
  int per_wg;               // tiles per workgroup (<= tiles_per_frame)
  int dc_diffed;            // coefficient input holds DC differences (drop-in)
  int seg_dc_inline;        // coefficient input: first DC of each segment from the raw DCs
  const int16_t *dc_pred;   // coefficient input, inline: DC predictor per frame [4] (null: 0)
  uint32_t *tok;            // token mode: per segment SEG_TOK tokens (token 0 in tok0)
  uint32_t *tok0;           // token mode: per segment its first token (the first block's DC)
  uint32_t *seg_ntok;       // token mode: tokens per segment
  uint32_t *hist;           // token mode: per frame [4][257] histograms
  // coefficient mode: per K1 N-tile (global tile * 3 + nt) the 16-bit mask of
  // its blocks k_fix_blocks must recompute; all zero between launches (K1
  // stores only nonzero masks, k_fix_blocks zeroes what it consumes)
  uint16_t *fix_mask;
  unsigned long long *wtime;  // diagnostics only (MIJ_K1_WTIME): per wave start, end, tiles,
                              // then 5 phase times (K1_WTIME_WORDS words per wave)
  int rgb;                  // input bytes in R, G, B order (PPM) instead of B, G, R
  const int2 *fdims;        // per-frame image size (region batches), null: the canvas
  uint16_t *audit;          // tests (mij_batch_audit): per frame, block, lane group g the 16
                            // straddle bits of zigzag 16g..16g+15; null in every product launch
  int *err_zero;            // an encode's first K1: workgroup 0 zeroes these per-frame error
  int nerr_zero;            // words (k_tables on write them), instead of a memset launch
};
constexpr int K1_WTIME_WORDS = 8;
// K1 diagnostic switches (timing attribution; outputs are wrong when set)
constexpr int K1F_NO_LUT = 1, K1F_NO_REPLAY = 2, K1F_NO_COLOUR = 4, K1F_NO_DCT = 8,
              K1F_NO_STORE = 16, K1F_NO_QUANT = 32, K1F_NO_MFMA = 64,
              K1F_LINEAR_STORE = 128, K1F_PLAIN_STORE = 256,
              K1F_NO_HIST = 512, K1F_NO_TOKSTORE = 1024,
              K1F_EXTRA_LDS = 2048, K1F_NO_EMIT = 4096, K1F_NO_ACLOOP = 8192,
              K1F_NO_DMAWAIT = 16384,
              K1F_REPLAY_NO_FP64 = 32768,  // replay pass without its FP64 rounds
              K1F_COUNT_PASSES = 65536,    // the replay counter counts passes
              K1F_COUNT_LUMA = 131072;     // ... and replays of luma N-tiles only

struct EntArgs {
  Geom g;
  int nframes;
  const int16_t *coef;
  const int16_t *dc;        // raw DC per block (K1)
  uint32_t *hist;           // per frame [4][257]
  const uint32_t *ehuf;     // per frame [4][256] = len << 16 | code
  uint32_t *tok;            // per segment SEG_TOK tokens (token 0 in tok0)
  uint32_t *tok0;           // per segment its first token
  const uint32_t *seg_ntok; // per segment token count
  uint32_t *seg_bits;       // per segment bits
  uint64_t *seg_off;        // per segment bit offset inside its scan
  uint64_t *scan_bits;      // per frame [3]
  uint32_t *raw;            // per frame: 3 component bit buffers (big-endian words)
  const HuffCode *hc;       // per frame [4]
  const Tables *tab;
  uint8_t *out;             // per frame out_cap bytes
  uint64_t *out_len;        // per frame
  int *err;                 // per frame error flag
  // one large frame split into bands (mij_band_*): per frame [4]
  const int16_t *dc_pred;   // DC predictor of each component's first block (null: 0)
  const uint32_t *bit_base; // bit offset of each scan inside its first word (null: 0)
  uint32_t *ffc;            // per frame [3][emit_chunks]: 0xFF bytes per EMIT_CH chunk
  uint32_t *choff;          // per frame [3][emit_chunks]: output offset of each chunk (inside
                            // its frame; band stuffing: inside its scan, see scan_base)
  uint64_t *scan_base;      // per frame [3]: band stuffing, a scan's first byte in the band's buffer
  unsigned long long *pack_state;  // k_pack_flat: per pack group, flag << 62 | bits
  unsigned int *pack_ticket;       // k_pack_flat: next group to claim, per scan
  unsigned long long *dbg;         // diagnostics only (MIJ_PACK_TIME, diag build)
  const int2 *fdims;               // per-frame image size (region batches), null: the canvas
  uint32_t *seam;                  // per pack group: its first word when shared with the group
                                   // before it (null: edge words OR-ed onto all-zero scan buffers;
                                   // set: k_seam_fix ORs them in, nothing needs zeroed buffers)
  int emit_slots;                  // k_emit_count / k_emit_write workgroups per frame (0: EMIT_SLOTS)
  int pack_wide;                   // k_pack_flat with a 2 * PACK_WORDS window (high quality)
  int pack_ls[2];                  // k_pack_flat groups: 32 << pack_ls[chroma] segments of a scan
  int zero_pack;                   // k_tables_1w also zeroes k_pack_flat's look-back words and tickets
  int seg_dc;                      // k_tables: compute the segment-first DC tokens first (k_seg_dc)
  int tab_dc_only;                 // k_tables_1w: the DC tables only (k_segdc_actab built the AC ones)
  int dc_last;                     // k_segdc_actab: a frame's last segment-DC workgroup builds its two
                                   // DC tables (and zeroes the pack state): no k_tables_1w launch
  uint32_t *dcx;                   // dc_last: per frame 64 words -- the segment-first DCs' class
                                   // counts [luma, chroma][16] and the arrivals [32]; left zeroed
  int ff_pack;                     // seam mode: k_pack_flat / k_seam_fix count the 0xFF bytes of every
                                   // EMIT_CH chunk into ffc as they store (k_emit_count not run;
                                   // k_emit_write leaves the counts zeroed)
  int seam_in_scan;                // seam mode with ff_pack: k_emit_scan fixes its frame's seams
                                   // first, no k_seam_fix launch (small batches: one launch fewer;
                                   // on large ones the per-frame serial fixes cost more than it)
};

// The packing's groups (k_pack_flat, k_seam_fix): per frame gy luma groups,
// then gc Cb and gc Cr, of 32 << pack_ls[chroma] segments each; their
// per-group arrays (pack_state, seam) keep the stride of the 32-segment
// groups whatever the group size, so per-frame offsets do not depend on it.
struct PackGrid {
  int gy, gc, gpf, stride;
};
__host__ __device__ inline int pack_groups(int ns, int ls) { return (ns + (PACK_SEGS << ls) - 1) >> (5 + ls); }
__host__ __device__ inline int pack_stride(const Geom &g) { return pack_groups(g.nsy, 0) + 2 * pack_groups(g.nsc, 0); }
__host__ __device__ inline PackGrid pack_grid(const EntArgs &a) {
  PackGrid p;
  p.gy = pack_groups(a.g.nsy, a.pack_ls[0]);
  p.gc = pack_groups(a.g.nsc, a.pack_ls[1]);
  p.gpf = p.gy + 2 * p.gc;
  p.stride = pack_stride(a.g);
  return p;
}


// EMIT_CH chunks of the largest scan buffer (the per-scan stride of EntArgs::ffc)
__host__ __device__ inline long long emit_chunks(const Geom &g) {
  return (g.raw_words[0] * 4 + EMIT_CH - 1) / EMIT_CH;
}

}  // namespace mij
