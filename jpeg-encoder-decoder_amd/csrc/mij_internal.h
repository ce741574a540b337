// mij_internal.h -- shared definitions between the gfx950 kernels
// (mij_kernels.hip) and the host runtime (mij_api.hip).  Not a public header:
// the C ABI lives in include/mijpeg.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mij {

// ---- tiling of the fused colour+DCT kernel (K1) ---------------------------
// One wave owns a 128x16-pixel tile = 8 MCUs = 32 Y blocks (two block rows of
// 16) + 8 Cb + 8 Cr blocks: exactly three 16-block MFMA N-tiles.
constexpr int TILE_W = 128;
constexpr int TILE_H = 16;
constexpr int LDS_BLK = 80;          // bytes per staged 8x8 block (64 + pad)
constexpr int LDS_WAVE = 48 * LDS_BLK;  // 32 Y + 16 chroma blocks per wave
constexpr int K1_WAVES = 4;

// ---- entropy stage chunking -----------------------------------------------
// A chunk is CHUNK consecutive blocks of ONE component of ONE frame; it is the
// work unit of the statistics / bit-count / pack kernels and the unit of the
// per-scan offset scan.
constexpr int CHUNK = 256;
constexpr int MAX_BLOCK_BITS = 1729;  // 28 DC + 63 * 27 AC bits
// LDS words a chunk may need when packed (+2 for the unaligned head/tail)
constexpr int CHUNK_WORDS = (CHUNK * MAX_BLOCK_BITS + 31) / 32 + 2;

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
  int cy, cc, cpf;      // chunks: luma, per chroma plane, per frame
  long long coef_fs;    // coefficient elements per frame = nblk * 64
  long long raw_words[3];   // raw bit-buffer capacity per component (words)
  long long raw_fs;         // words per frame
  long long out_cap;        // output bytes per frame
};

// Device-resident constant tables for one quality setting.
struct Tables {
  int4 mfma_a[12 * 64];   // A fragments: 4 M-tiles x 3 digits x 64 lanes
  float qfac[2][64];      // zigzag order: 1 / (2^21 * q)
  float qtau[2][64];      // zigzag order: proven error bound (t units)
  int qint[2][64];        // zigzag order: integer quantizer
  int dqt[2][64];         // zigzag order: DQT bytes
  double cosd[64];        // encoder.c:8-16 constants
  uint32_t lut[3][2048];  // colour-exception bitmaps (Y by R,G; Cb by G,B; Cr by G,R)
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
};

struct EntArgs {
  Geom g;
  int nframes;
  const int16_t *coef;
  const int16_t *dc;        // raw DCs (dc_mode 0)
  int dc_mode;              // 0: DC raw, diff from dc[]; 1: coef holds DC diff
  uint32_t *hist;           // per frame [4][257]
  const uint32_t *ehuf;     // per frame [4][256] = len << 16 | code
  uint32_t *tok;            // per block 64 tokens (k_tokens)
  uint8_t *hdr;             // per block: #AC tokens | EOB << 7
  uint32_t *bits;           // per block (frame-major)
  uint64_t *chunk_bits;     // per chunk
  uint64_t *chunk_off;      // per chunk: bit offset inside its scan
  uint64_t *scan_bits;      // per frame [3]
  uint32_t *raw;            // per frame: 3 component bit buffers (big-endian words)
  const HuffCode *hc;       // per frame [4]
  const Tables *tab;
  uint8_t *out;             // per frame out_cap bytes
  uint64_t *out_len;        // per frame
  int *err;                 // per frame error flag
};

}  // namespace mij
