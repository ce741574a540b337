// mij_api.hip -- host runtime and C ABI of libmijpeg.so (include/mijpeg.h).
//
// The drop-in entry points rgb_to_dct / init_huffman / write_jpg keep the
// reference's signatures (include/encoder.h:10-12) and run every stage as a
// HIP kernel (mij_kernels.hip).  The batch API keeps frames, coefficients and
// bitstreams resident in HBM and is what bench.py measures.
#include <math.h>
#include <stdarg.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "mij_host.h"
#include "mij_internal.h"
#include "mijpeg.h"
#include "mij_testing.h"

namespace mij {
// launch wrappers (mij_kernels.hip)
int k1_grid(int device, long long ntiles, int mode);
hipError_t launch_colour_lut(uint32_t *lut, hipStream_t s);
hipError_t launch_k1(const K1Args &a, int grid, int mode, hipStream_t s);
hipError_t launch_fix_blocks(const K1Args &a, hipStream_t s);
hipError_t launch_seg_dc(const EntArgs &a, hipStream_t s);
hipError_t launch_segdc_actab(const EntArgs &a, hipStream_t s);
hipError_t launch_dc_diff(int16_t *coef, const int16_t *dc, const Geom &g, int nframes,
                          const int2 *fd, hipStream_t s);
hipError_t launch_tables(const EntArgs &a, hipStream_t s);
hipError_t launch_ehuf_struct(const HuffCode *hc, uint32_t *ehuf, hipStream_t s);
hipError_t launch_bits(const EntArgs &a, hipStream_t s);
hipError_t launch_scan(const EntArgs &a, hipStream_t s);
hipError_t launch_pack(const EntArgs &a, hipStream_t s, bool state_zeroed = false);
hipError_t launch_emit(const EntArgs &a, hipStream_t s);
hipError_t launch_seam_fix(const EntArgs &a, hipStream_t s);
hipError_t launch_or_words(uint32_t *dst, const uint32_t *src, long long n, hipStream_t s);
hipError_t launch_move_pieces(uint32_t *raw, const Geom &g, uint32_t *dst,
                              const unsigned long long *d_pieces, int npieces, long long max_words, long long cap,
                              hipStream_t s);
hipError_t launch_or_pieces(uint32_t *raw, const Geom &g, const uint32_t *src,
                            const unsigned long long *d_pieces, int npieces, long long max_words, hipStream_t s);
hipError_t launch_gather_regions(uint8_t *dst, long long slot_bytes, int pitch, const uint8_t *src,
                                 long long src_pitch, const int4 *regions, int n, int max_h,
                                 hipStream_t s);
hipError_t launch_mfma_probe(const int4 *A, const int4 *B, int4 *D, hipStream_t s);
hipError_t launch_band_last(const int16_t *dc, const Geom &g, int n, int16_t *last, hipStream_t s);
hipError_t launch_band_bound(const EntArgs &a, unsigned long long *acc, unsigned long long *bound, hipStream_t s);
hipError_t launch_band_count(const unsigned long long *scan_bits, int n, unsigned long long *pieces,
                             unsigned long long *bits, hipStream_t s);
hipError_t launch_or_shift_pieces(uint32_t *raw, const Geom &g, const uint32_t *src,
                                  const unsigned long long *d_pieces, int npieces, long long max_words, hipStream_t s);
hipError_t launch_band_stuff(const EntArgs &a, const unsigned long long *allbits, int world, int rank,
                             unsigned long long *rec, unsigned long long *total, uint8_t *dst, unsigned long long cap,
                             hipStream_t s);
hipError_t launch_band_join(const EntArgs &a, const unsigned long long *allrec, int world, unsigned long long stride,
                            unsigned long long *pieces, const uint8_t *src, hipStream_t s);
hipError_t launch_band_assembly(const unsigned long long *allbits, int world, int n, unsigned long long stride,
                                unsigned long long *pieces, unsigned long long *scan_bits, int *over, hipStream_t s);
}  // namespace mij

using namespace mij;

// ---------------------------------------------------------------------------
// error state
// ---------------------------------------------------------------------------
static thread_local int g_err = MIJ_OK;

static thread_local char g_msg[256];  // text of this thread's last failure
static int vfail(int code, const char *fmt, va_list ap) {
  g_err = code;
  va_list aq;
  va_copy(aq, ap);
  vsnprintf(g_msg, sizeof g_msg, fmt, aq);
  va_end(aq);
  fprintf(stderr, "mijpeg: %s\n", g_msg);
  return code;
}
static int fail(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfail(code, fmt, ap);
  va_end(ap);
  return code;
}
// for the other host translation units (mij_stream.hip)
int mij_frame_fail(int ferr, const char *what, int frame) {
  switch (ferr) {
    case FERR_SPIN:
      return fail(MIJ_EHANG, "%s %d: a device-side wait outlasted its bound (a pack group's look-back "
                  "publication lost, or a stale pack ticket)", what, frame);
    case FERR_OVERFLOW: return fail(MIJ_ENOSPC, "%s %d: bits past the scan buffer", what, frame);
    case FERR_ASSEMBLY: return fail(MIJ_ENOSPC, "%s %d: a band piece outside its buffer", what, frame);
  }
  return fail(MIJ_ETABLE, "%s %d: Huffman table construction failed", what, frame);
}
int mij_fail(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfail(code, fmt, ap);
  va_end(ap);
  return code;
}
void mij_clear_error() { g_err = MIJ_OK; }

// Diagnostic switches (per-wave clocks, K1 attribution flags, timing dumps)
// read from the environment in the diagnostic build only (make diag); the
// product library ignores them.
#ifdef MIJ_K1_DIAG
static int diag_env(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}
static const char *diag_str(const char *name) { return getenv(name); }
#else
static constexpr int diag_env(const char *, int dflt) { return dflt; }
static constexpr const char *diag_str(const char *) { return nullptr; }
#endif

#define HIP_TRY(x)                                                          \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess)                                                   \
      return fail(MIJ_EHIP, "%s failed: %s", #x, hipGetErrorString(e_));    \
  } while (0)

extern "C" int mij_last_error(void) { return g_err; }

extern "C" const char *mij_last_message(void) { return g_msg; }

extern "C" const char *mij_strerror(int code) {
  switch (code) {
    case MIJ_OK: return "ok";
    case MIJ_EINVAL: return "invalid argument";
    case MIJ_ENODEV: return "no usable HIP device";
    case MIJ_EHIP: return "HIP runtime error";
    case MIJ_ENOSPC: return "output buffer too small";
    case MIJ_ETABLE: return "Huffman table outside the reference's defined behaviour";
    case MIJ_EPPM: return "PPM rejected (utils/original.c read_ppm rules)";
    case MIJ_EIO: return "file I/O error";
    case MIJ_EJPEG: return "JPEG stream rejected (not a baseline 4:2:0 three-scan JFIF, or corrupt)";
    case MIJ_EHANG: return "device-side wait outlasted its bound (corrupted device state)";
  }
  return "unknown error";
}

extern "C" const char *mij_build_target(void) { return "gfx950"; }

// ---------------------------------------------------------------------------
// geometry and constant tables
// ---------------------------------------------------------------------------
static const int k_luma_q[64] = {  // encoder.c:18-26
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const int k_chroma_q[64] = {  // encoder.c:28-36
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
static const int k_zz[64] = {  // encoder.c:38-46
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

static long long round_up(long long v, long long m) { return (v + m - 1) / m * m; }

static bool valid_dims(int w, int h) { return w > 0 && h > 0 && w % 16 == 0 && h % 16 == 0; }

static Geom make_geom(int w, int h) {
  Geom g;
  memset(&g, 0, sizeof(g));
  g.w = w;
  g.h = h;
  g.nY = w * h / 64;
  g.nC = w * h / 256;
  g.nblk = g.nY + 2 * g.nC;
  g.tiles_x = (w + TILE_W - 1) / TILE_W;
  g.tiles_per_frame = g.tiles_x * (h / TILE_H);
  g.nsy = (h / 8) * g.tiles_x;
  g.nsc = (h / 16) * g.tiles_x;
  g.nseg = g.nsy + 2 * g.nsc;
  g.coef_fs = (long long)g.nblk * 64;
  g.raw_words[0] = round_up((long long)g.nY * MAX_BLOCK_BITS / 32 + 16, 64);
  g.raw_words[1] = round_up((long long)g.nC * MAX_BLOCK_BITS / 32 + 16, 64);
  g.raw_words[2] = g.raw_words[1];
  g.raw_fs = g.raw_words[0] + g.raw_words[1] + g.raw_words[2];
  g.out_cap = round_up((long long)g.nblk * 434 + 4096, 256);
  div_magic((uint32_t)g.tiles_per_frame, g.tpf_m, g.tpf_s);
  div_magic((uint32_t)g.tiles_x, g.tx_m, g.tx_s);
  return g;
}

extern "C" size_t mij_max_jpg_bytes(int w, int h) {
  if (!valid_dims(w, h)) return 0;
  return (size_t)make_geom(w, h).out_cap;
}

// original.c:504-509
static void quality_tables(int quality, int lq[64], int cq[64]) {
  for (int i = 0; i < 64; i++) {
    double l = (100 - quality) / 50.0 * k_luma_q[i];
    double c = (100 - quality) / 50.0 * k_chroma_q[i];
    l = l < 1 ? 1 : (l > 255 ? 255 : l);
    c = c < 1 ? 1 : (c > 255 ? 255 : c);
    lq[i] = (int)l;
    cq[i] = (int)c;
  }
}

// Host-built constant tables (A-operand digits, quantizer factors/bounds,
// cosines); the colour-exception bitmaps are built on the device.
static void fill_tables(int quality, Tables *t) {
  memset(t, 0, sizeof(*t));
  for (int i = 0; i < 64; i++)  // utils/lookup.c:10 == encoder.c:8-16
    t->cosd[i] = cos((double)(2 * (i / 8) + 1) * (i % 8) * M_PI / 16);
  int q[2][64];
  quality_tables(quality, q[0], q[1]);
  for (int c = 0; c < 2; c++)
    for (int z = 0; z < 64; z++) {
      t->qint[c][z] = q[c][k_zz[z]];
      t->dqt[c][z] = q[c][k_zz[z]];
    }
  // The luma prescale of the A rows: zigzag group g = z / 16
  // gets s_g = floor(log2(min luma AC q in the group)), row z the factor
  // 2^s_g / q_z <= 1, so the weights stay inside the unscaled digit ranges
  // and |N'| <= |N| < 2^31; a luma coefficient is then t = N' / 2^(21 + s_g).
  int sg[4];
  for (int g = 0; g < 4; g++) {
    int qmin = 256;
    for (int z = 16 * g; z < 16 * g + 16; z++)
      if (z) qmin = t->qint[0][z] < qmin ? t->qint[0][z] : qmin;
    int s = 0;
    while ((2 << s) <= qmin) s++;
    sg[g] = s;
    t->kq[g] = 21 + s;
  }
  for (int z = 1; z < 64; z++) {
    // chroma in fp32 on the luma-scaled N' (z = 0, the DC: exact from the pixel sum)
    const double fac = (double)t->qint[0][z] / ((double)t->qint[1][z] * ldexp(1.0, 21 + sg[z >> 4]));
    t->qfac[1][z] = (float)fac;
  }
  // DC ties (K1 dc_tie): at |S| = 8qK the reference computes
  // (int)(((S * M_SQRT1_2) * M_SQRT1_2) / 4 / q) (encoder.c:87-109 with the
  // frequency-0 cosines exactly 1.0), which is K or K - 1
  for (int c = 0; c < 2; c++) {
    const int q0 = q[c][0];
    for (int K = 1; K < 32 * DCTIE_WORDS && 8 * q0 * K <= 8192; K++) {
      volatile double f = (double)(8 * q0 * K);  // volatile: keep the reference's rounding steps
      f = f * M_SQRT1_2;
      f = f * M_SQRT1_2;
      f = f / 4;
      const int r = (int)(f / q0);
      if (r != K) t->dctie[c][K >> 5] |= 1u << (K & 31);
    }
  }
  // A fragments of v_mfma_i32_16x16x64_i8: lane l holds row (l & 15) and the
  // 16 k-values 16*(l>>4) .. +15.  Row r of M-tile m is zigzag coefficient
  // z = 16*(r>>2) + 4m + (r&3); k = pixel index y*8+x of the block.
  for (int m = 0; m < 4; m++)
    for (int lane = 0; lane < 64; lane++) {
      const int row = lane & 15, kg = lane >> 4;
      const int z = 16 * (row >> 2) + 4 * m + (row & 3);
      const int rz = k_zz[z], v = rz >> 3, u = rz & 7;
      int8_t dig[3][16];
      for (int j = 0; j < 16; j++) {
        const int p = 16 * kg + j, y = p >> 3, x = p & 7;
        long long W;
        if (z == 0) {
          dig[0][j] = 0;
          dig[1][j] = 0;
          dig[2][j] = 1;  // DC row: exact pixel sum in digit 0
          continue;
        }
        double k = t->cosd[y * 8 + v] * t->cosd[x * 8 + u];
        if (u == 0) k *= M_SQRT1_2;
        if (v == 0) k *= M_SQRT1_2;
        W = llround(k * ldexp(1.0, 19 + sg[z >> 4]) / t->qint[0][z]);  // 2^19 * 2^s_g / q_z
        const long long d0 = ((W + 64) & 127) - 64;
        const long long w1 = (W - d0) >> 7;
        const long long d1 = ((w1 + 64) & 127) - 64;
        const long long d2 = (w1 - d1) >> 7;
        dig[0][j] = (int8_t)d2;
        dig[1][j] = (int8_t)d1;
        dig[2][j] = (int8_t)d0;
      }
      for (int d = 0; d < 3; d++) memcpy(&t->mfma_a[(m * 3 + d) * 64 + lane], dig[d], 16);
    }
  // K1's chroma all-AC-zero test (Tables::czl): the reference's |F/q| < 1
  // wherever |N'| + 4096 (the integer DCT's error bound, L1 / 2 <= 4096)
  // stays below (1 - 1e-6) / qfac (its unit); the test runs where all-zero
  // chroma N-tiles are common (smallest chroma AC quantiser >= 9: Q <= 75)
  {
    int qmin = 256;
    for (int z = 0; z < 64; z++) {
      const double lim = z ? (double)t->qint[1][z] * ldexp(1.0, 21 + sg[z >> 4]) / t->qint[0][z] * (1.0 - 2e-6) - 6000.0
                           : (double)(1 << 30);
      t->czl[z] = lim > (double)(1 << 30) ? (1 << 30) : (int)lim;
      if (z) qmin = t->qint[1][z] < qmin ? t->qint[1][z] : qmin;
    }
    t->cz_on = qmin >= 9;
  }
}

// ---------------------------------------------------------------------------
// batch pipeline
// ---------------------------------------------------------------------------
struct mij_batch {
  int dev = 0;
  hipStream_t stream = nullptr;  // where the batch enqueues: its own, or the caller's (mij_batch_set_stream)
  hipStream_t own_stream = nullptr;
  hipEvent_t ev_switch = nullptr;  // orders a stream switch after the work before it
  Geom g;
  int cap = 0, quality = 50;
  Tables *d_tab = nullptr;
  uint8_t *d_in = nullptr;
  bool own_in = false;
  long long in_fs = 0;
  int pitch = 0;
  int16_t *d_coef = nullptr, *d_dc = nullptr;
  uint32_t *d_hist = nullptr, *d_ehuf = nullptr, *d_raw = nullptr;
  uint32_t *d_tok = nullptr, *d_tok0 = nullptr, *d_seg_ntok = nullptr, *d_seg_bits = nullptr;
  uint64_t *d_seg_off = nullptr, *d_scan_bits = nullptr, *d_out_len = nullptr;
  HuffCode *d_hc = nullptr;
  uint8_t *d_out = nullptr;
  int *d_err = nullptr;
  unsigned *d_replays = nullptr;
  uint32_t *d_ffc = nullptr;      // k_emit_count: 0xFF bytes per scan chunk
  uint32_t *d_choff = nullptr;    // k_emit_scan: output offset per scan chunk
  uint64_t *d_scan_base = nullptr;  // band stuffing: each scan's first byte in the band's buffer
  uint32_t *d_seam = nullptr;     // k_pack_flat -> k_seam_fix: shared first word per pack group
  unsigned long long *d_pack_state = nullptr;  // k_pack_flat look-back words, per pack group
  unsigned *d_pack_ticket = nullptr;
  uint32_t *d_dcx = nullptr;      // k_segdc_actab (dc_last): per frame 64 words, left zeroed
  uint16_t *d_fixmask = nullptr;  // K1 fix masks: per N-tile (tile * 3 + nt), zero between launches
  uint16_t *d_audit = nullptr;    // mij_batch_audit: per frame, block, lane group 16 straddle bits
  size_t audit_cap = 0;
  bool audit = false;             // the next coefficient K1 launch is the audit variant
  // bands of one large frame (mij_band_*, mij_assemble_*): per frame [4]
  int16_t *d_dcpred = nullptr;
  uint32_t *d_bitbase = nullptr;
  uint32_t *d_stage = nullptr;      // H2D staging for mij_assemble_words / _pieces
  size_t stage_words = 0;
  unsigned long long *d_pieces = nullptr;  // mij_assemble_pieces: piece table
  size_t pieces_cap = 0;
  // an assembler (mij_assembler_create): only what the JFIF assembly of
  // whole frames from band words needs -- tables, scan buffers, outputs
  bool assembler = false;
  std::vector<unsigned long long> band_words;  // per frame x 3: packed words after mij_band_pack
  int band_async_n = 0;                        // frames of the last mij_band_pack_async
  int asm_tables_n = 0;                        // frames of the last mij_assemble_tables_async
  int hist_zero_n = 0;  // frames 0..n-1 of d_hist left zeroed by the last encode's k_tables_1w
  int band_hist_zero = 0;  // frames 0..n-1 of d_hist left zeroed by mij_band_tables_async's k_band_bound
  int hist_zero_after = 0;  // set by run_entropy: the frames its k_tables_1w zeroed
  unsigned long long *d_bound_acc = nullptr;   // k_band_bound: {sum, arrivals}, left zeroed by its last workgroup
  // region batches (mij_batch_set_frame_dims / _gather_regions): per-frame
  // image size inside the canvas slots; d_frame stages a host frame
  int2 *d_fdims = nullptr;
  int4 *d_regions = nullptr;
  bool use_fdims = false;
  std::vector<int2> h_fdims;
  uint8_t *d_frame = nullptr;
  size_t frame_cap = 0;
  // the band packing needs all-zero scan buffers; k_emit_write leaves them so, the
  // band paths (k_scan + k_pack_flat, no emit) and the assembler's ORed words
  // before mij_assemble_end do not.  raw_dirty = frames 0..raw_dirty-1 may
  // hold words (0: every scan buffer is zero)
  int raw_dirty = 0;
  bool keep_coefs = false;  // encode also writes coefficient planes
  bool rgb = false;         // input frames in R, G, B byte order (PPM) instead of B, G, R
  bool split = false;       // true: K1 writes coefficients, a second pass tokenizes;
                            // false (default): K1 emits the tokens itself
  // sub-batch overlap (mij_batch_set_overlap): entropy stages on stream2
  int overlap = 1;
  hipStream_t stream2 = nullptr;
  hipEvent_t ov_k1[16] = {}, ov_done = nullptr;
  bool timing = false;
  int k1_err_zero = 0;  // frames whose error words the next run_k1 zeroes
  // mij_batch_set_option (include/mijpeg.h): entropy-stage variants
  int opt[MIJ_OPT_COUNT] = {1, 1, 1, 0, -1, 0, 1, 0, -1};
  static constexpr int HIST = 64;
  hipEvent_t evh[HIST][MIJ_NSTAGES] = {};  // per-step events while timing is on
  hipEvent_t *ev = evh[0];       // current step's events
  long long steps = 0;
  int last_frames = 0;
};

template <class T>
static hipError_t dalloc(T **p, size_t count) {
  return hipMalloc((void **)p, count * sizeof(T) + 256);
}

static void batch_free(mij_batch *b) {
  if (!b) return;
  hipSetDevice(b->dev);
  if (b->stream && b->stream != b->own_stream) hipStreamSynchronize(b->stream);
  if (b->own_stream) hipStreamSynchronize(b->own_stream);
  void *ptrs[] = {b->d_tab, b->own_in ? b->d_in : nullptr, b->d_coef, b->d_dc, b->d_hist,
                  b->d_ehuf, b->d_raw, b->d_tok, b->d_tok0, b->d_seg_ntok, b->d_seg_bits, b->d_seg_off,
                  b->d_scan_bits, b->d_out_len, b->d_hc, b->d_out, b->d_err, b->d_replays,
                  b->d_dcpred, b->d_bitbase, b->d_stage, b->d_fixmask, b->d_audit, b->d_ffc, b->d_choff, b->d_scan_base,
                  b->d_seam, b->d_pack_state, b->d_pack_ticket, b->d_fdims, b->d_frame, b->d_regions, b->d_pieces,
                  b->d_bound_acc, b->d_dcx};
  for (void *p : ptrs)
    if (p) hipFree(p);
  for (auto &row : b->evh)
    for (auto &e : row)
      if (e) hipEventDestroy(e);
  for (auto &e : b->ov_k1)
    if (e) hipEventDestroy(e);
  if (b->ov_done) hipEventDestroy(b->ov_done);
  if (b->stream2) {
    hipStreamSynchronize(b->stream2);
    hipStreamDestroy(b->stream2);
  }
  if (b->ev_switch) hipEventDestroy(b->ev_switch);
  if (b->own_stream) hipStreamDestroy(b->own_stream);
  delete b;
}

static int check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return fail(MIJ_ENODEV, "no HIP device visible (the HIP path has no CPU fallback)");
  if (device < 0 || device >= n) return fail(MIJ_ENODEV, "device %d out of range (%d)", device, n);
  return MIJ_OK;
}

static int batch_init(mij_batch *b, int device, int w, int h, int frames, int quality, bool assembler = false) {
  if (check_device(device)) return g_err;
  b->dev = device;
  b->assembler = assembler;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
  b->own_stream = b->stream;
  b->g = make_geom(w, h);
  b->cap = frames;
  b->quality = quality;
  const Geom &g = b->g;
  const long long F = frames;
  HIP_TRY(dalloc(&b->d_tab, 1));
  {
    Tables *t = new Tables;
    fill_tables(quality, t);
    hipError_t e = hipMemcpy(b->d_tab, t, sizeof(Tables), hipMemcpyHostToDevice);
    delete t;
    HIP_TRY(e);
    uint32_t *lut = &b->d_tab->lut[0][0];
    HIP_TRY(hipMemsetAsync(lut, 0, sizeof(uint32_t) * 3 * LUT_WORDS, b->stream));
    HIP_TRY(launch_colour_lut(lut, b->stream));
  }
  b->pitch = w * 3;
  b->in_fs = (long long)w * h * 3;
  if (!assembler) {
    HIP_TRY(dalloc(&b->d_in, F * b->in_fs));
    b->own_in = true;
    HIP_TRY(dalloc(&b->d_coef, F * g.coef_fs));
    HIP_TRY(dalloc(&b->d_dc, F * g.nblk));
    HIP_TRY(dalloc(&b->d_tok, F * g.nseg * SEG_TOK));
    HIP_TRY(dalloc(&b->d_tok0, F * g.nseg));
    HIP_TRY(dalloc(&b->d_seg_ntok, F * g.nseg));
    HIP_TRY(dalloc(&b->d_seg_bits, F * g.nseg));
    HIP_TRY(dalloc(&b->d_seg_off, F * g.nseg));
    HIP_TRY(dalloc(&b->d_fixmask, F * g.tiles_per_frame * 3));
    HIP_TRY(hipMemsetAsync(b->d_fixmask, 0, sizeof(uint16_t) * F * g.tiles_per_frame * 3, b->stream));
    HIP_TRY(dalloc(&b->d_pack_state, F * pack_stride(g)));
    HIP_TRY(dalloc(&b->d_pack_ticket, F * 3));  // one per scan
    HIP_TRY(dalloc(&b->d_dcx, F * 64));
    HIP_TRY(hipMemsetAsync(b->d_dcx, 0, sizeof(uint32_t) * F * 64, b->stream));
    HIP_TRY(dalloc(&b->d_seam, F * pack_stride(g)));
    HIP_TRY(dalloc(&b->d_regions, F));
  }
  HIP_TRY(dalloc(&b->d_hist, F * 4 * 257));
  HIP_TRY(dalloc(&b->d_ehuf, F * 4 * 256));
  HIP_TRY(dalloc(&b->d_raw, F * g.raw_fs));
  HIP_TRY(hipMemsetAsync(b->d_raw, 0, sizeof(uint32_t) * F * g.raw_fs, b->stream));
  HIP_TRY(dalloc(&b->d_scan_bits, F * 3));
  HIP_TRY(dalloc(&b->d_out_len, F));
  HIP_TRY(dalloc(&b->d_hc, F * 4));
  HIP_TRY(dalloc(&b->d_out, F * g.out_cap));
  HIP_TRY(dalloc(&b->d_err, F));
  HIP_TRY(dalloc(&b->d_replays, 1));
  HIP_TRY(dalloc(&b->d_ffc, F * 3 * emit_chunks(g)));
  HIP_TRY(dalloc(&b->d_choff, F * 3 * emit_chunks(g)));
  HIP_TRY(dalloc(&b->d_scan_base, F * 3));
  HIP_TRY(hipMemsetAsync(b->d_ffc, 0, sizeof(uint32_t) * F * 3 * emit_chunks(g), b->stream));  // (ff_pack adds)
  HIP_TRY(hipMemsetAsync(b->d_replays, 0, sizeof(unsigned), b->stream));
  HIP_TRY(dalloc(&b->d_fdims, F));
  b->h_fdims.assign((size_t)F, make_int2(w, h));
  HIP_TRY(dalloc(&b->d_dcpred, F * 4));
  HIP_TRY(dalloc(&b->d_bitbase, F * 4));
  HIP_TRY(hipMemsetAsync(b->d_dcpred, 0, sizeof(int16_t) * F * 4, b->stream));
  HIP_TRY(hipMemsetAsync(b->d_bitbase, 0, sizeof(uint32_t) * F * 4, b->stream));
  b->band_words.assign((size_t)F * 3, 0);
  for (auto &row : b->evh)
    for (auto &e : row) HIP_TRY(hipEventCreate(&e));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" mij_batch *mij_batch_create(int device, int width, int height, int max_frames,
                                       int quality) {
  if (!valid_dims(width, height) || max_frames < 1 || quality < 1 || quality > 100) {
    fail(MIJ_EINVAL, "batch_create: bad geometry %dx%d x%d or quality %d", width, height,
         max_frames, quality);
    return nullptr;
  }
  mij_batch *b = new mij_batch;
  if (batch_init(b, device, width, height, max_frames, quality)) {
    batch_free(b);
    return nullptr;
  }
  g_err = MIJ_OK;
  return b;
}

extern "C" mij_batch *mij_assembler_create(int device, int width, int height, int max_frames,
                                           int quality) {
  if (!valid_dims(width, height) || max_frames < 1 || quality < 1 || quality > 100) {
    fail(MIJ_EINVAL, "assembler_create: bad geometry %dx%d x%d or quality %d", width, height,
         max_frames, quality);
    return nullptr;
  }
  mij_batch *b = new mij_batch;
  if (batch_init(b, device, width, height, max_frames, quality, true)) {
    batch_free(b);
    return nullptr;
  }
  g_err = MIJ_OK;
  return b;
}

// entry points that run the encoder itself: not on an assembler
static int pipe_check(const mij_batch *b, const char *what) {
  if (!b) return fail(MIJ_EINVAL, "%s: null batch", what);
  if (b->assembler) return fail(MIJ_EINVAL, "%s: an assembler only assembles band words", what);
  return MIJ_OK;
}

extern "C" void mij_batch_destroy(mij_batch *b) { batch_free(b); }

extern "C" void *mij_batch_stream(mij_batch *b) { return b ? (void *)b->stream : nullptr; }

extern "C" int mij_batch_set_stream(mij_batch *b, void *stream) {
  if (!b) return fail(MIJ_EINVAL, "set_stream: null batch");
  HIP_TRY(hipSetDevice(b->dev));
  const hipStream_t s = stream ? (hipStream_t)stream : b->own_stream;
  if (s == b->stream) return MIJ_OK;
  // the new stream runs after everything enqueued so far on the old one
  if (!b->ev_switch) HIP_TRY(hipEventCreateWithFlags(&b->ev_switch, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(b->ev_switch, b->stream));
  HIP_TRY(hipStreamWaitEvent(s, b->ev_switch, 0));
  b->stream = s;
  return MIJ_OK;
}

// slots first..first+n-1 hold canvas-sized frames again; a region batch
// whose slots are then all canvas-sized is a plain batch
static int canvas_frames(mij_batch *b, int first, int n) {
  if (!b->use_fdims) return MIJ_OK;
  const int2 cv = make_int2(b->g.w, b->g.h);
  for (int i = first; i < first + n; i++) b->h_fdims[i] = cv;
  bool all = true;
  for (const int2 &d : b->h_fdims) all = all && d.x == cv.x && d.y == cv.y;
  if (all) {
    b->use_fdims = false;
    return MIJ_OK;
  }
  HIP_TRY(hipMemcpyAsync(b->d_fdims + first, b->h_fdims.data() + first, sizeof(int2) * n,
                         hipMemcpyHostToDevice, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));  // pageable source
  return MIJ_OK;
}

extern "C" int mij_batch_upload(mij_batch *b, const uint8_t *bgr, int first, int nframes) {
  if (pipe_check(b, "upload")) return g_err;
  if (!bgr || first < 0 || nframes < 1 || first + nframes > b->cap)
    return fail(MIJ_EINVAL, "upload: bad args");
  if (!b->own_in) return fail(MIJ_EINVAL, "upload: batch reads external device input");
  HIP_TRY(hipSetDevice(b->dev));
  // full frames: the uploaded slots are canvas-sized again (set_frame_dims
  // after, if wanted); the other slots keep their sizes
  if (canvas_frames(b, first, nframes)) return g_err;
  HIP_TRY(hipMemcpyAsync(b->d_in + (long long)first * b->in_fs, bgr, (size_t)nframes * b->in_fs,
                         hipMemcpyHostToDevice, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_batch_set_input(mij_batch *b, const void *d_bgr, long long frame_stride,
                                   int pitch) {
  if (pipe_check(b, "set_input")) return g_err;
  if (!d_bgr || ((uintptr_t)d_bgr & 15) || (pitch & 15) || (frame_stride & 15) ||
      pitch < b->g.w * 3)
    return fail(MIJ_EINVAL, "set_input: pointer, pitch and frame stride must be 16-byte "
                            "aligned, pitch >= 3*w");
  HIP_TRY(hipSetDevice(b->dev));
  if (b->own_in && b->d_in) HIP_TRY(hipFree(b->d_in));
  b->own_in = false;
  b->use_fdims = false;  // full frames: the batch geometry again
  b->d_in = (uint8_t *)d_bgr;
  b->in_fs = frame_stride;
  b->pitch = pitch;
  return MIJ_OK;
}

// a 64-segment pack group at Q >= 85 outgrows a 4096-word window (config
// 5: Q=90 luma groups ~4.8k words): the wider window keeps it on the
// one-window path (A/B: MIJ_PACK_WIDE=0/1)
static int ent_args_pack_wide(const mij_batch *b) {
  const int v = b->opt[MIJ_OPT_PACK_WIDE];
  return v >= 0 ? v : (b->quality >= PACK_WIDE_MIN_Q ? 1 : 0);
}

// the packing's group sizes (32 << ls segments): larger groups spread the
// per-group fixed cost (ticket, counts, look-back) over more tokens, as long
// as the group's bits stay inside one LDS window at the quality's typical
// entropy (MIJ_OPT_PACK_SEGS overrides; A/B profiles/r05/pack_segs)
static void ent_args_pack_ls(const mij_batch *b, int nframes, int ls[2]) {
  const int v = b->opt[MIJ_OPT_PACK_SEGS];
  if (v >= 0) {
    ls[0] = v % 4;
    ls[1] = v / 4;
    return;
  }
  // (config 3, profiles/r05/pack_segs/ab.txt: luma 128 segments to Q=70,
  // 64 to Q=92, 32 above; chroma 256 to Q=97, 128 above.  At Q=50 that is
  // 0.43 ms against 0.63 with 64 / 64; at Q=95 2.0 against 3.6)
  ls[0] = b->quality <= 70 ? 2 : (b->quality <= 92 ? 1 : 0);
  ls[1] = b->quality <= 97 ? 3 : 2;
  // A small batch cannot fill the GPU with large groups, and then a group's
  // latency is the packing's: smaller groups until the launch has about half
  // of the 2048 workgroups 256 CUs hold (one 1920x1280 frame: 32-segment
  // groups, pack 31 -> 23 us)
  const long long nf = nframes > 0 ? nframes : 1;
  while (ls[0] > 0 && nf * pack_groups(b->g.nsy, ls[0]) < 1024) ls[0]--;
  while (ls[1] > 0 && nf * 2 * pack_groups(b->g.nsc, ls[1]) < 1024) ls[1]--;
}

// band: the mij_band_* calls, whose per-frame DC predictors and in-word scan
// start bits live in d_dcpred / d_bitbase; every other pipeline reads both as
// 0 (null), so a band call leaves no state behind for the next encode
static EntArgs ent_args(mij_batch *b, int nframes, int f0 = 0, bool band = false) {
  b->hist_zero_n = 0;  // every path through here may write the histograms
  EntArgs a;
  memset(&a, 0, sizeof(a));
  a.g = b->g;
  a.nframes = nframes;
  a.coef = b->d_coef;
  a.dc = b->d_dc;
  a.hist = b->d_hist;
  a.ehuf = b->d_ehuf;
  a.tok = b->d_tok;
  a.tok0 = b->d_tok0;
  a.seg_ntok = b->d_seg_ntok;
  a.seg_bits = b->d_seg_bits;
  a.seg_off = b->d_seg_off;
  a.scan_bits = b->d_scan_bits;
  a.raw = b->d_raw;
  a.hc = b->d_hc;
  a.tab = b->d_tab;
  a.out = b->d_out;
  a.out_len = b->d_out_len;
  a.err = b->d_err;
  a.dc_pred = band ? b->d_dcpred : nullptr;
  a.bit_base = band ? b->d_bitbase : nullptr;
  a.ffc = b->d_ffc;
  a.choff = b->d_choff;
  a.scan_base = b->d_scan_base;
  a.pack_state = b->d_pack_state;
  a.pack_ticket = b->d_pack_ticket;
  a.dcx = b->d_dcx;
  a.fdims = b->use_fdims ? b->d_fdims : nullptr;
  // JFIF-assembly workgroups per frame (its chunks dealt round-robin over
  // the three scans; A/B per scan in round 2, profiles/r02/emit_slots_ab.txt):
  // 48 on large batches at any quality (round 6 sweep on config 3,
  // scripts/emit_sweep.sh, profiles/r06/probe/emit_slots.txt: emit 0.146 ms
  // at 48 against 0.154-0.189 at 16-384 for Q=50, 0.383 against 0.401 at the
  // former 192 for Q=90), about 4096 per launch on frames of 8 Mpixels and
  // more (config 4: few scans of hundreds of chunks each; 1536 per frame for
  // one or two frames, 512 for config 4's eight: its assembly 0.094-0.097 ms
  // at 1536, 0.089 at 512, profiles/r06/probe/c4_emit_slots.txt), 192
  // otherwise (a single frame needs the width)
  const int slots_opt = b->opt[MIJ_OPT_EMIT_SLOTS];
  a.emit_slots = slots_opt > 0                                 ? slots_opt
                 : nframes >= 43                               ? 48
                 : ((long long)b->g.w * b->g.h >= (8 << 20))    ? std::max(192, std::min(1536, 4096 / nframes))
                                                                : 192;
  a.pack_wide = ent_args_pack_wide(b);
  ent_args_pack_ls(b, nframes, a.pack_ls);
  if (f0) {  // sub-batch: frames f0.. of the batch (every per-frame array shifted)
    const Geom &g = b->g;
    const long long F = f0, gpf = pack_stride(g);
    a.coef += F * g.coef_fs;
    a.dc += F * g.nblk;
    a.hist += F * 4 * 257;
    a.ehuf += F * 4 * 256;
    a.tok += F * g.nseg * SEG_TOK;
    a.tok0 += F * g.nseg;
    a.seg_ntok += F * g.nseg;
    a.seg_bits += F * g.nseg;
    a.seg_off += F * g.nseg;
    a.scan_bits += F * 3;
    a.raw += F * g.raw_fs;
    a.hc += F * 4;
    a.out += F * g.out_cap;
    a.out_len += F;
    a.err += F;
    if (a.dc_pred) a.dc_pred += F * 4;
    if (a.bit_base) a.bit_base += F * 4;
    a.ffc += F * 3 * emit_chunks(g);
    a.choff += F * 3 * emit_chunks(g);
    a.scan_base += F * 3;
    a.pack_state += F * gpf;
    a.pack_ticket += F * 3;
    if (a.dcx) a.dcx += F * 64;
    if (a.fdims) a.fdims += F;
  }
  return a;
}

// mode: K1 mode bits (1 coefficient planes out, 2 tokens + histograms out,
// 4 coefficient planes in)
static int run_k1(mij_batch *b, int nframes, int mode, int dc_diffed = 0, int seg_dc_inline = 0, int f0 = 0,
                  bool stage_events = true) {
  // a token-emitting K1 (modes 2, 3, 6: the band calls too) adds onto d_hist:
  // the next encode must zero it again
  if (mode & 2) b->hist_zero_n = b->band_hist_zero = 0;
  K1Args k;
  memset(&k, 0, sizeof(k));
  k.in = b->d_in;
  k.in_fs = b->in_fs;
  k.pitch = b->pitch;
  k.nframes = nframes;
  k.g = b->g;
  k.coef = b->d_coef;
  k.dc = b->d_dc;
  k.tab = b->d_tab;
  k.replays = b->d_replays;
  k.tok = b->d_tok;
  k.tok0 = b->d_tok0;
  k.seg_ntok = b->d_seg_ntok;
  k.hist = b->d_hist;
  k.fix_mask = b->d_fixmask;
  k.audit = b->audit && mode == 1 ? b->d_audit : nullptr;
  k.rgb = b->rgb && (mode & 4) == 0;  // pixel-input variants
  k.fdims = b->use_fdims ? b->d_fdims : nullptr;
  if (b->k1_err_zero) {  // the encode's first K1 zeroes its error words
    k.err_zero = b->d_err;
    k.nerr_zero = b->k1_err_zero;
    b->k1_err_zero = 0;
  }
  if (f0) {  // sub-batch: frames f0.. (per-frame arrays shifted; mode 2 only)
    const Geom &g = b->g;
    const long long F = f0;
    k.in += F * b->in_fs;
    k.coef += F * g.coef_fs;
    k.dc += F * g.nblk;
    k.tok += F * g.nseg * SEG_TOK;
    k.tok0 += F * g.nseg;
    k.seg_ntok += F * g.nseg;
    k.hist += F * 4 * 257;
    if (k.fdims) k.fdims += F;
  }
  static const int k1_flags = diag_env("MIJ_K1_FLAGS", 0);
  k.flags = k1_flags;
  const long long ntiles = (long long)nframes * b->g.tiles_per_frame;
  long long grid = k1_grid(b->dev, ntiles, mode);
  long long per_wg = (ntiles + grid - 1) / grid;
  if (per_wg > b->g.tiles_per_frame) per_wg = b->g.tiles_per_frame;  // <= 2 frames per WG
  grid = (ntiles + per_wg - 1) / per_wg;
  k.per_wg = (int)per_wg;
  k.dc_diffed = dc_diffed;
  k.seg_dc_inline = seg_dc_inline;
  // the coefficient variant marks hazard blocks in the fix masks;
  // k_fix_blocks recomputes them in FP64 right after it, on the same stream
  // diagnostics (MIJ_K1_WTIME with the diag build): per-wave lifetimes of K1
  static const bool wtime = diag_env("MIJ_K1_WTIME", 0) != 0;
  unsigned long long *d_wt = nullptr;
  const long long nw = grid * 16;
  if (wtime && (mode == 1 || mode == 2)) {
    HIP_TRY(hipMalloc(&d_wt, sizeof(unsigned long long) * K1_WTIME_WORDS * nw));
    HIP_TRY(hipMemsetAsync(d_wt, 0, sizeof(unsigned long long) * K1_WTIME_WORDS * nw, b->stream));
    k.wtime = d_wt;
  }
  HIP_TRY(launch_k1(k, (int)grid, mode, b->stream));
  if (d_wt) {
    const int WW = K1_WTIME_WORDS;
    std::vector<unsigned long long> h(WW * nw);
    HIP_TRY(hipMemcpyAsync(h.data(), d_wt, sizeof(unsigned long long) * WW * nw, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipFree(d_wt));
    unsigned long long s0 = ~0ull, e1 = 0, e0 = ~0ull;
    double sum = 0, smin = 1e30, smax = 0, ph[5] = {0, 0, 0, 0, 0};
    long long n = 0, tiles = 0;
    for (long long i = 0; i < nw; i++) {
      if (!h[WW * i + 1]) continue;
      const unsigned long long a0 = h[WW * i], a1 = h[WW * i + 1];
      s0 = std::min(s0, a0); e1 = std::max(e1, a1); e0 = std::min(e0, a1);
      const double d = (double)(a1 - a0);
      sum += d; smin = std::min(smin, d); smax = std::max(smax, d); n++; tiles += (long long)h[WW * i + 2];
      for (int k = 0; k < 5; k++) ph[k] += (double)h[WW * i + 3 + k];
    }
    if (const char *path = diag_str("MIJ_K1_WTIME_DUMP")) {  // raw per-wave records
      if (FILE *fp = fopen(path, "ab")) { fwrite(h.data(), sizeof(unsigned long long), WW * nw, fp); fclose(fp); }
    }
    // s_memrealtime ticks at 100 MHz; the phases are s_memtime (shader clock) per tile
    fprintf(stderr, "K1 waves %lld tiles %lld: span %.1f us, first end %.1f us, wave life mean %.1f min %.1f max %.1f us\n",
            n, tiles, (e1 - s0) / 100.0, (e0 - s0) / 100.0, sum / n / 100.0, smin / 100.0, smax / 100.0);
    if (tiles)
      fprintf(stderr, "K1 phases, clocks per tile: dma-wait %.0f colour %.0f dma-issue %.0f dct+quant %.0f store/emit %.0f\n",
              ph[0] / tiles, ph[1] / tiles, ph[2] / tiles, ph[3] / tiles, ph[4] / tiles);
  }
  if (b->timing && mode != 6 && stage_events) HIP_TRY(hipEventRecord(b->ev[1], b->stream));
  if (mode == 1) HIP_TRY(launch_fix_blocks(k, b->stream));
  if (b->timing && mode != 6 && stage_events) HIP_TRY(hipEventRecord(b->ev[2], b->stream));
  return MIJ_OK;
}

// Stages after K1 emitted the token streams and histograms (the histograms
// must have been zeroed before K1).  dc_fix: the segments' first DC tokens
// are still to compute (K1 from pixels); tables_given: the caller's huff_code
// structs are already in d_hc and d_ehuf (drop-in write_jpg).
static int run_entropy(mij_batch *b, int nframes, bool dc_fix, bool tables_given, int f0 = 0,
                       hipStream_t st = nullptr) {
  b->band_hist_zero = 0;  // (its segment DCs add onto d_hist)
  EntArgs a = ent_args(b, nframes, f0);
  const bool t = b->timing && !st;  // (sub-batches: no stage events)
  if (!st) st = b->stream;
  // segment-first DC tokens: inside k_tables (its DC-table waves), or on
  // their own when the caller's tables are given
  static const int segdc_dbg = diag_env("MIJ_SEGDC_DBG", 0);  // diag build
  // (A/B: MIJ_OPT_SEGDC_FUSED=1 runs them in k_tables' DC waves -- two waves
  // per frame, 0.11 ms of a config-3 launch against a few us spread over the chip)
  const bool segdc_fused = b->opt[MIJ_OPT_SEGDC_FUSED] != 0;
  a.seg_dc = dc_fix && !tables_given && segdc_fused ? 1 | segdc_dbg : 0;
  // diagnostics (MIJ_TAB_TIME with the diag build): per-wave phase clocks of k_tables
  static const bool ttime = diag_env("MIJ_TAB_TIME", 0) != 0;
  // the AC tables beside the segment DCs (they need only K1's histograms),
  // the DC tables after (A/B: MIJ_OPT_ACTAB=0; profiles/r03/qsweep/actab_ab.txt:
  // segment DCs + tables 0.077 -> 0.062 ms at config 3 Q=50, 0.102 -> 0.075
  // at Q=90).  Not on small batches: one frame's four tables take as long
  // as its AC tables, and the DC tables after them add 10 us.
  // dc_last: the DC tables in the same launch, built by each frame's last
  // segment-DC workgroup while the AC tables' waves still merge (no
  // k_tables_1w launch) -- on batches of up to 64 frames (profiles/r06/dc_last:
  // one 1920x1280 frame 0.062 -> 0.059 ms, 16 frames 0.173 -> 0.162, 64
  // frames 0.354 -> 0.348; at 256 frames of 3840x2160 the tables after the
  // launch are faster: 3.63 against 3.70 ms)
  static const int dc_last_max = diag_env("MIJ_DC_LAST_MAX", 64);
  const bool dc_last = dc_fix && !a.seg_dc && !tables_given && !ttime && b->opt[MIJ_OPT_ACTAB] &&
                       nframes <= dc_last_max && b->d_dcx;
  const bool actab =
      dc_last || (dc_fix && !a.seg_dc && !tables_given && !ttime && b->opt[MIJ_OPT_ACTAB] && nframes >= 16);
  if (actab) {
    static const int dc_last_nozero = diag_env("MIJ_DC_LAST_NOZERO", 0);  // (diag: the packing zeroes its state)
    a.zero_pack = dc_last && dc_last_nozero ? 0 : 1;  // (the AC workgroups zero the counts they read)
    a.dc_last = dc_last;
    HIP_TRY(launch_segdc_actab(a, st));
  } else if (dc_fix && !a.seg_dc) {
    HIP_TRY(launch_seg_dc(a, st));
  }
  if (t) HIP_TRY(hipEventRecord(b->ev[4], st));
  if (!tables_given && ttime) {
    EntArgs at = a;
    const size_t nt = (size_t)nframes * 4 * 10;
    HIP_TRY(hipMalloc(&at.dbg, sizeof(unsigned long long) * nt));
    HIP_TRY(hipMemsetAsync(at.dbg, 0, sizeof(unsigned long long) * nt, st));
    HIP_TRY(launch_tables(at, st));
    std::vector<unsigned long long> h(nt);
    HIP_TRY(hipMemcpyAsync(h.data(), at.dbg, sizeof(unsigned long long) * nt, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipFree(at.dbg));
    // s_memtime: shader clocks; phases 0-1 load, 1-2 sort, 2-3 merges, 3-4
    // depths, 4-5 counts + limit, 5-6 symbol order, 6-7 codes + stores
    for (int kind = 0; kind < 2; kind++) {
      double ph[8] = {0};
      int cnt = 0;
      for (int f = 0; f < nframes; f++)
        for (int tt = kind; tt < 4; tt += 2) {
          const unsigned long long *r = &h[((size_t)f * 4 + tt) * 10];
          if (!r[7]) continue;
          for (int k = 0; k < 7; k++) ph[k] += (double)(r[k + 1] - r[k]);
          ph[7] += (double)(r[0] - r[8]);  // kernel entry -> table start (DC waves: the segment DCs)
          cnt++;
        }
      if (cnt)
        fprintf(stderr, "k_tables %s waves %d, clocks: pre %.0f load %.0f sort %.0f merge %.0f depth %.0f limit %.0f order %.0f codes %.0f\n",
                kind ? "AC" : "DC", cnt, ph[7] / cnt, ph[0] / cnt, ph[1] / cnt, ph[2] / cnt, ph[3] / cnt, ph[4] / cnt,
                ph[5] / cnt, ph[6] / cnt);
    }
    {  // one frame's span: first wave entry to last wave end
      double span = 0;
      for (int f = 0; f < nframes; f++) {
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int tt = 0; tt < 4; tt++) {
          const unsigned long long *r = &h[((size_t)f * 4 + tt) * 10];
          t0 = std::min(t0, r[8]);
          t1 = std::max(t1, r[7]);
        }
        span += (double)(t1 - t0);
      }
      double sw = 0, ww = 0, ent = 0;
      for (int f = 0; f < nframes; f++)
        for (int tt = 0; tt < 4; tt += 2) {
          const unsigned long long *r = &h[((size_t)f * 4 + tt) * 10];
          sw += (double)(r[9] - r[8]);
          ww += (double)(r[0] - r[9]);
        }
      for (int f = 0; f < nframes; f++) {
        unsigned long long e0 = ~0ull, e1 = 0;
        for (int tt = 0; tt < 4; tt++) {
          e0 = std::min(e0, h[((size_t)f * 4 + tt) * 10 + 8]);
          e1 = std::max(e1, h[((size_t)f * 4 + tt) * 10 + 8]);
        }
        ent += (double)(e1 - e0);
      }
      if (nframes == 1)
        for (int tt = 0; tt < 4; tt++) {
          const unsigned long long *r = &h[(size_t)tt * 10];
          fprintf(stderr, "k_tables wave %d: entry +%lld start +%lld end +%lld; phases %lld %lld %lld %lld %lld %lld %lld\n", tt,
                  (long long)(r[8] - h[8]), (long long)(r[0] - h[8]), (long long)(r[7] - h[8]), (long long)(r[1] - r[0]),
                  (long long)(r[2] - r[1]), (long long)(r[3] - r[2]), (long long)(r[4] - r[3]), (long long)(r[5] - r[4]),
                  (long long)(r[6] - r[5]), (long long)(r[7] - r[6]));
        }
      fprintf(stderr, "k_tables frame span %.0f clocks; DC waves: segment DCs %.0f, wait %.0f; wave entry spread %.0f\n",
              span / nframes, sw / (2.0 * nframes), ww / (2.0 * nframes), ent / nframes);
    }
  } else if (!tables_given && !dc_last) {
    a.zero_pack = !a.seg_dc;  // one wave per table: it zeroes the pack state too
    a.tab_dc_only = actab;
    HIP_TRY(launch_tables(a, st));
    a.tab_dc_only = 0;
  }
  b->hist_zero_after = (f0 == 0 && a.zero_pack) ? nframes : 0;
  if (t) HIP_TRY(hipEventRecord(b->ev[5], st));
  // segment bits, scan offsets and packing in one look-back pass
  // Seam mode (default; MIJ_OPT_SEAM=0 for the A/B): every scan word is stored
  // whole by one pack group; a group's first word, when shared with the group
  // before it, goes to seam[] and k_seam_fix ORs it in after the packing --
  // the scan buffers need not start zeroed (no atomics in k_pack_flat), and
  // k_emit_write does not zero them after reading.  The other paths (bands,
  // assembly) still OR onto zero: they clear what this leaves (raw_dirty).
  if (b->opt[MIJ_OPT_SEAM] && b->d_seam) {
    a.seam = b->d_seam + (long long)f0 * pack_stride(b->g);
    // the 0xFF bytes of every emit chunk counted as the words are stored
    // (no k_emit_count pass over the scan words; A/B: MIJ_OPT_FF_PACK=0)
    a.ff_pack = b->opt[MIJ_OPT_FF_PACK] != 0;
    b->raw_dirty = std::max(b->raw_dirty, f0 + nframes);
  } else if (b->raw_dirty) {
    HIP_TRY(hipMemsetAsync(b->d_raw, 0, sizeof(uint32_t) * b->raw_dirty * b->g.raw_fs, st));
    b->raw_dirty = 0;
  }
  // diagnostics (MIJ_PACK_TIME with the diag build): per-group phase times of k_pack_flat
  static const bool ptime = diag_env("MIJ_PACK_TIME", 0) != 0;
  const long long nwords = (long long)nframes * pack_stride(b->g);  // per-group words (look-back, seam)
  if (ptime) {
    HIP_TRY(hipMalloc(&a.dbg, sizeof(unsigned long long) * 6 * nwords));
    HIP_TRY(hipMemsetAsync(a.dbg, 0, sizeof(unsigned long long) * 6 * nwords, st));
  }
  if (b->opt[OPT_TEST_FAULT_TICKET] && f0 == 0) {
    // fault injection (tests): frame 0's luma ticket starts past group 0
    const int v = b->opt[OPT_TEST_FAULT_TICKET];
    b->opt[OPT_TEST_FAULT_TICKET] = 0;
    if (!a.zero_pack) {
      HIP_TRY(hipMemsetAsync(a.pack_state, 0, sizeof(unsigned long long) * nwords, st));
      HIP_TRY(hipMemsetAsync(a.pack_ticket, 0, sizeof(unsigned) * 3 * nframes, st));
    }
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)a.pack_ticket, v, 1, st));
    HIP_TRY(launch_pack(a, st, true));
  } else {
    HIP_TRY(launch_pack(a, st, a.zero_pack != 0));
  }
  // the seam fixes inside k_emit_scan on small batches (one frame: 0.080 ->
  // 0.073 ms with the error words zeroed by K1; at config 3 the per-frame
  // serial fixes cost emit ~20 us, more than the launch)
  a.seam_in_scan = a.seam && a.ff_pack && nframes < 16;
  if (a.seam && !a.seam_in_scan) HIP_TRY(launch_seam_fix(a, st));
  if (ptime) {
    std::vector<unsigned long long> h(6 * nwords);
    HIP_TRY(hipMemcpyAsync(h.data(), a.dbg, sizeof(unsigned long long) * 6 * nwords, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipFree(a.dbg));
    a.dbg = nullptr;
    // k_pack_flat's stamps: start, counts ready, sweep done, look-back done,
    // end, [5] ticket and code table in (groups on the windowed path are not
    // stamped); luma and chroma groups apart
    const PackGrid P = pack_grid(a);
    double ph[2][5] = {{0}};
    long long cnt[2] = {0, 0};
    unsigned long long t0 = ~0ull, t1 = 0;
    for (long long g = 0; g < nwords; g++) {
      const unsigned long long *r = &h[6 * g];
      if (!r[4]) continue;
      const int kind = (g % P.stride) >= P.gy;
      for (int k = 0; k < 4; k++) ph[kind][k] += (double)(r[k + 1] - r[k]);
      ph[kind][4] += (double)(r[5] - r[0]);
      cnt[kind]++;
      t0 = std::min(t0, r[0]);
      t1 = std::max(t1, r[4]);
    }
    // s_memrealtime ticks at 100 MHz
    for (int kind = 0; kind < 2; kind++)
      if (cnt[kind])
        fprintf(stderr, "pack %s groups %lld (%d segments): span %.1f us, per group: ticket+counts %.2f us "
                "(ticket + code table %.2f), sweep %.2f us, look-back %.2f us, store %.2f us\n",
                kind ? "chroma" : "luma", cnt[kind], PACK_SEGS << a.pack_ls[kind], (t1 - t0) / 100.0,
                ph[kind][0] / cnt[kind] / 100.0, ph[kind][4] / cnt[kind] / 100.0, ph[kind][1] / cnt[kind] / 100.0,
                ph[kind][2] / cnt[kind] / 100.0, ph[kind][3] / cnt[kind] / 100.0);
  }
  if (t) HIP_TRY(hipEventRecord(b->ev[6], st));
  HIP_TRY(launch_emit(a, st));
  if (t) HIP_TRY(hipEventRecord(b->ev[7], st));
  return MIJ_OK;
}

static int encode_frames(mij_batch *b, int nframes) {
  if (nframes > b->hist_zero_n)
    HIP_TRY(hipMemsetAsync(b->d_hist, 0, sizeof(uint32_t) * nframes * 4 * 257, b->stream));
  b->hist_zero_n = 0;
  // region batches: K1 skips the canvas tiles outside a frame, so their
  // segments must read as empty
  if (b->use_fdims && b->rgb) return fail(MIJ_EINVAL, "encode: region batches read B, G, R frames");
  if (b->use_fdims)
    HIP_TRY(hipMemsetAsync(b->d_seg_ntok, 0, sizeof(uint32_t) * nframes * b->g.nseg, b->stream));
  // (d_err: zeroed by the first K1 below -- nothing before k_tables writes it;
  // a memset launch is 4-5 us of a one-frame step)
  b->k1_err_zero = nframes;
  if (b->timing) HIP_TRY(hipEventRecord(b->ev[0], b->stream));
  const int nsub = std::min(b->overlap, nframes);
  if (!b->split && !b->keep_coefs && nsub > 1) {
    // sub-batches: K1 of sub-batch k on the batch stream, its entropy stages
    // on stream2 behind it, concurrent with K1 of sub-batch k + 1; the batch
    // stream then waits for stream2, so syncing it covers the whole encode
    const int per = (nframes + nsub - 1) / nsub;
    for (int k = 0, f0 = 0; f0 < nframes; k++, f0 += per) {
      const int nk = std::min(per, nframes - f0);
      if (run_k1(b, nk, 2, 0, 0, f0, false)) return g_err;
      HIP_TRY(hipEventRecord(b->ov_k1[k], b->stream));
      HIP_TRY(hipStreamWaitEvent(b->stream2, b->ov_k1[k], 0));
      if (run_entropy(b, nk, true, false, f0, b->stream2)) return g_err;
    }
    if (b->timing)
      for (int e = 1; e <= 3; e++) HIP_TRY(hipEventRecord(b->ev[e], b->stream));  // K1 over all sub-batches
    HIP_TRY(hipEventRecord(b->ov_done, b->stream2));
    HIP_TRY(hipStreamWaitEvent(b->stream, b->ov_done, 0));
    if (b->timing)
      for (int e = 4; e < MIJ_NSTAGES; e++) HIP_TRY(hipEventRecord(b->ev[e], b->stream));
    return MIJ_OK;
  }
  if (b->split) {
    if (run_k1(b, nframes, 1)) return g_err;  // records events 1 and 2 around the fixer
    if (run_k1(b, nframes, 6, 0, 1)) return g_err;  // segment-first DCs inline: no k_seg_dc
  } else {
    if (run_k1(b, nframes, b->keep_coefs ? 3 : 2)) return g_err;  // events 1 and 2 (no fixer)
  }
  if (b->timing) HIP_TRY(hipEventRecord(b->ev[3], b->stream));
  if (run_entropy(b, nframes, !b->split, false)) return g_err;
  // (run_entropy's k_tables_1w zeroed the counts it read)
  b->hist_zero_n = b->hist_zero_after;
  return MIJ_OK;
}

static void next_slot(mij_batch *b) {
  if (b->timing) b->ev = b->evh[b->steps++ % mij_batch::HIST];
}

extern "C" int mij_batch_encode(mij_batch *b, int nframes) {
  if (pipe_check(b, "encode")) return g_err;
  if (nframes < 1 || nframes > b->cap) return fail(MIJ_EINVAL, "encode: bad frame count");
  HIP_TRY(hipSetDevice(b->dev));
  next_slot(b);
  if (encode_frames(b, nframes)) return g_err;
  b->last_frames = nframes;
  return MIJ_OK;
}

extern "C" int mij_batch_keep_coefs(mij_batch *b, int on) {
  if (pipe_check(b, "keep_coefs")) return g_err;
  b->keep_coefs = on != 0;
  return MIJ_OK;
}

extern "C" int mij_batch_set_rgb(mij_batch *b, int on) {
  if (pipe_check(b, "set_rgb")) return g_err;
  b->rgb = on != 0;
  return MIJ_OK;
}

// ---- region batches --------------------------------
static int check_frame_dims(const mij_batch *b, int w, int h, const char *what, int i) {
  if (!valid_dims(w, h) || w > b->g.w || h > b->g.h)
    return fail(MIJ_EINVAL, "%s: frame %d is %dx%d (multiples of 16, at most the batch's %dx%d)", what, i,
                w, h, b->g.w, b->g.h);
  return MIJ_OK;
}

// per-frame sizes, queued on the batch stream (the kernels read them there)
static int upload_frame_dims(mij_batch *b, const int2 *wh, int n) {
  for (int i = 0; i < b->cap; i++) b->h_fdims[i] = i < n ? wh[i] : make_int2(b->g.w, b->g.h);
  HIP_TRY(hipMemcpyAsync(b->d_fdims, b->h_fdims.data(), sizeof(int2) * b->cap, hipMemcpyHostToDevice,
                         b->stream));
  // the pageable source is read before the call returns only with a sync
  HIP_TRY(hipStreamSynchronize(b->stream));
  b->use_fdims = true;
  return MIJ_OK;
}

extern "C" int mij_batch_set_frame_dims(mij_batch *b, const int *wh, int nframes) {
  if (!b) return fail(MIJ_EINVAL, "set_frame_dims: null batch");
  HIP_TRY(hipSetDevice(b->dev));
  if (!wh) {
    b->use_fdims = false;
    return MIJ_OK;
  }
  if (nframes < 1 || nframes > b->cap) return fail(MIJ_EINVAL, "set_frame_dims: bad frame count");
  std::vector<int2> v(nframes);
  for (int i = 0; i < nframes; i++) {
    if (check_frame_dims(b, wh[2 * i], wh[2 * i + 1], "set_frame_dims", i)) return g_err;
    v[i] = make_int2(wh[2 * i], wh[2 * i + 1]);
  }
  return upload_frame_dims(b, v.data(), nframes);
}

// regions of one frame in device memory (rows src_pitch bytes apart, frame
// frame_w x frame_h pixels) into slots 0..n-1, each slot's size set to its
// region's; one gather launch on the batch stream
static int gather_regions(mij_batch *b, const uint8_t *d_src, long long src_pitch, int frame_w,
                          int frame_h, const area_t *regions, int n) {
  if (!b->own_in) return fail(MIJ_EINVAL, "regions: batch reads external device input");
  if (n < 1 || n > b->cap || !regions) return fail(MIJ_EINVAL, "regions: bad region count %d", n);
  std::vector<int4> r(n);
  std::vector<int2> wh(n);
  int max_h = 0;
  for (int i = 0; i < n; i++) {
    const area_t d = regions[i];
    if (check_frame_dims(b, d.w, d.h, "regions", i)) return g_err;
    if (d.x < 0 || d.y < 0 || d.x + d.w > frame_w || d.y + d.h > frame_h)
      return fail(MIJ_EINVAL, "regions: region %d (%d,%d %dx%d) outside the %dx%d frame", i, d.x, d.y,
                  d.w, d.h, frame_w, frame_h);
    r[i] = make_int4(d.x, d.y, d.w, d.h);
    wh[i] = make_int2(d.w, d.h);
    max_h = d.h > max_h ? d.h : max_h;
  }
  HIP_TRY(hipMemcpyAsync(b->d_regions, r.data(), sizeof(int4) * n, hipMemcpyHostToDevice, b->stream));
  HIP_TRY(launch_gather_regions(b->d_in, b->in_fs, b->pitch, d_src, src_pitch, b->d_regions, n, max_h,
                                b->stream));
  return upload_frame_dims(b, wh.data(), n);  // synchronises (pageable sources)
}

extern "C" int mij_batch_gather_regions(mij_batch *b, const void *d_frame, long long pitch, int frame_w,
                                        int frame_h, const area_t *regions, int n) {
  if (pipe_check(b, "gather_regions")) return g_err;
  if (!d_frame || pitch < 3LL * frame_w) return fail(MIJ_EINVAL, "gather_regions: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  return gather_regions(b, (const uint8_t *)d_frame, pitch, frame_w, frame_h, regions, n);
}

extern "C" int mij_batch_upload_regions(mij_batch *b, const uint8_t *bgr, int stride_px, int frame_h,
                                        const area_t *regions, int n) {
  if (pipe_check(b, "upload_regions")) return g_err;
  if (!bgr || stride_px < 16 || frame_h < 16) return fail(MIJ_EINVAL, "upload_regions: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  const size_t bytes = (size_t)stride_px * frame_h * 3;
  if (bytes > b->frame_cap) {
    if (b->d_frame) HIP_TRY(hipFree(b->d_frame));
    b->d_frame = nullptr;
    b->frame_cap = 0;
    HIP_TRY(hipMalloc((void **)&b->d_frame, bytes));
    b->frame_cap = bytes;
  }
  HIP_TRY(hipMemcpyAsync(b->d_frame, bgr, bytes, hipMemcpyHostToDevice, b->stream));
  return gather_regions(b, b->d_frame, 3LL * stride_px, stride_px, frame_h, regions, n);
}

// ---- asynchronous host transfers for the streaming engine (mij_stream.hip):
// queued on the batch stream, no synchronisation
// (runs on the stream's reader threads: the checks of pipe_check -- no
// assembler -- are inline, and a region batch is refused outright, so no slot
// needs canvas_frames' size reset; the caller re-raises a failure's message
// on its own thread, mij_stream.hip join_read)
int mij_batch_upload_slot_async(mij_batch *b, const uint8_t *host, int slot, void *stream) {
  if (!b || b->assembler || !host || slot < 0 || slot >= b->cap || !b->own_in || b->use_fdims)
    return fail(MIJ_EINVAL, "upload_slot_async: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipMemcpyAsync(b->d_in + (long long)slot * b->in_fs, host, (size_t)b->in_fs, hipMemcpyHostToDevice,
                         stream ? (hipStream_t)stream : b->stream));
  return MIJ_OK;
}
int mij_batch_lengths_async(mij_batch *b, uint64_t *h_len, int *h_err, int nframes) {
  if (!b || nframes < 1 || nframes > b->cap) return fail(MIJ_EINVAL, "lengths_async: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipMemcpyAsync(h_len, b->d_out_len, sizeof(uint64_t) * nframes, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipMemcpyAsync(h_err, b->d_err, sizeof(int) * nframes, hipMemcpyDeviceToHost, b->stream));
  return MIJ_OK;
}
int mij_batch_output_async(mij_batch *b, int frame, uint8_t *dst, size_t n) {
  if (!b || frame < 0 || frame >= b->cap || n > (size_t)b->g.out_cap)
    return fail(MIJ_EINVAL, "output_async: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipMemcpyAsync(dst, b->d_out + (long long)frame * b->g.out_cap, n, hipMemcpyDeviceToHost, b->stream));
  return MIJ_OK;
}

extern "C" int mij_batch_set_split(mij_batch *b, int on) {
  if (pipe_check(b, "set_split")) return g_err;
  b->split = on != 0;
  return MIJ_OK;
}

extern "C" int mij_batch_set_overlap(mij_batch *b, int nsub) {
  if (pipe_check(b, "set_overlap")) return g_err;
  if (nsub < 1 || nsub > 16) return fail(MIJ_EINVAL, "set_overlap: 1..16 sub-batches");
  HIP_TRY(hipSetDevice(b->dev));
  if (nsub > 1 && !b->stream2) {
    // the entropy stream at the highest priority: its small workgroups take
    // the CU room the running K1 leaves before the next K1's do
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(hipStreamCreateWithPriority(&b->stream2, hipStreamNonBlocking, b->opt[MIJ_OPT_OVERLAP_PRIO] ? hi : lo));
    for (auto &e : b->ov_k1) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&b->ov_done, hipEventDisableTiming));
  }
  b->overlap = nsub;
  return MIJ_OK;
}

extern "C" int mij_batch_set_option(mij_batch *b, int opt, int value) {
  // (an assembler emits the frames: its emission slots are its one option)
  if (!(b && b->assembler && opt == MIJ_OPT_EMIT_SLOTS) && pipe_check(b, "set_option")) return g_err;
  if (opt < 0 || opt >= MIJ_OPT_COUNT) return fail(MIJ_EINVAL, "set_option: unknown option %d", opt);
  if (opt == OPT_TEST_FAULT_TICKET) return fail(MIJ_EINVAL, "set_option: unknown option %d", opt);
  const bool binary = opt != MIJ_OPT_PACK_WIDE && opt != MIJ_OPT_EMIT_SLOTS && opt != MIJ_OPT_PACK_SEGS;
  if ((binary && value != 0 && value != 1) || (opt == MIJ_OPT_PACK_WIDE && (value < -1 || value > 1)) ||
      (opt == MIJ_OPT_EMIT_SLOTS && (value < 0 || value > 4096)) ||
      (opt == MIJ_OPT_PACK_SEGS && (value < -1 || value > 15)))
    return fail(MIJ_EINVAL, "set_option: value %d out of range for option %d", value, opt);
  if (opt == MIJ_OPT_OVERLAP_PRIO && b->stream2)
    return fail(MIJ_EINVAL, "set_option: the overlap stream exists already (set the priority before set_overlap)");
  b->opt[opt] = value;
  return MIJ_OK;
}

extern "C" int mij_batch_get_option(mij_batch *b, int opt) {
  if (!b || opt < 0 || opt >= MIJ_OPT_COUNT || opt == OPT_TEST_FAULT_TICKET)
    return fail(MIJ_EINVAL, "get_option: bad args"), -2;
  return b->opt[opt];
}

// test-only (csrc/mij_testing.h, not the public header): arm the stale-ticket
// fault for the next encode; returns the value that was armed before
extern "C" int mij_test_stale_ticket(mij_batch *b, int v) {
  if (!b || v < 0 || v > 1 << 20) return fail(MIJ_EINVAL, "test_stale_ticket: bad args"), -2;
  const int old = b->opt[OPT_TEST_FAULT_TICKET];
  b->opt[OPT_TEST_FAULT_TICKET] = v;
  return old;
}

extern "C" int mij_batch_dct(mij_batch *b, int nframes) {
  if (pipe_check(b, "dct")) return g_err;
  if (nframes < 1 || nframes > b->cap) return fail(MIJ_EINVAL, "dct: bad frame count");
  HIP_TRY(hipSetDevice(b->dev));
  next_slot(b);
  if (b->timing) HIP_TRY(hipEventRecord(b->ev[0], b->stream));
  if (run_k1(b, nframes, 1)) return g_err;  // events 1, 2
  if (b->timing)
    for (int k = 3; k < MIJ_NSTAGES; k++) HIP_TRY(hipEventRecord(b->ev[k], b->stream));
  return MIJ_OK;
}

// measurement only: K1's memory traffic without its arithmetic (k_mcu_dct
// <COEF_OUT | FLOOR>) on frames 0..n-1, timed like mij_batch_dct (stage
// events); the coefficient planes are left holding garbage
extern "C" int mij_batch_pattern_floor(mij_batch *b, int nframes) {
  if (pipe_check(b, "pattern_floor")) return g_err;
  if (nframes < 1 || nframes > b->cap) return fail(MIJ_EINVAL, "pattern_floor: bad frame count");
  if (b->rgb || b->use_fdims) return fail(MIJ_EINVAL, "pattern_floor: plain B, G, R batches only");
  HIP_TRY(hipSetDevice(b->dev));
  next_slot(b);
  if (b->timing) HIP_TRY(hipEventRecord(b->ev[0], b->stream));
  if (run_k1(b, nframes, 1 | 64)) return g_err;  // K1M_COEF_OUT | K1M_FLOOR; events 1, 2
  if (b->timing)
    for (int k = 3; k < MIJ_NSTAGES; k++) HIP_TRY(hipEventRecord(b->ev[k], b->stream));
  return MIJ_OK;
}

// tests: the coefficient K1 on frames 0..n-1 through its audit variant,
// which also exports every block's fast-path keep/replay decisions
extern "C" int mij_batch_audit(mij_batch *b, int nframes, uint16_t *masks) {
  if (pipe_check(b, "audit")) return g_err;
  if (nframes < 1 || nframes > b->cap || !masks) return fail(MIJ_EINVAL, "audit: bad arguments");
  if (b->rgb || b->use_fdims) return fail(MIJ_EINVAL, "audit: plain B, G, R batches only");
  HIP_TRY(hipSetDevice(b->dev));
  const size_t n = (size_t)nframes * b->g.nblk * 4;
  if (b->audit_cap < n) {
    if (b->d_audit) HIP_TRY(hipFree(b->d_audit));
    b->d_audit = nullptr;
    b->audit_cap = 0;
    HIP_TRY(dalloc(&b->d_audit, n));
    b->audit_cap = n;
  }
  HIP_TRY(hipMemsetAsync(b->d_audit, 0, sizeof(uint16_t) * n, b->stream));
  b->audit = true;
  const int rc = run_k1(b, nframes, 1);
  b->audit = false;
  if (rc) return g_err;
  HIP_TRY(hipMemcpyAsync(masks, b->d_audit, sizeof(uint16_t) * n, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_batch_sync(mij_batch *b) {
  if (!b) return fail(MIJ_EINVAL, "sync: null batch");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_batch_set_timing(mij_batch *b, int on) {
  if (!b) return fail(MIJ_EINVAL, "set_timing: null batch");
  b->timing = on != 0;
  b->steps = 0;
  b->ev = b->evh[0];
  return MIJ_OK;
}

static float elapsed(hipEvent_t a, hipEvent_t z) {
  float v = -1.0f;
  if (hipEventElapsedTime(&v, a, z) != hipSuccess) v = -1.0f;
  return v;
}

// stage i spans events (i, i+1); the last one is the whole encode
// events: 0 start, 1 after K1, 2 after the fixer, 3 after tokenize, 4 after
// the segment DC fixup, 5 after the tables, 6 after pack, 7 after emit
static const int k_stage_pairs[MIJ_NSTAGES][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4},
                                                  {4, 5}, {5, 6}, {6, 7}, {0, 7}};

extern "C" int mij_batch_stage_history(mij_batch *b, float *ms, int steps) {
  if (!b || !ms || steps < 1) return fail(MIJ_EINVAL, "stage_history: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipStreamSynchronize(b->stream));
  long long have = b->steps < mij_batch::HIST ? b->steps : mij_batch::HIST;
  int n = (int)(steps < have ? steps : have);
  for (int i = 0; i < n; i++) {
    const long long step = b->steps - n + i;
    hipEvent_t *e = b->evh[step % mij_batch::HIST];
    for (int k = 0; k < MIJ_NSTAGES; k++) ms[i * MIJ_NSTAGES + k] = elapsed(e[k_stage_pairs[k][0]], e[k_stage_pairs[k][1]]);
  }
  return n;
}

extern "C" int mij_batch_stage_ms(mij_batch *b, float *ms, int n) {
  if (!b || !ms) return fail(MIJ_EINVAL, "stage_ms: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipStreamSynchronize(b->stream));
  for (int i = 0; i < n && i < MIJ_NSTAGES; i++) ms[i] = elapsed(b->ev[k_stage_pairs[i][0]], b->ev[k_stage_pairs[i][1]]);
  return MIJ_OK;
}

extern "C" unsigned long long mij_batch_token_count(mij_batch *b, int nframes) {
  if (!b || b->assembler || nframes < 1 || nframes > b->cap) return 0;
  hipSetDevice(b->dev);
  hipStreamSynchronize(b->stream);
  std::vector<uint32_t> v((size_t)nframes * b->g.nseg);
  if (hipMemcpy(v.data(), b->d_seg_ntok, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return 0;
  unsigned long long n = 0;
  for (uint32_t x : v) n += x;
  return n;
}

extern "C" int mij_batch_geometry(mij_batch *b, long long *out, int n) {
  if (!b || !out) return fail(MIJ_EINVAL, "geometry: bad args");
  // ... then k_pack_flat's LDS window (words) at this batch's quality
  const long long win = ent_args_pack_wide(b) ? PACK_WIDE_WORDS : PACK_WORDS;
  const long long v[] = {b->g.w, b->g.h, b->g.nblk, b->g.nseg, b->g.tiles_per_frame, win};
  const int nv = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < nv; i++) out[i] = v[i];
  return MIJ_OK;
}

extern "C" unsigned long long mij_batch_replays(mij_batch *b) {
  if (!b) return 0;
  unsigned v = 0;
  hipSetDevice(b->dev);
  hipStreamSynchronize(b->stream);
  hipMemcpy(&v, b->d_replays, sizeof(v), hipMemcpyDeviceToHost);
  return v;
}

extern "C" int mij_batch_lengths(mij_batch *b, size_t *lens, int nframes) {
  if (!b || !lens || nframes < 1 || nframes > b->cap) return fail(MIJ_EINVAL, "lengths: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipStreamSynchronize(b->stream));
  std::vector<uint64_t> v(nframes);
  HIP_TRY(hipMemcpy(v.data(), b->d_out_len, sizeof(uint64_t) * nframes, hipMemcpyDeviceToHost));
  for (int i = 0; i < nframes; i++) lens[i] = (size_t)v[i];
  return MIJ_OK;
}

extern "C" int mij_batch_output(mij_batch *b, int frame, uint8_t *dst, size_t cap, size_t *len) {
  if (!b || frame < 0 || frame >= b->cap) return fail(MIJ_EINVAL, "output: bad frame");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipStreamSynchronize(b->stream));
  uint64_t n = 0;
  int err = 0;
  HIP_TRY(hipMemcpy(&n, b->d_out_len + frame, sizeof(n), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&err, b->d_err + frame, sizeof(err), hipMemcpyDeviceToHost));
  if (err) return mij_frame_fail(err, "frame", frame);
  if (len) *len = (size_t)n;
  if (dst) {
    if (cap < n) return fail(MIJ_ENOSPC, "output: need %llu bytes", (unsigned long long)n);
    HIP_TRY(hipMemcpy(dst, b->d_out + (long long)frame * b->g.out_cap, n, hipMemcpyDeviceToHost));
  }
  return MIJ_OK;
}

extern "C" int mij_batch_coefs(mij_batch *b, int frame, int16_t *Y, int16_t *Cb, int16_t *Cr,
                               int diffed) {
  if (pipe_check(b, "coefs")) return g_err;
  if (frame < 0 || frame >= b->cap) return fail(MIJ_EINVAL, "coefs: bad frame");
  HIP_TRY(hipSetDevice(b->dev));
  const Geom &g0 = b->g;
  // the frame's own planes (region batches: its w x h, not the canvas)
  const FGeom g = frame_geom(g0, b->use_fdims ? b->h_fdims.data() : nullptr, frame);
  int16_t *base = b->d_coef + (long long)frame * g0.coef_fs;
  int16_t *tmp = nullptr;
  if (diffed) {  // differenced copy, leaving the batch's planes raw
    HIP_TRY(hipMalloc((void **)&tmp, sizeof(int16_t) * g0.coef_fs));
    HIP_TRY(hipMemcpyAsync(tmp, base, sizeof(int16_t) * g0.coef_fs, hipMemcpyDeviceToDevice,
                           b->stream));
    HIP_TRY(launch_dc_diff(tmp, b->d_dc + (long long)frame * g0.nblk, g0, 1,
                           b->use_fdims ? b->d_fdims + frame : nullptr, b->stream));
    base = tmp;
  }
  HIP_TRY(hipStreamSynchronize(b->stream));
  hipError_t e = hipMemcpy(Y, base, sizeof(int16_t) * g.nY * 64, hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    e = hipMemcpy(Cb, base + (long long)g.nY * 64, sizeof(int16_t) * g.nC * 64,
                  hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    e = hipMemcpy(Cr, base + (long long)(g.nY + g.nC) * 64, sizeof(int16_t) * g.nC * 64,
                  hipMemcpyDeviceToHost);
  if (tmp) hipFree(tmp);
  HIP_TRY(e);
  return MIJ_OK;
}

extern "C" int mij_batch_tables(mij_batch *b, int frame, huff_code out[4]) {
  if (!b || !out || frame < 0 || frame >= b->cap) return fail(MIJ_EINVAL, "tables: bad args");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipStreamSynchronize(b->stream));
  HIP_TRY(hipMemcpy(out, b->d_hc + (long long)frame * 4, sizeof(HuffCode) * 4,
                    hipMemcpyDeviceToHost));
  return MIJ_OK;
}

// ---------------------------------------------------------------------------
// drop-in entry points: one lazily created single-frame pipeline
// ---------------------------------------------------------------------------
static std::mutex g_mu;
static mij_batch *g_ctx = nullptr;
static int g_stride = 320;  // define.h:3 WIDTH
static int g_quality = 50;

static int drop_device() {
  const char *e = getenv("MIJ_DEVICE");
  return e ? atoi(e) : 0;
}

static mij_batch *ctx_for(int w, int h, int quality) {
  if (g_ctx && g_ctx->g.w == w && g_ctx->g.h == h && g_ctx->quality == quality) return g_ctx;
  batch_free(g_ctx);
  g_ctx = mij_batch_create(drop_device(), w, h, 1, quality);
  return g_ctx;
}

// for the other host translation units (the drop-in detector, mij_detect.hip)
int mij_drop_stride() {
  std::lock_guard<std::mutex> l(g_mu);
  return g_stride;
}
int mij_drop_device() { return drop_device(); }

extern "C" int mij_set_input_stride(int stride_px) {
  if (stride_px < 16) return fail(MIJ_EINVAL, "stride %d", stride_px);
  std::lock_guard<std::mutex> l(g_mu);
  g_stride = stride_px;
  return MIJ_OK;
}

extern "C" int mij_set_quality(int quality) {
  if (quality < 1 || quality > 100) return fail(MIJ_EINVAL, "quality %d", quality);
  std::lock_guard<std::mutex> l(g_mu);
  g_quality = quality;
  return MIJ_OK;
}

static int upload_region(mij_batch *b, const uint8_t *in, int stride, area_t d) {
  if (d.x < 0 || d.y < 0 || d.x + d.w > stride)
    return fail(MIJ_EINVAL, "region x=%d w=%d outside stride %d", d.x, d.w, stride);
  const uint8_t *src = in + ((size_t)d.y * stride + d.x) * 3;
  HIP_TRY(hipMemcpy2DAsync(b->d_in, (size_t)d.w * 3, src, (size_t)stride * 3, (size_t)d.w * 3,
                           d.h, hipMemcpyHostToDevice, b->stream));
  return MIJ_OK;
}

static int upload_planes(mij_batch *b, const int16_t *Y, const int16_t *Cb, const int16_t *Cr) {
  const Geom &g = b->g;
  HIP_TRY(hipMemcpyAsync(b->d_coef, Y, sizeof(int16_t) * g.nY * 64, hipMemcpyHostToDevice,
                         b->stream));
  HIP_TRY(hipMemcpyAsync(b->d_coef + (long long)g.nY * 64, Cb, sizeof(int16_t) * g.nC * 64,
                         hipMemcpyHostToDevice, b->stream));
  HIP_TRY(hipMemcpyAsync(b->d_coef + (long long)(g.nY + g.nC) * 64, Cr,
                         sizeof(int16_t) * g.nC * 64, hipMemcpyHostToDevice, b->stream));
  return MIJ_OK;
}

extern "C" void rgb_to_dct(uint8_t *in, int16_t *Y, int16_t *Cb, int16_t *Cr, area_t dims) {
  std::lock_guard<std::mutex> l(g_mu);
  g_err = MIJ_OK;
  if (!in || !Y || !Cb || !Cr || !valid_dims(dims.w, dims.h)) {
    fail(MIJ_EINVAL, "rgb_to_dct: null buffer or dims %dx%d not multiples of 16", dims.w, dims.h);
    return;
  }
  mij_batch *b = ctx_for(dims.w, dims.h, g_quality);
  if (!b) return;
  if (upload_region(b, in, g_stride, dims)) return;
  if (run_k1(b, 1, 1)) return;
  if (launch_dc_diff(b->d_coef, b->d_dc, b->g, 1, nullptr, b->stream) != hipSuccess) {
    fail(MIJ_EHIP, "dc_diff launch failed");
    return;
  }
  const Geom &g = b->g;
  if (hipStreamSynchronize(b->stream) != hipSuccess ||
      hipMemcpy(Y, b->d_coef, sizeof(int16_t) * g.nY * 64, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(Cb, b->d_coef + (long long)g.nY * 64, sizeof(int16_t) * g.nC * 64,
                hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(Cr, b->d_coef + (long long)(g.nY + g.nC) * 64, sizeof(int16_t) * g.nC * 64,
                hipMemcpyDeviceToHost) != hipSuccess)
    fail(MIJ_EHIP, "rgb_to_dct: device copy failed");
}

extern "C" void init_huffman(int16_t *Y, int16_t *Cb, int16_t *Cr, area_t dims,
                             huff_code Luma[2], huff_code Chroma[2]) {
  std::lock_guard<std::mutex> l(g_mu);
  g_err = MIJ_OK;
  if (!Y || !Cb || !Cr || !Luma || !Chroma || !valid_dims(dims.w, dims.h)) {
    fail(MIJ_EINVAL, "init_huffman: bad arguments");
    return;
  }
  mij_batch *b = ctx_for(dims.w, dims.h, g_quality);
  if (!b || upload_planes(b, Y, Cb, Cr)) return;
  EntArgs a = ent_args(b, 1);
  if (hipMemsetAsync(b->d_hist, 0, sizeof(uint32_t) * 4 * 257, b->stream) != hipSuccess ||
      hipMemsetAsync(b->d_err, 0, sizeof(int), b->stream) != hipSuccess || run_k1(b, 1, 6, 1) ||
      launch_tables(a, b->stream) != hipSuccess) {
    fail(MIJ_EHIP, "init_huffman: launch failed");
    return;
  }
  HuffCode t[4];
  int err = 0;
  if (hipStreamSynchronize(b->stream) != hipSuccess ||
      hipMemcpy(t, b->d_hc, sizeof(t), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) {
    fail(MIJ_EHIP, "init_huffman: device copy failed");
    return;
  }
  if (err) mij_frame_fail(err, "init_huffman: frame", 0);
  memcpy(&Luma[0], &t[0], sizeof(HuffCode));
  memcpy(&Luma[1], &t[1], sizeof(HuffCode));
  memcpy(&Chroma[0], &t[2], sizeof(HuffCode));
  memcpy(&Chroma[1], &t[3], sizeof(HuffCode));
}

extern "C" size_t write_jpg(FILE *f, uint8_t *jpg, int16_t *Y, int16_t *Cb, int16_t *Cr,
                            area_t dims, huff_code Luma[2], huff_code Chroma[2]) {
  std::lock_guard<std::mutex> l(g_mu);
  g_err = MIJ_OK;
  if (!jpg || !Y || !Cb || !Cr || !Luma || !Chroma || !valid_dims(dims.w, dims.h)) {
    fail(MIJ_EINVAL, "write_jpg: bad arguments");
    return 0;
  }
  mij_batch *b = ctx_for(dims.w, dims.h, g_quality);
  if (!b || upload_planes(b, Y, Cb, Cr)) return 0;
  HuffCode t[4];
  memcpy(&t[0], &Luma[0], sizeof(HuffCode));
  memcpy(&t[1], &Luma[1], sizeof(HuffCode));
  memcpy(&t[2], &Chroma[0], sizeof(HuffCode));
  memcpy(&t[3], &Chroma[1], sizeof(HuffCode));
  if (hipMemcpyAsync(b->d_hc, t, sizeof(t), hipMemcpyHostToDevice, b->stream) != hipSuccess ||
      hipMemsetAsync(b->d_err, 0, sizeof(int), b->stream) != hipSuccess ||
      launch_ehuf_struct(b->d_hc, b->d_ehuf, b->stream) != hipSuccess) {
    fail(MIJ_EHIP, "write_jpg: table upload failed");
    return 0;
  }
  if (hipMemsetAsync(b->d_hist, 0, sizeof(uint32_t) * 4 * 257, b->stream) != hipSuccess ||
      run_k1(b, 1, 6, 1) || run_entropy(b, 1, false, true))
    return 0;
  size_t n = 0;
  if (hipStreamSynchronize(b->stream) != hipSuccess) {
    fail(MIJ_EHIP, "write_jpg: stream failed");
    return 0;
  }
  uint64_t n64 = 0;
  if (hipMemcpy(&n64, b->d_out_len, sizeof(n64), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(jpg, b->d_out, n64, hipMemcpyDeviceToHost) != hipSuccess) {
    fail(MIJ_EHIP, "write_jpg: device copy failed");
    return 0;
  }
  n = (size_t)n64;
  if (f && fwrite(jpg, 1, n, f) != n) fail(MIJ_EINVAL, "write_jpg: short write to FILE*");
  return n;
}

extern "C" int mij_encode(const uint8_t *bgr, int stride_px, area_t dims, int quality,
                          uint8_t *out, size_t cap, size_t *out_len) {
  std::lock_guard<std::mutex> l(g_mu);
  g_err = MIJ_OK;
  if (!bgr || !out || !valid_dims(dims.w, dims.h) || quality < 1 || quality > 100)
    return fail(MIJ_EINVAL, "mij_encode: bad arguments");
  mij_batch *b = ctx_for(dims.w, dims.h, quality);
  if (!b) return g_err;
  if (upload_region(b, bgr, stride_px, dims)) return g_err;
  if (encode_frames(b, 1)) return g_err;
  size_t n = 0;
  if (mij_batch_output(b, 0, nullptr, 0, &n)) return g_err;
  if (n > cap) return fail(MIJ_ENOSPC, "mij_encode: need %zu bytes", n);
  if (mij_batch_output(b, 0, out, cap, &n)) return g_err;
  if (out_len) *out_len = n;
  return MIJ_OK;
}

// main.c:142-155 in one call: every region of a BGR frame its own JPEG, all
// regions through one region batch (canvas = the largest region)
static mij_batch *g_rctx = nullptr;

extern "C" int mij_encode_regions(const uint8_t *bgr, int stride_px, int frame_h, const area_t *regions,
                                  int n, int quality, uint8_t *out, size_t cap, size_t *lens) {
  std::lock_guard<std::mutex> l(g_mu);
  g_err = MIJ_OK;
  if (!bgr || !regions || n < 1 || !out || !lens || quality < 1 || quality > 100)
    return fail(MIJ_EINVAL, "mij_encode_regions: bad arguments");
  int W = 16, H = 16;
  for (int i = 0; i < n; i++) {
    if (!valid_dims(regions[i].w, regions[i].h))
      return fail(MIJ_EINVAL, "mij_encode_regions: region %d is %dx%d", i, regions[i].w, regions[i].h);
    W = regions[i].w > W ? regions[i].w : W;
    H = regions[i].h > H ? regions[i].h : H;
  }
  if (!g_rctx || g_rctx->g.w < W || g_rctx->g.h < H || g_rctx->cap < n || g_rctx->quality != quality) {
    const int cw = g_rctx && g_rctx->g.w > W ? g_rctx->g.w : W;
    const int ch = g_rctx && g_rctx->g.h > H ? g_rctx->g.h : H;
    const int cn = g_rctx && g_rctx->cap > n ? g_rctx->cap : n;
    batch_free(g_rctx);
    g_rctx = mij_batch_create(drop_device(), cw, ch, cn, quality);
    if (!g_rctx) return g_err;
  }
  mij_batch *b = g_rctx;
  if (mij_batch_upload_regions(b, bgr, stride_px, frame_h, regions, n)) return g_err;
  if (encode_frames(b, n)) return g_err;
  std::vector<size_t> len(n);
  if (mij_batch_lengths(b, len.data(), n)) return g_err;
  std::vector<int> err(n);
  HIP_TRY(hipMemcpy(err.data(), b->d_err, sizeof(int) * n, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; i++)
    if (err[i]) return mij_frame_fail(err[i], "mij_encode_regions: region", i);
  size_t off = 0;
  for (int i = 0; i < n; i++) {
    lens[i] = len[i];
    if (off + len[i] > cap) return fail(MIJ_ENOSPC, "mij_encode_regions: need more than %zu bytes", cap);
    HIP_TRY(hipMemcpyAsync(out + off, b->d_out + (long long)i * b->g.out_cap, len[i], hipMemcpyDeviceToHost,
                           b->stream));
    off += len[i];
  }
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

// ---------------------------------------------------------------------------
// one large frame over several ranks
//
// Rank r encodes band r (an MCU-row range) of each frame as the frames of its
// own batch (width x band rows); the caller moves four small things between
// ranks (RCCL in sharding.py).  DC differencing, the Huffman statistics and
// the bit positions are the only couplings between bands (encoder.c:168-177,
// :360-381, :462-502): each band's first DC is predicted from the previous
// band's last DC, the tables are built from the summed histograms, and each
// band's share of a scan starts at the sum of the earlier bands' bits.
// ---------------------------------------------------------------------------
static int band_check(mij_batch *b, int n, const char *what, bool assembling = false) {
  if (!b || n < 1 || n > b->cap) return fail(MIJ_EINVAL, "%s: bad frame count", what);
  if (!assembling && pipe_check(b, what)) return g_err;
  HIP_TRY(hipSetDevice(b->dev));
  return MIJ_OK;
}

extern "C" int mij_band_analyze(mij_batch *b, int n, int16_t *last_dc) {
  if (band_check(b, n, "band_analyze")) return g_err;
  if (!last_dc) return fail(MIJ_EINVAL, "band_analyze: null last_dc");
  HIP_TRY(hipMemsetAsync(b->d_hist, 0, sizeof(uint32_t) * n * 4 * 257, b->stream));
  HIP_TRY(hipMemsetAsync(b->d_err, 0, sizeof(int) * n, b->stream));
  // the fused K1: tokens and histograms straight from the pixels; each
  // segment's first DC token waits for mij_band_histograms (k_seg_dc), which
  // knows the band's predictors by then
  if (run_k1(b, n, 2)) return g_err;
  const Geom &g = b->g;
  const long long last[3] = {g.nY - 1, g.nY + g.nC - 1, g.nY + 2LL * g.nC - 1};
  // every frame's last raw DC of a component: one strided copy per component
  for (int c = 0; c < 3; c++)
    HIP_TRY(hipMemcpy2DAsync(last_dc + c, 3 * sizeof(int16_t), b->d_dc + last[c], sizeof(int16_t) * g.nblk,
                             sizeof(int16_t), n, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_band_histograms(mij_batch *b, int n, const int16_t *prev_dc, uint32_t *hist) {
  if (band_check(b, n, "band_histograms")) return g_err;
  b->band_hist_zero = 0;
  if (!prev_dc || !hist) return fail(MIJ_EINVAL, "band_histograms: null argument");
  std::vector<int16_t> pred((size_t)n * 4, 0);
  for (int f = 0; f < n; f++)
    for (int c = 0; c < 3; c++) pred[f * 4 + c] = prev_dc[f * 3 + c];
  HIP_TRY(hipMemcpyAsync(b->d_dcpred, pred.data(), sizeof(int16_t) * n * 4, hipMemcpyHostToDevice,
                         b->stream));
  EntArgs a = ent_args(b, n, 0, true);
  HIP_TRY(launch_seg_dc(a, b->stream));
  HIP_TRY(hipMemcpyAsync(hist, b->d_hist, sizeof(uint32_t) * n * 4 * 257, hipMemcpyDeviceToHost,
                         b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

static int upload_hist_tables(mij_batch *b, int n, const uint32_t *hist) {
  b->band_hist_zero = 0;
  HIP_TRY(hipMemcpyAsync(b->d_hist, hist, sizeof(uint32_t) * n * 4 * 257, hipMemcpyHostToDevice,
                         b->stream));
  HIP_TRY(hipMemsetAsync(b->d_err, 0, sizeof(int) * n, b->stream));
  EntArgs a = ent_args(b, n);
  HIP_TRY(launch_tables(a, b->stream));
  return MIJ_OK;
}

// ---------------------------------------------------------------------------
// the same band protocol, device-resident: every argument
// and result is device memory, every call only enqueues on the batch stream
// (mij_batch_stream), so the caller's collectives can run on that stream
// between the calls and nothing waits for the host.  Table failures stay in
// the frames' error flags (the root's mij_batch_output reports them).
// ---------------------------------------------------------------------------
static int ensure_pieces(mij_batch *b, size_t n) {
  if (b->pieces_cap >= n) return MIJ_OK;
  // (a buffer the stream may still read: wait for it before freeing)
  if (b->d_pieces) {
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipFree(b->d_pieces));
  }
  b->d_pieces = nullptr;
  b->pieces_cap = 0;
  HIP_TRY(dalloc(&b->d_pieces, n * 4));
  b->pieces_cap = n;
  return MIJ_OK;
}

extern "C" int mij_band_analyze_async(mij_batch *b, int n, int16_t *d_last) {
  if (band_check(b, n, "band_analyze_async")) return g_err;
  if (!d_last) return fail(MIJ_EINVAL, "band_analyze_async: null d_last");
  // (the last step's k_band_bound zeroed the histograms it read, and K1
  // zeroes the error words: no fills on the band stream's critical path)
  if (n > b->band_hist_zero) HIP_TRY(hipMemsetAsync(b->d_hist, 0, sizeof(uint32_t) * n * 4 * 257, b->stream));
  b->k1_err_zero = n;
  if (run_k1(b, n, 2)) return g_err;
  HIP_TRY(launch_band_last(b->d_dc, b->g, n, d_last, b->stream));
  return MIJ_OK;
}

extern "C" int mij_band_histograms_async(mij_batch *b, int n, const int16_t *d_prev, uint32_t *d_hist) {
  if (band_check(b, n, "band_histograms_async")) return g_err;
  b->band_hist_zero = 0;
  if (!d_hist) return fail(MIJ_EINVAL, "band_histograms_async: null d_hist");
  // the previous band's last DCs are read in place (null: band 0, zeros)
  EntArgs a = ent_args(b, n);
  a.dc_pred = d_prev;
  HIP_TRY(launch_seg_dc(a, b->stream));
  HIP_TRY(hipMemcpyAsync(d_hist, b->d_hist, sizeof(uint32_t) * n * 4 * 257, hipMemcpyDeviceToDevice, b->stream));
  return MIJ_OK;
}

extern "C" int mij_band_tables_async(mij_batch *b, int n, const uint32_t *d_ghist, uint64_t *d_bound) {
  if (band_check(b, n, "band_tables_async")) return g_err;
  if (!d_ghist || !d_bound) return fail(MIJ_EINVAL, "band_tables_async: null argument");
  if (ensure_pieces(b, (size_t)n * 3)) return g_err;
  // the tables from the summed histograms (read in place), then the band's
  // words bounded from its own histograms and those code lengths: the caller
  // sizes the word exchange from the bound while the band packs
  EntArgs a = ent_args(b, n);
  a.hist = const_cast<uint32_t *>(d_ghist);
  HIP_TRY(launch_tables(a, b->stream));
  if (!b->d_bound_acc) {
    HIP_TRY(dalloc(&b->d_bound_acc, 2));
    HIP_TRY(hipMemsetAsync(b->d_bound_acc, 0, 2 * sizeof(unsigned long long), b->stream));
  }
  HIP_TRY(launch_band_bound(ent_args(b, n), b->d_bound_acc, (unsigned long long *)d_bound, b->stream));
  b->band_hist_zero = n;  // (k_band_bound zeroes the band's histograms it reads)
  b->band_async_n = -n;  // tables built, not packed yet
  return MIJ_OK;
}

extern "C" int mij_band_pack_async(mij_batch *b, int n, uint64_t *d_bits) {
  if (band_check(b, n, "band_pack_async")) return g_err;
  if (!d_bits) return fail(MIJ_EINVAL, "band_pack_async: null d_bits");
  if (b->band_async_n != -n) return fail(MIJ_EINVAL, "band_pack_async: needs mij_band_tables_async of the same frames first");
  // every scan of the band packed from bit 0 (the root shifts it to its
  // place): no band waits for the bit counts of the bands before it
  if (b->raw_dirty) HIP_TRY(hipMemsetAsync(b->d_raw, 0, sizeof(uint32_t) * b->raw_dirty * b->g.raw_fs, b->stream));
  b->raw_dirty = n;
  EntArgs a = ent_args(b, n);
  HIP_TRY(launch_pack(a, b->stream, true));  // (k_band_bound zeroed its state)
  HIP_TRY(launch_band_count((const unsigned long long *)b->d_scan_bits, n, b->d_pieces,
                            (unsigned long long *)d_bits, b->stream));
  b->band_async_n = n;
  return MIJ_OK;
}

extern "C" int mij_band_words_async(mij_batch *b, int n, uint32_t *d_dst, size_t cap_words) {
  if (band_check(b, n, "band_words_async")) return g_err;
  if (!d_dst || n != b->band_async_n) return fail(MIJ_EINVAL, "band_words_async: needs mij_band_pack_async of the same frames first");
  // the move table of mij_band_pack_async, words of frames 0..n-1 in (frame,
  // scan) order into d_dst (cap_words long: words beyond it are dropped, and
  // the root's assembly sees the overflow in the counts), zeroed behind
  // (no piece is longer than the caller's buffer: its length sizes the grid)
  HIP_TRY(launch_move_pieces(b->d_raw, b->g, d_dst, b->d_pieces, n * 3, std::max<long long>((long long)cap_words, 1024),
                             (long long)cap_words, b->stream));
  if (n >= b->raw_dirty) b->raw_dirty = 0;
  return MIJ_OK;
}

extern "C" int mij_assemble_tables_async(mij_batch *b, int n, const uint32_t *d_ghist) {
  if (band_check(b, n, "assemble_tables_async", true)) return g_err;
  if (!d_ghist) return fail(MIJ_EINVAL, "assemble_tables_async: null d_ghist");
  HIP_TRY(hipMemsetAsync(b->d_err, 0, sizeof(int) * n, b->stream));
  EntArgs a = ent_args(b, n);
  a.hist = const_cast<uint32_t *>(d_ghist);  // (read in place: k_tables only reads it)
  HIP_TRY(launch_tables(a, b->stream));
  b->asm_tables_n = n;
  return MIJ_OK;
}

extern "C" int mij_copy_to_host_async(mij_batch *b, void *h_dst, const void *d_src, size_t bytes) {
  if (!b || !h_dst || !d_src) return fail(MIJ_EINVAL, "copy_to_host_async: null argument");
  HIP_TRY(hipSetDevice(b->dev));
  HIP_TRY(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, b->stream));
  return MIJ_OK;
}

extern "C" int mij_assemble_async(mij_batch *b, int n, const uint64_t *d_allbits, int world, const uint32_t *d_src,
                                  size_t stride_words) {
  if (band_check(b, n, "assemble_async", true)) return g_err;
  if (!d_allbits || !d_src || world < 1) return fail(MIJ_EINVAL, "assemble_async: bad arguments");
  if (n != b->asm_tables_n) return fail(MIJ_EINVAL, "assemble_async: needs mij_assemble_tables_async of the same frames first");
  if (ensure_pieces(b, (size_t)world * n * 3)) return g_err;
  // the pieces' boundary words are OR-ed: the scans must start zeroed (a
  // finished assembly leaves them so: k_emit_write zeroes what it reads)
  if (b->raw_dirty) HIP_TRY(hipMemsetAsync(b->d_raw, 0, sizeof(uint32_t) * b->raw_dirty * b->g.raw_fs, b->stream));
  b->raw_dirty = std::max(b->raw_dirty, n);
  EntArgs a = ent_args(b, n);
  HIP_TRY(launch_band_assembly((const unsigned long long *)d_allbits, world, n, stride_words, b->d_pieces,
                               (unsigned long long *)b->d_scan_bits, b->d_err, b->stream));
  HIP_TRY(launch_or_shift_pieces(b->d_raw, b->g, d_src, b->d_pieces, world * n * 3, (long long)stride_words,
                                 b->stream));
  HIP_TRY(launch_emit(a, b->stream));  // k_emit_write zeroes the words it reads
  if (n >= b->raw_dirty) b->raw_dirty = 0;
  b->asm_tables_n = 0;
  b->last_frames = n;
  return MIJ_OK;
}

// Distributed JFIF emission (include/mijpeg.h): the band's interiors stuffed
// on its own GPU, the root joins them (k_band_* in mij_kernels.hip)
extern "C" int mij_band_stuff_async(mij_batch *b, int n, const uint64_t *d_allbits, int world, int rank,
                                    uint64_t *d_rec, uint64_t *d_total, uint8_t *d_dst, size_t cap) {
  if (band_check(b, n, "band_stuff_async")) return g_err;
  if (!d_allbits || !d_rec || !d_total || !d_dst || world < 1 || rank < 0 || rank >= world)
    return fail(MIJ_EINVAL, "band_stuff_async: bad arguments");
  if (n != b->band_async_n) return fail(MIJ_EINVAL, "band_stuff_async: needs mij_band_pack_async of the same frames first");
  EntArgs a = ent_args(b, n, 0, true);  // (bit_base: the heads' shifts)
  a.ff_pack = 0;
  HIP_TRY(launch_band_stuff(a, (const unsigned long long *)d_allbits, world, rank, (unsigned long long *)d_rec,
                            (unsigned long long *)d_total, d_dst, (unsigned long long)cap, b->stream));
  // the heads' shifts k_band_stuff_prep kept in the bit bases: reset, so no
  // band call after this one finds them
  HIP_TRY(hipMemsetAsync(b->d_bitbase, 0, sizeof(uint32_t) * n * 4, b->stream));
  b->band_async_n = 0;  // the scan words are consumed (zeroed)
  if (n >= b->raw_dirty) b->raw_dirty = 0;
  return MIJ_OK;
}

extern "C" int mij_assemble_stuffed_async(mij_batch *b, int n, const uint64_t *d_allrec, int world,
                                          const uint8_t *d_src, size_t stride) {
  if (band_check(b, n, "assemble_stuffed_async", true)) return g_err;
  if (!d_allrec || !d_src || world < 1) return fail(MIJ_EINVAL, "assemble_stuffed_async: bad arguments");
  if (n != b->asm_tables_n)
    return fail(MIJ_EINVAL, "assemble_stuffed_async: needs mij_assemble_tables_async of the same frames first");
  if (ensure_pieces(b, (size_t)world * n * 3)) return g_err;
  EntArgs a = ent_args(b, n);
  HIP_TRY(launch_band_join(a, (const unsigned long long *)d_allrec, world, (unsigned long long)stride, b->d_pieces,
                           d_src, b->stream));
  b->asm_tables_n = 0;
  b->last_frames = n;
  return MIJ_OK;
}

// tests: the four tables of frames 0..n-1 from given counts (k_tables alone)
extern "C" int mij_batch_build_tables(mij_batch *b, int n, const uint32_t *hist) {
  if (band_check(b, n, "build_tables", true)) return g_err;
  if (!hist) return fail(MIJ_EINVAL, "build_tables: null hist");
  if (upload_hist_tables(b, n, hist)) return g_err;
  std::vector<int> err((size_t)n);
  HIP_TRY(hipMemcpyAsync(err.data(), b->d_err, sizeof(int) * n, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  for (int f = 0; f < n; f++)
    if (err[f]) return mij_frame_fail(err[f], "frame", f);
  return MIJ_OK;
}

extern "C" int mij_band_tables(mij_batch *b, int n, const uint32_t *hist, unsigned long long *bits) {
  if (band_check(b, n, "band_tables")) return g_err;
  if (!hist || !bits) return fail(MIJ_EINVAL, "band_tables: null argument");
  if (upload_hist_tables(b, n, hist)) return g_err;
  HIP_TRY(hipMemsetAsync(b->d_bitbase, 0, sizeof(uint32_t) * n * 4, b->stream));
  EntArgs a = ent_args(b, n, 0, true);
  HIP_TRY(launch_bits(a, b->stream));
  HIP_TRY(launch_scan(a, b->stream));
  HIP_TRY(hipMemcpyAsync(bits, b->d_scan_bits, sizeof(uint64_t) * n * 3, hipMemcpyDeviceToHost,
                         b->stream));
  std::vector<int> err((size_t)n);
  HIP_TRY(hipMemcpyAsync(err.data(), b->d_err, sizeof(int) * n, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  for (int f = 0; f < n; f++)
    if (err[f]) return mij_frame_fail(err[f], "band frame", f);
  return MIJ_OK;
}

extern "C" int mij_band_pack(mij_batch *b, int n, const unsigned long long *bit_offset,
                             unsigned long long *nwords) {
  if (band_check(b, n, "band_pack")) return g_err;
  if (!bit_offset) return fail(MIJ_EINVAL, "band_pack: null bit_offset");
  std::vector<uint32_t> base((size_t)n * 4, 0);
  for (int f = 0; f < n; f++)
    for (int c = 0; c < 3; c++) base[f * 4 + c] = (uint32_t)(bit_offset[f * 3 + c] & 31);
  HIP_TRY(hipMemcpyAsync(b->d_bitbase, base.data(), sizeof(uint32_t) * n * 4, hipMemcpyHostToDevice,
                         b->stream));
  EntArgs a = ent_args(b, n, 0, true);
  // the band packing needs all-zero scan buffers: mij_band_words_all moves the band
  // words out and zeroes them; a band packed but never moved leaves them dirty
  if (b->raw_dirty) HIP_TRY(hipMemsetAsync(b->d_raw, 0, sizeof(uint32_t) * b->raw_dirty * b->g.raw_fs, b->stream));
  b->raw_dirty = n;
  HIP_TRY(launch_pack(a, b->stream));
  std::vector<unsigned long long> tot((size_t)n * 3);
  HIP_TRY(hipMemcpyAsync(tot.data(), b->d_scan_bits, sizeof(uint64_t) * n * 3,
                         hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  for (int i = 0; i < n * 3; i++) {
    b->band_words[i] = (tot[i] + 31) >> 5;  // scan bits include the in-word start offset
    if (nwords) nwords[i] = b->band_words[i];
  }
  return MIJ_OK;
}

static uint32_t *scan_words(mij_batch *b, int frame, int comp) {
  const Geom &g = b->g;
  return b->d_raw + (long long)frame * g.raw_fs +
         (comp == 0 ? 0 : g.raw_words[0] + (comp == 2 ? g.raw_words[1] : 0));
}

extern "C" int mij_band_words(mij_batch *b, int frame, int comp, void *dst, size_t cap_words,
                              int dst_on_device) {
  if (pipe_check(b, "band_words")) return g_err;
  if (frame < 0 || frame >= b->cap || comp < 0 || comp > 2 || !dst)
    return fail(MIJ_EINVAL, "band_words: bad arguments");
  HIP_TRY(hipSetDevice(b->dev));
  const unsigned long long nw = b->band_words[frame * 3 + comp];
  if (cap_words < nw) return fail(MIJ_ENOSPC, "band_words: need %llu words", nw);
  HIP_TRY(hipMemcpyAsync(dst, scan_words(b, frame, comp), nw * 4,
                         dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_band_words_all(mij_batch *b, int n, void *dst, size_t cap_words, int dst_on_device) {
  if (band_check(b, n, "band_words_all")) return g_err;
  if (!dst) return fail(MIJ_EINVAL, "band_words_all: null dst");
  unsigned long long total = 0;
  for (int i = 0; i < 3 * n; i++) total += b->band_words[i];
  if (cap_words < total) return fail(MIJ_ENOSPC, "band_words_all: need %llu words", total);
  // (frame, comp) order, moved (and zeroed behind) in one launch, then one
  // copy to a host destination, one synchronisation
  HIP_TRY(hipSetDevice(b->dev));
  std::vector<unsigned long long> pcs;
  long long max_words = 0;
  unsigned long long at = 0;
  for (int i = 0; i < 3 * n; i++) {
    const unsigned long long nw = b->band_words[i];
    if (nw) pcs.insert(pcs.end(), {(unsigned long long)i, nw, at});
    max_words = std::max(max_words, (long long)nw);
    at += nw;
  }
  const int np = (int)(pcs.size() / 3);
  uint32_t *d = (uint32_t *)dst;
  if (!dst_on_device && total) {
    if (b->stage_words < total) {
      if (b->d_stage) HIP_TRY(hipFree(b->d_stage));
      b->d_stage = nullptr;
      HIP_TRY(dalloc(&b->d_stage, total));
      b->stage_words = total;
    }
    d = b->d_stage;
  }
  if (np) {
    if (b->pieces_cap < (size_t)np) {
      if (b->d_pieces) HIP_TRY(hipFree(b->d_pieces));
      b->d_pieces = nullptr;
      HIP_TRY(dalloc(&b->d_pieces, (size_t)np * 4));
      b->pieces_cap = (size_t)np;
    }
    HIP_TRY(hipMemcpyAsync(b->d_pieces, pcs.data(), sizeof(unsigned long long) * pcs.size(), hipMemcpyHostToDevice,
                           b->stream));
    HIP_TRY(launch_move_pieces(b->d_raw, b->g, d, b->d_pieces, np, max_words, (long long)total, b->stream));
  }
  if (!dst_on_device && total)
    HIP_TRY(hipMemcpyAsync(dst, d, total * 4, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  // the words of frames 0..n-1 have left the buffers (a scan's words, its
  // in-word start offset included, are its band_words); frames a wider
  // mij_band_pack covered beyond n still hold theirs
  if (n >= b->raw_dirty) b->raw_dirty = 0;
  return MIJ_OK;
}

extern "C" int mij_assemble_pieces(mij_batch *b, const void *src, size_t src_words, int src_on_device,
                                   const unsigned long long *pieces, int npieces) {
  if (!b || npieces < 0 || (npieces && (!src || !pieces)))
    return fail(MIJ_EINVAL, "assemble_pieces: bad arguments");
  long long max_words = 0;
  for (int i = 0; i < npieces; i++) {
    const unsigned long long *p = pieces + 4 * i;
    const unsigned long long fc = p[0], f = fc / 3, c = fc % 3;
    if (f >= (unsigned long long)b->cap || p[1] + p[3] > (unsigned long long)b->g.raw_words[c] ||
        p[2] + p[3] > src_words)
      return fail(MIJ_ENOSPC, "assemble_pieces: piece %d (frame %llu comp %llu) out of bounds", i, f, c);
    max_words = std::max(max_words, (long long)p[3]);
  }
  if (!npieces || !max_words) return MIJ_OK;
  HIP_TRY(hipSetDevice(b->dev));
  const uint32_t *s32 = (const uint32_t *)src;
  if (!src_on_device) {
    if (b->stage_words < src_words) {
      if (b->d_stage) HIP_TRY(hipFree(b->d_stage));
      b->d_stage = nullptr;
      HIP_TRY(dalloc(&b->d_stage, src_words));
      b->stage_words = src_words;
    }
    HIP_TRY(hipMemcpyAsync(b->d_stage, src, src_words * 4, hipMemcpyHostToDevice, b->stream));
    s32 = b->d_stage;
  }
  if (b->pieces_cap < (size_t)npieces) {
    if (b->d_pieces) HIP_TRY(hipFree(b->d_pieces));
    b->d_pieces = nullptr;
    HIP_TRY(dalloc(&b->d_pieces, (size_t)npieces * 4));
    b->pieces_cap = (size_t)npieces;
  }
  HIP_TRY(hipMemcpyAsync(b->d_pieces, pieces, sizeof(unsigned long long) * 4 * npieces, hipMemcpyHostToDevice,
                         b->stream));
  HIP_TRY(launch_or_pieces(b->d_raw, b->g, s32, b->d_pieces, npieces, max_words, b->stream));
  // the caller may release or reuse src (and pieces) once this returns
  HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_assemble_begin(mij_batch *b, int n, const uint32_t *hist) {
  if (band_check(b, n, "assemble_begin", true)) return g_err;
  if (!hist) return fail(MIJ_EINVAL, "assemble_begin: null hist");
  HIP_TRY(hipMemsetAsync(b->d_raw, 0, sizeof(uint32_t) * n * b->g.raw_fs, b->stream));
  // the words ORed in before mij_assemble_end leave frames 0..n-1 dirty
  b->raw_dirty = std::max(b->raw_dirty, n);
  return upload_hist_tables(b, n, hist);
}

extern "C" int mij_assemble_words(mij_batch *b, int frame, int comp, unsigned long long first_word,
                                  const void *src, size_t nwords, int src_on_device) {
  if (!b || frame < 0 || frame >= b->cap || comp < 0 || comp > 2 || (!src && nwords))
    return fail(MIJ_EINVAL, "assemble_words: bad arguments");
  if (first_word + nwords > (unsigned long long)b->g.raw_words[comp])
    return fail(MIJ_ENOSPC, "assemble_words: words beyond the scan buffer");
  HIP_TRY(hipSetDevice(b->dev));
  const uint32_t *s32 = (const uint32_t *)src;
  if (!src_on_device && nwords) {
    if (b->stage_words < nwords) {
      if (b->d_stage) HIP_TRY(hipFree(b->d_stage));
      b->d_stage = nullptr;
      HIP_TRY(dalloc(&b->d_stage, nwords));
      b->stage_words = nwords;
    }
    HIP_TRY(hipMemcpyAsync(b->d_stage, src, nwords * 4, hipMemcpyHostToDevice, b->stream));
    s32 = b->d_stage;
  }
  // neighbouring bands share at most their boundary word: OR-combine
  HIP_TRY(launch_or_words(scan_words(b, frame, comp) + first_word, s32, (long long)nwords, b->stream));
  if (!src_on_device) HIP_TRY(hipStreamSynchronize(b->stream));
  return MIJ_OK;
}

extern "C" int mij_assemble_end(mij_batch *b, int n, const unsigned long long *total_bits) {
  if (band_check(b, n, "assemble_end", true)) return g_err;
  if (!total_bits) return fail(MIJ_EINVAL, "assemble_end: null total_bits");
  HIP_TRY(hipMemcpyAsync(b->d_scan_bits, total_bits, sizeof(uint64_t) * n * 3,
                         hipMemcpyHostToDevice, b->stream));
  EntArgs a = ent_args(b, n);
  HIP_TRY(launch_emit(a, b->stream));  // k_emit_write zeroes the words it reads
  if (n >= b->raw_dirty) b->raw_dirty = 0;
  b->last_frames = n;
  return MIJ_OK;
}

// ---------------------------------------------------------------------------
// diagnostics
// ---------------------------------------------------------------------------
extern "C" int mij_probe_mfma(const int8_t *A, const int8_t *B, int32_t *D) {
  if (check_device(drop_device())) return g_err;
  HIP_TRY(hipSetDevice(drop_device()));
  int4 *dA, *dB, *dD;
  HIP_TRY(hipMalloc((void **)&dA, 64 * 16));
  HIP_TRY(hipMalloc((void **)&dB, 64 * 16));
  HIP_TRY(hipMalloc((void **)&dD, 64 * 16));
  HIP_TRY(hipMemcpy(dA, A, 64 * 16, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dB, B, 64 * 16, hipMemcpyHostToDevice));
  HIP_TRY(launch_mfma_probe(dA, dB, dD, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(D, dD, 64 * 16, hipMemcpyDeviceToHost));
  hipFree(dA);
  hipFree(dB);
  hipFree(dD);
  return MIJ_OK;
}

extern "C" int mij_colour_lut(uint32_t *out) {
  std::lock_guard<std::mutex> l(g_mu);
  mij_batch *b = ctx_for(16, 16, g_quality);
  if (!b) return g_err;
  HIP_TRY(hipStreamSynchronize(b->stream));
  HIP_TRY(hipMemcpy(out, &b->d_tab->lut[0][0], sizeof(uint32_t) * 3 * LUT_WORDS,
                    hipMemcpyDeviceToHost));
  return MIJ_OK;
}
