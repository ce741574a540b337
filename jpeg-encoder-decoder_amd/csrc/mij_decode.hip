// mij_decode.hip -- round-trip verifier: baseline JFIF -> quantized
// coefficient planes on the GPU (the reference has
// no decoder, func_tester.c:1262-1309 checks its output with libjpeg).
//
// Scope: the streams this library and the reference write (encoder.c:549-644):
// 8-bit baseline, 3 components Y 2x2 / Cb 1x1 / Cr 1x1, three
// non-interleaved scans, no restart markers.  The output is the encoder's
// own coefficient layout (encoder.c:158-178): per component, blocks in
// raster order, 64 zigzag-ordered coefficients per block, the DC as the
// coded difference -- so decode(encode(x)) can be compared bit-exactly with
// rgb_to_dct(x) at any size.
//
// Host: marker parsing (SOI, APP0, DQT, DHT, SOF0, SOS, EOI), canonical
// Huffman tables with a 9-bit lookahead, and the scans copied unstuffed
// into one pinned staging blob.  Device: every scan is cut into 512-bit
// chunks, one lane per chunk.  Entropy decoding is sequential by
// construction, so the chunks' entry states (bit position, coefficient
// index) are found by self-synchronisation: each chunk first decodes from
// its own first bit as if a block began there, then repeatedly from the
// exit state of its predecessor until no entry changes (2-3 passes).  A
// per-scan prefix sum of the blocks each chunk starts gives every chunk its
// output block, and a final pass writes the nonzero coefficients into the
// zeroed planes.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "mij_host.h"

#define HIP_TRY(x)                                                                 \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess)                                                          \
      return mij_fail(MIJ_EHIP, "%s failed: %s", #x, hipGetErrorString(e_));       \
  } while (0)

namespace mij {

constexpr int LOOK = 9;

// One canonical Huffman table (ISO/IEC 10918-1 F.2.2.3 decoding procedure).
struct DecTab {
  uint16_t look[1 << LOOK];  // (length << 8) | symbol, 0 = longer than LOOK
  int32_t maxcode[18];       // largest code of each length, -1 if none
  int32_t valoff[17];        // index of the first symbol of a length - its code
  uint8_t val[256];
};

struct DecJob {
  long long data;   // byte offset of the UNSTUFFED scan in the blob (8-aligned)
  long long nbits;  // its length in bits (the pad bits included)
  long long out;    // first int16 of the component's plane
  int nblocks;
  int dc, ac;       // table indices
  int chunk0, nchunks;  // global ids of the scan's chunks
};

// chunk c of a scan covers bits [c*CHUNK, (c+1)*CHUNK): a symbol belongs to
// the chunk its first bit lies in.  512: measured against 1024 / 2048 / 4096
// on 256 config-3 streams, 16.3 / 17.7 / 21.1 / 23.9 ms per decode call.
constexpr int CHUNK = 512;

// MSB-first bit window over an unstuffed, 8-byte aligned, zero-padded scan
struct Bits {
  const unsigned long long *w;
  long long cw = -2;  // index of the word pair held (none yet)
  unsigned long long hi = 0, lo = 0;
  __device__ unsigned long long window(long long pos) {
    const long long i = pos >> 6;
    if (i != cw) {
      if (i == cw + 1) {
        hi = lo;
        lo = __builtin_bswap64(w[i + 1]);
      } else {
        hi = __builtin_bswap64(w[i]);
        lo = __builtin_bswap64(w[i + 1]);
      }
      cw = i;
    }
    const int sh = pos & 63;
    return sh ? (hi << sh) | (lo >> (64 - sh)) : hi;
  }
};

// one symbol (+ its magnitude bits) at pos; returns bits consumed, or 0 on
// an invalid code.  F.2.2.3 DECODE with a LOOK-bit table, F.2.2.1 EXTEND
__device__ __forceinline__ int decode_one(Bits &br, long long pos, const DecTab &t, int &sym, int &val) {
  const unsigned long long win = br.window(pos);
  int len;
  const uint32_t e = t.look[win >> (64 - LOOK)];
  if (e) {
    len = e >> 8;
    sym = e & 255;
  } else {
    len = 0;
    for (int l = LOOK + 1; l <= 16; l++) {
      const int32_t code = (int32_t)(win >> (64 - l));
      if (code <= t.maxcode[l]) {
        len = l;
        sym = t.val[t.valoff[l] + code];
        break;
      }
    }
    if (!len) return 0;
  }
  const int s = sym & 15;
  if (s) {
    // magnitude bits follow the code; the window holds >= 64 - 16 bits
    const int v = (int)((win << len) >> (64 - s));
    val = v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;  // negatives are ~|v| (encoder.c:442-444)
  } else {
    val = 0;
  }
  return len + s;
}

// Decodes from (pos, k) until pos reaches `stop` or `blocks_left` blocks
// have ended.  k = next coefficient index (0 = a DC symbol is next).
// Returns the number of blocks started; pos/k are the state after the last
// symbol.  WRITE: coefficients go to out[64*blk + zigzag index] (nonzeros
// only; the planes are zeroed first).  *bad = invalid code met.
template <bool WRITE>
__device__ int decode_span(Bits &br, long long &pos, int &k, long long stop, const DecTab &dc,
                           const DecTab &ac, int16_t *out, long long blk, long long blocks_left,
                           bool *bad) {
  int started = 0;
  *bad = false;
  while (pos < stop) {
    int sym, val;
    if (k == 0) {
      if (blocks_left <= 0) break;
      const int n = decode_one(br, pos, dc, sym, val);
      if (!n || sym > 15) {
        *bad = true;
        break;
      }
      pos += n;
      if (WRITE && val) out[64 * blk] = (int16_t)val;
      started++;
      k = 1;
    } else {
      const int n = decode_one(br, pos, ac, sym, val);
      if (!n) {
        *bad = true;
        break;
      }
      pos += n;
      const int r = sym >> 4;
      if (sym & 15) {
        k += r;
        if (k > 63) {
          *bad = true;
          break;
        }
        if (WRITE) out[64 * blk + k] = (int16_t)val;
        k++;
      } else if (r == 15) {
        k += 16;  // ZRL
      } else {
        k = 64;   // EOB
      }
    }
    if (k >= 64) {
      k = 0;
      blk++;
      blocks_left--;
    }
  }
  return started;
}

__device__ __forceinline__ int job_of(const DecJob *jobs, int njobs, int c) {
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].chunk0 <= c) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Self-synchronising pass (Weissenberger & Schmidt, ICPP 2018): chunk c
// decodes from its entry state to its end.  First pass: every chunk starts
// at its first bit as if a block began there (exact for chunk 0 of a
// scan).  Later passes: the entry of chunk c is the exit of chunk c-1 from
// the previous pass; a chunk whose entry did not change keeps its result.
// Huffman streams resynchronise within a few symbols, so 2-3 passes settle.
struct SyncArgs {
  const uint8_t *blob;
  const DecJob *jobs;
  int njobs, nchunks;
  const DecTab *tabs;
  long long *entry_pos, *exit_in, *exit_out;  // pos * 64 + k packed
  int *nblk;
  int *changed;
  int first;
};

__device__ __forceinline__ long long pack_state(long long pos, int k) { return pos * 64 + k; }

__global__ __launch_bounds__(256) void k_dec_sync(SyncArgs a) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.nchunks) return;
  const DecJob &job = a.jobs[job_of(a.jobs, a.njobs, c)];
  const int lc = c - job.chunk0;
  long long entry;
  if (a.first || lc == 0) {
    entry = pack_state((long long)lc * CHUNK, 0);
    if (!a.first) {
      a.exit_out[c] = a.exit_in[c];
      return;
    }
  } else {
    entry = a.exit_in[c - 1];
    if (entry < 0) entry = pack_state((long long)lc * CHUNK, 0);  // predecessor met a bad code
    if (entry == a.entry_pos[c]) {
      a.exit_out[c] = a.exit_in[c];
      return;
    }
    *a.changed = 1;
  }
  a.entry_pos[c] = entry;
  Bits br{(const unsigned long long *)(a.blob + job.data)};
  long long pos = entry >> 6;
  int k = (int)(entry & 63);
  const long long stop = min((long long)(lc + 1) * CHUNK, job.nbits);
  bool bad;
  const int n = decode_span<false>(br, pos, k, stop, a.tabs[job.dc], a.tabs[job.ac], nullptr, 0,
                                   (long long)job.nblocks, &bad);
  a.nblk[c] = n;
  a.exit_out[c] = bad ? -1 : pack_state(pos, k);
}

// per scan: exclusive scan of the chunks' block counts (one workgroup per
// scan, sequential over 256-chunk tiles) and the total check
__global__ __launch_bounds__(256) void k_dec_scan(const DecJob *jobs, const int *nblk, long long *base,
                                                  int *status) {
  __shared__ long long part[256];
  const DecJob job = jobs[blockIdx.x];
  long long carry = 0;
  for (int t0 = 0; t0 < job.nchunks; t0 += 256) {
    const int t = t0 + threadIdx.x;
    const long long v = t < job.nchunks ? nblk[job.chunk0 + t] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const long long add = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (t < job.nchunks) base[job.chunk0 + t] = carry + part[threadIdx.x] - v;
    const long long tot = part[255];
    __syncthreads();
    carry += tot;
  }
  // a chunk that decodes the last block may go on through the pad bits
  // (and count garbage blocks there); fewer blocks than the frame needs is
  // a truncated stream
  if (threadIdx.x == 0) status[blockIdx.x] = carry >= job.nblocks ? 0 : 5;
}

// final pass: every chunk decodes from its settled entry and writes.  A
// lane assembles each block in its own LDS slot (128 B) and stores it whole
// (8 x 16 B, zeros included: no memset of the planes).  A block split
// between two chunks is stored in halves with 2-byte stores: the lane that
// started it writes positions [first, k_exit), the next lane [k_entry, 64)
// -- the settled states make k_exit == k_entry.
__global__ __launch_bounds__(256) void k_dec_write(SyncArgs a, const long long *base, int16_t *coefs,
                                                   int *status) {
  __shared__ int4 slot[256][8];
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.nchunks) return;
  const int j = job_of(a.jobs, a.njobs, c);
  const DecJob &job = a.jobs[j];
  const int lc = c - job.chunk0;
  const long long entry = a.entry_pos[c];
  long long pos = entry >> 6;
  int k = (int)(entry & 63);
  // the block in progress at the entry was started by an earlier chunk
  long long blk = base[c] - (k ? 1 : 0);
  if (blk >= job.nblocks) return;  // pad bits after the last block
  Bits br{(const unsigned long long *)(a.blob + job.data)};
  const long long stop = min((long long)(lc + 1) * CHUNK, job.nbits);
  const DecTab &dc = a.tabs[job.dc], &ac = a.tabs[job.ac];
  int4 *sl = slot[threadIdx.x];
  int16_t *b16 = (int16_t *)sl;
  int16_t *out = coefs + job.out;
#pragma unroll
  for (int q = 0; q < 8; q++) sl[q] = int4{0, 0, 0, 0};
  int first = k;
  bool bad = false;
  while (pos < stop && blk < job.nblocks) {
    int sym, val;
    const int n = decode_one(br, pos, k ? ac : dc, sym, val);
    if (!n) {
      bad = true;
      break;
    }
    pos += n;
    if (k == 0) {
      if (sym > 15) {
        bad = true;
        break;
      }
      b16[0] = (int16_t)val;
      k = 1;
    } else {
      const int r = sym >> 4;
      if (sym & 15) {
        k += r;
        if (k > 63) {
          bad = true;
          break;
        }
        b16[k++] = (int16_t)val;
      } else {
        k = r == 15 ? k + 16 : 64;  // ZRL / EOB
      }
    }
    if (k >= 64) {  // block complete: store it, clear the slot
      int16_t *o = out + 64 * blk;
      if (first == 0) {
#pragma unroll
        for (int q = 0; q < 8; q++) ((int4 *)o)[q] = sl[q];
      } else {
        for (int t = first; t < 64; t++) o[t] = b16[t];
      }
#pragma unroll
      for (int q = 0; q < 8; q++) sl[q] = int4{0, 0, 0, 0};
      first = 0;
      k = 0;
      blk++;
    }
  }
  if (!bad && k && blk < job.nblocks) {  // block continues in the next chunk
    int16_t *o = out + 64 * blk;
    for (int t = first; t < k; t++) o[t] = b16[t];
  }
  if (bad) atomicMax(&status[j], 6);
}

}  // namespace mij

// ---------------------------------------------------------------------------
// host: JFIF parsing
// ---------------------------------------------------------------------------
namespace {

struct Parsed {
  int w = 0, h = 0;
  uint8_t dqt[2][64];
  bool have_dqt[2] = {false, false};
  mij::DecTab tab[4];  // DC0, AC0 (luma), DC1, AC1 (chroma): index 2*Th + Tc
  bool have_tab[4] = {false, false, false, false};
  struct Scan {
    int comp, td, ta;
    long long data, end;
  } scan[3];
  int nscans = 0;
  int comp_seen = 0;  // components that already have a scan (bit c)
};

int be16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

int build_table(mij::DecTab &t, const uint8_t counts[16], const uint8_t *syms, int nsyms) {
  memset(&t, 0, sizeof t);
  memcpy(t.val, syms, nsyms);
  int code = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    const int c = counts[l - 1];
    t.valoff[l] = k - code;
    t.maxcode[l] = c ? code + c - 1 : -1;
    for (int i = 0; i < c; i++, k++, code++) {
      if (l <= mij::LOOK) {
        const int sh = mij::LOOK - l;
        for (int f = 0; f < (1 << sh); f++) t.look[(code << sh) | f] = (uint16_t)((l << 8) | syms[k]);
      }
    }
    if (code > (1 << l)) return -1;  // over-subscribed
    code <<= 1;
  }
  t.maxcode[17] = 0x7fffffff;
  return 0;
}

int parse(const uint8_t *s, size_t n, Parsed &P, int frame) {
#define BAD(...) return mij_fail(MIJ_EJPEG, __VA_ARGS__)
  if (n < 4 || s[0] != 0xFF || s[1] != 0xD8) BAD("stream %d: no SOI", frame);
  size_t i = 2;
  while (i + 4 <= n) {
    if (s[i] != 0xFF) BAD("stream %d: marker expected at byte %zu", frame, i);
    const int m = s[i + 1];
    if (m == 0xFF) {  // fill byte
      i++;
      continue;
    }
    if (m == 0xD9) break;  // EOI
    const int len = be16(s + i + 2);
    if (len < 2 || i + 2 + len > n) BAD("stream %d: segment 0x%02X length %d", frame, m, len);
    const uint8_t *q = s + i + 4;
    const int body = len - 2;
    if (m == 0xDB) {  // DQT, 8-bit, possibly several tables
      for (int o = 0; o + 65 <= body; o += 65) {
        const int tq = q[o] & 15;
        if ((q[o] >> 4) || tq > 1) BAD("stream %d: DQT Pq/Tq %02X", frame, q[o]);
        memcpy(P.dqt[tq], q + o + 1, 64);
        P.have_dqt[tq] = true;
      }
    } else if (m == 0xC4) {  // DHT, possibly several tables
      int o = 0;
      while (o + 17 <= body) {
        const int tc = q[o] >> 4, th = q[o] & 15;
        if (tc > 1 || th > 1) BAD("stream %d: DHT Tc/Th %02X", frame, q[o]);
        int nsym = 0;
        for (int l = 0; l < 16; l++) nsym += q[o + 1 + l];
        if (nsym > 256 || o + 17 + nsym > body) BAD("stream %d: DHT symbol count %d", frame, nsym);
        if (build_table(P.tab[2 * th + tc], q + o + 1, q + o + 17, nsym))
          BAD("stream %d: DHT code over-subscribed", frame);
        P.have_tab[2 * th + tc] = true;
        o += 17 + nsym;
      }
    } else if (m == 0xC0) {  // SOF0
      if (body < 15 || q[0] != 8 || q[5] != 3) BAD("stream %d: SOF0 not 8-bit 3-component", frame);
      P.h = be16(q + 1);
      P.w = be16(q + 3);
      const uint8_t want[3][3] = {{1, 0x22, 0}, {2, 0x11, 1}, {3, 0x11, 1}};
      for (int c = 0; c < 3; c++)
        if (memcmp(q + 6 + 3 * c, want[c], 3)) BAD("stream %d: SOF0 component %d is not 4:2:0", frame, c);
      if (P.w <= 0 || P.h <= 0 || P.w % 16 || P.h % 16) BAD("stream %d: %dx%d", frame, P.w, P.h);
    } else if (m == 0xC1 || m == 0xC2 || m == 0xC3 || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) {
      BAD("stream %d: SOF 0x%02X is not baseline", frame, m);
    } else if (m == 0xDA) {  // SOS + entropy data
      if (P.nscans >= 3 || body < 6 || q[0] != 1) BAD("stream %d: SOS (only 1-component scans)", frame);
      if (q[3] != 0 || q[4] != 63 || q[5] != 0) BAD("stream %d: SOS Ss/Se/AhAl", frame);
      Parsed::Scan &sc = P.scan[P.nscans++];
      sc.comp = q[1] - 1;
      sc.td = q[2] >> 4;
      sc.ta = q[2] & 15;
      if (sc.comp < 0 || sc.comp > 2 || sc.td > 1 || sc.ta > 1) BAD("stream %d: SOS component", frame);
      // each component exactly once: a repeated scan would leave another
      // component's plane unwritten (it keeps the previous call's values)
      if (P.comp_seen & (1 << sc.comp)) BAD("stream %d: SOS repeats component %d", frame, sc.comp + 1);
      P.comp_seen |= 1 << sc.comp;
      size_t e = i + 2 + len;
      sc.data = (long long)e;
      // entropy data ends at the next marker: a 0xFF followed by neither
      // 0x00 (stuffing) nor 0xFF.  The end-of-scan pad byte is never
      // stuffed (encoder.c:425-432), so "FF FF xx" is a pad byte that still
      // holds the scan's last bits, then the marker: it is kept as data.
      for (;;) {
        const uint8_t *f = (const uint8_t *)memchr(s + e, 0xFF, n - e);
        if (!f || (size_t)(f - s) + 1 >= n) BAD("stream %d: scan %d runs to the end", frame, P.nscans);
        e = f - s;
        if (s[e + 1] == 0x00) {
          e += 2;
          continue;
        }
        if (s[e + 1] == 0xFF) {
          e += 1;
          continue;
        }
        break;
      }
      sc.end = (long long)e;
      i = e;
      continue;
    }
    i += 2 + len;  // APPn, COM, anything else: skipped
  }
  if (!P.w || P.nscans != 3) BAD("stream %d: missing SOF0 or scans (%d)", frame, P.nscans);
  for (int k = 0; k < 3; k++) {
    const auto &sc = P.scan[k];
    if (!P.have_tab[2 * sc.td] || !P.have_tab[2 * sc.ta + 1]) BAD("stream %d: scan %d table missing", frame, k);
  }
  return MIJ_OK;
#undef BAD
}

}  // namespace

struct mij_decoder {
  int dev = 0;
  hipStream_t stream = nullptr;
  int max_w = 0, max_h = 0, cap = 0;
  size_t blob_cap = 0;
  uint8_t *d_blob = nullptr, *h_blob = nullptr;
  int16_t *d_coef = nullptr;
  mij::DecTab *d_tabs = nullptr;
  mij::DecJob *d_jobs = nullptr;
  int *d_status = nullptr;
  int *d_changed = nullptr;
  long long *d_entry = nullptr, *d_exit[2] = {nullptr, nullptr}, *d_base = nullptr;
  int *d_nblk = nullptr;
  int chunk_cap = 0, job_cap = 1 << 30, last_passes = 0;
  std::vector<Parsed> parsed;
  long long plane_px = 0;  // max_w * max_h: Y plane; Cb/Cr a quarter each
  int n = 0;
};

static void decoder_free(mij_decoder *d) {
  if (!d) return;
  hipSetDevice(d->dev);
  if (d->stream) hipStreamSynchronize(d->stream);
  hipFree(d->d_blob);
  hipFree(d->d_coef);
  hipFree(d->d_tabs);
  hipFree(d->d_jobs);
  hipFree(d->d_status);
  hipFree(d->d_changed);
  hipFree(d->d_entry);
  hipFree(d->d_exit[0]);
  hipFree(d->d_exit[1]);
  hipFree(d->d_nblk);
  hipFree(d->d_base);
  if (d->h_blob) hipHostFree(d->h_blob);
  if (d->stream) hipStreamDestroy(d->stream);
  delete d;
}

extern "C" mij_decoder *mij_decoder_create(int device, int max_w, int max_h, int max_frames) {
  mij_clear_error();
  if (max_w < 16 || max_h < 16 || max_w % 16 || max_h % 16 || max_frames < 1) {
    mij_fail(MIJ_EINVAL, "decoder_create: %dx%d x%d", max_w, max_h, max_frames);
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
    mij_fail(MIJ_ENODEV, "no HIP device %d (the HIP path has no CPU fallback)", device);
    return nullptr;
  }
  auto *d = new mij_decoder();
  d->dev = device;
  d->max_w = max_w;
  d->max_h = max_h;
  d->cap = max_frames;
  d->plane_px = (long long)max_w * max_h;
  auto init = [&]() -> int {
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    HIP_TRY(hipMalloc((void **)&d->d_coef, (size_t)max_frames * d->plane_px * 3 / 2 * sizeof(int16_t)));
    HIP_TRY(hipMalloc((void **)&d->d_tabs, (size_t)max_frames * 4 * sizeof(mij::DecTab)));
    HIP_TRY(hipMalloc((void **)&d->d_jobs, (size_t)max_frames * 3 * sizeof(mij::DecJob)));
    HIP_TRY(hipMalloc((void **)&d->d_status, (size_t)max_frames * 3 * sizeof(int)));
    HIP_TRY(hipMalloc((void **)&d->d_changed, sizeof(int)));
    return MIJ_OK;
  };
  if (init()) {
    decoder_free(d);
    return nullptr;
  }
  return d;
}

extern "C" void mij_decoder_destroy(mij_decoder *d) { decoder_free(d); }

static int decoder_stage(mij_decoder *d, size_t total) {
  if (total <= d->blob_cap) return MIJ_OK;
  hipFree(d->d_blob);
  if (d->h_blob) hipHostFree(d->h_blob);
  d->d_blob = nullptr;
  d->h_blob = nullptr;
  d->blob_cap = 0;
  const size_t cap = total + total / 4 + 4096;
  HIP_TRY(hipMalloc((void **)&d->d_blob, cap));
  HIP_TRY(hipHostMalloc((void **)&d->h_blob, cap));
  d->blob_cap = cap;
  return MIJ_OK;
}

// Parses n streams, stages them in one device blob and decodes every scan.
// Synchronous; the coefficients stay on the device (mij_decoder_coefs).
// Unstuffed copy of scan bytes [b, e) of stream s into dst; returns bytes
static size_t unstuff(uint8_t *dst, const uint8_t *s, size_t b, size_t e) {
  size_t o = 0;
  while (b < e) {
    const uint8_t *f = (const uint8_t *)memchr(s + b, 0xFF, e - b);
    const size_t stop = f ? (size_t)(f - s) + 1 : e;  // through the 0xFF
    memcpy(dst + o, s + b, stop - b);
    o += stop - b;
    b = stop;
    if (f && b < e && s[b] == 0x00) b++;  // stuffed zero (B.1.1.5)
  }
  return o;
}

static int decoder_buffers(mij_decoder *d, int nchunks, int njobs) {
  if (nchunks <= d->chunk_cap && njobs <= d->job_cap) return MIJ_OK;
  // null each pointer once freed: a failed hipMalloc below must not leave
  // one dangling for the next call or decoder_free to free again
  for (void **p : {(void **)&d->d_entry, (void **)&d->d_exit[0], (void **)&d->d_exit[1], (void **)&d->d_nblk,
                   (void **)&d->d_base}) {
    hipFree(*p);
    *p = nullptr;
  }
  d->chunk_cap = 0;
  const size_t n = (size_t)nchunks + nchunks / 4 + 1024;
  HIP_TRY(hipMalloc((void **)&d->d_entry, n * sizeof(long long)));
  HIP_TRY(hipMalloc((void **)&d->d_exit[0], n * sizeof(long long)));
  HIP_TRY(hipMalloc((void **)&d->d_exit[1], n * sizeof(long long)));
  HIP_TRY(hipMalloc((void **)&d->d_nblk, n * sizeof(int)));
  HIP_TRY(hipMalloc((void **)&d->d_base, n * sizeof(long long)));
  d->chunk_cap = (int)n;
  return MIJ_OK;
}

// Parses n streams, stages their unstuffed scans in one device blob and
// decodes every scan chunk-parallel.  Synchronous; the coefficients stay on
// the device (mij_decoder_coefs).
extern "C" int mij_decoder_decode(mij_decoder *d, const uint8_t *const *jpgs, const size_t *lens, int n) {
  mij_clear_error();
  if (!d || !jpgs || !lens || n < 1 || n > d->cap) return mij_fail(MIJ_EINVAL, "decoder_decode: bad args");
  HIP_TRY(hipSetDevice(d->dev));
  d->n = 0;  // set to n only once every stream decoded cleanly
  d->parsed.assign(n, Parsed());
  // host work per stream in parallel: parse (finds the scan ends), then
  // unstuff each scan into its slot (sized by the raw length, an upper bound)
  const int nth = std::max(1, std::min(n, (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()))));
  auto parallel = [&](auto &&fn) {
    std::atomic<int> next{0};
    std::vector<std::thread> pool;
    for (int t = 1; t < nth; t++)
      pool.emplace_back([&] { for (int f; (f = next++) < n;) fn(f); });
    for (int f; (f = next++) < n;) fn(f);
    for (auto &th : pool) th.join();
  };
  std::vector<int> prc(n, MIJ_OK);
  for (int f = 0; f < n; f++)
    if (!jpgs[f]) return mij_fail(MIJ_EINVAL, "decoder_decode: stream %d is NULL", f);
  parallel([&](int f) { prc[f] = parse(jpgs[f], lens[f], d->parsed[f], f); });
  for (int f = 0; f < n; f++) {
    if (prc[f]) return mij_fail(prc[f], "decoder_decode: stream %d rejected", f);
    const Parsed &P = d->parsed[f];
    if (P.w > d->max_w || P.h > d->max_h)
      return mij_fail(MIJ_EINVAL, "stream %d: %dx%d exceeds the decoder's %dx%d", f, P.w, P.h, d->max_w, d->max_h);
  }
  // slots: raw scan length + >= 16 zero bytes, 8-aligned
  std::vector<size_t> slot(3 * (size_t)n);
  size_t off = 0;
  for (int f = 0; f < n; f++)
    for (int k = 0; k < 3; k++) {
      slot[3 * f + k] = off;
      const auto &sc = d->parsed[f].scan[k];
      off = (off + (size_t)(sc.end - sc.data) + 16 + 7) & ~(size_t)7;
    }
  if (int rc = decoder_stage(d, off)) return rc;
  std::vector<mij::DecTab> tabs(4 * (size_t)n);
  std::vector<mij::DecJob> jobs(3 * (size_t)n);
  const long long fs = d->plane_px * 3 / 2;  // int16 per frame slot
  parallel([&](int f) {
    const Parsed &P = d->parsed[f];
    for (int t = 0; t < 4; t++) tabs[4 * f + t] = P.tab[t];
    const long long ny = (long long)P.w * P.h;
    const long long base[3] = {f * fs, f * fs + ny, f * fs + ny + ny / 4};
    for (int k = 0; k < 3; k++) {
      const auto &sc = P.scan[k];
      const size_t at = slot[3 * f + k];
      const size_t len = unstuff(d->h_blob + at, jpgs[f], (size_t)sc.data, (size_t)sc.end);
      const size_t next = (at + (size_t)(sc.end - sc.data) + 16 + 7) & ~(size_t)7;
      memset(d->h_blob + at + len, 0, next - at - len);
      mij::DecJob &j = jobs[3 * f + k];
      j.data = (long long)at;
      j.nbits = 8LL * (long long)len;
      j.out = base[sc.comp];
      j.nblocks = (int)(sc.comp ? ny / 256 : ny / 64);
      j.dc = 4 * f + 2 * sc.td;
      j.ac = 4 * f + 2 * sc.ta + 1;
    }
  });
  int nchunks = 0, max_chunks = 1;
  for (auto &j : jobs) {
    j.chunk0 = nchunks;
    j.nchunks = std::max(1, (int)((j.nbits + mij::CHUNK - 1) / mij::CHUNK));
    nchunks += j.nchunks;
    max_chunks = std::max(max_chunks, j.nchunks);
  }
  const int nj = 3 * n;
  if (int rc = decoder_buffers(d, nchunks, nj)) return rc;
  HIP_TRY(hipMemcpyAsync(d->d_blob, d->h_blob, off, hipMemcpyHostToDevice, d->stream));
  HIP_TRY(hipMemcpyAsync(d->d_tabs, tabs.data(), tabs.size() * sizeof(mij::DecTab), hipMemcpyHostToDevice,
                         d->stream));
  HIP_TRY(hipMemcpyAsync(d->d_jobs, jobs.data(), jobs.size() * sizeof(mij::DecJob), hipMemcpyHostToDevice,
                         d->stream));
  HIP_TRY(hipMemsetAsync(d->d_status, 0, nj * sizeof(int), d->stream));
  mij::SyncArgs a{d->d_blob, d->d_jobs, nj, nchunks, d->d_tabs, d->d_entry, d->d_exit[1], d->d_exit[0],
                  d->d_nblk, d->d_changed, 1};
  const dim3 grid((nchunks + 255) / 256);
  hipLaunchKernelGGL(mij::k_dec_sync, grid, dim3(256), 0, d->stream, a);
  HIP_TRY(hipGetLastError());
  int cur = 0, passes = 1;
  for (;; passes++) {
    // every pass settles at least one more chunk of each scan, so this bound
    // is never reached by a valid stream (badly synchronising content, e.g.
    // Q=100 noise with blocks longer than a chunk, only costs more passes)
    if (passes > max_chunks + 1) return mij_fail(MIJ_EJPEG, "decoder: chunk states did not settle");
    HIP_TRY(hipMemsetAsync(d->d_changed, 0, sizeof(int), d->stream));
    a.first = 0;
    a.exit_in = d->d_exit[cur];
    a.exit_out = d->d_exit[!cur];
    hipLaunchKernelGGL(mij::k_dec_sync, grid, dim3(256), 0, d->stream, a);
    HIP_TRY(hipGetLastError());
    cur = !cur;
    int changed = 0;
    HIP_TRY(hipMemcpyAsync(&changed, d->d_changed, sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    if (!changed) break;
  }
  d->last_passes = passes;
  hipLaunchKernelGGL(mij::k_dec_scan, dim3(nj), dim3(256), 0, d->stream, d->d_jobs, d->d_nblk, d->d_base,
                     d->d_status);
  hipLaunchKernelGGL(mij::k_dec_write, grid, dim3(256), 0, d->stream, a, d->d_base, d->d_coef, d->d_status);
  HIP_TRY(hipGetLastError());
  std::vector<int> st(nj);
  HIP_TRY(hipMemcpyAsync(st.data(), d->d_status, nj * sizeof(int), hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  for (int j = 0; j < nj; j++)
    if (st[j]) return mij_fail(MIJ_EJPEG, "stream %d scan %d: corrupt entropy data (%d)", j / 3, j % 3, st[j]);
  d->n = n;
  return MIJ_OK;
}

extern "C" int mij_decoder_passes(mij_decoder *d) { return d ? d->last_passes : -1; }

extern "C" int mij_decoder_info(mij_decoder *d, int frame, int *w, int *h, uint8_t dqt[128]) {
  mij_clear_error();
  if (!d || frame < 0 || frame >= d->n) return mij_fail(MIJ_EINVAL, "decoder_info: bad frame");
  const Parsed &P = d->parsed[frame];
  if (w) *w = P.w;
  if (h) *h = P.h;
  if (dqt) {
    memcpy(dqt, P.dqt[0], 64);
    memcpy(dqt + 64, P.dqt[1], 64);
  }
  return MIJ_OK;
}

extern "C" int mij_decoder_coefs(mij_decoder *d, int frame, int16_t *Y, int16_t *Cb, int16_t *Cr) {
  mij_clear_error();
  if (!d || frame < 0 || frame >= d->n || !Y || !Cb || !Cr) return mij_fail(MIJ_EINVAL, "decoder_coefs: bad args");
  HIP_TRY(hipSetDevice(d->dev));
  const Parsed &P = d->parsed[frame];
  const long long ny = (long long)P.w * P.h;
  const int16_t *src = d->d_coef + frame * (d->plane_px * 3 / 2);
  HIP_TRY(hipMemcpyAsync(Y, src, ny * 2, hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipMemcpyAsync(Cb, src + ny, ny / 2, hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipMemcpyAsync(Cr, src + ny + ny / 4, ny / 2, hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return MIJ_OK;
}

extern "C" void *mij_decoder_device_coefs(mij_decoder *d, int frame) {
  if (!d || frame < 0 || frame >= d->n) return nullptr;
  return d->d_coef + frame * (d->plane_px * 3 / 2);
}
