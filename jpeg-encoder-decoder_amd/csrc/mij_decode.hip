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
// Huffman tables with a 9-bit lookahead.  Device: one lane per (frame,
// scan) decodes its scan sequentially: a 64-bit bit buffer refilled a byte
// at a time with the 0xFF 0x00 unstuffing inline, table lookups from the
// L1/L2-resident per-frame tables, coefficients written block by block.
// Entropy decoding of one scan is sequential by construction; the batch
// gives the parallelism (3 lanes per frame).
#include <hip/hip_runtime.h>
#include <string.h>

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
  long long data, end;  // scan bytes [data, end) in the stream blob
  long long out;        // first int16 of the component's plane
  int nblocks;
  int dc, ac;           // table indices
  int frame;
};

struct BitReader {
  const uint8_t *p;
  long long pos, end;
  unsigned long long acc;
  int n;
  int fed0;  // zero bytes fed past the scan's end
  __device__ void fill() {
    while (n <= 56) {
      uint32_t b = 0;
      if (pos < end) {
        b = p[pos++];
        if (b == 0xFF) pos++;  // stuffed 0x00 (B.1.1.5)
      } else {
        fed0++;
      }
      acc |= (unsigned long long)b << (56 - n);
      n += 8;
    }
  }
  __device__ uint32_t peek(int k) const { return (uint32_t)(acc >> (64 - k)); }
  __device__ void skip(int k) {
    acc <<= k;
    n -= k;
  }
};

__device__ __forceinline__ int decode_sym(BitReader &br, const DecTab &t) {
  br.fill();
  const uint32_t e = t.look[br.peek(LOOK)];
  if (e) {
    br.skip(e >> 8);
    return e & 255;
  }
  for (int l = LOOK + 1; l <= 16; l++) {
    const int32_t code = (int32_t)br.peek(l);
    if (code <= t.maxcode[l]) {
      br.skip(l);
      return t.val[t.valoff[l] + code];
    }
  }
  return -1;
}

// F.2.2.1 EXTEND: s magnitude bits; the encoder's negative form is ~|v|
// (encoder.c:442-444)
__device__ __forceinline__ int receive_extend(BitReader &br, int s) {
  if (!s) return 0;
  br.fill();
  const int v = (int)br.peek(s);
  br.skip(s);
  return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
}

__global__ __launch_bounds__(64) void k_decode_scans(const uint8_t *__restrict__ blob,
                                                     const DecJob *__restrict__ jobs, int njobs,
                                                     const DecTab *__restrict__ tabs,
                                                     int16_t *__restrict__ coefs,
                                                     int *__restrict__ status) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= njobs) return;
  const DecJob job = jobs[j];
  const DecTab &dc = tabs[job.dc];
  const DecTab &ac = tabs[job.ac];
  BitReader br{blob, job.data, job.end, 0ULL, 0, 0};
  int16_t *out = coefs + job.out;
  int err = 0;
  for (int b = 0; b < job.nblocks && !err; b++) {
    int16_t *blk = out + 64LL * b;
    int4 *o = (int4 *)blk;
#pragma unroll
    for (int q = 0; q < 8; q++) o[q] = int4{0, 0, 0, 0};
    const int s = decode_sym(br, dc);
    if (s < 0 || s > 15) {
      err = 1;
      break;
    }
    blk[0] = (int16_t)receive_extend(br, s);
    for (int k = 1; k < 64;) {
      const int rs = decode_sym(br, ac);
      if (rs < 0) {
        err = 2;
        break;
      }
      const int r = rs >> 4, sz = rs & 15;
      if (!sz) {
        if (r != 15) break;  // EOB
        k += 16;             // ZRL
        continue;
      }
      k += r;
      if (k > 63) {
        err = 3;
        break;
      }
      blk[k++] = (int16_t)receive_extend(br, sz);
    }
  }
  // bits consumed past the scan's bytes: truncated or corrupt stream
  if (!err && 8 * br.fed0 > br.n) err = 4;
  status[j] = err;
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
extern "C" int mij_decoder_decode(mij_decoder *d, const uint8_t *const *jpgs, const size_t *lens, int n) {
  mij_clear_error();
  if (!d || !jpgs || !lens || n < 1 || n > d->cap) return mij_fail(MIJ_EINVAL, "decoder_decode: bad args");
  HIP_TRY(hipSetDevice(d->dev));
  d->parsed.assign(n, Parsed());
  size_t total = 0;
  for (int f = 0; f < n; f++) {
    if (!jpgs[f]) return mij_fail(MIJ_EINVAL, "decoder_decode: stream %d is NULL", f);
    if (int rc = parse(jpgs[f], lens[f], d->parsed[f], f)) return rc;
    const Parsed &P = d->parsed[f];
    if (P.w > d->max_w || P.h > d->max_h)
      return mij_fail(MIJ_EINVAL, "stream %d: %dx%d exceeds the decoder's %dx%d", f, P.w, P.h, d->max_w, d->max_h);
    total += lens[f];
  }
  if (int rc = decoder_stage(d, total)) return rc;
  std::vector<mij::DecTab> tabs(4 * (size_t)n);
  std::vector<mij::DecJob> jobs(3 * (size_t)n);
  size_t off = 0;
  const long long fs = d->plane_px * 3 / 2;  // int16 per frame slot
  for (int f = 0; f < n; f++) {
    const Parsed &P = d->parsed[f];
    memcpy(d->h_blob + off, jpgs[f], lens[f]);
    for (int t = 0; t < 4; t++) tabs[4 * f + t] = P.tab[t];
    const long long ny = (long long)P.w * P.h;
    const long long base[3] = {f * fs, f * fs + ny, f * fs + ny + ny / 4};
    for (int k = 0; k < 3; k++) {
      const auto &sc = P.scan[k];
      mij::DecJob &j = jobs[3 * f + k];
      j.data = (long long)off + sc.data;
      j.end = (long long)off + sc.end;
      j.out = base[sc.comp];
      j.nblocks = (int)(sc.comp ? ny / 256 : ny / 64);
      j.dc = 4 * f + 2 * sc.td;
      j.ac = 4 * f + 2 * sc.ta + 1;
      j.frame = f;
    }
    off += lens[f];
  }
  d->n = n;
  HIP_TRY(hipMemcpyAsync(d->d_blob, d->h_blob, total, hipMemcpyHostToDevice, d->stream));
  HIP_TRY(hipMemcpyAsync(d->d_tabs, tabs.data(), tabs.size() * sizeof(mij::DecTab), hipMemcpyHostToDevice,
                         d->stream));
  HIP_TRY(hipMemcpyAsync(d->d_jobs, jobs.data(), jobs.size() * sizeof(mij::DecJob), hipMemcpyHostToDevice,
                         d->stream));
  const int nj = 3 * n;
  hipLaunchKernelGGL(mij::k_decode_scans, dim3((nj + 63) / 64), dim3(64), 0, d->stream, d->d_blob, d->d_jobs,
                     nj, d->d_tabs, d->d_coef, d->d_status);
  HIP_TRY(hipGetLastError());
  std::vector<int> st(nj);
  HIP_TRY(hipMemcpyAsync(st.data(), d->d_status, nj * sizeof(int), hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  for (int j = 0; j < nj; j++)
    if (st[j]) return mij_fail(MIJ_EJPEG, "stream %d scan %d: corrupt entropy data (%d)", j / 3, j % 3, st[j]);
  return MIJ_OK;
}

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
