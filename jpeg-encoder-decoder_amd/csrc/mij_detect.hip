// mij_detect.hip -- the change detector in front of the region encoder
// (reference main/brain.c, caller main.c:136-163).
//
// Device part (one launch per frame): k_detect reads the BGR frame once,
// forms the 4x4 box averages of brain.c:16-45 (one lane per subsampled
// pixel, 3 dwords from each of 4 rows: coalesced 12-byte runs), stores them
// as a packed R|G<<8|B<<16 plane, evaluates the weighted colour distance of
// brain.c:184-195 against the stored plane and ballots the > 600 test into
// one 64-bit word per 64 subsampled pixels of a row.
//
// Host part: the run extraction and the sequential area joining of
// brain.c:104-233 over the bit mask (a 3840x2160 frame has a 960x540 mask,
// 64 KB), then enlargeAdjust and the final merges.  The joining order and
// its quirks are the reference's.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "mij_host.h"

#define HIP_TRY(x)                                                                 \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess)                                                          \
      return mij_fail(MIJ_EHIP, "%s failed: %s", #x, hipGetErrorString(e_));       \
  } while (0)

namespace mij {

// brain.c:184-195.  The reference evaluates d^2 * (2 + cR/256) (and the B
// analogue) in FP64 with cR = (a+b)/2; every step there is an exact dyadic
// rational, so it equals floor(d^2 (1024+s) / 512) with s = a_R + b_R
// (B: floor(d^2 (1534-s) / 512)); the G term is 4 d^2.
__device__ __forceinline__ bool pixel_differs(uint32_t a, uint32_t b) {
  const int ar = a & 255, ag = (a >> 8) & 255, ab = (a >> 16) & 255;
  const int br = b & 255, bg = (b >> 8) & 255, bb = (b >> 16) & 255;
  const uint32_t s = ar + br;
  const uint32_t dr = (ar - br) * (ar - br), dg = (ag - bg) * (ag - bg), db = (ab - bb) * (ab - bb);
  const uint32_t t = ((dr * (1024 + s)) >> 9) + 4 * dg + ((db * (1534 - s)) >> 9);
  return t > 600;
}

// blockDim 256 (4 waves); grid (ceil(sw/256), sh).  FRAME: the current
// plane is computed from the frame and written; otherwise it is read.
// saved == nullptr: no comparison (subsample only).
template <bool FRAME>
__global__ __launch_bounds__(256) void k_detect(const uint8_t *__restrict__ frame, long long pitch,
                                                uint32_t *__restrict__ cur,
                                                const uint32_t *__restrict__ saved,
                                                unsigned long long *__restrict__ mask, int sw,
                                                int words) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  const bool in = x < sw;
  const long long idx = (long long)y * sw + x;
  uint32_t c = 0;
  if (in) {
    if constexpr (FRAME) {
      uint32_t sb = 0, sg = 0, sr = 0;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t *p = (const uint32_t *)(frame + (4LL * y + r) * pitch + 12LL * x);
        const uint32_t d0 = __builtin_nontemporal_load(p), d1 = __builtin_nontemporal_load(p + 1),
                       d2 = __builtin_nontemporal_load(p + 2);
        // bytes of 4 pixels: B G R B | G R B G | R B G R
        sb += ((d0 & 255) + (d0 >> 24) + ((d1 >> 16) & 255) + ((d2 >> 8) & 255));
        sg += (((d0 >> 8) & 255) + (d1 & 255) + (d1 >> 24) + ((d2 >> 16) & 255));
        sr += (((d0 >> 16) & 255) + ((d1 >> 8) & 255) + (d2 & 255) + (d2 >> 24));
      }
      c = (sr >> 4) | ((sg >> 4) << 8) | ((sb >> 4) << 16);
      cur[idx] = c;
    } else {
      c = cur[idx];
    }
  }
  if (!saved) return;
  const bool diff = in && pixel_differs(c, saved[in ? idx : 0]);
  const unsigned long long bits = __ballot(diff);
  const int wi = (blockIdx.x * 256 + (int)threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0 && wi < words) mask[(long long)y * words + wi] = bits;
}

}  // namespace mij

// ---------------------------------------------------------------------------
// host: area joining, brain.c:64-102, :104-233, :240-261
// ---------------------------------------------------------------------------
static bool area_invalid(const area_t &a) { return a.x < 0 || a.y < 0 || a.w < 0 || a.h < 0; }

// brain.c:86-102: w/h hold the right/bottom edges while scanning; after
// enlargeAdjust the same rule keeps the larger width/height (not the union)
static void sum_areas(area_t &a, const area_t b) {
  const bool ia = area_invalid(a), ib = area_invalid(b);
  if (ia && ib) a = area_t{-1, -1, -1, -1};
  else if (ia) a = b;
  else if (!ib) a = area_t{std::min(a.x, b.x), std::min(a.y, b.y), std::max(a.w, b.w), std::max(a.h, b.h)};
}

// brain.c:64-68 (edges form) and :70-74 (x, y, w, h form)
static bool touches_edges(const area_t &a, const area_t &b) {
  return !(a.x > b.w + 1 || a.w + 1 < b.x) && !(a.y > b.h + 1 || a.h + 1 < b.y);
}
static bool touches_sized(const area_t &a, const area_t &b) {
  return !(a.x > b.x + b.w + 2 || a.x + a.w + 2 < b.x) && !(a.y > b.y + b.h + 2 || a.y + a.h + 2 < b.y);
}

// brain.c:240-261: subsampled edges -> frame rectangle, sizes rounded up to
// 16, centred, clamped into the w x h frame
static void enlarge_adjust(area_t &a, int w, int h) {
  int aw = 4 * (a.w - a.x + 1), ah = 4 * (a.h - a.y + 1);
  int ax = 4 * a.x - (16 - aw % 16) / 2, ay = 4 * a.y - (16 - ah % 16) / 2;
  if (aw % 16) aw += 16 - aw % 16;
  if (ah % 16) ah += 16 - ah % 16;
  aw = std::min(aw, w);
  ah = std::min(ah, h);
  if (ax + aw > w) ax -= ax + aw - w;
  if (ay + ah > h) ay -= ay + ah - h;
  a = area_t{std::max(ax, 0), std::max(ay, 0), aw, ah};
}

// first position >= x whose bit equals `set` in one mask row (words*64
// positions; the kernel leaves the bits past sw clear)
static int find_bit(const unsigned long long *m, int words, int x, bool set) {
  int wi = x >> 6;
  if (wi >= words) return words * 64;
  unsigned long long v = (set ? m[wi] : ~m[wi]) & (~0ULL << (x & 63));
  while (!v) {
    if (++wi >= words) return words * 64;
    v = set ? m[wi] : ~m[wi];
  }
  return (wi << 6) + __builtin_ctzll(v);
}

// Runs of differing pixels of one sub-row in the reference's list form.  A
// run that reaches the right edge is never closed (brain.c:197-209 only
// counts a run when a non-differing pixel follows it), so it is not listed.
static int row_runs(const unsigned long long *m, int words, int sw, int y, pair_t *out) {
  int n = 0;
  for (int x = 0; x < sw;) {
    const int beg = find_bit(m, words, x, true);
    if (beg >= sw) break;
    const int stop = find_bit(m, words, beg, false);
    if (stop >= sw) break;  // open at the row end: dropped
    out[n++] = pair_t{beg, stop - 1, y, -1};
    x = stop + 1;
  }
  return n;
}

// brain.c:104-233 over the mask.  L = 2 lists of w/8 runs (main.c:35).
static int join_areas(const unsigned long long *mask, int words, int w, int h, area_t *outs,
                      pair_t *L0, pair_t *L1) {
  const int sw = w / 4, sh = h / 4, cap = w / 8;
  pair_t *L[2] = {L0, L1};
  for (int i = 0; i < 100; i++) outs[i] = area_t{-1, -1, -1, -1};
  for (int i = 0; i < cap; i++) L0[i] = L1[i] = pair_t{-1, -1, -1, -1};
  int n = 0, cur = 0, ncur = 0, nprev = 0;
  for (int y = 0; y < sh; y++) {
    pair_t *rk = L[cur], *rz = L[!cur];
    for (int k = 0; k < ncur; k++) {
      bool joined = false;
      for (int z = 0; z < nprev; z++) {
        if (rk[k].end < rz[z].beg - 1 || rk[k].beg > rz[z].end + 1) continue;
        joined = true;
        if (rk[k].done >= 0) {
          const int lo = std::min(rz[z].done, rk[k].done), hi = std::max(rz[z].done, rk[k].done);
          if (lo == hi) continue;
          sum_areas(outs[lo], outs[hi]);
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
          sum_areas(outs[rz[z].done], area_t{rk[k].beg, rk[k].row, rk[k].end, rk[k].row});
        }
      }
      if (joined) continue;
      if (n > 99) {  // brain.c:156-168: compaction, labels left as they are
        for (int i = 0; i < n; i++)
          for (int j = i + 1; j < n; j++)
            if (touches_edges(outs[i], outs[j])) {
              sum_areas(outs[i], outs[j]);
              n--;
              outs[j] = outs[n];
            }
        if (n > 99) return n;
      }
      rk[k].done = n;
      outs[n++] = area_t{rk[k].beg, rk[k].row, rk[k].end, rk[k].row};
    }
    cur = !cur;
    nprev = ncur;
    ncur = row_runs(mask + (long long)y * words, words, sw, y, L[cur]);
  }
  for (int i = 0; i < n; i++) enlarge_adjust(outs[i], w, h);
  for (int i = 0; i < n; i++)
    for (int j = i + 1; j < n; j++)
      if (touches_sized(outs[i], outs[j])) {
        sum_areas(outs[i], outs[j]);
        n--;
        outs[j] = outs[n];
        j--;
      }
  for (int i = 0; i < n;) {
    if (outs[i].w < 32 && outs[i].h < 24) {
      n--;
      if (i < n) outs[i] = outs[n];
      outs[n] = area_t{-1, -1, -1, -1};
    } else {
      i++;
    }
  }
  return n;
}

// ---------------------------------------------------------------------------
// detector object
// ---------------------------------------------------------------------------
struct mij_detector {
  int dev = 0;
  hipStream_t stream = nullptr;
  int w = 0, h = 0, sw = 0, sh = 0, words = 0;
  uint32_t *d_plane[2] = {nullptr, nullptr};  // [0] current, [1] stored
  unsigned long long *d_mask = nullptr, *h_mask = nullptr;
  uint8_t *d_frame = nullptr;                  // host-frame uploads
  size_t frame_bytes = 0;
  std::vector<pair_t> lists;                   // 2 x w/8 runs
};

static void detector_free(mij_detector *d) {
  if (!d) return;
  hipSetDevice(d->dev);
  if (d->stream) hipStreamSynchronize(d->stream);
  for (auto *p : d->d_plane) hipFree(p);
  hipFree(d->d_mask);
  hipFree(d->d_frame);
  if (d->h_mask) hipHostFree(d->h_mask);
  if (d->stream) hipStreamDestroy(d->stream);
  delete d;
}

static int detector_init(mij_detector *d, int device, int w, int h) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return mij_fail(MIJ_ENODEV, "no HIP device visible (the HIP path has no CPU fallback)");
  if (device < 0 || device >= n) return mij_fail(MIJ_ENODEV, "device %d out of range (%d)", device, n);
  d->dev = device;
  d->w = w;
  d->h = h;
  d->sw = w / 4;
  d->sh = h / 4;
  d->words = (d->sw + 63) / 64;
  d->lists.assign(2 * (size_t)(w / 8), pair_t{-1, -1, -1, -1});
  const size_t plane = (size_t)d->sw * d->sh * sizeof(uint32_t);
  const size_t mwords = (size_t)d->words * d->sh;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  for (auto &p : d->d_plane) {
    HIP_TRY(hipMalloc((void **)&p, plane));
    HIP_TRY(hipMemsetAsync(p, 0, plane, d->stream));  // main.c:33 static saved[]
  }
  HIP_TRY(hipMalloc((void **)&d->d_mask, mwords * sizeof(unsigned long long)));
  HIP_TRY(hipHostMalloc((void **)&d->h_mask, mwords * sizeof(unsigned long long)));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return MIJ_OK;
}

extern "C" mij_detector *mij_detector_create(int device, int width, int height) {
  mij_clear_error();
  if (width < 16 || height < 16 || width % 4 || height % 4) {
    mij_fail(MIJ_EINVAL, "detector_create: frame %dx%d (multiples of 4, at least 16)", width, height);
    return nullptr;
  }
  auto *d = new mij_detector();
  if (detector_init(d, device, width, height)) {
    detector_free(d);
    return nullptr;
  }
  return d;
}

extern "C" void mij_detector_destroy(mij_detector *d) { detector_free(d); }

static int launch_detect(mij_detector *d, const void *frame, long long pitch, bool compare) {
  const dim3 grid((d->sw + 255) / 256, d->sh);
  if (frame) {
    if (pitch < 3LL * d->w || (pitch & 3) || ((uintptr_t)frame & 3))
      return mij_fail(MIJ_EINVAL, "detector: frame pitch %lld / pointer not 4-byte aligned or short", pitch);
    hipLaunchKernelGGL(mij::k_detect<true>, grid, dim3(256), 0, d->stream, (const uint8_t *)frame,
                       pitch, d->d_plane[0], compare ? d->d_plane[1] : nullptr, d->d_mask, d->sw,
                       d->words);
  } else {
    hipLaunchKernelGGL(mij::k_detect<false>, grid, dim3(256), 0, d->stream, nullptr, 0LL,
                       d->d_plane[0], d->d_plane[1], d->d_mask, d->sw, d->words);
  }
  HIP_TRY(hipGetLastError());
  return MIJ_OK;
}

static int finish_compare(mij_detector *d, area_t *outs, int *count, pair_t *lists) {
  const size_t mwords = (size_t)d->words * d->sh;
  HIP_TRY(hipMemcpyAsync(d->h_mask, d->d_mask, mwords * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  pair_t *L = lists ? lists : d->lists.data();
  const int n = join_areas(d->h_mask, d->words, d->w, d->h, outs, L, L + d->w / 8);
  if (count) *count = n;
  return MIJ_OK;
}

extern "C" int mij_detector_subsample(mij_detector *d, const void *d_frame, long long pitch) {
  mij_clear_error();
  if (!d || !d_frame) return mij_fail(MIJ_EINVAL, "detector_subsample: null argument");
  HIP_TRY(hipSetDevice(d->dev));
  return launch_detect(d, d_frame, pitch, false);
}

extern "C" int mij_detector_compare(mij_detector *d, area_t outs[100], int *count) {
  mij_clear_error();
  if (!d || !outs) return mij_fail(MIJ_EINVAL, "detector_compare: null argument");
  HIP_TRY(hipSetDevice(d->dev));
  if (int rc = launch_detect(d, nullptr, 0, true)) return rc;
  return finish_compare(d, outs, count, nullptr);
}

extern "C" int mij_detector_step(mij_detector *d, const void *d_frame, long long pitch, area_t outs[100],
                                 int *count) {
  mij_clear_error();
  if (!d || !d_frame || !outs) return mij_fail(MIJ_EINVAL, "detector_step: null argument");
  HIP_TRY(hipSetDevice(d->dev));
  if (int rc = launch_detect(d, d_frame, pitch, true)) return rc;
  return finish_compare(d, outs, count, nullptr);
}

extern "C" int mij_detector_launch(mij_detector *d, const void *d_frame, long long pitch) {
  mij_clear_error();
  if (!d || !d_frame) return mij_fail(MIJ_EINVAL, "detector_launch: null argument");
  HIP_TRY(hipSetDevice(d->dev));
  return launch_detect(d, d_frame, pitch, true);
}

extern "C" int mij_detector_store(mij_detector *d) {
  mij_clear_error();
  if (!d) return mij_fail(MIJ_EINVAL, "detector_store: null detector");
  HIP_TRY(hipSetDevice(d->dev));
  HIP_TRY(hipMemcpyAsync(d->d_plane[1], d->d_plane[0], (size_t)d->sw * d->sh * sizeof(uint32_t),
                         hipMemcpyDeviceToDevice, d->stream));
  return MIJ_OK;
}

extern "C" int mij_detector_upload(mij_detector *d, const uint8_t *bgr, long long pitch,
                                   const void **d_frame) {
  mij_clear_error();
  if (!d || !bgr) return mij_fail(MIJ_EINVAL, "detector_upload: null argument");
  if (!pitch) pitch = 3LL * d->w;
  if (pitch < 3LL * d->w || (pitch & 3)) return mij_fail(MIJ_EINVAL, "detector_upload: pitch %lld", pitch);
  HIP_TRY(hipSetDevice(d->dev));
  const size_t bytes = (size_t)pitch * d->h;
  if (d->frame_bytes < bytes) {
    hipFree(d->d_frame);
    d->d_frame = nullptr;
    d->frame_bytes = 0;
    HIP_TRY(hipMalloc((void **)&d->d_frame, bytes));
    d->frame_bytes = bytes;
  }
  HIP_TRY(hipMemcpyAsync(d->d_frame, bgr, bytes, hipMemcpyHostToDevice, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  if (d_frame) *d_frame = d->d_frame;
  return MIJ_OK;
}

extern "C" int mij_detector_get_plane(mij_detector *d, int which, uint8_t *rgb) {
  mij_clear_error();
  if (!d || !rgb || which < 0 || which > 1) return mij_fail(MIJ_EINVAL, "detector_get_plane: bad args");
  HIP_TRY(hipSetDevice(d->dev));
  std::vector<uint32_t> p((size_t)d->sw * d->sh);
  HIP_TRY(hipMemcpyAsync(p.data(), d->d_plane[which], p.size() * 4, hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  for (size_t i = 0; i < p.size(); i++) {
    rgb[3 * i] = p[i] & 255;
    rgb[3 * i + 1] = (p[i] >> 8) & 255;
    rgb[3 * i + 2] = (p[i] >> 16) & 255;
  }
  return MIJ_OK;
}

extern "C" int mij_detector_set_plane(mij_detector *d, int which, const uint8_t *rgb) {
  mij_clear_error();
  if (!d || !rgb || which < 0 || which > 1) return mij_fail(MIJ_EINVAL, "detector_set_plane: bad args");
  HIP_TRY(hipSetDevice(d->dev));
  std::vector<uint32_t> p((size_t)d->sw * d->sh);
  for (size_t i = 0; i < p.size(); i++)
    p[i] = rgb[3 * i] | (uint32_t)rgb[3 * i + 1] << 8 | (uint32_t)rgb[3 * i + 2] << 16;
  HIP_TRY(hipMemcpyAsync(d->d_plane[which], p.data(), p.size() * 4, hipMemcpyHostToDevice, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return MIJ_OK;
}

extern "C" int mij_detector_mask(mij_detector *d, unsigned long long *dst, size_t cap_words, int *words) {
  mij_clear_error();
  if (!d) return mij_fail(MIJ_EINVAL, "detector_mask: null detector");
  const size_t mwords = (size_t)d->words * d->sh;
  if (words) *words = d->words;
  if (!dst) return MIJ_OK;
  if (cap_words < mwords) return mij_fail(MIJ_ENOSPC, "detector_mask: %zu words needed", mwords);
  memcpy(dst, d->h_mask, mwords * sizeof(unsigned long long));
  return MIJ_OK;
}

extern "C" void *mij_detector_stream(mij_detector *d) { return d ? (void *)d->stream : nullptr; }

// ---------------------------------------------------------------------------
// drop-in entry points (include/brain.h:7-10) on WIDTH x HEIGHT frames
// ---------------------------------------------------------------------------
static std::mutex g_dmu;
static mij_detector *g_det = nullptr;
static int g_height = 240;  // define.h:4 HEIGHT

extern "C" int mij_set_frame_height(int height) {
  if (height < 16 || height % 4) return mij_fail(MIJ_EINVAL, "frame height %d", height);
  std::lock_guard<std::mutex> l(g_dmu);
  g_height = height;
  return MIJ_OK;
}

static mij_detector *drop_detector() {
  const int w = mij_drop_stride(), h = g_height;
  if (g_det && g_det->w == w && g_det->h == h) return g_det;
  detector_free(g_det);
  g_det = mij_detector_create(mij_drop_device(), w, h);
  return g_det;
}

extern "C" void subsample(FILE *f, uint8_t *in, uint8_t *out) {
  std::lock_guard<std::mutex> l(g_dmu);
  mij_detector *d = drop_detector();
  const void *frame = nullptr;
  if (!d || mij_detector_upload(d, in, 0, &frame) || mij_detector_subsample(d, frame, 3LL * d->w) ||
      mij_detector_get_plane(d, 0, out))
    return;
  if (f) {  // brain.c:22 header, :29-42 the bytes
    fprintf(f, "P6\n%i %i\n255\n", d->w / 4, d->h / 4);
    fwrite(out, 1, 3ULL * d->sw * d->sh, f);
  }
}

extern "C" void store(uint8_t *in, uint8_t *saved) {  // brain.c:53-60, a host copy
  std::lock_guard<std::mutex> l(g_dmu);
  const size_t n = 3ULL * (mij_drop_stride() / 4) * (g_height / 4);
  memmove(saved, in, n);
}

extern "C" uint8_t compare(uint8_t *in, uint8_t *saved, area_t *outs, pair_t (*differences)[]) {
  std::lock_guard<std::mutex> l(g_dmu);
  mij_detector *d = drop_detector();
  int n = 0;
  if (!d || mij_detector_set_plane(d, 0, in) || mij_detector_set_plane(d, 1, saved) ||
      launch_detect(d, nullptr, 0, true) ||
      finish_compare(d, outs, &n, differences ? (pair_t *)differences : nullptr))
    return 0;
  return (uint8_t)n;
}

extern "C" void enlargeAdjust(area_t *a) {
  std::lock_guard<std::mutex> l(g_dmu);
  if (a) enlarge_adjust(*a, mij_drop_stride(), g_height);
}
