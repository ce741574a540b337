// mij_stream.hip -- PPM ingest and the streaming encoder (host code of
// libmijpeg.so).
//
// * mij_ppm_header / mij_ppm_read: the reference's PPM reader
//   (utils/original.c:294-365) restated with its acceptance rules intact.
// * mij_stream_*: PPM files (or host frames) -> JPEG files (or host buffers)
//   through two device batches used in ping-pong.  Chunk k+1 is read into
//   pinned memory by host threads while the GPU encodes chunk k; every chunk
//   is uploaded, encoded, its lengths fetched, its bytes copied back and
//   written out by host threads, overlapped with the other batch's chunk.
//   Frames stay in PPM byte order (R, G, B): K1 swaps channels as it loads.
//   Three pinned input buffers: the reader threads fill chunk k+1 while chunk
//   k uploads and the bytes of chunk k-1 are written, so the PCIe upload
//   (the bound of a host-fed stream) runs back to back; each frame's upload is
//   enqueued by its reader thread as soon as the frame is in pinned memory.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "mij_host.h"

// ---------------------------------------------------------------------------
// PPM header, utils/original.c:294-365
// ---------------------------------------------------------------------------
// On success the stream is positioned at the first pixel byte.
static int ppm_parse(FILE *f, const char *path, int *w, int *h, long long *off) {
  // :296-300 magic number; :302-303 a newline right after it
  if (fgetc(f) != 'P' || fgetc(f) != '6')
    return mij_fail(MIJ_EPPM, "%s: Could not find magic number for this PPM!", path);
  if (fgetc(f) != '\n') return mij_fail(MIJ_EPPM, "%s: Could not parse the PPM file properly", path);
  // :305-316 lines until the first one that is not a '#' comment (the
  // reference's unbounded line loop is bounded here: 1023 bytes and a
  // newline before EOF, otherwise a parse error)
  char buf[1024];
  for (;;) {
    int n = 0, c;
    while ((c = fgetc(f)) != '\n') {
      if (c == EOF || n == 1023) return mij_fail(MIJ_EPPM, "%s: Could not parse the PPM file properly", path);
      buf[n++] = (char)c;
    }
    buf[n] = '\0';
    if (buf[0] != '#') break;
  }
  int W = 0, H = 0, depth = 0;
  if (sscanf(buf, "%d %d\n", &W, &H) != 2)  // :318
    return mij_fail(MIJ_EPPM, "%s: Could not parse the PPM file properly", path);
  if (W % 16 != 0 || H % 16 != 0)  // :324-328
    return mij_fail(MIJ_EPPM, "%s: Only pictures with dimensions which are multiples of 16 are supported!", path);
  // :330-331 -- "%d\n": the newline directive skips every whitespace byte,
  // including leading pixel bytes 0x09-0x0d / 0x20 (the length check below
  // then rejects the file, as the reference does)
  if (fscanf(f, "%d\n", &depth) != 1) return mij_fail(MIJ_EPPM, "%s: Could not parse the PPM file properly", path);
  if (depth != 255)  // :333-337
    return mij_fail(MIJ_EPPM, "%s: For simplicity, only a bit-depth of 256 is supported!", path);
  // :339-344 the rest of the file is exactly the pixels
  const long pos = ftell(f);
  if (pos < 0 || fseek(f, 0L, SEEK_END) != 0) return mij_fail(MIJ_EIO, "%s: cannot seek", path);
  const long end = ftell(f);
  if (fseek(f, pos, SEEK_SET) != 0) return mij_fail(MIJ_EIO, "%s: cannot seek", path);
  if ((long long)(end - pos) != 3LL * W * H)
    return mij_fail(MIJ_EPPM, "%s: Could not parse the PPM file properly", path);
  if (W <= 0 || H <= 0) return mij_fail(MIJ_EINVAL, "%s: empty image %dx%d", path, W, H);
  *w = W;
  *h = H;
  *off = pos;
  return MIJ_OK;
}

extern "C" int mij_ppm_header(const char *path, int *w, int *h, long long *data_offset) {
  if (!path || !w || !h) return mij_fail(MIJ_EINVAL, "ppm_header: null argument");
  FILE *f = fopen(path, "rb");
  if (!f) return mij_fail(MIJ_EIO, "Cannot open file '%s'!", path);
  long long off = 0;
  const int rc = ppm_parse(f, path, w, h, &off);
  fclose(f);
  if (rc) return rc;
  if (data_offset) *data_offset = off;
  mij_clear_error();
  return MIJ_OK;
}

static void swap_rb(uint8_t *row, int w) {
  for (int x = 0; x < w; x++) std::swap(row[3 * x], row[3 * x + 2]);
}

// reads one PPM into dst; expect_w/h > 0 also checks the geometry
static int ppm_load(const char *path, uint8_t *dst, size_t cap, int pitch, int to_bgr, int expect_w,
                    int expect_h) {
  FILE *f = fopen(path, "rb");
  if (!f) return mij_fail(MIJ_EIO, "Cannot open file '%s'!", path);
  int w = 0, h = 0;
  long long off = 0;
  int rc = ppm_parse(f, path, &w, &h, &off);
  if (!rc && expect_w > 0 && (w != expect_w || h != expect_h))
    rc = mij_fail(MIJ_EINVAL, "%s: %dx%d, the stream encodes %dx%d", path, w, h, expect_w, expect_h);
  if (!rc && (pitch < 3 * w || (size_t)(h - 1) * pitch + 3 * (size_t)w > cap))
    rc = mij_fail(MIJ_ENOSPC, "%s: destination too small", path);
  if (!rc) {
    if (pitch == 3 * w) {
      if (fread(dst, 1, (size_t)3 * w * h, f) != (size_t)3 * w * h) rc = mij_fail(MIJ_EIO, "%s: short read", path);
    } else {
      for (int y = 0; y < h && !rc; y++)
        if (fread(dst + (size_t)y * pitch, 1, (size_t)3 * w, f) != (size_t)3 * w)
          rc = mij_fail(MIJ_EIO, "%s: short read", path);
    }
  }
  fclose(f);
  if (!rc && to_bgr)
    for (int y = 0; y < h; y++) swap_rb(dst + (size_t)y * pitch, w);
  return rc;
}

extern "C" int mij_ppm_read(const char *path, uint8_t *dst, size_t cap, int dst_pitch, int to_bgr) {
  if (!path || !dst) return mij_fail(MIJ_EINVAL, "ppm_read: null argument");
  const int rc = ppm_load(path, dst, cap, dst_pitch, to_bgr, 0, 0);
  if (!rc) mij_clear_error();
  return rc;
}

// ---------------------------------------------------------------------------
// streaming encoder
// ---------------------------------------------------------------------------
#define S_TRY(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess)                                                     \
      return mij_fail(MIJ_EHIP, "%s: %s", #x, hipGetErrorString(e_));         \
  } while (0)

constexpr int NIN = 3;  // pinned input buffers

struct mij_stream {
  int dev = 0, w = 0, h = 0, chunk = 0, threads = 1;
  size_t fbytes = 0;
  mij_batch *b[2] = {nullptr, nullptr};
  hipStream_t st[2] = {nullptr, nullptr};
  uint8_t *h_in[NIN] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_up[NIN] = {};  // the upload out of h_in[i] has completed
  // uploads on a stream of their own, so that a chunk's uploads never queue
  // ahead of another chunk's D2H copies on a batch stream; ev_in_free[i]:
  // batch i's encode has read its input (the next chunk may overwrite it)
  hipStream_t st_up = nullptr;
  hipEvent_t ev_in_free[2] = {};
  uint64_t *h_len[2] = {nullptr, nullptr};
  int *h_err[2] = {nullptr, nullptr};
  uint8_t *h_out[2] = {nullptr, nullptr};
  size_t h_out_cap[2] = {0, 0};
  std::vector<size_t> off[2];
  hipEvent_t ev_len[2] = {}, ev_out[2] = {}, ev_t0[2] = {}, ev_t1[2] = {};
  double stats[MIJ_STREAM_NSTATS] = {};
};

static void stream_free(mij_stream *s) {
  if (!s) return;
  hipSetDevice(s->dev);
  for (int i = 0; i < NIN; i++) {
    if (s->h_in[i]) hipHostFree(s->h_in[i]);
    if (s->ev_up[i]) hipEventDestroy(s->ev_up[i]);
  }
  if (s->st_up) {
    hipStreamSynchronize(s->st_up);
    hipStreamDestroy(s->st_up);
  }
  for (int i = 0; i < 2; i++) {
    if (s->ev_in_free[i]) hipEventDestroy(s->ev_in_free[i]);
    if (s->st[i]) hipStreamSynchronize(s->st[i]);
    if (s->b[i]) mij_batch_destroy(s->b[i]);
    if (s->h_len[i]) hipHostFree(s->h_len[i]);
    if (s->h_err[i]) hipHostFree(s->h_err[i]);
    if (s->h_out[i]) hipHostFree(s->h_out[i]);
    for (hipEvent_t e : {s->ev_len[i], s->ev_out[i], s->ev_t0[i], s->ev_t1[i]})
      if (e) hipEventDestroy(e);
  }
  delete s;
}

static int stream_init(mij_stream *s, int device, int w, int h, int chunk, int quality, int threads) {
  s->dev = device;
  s->w = w;
  s->h = h;
  s->chunk = chunk;
  s->threads = threads > 0 ? threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  s->fbytes = (size_t)3 * w * h;
  for (int i = 0; i < 2; i++) {
    s->b[i] = mij_batch_create(device, w, h, chunk, quality);
    if (!s->b[i]) return mij_last_error();
    if (mij_batch_set_rgb(s->b[i], 1)) return mij_last_error();
    s->st[i] = (hipStream_t)mij_batch_stream(s->b[i]);
  }
  S_TRY(hipSetDevice(device));
  S_TRY(hipStreamCreateWithFlags(&s->st_up, hipStreamNonBlocking));
  for (int i = 0; i < 2; i++) S_TRY(hipEventCreateWithFlags(&s->ev_in_free[i], hipEventDisableTiming));
  for (int i = 0; i < NIN; i++) {
    S_TRY(hipHostMalloc((void **)&s->h_in[i], s->fbytes * chunk, hipHostMallocDefault));
    S_TRY(hipEventCreateWithFlags(&s->ev_up[i], hipEventDisableTiming));
  }
  for (int i = 0; i < 2; i++) {
    S_TRY(hipHostMalloc((void **)&s->h_len[i], sizeof(uint64_t) * chunk, hipHostMallocDefault));
    S_TRY(hipHostMalloc((void **)&s->h_err[i], sizeof(int) * chunk, hipHostMallocDefault));
    s->h_out_cap[i] = std::max<size_t>(1 << 20, s->fbytes / 4 * chunk);  // grows on demand
    S_TRY(hipHostMalloc((void **)&s->h_out[i], s->h_out_cap[i], hipHostMallocDefault));
    s->off[i].assign(chunk + 1, 0);
    for (hipEvent_t *e : {&s->ev_len[i], &s->ev_out[i], &s->ev_t0[i], &s->ev_t1[i]}) S_TRY(hipEventCreate(e));
  }
  return MIJ_OK;
}

extern "C" mij_stream *mij_stream_create(int device, int width, int height, int chunk_frames,
                                         int quality, int host_threads) {
  if (width <= 0 || height <= 0 || width % 16 || height % 16 || chunk_frames < 1 || quality < 1 ||
      quality > 100) {
    mij_fail(MIJ_EINVAL, "stream_create: bad geometry %dx%d, chunk %d or quality %d", width, height,
             chunk_frames, quality);
    return nullptr;
  }
  mij_stream *s = new mij_stream;
  if (stream_init(s, device, width, height, chunk_frames, quality, host_threads)) {
    stream_free(s);
    return nullptr;
  }
  mij_clear_error();
  return s;
}

extern "C" void mij_stream_destroy(mij_stream *s) { stream_free(s); }

extern "C" int mij_stream_stats(mij_stream *s, double *out, int n) {
  if (!s || !out) return mij_fail(MIJ_EINVAL, "stream_stats: null argument");
  for (int i = 0; i < n && i < MIJ_STREAM_NSTATS; i++) out[i] = s->stats[i];
  return MIJ_OK;
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// runs job(i) for i in [0, n) on up to `threads` host threads; returns the
// first nonzero result (by index) or 0.  A failing job's error (thread-local
// to the worker that ran it) is raised again on the calling thread.
static int parallel_for(int n, int threads, const std::function<int(int)> &job, int *failed) {
  std::vector<int> rc(n, 0);
  std::vector<std::string> msg(n);
  std::atomic<int> next{0};
  auto worker = [&]() {
    for (int i; (i = next.fetch_add(1)) < n;)
      if ((rc[i] = job(i))) msg[i] = mij_last_message();
  };
  const int nt = std::min(n, threads);
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; t++) pool.emplace_back(worker);
  worker();
  for (auto &t : pool) t.join();
  for (int i = 0; i < n; i++)
    if (rc[i]) {
      if (failed) *failed = i;
      return mij_fail(rc[i], "%s", msg[i].c_str());
    }
  return 0;
}

// fill(i, dst): frame i into pinned dst (fbytes, RGB rows); drain(i, src, len)
using FillFn = std::function<int(int, uint8_t *)>;
using DrainFn = std::function<int(int, const uint8_t *, size_t)>;

static int stream_run(mij_stream *s, int n, const FillFn &fill, const DrainFn &drain, int *failed) {
  if (failed) *failed = -1;
  S_TRY(hipSetDevice(s->dev));
  for (double &v : s->stats) v = 0.0;
  const double t_start = now_s();
  const int nchunks = (n + s->chunk - 1) / s->chunk;
  // diagnostics (MIJ_STREAM_TRACE=1): per chunk, host times of its read,
  // enqueue and drain steps and device times of its uploads and encode, to
  // stderr after the run
  static const bool trace = getenv("MIJ_STREAM_TRACE") && atoi(getenv("MIJ_STREAM_TRACE"));
  struct Tr {
    double r0 = 0, r1 = 0, enq = 0, len = 0, out = 0, wr = 0;
    hipEvent_t up = nullptr, enc = nullptr;
  };
  std::vector<Tr> tr(trace ? nchunks : 0);
  hipEvent_t tr0 = nullptr;
  if (trace) {
    S_TRY(hipEventCreate(&tr0));
    S_TRY(hipEventRecord(tr0, s->st[0]));
    for (Tr &x : tr) {
      S_TRY(hipEventCreate(&x.up));
      S_TRY(hipEventCreate(&x.enc));
    }
  }
  auto count = [&](int k) { return std::min(s->chunk, n - k * s->chunk); };
  // reader and writer pools share the host threads (writes are small)
  const int wthreads = std::max(1, s->threads / 4), rthreads = std::max(1, s->threads - wthreads);

  // chunk k's files into pinned buffer k % NIN (its previous upload, of chunk
  // k - NIN, has completed: the caller waited for that event); runs on its
  // own thread, ahead of the GPU work
  struct Read {
    std::thread th;
    int rc = MIJ_OK, bad = -1;
    double secs = 0.0;
    std::string msg;  // the reader thread's error, raised again by join_read
  } rd[NIN];
  auto start_read = [&](int k) -> int {
    Read &r = rd[k % NIN];
    r.rc = MIJ_OK;
    r.bad = -1;
    r.msg.clear();
    // batch k & 1's input is free once chunk k - 2's encode has run (its
    // uploads wait for that on the upload stream; the reads do not)
    if (k >= 2) S_TRY(hipStreamWaitEvent(s->st_up, s->ev_in_free[k & 1], 0));
    r.th = std::thread([&, k]() {
      const int first = k * s->chunk, cnt = count(k);
      uint8_t *dst = s->h_in[k % NIN];
      const double t0 = now_s();
      if (trace) tr[k].r0 = t0 - t_start;
      // each frame's upload enqueued on the upload stream as soon as it is
      // read (the copies run while the chunk's other files are read: no
      // chunk-long read before the first byte crosses PCIe)
      mij_batch *bk = s->b[k & 1];
      r.rc = parallel_for(cnt, rthreads, [&](int i) {
        uint8_t *fd = dst + (size_t)i * s->fbytes;
        const int rc = fill(first + i, fd);
        return rc ? rc : mij_batch_upload_slot_async(bk, fd, i, s->st_up);
      }, &r.bad);
      if (r.rc && r.bad >= 0) r.bad += first;
      if (r.rc) {
        r.msg = mij_last_message();
      } else {
        // every upload of chunk k is on the upload stream now, and nothing
        // of chunk k + 1 yet (start_read(k + 1) runs after join_read(k)):
        // the event covers exactly this chunk's copies
        if (hipEventRecord(s->ev_up[k % NIN], s->st_up) != hipSuccess ||
            (trace && hipEventRecord(tr[k].up, s->st_up) != hipSuccess)) {
          r.rc = MIJ_EHIP;
          r.msg = "stream: recording a chunk's upload event failed";
        }
      }
      r.secs = now_s() - t0;
      if (trace) tr[k].r1 = now_s() - t_start;
    });
    return MIJ_OK;
  };
  auto join_read = [&](int k) -> int {
    Read &r = rd[k % NIN];
    if (r.th.joinable()) r.th.join();
    s->stats[1] += r.secs;
    if (r.rc && failed) *failed = r.bad;
    // (the reader thread's error is thread-local to it: raised again here,
    // on the caller's thread, naming the frame)
    if (r.rc) return r.bad >= 0 ? mij_fail(r.rc, "stream: frame %d: %s", r.bad, r.msg.c_str())
                                : mij_fail(r.rc, "%s", r.msg.c_str());
    return r.rc;
  };

  auto enqueue = [&](int k) -> int {
    const int sl = k & 1, cnt = count(k);
    int rc;
    // (the reader thread recorded ev_up[k % NIN] after chunk k's last
    // upload: buffer k % NIN is free and the batch's input is in once it
    // completes)
    if (trace) tr[k].enq = now_s() - t_start;
    S_TRY(hipStreamWaitEvent(s->st[sl], s->ev_up[k % NIN], 0));
    S_TRY(hipEventRecord(s->ev_t0[sl], s->st[sl]));
    if ((rc = mij_batch_encode(s->b[sl], cnt))) return rc;
    S_TRY(hipEventRecord(s->ev_t1[sl], s->st[sl]));
    S_TRY(hipEventRecord(s->ev_in_free[sl], s->st[sl]));
    if (trace) S_TRY(hipEventRecord(tr[k].enc, s->st[sl]));
    if ((rc = mij_batch_lengths_async(s->b[sl], s->h_len[sl], s->h_err[sl], cnt))) return rc;
    S_TRY(hipEventRecord(s->ev_len[sl], s->st[sl]));
    s->stats[5] += (double)cnt * s->fbytes;
    return MIJ_OK;
  };

  auto finish = [&](int k) -> int {
    const int sl = k & 1, first = k * s->chunk, cnt = count(k);
    S_TRY(hipEventSynchronize(s->ev_len[sl]));
    if (trace) tr[k].len = now_s() - t_start;
    std::vector<size_t> &off = s->off[sl];
    off[0] = 0;
    for (int i = 0; i < cnt; i++) {
      if (s->h_err[sl][i]) {
        if (failed) *failed = first + i;
        return mij_frame_fail(s->h_err[sl][i], "stream: frame", first + i);
      }
      off[i + 1] = off[i] + (size_t)s->h_len[sl][i];
    }
    if (off[cnt] > s->h_out_cap[sl]) {  // the previous D2H into this slot has completed
      S_TRY(hipHostFree(s->h_out[sl]));
      s->h_out_cap[sl] = off[cnt] + off[cnt] / 4;
      S_TRY(hipHostMalloc((void **)&s->h_out[sl], s->h_out_cap[sl], hipHostMallocDefault));
    }
    for (int i = 0; i < cnt; i++) {
      const int rc = mij_batch_output_async(s->b[sl], i, s->h_out[sl] + off[i], (size_t)s->h_len[sl][i]);
      if (rc) return rc;
    }
    S_TRY(hipEventRecord(s->ev_out[sl], s->st[sl]));
    S_TRY(hipEventSynchronize(s->ev_out[sl]));
    if (trace) tr[k].out = now_s() - t_start;
    float ms = 0.f;
    S_TRY(hipEventElapsedTime(&ms, s->ev_t0[sl], s->ev_t1[sl]));
    s->stats[3] += ms * 1e-3;
    const double t0 = now_s();
    int bad = -1;
    // (the last chunk's files on every host thread: nothing is read by then)
    const int rc = parallel_for(cnt, k == nchunks - 1 ? s->threads : wthreads,
                                [&](int i) { return drain(first + i, s->h_out[sl] + off[i], off[i + 1] - off[i]); }, &bad);
    s->stats[2] += now_s() - t0;
    if (trace) tr[k].wr = now_s() - t_start;
    s->stats[4] += cnt;
    s->stats[6] += (double)off[cnt];
    if (rc && failed) *failed = first + bad;
    return rc;
  };

  // chunk k: read (reader thread, one chunk ahead) -> upload + encode + lengths
  // (batch k & 1's stream) -> D2H + file writes (this thread, after chunk
  // k + 1 is enqueued).  Buffer k % NIN is refilled with chunk k + NIN only
  // after its upload event.
  int rc = MIJ_OK;
  if (nchunks) rc = start_read(0);
  for (int k = 0; k < nchunks && !rc; k++) {
    rc = join_read(k);
    if (!rc && k + 1 < nchunks) {
      if (k + 1 >= NIN) S_TRY(hipEventSynchronize(s->ev_up[(k + 1) % NIN]));
      rc = start_read(k + 1);
    }
    if (!rc) rc = enqueue(k);
    if (!rc && k >= 1) rc = finish(k - 1);  // chunk k - 1 drains while k uploads and k + 1 is read
  }
  if (!rc && nchunks) rc = finish(nchunks - 1);
  for (auto &r : rd)
    if (r.th.joinable()) r.th.join();  // (an error left a read running)
  if (rc) {  // drain what is still queued before returning
    hipStreamSynchronize(s->st_up);
    hipStreamSynchronize(s->st[0]);
    hipStreamSynchronize(s->st[1]);
  }
  s->stats[0] = now_s() - t_start;
  if (trace) {
    hipDeviceSynchronize();
    for (int k = 0; k < nchunks; k++) {
      float up = 0.f, enc = 0.f;
      hipEventElapsedTime(&up, tr0, tr[k].up);
      hipEventElapsedTime(&enc, tr0, tr[k].enc);
      fprintf(stderr, "stream chunk %d: read %.2f-%.2f ms, enqueued %.2f, uploads done %.2f (device), "
              "encoded %.2f (device), lengths %.2f, bytes back %.2f, files written %.2f\n", k, 1e3 * tr[k].r0,
              1e3 * tr[k].r1, 1e3 * tr[k].enq, up, enc, 1e3 * tr[k].len, 1e3 * tr[k].out, 1e3 * tr[k].wr);
      hipEventDestroy(tr[k].up);
      hipEventDestroy(tr[k].enc);
    }
    fprintf(stderr, "stream run %.2f ms\n", 1e3 * s->stats[0]);
    hipEventDestroy(tr0);
  }
  if (!rc) mij_clear_error();
  return rc;
}

extern "C" int mij_stream_encode_files(mij_stream *s, const char *const *in_paths,
                                       const char *const *out_paths, int n, int *failed) {
  if (!s || !in_paths || !out_paths || n < 0) return mij_fail(MIJ_EINVAL, "stream_encode_files: bad args");
  auto fill = [&](int i, uint8_t *dst) -> int {
    return ppm_load(in_paths[i], dst, s->fbytes, 3 * s->w, 0, s->w, s->h);
  };
  auto drain = [&](int i, const uint8_t *src, size_t len) -> int {
    FILE *f = fopen(out_paths[i], "wb");
    if (!f) return mij_fail(MIJ_EIO, "cannot create '%s'", out_paths[i]);
    const bool ok = fwrite(src, 1, len, f) == len;
    return (fclose(f) == 0 && ok) ? MIJ_OK : mij_fail(MIJ_EIO, "cannot write '%s'", out_paths[i]);
  };
  return stream_run(s, n, fill, drain, failed);
}

extern "C" int mij_stream_encode_frames(mij_stream *s, const uint8_t *const *rgb, int n,
                                        uint8_t *const *outs, const size_t *caps, size_t *lens) {
  if (!s || !rgb || !outs || !caps || !lens || n < 0) return mij_fail(MIJ_EINVAL, "stream_encode_frames: bad args");
  auto fill = [&](int i, uint8_t *dst) -> int {
    memcpy(dst, rgb[i], s->fbytes);
    return MIJ_OK;
  };
  auto drain = [&](int i, const uint8_t *src, size_t len) -> int {
    lens[i] = len;
    if (len > caps[i]) return mij_fail(MIJ_ENOSPC, "stream: frame %d needs %zu bytes", i, len);
    memcpy(outs[i], src, len);
    return MIJ_OK;
  };
  return stream_run(s, n, fill, drain, nullptr);
}
