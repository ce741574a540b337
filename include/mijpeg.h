/*
 * mijpeg.h -- C ABI of the MI355X-native (gfx950) JPEG block-encode path.
 *
 * Drop-in replacement for the reference's encoder
 * (MattiaDallaCosta/JPEG-encoder-decoder include/encoder.h:10-12,
 * include/structs.h:5-18): a C host that includes this header instead of
 * encoder.h and links libmijpeg.so gets the same three entry points with the
 * same signatures, argument meaning, buffer ownership and output bytes; the
 * work runs as HIP kernels on the GPU.  See INTEGRATION.md.
 *
 * Plain C types only: no HIP/torch types cross this boundary.
 */
#ifndef MIJPEG_H
#define MIJPEG_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- types: layout-identical to the reference --------------------------- */

/* include/structs.h:5-13 (ISO/IEC 10918-1 K.2 table state). */
typedef struct __huff_code {
    int sym_freq[257];
    int code_len[257];
    int next[257];
    int code_len_freq[32];
    int sym_sorted[256];
    int sym_code_len[256];
    int sym_code[256];
} huff_code;

/* include/structs.h:15-18: a sub-rectangle of the input frame; w and h must
 * be multiples of 16 (the reference silently produced garbage otherwise,
 * this library rejects them, see mij_last_error). */
typedef struct {
    int x, y;
    int w, h;
} area_t;

/* ---- drop-in entry points ------------------------------------------------ */

/* Replaces encoder.h:10 / encoder.c:158-178.  `in` is a BGR888 frame whose
 * row stride is the reference's compile-time WIDTH (define.h:3, 320 px) or
 * the value set with mij_set_input_stride().  Writes the quantized, zigzagged
 * coefficients with DC differences into Y[w*h], Cb[w*h/4], Cr[w*h/4] (block
 * raster order per component). */
void rgb_to_dct(uint8_t *in, int16_t *Y, int16_t *Cb, int16_t *Cr, area_t dims);

/* Replaces encoder.h:11 / encoder.c:360-381: fills the four optimized
 * Huffman tables (Luma[0]=DC, Luma[1]=AC, Chroma[0]=DC, Chroma[1]=AC);
 * every field ends in the state the reference leaves it in. */
void init_huffman(int16_t *Y, int16_t *Cb, int16_t *Cr, area_t dims,
                  huff_code Luma[2], huff_code Chroma[2]);

/* Replaces encoder.h:12 / encoder.c:549-644: writes the JFIF stream to `f`
 * (may be NULL here, unlike the reference) and to jpg[], returns its size
 * (0 on error).  jpg must hold mij_max_jpg_bytes(w, h) bytes to be safe. */
size_t write_jpg(FILE *f, uint8_t *jpg, int16_t *Y, int16_t *Cb, int16_t *Cr,
                 area_t dims, huff_code Luma[2], huff_code Chroma[2]);

/* ---- extensions ----------------------------------------------------------- */

/* Runtime replacement for define.h:3 WIDTH (input row stride in pixels used
 * by rgb_to_dct).  Default 320.  Returns 0 or an error code. */
int mij_set_input_stride(int stride_px);

/* Quality factor for the drop-in calls, scaled like utils/original.c:504-509.
 * Default 50 == the reference's fixed tables (encoder.c:18-36). */
int mij_set_quality(int quality);

/* Error reporting (the reference has none: encoder.c returns void). */
enum {
    MIJ_OK = 0,
    MIJ_EINVAL = 1,     /* dims not multiples of 16, bad stride/quality, ... */
    MIJ_ENODEV = 2,     /* no usable HIP device / runtime */
    MIJ_EHIP = 3,       /* a HIP runtime call failed */
    MIJ_ENOSPC = 4,     /* output capacity too small */
    MIJ_ETABLE = 5,     /* Huffman construction outside the reference's
                           defined behaviour (code length >= 32 etc.) */
    MIJ_EPPM = 6,       /* PPM rejected by the rules of utils/original.c:294-365 */
    MIJ_EIO = 7,        /* file could not be opened, read or written */
    MIJ_EJPEG = 8,      /* decoder: stream outside the supported JFIF subset or corrupt */
    MIJ_EHANG = 9       /* a device-side wait (pack look-back, ticket) outlasted its
                           bound: the frame's device state was corrupted; the
                           frame fails instead of the launch hanging */
};
int mij_last_error(void);
const char *mij_strerror(int code);
/* Text of the calling thread's last failure ("" before any): what was wrong
 * with which argument, beyond the code mij_last_error returns. */
const char *mij_last_message(void);

/* Worst-case size of an encoded w x h frame (all 63 AC coefficients coded at
 * 27 bits, every byte stuffed). */
size_t mij_max_jpg_bytes(int w, int h);

/* Whole path host->host (rgb_to_dct -> init_huffman -> write_jpg without the
 * host round trips of the three-call split).  `bgr` + stride_px describe the
 * frame, dims the region.  Returns MIJ_OK and the size in *out_len. */
int mij_encode(const uint8_t *bgr, int stride_px, area_t dims, int quality,
               uint8_t *out, size_t cap, size_t *out_len);

/* ---- device-resident batch pipeline (throughput path) ---------------------
 * A batch object owns the device buffers for up to max_frames frames of one
 * geometry; frames are independent (own tables, own JFIF stream).  All work
 * is queued on the batch's HIP stream; outputs stay in HBM until fetched. */
typedef struct mij_batch mij_batch;

mij_batch *mij_batch_create(int device, int width, int height, int max_frames,
                            int quality);
void mij_batch_destroy(mij_batch *b);
/* packed BGR888 frames (width*height*3 bytes each) from host memory into
 * batch slots first .. first+nframes-1 */
int mij_batch_upload(mij_batch *b, const uint8_t *bgr, int first, int nframes);
/* or point the batch at frames already in device memory (not owned):
 * frame i starts at d_bgr + i*frame_stride, rows pitch bytes apart
 * (pointer, pitch and frame stride 16-byte aligned: K1 streams rows with
 * 16-byte LDS-DMA loads) */
int mij_batch_set_input(mij_batch *b, const void *d_bgr, long long frame_stride,
                        int pitch);
int mij_batch_encode(mij_batch *b, int nframes);     /* full path, async */
/* pipeline: fused (default) -- K1 emits the symbol tokens directly, the
 * coefficient planes never reach HBM; split (set_split(b, 1)) -- K1 writes
 * zigzag coefficient planes and a second pass tokenizes them.  Same output
 * bytes either way. */
int mij_batch_set_split(mij_batch *b, int on);
/* fused pipeline: encode in nsub sub-batches (1 = off, at most 16), the
 * entropy stages of sub-batch k on a second stream behind K1 of sub-batch k,
 * concurrent with K1 of sub-batch k + 1.  Same output bytes; stage timing
 * then reports K1 over all sub-batches ([0]) and the whole encode ([7]). */
int mij_batch_set_overlap(mij_batch *b, int nsub);
/* Entropy-stage variants of the fused pipeline.  Every setting gives the
 * same output bytes; the defaults are the measured-fastest ones and the
 * others exist for A/B timing (bench.py --opt NAME=V) and are covered by
 * tests/test_options.py.
 *   MIJ_OPT_SEAM          1 (default): every scan word stored whole, shared
 *                         group edge words ORed in afterwards; 0: edge words
 *                         ORed onto zeroed scan buffers (the band paths' form)
 *   MIJ_OPT_FF_PACK       1 (default, seam mode only): the packing counts the
 *                         0xFF bytes of every output chunk; 0: a counting pass
 *   MIJ_OPT_ACTAB         1 (default): on batches of >= 16 frames the AC
 *                         tables are built beside the segment DCs; 0: after
 *   MIJ_OPT_SEGDC_FUSED   0 (default); 1: the segment DCs inside the table
 *                         kernel's DC waves
 *   MIJ_OPT_PACK_WIDE     -1 (default: the wide window from quality 85);
 *                         0 / 1 force the default / wide pack window
 *   MIJ_OPT_EMIT_SLOTS    0 (default: chosen from frame count, size and Q);
 *                         > 0: JFIF-assembly workgroups per frame
 *   MIJ_OPT_OVERLAP_PRIO  1 (default): the overlap stream (set_overlap) at
 *                         the highest priority; 0: the lowest
 *   (7 is reserved: an internal fault-injection hook of the test suite,
 *   not settable through this call)
 *   MIJ_OPT_PACK_SEGS     -1 (default: chosen from the quality); otherwise
 *                         ly + 4 * lc (0..15): the packing's groups take
 *                         32 << ly luma and 32 << lc chroma segments */
enum {
  MIJ_OPT_SEAM = 0,
  MIJ_OPT_FF_PACK = 1,
  MIJ_OPT_ACTAB = 2,
  MIJ_OPT_SEGDC_FUSED = 3,
  MIJ_OPT_PACK_WIDE = 4,
  MIJ_OPT_EMIT_SLOTS = 5,
  MIJ_OPT_OVERLAP_PRIO = 6,
  /* 7: reserved */
  MIJ_OPT_PACK_SEGS = 8,
  MIJ_OPT_COUNT = 9
};
int mij_batch_set_option(mij_batch *b, int opt, int value);
int mij_batch_get_option(mij_batch *b, int opt);
/* input frames in R, G, B byte order (PPM files, brain.c:25-42) instead of the
 * encoder's B, G, R (encoder.c:133); the channels are swapped inside K1, at no
 * cost.  Both pipelines. */
int mij_batch_set_rgb(mij_batch *b, int on);
/* fused pipeline only: also keep the coefficient planes (for
 * mij_batch_coefs); the split pipeline always has them */
int mij_batch_keep_coefs(mij_batch *b, int on);
int mij_batch_dct(mij_batch *b, int nframes);        /* K1 only, async */
/* Measurement only (bench.py): K1's memory traffic without its arithmetic --
 * the coefficient variant's persistent grid, tile claims, LDS-DMA of the BGR
 * tiles one tile ahead and whole-line coefficient + raw-DC stores -- on
 * frames 0..n-1, timed like mij_batch_dct; the coefficient planes are left
 * holding garbage.  Its time is the floor of K1's access pattern on this GPU.
 * Plain B, G, R batches only; async. */
int mij_batch_pattern_floor(mij_batch *b, int nframes);
int mij_batch_sync(mij_batch *b);
int mij_batch_output(mij_batch *b, int frame, uint8_t *dst, size_t cap,
                     size_t *len);
int mij_batch_lengths(mij_batch *b, size_t *lens, int nframes);
/* quantized zigzag coefficient planes of a frame; diffed != 0 applies the DC
 * differencing of encoder.c:168-177 (as rgb_to_dct returns them) */
int mij_batch_coefs(mij_batch *b, int frame, int16_t *Y, int16_t *Cb,
                    int16_t *Cr, int diffed);
int mij_batch_tables(mij_batch *b, int frame, huff_code out[4]);
/* timing: when enabled, HIP events bracket each stage of the next encode;
 * mij_batch_stage_ms returns up to n (<= MIJ_NSTAGES) stage durations (ms) of
 * the last one: [0]=K1 colour+DCT+quant (+tokens when fused), [1]=fix (FP64
 * re-encode of the blocks K1 listed), [2]=tokenize (split pipeline),
 * [3]=stats (segment DC fixup, fused pipeline), [4]=tables, [5]=pack
 * (segment bits + offsets + bit packing), [6]=emit (JFIF assembly),
 * [7]=whole encode */
#define MIJ_NSTAGES 8
int mij_batch_set_timing(mij_batch *b, int on);
int mij_batch_stage_ms(mij_batch *b, float *ms, int n);
/* the same for each of the last `steps` encodes (<= 64) issued while timing
 * was on, oldest first: ms[step*MIJ_NSTAGES + stage]; returns the count filled */
int mij_batch_stage_history(mij_batch *b, float *ms, int steps);
/* symbol tokens K1 emitted for the last encode of nframes frames (4 bytes
 * each; used for the bandwidth accounting of the fused kernel) */
unsigned long long mij_batch_token_count(mij_batch *b, int nframes);
/* {w, h, 8x8 blocks per frame, segments per frame, K1 tiles per frame,
 *  the pack kernel's LDS window in words at the batch's quality}: the first n */
int mij_batch_geometry(mij_batch *b, long long *out, int n);
/* FP64 fix-ups since creation: blocks re-encoded by the fix-up kernel after
 * K1 (split pipeline) plus coefficients replayed in place (fused pipeline) */
unsigned long long mij_batch_replays(mij_batch *b);
/* the batch's hipStream_t, as an opaque pointer */
void *mij_batch_stream(mij_batch *b);
/* Enqueue the batch's work on the caller's stream (null: its own again).
 * Work enqueued after the switch runs after the work enqueued before it (an
 * event on the old stream).  The root's assembler runs its assembly on the
 * band batch's stream this way (sharding.encode_banded_dev), so the band's
 * word move, the assembly and the next step's K1 follow each other in one
 * queue instead of through cross-queue waits (~13 us each on config 4).
 * Switch back (null) before destroying either batch. */
int mij_batch_set_stream(mij_batch *b, void *stream);

/* ---- region batches: many areas of one frame -----
 * The reference's workload (main.c:142-155): the change detector returns up
 * to 100 rectangles of a frame and each is encoded on its own with
 * rgb_to_dct / init_huffman / write_jpg.  A region batch does all of them in
 * one launch sequence: the batch is created with the largest region's size
 * (the canvas) and slot i holds region i, w_i x h_i, at the top-left of its
 * slot.  Each region gets its own tables and JFIF (SOF0 = w_i x h_i); the
 * bytes are those of the three drop-in calls on that region. */
/* per-frame sizes of the next encodes (multiples of 16, at most the batch
 * geometry); wh = {w0, h0, w1, h1, ...}; NULL restores the batch geometry.
 * A full-frame mij_batch_upload / mij_batch_set_input also restores it: call
 * this after uploading when the uploaded frames are smaller than the canvas. */
int mij_batch_set_frame_dims(mij_batch *b, const int *wh, int nframes);
/* regions of a device-resident BGR frame (rows pitch bytes apart) into
 * slots 0..n-1 (one gather launch) and their sizes as the frame dims */
int mij_batch_gather_regions(mij_batch *b, const void *d_frame, long long pitch,
                             int frame_w, int frame_h, const area_t *regions, int n);
/* the same from a host frame of stride_px pixels per row (uploaded once) */
int mij_batch_upload_regions(mij_batch *b, const uint8_t *bgr, int stride_px, int frame_h,
                             const area_t *regions, int n);
/* one call: every region of a host BGR frame to its own JPEG; the n streams
 * are written back to back into out (cap bytes), their lengths into lens */
int mij_encode_regions(const uint8_t *bgr, int stride_px, int frame_h, const area_t *regions,
                       int n, int quality, uint8_t *out, size_t cap, size_t *lens);

/* ---- PPM ingest -----------------------------------
 * Header rules of the reference's reader, utils/original.c:294-365, kept
 * exactly: "P6" then a newline straight after it; then lines up to the first
 * one that does not start with '#' (comment lines, :303-316), which must hold
 * "W H" (sscanf "%d %d", :318); W and H multiples of 16 (:324-328); the depth
 * read with fscanf("%d\n") -- which also swallows whitespace bytes that begin
 * the pixel data, so such a file then fails the length check, as in the
 * reference -- must be 255 (:330-337); the bytes left must be exactly 3*W*H
 * (:339-344).  Extra rules where the reference is undefined: a line longer
 * than 1023 bytes or missing its newline is a parse error, W or H <= 0 is
 * rejected.  Errors: MIJ_EIO (open/read), MIJ_EPPM (rules above). */
int mij_ppm_header(const char *path, int *w, int *h, long long *data_offset);
/* pixels of a PPM into dst (rows dst_pitch bytes apart); to_bgr != 0 swaps
 * to the encoder's B, G, R order (what rgb_to_dct / mij_encode expect) */
int mij_ppm_read(const char *path, uint8_t *dst, size_t cap, int dst_pitch, int to_bgr);

/* ---- streaming encoder: PPM files -> .jpg files ----------------------------
 * Frames of one geometry flow through two batches in ping-pong: host threads
 * read chunk k+1 into pinned memory (no channel swap: K1 reads RGB) while the
 * GPU encodes chunk k; each chunk is uploaded, encoded, its lengths fetched,
 * its JPEG bytes copied back and written by host threads, all overlapped with
 * the other batch's chunk.  Output bytes are those of mij_encode /
 * write_jpg for the same image. */
typedef struct mij_stream mij_stream;
mij_stream *mij_stream_create(int device, int width, int height, int chunk_frames,
                              int quality, int host_threads);
void mij_stream_destroy(mij_stream *s);
/* encode n PPM files (all width x height) to out_paths; stops at the first
 * failing file (its index in *failed, -1 if none) */
int mij_stream_encode_files(mij_stream *s, const char *const *in_paths,
                            const char *const *out_paths, int n, int *failed);
/* in-memory variant: n RGB frames (packed rows) -> outs[i] (caps[i] bytes),
 * lengths in lens[i] */
int mij_stream_encode_frames(mij_stream *s, const uint8_t *const *rgb, int n,
                             uint8_t *const *outs, const size_t *caps, size_t *lens);
/* seconds of the last encode_*: {wall, host read, host write, gpu (events),
 * frames, bytes in, bytes out} */
#define MIJ_STREAM_NSTATS 7
int mij_stream_stats(mij_stream *s, double *out, int n);

/* ---- one large frame over several ranks -------
 * Rank r encodes band r -- an MCU-row range [row0, row0 + rows) with rows a
 * multiple of 16 -- of each of n frames as frames 0..n-1 of its own batch
 * (created for width x rows, input pointing at the band's first row).  The
 * caller moves four small things between ranks (sharding.py does it with
 * torch.distributed / RCCL):
 *   1. mij_band_analyze    -> last raw DC per component      [n*3]  all-gather
 *   2. mij_band_histograms(previous band's last DCs, 0 for band 0)
 *                          -> the band's symbol counts       [n*4*257] all-reduce(sum)
 *   3. mij_band_tables(summed counts) -> bits per scan       [n*3]  all-gather, exclusive scan
 *   4. mij_band_pack(global bit offset of the band in each scan)
 *      mij_band_words(frame, comp) -> packed big-endian words; word 0 is
 *      global word offset/32 of that scan (bits before the offset are 0)  gather
 * One rank assembles on a batch of the whole frame: mij_assemble_begin
 * (summed counts -> tables), mij_assemble_words per band and component (OR:
 * neighbouring bands share at most one word), mij_assemble_end(total bits per
 * scan) -> 0xFF stuffing, pads, headers; then mij_batch_output. */
int mij_band_analyze(mij_batch *b, int n, int16_t *last_dc);
int mij_band_histograms(mij_batch *b, int n, const int16_t *prev_dc, uint32_t *hist);
int mij_band_tables(mij_batch *b, int n, const uint32_t *hist, unsigned long long *bits);
int mij_band_pack(mij_batch *b, int n, const unsigned long long *bit_offset,
                  unsigned long long *nwords);
int mij_band_words(mij_batch *b, int frame, int comp, void *dst, size_t cap_words,
                   int dst_on_device);
int mij_assemble_begin(mij_batch *b, int n, const uint32_t *hist);
int mij_assemble_words(mij_batch *b, int frame, int comp, unsigned long long first_word,
                       const void *src, size_t nwords, int src_on_device);
int mij_assemble_end(mij_batch *b, int n, const unsigned long long *total_bits);
/* The same exchange in one call per side (what sharding.encode_banded uses):
 * mij_band_words_all copies every scan's band words of frames 0..n-1, in
 * (frame, comp) order, into one buffer (word counts from mij_band_pack);
 * mij_assemble_pieces ORs pieces of one buffer (the gathered band words of
 * all ranks) into the scans in one launch: piece i = pieces[4i..4i+3] =
 * {frame * 3 + comp, first word in the scan, first word in src, words}.  Both
 * return once the copy is done (src / dst may be reused).
 * mij_assembler_create makes a batch that only assembles (tables, scan
 * buffers, outputs: no input, coefficient or token buffers); use it with
 * mij_assemble_begin / _pieces / _words / _end and the output calls. */
int mij_band_words_all(mij_batch *b, int n, void *dst, size_t cap_words, int dst_on_device);
int mij_assemble_pieces(mij_batch *b, const void *src, size_t src_words, int src_on_device,
                        const unsigned long long *pieces, int npieces);
mij_batch *mij_assembler_create(int device, int width, int height, int max_frames, int quality);

/* The same exchange steps, device-resident: every pointer is device memory
 * and every call only enqueues work on the batch's stream (mij_batch_stream)
 * -- nothing waits for the host, so the caller's collectives (RCCL on that
 * same stream) run between the calls.  Shapes: last/prev int16 [n][4]
 * (component c at [f][c]), hist uint32 [n][4][257],
 * bits uint64 [3n + 1] (a band's bits per (frame, scan), then its word
 * count), allbits uint64 [world][3n + 1] (every band's bits, rank order).
 *   band_analyze_async     K1 over the band; its last raw DCs -> d_last
 *   band_histograms_async  the segments' first DC tokens from the previous
 *                          band's last DCs (d_prev; null for band 0: zeros);
 *                          the band's histograms -> d_hist (sum them over
 *                          the bands)
 *   band_tables_async      tables from the summed histograms; an upper bound
 *                          of the band's words (its histograms weighted by
 *                          the code lengths, +3 per frame) -> *d_bound, so
 *                          the caller can size the word exchange while the
 *                          band packs
 *   band_pack_async        every scan of the band packed from bit 0 -> d_bits
 *   band_words_async       moves those words, (frame, scan) order, to d_dst
 *                          (cap_words long; words beyond it are dropped and
 *                          the root's assembly fails those frames)
 *   assemble_tables_async  (root) the tables from the summed histograms (may
 *                          run while the bands pack)
 *   assemble_async         (root) every band's words shifted to its bit
 *                          position (the sum of the earlier bands' bits) and
 *                          OR-ed into the scans from d_src (band r's words at
 *                          row r, stride_words apart), then the JFIF
 *                          assembly; read the frames with mij_batch_output.
 * Replaces the host protocol's mij_band_analyze / _histograms / _tables /
 * _pack / _words_all and mij_assemble_begin / _pieces / _end. */
int mij_band_analyze_async(mij_batch *b, int n, int16_t *d_last);
int mij_band_histograms_async(mij_batch *b, int n, const int16_t *d_prev, uint32_t *d_hist);
int mij_band_tables_async(mij_batch *b, int n, const uint32_t *d_ghist, uint64_t *d_bound);
int mij_band_pack_async(mij_batch *b, int n, uint64_t *d_bits);
int mij_band_words_async(mij_batch *b, int n, uint32_t *d_dst, size_t cap_words);
int mij_assemble_tables_async(mij_batch *b, int n, const uint32_t *d_ghist);
int mij_assemble_async(mij_batch *b, int n, const uint64_t *d_allbits, int world, const uint32_t *d_src,
                       size_t stride_words);
/* A device-to-host copy of `bytes` on the batch's stream (the word bounds
 * and stuffed totals of the device protocol, read by the host to size the
 * word exchange): ordered after the collectives and launches enqueued on
 * that stream before it, so the caller waits for just those (an event on the
 * batch's stream) and not for a copy queued behind the packing on another
 * stream.  h_dst must be pinned host memory. */
int mij_copy_to_host_async(mij_batch *b, void *h_dst, const void *d_src, size_t bytes);
/* Distributed JFIF emission (the config-4 bands, sharding.encode_banded_dev
 * with emit="bands"): after mij_band_pack_async and the all-gather of every
 * band's d_bits into d_allbits [world][3n + 1], band `rank` stuffs the bytes
 * of the final scans that lie wholly inside it (encoder.c:403-408) into
 * d_dst (cap bytes), frames and scans in order; d_rec [n][3][4] (u64) gets
 * per scan {stuffed bytes, band bits, head bits << 8 | head count, tail bits
 * << 8 | tail count} (head: the <= 7 bits completing the byte the bands
 * before began; tail: the bits after the last whole byte) and *d_total the
 * band's stuffed bytes.  The band's scan words are consumed. */
int mij_band_stuff_async(mij_batch *b, int n, const uint64_t *d_allbits, int world, int rank,
                         uint64_t *d_rec, uint64_t *d_total, uint8_t *d_dst, size_t cap);
/* root, after mij_assemble_tables_async: frames 0..n-1 from every band's
 * records d_allrec [world][n][3][4] and stuffed bytes d_src [world][stride]:
 * headers, the seam bytes between bands (stuffed when 0xFF), the pads
 * (encoder.c:425-432), EOI, the interiors copied into place */
int mij_assemble_stuffed_async(mij_batch *b, int n, const uint64_t *d_allrec, int world,
                               const uint8_t *d_src, size_t stride);

/* ---- diagnostics used by the test-suite -----------------------------------*/
/* 16x16x64 i8 MFMA layout probe: A, B are 64 lanes x 16 int8, D 64 x 4 int32 */
int mij_probe_mfma(const int8_t *A, const int8_t *B, int32_t *D);
/* colour-exception bitmaps as built on the device: 3 x 1024 words; bit
 * (R<<7 | G>>1) of table 0 (Y), (G<<7 | B>>1) of table 1 (Cb, R == G),
 * (G<<7 | R>>1) of table 2 (Cr, B == G); see DESIGN.md */
int mij_colour_lut(uint32_t *out);
/* Tests: runs the coefficient K1 (as mij_batch_dct) on frames 0..n-1 of a
 * plain B, G, R batch through its audit variant and copies out every
 * block's fast-path decisions: masks[(f * nblk + blk) * 4 + g] bit k set =
 * zigzag coefficient 16 g + k straddled a truncation boundary (replayed in
 * FP64), blocks in the batch's coefficient order (Y, Cb, Cr). */
int mij_batch_audit(mij_batch *b, int nframes, uint16_t *masks);
/* Tests: the four optimized tables of frames 0..n-1 built from given counts
 * hist[f][4][257] (DC-Y, AC-Y, DC-C, AC-C; entry 256 is ignored, the
 * reserved count of encoder.c:367 is 1); read them with mij_batch_tables.
 * MIJ_ETABLE when a frame's counts have no valid table (mij_last_message). */
int mij_batch_build_tables(mij_batch *b, int n, const uint32_t *hist);
/* name of the code object target the library was built for ("gfx950") */
const char *mij_build_target(void);

/* ---- change detector (reference main/brain.c) ------
 * The reference's per-frame loop (main.c:136-163) subsamples the camera frame
 * 4x4 (brain.c:16-45), compares it with the stored subsampled frame
 * (brain.c:104-233: weighted colour distance > 600 per subsampled pixel,
 * runs of differing pixels joined into at most 100 areas, enlarged to
 * multiples of 16 in frame pixels) and encodes each area.  Here the
 * subsample and the per-pixel test run as one HIP kernel over a
 * device-resident frame that writes one bit per subsampled pixel; the run
 * joining, which is sequential in the reference and keeps its quirks (see
 * DESIGN.md), runs on the host over the runs of that bit mask. */

/* include/structs.h:20-22 */
typedef struct {
    int beg, end, row, done;
} pair_t;

typedef struct mij_detector mij_detector;
/* frame geometry: width and height multiples of 4 (the reference: 320x240);
 * the stored plane starts as zeros, like main.c:33's static `saved` */
mij_detector *mij_detector_create(int device, int width, int height);
void mij_detector_destroy(mij_detector *d);
/* brain.c:16-45 on a device BGR frame (rows pitch bytes apart, pitch and
 * pointer 4-byte aligned) into the detector's current plane */
int mij_detector_subsample(mij_detector *d, const void *d_frame, long long pitch);
/* brain.c:104-233: current plane vs stored plane -> outs[100], *count */
int mij_detector_compare(mij_detector *d, area_t outs[100], int *count);
/* subsample + compare in one kernel launch (main.c:140-143) */
int mij_detector_step(mij_detector *d, const void *d_frame, long long pitch, area_t outs[100],
                      int *count);
/* the step's kernel alone, asynchronous on the detector's stream (the mask
 * stays on the device; for timing) */
int mij_detector_launch(mij_detector *d, const void *d_frame, long long pitch);
/* brain.c:53-60 / main.c:161: stored plane := current plane (device copy) */
int mij_detector_store(mij_detector *d);
/* host BGR frame (height rows pitch bytes apart; pitch 0 = 3*width) into the
 * detector's frame buffer, same pitch; *d_frame receives its device address */
int mij_detector_upload(mij_detector *d, const uint8_t *bgr, long long pitch, const void **d_frame);
/* plane 0 = current, 1 = stored, in the reference's layout (R, G, B bytes per
 * subsampled pixel, (width/4)*(height/4)*3 bytes): read back / set */
int mij_detector_get_plane(mij_detector *d, int which, uint8_t *rgb);
int mij_detector_set_plane(mij_detector *d, int which, const uint8_t *rgb);
/* the kernel's bit mask of the last compare: one row of `words` 64-bit words
 * per subsampled row (bit x%64 of word x/64 = pixel x differs) */
int mij_detector_mask(mij_detector *d, unsigned long long *dst, size_t cap_words, int *words);
void *mij_detector_stream(mij_detector *d);

/* ---- round-trip verifier ---------------------------
 * The reference has no decoder.  mij_decoder turns baseline JFIF streams of
 * the shape encoder.c:549-644 writes (8-bit, Y 2x2 + Cb + Cr 1x1, three
 * one-component scans, no restarts) back into the encoder's coefficient
 * layout: per component, blocks in raster order, 64 zigzag-ordered
 * quantized coefficients, DC as the coded difference (= rgb_to_dct's
 * output), so encode -> decode can be checked bit-exactly at any size.
 * Entropy decoding runs on the GPU, one lane per 512-bit chunk of every
 * scan, the chunks' entry states found by self-synchronisation. */
typedef struct mij_decoder mij_decoder;
mij_decoder *mij_decoder_create(int device, int max_w, int max_h, int max_frames);
void mij_decoder_destroy(mij_decoder *d);
/* n host streams; synchronous; MIJ_EJPEG names the stream on failure */
int mij_decoder_decode(mij_decoder *d, const uint8_t *const *jpgs, const size_t *lens, int n);
/* frame size and the two DQT tables (zigzag order) of stream `frame` */
int mij_decoder_info(mij_decoder *d, int frame, int *w, int *h, uint8_t dqt[128]);
/* Y[w*h], Cb[w*h/4], Cr[w*h/4] of stream `frame` (host copies) */
int mij_decoder_coefs(mij_decoder *d, int frame, int16_t *Y, int16_t *Cb, int16_t *Cr);
/* self-synchronisation passes the last decode needed */
int mij_decoder_passes(mij_decoder *d);
/* device address of stream `frame`'s planes (Y, then Cb, then Cr) */
void *mij_decoder_device_coefs(mij_decoder *d, int frame);

/* Drop-in entry points of include/brain.h:7-10, on frames of
 * mij_set_input_stride() x mij_set_frame_height() pixels (define.h:3-4,
 * 320x240 by default).  subsample writes the PPM copy to f when f is not
 * NULL (brain.c:22, :29-42).  compare uses differences (2 rows of WIDTH/8
 * runs, main.c:35) as scratch like the reference.  Errors: mij_last_error. */
int mij_set_frame_height(int height);
void subsample(FILE *f, uint8_t *in, uint8_t *out);
void store(uint8_t *in, uint8_t *saved);
uint8_t compare(uint8_t *in, uint8_t *saved, area_t *outs, pair_t (*differences)[]);
void enlargeAdjust(area_t *a);

#ifdef __cplusplus
}
#endif
#endif /* MIJPEG_H */
