// mij_host.h -- host-side helpers shared between the translation units of
// libmijpeg.so (mij_api.hip <-> mij_stream.hip).  Not a public header.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "mijpeg.h"

// error state of the C ABI (mij_last_error): set and print like the API does
int mij_fail(int code, const char *fmt, ...);
void mij_clear_error();
// a frame's device error code (mij_internal.h FERR_*) as the C ABI's error,
// naming `what` and the frame
int mij_frame_fail(int ferr, const char *what, int frame);

// asynchronous transfers on the batch's stream (no synchronisation)
// one frame into slot `slot` on the batch stream (or `stream`), for host threads uploading
// the frames of a chunk as each is read: distinct slots may be uploaded from
// different threads at once (only the copy is enqueued: a stream's batches never hold region
// sizes, which mij_batch_upload resets)
int mij_batch_upload_slot_async(mij_batch *b, const uint8_t *host, int slot, void *stream = nullptr);
int mij_batch_lengths_async(mij_batch *b, uint64_t *h_len, int *h_err, int nframes);
int mij_batch_output_async(mij_batch *b, int frame, uint8_t *dst, size_t n);

// drop-in state shared with the detector's drop-in calls (mij_detect.hip)
int mij_drop_stride();   // define.h:3 WIDTH, as set by mij_set_input_stride
int mij_drop_device();   // MIJ_DEVICE or 0
