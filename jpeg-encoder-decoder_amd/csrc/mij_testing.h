/* mij_testing.h -- test-only entry points of libmijpeg.so.  Not part of the
 * public C ABI (include/mijpeg.h); the test suite binds them by name. */
#ifndef MIJ_TESTING_H
#define MIJ_TESTING_H
#include "mijpeg.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Fault injection: v > 0 makes the next encode's packing start frame 0's luma
 * pack ticket at v, as a stale ticket word would (pack group 0 never runs,
 * the groups after it wait on its look-back word); the frame must fail with
 * MIJ_EHANG within the device-wait bound instead of hanging the launch.
 * Consumed by that encode.  Returns the value armed before (0 once consumed),
 * or -2 on bad arguments. */
int mij_test_stale_ticket(mij_batch *b, int v);
#ifdef __cplusplus
}
#endif
#endif
