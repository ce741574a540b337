/* tests/colour_check.c -- exhaustive machine check of K1's fp32 colour rules
 *  over all 2^24 (B, G, R) colours.
 *
 * Restates bit for bit what convert4 (csrc/mij_kernels.hip) computes per
 * pixel -- byte -> fp32, dr = R - G, db = B - G, then per channel a two-fma
 * chain and one rounding add (v_pk_fma_f32 / v_pk_add_f32 are per element
 * IEEE fp32 operations with round-to-nearest-even) -- and compares with the
 * exact values of encoder.c:133-135 in integer arithmetic:
 *   Y  = (299 R + 587 G + 114 B) / 1000
 *   Cb = 128 + (500000 B - 168736 R - 331264 G) / 10^6
 *   Cr = 128 + (500000 R - 418688 G -  81312 B) / 10^6
 * Asserted for every colour:
 *   Y : bits(fl(Yc + 12288)) = 0x46400000 + 1024 floor(Y) + j with j = 0
 *       exactly when Y is an integer (so floor(Y) = bits 10-17 and the
 *       integer-point flag is "low 10 bits zero");
 *   Cb/Cr: bits(fl(c + 1.5 2^23)) - 0x4B400000 = floor(exact) (the -0.5 +
 *       2^-16 bias in CH_BIAS turns the rounding into a floor; at exact
 *       integers it gives the integer itself).
 * The reference's own FP64 evaluation differs from these floors only at
 * integer points (the colour-exception bitmaps, tested on the GPU against
 * tests/golden/colour_exceptions.npz).
 * Prints one JSON line; exit status 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

static long long floordiv(long long a, long long b) {
  long long q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
  return q;
}

int main(void) {
  const float CH_BIAS = 127.5f + 0x1p-16f, MAGIC = 12582912.0f, YMAGIC = 12288.0f;
  long long bad_y = 0, bad_flag = 0, bad_cb = 0, bad_cr = 0, y_int = 0, cb_int = 0, cr_int = 0;
  for (int R = 0; R < 256; R++)
    for (int G = 0; G < 256; G++)
      for (int B = 0; B < 256; B++) {
        const float fr = (float)R, fg = (float)G, fb = (float)B;
        const float dr = fr - fg, db = fb - fg;
        const float yc = fmaf(0.114f, db, fmaf(0.299f, dr, fg));
        const uint32_t yb = fbits(yc + YMAGIC);
        const long long S = 299LL * R + 587LL * G + 114LL * B;
        const int yint = S % 1000 == 0;
        y_int += yint;
        if (((yb >> 10) & 0xFFu) != (uint32_t)(S / 1000) || (yb >> 18) != (0x46400000u >> 18)) bad_y++;
        if (((yb & 0x3FFu) == 0) != yint) bad_flag++;
        const float cb = fmaf(-0.168736f, dr, fmaf(0.5f, db, CH_BIAS)) + MAGIC;
        const float cr = fmaf(-0.081312f, db, fmaf(0.5f, dr, CH_BIAS)) + MAGIC;
        const long long ncb = 128000000LL + 500000LL * B - 168736LL * R - 331264LL * G;
        const long long ncr = 128000000LL + 500000LL * R - 418688LL * G - 81312LL * B;
        cb_int += ncb % 1000000 == 0;
        cr_int += ncr % 1000000 == 0;
        if ((long long)(fbits(cb) - 0x4B400000u) != floordiv(ncb, 1000000)) bad_cb++;
        if ((long long)(fbits(cr) - 0x4B400000u) != floordiv(ncr, 1000000)) bad_cr++;
      }
  printf("{\"colours\": %d, \"bad_y\": %lld, \"bad_y_flag\": %lld, \"bad_cb\": %lld, \"bad_cr\": %lld, "
         "\"y_integer_points\": %lld, \"cb_integer_points\": %lld, \"cr_integer_points\": %lld}\n",
         1 << 24, bad_y, bad_flag, bad_cb, bad_cr, y_int, cb_int, cr_int);
  return (bad_y | bad_flag | bad_cb | bad_cr) ? 1 : 0;
}
