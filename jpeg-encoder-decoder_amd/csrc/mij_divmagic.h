// mij_divmagic.h -- division by a run-time constant as a multiply-high:
// K1 turns its tile index into (frame, tile row, tile column) per tile on
// the scalar unit (mij_internal.h Geom::tpf_m/tx_m).  Plain C++ so that
// tests/div_check.cpp can check it on the host.
#pragma once
#include <stdint.h>
#ifndef __host__
#define __host__
#define __device__
#endif

namespace mij {

// s = the smallest value with 2^s >= d, m = floor(2^(32+s) / d) + 1 - 2^32:
// (umulhi(n, m) + n) >> s == n / d for 0 <= n < 2^31 and 1 <= d < 2^31
// (the round-up method: M = m + 2^32 = ceil(2^(32+s) / d) errs by at most
// 2^s / d < 2 in d M - 2^(32+s), exact for every n < 2^32; n < 2^31 keeps the
// 32-bit sum from overflowing).  tests/test_abi.py::test_division_magic.
inline void div_magic(uint32_t d, uint32_t &m, uint32_t &s) {
  uint32_t k = 0;
  while ((1ull << k) < d) k++;
  s = k;
  m = (uint32_t)(((1ull << (32 + k)) / d) + 1 - (1ull << 32));
}
__host__ __device__ inline uint32_t div_by(uint32_t n, uint32_t m, uint32_t s) {
#ifdef __HIP_DEVICE_COMPILE__
  return (__umulhi(n, m) + n) >> s;
#else
  return ((uint32_t)(((unsigned long long)n * m) >> 32) + n) >> s;
#endif
}

}  // namespace mij
