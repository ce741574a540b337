// tests/div_check.cpp -- host check of mij_divmagic.h (K1's scalar tile
// division): exhaustive n < 2^24 and a strided sweep to 2^31 for every
// divisor d < 2^12, then sampled large divisors.  Prints the divisor count.
#include <stdio.h>
#include <stdlib.h>
#include "mij_divmagic.h"

static int check(uint32_t d, uint32_t nmax_exh) {
  uint32_t m, s;
  mij::div_magic(d, m, s);
  for (uint32_t n = 0; n < nmax_exh; n++)
    if (mij::div_by(n, m, s) != n / d) { printf("FAIL d=%u n=%u\n", d, n); return 1; }
  for (uint64_t n = nmax_exh; n < (1ull << 31); n += 9973 + (n % 1021))
    if (mij::div_by((uint32_t)n, m, s) != (uint32_t)n / d) { printf("FAIL d=%u n=%llu\n", d, (unsigned long long)n); return 1; }
  const uint32_t top = 0x7FFFFFFFu;
  for (uint32_t n = top - 4096; n != 0 && n <= top; n++)
    if (mij::div_by(n, m, s) != n / d) { printf("FAIL d=%u n=%u\n", d, n); return 1; }
  return 0;
}

int main() {
  int nd = 0;
  for (uint32_t d = 1; d < 4096; d++, nd++)
    if (check(d, d < 64 ? (1u << 22) : (1u << 16))) return 1;
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 2000; i++, nd++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    const uint32_t d = (uint32_t)(x % 0x7FFFFFFFull) + 1;
    if (check(d, 1u << 12)) return 1;
  }
  printf("ok %d divisors\n", nd);
  return 0;
}
