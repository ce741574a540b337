// scripts/micro/fetch_check.hip -- k_tables' lane-partner fetches (DPP /
// permlane swaps), 32- and 64-bit: lane i must read lane i ^ J (i ^ (K - 1))
#include "../../jpeg-encoder-decoder_amd/csrc/mij_kernels.hip"
#include <cstdio>
namespace mij {
__global__ void k_fetch(int *out) {
  const int lane = threadIdx.x;
  const uint32_t v = 1000 + lane;
  const unsigned long long w = (1ull << 40) + lane;
  int o = 0;
  out[64 * o++ + lane] = (int)xor_fetch32<1>(v, lane);
  out[64 * o++ + lane] = (int)xor_fetch32<2>(v, lane);
  out[64 * o++ + lane] = (int)xor_fetch32<4>(v, lane);
  out[64 * o++ + lane] = (int)xor_fetch32<8>(v, lane);
  out[64 * o++ + lane] = (int)xor_fetch32<16>(v, lane);
  out[64 * o++ + lane] = (int)xor_fetch32<32>(v, lane);
  out[64 * o++ + lane] = (int)flip_fetch32<2>(v, lane);
  out[64 * o++ + lane] = (int)flip_fetch32<4>(v, lane);
  out[64 * o++ + lane] = (int)flip_fetch32<8>(v, lane);
  out[64 * o++ + lane] = (int)flip_fetch32<16>(v, lane);
  out[64 * o++ + lane] = (int)flip_fetch32<32>(v, lane);
  out[64 * o++ + lane] = (int)flip_fetch32<64>(v, lane);
  out[64 * o++ + lane] = (int)(xor_fetch<4>(w, lane) - (1ull << 40)) + 1000;
  out[64 * o++ + lane] = (int)(xor_fetch<16>(w, lane) - (1ull << 40)) + 1000;
  out[64 * o++ + lane] = (int)(flip_fetch<64>(w, lane) - (1ull << 40)) + 1000;
}
}  // namespace mij
int main() {
  int *d;
  hipMalloc(&d, 64 * 15 * 4);
  hipLaunchKernelGGL(mij::k_fetch, dim3(1), dim3(64), 0, 0, d);
  int h[64 * 15];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char *nm[15] = {"x1", "x2", "x4", "x8", "x16", "x32", "f2", "f4", "f8", "f16", "f32", "f64", "x4_64", "x16_64", "f64_64"};
  const int want_x[15] = {1, 2, 4, 8, 16, 32, 1, 3, 7, 15, 31, 63, 4, 16, 63};
  for (int o = 0; o < 15; o++) {
    int bad = 0;
    for (int l = 0; l < 64; l++) bad += h[64 * o + l] != 1000 + (l ^ want_x[o]);
    printf("%s bad %d (lane0 %d lane5 %d)\n", nm[o], bad, h[64 * o] - 1000, h[64 * o + 5] - 1000);
  }
  return 0;
}
