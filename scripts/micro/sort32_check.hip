// scripts/micro/sort32_check.hip -- the 32- and 64-bit register bitonic sorts
// of k_tables against std::sort on random keys (one wave, 256 keys)
#include "../../jpeg-encoder-decoder_amd/csrc/mij_kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
namespace mij {
__global__ void k_sort_check(const uint32_t *in, uint32_t *out32, unsigned long long *out64) {
  const int lane = threadIdx.x;
  uint32_t k32[4];
  unsigned long long k[4];
  for (int r = 0; r < 4; r++) {
    k32[r] = in[lane + 64 * r];
    k[r] = k32[r] == ~0u ? ~0ull : ((unsigned long long)k32[r] << 20);
  }
  bsort_level32<2>(k32, lane);
  bsort_level<2>(k, lane);
  for (int r = 0; r < 4; r++) {
    out32[lane + 64 * r] = k32[r];
    out64[lane + 64 * r] = k[r];
  }
}
}  // namespace mij
int main() {
  std::vector<uint32_t> h(256);
  srand(5);
  for (int i = 0; i < 256; i++) h[i] = (rand() % 4) ? (uint32_t)((rand() % 4) << 9 | (256 - i)) : ~0u;
  uint32_t *din, *d32;
  unsigned long long *d64;
  hipMalloc(&din, 1024); hipMalloc(&d32, 1024); hipMalloc(&d64, 2048);
  hipMemcpy(din, h.data(), 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mij::k_sort_check, dim3(1), dim3(64), 0, 0, din, d32, d64);
  std::vector<uint32_t> o32(256);
  std::vector<unsigned long long> o64(256);
  hipMemcpy(o32.data(), d32, 1024, hipMemcpyDeviceToHost);
  hipMemcpy(o64.data(), d64, 2048, hipMemcpyDeviceToHost);
  std::vector<uint32_t> want = h;
  std::sort(want.begin(), want.end());
  int bad32 = 0, bad64 = 0;
  for (int i = 0; i < 256; i++) {
    if (o32[i] != want[i]) { if (bad32 < 5) printf("32: %d got %08x want %08x\n", i, o32[i], want[i]); bad32++; }
    const unsigned long long w = want[i] == ~0u ? ~0ull : ((unsigned long long)want[i] << 20);
    if (o64[i] != w) { if (bad64 < 5) printf("64: %d got %llx want %llx\n", i, o64[i], w); bad64++; }
  }
  printf("bad32 %d bad64 %d\n", bad32, bad64);
  return 0;
}
