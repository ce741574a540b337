// scripts/micro/mfma_overlap.hip -- does an i8 MFMA (v_mfma_i32_16x16x64_i8)
// take VALU issue cycles from the waves beside it?  3 waves per SIMD (the K1
// occupancy); per wave a loop of fast VALU (v_add_f32 chains) and/or MFMAs on
// independent accumulators.  If VALU and MFMA overlap, mix ~ max(valu, mfma);
// if the MFMA blocks VALU issue, mix ~ valu + mfma.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
#define V8 "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
template <int NV, int NM>
__global__ __launch_bounds__(256) void k(int *out, int iters) {
  float f0 = threadIdx.x, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
  const float inc = 1e-7f * (float)(threadIdx.x & 1);
  v4i a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
  v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
      for (int v = 0; v < NV; v++)
        asm volatile(V8 : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(inc));
      if (NM > 0) {
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
        if (NM > 1) c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
        if (NM > 2) c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
        if (NM > 3) c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
      }
    }
  }
  v4i s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3] + (int)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
}
template <int NV, int NM>
static void run(const char *name, int *buf) {
  // 256 CUs x 3 workgroups of 256 threads = 3 waves per SIMD
  const int grid = 256 * 3, block = 256, iters = 4000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k<NV, NM>), dim3(grid), dim3(block), 0, 0, buf, 10);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k<NV, NM>), dim3(grid), dim3(block), 0, 0, buf, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  // per wave-iteration-step: NV*8 VALU + NM MFMA; 3 waves per SIMD
  const double steps = (double)iters * 4;
  printf("%-28s %.3f ms  SIMD-cycles per step @2.4GHz (3 waves) = %.1f\n", name, ms, ms * 1e-3 * 2.4e9 / steps);
}
int main() {
  int *buf;
  (void)hipMalloc(&buf, 256 * 3 * 256 * 4);
  run<1, 0>("valu 8", buf);
  run<2, 0>("valu 16", buf);
  run<4, 0>("valu 32", buf);
  run<0, 1>("mfma 1", buf);
  run<0, 2>("mfma 2", buf);
  run<0, 4>("mfma 4", buf);
  run<1, 1>("valu 8 + mfma 1", buf);
  run<2, 1>("valu 16 + mfma 1", buf);
  run<4, 1>("valu 32 + mfma 1", buf);
  run<2, 2>("valu 16 + mfma 2", buf);
  run<4, 2>("valu 32 + mfma 2", buf);
  run<4, 4>("valu 32 + mfma 4", buf);
  return 0;
}
