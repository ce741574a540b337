// fp64 vs fp32 vector issue rate on gfx950 (independent chains, no memory)
#include <hip/hip_runtime.h>
#include <cstdio>
template <typename T>
__global__ void k_fma(T *out, T a, T b, int iters) {
  T x[8];
  for (int i = 0; i < 8; i++) x[i] = (T)(threadIdx.x + i);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = x[i] * a + b;
  }
  T s = 0;
  for (int i = 0; i < 8; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <typename T>
__global__ void k_muladd(T *out, T a, T b, int iters) {  // separate mul and add (reference op order)
  T x[8];
  for (int i = 0; i < 8; i++) x[i] = (T)(threadIdx.x + i);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_elementwise_canonicalize(x[i] * a) + b;
  }
  T s = 0;
  for (int i = 0; i < 8; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cvt(double *out, unsigned v, int iters) {
  double s[8] = {0};
  unsigned u = v + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) { s[i] += (double)((u >> (i * 3)) & 255u); }
    u = u * 1664525u + 1013904223u;
  }
  double t = 0;
  for (int i = 0; i < 8; i++) t += s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
template <typename K, typename... A>
float timeit(K k, int grid, A... args) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, args...);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, args...);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); return ms;
}
int main() {
  const int grid = 256 * 8, iters = 4096;
  void *buf; hipMalloc(&buf, grid * 256 * 8);
  const double ops = (double)grid * 256 * iters * 8;  // lane-ops
  float t;
  t = timeit(k_fma<float>, grid, (float *)buf, 0.999f, 0.5f, iters);
  printf("f32 fma     %.3f ms  %.1f Glane-op/s  wave-instr/SIMD/clk(2.4GHz) %.3f\n", t, ops / t / 1e6, ops / 64 / (t * 1e-3) / 1024 / 2.4e9);
  t = timeit(k_fma<double>, grid, (double *)buf, 0.999, 0.5, iters);
  printf("f64 fma     %.3f ms  %.1f Glane-op/s  wave-instr/SIMD/clk(2.4GHz) %.3f\n", t, ops / t / 1e6, ops / 64 / (t * 1e-3) / 1024 / 2.4e9);
  t = timeit(k_muladd<double>, grid, (double *)buf, 0.999, 0.5, iters);
  printf("f64 mul+add %.3f ms  (2 ops each) %.3f wave-instr/SIMD/clk\n", t, 2 * ops / 64 / (t * 1e-3) / 1024 / 2.4e9);
  t = timeit(k_cvt, grid, (double *)buf, 7u, iters);
  printf("cvt_f64_u32+add+bfe %.3f ms\n", t);
  return 0;
}
