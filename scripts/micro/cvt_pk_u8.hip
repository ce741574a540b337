// scripts/micro/cvt_pk_u8.hip -- semantics probe: does v_cvt_pk_u8_f32 truncate
// or round, and does it clamp?  hipcc --offload-arch=gfx950 -o /tmp/cvt cvt_pk_u8.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float *in, unsigned *out, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  unsigned r;
  asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, 0" : "=v"(r) : "v"(in[i]));
  out[i] = r;
}
int main() {
  const float v[] = {0.0f, 0.4f, 0.5f, 0.6f, 1.5f, 1.7f, 2.5f, 3.49f, 3.5f, 254.99f, 255.4f, 255.6f, 256.2f, -0.3f, -1.0f, 17.9999f};
  const int n = sizeof(v) / sizeof(v[0]);
  float *d_in; unsigned *d_out; unsigned h[64];
  hipMalloc(&d_in, sizeof v); hipMalloc(&d_out, sizeof(unsigned) * n);
  hipMemcpy(d_in, v, sizeof v, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d_in, d_out, n);
  hipMemcpy(h, d_out, sizeof(unsigned) * n, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; i++) printf("%g -> %u\n", v[i], h[i]);
  return 0;
}
