// Issue cost of individual VALU instructions on gfx950: 16 independent
// instances per loop iteration, 8 waves per SIMD; cycles measured with
// s_memtime inside each wave and by wall clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP16(X) X X X X X X X X X X X X X X X X
#define KERNEL(name, INSTR)                                                        \
  __global__ void name(unsigned *out, int iters, unsigned long long *cyc) {       \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,  \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                \
    unsigned long long t0 = __builtin_readcyclecounter();                          \
    for (int it = 0; it < iters; it++) {                                           \
      asm volatile(REP16(INSTR) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), \
                   "+v"(a5), "+v"(a6), "+v"(a7));                                  \
    }                                                                              \
    unsigned long long t1 = __builtin_readcyclecounter();                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;                       \
  }
#define KERNEL64(name, INSTR)                                                      \
  __global__ void name(unsigned *out, int iters, unsigned long long *cyc) {       \
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;    \
    unsigned long long t0 = __builtin_readcyclecounter();                          \
    for (int it = 0; it < iters; it++) {                                           \
      asm volatile(REP16(INSTR) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));         \
    }                                                                              \
    unsigned long long t1 = __builtin_readcyclecounter();                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);     \
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;                       \
  }
// each INSTR line issues 8 independent ops (one per register)
#define OPS(op) op " %0, %0, %1\n" op " %1, %1, %2\n" op " %2, %2, %3\n" op " %3, %3, %4\n" \
                op " %4, %4, %5\n" op " %5, %5, %6\n" op " %6, %6, %7\n" op " %7, %7, %0\n"
KERNEL(k_add_u32, OPS("v_add_u32"))
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %2\nv_fma_f32 %1, %1, %2, %3\nv_fma_f32 %2, %2, %3, %4\nv_fma_f32 %3, %3, %4, %5\nv_fma_f32 %4, %4, %5, %6\nv_fma_f32 %5, %5, %6, %7\nv_fma_f32 %6, %6, %7, %0\nv_fma_f32 %7, %7, %0, %1\n")
KERNEL64(k_pk_fma, "v_pk_fma_f32 %0, %0, %1, %2\nv_pk_fma_f32 %1, %1, %2, %3\nv_pk_fma_f32 %2, %2, %3, %0\nv_pk_fma_f32 %3, %3, %0, %1\nv_pk_fma_f32 %0, %0, %1, %2\nv_pk_fma_f32 %1, %1, %2, %3\nv_pk_fma_f32 %2, %2, %3, %0\nv_pk_fma_f32 %3, %3, %0, %1\n")
KERNEL(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %1\nv_cvt_f32_u32 %1, %2\nv_cvt_f32_u32 %2, %3\nv_cvt_f32_u32 %3, %4\nv_cvt_f32_u32 %4, %5\nv_cvt_f32_u32 %5, %6\nv_cvt_f32_u32 %6, %7\nv_cvt_f32_u32 %7, %0\n")
KERNEL(k_cvt_i32_f32, "v_cvt_i32_f32 %0, %1\nv_cvt_i32_f32 %1, %2\nv_cvt_i32_f32 %2, %3\nv_cvt_i32_f32 %3, %4\nv_cvt_i32_f32 %4, %5\nv_cvt_i32_f32 %5, %6\nv_cvt_i32_f32 %6, %7\nv_cvt_i32_f32 %7, %0\n")
KERNEL(k_cvt_ubyte, "v_cvt_f32_ubyte1 %0, %1\nv_cvt_f32_ubyte2 %1, %2\nv_cvt_f32_ubyte1 %2, %3\nv_cvt_f32_ubyte2 %3, %4\nv_cvt_f32_ubyte1 %4, %5\nv_cvt_f32_ubyte2 %5, %6\nv_cvt_f32_ubyte1 %6, %7\nv_cvt_f32_ubyte2 %7, %0\n")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 3, %1\nv_lshl_or_b32 %1, %1, 3, %2\nv_lshl_or_b32 %2, %2, 3, %3\nv_lshl_or_b32 %3, %3, 3, %4\nv_lshl_or_b32 %4, %4, 3, %5\nv_lshl_or_b32 %5, %5, 3, %6\nv_lshl_or_b32 %6, %6, 3, %7\nv_lshl_or_b32 %7, %7, 3, %0\n")
KERNEL(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %2\nv_dot4_u32_u8 %1, %1, %2, %3\nv_dot4_u32_u8 %2, %2, %3, %4\nv_dot4_u32_u8 %3, %3, %4, %5\nv_dot4_u32_u8 %4, %4, %5, %6\nv_dot4_u32_u8 %5, %5, %6, %7\nv_dot4_u32_u8 %6, %6, %7, %0\nv_dot4_u32_u8 %7, %7, %0, %1\n")
KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2\nv_mad_u32_u24 %1, %1, %2, %3\nv_mad_u32_u24 %2, %2, %3, %4\nv_mad_u32_u24 %3, %3, %4, %5\nv_mad_u32_u24 %4, %4, %5, %6\nv_mad_u32_u24 %5, %5, %6, %7\nv_mad_u32_u24 %6, %6, %7, %0\nv_mad_u32_u24 %7, %7, %0, %1\n")
KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %1\nv_mul_hi_u32 %1, %1, %2\nv_mul_hi_u32 %2, %2, %3\nv_mul_hi_u32 %3, %3, %4\nv_mul_hi_u32 %4, %4, %5\nv_mul_hi_u32 %5, %5, %6\nv_mul_hi_u32 %6, %6, %7\nv_mul_hi_u32 %7, %7, %0\n")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2\nv_perm_b32 %1, %1, %2, %3\nv_perm_b32 %2, %2, %3, %4\nv_perm_b32 %3, %3, %4, %5\nv_perm_b32 %4, %4, %5, %6\nv_perm_b32 %5, %5, %6, %7\nv_perm_b32 %6, %6, %7, %0\nv_perm_b32 %7, %7, %0, %1\n")
KERNEL64(k_fma_f64, "v_fma_f64 %0, %0, %1, %2\nv_fma_f64 %1, %1, %2, %3\nv_fma_f64 %2, %2, %3, %0\nv_fma_f64 %3, %3, %0, %1\nv_fma_f64 %0, %0, %1, %2\nv_fma_f64 %1, %1, %2, %3\nv_fma_f64 %2, %2, %3, %0\nv_fma_f64 %3, %3, %0, %1\n")
KERNEL64(k_pk_add, "v_pk_add_f32 %0, %0, %1\nv_pk_add_f32 %1, %1, %2\nv_pk_add_f32 %2, %2, %3\nv_pk_add_f32 %3, %3, %0\nv_pk_add_f32 %0, %0, %1\nv_pk_add_f32 %1, %1, %2\nv_pk_add_f32 %2, %2, %3\nv_pk_add_f32 %3, %3, %0\n")
KERNEL64(k_lshl_u64, "v_lshlrev_b64 %0, 3, %1\nv_lshlrev_b64 %1, 3, %2\nv_lshlrev_b64 %2, 3, %3\nv_lshlrev_b64 %3, 3, %0\nv_lshlrev_b64 %0, 3, %1\nv_lshlrev_b64 %1, 3, %2\nv_lshlrev_b64 %2, 3, %3\nv_lshlrev_b64 %3, 3, %0\n")

template <typename K>
void run(const char *name, K k, unsigned *buf, unsigned long long *cyc, int waves_per_simd) {
  const int iters = 2000, block = 256;
  const int grid = 256 * waves_per_simd;  // 4 waves per block, 256 CUs
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, iters, cyc);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, iters, cyc);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double instr = (double)grid * 4 * iters * 128;  // wave-instructions
  const double per_simd = instr / 1024;
  printf("%-14s w/SIMD=%d  %.3f ms  wave-cycles/instr(wall@2.4GHz)=%.2f  (cyclecounter/instr per wave %.2f)\n",
         name, waves_per_simd, ms, ms * 1e-3 * 2.4e9 / per_simd, (double)c / (iters * 128.0));
}
int main() {
  unsigned *buf; unsigned long long *cyc;
  (void)hipMalloc(&buf, 256 * 8 * 256 * 4 * 4); (void)hipMalloc(&cyc, 8);
  for (int w : {2, 8}) {
    run("add_u32", k_add_u32, buf, cyc, w);
    run("fma_f32", k_fma_f32, buf, cyc, w);
    run("pk_fma_f32", k_pk_fma, buf, cyc, w);
    run("cvt_f32_u32", k_cvt_f32_u32, buf, cyc, w);
    run("cvt_i32_f32", k_cvt_i32_f32, buf, cyc, w);
    run("cvt_f32_ubyte", k_cvt_ubyte, buf, cyc, w);
    run("lshl_or", k_lshl_or, buf, cyc, w);
    run("dot4_u32_u8", k_dot4, buf, cyc, w);
    run("mad_u32_u24", k_mad_u24, buf, cyc, w);
    run("mul_hi_u32", k_mul_hi, buf, cyc, w);
    run("perm_b32", k_perm, buf, cyc, w);
    run("fma_f64", k_fma_f64, buf, cyc, w);
    run("pk_add_f32", k_pk_add, buf, cyc, w);
    run("lshlrev_b64", k_lshl_u64, buf, cyc, w);
  }
  return 0;
}
