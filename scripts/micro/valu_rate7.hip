// scripts/micro/valu_rate7.hip -- gfx950 VALU issue costs, round 5: mixed-precision
// forms (fma_mix, dot2 f16), the conversions, and the integer ops the token K1 uses
// (8 waves per SIMD, 8 independent chains per wave; same harness as valu_rate6)
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
__global__ void k0(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_fma_mix_f32 %0, %0, %1, %0 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %1, %1, %2, %1 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %2, %2, %3, %2 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %3, %3, %4, %3 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %4, %4, %5, %4 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %5, %5, %6, %5 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %6, %6, %7, %6 op_sel_hi:[1,0,0]\nv_fma_mix_f32 %7, %7, %0, %7 op_sel_hi:[1,0,0]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k1(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_fma_mix_f32 %0, %0, %1, %0 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %1, %1, %2, %1 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %2, %2, %3, %2 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %3, %3, %4, %3 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %4, %4, %5, %4 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %5, %5, %6, %5 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %6, %6, %7, %6 op_sel_hi:[0,0,0]\nv_fma_mix_f32 %7, %7, %0, %7 op_sel_hi:[0,0,0]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k2(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_fma_mix_f32 %0, %1, %1, %0 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %1, %2, %2, %1 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %2, %3, %3, %2 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %3, %4, %4, %3 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %4, %5, %5, %4 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %5, %6, %6, %5 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %6, %7, %7, %6 op_sel:[0,1,0] op_sel_hi:[1,1,0]\nv_fma_mix_f32 %7, %0, %0, %7 op_sel:[0,1,0] op_sel_hi:[1,1,0]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k3(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_dot2_f32_f16 %0, %1, %1, %0\nv_dot2_f32_f16 %1, %2, %2, %1\nv_dot2_f32_f16 %2, %3, %3, %2\nv_dot2_f32_f16 %3, %4, %4, %3\nv_dot2_f32_f16 %4, %5, %5, %4\nv_dot2_f32_f16 %5, %6, %6, %5\nv_dot2_f32_f16 %6, %7, %7, %6\nv_dot2_f32_f16 %7, %0, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k4(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_dot2c_f32_f16 %0, %1, %1\nv_dot2c_f32_f16 %1, %2, %2\nv_dot2c_f32_f16 %2, %3, %3\nv_dot2c_f32_f16 %3, %4, %4\nv_dot2c_f32_f16 %4, %5, %5\nv_dot2c_f32_f16 %5, %6, %6\nv_dot2c_f32_f16 %6, %7, %7\nv_dot2c_f32_f16 %7, %0, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k5(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_cvt_f32_f16 %0, %1\nv_cvt_f32_f16 %1, %2\nv_cvt_f32_f16 %2, %3\nv_cvt_f32_f16 %3, %4\nv_cvt_f32_f16 %4, %5\nv_cvt_f32_f16 %5, %6\nv_cvt_f32_f16 %6, %7\nv_cvt_f32_f16 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k6(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_cvt_f32_ubyte1 %0, %1\nv_cvt_f32_ubyte1 %1, %2\nv_cvt_f32_ubyte1 %2, %3\nv_cvt_f32_ubyte1 %3, %4\nv_cvt_f32_ubyte1 %4, %5\nv_cvt_f32_ubyte1 %5, %6\nv_cvt_f32_ubyte1 %6, %7\nv_cvt_f32_ubyte1 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k7(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_pk_fma_f16 %0, %0, %1, %0\nv_pk_fma_f16 %1, %1, %2, %1\nv_pk_fma_f16 %2, %2, %3, %2\nv_pk_fma_f16 %3, %3, %4, %3\nv_pk_fma_f16 %4, %4, %5, %4\nv_pk_fma_f16 %5, %5, %6, %5\nv_pk_fma_f16 %6, %6, %7, %6\nv_pk_fma_f16 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k8(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_dot4_u32_u8 %0, %1, %1, %0\nv_dot4_u32_u8 %1, %2, %2, %1\nv_dot4_u32_u8 %2, %3, %3, %2\nv_dot4_u32_u8 %3, %4, %4, %3\nv_dot4_u32_u8 %4, %5, %5, %4\nv_dot4_u32_u8 %5, %6, %6, %5\nv_dot4_u32_u8 %6, %7, %7, %6\nv_dot4_u32_u8 %7, %0, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k9(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_add3_u32 %0, %0, %1, %0\nv_add3_u32 %1, %1, %2, %1\nv_add3_u32 %2, %2, %3, %2\nv_add3_u32 %3, %3, %4, %3\nv_add3_u32 %4, %4, %5, %4\nv_add3_u32 %5, %5, %6, %5\nv_add3_u32 %6, %6, %7, %6\nv_add3_u32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k10(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_or3_b32 %0, %0, %1, %0\nv_or3_b32 %1, %1, %2, %1\nv_or3_b32 %2, %2, %3, %2\nv_or3_b32 %3, %3, %4, %3\nv_or3_b32 %4, %4, %5, %4\nv_or3_b32 %5, %5, %6, %5\nv_or3_b32 %6, %6, %7, %6\nv_or3_b32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k11(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_xad_u32 %0, %0, %1, %0\nv_xad_u32 %1, %1, %2, %1\nv_xad_u32 %2, %2, %3, %2\nv_xad_u32 %3, %3, %4, %3\nv_xad_u32 %4, %4, %5, %4\nv_xad_u32 %5, %5, %6, %5\nv_xad_u32 %6, %6, %7, %6\nv_xad_u32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k12(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_and_or_b32 %0, %0, %1, %0\nv_and_or_b32 %1, %1, %2, %1\nv_and_or_b32 %2, %2, %3, %2\nv_and_or_b32 %3, %3, %4, %3\nv_and_or_b32 %4, %4, %5, %4\nv_and_or_b32 %5, %5, %6, %5\nv_and_or_b32 %6, %6, %7, %6\nv_and_or_b32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k13(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_ffbl_b32 %0, %1\nv_ffbl_b32 %1, %2\nv_ffbl_b32 %2, %3\nv_ffbl_b32 %3, %4\nv_ffbl_b32 %4, %5\nv_ffbl_b32 %5, %6\nv_ffbl_b32 %6, %7\nv_ffbl_b32 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k14(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %2, %1 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %3, %2 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %4, %3 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %5, %4 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %6, %5 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %7, %6 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %0, %7 row_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k15(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %5 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %6 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %7 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k16(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_pk_add_f32 %0, %0, %0\nv_pk_add_f32 %1, %1, %1\nv_pk_add_f32 %2, %2, %2\nv_pk_add_f32 %3, %3, %3\nv_pk_add_f32 %4, %4, %4\nv_pk_add_f32 %5, %5, %5\nv_pk_add_f32 %6, %6, %6\nv_pk_add_f32 %7, %7, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k17(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_pk_mul_f32 %0, %0, %0\nv_pk_mul_f32 %1, %1, %1\nv_pk_mul_f32 %2, %2, %2\nv_pk_mul_f32 %3, %3, %3\nv_pk_mul_f32 %4, %4, %4\nv_pk_mul_f32 %5, %5, %5\nv_pk_mul_f32 %6, %6, %6\nv_pk_mul_f32 %7, %7, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k18(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_cvt_pk_u8_f32 %0, %1, 1, %0\nv_cvt_pk_u8_f32 %1, %2, 1, %1\nv_cvt_pk_u8_f32 %2, %3, 1, %2\nv_cvt_pk_u8_f32 %3, %4, 1, %3\nv_cvt_pk_u8_f32 %4, %5, 1, %4\nv_cvt_pk_u8_f32 %5, %6, 1, %5\nv_cvt_pk_u8_f32 %6, %7, 1, %6\nv_cvt_pk_u8_f32 %7, %0, 1, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k19(unsigned *out, int iters) {
  unsigned long long a[8];
  for (int j = 0; j < 8; j++) a[j] = threadIdx.x + j;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_lshlrev_b64 %0, 7, %0\nv_lshlrev_b64 %1, 7, %1\nv_lshlrev_b64 %2, 7, %2\nv_lshlrev_b64 %3, 7, %3\nv_lshlrev_b64 %4, 7, %4\nv_lshlrev_b64 %5, 7, %5\nv_lshlrev_b64 %6, 7, %6\nv_lshlrev_b64 %7, 7, %7\n") : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) :: "vcc");
  unsigned long long x = 0; for (int j = 0; j < 8; j++) x ^= a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)x;
}
__global__ void k20(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_bfe_u32 %0, %1, 3, 5\nv_bfe_u32 %1, %2, 3, 5\nv_bfe_u32 %2, %3, 3, 5\nv_bfe_u32 %3, %4, 3, 5\nv_bfe_u32 %4, %5, 3, 5\nv_bfe_u32 %5, %6, 3, 5\nv_bfe_u32 %6, %7, 3, 5\nv_bfe_u32 %7, %0, 3, 5\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k21(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_cmp_ne_u32_e32 vcc, %0, %1\nv_cmp_ne_u32_e32 vcc, %1, %2\nv_cmp_ne_u32_e32 vcc, %2, %3\nv_cmp_ne_u32_e32 vcc, %3, %4\nv_cmp_ne_u32_e32 vcc, %4, %5\nv_cmp_ne_u32_e32 vcc, %5, %6\nv_cmp_ne_u32_e32 vcc, %6, %7\nv_cmp_ne_u32_e32 vcc, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static void run(const char *name, void (*k)(unsigned *, int), unsigned *buf) {
  const int grid = 256 * 8, block = 256, iters = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, 10);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double per_simd = (double)grid * 4 * iters * 64 / 1024;  // wave-instructions per SIMD
  printf("%-20s %.3f ms  wave-cycles/instr @2.4GHz = %.2f\n", name, ms, ms * 1e-3 * 2.4e9 / per_simd);
}
int main() {
  unsigned *buf;
  (void)hipMalloc(&buf, 256 * 8 * 256 * 4);
  run("fma_mix_f16src", k0, buf);
  run("fma_mix_f32all", k1, buf);
  run("fma_mix_2f16", k2, buf);
  run("dot2_f32_f16", k3, buf);
  run("dot2c_f32_f16", k4, buf);
  run("cvt_f32_f16", k5, buf);
  run("cvt_f32_ubyte1", k6, buf);
  run("pk_fma_f16", k7, buf);
  run("dot4_u32_u8", k8, buf);
  run("add3_u32", k9, buf);
  run("or3_b32", k10, buf);
  run("xad_u32", k11, buf);
  run("and_or_b32", k12, buf);
  run("ffbl_b32", k13, buf);
  run("add_u32_dpp", k14, buf);
  run("mov_b32_dpp", k15, buf);
  run("pk_add_f32_v", k16, buf);
  run("pk_mul_f32_v", k17, buf);
  run("cvt_pk_u8_f32", k18, buf);
  run("lshlrev_b64", k19, buf);
  run("bfe_u32", k20, buf);
  run("cmp_ne_u32", k21, buf);
  return 0;
}
