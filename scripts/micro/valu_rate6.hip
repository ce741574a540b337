// scripts/micro/valu_rate6.hip -- gfx950 VALU issue costs of the ops the integer-domain
// quantisation uses, with VGPR / SGPR / literal operands (8 waves per SIMD, 8
// independent chains per wave)
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
__global__ void k0(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_sub_u32_e64 %0, %0, %1 clamp\nv_sub_u32_e64 %1, %1, %2 clamp\nv_sub_u32_e64 %2, %2, %3 clamp\nv_sub_u32_e64 %3, %3, %4 clamp\nv_sub_u32_e64 %4, %4, %5 clamp\nv_sub_u32_e64 %5, %5, %6 clamp\nv_sub_u32_e64 %6, %6, %7 clamp\nv_sub_u32_e64 %7, %7, %0 clamp\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k1(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_sub_u32_e64 %0, %0, %1\nv_sub_u32_e64 %1, %1, %2\nv_sub_u32_e64 %2, %2, %3\nv_sub_u32_e64 %3, %3, %4\nv_sub_u32_e64 %4, %4, %5\nv_sub_u32_e64 %5, %5, %6\nv_sub_u32_e64 %6, %6, %7\nv_sub_u32_e64 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k2(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_pk_sub_i16 %0, %0, %1\nv_pk_sub_i16 %1, %1, %2\nv_pk_sub_i16 %2, %2, %3\nv_pk_sub_i16 %3, %3, %4\nv_pk_sub_i16 %4, %4, %5\nv_pk_sub_i16 %5, %5, %6\nv_pk_sub_i16 %6, %6, %7\nv_pk_sub_i16 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k3(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_lshrrev_b32 %0, %1, %0\nv_lshrrev_b32 %1, %2, %1\nv_lshrrev_b32 %2, %3, %2\nv_lshrrev_b32 %3, %4, %3\nv_lshrrev_b32 %4, %5, %4\nv_lshrrev_b32 %5, %6, %5\nv_lshrrev_b32 %6, %7, %6\nv_lshrrev_b32 %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k4(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_xor_b32 %0, 0x12345, %0\nv_xor_b32 %1, 0x12345, %1\nv_xor_b32 %2, 0x12345, %2\nv_xor_b32 %3, 0x12345, %3\nv_xor_b32 %4, 0x12345, %4\nv_xor_b32 %5, 0x12345, %5\nv_xor_b32 %6, 0x12345, %6\nv_xor_b32 %7, 0x12345, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k5(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("s_mov_b32 s4, 0x12345\n" REP8("v_xor_b32 %0, s4, %0\nv_xor_b32 %1, s4, %1\nv_xor_b32 %2, s4, %2\nv_xor_b32 %3, s4, %3\nv_xor_b32 %4, s4, %4\nv_xor_b32 %5, s4, %5\nv_xor_b32 %6, s4, %6\nv_xor_b32 %7, s4, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k6(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_bitop3_b32 %0, %0, %1, %0 bitop3:0xe8\nv_bitop3_b32 %1, %1, %2, %1 bitop3:0xe8\nv_bitop3_b32 %2, %2, %3, %2 bitop3:0xe8\nv_bitop3_b32 %3, %3, %4, %3 bitop3:0xe8\nv_bitop3_b32 %4, %4, %5, %4 bitop3:0xe8\nv_bitop3_b32 %5, %5, %6, %5 bitop3:0xe8\nv_bitop3_b32 %6, %6, %7, %6 bitop3:0xe8\nv_bitop3_b32 %7, %7, %0, %7 bitop3:0xe8\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k7(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("s_mov_b32 s4, 0xffff\n" REP8("v_bitop3_b32 %0, %0, %1, s4 bitop3:0xe8\nv_bitop3_b32 %1, %1, %2, s4 bitop3:0xe8\nv_bitop3_b32 %2, %2, %3, s4 bitop3:0xe8\nv_bitop3_b32 %3, %3, %4, s4 bitop3:0xe8\nv_bitop3_b32 %4, %4, %5, s4 bitop3:0xe8\nv_bitop3_b32 %5, %5, %6, s4 bitop3:0xe8\nv_bitop3_b32 %6, %6, %7, s4 bitop3:0xe8\nv_bitop3_b32 %7, %7, %0, s4 bitop3:0xe8\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k8(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("s_mov_b32 s4, 0x5040100\n" REP8("v_perm_b32 %0, %0, %1, s4\nv_perm_b32 %1, %1, %2, s4\nv_perm_b32 %2, %2, %3, s4\nv_perm_b32 %3, %3, %4, s4\nv_perm_b32 %4, %4, %5, s4\nv_perm_b32 %5, %5, %6, s4\nv_perm_b32 %6, %6, %7, s4\nv_perm_b32 %7, %7, %0, s4\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k9(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_cvt_pk_i16_i32 %0, %0, %1\nv_cvt_pk_i16_i32 %1, %1, %2\nv_cvt_pk_i16_i32 %2, %2, %3\nv_cvt_pk_i16_i32 %3, %3, %4\nv_cvt_pk_i16_i32 %4, %4, %5\nv_cvt_pk_i16_i32 %5, %5, %6\nv_cvt_pk_i16_i32 %6, %6, %7\nv_cvt_pk_i16_i32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k10(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_med3_i32 %0, %0, %1, 0\nv_med3_i32 %1, %1, %2, 0\nv_med3_i32 %2, %2, %3, 0\nv_med3_i32 %3, %3, %4, 0\nv_med3_i32 %4, %4, %5, 0\nv_med3_i32 %5, %5, %6, 0\nv_med3_i32 %6, %6, %7, 0\nv_med3_i32 %7, %7, %0, 0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k11(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_fma_f32 %0, |%0|, %1, 1.0\nv_fma_f32 %1, |%1|, %2, 1.0\nv_fma_f32 %2, |%2|, %3, 1.0\nv_fma_f32 %3, |%3|, %4, 1.0\nv_fma_f32 %4, |%4|, %5, 1.0\nv_fma_f32 %5, |%5|, %6, 1.0\nv_fma_f32 %6, |%6|, %7, 1.0\nv_fma_f32 %7, |%7|, %0, 1.0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k12(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("s_mov_b32 s4, 0x3f800000\n" REP8("v_fma_f32 %0, %0, %1, s4\nv_fma_f32 %1, %1, %2, s4\nv_fma_f32 %2, %2, %3, s4\nv_fma_f32 %3, %3, %4, s4\nv_fma_f32 %4, %4, %5, s4\nv_fma_f32 %5, %5, %6, s4\nv_fma_f32 %6, %6, %7, s4\nv_fma_f32 %7, %7, %0, s4\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k13(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_cvt_f32_i32 %0, %0\nv_cvt_f32_i32 %1, %1\nv_cvt_f32_i32 %2, %2\nv_cvt_f32_i32 %3, %3\nv_cvt_f32_i32 %4, %4\nv_cvt_f32_i32 %5, %5\nv_cvt_f32_i32 %6, %6\nv_cvt_f32_i32 %7, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k14(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_mul_f32 %0, %0, %1\nv_mul_f32 %1, %1, %2\nv_mul_f32 %2, %2, %3\nv_mul_f32 %3, %3, %4\nv_mul_f32 %4, %4, %5\nv_mul_f32 %5, %5, %6\nv_mul_f32 %6, %6, %7\nv_mul_f32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k15(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("s_mov_b32 s4, 3\n" REP8("v_lshrrev_b32 %0, s4, %0\nv_lshrrev_b32 %1, s4, %1\nv_lshrrev_b32 %2, s4, %2\nv_lshrrev_b32 %3, s4, %3\nv_lshrrev_b32 %4, s4, %4\nv_lshrrev_b32 %5, s4, %5\nv_lshrrev_b32 %6, s4, %6\nv_lshrrev_b32 %7, s4, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k16(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_ashrrev_i32 %0, 31, %0\nv_ashrrev_i32 %1, 31, %1\nv_ashrrev_i32 %2, 31, %2\nv_ashrrev_i32 %3, 31, %3\nv_ashrrev_i32 %4, 31, %4\nv_ashrrev_i32 %5, 31, %5\nv_ashrrev_i32 %6, 31, %6\nv_ashrrev_i32 %7, 31, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k17(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_sad_u32 %0, %0, %1, %0\nv_sad_u32 %1, %1, %2, %1\nv_sad_u32 %2, %2, %3, %2\nv_sad_u32 %3, %3, %4, %3\nv_sad_u32 %4, %4, %5, %4\nv_sad_u32 %5, %5, %6, %5\nv_sad_u32 %6, %6, %7, %6\nv_sad_u32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k18(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("s_mov_b32 s4, 3\n" REP8("v_add_u32 %0, s4, %0\nv_add_u32 %1, s4, %1\nv_add_u32 %2, s4, %2\nv_add_u32 %3, s4, %3\nv_add_u32 %4, s4, %4\nv_add_u32 %5, s4, %5\nv_add_u32 %6, s4, %6\nv_add_u32 %7, s4, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k19(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile("" REP8("v_and_b32 %0, 0xff00ff, %0\nv_and_b32 %1, 0xff00ff, %1\nv_and_b32 %2, 0xff00ff, %2\nv_and_b32 %3, 0xff00ff, %3\nv_and_b32 %4, 0xff00ff, %4\nv_and_b32 %5, 0xff00ff, %5\nv_and_b32 %6, 0xff00ff, %6\nv_and_b32 %7, 0xff00ff, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4");
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
  run("sub_u32_clamp", k0, buf);
  run("sub_u32_e64", k1, buf);
  run("pk_sub_i16", k2, buf);
  run("lshrrev_vv", k3, buf);
  run("xor_lit", k4, buf);
  run("xor_sgpr", k5, buf);
  run("bitop3_vvv", k6, buf);
  run("bitop3_vvs", k7, buf);
  run("perm_b32_s", k8, buf);
  run("cvt_pk_i16_i32", k9, buf);
  run("med3_i32", k10, buf);
  run("fma_f32_abs", k11, buf);
  run("fma_f32_vvs", k12, buf);
  run("cvt_f32_i32", k13, buf);
  run("mul_f32", k14, buf);
  run("lshrrev_s", k15, buf);
  run("ashrrev_k", k16, buf);
  run("sad_u32", k17, buf);
  run("add_u32_s", k18, buf);
  run("and_lit", k19, buf);
  return 0;
}
