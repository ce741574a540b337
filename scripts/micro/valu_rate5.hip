// scripts/micro/valu_rate5.hip -- gfx950 VALU issue costs: 64-bit shifts and others (made by gen5.py)
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
__global__ void k0(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshlrev_b64 %0, 7, %0\nv_lshlrev_b64 %1, 7, %1\nv_lshlrev_b64 %2, 7, %2\nv_lshlrev_b64 %3, 7, %3\nv_lshlrev_b64 %0, 7, %0\nv_lshlrev_b64 %1, 7, %1\nv_lshlrev_b64 %2, 7, %2\nv_lshlrev_b64 %3, 7, %3\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
__global__ void k1(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshl_add_u64 %0, %0, 2, %1\nv_lshl_add_u64 %1, %1, 2, %2\nv_lshl_add_u64 %2, %2, 2, %3\nv_lshl_add_u64 %3, %3, 2, %0\nv_lshl_add_u64 %0, %0, 2, %1\nv_lshl_add_u64 %1, %1, 2, %2\nv_lshl_add_u64 %2, %2, 2, %3\nv_lshl_add_u64 %3, %3, 2, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
__global__ void k2(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshl_add_u64 %0, %0, 4, %1\nv_lshl_add_u64 %1, %1, 4, %2\nv_lshl_add_u64 %2, %2, 4, %3\nv_lshl_add_u64 %3, %3, 4, %0\nv_lshl_add_u64 %0, %0, 4, %1\nv_lshl_add_u64 %1, %1, 4, %2\nv_lshl_add_u64 %2, %2, 4, %3\nv_lshl_add_u64 %3, %3, 4, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
__global__ void k3(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshrrev_b64 %0, 7, %0\nv_lshrrev_b64 %1, 7, %1\nv_lshrrev_b64 %2, 7, %2\nv_lshrrev_b64 %3, 7, %3\nv_lshrrev_b64 %0, 7, %0\nv_lshrrev_b64 %1, 7, %1\nv_lshrrev_b64 %2, 7, %2\nv_lshrrev_b64 %3, 7, %3\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
__global__ void k4(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_add_u32 %0, %0, %1\nv_add_u32 %1, %1, %2\nv_add_u32 %2, %2, %3\nv_add_u32 %3, %3, %4\nv_add_u32 %4, %4, %5\nv_add_u32 %5, %5, %6\nv_add_u32 %6, %6, %7\nv_add_u32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k5(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_and_or_b32 %0, %0, 63, %1\nv_and_or_b32 %1, %1, 63, %2\nv_and_or_b32 %2, %2, 63, %3\nv_and_or_b32 %3, %3, 63, %4\nv_and_or_b32 %4, %4, 63, %5\nv_and_or_b32 %5, %5, 63, %6\nv_and_or_b32 %6, %6, 63, %7\nv_and_or_b32 %7, %7, 63, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k6(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_or3_b32 %0, %0, %1, 1\nv_or3_b32 %1, %1, %2, 1\nv_or3_b32 %2, %2, %3, 1\nv_or3_b32 %3, %3, %4, 1\nv_or3_b32 %4, %4, %5, 1\nv_or3_b32 %5, %5, %6, 1\nv_or3_b32 %6, %6, %7, 1\nv_or3_b32 %7, %7, %0, 1\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k7(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_dot4_i32_i8 %0, %0, %1, %0\nv_dot4_i32_i8 %1, %1, %2, %1\nv_dot4_i32_i8 %2, %2, %3, %2\nv_dot4_i32_i8 %3, %3, %4, %3\nv_dot4_i32_i8 %4, %4, %5, %4\nv_dot4_i32_i8 %5, %5, %6, %5\nv_dot4_i32_i8 %6, %6, %7, %6\nv_dot4_i32_i8 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k8(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_dot4_u32_u8 %0, %0, %1, %0\nv_dot4_u32_u8 %1, %1, %2, %1\nv_dot4_u32_u8 %2, %2, %3, %2\nv_dot4_u32_u8 %3, %3, %4, %3\nv_dot4_u32_u8 %4, %4, %5, %4\nv_dot4_u32_u8 %5, %5, %6, %5\nv_dot4_u32_u8 %6, %6, %7, %6\nv_dot4_u32_u8 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k9(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mul_hi_u32_u24 %0, %0, %1\nv_mul_hi_u32_u24 %1, %1, %2\nv_mul_hi_u32_u24 %2, %2, %3\nv_mul_hi_u32_u24 %3, %3, %4\nv_mul_hi_u32_u24 %4, %4, %5\nv_mul_hi_u32_u24 %5, %5, %6\nv_mul_hi_u32_u24 %6, %6, %7\nv_mul_hi_u32_u24 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k10(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mul_lo_u32 %0, %0, %1\nv_mul_lo_u32 %1, %1, %2\nv_mul_lo_u32 %2, %2, %3\nv_mul_lo_u32 %3, %3, %4\nv_mul_lo_u32 %4, %4, %5\nv_mul_lo_u32 %5, %5, %6\nv_mul_lo_u32 %6, %6, %7\nv_mul_lo_u32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k11(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_alignbyte_b32 %0, %0, %1, 2\nv_alignbyte_b32 %1, %1, %2, 2\nv_alignbyte_b32 %2, %2, %3, 2\nv_alignbyte_b32 %3, %3, %4, 2\nv_alignbyte_b32 %4, %4, %5, 2\nv_alignbyte_b32 %5, %5, %6, 2\nv_alignbyte_b32 %6, %6, %7, 2\nv_alignbyte_b32 %7, %7, %0, 2\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k12(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]\nv_pk_mov_b32 %1, %1, %2 op_sel:[1,0]\nv_pk_mov_b32 %2, %2, %3 op_sel:[1,0]\nv_pk_mov_b32 %3, %3, %0 op_sel:[1,0]\nv_pk_mov_b32 %0, %0, %1 op_sel:[1,0]\nv_pk_mov_b32 %1, %1, %2 op_sel:[1,0]\nv_pk_mov_b32 %2, %2, %3 op_sel:[1,0]\nv_pk_mov_b32 %3, %3, %0 op_sel:[1,0]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
__global__ void k13(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mov_b64 %0, %1\nv_mov_b64 %1, %2\nv_mov_b64 %2, %3\nv_mov_b64 %3, %0\nv_mov_b64 %0, %1\nv_mov_b64 %1, %2\nv_mov_b64 %2, %3\nv_mov_b64 %3, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
__global__ void k14(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_sub_u32 %0, %0, %1\nv_sub_u32 %1, %1, %2\nv_sub_u32 %2, %2, %3\nv_sub_u32 %3, %3, %4\nv_sub_u32 %4, %4, %5\nv_sub_u32 %5, %5, %6\nv_sub_u32 %6, %6, %7\nv_sub_u32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k15(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshrrev_b32 %0, %1, %0\nv_lshrrev_b32 %1, %2, %1\nv_lshrrev_b32 %2, %3, %2\nv_lshrrev_b32 %3, %4, %3\nv_lshrrev_b32 %4, %5, %4\nv_lshrrev_b32 %5, %6, %5\nv_lshrrev_b32 %6, %7, %6\nv_lshrrev_b32 %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k16(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_ashrrev_i32 %0, %1, %0\nv_ashrrev_i32 %1, %2, %1\nv_ashrrev_i32 %2, %3, %2\nv_ashrrev_i32 %3, %4, %3\nv_ashrrev_i32 %4, %5, %4\nv_ashrrev_i32 %5, %6, %5\nv_ashrrev_i32 %6, %7, %6\nv_ashrrev_i32 %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k17(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_add_f32 %0, %0, %1\nv_add_f32 %1, %1, %2\nv_add_f32 %2, %2, %3\nv_add_f32 %3, %3, %4\nv_add_f32 %4, %4, %5\nv_add_f32 %5, %5, %6\nv_add_f32 %6, %6, %7\nv_add_f32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k18(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cvt_f32_ubyte1 %0, %1\nv_cvt_f32_ubyte1 %1, %2\nv_cvt_f32_ubyte1 %2, %3\nv_cvt_f32_ubyte1 %3, %4\nv_cvt_f32_ubyte1 %4, %5\nv_cvt_f32_ubyte1 %5, %6\nv_cvt_f32_ubyte1 %6, %7\nv_cvt_f32_ubyte1 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k19(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_sad_u8 %0, %0, %1, %0\nv_sad_u8 %1, %1, %2, %1\nv_sad_u8 %2, %2, %3, %2\nv_sad_u8 %3, %3, %4, %3\nv_sad_u8 %4, %4, %5, %4\nv_sad_u8 %5, %5, %6, %5\nv_sad_u8 %6, %6, %7, %6\nv_sad_u8 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k20(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_bitop3_b32 %0, %0, %1, 64 bitop3:0x6c\nv_bitop3_b32 %1, %1, %2, 64 bitop3:0x6c\nv_bitop3_b32 %2, %2, %3, 64 bitop3:0x6c\nv_bitop3_b32 %3, %3, %4, 64 bitop3:0x6c\nv_bitop3_b32 %4, %4, %5, 64 bitop3:0x6c\nv_bitop3_b32 %5, %5, %6, 64 bitop3:0x6c\nv_bitop3_b32 %6, %6, %7, 64 bitop3:0x6c\nv_bitop3_b32 %7, %7, %0, 64 bitop3:0x6c\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k21(unsigned *out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_add_u16 %0, %0, %1\nv_pk_add_u16 %1, %1, %2\nv_pk_add_u16 %2, %2, %3\nv_pk_add_u16 %3, %3, %4\nv_pk_add_u16 %4, %4, %5\nv_pk_add_u16 %5, %5, %6\nv_pk_add_u16 %6, %6, %7\nv_pk_add_u16 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k22(unsigned *out, int iters) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; unsigned c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mad_u64_u32 %0, s[4:5], %5, 7, %0\nv_mad_u64_u32 %1, s[4:5], %6, 7, %1\nv_mad_u64_u32 %2, s[4:5], %7, 7, %2\nv_mad_u64_u32 %3, s[4:5], %4, 7, %3\nv_mad_u64_u32 %0, s[4:5], %5, 7, %0\nv_mad_u64_u32 %1, s[4:5], %6, 7, %1\nv_mad_u64_u32 %2, s[4:5], %7, 7, %2\nv_mad_u64_u32 %3, s[4:5], %4, 7, %3\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) :: "vcc", "s4", "s5");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3) ^ c0 ^ c1 ^ c2 ^ c3;
}
template <typename K>
void run(const char *name, K k, unsigned *buf) {
  const int iters = 1000, block = 256, grid = 256 * 8;
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
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
  run("lshlrev_b64_7", k0, buf);
  run("lshl_add_u64_2", k1, buf);
  run("lshl_add_u64_4", k2, buf);
  run("lshrrev_b64_7", k3, buf);
  run("add_u32_vv", k4, buf);
  run("and_or_b32", k5, buf);
  run("or3_b32", k6, buf);
  run("dot4_i32_i8", k7, buf);
  run("dot4_u32_u8", k8, buf);
  run("mul_hi_u32_u24", k9, buf);
  run("mul_lo_u32", k10, buf);
  run("alignbyte_k2", k11, buf);
  run("pk_mov_b32", k12, buf);
  run("mov_b64", k13, buf);
  run("sub_u32_vv", k14, buf);
  run("lshrrev_b32_vv", k15, buf);
  run("ashrrev_i32_vv", k16, buf);
  run("add_f32_vv", k17, buf);
  run("cvt_f32_ubyte1", k18, buf);
  run("sad_u8", k19, buf);
  run("bitop3_vv", k20, buf);
  run("pk_add_u16", k21, buf);
  run("mad_u64_u32", k22, buf);
  return 0;
}
