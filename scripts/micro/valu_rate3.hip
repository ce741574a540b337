// scripts/micro/valu_rate3.hip -- issue cost of candidate VALU forms on gfx950 (generated)
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
__global__ void k0(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k1(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshlrev_b32 %0, %0, %1\nv_lshlrev_b32 %1, %1, %2\nv_lshlrev_b32 %2, %2, %3\nv_lshlrev_b32 %3, %3, %4\nv_lshlrev_b32 %4, %4, %5\nv_lshlrev_b32 %5, %5, %6\nv_lshlrev_b32 %6, %6, %7\nv_lshlrev_b32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k2(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_lshrrev_b32 %0, 7, %0\nv_lshrrev_b32 %1, 7, %1\nv_lshrrev_b32 %2, 7, %2\nv_lshrrev_b32 %3, 7, %3\nv_lshrrev_b32 %4, 7, %4\nv_lshrrev_b32 %5, 7, %5\nv_lshrrev_b32 %6, 7, %6\nv_lshrrev_b32 %7, 7, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k3(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_ashrrev_i32 %0, 7, %0\nv_ashrrev_i32 %1, 7, %1\nv_ashrrev_i32 %2, 7, %2\nv_ashrrev_i32 %3, 7, %3\nv_ashrrev_i32 %4, 7, %4\nv_ashrrev_i32 %5, 7, %5\nv_ashrrev_i32 %6, 7, %6\nv_ashrrev_i32 %7, 7, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k4(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_or_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %1, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %2, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %3, %4, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %4, %5, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %5, %6, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %6, %7, %6 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\nv_or_b32_sdwa %7, %0, %7 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k5(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_sub_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %1, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %2, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %3, %4, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %4, %5, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %5, %6, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %6, %7, %6 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\nv_sub_u32_sdwa %7, %0, %7 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_1\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k6(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cvt_f32_ubyte0 %0, %1\nv_cvt_f32_ubyte0 %1, %2\nv_cvt_f32_ubyte0 %2, %3\nv_cvt_f32_ubyte0 %3, %4\nv_cvt_f32_ubyte0 %4, %5\nv_cvt_f32_ubyte0 %5, %6\nv_cvt_f32_ubyte0 %6, %7\nv_cvt_f32_ubyte0 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k7(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_sub_f32 %0, %0, %1\nv_sub_f32 %1, %1, %2\nv_sub_f32 %2, %2, %3\nv_sub_f32 %3, %3, %4\nv_sub_f32 %4, %4, %5\nv_sub_f32 %5, %5, %6\nv_sub_f32 %6, %6, %7\nv_sub_f32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k8(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_add_f32_e64 %0, |%0|, %1\nv_add_f32_e64 %1, |%1|, %2\nv_add_f32_e64 %2, |%2|, %3\nv_add_f32_e64 %3, |%3|, %4\nv_add_f32_e64 %4, |%4|, %5\nv_add_f32_e64 %5, |%5|, %6\nv_add_f32_e64 %6, |%6|, %7\nv_add_f32_e64 %7, |%7|, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k9(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_max_f32 %0, %0, %1\nv_max_f32 %1, %1, %2\nv_max_f32 %2, %2, %3\nv_max_f32 %3, %3, %4\nv_max_f32 %4, %4, %5\nv_max_f32 %5, %5, %6\nv_max_f32 %6, %6, %7\nv_max_f32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k10(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_min_f32 %0, %0, %1\nv_min_f32 %1, %1, %2\nv_min_f32 %2, %2, %3\nv_min_f32 %3, %3, %4\nv_min_f32 %4, %4, %5\nv_min_f32 %5, %5, %6\nv_min_f32 %6, %6, %7\nv_min_f32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k11(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_max_u32 %0, %0, %1\nv_max_u32 %1, %1, %2\nv_max_u32 %2, %2, %3\nv_max_u32 %3, %3, %4\nv_max_u32 %4, %4, %5\nv_max_u32 %5, %5, %6\nv_max_u32 %6, %6, %7\nv_max_u32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k12(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_bitop3_b32 %0, %0, %1, 64 bitop3:0xf8\nv_bitop3_b32 %1, %1, %2, 64 bitop3:0xf8\nv_bitop3_b32 %2, %2, %3, 64 bitop3:0xf8\nv_bitop3_b32 %3, %3, %4, 64 bitop3:0xf8\nv_bitop3_b32 %4, %4, %5, 64 bitop3:0xf8\nv_bitop3_b32 %5, %5, %6, 64 bitop3:0xf8\nv_bitop3_b32 %6, %6, %7, 64 bitop3:0xf8\nv_bitop3_b32 %7, %7, %0, 64 bitop3:0xf8\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k13(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_and_b32 %0, 0x4b0000ff, %0\nv_and_b32 %1, 0x4b0000ff, %1\nv_and_b32 %2, 0x4b0000ff, %2\nv_and_b32 %3, 0x4b0000ff, %3\nv_and_b32 %4, 0x4b0000ff, %4\nv_and_b32 %5, 0x4b0000ff, %5\nv_and_b32 %6, 0x4b0000ff, %6\nv_and_b32 %7, 0x4b0000ff, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k14(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_fmac_f32 %0, %1, %0\nv_fmac_f32 %1, %2, %1\nv_fmac_f32 %2, %3, %2\nv_fmac_f32 %3, %4, %3\nv_fmac_f32 %4, %5, %4\nv_fmac_f32 %5, %6, %5\nv_fmac_f32 %6, %7, %6\nv_fmac_f32 %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k15(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_fmamk_f32 %0, %0, 0x3e991687, %1\nv_fmamk_f32 %1, %1, 0x3e991687, %2\nv_fmamk_f32 %2, %2, 0x3e991687, %3\nv_fmamk_f32 %3, %3, 0x3e991687, %4\nv_fmamk_f32 %4, %4, 0x3e991687, %5\nv_fmamk_f32 %5, %5, 0x3e991687, %6\nv_fmamk_f32 %6, %6, 0x3e991687, %7\nv_fmamk_f32 %7, %7, 0x3e991687, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k16(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_fma_f16 %0, %0, %1, %0\nv_pk_fma_f16 %1, %1, %2, %1\nv_pk_fma_f16 %2, %2, %3, %2\nv_pk_fma_f16 %3, %3, %4, %3\nv_pk_fma_f16 %4, %4, %5, %4\nv_pk_fma_f16 %5, %5, %6, %5\nv_pk_fma_f16 %6, %6, %7, %6\nv_pk_fma_f16 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k17(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_add_f16 %0, %0, %1\nv_pk_add_f16 %1, %1, %2\nv_pk_add_f16 %2, %2, %3\nv_pk_add_f16 %3, %3, %4\nv_pk_add_f16 %4, %4, %5\nv_pk_add_f16 %5, %5, %6\nv_pk_add_f16 %6, %6, %7\nv_pk_add_f16 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k18(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_dot2_f32_f16 %0, %0, %1, %0\nv_dot2_f32_f16 %1, %1, %2, %1\nv_dot2_f32_f16 %2, %2, %3, %2\nv_dot2_f32_f16 %3, %3, %4, %3\nv_dot2_f32_f16 %4, %4, %5, %4\nv_dot2_f32_f16 %5, %5, %6, %5\nv_dot2_f32_f16 %6, %6, %7, %6\nv_dot2_f32_f16 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k19(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_dot2c_f32_f16 %0, %1, %0\nv_dot2c_f32_f16 %1, %2, %1\nv_dot2c_f32_f16 %2, %3, %2\nv_dot2c_f32_f16 %3, %4, %3\nv_dot2c_f32_f16 %4, %5, %4\nv_dot2c_f32_f16 %5, %6, %5\nv_dot2c_f32_f16 %6, %7, %6\nv_dot2c_f32_f16 %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k20(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_mul_lo_u16 %0, %0, %1\nv_pk_mul_lo_u16 %1, %1, %2\nv_pk_mul_lo_u16 %2, %2, %3\nv_pk_mul_lo_u16 %3, %3, %4\nv_pk_mul_lo_u16 %4, %4, %5\nv_pk_mul_lo_u16 %5, %5, %6\nv_pk_mul_lo_u16 %6, %6, %7\nv_pk_mul_lo_u16 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k21(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_add_u16 %0, %0, %1\nv_pk_add_u16 %1, %1, %2\nv_pk_add_u16 %2, %2, %3\nv_pk_add_u16 %3, %3, %4\nv_pk_add_u16 %4, %4, %5\nv_pk_add_u16 %5, %5, %6\nv_pk_add_u16 %6, %6, %7\nv_pk_add_u16 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k22(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_pk_lshlrev_b16 %0, 7, %0 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %1, 7, %1 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %2, 7, %2 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %3, 7, %3 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %4, 7, %4 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %5, 7, %5 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %6, 7, %6 op_sel_hi:[0,1]\nv_pk_lshlrev_b16 %7, 7, %7 op_sel_hi:[0,1]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k23(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_sad_u32 %0, %0, %1, %0\nv_sad_u32 %1, %1, %2, %1\nv_sad_u32 %2, %2, %3, %2\nv_sad_u32 %3, %3, %4, %3\nv_sad_u32 %4, %4, %5, %4\nv_sad_u32 %5, %5, %6, %5\nv_sad_u32 %6, %6, %7, %6\nv_sad_u32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k24(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cndmask_b32 %0, %0, %1, vcc\nv_cndmask_b32 %1, %1, %2, vcc\nv_cndmask_b32 %2, %2, %3, vcc\nv_cndmask_b32 %3, %3, %4, vcc\nv_cndmask_b32 %4, %4, %5, vcc\nv_cndmask_b32 %5, %5, %6, vcc\nv_cndmask_b32 %6, %6, %7, vcc\nv_cndmask_b32 %7, %7, %0, vcc\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k25(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %5 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %6 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %7 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k26(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %2, %1 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %3, %2 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %4, %3 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %5, %4 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %6, %5 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %7, %6 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %0, %7 row_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k27(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_xad_u32 %0, %0, %1, %0\nv_xad_u32 %1, %1, %2, %1\nv_xad_u32 %2, %2, %3, %2\nv_xad_u32 %3, %3, %4, %3\nv_xad_u32 %4, %4, %5, %4\nv_xad_u32 %5, %5, %6, %5\nv_xad_u32 %6, %6, %7, %6\nv_xad_u32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k28(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_add3_u32 %0, %0, %1, %0\nv_add3_u32 %1, %1, %2, %1\nv_add3_u32 %2, %2, %3, %2\nv_add3_u32 %3, %3, %4, %3\nv_add3_u32 %4, %4, %5, %4\nv_add3_u32 %5, %5, %6, %5\nv_add3_u32 %6, %6, %7, %6\nv_add3_u32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k29(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_bfi_b32 %0, %0, %1, %0\nv_bfi_b32 %1, %1, %2, %1\nv_bfi_b32 %2, %2, %3, %2\nv_bfi_b32 %3, %3, %4, %3\nv_bfi_b32 %4, %4, %5, %4\nv_bfi_b32 %5, %5, %6, %5\nv_bfi_b32 %6, %6, %7, %6\nv_bfi_b32 %7, %7, %0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k30(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cvt_pk_u16_u32 %0, %0, %1\nv_cvt_pk_u16_u32 %1, %1, %2\nv_cvt_pk_u16_u32 %2, %2, %3\nv_cvt_pk_u16_u32 %3, %3, %4\nv_cvt_pk_u16_u32 %4, %4, %5\nv_cvt_pk_u16_u32 %5, %5, %6\nv_cvt_pk_u16_u32 %6, %6, %7\nv_cvt_pk_u16_u32 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k31(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cvt_f32_i32 %0, %1\nv_cvt_f32_i32 %1, %2\nv_cvt_f32_i32 %2, %3\nv_cvt_f32_i32 %3, %4\nv_cvt_f32_i32 %4, %5\nv_cvt_f32_i32 %5, %6\nv_cvt_f32_i32 %6, %7\nv_cvt_f32_i32 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k32(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mul_i32_i24 %0, %0, %1\nv_mul_i32_i24 %1, %1, %2\nv_mul_i32_i24 %2, %2, %3\nv_mul_i32_i24 %3, %3, %4\nv_mul_i32_i24 %4, %4, %5\nv_mul_i32_i24 %5, %5, %6\nv_mul_i32_i24 %6, %6, %7\nv_mul_i32_i24 %7, %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k33(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_perm_b32 %0, %0, %1, %1\nv_perm_b32 %1, %1, %2, %2\nv_perm_b32 %2, %2, %3, %3\nv_perm_b32 %3, %3, %4, %4\nv_perm_b32 %4, %4, %5, %5\nv_perm_b32 %5, %5, %6, %6\nv_perm_b32 %6, %6, %7, %7\nv_perm_b32 %7, %7, %0, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k34(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0) : "vcc");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_mov_b32 %0, %1\nv_mov_b32 %1, %2\nv_mov_b32 %2, %3\nv_mov_b32 %3, %4\nv_mov_b32 %4, %5\nv_mov_b32 %5, %6\nv_mov_b32 %6, %7\nv_mov_b32 %7, %0\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k100(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0\ns_mov_b64 s[4:5], vcc" :: "v"(a0) : "vcc", "s4", "s5");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cndmask_b32_e64 %0, %0, %1, s[4:5]\nv_cndmask_b32_e64 %1, %1, %2, s[4:5]\nv_cndmask_b32_e64 %2, %2, %3, s[4:5]\nv_cndmask_b32_e64 %3, %3, %4, s[4:5]\nv_cndmask_b32_e64 %4, %4, %5, s[4:5]\nv_cndmask_b32_e64 %5, %5, %6, s[4:5]\nv_cndmask_b32_e64 %6, %6, %7, s[4:5]\nv_cndmask_b32_e64 %7, %7, %0, s[4:5]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k101(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0\ns_mov_b64 s[4:5], vcc" :: "v"(a0) : "vcc", "s4", "s5");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_add_u32 %0, s4, %0\nv_add_u32 %1, s4, %1\nv_add_u32 %2, s4, %2\nv_add_u32 %3, s4, %3\nv_add_u32 %4, s4, %4\nv_add_u32 %5, s4, %5\nv_add_u32 %6, s4, %6\nv_add_u32 %7, s4, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ void k102(unsigned *out, int iters, unsigned long long *cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0\ns_mov_b64 s[4:5], vcc" :: "v"(a0) : "vcc", "s4", "s5");
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++)
    asm volatile(REP8("v_cmp_gt_u32 vcc, %0, %1\nv_cndmask_b32 %0, %0, %1, vcc\nv_cmp_gt_u32 vcc, %1, %2\nv_cndmask_b32 %1, %1, %2, vcc\nv_cmp_gt_u32 vcc, %2, %3\nv_cndmask_b32 %2, %2, %3, vcc\nv_cmp_gt_u32 vcc, %3, %4\nv_cndmask_b32 %3, %3, %4, vcc\nv_cmp_gt_u32 vcc, %4, %5\nv_cndmask_b32 %4, %4, %5, vcc\nv_cmp_gt_u32 vcc, %5, %6\nv_cndmask_b32 %5, %5, %6, vcc\nv_cmp_gt_u32 vcc, %6, %7\nv_cndmask_b32 %6, %6, %7, vcc\nv_cmp_gt_u32 vcc, %7, %0\nv_cndmask_b32 %7, %7, %0, vcc\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s4", "s5");
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
template <typename K>
void run(const char *name, K k, unsigned *buf, unsigned long long *cyc, int waves_per_simd) {
  const int iters = 1000, block = 256, grid = 256 * waves_per_simd;
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, iters, cyc);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, buf, iters, cyc);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double per_simd = (double)grid * 4 * iters * 64 / 1024;  // wave-instructions per SIMD
  printf("%-20s w/SIMD=%d %.3f ms  wave-cycles/instr @2.4GHz = %.2f\n", name, waves_per_simd, ms, ms * 1e-3 * 2.4e9 / per_simd);
}
int main() {
  unsigned *buf; unsigned long long *cyc;
  (void)hipMalloc(&buf, 256 * 8 * 256 * 4 * 4); (void)hipMalloc(&cyc, 8);
  run("lshlrev_k7", k0, buf, cyc, 8);
  run("lshlrev_vv", k1, buf, cyc, 8);
  run("lshrrev_k7", k2, buf, cyc, 8);
  run("ashrrev_k7", k3, buf, cyc, 8);
  run("or_sdwa_b1", k4, buf, cyc, 8);
  run("sub_u32_sdwa", k5, buf, cyc, 8);
  run("cvt_f32_ubyte_sdwa?", k6, buf, cyc, 8);
  run("sub_f32", k7, buf, cyc, 8);
  run("add_f32_abs", k8, buf, cyc, 8);
  run("max_f32", k9, buf, cyc, 8);
  run("min_f32", k10, buf, cyc, 8);
  run("max_u32", k11, buf, cyc, 8);
  run("bitop3_k", k12, buf, cyc, 8);
  run("and_lit", k13, buf, cyc, 8);
  run("fmac_f32", k14, buf, cyc, 8);
  run("fmamk_f32", k15, buf, cyc, 8);
  run("pk_fma_f16", k16, buf, cyc, 8);
  run("pk_add_f16", k17, buf, cyc, 8);
  run("dot2_f32_f16", k18, buf, cyc, 8);
  run("dot2c_f32_f16", k19, buf, cyc, 8);
  run("pk_mul_lo_u16", k20, buf, cyc, 8);
  run("pk_add_u16", k21, buf, cyc, 8);
  run("pk_lshlrev_b16", k22, buf, cyc, 8);
  run("sad_u32", k23, buf, cyc, 8);
  run("cndmask_vcc", k24, buf, cyc, 8);
  run("mov_dpp_shr1", k25, buf, cyc, 8);
  run("add_u32_dpp", k26, buf, cyc, 8);
  run("xad_u32", k27, buf, cyc, 8);
  run("add3_u32", k28, buf, cyc, 8);
  run("bfi_b32", k29, buf, cyc, 8);
  run("cvt_pk_u16_u32", k30, buf, cyc, 8);
  run("cvt_f32_i32", k31, buf, cyc, 8);
  run("mul_i32_i24", k32, buf, cyc, 8);
  run("perm_k", k33, buf, cyc, 8);
  run("readfirstlane?", k34, buf, cyc, 8);
  run("cndmask_e64_s", k100, buf, cyc, 8);
  run("add_u32_sgpr", k101, buf, cyc, 8);
  run("cmp_then_cndmask", k102, buf, cyc, 8);
  return 0;
}
