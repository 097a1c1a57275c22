#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
constexpr int ITERS=2048;
__global__ __launch_bounds__(256) void k0(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k1(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_max_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_u32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_max_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k2(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k3(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k4(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_u16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k5(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u16 %0, %0, %8\nv_max_u16 %1, %1, %8\nv_max_u16 %2, %2, %8\nv_max_u16 %3, %3, %8\nv_max_u16 %4, %4, %8\nv_max_u16 %5, %5, %8\nv_max_u16 %6, %6, %8\nv_max_u16 %7, %7, %8\nv_max_u16 %0, %0, %8\nv_max_u16 %1, %1, %8\nv_max_u16 %2, %2, %8\nv_max_u16 %3, %3, %8\nv_max_u16 %4, %4, %8\nv_max_u16 %5, %5, %8\nv_max_u16 %6, %6, %8\nv_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k6(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u16_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k7(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u16 %0, %0, %8\nv_max_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %2, %2, %8\nv_max_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %4, %4, %8\nv_max_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %6, %6, %8\nv_max_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %0, %0, %8\nv_max_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %2, %2, %8\nv_max_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %4, %4, %8\nv_max_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_max_u16 %6, %6, %8\nv_max_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k8(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_perm_b32 %1, %1, %8, %8\nv_pk_max_u16 %2, %2, %8\nv_perm_b32 %3, %3, %8, %8\nv_pk_max_u16 %4, %4, %8\nv_perm_b32 %5, %5, %8, %8\nv_pk_max_u16 %6, %6, %8\nv_perm_b32 %7, %7, %8, %8\nv_pk_max_u16 %0, %0, %8\nv_perm_b32 %1, %1, %8, %8\nv_pk_max_u16 %2, %2, %8\nv_perm_b32 %3, %3, %8, %8\nv_pk_max_u16 %4, %4, %8\nv_perm_b32 %5, %5, %8, %8\nv_pk_max_u16 %6, %6, %8\nv_perm_b32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k9(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_max_u16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_u16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_u16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_u16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_max_u16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_u16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_u16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k10(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_xor_b32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_xor_b32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_xor_b32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_xor_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k11(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_u16 %0, %0, %8\nv_add_u16 %1, %1, %8\nv_add_u16 %2, %2, %8\nv_add_u16 %3, %3, %8\nv_add_u16 %4, %4, %8\nv_add_u16 %5, %5, %8\nv_add_u16 %6, %6, %8\nv_add_u16 %7, %7, %8\nv_add_u16 %0, %0, %8\nv_add_u16 %1, %1, %8\nv_add_u16 %2, %2, %8\nv_add_u16 %3, %3, %8\nv_add_u16 %4, %4, %8\nv_add_u16 %5, %5, %8\nv_add_u16 %6, %6, %8\nv_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k12(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_sub_u16_e64 %0, %0, %8 clamp\nv_sub_u16_e64 %1, %1, %8 clamp\nv_sub_u16_e64 %2, %2, %8 clamp\nv_sub_u16_e64 %3, %3, %8 clamp\nv_sub_u16_e64 %4, %4, %8 clamp\nv_sub_u16_e64 %5, %5, %8 clamp\nv_sub_u16_e64 %6, %6, %8 clamp\nv_sub_u16_e64 %7, %7, %8 clamp\nv_sub_u16_e64 %0, %0, %8 clamp\nv_sub_u16_e64 %1, %1, %8 clamp\nv_sub_u16_e64 %2, %2, %8 clamp\nv_sub_u16_e64 %3, %3, %8 clamp\nv_sub_u16_e64 %4, %4, %8 clamp\nv_sub_u16_e64 %5, %5, %8 clamp\nv_sub_u16_e64 %6, %6, %8 clamp\nv_sub_u16_e64 %7, %7, %8 clamp\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k13(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_i16_e64 %0, %0, %8\nv_max_i16_e64 %1, %1, %8\nv_max_i16_e64 %2, %2, %8\nv_max_i16_e64 %3, %3, %8\nv_max_i16_e64 %4, %4, %8\nv_max_i16_e64 %5, %5, %8\nv_max_i16_e64 %6, %6, %8\nv_max_i16_e64 %7, %7, %8\nv_max_i16_e64 %0, %0, %8\nv_max_i16_e64 %1, %1, %8\nv_max_i16_e64 %2, %2, %8\nv_max_i16_e64 %3, %3, %8\nv_max_i16_e64 %4, %4, %8\nv_max_i16_e64 %5, %5, %8\nv_max_i16_e64 %6, %6, %8\nv_max_i16_e64 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k14(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k15(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_f16 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_max_f16 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_max_f16 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_max_f16 %6, %6, %8\nv_max_f16 %7, %7, %8\nv_max_f16 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_max_f16 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_max_f16 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_max_f16 %6, %6, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k16(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_u32_e64 %0, %0, %8\nv_add_u32_e64 %1, %1, %8\nv_add_u32_e64 %2, %2, %8\nv_add_u32_e64 %3, %3, %8\nv_add_u32_e64 %4, %4, %8\nv_add_u32_e64 %5, %5, %8\nv_add_u32_e64 %6, %6, %8\nv_add_u32_e64 %7, %7, %8\nv_add_u32_e64 %0, %0, %8\nv_add_u32_e64 %1, %1, %8\nv_add_u32_e64 %2, %2, %8\nv_add_u32_e64 %3, %3, %8\nv_add_u32_e64 %4, %4, %8\nv_add_u32_e64 %5, %5, %8\nv_add_u32_e64 %6, %6, %8\nv_add_u32_e64 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k17(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_mul_u32_u24 %0, %0, %8\nv_mul_u32_u24 %1, %1, %8\nv_mul_u32_u24 %2, %2, %8\nv_mul_u32_u24 %3, %3, %8\nv_mul_u32_u24 %4, %4, %8\nv_mul_u32_u24 %5, %5, %8\nv_mul_u32_u24 %6, %6, %8\nv_mul_u32_u24 %7, %7, %8\nv_mul_u32_u24 %0, %0, %8\nv_mul_u32_u24 %1, %1, %8\nv_mul_u32_u24 %2, %2, %8\nv_mul_u32_u24 %3, %3, %8\nv_mul_u32_u24 %4, %4, %8\nv_mul_u32_u24 %5, %5, %8\nv_mul_u32_u24 %6, %6, %8\nv_mul_u32_u24 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k18(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_cndmask_b32_e64 %0, %0, %8, s[0:1]\nv_cndmask_b32_e64 %1, %1, %8, s[0:1]\nv_cndmask_b32_e64 %2, %2, %8, s[0:1]\nv_cndmask_b32_e64 %3, %3, %8, s[0:1]\nv_cndmask_b32_e64 %4, %4, %8, s[0:1]\nv_cndmask_b32_e64 %5, %5, %8, s[0:1]\nv_cndmask_b32_e64 %6, %6, %8, s[0:1]\nv_cndmask_b32_e64 %7, %7, %8, s[0:1]\nv_cndmask_b32_e64 %0, %0, %8, s[0:1]\nv_cndmask_b32_e64 %1, %1, %8, s[0:1]\nv_cndmask_b32_e64 %2, %2, %8, s[0:1]\nv_cndmask_b32_e64 %3, %3, %8, s[0:1]\nv_cndmask_b32_e64 %4, %4, %8, s[0:1]\nv_cndmask_b32_e64 %5, %5, %8, s[0:1]\nv_cndmask_b32_e64 %6, %6, %8, s[0:1]\nv_cndmask_b32_e64 %7, %7, %8, s[0:1]\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k19(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_mov_b32 %0, %8\nv_mov_b32 %1, %8\nv_mov_b32 %2, %8\nv_mov_b32 %3, %8\nv_mov_b32 %4, %8\nv_mov_b32 %5, %8\nv_mov_b32 %6, %8\nv_mov_b32 %7, %8\nv_mov_b32 %0, %8\nv_mov_b32 %1, %8\nv_mov_b32 %2, %8\nv_mov_b32 %3, %8\nv_mov_b32 %4, %8\nv_mov_b32 %5, %8\nv_mov_b32 %6, %8\nv_mov_b32 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k20(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max3_u32 %0, %0, %8, %8\nv_max3_u32 %1, %1, %8, %8\nv_max3_u32 %2, %2, %8, %8\nv_max3_u32 %3, %3, %8, %8\nv_max3_u32 %4, %4, %8, %8\nv_max3_u32 %5, %5, %8, %8\nv_max3_u32 %6, %6, %8, %8\nv_max3_u32 %7, %7, %8, %8\nv_max3_u32 %0, %0, %8, %8\nv_max3_u32 %1, %1, %8, %8\nv_max3_u32 %2, %2, %8, %8\nv_max3_u32 %3, %3, %8, %8\nv_max3_u32 %4, %4, %8, %8\nv_max3_u32 %5, %5, %8, %8\nv_max3_u32 %6, %6, %8, %8\nv_max3_u32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
typedef void(*KF)(uint32_t*,uint32_t);
KF ks[]={k0,k1,k2,k3,k4,k5,k6,k7,k8,k9,k10,k11,k12,k13,k14,k15,k16,k17,k18,k19,k20};
const char*names[]={"16 pk_max_u16","8 pk_max + 8 max_u32","8 pk_max + 8 add_u32","8 max_u32 + 8 add_u32","8 pk_max + 8 max_u16","16 max_u16","16 max_u16 sdwa hi","8 max_u16 + 8 max_u16_sdwa","8 pk_max + 8 perm","8 max_u32 + 8 max_u16","8 pk_max + 8 xor","16 add_u16","16 sub_u16 clamp","16 max_i16_e64","16 pk_add_u16","16 max_f16","16 add_u32 e64","16 mul_u32_u24","16 cndmask sgpr","16 mov_b32","16 max3_u32 (2x max work)"};
int main(){uint32_t*out;(void)hipMalloc(&out,256*256*8*4);
 for(int v=0;v<(int)(sizeof(ks)/sizeof(ks[0]));++v){ printf("%-30s",names[v]);
  for(int W: {2,4,8}){int blocks=256*W; hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   hipEvent_t e0,e1;(void)hipEventCreate(&e0);(void)hipEventCreate(&e1);(void)hipEventRecord(e0);
   for(int rep=0;rep<3;++rep) hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   (void)hipEventRecord(e1);(void)hipEventSynchronize(e1);
   float ms;(void)hipEventElapsedTime(&ms,e0,e1); double ninst=3.0*ITERS*16*blocks*4;
   printf("  W=%d %.2f", W, ms*1e-3*2.4e9/(ninst/1024));}
  printf("   cyc/inst/SIMD\n");}
 return 0;}