#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
constexpr int ITERS=2048;
__global__ __launch_bounds__(256) void k0(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k1(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_sub_u32 %0, %0, %8\nv_sub_u32 %1, %1, %8\nv_sub_u32 %2, %2, %8\nv_sub_u32 %3, %3, %8\nv_sub_u32 %4, %4, %8\nv_sub_u32 %5, %5, %8\nv_sub_u32 %6, %6, %8\nv_sub_u32 %7, %7, %8\nv_sub_u32 %0, %0, %8\nv_sub_u32 %1, %1, %8\nv_sub_u32 %2, %2, %8\nv_sub_u32 %3, %3, %8\nv_sub_u32 %4, %4, %8\nv_sub_u32 %5, %5, %8\nv_sub_u32 %6, %6, %8\nv_sub_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k2(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_i32 %0, %0, %8\nv_max_i32 %1, %1, %8\nv_max_i32 %2, %2, %8\nv_max_i32 %3, %3, %8\nv_max_i32 %4, %4, %8\nv_max_i32 %5, %5, %8\nv_max_i32 %6, %6, %8\nv_max_i32 %7, %7, %8\nv_max_i32 %0, %0, %8\nv_max_i32 %1, %1, %8\nv_max_i32 %2, %2, %8\nv_max_i32 %3, %3, %8\nv_max_i32 %4, %4, %8\nv_max_i32 %5, %5, %8\nv_max_i32 %6, %6, %8\nv_max_i32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k3(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_max_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_u32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_max_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k4(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_min_i32 %0, %0, %8\nv_min_i32 %1, %1, %8\nv_min_i32 %2, %2, %8\nv_min_i32 %3, %3, %8\nv_min_i32 %4, %4, %8\nv_min_i32 %5, %5, %8\nv_min_i32 %6, %6, %8\nv_min_i32 %7, %7, %8\nv_min_i32 %0, %0, %8\nv_min_i32 %1, %1, %8\nv_min_i32 %2, %2, %8\nv_min_i32 %3, %3, %8\nv_min_i32 %4, %4, %8\nv_min_i32 %5, %5, %8\nv_min_i32 %6, %6, %8\nv_min_i32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k5(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_and_b32 %0, %0, %8\nv_and_b32 %1, %1, %8\nv_and_b32 %2, %2, %8\nv_and_b32 %3, %3, %8\nv_and_b32 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_and_b32 %6, %6, %8\nv_and_b32 %7, %7, %8\nv_and_b32 %0, %0, %8\nv_and_b32 %1, %1, %8\nv_and_b32 %2, %2, %8\nv_and_b32 %3, %3, %8\nv_and_b32 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_and_b32 %6, %6, %8\nv_and_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k6(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_xor_b32 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_xor_b32 %2, %2, %8\nv_xor_b32 %3, %3, %8\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_xor_b32 %6, %6, %8\nv_xor_b32 %7, %7, %8\nv_xor_b32 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_xor_b32 %2, %2, %8\nv_xor_b32 %3, %3, %8\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_xor_b32 %6, %6, %8\nv_xor_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k7(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_lshlrev_b32 %0, %8, %0\nv_lshlrev_b32 %1, %8, %1\nv_lshlrev_b32 %2, %8, %2\nv_lshlrev_b32 %3, %8, %3\nv_lshlrev_b32 %4, %8, %4\nv_lshlrev_b32 %5, %8, %5\nv_lshlrev_b32 %6, %8, %6\nv_lshlrev_b32 %7, %8, %7\nv_lshlrev_b32 %0, %8, %0\nv_lshlrev_b32 %1, %8, %1\nv_lshlrev_b32 %2, %8, %2\nv_lshlrev_b32 %3, %8, %3\nv_lshlrev_b32 %4, %8, %4\nv_lshlrev_b32 %5, %8, %5\nv_lshlrev_b32 %6, %8, %6\nv_lshlrev_b32 %7, %8, %7\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k8(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_f32 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_add_f32 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_add_f32 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_add_f32 %6, %6, %8\nv_add_f32 %7, %7, %8\nv_add_f32 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_add_f32 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_add_f32 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_add_f32 %6, %6, %8\nv_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k9(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_f32 %0, %0, %8\nv_max_f32 %1, %1, %8\nv_max_f32 %2, %2, %8\nv_max_f32 %3, %3, %8\nv_max_f32 %4, %4, %8\nv_max_f32 %5, %5, %8\nv_max_f32 %6, %6, %8\nv_max_f32 %7, %7, %8\nv_max_f32 %0, %0, %8\nv_max_f32 %1, %1, %8\nv_max_f32 %2, %2, %8\nv_max_f32 %3, %3, %8\nv_max_f32 %4, %4, %8\nv_max_f32 %5, %5, %8\nv_max_f32 %6, %6, %8\nv_max_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k10(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_min_f32 %0, %0, %8\nv_min_f32 %1, %1, %8\nv_min_f32 %2, %2, %8\nv_min_f32 %3, %3, %8\nv_min_f32 %4, %4, %8\nv_min_f32 %5, %5, %8\nv_min_f32 %6, %6, %8\nv_min_f32 %7, %7, %8\nv_min_f32 %0, %0, %8\nv_min_f32 %1, %1, %8\nv_min_f32 %2, %2, %8\nv_min_f32 %3, %3, %8\nv_min_f32 %4, %4, %8\nv_min_f32 %5, %5, %8\nv_min_f32 %6, %6, %8\nv_min_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k11(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\nv_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k12(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_mul_f32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_mul_f32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_mul_f32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_mul_f32 %6, %6, %8\nv_mul_f32 %7, %7, %8\nv_mul_f32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_mul_f32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_mul_f32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_mul_f32 %6, %6, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k13(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max3_f32 %0, %0, %8, %8\nv_max3_f32 %1, %1, %8, %8\nv_max3_f32 %2, %2, %8, %8\nv_max3_f32 %3, %3, %8, %8\nv_max3_f32 %4, %4, %8, %8\nv_max3_f32 %5, %5, %8, %8\nv_max3_f32 %6, %6, %8, %8\nv_max3_f32 %7, %7, %8, %8\nv_max3_f32 %0, %0, %8, %8\nv_max3_f32 %1, %1, %8, %8\nv_max3_f32 %2, %2, %8, %8\nv_max3_f32 %3, %3, %8, %8\nv_max3_f32 %4, %4, %8, %8\nv_max3_f32 %5, %5, %8, %8\nv_max3_f32 %6, %6, %8, %8\nv_max3_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k14(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max3_i32 %0, %0, %8, %8\nv_max3_i32 %1, %1, %8, %8\nv_max3_i32 %2, %2, %8, %8\nv_max3_i32 %3, %3, %8, %8\nv_max3_i32 %4, %4, %8, %8\nv_max3_i32 %5, %5, %8, %8\nv_max3_i32 %6, %6, %8, %8\nv_max3_i32 %7, %7, %8, %8\nv_max3_i32 %0, %0, %8, %8\nv_max3_i32 %1, %1, %8, %8\nv_max3_i32 %2, %2, %8, %8\nv_max3_i32 %3, %3, %8, %8\nv_max3_i32 %4, %4, %8, %8\nv_max3_i32 %5, %5, %8, %8\nv_max3_i32 %6, %6, %8, %8\nv_max3_i32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k15(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_med3_i32 %0, %0, %8, %8\nv_med3_i32 %1, %1, %8, %8\nv_med3_i32 %2, %2, %8, %8\nv_med3_i32 %3, %3, %8, %8\nv_med3_i32 %4, %4, %8, %8\nv_med3_i32 %5, %5, %8, %8\nv_med3_i32 %6, %6, %8, %8\nv_med3_i32 %7, %7, %8, %8\nv_med3_i32 %0, %0, %8, %8\nv_med3_i32 %1, %1, %8, %8\nv_med3_i32 %2, %2, %8, %8\nv_med3_i32 %3, %3, %8, %8\nv_med3_i32 %4, %4, %8, %8\nv_med3_i32 %5, %5, %8, %8\nv_med3_i32 %6, %6, %8, %8\nv_med3_i32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k16(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add3_u32 %0, %0, %8, %8\nv_add3_u32 %1, %1, %8, %8\nv_add3_u32 %2, %2, %8, %8\nv_add3_u32 %3, %3, %8, %8\nv_add3_u32 %4, %4, %8, %8\nv_add3_u32 %5, %5, %8, %8\nv_add3_u32 %6, %6, %8, %8\nv_add3_u32 %7, %7, %8, %8\nv_add3_u32 %0, %0, %8, %8\nv_add3_u32 %1, %1, %8, %8\nv_add3_u32 %2, %2, %8, %8\nv_add3_u32 %3, %3, %8, %8\nv_add3_u32 %4, %4, %8, %8\nv_add3_u32 %5, %5, %8, %8\nv_add3_u32 %6, %6, %8, %8\nv_add3_u32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k17(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_mad_u32_u24 %0, %0, %8, %8\nv_mad_u32_u24 %1, %1, %8, %8\nv_mad_u32_u24 %2, %2, %8, %8\nv_mad_u32_u24 %3, %3, %8, %8\nv_mad_u32_u24 %4, %4, %8, %8\nv_mad_u32_u24 %5, %5, %8, %8\nv_mad_u32_u24 %6, %6, %8, %8\nv_mad_u32_u24 %7, %7, %8, %8\nv_mad_u32_u24 %0, %0, %8, %8\nv_mad_u32_u24 %1, %1, %8, %8\nv_mad_u32_u24 %2, %2, %8, %8\nv_mad_u32_u24 %3, %3, %8, %8\nv_mad_u32_u24 %4, %4, %8, %8\nv_mad_u32_u24 %5, %5, %8, %8\nv_mad_u32_u24 %6, %6, %8, %8\nv_mad_u32_u24 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k18(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_bitop3_b32 %0, %0, %8, %8 bitop3:0x6c\nv_bitop3_b32 %1, %1, %8, %8 bitop3:0x6c\nv_bitop3_b32 %2, %2, %8, %8 bitop3:0x6c\nv_bitop3_b32 %3, %3, %8, %8 bitop3:0x6c\nv_bitop3_b32 %4, %4, %8, %8 bitop3:0x6c\nv_bitop3_b32 %5, %5, %8, %8 bitop3:0x6c\nv_bitop3_b32 %6, %6, %8, %8 bitop3:0x6c\nv_bitop3_b32 %7, %7, %8, %8 bitop3:0x6c\nv_bitop3_b32 %0, %0, %8, %8 bitop3:0x6c\nv_bitop3_b32 %1, %1, %8, %8 bitop3:0x6c\nv_bitop3_b32 %2, %2, %8, %8 bitop3:0x6c\nv_bitop3_b32 %3, %3, %8, %8 bitop3:0x6c\nv_bitop3_b32 %4, %4, %8, %8 bitop3:0x6c\nv_bitop3_b32 %5, %5, %8, %8 bitop3:0x6c\nv_bitop3_b32 %6, %6, %8, %8 bitop3:0x6c\nv_bitop3_b32 %7, %7, %8, %8 bitop3:0x6c\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k19(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_perm_b32 %1, %1, %8, %8\nv_perm_b32 %2, %2, %8, %8\nv_perm_b32 %3, %3, %8, %8\nv_perm_b32 %4, %4, %8, %8\nv_perm_b32 %5, %5, %8, %8\nv_perm_b32 %6, %6, %8, %8\nv_perm_b32 %7, %7, %8, %8\nv_perm_b32 %0, %0, %8, %8\nv_perm_b32 %1, %1, %8, %8\nv_perm_b32 %2, %2, %8, %8\nv_perm_b32 %3, %3, %8, %8\nv_perm_b32 %4, %4, %8, %8\nv_perm_b32 %5, %5, %8, %8\nv_perm_b32 %6, %6, %8, %8\nv_perm_b32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k20(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_cndmask_b32 %0, %0, %8, vcc\nv_cndmask_b32 %1, %1, %8, vcc\nv_cndmask_b32 %2, %2, %8, vcc\nv_cndmask_b32 %3, %3, %8, vcc\nv_cndmask_b32 %4, %4, %8, vcc\nv_cndmask_b32 %5, %5, %8, vcc\nv_cndmask_b32 %6, %6, %8, vcc\nv_cndmask_b32 %7, %7, %8, vcc\nv_cndmask_b32 %0, %0, %8, vcc\nv_cndmask_b32 %1, %1, %8, vcc\nv_cndmask_b32 %2, %2, %8, vcc\nv_cndmask_b32 %3, %3, %8, vcc\nv_cndmask_b32 %4, %4, %8, vcc\nv_cndmask_b32 %5, %5, %8, vcc\nv_cndmask_b32 %6, %6, %8, vcc\nv_cndmask_b32 %7, %7, %8, vcc\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k21(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_i16 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_max_i16 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_max_i16 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_max_i16 %6, %6, %8\nv_max_i16 %7, %7, %8\nv_max_i16 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_max_i16 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_max_i16 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_max_i16 %6, %6, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k22(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_i16 %0, %0, %8\nv_pk_max_i16 %1, %1, %8\nv_pk_max_i16 %2, %2, %8\nv_pk_max_i16 %3, %3, %8\nv_pk_max_i16 %4, %4, %8\nv_pk_max_i16 %5, %5, %8\nv_pk_max_i16 %6, %6, %8\nv_pk_max_i16 %7, %7, %8\nv_pk_max_i16 %0, %0, %8\nv_pk_max_i16 %1, %1, %8\nv_pk_max_i16 %2, %2, %8\nv_pk_max_i16 %3, %3, %8\nv_pk_max_i16 %4, %4, %8\nv_pk_max_i16 %5, %5, %8\nv_pk_max_i16 %6, %6, %8\nv_pk_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k23(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_pk_mad_u16 %1, %1, %8, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_pk_mad_u16 %3, %3, %8, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_pk_mad_u16 %5, %5, %8, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_pk_mad_u16 %7, %7, %8, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_pk_mad_u16 %1, %1, %8, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_pk_mad_u16 %3, %3, %8, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_pk_mad_u16 %5, %5, %8, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_pk_mad_u16 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k24(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_add_f16 %0, %0, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_add_f16 %2, %2, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_add_f16 %4, %4, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_add_f16 %6, %6, %8\nv_pk_add_f16 %7, %7, %8\nv_pk_add_f16 %0, %0, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_add_f16 %2, %2, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_add_f16 %4, %4, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_add_f16 %6, %6, %8\nv_pk_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k25(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_f16 %0, %0, %8\nv_pk_max_f16 %1, %1, %8\nv_pk_max_f16 %2, %2, %8\nv_pk_max_f16 %3, %3, %8\nv_pk_max_f16 %4, %4, %8\nv_pk_max_f16 %5, %5, %8\nv_pk_max_f16 %6, %6, %8\nv_pk_max_f16 %7, %7, %8\nv_pk_max_f16 %0, %0, %8\nv_pk_max_f16 %1, %1, %8\nv_pk_max_f16 %2, %2, %8\nv_pk_max_f16 %3, %3, %8\nv_pk_max_f16 %4, %4, %8\nv_pk_max_f16 %5, %5, %8\nv_pk_max_f16 %6, %6, %8\nv_pk_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k26(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_fma_f16 %0, %0, %8, %8\nv_pk_fma_f16 %1, %1, %8, %8\nv_pk_fma_f16 %2, %2, %8, %8\nv_pk_fma_f16 %3, %3, %8, %8\nv_pk_fma_f16 %4, %4, %8, %8\nv_pk_fma_f16 %5, %5, %8, %8\nv_pk_fma_f16 %6, %6, %8, %8\nv_pk_fma_f16 %7, %7, %8, %8\nv_pk_fma_f16 %0, %0, %8, %8\nv_pk_fma_f16 %1, %1, %8, %8\nv_pk_fma_f16 %2, %2, %8, %8\nv_pk_fma_f16 %3, %3, %8, %8\nv_pk_fma_f16 %4, %4, %8, %8\nv_pk_fma_f16 %5, %5, %8, %8\nv_pk_fma_f16 %6, %6, %8, %8\nv_pk_fma_f16 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k27(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_pk_maximum3_f16 %1, %1, %8, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_pk_maximum3_f16 %3, %3, %8, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_pk_maximum3_f16 %5, %5, %8, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_pk_maximum3_f16 %7, %7, %8, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_pk_maximum3_f16 %1, %1, %8, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_pk_maximum3_f16 %3, %3, %8, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_pk_maximum3_f16 %5, %5, %8, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_pk_maximum3_f16 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k28(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_f16 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_max_f16 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_max_f16 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_max_f16 %6, %6, %8\nv_max_f16 %7, %7, %8\nv_max_f16 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_max_f16 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_max_f16 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_max_f16 %6, %6, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k29(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_f16 %0, %0, %8\nv_add_f16 %1, %1, %8\nv_add_f16 %2, %2, %8\nv_add_f16 %3, %3, %8\nv_add_f16 %4, %4, %8\nv_add_f16 %5, %5, %8\nv_add_f16 %6, %6, %8\nv_add_f16 %7, %7, %8\nv_add_f16 %0, %0, %8\nv_add_f16 %1, %1, %8\nv_add_f16 %2, %2, %8\nv_add_f16 %3, %3, %8\nv_add_f16 %4, %4, %8\nv_add_f16 %5, %5, %8\nv_add_f16 %6, %6, %8\nv_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k30(uint32_t*out,uint32_t seed){
  uint64_t b=seed+threadIdx.x; uint64_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_add_f32 %0, %0, %8\nv_pk_add_f32 %1, %1, %8\nv_pk_add_f32 %2, %2, %8\nv_pk_add_f32 %3, %3, %8\nv_pk_add_f32 %4, %4, %8\nv_pk_add_f32 %5, %5, %8\nv_pk_add_f32 %6, %6, %8\nv_pk_add_f32 %7, %7, %8\nv_pk_add_f32 %0, %0, %8\nv_pk_add_f32 %1, %1, %8\nv_pk_add_f32 %2, %2, %8\nv_pk_add_f32 %3, %3, %8\nv_pk_add_f32 %4, %4, %8\nv_pk_add_f32 %5, %5, %8\nv_pk_add_f32 %6, %6, %8\nv_pk_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k31(uint32_t*out,uint32_t seed){
  uint64_t b=seed+threadIdx.x; uint64_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_fma_f32 %0, %0, %8, %8\nv_pk_fma_f32 %1, %1, %8, %8\nv_pk_fma_f32 %2, %2, %8, %8\nv_pk_fma_f32 %3, %3, %8, %8\nv_pk_fma_f32 %4, %4, %8, %8\nv_pk_fma_f32 %5, %5, %8, %8\nv_pk_fma_f32 %6, %6, %8, %8\nv_pk_fma_f32 %7, %7, %8, %8\nv_pk_fma_f32 %0, %0, %8, %8\nv_pk_fma_f32 %1, %1, %8, %8\nv_pk_fma_f32 %2, %2, %8, %8\nv_pk_fma_f32 %3, %3, %8, %8\nv_pk_fma_f32 %4, %4, %8, %8\nv_pk_fma_f32 %5, %5, %8, %8\nv_pk_fma_f32 %6, %6, %8, %8\nv_pk_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k32(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_co_u32 %0, vcc, %0, %8\nv_add_co_u32 %1, vcc, %1, %8\nv_add_co_u32 %2, vcc, %2, %8\nv_add_co_u32 %3, vcc, %3, %8\nv_add_co_u32 %4, vcc, %4, %8\nv_add_co_u32 %5, vcc, %5, %8\nv_add_co_u32 %6, vcc, %6, %8\nv_add_co_u32 %7, vcc, %7, %8\nv_add_co_u32 %0, vcc, %0, %8\nv_add_co_u32 %1, vcc, %1, %8\nv_add_co_u32 %2, vcc, %2, %8\nv_add_co_u32 %3, vcc, %3, %8\nv_add_co_u32 %4, vcc, %4, %8\nv_add_co_u32 %5, vcc, %5, %8\nv_add_co_u32 %6, vcc, %6, %8\nv_add_co_u32 %7, vcc, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k33(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_sub_u16 %0, %0, %8\nv_sub_u16 %1, %1, %8\nv_sub_u16 %2, %2, %8\nv_sub_u16 %3, %3, %8\nv_sub_u16 %4, %4, %8\nv_sub_u16 %5, %5, %8\nv_sub_u16 %6, %6, %8\nv_sub_u16 %7, %7, %8\nv_sub_u16 %0, %0, %8\nv_sub_u16 %1, %1, %8\nv_sub_u16 %2, %2, %8\nv_sub_u16 %3, %3, %8\nv_sub_u16 %4, %4, %8\nv_sub_u16 %5, %5, %8\nv_sub_u16 %6, %6, %8\nv_sub_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k34(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_dot2_u32_u16 %0, %0, %8, %8\nv_dot2_u32_u16 %1, %1, %8, %8\nv_dot2_u32_u16 %2, %2, %8, %8\nv_dot2_u32_u16 %3, %3, %8, %8\nv_dot2_u32_u16 %4, %4, %8, %8\nv_dot2_u32_u16 %5, %5, %8, %8\nv_dot2_u32_u16 %6, %6, %8, %8\nv_dot2_u32_u16 %7, %7, %8, %8\nv_dot2_u32_u16 %0, %0, %8, %8\nv_dot2_u32_u16 %1, %1, %8, %8\nv_dot2_u32_u16 %2, %2, %8, %8\nv_dot2_u32_u16 %3, %3, %8, %8\nv_dot2_u32_u16 %4, %4, %8, %8\nv_dot2_u32_u16 %5, %5, %8, %8\nv_dot2_u32_u16 %6, %6, %8, %8\nv_dot2_u32_u16 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k35(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_sad_u32 %0, %0, %8, %8\nv_sad_u32 %1, %1, %8, %8\nv_sad_u32 %2, %2, %8, %8\nv_sad_u32 %3, %3, %8, %8\nv_sad_u32 %4, %4, %8, %8\nv_sad_u32 %5, %5, %8, %8\nv_sad_u32 %6, %6, %8, %8\nv_sad_u32 %7, %7, %8, %8\nv_sad_u32 %0, %0, %8, %8\nv_sad_u32 %1, %1, %8, %8\nv_sad_u32 %2, %2, %8, %8\nv_sad_u32 %3, %3, %8, %8\nv_sad_u32 %4, %4, %8, %8\nv_sad_u32 %5, %5, %8, %8\nv_sad_u32 %6, %6, %8, %8\nv_sad_u32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k36(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_i32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %1, %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %2, %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %3, %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %4, %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %5, %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %6, %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %7, %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %1, %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %2, %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %3, %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %4, %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %5, %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %6, %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %7, %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k37(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_mov_b32_dpp %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
typedef void(*KF)(uint32_t*,uint32_t);
KF ks[]={k0,k1,k2,k3,k4,k5,k6,k7,k8,k9,k10,k11,k12,k13,k14,k15,k16,k17,k18,k19,k20,k21,k22,k23,k24,k25,k26,k27,k28,k29,k30,k31,k32,k33,k34,k35,k36,k37};
const char*names[]={"v_add_u32","v_sub_u32","v_max_i32","v_max_u32","v_min_i32","v_and_b32","v_xor_b32","v_lshlrev_b32","v_add_f32","v_max_f32","v_min_f32","v_fma_f32","v_mul_f32","v_max3_f32","v_max3_i32","v_med3_i32","v_add3_u32","v_mad_u32_u24","v_bitop3_b32","v_perm_b32","v_cndmask_b32","v_max_i16","v_pk_max_i16","v_pk_mad_u16","v_pk_add_f16","v_pk_max_f16","v_pk_fma_f16","v_pk_maximum3_f16","v_max_f16","v_add_f16","v_pk_add_f32","v_pk_fma_f32","v_add_co_u32","v_sub_u16","v_dot2_u32_u16","v_sad_u32","v_max_i32_dpp","v_mov_b32_dpp"};
int main(){uint32_t*out;hipMalloc(&out,256*256*8*4);
 for(int v=0;v<(int)(sizeof(ks)/sizeof(ks[0]));++v){ printf("%-20s",names[v]);
  for(int W: {2,4,8}){int blocks=256*W; hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   hipEvent_t e0,e1;hipEventCreate(&e0);hipEventCreate(&e1);hipEventRecord(e0);
   hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);hipEventRecord(e1);hipEventSynchronize(e1);
   float ms;hipEventElapsedTime(&ms,e0,e1); double ninst=(double)ITERS*16*blocks*4; // wave instrs
   printf("  W=%d %.2f cyc/inst/SIMD", W, ms*1e-3*2.4e9/(ninst/1024));}
  printf("\n");}
 return 0;}