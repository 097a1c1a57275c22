#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
constexpr int ITERS=2048;
__global__ __launch_bounds__(256) void k0(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_f32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k1(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_mul_f32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k2(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k3(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_and_b32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_and_b32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_and_b32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_and_b32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_and_b32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_and_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k4(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_i16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k5(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_add_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_add_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k6(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_mov_b32 %1, %8\nv_pk_max_u16 %2, %2, %8\nv_mov_b32 %3, %8\nv_pk_max_u16 %4, %4, %8\nv_mov_b32 %5, %8\nv_pk_max_u16 %6, %6, %8\nv_mov_b32 %7, %8\nv_pk_max_u16 %0, %0, %8\nv_mov_b32 %1, %8\nv_pk_max_u16 %2, %2, %8\nv_mov_b32 %3, %8\nv_pk_max_u16 %4, %4, %8\nv_mov_b32 %5, %8\nv_pk_max_u16 %6, %6, %8\nv_mov_b32 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k7(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_fma_f32 %1, %1, %8, %8\nv_pk_max_u16 %2, %2, %8\nv_fma_f32 %3, %3, %8, %8\nv_pk_max_u16 %4, %4, %8\nv_fma_f32 %5, %5, %8, %8\nv_pk_max_u16 %6, %6, %8\nv_fma_f32 %7, %7, %8, %8\nv_pk_max_u16 %0, %0, %8\nv_fma_f32 %1, %1, %8, %8\nv_pk_max_u16 %2, %2, %8\nv_fma_f32 %3, %3, %8, %8\nv_pk_max_u16 %4, %4, %8\nv_fma_f32 %5, %5, %8, %8\nv_pk_max_u16 %6, %6, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k8(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_max_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_f32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_max_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k9(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_add_f16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k10(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_f16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k11(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_sub_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_sub_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_sub_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_sub_f32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_sub_f32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_sub_f32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_sub_f32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_sub_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k12(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k13(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_add_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_f32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_add_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k14(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_mul_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_mul_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_mul_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_mul_f32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_mul_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_mul_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_mul_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k15(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k16(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_and_b32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_and_b32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_and_b32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_and_b32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_and_b32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_and_b32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_and_b32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_and_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k17(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_max_i16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_max_i16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_max_i16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_max_i16 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_max_i16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_max_i16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_max_i16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k18(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_add_u16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_u16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_u16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_u16 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_add_u16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_u16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_u16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k19(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_mov_b32 %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_mov_b32 %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_mov_b32 %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_mov_b32 %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_mov_b32 %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_mov_b32 %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_mov_b32 %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_mov_b32 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k20(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k21(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_max_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_max_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_max_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_max_f32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_max_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_max_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_max_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_max_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k22(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_pk_add_f16 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_pk_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k23(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_max_f16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_max_f16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_max_f16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_max_f16 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_max_f16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_max_f16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_max_f16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k24(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_sub_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_sub_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_sub_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_sub_f32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_sub_f32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_sub_f32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_sub_f32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_sub_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k25(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_pk_max_u16 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k26(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_add_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_f32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_add_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k27(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_mul_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_mul_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_mul_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_mul_f32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_mul_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_mul_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_mul_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k28(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k29(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_and_b32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_and_b32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_and_b32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_and_b32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_and_b32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_and_b32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_and_b32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_and_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k30(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_max_i16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_max_i16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_max_i16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_max_i16 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_max_i16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_max_i16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_max_i16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k31(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_add_u16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_u16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_u16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_u16 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_add_u16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_u16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_u16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k32(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_mov_b32 %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_mov_b32 %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_mov_b32 %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_mov_b32 %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_mov_b32 %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_mov_b32 %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_mov_b32 %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_mov_b32 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k33(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_perm_b32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_perm_b32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_perm_b32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\nv_perm_b32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_perm_b32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_perm_b32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_perm_b32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k34(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_max_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_max_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_max_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_max_f32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_max_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_max_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_max_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_max_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k35(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_pk_add_f16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_pk_add_f16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_pk_add_f16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_pk_add_f16 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_pk_add_f16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_pk_add_f16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_pk_add_f16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_pk_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k36(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_max_f16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_max_f16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_max_f16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_max_f16 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_max_f16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_max_f16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_max_f16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k37(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_sub_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_sub_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_sub_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_sub_f32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_sub_f32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_sub_f32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_sub_f32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_sub_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k38(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_pk_max_u16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_pk_max_u16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_pk_max_u16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_pk_max_u16 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_pk_max_u16 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_pk_max_u16 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_pk_max_u16 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k39(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_add_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_add_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_add_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_add_f32 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_add_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_add_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_add_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k40(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_mul_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_mul_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_mul_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_mul_f32 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_mul_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_mul_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_mul_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k41(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k42(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_and_b32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_and_b32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_and_b32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_and_b32 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_and_b32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_and_b32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_and_b32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_and_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k43(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_max_i16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_max_i16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_max_i16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_max_i16 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_max_i16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_max_i16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_max_i16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k44(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_add_u16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_add_u16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_add_u16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_add_u16 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_add_u16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_add_u16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_add_u16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k45(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_mov_b32 %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_mov_b32 %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_mov_b32 %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_mov_b32 %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_mov_b32 %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_mov_b32 %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_mov_b32 %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_mov_b32 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k46(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k47(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_max_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_max_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_max_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_max_f32 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_max_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_max_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_max_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_max_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k48(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_pk_add_f16 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_pk_add_f16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_pk_add_f16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_pk_add_f16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_pk_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k49(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_max_f16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_max_f16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_max_f16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_max_f16 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_max_f16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_max_f16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_max_f16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k50(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_sub_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_sub_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_sub_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_sub_f32 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_sub_f32 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_sub_f32 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_sub_f32 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_sub_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k51(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mad_u16 %0, %0, %8, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_pk_max_u16 %7, %7, %8\nv_pk_mad_u16 %0, %0, %8, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_mad_u16 %2, %2, %8, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_mad_u16 %4, %4, %8, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_mad_u16 %6, %6, %8, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k52(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_f32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k53(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_mul_f32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k54(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k55(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_and_b32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_and_b32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_and_b32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_and_b32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_and_b32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_and_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k56(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_i16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k57(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_add_u16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_add_u16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k58(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_mov_b32 %1, %8\nv_max_u32 %2, %2, %8\nv_mov_b32 %3, %8\nv_max_u32 %4, %4, %8\nv_mov_b32 %5, %8\nv_max_u32 %6, %6, %8\nv_mov_b32 %7, %8\nv_max_u32 %0, %0, %8\nv_mov_b32 %1, %8\nv_max_u32 %2, %2, %8\nv_mov_b32 %3, %8\nv_max_u32 %4, %4, %8\nv_mov_b32 %5, %8\nv_max_u32 %6, %6, %8\nv_mov_b32 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k59(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_fma_f32 %1, %1, %8, %8\nv_max_u32 %2, %2, %8\nv_fma_f32 %3, %3, %8, %8\nv_max_u32 %4, %4, %8\nv_fma_f32 %5, %5, %8, %8\nv_max_u32 %6, %6, %8\nv_fma_f32 %7, %7, %8, %8\nv_max_u32 %0, %0, %8\nv_fma_f32 %1, %1, %8, %8\nv_max_u32 %2, %2, %8\nv_fma_f32 %3, %3, %8, %8\nv_max_u32 %4, %4, %8\nv_fma_f32 %5, %5, %8, %8\nv_max_u32 %6, %6, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k60(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_max_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_f32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_max_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k61(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_pk_add_f16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_pk_add_f16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_pk_add_f16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_pk_add_f16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_pk_add_f16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_pk_add_f16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_pk_add_f16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_pk_add_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k62(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_f16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_max_f16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_f16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_f16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_f16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k63(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_sub_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_sub_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_sub_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_sub_f32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_sub_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_sub_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_sub_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_sub_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k64(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
typedef void(*KF)(uint32_t*,uint32_t);
KF ks[]={k0,k1,k2,k3,k4,k5,k6,k7,k8,k9,k10,k11,k12,k13,k14,k15,k16,k17,k18,k19,k20,k21,k22,k23,k24,k25,k26,k27,k28,k29,k30,k31,k32,k33,k34,k35,k36,k37,k38,k39,k40,k41,k42,k43,k44,k45,k46,k47,k48,k49,k50,k51,k52,k53,k54,k55,k56,k57,k58,k59,k60,k61,k62,k63,k64};
const char*names[]={"pk_max_u16+add_f32","pk_max_u16+mul_f32","pk_max_u16+add_u32","pk_max_u16+and_b32","pk_max_u16+max_i16","pk_max_u16+add_u16","pk_max_u16+mov_b32","pk_max_u16+fma_f32","pk_max_u16+max_f32","pk_max_u16+pk_add_f16","pk_max_u16+max_f16","pk_max_u16+sub_f32","pk_max_u16+pk_max_u16","pk_max3_f16+add_f32","pk_max3_f16+mul_f32","pk_max3_f16+add_u32","pk_max3_f16+and_b32","pk_max3_f16+max_i16","pk_max3_f16+add_u16","pk_max3_f16+mov_b32","pk_max3_f16+fma_f32","pk_max3_f16+max_f32","pk_max3_f16+pk_add_f16","pk_max3_f16+max_f16","pk_max3_f16+sub_f32","pk_max3_f16+pk_max_u16","perm+add_f32","perm+mul_f32","perm+add_u32","perm+and_b32","perm+max_i16","perm+add_u16","perm+mov_b32","perm+fma_f32","perm+max_f32","perm+pk_add_f16","perm+max_f16","perm+sub_f32","perm+pk_max_u16","pk_mad_u16+add_f32","pk_mad_u16+mul_f32","pk_mad_u16+add_u32","pk_mad_u16+and_b32","pk_mad_u16+max_i16","pk_mad_u16+add_u16","pk_mad_u16+mov_b32","pk_mad_u16+fma_f32","pk_mad_u16+max_f32","pk_mad_u16+pk_add_f16","pk_mad_u16+max_f16","pk_mad_u16+sub_f32","pk_mad_u16+pk_max_u16","max_u32+add_f32","max_u32+mul_f32","max_u32+add_u32","max_u32+and_b32","max_u32+max_i16","max_u32+add_u16","max_u32+mov_b32","max_u32+fma_f32","max_u32+max_f32","max_u32+pk_add_f16","max_u32+max_f16","max_u32+sub_f32","max_u32+pk_max_u16"};
int main(){uint32_t*out;(void)hipMalloc(&out,256*256*8*4);
 for(int v=0;v<(int)(sizeof(ks)/sizeof(ks[0]));++v){ printf("%-24s",names[v]);
  for(int W: {8}){int blocks=256*W; hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   hipEvent_t e0,e1;(void)hipEventCreate(&e0);(void)hipEventCreate(&e1);(void)hipEventRecord(e0);
   for(int rep=0;rep<3;++rep) hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   (void)hipEventRecord(e1);(void)hipEventSynchronize(e1);
   float ms;(void)hipEventElapsedTime(&ms,e0,e1); double ninst=3.0*ITERS*16*blocks*4;
   printf("  W=%d %.2f cyc/inst  (%.2f per pair)", W, ms*1e-3*2.4e9/(ninst/1024), 2*ms*1e-3*2.4e9/(ninst/1024));}
  printf("\n");}
 return 0;}