#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
constexpr int ITERS=2048;
__global__ __launch_bounds__(256) void k0(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_fmac_f32 %0, %8, %8\nv_fmac_f32 %1, %8, %8\nv_fmac_f32 %2, %8, %8\nv_fmac_f32 %3, %8, %8\nv_fmac_f32 %4, %8, %8\nv_fmac_f32 %5, %8, %8\nv_fmac_f32 %6, %8, %8\nv_fmac_f32 %7, %8, %8\nv_fmac_f32 %0, %8, %8\nv_fmac_f32 %1, %8, %8\nv_fmac_f32 %2, %8, %8\nv_fmac_f32 %3, %8, %8\nv_fmac_f32 %4, %8, %8\nv_fmac_f32 %5, %8, %8\nv_fmac_f32 %6, %8, %8\nv_fmac_f32 %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k1(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\nv_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k2(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_mul_f32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_mul_f32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_mul_f32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_mul_f32 %6, %6, %8\nv_mul_f32 %7, %7, %8\nv_mul_f32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_mul_f32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_mul_f32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_mul_f32 %6, %6, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k3(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_cmp_eq_u32 vcc, %0, %8\nv_cmp_eq_u32 vcc, %1, %8\nv_cmp_eq_u32 vcc, %2, %8\nv_cmp_eq_u32 vcc, %3, %8\nv_cmp_eq_u32 vcc, %4, %8\nv_cmp_eq_u32 vcc, %5, %8\nv_cmp_eq_u32 vcc, %6, %8\nv_cmp_eq_u32 vcc, %7, %8\nv_cmp_eq_u32 vcc, %0, %8\nv_cmp_eq_u32 vcc, %1, %8\nv_cmp_eq_u32 vcc, %2, %8\nv_cmp_eq_u32 vcc, %3, %8\nv_cmp_eq_u32 vcc, %4, %8\nv_cmp_eq_u32 vcc, %5, %8\nv_cmp_eq_u32 vcc, %6, %8\nv_cmp_eq_u32 vcc, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc","s0","s1");
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k4(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_cmp_eq_u32_e64 s[0:1], %0, %8\nv_cmp_eq_u32_e64 s[0:1], %1, %8\nv_cmp_eq_u32_e64 s[0:1], %2, %8\nv_cmp_eq_u32_e64 s[0:1], %3, %8\nv_cmp_eq_u32_e64 s[0:1], %4, %8\nv_cmp_eq_u32_e64 s[0:1], %5, %8\nv_cmp_eq_u32_e64 s[0:1], %6, %8\nv_cmp_eq_u32_e64 s[0:1], %7, %8\nv_cmp_eq_u32_e64 s[0:1], %0, %8\nv_cmp_eq_u32_e64 s[0:1], %1, %8\nv_cmp_eq_u32_e64 s[0:1], %2, %8\nv_cmp_eq_u32_e64 s[0:1], %3, %8\nv_cmp_eq_u32_e64 s[0:1], %4, %8\nv_cmp_eq_u32_e64 s[0:1], %5, %8\nv_cmp_eq_u32_e64 s[0:1], %6, %8\nv_cmp_eq_u32_e64 s[0:1], %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc","s0","s1");
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k5(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_cndmask_b32 %0, %0, %8, vcc\nv_cndmask_b32 %1, %1, %8, vcc\nv_cndmask_b32 %2, %2, %8, vcc\nv_cndmask_b32 %3, %3, %8, vcc\nv_cndmask_b32 %4, %4, %8, vcc\nv_cndmask_b32 %5, %5, %8, vcc\nv_cndmask_b32 %6, %6, %8, vcc\nv_cndmask_b32 %7, %7, %8, vcc\nv_cndmask_b32 %0, %0, %8, vcc\nv_cndmask_b32 %1, %1, %8, vcc\nv_cndmask_b32 %2, %2, %8, vcc\nv_cndmask_b32 %3, %3, %8, vcc\nv_cndmask_b32 %4, %4, %8, vcc\nv_cndmask_b32 %5, %5, %8, vcc\nv_cndmask_b32 %6, %6, %8, vcc\nv_cndmask_b32 %7, %7, %8, vcc\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k6(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_cndmask_b32_e64 %0, %0, %8, s[2:3]\nv_cndmask_b32_e64 %1, %1, %8, s[2:3]\nv_cndmask_b32_e64 %2, %2, %8, s[2:3]\nv_cndmask_b32_e64 %3, %3, %8, s[2:3]\nv_cndmask_b32_e64 %4, %4, %8, s[2:3]\nv_cndmask_b32_e64 %5, %5, %8, s[2:3]\nv_cndmask_b32_e64 %6, %6, %8, s[2:3]\nv_cndmask_b32_e64 %7, %7, %8, s[2:3]\nv_cndmask_b32_e64 %0, %0, %8, s[2:3]\nv_cndmask_b32_e64 %1, %1, %8, s[2:3]\nv_cndmask_b32_e64 %2, %2, %8, s[2:3]\nv_cndmask_b32_e64 %3, %3, %8, s[2:3]\nv_cndmask_b32_e64 %4, %4, %8, s[2:3]\nv_cndmask_b32_e64 %5, %5, %8, s[2:3]\nv_cndmask_b32_e64 %6, %6, %8, s[2:3]\nv_cndmask_b32_e64 %7, %7, %8, s[2:3]\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k7(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k8(uint32_t*out,uint32_t seed){
  typedef float f2 __attribute__((ext_vector_type(2)));
  float b0=seed+threadIdx.x; f2 b={b0,b0+1}; f2 r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_mul_f32 %0, %0, %8\nv_pk_mul_f32 %1, %1, %8\nv_pk_mul_f32 %2, %2, %8\nv_pk_mul_f32 %3, %3, %8\nv_pk_mul_f32 %4, %4, %8\nv_pk_mul_f32 %5, %5, %8\nv_pk_mul_f32 %6, %6, %8\nv_pk_mul_f32 %7, %7, %8\nv_pk_mul_f32 %0, %0, %8\nv_pk_mul_f32 %1, %1, %8\nv_pk_mul_f32 %2, %2, %8\nv_pk_mul_f32 %3, %3, %8\nv_pk_mul_f32 %4, %4, %8\nv_pk_mul_f32 %5, %5, %8\nv_pk_mul_f32 %6, %6, %8\nv_pk_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  f2 x=r0+r1+r2+r3+r4+r5+r6+r7; out[blockIdx.x*256+threadIdx.x]=(uint32_t)(x.x+x.y);}
__global__ __launch_bounds__(256) void k9(uint32_t*out,uint32_t seed){
  typedef float f2 __attribute__((ext_vector_type(2)));
  float b0=seed+threadIdx.x; f2 b={b0,b0+1}; f2 r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_fma_f32 %0, %0, %8, %8\nv_pk_fma_f32 %1, %1, %8, %8\nv_pk_fma_f32 %2, %2, %8, %8\nv_pk_fma_f32 %3, %3, %8, %8\nv_pk_fma_f32 %4, %4, %8, %8\nv_pk_fma_f32 %5, %5, %8, %8\nv_pk_fma_f32 %6, %6, %8, %8\nv_pk_fma_f32 %7, %7, %8, %8\nv_pk_fma_f32 %0, %0, %8, %8\nv_pk_fma_f32 %1, %1, %8, %8\nv_pk_fma_f32 %2, %2, %8, %8\nv_pk_fma_f32 %3, %3, %8, %8\nv_pk_fma_f32 %4, %4, %8, %8\nv_pk_fma_f32 %5, %5, %8, %8\nv_pk_fma_f32 %6, %6, %8, %8\nv_pk_fma_f32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  f2 x=r0+r1+r2+r3+r4+r5+r6+r7; out[blockIdx.x*256+threadIdx.x]=(uint32_t)(x.x+x.y);}
__global__ __launch_bounds__(256) void k10(uint32_t*out,uint32_t seed){
  typedef float f2 __attribute__((ext_vector_type(2)));
  float b0=seed+threadIdx.x; f2 b={b0,b0+1}; f2 r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_fma_f32 %0, %8, %0, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %1, %8, %1, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %2, %8, %2, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %3, %8, %3, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %4, %8, %4, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %5, %8, %5, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %6, %8, %6, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %7, %8, %7, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %0, %8, %0, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %1, %8, %1, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %2, %8, %2, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %3, %8, %3, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %4, %8, %4, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %5, %8, %5, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %6, %8, %6, %8 op_sel_hi:[0,1,1]\nv_pk_fma_f32 %7, %8, %7, %8 op_sel_hi:[0,1,1]\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  f2 x=r0+r1+r2+r3+r4+r5+r6+r7; out[blockIdx.x*256+threadIdx.x]=(uint32_t)(x.x+x.y);}
__global__ __launch_bounds__(256) void k11(uint32_t*out,uint32_t seed){
  typedef float f2 __attribute__((ext_vector_type(2)));
  float b0=seed+threadIdx.x; f2 b={b0,b0+1}; f2 r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_add_f32 %0, %0, %8\nv_pk_add_f32 %1, %1, %8\nv_pk_add_f32 %2, %2, %8\nv_pk_add_f32 %3, %3, %8\nv_pk_add_f32 %4, %4, %8\nv_pk_add_f32 %5, %5, %8\nv_pk_add_f32 %6, %6, %8\nv_pk_add_f32 %7, %7, %8\nv_pk_add_f32 %0, %0, %8\nv_pk_add_f32 %1, %1, %8\nv_pk_add_f32 %2, %2, %8\nv_pk_add_f32 %3, %3, %8\nv_pk_add_f32 %4, %4, %8\nv_pk_add_f32 %5, %5, %8\nv_pk_add_f32 %6, %6, %8\nv_pk_add_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  f2 x=r0+r1+r2+r3+r4+r5+r6+r7; out[blockIdx.x*256+threadIdx.x]=(uint32_t)(x.x+x.y);}
__global__ __launch_bounds__(256) void k12(uint32_t*out,uint32_t seed){
  typedef float f2 __attribute__((ext_vector_type(2)));
  float b0=seed+threadIdx.x; f2 b={b0,b0+1}; f2 r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_mov_b64 %0, %8\nv_mov_b64 %1, %8\nv_mov_b64 %2, %8\nv_mov_b64 %3, %8\nv_mov_b64 %4, %8\nv_mov_b64 %5, %8\nv_mov_b64 %6, %8\nv_mov_b64 %7, %8\nv_mov_b64 %0, %8\nv_mov_b64 %1, %8\nv_mov_b64 %2, %8\nv_mov_b64 %3, %8\nv_mov_b64 %4, %8\nv_mov_b64 %5, %8\nv_mov_b64 %6, %8\nv_mov_b64 %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  f2 x=r0+r1+r2+r3+r4+r5+r6+r7; out[blockIdx.x*256+threadIdx.x]=(uint32_t)(x.x+x.y);}
__global__ __launch_bounds__(256) void k13(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_perm_b32 %1, %1, %8, %8\nv_perm_b32 %2, %2, %8, %8\nv_perm_b32 %3, %3, %8, %8\nv_perm_b32 %4, %4, %8, %8\nv_perm_b32 %5, %5, %8, %8\nv_perm_b32 %6, %6, %8, %8\nv_perm_b32 %7, %7, %8, %8\nv_perm_b32 %0, %0, %8, %8\nv_perm_b32 %1, %1, %8, %8\nv_perm_b32 %2, %2, %8, %8\nv_perm_b32 %3, %3, %8, %8\nv_perm_b32 %4, %4, %8, %8\nv_perm_b32 %5, %5, %8, %8\nv_perm_b32 %6, %6, %8, %8\nv_perm_b32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k14(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  asm volatile("s_mov_b64 s[2:3], -1" ::: "s2","s3");
  for(int it=0;it<ITERS;++it) asm volatile("v_bfi_b32 %0, %0, %8, %8\nv_bfi_b32 %1, %1, %8, %8\nv_bfi_b32 %2, %2, %8, %8\nv_bfi_b32 %3, %3, %8, %8\nv_bfi_b32 %4, %4, %8, %8\nv_bfi_b32 %5, %5, %8, %8\nv_bfi_b32 %6, %6, %8, %8\nv_bfi_b32 %7, %7, %8, %8\nv_bfi_b32 %0, %0, %8, %8\nv_bfi_b32 %1, %1, %8, %8\nv_bfi_b32 %2, %2, %8, %8\nv_bfi_b32 %3, %3, %8, %8\nv_bfi_b32 %4, %4, %8, %8\nv_bfi_b32 %5, %5, %8, %8\nv_bfi_b32 %6, %6, %8, %8\nv_bfi_b32 %7, %7, %8, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
__global__ __launch_bounds__(256) void k15(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_fmac_f32 %0, %8, %8\nv_mul_f32 %4, %4, %8\nv_fmac_f32 %1, %8, %8\nv_mul_f32 %5, %5, %8\nv_fmac_f32 %2, %8, %8\nv_mul_f32 %6, %6, %8\nv_fmac_f32 %3, %8, %8\nv_mul_f32 %7, %7, %8\nv_fmac_f32 %0, %8, %8\nv_mul_f32 %4, %4, %8\nv_fmac_f32 %1, %8, %8\nv_mul_f32 %5, %5, %8\nv_fmac_f32 %2, %8, %8\nv_mul_f32 %6, %6, %8\nv_fmac_f32 %3, %8, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b));
  out[blockIdx.x*256+threadIdx.x]=(uint32_t)(r0^r1^r2^r3^r4^r5^r6^r7);}
typedef void(*K)(uint32_t*,uint32_t);
K ks[]={k0,k1,k2,k3,k4,k5,k6,k7,k8,k9,k10,k11,k12,k13,k14,k15};
const char*names[]={"v_fmac_f32","v_fma_f32","v_mul_f32","v_cmp_e32_vcc","v_cmp_e64_sgpr","v_cndmask_e32","v_cndmask_e64","v_mov_b32_dpp","v_pk_mul_f32","v_pk_fma_f32","v_pk_fma_bcast","v_pk_add_f32","v_mov_b64","v_perm_b32","v_bfi_b32","mix_fmac_mul"};
int main(){uint32_t*out;hipMalloc(&out,256*256*8*4);
 for(int v=0;v<(int)(sizeof(ks)/sizeof(ks[0]));++v){ printf("%-20s",names[v]);
  for(int W: {2,4,8}){int blocks=256*W; hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   hipEvent_t e0,e1;hipEventCreate(&e0);hipEventCreate(&e1);hipEventRecord(e0);
   hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);hipEventRecord(e1);hipEventSynchronize(e1);
   float ms;hipEventElapsedTime(&ms,e0,e1); double ninst=(double)ITERS*16*blocks*4;
   printf("  W=%d %.2f", W, ms*1e-3*2.4e9/(ninst/1024));}
  printf("\n");}
 return 0;}
