#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
constexpr int ITERS=2048;
__global__ __launch_bounds__(256) void k0(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k1(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k2(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\nv_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k3(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k4(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k5(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\nv_pk_max_u16 %0, %0, %8\nv_pk_max_u16 %1, %1, %8\nv_pk_max_u16 %2, %2, %8\nv_pk_max_u16 %3, %3, %8\nv_pk_max_u16 %4, %4, %8\nv_pk_max_u16 %5, %5, %8\nv_pk_max_u16 %6, %6, %8\nv_pk_max_u16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k6(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_u32 %0, %0, %8\nv_sub_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_sub_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_sub_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_sub_u32 %7, %7, %8\nv_add_u32 %0, %0, %8\nv_sub_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_sub_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_sub_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_sub_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k7(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_u32 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_xor_b32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_xor_b32 %7, %7, %8\nv_add_u32 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_xor_b32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_xor_b32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k8(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_pk_maximum3_f16 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\nv_pk_maximum3_f16 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_pk_maximum3_f16 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_pk_maximum3_f16 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_pk_maximum3_f16 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k9(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_perm_b32 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\nv_perm_b32 %0, %0, %8, %8\nv_add_u32 %1, %1, %8\nv_perm_b32 %2, %2, %8, %8\nv_add_u32 %3, %3, %8\nv_perm_b32 %4, %4, %8, %8\nv_add_u32 %5, %5, %8\nv_perm_b32 %6, %6, %8, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k10(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_i16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_i16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_i16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_i16 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_max_i16 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_i16 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_i16 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_i16 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k11(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_i16 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_max_i16 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_max_i16 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_max_i16 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_max_i16 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k12(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_add_f32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_f32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_f32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_f32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_add_f32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_f32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_f32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_f32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k13(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_add_u32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
__global__ __launch_bounds__(256) void k14(uint32_t*out,uint32_t seed){
  uint32_t b=seed+threadIdx.x; uint32_t r0=b,r1=b+1,r2=b+2,r3=b+3,r4=b+4,r5=b+5,r6=b+6,r7=b+7;
  for(int it=0;it<ITERS;++it) asm volatile("v_max_u32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_mul_f32 %7, %7, %8\nv_max_u32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_max_u32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_mul_f32 %7, %7, %8\n":"+v"(r0),"+v"(r1),"+v"(r2),"+v"(r3),"+v"(r4),"+v"(r5),"+v"(r6),"+v"(r7):"v"(b):"vcc");
  out[blockIdx.x*256+threadIdx.x]=r0^r1^r2^r3^r4^r5^r6^r7;}
typedef void(*KF)(uint32_t*,uint32_t);
KF ks[]={k0,k1,k2,k3,k4,k5,k6,k7,k8,k9,k10,k11,k12,k13,k14};
const char*names[]={"alt pk/add","4pk 4add x2","8pk 8add","2pk 2add x4","16 add","16 pk","alt add/sub","alt add/xor","alt max3f/add","alt perm/add","alt max_i16/add","alt max_u32/max_i16","alt add_f32/add_u32","alt max_u32/add_u32","alt max_u32/mul_f32"};
int main(){uint32_t*out;(void)hipMalloc(&out,256*256*8*4);
 for(int v=0;v<(int)(sizeof(ks)/sizeof(ks[0]));++v){ printf("%-24s",names[v]);
  for(int W: {2,4,8}){int blocks=256*W; hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   hipEvent_t e0,e1;(void)hipEventCreate(&e0);(void)hipEventCreate(&e1);(void)hipEventRecord(e0);
   for(int rep=0;rep<3;++rep) hipLaunchKernelGGL(ks[v],dim3(blocks),dim3(256),0,0,out,1u);
   (void)hipEventRecord(e1);(void)hipEventSynchronize(e1);
   float ms;(void)hipEventElapsedTime(&ms,e0,e1); double ninst=3.0*ITERS*16*blocks*4;
   printf("  W=%d %.2f", W, ms*1e-3*2.4e9/(ninst/1024));}
  printf("   cyc/inst/SIMD\n");}
 return 0;}