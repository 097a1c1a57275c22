// Issue-rate microbenchmark of the VALU ops the wavefront kernels use (gfx950).
// Each wave runs ITERS x 16 instructions; reports shader cycles per wave
// instruction per SIMD (s_memtime) for W resident waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int ITERS = 4096;

#define BODY16(INS)                                                                        \
    asm volatile(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
                 INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n" \
                 INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
                 INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n" \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(b))
#define DEP16(INS)                                                                          \
    asm volatile(INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" \
                 INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" \
                 INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" \
                 INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" INS " %0, %0, %1\n" \
                 : "+v"(r0) : "v"(b))

template <int V>
__global__ __launch_bounds__(256) void ub(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t b = seed + threadIdx.x;
    uint32_t r0 = b, r1 = b + 1, r2 = b + 2, r3 = b + 3, r4 = b + 4, r5 = b + 5, r6 = b + 6, r7 = b + 7;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        if (V == 0) BODY16("v_pk_max_i16");
        if (V == 1) BODY16("v_max_i32");
        if (V == 2) BODY16("v_pk_add_u16");
        if (V == 3) BODY16("v_pk_sub_u16");
        if (V == 4) DEP16("v_pk_max_i16");
        if (V == 5) DEP16("v_max_i32");
        if (V == 6) BODY16("v_add_u32");
        if (V == 7) BODY16("v_pk_min_u16");
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    const char *names[] = {"v_pk_max_i16 indep", "v_max_i32 indep", "v_pk_add_u16 indep", "v_pk_sub_u16 indep",
                           "v_pk_max_i16 dep", "v_max_i32 dep", "v_add_u32 indep", "v_pk_min_u16 indep"};
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 256 * 8 * cus * sizeof(uint32_t) * 2);
    hipMalloc(&cyc, 4 * 8 * cus * sizeof(uint64_t) * 2);
    uint64_t *h = (uint64_t *)malloc(4 * 8 * cus * sizeof(uint64_t) * 2);
    void (*ks[])(uint32_t *, uint64_t *, uint32_t) = {ub<0>, ub<1>, ub<2>, ub<3>, ub<4>, ub<5>, ub<6>, ub<7>};
    printf("CUs %d\n", cus);
    for (int v = 0; v < 8; ++v) {
        for (int W : {1, 2, 3, 4, 8}) {
            const int blocks = cus * W;
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, out, cyc, 1u);
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, out, cyc, 1u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h, cyc, blocks * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost);
            double avg = 0;
            for (int i = 0; i < blocks * 4; ++i) avg += h[i];
            avg /= blocks * 4;
            const double ninst = (double)ITERS * 16;
            // s_memtime cycles per instruction of one wave; SIMD cost = that / W
            printf("%-20s W=%d  wave cyc/inst %.2f  SIMD cyc/inst %.2f  ms %.3f  lane-ops/s %.2fT\n", names[v], W,
                   avg / ninst, avg / ninst / W, ms, ninst * 64 * 4 * blocks / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
