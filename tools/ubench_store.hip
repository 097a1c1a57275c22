// ubench_store.hip — write bandwidth of 8-byte-per-lane stores on gfx950, to price the
// direction-flag stream of the packed traceback kernels (profiles/r02_tb_store_ab.md).
// Each wave writes `iters` rounds of 64 x 8 B; pattern 0: one 512-byte run per store,
// pattern 1: four 128-byte runs 40 KB apart (lane groups of different pairs);
// `valu` independent VALU ops between stores model the DP work around them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void st(uint2 *out, uint32_t iters, int pattern, int valu, uint64_t wave_span) {
    const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
    uint2 *base = out + (uint64_t)wave * wave_span;
    uint32_t a = lane, b = lane * 3u;
    for (uint32_t i = 0; i < iters; ++i) {
        for (int v = 0; v < valu; ++v) { a = a * 5u + b; b ^= a >> 3; }
        uint64_t off = pattern == 0 ? (uint64_t)i * 64 + lane
                                    : (uint64_t)(lane >> 4) * (wave_span / 4) + (uint64_t)i * 16 + (lane & 15);
        base[off] = make_uint2(a, b + i);
    }
}

int main(int argc, char **argv) {
    const int pattern = argc > 1 ? atoi(argv[1]) : 0, valu = argc > 2 ? atoi(argv[2]) : 0;
    const uint32_t waves = 12500 * 2, iters = 1600;   // 25 K waves x 1600 x 512 B = 20.5 GB? scaled below
    const uint32_t it = iters / 4;                     // 5.1 GB total
    const uint64_t span = (uint64_t)it * 64;           // uint2 per wave
    uint2 *d;
    if (hipMalloc(&d, (uint64_t)waves * span * 8 + 64)) { printf("alloc failed\n"); return 1; }
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int r = 0; r < 4; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(st, dim3(waves / 4), dim3(256), 0, 0, d, it, pattern, valu, span);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0; hipEventElapsedTime(&ms, e0, e1);
        const double bytes = (double)waves * it * 512;
        printf("pattern %d valu %d: %.3f ms, %.2f GB, %.2f TB/s\n", pattern, valu, ms, bytes / 1e9, bytes / ms / 1e9);
    }
    hipFree(d);
    return 0;
}
