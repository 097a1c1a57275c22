// ubench_issue.hip — VALU issue cost per wave64 instruction on one SIMD (gfx950), measured the
// way /opt/skills/guides/MI355X_MICROARCH.md prescribes: independent instructions, 16 chains,
// every source operand in a different VGPR bank from the destination (bank = index % 4; the
// registers are named in the asm, v32..v63, and declared clobbered), timed in shader cycles
// by s_memtime inside the kernel (no assumed clock, no launch overhead).  W waves per SIMD
// (W blocks of 4 waves per CU): cycles per instruction per SIMD = wave cycles / (W * count).
// W = 1 is one wave's own issue cost (the guide's "one wave alone"), W >= 2 the SIMD's rate.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_issue.hip -o tools/ubench_issue
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int ITERS = 512;
constexpr int PER_ITER = 32;   // 16 chains, the body twice (packed fp32: 8 pair chains, the body four times)

#define CLOB                                                                                               \
    "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", \
        "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60",    \
        "v61", "v62", "v63"

// chain d in v32..v47; sources from v48..v63 at banks d+1, d+2 (mod 4)
#define S2(op, d, s) op " v" #d ", v" #d ", v" #s "\n"
#define S3(op, d, s, t) op " v" #d ", v" #d ", v" #s ", v" #t "\n"
#define BODY2(op)                                                                                           \
    S2(op, 32, 49) S2(op, 33, 50) S2(op, 34, 51) S2(op, 35, 52) S2(op, 36, 53) S2(op, 37, 54) S2(op, 38, 55) \
    S2(op, 39, 56) S2(op, 40, 57) S2(op, 41, 58) S2(op, 42, 59) S2(op, 43, 60) S2(op, 44, 61) S2(op, 45, 62) \
    S2(op, 46, 63) S2(op, 47, 48)
#define BODY3(op)                                                                                           \
    S3(op, 32, 49, 50) S3(op, 33, 50, 51) S3(op, 34, 51, 52) S3(op, 35, 52, 53) S3(op, 36, 53, 54)         \
    S3(op, 37, 54, 55) S3(op, 38, 55, 56) S3(op, 39, 56, 57) S3(op, 40, 57, 58) S3(op, 41, 58, 59)         \
    S3(op, 42, 59, 60) S3(op, 43, 60, 61) S3(op, 44, 61, 62) S3(op, 45, 62, 63) S3(op, 46, 63, 48)         \
    S3(op, 47, 48, 49)
// the same three-source ops with every operand in the destination's bank (bank conflicts)
#define BODY3C(op)                                                                                          \
    S3(op, 32, 48, 52) S3(op, 33, 49, 53) S3(op, 34, 50, 54) S3(op, 35, 51, 55) S3(op, 36, 56, 60)         \
    S3(op, 37, 57, 61) S3(op, 38, 58, 62) S3(op, 39, 59, 63) S3(op, 40, 48, 52) S3(op, 41, 49, 53)         \
    S3(op, 42, 50, 54) S3(op, 43, 51, 55) S3(op, 44, 56, 60) S3(op, 45, 57, 61) S3(op, 46, 58, 62)         \
    S3(op, 47, 59, 63)
// packed fp32 (64-bit register pairs): 8 chains, each counted once, the body four times
#define P2(op, d, e, s, t) op " v[" #d ":" #e "], v[" #d ":" #e "], v[" #s ":" #t "]\n"
#define P3(op, d, e, s, t, u, v) op " v[" #d ":" #e "], v[" #d ":" #e "], v[" #s ":" #t "], v[" #u ":" #v "]\n"
#define BODYP2(op)                                                                                          \
    P2(op, 32, 33, 50, 51) P2(op, 34, 35, 52, 53) P2(op, 36, 37, 54, 55) P2(op, 38, 39, 56, 57)              \
    P2(op, 40, 41, 58, 59) P2(op, 42, 43, 60, 61) P2(op, 44, 45, 62, 63) P2(op, 46, 47, 48, 49)
#define BODYP3(op)                                                                                          \
    P3(op, 32, 33, 50, 51, 54, 55) P3(op, 34, 35, 52, 53, 58, 59) P3(op, 36, 37, 54, 55, 58, 59)             \
    P3(op, 38, 39, 56, 57, 60, 61) P3(op, 40, 41, 58, 59, 62, 63) P3(op, 42, 43, 60, 61, 48, 49)             \
    P3(op, 44, 45, 62, 63, 50, 51) P3(op, 46, 47, 48, 49, 52, 53)
#define INIT                                                                                                \
    "v_mov_b32 v32, 0x3c003c00\nv_mov_b32 v33, 0x3c003c00\nv_mov_b32 v34, 0x3c003c00\nv_mov_b32 v35, 0x3c003c00\nv_mov_b32 v36, 0x3c003c00\n"          \
    "v_mov_b32 v37, 0x3c003c00\nv_mov_b32 v38, 0x3c003c00\nv_mov_b32 v39, 0x3c003c00\nv_mov_b32 v40, 0x3c003c00\nv_mov_b32 v41, 0x3c003c00\n"         \
    "v_mov_b32 v42, 0x3c003c00\nv_mov_b32 v43, 0x3c003c00\nv_mov_b32 v44, 0x3c003c00\nv_mov_b32 v45, 0x3c003c00\nv_mov_b32 v46, 0x3c003c00\n"     \
    "v_mov_b32 v47, 0x3c003c00\nv_mov_b32 v48, 0x3c003c00\nv_mov_b32 v49, 0x3c003c00\nv_mov_b32 v50, 0x3c003c00\n" \
    "v_mov_b32 v51, 0x3c003c00\nv_mov_b32 v52, 0x3c003c00\nv_mov_b32 v53, 0x3c003c00\n"                 \
    "v_mov_b32 v54, 0x3c003c00\nv_mov_b32 v55, 0x3c003c00\nv_mov_b32 v56, 0x3c003c00\n"                 \
    "v_mov_b32 v57, 0x3c003c00\nv_mov_b32 v58, 0x3c003c00\nv_mov_b32 v59, 0x3c003c00\n"                 \
    "v_mov_b32 v60, 0x3c003c00\nv_mov_b32 v61, 0x3c003c00\nv_mov_b32 v62, 0x3c003c00\n"                 \
    "v_mov_b32 v63, 0x3c003c00\n"

#define KERNEL(name, body)                                                               \
    __global__ __launch_bounds__(256) void name(long long *cyc) {                        \
        asm volatile(INIT ::: CLOB);                                                     \
        const long long t0 = clock64();                                                  \
        for (int it = 0; it < ITERS; ++it) asm volatile(body body ::: CLOB);             \
        const long long t1 = clock64();                                                  \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0; \
    }

KERNEL(k_add_u32, BODY2("v_add_u32"))
KERNEL(k_sub_u32, BODY2("v_sub_u32"))
KERNEL(k_and_b32, BODY2("v_and_b32"))
KERNEL(k_max_i32, BODY2("v_max_i32"))
KERNEL(k_lshlrev_b32, BODY2("v_lshlrev_b32"))
KERNEL(k_add_f32, BODY2("v_add_f32"))
KERNEL(k_mul_f32, BODY2("v_mul_f32"))
KERNEL(k_max_f32, BODY2("v_max_f32"))
KERNEL(k_fma_f32, BODY3("v_fma_f32"))
KERNEL(k_fmac_f32, BODY2("v_fmac_f32"))
KERNEL(k_add3_u32, BODY3("v_add3_u32"))
KERNEL(k_max3_i32, BODY3("v_max3_i32"))
KERNEL(k_perm_b32, BODY3("v_perm_b32"))
KERNEL(k_bitop3_b32, BODY3("v_and_or_b32"))
KERNEL(k_pk_add_u16, BODY2("v_pk_add_u16"))
KERNEL(k_pk_sub_i16, BODY2("v_pk_sub_i16"))
KERNEL(k_pk_max_u16, BODY2("v_pk_max_u16"))
KERNEL(k_pk_mad_u16, BODY3("v_pk_mad_u16"))
KERNEL(k_pk_max_f16, BODY2("v_pk_max_f16"))
KERNEL(k_pk_maximum3_f16, BODY3("v_pk_maximum3_f16"))
KERNEL(k_fma_f32_conflict, BODY3C("v_fma_f32"))
KERNEL(k_pk_fma_f32, BODYP3("v_pk_fma_f32") BODYP3("v_pk_fma_f32"))
KERNEL(k_pk_mul_f32, BODYP2("v_pk_mul_f32") BODYP2("v_pk_mul_f32"))
KERNEL(k_pk_add_f32, BODYP2("v_pk_add_f32") BODYP2("v_pk_add_f32"))

typedef void (*Fn)(long long *);
static const Fn ks[] = {k_add_u32,   k_sub_u32,    k_and_b32,   k_max_i32,    k_lshlrev_b32, k_add_f32,
                        k_mul_f32,   k_max_f32,    k_fma_f32,   k_fmac_f32,   k_add3_u32,    k_max3_i32,
                        k_perm_b32,  k_bitop3_b32, k_pk_add_u16, k_pk_sub_i16, k_pk_max_u16, k_pk_mad_u16,
                        k_pk_max_f16, k_pk_maximum3_f16, k_fma_f32_conflict, k_pk_fma_f32, k_pk_mul_f32,
                        k_pk_add_f32};
static const char *names[] = {"v_add_u32",    "v_sub_u32",    "v_and_b32",    "v_max_i32",     "v_lshlrev_b32",
                              "v_add_f32",    "v_mul_f32",    "v_max_f32",    "v_fma_f32",     "v_fmac_f32",
                              "v_add3_u32",   "v_max3_i32",   "v_perm_b32",   "v_and_or_b32",  "v_pk_add_u16",
                              "v_pk_sub_i16", "v_pk_max_u16", "v_pk_mad_u16", "v_pk_max_f16",  "v_pk_maximum3_f16",
                              "v_fma_f32_bank_conflict", "v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32"};

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    long long *cyc;
    hipMalloc(&cyc, (size_t)cus * 8 * 4 * sizeof(long long));
    printf("{\"cus\": %d, \"iters\": %d, \"per_iter\": %d, \"unit\": \"cycles per wave64 instruction per SIMD "
           "(s_memtime, median over waves)\", \"ops\": {",
           cus, ITERS, PER_ITER);
    const int n = (int)(sizeof(ks) / sizeof(ks[0]));
    for (int v = 0; v < n; ++v) {
        printf("%s\"%s\": {", v ? ", " : "", names[v]);
        const int Ws[] = {1, 2, 4, 8};
        for (int wi = 0; wi < 4; ++wi) {
            const int W = Ws[wi], blocks = cus * W;
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, cyc);   // warm-up
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, cyc);
            hipDeviceSynchronize();
            std::vector<long long> h((size_t)blocks * 4);
            hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.end());
            const double med = (double)h[h.size() / 2];
            const double per = med / ((double)ITERS * PER_ITER * W);
            printf("%s\"W%d\": %.3f", wi ? ", " : "", W, per);
        }
        printf("}");
    }
    printf("}}\n");
    return 0;
}
