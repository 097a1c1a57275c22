// rclass.hip — the WITH_START reverse passes (start.hpp) with the register axis sized per block.
//
// A packed wavefront instance covers G*R register-axis positions (the query for LOCAL, the
// target for SEMI); a lane runs all R of its rows on every step whether or not they hold a real
// base.  The reverse pass's register-axis lengths vary from pair to pair (SEMI: the reversed
// target L = tl - 8*gend_reg, 151..182 for config 4; LOCAL: the query words up to the end
// cell, 8..152 for config 2), and its slots are sorted so that a block's pairs have one length
// class (start.hpp rev_bucket).  These kernels hold the kernel body (wf16_body.inc) for several
// R and run, per block, the smallest R whose G*R covers the block's longest padded register
// axis: the same cells, results and tie-breaks as the largest instance (a pair's pad rows hold
// N past its length in both), with R rows of work per step instead of the maximum.  The
// block's choice is uniform: every wave reads the same lengths.
#include "wavefront16.hpp"

namespace gx {

// the block's longest padded register axis.  The reverse pass's slots are sorted longest first
// by exactly these words (start.hpp rev_bucket: SEMI the reversed target's, LOCAL the reversed
// query's first), so it is the block's first slot's: two scalar loads (A.perm_xkey).  Otherwise
// the maximum over the block's slots.  (A pair longer than the chosen G*R declines its block to the
// int32 kernel: wf16_body.inc's `other`.)
template <int ALGO_, int G>
__device__ __forceinline__ uint32_t block_xpad(const WfArgs &A) {
    constexpr bool TR = ALGO_ == WF16_SEMI_STOP;   // SEMI: X = target
    constexpr uint32_t ppb = kWavesPerBlock * 2 * (64 / G);
    const uint32_t base = blockIdx.x * ppb;
    if (A.perm && A.perm_xkey) {
        const uint32_t p0 = A.perm[base];
        return ((TR ? A.tlen[p0] : A.qlen[p0]) + 7u) & ~7u;
    }
    // unsorted, or sorted by another key (LOCAL's slot sort drops the query key when its
    // two-key histogram would not fit LDS): the maximum over the block's slots
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t m = 0;
    for (uint32_t i = lane; i < ppb; i += 64) {
        const uint32_t idx = base + i;
        if (idx < A.n) {
            const uint32_t pr = A.perm ? A.perm[idx] : idx;
            m = max(m, ((TR ? A.tlen[pr] : A.qlen[pr]) + 7u) & ~7u);
        }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) m = max(m, (uint32_t)__shfl_xor(m, s));
    return m;
}

// Two forms of the class kernel, R0 < R1 < ... ascending (0 = unused), the largest the plan's
// instance (it covers every slot):
//  * wf16_rclass_kernel: one copy of the kernel body (wf16_body.inc) per R, each in its own
//    block scope of the kernel -- the SEMI reverse pass (as a device function its sweep issued
//    more instructions per step, as wf16_kernel's did);
//  * wf16_rclass_fn_kernel: the body as a device function per R -- the LOCAL reverse pass (in
//    block scopes the R = 19 sweep spilled, 80 B per lane, 8 scratch accesses per loop trip).
template <int ALGO_, int G, int R0, int R1, int R2, int R3, int R4, int R5>
__global__ __launch_bounds__(kBlock, wf16_waves(ALGO_, R5 ? R5 : R4 ? R4 : R3)) void wf16_rclass_kernel(WfArgs A) {
    const uint32_t need = block_xpad<ALGO_, G>(A);
    const uint32_t wf16_bid = blockIdx.x, wf16_bl = blockIdx.x, wf16_p0 = 0, wf16_lds = A.lds_stride;
    if (need <= (uint32_t)(G * R0)) {
        constexpr int R = R0;
#include "wf16_body.inc"
    } else if (need <= (uint32_t)(G * R1)) {
        constexpr int R = R1;
#include "wf16_body.inc"
    } else if (need <= (uint32_t)(G * R2)) {
        constexpr int R = R2;
#include "wf16_body.inc"
    } else if (R4 == 0 || need <= (uint32_t)(G * R3)) {
        constexpr int R = R3;
#include "wf16_body.inc"
    } else if constexpr (R4 != 0) {
        if (R5 == 0 || need <= (uint32_t)(G * R4)) {
            constexpr int R = R4;
#include "wf16_body.inc"
        } else if constexpr (R5 != 0) {
            constexpr int R = R5;
#include "wf16_body.inc"
        }
    }
}

template <int ALGO_, int G, int R>
__device__ __attribute__((always_inline)) void wf16_body(const WfArgs &A) {
    const uint32_t wf16_bid = blockIdx.x, wf16_bl = blockIdx.x, wf16_p0 = 0, wf16_lds = A.lds_stride;
#include "wf16_body.inc"
}

template <int... Rs>
constexpr int rmax() {
    int m = 0;
    ((m = Rs > m ? Rs : m), ...);
    return m;
}

template <int ALGO_, int G, int... Rs>
__global__ __launch_bounds__(kBlock, wf16_waves(ALGO_, rmax<Rs...>())) void wf16_rclass_fn_kernel(WfArgs A) {
    const uint32_t need = block_xpad<ALGO_, G>(A);
    bool done = false;
    ((done ? void() : need <= (uint32_t)(G * Rs) ? (wf16_body<ALGO_, G, Rs>(A), done = true, void()) : void()), ...);
}

// The class sets, by the plan's instance (NULL: no class kernel, the plan's instance runs):
//  * SEMI TAIL=TARGET reverse pass, G = 8 up to 184 target columns: every padded length
//    152..184 of config 4 has its own R;
//  * LOCAL reverse pass (f16 / u16 keys), G = 8 up to 152 query rows.
Wf16Fn wf16_rclass_lookup(int algo, int G, int R) {
    if (G != 8) return nullptr;
    if (algo == WF16_SEMI_STOP && R == 23) return &wf16_rclass_kernel<WF16_SEMI_STOP, 8, 16, 19, 20, 21, 22, 23>;
    if (algo == WF16_LOCAL_RS && R == 19) return &wf16_rclass_fn_kernel<WF16_LOCAL_RS, 8, 4, 8, 12, 16, 19>;
    if (algo == WF16_LOCAL_U16_RS && R == 19) return &wf16_rclass_fn_kernel<WF16_LOCAL_U16_RS, 8, 4, 8, 12, 16, 19>;
    return nullptr;
}

}  // namespace gx
