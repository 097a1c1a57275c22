// wavefront16.hpp — packed-int16 segmented wavefront for LOCAL score + ends.
//
// Same sweep as wavefront.hpp (G lanes per group, R query rows per lane, one
// column per step, DPP wave_shr:1 hand-off), but every VGPR holds TWO pairs:
// the low 16 bits belong to pair 2*slot and the high 16 bits to pair
// 2*slot+1, so each v_pk_* instruction advances two DP cells.  The cell
// update is GASAL2's CORE_LOCAL_COMPUTE (local_kernel_template.h:19-30):
//   tmp = H(r-1,c-1) + s;  H = max(tmp, F, E, 0);
//   E'  = max(tmp - OE, E - e);  F' = max(tmp - OE, F - e)
// with E and F kept clamped at 0 (max(E,0) obeys the same recurrence when
// e >= 0, and values below 0 never reach H), so H = max(tmp, F, E) and the
// gap decay is one saturating v_pk_sub_u16.  The per-row maximum is tracked
// as a 16-bit key (H << 8 | 255 - c); the strip-major first maximum (SURVEY
// Q1) is resolved at the end exactly as in the int32 kernel.
//
// Exactness domain (checked by the planner): every H <= 255 (a * min(ql,tl)),
// padded targets <= 256 columns, e >= 0, o + e <= 16000.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wavefront.hpp"

namespace gx {

typedef short pk_s2 __attribute__((ext_vector_type(2)));
typedef unsigned short pk_u2 __attribute__((ext_vector_type(2)));
#define GX_AS(T, x) __builtin_bit_cast(T, x)

// Plain vector expressions; the "1" of pk_min_u16 arrives as a kernel
// argument so the compiler cannot turn min(x,1)*D + M into compare/select.
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, __builtin_elementwise_min(GX_AS(pk_u2, a), GX_AS(pk_u2, b)));
}
__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t b, uint32_t c) {
    return GX_AS(uint32_t, GX_AS(pk_u2, a) * GX_AS(pk_u2, b) + GX_AS(pk_u2, c));
}
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, __builtin_elementwise_max(GX_AS(pk_s2, a), GX_AS(pk_s2, b)));
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, __builtin_elementwise_max(GX_AS(pk_u2, a), GX_AS(pk_u2, b)));
}
__device__ __forceinline__ uint32_t pk_subsat_u16(uint32_t a, uint32_t b) {   // max(a - b, 0), a,b >= 0
    return GX_AS(uint32_t, __builtin_elementwise_sub_sat(GX_AS(pk_u2, a), GX_AS(pk_u2, b)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, GX_AS(pk_s2, a) + GX_AS(pk_s2, b));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, GX_AS(pk_s2, a) - GX_AS(pk_s2, b));
}
__device__ __forceinline__ uint32_t pk_bcast(int32_t v) { return ((uint32_t)v & 0xFFFFu) * 0x10001u; }

#ifndef GX_WF16_WAVES
#define GX_WF16_WAVES 3   // waves per SIMD the register allocator must allow
#endif

constexpr uint32_t kPkInvalid = 0xFFu;   // target/query code outside the padded grid
constexpr int32_t kPkNeg = -16384;       // substitution score of an outside cell

// One column step: rows read the previous column's H from Hin and write the
// new H to Hout (ping-pong arrays, so no register copies on the back edge).
template <int R, bool EXACT>
__device__ __forceinline__ void wf16_step(const uint32_t t, const int32_t c, const uint32_t diag_top,
                                          const uint32_t f_top, const uint32_t (&q)[R],
                                          const uint32_t (&Hin)[R], uint32_t (&Hout)[R], uint32_t (&Ek)[R],
                                          uint32_t (&key)[R], uint32_t &f_out, const uint32_t OEp,
                                          const uint32_t EXTp, const uint32_t NVALp, const uint32_t Ap,
                                          const uint32_t NSp, const uint32_t DAp, const uint32_t ONEp) {
    const uint32_t INVp = 0x00FF00FFu;
    const uint32_t NEGp = pk_bcast(kPkNeg);
    // per-column substitution constants, per half:
    //   ordinary base : M = a,   D = -(a+b)   (s = M + D * [q != t])
    //   N (N_CODE)    : M = NS,  D = 0
    //   outside grid  : M = NEG, D = 0
    const uint32_t notN = pk_min_u16(t ^ NVALp, ONEp);
    const uint32_t notI = pk_min_u16(t ^ INVp, ONEp);
    const uint32_t live = pk_mad_u16(notN, notI, 0u);
    uint32_t M = pk_mad_u16(notI, pk_sub(pk_mad_u16(notN, pk_sub(Ap, NSp), NSp), NEGp), NEGp);
    uint32_t D = pk_mad_u16(live, DAp, 0u);
    uint32_t NSt = 0;
    if (EXACT) NSt = pk_mad_u16(notI, pk_sub(NSp, NEGp), NEGp);   // query-N score this column
    // opaque per-column constants: keeps the compiler from re-deriving them per row
    asm volatile("" : "+v"(M), "+v"(D), "+v"(NSt));
    const bool kc = c >= 0 && c < 256;
    const uint32_t invc = kc ? pk_bcast(255 - c) : 0u;
    const uint32_t kmul = kc ? (ONEp << 8) : 0u;                  // key = H*256 + 255-c
    uint32_t diag = diag_top, f = f_top;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t mis = pk_min_u16(q[k] ^ t, ONEp);
        uint32_t sc = pk_mad_u16(mis, D, M);
        if (EXACT) {   // LOCAL N rule for query N (pad rows included): s = NSt
            const uint32_t isN = ONEp ^ pk_min_u16(q[k] ^ NVALp, ONEp);
            sc = pk_mad_u16(isN, pk_sub(NSt, sc), sc);
        }
        const uint32_t tmp = pk_add(diag, sc);
        const uint32_t H = pk_max_i16(pk_max_i16(tmp, f), Ek[k]);
        const uint32_t toe = pk_sub(tmp, OEp);
        Ek[k] = pk_max_i16(toe, pk_subsat_u16(Ek[k], EXTp));
        f = pk_max_i16(toe, pk_subsat_u16(f, EXTp));
        key[k] = pk_max_u16(key[k], pk_mad_u16(H, kmul, invc));
        diag = Hin[k];
        Hout[k] = H;
    }
    f_out = f;
}

template <int G, int R, bool EXACT>
__device__ __forceinline__ void wf16_body(const WfArgs &A, const uint32_t *tcol, const uint32_t lg,
                                          const uint32_t nsteps, const uint32_t (&q)[R],
                                          uint32_t (&key)[R]) {
    const uint32_t OEp = pk_bcast(A.o + A.e);
    const uint32_t EXTp = pk_bcast(A.e);
    const uint32_t NVALp = pk_bcast(A.nval);
    const int32_t NS = A.has_npen ? -A.npen : 0;
    const uint32_t Ap = pk_bcast(A.a), NSp = pk_bcast(NS);
    const uint32_t DAp = pk_bcast(-(A.a + A.b));
    const uint32_t ONEp = A.one;
    uint32_t HA[R], HB[R], Ek[R];
#pragma unroll
    for (int k = 0; k < R; ++k) { HA[k] = 0; HB[k] = 0; Ek[k] = 0; key[k] = 0; }
    uint32_t recvH = 0, prevRecvH = 0, recvF = 0, f = 0;
    const bool top = lg == 0;
    int32_t c = -(int32_t)lg;
    uint32_t tnext = tcol[c + G];
    // two columns per iteration (the odd tail step reads only "outside" columns)
    for (uint32_t s = 0; s < nsteps; s += 2, c += 2) {
        uint32_t t = tnext;
        tnext = tcol[c + 1 + G];
        wf16_step<R, EXACT>(t, c, top ? 0u : prevRecvH, top ? 0u : recvF, q, HA, HB, Ek, key, f, OEp, EXTp,
                            NVALp, Ap, NSp, DAp, ONEp);
        prevRecvH = recvH;
        recvH = (uint32_t)shr_lane((int32_t)HB[R - 1]);
        recvF = (uint32_t)shr_lane((int32_t)f);
        t = tnext;
        tnext = tcol[c + 2 + G];
        wf16_step<R, EXACT>(t, c + 1, top ? 0u : prevRecvH, top ? 0u : recvF, q, HB, HA, Ek, key, f, OEp,
                            EXTp, NVALp, Ap, NSp, DAp, ONEp);
        prevRecvH = recvH;
        recvH = (uint32_t)shr_lane((int32_t)HA[R - 1]);
        recvF = (uint32_t)shr_lane((int32_t)f);
    }
}

template <int G, int R>
__global__ __launch_bounds__(kBlock, GX_WF16_WAVES) void wf16_local_kernel(WfArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int S = 64 / G;            // lane groups per wave
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1), slot = lane / G;
    const uint32_t pair0 = (blockIdx.x * kWavesPerBlock + wave) * (2 * S);
    uint32_t pr[2], ql[2], tl[2], qo[2], to[2], qpad[2], tpad[2];
    bool valid[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        pr[h] = pair0 + 2 * slot + h;
        valid[h] = pr[h] < A.n;
        ql[h] = valid[h] ? A.qlen[pr[h]] : 0;
        tl[h] = valid[h] ? A.tlen[pr[h]] : 0;
        qo[h] = valid[h] ? A.qoff[pr[h]] : 0;
        to[h] = valid[h] ? A.toff[pr[h]] : 0;
        qpad[h] = (ql[h] + 7u) & ~7u;
        tpad[h] = (tl[h] + 7u) & ~7u;
    }
    uint32_t tmaxw = max(tpad[0], tpad[1]);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) tmaxw = max(tmaxw, (uint32_t)__shfl_xor(tmaxw, m));
    // ---- stage both pairs' targets, one uint32 per column (lo: pair 0, hi: pair 1),
    //      columns [-G, tmaxw + G) so that out-of-range steps read "outside" ----
    const uint32_t words = A.lds_stride >> 2;            // >= tmaxw + 2G + 4, multiple of 4
    uint32_t *wl = reinterpret_cast<uint32_t *>(lds) + (size_t)wave * S * words;
    for (uint32_t base = 0; base < S * (words >> 2); base += 64) {
        const uint32_t idx = base + lane;
        const uint32_t ps = min(idx / (words >> 2), (uint32_t)S - 1);
        const uint32_t c0 = 4 * (idx - ps * (words >> 2)) - G;   // first column of this quad
        uint32_t v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t tp = __shfl(tpad[h], ps * G), tof = __shfl(to[h], ps * G);
            v[h] = 0xFFFFFFFFu;
            if ((int32_t)c0 >= 0 && c0 < tp) v[h] = load4_codes(A.t, tof, c0 >> 2, A.packed);
        }
        if (idx < S * (words >> 2)) {
            uint4 w;
            w.x = (v[0] & 0xFFu) | ((v[1] & 0xFFu) << 16);
            w.y = ((v[0] >> 8) & 0xFFu) | (((v[1] >> 8) & 0xFFu) << 16);
            w.z = ((v[0] >> 16) & 0xFFu) | (((v[1] >> 16) & 0xFFu) << 16);
            w.w = (v[0] >> 24) | ((v[1] >> 24) << 16);
            reinterpret_cast<uint4 *>(wl + ps * words)[idx - ps * (words >> 2)] = w;
        }
    }
    __syncthreads();
    // ---- the lane's query rows, both pairs ----
    uint32_t q[R];
    bool has_n = false;
    const uint32_t r0 = lg * R;
#pragma unroll
    for (int k = 0; k < R; k += 4) {
        uint32_t v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            v[h] = 0xFFFFFFFFu;
            if (valid[h] && r0 + k < qpad[h]) v[h] = load4_codes(A.q, qo[h], (r0 + k) >> 2, A.packed);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t c0 = (v[0] >> (8 * j)) & 0xFFu, c1 = (v[1] >> (8 * j)) & 0xFFu;
            q[k + j] = (c0 & 15u) | ((c1 & 15u) << 16);        // rows past the grid: any code
            has_n |= ((int32_t)c0 == A.nval && r0 + k + j < ql[0]) || ((int32_t)c1 == A.nval && r0 + k + j < ql[1]);
        }
    }
    const uint32_t nsteps = tmaxw + G - 1;
    const uint32_t *tcol = wl + slot * words;
    uint32_t key[R];
    if (A.force_exact || __any(has_n))
        wf16_body<G, R, true>(A, tcol, lg, nsteps, q, key);
    else
        wf16_body<G, R, false>(A, tcol, lg, nsteps, q, key);

    // ---- strip-major first maximum per pair (Q1) ----
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint64_t best = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint32_t r = r0 + k;
            const uint32_t kk = (key[k] >> (16 * h)) & 0xFFFFu;
            const uint32_t H = kk >> 8;
            if (r < qpad[h] && H > 0) {
                const uint32_t col = 255u - (kk & 0xFFu);
                const uint32_t ord = (((col >> 3) * qpad[h] + r) << 3) + (col & 7);
                const uint64_t cand = ((uint64_t)H << 32) | (0xFFFFFFFFu - ord);
                best = cand > best ? cand : best;
            }
        }
        best = group_max_u64<G>(best);
        if (valid[h] && lg == 0) {
            int32_t H = (int32_t)(best >> 32), qe = 0, te = 0;
            if (H > 0) {
                const uint32_t ord = 0xFFFFFFFFu - (uint32_t)best;
                const uint32_t rest = ord >> 3;
                qe = (int32_t)(rest % qpad[h]);
                te = (int32_t)((rest / qpad[h]) * 8 + (ord & 7));
            }
            A.score[pr[h]] = H;
            if (A.qend) A.qend[pr[h]] = qe;
            if (A.tend) A.tend[pr[h]] = te;
        }
    }
}

}  // namespace gx
