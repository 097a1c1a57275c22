// wavefront16.hpp — packed-int16 segmented wavefront for LOCAL score + ends.
//
// Same sweep as wavefront.hpp (G lanes per group, R query rows per lane, one
// column per step, DPP wave_shr:1 hand-off), but every VGPR holds TWO pairs:
// the low 16 bits belong to pair 2*slot and the high 16 bits to pair
// 2*slot+1.  The cell update is GASAL2's CORE_LOCAL_COMPUTE
// (local_kernel_template.h:19-30):
//   tmp = H(r-1,c-1) + s;  H = max(tmp, F, E, 0);
//   E'  = max(tmp - OE, E - e);  F' = max(tmp - OE, F - e)
//
// Instruction economics on gfx950 (tools/ubench_ops.hip, measured): every
// v_pk_* op, v_max/min_*32, v_bitop3 and DPP issue at 4 cycles per wave64,
// while v_add_u32 / v_sub_u32 / v_and / v_xor issue at 2.  So the cell is
// written to use 32-bit adds/subtracts on the packed pair wherever no carry
// or borrow can cross from the low half into the high half:
//   * every DP value is stored with a bias B = 0x8000 (H = 0 <-> B), and the
//     local floor is applied once per cell on tmp - OE (toe = max(., B)), so
//     E and F never drop below B (max(E,0) obeys the same recurrence when
//     e >= 0, and values below 0 never reach H): all four subtractions are
//     borrow-free v_sub_u32;
//   * the substitution score is s = M_c - min(x, AB_c) where x = (q ^ t) &
//     mask holds the two codes' nibble at bit 8 or 12 of each half (so a
//     mismatch gives x >= 256 >= AB_c = a + b), M_c / AB_c are per-column
//     constants (a / a+b for bases, N rule / 0 for N columns, 0 / 0 outside
//     the grid): one v_bitop3, one v_pk_min_u16, then tmp = diag - m + M_c.
// Per row: 9 half-rate + 4 full-rate instructions for two cells.  The per-row
// maximum is a 16-bit key (H << 8 | 255 - c), unaffected by the bias since
// B * 256 = 0 mod 2^16; the strip-major first maximum is resolved
// at the end exactly as in the int32 kernel.
//
// Exactness domain (checked by the planner, packed16_ok): every H <= 255
// (a * min(ql,tl)), padded targets <= 256 columns, a + b <= 256, e >= 0,
// o + e <= 16000, N penalty <= 16000.
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
// 32-bit add/sub used on a packed pair; exact per half when no carry/borrow
// crosses bit 16 (guaranteed by the bias invariants above).
__device__ __forceinline__ uint32_t pk_addnc(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t pk_subnb(uint32_t a, uint32_t b) { return a - b; }
__device__ __forceinline__ uint32_t pk_bcast(int32_t v) { return ((uint32_t)v & 0xFFFFu) * 0x10001u; }

#ifndef GX_WF16_PINGPONG
#define GX_WF16_PINGPONG 1
#endif
#ifndef GX_WF16_WAVES
#define GX_WF16_WAVES 3   // waves per SIMD the register allocator must allow
#endif

constexpr uint32_t kPkInvalid = 0xFFu;   // target/query code outside the padded grid
constexpr uint32_t kPkBias = 0x8000u;    // stored value of H = 0

// Per-column constants of one step (both halves).
struct Col16 {
    uint32_t trep;   // target nibble at bits 8 and 12 of each half
    uint32_t ab;     // a + b for a base column, 0 for N / outside
    uint32_t m;      // a for a base column, N rule score for N, 0 outside
    uint32_t qn;     // EXACT only: m - (N-row score) >= 0
};

template <bool NPEN, bool EXACT>
__device__ __forceinline__ Col16 col16(const uint32_t t, const uint32_t NVALp, const uint32_t Ap, const uint32_t ABp,
                                       const uint32_t NSp, const uint32_t ONEp) {
    const uint32_t INVp = 0x00FF00FFu;
    const uint32_t notN = pk_min_u16(t ^ NVALp, ONEp);
    const uint32_t notI = pk_min_u16(t ^ INVp, ONEp);
    const uint32_t live = pk_mad_u16(notN, notI, 0u);
    Col16 C;
    C.trep = pk_mad_u16(t & 0x000F000Fu, 0x11001100u, 0u);
    C.ab = pk_mad_u16(live, ABp, 0u);
    // N column: M = NS (<= 0), outside: 0, base: a
    C.m = NPEN ? pk_mad_u16(notI, pk_mad_u16(notN, pk_sub(Ap, NSp), NSp), 0u)
               : pk_mad_u16(live, Ap, 0u);
    C.qn = 0;
    if (EXACT) C.qn = pk_sub(C.m, pk_mad_u16(notI, NSp, 0u));   // base: a - NS, N col: 0, outside: 0
    // opaque per-column constants: keeps the compiler from re-deriving them per row
    asm volatile("" : "+v"(C.ab), "+v"(C.m), "+v"(C.qn));
    return C;
}

// One column step: rows read the previous column's H from Hin and write the
// new H to Hout (ping-pong arrays, so no register copies on the back edge).
template <int R, bool NPEN, bool EXACT>
__device__ __forceinline__ void wf16_step(const Col16 &C, const int32_t c, const uint32_t diag_top,
                                          const uint32_t f_top, const uint32_t (&qp)[(R + 1) / 2],
                                          const uint32_t (&Hin)[R], uint32_t (&Hout)[R], uint32_t (&Ek)[R],
                                          uint32_t (&key)[R], uint32_t &f_out, const uint32_t OE,
                                          const uint32_t EXT, const uint32_t NREP, const uint32_t ONEp) {
    const uint32_t BB = kPkBias * 0x10001u;
    const bool kc = c >= 0 && c < 256;
    const uint32_t invc = kc ? pk_bcast(255 - c) : 0u;
    const uint32_t kmul = kc ? (ONEp << 8) : 0u;                  // key = H*256 + 255-c
    uint32_t diag = diag_top, f = f_top;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t mask = 0x0F000F00u << (4 * (k & 1));
        const uint32_t q = qp[k >> 1];
        uint32_t m = pk_min_u16((q ^ C.trep) & mask, C.ab);
        if (EXACT) {   // query N (LOCAL N rule): m = qn for that row
            const uint32_t notNq = pk_min_u16((q ^ NREP) & mask, ONEp);
            m = pk_mad_u16(notNq, pk_sub(m, C.qn), C.qn);
        }
        const uint32_t tmp = NPEN ? pk_add(pk_subnb(diag, m), C.m) : pk_addnc(pk_subnb(diag, m), C.m);
        const uint32_t H = pk_max_u16(pk_max_u16(tmp, f), Ek[k]);
        const uint32_t toe = pk_max_u16(pk_subnb(tmp, OE), BB);
        Ek[k] = pk_max_u16(toe, pk_subnb(Ek[k], EXT));
        f = pk_max_u16(toe, pk_subnb(f, EXT));
        key[k] = pk_max_u16(key[k], pk_mad_u16(H, kmul, invc));
        diag = Hin[k];
        Hout[k] = H;
    }
    f_out = f;
}

template <int G, int R, bool NPEN, bool EXACT>
__device__ __forceinline__ void wf16_body(const WfArgs &A, const uint2 *tcol, const uint32_t lg,
                                          const uint32_t nsteps, const uint32_t (&qp)[(R + 1) / 2],
                                          uint32_t (&key)[R]) {
    const uint32_t BB = kPkBias * 0x10001u;
    const uint32_t OE = pk_bcast(A.o + A.e);
    const uint32_t EXT = pk_bcast(A.e);
    const uint32_t NVALp = pk_bcast(A.nval);
    const uint32_t NREP = pk_bcast(A.nval * 0x1100);
    const int32_t NS = A.has_npen ? -A.npen : 0;
    const uint32_t Ap = pk_bcast(A.a), NSp = pk_bcast(NS), ABp = pk_bcast(A.a + A.b);
    const uint32_t ONEp = A.one;
    uint32_t HA[R], Ek[R];
#if GX_WF16_PINGPONG
    uint32_t HB[R];
#else
    uint32_t (&HB)[R] = HA;   // one array: the compiler renames with a copy per row
#endif
#pragma unroll
    for (int k = 0; k < R; ++k) { HA[k] = BB; HB[k] = BB; Ek[k] = BB; key[k] = 0; }
    uint32_t recvH = BB, prevRecvH = BB, recvF = BB, f = BB;
    const bool top = lg == 0;
    int32_t c = -(int32_t)lg;
    uint32_t tnext = tcol[c + G].y;
    // two columns per iteration (the odd tail step reads only "outside" columns)
    for (uint32_t s = 0; s < nsteps; s += 2, c += 2) {
        Col16 C = col16<NPEN, EXACT>(tnext, NVALp, Ap, ABp, NSp, ONEp);
        tnext = tcol[c + 1 + G].y;
        wf16_step<R, NPEN, EXACT>(C, c, top ? BB : prevRecvH, top ? BB : recvF, qp, HA, HB, Ek, key, f, OE, EXT,
                                  NREP, ONEp);
        prevRecvH = recvH;
        recvH = (uint32_t)shr_lane((int32_t)HB[R - 1]);
        recvF = (uint32_t)shr_lane((int32_t)f);
        C = col16<NPEN, EXACT>(tnext, NVALp, Ap, ABp, NSp, ONEp);
        tnext = tcol[c + 2 + G].y;
        wf16_step<R, NPEN, EXACT>(C, c + 1, top ? BB : prevRecvH, top ? BB : recvF, qp, HB, HA, Ek, key, f, OE,
                                  EXT, NREP, ONEp);
        prevRecvH = recvH;
        recvH = (uint32_t)shr_lane((int32_t)HA[R - 1]);
        recvF = (uint32_t)shr_lane((int32_t)f);
    }
}

// ---------------------------------------------------------------------------
// Fast path (every code of the block is A/C/G/T, query N only in pad rows).
//
// Substitution: each staged column holds two 4-byte tables T0/T1 (pair 0 /
// pair 1), byte j = score(query letter j, target) + K >= 0; one v_perm_b32
// per row picks byte l0 of T0 into the low half and byte 4+l1 of T1 into the
// high half (selector bytes 1 and 3 = 0x0C give 0).
//
// Representation: every DP value is stored as value + B with B chosen so that
// all stored values stay inside the positive, normal f16 range
// [0x0400, 0x7BFF], where the f16 order of the bit patterns equals their
// integer order — so v_pk_maximum3_f16 is an exact 3-way integer max on both
// halves (bit patterns in, one of them out):
//   t1 = diag + v;  tmp = t1 - K;  H = max3(tmp, F, E)
//   toe = t1 - (OE + K);  E' = max3(toe, E - e, B);  F' = max3(toe, F - e, B)
// (GASAL2's local core, local_kernel_template.h:19-30; flooring E and F at 0
// is exact: values below 0 never reach H, and H >= 0 follows).  Adds and
// subtracts are 32-bit on the packed pair and never carry across bit 16.
// Per row: perm, 5 add/sub, 3 maximum3 and the key mad + max = 11
// instructions for two cells (the int16 general path below needs 14).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pk_max3_f16bits(uint32_t a, uint32_t b, uint32_t c) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 x = GX_AS(h2, a), y = GX_AS(h2, b), z = GX_AS(h2, c);
    return GX_AS(uint32_t, __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z));
}

// A/C/G/T nibble -> 0..3, N -> 4, anything else -> 5
__device__ __forceinline__ uint32_t letter_of(uint32_t nib, int32_t nval) {
    if ((int32_t)nib == nval) return 4;
    const uint64_t lut = 0x5555555555555555ull & ~(0xFull << 4) & ~(0xFull << 12) & ~(0xFull << 28) & ~(0xFull << 16);
    const uint64_t set = (0ull << 4) | (1ull << 12) | (2ull << 28) | (3ull << 16);   // A=1 C=3 G=7 T=4
    return (uint32_t)(((lut | set) >> (4 * (nib & 15u))) & 15u);
}

// Offsets of the fast path (the host planner checks the range, dispatch.hip).
struct Fast16 {
    int32_t k;      // table offset, >= max(b, N penalty)
    int32_t base;   // B: stored value of 0
};
__device__ __forceinline__ Fast16 fast16_params(const WfArgs &A) {
    Fast16 F;
    F.k = max(A.b, A.has_npen ? A.npen : 0);
    F.base = 0x0400 + A.o + A.e + F.k + 16;
    return F;
}

template <int R>
__device__ __forceinline__ void wf16f_step(const uint2 T, const int32_t c, const uint32_t diag_top,
                                           const uint32_t f_top, const uint32_t (&qs)[R], const uint32_t (&Hin)[R],
                                           uint32_t (&Hout)[R], uint32_t (&Ek)[R], uint32_t (&key)[R],
                                           uint32_t &f_out, const uint32_t KK, const uint32_t OEK, const uint32_t EXT,
                                           const uint32_t BB, const uint32_t KMUL, const uint32_t bshift) {
    const uint32_t col = (c >= 0 && c < 256) ? (uint32_t)(255 - c) : 0u;
    const uint32_t invc = ((col - bshift) & 0xFFFFu) * 0x10001u;   // key = H*256 + col (mod 2^16)
    uint32_t diag = diag_top, f = f_top;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t v = __builtin_amdgcn_perm(T.y, T.x, qs[k]);
        const uint32_t t1 = pk_addnc(diag, v);
        const uint32_t tmp = pk_subnb(t1, KK);
        const uint32_t toe = pk_subnb(t1, OEK);
        const uint32_t H = pk_max3_f16bits(tmp, f, Ek[k]);
        Ek[k] = pk_max3_f16bits(toe, pk_subnb(Ek[k], EXT), BB);
        f = pk_max3_f16bits(toe, pk_subnb(f, EXT), BB);
        key[k] = pk_max_u16(key[k], pk_mad_u16(H, KMUL, invc));
        diag = Hin[k];
        Hout[k] = H;
    }
    f_out = f;
}

template <int G, int R>
__device__ __forceinline__ void wf16f_body(const WfArgs &A, const uint2 *tcol, const uint32_t lg,
                                           const uint32_t nsteps, const uint32_t (&qs)[R], uint32_t (&key)[R]) {
    const Fast16 P = fast16_params(A);
    const uint32_t BB = (uint32_t)P.base * 0x10001u;
    const uint32_t KK = pk_bcast(P.k);
    const uint32_t OEK = pk_bcast(A.o + A.e + P.k);
    const uint32_t EXT = pk_bcast(A.e);
    const uint32_t KMUL = A.one << 8;
    const uint32_t bshift = ((uint32_t)P.base << 8) & 0xFFFFu;
    uint32_t HA[R], HB[R], Ek[R];
#pragma unroll
    for (int k = 0; k < R; ++k) { HA[k] = BB; HB[k] = BB; Ek[k] = BB; key[k] = 0; }
    uint32_t recvH = BB, prevRecvH = BB, recvF = BB, f = BB;
    const bool top = lg == 0;
    int32_t c = -(int32_t)lg;
    uint2 tnext = tcol[c + G];
    for (uint32_t s = 0; s < nsteps; s += 2, c += 2) {
        uint2 T = tnext;
        tnext = tcol[c + 1 + G];
        wf16f_step<R>(T, c, top ? BB : prevRecvH, top ? BB : recvF, qs, HA, HB, Ek, key, f, KK, OEK, EXT, BB, KMUL,
                      bshift);
        prevRecvH = recvH;
        recvH = (uint32_t)shr_lane((int32_t)HB[R - 1]);
        recvF = (uint32_t)shr_lane((int32_t)f);
        T = tnext;
        tnext = tcol[c + 2 + G];
        wf16f_step<R>(T, c + 1, top ? BB : prevRecvH, top ? BB : recvF, qs, HB, HA, Ek, key, f, KK, OEK, EXT, BB,
                      KMUL, bshift);
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
    // ---- stage both pairs' target codes, one uint2 per column (.y = lo: pair 0 code,
    //      hi: pair 1 code; .x = later the fast path's T0), columns [-G, tmaxw + G)
    //      so that out-of-range steps read "outside" ----
    const uint32_t words = A.lds_stride >> 3;            // columns per slot, >= tmaxw + 2G + 4, multiple of 4
    uint2 *wl = reinterpret_cast<uint2 *>(lds) + (size_t)wave * S * words;
    bool other = false;                                  // a code the fast path cannot score
    for (uint32_t base = 0; base < S * (words >> 2); base += 64) {
        const uint32_t idx = base + lane;
        const uint32_t ps = min(idx / (words >> 2), (uint32_t)S - 1);
        const uint32_t c0 = 4 * (idx - ps * (words >> 2)) - G;   // first column of this quad
        uint32_t v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t tp = __shfl(tpad[h], ps * G), tof = __shfl(to[h], ps * G);
            v[h] = 0xFFFFFFFFu;
            if ((int32_t)c0 >= 0 && c0 < tp) {
                v[h] = load4_codes(A.t, tof, c0 >> 2, A.packed);
#pragma unroll
                for (int j = 0; j < 4; ++j) other |= letter_of((v[h] >> (8 * j)) & 15u, A.nval) == 5;
            }
        }
        if (idx < S * (words >> 2)) {
            uint2 *dst = wl + ps * words + 4 * (idx - ps * (words >> 2));
#pragma unroll
            for (int j = 0; j < 4; ++j)
                dst[j] = make_uint2(0u, ((v[0] >> (8 * j)) & 0xFFu) | (((v[1] >> (8 * j)) & 0xFFu) << 16));
        }
    }
    // ---- query codes: letter per row and pair, N / foreign-code census ----
    const uint32_t r0 = lg * R;
    bool has_n = false;
    uint32_t qs[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t r = r0 + k;
        qs[k] = 0x0C000C00u | 0x000C000Cu;    // selector "constant 0" for rows outside the query
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (valid[h] && r < qpad[h]) {
                const uint32_t cde = A.packed ? (load4_codes(A.q, qo[h], r >> 2, 1) >> (8 * (r & 3))) & 15u
                                              : (uint32_t)A.q[qo[h] + r] & 15u;
                const uint32_t l = letter_of(cde, A.nval);
                has_n |= l == 4 && r < ql[h];
                other |= l == 5 || (l == 4) != (r >= ql[h]);   // pad rows must be N (fast path scores them -K)
                if (l < 4) qs[k] = (qs[k] & ~(0xFFu << (16 * h))) | ((l + 4 * h) << (16 * h));
            }
        }
    }
    const bool fast = A.fast16 && !A.force_exact && !__syncthreads_or(other);
    const uint32_t nsteps = tmaxw + G - 1;
    const uint2 *tcol = wl + slot * words;
    uint32_t key[R];
    if (fast) {
        // codes -> per-column score tables (byte j = score(letter j, t) + Kt; Kt outside the grid)
        const int32_t K = fast16_params(A).k;
        const int32_t NS = A.has_npen ? -A.npen : 0;
        const uint32_t mis = (uint32_t)(K - A.b) * 0x01010101u, nrow = (uint32_t)(NS + K) * 0x01010101u;
        const uint32_t outside = (uint32_t)K * 0x01010101u;
        for (uint32_t e = lane; e < S * words; e += 64) {
            const uint32_t cw = wl[e].y;
            uint32_t tab[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t t = (cw >> (16 * h)) & 0xFFu;
                const uint32_t l = t == 0xFFu ? 6u : letter_of(t, A.nval);
                tab[h] = l == 6 ? outside : l == 4 ? nrow
                                                   : (mis & ~(0xFFu << (8 * l))) | ((uint32_t)(A.a + K) << (8 * l));
            }
            wl[e] = make_uint2(tab[0], tab[1]);
        }
        __syncthreads();
        wf16f_body<G, R>(A, tcol, lg, nsteps, qs, key);
    } else {
        // general path: nibble codes, row k's nibble at bit 8 + 4*(k&1) of each half
        uint32_t qp[(R + 1) / 2];
#pragma unroll
        for (int j = 0; j < (R + 1) / 2; ++j) qp[j] = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint32_t r = r0 + k;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t cde = 0;
                if (valid[h] && r < qpad[h])
                    cde = A.packed ? (load4_codes(A.q, qo[h], r >> 2, 1) >> (8 * (r & 3))) & 15u
                                   : (uint32_t)A.q[qo[h] + r] & 15u;
                qp[k >> 1] |= cde << (8 + 4 * (k & 1) + 16 * h);
            }
        }
        const bool npen = A.has_npen && A.npen != 0;
        const bool exact = A.force_exact || __any(has_n);
        if (npen) {
            if (exact) wf16_body<G, R, true, true>(A, tcol, lg, nsteps, qp, key);
            else wf16_body<G, R, true, false>(A, tcol, lg, nsteps, qp, key);
        } else {
            if (exact) wf16_body<G, R, false, true>(A, tcol, lg, nsteps, qp, key);
            else wf16_body<G, R, false, false>(A, tcol, lg, nsteps, qp, key);
        }
    }

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
