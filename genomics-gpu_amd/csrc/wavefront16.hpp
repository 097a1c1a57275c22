// wavefront16.hpp — packed two-pairs-per-lane wavefront kernels (LOCAL, GLOBAL,
// SEMI-GLOBAL score paths) for gfx950.
//
// Sweep: as wavefront.hpp — a group of G lanes owns a DP matrix; lane lg holds
// R consecutive positions of the "register axis" sequence X and, at step s,
// computes position y = s - lg of the "step axis" sequence Y for all its R
// positions, top to bottom; the last position's values go to lane lg+1 by DPP
// wave_shr:1.  Every VGPR holds TWO pairs: low 16 bits pair 2*slot, high 16
// bits pair 2*slot+1.
//   LOCAL, GLOBAL: X = query (rows), Y = target (columns) — the reference's
//                  orientation (local_kernel_template.h, global.h).
//   SEMI:          X = target, Y = query (transposed), so that the last query
//                  row — the only row the TAIL=TARGET result reads
//                  (semiglobal_kernel_template.h:160-178) — is one step, read
//                  once, instead of a per-cell running key.
//
// Substitution: the step-axis sequence is staged in LDS as per-position score
// tables, two 4-byte tables per uint2 (pair 0 / pair 1): byte j =
// score(X letter j, Y code) + K >= 0.  One v_perm_b32 per cell-pair picks byte
// l0 of table 0 into the low half and byte 4+l1 of table 1 into the high half
// (selector bytes 1 and 3 = 0x0C give 0).  Blocks with codes other than
// A/C/G/T on the register axis (or other than A/C/G/T/N on the step axis) are
// declined: the kernel marks them in `handled` and the int32 kernel
// (wavefront.hpp) aligns exactly those pairs afterwards (dispatch.hip).
//
// Arithmetic: every stored DP value is value + B with B chosen so that all
// stored values stay inside the positive, normal f16 range [0x0400, 0x7BFF],
// where the f16 order of the bit patterns equals their integer order — so
// v_pk_maximum3_f16 is an exact 3-way integer max on both halves, and 32-bit
// adds/subtracts on the packed pair never carry across bit 16.  Issue cost on
// gfx950 (profiles/r01_valu_issue_rates.md): v_pk_*, maximum3 and v_perm issue
// at 4 cycles per wave64, v_add/sub_u32 at 2.
//
//   LOCAL  (local_kernel_template.h:19-30; floors at B are exact because
//           values below 0 never reach H):
//     t1 = diag + v; tmp = t1 - K; toe = t1 - (OE + K); H = max3(tmp, F, E)
//     E' = max3(toe, E - e, B); F' = max3(toe, F - e, B); key = max(key, H*256 + 255-c)
//     11 instructions per two cells.
//   GLOBAL (global.h:4-12; the NEG floors never bind for reachable values):
//     same without the key and with NEG in place of B: 9 instructions.
//   SEMI   (semiglobal_kernel_template.h:17-28, H-based Gotoh; values stored
//           as H - OE, every value drifting by e per anti-diagonal, so that the
//           gap extensions vanish and the table offset K = OE + e folds the + OE):
//     tmp = diag + v; F = max(Hup, F); E = max(Hleft, E);
//     H' = max3(tmp, F, E) - o: 6 instructions (8 before the drift).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "wavefront.hpp"

namespace gx {

typedef unsigned short pk_u2 __attribute__((ext_vector_type(2)));
#define GX_AS(T, x) __builtin_bit_cast(T, x)

__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t b, uint32_t c) {
    return GX_AS(uint32_t, GX_AS(pk_u2, a) * GX_AS(pk_u2, b) + GX_AS(pk_u2, c));
}
// c's low half added to both halves (a splat the compiler issues as op_sel_hi on an SGPR)
__device__ __forceinline__ uint32_t pk_mad_u16_lo(uint32_t a, uint32_t b, uint32_t c) {
    const pk_u2 cc = {(uint16_t)c, (uint16_t)c};
    return GX_AS(uint32_t, GX_AS(pk_u2, a) * GX_AS(pk_u2, b) + cc);
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, __builtin_elementwise_max(GX_AS(pk_u2, a), GX_AS(pk_u2, b)));
}
// 32-bit add/sub used on a packed pair; exact per half when no carry/borrow
// crosses bit 16 (guaranteed by the value-range invariants above).
__device__ __forceinline__ uint32_t pk_addnc(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t pk_subnb(uint32_t a, uint32_t b) { return a - b; }
__device__ __forceinline__ uint32_t pk_bcast(int32_t v) { return ((uint32_t)v & 0xFFFFu) * 0x10001u; }
// exact integer 3-way max of bit patterns in [0x0400, 0x7BFF] (positive normal f16)
__device__ __forceinline__ uint32_t pk_max3(uint32_t a, uint32_t b, uint32_t c) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 x = GX_AS(h2, a), y = GX_AS(h2, b), z = GX_AS(h2, c);
    return GX_AS(uint32_t, __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z));
}

constexpr int kW16_TB_WAVES = 2;   // GLOBAL + traceback kernel
#ifndef GX_LOCAL_FENCE
#define GX_LOCAL_FENCE 0   // A/B: scheduling fences after the LOCAL sweep's table reads
#endif
#ifndef GX_LOCAL_IL2
#define GX_LOCAL_IL2 1     // the LOCAL sweep's rows in interleaved pairs (+1.0 %, profiles/r06/ab)
#endif
#ifndef GX_SEMI_IL2
#define GX_SEMI_IL2 0      // A/B: the SEMI sweep's rows in interleaved pairs (-1.3 % on config 4)
#endif
#ifndef GX_GLOBAL_IL2
#define GX_GLOBAL_IL2 1    // the GLOBAL sweep's rows in interleaved pairs (NW +1.4 %, config 3 +2-4 %)
#endif
#ifndef GX_TB_IL2
#define GX_TB_IL2 1        // the traceback sweeps' rows in interleaved pairs (LOCAL+TB +0.7 %)
#endif
#ifndef GX_CP_ST16
#define GX_CP_ST16 0       // A/B: the config-3 sweep's checkpoint and stream stores 16 bytes wide
#endif
#ifndef GX_SEMI_PH4
#define GX_SEMI_PH4 1      // the SEMI sweep's reset code only in its first G steps (+1.0 %)
#endif
#ifndef GX_LTB_KA0
#define GX_LTB_KA0 1      // GX_LOCAL_KA0 in the LOCAL+TB kernel (step_local_tb_dr): 2,964 -> 3,144 GCUPS
                          // (its two waves per SIMD issued the two scalar addend subtracts per row)
#endif
#ifndef GX_LOCAL_KA0
#define GX_LOCAL_KA0 1     // one key addend for every row (keys offset by e*k*M, taken off after the sweep): +0.6 %
#endif
#ifndef GX_LOCAL_ATIE
#define GX_LOCAL_ATIE 1    // the LOCAL keys' scalar addends kept as a chain (with IL2: +2.4 %, profiles/r06/ab)
#endif
#ifndef GX_WF16_WAVES
#define GX_WF16_WAVES 3   // waves per SIMD the register allocator must allow
#endif
constexpr int kW16_K2_WAVES = 2;    // LOCAL over 257..512 target columns (a 3-wave build spills)
constexpr int kW16_LTB_WAVES = 2;   // LOCAL + traceback kernel

// A/C/G/T nibble -> 0..3, N -> 4, anything else -> 5
__device__ __forceinline__ uint32_t letter_of(uint32_t nib, int32_t nval) {
    if ((int32_t)nib == nval) return 4;
    const uint64_t lut = 0x5555555555555555ull & ~(0xFull << 4) & ~(0xFull << 12) & ~(0xFull << 28) & ~(0xFull << 16);
    const uint64_t set = (0ull << 4) | (1ull << 12) | (2ull << 28) | (3ull << 16);   // A=1 C=3 G=7 T=4
    return (uint32_t)(((lut | set) >> (4 * (nib & 15u))) & 15u);
}

// every G-lane group of a wave ballot has a bit set
template <int G>
__device__ __forceinline__ bool groups_all(uint64_t b) {
    constexpr uint64_t low = G == 64 ? 1ull : G == 32 ? 0x0000000100000001ull : G == 16 ? 0x0001000100010001ull
                                                                                      : 0x0101010101010101ull;
#pragma unroll
    for (int sh = 1; sh < G; sh <<= 1) b |= b >> sh;
    return (b & low) == low;
}

// Value-range constants of one launch (dispatch.hip packed16_ok checks that the
// stored values stay inside [0x0400, 0x7BFF] for these).
struct Pk16 {
    int32_t k;      // table offset
    int32_t base;   // stored value of 0
    int32_t neg;    // stored "minus infinity" (below every reachable value)
    int32_t drift;  // GLOBAL: a value of cell (r, c) is stored + drift*(r + c)
};
template <int ALGO>
__device__ __forceinline__ Pk16 pk16_params(const WfArgs &A) {
    Pk16 P;
    const int32_t OE = A.o + A.e;
    if (ALGO == WF_LOCAL) {
        P.k = max(A.b, A.has_npen ? A.npen : 0);
        P.base = 0x0400 + OE + P.k + 16;
        P.neg = P.base;
        P.drift = 0;
    } else {
        P.k = (ALGO == WF_SEMI) ? OE + A.e : max(A.b, A.has_npen ? A.npen : 0);   // SEMI: step_semi's frame
        P.drift = 0;
        if (ALGO == WF_GLOBAL) {       // drift e, table offset K >= 2e (step_global)
            P.drift = A.e;
            P.k = max(2 * ((P.k + 1) >> 1), 2 * A.e);
        }
        P.neg = 0x0400 + 2 * A.e + 16;
        P.base = P.neg + A.vmin;
    }
    return P;
}

// ---------------------------------------------------------------------------
// LOCAL step: registers = query rows, one target column per step.
// ---------------------------------------------------------------------------
// Per-row keys H*256 + (255 - column) in 16 bits cover 256 columns.  Targets up
// to 512 columns (KM != 0) keep a second key per row for columns 256..511:
// KM = 1 while lanes straddle column 256 (each lane feeds the key of its own
// column's half, the other gets a 0 candidate), KM = 2 once every lane is past it.
//
// KU (A.kf16 launches, dispatch.hip): keys as f16 patterns 0x0400 + H*C + (C-1-c),
// C = the launch's padded target length, so one v_pk_maximum3 folds two columns'
// candidates into a row's key: KU = 1 (first step of a pair) updates no key, KU = 2
// takes max3(key, cand(Hin = the previous column's H, invp), cand(H, invn)) — 3
// instructions per two cells instead of 4 (10.5 per cell pair instead of 11).
template <int R, int KM = 0, int KU = 0>
__device__ __forceinline__ void step_local(const uint2 T, const int32_t c, const uint32_t diag_top,
                                           const uint32_t f_top, const uint32_t (&xs)[R], const uint32_t (&Hin)[R],
                                           uint32_t (&Hout)[R], uint32_t (&Ek)[R], uint32_t (&key)[R],
                                           uint32_t (&key2)[R], uint32_t &f_out, const uint32_t KK,
                                           const uint32_t OEK, const uint32_t EXT, const uint32_t BB,
                                           const uint32_t KMUL, const uint32_t bshift, const uint32_t invp = 0,
                                           const uint32_t invn = 0) {
    const bool hi = KM != 0 && c >= 256;
    const uint32_t col = (c >= 0 && c < 256) ? (uint32_t)(255 - c) : 0u;
    const uint32_t col2 = (c >= 256 && c < 512) ? (uint32_t)(511 - c) : 0u;
    const uint32_t kmA = hi ? 0u : KMUL, kmB = hi ? KMUL : 0u;
    const uint32_t invc = hi ? 0u : ((col - bshift) & 0xFFFFu) * 0x10001u;   // key = H*256 + col (mod 2^16)
    const uint32_t invc2 = hi ? ((col2 - bshift) & 0xFFFFu) * 0x10001u : 0u;
    uint32_t diag = diag_top, f = f_top;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t v = __builtin_amdgcn_perm(T.y, T.x, xs[k]);
        const uint32_t t1 = pk_addnc(diag, v);
        const uint32_t tmp = pk_subnb(t1, KK);
        const uint32_t toe = pk_subnb(t1, OEK);
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        Ek[k] = pk_max3(toe, pk_subnb(Ek[k], EXT), BB);
        f = pk_max3(toe, pk_subnb(f, EXT), BB);
        if (KU == 2) key[k] = pk_max3(key[k], pk_mad_u16(Hin[k], KMUL, invp), pk_mad_u16(H, KMUL, invn));
        if (KU == 0 && KM != 2) key[k] = pk_max_u16(key[k], pk_mad_u16(H, kmA, invc));
        if (KU == 0 && KM != 0) key2[k] = pk_max_u16(key2[k], pk_mad_u16(H, kmB, invc2));
        diag = Hin[k];
        Hout[k] = H;
    }
    f_out = f;
}

// ---------------------------------------------------------------------------
// LOCAL step in the e-drift frame (A.kf16 launches): cell (r, c) stores value + B +
// e(r+c), so neither E nor F pays its extension subtract (each one measured at ~9 %
// of the kernel, profiles/r03_local_drift_ab.md).  The floor at 0 moves with the
// frame: FL[k] = B + e(r + c + 1), E's floor for the next column, one add per cell
// off the dependency chains; F is left unfloored (E >= 0 already floors H, and H =
// max(tmp, E, F) is the same for every F <= 0).  tmp = diag + v - (K - 2e), toe =
// diag + v - (K - 2e + o).  Keys: the f16 patterns of step_local KU, from H^ less
// FL - 2e (borrow-free 32-bit subtracts: Hin = H^(r, c) >= FL - 2e, H >= FL - e),
// two columns per v_pk_maximum3 (KEYS: the second step of a pair).
// ---------------------------------------------------------------------------
// U16 (WF16_LOCAL_U16 launches): the keys are plain u16 integers H*C + (C-1-c), ordered by
// two v_pk_max_u16 instead of one f16-pattern v_pk_maximum3 (one instruction more per two
// cells), so (Hmax + 1) * C may reach 65536 instead of 0x7800: 150 bp at match 2, where the
// round-3 planner fell back to the int32 kernel (2,627 GCUPS)
template <int R, bool KEYS, bool U16 = false, bool KA0 = false>
__device__ __forceinline__ void step_local_dr(const uint2 T, const uint32_t diag_top, const uint32_t f_top,
                                              const uint32_t (&xs)[R], const uint32_t (&Hin)[R], uint32_t (&Hout)[R],
                                              uint32_t (&Ek)[R], uint32_t (&key)[R], uint32_t (&FL)[R],
                                              uint32_t &f_out, const uint32_t KX, const uint32_t OEX,
                                              const uint32_t EXT, const uint32_t KMUL, const uint32_t invp,
                                              const uint32_t invn, const uint32_t EXT2, const uint32_t MK16 = 0) {
    uint32_t diag = diag_top, f = f_top;
    // row 0's addends (invp / invn: the candidates' bases), then one scalar subtract per row
    const uint32_t g20 = (FL[0] - EXT2) & 0xFFFFu, EM = (EXT2 >> 1 & 0xFFFFu) * MK16;   // e * M
    uint32_t a1 = invp - g20 * MK16, a2 = invn - g20 * MK16;
#if GX_LOCAL_IL2
    // A/B: two rows' independent parts interleaved (table byte, diagonal add, the two offsets), pinned
    // stage by stage with empty asm ties, so that no instruction waits on the one just before it
    constexpr int R2 = R & ~1;
#pragma unroll
    for (int k = 0; k < R2; k += 2) {
        uint32_t v0 = __builtin_amdgcn_perm(T.y, T.x, xs[k]), v1 = __builtin_amdgcn_perm(T.y, T.x, xs[k + 1]);
        asm volatile("" : "+v"(v0), "+v"(v1));
        uint32_t t0 = pk_addnc(diag, v0), t1 = pk_addnc(Hin[k], v1);
        asm volatile("" : "+v"(t0), "+v"(t1));
        uint32_t tmp0 = pk_subnb(t0, KX), tmp1 = pk_subnb(t1, KX), toe0 = pk_subnb(t0, OEX), toe1 = pk_subnb(t1, OEX);
        asm volatile("" : "+v"(tmp0), "+v"(tmp1), "+v"(toe0), "+v"(toe1));
        const uint32_t H0 = pk_max3(tmp0, f, Ek[k]);
        const uint32_t f1 = pk_max_u16(toe0, f);
        Ek[k] = pk_max3(toe0, Ek[k], FL[k]);
        const uint32_t H1 = pk_max3(tmp1, f1, Ek[k + 1]);
        f = pk_max_u16(toe1, f1);
        Ek[k + 1] = pk_max3(toe1, Ek[k + 1], FL[k + 1]);
        if (KEYS) {
            if (U16)
                key[k] = pk_max_u16(key[k], pk_max_u16(pk_mad_u16_lo(Hin[k], KMUL, a1), pk_mad_u16_lo(H0, KMUL, a2)));
            else
                key[k] = pk_max3(key[k], pk_mad_u16_lo(Hin[k], KMUL, a1), pk_mad_u16_lo(H0, KMUL, a2));
            if (!KA0) {
                a1 -= EM;
                a2 -= EM;
            }
            if (U16)
                key[k + 1] = pk_max_u16(key[k + 1], pk_max_u16(pk_mad_u16_lo(Hin[k + 1], KMUL, a1),
                                                               pk_mad_u16_lo(H1, KMUL, a2)));
            else
                key[k + 1] = pk_max3(key[k + 1], pk_mad_u16_lo(Hin[k + 1], KMUL, a1), pk_mad_u16_lo(H1, KMUL, a2));
            if (!KA0) {
                a1 -= EM;
                a2 -= EM;
#if GX_LOCAL_ATIE
                asm volatile("" : "+s"(a1), "+s"(a2));
#endif
            }
        }
        FL[k] = pk_addnc(FL[k], EXT);
        FL[k + 1] = pk_addnc(FL[k + 1], EXT);
        diag = Hin[k + 1];
        Hout[k] = H0;
        Hout[k + 1] = H1;
    }
#pragma unroll
    for (int k = R2; k < R; ++k) {
#else
#pragma unroll
    for (int k = 0; k < R; ++k) {
#endif
        const uint32_t v = __builtin_amdgcn_perm(T.y, T.x, xs[k]);
        const uint32_t t1 = pk_addnc(diag, v);
        const uint32_t tmp = pk_subnb(t1, KX);
        const uint32_t toe = pk_subnb(t1, OEX);
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        Ek[k] = pk_max3(toe, Ek[k], FL[k]);
        if (KEYS) {
            // key = (H^ - g2) * M + base = H^ * M + (base - g2 * M) (mod 2^16): the addend is the
            // same in every lane (FL and the step's bases are wave-uniform), so it is scalar work
            // and a cell pair's keys cost two mads and one max (the subtracts are gone)
            if (U16)
                key[k] = pk_max_u16(key[k], pk_max_u16(pk_mad_u16_lo(Hin[k], KMUL, a1), pk_mad_u16_lo(H, KMUL, a2)));
            else
                key[k] = pk_max3(key[k], pk_mad_u16_lo(Hin[k], KMUL, a1), pk_mad_u16_lo(H, KMUL, a2));
            if (!KA0) {
                a1 -= EM;   // row k + 1: FL one e higher
                a2 -= EM;
#if GX_LOCAL_ATIE
                // keep the addends a chain of one subtract per row: left alone, the compiler rebuilt each
                // row's from FL[k] (a subtract, a multiply and an add: 3 SALU per row instead of 1)
                asm volatile("" : "+s"(a1), "+s"(a2));
#endif
            }
        }
        FL[k] = pk_addnc(FL[k], EXT);
        f = pk_max_u16(toe, f);
        diag = Hin[k];
        Hout[k] = H;
    }
    f_out = f;
}

// ---------------------------------------------------------------------------
// GLOBAL step: as LOCAL without the floor at 0 and without keys.
// ---------------------------------------------------------------------------
// Values drift by the gap extension: cell (r, c) is stored as value + B + e*(r+c)
// (D = e), so E and F, which move one anti-diagonal and fall by e per step, stay
// put: E' = max3(toe, E, NEG) with toe = tmp - OE + e, no extension subtract.  The
// diagonal gains 2e: with table offset K (bytes s + K >= 0) tmp = diag + v - KX,
// KX = K - 2e >= 0 (K = max(2*ceil(max(b, npen)/2), 2e)); toe = diag + v - (KX +
// OE - e).  7 instructions per two cells (8 with the round-2 drift K/2, which
// left an extension add).  32-bit adds/subtracts of per-half constants, exact.
// SYNC: row by row (an empty asm ties each row's E and F): the band kernels' sweeps, whose
// consecutive steps are independent of each other, were otherwise scheduled into spills
template <int R, bool SYNC = false>
__device__ __forceinline__ void step_global(const uint2 T, const uint32_t diag_top, const uint32_t f_top,
                                            const uint32_t (&xs)[R], const uint32_t (&Hin)[R], uint32_t (&Hout)[R],
                                            uint32_t (&Ek)[R], uint32_t &f_out, const uint32_t KX,
                                            const uint32_t OEX, const uint32_t NN) {
    uint32_t diag = diag_top, f = f_top;
#if GX_GLOBAL_IL2
    constexpr int R2 = R & ~1;
#pragma unroll
    for (int k = 0; k < R2; k += 2) {
        uint32_t v0 = __builtin_amdgcn_perm(T.y, T.x, xs[k]), v1 = __builtin_amdgcn_perm(T.y, T.x, xs[k + 1]);
        asm volatile("" : "+v"(v0), "+v"(v1));
        uint32_t t0 = pk_addnc(diag, v0), t1 = pk_addnc(Hin[k], v1);
        asm volatile("" : "+v"(t0), "+v"(t1));
        uint32_t tmp0 = pk_subnb(t0, KX), tmp1 = pk_subnb(t1, KX), toe0 = pk_subnb(t0, OEX), toe1 = pk_subnb(t1, OEX);
        asm volatile("" : "+v"(tmp0), "+v"(tmp1), "+v"(toe0), "+v"(toe1));
        const uint32_t H0 = pk_max3(tmp0, f, Ek[k]);
        Ek[k] = pk_max3(toe0, Ek[k], NN);
        const uint32_t f1 = pk_max3(toe0, f, NN);
        const uint32_t H1 = pk_max3(tmp1, f1, Ek[k + 1]);
        Ek[k + 1] = pk_max3(toe1, Ek[k + 1], NN);
        f = pk_max3(toe1, f1, NN);
        diag = Hin[k + 1];
        Hout[k] = H0;
        Hout[k + 1] = H1;
        if (SYNC) asm volatile("" : "+v"(Ek[k]), "+v"(Ek[k + 1]), "+v"(f));
    }
#pragma unroll
    for (int k = R2; k < R; ++k) {
#else
#pragma unroll
    for (int k = 0; k < R; ++k) {
#endif
        const uint32_t v = __builtin_amdgcn_perm(T.y, T.x, xs[k]);
        const uint32_t t1 = pk_addnc(diag, v);
        const uint32_t tmp = pk_subnb(t1, KX);
        const uint32_t toe = pk_subnb(t1, OEX);
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        Ek[k] = pk_max3(toe, Ek[k], NN);
        f = pk_max3(toe, f, NN);
        diag = Hin[k];
        Hout[k] = H;
        if (SYNC) asm volatile("" : "+v"(Ek[k]), "+v"(f));
    }
    f_out = f;
}

// ---------------------------------------------------------------------------
// GLOBAL step with traceback flags (global.h:14-26).  The
// reference's nibble per cell is low2 = (H == tmp) ? (s < 0) : ((H == F) ? 3 : 2),
// bit2 = E extended, bit3 = F extended; here each cell records four "differs"
// flags and tb_kernel rebuilds the nibble (s < 0 it takes from the sequences):
//   u = [H != tmp], w = [H != F], x = [toe > E - e], y = [toe > F - e]
// (x, y are the reference's own "not extended" tests).  A flag is bit 15 of the
// per-half difference B - A (one v_pk_sub_u16): [A != B] for A >= B, [A > B] for
// |A - B| < 0x7800 (round 2 used (A + 0x7FFF) - B as two
// 32-bit ops with no carry/borrow across a half, 6 instructions for 4 flags instead
// of 4); v_perm's sign selectors turn two such bits into 0x00/0xFF bytes and one
// v_and_or places them: step j of a 4-step window owns bits j (u), 4+j (w),
// 8+j (x) and 12+j (y) of each 16-bit half of dw.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t tb_flag(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, GX_AS(pk_u2, b) - GX_AS(pk_u2, a));
}
// (a & m) | b as one v_bitop3_b32 (truth table 0xEA); the compiler would
// otherwise split the two merges of a row into and, and, or3
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(a, m, b, 0xEA);
}

// ---------------------------------------------------------------------------
// LOCAL + traceback in the e-drift frame (WF16_LOCAL_TBD): step_local_dr's cell (no E or F
// extension subtract, E floored at FL, F unfloored as the reference's) plus the four
// "differs" flags of step_local_tb in the same skewed layout: u = [H != tmp], w = [H != F],
// x = [E' != E - e], y = [F' != F - e] -- in the frame E - e and F - e are the stored E^ and F^.
// With F unfloored, w and y are the reference's own tests on every cell; x differs from the
// reference only where E is floored (E <= 0), never on a gap run the walk follows (it stops
// before H = 0, get_tb.h:100-103).  Keys: the wave-uniform addends of step_local_dr
// (step_local_dr), two columns per v_pk_maximum3 on the KEYS steps.  15.5 instructions per cell
// pair instead of step_local_tb's 19.
// ---------------------------------------------------------------------------
template <int R, bool KEYS, bool KA0 = false>
__device__ __forceinline__ void step_local_tb_dr(const uint2 T, const uint32_t diag_top, const uint32_t f_top,
                                                 const uint32_t (&xs)[R], const uint32_t (&Hin)[R],
                                                 uint32_t (&Hout)[R], uint32_t (&Ek)[R], uint32_t (&key)[R],
                                                 uint32_t &FL0, uint32_t (&dw)[R], uint32_t &f_out,
                                                 const uint32_t KX, const uint32_t OEX, const uint32_t EXT,
                                                 const uint32_t KMUL, const uint32_t invp, const uint32_t invn,
                                                 const uint32_t EXT2, const uint32_t MK16, const int j) {
    const uint32_t M1 = 0x01010101u << j, M2 = 0x10101010u << j;
    uint32_t diag = diag_top, f = f_top;
    // the rows' floors FL0 + k e are formed per row from row 0's (scalar adds): an array of R
    // floors in scalar registers overflowed them at this kernel's two waves (readlane spills)
    const uint32_t g20 = (FL0 - EXT2) & 0xFFFFu, EM = ((EXT2 >> 1) & 0xFFFFu) * MK16;
    uint32_t a1 = invp - g20 * MK16, a2 = invn - g20 * MK16, flk = FL0;
    auto cell = [&](const int k, const uint32_t tmp, const uint32_t toe) __attribute__((always_inline)) {
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        const uint32_t En = pk_max3(toe, Ek[k], flk);
        const uint32_t Fn = pk_max_u16(toe, f);
        const uint32_t fu = tb_flag(H, tmp), fw = tb_flag(H, f), fx = tb_flag(toe, Ek[k]), fy = tb_flag(toe, f);
        const uint32_t m1 = __builtin_amdgcn_perm(fx, fu, 0x0B090A08u);
        const uint32_t m2 = __builtin_amdgcn_perm(fy, fw, 0x0B090A08u);
        dw[k] = and_or(m2, M2, j == 0 ? (m1 & M1) : and_or(m1, M1, dw[k]));
        if (KEYS) {
            key[k] = pk_max3(key[k], pk_mad_u16_lo(Hin[k], KMUL, a1), pk_mad_u16_lo(H, KMUL, a2));
            if (!KA0) {
                a1 -= EM;
                a2 -= EM;
            }
        }
        flk = pk_addnc(flk, EXT);
        Ek[k] = En;
        f = Fn;
        Hout[k] = H;
        if (KEYS && !KA0) asm volatile("" : "+v"(dw[k]), "+v"(f), "+s"(a1), "+s"(a2), "+s"(flk));
        else asm volatile("" : "+v"(dw[k]), "+v"(f), "+s"(flk));
    };
#if GX_TB_IL2
    constexpr int R2 = R & ~1;
#pragma unroll
    for (int k = 0; k < R2; k += 2) {
        uint32_t v0 = __builtin_amdgcn_perm(T.y, T.x, xs[k]), v1 = __builtin_amdgcn_perm(T.y, T.x, xs[k + 1]);
        asm volatile("" : "+v"(v0), "+v"(v1));
        uint32_t t0 = pk_addnc(diag, v0), t1 = pk_addnc(Hin[k], v1);
        asm volatile("" : "+v"(t0), "+v"(t1));
        uint32_t tmp0 = pk_subnb(t0, KX), tmp1 = pk_subnb(t1, KX), toe0 = pk_subnb(t0, OEX), toe1 = pk_subnb(t1, OEX);
        asm volatile("" : "+v"(tmp0), "+v"(tmp1), "+v"(toe0), "+v"(toe1));
        cell(k, tmp0, toe0);
        cell(k + 1, tmp1, toe1);
        diag = Hin[k + 1];
    }
    if (R & 1) {
        constexpr int k = R - 1;
        const uint32_t t1 = pk_addnc(diag, __builtin_amdgcn_perm(T.y, T.x, xs[k]));
        cell(k, pk_subnb(t1, KX), pk_subnb(t1, OEX));
    }
#else
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t v = __builtin_amdgcn_perm(T.y, T.x, xs[k]);
        const uint32_t t1 = pk_addnc(diag, v);
        const uint32_t tmp = pk_subnb(t1, KX);
        const uint32_t toe = pk_subnb(t1, OEX);
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        const uint32_t En = pk_max3(toe, Ek[k], flk);
        const uint32_t Fn = pk_max_u16(toe, f);
        const uint32_t fu = tb_flag(H, tmp), fw = tb_flag(H, f), fx = tb_flag(toe, Ek[k]), fy = tb_flag(toe, f);
        const uint32_t m1 = __builtin_amdgcn_perm(fx, fu, 0x0B090A08u);
        const uint32_t m2 = __builtin_amdgcn_perm(fy, fw, 0x0B090A08u);
        dw[k] = and_or(m2, M2, j == 0 ? (m1 & M1) : and_or(m1, M1, dw[k]));
        if (KEYS) {
            key[k] = pk_max3(key[k], pk_mad_u16_lo(Hin[k], KMUL, a1), pk_mad_u16_lo(H, KMUL, a2));
            a1 -= EM;
            a2 -= EM;
        }
        flk = pk_addnc(flk, EXT);   // row k + 1: one e higher
        Ek[k] = En;
        f = Fn;
        diag = Hin[k];
        Hout[k] = H;
        // row by row, the scalar chains too (the scheduler otherwise spills, VGPRs and SGPRs)
        if (KEYS) asm volatile("" : "+v"(dw[k]), "+v"(f), "+s"(a1), "+s"(a2), "+s"(flk));
        else asm volatile("" : "+v"(dw[k]), "+v"(f), "+s"(flk));
    }
#endif
    FL0 = pk_addnc(FL0, EXT);   // the next step
    f_out = f;
}

template <int R, bool SYNC = false>
__device__ __forceinline__ void step_global_tb(const uint2 T, const uint32_t diag_top, const uint32_t f_top,
                                               const uint32_t (&xs)[R], const uint32_t (&Hin)[R],
                                               uint32_t (&Hout)[R], uint32_t (&Ek)[R], uint32_t (&dw)[R],
                                               uint32_t &f_out, const uint32_t KX, const uint32_t OEX,
                                               const uint32_t NN, const int j) {
    const uint32_t M1 = 0x01010101u << j, M2 = 0x10101010u << j;
    uint32_t diag = diag_top, f = f_top, tx = T.x, ty = T.y;
#if GX_TB_IL2
    auto cell = [&](const int k, const uint32_t tmp, const uint32_t toe) __attribute__((always_inline)) {
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        const uint32_t em = Ek[k], fm = f;
        const uint32_t En = pk_max3(toe, em, NN);
        const uint32_t Fn = pk_max3(toe, fm, NN);
        const uint32_t fu = tb_flag(H, tmp), fw = tb_flag(H, f), fx = tb_flag(toe, em), fy = tb_flag(toe, fm);
        const uint32_t m1 = __builtin_amdgcn_perm(fx, fu, 0x0B090A08u);
        const uint32_t m2 = __builtin_amdgcn_perm(fy, fw, 0x0B090A08u);
        dw[k] = and_or(m2, M2, j == 0 ? (m1 & M1) : and_or(m1, M1, dw[k]));
        Ek[k] = En;
        f = Fn;
        Hout[k] = H;
        if (SYNC) asm volatile("" : "+v"(dw[k]), "+v"(f));
    };
    constexpr int R2 = R & ~1;
#pragma unroll
    for (int k = 0; k < R2; k += 2) {
        uint32_t v0 = __builtin_amdgcn_perm(ty, tx, xs[k]), v1 = __builtin_amdgcn_perm(ty, tx, xs[k + 1]);
        asm volatile("" : "+v"(v0), "+v"(v1));
        uint32_t t0 = pk_addnc(diag, v0), t1 = pk_addnc(Hin[k], v1);
        asm volatile("" : "+v"(t0), "+v"(t1));
        uint32_t tmp0 = pk_subnb(t0, KX), tmp1 = pk_subnb(t1, KX), toe0 = pk_subnb(t0, OEX), toe1 = pk_subnb(t1, OEX);
        asm volatile("" : "+v"(tmp0), "+v"(tmp1), "+v"(toe0), "+v"(toe1));
        cell(k, tmp0, toe0);
        cell(k + 1, tmp1, toe1);
        diag = Hin[k + 1];
    }
    if (R & 1) {
        constexpr int k = R - 1;
        const uint32_t t1 = pk_addnc(diag, __builtin_amdgcn_perm(ty, tx, xs[k]));
        cell(k, pk_subnb(t1, KX), pk_subnb(t1, OEX));
    }
#else
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t v = __builtin_amdgcn_perm(ty, tx, xs[k]);
        const uint32_t t1 = pk_addnc(diag, v);           // drift e: see step_global
        const uint32_t tmp = pk_subnb(t1, KX);
        const uint32_t toe = pk_subnb(t1, OEX);
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        const uint32_t em = Ek[k], fm = f;               // E - e and F - e, in the frame
        const uint32_t En = pk_max3(toe, em, NN);
        const uint32_t Fn = pk_max3(toe, fm, NN);
        const uint32_t fu = tb_flag(H, tmp), fw = tb_flag(H, f), fx = tb_flag(toe, em), fy = tb_flag(toe, fm);
        // bytes: [u, x] per half and [w, y] per half, 0x00 / 0xFF
        const uint32_t m1 = __builtin_amdgcn_perm(fx, fu, 0x0B090A08u);
        const uint32_t m2 = __builtin_amdgcn_perm(fy, fw, 0x0B090A08u);
        dw[k] = and_or(m2, M2, j == 0 ? (m1 & M1) : and_or(m1, M1, dw[k]));
        Ek[k] = En;
        f = Fn;
        diag = Hin[k];
        Hout[k] = H;
        // SYNC: each row's flags before the next row (the band pass deferred them all to the
        // window's store otherwise: 345 spilled VGPRs; 120 VGPRs with it)
        if (SYNC) asm volatile("" : "+v"(dw[k]), "+v"(f));
    }
#endif
    f_out = f;
}

// ---------------------------------------------------------------------------
// LOCAL step with traceback flags (local_kernel_template.h:45-60 nibbles): the
// LOCAL update of step_local plus the four "differs" flags of step_global_tb.
// E and F are floored at 0 here (the reference's are not); on every cell the
// walk visits (H > 0, gap values > 0, get_tb.h:100-103 stops before H = 0)
// the flags agree: u = [H != tmp] is unchanged, w = [H != F] differs only
// where H = 0, x/y only where the floored value's successor is <= 0.
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void step_local_tb(const uint2 T, const int32_t c, const uint32_t diag_top,
                                              const uint32_t f_top, const uint32_t (&xs)[R], const uint32_t (&Hin)[R],
                                              uint32_t (&Hout)[R], uint32_t (&Ek)[R], uint32_t (&key)[R],
                                              uint32_t (&dw)[R], uint32_t &f_out, const uint32_t KK,
                                              const uint32_t OEK, const uint32_t EXT, const uint32_t BB,
                                              const uint32_t KMUL, const uint32_t bshift, const int j) {
    const uint32_t M1 = 0x01010101u << j, M2 = 0x10101010u << j;
    const uint32_t col = (c >= 0 && c < 256) ? (uint32_t)(255 - c) : 0u;
    const uint32_t invc = ((col - bshift) & 0xFFFFu) * 0x10001u;   // key = H*256 + col (mod 2^16)
    uint32_t diag = diag_top, f = f_top;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t v = __builtin_amdgcn_perm(T.y, T.x, xs[k]);
        const uint32_t t1 = pk_addnc(diag, v);
        const uint32_t tmp = pk_subnb(t1, KK);
        const uint32_t toe = pk_subnb(t1, OEK);
        const uint32_t H = pk_max3(tmp, f, Ek[k]);
        const uint32_t em = pk_subnb(Ek[k], EXT), fm = pk_subnb(f, EXT);
        const uint32_t En = pk_max3(toe, em, BB);
        const uint32_t Fn = pk_max3(toe, fm, BB);
        key[k] = pk_max_u16(key[k], pk_mad_u16(H, KMUL, invc));
        const uint32_t fu = tb_flag(H, tmp), fw = tb_flag(H, f), fx = tb_flag(toe, em), fy = tb_flag(toe, fm);
        const uint32_t m1 = __builtin_amdgcn_perm(fx, fu, 0x0B090A08u);
        const uint32_t m2 = __builtin_amdgcn_perm(fy, fw, 0x0B090A08u);
        dw[k] = and_or(m2, M2, j == 0 ? (m1 & M1) : and_or(m1, M1, dw[k]));
        Ek[k] = En;
        f = Fn;
        diag = Hin[k];
        Hout[k] = H;
    }
    f_out = f;
}

// ---------------------------------------------------------------------------
// SEMI step (transposed): registers = target columns, one query row per step.
// Values drift by e per anti-diagonal (semi_frame below): cell (r, c) stores
//   F^ = B + F + e(r+c),  E^ = B + E + e(r+c),  Hm^ = B + H - OE + e(r+c) + e,
// so the gap extensions cost nothing, F(r,c) = max(Hm(r-1,c), F(r-1,c) - e) is
// max(Hm^(r-1,c), F^(r-1,c)) and E likewise, the diagonal H(r-1,c-1) + s is
// Hm^(r-1,c-1) + (s + OE + e) (table offset K = OE + e) and Hm^ = max3 - o:
// 6 instructions per two cells instead of 8.  In: diag_top = Hm^(r-1, c0-1),
// hl/el = Hm^(r, c0-1) / E^(r, c0-1) entering the lane's first column.
// ---------------------------------------------------------------------------
// PV > 0 (TAIL=QUERY/BOTH kernel): the last PV registers may hold pad columns of the
// target, which the reference scores by its N rule (Q6/Q7, read by Q11); their selector
// picks the constant 0 and pv adds the N score + K per half (0 for real columns).
template <int R, int PV = 0>
__device__ __forceinline__ void step_semi(const uint2 T, const uint32_t diag_top, uint32_t &hl, uint32_t &el,
                                          const uint32_t (&xs)[R], const uint32_t (&Hin)[R], uint32_t (&Hout)[R],
                                          uint32_t (&Fk)[R], const uint32_t GO, const uint32_t *pv = nullptr) {
    uint32_t diag = diag_top, h = hl, e = el;
#if GX_SEMI_IL2
    constexpr int R2 = R & ~1;
#pragma unroll
    for (int k = 0; k < R2; k += 2) {
        uint32_t v0 = __builtin_amdgcn_perm(T.y, T.x, xs[k]), v1 = __builtin_amdgcn_perm(T.y, T.x, xs[k + 1]);
        if (PV > 0 && k >= R - PV) v0 = pk_addnc(v0, pv[k - (R - PV)]);
        if (PV > 0 && k + 1 >= R - PV) v1 = pk_addnc(v1, pv[k + 1 - (R - PV)]);
        asm volatile("" : "+v"(v0), "+v"(v1));
        uint32_t t0 = pk_addnc(diag, v0), t1 = pk_addnc(Hin[k], v1);
        uint32_t F0 = pk_max_u16(Hin[k], Fk[k]), F1 = pk_max_u16(Hin[k + 1], Fk[k + 1]);
        asm volatile("" : "+v"(t0), "+v"(t1), "+v"(F0), "+v"(F1));
        e = pk_max_u16(h, e);
        h = pk_subnb(pk_max3(t0, F0, e), GO);
        Hout[k] = h;
        e = pk_max_u16(h, e);
        h = pk_subnb(pk_max3(t1, F1, e), GO);
        Hout[k + 1] = h;
        Fk[k] = F0;
        Fk[k + 1] = F1;
        diag = Hin[k + 1];
    }
#pragma unroll
    for (int k = R2; k < R; ++k) {
#else
#pragma unroll
    for (int k = 0; k < R; ++k) {
#endif
        uint32_t v = __builtin_amdgcn_perm(T.y, T.x, xs[k]);
        if (PV > 0 && k >= R - PV) v = pk_addnc(v, pv[k - (R - PV)]);
        const uint32_t tmp = pk_addnc(diag, v);                     // H(r-1,c-1) + s
        Fk[k] = pk_max_u16(Hin[k], Fk[k]);                           // F(r,c)
        e = pk_max_u16(h, e);                                        // E(r,c)
        h = pk_subnb(pk_max3(tmp, Fk[k], e), GO);                    // H(r,c) - OE
        diag = Hin[k];
        Hout[k] = h;
    }
    hl = h;
    el = e;
}

// ---------------------------------------------------------------------------
// Direction-flag stores of the packed traceback kernels, one 4-step window w.
// A chunk is 4 rows x 4 steps of one pair (8 bytes, rows k..k+3 of lane lg).
//  * per pair (tb_q8 = 0; sorted launches): window w of a pair holds G*R uint16,
//    row lg*R + k at ((k/4)*G + lg)*4 + k%4, so a lane group's store is 8*G
//    contiguous bytes;
//  * interleaved (tb_q8 = 1; unsorted launches, whose waves hold 8 consecutive
//    pairs): the 8 pairs of a wave share one region at pair (p & ~7), chunk
//    ((w*R/4 + k/4)*G + lg)*8 + (p & 7).  A lane's two halves are adjacent pairs,
//    so it stores both chunks as one 16-byte word and a wave's store is 1 KB
//    contiguous; walks of neighbouring pairs that sit at the same cell read the
//    same line (tb_kernel, profiles/r03_tb_walk.md).
// ---------------------------------------------------------------------------
template <int G, int R>
__device__ __forceinline__ void tb_store_window(const WfArgs &A, const uint32_t (&pr)[2], const bool (&valid)[2],
                                                const uint32_t (&W16)[2], const uint32_t w, const uint32_t lg,
                                                const uint32_t (&dw)[R]) {
    if (A.tb_q8) {
        if ((valid[0] && w < W16[0]) || (valid[1] && w < W16[1])) {
            uint4 *dst = reinterpret_cast<uint4 *>(A.tb + (uint64_t)(pr[0] & ~7u) * A.tb_pair_words) +
                         ((uint64_t)w * (R / 4) * G + lg) * 4 + ((pr[0] & 7u) >> 1);
#pragma unroll
            for (int k = 0; k < R; k += 4)
                dst[(k / 4) * G * 4] = make_uint4(__builtin_amdgcn_perm(dw[k + 1], dw[k], 0x05040100u),
                                                  __builtin_amdgcn_perm(dw[k + 3], dw[k + 2], 0x05040100u),
                                                  __builtin_amdgcn_perm(dw[k + 1], dw[k], 0x07060302u),
                                                  __builtin_amdgcn_perm(dw[k + 3], dw[k + 2], 0x07060302u));
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (valid[h] && w < W16[h]) {
            uint16_t *dst = reinterpret_cast<uint16_t *>(A.tb + (uint64_t)pr[h] * A.tb_pair_words) +
                            (uint64_t)w * (G * R) + lg * 4;
            const uint32_t sel = h ? 0x07060302u : 0x05040100u;
#pragma unroll
            for (int k = 0; k < R; k += 4)
                *reinterpret_cast<uint2 *>(dst + k * G) =
                    make_uint2(__builtin_amdgcn_perm(dw[k + 1], dw[k], sel), __builtin_amdgcn_perm(dw[k + 3], dw[k + 2], sel));
        }
    }
}

// ---------------------------------------------------------------------------
// The kernel.
// ---------------------------------------------------------------------------
constexpr int WF16_GLOBAL_TB = 3;     // GLOBAL with traceback words (wavefront16 only)
constexpr int WF16_LOCAL_TB = 4;      // LOCAL with traceback words (wavefront16 only)
constexpr int WF16_LOCAL_K2 = 5;      // LOCAL, padded targets of 257..512 columns (two keys per row)
constexpr int WF16_SEMI_TQ = 6;       // SEMI with TAIL = QUERY / BOTH: the last padded column's rows (Q11)
// GLOBAL + traceback by band recomputation (dispatch.hip, plan tb_band):
//  * WF16_GLOBAL_CP: the score-only GLOBAL sweep (step_global, no flags) that also stores, for
//    every lane lg, its R rows' (H, E) at the column left of its band window [L, L + wd), L =
//    max(lg*R - w, 0), and its bottom row's hand-off (H, F) over the window of the lane below;
//  * then, in the same kernel (band_pass), every lane recomputes its R x wd window from those
//    values alone, with the direction flags of step_global_tb (identical inputs, identical
//    flags), one 4-column window of flags at a time into bflags.  tb_kernel walks the band and
//    hands the pairs whose path leaves it to a WF16_GLOBAL_TB launch over the full matrix
//    (dispatch.hip).
// Per cell pair the sweep issues 7 instructions instead of step_global_tb's 15; the band is
// R x wd of every lane's G*R x (ypad) cells (config 3, w = 12: 44 of 304 columns).
// entries per lane of the band hand-off stream: wd + 1 used, rounded up to blocks of 4, plus the
// two blocks the band pass prefetches past its last one
__host__ __device__ constexpr uint32_t band_stream_words(uint32_t wd) { return ((wd + 1 + 3) & ~3u) + 8; }
constexpr int WF16_GLOBAL_CP = 7;
// SEMI TAIL=TARGET reverse pass of WITH_START (start.hpp, A.stop): the forward instances keep
// no stop branch, whose per-column constants the compiler hoisted out of the sweep and spilled
// (config 4: 32 B of scratch per lane, 0.73 GB of traffic per launch)
constexpr int WF16_SEMI_STOP = 9;
constexpr int WF16_LOCAL_U16 = 10;    // LOCAL score + ends in the e-drift frame, u16 keys (step_local_dr U16)
constexpr int WF16_LOCAL_RS = 11;     // LOCAL reverse pass of WITH_START (A.lstop early stop), f16 keys
constexpr int WF16_LOCAL_U16_RS = 12; // the same with u16 keys (local_rs.hip instances)
// LOCAL with f16-pattern keys by step segments: key = H*M + (M-1-t), t = the step within a
// segment of M = 2^kseg_shift steps (lane lg: columns [jM - lg, (j+1)M - lg)), so the range
// is (Hmax + 1) * M <= 0x7800 whatever the target length; at each segment's end (the same step
// in every lane: no masked work) the keys go to A.kseg and restart; the final merge takes per
// row the first segment holding its maximum (later columns win only when strictly higher)
constexpr int WF16_LOCAL_SEG = 13;
constexpr int WF16_LOCAL_TBD = 14;    // LOCAL + traceback in the e-drift frame (step_local_tb_dr)
constexpr int WF16_LOCAL_SEGR = 15;   // WF16_LOCAL_SEG with the finished segments' best per row in registers
constexpr int kW16_LTBD_WAVES = 2;
constexpr int kW16_TQ_WAVES = 3;
constexpr int kW16_TQ_BIG_WAVES = 3;   // R > 20: 3 waves spill (R = 23: 20 VGPRs) and still beat 2 (profiles/r03_semi_tq_waves_ab.md)
constexpr int kW16_CP_WAVES = 3;    // GLOBAL score sweep with band checkpoints, then its band pass

// waves per SIMD the register allocator must allow, per instance
__host__ __device__ constexpr int wf16_waves(int algo, int R) {
    return algo == WF16_GLOBAL_TB ? kW16_TB_WAVES
           : algo == WF16_LOCAL_TB ? kW16_LTB_WAVES
           : algo == WF16_LOCAL_TBD ? (R <= 12 ? 3 : kW16_LTBD_WAVES)   // G16R12: the 3-wave A/B shape
           : algo == WF16_LOCAL_SEGR ? 2                                 // 2R more VGPRs than WF16_LOCAL_SEG
           : algo == WF16_LOCAL_K2 ? kW16_K2_WAVES
           : algo == WF16_SEMI_TQ ? (R > 20 ? kW16_TQ_BIG_WAVES : kW16_TQ_WAVES)
           : algo == WF16_GLOBAL_CP ? kW16_CP_WAVES
           : GX_WF16_WAVES;
}

template <int ALGO_, int G, int R>
__global__ __launch_bounds__(kBlock, wf16_waves(ALGO_, R)) void wf16_kernel(WfArgs A) {
    const uint32_t wf16_bid = blockIdx.x, wf16_bl = blockIdx.x, wf16_p0 = 0, wf16_lds = A.lds_stride;
#include "wf16_body.inc"
}

// One launch, two shapes: blocks [0, A.tail_b0) run (G1, R1) over slots [0, A.tail_p0), the rest run
// (G2, R2) -- more lanes per pair, fewer rows per lane, so a wave is a third as long -- over the
// slots from A.tail_p0 on.  Blocks are dispatched in order, so the short waves fill the slots the
// long ones leave at the end of the launch instead of the last long waves running alone (a launch
// of W waves over S resident slots ends with about one wave time at a fraction of the chip:
// config 2 ran 1.7 % faster at 983,040 pairs, 20 full rounds, than at 1 M, profiles/r06/tail/).
// The flags in A.handled follow the blocks (A.skip_* tell the int32 kernel their slot ranges).
template <int ALGO_, int G1, int R1, int G2, int R2>
__global__ __launch_bounds__(kBlock, wf16_waves(ALGO_, R1)) void wf16_mix_kernel(WfArgs A) {
    if (blockIdx.x < A.tail_b0) {
        constexpr int G = G1, R = R1;
        const uint32_t wf16_bid = blockIdx.x, wf16_bl = blockIdx.x, wf16_p0 = 0, wf16_lds = A.lds_stride;
#include "wf16_body.inc"
    } else {
        constexpr int G = G2, R = R2;
        const uint32_t wf16_bid = blockIdx.x, wf16_bl = blockIdx.x - A.tail_b0, wf16_p0 = A.tail_p0,
                       wf16_lds = A.tail_lds;
#include "wf16_body.inc"
    }
}

// SEMI TAIL=QUERY/BOTH instances, G = 8, R = 1..32 (semi_tq.hip; one per padded target
// length 8R): NULL outside that range
using Wf16Fn = void (*)(WfArgs);
Wf16Fn wf16_tq_lookup(int R);
// LOCAL e-drift instances with u16 keys and/or the reverse pass's early stop (local_rs.hip):
// NULL for shapes outside kShapes16
Wf16Fn wf16_local_lookup(int G, int R, bool u16, bool rs, bool seg = false);
// WITH_START reverse passes with the register axis sized per block (rclass.hip): NULL when the
// plan's instance (algo, G, R) has no class set
Wf16Fn wf16_rclass_lookup(int algo, int G, int R);

}  // namespace gx
