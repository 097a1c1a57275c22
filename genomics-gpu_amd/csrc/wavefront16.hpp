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
template <int R, bool KEYS, bool U16 = false>
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
#pragma unroll
    for (int k = 0; k < R; ++k) {
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
            a1 -= EM;   // row k + 1: FL one e higher
            a2 -= EM;
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
#pragma unroll
    for (int k = 0; k < R; ++k) {
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
template <int R, bool KEYS>
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
#pragma unroll
    for (int k = 0; k < R; ++k) {
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
constexpr int kW16_LTBD_WAVES = 2;
constexpr int kW16_TQ_WAVES = 3;
constexpr int kW16_TQ_BIG_WAVES = 3;   // R > 20: 3 waves spill (R = 23: 20 VGPRs) and still beat 2 (profiles/r03_semi_tq_waves_ab.md)
constexpr int kW16_CP_WAVES = 3;    // GLOBAL score sweep with band checkpoints, then its band pass

template <int ALGO_, int G, int R>
__global__ __launch_bounds__(kBlock, ALGO_ == WF16_GLOBAL_TB ? kW16_TB_WAVES
                                   : ALGO_ == WF16_LOCAL_TB ? kW16_LTB_WAVES
                                   : ALGO_ == WF16_LOCAL_TBD ? kW16_LTBD_WAVES
                                   : ALGO_ == WF16_LOCAL_K2 ? kW16_K2_WAVES
                                   : ALGO_ == WF16_SEMI_TQ ? (R > 20 ? kW16_TQ_BIG_WAVES : kW16_TQ_WAVES)
                                   : ALGO_ == WF16_GLOBAL_CP ? kW16_CP_WAVES
                                   : GX_WF16_WAVES) void wf16_kernel(WfArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr bool GTB = ALGO_ == WF16_GLOBAL_TB;
    constexpr bool GCP = ALGO_ == WF16_GLOBAL_CP;
    constexpr bool GT = GTB || GCP;   // the traceback kernels' declines and start-cell capture
    constexpr bool LTB = ALGO_ == WF16_LOCAL_TB;
    constexpr bool K2 = ALGO_ == WF16_LOCAL_K2;
    constexpr bool KU16 = ALGO_ == WF16_LOCAL_U16 || ALGO_ == WF16_LOCAL_U16_RS;
    constexpr bool LRS = ALGO_ == WF16_LOCAL_RS || ALGO_ == WF16_LOCAL_U16_RS;   // (the check costs VGPRs)
    constexpr bool KSEG = ALGO_ == WF16_LOCAL_SEG;
    constexpr bool LTBD = ALGO_ == WF16_LOCAL_TBD;
    // TQ: one launch per class of equal padded target length G*R (dispatch.hip), so the
    // last padded column is always register R - 1 of lane G - 1
    constexpr bool TQ = ALGO_ == WF16_SEMI_TQ;
    static_assert(!TQ || G == 8, "TAIL=QUERY/BOTH instances are G = 8");
    constexpr bool STOPK = ALGO_ == WF16_SEMI_STOP;
    constexpr int ALGO = GT ? WF_GLOBAL : (LTB || K2 || KU16 || LRS || KSEG || LTBD) ? WF_LOCAL : (TQ || STOPK) ? WF_SEMI : ALGO_;
    constexpr int S = 64 / G;            // lane groups per wave
    constexpr bool TR = ALGO == WF_SEMI; // transposed: X = target, Y = query
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1), slot = lane / G;
    // a launch over a device-side count (the traceback fallback list): whole blocks past it leave
    const uint32_t nn = A.n_dev ? min(*A.n_dev, A.n) : A.n;
    if (A.n_dev && blockIdx.x * (uint32_t)(kWavesPerBlock * 2 * S) >= nn) return;
    const uint32_t wv = blockIdx.x * kWavesPerBlock + wave;   // wave index of the launch
    const uint32_t pair0 = (TQ ? A.slot0 : 0u) + wv * (2 * S);
    uint32_t pr[2], xl[2], yl[2], xo[2], yo[2], xpad[2], ypad[2];
    bool valid[2];
    const uint8_t *X = TR ? A.t : A.q, *Y = TR ? A.q : A.t;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t idx = pair0 + 2 * slot + h;   // slot; the pair is perm[slot] when sorted
        valid[h] = idx < nn;
        pr[h] = (valid[h] && A.perm) ? A.perm[idx] : idx;
        const uint32_t ql = valid[h] ? A.qlen[pr[h]] : 0, tl = valid[h] ? A.tlen[pr[h]] : 0;
        const uint32_t qo = valid[h] ? A.qoff[pr[h]] : 0, to = valid[h] ? A.toff[pr[h]] : 0;
        xl[h] = TR ? tl : ql; yl[h] = TR ? ql : tl;
        xo[h] = TR ? to : qo; yo[h] = TR ? qo : to;
        xpad[h] = (xl[h] + 7u) & ~7u;
        ypad[h] = (yl[h] + 7u) & ~7u;
    }
    uint32_t ymaxw = max(ypad[0], ypad[1]);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) ymaxw = max(ymaxw, (uint32_t)__shfl_xor(ymaxw, m));

    const Pk16 P = pk16_params<ALGO>(A);
    const int32_t NS = A.has_npen ? -A.npen : 0;
    // table bytes for a Y code (per X letter j): match / mismatch / N / outside
    const int32_t nrule = (ALGO == WF_GLOBAL) ? (A.has_npen ? NS : -A.b) : NS;   // gasal_kernels.h:44-54
    const uint32_t t_mis = (uint32_t)(P.k - A.b) * 0x01010101u;
    const uint32_t t_n = (uint32_t)(nrule + P.k) * 0x01010101u;
    const uint32_t t_out = (uint32_t)P.k * 0x01010101u;            // score 0
    const uint32_t t_match = (uint32_t)(A.a + P.k);

    // ---- stage the step-axis sequences as score tables, one uint2 per position
    //      (x: pair 0, y: pair 1), positions [-G, ymaxw + G) ----
    const uint32_t words = A.lds_stride >> 3;            // positions per slot, >= ymaxw + 2G + 4, multiple of 4
    uint2 *wl = reinterpret_cast<uint2 *>(lds) + (size_t)wave * S * words;
    bool other = false;                                  // a code the packed path cannot score
    for (uint32_t base = 0; base < S * (words >> 2); base += 64) {
        const uint32_t idx = base + lane;
        const uint32_t ps = min(idx / (words >> 2), (uint32_t)S - 1);
        const uint32_t y0 = 4 * (idx - ps * (words >> 2)) - G;   // first position of this quad
        uint32_t tab[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t yp = __shfl(ypad[h], ps * G), yof = __shfl(yo[h], ps * G);
            const uint32_t ylen = __shfl(yl[h], ps * G);
            uint32_t v = 0;
            const bool in = (int32_t)y0 >= 0 && y0 < yp;
            if (in) v = load4_codes_dir(A, Y, yof, ylen, y0 >> 2);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t l = in ? letter_of((v >> (8 * j)) & 15u, A.nval) : 6u;
                other |= l == 5;
                // traceback reads the first pad query row, scored here as -K: exact for
                // pad x base columns, not for pad x real-N columns (N == N is a match)
                if (GT && !A.has_npen) other |= l == 4 && y0 + j < ylen;
                if (GT) other |= in && y0 + j >= ylen && l != 4;   // start-cell fix assumes N pads
                tab[h][j] = l == 6 ? t_out : l == 4 ? t_n : (t_mis & ~(0xFFu << (8 * l))) | (t_match << (8 * l));
            }
        }
        if (idx < S * (words >> 2)) {
            uint2 *dst = wl + ps * words + 4 * (idx - ps * (words >> 2));
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[j] = make_uint2(tab[0][j], tab[1][j]);
        }
    }
    // ---- register-axis letters: selector bytes 0 / 2 (0x0C = constant 0 outside) ----
    const uint32_t r0 = lg * R;
    uint32_t xs[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t r = r0 + k;
        xs[k] = 0x0C0C0C0Cu;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (valid[h] && r < xpad[h]) {
                // (WITH_START reverse pass: position r of "the first xl bases, reversed", N past xl)
                const uint32_t pos = A.rev ? xl[h] - 1u - r : r;
                const uint32_t cde = A.rev && r >= xl[h] ? (uint32_t)A.nval
                                     : A.packed ? (load4_codes(X, xo[h], pos >> 2, 1) >> (8 * (pos & 3))) & 15u
                                                : (uint32_t)X[xo[h] + pos] & 15u;
                const uint32_t l = letter_of(cde, A.nval);
                if (r < xl[h]) {
                    other |= l >= 4;                 // real positions must be A/C/G/T
                    xs[k] = (xs[k] & ~(0xFFu << (16 * h))) | ((l + 4 * h) << (16 * h));
                } else if (ALGO == WF_LOCAL || GT || TQ) {
                    other |= l != 4;                 // pads must be N (LOCAL: scored -K here, dominated;
                }                                    // TQ: scored by the N rule through pv)
            }
        }
    }
    // TQ: pad columns sit in the last PV registers (of the last lanes); their N-rule score
    constexpr int PV = TQ ? (R < 7 ? R : 7) : 0;
    uint32_t pv[PV > 0 ? PV : 1];
    if constexpr (TQ) {
        const int32_t nrule = A.has_npen ? -A.npen : 0;   // gasal_kernels.h:44-51 LOCAL macro (semi-global uses it)
#pragma unroll
        for (int j = 0; j < PV; ++j) {
            const uint32_t r = r0 + (R - PV) + j;
            pv[j] = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (valid[h] && r >= xl[h] && r < xpad[h]) pv[j] |= (uint32_t)(nrule + P.k) << (16 * h);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) other |= valid[h] && xpad[h] != (uint32_t)(G * R);   // the launch's class
    }
    const bool fast = A.fast16 && !A.force_exact && !__syncthreads_or(other);
    if constexpr (TQ) {
        // flags per slot: class launches cover slot ranges that need not align to blocks
        if (lg == 0)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (valid[h]) A.handled[pair0 + 2 * slot + h] = fast ? 1 : 0;
    } else if (threadIdx.x == 0) {
        A.handled[blockIdx.x] = fast ? 1 : 0;
    }
    if (!fast) return;                                   // the int32 kernel takes this block

    const uint32_t nsteps = ymaxw + G - 1;
    const uint2 *tcol = wl + slot * words;
    const uint32_t EXT = pk_bcast(A.e);
    const uint32_t GO = pk_bcast(A.o);                   // SEMI: Hm^ = max3 - o (step_semi's frame)
    const uint32_t BB = (uint32_t)P.base * 0x10001u;
    const uint32_t NN = (uint32_t)P.neg * 0x10001u;
    const bool top = lg == 0;
    int32_t c = -(int32_t)lg;                            // step-axis position of this lane

    auto band_pass = [&]() __attribute__((always_inline)) {
      if constexpr (GCP) {
        // Band recomputation (the WF16_GLOBAL_CP kernel once its sweep is done): lane lg's rows r0..r0+R-1 over the columns
        // [L, L + wd), L = max(r0 - w, 0), from the state WF16_GLOBAL_CP stored (same frame,
        // same tables, so step_global_tb sees the inputs the full traceback sweep would).
        // Entering column L: H(r, L - 1) and E(r, L) of the lane's rows (the left boundary of
        // global.h:57-60 when L = 0); per column c: the upper lane's H(r0 - 1, c - 1) and
        // F(r0, c) (stream entries c - L and c - L + 1), or the top boundary for lane 0.
        static_assert(R % 4 == 0, "band windows store flags in groups of 4 rows");
        const int32_t pb = P.base, go = A.o, ge = A.e, D = P.drift;
        const uint32_t KX = pk_bcast(P.k - 2 * D), OEX = pk_bcast(P.k - 2 * D + A.o + A.e - D);
        const uint32_t WD = A.band_wd;
        const int32_t L = max((int32_t)r0 - (int32_t)A.band_w, 0);
        // (element by element: a whole-array copy here became one <R x i32> value, a register
        // tuple the allocator could only place by spilling ~350 VGPRs)
        uint32_t HA[R], HB[R], Ek[R], dw[R];
        const uint32_t *cpw = A.cp + ((size_t)wv * 64 + lane) * (2 * R);
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int32_t r = (int32_t)r0 + k;
            // H(r, -1) (Q2) at anti-diagonal r - 1, E(r, 0) = -inf; else the sweep's checkpoint
            HA[k] = L == 0 ? (uint32_t)(pb + D * (r - 1) - (r <= 0 ? 0 : go + ge * r)) * 0x10001u : cpw[k];
            Ek[k] = L == 0 ? NN : cpw[R + k];
            HB[k] = HA[k];
            dw[k] = 0;
        }
        // the upper lane's stream (lane 0 reads a neighbour's and ignores it), [wave][lane][SW]:
        // blocks of 4 entries as two 16-byte loads, the block two ahead in flight (the loads
        // of one entry two steps ahead stalled the pass on their latency)
        const uint32_t SW = band_stream_words(WD);
        const uint4 *sp = reinterpret_cast<const uint4 *>(A.stm + ((size_t)wv * 64 + (lane ? lane - 1 : 0)) * SW);
        uint4 B0a = sp[0], B0b = sp[1], B1a = sp[2], B1b = sp[3];
        // a window from column 0 starts at the left boundary: H(r0 - 1, -1) (Q2; lane 0 of the
        // sweep never runs column -1, so lane 1's entry 0 is not stored)
        if (L == 0) B0a.x = (uint32_t)(pb + D * ((int32_t)r0 - 2) - (r0 <= 1 ? 0 : go + ge * ((int32_t)r0 - 1))) * 0x10001u;
        uint4 *bf = A.bflags + ((size_t)wv * 64 + lane) * (WD / 4) * (R / 4);
        const bool any = valid[0] || valid[1];
        c = L;
        uint32_t fdummy = NN;
        // entry t: (H(r0 - 1, c - 1), F(r0, c)) for c = L + t - 1 ... step j of a block takes the
        // diagonal from entry j and F from entry j + 1
        auto bstep = [&](const int j, uint32_t (&Hin)[R], uint32_t (&Hout)[R], const uint32_t hd, const uint32_t fu)
            __attribute__((always_inline)) {
            const uint2 T = tcol[c + G];
            // H(-1, c - 1) at anti-diagonal c - 2 (the GLOBAL branch's dtop)
            const uint32_t dtop = (uint32_t)(pb + D * (c - 2) - (c <= 0 ? 0 : go + ge * c)) * 0x10001u;
            step_global_tb<R, true>(T, top ? dtop : hd, top ? NN : fu, xs, Hin, Hout, Ek, dw, fdummy, KX, OEX, NN, j);
            ++c;
        };
        // columns past ymaxw (the wave's widest padded target; the walk starts at most at column
        // tl <= ymaxw, Q9) are never visited: a lane whose window runs past them stops there
        // (the table reads of those columns fell outside the slot's staged positions)
        const uint32_t tmax = (uint32_t)L <= ymaxw ? min(WD, (ymaxw + 1u - (uint32_t)L + 3u) & ~3u) : 0u;
        for (uint32_t t = 0; t < WD; t += 4) {
            if (t >= tmax) break;                                    // (lane-divergent: no DPP in the band pass)
            const uint4 B2a = sp[t / 2 + 4], B2b = sp[t / 2 + 5];   // entries t + 8 .. t + 11
            bstep(0, HA, HB, B0a.x, B0a.w);
            bstep(1, HB, HA, B0a.z, B0b.y);
            bstep(2, HA, HB, B0b.x, B0b.w);
            bstep(3, HB, HA, B0b.z, B1a.y);
            B0a = B1a; B0b = B1b; B1a = B2a; B1b = B2b;
            if (any) {
                uint4 *dst = bf + (t / 4) * (R / 4);
#pragma unroll
                for (int k = 0; k < R; k += 4)
                    dst[k / 4] = make_uint4(__builtin_amdgcn_perm(dw[k + 1], dw[k], 0x05040100u),
                                            __builtin_amdgcn_perm(dw[k + 3], dw[k + 2], 0x05040100u),
                                            __builtin_amdgcn_perm(dw[k + 1], dw[k], 0x07060302u),
                                            __builtin_amdgcn_perm(dw[k + 3], dw[k + 2], 0x07060302u));
            }
        }
      }
    };

    if (ALGO == WF_LOCAL) {
        const uint32_t KK = pk_bcast(P.k), OEK = pk_bcast(A.o + A.e + P.k);
        const uint32_t KMUL = A.one << 8;
        const uint32_t bshift = ((uint32_t)P.base << 8) & 0xFFFFu;
        uint32_t HA[R], HB[R], Ek[R], key[R], key2[K2 ? R : 1];
        uint32_t jseg = 0;   // KSEG: segments saved to A.kseg (the live one is segment jseg)
#pragma unroll
        for (int k = 0; k < R; ++k) { HA[k] = BB; HB[k] = BB; Ek[k] = BB; key[k] = 0; }
#pragma unroll
        for (int k = 0; k < (K2 ? R : 1); ++k) key2[k] = 0;
        uint32_t recvH = BB, prevRecvH = BB, recvF = BB, f = BB;
        uint2 tnext = tcol[c + G];
        if constexpr (LTB) {
            // direction flags in the skewed layout of the GLOBAL+TB kernel (see there)
            static_assert(R % 4 == 0, "LOCAL+TB packed shapes need R % 4 == 0");
            uint32_t dw[R];
#pragma unroll
            for (int k = 0; k < R; ++k) dw[k] = 0;
            uint32_t W16[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) W16[h] = (ypad[h] + G + 2) >> 2;
            auto qstep = [&](const int j, uint32_t (&Hin)[R], uint32_t (&Hout)[R]) __attribute__((always_inline)) {
                const uint2 T = tnext;
                tnext = tcol[c + j + 1 + G];
                step_local_tb<R>(T, c + j, top ? BB : prevRecvH, top ? BB : recvF, xs, Hin, Hout, Ek, key, dw, f, KK,
                                 OEK, EXT, BB, KMUL, bshift, j);
                prevRecvH = recvH;
                recvH = (uint32_t)shr_lane((int32_t)Hout[R - 1]);
                recvF = (uint32_t)shr_lane((int32_t)f);
            };
            for (uint32_t s = 0; s < nsteps; s += 4, c += 4) {
                qstep(0, HA, HB);
                qstep(1, HB, HA);
                qstep(2, HA, HB);
                qstep(3, HB, HA);
                tb_store_window<G, R>(A, pr, valid, W16, s >> 2, lg, dw);   // layout: see tb_store_window
            }
        } else {
            uint32_t s = 0;
            // two steps (ping-pong HA/HB) per iteration, up to step `end`
            auto sweep = [&](auto kmc, const uint32_t end) __attribute__((always_inline)) {
                constexpr int KM = decltype(kmc)::value;
                auto &k2 = *reinterpret_cast<uint32_t(*)[R]>(K2 ? key2 : key);   // unused unless K2
                for (; s < end; s += 2, c += 2) {
                    uint2 T = tnext;
                    tnext = tcol[c + 1 + G];
                    step_local<R, KM>(T, c, top ? BB : prevRecvH, top ? BB : recvF, xs, HA, HB, Ek, key, k2, f, KK,
                                      OEK, EXT, BB, KMUL, bshift);
                    prevRecvH = recvH;
                    recvH = (uint32_t)shr_lane((int32_t)HB[R - 1]);
                    recvF = (uint32_t)shr_lane((int32_t)f);
                    T = tnext;
                    tnext = tcol[c + 2 + G];
                    step_local<R, KM>(T, c + 1, top ? BB : prevRecvH, top ? BB : recvF, xs, HB, HA, Ek, key, k2, f,
                                      KK, OEK, EXT, BB, KMUL, bshift);
                    prevRecvH = recvH;
                    recvH = (uint32_t)shr_lane((int32_t)HA[R - 1]);
                    recvF = (uint32_t)shr_lane((int32_t)f);
                }
            };
            if constexpr (K2) {
                // lane lg reaches column 256 at step 256 + lg
                sweep(std::integral_constant<int, 0>{}, min(nsteps, 256u));
                sweep(std::integral_constant<int, 1>{}, min(nsteps, 256u + G));
                sweep(std::integral_constant<int, 2>{}, nsteps);
            } else if (A.kf16) {
                // the e-drift frame (step_local_dr); f16-pattern keys 0x0400 + H*C + (C-1-c)
                // for the columns c < C, 0x0400 + H*C elsewhere (H = 0 left of the matrix;
                // right of the padded target no cell beats the real columns' maximum).
                // Lane lg starts at column c0 = -lg with "0 in the frame" everywhere, which
                // the garbage columns keep exactly (score 0, E at its floor), so they reach
                // column -1 as the left boundary H = E = 0.  Top lane: diag H(-1, c-1) = 0,
                // F(0, c) <= 0 (BB).
                const uint32_t C = A.kf16;
                // key multiplier: KSEG's segment length M, else the step range C + G (
                // keys rank steps, not columns, so that their addend is wave-uniform) or C
                const uint32_t CP = C + G;
                const uint32_t MK = KSEG ? (1u << A.kseg_shift) : CP, KMC = A.one * MK;
                const int32_t ge = A.e, pbv = P.base;
                const uint32_t EXT2 = pk_bcast(2 * ge);
                const uint32_t KXD = (uint32_t)((P.k - 2 * ge) * 0x10001),
                               OEXD = (uint32_t)((P.k - 2 * ge + A.o) * 0x10001);
                constexpr uint32_t KOFS = KU16 ? 0u : 0x0400u;   // u16 keys need no f16 offset
                uint32_t segend = MK;                            // KSEG: the current segment's end step
                uint32_t KMV = KMC;
                asm volatile("" : "+v"(KMV));   // the multiplier in a VGPR: the mads' scalar operand is the addend
                // the key base of the candidate at step ss: KOFS + (end - 1 - ss) + add * M, end = the
                // segment's end step (KSEG) or C + G; the garbage columns left of the matrix hold H = 0
                // and those right of it less than the maximum, so no column test is needed
                auto inv = [&](uint32_t ss, uint32_t add) __attribute__((always_inline)) {
                    return (KOFS + ((KSEG ? segend : CP) - 1u - ss) + add * MK) & 0xFFFFu;
                };
                // Each lane keeps the frame shifted by its own constant, e(k + s) instead of
                // e(r + c) (r = lg*R + k, c = s - lg): every floor FL[k] = B + e(k + s + 1) is
                // then the same in all lanes (scalar registers, s_add per step) and the
                // values a lane receives from the lane above drop by e(R - 1).
                uint32_t FL[R];
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    key[k] = KOFS * 0x10001u;
                    HA[k] = (uint32_t)(pbv + ge * (k - 1)) * 0x10001u;   // H^(r, c0 - 1) = 0
                    Ek[k] = (uint32_t)(pbv + ge * k) * 0x10001u;         // E^(r, c0) = its floor
                    FL[k] = (uint32_t)(pbv + ge * (k + 1)) * 0x10001u;   // floor of E(r, c0 + 1)
                }
                const uint32_t ADJ = pk_bcast(ge * (R - 1));
                // the diagonals of the first two steps, which no upper-lane step hands over
                // (lane 1's upper lane has no garbage column -1): H = 0 at k = -1, s - 1
                prevRecvH = (uint32_t)(pbv - 2 * ge) * 0x10001u;
                recvH = (uint32_t)(pbv - ge) * 0x10001u;
                // WITH_START reverse pass (A.lstop, start.hpp): no cell exceeds the forward score
                // S, so a key >= KOFS + S*C + (C-1-m) is a cell reaching S in a column <= m.  Once
                // lane G-1 has finished the strips up to column m and every pair has such a cell,
                // its first one in strip-major order (Q1) is settled: the sweep stops there
                // (local_kernel_template.h:441-511 stops at the first cell reaching the score).
                int32_t sstop[2] = {0, 0};
                if (LRS) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) sstop[h] = valid[h] ? A.lstop[pr[h]] : 0;
                }
                if constexpr (LTBD) {
                    // four steps per window of direction flags (tb_store_window, the LOCAL_TB layout);
                    // the keys of two columns on the second step of each pair
                    static_assert(R % 4 == 0, "LOCAL+TB packed shapes need R % 4 == 0");
                    uint32_t dw[R];
#pragma unroll
                    for (int k = 0; k < R; ++k) dw[k] = 0;
                    uint32_t W16[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) W16[h] = (ypad[h] + G + 2) >> 2;
                    uint32_t FL0 = FL[0];
                    auto tstep = [&](auto keysc, const int j, uint32_t (&Hin)[R], uint32_t (&Hout)[R])
                        __attribute__((always_inline)) {
                        constexpr bool KEYS = decltype(keysc)::value;
                        const uint2 T = tnext;
                        tnext = tcol[c + j + 1 + G];
                        const uint32_t dt = (uint32_t)(pbv + ge * (c + j - 2)) * 0x10001u;   // lane 0: H^(-1, c + j - 1)
                        step_local_tb_dr<R, KEYS>(T, top ? dt : prevRecvH, top ? BB : recvF, xs, Hin, Hout, Ek, key, FL0,
                                                  dw, f, KXD, OEXD, EXT, KMV, KEYS ? inv(s + j - 1, 0) : 0u,
                                                  KEYS ? inv(s + j, (uint32_t)(-ge)) : 0u, EXT2, MK, j);
                        prevRecvH = recvH;
                        recvH = pk_subnb((uint32_t)shr_lane((int32_t)Hout[R - 1]), ADJ);
                        recvF = pk_subnb((uint32_t)shr_lane((int32_t)f), ADJ);
                    };
                    for (; s < nsteps; s += 4, c += 4) {
                        tstep(std::false_type{}, 0, HA, HB);
                        tstep(std::true_type{}, 1, HB, HA);
                        tstep(std::false_type{}, 2, HA, HB);
                        tstep(std::true_type{}, 3, HB, HA);
                        tb_store_window<G, R>(A, pr, valid, W16, s >> 2, lg, dw);   // layout: see tb_store_window
                    }
                }
                for (; !LTBD && s < nsteps; s += 2, c += 2) {
                    if (KSEG && s == segend && jseg < A.kseg_n) {   // wave-uniform: a segment ends
                        // [wave][segment][lane][R]: one base address, immediate offsets
                        uint32_t *dst = A.kseg + (((size_t)wv * A.kseg_n + jseg) * 64 + lane) * R;
#pragma unroll
                        for (int k = 0; k < R; ++k) { dst[k] = key[k]; key[k] = KOFS * 0x10001u; }
                        ++jseg;
                        segend += MK;
                    }
                    uint2 T = tnext;
                    tnext = tcol[c + 1 + G];
                    const uint32_t dt0 = (uint32_t)(pbv + ge * (c - 2)) * 0x10001u;   // lane 0: H^(-1, c - 1)
                    step_local_dr<R, false, KU16>(T, top ? dt0 : prevRecvH, top ? BB : recvF, xs, HA, HB, Ek, key, FL, f,
                                            KXD, OEXD, EXT, KMC, 0u, 0u, EXT2);
                    prevRecvH = recvH;
                    recvH = pk_subnb((uint32_t)shr_lane((int32_t)HB[R - 1]), ADJ);
                    recvF = pk_subnb((uint32_t)shr_lane((int32_t)f), ADJ);
                    T = tnext;
                    tnext = tcol[c + 2 + G];
                    const uint32_t dt1 = (uint32_t)(pbv + ge * (c - 1)) * 0x10001u;
                    step_local_dr<R, true, KU16>(T, top ? dt1 : prevRecvH, top ? BB : recvF, xs, HB, HA, Ek, key, FL, f,
                                           KXD, OEXD, EXT, KMV, inv(s, 0), inv(s + 1, (uint32_t)(-ge)), EXT2, MK);
                    prevRecvH = recvH;
                    recvH = pk_subnb((uint32_t)shr_lane((int32_t)HA[R - 1]), ADJ);
                    recvF = pk_subnb((uint32_t)shr_lane((int32_t)f), ADJ);
                    if (LRS && (s & 7u) == 6u) {
                        const int32_t cl = (int32_t)s + 1 - (G - 1);                // lane G-1's last column
                        const int32_t m = min(((cl + 1) & ~7) - 1, (int32_t)C - 1);   // last settled strip's end
                        if (m >= 0) {
                            uint32_t mx = key[0];
#pragma unroll
                            for (int k = 1; k < R; ++k) mx = pk_max_u16(mx, key[k]);
                            bool hit[2];
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                // (the key of column m: step m + lg)
                                const uint32_t thr = KOFS + (uint32_t)sstop[h] * MK +
                                                     (CP - 1u - (uint32_t)m - lg);
                                hit[h] = !valid[h] || sstop[h] <= 0 || ((mx >> (16 * h)) & 0xFFFFu) >= thr;
                            }
                            if (groups_all<G>(__ballot(hit[0])) && groups_all<G>(__ballot(hit[1]))) break;
                        }
                    }
                }
            } else {
                sweep(std::integral_constant<int, 0>{}, nsteps);
            }
        }
        // ---- strip-major first maximum per pair (Q1) ----
        // e-drift keys (A.kf16; not K2 / KSEG / the round-2 TB kernel): key = KOFS + H*C' + (C'-1-s),
        // C' = C + G, s = the step (column c = s - lg).  Decoding every row's key took a 32-bit
        // division per row and half (4 quarter-rate multiplies each, ~6 % of the config-2 kernel);
        // instead the lane's largest H comes from its largest key (one division per half), and
        // among the rows holding it the strip-major first cell is a packed minimum of the 16-bit
        // codes (strip << 8 | k << 3 | col & 7), rows below that H masked to 0xFFFF.  Rows past
        // the pair's padded query (garbage rows) never hold a larger H than the last real row
        // above them in the lane, and tie it only in a later row of the same or a later strip.
        uint64_t bestv[2] = {0, 0};
        static_assert(R <= 32, "row index of the merge codes: 5 bits");
        const bool fastkey = !K2 && !LTB && !KSEG && A.kf16 && A.kf16 + G <= 2048;   // strip: 8 bits
        if (fastkey) {
            const uint32_t C = A.kf16 + G;
            constexpr uint32_t KOFS_ = KU16 ? 0u : 0x0400u;
            uint32_t km = key[0];
#pragma unroll
            for (int k = 1; k < R; ++k) km = pk_max_u16(km, key[k]);
            uint32_t thr = 0, Hm[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                Hm[h] = (((km >> (16 * h)) & 0xFFFFu) - KOFS_) / C;
                thr |= (KOFS_ + Hm[h] * C) << (16 * h);
            }
            const uint32_t cb = pk_bcast((int32_t)(C - 1u - lg));   // col = cb - (key - thr)
            const pk_u2 one = {1, 1}, ffff = {0xFFFF, 0xFFFF};
            uint32_t bc = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const uint32_t t = GX_AS(uint32_t, GX_AS(pk_u2, key[k]) - GX_AS(pk_u2, thr));
                const pk_u2 below = __builtin_elementwise_min(__builtin_elementwise_sub_sat(GX_AS(pk_u2, thr),
                                                                                            GX_AS(pk_u2, key[k])), one);
                const uint32_t col = GX_AS(uint32_t, GX_AS(pk_u2, cb) - GX_AS(pk_u2, t));
                // (a 16-bit shift per half: the masked rows' col is garbage, and a 32-bit shift would
                // carry its high bits into the other half's code)
                const pk_u2 sh5 = {5, 5};
                const uint32_t code = GX_AS(uint32_t, GX_AS(pk_u2, col & 0xFFF8FFF8u) << sh5) | (col & 0x00070007u) |
                                      ((uint32_t)(k << 3) * 0x10001u) | GX_AS(uint32_t, below * ffff);
                bc = GX_AS(uint32_t, __builtin_elementwise_min(GX_AS(pk_u2, bc), GX_AS(pk_u2, code)));
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t c16 = (bc >> (16 * h)) & 0xFFFFu, k = (c16 >> 3) & 31u, r = r0 + k;
                if (Hm[h] > 0 && c16 != 0xFFFFu && r < xpad[h]) {
                    const uint32_t ord = (((c16 >> 8) * xpad[h] + r) << 3) + (c16 & 7u);
                    bestv[h] = ((uint64_t)Hm[h] << 32) | (0xFFFFFFFFu - ord);
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint64_t best = bestv[h];
#pragma unroll
            for (int k = 0; k < R && !fastkey; ++k) {
                const uint32_t r = r0 + k;
                const uint32_t kk = (key[k] >> (16 * h)) & 0xFFFFu;
                uint32_t H = kk >> 8, col = 255u - (kk & 0xFFu);
                if (KSEG) {
                    // the first segment holding the row's maximum: the saved segments in order, then
                    // the live one (keys 0x0400 + H*M + (M-1-t), t = the step within the segment)
                    const uint32_t ms = A.kseg_shift;
                    H = 0;
                    col = 0;
                    auto seg = [&](const uint32_t j, const uint32_t kv) __attribute__((always_inline)) {
                        const uint32_t x = ((kv >> (16 * h)) & 0xFFFFu) - 0x0400u;
                        const uint32_t Hj = x >> ms, t = x & ((1u << ms) - 1u);
                        if (Hj > H) { H = Hj; col = ((j + 1) << ms) - 1u - t - lg; }
                    };
                    const uint32_t *src = A.kseg + ((size_t)wv * A.kseg_n * 64 + lane) * R + k;
                    for (uint32_t j = 0; j < jseg; ++j) seg(j, src[(size_t)j * (64 * R)]);
                    seg(jseg, key[k]);
                }
                if constexpr (K2) {   // columns 256..511: later, so they win only when strictly higher
                    const uint32_t k2v = (key2[k] >> (16 * h)) & 0xFFFFu;
                    if ((k2v >> 8) > H) { H = k2v >> 8; col = 511u - (k2v & 0xFFu); }
                }
                if (r < xpad[h] && H > 0) {
                    const uint32_t ord = (((col >> 3) * xpad[h] + r) << 3) + (col & 7);
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
                    qe = (int32_t)(rest % xpad[h]);
                    te = (int32_t)((rest / xpad[h]) * 8 + (ord & 7));
                }
                A.score[pr[h]] = H;                                   // local :428-430
                if (A.qend) A.qend[pr[h]] = qe;
                if (A.tend) A.tend[pr[h]] = te;
            }
        }
    } else if (ALGO == WF_GLOBAL) {
        // boundaries (global.h:57-71, Q2): H(r,-1) = -(o+e*r) (0 for r = 0), E = -inf;
        // top: H(-1,c-1) = -(o+e*c) (0 for c = 0), F = -inf.  Lanes sweep garbage
        // columns c < -1 first and reset to the left boundary at c = -1.
        const int32_t pb = P.base, go = A.o, ge = A.e, D = P.drift;   // D = e (step_global)
        const uint32_t KX = pk_bcast(P.k - 2 * D), OEX = pk_bcast(P.k - 2 * D + A.o + A.e - D);
        // H(r, -1) (Q2), stored at anti-diagonal r - 1
        auto left = [=](int32_t r) -> uint32_t {
            return (uint32_t)(pb + D * (r - 1) - (r <= 0 ? 0 : go + ge * r)) * 0x10001u;
        };
        uint32_t HA[R], HB[R], Ek[R];
        uint32_t dw[GTB ? R : 1];                      // traceback nibbles: last 4 steps per half
#pragma unroll
        for (int k = 0; k < R; ++k) { HA[k] = left((int32_t)(r0 + k)); HB[k] = HA[k]; Ek[k] = NN; }
#pragma unroll
        for (int k = 0; k < (GTB ? R : 1); ++k) dw[k] = 0;
        uint32_t recvH = left((int32_t)r0 - 1), prevRecvH = recvH, recvF = NN, f = NN;
        uint32_t kq_lane[2], kq[2], kp_lane[2], kp[2];
        bool fixable[2];
        int32_t score[2] = {0, 0}, fixv[2] = {0, 0};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            kq_lane[h] = (xl[h] - 1) / R;
            kq[h] = (xl[h] - 1) - kq_lane[h] * R;
            // traceback starts at (row ql, column tl); when both are pad
            // positions this kernel scores that cell -K instead of N==N, and records
            // its H so tb_kernel can redo the cell's low two bits
            fixable[h] = GT && valid[h] && xl[h] < xpad[h] && yl[h] < ypad[h];
            kp_lane[h] = xl[h] / R;
            kp[h] = xl[h] - kp_lane[h] * R;
        }
        // GCP: lane lg's band window starts at column L = max(r0 - w, 0): its rows' H(r, L - 1)
        // and E(r, L) are stored after the step at column L - 1 (none when L = 0: the left
        // boundary); the lane below's window starts at Ld = max(r0 + R - w, 0), and this lane's
        // bottom-row hand-off (H(r0 + R - 1, c), F(r0 + R, c)) is stored for c in [Ld - 1, Ld + wd]
        const int32_t cs_own = GCP ? max((int32_t)r0 - (int32_t)A.band_w, 0) - 1 : -1;
        const int32_t cs_dn = GCP ? max((int32_t)(r0 + R) - (int32_t)A.band_w, 0) - 1 : 0;
        const bool cp_on = GCP && (valid[0] || valid[1]);
        const bool st_on = cp_on && lg + 1 < G;
        uint32_t *cpw = GCP ? A.cp + ((size_t)wv * 64 + lane) * (2 * R) : nullptr;   // [wave][lane][2R]
        uint2 *stw = GCP ? A.stm + ((size_t)wv * 64 + lane) * band_stream_words(A.band_wd) : nullptr;   // [wave][lane][SW]
        uint2 tnext = tcol[c + G];
        // Capture window: the steps at which some lane of the wave holds a cell to capture --
        // row xl - 1 at column yl - 1 (the score, global.h:98-103,299) and, for traceback, row
        // xl at column yl (the start cell, tb_kernel) -- so that the steps outside it carry no
        // capture code: its per-register selects, if-converted, ran on every step (597 VALU
        // instructions per two steps of G16R20 instead of ~300, kernel_census.py).
        uint32_t cap_lo = 0xFFFFFFFFu, cap_hi = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (valid[h]) {
                const uint32_t sq = yl[h] - 1 + kq_lane[h];
                cap_lo = min(cap_lo, sq);
                cap_hi = max(cap_hi, sq);
                if (fixable[h]) {
                    const uint32_t sf = yl[h] + kp_lane[h];
                    cap_lo = min(cap_lo, sf);
                    cap_hi = max(cap_hi, sf);
                }
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            cap_lo = min(cap_lo, (uint32_t)__shfl_xor(cap_lo, m));
            cap_hi = max(cap_hi, (uint32_t)__shfl_xor(cap_hi, m));
        }
        // FLG bit 0: a lane may reach column -1 (its reset to the left boundary) in this
        // phase; bit 1: captures
        auto half_step = [&](auto flg, const int32_t cc, const int j, uint32_t (&Hin)[R], uint32_t (&Hout)[R]) __attribute__((always_inline)) {
            constexpr int FLG = decltype(flg)::value;
            const uint2 T = tnext;
            tnext = tcol[cc + 1 + G];
            if ((FLG & 1) && cc == -1) {
                int32_t rr = (int32_t)r0;
                asm volatile("" : "+v"(rr));   // keep the R boundary values out of loop-invariant registers
#pragma unroll
                for (int k = 0; k < R; ++k) { Hout[k] = left(rr + k); Ek[k] = NN; }
                f = NN;
                if (GTB && j == 0) {
#pragma unroll
                    for (int k = 0; k < R; ++k) dw[k] = 0;   // the window's flags are OR-ed in
                }
            } else {
                // H(-1, c-1) at anti-diagonal c - 2
                const uint32_t dtop = (uint32_t)(pb + D * (cc - 2) - (cc <= 0 ? 0 : go + ge * cc)) * 0x10001u;
                if constexpr (GTB)
                    step_global_tb<R>(T, top ? dtop : prevRecvH, top ? NN : recvF, xs, Hin, Hout, Ek, dw, f, KX,
                                      OEX, NN, j);
                else
                    step_global<R, GCP>(T, top ? dtop : prevRecvH, top ? NN : recvF, xs, Hin, Hout, Ek, f, KX, OEX, NN);
                if constexpr ((FLG & 2) != 0) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if (valid[h] && cc == (int32_t)yl[h] - 1 && lg == kq_lane[h]) {   // global.h:98-103,299
                            uint32_t v = 0;
#pragma unroll
                            for (int k = 0; k < R; ++k) v = (k == (int)kq[h]) ? Hout[k] : v;
                            score[h] = (int32_t)((v >> (16 * h)) & 0xFFFFu) - pb - D * (int32_t)(xl[h] + yl[h] - 2);
                        }
                        if (fixable[h] && cc == (int32_t)yl[h] && lg == kp_lane[h]) {
                            uint32_t v = 0;
#pragma unroll
                            for (int k = 0; k < R; ++k) v = (k == (int)kp[h]) ? Hout[k] : v;
                            fixv[h] = (int32_t)((v >> (16 * h)) & 0xFFFFu) - pb - D * (int32_t)(xl[h] + yl[h]);
                        }
                    }
                }
            }
            if constexpr (GCP) {
                if (cp_on && cc == cs_own) {
#pragma unroll
                    for (int k = 0; k < R; k += 2) {
                        *reinterpret_cast<uint2 *>(cpw + k) = make_uint2(Hout[k], Hout[k + 1]);
                        *reinterpret_cast<uint2 *>(cpw + R + k) = make_uint2(Ek[k], Ek[k + 1]);
                    }
                }
                const uint32_t t = (uint32_t)(cc - cs_dn);
                if (st_on && t <= A.band_wd) stw[t] = make_uint2(Hout[R - 1], f);
            }
            prevRecvH = recvH;
            recvH = (uint32_t)shr_lane((int32_t)Hout[R - 1]);
            recvF = (uint32_t)shr_lane((int32_t)f);
        };
        // Direction flags (GTB), skewed layout (read by tb_kernel): windows w = (column + lane)
        // / 4 holding the 4-step window's flags, every lane stores after the same steps
        // (tb_store_window: per pair, or 8 pairs interleaved).
        static_assert(!GTB || R % 4 == 0, "GLOBAL+TB packed shapes need R % 4 == 0");
        uint32_t W16[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) W16[h] = (ypad[h] + G + 2) >> 2;
        constexpr uint32_t STEP = GTB ? 4 : 2;
        uint32_t s = 0;
        auto run = [&](auto flg, const uint32_t end) __attribute__((always_inline)) {
            for (; s < end; s += STEP, c += STEP) {
                if constexpr (GTB) {
                    half_step(flg, c, 0, HA, HB);
                    half_step(flg, c + 1, 1, HB, HA);
                    half_step(flg, c + 2, 2, HA, HB);
                    half_step(flg, c + 3, 3, HB, HA);
                    tb_store_window<G, R>(A, pr, valid, W16, s >> 2, lg, dw);   // layout: see tb_store_window
                } else {
                    half_step(flg, c, 0, HA, HB);
                    half_step(flg, c + 1, 1, HB, HA);
                }
            }
        };
        // steps [0, G): lanes reset at column -1 (step lg - 1), captures of short pairs too;
        // then steady steps, the capture window, steady steps
        // (the full-matrix traceback kernel, now the band's fallback, keeps one loop: four copies
        // of its flag sweep did not fit 256 VGPRs)
        const uint32_t up = (cap_hi + STEP) & ~(STEP - 1);
        if constexpr (GTB) {
            run(std::integral_constant<int, 3>{}, nsteps);
        } else {
            run(std::integral_constant<int, 3>{}, min(nsteps, (uint32_t)G));
            run(std::integral_constant<int, 0>{}, min(nsteps, cap_lo & ~(STEP - 1)));
            run(std::integral_constant<int, 2>{}, min(nsteps, up));
            run(std::integral_constant<int, 0>{}, nsteps);
        }
        if constexpr (GTB || GCP) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (fixable[h] && lg == kp_lane[h]) A.tbfix[pr[h]] = fixv[h];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (valid[h] && lg == kq_lane[h]) A.score[pr[h]] = score[h];
        if constexpr (GCP) {
            // the band pass right behind the sweep, in the same wave: no second prologue, and the
            // checkpoints and hand-offs just written (this wave's own stores) are read from L2
            __threadfence_block();
            band_pass();
        }
    } else {
        // SEMI, transposed: c is the query row of this step, registers are the
        // target columns lg*R + k.  Boundaries (semiglobal_kernel_template.h):
        //   left  H(r,-1) = head_q ? 0 : -(o+e*r) (0 for r = 0); E(r,-1) = head_q ? 0 : -inf  (:87-99, Q2)
        //   top   diag into (0,c): head_t ? 0 : -(o+e*c) (0 for c = 0)                         (:127)
        //         F(0,c) = hu(c) - OE, hu(c) = head_t ? 0 : -(o+e*c)                           (:125, Q3)
        // Lanes sweep garbage rows r < -1 first and reset to row -1 at r = -1.
        // Every value is stored in step_semi's frame (+ e per anti-diagonal, Hm^ one e
        // more): Hm^(r, c) = B + H - OE + e(r + c + 1); reads subtract it again.
        const bool head_q = (A.head == 1 || A.head == 3), head_t = (A.head == 2 || A.head == 3);
        const int32_t oe = A.o + A.e, pb = P.base, go = A.o, ge = A.e;
        auto hm = [=](int32_t val, int32_t r, int32_t c) -> uint32_t {   // Hm^ of H value val at (r, c)
            return (uint32_t)(pb + val - oe + ge * (r + c + 1)) * 0x10001u;
        };
        auto hleft = [=](int32_t r) -> uint32_t {      // Hm^(r, -1); r = -1 gives H(-1,-1) = 0
            return (uint32_t)(pb - oe + (head_q ? 0 : (r <= 0 ? 0 : -(go + ge * r))) + ge * r) * 0x10001u;
        };
        // E^(r, -1): 0 (HEAD=QUERY/BOTH) at frame e(r - 1), else -inf (NN is below every
        // value the frame can hold and, undecayed, stays there)
        auto eleft = [=](int32_t r) -> uint32_t { return head_q ? (uint32_t)(pb + ge * (r - 1)) * 0x10001u : NN; };
        uint32_t HA[R], HB[R], Fk[R];
        auto reset = [&](uint32_t (&H)[R]) __attribute__((always_inline)) {
            // computed where used: hoisting 2R loop-invariant values out of the sweep would spill
            int32_t c0 = (int32_t)r0;
            asm volatile("" : "+v"(c0));
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int32_t col = c0 + k;
                const int32_t hd = head_t ? 0 : -(go + ge * (col + 1));   // H(-1,col) as diag of (0,col+1)
                const int32_t hu = head_t ? 0 : -(go + ge * col);         // H(-1,col) as F source (Q3)
                H[k] = hm(hd, -1, col);
                Fk[k] = (uint32_t)(pb + hu - oe + ge * col) * 0x10001u;   // F^(0,col) = hu - OE exactly (>= H[k])
            }
        };
        reset(HA);
#pragma unroll
        for (int k = 0; k < R; ++k) HB[k] = HA[k];
        // TAIL=TARGET: max over the last query row, columns < tl, first (smallest) column.
        // Reverse pass (A.stop, start.hpp): values >= the forward score rank first,
        // by smallest 8-column strip, then value, then first column (bit 31 set).
        uint32_t best[2] = {0, 0};
        uint32_t bestq[2] = {0, 0};                     // TQ: key (H, -row) of the last padded column
        const bool tail_t = !TQ || A.tail == 3;         // the last-row maximum (TAIL TARGET / BOTH)
        int32_t thrp[2] = {0x7FFFFFFF, 0x7FFFFFFF};
        if (STOPK) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (valid[h]) thrp[h] = A.stop[pr[h]] + pb - oe + ge * (int32_t)(yl[h] + G * R);   // its key-frame pattern
        }
        // Lane lg's first real step (row 0, column r0) takes its diagonal from the
        // upper lane's reset at row -1, i.e. H(-1, r0 - 1).  Lanes lg >= 2 receive it
        // by the hand-off of that reset step; lane 1's upper lane (lane 0) has no
        // reset step, so the value is seeded here.  Seeding it with the lane's own
        // H(-1, r0 + R - 1) made cell (0, R) of lane 1 wrong with HEAD=NONE, which
        // surfaced on few-row shapes (the diagonal entry at column R is cheap there).
        const uint32_t hd_up = hm(head_t ? 0 : (r0 == 0 ? 0 : -(go + ge * (int32_t)r0)), -1, (int32_t)r0 - 1);
        uint32_t recvH = hd_up, prevRecvH = hd_up, recvE = NN, hl = 0, el = 0;
        uint2 tnext = tcol[c + G];
        auto half_step = [&](const int32_t cc, uint32_t (&Hin)[R], uint32_t (&Hout)[R]) __attribute__((always_inline)) {
            const uint2 T = tnext;
            tnext = tcol[cc + 1 + G];
            if (cc == -1) {
                reset(Hout);
            } else {
                hl = top ? hleft(cc) : recvH;
                el = top ? eleft(cc) : recvE;
                step_semi<R, PV>(T, top ? hleft(cc - 1) : prevRecvH, hl, el, xs, Hin, Hout, Fk, GO, pv);
                if constexpr (TQ) {
                    // semiglobal :185-193 (Q11): H of row cc at the last padded column, which is
                    // register R - 1 of lane G - 1 (the other lanes' keys are never read);
                    // the largest key is the first row of the maximum
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        // rows compared in one frame: cell (cc, G*R - 1) + e*(yl - cc), which is
                        // the old-frame pattern + e*(yl + G*R) and positive for cc < yl
                        const uint32_t v = ((Hout[R - 1] >> (16 * h)) & 0xFFFFu) + (uint32_t)ge * (yl[h] - (uint32_t)cc);
                        const uint32_t cand = (uint32_t)cc < yl[h] ? (v << 16) | (0xFFFFu - (uint32_t)cc) : 0u;
                        bestq[h] = cand > bestq[h] ? cand : bestq[h];
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (tail_t && valid[h] && cc == (int32_t)yl[h] - 1) {       // semiglobal :160-178
                        // columns compared in one frame: cell (yl - 1, col) + e*(G*R - col), the
                        // old-frame pattern + e*(yl + G*R) (thrp too); positive.  The offset is
                        // formed here, from an opaque base: R hoisted per-column constants spill
                        uint32_t fo = (uint32_t)ge * ((uint32_t)(G * R) - r0);
                        asm volatile("" : "+v"(fo));
#pragma unroll
                        for (int k = 0; k < R; ++k) {
                            const uint32_t col = r0 + k;
                            const uint32_t v = ((Hout[k] >> (16 * h)) & 0xFFFFu) + fo;
                            fo -= (uint32_t)ge;
                            const uint32_t cand =
                                col >= xl[h] ? 0u
                                : STOPK && (int32_t)v >= thrp[h]
                                    ? 0x80000000u | ((255u - (col >> 3)) << 23) | (v << 8) | (255u - (col & 7u))
                                    : (v << 16) | (0xFFFFu - col);
                            best[h] = cand > best[h] ? cand : best[h];
                        }
                    }
                }
            }
            prevRecvH = recvH;
            recvH = (uint32_t)shr_lane((int32_t)Hout[R - 1]);
            recvE = (uint32_t)shr_lane((int32_t)el);
        };
        for (uint32_t s = 0; s < nsteps; s += 2, c += 2) {
            half_step(c, HA, HB);
            half_step(c + 1, HB, HA);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t b = best[h];
#pragma unroll
            for (int m = 1; m < G; m <<= 1) b = max(b, (uint32_t)__shfl_xor(b, m));
            const uint32_t bq = TQ ? (uint32_t)__shfl(bestq[h], (int)(slot * G + G - 1)) : 0u;
            if (valid[h] && lg == 0) {
                // semiglobal :49,63-64,206-218 (Q10): q_end = tl, t_end = column of the max
                // keys hold the old-frame pattern + e*(yl + G*R) (see the captures)
                const int32_t kof = pb - oe + ge * (int32_t)(yl[h] + G * R);
                int32_t score = -32768, qe = (int32_t)xl[h], te = (int32_t)yl[h];
                if (b & 0x80000000u) {
                    score = (int32_t)((b >> 8) & 0x7FFFu) - kof;
                    te = (int32_t)(8 * (255u - ((b >> 23) & 255u)) + (255u - (b & 255u)));
                } else if (b != 0) {
                    score = (int32_t)(b >> 16) - kof;
                    te = (int32_t)(0xFFFFu - (b & 0xFFFFu));
                }
                if (TQ && bq != 0) {
                    // :185-203: a row of the last padded column strictly above the maximum so
                    // far moves the end to (row, ...); then t_end = ql unless that row is tl
                    const int32_t vq = (int32_t)(bq >> 16) - kof;
                    if (vq > score) { score = vq; qe = (int32_t)(0xFFFFu - (bq & 0xFFFFu)); }
                }
                if (TQ && qe != (int32_t)xl[h]) te = (int32_t)yl[h];
                A.score[pr[h]] = score;
                if (A.qend) A.qend[pr[h]] = qe;
                if (A.tend) A.tend[pr[h]] = te;
            }
        }
    }
}

// SEMI TAIL=QUERY/BOTH instances, G = 8, R = 1..32 (semi_tq.hip; one per padded target
// length 8R): NULL outside that range
using Wf16Fn = void (*)(WfArgs);
Wf16Fn wf16_tq_lookup(int R);
// LOCAL e-drift instances with u16 keys and/or the reverse pass's early stop (local_rs.hip):
// NULL for shapes outside kShapes16
Wf16Fn wf16_local_lookup(int G, int R, bool u16, bool rs, bool seg = false);

}  // namespace gx
