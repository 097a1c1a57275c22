// banded16.hpp — the banded-tiled LOCAL kernel (kernels/banded.h:10-139) with
// two pairs per lane in the 16-bit halves of every register.
//
// The reference's band is a staircase of 8x8 tiles: strip i (8 target columns)
// covers query tiles [max(0, i - kother + 1), min(k_band/8 + i, QR)) with
// kother = TR - (QR - k_band/8) (banded.h:35, :73-75), so at k_band = 16 only
// 30 % of a 150 x 182 rectangle is computed.  Lanes over rows (the wavefront
// kernels) would idle outside that diagonal band, so the band stays one lane
// per pair — but a lane carries two pairs of the same tile geometry (QR, TR),
// whose loops are then identical, and computes both with packed 16-bit
// arithmetic: values stored as value + B inside the positive normal f16 range,
// where v_pk_maximum3_f16 is an exact 3-way max on both halves
// (wavefront16.hpp).  Per cell of both pairs: v_perm (substitution byte of the
// column's table selected by the row's letter), v_add3 (diag + s, the diagonal
// taken from the row above's H - OE), F and E (one sub + one maximum3 each,
// floored at 0: exact for H, see below), H (maximum3), H - OE (feeds E of the
// next column and F and the diagonal of the next row) and the (H, column) key
// (v_pk_mad_u16): 9 instructions for two cells, about 12 with the per-row
// first-maximum update, against about 16 per cell in the int32 kernel.
//
// A lane runs strips i and i + 1 in one pass over their rows: strip i's (H, E)
// at its last column feeds strip i + 1 directly, so the [row][lane] row buffer
// is read and written once per two strips, and rows entering the band for the
// first time start from the initial 0 without a load.  The next tile's row
// buffer entries and query words are loaded one tile ahead.
//
// Semantics kept from banded.h: textbook Gotoh on H (F from the H above, E
// from the H on the left, :94-102); (H, E) of every row carried between strips
// in a row buffer that starts at 0 (:61-63, :83-84, :108-111); h, f, p reset
// to 0 at every strip start (:69-73), so cells outside the band act as H = E =
// F = 0; the first strict maximum in strip-major order (FIND_MAX, :104, :113).
// E and F are floored at 0 here (the reference floors only H): the stored
// value is then max(E, 0), which gives the same H everywhere (a negative E or F
// never beats the 0 floor of H) and propagates as max(E - e, H - OE, 0).
//
// Declined (flag in `todo`, the int32 kernel aligns the pair afterwards): a
// base other than A/C/G/T inside a sequence (the N rule), and the second pair
// of a lane whose tile geometry differs from the first.  Pad cells (past ql or
// tl, N_CODE in the reference) score -b here instead of the N rule's 0 or
// -N_PENALTY: pads are the last rows and the last columns, so they feed only
// other pad cells, and with a score <= 0 a pad H never exceeds the maximum of
// the cells it is computed from, which were visited earlier — the strict
// maximum, its row and its column are unchanged (the planner takes this path
// only when the N score is <= 0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wavefront16.hpp"

namespace gx {

#ifndef GX_BAND16_WAVES
#define GX_BAND16_WAVES 3   // waves per SIMD (a few spills; 3.3 % faster than 2 waves at 184 VGPRs)
#endif

struct BandArgs {
    const uint32_t *qw, *tw;           // packed 4-bit words of the batch
    const uint32_t *qoff, *toff, *qlen, *tlen;
    const uint32_t *perm;              // slot -> pair (NULL: identity)
    int32_t *score, *qend, *tend;
    uint8_t *todo;                     // per pair: 1 = the int32 kernel aligns it
    uint2 *rows;                       // [row][lane]: (H, E) of both halves
    uint32_t n, n_lanes;
    int32_t a, b, oe, e, kbw, nval;
    uint32_t base;                     // stored value of 0
};

// exact u16x2 multiply-add in one VOP3P op (the compiler splits a multiply by 8
// into a shift and an add)
__device__ __forceinline__ uint32_t band_key(uint32_t h, uint32_t c) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, 8, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(h), "s"(c));
    return r;
}

// [x != y] per 16-bit half as 0x0000 / 0xFFFF, for x >= y per half
__device__ __forceinline__ uint32_t band_ne_mask(uint32_t x, uint32_t y) {
    const uint32_t d = pk_subnb(x, y);                                   // no borrow: x >= y per half
    const uint32_t one = GX_AS(uint32_t, __builtin_elementwise_min(GX_AS(pk_u2, d), GX_AS(pk_u2, 0x00010001u)));
    return GX_AS(uint32_t, GX_AS(pk_u2, 0u) - GX_AS(pk_u2, one));
}

// Running first maximum of one strip, both halves: key = H*8 + (7 - column) + 0x400,
// updated by a row only when the row's H is strictly higher (its B7 = key | 7).
struct BandBest {
    uint32_t key, b7, row;
};
__device__ __forceinline__ void band_row_max(BandBest &B, const uint32_t (&key)[8], uint32_t rr) {
    const uint32_t m1 = pk_max3(key[0], key[1], key[2]), m2 = pk_max3(key[3], key[4], key[5]);
    const uint32_t rk = pk_max3(pk_max3(key[6], key[7], m1), m2, m2);
    const uint32_t t = pk_max_u16(rk, B.b7);
    const uint32_t msk = band_ne_mask(t, B.b7);
    B.key = (B.key & ~msk) | (rk & msk);
    B.row = (B.row & ~msk) | (rr & msk);
    B.b7 = t | 0x00070007u;
}

// One row of 8 columns of one strip for both halves (banded.h:86-107).  The
// diagonal H(r-1, c-1) is not kept: it is hoe[c-1] + OE of the row above, so
// tmp = (H(r-1, c-1) - OE) + v + (OE - K) is one v_add3 (C = OE - K per half,
// exact in 32 bits because every half's result stays inside its window).
__device__ __forceinline__ void band_row(const uint32_t (&T0)[8], const uint32_t (&T1)[8], uint32_t sel,
                                         uint32_t (&hoe)[8], uint32_t (&f)[8], uint32_t &hol, uint32_t &left,
                                         uint32_t &e, uint32_t (&key)[8], const uint32_t (&KC)[8], uint32_t BB,
                                         uint32_t OE2, uint32_t EXT, uint32_t C) {
    uint32_t dg = hol;                      // H(r-1, -1) - OE
    uint32_t loe = pk_subnb(left, OE2);     // H(r, -1) - OE
    hol = loe;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const uint32_t v = __builtin_amdgcn_perm(T1[m], T0[m], sel);
        const uint32_t up = hoe[m];         // H(r-1, c) - OE
        const uint32_t fm = pk_max3(up, pk_subnb(f[m], EXT), BB);
        const uint32_t tmp = dg + v + C;
        e = pk_max3(loe, pk_subnb(e, EXT), BB);
        const uint32_t H = pk_max3(tmp, fm, e);
        f[m] = fm;
        left = H;
        loe = pk_subnb(H, OE2);
        hoe[m] = loe;
        dg = up;
        key[m] = band_key(H, KC[m]);
    }
}

// letters as nibbles 0..3 ((code >> 1) & 3: A 0, C 1, T 2, G 3); valid codes 1, 3, 4, 7
__device__ __forceinline__ bool band_word_ok(uint32_t w, uint32_t nreal) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) ok &= (uint32_t)k >= nreal || ((0x9Au >> ((w >> (28 - 4 * k)) & 15u)) & 1u);
    return ok;
}

// the 8 substitution tables of one strip for one pair: byte l = score(l, t) + b;
// pad columns (past tl) score -b in every row
__device__ __forceinline__ bool band_tables(uint32_t g, uint32_t col0, uint32_t tl, uint32_t match, uint32_t (&T)[8]) {
    bool ok = true;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const uint32_t c = (g >> (28 - 4 * m)) & 15u;
        const bool real = col0 + m < tl, valid = (0x9Au >> c) & 1u;
        ok &= !real || valid;
        T[m] = (real && valid) ? match << (8 * ((c >> 1) & 3u)) : 0u;
    }
    return ok;
}

__global__ __launch_bounds__(256, GX_BAND16_WAVES) void band16_kernel(BandArgs A) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= A.n_lanes) return;
    const uint32_t s0 = 2 * lane, s1 = s0 + 1;
    const uint32_t pa = A.perm ? A.perm[s0] : s0;
    const uint32_t qla = A.qlen[pa], tla = A.tlen[pa];
    const uint32_t QR = (qla + 7) >> 3, TR = (tla + 7) >> 3;
    uint32_t pb = pa;
    if (s1 < A.n) {
        const uint32_t c = A.perm ? A.perm[s1] : s1;
        if (((A.qlen[c] + 7) >> 3) == QR && ((A.tlen[c] + 7) >> 3) == TR) pb = c;
        else A.todo[c] = 1;
    }
    const bool two = pb != pa;
    const uint32_t qlb = A.qlen[pb], tlb = A.tlen[pb];
    const uint32_t *qwa = A.qw + (A.qoff[pa] >> 3), *qwb = A.qw + (A.qoff[pb] >> 3);
    const uint32_t *twa = A.tw + (A.toff[pa] >> 3), *twb = A.tw + (A.toff[pb] >> 3);
    const uint32_t BB = A.base * 0x10001u, OE2 = (uint32_t)A.oe * 0x10001u, EXT = (uint32_t)A.e * 0x10001u;
    const uint32_t C = OE2 - (uint32_t)A.b * 0x10001u, MATCH = (uint32_t)(A.a + A.b);
    uint2 *rows = A.rows + lane;
    const size_t rs = A.n_lanes;
    // key = H*8 + (7 - column in strip) + 0x400 = H_stored*8 + KC[m]  (mod 2^16)
    uint32_t KC[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) KC[m] = ((uint32_t)(7 - m + 0x400 - 8 * (int32_t)A.base) & 0xFFFFu) * 0x10001u;
    // the query is read once per strip: check its letters once
    bool ok_a = true, ok_b = true;
    for (uint32_t j = 0; j < QR; ++j) {
        ok_a &= band_word_ok(qwa[j], qla - 8 * j);
        ok_b &= band_word_ok(qwb[j], qlb - 8 * j);
    }
    // pad rows of the last query tile: letter nibble 0xC (selector byte 0x0C = 0,
    // score -b) for the low half, 0x8 (+4 = 0x0C) for the high half
    const uint32_t kpa = qla - 8 * (QR - 1), kpb = qlb - 8 * (QR - 1);
    const uint32_t pma = kpa >= 8 ? 0u : (1u << (4 * (8 - kpa))) - 1u;
    const uint32_t pmb = kpb >= 8 ? 0u : (1u << (4 * (8 - kpb))) - 1u;
    int32_t gma = 0, gmb = 0, xa = 0, xb = 0, ya = 0, yb = 0;   // FIND_MAX state (banded.h:104, :113)
    const int32_t kother = (int32_t)TR - ((int32_t)QR - A.kbw);   // banded.h:35
    // strips i and i + 1 in one pass over their rows: strip i's (H, E) at its last
    // column feeds strip i + 1 directly, so the row buffer is read and written once
    // per two strips
    for (int32_t i = 0; i < (int32_t)TR; i += 2) {
        const bool hasB = i + 1 < (int32_t)TR;
        uint32_t TA0[8], TA1[8], TB0[8], TB1[8];
        ok_a &= band_tables(twa[i], 8 * i, tla, MATCH, TA0);
        ok_b &= band_tables(twb[i], 8 * i, tlb, MATCH, TA1);
        if (hasB) {
            ok_a &= band_tables(twa[i + 1], 8 * i + 8, tla, MATCH, TB0);
            ok_b &= band_tables(twb[i + 1], 8 * i + 8, tlb, MATCH, TB1);
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) TB0[m] = TB1[m] = 0u;
        }
        uint32_t hoeA[8], fA[8], hoeB[8], fB[8], holA = BB - OE2, holB = BB - OE2;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            hoeA[m] = hoeB[m] = BB - OE2;
            fA[m] = fB[m] = BB;
        }
        const int32_t j0A = max(0, i - kother + 1), j1A = min(A.kbw + i, (int32_t)QR);   // banded.h:73-75
        const int32_t j0B = max(0, i + 1 - kother + 1), j1B = hasB ? min(A.kbw + i + 1, (int32_t)QR) : j1A;
        // row tiles >= fresh were never written (j1 only grows): their (H, E) is the
        // initial 0 (banded.h:61-63) without a load
        const int32_t fresh = i == 0 ? 0 : min(A.kbw + i - 1, (int32_t)QR);
        BandBest bA = {0x04070407u, 0x04070407u, 0u}, bB = bA;
        // one tile of 8 rows: strip i (DA), strip i + 1 (DB), or both; three loops so
        // that no row branches (the register rotation of p / left stays free)
        // row-buffer entries and query words of the tile, loaded one tile ahead
        // (tiles >= fresh start at the initial 0 without a load)
        uint2 cur[8];
        uint32_t cwa = 0, cwb = 0;
        auto load = [&](int32_t j, uint2 (&dst)[8], uint32_t &wa, uint32_t &wb) {
            if (j < fresh) {
#pragma unroll
                for (int k = 0; k < 8; ++k) dst[k] = rows[((uint32_t)j * 8 + k) * rs];
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) dst[k] = make_uint2(BB, BB);
            }
            if (j < (int32_t)QR) { wa = qwa[j]; wb = qwb[j]; }
        };
        auto tile = [&](int32_t j, auto DA, auto DB) {
            constexpr bool doA = decltype(DA)::value, doB = decltype(DB)::value;
            uint2 nxt[8];
            uint32_t nwa = 0, nwb = 0;
            load(j + 1, nxt, nwa, nwb);
            uint32_t la = (cwa >> 1) & 0x33333333u, lb = (cwb >> 1) & 0x33333333u;
            if (j == (int32_t)QR - 1) { la = (la & ~pma) | (0xCCCCCCCCu & pma); lb = (lb & ~pmb) | (0x88888888u & pmb); }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t rr = ((uint32_t)j * 8 + k) * 0x10001u;
                const uint32_t sel = (((la >> (28 - 4 * k)) & 15u) | (((lb >> (28 - 4 * k)) & 15u) << 16)) + 0x0C040C00u;
                uint32_t left = cur[k].x, e = cur[k].y, key[8];
                if (doA) {
                    band_row(TA0, TA1, sel, hoeA, fA, holA, left, e, key, KC, BB, OE2, EXT, C);
                    band_row_max(bA, key, rr);
                }
                if (doB) {
                    band_row(TB0, TB1, sel, hoeB, fB, holB, left, e, key, KC, BB, OE2, EXT, C);
                    band_row_max(bB, key, rr);
                    rows[((uint32_t)j * 8 + k) * rs] = make_uint2(left, e);
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
            cwa = nwa; cwb = nwb;
        };
        // the tiles a pass visits are contiguous from here (j0B <= j0A + 1 <= j1A when
        // strip i's band is not empty)
        load(j0A < j1A || !hasB ? j0A : j0B, cur, cwa, cwb);
        using T_ = std::true_type;
        using F_ = std::false_type;
        if (!hasB) {
            for (int32_t j = j0A; j < j1A; ++j) tile(j, T_{}, F_{});
        } else {
            // tiles of strip i: [j0A, j1A), of strip i + 1: [j0B, j1B), j0B >= j0A, j1B >= j1A
            for (int32_t j = j0A; j < min(j1A, j0B); ++j) tile(j, T_{}, F_{});   // above strip i + 1's band
            for (int32_t j = j0B; j < j1A; ++j) tile(j, T_{}, T_{});
            for (int32_t j = max(j0B, j1A); j < j1B; ++j) tile(j, F_{}, T_{});   // below strip i's band
        }
        // strip-major order: strip i's first maximum, then strip i + 1's, each only
        // when strictly above the maximum so far
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const BandBest &b = s ? bB : bA;
            const int32_t col0 = 8 * (i + s) + 7;
            const int32_t ka = (int32_t)(b.key & 0xFFFFu) - 0x400, kb = (int32_t)(b.key >> 16) - 0x400;
            if ((ka >> 3) > gma) { gma = ka >> 3; ya = col0 - (ka & 7); xa = (int32_t)(b.row & 0xFFFFu); }
            if ((kb >> 3) > gmb) { gmb = kb >> 3; yb = col0 - (kb & 7); xb = (int32_t)(b.row >> 16); }
        }
    }
    A.score[pa] = gma;
    if (A.qend) A.qend[pa] = xa;
    if (A.tend) A.tend[pa] = ya;
    if (!ok_a) A.todo[pa] = 1;
    if (two) {
        A.score[pb] = gmb;
        if (A.qend) A.qend[pb] = xb;
        if (A.tend) A.tend[pb] = yb;
        if (!ok_b) A.todo[pb] = 1;
    }
}

// sort key of the tile geometry (counting sort by start.hpp's kernels, REV_PLAIN
// mode, which buckets ceil(len / 8)): len = 8 * ((QR - 1) * TRW + TR)
__global__ __launch_bounds__(256) void band16_key_kernel(const uint32_t *qlen, const uint32_t *tlen, uint32_t n,
                                                         uint32_t trw, uint32_t *klen) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t QR = max((qlen[k] + 7) >> 3, 1u), TR = max((tlen[k] + 7) >> 3, 1u);
    klen[k] = 8 * ((QR - 1) * trw + TR);
}

}  // namespace gx
