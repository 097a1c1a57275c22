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
// column's table selected by the row's letter), add/sub (diag + s), F and E
// (one sub + one maximum3 each, floored at 0: exact for H, see below), H
// (maximum3), H - OE (feeds E of the next column and F of the next row) and
// the (H, column) key (v_pk_mad_u16): 10 instructions for two cells, against
// about 16 per cell in the int32 kernel.
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

__global__ __launch_bounds__(256) void band16_kernel(BandArgs A) {
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
    const uint32_t KK = (uint32_t)A.b * 0x10001u, MATCH = (uint32_t)(A.a + A.b);
    uint2 *rows = A.rows + lane;
    const size_t rs = A.n_lanes;
    for (uint32_t r = 0; r < QR * 8; ++r) rows[r * rs] = make_uint2(BB, BB);
    // key = H*8 + (7 - column in strip) + 0x400 = H_stored*8 + KC[m]  (mod 2^16)
    uint32_t KC[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) KC[m] = ((uint32_t)(7 - m + 0x400 - 8 * (int32_t)A.base) & 0xFFFFu) * 0x10001u;
    bool bad_a = false, bad_b = false;
    int32_t maxa = 0, maxb = 0, xa = 0, xb = 0, ya = 0, yb = 0;
    const int32_t kother = (int32_t)TR - ((int32_t)QR - A.kbw);   // banded.h:35
    for (int32_t i = 0; i < (int32_t)TR; ++i) {
        // the strip's 8 substitution tables per pair: byte l = score(l, t) + b
        uint32_t T0[8], T1[8];
        const uint32_t ga = twa[i], gb = twb[i];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t col = (uint32_t)i * 8 + m;
            const uint32_t la = letter_of((ga >> (28 - 4 * m)) & 15u, A.nval);
            const uint32_t lb = letter_of((gb >> (28 - 4 * m)) & 15u, A.nval);
            const bool ra = col < tla, rb = col < tlb;
            bad_a |= ra && la > 3;
            bad_b |= rb && lb > 3;
            T0[m] = (ra && la < 4) ? MATCH << (8 * la) : 0u;
            T1[m] = (rb && lb < 4) ? MATCH << (8 * lb) : 0u;
        }
        uint32_t hoe[8], f[8], p[8];   // row above: H - OE, F, and diag H(r-1, c-1)
#pragma unroll
        for (int m = 0; m < 8; ++m) { hoe[m] = BB - OE2; f[m] = BB; p[m] = BB; }
        const int32_t j0 = max(0, i - kother + 1), j1 = min(A.kbw + i, (int32_t)QR);   // banded.h:73-75
        // the tile's 8 row-buffer entries and query words, loaded one tile ahead
        uint2 cur[8];
        uint32_t wa = 0, wb = 0;
        if (j0 < j1) {
            wa = qwa[j0]; wb = qwb[j0];
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = rows[((uint32_t)j0 * 8 + k) * rs];
        }
        for (int32_t j = j0; j < j1; ++j) {
            uint2 nxt[8];
            uint32_t nwa = 0, nwb = 0;
            if (j + 1 < j1) {
                nwa = qwa[j + 1]; nwb = qwb[j + 1];
#pragma unroll
                for (int k = 0; k < 8; ++k) nxt[k] = rows[((uint32_t)j * 8 + 8 + k) * rs];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t r = (uint32_t)j * 8 + k;
                const uint32_t la = letter_of((wa >> (28 - 4 * k)) & 15u, A.nval);
                const uint32_t lb = letter_of((wb >> (28 - 4 * k)) & 15u, A.nval);
                const bool ra = r < qla, rb = r < qlb;
                bad_a |= ra && la > 3;
                bad_b |= rb && lb > 3;
                const uint32_t sa = (ra && la < 4) ? la : 0x0Cu, sb = (rb && lb < 4) ? lb + 4 : 0x0Cu;
                const uint32_t sel = sa | 0x0C00u | (sb << 16) | 0x0C000000u;
                uint32_t left = cur[k].x, e = cur[k].y;        // H, E of the row at the previous strip's last column
                uint32_t loe = left - OE2;
                uint32_t key[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const uint32_t v = __builtin_amdgcn_perm(T1[m], T0[m], sel);
                    const uint32_t fm = pk_max3(hoe[m], pk_subnb(f[m], EXT), BB);
                    const uint32_t tmp = pk_subnb(pk_addnc(p[m], v), KK);
                    e = pk_max3(loe, pk_subnb(e, EXT), BB);
                    const uint32_t H = pk_max3(tmp, fm, e);
                    f[m] = fm;
                    p[m] = left;
                    left = H;
                    loe = pk_subnb(H, OE2);
                    hoe[m] = loe;
                    key[m] = pk_mad_u16(H, 0x00080008u, KC[m]);
                }
                rows[r * rs] = make_uint2(left, e);
                const uint32_t m1 = pk_max3(key[0], key[1], key[2]), m2 = pk_max3(key[3], key[4], key[5]);
                const uint32_t rk = pk_max3(pk_max3(key[6], key[7], m1), m2, m2);
                const int32_t ka = (int32_t)(rk & 0xFFFFu) - 0x400, kb = (int32_t)(rk >> 16) - 0x400;
                if ((ka >> 3) > maxa) { maxa = ka >> 3; ya = i * 8 + 7 - (ka & 7); xa = (int32_t)r; }
                if ((kb >> 3) > maxb) { maxb = kb >> 3; yb = i * 8 + 7 - (kb & 7); xb = (int32_t)r; }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
            wa = nwa; wb = nwb;
        }
    }
    A.score[pa] = maxa;
    if (A.qend) A.qend[pa] = xa;
    if (A.tend) A.tend[pa] = ya;
    if (bad_a) A.todo[pa] = 1;
    if (two) {
        A.score[pb] = maxb;
        if (A.qend) A.qend[pb] = xb;
        if (A.tend) A.tend[pb] = yb;
        if (bad_b) A.todo[pb] = 1;
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
