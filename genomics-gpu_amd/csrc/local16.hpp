// local16.hpp — LOCAL with the second-best result (local_kernel_template.h:
// 72-430, secondBest: :145-150, :160-164, :412-418) as two pairs per lane in
// the 16-bit halves of every register.
//
// Why not the wavefront: the second-best update of a cell,
//     if (max2 < H && maxHH > H) { max2 = H; y2 = column }   (after FIND_MAX),
// reads the running maximum in strip-major order at that cell, a prefix that an
// anti-diagonal sweep does not have.  So the pairs walk the rectangle in the
// reference's own order (8-column strips, rows, columns), a lane per two pairs
// of one tile geometry, as banded16.hpp does, with the LOCAL cell update of
// wavefront16.hpp (Q4: F and E from tmp; E and F floored at 0, exact for H).
//
// Per row the cells give, per half: the first maximum (key H*8 + 7 - column,
// the strictly higher row wins) and the second-best candidates: a cell counts
// iff H < Q, Q the running maximum before it (then maxHH > H after FIND_MAX;
// a candidate only raises max2, so the row's largest candidate, first in its
// row, is the reference's sequential result).  Q itself is carried from cell
// to cell and row to row.  Per row: x2 = (prev2 < maxHH) ? row : x2;
// prev2 = max(max2, prev2) (:412-418, the reference compares prev2 with maxHH).
//
// N: the N rule (gasal_kernels.h:49-51) holds for pads: pad columns get tables
// of the N score, pad rows (the last tile) a patched byte; pad cells can update
// the second best (Q13), so they are computed exactly.  A real N or another
// letter inside a sequence, or a second pair of another tile geometry, is
// declined to gen_local_kernel (todo).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "banded16.hpp"

namespace gx {

struct Local16Args {
    const uint32_t *qw, *tw;
    const uint32_t *qoff, *toff, *qlen, *tlen;
    const uint32_t *perm;              // slot -> pair (NULL: identity)
    int32_t *score, *qend, *tend, *score2, *qend2, *tend2;
    uint8_t *todo;
    uint2 *rows;                       // [wave][row][64 lanes]: (H, E) of both halves
    uint32_t n, n_lanes, rows_cap;     // rows_cap: rows per wave (padded query length)
    int32_t a, b, oe, e, nval, sn;     // sn: the N score (0, or -N_PENALTY)
    uint32_t k, base;                  // table offset, stored value of 0
};

// 0x0000 / 0xFFFF per 16-bit half: [d != 0] (v_pk_mad_u16 saturates d * 0xFFFF)
__device__ __forceinline__ uint32_t l16_nz_mask(uint32_t d) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, -1, 0 op_sel_hi:[1,0,0] clamp" : "=v"(r) : "v"(d));
    return r;
}
// max(x - y, 0) per unsigned 16-bit half
__device__ __forceinline__ uint32_t l16_satsub(uint32_t x, uint32_t y) {
    uint32_t d;
    asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(d) : "v"(x), "v"(y));
    return d;
}

template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void local2nd16_kernel(Local16Args A) {
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
    const uint32_t MK = (uint32_t)(-(int32_t)A.k) * 0x10001u;
    const uint32_t BYTE_M = (uint32_t)(A.a + (int32_t)A.k), BYTE_X = (uint32_t)((int32_t)A.k - A.b);
    const uint32_t BYTE_N = (uint32_t)(A.sn + (int32_t)A.k), SNK = BYTE_N * 0x10001u;
    // maxHH in key units with column bits 0: (Q - B)*8 + 0x400
    const uint32_t QK = ((uint32_t)(0x400 - 8 * (int32_t)A.base) & 0xFFFFu) * 0x10001u;
    // row buffer [wave][row][64 lanes]: the 8 rows of a tile at immediate offsets
    uint2 *rw = A.rows + (size_t)(lane >> 6) * A.rows_cap * 64 + (lane & 63);
    uint32_t KC[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) KC[m] = ((uint32_t)(7 - m + 0x400 - 8 * (int32_t)A.base) & 0xFFFFu) * 0x10001u;
    // letters checked once (the query is read again in every strip)
    bool ok_a = true, ok_b = true;
    for (uint32_t j = 0; j < QR; ++j) {
        ok_a &= band_word_ok(qwa[j], qla - 8 * j);
        ok_b &= band_word_ok(qwb[j], qlb - 8 * j);
    }
    const uint32_t kpa = qla - 8 * (QR - 1), kpb = qlb - 8 * (QR - 1);
    BandBest b1 = {0x04070407u, 0u, 0u};             // first maximum (key, row)
    uint32_t k2 = 0x04070407u;                       // second best key
    uint32_t strip1 = 0, strip2 = 0;                 // strip of b1 / of k2 (16 bits per half)
    uint32_t Q = BB, x2 = 0;                         // running maximum (stored), maxXY_x_second
    uint32_t T0[8], T1[8], f[8], p[8];
    // one row of the strip; PAD: the row may be a pad row of either half (last tile)
    auto row = [&](uint32_t rr, uint2 he, uint2 *dst, uint32_t sel, uint32_t padm, auto pad_t) {
        constexpr bool PAD = decltype(pad_t)::value;
        uint32_t left = he.x, e = he.y;   // H, E at the previous strip's last column
        const uint32_t Q0 = Q;
        uint32_t key[8], cand[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            uint32_t v = __builtin_amdgcn_perm(T1[m], T0[m], sel);
            if (PAD) v = (v & ~padm) | (SNK & padm);
            const uint32_t tmp = p[m] + v + MK;
            const uint32_t toe = pk_subnb(tmp, OE2);
            const uint32_t H = pk_max3(tmp, f[m], e);
            f[m] = pk_max3(toe, pk_subnb(f[m], EXT), BB);
            e = pk_max3(toe, pk_subnb(e, EXT), BB);
            key[m] = band_key(H, KC[m]);
            // second best: the cell counts iff H < the running maximum after it
            Q = pk_max_u16(Q, H);
            cand[m] = key[m] & l16_nz_mask(pk_subnb(Q, H));
            p[m] = left;
            left = H;
        }
        *dst = make_uint2(left, e);
        // first maximum: the row's largest key when the row raised the running maximum
        const uint32_t m1 = pk_max3(key[0], key[1], key[2]), m2 = pk_max3(key[3], key[4], key[5]);
        const uint32_t rk = pk_max3(pk_max3(key[6], key[7], m1), m2, m2);
        const uint32_t msk = l16_nz_mask(pk_subnb(Q, Q0));
        b1.key = (b1.key & ~msk) | (rk & msk);
        b1.row = (b1.row & ~msk) | (rr & msk);
        // x2 = (prev_maxHH_second < maxHH) ? r : x2 with prev_maxHH_second = max2 before
        // this row (max2 only grows): max2 < maxHH iff max2*8 + 7 < maxHH*8 in key units
        const uint32_t b27 = k2 | 0x00070007u;
        const uint32_t xm = l16_nz_mask(l16_satsub(band_key(Q, QK), b27));
        x2 = (x2 & ~xm) | (rr & xm);
        // second best: the row's largest candidate when its H is strictly above max2
        const uint32_t c1 = pk_max3(cand[0], cand[1], cand[2]), c2 = pk_max3(cand[3], cand[4], cand[5]);
        const uint32_t acc2 = pk_max3(pk_max3(cand[6], cand[7], c1), c2, c2);
        const uint32_t msk2 = l16_nz_mask(l16_satsub(acc2, b27));
        k2 = (k2 & ~msk2) | (acc2 & msk2);
    };
    // tiles in strip-major order, the next tile's row buffer entries and query words
    // loaded while this one computes (strip 0 starts from (0, 0) without loads; a
    // one-tile query (QR == 1) reloads its rows after storing them)
    uint2 nx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) nx[k] = make_uint2(BB, BB);
    uint32_t nqa = qwa[0], nqb = qwb[0];
    for (uint32_t i = 0; i < TR; ++i) {
        // substitution tables of the strip, byte l = s(l, t) + K; pad and N columns: the N score
        const uint32_t ga = twa[i], gb = twb[i];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t col = i * 8 + m;
            const uint32_t ca = (ga >> (28 - 4 * m)) & 15u, cb = (gb >> (28 - 4 * m)) & 15u;
            const bool na = col >= tla || ca == (uint32_t)A.nval, nb = col >= tlb || cb == (uint32_t)A.nval;
            ok_a &= na || ((0x9Au >> ca) & 1u);
            ok_b &= nb || ((0x9Au >> cb) & 1u);
            T0[m] = na ? BYTE_N * 0x01010101u : BYTE_X * 0x01010101u + ((BYTE_M - BYTE_X) << (8 * ((ca >> 1) & 3u)));
            T1[m] = nb ? BYTE_N * 0x01010101u : BYTE_X * 0x01010101u + ((BYTE_M - BYTE_X) << (8 * ((cb >> 1) & 3u)));
            f[m] = BB; p[m] = BB;
        }
        const uint32_t key0 = b1.key, k20 = k2;
        for (uint32_t j = 0; j < QR; ++j) {
            uint2 cu[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) cu[k] = nx[k];
            const uint32_t qa = nqa, qb = nqb;
            const uint32_t nj = j + 1 < QR ? j + 1 : 0;
            // the next tile is in strip 0 (its rows start at 0), in a later strip with
            // QR > 1 (prefetch) or the same tile of the next strip (QR == 1, below)
            const bool later = j + 1 == QR ? i + 1 < TR : i > 0;
            uint2 *rb = rw + (size_t)j * 8 * 64;
            if (later && QR > 1) {
                const uint2 *nb = rw + (size_t)nj * 8 * 64;
#pragma unroll
                for (int k = 0; k < 8; ++k) nx[k] = nb[k * 64];
            }
            if (nj != j) { nqa = qwa[nj]; nqb = qwb[nj]; }
            const uint32_t la = (qa >> 1) & 0x33333333u, lb = ((qb >> 1) & 0x33333333u) + 0x44444444u;
            if (j + 1 < QR) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t sel = ((la >> (28 - 4 * k)) & 15u) | (((lb >> (28 - 4 * k)) & 15u) << 16) | 0x0C000C00u;
                    row((j * 8 + k) * 0x10001u, cu[k], rb + k * 64, sel, 0u, std::false_type{});
                }
            } else {   // the last tile: pad rows of either half score the N score
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t sel = ((la >> (28 - 4 * k)) & 15u) | (((lb >> (28 - 4 * k)) & 15u) << 16) | 0x0C000C00u;
                    const uint32_t padm = ((uint32_t)k >= kpa ? 0x0000FFFFu : 0u) | ((uint32_t)k >= kpb ? 0xFFFF0000u : 0u);
                    row((j * 8 + k) * 0x10001u, cu[k], rb + k * 64, sel, padm, std::true_type{});
                }
            }
            if (QR == 1 && i + 1 < TR) {
#pragma unroll
                for (int k = 0; k < 8; ++k) nx[k] = rb[k * 64];
            }
        }
        // strips of the maxima: the keys only grow, so a changed key was set in this strip
        const uint32_t ss = i * 0x10001u;
        const uint32_t c1 = l16_nz_mask(b1.key - key0), c2 = l16_nz_mask(k2 - k20);
        strip1 = (strip1 & ~c1) | (ss & c1);
        strip2 = (strip2 & ~c2) | (ss & c2);
    }
    auto out = [&](uint32_t pair, uint32_t half, bool ok) {
        const uint32_t sh = 16 * half;
        const int32_t c1 = (int32_t)((b1.key >> sh) & 0xFFFFu) - 0x400, c2 = (int32_t)((k2 >> sh) & 0xFFFFu) - 0x400;
        A.score[pair] = c1 >> 3;
        if (A.qend) A.qend[pair] = (int32_t)((b1.row >> sh) & 0xFFFFu);
        if (A.tend) A.tend[pair] = (int32_t)((strip1 >> sh) & 0xFFFFu) * 8 + 7 - (c1 & 7);
        if (A.score2) A.score2[pair] = c2 >> 3;
        if (A.qend2) A.qend2[pair] = (int32_t)((x2 >> sh) & 0xFFFFu);
        if (A.tend2) A.tend2[pair] = (int32_t)((strip2 >> sh) & 0xFFFFu) * 8 + 7 - (c2 & 7);
        if (!ok) A.todo[pair] = 1;
    };
    out(pa, 0, ok_a);
    if (two) out(pb, 1, ok_b);
}

}  // namespace gx
