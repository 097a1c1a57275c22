// ksw16.hpp — KSW (ksw_kernel_template.h:47-199: BWA's ksw_extend with GASAL2's tile
// skip and Q16 end rule) as two pairs per lane in the 16-bit halves of every register.
//
// The reference is thread per pair and so is gen_ksw_kernel (generic.hpp); its row
// loop is sequential (the row's beg/end trimming needs the whole previous row), so the
// MI355X form keeps the row-by-row walk and packs two pairs, slots 2t and 2t + 1, into
// one lane.  The halves share the column index j; each keeps its own beg/end/skip and
// row bookkeeping (scalars per half, once per row).  The column loop runs over the
// union of the two pairs' (and the wave's) ranges:
//  * left of a pair's beg every stored entry is (0, 0) (the scan that sets beg stops at
//    the first non-zero entry, and entries left of it are never written again), the
//    row starts with f = 0 and h1 = 0 (beg > 0), so the cells there compute and store
//    zeros: exactly the reference's untouched entries;
//  * at j == end the half stores (H(i, end-1), 0) — the reference's eh[end] = {h1, 0};
//  * right of end, and in rows where the half is idle (past its target, or skipping
//    the rest of a tile after m == 0), the half keeps its stored bytes.
// Per cell (two cells per lane): v_perm unpacks H(i-1, j-1) and E(i, j) from the 8-bit
// entry bytes (biased by 0x800, so v_pk_maximum3_f16 is an exact integer max), a
// per-row v_perm table gives both substitution scores from a per-column selector
// word, M = M ? M + s : 0 (mask + bfi; M < 0 is clamped by the maxes as in the
// reference), H, E', F' by maximum3, the running maximum and its last column as a
// 16-bit key H*256 + j + 1, and the stored entry merged under per-byte masks.  The
// first / last non-zero stored entry of the row (the reference's trimming scans) are
// a min / max over the stored words.
//
// A pair is taken when its bound (seed + gain * min(ql, tl)) fits the 8-bit entries,
// ql <= 254 and its query is A/C/G/T only (the targets may hold anything: a target
// row's table scores every query code); both pairs of a lane must qualify, otherwise
// both stay for gen_ksw_kernel (todo untouched).  Taken pairs get todo = 0xFF.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "generic.hpp"
#include "local16.hpp"
#include "wavefront16.hpp"

namespace gx {

__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return GX_AS(uint32_t, __builtin_elementwise_min(GX_AS(pk_u2, a), GX_AS(pk_u2, b)));
}

struct Ksw16Args {
    const uint32_t *qw, *tw;                   // packed words (4-bit codes, first in bits 31:28)
    const uint32_t *qoff, *toff, *qlen, *tlen, *seed;
    int32_t *score, *qend, *tend;
    uint8_t *todo;
    uint32_t *ent;                             // [column][lane]: bytes hA, eA, hB, eB
    uint32_t *sel;                             // [column / 2][lane]: per column cA | (4 + cB) << 8
    uint32_t n, n_lanes, cols;                 // cols: entry columns (max query + 2), even
    uint32_t stride;                           // lanes per column row: the grid's threads
    int32_t a, b, o, e, nval, has_npen, npen;
    int32_t kofs;                              // table bias K: every score + K in [0, 255]
};

// A/C/G/T nibble -> 0..3 (A 1, C 3, G 7, T 4), anything else -> 4
__device__ __forceinline__ uint32_t ksw16_code(uint32_t nib) {
    return nib == 1 ? 0u : nib == 3 ? 1u : nib == 7 ? 2u : nib == 4 ? 3u : 4u;
}

// the first row of one pair: eh[0].h = h0, eh[1].h = h0 - oe (or 0), then - e while > e
__device__ __forceinline__ uint32_t ksw16_first_row(uint32_t j, uint32_t h0, int32_t oe, int32_t e, uint32_t qlen) {
    if (j == 0) return h0;
    int32_t h = (int32_t)h0 > oe ? (int32_t)h0 - oe : 0;
    for (uint32_t k = 2; k <= j; ++k) {
        if (k > qlen || h <= e) return 0;
        h -= e;
    }
    return j <= qlen ? (uint32_t)h : 0u;
}

#ifndef GX_KSW16_WAVES
#define GX_KSW16_WAVES 8   // waves per SIMD the register allocator must allow (A/B: 7)
#endif
// QC = 0: entries in the global [column][lane] array (any query up to 254).  QC > 0: the
// row of entries in QC registers of the lane and the selector words in LDS
// ([wave][column / 2][lane]), for queries up to QC - 2: no entry traffic at all (the
// global form moves ~84 GB per 1 M config-2 pairs and is HBM-bound, profiles/r03_ksw16.md).
template <int QC>
__global__ __launch_bounds__(256, QC == 0 ? GX_KSW16_WAVES : QC <= 64 ? 4 : QC <= 128 ? 3 : 2) void ksw16_kernel(Ksw16Args A) {
    extern __shared__ uint32_t ksw16_lds[];
    constexpr bool REG = QC > 0;
    const uint32_t lane_id = blockIdx.x * blockDim.x + threadIdx.x;
    constexpr uint32_t BIAS = 0x0800u, BIAS2 = 0x08000800u;
    const int32_t oe = A.o + A.e;
    // ---- the two pairs of this lane and whether both qualify ----
    bool valid[2], take = lane_id < A.n_lanes;
    uint32_t pr[2], ql[2] = {0, 0}, tl[2] = {0, 0}, h0[2] = {0, 0}, qo[2] = {0, 0}, to[2] = {0, 0};
    int step = max(max(A.a, -A.b), 0);
    if (A.has_npen) step = max(step, -A.npen);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        pr[h] = 2 * lane_id + h;
        valid[h] = take && pr[h] < A.n;
        if (valid[h]) {
            ql[h] = A.qlen[pr[h]]; tl[h] = A.tlen[pr[h]];
            h0[h] = A.seed[pr[h]];
            qo[h] = A.qoff[pr[h]] >> 3; to[h] = A.toff[pr[h]] >> 3;
            const uint64_t bound = (uint64_t)h0[h] + (uint64_t)step * min(ql[h], tl[h]);
            if (bound > 255u || ql[h] > 254u || ql[h] == 0 || A.todo[pr[h]] != 0) take = false;
            for (uint32_t w = 0; take && w < (ql[h] + 7) / 8; ++w) {
                const uint32_t word = A.qw[qo[h] + w];
                for (uint32_t k = 0; k < 8 && 8 * w + k < ql[h]; ++k)
                    if (ksw16_code((word >> (28 - 4 * k)) & 15u) > 3) take = false;
            }
        }
    }
    if (!valid[0]) take = false;
    // lanes that do not take their pairs still run the wave's loops, idle
    bool act_pair[2] = {take && valid[0], take && valid[1]};
    uint32_t qmax = max(act_pair[0] ? ql[0] : 0u, act_pair[1] ? ql[1] : 0u);
    qmax = (uint32_t)ksw_wave_max((int)qmax);
    const uint32_t stride = A.stride;                    // >= every lane of the grid
    uint32_t *ent = A.ent + lane_id;
    uint32_t *selp = REG ? ksw16_lds + (threadIdx.x >> 6) * (QC / 2) * 64 + (threadIdx.x & 63) : A.sel + lane_id;
    const uint32_t sstride = REG ? 64u : stride;
    uint32_t reg[REG ? QC : 1];
    // ---- selector words and the first row ----
    {
        for (uint32_t j = 0; j < qmax + 2; j += 2) {
            uint32_t s = 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t jj = j + u;
                uint32_t cA = 0, cB = 0;
                if (act_pair[0] && jj < ql[0]) cA = ksw16_code((A.qw[qo[0] + (jj >> 3)] >> (28 - 4 * (jj & 7))) & 15u);
                if (act_pair[1] && jj < ql[1]) cB = ksw16_code((A.qw[qo[1] + (jj >> 3)] >> (28 - 4 * (jj & 7))) & 15u);
                s |= (cA | ((4u + cB) << 8)) << (16 * u);
            }
            if (j / 2 < (A.cols + 1) / 2) selp[(size_t)(j / 2) * sstride] = s;
        }
        if constexpr (REG) {
            // eh[0] = h0, eh[1] = v1 = max(h0 - oe, 0), eh[j] = eh[j-1] - e while eh[j-1] > e and
            // j <= qlen: eh[j] = v1 - (j-1)e where j <= qlen and v1 > (j-1)e, else 0 (closed form)
            int32_t v1[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) v1[h] = act_pair[h] ? max((int32_t)h0[h] - oe, 0) : 0;
#pragma unroll
            for (int j = 0; j < QC; ++j) {
                uint32_t w = 0;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    int32_t v;
                    if (j == 0) v = act_pair[h] ? (int32_t)h0[h] : 0;
                    else {
                        const int32_t t = v1[h] - (j - 1) * A.e;
                        v = ((uint32_t)j <= ql[h] && t > 0) ? t : 0;
                    }
                    w |= (uint32_t)v << (16 * h);
                }
                reg[j] = w;
            }
        } else {
            for (uint32_t j = 0; j < qmax + 2 && j < A.cols; ++j) {
                uint32_t w = 0;
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (act_pair[h]) w |= ksw16_first_row(j, h0[h], oe, A.e, ql[h]) << (16 * h);
                ent[(size_t)j * stride] = w;
            }
        }
    }
    // ---- per-half row state (the reference's scalars) ----
    int32_t beg[2] = {0, 0}, end[2], mx[2], mx_i[2] = {-1, -1}, mx_j[2] = {-1, -1}, mx_ie[2] = {-1, -1},
            gsc[2] = {-1, -1};
    bool skip[2] = {false, false};
    uint32_t gpac[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h) { end[h] = (int32_t)ql[h]; mx[h] = (int32_t)h0[h]; }
    const int32_t nsc = A.has_npen ? -A.npen : 0;
    const uint32_t K = (uint32_t)A.kofs;
    const uint32_t OE2 = (uint32_t)oe * 0x10001u, EXT2 = (uint32_t)A.e * 0x10001u;
    const uint32_t NEGK = 0u - K * 0x10001u;
    int imax = max(act_pair[0] ? (int)tl[0] : 0, act_pair[1] ? (int)tl[1] : 0);
    imax = ksw_wave_max(imax);
    for (int i = 0; i < imax; ++i) {
        bool act[2];
        uint32_t T[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if ((i & 7) == 0) {
                skip[h] = false;
                if (act_pair[h] && i < (int)tl[h]) gpac[h] = A.tw[to[h] + (i >> 3)];
            }
            act[h] = act_pair[h] && i < (int)tl[h] && !skip[h];
            // substitution bytes of this row for query codes A, C, G, T (+ K)
            const uint32_t g = (gpac[h] >> (28 - 4 * (i & 7))) & 15u;
            const bool gN = (int32_t)g == A.nval;
            uint32_t t = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t nib = c == 0 ? 1u : c == 1 ? 3u : c == 2 ? 7u : 4u;
                const int32_t sc = (gN || (int32_t)nib == A.nval) ? nsc : (nib == g ? A.a : -A.b);   // g_sub_local
                t |= ((uint32_t)(sc + (int32_t)K) & 0xFFu) << (8 * c);
            }
            T[h] = t;
        }
        // the wave's column range: the active halves' [beg, end]
        int jlo = 0x7FFFFFFF, jhi = -1;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (act[h]) { jlo = min(jlo, beg[h]); jhi = max(jhi, end[h]); }
        jlo = -ksw_wave_max(-jlo);
        jhi = ksw_wave_max(jhi);
        if (jhi < 0) continue;   // no active half in the wave (every lane of it agrees)
        // row-start values per half: h1 = H(i, beg-1), f = 0 (biased)
        uint32_t H1 = 0, F = BIAS2;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int32_t v = 0;
            if (act[h] && beg[h] == 0) v = max((int32_t)h0[h] - (A.o + A.e * (i + 1)), 0);
            H1 |= ((uint32_t)v + BIAS) << (16 * h);
        }
        // per-half column bounds as j+1 < end+1 (store the cell), j+1 < end+2 (store eh[end]);
        // an idle half gets 0 / 0: it stores nothing
        uint32_t ENDP1 = 0, ENDP2 = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (act[h]) { ENDP1 |= (uint32_t)(end[h] + 1) << (16 * h); ENDP2 |= (uint32_t)(end[h] + 2) << (16 * h); }
        uint32_t mkey = 0, first2 = 0xFFFFFFFFu, last2 = 0;
        // columns in pairs from an even start (the extra cells left of every active half's
        // beg compute zeros; right of every end they keep their bytes); wave-uniform bounds
        const int j0 = __builtin_amdgcn_readfirstlane(jlo) & ~1, j1 = __builtin_amdgcn_readfirstlane(jhi);
        uint32_t JP = (uint32_t)(j0 + 1) * 0x10001u;          // j + 1 per half
        uint32_t *pe = ent + (size_t)j0 * stride;
        const uint32_t *ps = selp + (size_t)(j0 >> 1) * sstride;
        auto cell = [&](const uint32_t w, const uint32_t selw, uint32_t &dst) {
            const uint32_t H2 = __builtin_amdgcn_perm(0x08080808u, w, 0x04020400u);   // {hA, 8, hB, 8}: h + 0x800
            const uint32_t E2 = __builtin_amdgcn_perm(0x08080808u, w, 0x04030401u);
            const uint32_t nzM = l16_nz_mask(w & 0x00FF00FFu);                       // [H(i-1, j-1) != 0]
            const uint32_t sc2 = __builtin_amdgcn_perm(T[1], T[0], selw);           // {sA + K, 0, sB + K, 0}
            const uint32_t Msc = H2 + sc2 + NEGK;                                   // M + s, biased
            const uint32_t Mp = __builtin_amdgcn_bitop3_b32(Msc, nzM, BIAS2, 0xE2);  // nz ? M + s : 0
            const uint32_t Hn = pk_max3(Mp, E2, F);
            const uint32_t t = Mp - OE2;
            const uint32_t En = pk_max3(E2 - EXT2, t, BIAS2);
            F = pk_max3(F - EXT2, t, BIAS2);
            // masks: lt = [j < end] (the cell), le = [j <= end] (eh[end] too)
            const uint32_t d1 = GX_AS(uint32_t, GX_AS(pk_u2, JP) - GX_AS(pk_u2, ENDP1));
            const uint32_t d2 = GX_AS(uint32_t, GX_AS(pk_u2, JP) - GX_AS(pk_u2, ENDP2));
            const uint32_t lt16 = __builtin_amdgcn_perm(d1, d1, 0x0B0B0A0Au);
            mkey = pk_max_u16(mkey, pk_mad_u16(Hn, 0x01000100u, JP) & lt16);
            // stored bytes: h = H(i, j-1) where j <= end, e = E' where j < end, else the old byte
            // (e is 0 at j == end: E' masked by lt; then the new bytes where j <= end, else the old)
            const uint32_t wn = __builtin_amdgcn_perm(En & lt16, H1, 0x06020400u);
            const uint32_t mle = __builtin_amdgcn_perm(d2, d2, 0x09090808u);
            const uint32_t ws = __builtin_amdgcn_bitop3_b32(wn, w, mle, 0xE4);        // le ? wn : w
            dst = ws;
            const uint32_t nz = l16_nz_mask(ws);
            first2 = pk_min_u16(first2, JP | ~nz);
            last2 = pk_max_u16(last2, JP & nz);
            // H1 stops at the half's last cell: the stored h at j == end is H(i, end-1), and
            // after the row H1 holds it for the Q16 rule
            H1 = __builtin_amdgcn_bitop3_b32(Hn, H1, lt16, 0xE4);                   // lt ? Hn : H1
            JP += 0x10001u;
        };
        if constexpr (REG) {
            // blocks of 8 columns, unrolled over the register row; blocks wholly outside
            // [j0, j1] are skipped (wave-uniform branch)
#pragma unroll
            for (int blk = 0; blk < QC / 8; ++blk) {
                if (blk * 8 + 7 < j0 || blk * 8 > j1) continue;
                JP = (uint32_t)(blk * 8 + 1) * 0x10001u;
#pragma unroll
                for (int k = 0; k < 8; k += 2) {
                    const int j = blk * 8 + k;
                    const uint32_t sw = selp[(j >> 1) * 64];
                    cell(reg[j], __builtin_amdgcn_perm(0x0C0C0C0Cu, sw, 0x04010400u), reg[j]);
                    cell(reg[j + 1], __builtin_amdgcn_perm(0x0C0C0C0Cu, sw, 0x04030402u), reg[j + 1]);
                }
            }
        } else {
            for (int j = j0; j <= j1; j += 2) {
                const uint32_t sw = *ps;
                const uint32_t w0 = pe[0], w1 = pe[stride];
                cell(w0, __builtin_amdgcn_perm(0x0C0C0C0Cu, sw, 0x04010400u), pe[0]);
                cell(w1, __builtin_amdgcn_perm(0x0C0C0C0Cu, sw, 0x04030402u), pe[stride]);
                pe += 2 * stride;
                ps += sstride;
            }
        }
        // ---- row end per half (ksw_kernel_template.h:160-186) ----
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (!act[h]) continue;
            const int32_t e_ = end[h];
            // H(i, end-1): H1 stopped at the half's last cell (biased)
            const int32_t h1 = (int32_t)((H1 >> (16 * h)) & 0xFFFFu) - (int32_t)BIAS;
            if (e_ == (int32_t)ql[h] || (ql[h] & 7u) == 0) {                   // Q16
                mx_ie[h] = gsc[h] > h1 ? mx_ie[h] : i;
                gsc[h] = gsc[h] > h1 ? gsc[h] : h1;
            }
            const uint32_t kk = (mkey >> (16 * h)) & 0xFFFFu;
            const int32_t m = (int32_t)(kk >> 8), mj = (int32_t)(kk & 0xFFu) - 1;
            if (m == 0) { skip[h] = true; continue; }
            if (m > mx[h]) { mx[h] = m; mx_i[h] = i; mx_j[h] = mj; }
            const int32_t fst = (int32_t)((first2 >> (16 * h)) & 0xFFFFu) - 1;   // 0xFFFF - 1 when none
            const int32_t lst = (int32_t)((last2 >> (16 * h)) & 0xFFFFu) - 1;    // -1 when none
            const int32_t nb = min(fst, e_);
            int32_t l = lst;
            if (l < nb) l = nb - 1;
            beg[h] = nb;
            end[h] = l + 2 < (int32_t)ql[h] ? l + 2 : (int32_t)ql[h];
        }
    }
    if (!take) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (!valid[h]) continue;
        A.todo[pr[h]] = 0xFF;
        if (gsc[h] <= 0 || gsc[h] <= mx[h] - 5) {
            A.score[pr[h]] = mx[h];
            if (A.qend) A.qend[pr[h]] = mx_j[h] + 1;
            if (A.tend) A.tend[pr[h]] = mx_i[h] + 1;
        } else {
            A.score[pr[h]] = gsc[h];
            if (A.qend) A.qend[pr[h]] = (int32_t)ql[h];
            if (A.tend) A.tend[pr[h]] = mx_ie[h] + 1;
        }
    }
}

}  // namespace gx
