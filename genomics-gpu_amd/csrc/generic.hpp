// generic.hpp — thread-per-pair HIP kernels that walk the DP in the
// reference's own strip-major order.  They serve the configurations whose
// results depend on that order beyond the final maximum (local/semi-global
// second-best, the WITH_START reverse passes), the data-dependent banded and
// KSW kernels, and lengths beyond the wavefront kernels' register budget.
// Row buffers live in a pair-interleaved global workspace ([row][pair]) so
// that the 64 lanes of a wave touch consecutive words.
//
// Reference (Non-CDP/GASAL2/src): kernels/local_kernel_template.h:71-519,
// kernels/semiglobal_kernel_template.h:39-388, kernels/banded.h:10-139,
// kernels/ksw_kernel_template.h:46-199, kernels/get_tb.h:4-149,
// kernels/pack_rc_seqs.h:13-212.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gx {

struct GenArgs {
    const uint32_t *qw, *tw;          // packed words of the whole batch
    const uint32_t *qoff, *toff, *qlen, *tlen;
    const uint32_t *seed;
    int32_t *score, *qend, *tend, *qstart, *tstart;
    int32_t *score2, *qend2, *tend2;
    uint32_t *tb;                     // direction words (LOCAL WITH_TB), tb_pair_words per pair
    uint64_t tb_pair_words;
    int16_t *rowH, *rowE;             // [row][pair] scratch, rows_cap rows
    uint32_t rows_cap;
    uint32_t *rev;                    // [word][pair] scratch for semi-global WITH_START, 2*rev_words
    uint32_t rev_words;
    uint32_t n;
    int32_t a, b, o, e, nval, has_npen, npen;
    int32_t start_pos, second, head, tail, kbw, maxq;
    const uint8_t *todo;              // banded / local: only the pairs the packed kernel declined (NULL: all)
};

__device__ __forceinline__ uint32_t gcode(const uint32_t *w, uint32_t pos) {
    return (w[pos >> 3] >> (28 - ((pos & 7) << 2))) & 15u;
}
__device__ __forceinline__ int32_t g_sub_local(const GenArgs &A, uint32_t q, uint32_t t) {
    int32_t v = (q == t) ? A.a : -A.b;
    if ((int32_t)q == A.nval || (int32_t)t == A.nval) v = A.has_npen ? -A.npen : 0;
    return v;
}

// ---------------------------------------------------------------- local ----
__global__ __launch_bounds__(256) void gen_local_kernel(GenArgs A) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= A.n) return;
    if (A.todo && !A.todo[tid]) return;   // aligned by local2nd16_kernel
    const uint32_t ql = A.qlen[tid], tl = A.tlen[tid];
    const uint32_t *qw = A.qw + (A.qoff[tid] >> 3);
    const uint32_t *tw = A.tw + (A.toff[tid] >> 3);
    const uint32_t QR = (ql + 7) >> 3, TR = (tl + 7) >> 3, Q8 = QR * 8;
    const bool tb = A.start_pos == 2, second = A.second != 0;
    const int32_t OE = A.o + A.e;
#define RH(r) A.rowH[(size_t)(r) * A.n + tid]
#define RE(r) A.rowE[(size_t)(r) * A.n + tid]
    for (uint32_t r = 0; r < Q8; r++) { RH(r) = 0; RE(r) = 0; }
    int32_t h[9], f[9], p[9];
    int32_t maxHH = 0, maxY = 0, prevMax = 0, maxX = 0, max2 = 0, prev2 = 0, x2 = 0, y2 = 0;
    for (uint32_t i = 0; i < TR; i++) {
        for (int m = 0; m < 9; m++) h[m] = f[m] = p[m] = 0;
        const int32_t gidx = (int32_t)(i << 3);
        const uint32_t gpac = tw[i];
        for (uint32_t r = 0; r < Q8; r++) {
            const uint32_t qb = gcode(qw, r);
            uint32_t dword = 0;
            h[0] = RH(r);
            int32_t e = RE(r);
#pragma unroll
            for (int m = 1; m <= 8; m++) {
                const uint32_t tbase = (gpac >> (28 - 4 * (m - 1))) & 15u;
                const int32_t tmp = p[m] + g_sub_local(A, qb, tbase);
                const int32_t H = max(max(max(tmp, f[m]), e), 0);
                if (tb) {
                    const int sh = 28 - ((m - 1) << 2);
                    const uint32_t mxo = (tmp >= p[m]) ? 0u : 1u;
                    dword |= (H == tmp) ? (mxo << sh) : ((H == f[m]) ? (3u << sh) : (2u << sh));
                    dword |= ((tmp - OE) > (f[m] - A.e)) ? 0u : (1u << (sh + 3));
                    dword |= ((tmp - OE) > (e - A.e)) ? 0u : (1u << (sh + 2));
                }
                f[m] = max(tmp - OE, f[m] - A.e);
                e = max(tmp - OE, e - A.e);
                if (maxHH < H) { maxY = gidx + m - 1; maxHH = H; }
                if (second && max2 < H && maxHH > H) { y2 = gidx + m - 1; max2 = H; }
                h[m] = H;
                p[m] = h[m - 1];
            }
            RH(r) = (int16_t)h[8];
            RE(r) = (int16_t)e;
            if (tb) A.tb[(uint64_t)tid * A.tb_pair_words + (uint64_t)i * Q8 + r] = dword;
            maxX = (prevMax < maxHH) ? (int32_t)r : maxX;
            if (second) { x2 = (prev2 < maxHH) ? (int32_t)r : x2; prev2 = max(max2, prev2); }
            prevMax = max(maxHH, prevMax);
        }
    }
    A.score[tid] = maxHH;
    if (A.qend) A.qend[tid] = maxX;
    if (A.tend) A.tend[tid] = maxY;
    if (second) {
        if (A.score2) A.score2[tid] = max2;
        if (A.qend2) A.qend2[tid] = x2;
        if (A.tend2) A.tend2[tid] = y2;
    }
    if (A.start_pos == 1) {   // WITH_START reverse pass (local :441-511)
        const int32_t fwd = maxHH;
        const int32_t rend_reg = min((maxX >> 3) + 1, (int32_t)QR);
        const int32_t gend_reg = min((maxY >> 3) + 1, (int32_t)TR);
        int32_t mH = 0, pM = 0, sx = 0, sy = 0;
        for (uint32_t r = 0; r < Q8; r++) { RH(r) = 0; RE(r) = 0; }
        int32_t gidx = (gend_reg << 3) + 8 - 1;
        for (int32_t i = 0; i < gend_reg && mH < fwd; i++) {
            for (int m = 0; m < 9; m++) h[m] = f[m] = p[m] = 0;
            const uint32_t gpac = tw[gend_reg - 1 - i];
            gidx -= 8;
            int32_t ridx = (rend_reg << 3) - 1;
            int32_t gi = 0;
            for (int32_t j = 0; j < rend_reg && mH < fwd; j++) {
                const uint32_t rpac = qw[rend_reg - 1 - j];
                for (int k = 0; k <= 28 && mH < fwd; k += 4) {
                    const uint32_t qb = (rpac >> k) & 15u;
                    h[0] = RH(gi);
                    int32_t e = RE(gi);
#pragma unroll
                    for (int m = 1; m <= 8; m++) {
                        const uint32_t tbase = (gpac >> (4 * (m - 1))) & 15u;
                        const int32_t tmp = p[m] + g_sub_local(A, qb, tbase);
                        const int32_t H = max(max(max(tmp, f[m]), e), 0);
                        f[m] = max(tmp - OE, f[m] - A.e);
                        e = max(tmp - OE, e - A.e);
                        if (mH < H) { sy = gidx + (m - 1); mH = H; }   // Q8
                        h[m] = H;
                        p[m] = h[m - 1];
                    }
                    RH(gi) = (int16_t)h[8];
                    RE(gi) = (int16_t)e;
                    sx = (pM < mH) ? ridx : sx;
                    pM = max(mH, pM);
                    ridx--; gi++;
                }
            }
        }
        if (A.qstart) A.qstart[tid] = sx;
        if (A.tstart) A.tstart[tid] = sy;
    }
#undef RH
#undef RE
}

// --------------------------------------------------------------- global ----
// GLOBAL beyond the wavefront shapes (padded query > 1280, or values outside
// the range where int32 arithmetic without the int16 row buffer is exact):
// kernels/global.h:30-303.  Left column H(r, -1) = -(o + e*r) with H(0, -1) = 0
// (Q2), top row only through the diagonal, F = -inf at every strip start, no
// N rule (GLOBAL macro), (H, E) carried between strips as int16 (Q5), score =
// H(ql-1, tl-1) captured on the row ql-1 of the last strip (:98-103, :299).
__global__ __launch_bounds__(256) void gen_global_kernel(GenArgs A) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= A.n) return;
    const uint32_t ql = A.qlen[tid], tl = A.tlen[tid];
    const uint32_t *qw = A.qw + (A.qoff[tid] >> 3);
    const uint32_t *tw = A.tw + (A.toff[tid] >> 3);
    const uint32_t QR = (ql + 7) >> 3, TR = (tl + 7) >> 3, Q8 = QR * 8;
    const bool tb = A.start_pos == 2;
    const int32_t OE = A.o + A.e;
    auto sub = [&](uint32_t q, uint32_t t) {   // DEV_GET_SUB_SCORE_GLOBAL (gasal_kernels.h:44-54)
        int32_t v = (q == t) ? A.a : -A.b;
        if (A.has_npen && ((int32_t)q == A.nval || (int32_t)t == A.nval)) v = -A.npen;
        return v;
    };
#define RH(r) A.rowH[(size_t)(r) * A.n + tid]
#define RE(r) A.rowE[(size_t)(r) * A.n + tid]
    for (uint32_t r = 0; r < Q8; r++) {
        RH(r) = (int16_t)(r == 0 ? 0 : -(A.o + A.e * (int32_t)r));
        RE(r) = (int16_t)-32768;
    }
    int32_t h[9], f[9], p[9], last[9];
    for (int m = 0; m < 9; m++) last[m] = 0;
    h[0] = 0; p[0] = 0;
    for (uint32_t i = 0; i < TR; i++) {
        const int32_t c0 = (int32_t)(i << 3);
        for (int m = 1; m < 9; m++) {                       // :67-71 (u = column + 1, r = column)
            const int32_t col = c0 + m - 1;
            h[m] = -(A.o + A.e * (col + 1));
            f[m] = -32768;
            p[m] = col == 0 ? 0 : -(A.o + A.e * col);
        }
        const uint32_t gpac = tw[i];
        for (uint32_t r = 0; r < Q8; r++) {
            const uint32_t qb = gcode(qw, r);
            uint32_t dword = 0;
            h[0] = RH(r);
            int32_t e = RE(r);
#pragma unroll
            for (int m = 1; m <= 8; m++) {
                const uint32_t tbase = (gpac >> (28 - 4 * (m - 1))) & 15u;
                const int32_t tmp = p[m] + sub(qb, tbase);
                const int32_t H = max(max(tmp, f[m]), e);
                if (tb) {                                   // CORE_GLOBAL_COMPUTE_TB (:14-26)
                    const int sh = 28 - ((m - 1) << 2);
                    const uint32_t mxo = (tmp >= p[m]) ? 0u : 1u;
                    dword |= (H == tmp) ? (mxo << sh) : ((H == f[m]) ? (3u << sh) : (2u << sh));
                    dword |= ((tmp - OE) > (f[m] - A.e)) ? 0u : (1u << (sh + 3));
                    dword |= ((tmp - OE) > (e - A.e)) ? 0u : (1u << (sh + 2));
                }
                f[m] = max(tmp - OE, f[m] - A.e);
                e = max(tmp - OE, e - A.e);
                h[m] = H;
                p[m] = h[m - 1];
            }
            RH(r) = (int16_t)h[8];
            RE(r) = (int16_t)e;
            if (tb) A.tb[(uint64_t)tid * A.tb_pair_words + (uint64_t)i * Q8 + r] = dword;
            if (r + 1 == ql)
                for (int m = 1; m < 9; m++) last[m] = h[m];
        }
    }
    A.score[tid] = last[8 - ((TR << 3) - tl)];
#undef RH
#undef RE
}

// ----------------------------------------------------------- semi-global ----
__device__ __forceinline__ void semi_rows_init(const GenArgs &A, uint32_t tid, uint32_t nrow) {
    const bool hq = (A.head == 1 || A.head == 3);
    for (uint32_t r = 0; r < nrow; r++) {
        A.rowH[(size_t)r * A.n + tid] = hq ? 0 : (int16_t)((r == 0) ? 0 : -(A.o + A.e * (int32_t)r));
        A.rowE[(size_t)r * A.n + tid] = hq ? 0 : (int16_t)-32768;
    }
}

template <bool REV>
__device__ void semi_pass(const GenArgs &A, uint32_t tid, const uint32_t *qw, const uint32_t *tw, uint32_t QR,
                          uint32_t TR, uint32_t ql, uint32_t tl, int32_t i0, bool early, int32_t fwd, bool second,
                          int32_t &maxHH, int32_t &maxY, int32_t &max2, int32_t &y2) {
    const int32_t OE = A.o + A.e;
    const bool ht = (A.head == 2 || A.head == 3);
    const bool tailT = (A.tail == 2 || A.tail == 3);
    int32_t h[9], f[9], p[9];
    int32_t u = 1, rr = 1;
    h[0] = 0; p[0] = 0;
    for (int32_t i = i0; i < (int32_t)TR && (!early || maxHH < fwd); i++) {
        const int32_t gidx = i << 3;
        if (ht) {
            for (int m = 0; m < 9; m++) { h[m] = 0; f[m] = -32768; p[m] = 0; }
        } else {
            for (int m = 1; m < 9; m++, u++, rr++) {
                h[m] = -(A.o + A.e * (u - 1));
                f[m] = -32768;
                p[m] = (rr == 1) ? 0 : -(A.o + A.e * (rr - 1));
            }
        }
        // negative strips (gend_reg < 0) read zero words, as in the oracle
        const uint32_t gpac = i < 0 ? 0u : (REV ? A.rev[(size_t)(A.rev_words + i) * A.n + tid] : tw[i]);
        uint32_t ridx = 0;
        for (uint32_t j = 0; j < QR && (!early || maxHH < fwd); j++) {
            const uint32_t rpac = REV ? A.rev[(size_t)j * A.n + tid] : qw[j];
            for (int k = 28; k >= 0; k -= 4) {
                const uint32_t qb = (rpac >> k) & 15u;
                h[0] = A.rowH[(size_t)ridx * A.n + tid];
                int32_t e = A.rowE[(size_t)ridx * A.n + tid];
                int32_t prev = h[0] - OE;
#pragma unroll
                for (int m = 1; m < 9; m++) {
                    const uint32_t tbase = (gpac >> (28 - 4 * (m - 1))) & 15u;
                    const int32_t s = g_sub_local(A, qb, tbase);
                    int32_t curr = h[m] - OE;
                    f[m] = max(curr, f[m] - A.e);
                    curr = p[m] + s;
                    curr = max(curr, f[m]);
                    e = max(prev, e - A.e);
                    curr = max(curr, e);
                    h[m] = curr;
                    p[m] = prev + OE;
                    prev = curr - OE;
                }
                A.rowH[(size_t)ridx * A.n + tid] = (int16_t)h[8];
                A.rowE[(size_t)ridx * A.n + tid] = (int16_t)e;
                ridx++;
                if (tailT && ridx == ql) {
                    for (int m = 1; m < 9; m++) {
                        const int32_t col = gidx + m - 1;
                        if (h[m] > maxHH && col < (int32_t)tl) { maxY = col; maxHH = h[m]; }
                        if (second && h[m] > max2 && h[m] < maxHH && col < (int32_t)tl) { y2 = col; max2 = h[m]; }
                    }
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void gen_semi_kernel(GenArgs A) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= A.n) return;
    const uint32_t ql = A.qlen[tid], tl = A.tlen[tid];
    const uint32_t *qw = A.qw + (A.qoff[tid] >> 3);
    const uint32_t *tw = A.tw + (A.toff[tid] >> 3);
    const uint32_t QR = (ql + 7) >> 3, TR = (tl + 7) >> 3;
    const bool second = A.second != 0;
    const bool tailQ = (A.tail == 1 || A.tail == 3);
    const uint32_t maxq = (uint32_t)A.maxq;            // rows scanned for TAIL QUERY (:187)
    int32_t maxHH = -32768, maxX = (int32_t)tl, maxY = (int32_t)ql;
    int32_t max2 = -32768, x2 = (int32_t)tl, y2 = (int32_t)ql;
    semi_rows_init(A, tid, A.rows_cap);
    semi_pass<false>(A, tid, qw, tw, QR, TR, ql, tl, 0, false, 0, second, maxHH, maxY, max2, y2);
    if (tailQ) {
        for (uint32_t m = 0; m < maxq; m++) {
            const int32_t v = A.rowH[(size_t)m * A.n + tid];
            if (v > maxHH && m < ql) { maxX = (int32_t)m; maxHH = v; }
            if (second && v > max2 && v < maxHH && m < tl) { x2 = (int32_t)m; max2 = v; }   // Q12
        }
        if (maxX != (int32_t)tl) maxY = (int32_t)ql;
        if (second && x2 != (int32_t)tl) y2 = (int32_t)ql;
    }
    A.score[tid] = maxHH;
    if (A.tend) A.tend[tid] = maxY;
    if (A.qend) A.qend[tid] = maxX;
    if (second) {
        if (A.score2) A.score2[tid] = max2;
        if (A.tend2) A.tend2[tid] = y2;
        if (A.qend2) A.qend2[tid] = x2;
    }
    if (A.start_pos == 1) {   // :227-383
        const uint32_t nw = A.rev_words;
        for (uint32_t w = 0; w < 2 * nw; w++) A.rev[(size_t)w * A.n + tid] = 0;
        for (int32_t i = (int32_t)ql - 1, k = 0; i >= 0; i--, k++) {
            const uint32_t sym = gcode(qw, (uint32_t)i);
            A.rev[(size_t)(k >> 3) * A.n + tid] |= sym << (28 - ((k & 7) << 2));
        }
        for (int32_t i = (int32_t)tl - 1, k = 0; i >= 0; i--, k++) {
            const uint32_t sym = gcode(tw, (uint32_t)i);
            A.rev[(size_t)(nw + (k >> 3)) * A.n + tid] |= sym << (28 - ((k & 7) << 2));
        }
        const int32_t fwd = maxHH;
        const int32_t d = (int32_t)TR - ((maxY >> 3) + 1);
        const int32_t gend_reg = d > 0 ? d - 1 : d;
        int32_t rmax = -32768, ry = 0, d2 = 0, dy = 0;
        semi_rows_init(A, tid, A.rows_cap);
        semi_pass<true>(A, tid, qw, tw, QR, TR, ql, tl, gend_reg, true, fwd, false, rmax, ry, d2, dy);
        if (tailQ) {
            for (uint32_t m = 0; m < maxq; m++) {
                const int32_t v = A.rowH[(size_t)m * A.n + tid];
                if (v > rmax && m < ql) { maxX = (int32_t)m; rmax = v; }
            }
            if (maxX != (int32_t)tl) ry = (int32_t)ql;
        }
        if (A.tstart) A.tstart[tid] = ((int32_t)tl - 1) - ry;
        if (A.qstart) A.qstart[tid] = ((int32_t)ql - 1) - maxX;
    }
}

// --------------------------------------------------------------- banded ----
__global__ __launch_bounds__(256) void gen_banded_kernel(GenArgs A) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= A.n) return;
    if (A.todo && !A.todo[tid]) return;
    const uint32_t ql = A.qlen[tid], tl = A.tlen[tid];
    const uint32_t *qw = A.qw + (A.qoff[tid] >> 3);
    const uint32_t *tw = A.tw + (A.toff[tid] >> 3);
    const int32_t QR = (int32_t)((ql + 7) >> 3), TR = (int32_t)((tl + 7) >> 3);
    const int32_t OE = A.o + A.e;
    for (int32_t r = 0; r < QR * 8; r++) { A.rowH[(size_t)r * A.n + tid] = 0; A.rowE[(size_t)r * A.n + tid] = 0; }
    int32_t h[9], f[9], p[9];
    int32_t maxHH = 0, prevMax = 0, maxX = 0, maxY = 0;
    const int32_t kother = TR - (QR - A.kbw);                         // banded.h:35
    for (int32_t i = 0; i < TR; i++) {
        for (int m = 0; m < 9; m++) h[m] = f[m] = p[m] = 0;
        const int32_t gidx = i << 3;
        int32_t ridx = max(0, i - kother + 1) << 3;
        const int32_t last_tile = min(A.kbw + i, QR);
        const uint32_t gpac = tw[i];
        for (int32_t j = ridx >> 3; j < last_tile; j++) {
            const uint32_t rpac = qw[j];
            for (int k = 28; k >= 0; k -= 4) {
                const uint32_t qb = (rpac >> k) & 15u;
                h[0] = A.rowH[(size_t)ridx * A.n + tid];
                int32_t e = A.rowE[(size_t)ridx * A.n + tid];
#pragma unroll
                for (int m = 1; m < 9; m++) {
                    const uint32_t tbase = (gpac >> (28 - 4 * (m - 1))) & 15u;
                    const int32_t s = g_sub_local(A, qb, tbase);
                    f[m] = max(h[m] - OE, f[m] - A.e);
                    int32_t hv = max(max(p[m] + s, f[m]), 0);
                    e = max(h[m - 1] - OE, e - A.e);
                    hv = max(hv, e);
                    h[m] = hv;
                    if (maxHH < hv) { maxY = gidx + (m - 1); maxHH = hv; }
                    p[m] = h[m - 1];
                }
                A.rowH[(size_t)ridx * A.n + tid] = (int16_t)h[8];
                A.rowE[(size_t)ridx * A.n + tid] = (int16_t)e;
                maxX = (prevMax < maxHH) ? ridx : maxX;
                prevMax = max(maxHH, prevMax);
                ridx++;
            }
        }
    }
    A.score[tid] = maxHH;
    if (A.qend) A.qend[tid] = maxX;
    if (A.tend) A.tend[tid] = maxY;
}

// ------------------------------------------------------------------ KSW ----
// eh[] of the reference (ksw_kernel_template.h:69) as (h, e) int32 pairs in one
// 8-byte entry, [column][pair]: one load and one store per cell.  The row's
// beg/end trimming scans (:181-186) are tracked while the row is computed (first
// and last stored entry that is not (0, 0)) instead of re-reading the row.
// Rows are iterated in lockstep by the wave (a lane that the reference would
// `break` out of a tile just sits the rows out), so that every row's column
// loop can start at the wave's smallest beg — the lanes then touch the same
// column, and the [column][pair] entries stay coalesced.
__device__ __forceinline__ int ksw_wave_min(int v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = min(v, __shfl_xor(v, m));
    return v;
}
__device__ __forceinline__ int ksw_wave_max(int v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = max(v, __shfl_xor(v, m));
    return v;
}

// The entry width is a level: 0 = (h, e) as two uint8 in 16 bits, 1 = two uint16 in
// 32 bits, 2 = int2 (both values are >= 0 and at most h0 + match * min(qlen, tlen)).
// Narrower entries cut the loop's traffic (603 -> 808 GCUPS); a pair whose bound does
// not fit its level is flagged (todo = level + 1) for the next instance.  The loop is
// then bound by its VALU work (profiles/r02_ksw_lds_ab.md).
//
// INLDS (level 0 only): the pair's entries live in LDS, [column][thread] uint16 of
// the block (2 * blockDim * (max qlen + 2) bytes, dispatch.hip sizes the block so
// two fit a CU), instead of the [column][pair] global array: no lockstep column
// start is needed (any mix of columns is bank-conflict free: a thread's bank is
// fixed by its index) and the row's entries never leave the CU.
template <int LEVEL, bool INLDS = false>
__global__ __launch_bounds__(256) void gen_ksw_kernel(GenArgs A, void *ehv, uint8_t *todo) {
    static_assert(!INLDS || LEVEL == 0, "LDS entries are the 8-bit level");
    extern __shared__ __attribute__((aligned(16))) uint16_t ksw_lds[];
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    // lanes past n, and pairs of the other instance, run the wave's row loop without work
    bool live = tid < A.n && (todo ? todo[tid] == LEVEL : LEVEL == 2);
    if (LEVEL < 2 && live) {
        // no cell gains more than max(match, -mismatch, -N_PENALTY, 0) over its diagonal
        // (a negative mismatch or N penalty is a gain), and gaps cost >= 0; negative gap
        // scores have no such bound and go to the int2 level
        int step = max(max(A.a, -A.b), 0);
        if (A.has_npen) step = max(step, -A.npen);
        const uint64_t bound = (A.o < 0 || A.e < 0) ? ~0ull
                                                    : (uint64_t)(A.seed ? A.seed[tid] : 0u) +
                                                          (uint64_t)step * min(A.qlen[tid], A.tlen[tid]);
        if (bound > (LEVEL == 0 ? 255u : 65535u)) { todo[tid] = LEVEL + 1; live = false; }
    }
    const uint32_t qlen = live ? A.qlen[tid] : 0u, tlen = live ? A.tlen[tid] : 0u;
    const uint32_t *qw = A.qw + (live ? A.qoff[tid] >> 3 : 0u);
    const uint32_t *tw = A.tw + (live ? A.toff[tid] >> 3 : 0u);
    const uint32_t h0 = (live && A.seed) ? A.seed[tid] : 0u;
    const int o_del = A.o, o_ins = A.o, e_del = A.e, e_ins = A.e;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    int2 *ehw = reinterpret_cast<int2 *>(ehv);
    uint32_t *ehn = reinterpret_cast<uint32_t *>(ehv);
    uint16_t *ehb = reinterpret_cast<uint16_t *>(ehv);
    auto put = [&](int j, int h, int e) {
        if (INLDS) ksw_lds[(uint32_t)j * blockDim.x + threadIdx.x] = (uint16_t)((uint32_t)h | ((uint32_t)e << 8));
        else if (LEVEL == 0) ehb[(size_t)j * A.n + tid] = (uint16_t)((uint32_t)h | ((uint32_t)e << 8));
        else if (LEVEL == 1) ehn[(size_t)j * A.n + tid] = (uint32_t)h | ((uint32_t)e << 16);
        else ehw[(size_t)j * A.n + tid] = make_int2(h, e);
    };
    auto get = [&](int j) {
        if (LEVEL == 0) {
            const uint32_t v = INLDS ? (uint32_t)ksw_lds[(uint32_t)j * blockDim.x + threadIdx.x]
                                     : (uint32_t)ehb[(size_t)j * A.n + tid];
            return make_int2((int)(v & 0xFFu), (int)(v >> 8));
        }
        if (LEVEL == 1) {
            const uint32_t v = ehn[(size_t)j * A.n + tid];
            return make_int2((int)(v & 0xFFFFu), (int)(v >> 16));
        }
        return ehw[(size_t)j * A.n + tid];
    };
    if (live) {
        for (uint32_t j = 0; j < qlen + 2; j++) put((int)j, 0, 0);
        int h = (int32_t)h0;       // the first row (:72-76)
        put(0, h, 0);
        h = (h0 > (uint32_t)oe_ins) ? (int32_t)(h0 - (uint32_t)oe_ins) : 0;
        put(1, h, 0);
        for (int j = 2; j <= (int)qlen && h > e_ins; ++j) { h -= e_ins; put(j, h, 0); }
    }
    int max_ = (int32_t)h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1;
    int beg = 0, end = (int)qlen;
    // target rows in tiles of 8 (TR = tlen/8 + 1 words, Q16); `m == 0` skips the rest
    // of the tile (:165-166), a row past tlen ends it (:101-102)
    const int imax = ksw_wave_max((int)tlen);
    bool skip = false;
    uint32_t gpac = 0;
    for (int i = 0; i < imax; ++i) {
        if ((i & 7) == 0) {
            skip = false;
            if (i < (int)tlen) gpac = tw[i >> 3];
        }
        const bool act = i < (int)tlen && !skip;
        const int jlo = INLDS ? beg : ksw_wave_min(act ? beg : 0x7FFFFFFF);
        if (!act) continue;
        const uint32_t gbase = (gpac >> (28 - 4 * (i & 7))) & 0x0F;
        // substitution scores of this row (g_sub_local): N in the target row scores every
        // cell N; otherwise match / mismatch, or N for an N in the query
        const int32_t nsc = A.has_npen ? -A.npen : 0;
        const bool gN = (int32_t)gbase == A.nval;
        const int32_t sc_eq = gN ? nsc : A.a, sc_ne = gN ? nsc : -A.b;
        int f = 0, h1, m = 0, mj = -1;
        if (beg == 0) {
            h1 = (int32_t)(h0 - (uint32_t)(o_del + e_del * (i + 1)));
            if (h1 < 0) h1 = 0;
        } else h1 = 0;
        int first = end, last = beg - 1;   // stored entries other than (0, 0) in [beg, end]
        uint32_t rpac = qw[(uint32_t)jlo >> 3];
        for (int j = jlo; j < end; ++j) {
            if ((j & 7) == 0) rpac = qw[(uint32_t)j >> 3];
            if (j < beg) continue;
            const uint32_t rbase = (rpac >> (28 - 4 * (j & 7))) & 0x0F;
            const int2 v = get(j);
            int M = v.x, e = v.y;
            const int hs = h1;           // H(i, j-1), stored for the next row
            int sc = rbase == gbase ? sc_eq : sc_ne;
            sc = (int32_t)rbase == A.nval ? nsc : sc;
            M = M ? M + sc : 0;
            const int h = max(max(M, e), f);
            h1 = h;
            mj = m > h ? mj : j;
            m = m > h ? m : h;
            e = max(max(e - e_del, M - oe_del), 0);   // (:122-131) t = max(M - oe, 0); e = max(e - e, t)
            put(j, hs, e);
            if ((hs | e) != 0) { first = min(first, j); last = j; }   // h, e >= 0
            f = max(max(f - e_ins, M - oe_ins), 0);
        }
        put(end, h1, 0);
        if (h1 != 0) { first = min(first, end); last = end; }
        // the reference's column index after its loops is qlen exactly when the
        // row ended at qlen or qlen is a multiple of 8 (Q16's extra word)
        if (end == (int)qlen || (qlen & 7u) == 0) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (m == 0) { skip = true; continue; }
        if (m > max_) { max_ = m; max_i = i; max_j = mj; }
        beg = min(first, end);                                  // :181-183
        if (last < beg) last = beg - 1;                         // the backward scan stops at beg
        end = last + 2 < (int)qlen ? last + 2 : (int)qlen;      // :184-186
    }
    if (!live) return;
    if (gscore <= 0 || gscore <= max_ - 5) {
        A.score[tid] = max_;
        if (A.qend) A.qend[tid] = max_j + 1;
        if (A.tend) A.tend[tid] = max_i + 1;
    } else {
        A.score[tid] = gscore;
        if (A.qend) A.qend[tid] = (int32_t)qlen;
        if (A.tend) A.tend[tid] = max_ie + 1;
    }
}

// ------------------------------------------------------------- traceback ----
struct TbArgs {
    const uint32_t *tb;
    uint64_t tb_pair_words;
    const uint32_t *qlen, *tlen, *qoff;
    const int32_t *score, *qend, *tend;
    int32_t *qstart, *tstart;
    uint8_t *cigar;
    uint64_t cigar_cap;                 // writable bytes at cigar: a CIGAR longer than its slot
                                        // runs into the next one, never past the buffer
    uint32_t *n_ops;
    uint32_t n;
    int32_t a, b, o, e;
    int32_t is_local;
    // pairs aligned by the packed GLOBAL+TB kernel (wavefront16.hpp) use its
    // skewed uint16 layout: flag per block of pk_ppb pairs, R rows per lane
    const uint8_t *pk_flags;
    uint32_t pk_ppb, pk_R, pk_G, pk_rmagic;   // pk_rmagic = ceil(2^32 / pk_R)
    uint32_t pk_q8;                     // packed chunks of 8 consecutive pairs interleaved (wavefront16.hpp tb_store_window)
    const int32_t *pk_fix;              // H' at the start cell (row ql, column tl) when both are pads
    const uint32_t *slot_of;            // pair -> slot of the DP launch when it ran sorted, or NULL
    int32_t sc_nn;                      // substitution score N vs N (GLOBAL rule)
    // sequences (as the wavefront kernels read them) for the flags' s < 0 bit
    const uint8_t *qseq, *tseq;
    const uint32_t *toff;
    int32_t seq_packed, nval, has_npen, npen;
    // band recomputation (wavefront16.hpp WF16_GLOBAL_CP band pass): packed pairs read the flags of
    // their lane's band window ([wave][64][wd/4][R/4] uint4, two pairs per entry); a path that
    // leaves the band appends its pair to fb_list and stops (its bytes so far are a prefix of
    // the CIGAR the full-matrix walk writes later)
    const uint4 *band;
    uint32_t band_w, band_wd, pk_ppw;   // pk_ppw: pairs (slots) per wave of the DP launch
    // a mixed-shape DP launch (wf16_mix_kernel): slots from pk_p1 on ran the second shape (pk_G2 x
    // pk_R2, band window band_wd2, buffers from band2 on), their flags from pk_b1 on, pk_ppb2 slots
    // each (pk_p1 = 0xFFFFFFFF: one shape)
    uint32_t pk_p1, pk_b1, pk_ppb2;
    const uint4 *band2;
    uint32_t band_wd2, pk_R2, pk_G2, pk_ppw2, pk_rmagic2;
    uint32_t *fb_list, *fb_count;
    // fallback walk: thread t walks pair list[t], t < *n_dev - n_dev_off; its slot in the DP launch is t
    // (tb_slot: its direction words at slot t of the capped buffer)
    const uint32_t *list, *n_dev;
    uint32_t n_dev_off, tb_slot;
};

// 8 codes of a sequence cached per thread (the walk moves one position at a time)
__device__ __forceinline__ uint32_t tb_code(const uint8_t *seq, uint32_t off, uint32_t pos, int packed, uint2 &v,
                                            int32_t &key) {
    const int32_t k = (int32_t)(pos >> 3);
    if (k != key) {
        key = k;
        v = packed ? make_uint2(reinterpret_cast<const uint32_t *>(seq)[(off >> 3) + (uint32_t)k], 0u)
                   : *reinterpret_cast<const uint2 *>(seq + off + 8u * (uint32_t)k);
    }
    const uint32_t p = pos & 7u;
    return packed ? (v.x >> (28 - 4 * p)) & 15u : ((p < 4 ? v.x : v.y) >> (8 * (p & 3u))) & 15u;
}
__device__ __forceinline__ uint32_t pick4(const uint4 &c, uint32_t k) {
    return k == 0 ? c.x : k == 1 ? c.y : k == 2 ? c.z : c.w;
}

__global__ __launch_bounds__(256) void tb_kernel(TbArgs A) {
    const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (t0 >= A.n || (A.n_dev && t0 + A.n_dev_off >= *A.n_dev)) return;
    const uint32_t tid = A.list ? A.list[t0] : t0;                          // the pair
    const uint32_t slot = A.list ? t0 : (A.slot_of ? A.slot_of[tid] : tid);   // its slot in the DP launch
    const uint32_t ql = A.qlen[tid], tl = A.tlen[tid];
    const uint32_t q8 = (ql + 7) & ~7u, tstrips = (tl + 7) >> 3;
    const uint32_t *tb = A.tb + (uint64_t)(A.tb_slot ? slot : tid) * A.tb_pair_words;
    const int32_t OE = A.o + A.e;
    int i, j, total = 0, curr = 0;
    if (A.is_local) { i = A.tend[tid]; j = A.qend[tid]; total = A.score[tid]; }
    else { i = (int)tl; j = (int)ql; }
    const bool reg2 = slot >= A.pk_p1;   // the second shape of a mixed DP launch
    const bool pk = A.pk_flags && A.pk_flags[reg2 ? A.pk_b1 + (slot - A.pk_p1) / A.pk_ppb2 : slot / A.pk_ppb];
    const bool bnd = pk && A.band;
    const uint32_t bslot = reg2 ? slot - A.pk_p1 : slot, bppw = reg2 ? A.pk_ppw2 : A.pk_ppw;
    const uint32_t bG = reg2 ? A.pk_G2 : A.pk_G, bR = reg2 ? A.pk_R2 : A.pk_R;
    const uint32_t bwd = reg2 ? A.band_wd2 : A.band_wd, bmagic = reg2 ? A.pk_rmagic2 : A.pk_rmagic;
    // band layout: this pair's half of its lane group's entries in wave bslot / bppw
    const uint2 *bnd2 = bnd ? reinterpret_cast<const uint2 *>(reg2 ? A.band2 : A.band) +
                                  ((uint64_t)(bslot / bppw) * 64 + ((bslot % bppw) >> 1) * bG) * ((bwd / 4) * (bR / 4)) * 2 +
                                  (slot & 1u)
                            : nullptr;
    // band path: the int32 kernel aligned a declined block's pairs without direction words (the
    // fallback launch, over the list, writes them into the capped buffer)
    bool out_of_band = A.band && !pk;
    // interleaved packed layout: the region of pairs (tid & ~7) .. (tid | 7), chunk c of this
    // pair at 8 * c + (tid & 7)
    const bool il8 = pk && A.pk_q8;
    const uint16_t *tb16 = reinterpret_cast<const uint16_t *>(il8 ? A.tb + (uint64_t)(tid & ~7u) * A.tb_pair_words : tb);
    // packed kernel: the start cell (ql, tl), both pads, was scored with the pad
    // row's -K instead of N==N.  Its E and F are exact, so with H' the value it
    // did compute, the true cell takes the diagonal iff score + sc(N,N) >= H'.
    bool fix_diag = pk && !A.is_local && (ql & 7) && (tl & 7) && A.score[tid] + A.sc_nn >= A.pk_fix[tid];
    uint8_t *out = A.cigar + A.qoff[tid];
    const uint64_t room = A.cigar_cap > A.qoff[tid] ? A.cigar_cap - A.qoff[tid] : 0;
    auto put = [&](int at, uint32_t byte) { if ((uint64_t)at < room) out[at] = (uint8_t)byte; };
    uint32_t prev = 0, opf = 0;
    int n_ops = 0, off = 0, count = 0, op_select = 3, op_shift = 0;
    // the walk reads one cell per step, mostly from consecutive rows: keep the
    // chunk it is in (16 bytes: 4 rows of words; 8 bytes: 4 rows of 16-bit flags) and the
    // current 8 codes of each sequence, so most steps make no memory access
    // (loaded once: the CIGAR byte stores may alias any input for the compiler)
    const uint32_t qoff = A.qoff[tid], toff = pk ? A.toff[tid] : 0u;
    uint4 chunk = make_uint4(0u, 0u, 0u, 0u);
    int64_t chunk_key = -1;
    uint2 qv = make_uint2(0u, 0u), tv = make_uint2(0u, 0u);
    int32_t qkey = -1, tkey = -1;
    while (!out_of_band && i >= 0 && j >= 0) {
        // get_tb.h:50-71: linear cell index over (strip, row, column); a start
        // one row past the padded query (j == q8) wraps to row 0 of the next strip
        const bool wrap = j >= (int)q8;
        const uint32_t strip = (uint32_t)(i >> 3) + (wrap ? 1u : 0u), row = wrap ? 0u : (uint32_t)j,
                       c7 = (uint32_t)i & 7u;
        uint32_t cell_op = 0;   // past the padded grid: 0
        if (strip < tstrips) {
            if (bnd) {
                // band window of the row's lane: columns [L, L + wd), flags of 4 x 4 chunks
                const uint32_t col = strip * 8 + c7;
                const uint32_t lane = __umulhi(row, bmagic), k = row - lane * bR;
                const int32_t L = max((int32_t)(lane * bR) - (int32_t)A.band_w, 0);
                const uint32_t t = (uint32_t)((int32_t)col - L);
                if (t >= bwd) { out_of_band = true; break; }
                const int64_t key = (((int64_t)lane * (bwd / 4) + (t >> 2)) * (bR / 4) + (k >> 2)) * 2;
                if (key != chunk_key) {
                    const uint2 c2 = bnd2[key];
                    chunk = make_uint4(c2.x, c2.y, 0u, 0u);
                    chunk_key = key;
                }
                const uint32_t fl = (((k & 2u) ? chunk.y : chunk.x) >> (16 * (k & 1u) + (t & 3u))) & 0xFFFFu;
                const uint32_t qc = tb_code(A.qseq, qoff, row, A.seq_packed, qv, qkey);
                const uint32_t tc = tb_code(A.tseq, toff, col, A.seq_packed, tv, tkey);
                int32_t sc = qc == tc ? A.a : -A.b;                                   // global.h rule
                if (A.has_npen && ((int32_t)qc == A.nval || (int32_t)tc == A.nval)) sc = -A.npen;
                const uint32_t u = fix_diag ? 0u : (fl & 1u);
                fix_diag = false;
                cell_op = (u ? ((fl & 16u) ? 2u : 3u) : (sc < 0 ? 1u : 0u)) | ((fl & 256u) ? 0u : 4u) |
                          ((fl & 4096u) ? 0u : 8u);
            } else if (pk) {
                // wavefront16.hpp step_global_tb flags -> the reference's nibble
                // window (column + lane) / 4 holds G*R entries, row lane*R + k at
                // ((k/4)*G + lane)*4 + k%4 (wavefront16.hpp): 4 rows per 8-byte chunk
                const uint32_t col = strip * 8 + c7;
                const uint32_t lane = __umulhi(row, A.pk_rmagic), k = row - lane * A.pk_R;
                const uint32_t s = col + lane;
                // one 8-byte chunk (4 rows x 4 steps) per miss: the walk is bound by the
                // lines it fetches (a 2 x 2 block of chunks per miss fetched 1.6x the lines
                // and took 1.19 ms instead of 0.70, profiles/r03_tb_walk.md)
                const int64_t key = il8 ? (((int64_t)(s >> 2) * (A.pk_R >> 2) + (k >> 2)) * A.pk_G + lane) * 32 + (tid & 7u) * 4
                                       : (int64_t)(s >> 2) * (A.pk_G * A.pk_R) + ((k >> 2) * A.pk_G + lane) * 4;
                if (key != chunk_key) {
                    const uint2 c2 = *reinterpret_cast<const uint2 *>(tb16 + key);
                    chunk = make_uint4(c2.x, c2.y, 0u, 0u);
                    chunk_key = key;
                }
                const uint32_t fl = (((k & 2u) ? chunk.y : chunk.x) >> (16 * (k & 1u) + (s & 3u))) & 0xFFFFu;
                const uint32_t qc = tb_code(A.qseq, qoff, row, A.seq_packed, qv, qkey);
                const uint32_t tc = tb_code(A.tseq, toff, col, A.seq_packed, tv, tkey);
                int32_t sc = qc == tc ? A.a : -A.b;                                   // global.h rule
                if (A.has_npen && ((int32_t)qc == A.nval || (int32_t)tc == A.nval)) sc = -A.npen;
                if (A.is_local && !A.has_npen && ((int32_t)qc == A.nval || (int32_t)tc == A.nval)) sc = 0;   // local N rule
                const uint32_t u = fix_diag ? 0u : (fl & 1u);
                fix_diag = false;
                cell_op = (u ? ((fl & 16u) ? 2u : 3u) : (sc < 0 ? 1u : 0u)) | ((fl & 256u) ? 0u : 4u) |
                          ((fl & 4096u) ? 0u : 8u);
            } else {
                const int64_t key = (int64_t)strip * q8 + (row & ~3u);
                if (key != chunk_key) { chunk = *reinterpret_cast<const uint4 *>(tb + key); chunk_key = key; }
                cell_op = (pick4(chunk, row & 3u) >> (28 - (c7 << 2))) & 15u;
            }
        }
        const uint32_t op = (cell_op >> op_shift) & (uint32_t)op_select;
        opf = (op == 0 || op_select == 3) ? op : (uint32_t)op_shift;
        op_select = (op == 0 || (op == 1 && op_select == 3)) ? 3 : 1;
        op_shift = (op == 0 || (op == 1 && op_select == 3)) ? 0 : ((op == 2 || op == 3) ? (int)op : op_shift);
        if (count < 63 && opf == prev) {
            count++;
        } else {
            if (count > 0) { put(off++, prev | (uint32_t)(count << 2)); n_ops++; }
            count = 1;
        }
        if (A.is_local) {
            curr += ((opf == 2 || opf == 3) && prev != opf) ? -OE
                  : ((opf == 2 || opf == 3) ? -A.e : (opf == 1 ? -A.b : A.a));
            if (curr == total) break;
        }
        prev = opf;
        i = (opf == 0 || opf == 1 || opf == 2) ? i - 1 : i;
        j = (opf == 0 || opf == 1 || opf == 3) ? j - 1 : j;
    }
    if (out_of_band) {   // the full-matrix fallback walks this pair again (dispatch.hip)
        A.fb_list[atomicAdd(A.fb_count, 1u)] = tid;
        return;
    }
    put(off++, prev | (uint32_t)(count << 2));
    n_ops++;
    if (!A.is_local) {
        while (i >= 0) { const int rc = (i + 1) <= 63 ? (i + 1) : 63; put(off++, 2u | (uint32_t)(rc << 2)); n_ops++; i -= 63; }
        while (j >= 0) { const int rc = (j + 1) <= 63 ? (j + 1) : 63; put(off++, 3u | (uint32_t)(rc << 2)); n_ops++; j -= 63; }
    } else {
        if (A.tstart) A.tstart[tid] = i;
        if (A.qstart) A.qstart[tid] = j;
    }
    A.n_ops[tid] = (uint32_t)n_ops;
}

// ------------------------------------------------------- pack / revcomp ----
// gasal_pack_kernel (pack_rc_seqs.h:13-53): 8 ASCII bytes -> one word of 4-bit
// codes, first byte in bits 31:28.  Grid-stride over whole words.
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t *in, uint32_t *out, uint32_t n_words) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < n_words; w += gridDim.x * blockDim.x) {
        const uint2 v = reinterpret_cast<const uint2 *>(in)[w];
        uint32_t p = 0;
        p |= (v.x & 15u) << 28; p |= ((v.x >> 8) & 15u) << 24; p |= ((v.x >> 16) & 15u) << 20; p |= ((v.x >> 24) & 15u) << 16;
        p |= (v.y & 15u) << 12; p |= ((v.y >> 8) & 15u) << 8; p |= ((v.y >> 16) & 15u) << 4; p |= (v.y >> 24) & 15u;
        out[w] = p;
    }
}

__device__ __forceinline__ uint32_t shl_c(uint32_t x, uint32_t s) { return s >= 32 ? 0u : x << s; }
__device__ __forceinline__ uint32_t shr_c(uint32_t x, uint32_t s) { return s >= 32 ? 0u : x >> s; }
__device__ __forceinline__ uint32_t nib_rev(uint32_t x) {
    // reverse the 8 nibbles: byte-reverse then swap nibbles within bytes
    x = __builtin_bswap32(x);
    return ((x & 0x0F0F0F0Fu) << 4) | ((x >> 4) & 0x0F0F0F0Fu);
}

__device__ void rc_one(uint32_t *W, uint32_t base, uint32_t len, uint8_t op, int32_t n_code) {
    const uint32_t regs = (len + 7) >> 3;
    if (regs == 0) return;
    const uint32_t swaps = (regs >> 1) + (regs & 1);
    auto RD = [&](int64_t idx) -> uint32_t { return ((int64_t)base + idx) >= 0 ? W[(int64_t)base + idx] : 0u; };
    if (op & 1) {   // pack_rc_seqs.h:109-167 (N count is 0 for N_CODE > 15)
        uint32_t nbr = 0;
        const uint32_t last = W[base + regs - 1];
        for (int jj = 0; jj < 32; jj += 4) nbr += ((int32_t)((last >> jj) & 15u) == n_code);
        nbr <<= 2;
        const uint32_t lowmask = shl_c(1u, nbr) - 1u;
        for (uint32_t i = 0; i < swaps; i++) {
            const int64_t a = (int64_t)regs - 2 - i, b = (int64_t)regs - 1 - i;
            const uint32_t r1 = W[base + i];
            const uint32_t r2 = shl_c(RD(a), 32 - nbr) | shr_c(RD(b), nbr);
            const uint32_t rv1 = nib_rev(r1), rv2 = nib_rev(r2);
            const uint32_t q1 = shl_c(rv1, nbr) | (RD(b) & lowmask);
            const uint32_t q2 = (RD(a) & (0xFFFFFFFFu - lowmask)) | shr_c(rv1, 32 - nbr);
            W[base + i] = rv2;
            W[base + b] = q1;
            if (i != swaps - 1 && (int64_t)base + a >= 0) W[base + a] = q2;
        }
    }
    if (op & 2) {   // :169-205 complement A<->T (1<->4), C<->G (3<->7)
        for (uint32_t i = 0; i < regs; i++) {
            uint32_t rp = W[base + i], o = 0;
            for (int k = 28; k >= 0; k -= 4) {
                uint32_t nt = (rp >> k) & 15u;
                nt = nt == 1 ? 4 : nt == 3 ? 7 : nt == 4 ? 1 : nt == 7 ? 3 : nt;
                o |= nt << k;
            }
            W[base + i] = o;
        }
    }
}

__global__ __launch_bounds__(256) void revcomp_kernel(uint32_t *qw, uint32_t *tw, const uint32_t *qlen,
                                                      const uint32_t *tlen, const uint32_t *qoff,
                                                      const uint32_t *toff, const uint8_t *qop,
                                                      const uint8_t *top, uint32_t n, int32_t n_code) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= n) return;
    if (qop[tid] == 0 && top[tid] == 0) return;
    rc_one(qw, qoff[tid] >> 3, qlen[tid], qop[tid], n_code);
    rc_one(tw, toff[tid] >> 3, tlen[tid], top[tid], n_code);
}

}  // namespace gx
