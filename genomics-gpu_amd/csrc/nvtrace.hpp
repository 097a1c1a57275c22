// nvtrace.hpp — nvbio's BatchedAlignmentTraceback (NvB/nvbio/alignment/batched.h:436,
// batched_inl.h:612-664) on MI355X: the full-DP traceback of the Gotoh and Smith-Waterman
// aligners, GLOBAL / LOCAL / SEMI_GLOBAL, one pair per thread.
//
// The reference runs one thread per job too: a checkpointed scoring pass that keeps the
// BestSink, then, checkpoint by checkpoint from the sink backwards, a recomputation of the
// submatrix's direction vectors and the walk through it (alignment_inl.h:365-465).  The
// checkpoints only bound the reference's storage; the values and flags of every cell are those of
// one full pass, so here each thread runs that pass once, storing its flags, then walks:
//   * recurrences and flags: gotoh/gotoh_inl.h:462-593 (PatternBlockingTag update_row: rows i =
//     text, columns j = pattern; F from the row above = DELETION, E from the left = INSERTION;
//     hdir = top > left ? (top > diag ? DEL : SUB) : (left > diag ? INS : SUB); extension bits on a
//     strictly greater extension; LOCAL: H == 0 -> SINK, :441-442) and sw/sw_inl.h:420-540, 380-400;
//   * boundaries: gotoh_inl.h:695 and the checkpoint context's init (:247-300), sw_inl.h:660-663,
//     243-251;
//   * the sink: BestSink keeps the last maximum in report order (stripes of 8 pattern columns,
//     then rows, then columns) for LOCAL; SEMI_GLOBAL reports H(i, M-1) per row, GLOBAL H(N-1, M-1)
//     (utils_inl.h:273-300);
//   * the walk: gotoh_inl.h:1806-1872 (H / E / F states), sw_inl.h:1653-1709, then the first row /
//     column of alignment_inl.h:442-459.
// Flags are one byte per cell, 8 cells of a row and stripe per store, interleaved across the
// launch's threads ([row][stripe][pair]: a wave's stores are contiguous).  The CPU restatement is
// oracle/nvbio_oracle.c orc_nv_traceback_one, pinned by nvbio-test's alignment_test.cu:778-792.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nvbanded.hpp"   // NvSymReader

namespace gx {

struct NvTbArgs {
    const uint32_t *pw, *poff;
    uint32_t pbits, pbig;
    const uint32_t *tw, *toff;
    uint32_t tlen0, tbits, tbig;
    int32_t match, mismatch, go, ge, del, ins;
    uint32_t n, max_m, max_n;
    uint8_t *dir;          // [text row][stripe of 8 pattern columns][n] x 8 bytes
    int32_t *row;          // [text row][n] int2: (H, E) of the previous stripe's last column
    int32_t *score;
    uint32_t *src, *snk;   // [2n] each: (x = text, y = pattern)
    uint8_t *ops;          // pair k's pushes at ops + k * ops_stride (push order)
    uint32_t ops_stride;
    uint32_t *n_ops;
};

__device__ __forceinline__ uint32_t nvtb_symbol(const uint32_t *w, uint32_t bits, uint32_t big, uint32_t s) {
    const uint32_t per = 32u / bits, p = s % per;
    const uint32_t sh = big ? 32u - bits * (p + 1u) : bits * p;
    return (w[s / per] >> sh) & (bits == 32u ? 0xFFFFFFFFu : ((1u << bits) - 1u));
}

// The walk's pushes into a pair's output (ops + k * ops_stride, push order): single bytes until the
// output reaches a 4-byte boundary, then one 32-bit store per 4 pushes.  A wave's byte stores each
// touch 64 different lines; this issues a quarter of them (band 7: 0.67 -> 0.41 ms per 262 K pairs,
// profiles/r05/nvbtb/).
struct NvPushes {
    uint8_t *out;
    uint32_t a0, head, acc, cnt;
    __device__ __forceinline__ explicit NvPushes(uint8_t *o)
        : out(o), a0((uint32_t)(reinterpret_cast<uintptr_t>(o) & 3u)), head(0), acc(0), cnt(0) {
        head = (4u - a0) & 3u;
    }
    __device__ __forceinline__ void push(uint32_t op) {
        const uint32_t a = (a0 + cnt) & 3u;
        if (cnt < head) {
            out[cnt] = (uint8_t)op;
        } else {
            acc |= op << (8u * a);
            if (a == 3u) { *reinterpret_cast<uint32_t *>(out + cnt - 3) = acc; acc = 0; }
        }
        ++cnt;
    }
    __device__ __forceinline__ void flush() {   // the pushes of the last, partial word
        if (cnt > head)
            for (uint32_t i = cnt - ((a0 + cnt) & 3u); i < cnt; ++i) out[i] = (uint8_t)(acc >> (8u * ((a0 + i) & 3u)));
    }
};

// TYPE: 0 GLOBAL, 1 LOCAL, 2 SEMI_GLOBAL (nvbio AlignmentType).  The pass runs in stripes of 8
// pattern columns, as the reference's PatternBlockingTag does: a stripe's H and F across its 8
// columns stay in registers, the (H, E) of its last column goes to the next stripe through one
// int2 per text row ([row][pair], A.row), and the 8 cells' flags of a row are one 8-byte store
// ([row][stripe][pair] uint2, A.dir) -- 3 bytes of memory traffic per cell instead of the 17 of
// a row-by-row pass that kept whole DP rows in memory.
template <bool GOTOH, int TYPE>
__global__ __launch_bounds__(256) void nv_traceback_kernel(NvTbArgs A) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.n) return;
    constexpr uint8_t SUB = 0, INS = 1, DEL = 2, SNK = 3, INS_EXT = 4, DEL_EXT = 8;
    constexpr uint32_t BAND = 8;   // gotoh_bandlen_selector / the SW stripes (and the LOCAL report order)
    const uint32_t p0 = A.poff[k], M = A.poff[k + 1] - p0;
    const uint32_t t0 = A.toff ? A.toff[k] : 0u, N = A.toff ? A.toff[k + 1] - t0 : A.tlen0;
    const uint32_t n = A.n;
    uint32_t *src = A.src + 2 * (size_t)k, *snk = A.snk + 2 * (size_t)k;
    A.n_ops[k] = 0;
    if (M == 0 || N == 0 || M > A.max_m || N > A.max_n || M + N > A.ops_stride) {
        src[0] = src[1] = snk[0] = snk[1] = 0xFFFFFFFFu;
        A.score[k] = INT32_MIN;
        return;
    }
    const int32_t Go = A.go, Ge = A.ge;
    const int32_t infimum = -32768 - (Go < Ge ? Go : Ge);
    const uint32_t stripes = (A.max_m + BAND - 1) / BAND;
    int2 *temp = reinterpret_cast<int2 *>(A.row) + k;   // [row][pair]
    uint2 *dir8 = reinterpret_cast<uint2 *>(A.dir);       // [row][stripe][pair]
    for (uint32_t i = 0; i < N; i++)   // the first column's left neighbours (the checkpoint context's init)
        temp[(size_t)i * n] = make_int2(TYPE == 0 ? (GOTOH ? Go + Ge * (int32_t)i : A.del * (int32_t)(i + 1)) : 0,
                                        TYPE == 1 ? 0 : infimum);
    int32_t best = INT32_MIN;
    uint32_t bx = 0xFFFFFFFFu, by = 0xFFFFFFFFu;
    int32_t last_h = 0;   // H(i, M-1) of the stripe holding column M-1
    for (uint32_t blk = 0; blk * BAND < M; blk++) {
        const uint32_t c0 = blk * BAND;
        uint32_t q[BAND];
        int32_t Hb[BAND + 1], Fb[BAND + 1];
#pragma unroll
        for (uint32_t j = 0; j < BAND; j++) q[j] = c0 + j < M ? nvtb_symbol(A.pw, A.pbits, A.pbig, p0 + c0 + j) : 0xFFFFu;
#pragma unroll
        for (uint32_t j = 0; j <= BAND; j++) {   // row -1: H(-1, c0 + j - 1)
            const int32_t cc = (int32_t)(c0 + j) - 1;
            Hb[j] = TYPE == 1 || cc < 0 ? 0 : GOTOH ? Go + Ge * cc : A.ins * (cc + 1);
            Fb[j] = infimum;
        }
        int32_t diag0 = Hb[0];
        for (uint32_t i = 0; i < N; i++) {
            const uint32_t r = nvtb_symbol(A.tw, A.tbits, A.tbig, t0 + i);
            const int2 tv = temp[(size_t)i * n];
            int32_t diagH = diag0;     // H(i-1, c0-1)
            diag0 = tv.x;
            Hb[0] = tv.x;              // H(i, c0-1)
            int32_t E = tv.y;          // E(i, c0-1)
            uint32_t flo = 0, fhi = 0;
#pragma unroll
            for (uint32_t j = 1; j <= BAND; j++) {
                const int32_t S = r == q[j - 1] ? A.match : A.mismatch;
                const int32_t up = Hb[j];
                const int32_t diag = diagH + S;
                int32_t h;
                uint32_t d;
                if constexpr (GOTOH) {
                    const int32_t ftop = Fb[j] + Ge, htop = up + Go;
                    const int32_t F = max(ftop, htop);
                    const uint32_t fdir = ftop > htop ? DEL_EXT : SUB;
                    const int32_t eleft = E + Ge, hleft = Hb[j - 1] + Go;
                    E = max(eleft, hleft);
                    const uint32_t edir = eleft > hleft ? INS_EXT : SUB;
                    Fb[j] = F;
                    h = max(max(E, F), diag);
                    if (TYPE == 1) h = max(h, 0);
                    const uint32_t hdir = F > E ? (F > diag ? DEL : SUB) : (E > diag ? INS : SUB);
                    d = (TYPE == 1 && h == 0 ? SNK : hdir) | edir | fdir;
                } else {
                    const int32_t top = up + A.del, lft = Hb[j - 1] + A.ins;
                    h = max(max(top, lft), diag);
                    if (TYPE == 1) h = max(h, 0);
                    const uint32_t hdir = top > lft ? (top > diag ? DEL : SUB) : (lft > diag ? INS : SUB);
                    d = TYPE == 1 && h == 0 ? SNK : hdir;
                }
                diagH = up;
                Hb[j] = h;
                if (j <= 4) flo |= d << (8 * (j - 1)); else fhi |= d << (8 * (j - 5));
                if (TYPE == 1 && c0 + j <= M && best <= h) {   // report order: stripe, row, column; the last maximum wins
                    best = h; bx = i + 1; by = c0 + j;
                }
                if (c0 + j == M) last_h = h;
            }
            dir8[((size_t)i * stripes + blk) * n + k] = make_uint2(flo, fhi);
            temp[(size_t)i * n] = make_int2(Hb[BAND], E);
            if (TYPE == 2 && c0 + BAND >= M && best <= last_h) { best = last_h; bx = i + 1; by = M; }
        }
    }
    if (TYPE == 0) { best = last_h; bx = N; by = M; }
    snk[0] = bx; snk[1] = by;
    const uint8_t *dir = A.dir;
    auto dcell = [&](uint32_t i, uint32_t j) -> uint8_t {
        return dir[(((size_t)i * stripes + j / BAND) * n + k) * 8 + (j % BAND)];
    };
    NvPushes out(A.ops + (size_t)k * A.ops_stride);
    int32_t row = (int32_t)bx, col = (int32_t)by - 1;
    int state = 0;   // H / E / F
    while (row > 0 && col >= 0) {
        const uint8_t op = dcell((uint32_t)(row - 1), (uint32_t)col);
        if constexpr (GOTOH) {
            const uint8_t h_op = op & 3u;
            if (TYPE == 1 && state == 0 && h_op == SNK) break;
            if (state == 1) {
                if ((op & INS_EXT) == 0) state = 0;
                --col; out.push(INS);
            } else if (state == 2) {
                if ((op & DEL_EXT) == 0) state = 0;
                --row; out.push(DEL);
            } else if (h_op == INS) {
                state = 1;
            } else if (h_op == DEL) {
                state = 2;
            } else {
                --col; --row; out.push(SUB);
            }
        } else {
            if (TYPE == 1 && op == SNK) break;
            if (op != DEL) --col;
            if (op != INS) --row;
            out.push(op);
        }
    }
    uint32_t sx = (uint32_t)row, sy = (uint32_t)(col + 1);
    if (TYPE != 1 && sx == 0)
        for (; sy > 0; --sy) out.push(INS);
    if (TYPE == 0 && sy == 0)
        for (; sx > 0; --sx) out.push(DEL);
    out.flush();
    src[0] = sx; src[1] = sy;
    A.n_ops[k] = out.cnt;
    A.score[k] = best;
}

// nvbio's BatchedBandedAlignmentTraceback<BAND_LEN, CHECKPOINTS> (batched.h:464,
// batched_banded_inl.h:248-297, banded_inl.h:352-427): one pair per thread, the band of B cells
// of the current pattern row in registers as in nv_banded_kernel (rows i = pattern symbols,
// entry j = text symbol i + j).  The reference scores with checkpoints, then recomputes each
// CHECKPOINTS-row window of flags and walks it; the flags are those of one pass, so the pass
// runs once and stores them (one byte per cell, 4 cells per word, [row][word][pair]: a wave's
// stores are contiguous), then the thread walks them:
//   * cells and flags: gotoh/gotoh_banded_inl.h:482-614, :323-339 (top = F = INSERTION, left =
//     E = DELETION; j = 0 has no E, j = B-1 no F; the E flag of cell j is cell j-1's update;
//     LOCAL and H == 0 -> SINK) and sw/sw_banded_inl.h:392-475, :268-279 (top + deletion, left +
//     insertion; the SW flags never hold SINK);
//   * the sink: LOCAL every cell in row-then-entry order, SEMI_GLOBAL the last row's entries
//     j < min(M + B - 1, N) - (M - 1), GLOBAL entry B-1; the last maximum wins;
//   * the walk: gotoh_banded_inl.h:895-962, sw_banded_inl.h:740-798.
// The CPU restatement is oracle/nvbio_oracle.c orc_nv_banded_traceback_one, pinned by
// alignment_test.cu:790-793 and :796-826 (4M1D3M with band 7, 147M2D3M with band 31).
struct NvBandTbArgs {
    const uint32_t *pw, *poff;
    uint32_t pbits, pbig;
    const uint32_t *tw, *toff;
    uint32_t tbits, tbig, tlen0;
    int32_t match, mismatch, go, ge, del, ins;
    uint32_t n, band, words, max_m;   // words = (band + 3) / 4 flag words per row
    uint32_t *dir;                     // [pattern row][word][n]
    int32_t *score;
    uint32_t *src, *snk;
    uint8_t *ops;
    uint32_t ops_stride;
    uint32_t *n_ops;
};

// EX: the band length is BMAX itself (nvBowtie's BAND_LEN 7 / 15 / 31 get their own code, as
// nvbio's template argument does), so the per-cell band tests fold at compile time
template <bool GOTOH, int TYPE, int BMAX, bool EX = false>
__global__ __launch_bounds__(256) void nv_banded_traceback_kernel(NvBandTbArgs A) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.n) return;
    constexpr uint32_t SUB = 0, INS = 1, DEL = 2, SNK = 3, INS_EXT = 4, DEL_EXT = 8;
    const uint32_t po = A.poff[k], M = A.poff[k + 1] - po;
    const bool shared = A.toff == nullptr;
    const uint32_t to = shared ? 0u : A.toff[k], N = shared ? A.tlen0 : A.toff[k + 1] - to;
    const uint32_t B = EX ? (uint32_t)BMAX : A.band, n = A.n;
    const uint32_t words = EX ? (uint32_t)(BMAX + 3) / 4 : A.words;
    uint32_t *src = A.src + 2 * (size_t)k, *snk = A.snk + 2 * (size_t)k;
    src[0] = src[1] = snk[0] = snk[1] = 0xFFFFFFFFu;
    A.n_ops[k] = 0;
    if (N < M || M > A.max_m || 2 * M + B > A.ops_stride) { A.score[k] = INT32_MIN; return; }
    const int32_t S_eq = A.match, S_ne = A.mismatch, Go = A.go, Ge = A.ge, Del = A.del, Ins = A.ins;
    const int32_t infimum = -32768 - max(Go, Ge);   // gotoh_banded_inl.h:446-448
    int32_t H[BMAX], F[BMAX];
    uint32_t tc[BMAX];
    NvSymReader pr, tr;
    pr.init(A.pw, A.pbits, A.pbig, po, M);
    tr.init(A.tw, A.tbits, A.tbig, to, N);
#pragma unroll
    for (int j = 0; j < BMAX; ++j) {
        if (GOTOH) H[j] = j == 0 ? 0 : (TYPE == 0 ? Go + (j - 1) * Ge : 0);
        else H[j] = TYPE == 0 ? j * Del : 0;
        F[j] = infimum;
        tc[j] = 255u;
    }
    uint32_t tnext = 0;
#pragma unroll
    for (int j = 0; j < BMAX - 1; ++j)
        if ((uint32_t)j + 1 < B) { tc[j] = tnext < N ? tr.next() : 255u; ++tnext; }
    int32_t best = INT32_MIN;
    uint32_t bx = 0xFFFFFFFFu, by = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < M; ++i) {
        const uint32_t q = pr.next();
        const uint32_t g_last = tnext < N ? tr.next() : 255u;
        ++tnext;
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j + 1 == B) tc[j] = g_last;
        int32_t E = 0, hprev = 0;
        uint32_t edir = SUB;
        uint32_t fw[(BMAX + 3) / 4];
#pragma unroll
        for (int w = 0; w < (BMAX + 3) / 4; ++w) fw[w] = 0;
#pragma unroll
        for (int j = 0; j < BMAX; ++j) {
            if ((uint32_t)j >= B) continue;   // (not break: the loop must unroll fully)
            const bool last = (uint32_t)j + 1 == B;
            const int jn = j + 1 < BMAX ? j + 1 : j;
            const int32_t diag = H[j] + (tc[j] == q ? S_eq : S_ne);
            int32_t hi;
            uint32_t d;
            if (GOTOH) {
                uint32_t fdir = SUB;
                if (!last) {
                    const int32_t ftop = F[jn] + Ge, htop = H[jn] + Go;
                    F[j] = max(ftop, htop);
                    fdir = ftop > htop ? DEL_EXT : SUB;
                } else {
                    F[j] = infimum;
                }
                uint32_t hdir;
                if (j == 0) { hi = max(F[0], diag); hdir = F[0] > diag ? INS : SUB; }
                else if (!last) { hi = max(max(F[j], E), diag); hdir = F[j] > E ? (F[j] > diag ? INS : SUB) : (E > diag ? DEL : SUB); }
                else { hi = max(E, diag); hdir = E > diag ? DEL : SUB; }
                if (TYPE == 1) {
                    hi = max(hi, 0);
                    if (hi == 0) hdir = SNK;
                    if (best <= hi) { best = hi; bx = i + j + 1; by = i + 1; }
                }
                d = hdir | (j == 0 ? SUB : edir) | fdir;
                H[j] = hi;
                if (j == 0) { E = hi + Go; edir = SUB; }
                else {
                    const int32_t eleft = E + Ge, ediag = hi + Go;
                    edir = eleft > ediag ? INS_EXT : SUB;
                    E = max(ediag, eleft);
                }
            } else {
                const int32_t top = H[jn] + Del, left = hprev + Ins;
                if (j == 0) { hi = max(top, diag); d = top > diag ? INS : SUB; }
                else if (!last) { hi = max(max(top, left), diag); d = top > left ? (top > diag ? INS : SUB) : (left > diag ? DEL : SUB); }
                else { hi = max(left, diag); d = left > diag ? DEL : SUB; }
                if (TYPE == 1) {
                    hi = max(hi, 0);
                    if (best <= hi) { best = hi; bx = i + j + 1; by = i + 1; }
                }
                H[j] = hi;
                hprev = hi;
            }
            fw[j / 4] |= d << (8 * (j % 4));
        }
#pragma unroll
        for (int w = 0; w < (BMAX + 3) / 4; ++w)
            if ((uint32_t)w < words) A.dir[((size_t)i * words + w) * n + k] = fw[w];
#pragma unroll
        for (int j = 0; j + 1 < BMAX; ++j)
            if ((uint32_t)j + 1 < B) tc[j] = tc[j + 1];
    }
    if (TYPE == 0) {
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j + 1 == B && best <= H[j]) { best = H[j]; bx = M + B - 1; by = M; }
    } else if (TYPE == 2) {
        const uint32_t m = min(M + B - 1, N) - (M - 1u);
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j < B && (j == 0 || (uint32_t)j < m) && best <= H[j]) { best = H[j]; bx = M + j; by = M; }
    }
    A.score[k] = best;
    snk[0] = bx; snk[1] = by;
    if (bx == 0xFFFFFFFFu || by == 0xFFFFFFFFu) return;
    // The walk reads its flags P rows at a time: when any lane of the wave steps above the rows it
    // holds, every active lane loads the P rows ending at its own row (P x words independent loads,
    // one memory latency), so the wave waits on memory about once per P rows instead of once per
    // step; the step's byte is picked from the held rows by selects.
    constexpr int P = 8, WW = (BMAX + 3) / 4;
    uint32_t held[P][WW];
    NvPushes out(A.ops + (size_t)k * A.ops_stride);
    int32_t e = (int32_t)(bx - by), row = (int32_t)by - 1;
    int32_t base = 0x7FFFFFFF;   // rows [base, base + P) held (none yet)
    int state = 0;   // H / E / F
    bool found = false;
    while (row >= 0) {
        if (__any(row < base)) {
            base = max(row - (P - 1), 0);
#pragma unroll
            for (int p = 0; p < P; ++p)
#pragma unroll
                for (int w = 0; w < WW; ++w)
                    if ((uint32_t)w < words)
                        held[p][w] = base + p <= row ? A.dir[((size_t)(base + p) * words + w) * n + k] : 0u;
        }
        const int32_t rr = row - base;
        uint32_t rowv[WW];
#pragma unroll
        for (int w = 0; w < WW; ++w) {
            rowv[w] = held[0][w];
#pragma unroll
            for (int p = 1; p < P; ++p) rowv[w] = rr == p ? held[p][w] : rowv[w];
        }
        const uint32_t wi = (uint32_t)e >> 2;
        uint32_t word = rowv[0];
#pragma unroll
        for (int w = 1; w < WW; ++w) word = wi == (uint32_t)w ? rowv[w] : word;
        const uint8_t op = (uint8_t)(word >> (8u * ((uint32_t)e & 3u)));
        if constexpr (GOTOH) {
            const uint8_t h_op = op & 3u;
            if (TYPE == 1 && state == 0 && h_op == SNK) { found = true; break; }
            if (state == 1) {
                if ((op & INS_EXT) == 0) state = 0;
                --e; out.push(DEL);
            } else if (state == 2) {
                if ((op & DEL_EXT) == 0) state = 0;
                ++e; --row; out.push(INS);
            } else if (h_op == DEL) {
                state = 1;
            } else if (h_op == INS) {
                state = 2;
            } else {
                --row; out.push(SUB);
            }
        } else {
            if (op == DEL) { --e; out.push(DEL); }
            else if (op == INS) { ++e; --row; out.push(INS); }
            else { --row; out.push(SUB); }
        }
    }
    out.flush();
    const uint32_t sy = found ? (uint32_t)row + 1 : 0u;
    src[0] = (uint32_t)e + sy; src[1] = sy;
    A.n_ops[k] = out.cnt;
}

}  // namespace gx
