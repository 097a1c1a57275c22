// nvbanded.hpp — nvbio's BatchedBandedAlignmentScore<BAND_LEN> (NvB/nvbio/alignment/
// batched.h:337, batched_banded_inl.h:44-75): one pair per thread, the band of BAND_LEN
// cells of the current pattern row in registers, as the reference's DeviceThreadScheduler
// runs it.  The row recurrences (band[j] = H(i, i + j)):
//   SW / ED   sw/sw_banded_inl.h:44-54 (row zero), :392-475 (rows), :494-510 (sinks);
//             ed/ed_banded_inl.h:63-78 (ED = SW with (0, -1, -1, -1))
//     j = 0:     max(band[1] + del, band[0] + S)               (no left)
//     0<j<B-1:   max3(band[j+1] + del, band[j-1]' + ins, band[j] + S)
//     j = B-1:   max(band[B-2]' + ins, band[B-1] + S)          (no top)
//   Gotoh     gotoh/gotoh_banded_inl.h:44-75 (row zero), :463-618 (rows), :642-659 (sinks)
//     F[j] = max(F[j+1] + Ge, H[j+1] + Go) (F[B-1] = infimum), E carried along the row
//     from E_1 = H[0]' + Go, E_{j+1} = max(H[j]' + Go, E_j + Ge); H = max3(F, E, diag)
//   LOCAL clamps at 0 and reports every cell; GLOBAL reports band[B-1] after the last
//   row; SEMI_GLOBAL band[j] for j < min(M + B - 1, N) - (M - 1).  A pair with
//   N < M is skipped (the BestSink keeps INT32_MIN).  Text symbols past N read as 255
//   (the reference's row-loop guard, sw_banded_inl.h:453).
// int32 arithmetic like the reference's; the band length is a launch argument up to the
// instance's BMAX (cells j >= band are never read: the j = band-1 cell takes the last
// cell's rule).  The pattern and text are read one packed word ahead of the symbol in use.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nvbio.hpp"
#include "nvbio16.hpp"   // pk_max3 (nv_banded16_kernel)

namespace gx {

struct NvBandArgs {
    const uint32_t *pw, *poff;      // pattern words, n + 1 symbol offsets
    uint32_t pbits, pbig;
    const uint32_t *tw, *toff;      // text words, n + 1 symbol offsets (NULL: one shared text of tlen0)
    uint32_t tbits, tbig, tlen0;
    int32_t *score;
    uint32_t n, band;
    int32_t match, mismatch, go, ge, del, ins;
};

// sequential reader of one packed string: symbol k of the string at set offset `off`,
// the word holding the next symbols loaded one word ahead
// (never past the string's last word: `len` symbols from `off`)
struct NvSymReader {
    const uint32_t *w;
    uint32_t bits, big, per, mask;
    uint64_t word, lastw;   // index of `cur`; the string's last word
    uint32_t cur, nxt, p;
    __device__ __forceinline__ void init(const uint32_t *words, uint32_t b, uint32_t be, uint64_t off, uint32_t len) {
        w = words; bits = b; big = be; per = 32u / b; mask = (1u << b) - 1u;
        word = off / per; p = (uint32_t)(off % per);
        lastw = len ? (off + len - 1) / per : word;
        cur = len ? w[word] : 0u;
        nxt = word + 1 <= lastw ? w[word + 1] : 0u;
    }
    __device__ __forceinline__ uint32_t next() {
        const uint32_t sh = big ? 32u - bits * (p + 1) : bits * p;
        const uint32_t s = (cur >> sh) & mask;
        if (++p == per) {
            p = 0; ++word; cur = nxt;
            nxt = word + 1 <= lastw ? w[word + 1] : 0u;
        }
        return s;
    }
};

template <int ALN, int TYPE, int BMAX, bool EX = false>   // EX: band length == BMAX (as nv_banded16_kernel)
__global__ __launch_bounds__(256) void nv_banded_kernel(NvBandArgs A) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= A.n) return;
    const uint32_t po = A.poff[tid], M = A.poff[tid + 1] - po;
    const bool shared = A.toff == nullptr;
    const uint32_t to = shared ? 0u : A.toff[tid], N = shared ? A.tlen0 : A.toff[tid + 1] - to;
    int32_t best = INT32_MIN;                              // BestSink (sink_inl.h:38-40, 59-68)
    const uint32_t B = EX ? (uint32_t)BMAX : A.band;
    if (N < M) { A.score[tid] = best; return; }            // gotoh_banded_inl.h:424, sw_banded_inl.h:365
    constexpr bool GOTOH = ALN == NV_GOTOH;
    const int32_t S_eq = A.match, S_ne = A.mismatch;
    const int32_t Go = A.go, Ge = A.ge, Del = A.del, Ins = A.ins;
    const int32_t infimum = -32768 - max(Go, Ge);         // gotoh_banded_inl.h:440-442
    int32_t H[BMAX], F[BMAX];
    uint32_t tc[BMAX];                                     // text symbols i + j of the current row
    NvSymReader pr, tr;
    pr.init(A.pw, A.pbits, A.pbig, po, M);
    tr.init(A.tw, A.tbits, A.tbig, to, N);
#pragma unroll
    for (int j = 0; j < BMAX; ++j) {
        if (GOTOH) H[j] = j == 0 ? 0 : (TYPE == NV_GLOBAL ? Go + (j - 1) * Ge : 0);
        else H[j] = TYPE == NV_GLOBAL ? j * Del : 0;
        F[j] = infimum;
        tc[j] = 255u;
    }
    uint32_t tnext = 0;                                    // text symbols read so far
#pragma unroll
    for (int j = 0; j < BMAX - 1; ++j)
        if ((uint32_t)j + 1 < B) { tc[j] = tnext < N ? tr.next() : 255u; ++tnext; }
    for (uint32_t i = 0; i < M; ++i) {
        const uint32_t q = pr.next();
        // the band's last cell reads text symbol i + B - 1 (255 past N)
        const uint32_t g_last = tnext < N ? tr.next() : 255u;
        ++tnext;
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j + 1 == B) tc[j] = g_last;
        int32_t E = 0, hprev = 0;
#pragma unroll
        for (int j = 0; j < BMAX; ++j) {
            if ((uint32_t)j >= B) break;
            const bool last = (uint32_t)j + 1 == B;
            const int32_t diag = H[j] + (tc[j] == q ? S_eq : S_ne);
            int32_t hi;
            if (GOTOH) {
                if (!last) F[j] = max(F[j + (j + 1 < BMAX ? 1 : 0)] + Ge, H[j + (j + 1 < BMAX ? 1 : 0)] + Go);
                else F[j] = infimum;
                hi = j == 0 ? max(F[0], diag) : last ? max(E, diag) : max(max(F[j], E), diag);
            } else {
                const int32_t top = last ? INT32_MIN / 2 : H[j + (j + 1 < BMAX ? 1 : 0)] + Del;
                hi = j == 0 ? max(top, diag) : max(max(top, hprev + Ins), diag);
            }
            if (TYPE == NV_LOCAL) { hi = max(hi, 0); best = max(best, hi); }
            H[j] = hi;
            hprev = hi;
            if (GOTOH) E = j == 0 ? hi + Go : max(hi + Go, E + Ge);
        }
        // shift the text window: row i + 1 reads symbols i + 1 + j
#pragma unroll
        for (int j = 0; j + 1 < BMAX; ++j)
            if ((uint32_t)j + 1 < B) tc[j] = tc[j + 1];
    }
    if (TYPE == NV_GLOBAL) {
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j + 1 == B) best = max(best, H[j]);
    } else if (TYPE == NV_SEMI) {
        const uint32_t m = min(M + B - 1, N) - (M - 1);
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j < B && (uint32_t)j < max(m, 1u)) best = max(best, H[j]);
    }
    A.score[tid] = best;
}


// ---------------------------------------------------------------------------
// Two pairs per lane in 16-bit halves (nv_banded16_kernel): slots 2t and 2t + 1 of the
// batch share a lane, the band registers hold both pairs' cells (low / high half), the
// arithmetic is nvbio16.hpp's: stored value = value + base inside the positive normal
// f16 range, so v_pk_maximum3_f16 is an exact 3-way max of both pairs and 32-bit adds
// never carry across halves; -inf is NEG = 0x0400, LOCAL floors E and F at 0 (exact
// for H: gaps never score > 0).  Substitution: per row a 4-byte table per half,
// byte t = [t == pattern symbol]·(match − mismatch) (symbols >= 4 select none), and a
// per-band-slot selector {tA, 0x0C, 4 + tB, 0x0C} of the two texts' 2-bit symbols (past
// a text's end: 0x0C, the constant 0, a mismatch as nvbio's 255); tmp = H + byte +
// mismatch is one v_add3.  The halves may differ in length: the row loop runs to the
// longer pattern and each half's sinks are taken at its own last row.
// 2-bit texts, gap scores <= 0, match - mismatch <= 255 and the value window are the
// host's conditions (batched.hip nvb16_ok); otherwise nv_banded_kernel runs.
// ---------------------------------------------------------------------------
struct NvBand16Args {
    const uint32_t *pw, *poff;      // pattern words, n + 1 symbol offsets
    uint32_t pbits, pbig;
    const uint32_t *tw, *toff;      // 2-bit text words, n + 1 offsets (NULL: one shared text of tlen0)
    uint32_t tbig, tlen0;
    int32_t *score;
    uint32_t n, n_lanes, band;
    int32_t match, mismatch, go, ge, del, ins;
    uint32_t base;                  // stored value of 0
};

// EX: the band length is BMAX itself (nvbio's BAND_LEN is a template argument; 8, 16 and
// 32 get their own code), so the band-slot tests fold at compile time
template <int ALN, int TYPE, int BMAX, bool EX = false>
__global__ __launch_bounds__(256) void nv_banded16_kernel(NvBand16Args A) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= A.n_lanes) return;
    constexpr bool GOTOH = ALN == NV_GOTOH;
    const bool shared = A.toff == nullptr;
    uint32_t M[2], N[2], po[2], to[2];
    bool valid[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t pr = 2 * lane + h;
        valid[h] = pr < A.n;
        const uint32_t pp = valid[h] ? pr : 2 * lane;
        po[h] = A.poff[pp]; M[h] = A.poff[pp + 1] - po[h];
        to[h] = shared ? 0u : A.toff[pp];
        N[h] = shared ? A.tlen0 : A.toff[pp + 1] - to[h];
    }
    const uint32_t Bn = EX ? (uint32_t)BMAX : A.band;
    const int32_t Bs = (int32_t)A.base;
    const uint32_t BB = A.base * 0x10001u, NEG = 0x04000400u;
    const uint32_t FLOOR = TYPE == NV_LOCAL ? BB : NEG;
    const uint32_t MIS = (uint32_t)A.mismatch * 0x10001u;
    const uint32_t GO = (uint32_t)(-A.go) * 0x10001u, GE = (uint32_t)(-A.ge) * 0x10001u;   // gaps <= 0
    const uint32_t DEL = (uint32_t)(-A.del) * 0x10001u, INS = (uint32_t)(-A.ins) * 0x10001u;
    const uint32_t dm = (uint32_t)(A.match - A.mismatch);
    uint32_t H[BMAX], F[BMAX], sel[BMAX];
    NvSymReader tr[2], prd[2];
    uint32_t tnext[2] = {0u, 0u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        prd[h].init(A.pw, A.pbits, A.pbig, po[h], M[h]);
        tr[h].init(A.tw, 2u, A.tbig, to[h], N[h]);
    }
    // text selector of the next symbol of each half: 2-bit code (high half + 4), or 0x0C past the end
    auto next_sel = [&]() {
        uint32_t sa = 0x0Cu, sb = 0x0Cu;
        if (tnext[0] < N[0]) sa = tr[0].next();
        if (tnext[1] < N[1]) sb = tr[1].next() + 4u;
        ++tnext[0]; ++tnext[1];
        return sa | 0x0C00u | (sb << 16) | 0x0C000000u;
    };
#pragma unroll
    for (int j = 0; j < BMAX; ++j) {
        int32_t v;
        if (GOTOH) v = j == 0 ? 0 : (TYPE == NV_GLOBAL ? A.go + (j - 1) * A.ge : 0);
        else v = TYPE == NV_GLOBAL ? j * A.del : 0;
        H[j] = (uint32_t)(v + Bs) * 0x10001u;
        F[j] = FLOOR;
        sel[j] = 0x0C0C0C0Cu;
    }
#pragma unroll
    for (int j = 0; j < BMAX - 1; ++j)
        if ((uint32_t)j + 1 < Bn) sel[j] = next_sel();
    // per-half sinks: taken at the half's last row (M == 0: from the row-zero band)
    uint32_t out[2] = {0u, 0u};
    bool have[2] = {false, false};
    uint32_t best = FLOOR;
    auto take = [&](int h) {
        uint32_t v = 0;
        if (TYPE == NV_GLOBAL) {
#pragma unroll
            for (int j = 0; j < BMAX; ++j)
                if ((uint32_t)j + 1 == Bn) v = H[j];
        } else if (TYPE == NV_SEMI) {
            const uint32_t m = min(M[h] + Bn - 1, N[h]) - (M[h] - 1);   // uint32 as the reference
            v = H[0];
#pragma unroll
            for (int j = 1; j < BMAX; ++j)
                if ((uint32_t)j < Bn && (uint32_t)j < m) v = pk_max3(v, H[j], v);
        } else {
            v = best;
        }
        out[h] = v;
        have[h] = true;
    };
#pragma unroll
    for (int h = 0; h < 2; ++h)
        if (M[h] == 0 && TYPE != NV_LOCAL) take(h);
    const uint32_t Mmax = max(M[0], M[1]);
    for (uint32_t i = 0; i < Mmax; ++i) {
        // this row's tables: TA (low half, v_perm's second source), TB (high half, first source)
        const uint32_t qa = i < M[0] ? prd[0].next() : 4u, qb = i < M[1] ? prd[1].next() : 4u;
        const uint32_t TA = qa < 4 ? dm << (8 * qa) : 0u, TB = qb < 4 ? dm << (8 * qb) : 0u;
        // the band's last slot reads text symbol i + B - 1
        const uint32_t snew = next_sel();
#pragma unroll
        for (int j = 0; j < BMAX; ++j)
            if ((uint32_t)j + 1 == Bn) sel[j] = snew;
        uint32_t E = 0, hprev = 0;
#pragma unroll
        for (int j = 0; j < BMAX; ++j) {
            if ((uint32_t)j >= Bn) break;
            const bool last = (uint32_t)j + 1 == Bn;
            const int jn = j + 1 < BMAX ? j + 1 : j;
            const uint32_t tmp = H[j] + __builtin_amdgcn_perm(TB, TA, sel[j]) + MIS;   // H(i-1, i+j-1) + S
            uint32_t hi;
            if (GOTOH) {
                F[j] = last ? NEG : pk_max3(F[jn] - GE, H[jn] - GO, FLOOR);
                if (j == 0) hi = pk_max3(F[0], tmp, TYPE == NV_LOCAL ? BB : tmp);
                else if (last) hi = pk_max3(E, tmp, TYPE == NV_LOCAL ? BB : tmp);
                else hi = pk_max3(F[j], E, tmp);
                E = j == 0 ? (TYPE == NV_LOCAL ? pk_max3(hi - GO, BB, BB) : hi - GO) : pk_max3(hi - GO, E - GE, FLOOR);
            } else {
                if (j == 0) hi = pk_max3(H[jn] - DEL, tmp, tmp);
                else if (last) hi = pk_max3(hprev - INS, tmp, tmp);
                else hi = pk_max3(H[jn] - DEL, hprev - INS, tmp);
                if (TYPE == NV_LOCAL) hi = pk_max3(hi, BB, BB);
            }
            if (TYPE == NV_LOCAL) best = pk_max3(best, hi, best);
            H[j] = hi;
            hprev = hi;
        }
        // shift the selector window: row i + 1 reads text i + 1 + j
#pragma unroll
        for (int j = 0; j + 1 < BMAX; ++j)
            if ((uint32_t)j + 1 < Bn) sel[j] = sel[j + 1];
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (i + 1 == M[h]) take(h);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (!valid[h]) continue;
        int32_t v = INT32_MIN;                                       // BestSink: nothing reported
        if (N[h] >= M[h] && have[h]) v = (int32_t)((out[h] >> (16 * h)) & 0xFFFFu) - Bs;
        A.score[2 * lane + h] = v;
    }
}

}  // namespace gx
