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

template <int ALN, int TYPE, int BMAX>
__global__ __launch_bounds__(256) void nv_banded_kernel(NvBandArgs A) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= A.n) return;
    const uint32_t po = A.poff[tid], M = A.poff[tid + 1] - po;
    const bool shared = A.toff == nullptr;
    const uint32_t to = shared ? 0u : A.toff[tid], N = shared ? A.tlen0 : A.toff[tid + 1] - to;
    int32_t best = INT32_MIN;                              // BestSink (sink_inl.h:38-40, 59-68)
    const uint32_t B = A.band;
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

}  // namespace gx
