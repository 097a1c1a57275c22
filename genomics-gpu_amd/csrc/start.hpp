// start.hpp — LOCAL WITH_START on the wavefront kernels.
//
// The reference finds the start of a local alignment with a second, reversed
// pass (Non-CDP/GASAL2/src/kernels/local_kernel_template.h:441-511): from the
// 8-base words holding the end cell (rend_reg = min((q_end>>3)+1, qregs), same
// for the target), it walks the query and target words backwards (each word's
// 8 bases backwards too) with the forward cell update, boundaries 0, and stops
// at the first cell — in its strip-major order over the reversed matrix —
// whose H reaches the forward score.  That cell's row is the query start; the
// target start is recorded as gidx + (m-1) while the column actually runs
// gidx - (m-1).
//
// The reversed rectangle contains the forward optimum and is a sub-problem of
// the forward one, so its maximum is the forward score, and "first cell
// reaching it" is the first strict maximum in strip-major order: exactly what
// the forward LOCAL wavefront kernel reports (its Q1 tie-break).  So the
// reverse pass is the same kernel run on materialised reversed sequences:
//   rev_prep_kernel   reversed target = target words gend_reg-1 .. 0, each
//                     word's bytes (or nibbles) reversed, length 8*gend_reg:
//                     the pad columns of the last word stay (they are N
//                     columns the reference scores, and they keep the 8-column
//                     strips aligned as the reference's reversed strips are).
//                     Reversed query = query positions Lq-1 .. 0, where Lq is
//                     8*rend_reg less the run of N codes at its end that lies at
//                     positions >= ql (the pads; after a reverse-complement
//                     pre-op the pad region can hold real bases, which stay):
//                     the reference's leading N rows are dropped.  They hold
//                     H = 0 (every path into them starts at the 0 boundary and
//                     scores N as 0 or -N_PENALTY) and only
//                     turn the E/F entering the first real row from 0 into
//                     negative values, which can never win against the 0 clamp
//                     nor feed a later positive E/F; row order inside a strip is
//                     unchanged, so the tie-break order is too.  The packed
//                     kernel needs real query rows to be A/C/G/T, which this
//                     keeps.  One slot of pad8(max) bytes per pair, so
//                     one-to-many offsets need no care.
//   rev_hist/rev_scan/rev_scatter  counting sort of the pairs by reversed
//                     target words, longest first: a wave's step count is set by
//                     its longest target, so slot i holds pair perm[i] and waves
//                     see similar lengths (unrelated pairs end early in the
//                     target and their reversed rectangles are short)
//   wavefront LOCAL   on (reversed query, reversed target), slot order
//   start_map_kernel  reversed end (r', c') -> q_start = Lq-1-r',
//                     t_start = 8*gend_reg-1-8*(c'>>3) + (c'&7)  (Q8);
//                     a forward score of 0 never enters the loop: (0, 0)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gx {

struct RevArgs {
    const uint8_t *q, *t;               // input batch (unpacked bytes or packed words)
    const uint32_t *qoff, *toff, *qlen, *tlen;
    const int32_t *qend, *tend;         // forward ends
    uint8_t *rq, *rt;                   // reversed slots: slot i at i*q8 / i*t8
    uint32_t *rqoff, *rtoff, *rqlen, *rtlen;
    uint32_t n, q8w, t8w;               // words (of 8 bases) per slot
    int32_t packed;
    uint32_t fill;                      // 8 pad bytes' value (N_CODE replicated), as two words
    uint32_t nval;                      // N_CODE & 0xF
    const uint32_t *perm;               // slot i -> pair perm[i]
};

__device__ __forceinline__ uint32_t start_regs(uint32_t len, int32_t end) {
    const uint32_t regs = (len + 7) >> 3;
    const uint32_t r = ((uint32_t)end >> 3) + 1;
    return r < regs ? r : regs;
}

// 8 bases of word `wi` of a sequence at byte offset `off`, reversed, as bytes
__device__ __forceinline__ uint2 rev_word(const uint8_t *seq, uint32_t off, uint32_t wi, int packed) {
    if (!packed) {
        const uint2 v = *reinterpret_cast<const uint2 *>(seq + off + 8u * wi);
        return make_uint2(__builtin_bswap32(v.y), __builtin_bswap32(v.x));
    }
    // packed word: base k at bits 31-4k; reversed byte k = base 7-k = bits 4k+3..4k
    const uint32_t w = reinterpret_cast<const uint32_t *>(seq)[(off >> 3) + wi];
    uint2 o;
    o.x = (w & 15u) | (((w >> 4) & 15u) << 8) | (((w >> 8) & 15u) << 16) | (((w >> 12) & 15u) << 24);
    o.y = ((w >> 16) & 15u) | (((w >> 20) & 15u) << 8) | (((w >> 24) & 15u) << 16) | (((w >> 28) & 15u) << 24);
    return o;
}

__device__ __forceinline__ uint32_t seq_byte(const uint8_t *seq, uint32_t off, uint32_t pos, int packed) {
    if (!packed) return seq[off + pos];
    const uint32_t w = reinterpret_cast<const uint32_t *>(seq)[(off >> 3) + (pos >> 3)];
    return (w >> (28 - 4 * (pos & 7))) & 15u;
}

__device__ __forceinline__ uint32_t rev_bucket(const uint32_t *tlen, const int32_t *tend, uint32_t k, uint32_t t8w) {
    return t8w - start_regs(tlen[k], tend[k]);          // 0 = longest
}

__global__ __launch_bounds__(256) void rev_hist_kernel(const uint32_t *tlen, const int32_t *tend, uint32_t n,
                                                       uint32_t t8w, uint32_t *hist) {
    extern __shared__ uint32_t cnt[];
    for (uint32_t i = threadIdx.x; i < t8w; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) atomicAdd(&cnt[rev_bucket(tlen, tend, k, t8w)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < t8w; i += blockDim.x)
        if (cnt[i]) atomicAdd(&hist[i], cnt[i]);
}

// exclusive prefix sum of hist[0, nb) into cursor, one block of 256 threads
__global__ __launch_bounds__(256) void rev_scan_kernel(const uint32_t *hist, uint32_t *cursor, uint32_t nb) {
    __shared__ uint32_t part[256];
    const uint32_t per = (nb + 255) / 256, b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
    uint32_t sum = 0;
    for (uint32_t i = b0; i < b1; ++i) sum += hist[i];
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int i = 0; i < 256; ++i) { const uint32_t v = part[i]; part[i] = run; run += v; }
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
    for (uint32_t i = b0; i < b1; ++i) { cursor[i] = run; run += hist[i]; }
}

__global__ __launch_bounds__(256) void rev_scatter_kernel(const uint32_t *tlen, const int32_t *tend, uint32_t n,
                                                          uint32_t t8w, uint32_t *cursor, uint32_t *perm) {
    extern __shared__ uint32_t cnt[];   // [t8w] counts, then [t8w] bases
    uint32_t *base = cnt + t8w;
    for (uint32_t i = threadIdx.x; i < t8w; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t b = 0, local = 0;
    if (k < n) { b = rev_bucket(tlen, tend, k, t8w); local = atomicAdd(&cnt[b], 1u); }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < t8w; i += blockDim.x)
        if (cnt[i]) base[i] = atomicAdd(&cursor[i], cnt[i]);
    __syncthreads();
    if (k < n) perm[base[b] + local] = k;
}

// one thread per (slot, 8-base word of the two reversed sequences of the slot's pair)
__global__ __launch_bounds__(256) void rev_prep_kernel(RevArgs A) {
    const uint32_t per = A.q8w + A.t8w;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)A.n * per) return;
    const uint32_t i = (uint32_t)(gid / per), w = (uint32_t)(gid - (uint64_t)i * per);
    const uint32_t k = A.perm[i];
    uint2 v = make_uint2(A.fill, A.fill);
    if (w < A.q8w) {
        const uint32_t ql = A.qlen[k], rr = start_regs(ql, A.qend[k]), off = A.qoff[k];
        uint32_t L = 8 * rr;
        while (L > ql && seq_byte(A.q, off, L - 1, A.packed) % 16u == A.nval) --L;
        if (8 * w < L) {
            // output byte j = query position L-1-8w-j; positions below 0 are pads
            const int32_t st = (int32_t)L - 8 - 8 * (int32_t)w;
            if (!A.packed) {
                const int32_t a0 = st >= 0 ? st / 8 : -1, sh = st - 8 * a0;
                const uint64_t *src = reinterpret_cast<const uint64_t *>(A.q + off);
                const uint64_t lo = a0 >= 0 ? src[a0] : 0ull, hi = sh ? src[a0 + 1] : 0ull;   // within word rr-1
                uint64_t x = sh ? ((lo >> (8 * sh)) | (hi << (64 - 8 * sh))) : lo;   // bytes st .. st+7
                x = __builtin_bswap64(x);                                          // byte j = position st+7-j
                const uint32_t keep = L - 8 * w;                                   // valid bytes (1..8)
                if (keep < 8) {
                    const uint64_t m = (1ull << (8 * keep)) - 1ull;
                    x = (x & m) | (((uint64_t)A.fill << 32 | A.fill) & ~m);
                }
                v = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
            } else {
                uint32_t b[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int32_t p = st + 7 - j;
                    b[j] = p >= 0 ? seq_byte(A.q, off, (uint32_t)p, 1) : (A.fill & 0xFFu);
                }
                v.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
                v.y = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
            }
        }
        *reinterpret_cast<uint2 *>(A.rq + (uint64_t)i * A.q8w * 8 + 8u * w) = v;
        if (w == 0) { A.rqoff[i] = i * A.q8w * 8; A.rqlen[i] = L; }
    } else {
        const uint32_t ww = w - A.q8w;
        const uint32_t regs = start_regs(A.tlen[k], A.tend[k]);
        if (ww < regs) v = rev_word(A.t, A.toff[k], regs - 1 - ww, A.packed);
        *reinterpret_cast<uint2 *>(A.rt + (uint64_t)i * A.t8w * 8 + 8u * ww) = v;
        if (ww == 0) { A.rtoff[i] = i * A.t8w * 8; A.rtlen[i] = regs * 8; }
    }
}

// one thread per slot i (pair perm[i])
__global__ __launch_bounds__(256) void start_map_kernel(const uint32_t *perm, const int32_t *score,
                                                        const uint32_t *rqlen, const uint32_t *tlen,
                                                        const int32_t *tend, const int32_t *rqend,
                                                        const int32_t *rtend, int32_t *qstart, int32_t *tstart,
                                                        uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = perm[i];
    int32_t qs = 0, ts = 0;
    if (score[k] > 0) {   // local_kernel_template.h:468 loop guard maxHH < fwd_score
        const int32_t gr = (int32_t)start_regs(tlen[k], tend[k]);
        const int32_t Lq = (int32_t)rqlen[i];
        const int32_t r = rqend[i], c = rtend[i];
        qs = Lq - 1 - r;                                       // ridx counts down (true rows)
        ts = 8 * gr - 1 - 8 * (c >> 3) + (c & 7);              // gidx + (m-1), Q8
    }
    if (qstart) qstart[k] = qs;
    if (tstart) tstart[k] = ts;
}

}  // namespace gx
