// start.hpp — WITH_START (LOCAL, and SEMI-GLOBAL with TAIL=TARGET) on the
// wavefront kernels.
//
// The reference finds start positions with a second, reversed DP pass that
// stops early.  Both reverse passes are the forward kernel of the same
// algorithm reading the forward sequences backwards (WfArgs::rev): each reversed
// sequence is "the first L bases of the original, reversed", N after L, read in
// place at the pair's own offsets (round 4 wrote them into slots first: a
// prep kernel of 0.33 ms per 1 M config-2 pairs).
//
// LOCAL (Non-CDP/GASAL2/src/kernels/local_kernel_template.h:441-511).  From the
// 8-base words holding the end cell (rend_reg = min((q_end>>3)+1, qregs), same
// for the target) the reference walks query and target words backwards (each
// word's bases backwards too) with the forward cell update and 0 boundaries,
// and stops at the first cell, in its strip-major order over the reversed
// matrix, whose H reaches the forward score.  That cell's row is the query
// start; the target start is recorded as gidx + (m-1) while the column runs
// gidx - (m-1).  The reversed rectangle contains the forward
// optimum and is a sub-problem of the forward one, so its maximum is the
// forward score and "first cell reaching it" is the first strict maximum in
// strip-major order: what the LOCAL kernel reports (Q1).
//   target: L = 8*gend_reg.  The last word's pad columns stay: they are N
//           columns the reference scores, and they keep the 8-column strips
//           aligned as the reference's reversed strips are.
//   query:  L = 8*rend_reg less the run of N codes at its end lying at
//           positions >= ql (the pads; after a reverse-complement pre-op the
//           pad region can hold real bases, which stay).  The reference's
//           leading N rows hold H = 0 (every path into them starts at the 0
//           boundary and scores N as 0 or -N_PENALTY) and only turn the E/F
//           entering the first real row from 0 into negative values, which can
//           never win against the 0 clamp nor feed a later positive E/F; row
//           order inside a strip is unchanged, so is the tie-break order.  The
//           packed kernel needs real query rows to be A/C/G/T, which this keeps.
//   map:    q_start = Lq-1-r', t_start = 8*gend_reg-1-8*(c'>>3) + (c'&7) (Q8);
//           a forward score of 0 never enters the loop: (0, 0).
//
// SEMI-GLOBAL, TAIL=TARGET (semiglobal_kernel_template.h:227-383).  The
// reference reverses the whole query and target, then runs the forward
// recurrence (same HEAD boundaries, restarted) over the reversed target from
// strip gend_reg = X > 0 ? X-1 : X, X = tregs - (t_end>>3) - 1, to the end,
// stopping after the first strip in which a last-row cell (column < tl)
// reaches the forward score; the result is the first maximum over the last
// row of the strips it ran.  Since every cell before that strip is below the
// forward score, that is the first maximum inside the stopping strip, or the
// first maximum overall when no strip stops it.  The wavefront kernels find it
// with a `stop` key (wavefront.hpp / wavefront16.hpp, WfArgs::stop).
//   query:  L = ql (pads after the last row never reach it; the reference's
//           zero codes there are not read by a TAIL=TARGET result)
//   target: the reversed target from column 8*gend_reg = the first
//           L = tl - 8*gend_reg original bases, reversed; strips stay aligned.
//   map:    t_start = tl-1 - (8*gend_reg + c'); q_start = ql-1 - tl (the
//           reverse pass leaves maxXY_x at ref_len, Q10); no last-row cell at
//           all leaves maxXY_y = 0.
//
// The reverse pass's slots are sorted by reversed target words, longest first
// (counting sort, perm: slot -> pair): a wave's step count is set by its longest
// target, and unrelated pairs end early, so their reversed rectangles are short.
// LOCAL sorts by the reversed query's words first: the class kernels of rclass.hip run
// each block with the rows its longest query needs.
// Lengths and results of the reverse pass are per pair.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace gx {

enum RevMode { REV_LOCAL = 0, REV_SEMI = 1, REV_PLAIN = 2 };   // PLAIN: sort by the lengths given

__device__ __forceinline__ uint32_t start_regs(uint32_t len, int32_t end) {
    const uint32_t regs = (len + 7) >> 3;
    const uint32_t r = ((uint32_t)end >> 3) + 1;
    return r < regs ? r : regs;
}

// semiglobal_kernel_template.h:273: first reversed-target strip of the reverse pass
__device__ __forceinline__ int32_t semi_gend_reg(uint32_t tl, int32_t tend) {
    const int32_t x = (int32_t)((tl + 7) >> 3) - ((tend >> 3) + 1);
    return x > 0 ? x - 1 : x;
}

// reversed target length of pair k
__device__ __forceinline__ uint32_t rev_tlen(int32_t mode, const uint32_t *tlen, const int32_t *tend, uint32_t k) {
    if (mode == REV_PLAIN) return tlen[k];
    if (mode == REV_LOCAL) return 8 * start_regs(tlen[k], tend[k]);
    const int32_t L = (int32_t)tlen[k] - 8 * semi_gend_reg(tlen[k], tend[k]);
    return (uint32_t)max(L, 0);
}

__device__ __forceinline__ uint32_t seq_byte(const uint8_t *seq, uint32_t off, uint32_t pos, int packed) {
    if (!packed) return seq[off + pos];
    const uint32_t w = reinterpret_cast<const uint32_t *>(seq)[(off >> 3) + (pos >> 3)];
    return (w >> (28 - 4 * (pos & 7))) & 15u;
}

// sort key of the reverse pass's slots: the reversed target length, or (LOCAL with the forward
// scores, whose sweep stops once the score is reached) the shorter of it and a span estimate of
// the alignment, 2 * ceil(score / match) + 16 columns -- a wave's step count is set by its
// slowest pair, so pairs that will stop early share waves.  LOCAL with qlen: first by the
// reversed query's words (the register axis, which rclass.hip sizes per block), then by that.
// (A heuristic: the results do not depend on the order.)  Buckets: (q8w + 1) x (t8w + 1) with
// qlen, t8w + 1 without; 0 = longest.
__device__ __forceinline__ uint32_t rev_bucket(int32_t mode, const uint32_t *tlen, const int32_t *tend, uint32_t k,
                                               uint32_t t8w, const int32_t *score = nullptr, int32_t a = 1,
                                               const uint32_t *qlen = nullptr, const int32_t *qend = nullptr,
                                               uint32_t q8w = 0) {
    uint32_t L = rev_tlen(mode, tlen, tend, k);
    if (score && mode == REV_LOCAL && a > 0) {
        const int32_t sc = max(score[k], 0);
        L = min(L, (uint32_t)(2 * ((sc + a - 1) / a) + 16));
    }
    const uint32_t b = t8w - min((L + 7) >> 3, t8w);
    if (!qlen || mode != REV_LOCAL) return b;
    const uint32_t qb = q8w - min(start_regs(qlen[k], qend[k]), q8w);
    return qb * (t8w + 1) + b;
}

// cnt[b] += the number of active lanes of the wave with bucket b, one LDS atomic per distinct
// bucket of the wave (a lane per bucket adds the whole group's count); returns the lane's position
// among them (the old count + its rank in the group).  The per-lane LDS atomics this replaces
// serialised on the few buckets of a batch (config 2: ~20 distinct, 48 us per 1 M pairs).
__device__ __forceinline__ uint32_t wave_bucket_add(uint32_t *cnt, uint32_t b, bool active) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t todo = __ballot(active);
    uint32_t pos = 0;
    while (todo) {                                   // wave-uniform: one pass per distinct bucket
        const int leader = __builtin_ctzll(todo);
        const uint32_t lb = __shfl(b, leader);
        const bool mine = active && b == lb;
        const uint64_t m = __ballot(mine);
        uint32_t base = 0;
        if ((int)lane == leader) base = atomicAdd(&cnt[lb], (uint32_t)__popcll(m));
        base = __shfl(base, leader);
        if (mine) pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        todo &= ~m;
    }
    return pos;
}

// The sort kernels walk the pairs grid-stride (sort_grid: at most 1,024 blocks) and add a
// block's counts to the global ones once: one global atomic per bucket and block of 256 pairs
// serialised on the batch's few buckets (0.45 ms per 10 M config-4 pairs, 0.08 ms per 1 M
// config-2 pairs).  nb: the bucket count (rev_bucket).
inline int sort_grid(uint32_t n) { return (int)std::min<uint32_t>((n + 255) / 256, 1024u); }

__global__ __launch_bounds__(256) void rev_hist_kernel(int32_t mode, const uint32_t *tlen, const int32_t *tend,
                                                       uint32_t n, uint32_t t8w, uint32_t *hist,
                                                       const int32_t *score = nullptr, int32_t a = 1,
                                                       const uint32_t *qlen = nullptr, const int32_t *qend = nullptr,
                                                       uint32_t q8w = 0, uint32_t nb = 0) {
    extern __shared__ uint32_t cnt[];   // nb buckets
    if (!nb) nb = t8w + 1;
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {   // wave-uniform trips
        const uint32_t k = base + threadIdx.x;
        (void)wave_bucket_add(cnt, k < n ? rev_bucket(mode, tlen, tend, k, t8w, score, a, qlen, qend, q8w) : 0u, k < n);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x)
        if (cnt[i]) atomicAdd(&hist[i], cnt[i]);
}

// exclusive prefix sum of hist[0, nb) into cursor, one block of 256 threads
__global__ __launch_bounds__(256) void rev_scan_kernel(const uint32_t *hist, uint32_t *cursor, uint32_t nb) {
    __shared__ uint32_t part[256];
    const uint32_t per = (nb + 255) / 256, b0 = min(threadIdx.x * per, nb), b1 = min(b0 + per, nb);
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

__global__ __launch_bounds__(256) void rev_scatter_kernel(int32_t mode, const uint32_t *tlen, const int32_t *tend,
                                                          uint32_t n, uint32_t t8w, uint32_t *cursor,
                                                          uint32_t *perm, uint32_t *inv = nullptr,
                                                          const int32_t *score = nullptr, int32_t a = 1,
                                                          const uint32_t *qlen = nullptr,
                                                          const int32_t *qend = nullptr, uint32_t q8w = 0,
                                                          uint32_t nb = 0) {
    extern __shared__ uint32_t cnt[];   // [nb] counts, then [nb] bases
    if (!nb) nb = t8w + 1;
    uint32_t *base = cnt + nb;
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    // the block's counts over all its pairs, one global reservation per bucket, then the positions
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < n; b0 += stride) {
        const uint32_t k = b0 + threadIdx.x;
        (void)wave_bucket_add(cnt, k < n ? rev_bucket(mode, tlen, tend, k, t8w, score, a, qlen, qend, q8w) : 0u, k < n);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
        if (cnt[i]) base[i] = atomicAdd(&cursor[i], cnt[i]);
        cnt[i] = 0;
    }
    __syncthreads();
    for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < n; b0 += stride) {
        const uint32_t k = b0 + threadIdx.x;
        const uint32_t b = k < n ? rev_bucket(mode, tlen, tend, k, t8w, score, a, qlen, qend, q8w) : 0u;
        const uint32_t local = wave_bucket_add(cnt, b, k < n);
        if (k < n) {
            perm[base[b] + local] = k;
            if (inv) inv[k] = base[b] + local;
        }
    }
}

// one thread per pair: the reversed lengths (LOCAL: the end words, less the trailing N pads, a
// loop of dependent byte loads done once per pair), which the reverse pass reads the forward
// sequences backwards with (WfArgs::rev)
__global__ __launch_bounds__(256) void rev_len_kernel(int32_t mode, const uint8_t *q, const uint32_t *qoff,
                                                      const uint32_t *qlen, const uint32_t *tlen, const int32_t *qend,
                                                      const int32_t *tend, int32_t packed, uint32_t nval, uint32_t n,
                                                      uint32_t *rqlen, uint32_t *rtlen) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t ql = qlen[k];
    uint32_t L = ql;
    if (mode == REV_LOCAL) {
        const uint32_t off = qoff[k];
        L = 8 * start_regs(ql, qend[k]);
        while (L > ql && seq_byte(q, off, L - 1, packed) % 16u == nval) --L;
    }
    rqlen[k] = L;
    rtlen[k] = rev_tlen(mode, tlen, tend, k);
}

// one thread per pair k: the reverse pass's ends -> the reference's start fields
__global__ __launch_bounds__(256) void start_map_kernel(int32_t mode, const int32_t *score, const uint32_t *qlen,
                                                        const uint32_t *rqlen, const uint32_t *tlen,
                                                        const int32_t *tend, const int32_t *rscore,
                                                        const int32_t *rqend, const int32_t *rtend, int32_t *qstart,
                                                        int32_t *tstart, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int32_t qs = 0, ts = 0;
    if (mode == REV_LOCAL) {
        if (score[k] > 0) {   // local_kernel_template.h:468 loop guard maxHH < fwd_score
            const int32_t gr = (int32_t)start_regs(tlen[k], tend[k]);
            const int32_t r = rqend[k], c = rtend[k];
            qs = (int32_t)rqlen[k] - 1 - r;                    // ridx counts down (true rows)
            ts = 8 * gr - 1 - 8 * (c >> 3) + (c & 7);          // gidx + (m-1), Q8
        }
    } else {
        const int32_t tl = (int32_t)tlen[k];
        const int32_t y = rscore[k] > -32768 ? 8 * semi_gend_reg(tlen[k], tend[k]) + rtend[k] : 0;
        ts = tl - 1 - y;                                       // semiglobal :380
        qs = (int32_t)qlen[k] - 1 - tl;                        // :381, maxXY_x = ref_len (Q10)
    }
    if (qstart) qstart[k] = qs;
    if (tstart) tstart[k] = ts;
}

}  // namespace gx
