// nvbio.hpp — scoring kernels behind the second front-end: nvbio's batched
// alignment score (NvB/nvbio/alignment/batched.h:44-87, sw-benchmark.cu:355-443).
//
// Semantics (TextBlockingTag, score only, BestSink):
//   Gotoh  (gotoh/gotoh_inl.h:985-1110 cell update, :1140-1260 + :1395-1420 boundaries
//          and sinks; utils.h:114-135 SimpleGotohScheme):
//     F(i,c) = max(F(i-1,c) + Ge, H(i-1,c) + Go)     E(i,c) = max(E(i,c-1) + Ge, H(i,c-1) + Go)
//     H(i,c) = max3(E, F, H(i-1,c-1) + S(p_i, t_c))   LOCAL: max(H, 0)
//     H(i,-1) = LOCAL ? 0 : Go + Ge*i,  E(i,-1) = LOCAL ? 0 : -inf   (gotoh_inl.h:80-86)
//     H(-1,c) = GLOBAL ? (c >= 0 ? Go + Ge*c : 0) : 0,  F(-1,c) = -inf
//   Smith-Waterman, linear gaps (sw/sw_inl.h:895-970, :1085-1215, utils.h:92-110):
//     H(i,c) = max3(H(i-1,c) + Ins, H(i,c-1) + Del, H(i-1,c-1) + S)   LOCAL: max(H, 0)
//     H(i,-1) = LOCAL ? 0 : Ins*(i+1),  H(-1,c) = GLOBAL ? Del*(c+1) : 0
//   Edit distance = Smith-Waterman with (0, -1, -1, -1) (ed/ed_inl.h:97, ed_utils.h:45-52).
//   S(p, t) = p == t ? match : mismatch.  Sinks (sink_inl.h:59-68, the best score is all
//   that sw-benchmark's stream writes out, sw-benchmark.cu:203-209): LOCAL every cell,
//   SEMI_GLOBAL the last pattern row, GLOBAL H(M-1, N-1).
//
// Layout: the pattern is the register axis (G lanes per pair, R rows per lane),
// the text the step axis, staged in LDS as 16-bit codes (pads never match: pattern
// pad 0xFFFE, text pad 0xFFFF); one text per block when every pair shares it (the
// sw-benchmark case: all reads against one reference).  int32 arithmetic; the host
// bounds |values| so the -inf stand-in never wins, as nvbio's infimum never does.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gx {

enum NvAligner { NV_ED = 0, NV_SW = 1, NV_GOTOH = 2 };
enum NvType { NV_GLOBAL = 0, NV_LOCAL = 1, NV_SEMI = 2 };   // nvbio AlignmentType order (alignment_base.h:54)

struct NvArgs {
    const uint32_t *pw, *poff;      // pattern words, n + 1 symbol offsets
    uint32_t pbits, pbig;
    const uint32_t *tw, *toff;      // text words, n + 1 symbol offsets (NULL: one shared text of tlen0)
    uint32_t tbits, tbig, tlen0;
    int32_t *score;
    int16_t *score16;
    uint32_t n;
    int32_t match, mismatch, go, ge, del, ins;
    uint32_t lds_stride;            // 16-bit codes per text slot (>= padded max text + G)
};

constexpr int32_t kNvInf = -(1 << 29);

__device__ __forceinline__ uint32_t nv_symbol(const uint32_t *w, uint32_t bits, uint32_t big, uint32_t s) {
    if (bits == 8) return (w[s >> 2] >> (big ? 24 - 8 * (s & 3) : 8 * (s & 3))) & 0xFFu;
    const uint32_t per = 32u / bits, p = s % per;
    const uint32_t sh = big ? 32u - bits * (p + 1) : bits * p;
    return (w[s / per] >> sh) & ((1u << bits) - 1u);
}

__device__ __forceinline__ int32_t nv_shr(int32_t v) {   // lane i <- lane i-1 (DPP wave_shr:1)
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false);
}

template <int ALN, int TYPE, int G, int R, bool MASK>
__global__ __launch_bounds__(256) void nv_kernel(NvArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint16_t nvlds[];
    constexpr int P = 64 / G;
    constexpr bool GOTOH = ALN == NV_GOTOH;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1), slot = lane / G;
    const uint32_t pair = (blockIdx.x * 4 + wave) * P + slot;
    const bool valid = pair < A.n;
    const bool shared_text = A.toff == nullptr;
    uint32_t M = 0, N = 0, po = 0, to = 0;
    if (valid) {
        po = A.poff[pair]; M = A.poff[pair + 1] - po;
        if (shared_text) N = A.tlen0;
        else { to = A.toff[pair]; N = A.toff[pair + 1] - to; }
    }
    const uint32_t stride = A.lds_stride;
    // ---- text codes in LDS (one copy per block when shared) ----
    uint16_t *mine;
    if (shared_text) {
        for (uint32_t i = threadIdx.x; i < stride; i += blockDim.x)
            nvlds[i] = i < A.tlen0 ? (uint16_t)nv_symbol(A.tw, A.tbits, A.tbig, i) : (uint16_t)0xFFFF;
        mine = nvlds;
    } else {
        uint16_t *wl = nvlds + (size_t)wave * P * stride;
        for (uint32_t ps = 0; ps < (uint32_t)P; ps++) {   // uniform trip counts: shuffles see all lanes
            const uint32_t pN = __shfl(N, ps * G), pto = __shfl(to, ps * G);
            for (uint32_t i = lane; i < stride; i += 64)
                wl[ps * stride + i] = i < pN ? (uint16_t)nv_symbol(A.tw, A.tbits, A.tbig, pto + i) : (uint16_t)0xFFFF;
        }
        mine = wl + slot * stride;
    }
    __syncthreads();

    // ---- the lane's pattern rows ----
    const uint32_t r0 = lg * R;
    uint32_t pc[R];
    int32_t Hk[R], Ek[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t r = r0 + k;
        pc[k] = (valid && r < M) ? nv_symbol(A.pw, A.pbits, A.pbig, po + r) : 0xFFFEu;
        if (GOTOH) {
            Hk[k] = TYPE == NV_LOCAL ? 0 : A.go + A.ge * (int32_t)r;
            Ek[k] = TYPE == NV_LOCAL ? 0 : kNvInf;
        } else {
            Hk[k] = TYPE == NV_LOCAL ? 0 : A.ins * (int32_t)(r + 1);
            Ek[k] = 0;
        }
    }
    uint32_t nmax = N;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor(nmax, m));
    const uint32_t nsteps = nmax + G - 1;
    const uint32_t last_lane = M ? (M - 1) / R : 0, last_k = M ? (M - 1) - last_lane * R : 0;
    int32_t best = INT32_MIN;                     // BestSink() (sink_inl.h:38-40)
    // from the lane above: H(r0-1, c), F(r0-1, c), H(r0-1, c-1).  rH starts as the left
    // boundary H(r0-1, -1): lane 1 takes it as its diagonal at column 0 (lane 0 never
    // runs a column -1 step to hand it down)
    const int32_t rb = (int32_t)r0 - 1;
    int32_t rH = (TYPE == NV_LOCAL || lg == 0) ? 0 : (GOTOH ? A.go + A.ge * rb : A.ins * (rb + 1));
    int32_t rF = kNvInf, pH = 0;
    for (uint32_t s = 0; s < nsteps; ++s) {
        const int32_t c = (int32_t)s - (int32_t)lg;
        int32_t Hup, Fup, Hdg;
        if (lg == 0) {
            if (TYPE == NV_GLOBAL) {
                Hup = GOTOH ? A.go + A.ge * c : A.del * (c + 1);
                Hdg = GOTOH ? (c >= 1 ? A.go + A.ge * (c - 1) : 0) : A.del * c;
            } else { Hup = 0; Hdg = 0; }
            Fup = kNvInf;
        } else { Hup = rH; Fup = rF; Hdg = pH; }
        if (c >= 0 && (uint32_t)c < stride) {
            const uint32_t tc = mine[c];
            const bool cin = (uint32_t)c < N;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int32_t S = (pc[k] == tc) ? A.match : A.mismatch;
                int32_t H;
                if (GOTOH) {
                    const int32_t F = max(Fup + A.ge, Hup + A.go);
                    const int32_t E = max(Ek[k] + A.ge, Hk[k] + A.go);
                    H = max(max(E, F), Hdg + S);
                    Ek[k] = E;
                    Fup = F;
                } else {
                    H = max(max(Hup + A.ins, Hk[k] + A.del), Hdg + S);
                }
                if (TYPE == NV_LOCAL) {
                    H = max(H, 0);
                    if (MASK) best = (cin && r0 + k < M) ? max(best, H) : best;
                    else best = max(best, H);
                }
                Hdg = Hk[k];
                Hk[k] = H;
                Hup = H;
            }
            if (TYPE != NV_LOCAL && lg == last_lane && cin) {
                int32_t h = 0;
#pragma unroll
                for (int k = 0; k < R; ++k) h = (k == (int)last_k) ? Hk[k] : h;
                if (TYPE == NV_SEMI) best = max(best, h);
                else if ((uint32_t)c == N - 1) best = h;
            }
        }
        // hand the bottom row down: H(r0+R-1, c) once active; before that Hk[R-1] still
        // holds the row's left boundary H(r0+R-1, -1), the diagonal the lane below needs
        // at its column 0
        pH = rH;
        rH = nv_shr(Hk[R - 1]);
        rF = nv_shr(Fup);
    }
    // LOCAL: the pair's best over its lanes
    if (TYPE == NV_LOCAL) {
#pragma unroll
        for (int m = 1; m < G; m <<= 1) best = max(best, __shfl_xor(best, m));
    }
    const bool writer = TYPE == NV_LOCAL ? lg == 0 : lg == last_lane;
    if (valid && writer) {
        int32_t v = best;
        if (M == 0) {   // no pattern rows: only the band initialisation reaches the sink
            v = TYPE == NV_SEMI ? (N ? 0 : INT32_MIN)
              : TYPE == NV_GLOBAL ? (N ? (GOTOH ? A.go + A.ge * (int32_t)(N - 1) : A.del * (int32_t)N) : INT32_MIN)
                                  : INT32_MIN;
        } else if (N == 0) v = INT32_MIN;
        if (A.score) A.score[pair] = v;
        if (A.score16) A.score16[pair] = (int16_t)v;   // sw-benchmark's int16 score vector
    }
}

}  // namespace gx
