// nvbio16.hpp — the nvbio front-end's scoring kernel (nvbio.hpp) with two pairs
// per lane group: the pattern rows of pair 2p in the low 16-bit half of every
// register, those of pair 2p + 1 in the high half, against the one text all
// pairs share (sw-benchmark's layout: reads against one reference,
// NvB/sw-benchmark/sw-benchmark.cu:355-443).  Same recurrences, boundaries and
// sinks as nv_kernel; same lane-group wavefront (G lanes, R pattern rows per
// lane, DPP hand-off of the bottom row).
//
// Arithmetic (as wavefront16.hpp): a stored value is value + B inside the
// positive normal f16 range [0x0400, 0x7BFF], where v_pk_maximum3_f16 orders the
// bit patterns like the integers: one instruction is an exact 3-way max on both
// pairs, and 32-bit adds of a packed pair never carry or borrow across halves.
// nvbio's -inf stand-in becomes NEG = 0x0400, below every reachable value; E and
// F are floored there (LOCAL: at 0, exact for H because gaps never score > 0).
//
// Substitution: nvbio scores equality only (S = p == t ? match : mismatch).  The
// text (2-bit, symbols 0..3) is staged in LDS as one 4-byte table per column,
// byte l = (l == t) ? match - mismatch : 0, and a row's selector picks the byte
// of its pattern symbol for each half (symbols >= 4, and pad rows, select the
// constant 0: a mismatch, as nvbio's never-matching N); tmp = Hdg + byte +
// mismatch is one v_add3.  Per cell of both pairs, Gotoh: v_perm, v_add3, F
// (2 sub + maximum3), E (2 sub + maximum3), H (maximum3): 9 instructions.
//
// Gotoh SEMI_GLOBAL / GLOBAL (FR): values drift by g = -ge per anti-diagonal, as in
// wavefront16.hpp's SEMI frame: F^ = B + F + g(r+c), E^ likewise, H^ = B + H + g(r+c)
// + (go - ge), so F(r,c) = max(F(r-1,c) + ge, H(r-1,c) + go) is max(F^up, H^up), E
// likewise, tmp^ = H^dg + byte + (mismatch + g - go) and H^ = max3 + (go - ge): 6
// instructions per cell of both pairs instead of 9.  Sinks compare a row's columns
// in one frame (+ g*(N-1-c)); the outputs take the frame off again.
//
// Sinks (sink_inl.h:59-68): LOCAL every cell (a running maximum3 over two cells
// per instruction; pad rows and columns score <= 0 and never exceed a real cell,
// which the host requires); SEMI_GLOBAL row M-1 of each pair at every column;
// GLOBAL H(M-1, N-1).  The row M-1 of either half is picked through per-row
// masks (mask[k] = 0xFFFF in the half whose last row is row k of this lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nvbio.hpp"
#include "wavefront16.hpp"

namespace gx {

struct Nv16Args {
    const uint32_t *pw, *poff;      // pattern words, n + 1 symbol offsets
    uint32_t pbits, pbig;
    const uint32_t *tw;             // 2-bit text symbols
    const uint32_t *toff;           // n + 1 symbol offsets of per-pair texts (SHARED: unused)
    uint32_t tbig, tlen0;           // tlen0: the shared text's length
    int32_t *score;
    int16_t *score16;
    uint32_t n;
    int32_t match, mismatch, go, ge, del, ins;
    uint32_t base;                  // stored value of 0
    uint32_t lds_cols;              // table entries per staged text (>= its length, multiple of 4)
};

__device__ __forceinline__ uint32_t nv16_dpp(uint32_t v) {   // lane i <- lane i-1 (DPP wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}

template <int ALN, int TYPE, int G, int R, bool SHARED>
__global__ __launch_bounds__(256) void nv16_kernel(Nv16Args A) {
    extern __shared__ __attribute__((aligned(16))) uint32_t nvt[];
    constexpr int P = 64 / G;
    constexpr bool GOTOH = ALN == NV_GOTOH;
    constexpr bool FR = GOTOH && TYPE != NV_LOCAL;   // the drift frame (header)
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1), grp = lane / G;
    const uint32_t pa = 2 * ((blockIdx.x * 4 + wave) * P + grp), pb = pa + 1;
    const bool va = pa < A.n, vb = pb < A.n;
    uint32_t Ma = 0, Mb = 0, poa = 0, pob = 0;
    if (va) { poa = A.poff[pa]; Ma = A.poff[pa + 1] - poa; }
    if (vb) { pob = A.poff[pb]; Mb = A.poff[pb + 1] - pob; }
    // ---- the text(s) as per-column tables (pads: all mismatch) ----
    const uint32_t dm = (uint32_t)(A.match - A.mismatch);
    const uint32_t cols = A.lds_cols;
    uint32_t Na = A.tlen0, Nb = A.tlen0, toa = 0, tob = 0;
    const uint32_t *Ta = nvt, *Tb = nvt;
    if (SHARED) {
        for (uint32_t c = threadIdx.x; c < cols; c += blockDim.x)
            nvt[c] = c < Na ? dm << (8 * nv_symbol(A.tw, 2, A.tbig, c)) : 0u;
    } else {
        // one slot per pair of the wave: slot 2*grp + half
        Na = Nb = 0;
        if (va) { toa = A.toff[pa]; Na = A.toff[pa + 1] - toa; }
        if (vb) { tob = A.toff[pb]; Nb = A.toff[pb + 1] - tob; }
        uint32_t *wl = nvt + (size_t)wave * 2 * P * cols;
        for (uint32_t ps = 0; ps < 2u * P; ++ps) {   // uniform trip counts: shuffles see all lanes
            const uint32_t src = (ps >> 1) * G;
            const uint32_t pN = __shfl((ps & 1) ? Nb : Na, src), pto = __shfl((ps & 1) ? tob : toa, src);
            for (uint32_t c = lane; c < cols; c += 64)
                wl[ps * cols + c] = c < pN ? dm << (8 * nv_symbol(A.tw, 2, A.tbig, pto + c)) : 0u;
        }
        Ta = wl + 2 * grp * cols;
        Tb = Ta + cols;
    }
    __syncthreads();
    const uint32_t N = max(Na, Nb);

    const int32_t B = (int32_t)A.base;
    const uint32_t BB = A.base * 0x10001u, NEG = 0x04000400u;
    const uint32_t FLOOR = TYPE == NV_LOCAL ? BB : NEG;
    const uint32_t MIS = (uint32_t)A.mismatch * 0x10001u;
    const uint32_t GO = (uint32_t)(-A.go) * 0x10001u, GE = (uint32_t)(-A.ge) * 0x10001u;   // gaps <= 0
    const uint32_t DEL = (uint32_t)(-A.del) * 0x10001u, INS = (uint32_t)(-A.ins) * 0x10001u;
    auto pk = [&](int32_t v) { return (uint32_t)(v + B) * 0x10001u; };
    // ---- the lane's pattern rows ----
    // BOT (one shared text, SEMI_GLOBAL): rows bottom-aligned per half, so both pairs'
    // last row M-1 is row R-1 of lane G-1 and the sink is one maximum per step.  The
    // rows above row 0 are virtual: they score every column with the constant byte
    // |mismatch| (v_perm's second source, selector 4), so tmp = Hdg and, from the free
    // top boundary H = 0 (F = -inf), each passes H = 0 down unchanged (E and F stay
    // below it: gap scores <= 0) — row 0 sees exactly nvbio's boundary.
    constexpr bool BOT = SHARED && TYPE == NV_SEMI;
    const uint32_t VCONST = (uint32_t)(-A.mismatch);
    const int32_t ra0 = (int32_t)(lg * R) - (BOT ? (int32_t)(G * R - Ma) : 0);
    const int32_t rb0 = (int32_t)(lg * R) - (BOT ? (int32_t)(G * R - Mb) : 0);
    const uint32_t last_a = Ma ? Ma - 1 : 0xFFFFFFFFu, last_b = Mb ? Mb - 1 : 0xFFFFFFFFu;
    uint32_t sel[R], Hk[R], Ek[R], msk[R];
    bool has_last = false;
    auto left = [&](int32_t r) {   // H(r, -1); virtual rows: 0
        if (TYPE == NV_LOCAL || r < 0) return 0;
        return GOTOH ? A.go + A.ge * r : A.ins * (r + 1);
    };
    auto pk2 = [&](int32_t a, int32_t b) { return (uint32_t)(a + B) | ((uint32_t)(b + B) << 16); };
    const int32_t g = -A.ge, dl = A.go - A.ge;           // FR: drift per anti-diagonal, H^ offset
    // FR: H^ of H value h at (r, c)
    auto fr = [&](int32_t h, int32_t r, int32_t c) { return h + g * (r + c) + dl; };
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int32_t ra = ra0 + k, rb = rb0 + k;
        const uint32_t ca = (va && ra >= 0 && ra < (int32_t)Ma) ? nv_symbol(A.pw, A.pbits, A.pbig, poa + ra) : 4u;
        const uint32_t cb = (vb && rb >= 0 && rb < (int32_t)Mb) ? nv_symbol(A.pw, A.pbits, A.pbig, pob + rb) : 4u;
        // SHARED: both halves read the one table (v_perm(VCONST, T, .)); otherwise the
        // high half's bytes come from the second source, selectors 4..7
        const uint32_t sa = ra < 0 ? 4u : (ca < 4 ? ca : 0x0Cu);
        const uint32_t sb = rb < 0 ? 4u : (cb < 4 ? cb + (SHARED ? 0u : 4u) : 0x0Cu);
        sel[k] = sa | 0x0C00u | (sb << 16) | 0x0C000000u;
        Hk[k] = FR ? pk2(fr(left(ra), ra, -1), fr(left(rb), rb, -1)) : pk2(left(ra), left(rb));
        Ek[k] = GOTOH ? (TYPE == NV_LOCAL ? BB : NEG) : 0u;
        msk[k] = ((uint32_t)ra == last_a ? 0x0000FFFFu : 0u) | ((uint32_t)rb == last_b ? 0xFFFF0000u : 0u);
        has_last |= msk[k] != 0u;
    }
    uint32_t nmax = N;
    if (!SHARED) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor(nmax, m));
    }
    const uint32_t nsteps = nmax + G - 1;
    // per-half column limits of the sinks (SEMI: c < N of the half; GLOBAL: c == N - 1)
    const uint32_t lastc_a = Na - 1, lastc_b = Nb - 1;
    uint32_t best = TYPE == NV_LOCAL ? BB : NEG;   // stored; NEG = no cell seen (BestSink, sink_inl.h:38-40)
    // from the lane above: H(r0-1, c), F(r0-1, c), H(r0-1, c-1); rH starts as the
    // left boundary H(r0-1, -1), lane 1's diagonal at column 0 (nvbio.hpp)
    uint32_t rH = lg == 0 ? BB
                : FR ? pk2(fr(left(ra0 - 1), ra0 - 1, -1), fr(left(rb0 - 1), rb0 - 1, -1))
                     : pk2(left(ra0 - 1), left(rb0 - 1));
    const uint32_t MISF = (uint32_t)(A.mismatch + g - A.go) * 0x10001u, DL = (uint32_t)dl * 0x10001u;
    uint32_t rF = NEG, pH = BB;
    for (uint32_t s = 0; s < nsteps; ++s) {
        const int32_t c = (int32_t)s - (int32_t)lg;
        uint32_t Hup, Fup, Hdg;
        if (lg == 0) {
            if (FR) {   // H of the row above the lane's first (-1; BOT: virtual rows per half), in the frame
                const int32_t hu = TYPE == NV_GLOBAL ? A.go + A.ge * c : 0;
                const int32_t hd = TYPE == NV_GLOBAL && c >= 1 ? A.go + A.ge * (c - 1) : 0;
                Hup = pk2(fr(hu, ra0 - 1, c), fr(hu, rb0 - 1, c));
                Hdg = pk2(fr(hd, ra0 - 1, c - 1), fr(hd, rb0 - 1, c - 1));
            } else if (TYPE == NV_GLOBAL) {
                Hup = pk(GOTOH ? A.go + A.ge * c : A.del * (c + 1));
                Hdg = pk(GOTOH ? (c >= 1 ? A.go + A.ge * (c - 1) : 0) : A.del * c);
            } else { Hup = BB; Hdg = BB; }
            Fup = NEG;
        } else { Hup = rH; Fup = rF; Hdg = pH; }
        if (c >= 0 && (uint32_t)c < N) {
            const uint32_t T = Ta[c], T1 = SHARED ? VCONST : Tb[c];
            uint32_t lbest = best;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const uint32_t v = __builtin_amdgcn_perm(T1, T, sel[k]);
                const uint32_t tmp = Hdg + v + MIS;
                uint32_t H;
                if (FR) {
                    const uint32_t tmp2 = Hdg + v + MISF;
                    const uint32_t F = pk_max_u16(Fup, Hup);
                    const uint32_t E = pk_max_u16(Ek[k], Hk[k]);
                    H = pk_max3(E, F, tmp2) + DL;
                    Ek[k] = E;
                    Fup = F;
                } else if (GOTOH) {
                    const uint32_t F = pk_max3(Fup - GE, Hup - GO, FLOOR);
                    const uint32_t E = pk_max3(Ek[k] - GE, Hk[k] - GO, FLOOR);
                    H = pk_max3(E, F, tmp);
                    Ek[k] = E;
                    Fup = F;
                } else {
                    H = pk_max3(Hup - INS, Hk[k] - DEL, tmp);
                    if (TYPE == NV_LOCAL) H = pk_max3(H, BB, BB);
                }
                if (TYPE == NV_LOCAL) {   // two rows per maximum3: Hup is still row k - 1's H here
                    if (k & 1) lbest = pk_max3(lbest, H, Hup);
                    else if (k == R - 1) lbest = pk_max3(lbest, H, H);
                }
                Hdg = Hk[k];
                Hk[k] = H;
                Hup = H;
            }
            if (TYPE == NV_LOCAL) best = lbest;
            if (BOT) {
                // FR: the row's columns in one frame, + g*(N-1-c) (c < N here)
                const uint32_t kof = FR ? (uint32_t)(g * (int32_t)(N - 1 - (uint32_t)c)) * 0x10001u : 0u;
                if (lg == G - 1) best = pk_max3(best, Hk[R - 1] + kof, best);
            } else if (TYPE != NV_LOCAL && has_last) {
                uint32_t h = 0, hm = 0;
#pragma unroll
                for (int k = 0; k < R; ++k) { h |= Hk[k] & msk[k]; hm |= msk[k]; }
                if (TYPE == NV_SEMI) {   // a half without its last row here, or past its text: +0
                    if (!SHARED) hm &= ((uint32_t)c < Na ? 0x0000FFFFu : 0u) | ((uint32_t)c < Nb ? 0xFFFF0000u : 0u);
                    // FR: + g*(N-1-c) per half, masked first so that no add carries across
                    const uint32_t off = FR ? (((uint32_t)(g * (int32_t)(Na - 1 - (uint32_t)c)) & 0xFFFFu) |
                                               ((uint32_t)(g * (int32_t)(Nb - 1 - (uint32_t)c)) << 16)) & hm
                                            : 0u;
                    h = (h & hm) + off;
                    best = pk_max3(best, h, best);
                } else if (SHARED) {
                    if ((uint32_t)c == N - 1) best = h;
                } else {
                    if ((uint32_t)c == lastc_a) best = (best & 0xFFFF0000u) | (h & 0x0000FFFFu);
                    if ((uint32_t)c == lastc_b) best = (best & 0x0000FFFFu) | (h & 0xFFFF0000u);
                }
            }
        }
        pH = rH;
        rH = nv16_dpp(Hk[R - 1]);
        rF = nv16_dpp(Fup);
    }
    // LOCAL: the pair's best over its lanes
    if (TYPE == NV_LOCAL) {
#pragma unroll
        for (int m = 1; m < G; m <<= 1) best = pk_max3(best, (uint32_t)__shfl_xor((int)best, m), best);
    }
    auto out = [&](bool valid, uint32_t pair, uint32_t M, uint32_t N, uint32_t half, bool writer) {
        if (!valid || !writer) return;
        int32_t v = (int32_t)((best >> (16 * half)) & 0xFFFFu) - B;
        if (FR) v -= dl + g * (int32_t)(M + N - 2);   // the frame at (M-1, N-1); SEMI keys: + g*(N-1-c)
        if (M == 0) {
            v = TYPE == NV_SEMI ? (N ? 0 : INT32_MIN)
              : TYPE == NV_GLOBAL ? (N ? (GOTOH ? A.go + A.ge * (int32_t)(N - 1) : A.del * (int32_t)N) : INT32_MIN)
                                  : INT32_MIN;
        } else if (N == 0) v = INT32_MIN;
        if (A.score) A.score[pair] = v;
        if (A.score16) A.score16[pair] = (int16_t)v;
    };
    const bool wa = TYPE == NV_LOCAL ? lg == 0 : BOT ? lg == G - 1 : (Ma ? (Ma - 1) / R == lg : lg == 0);
    const bool wb = TYPE == NV_LOCAL ? lg == 0 : BOT ? lg == G - 1 : (Mb ? (Mb - 1) / R == lg : lg == 0);
    out(va, pa, Ma, Na, 0, wa);
    out(vb, pb, Mb, Nb, 1, wb);
}

}  // namespace gx
