// wavefront.hpp — segmented anti-diagonal DP kernels for gfx950 (CDNA4).
//
// One 64-lane wavefront aligns 64/G pairs.  Each pair owns a group of G
// consecutive lanes; lane lg of the group owns the R consecutive query rows
// [lg*R, lg*R+R) and holds their H/E state (and score keys, and traceback
// words) in VGPRs.  At step s the lane computes column c = s - lg of its rows,
// top to bottom; the bottom row's H and the F leaving it are passed to lane
// lg+1 with one DPP wave_shr:1 each, so the group sweeps the DP matrix as an
// anti-diagonal band.  Targets are staged once per wave in LDS (byte codes);
// each step reads one byte per lane.  No row buffer touches memory.
//
// Semantics are those of the GASAL2 kernels (paths under Non-CDP/GASAL2/src):
//   LOCAL  gasal_local_kernel          kernels/local_kernel_template.h:71-519
//   GLOBAL gasal_global_kernel         kernels/global.h:30-303
//   SEMI   gasal_semi_global_kernel    kernels/semiglobal_kernel_template.h:39-388
// including the quirks listed in SURVEY.md §8 (Q1-Q7, Q9-Q11, Q15).  The
// reference walks the matrix strip-major (8-column strips, then rows, then the
// 8 columns); the first maximum in that order is recovered here from per-row
// keys (score, -column) merged at the end in (strip, row, column) order (Q1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gx {

enum WfAlgo { WF_LOCAL = 0, WF_GLOBAL = 1, WF_SEMI = 2 };

struct WfArgs {
    const uint8_t *q;          // unpacked bytes, or packed words (packed != 0)
    const uint8_t *t;
    const uint32_t *qoff, *toff, *qlen, *tlen;
    int32_t *score, *qend, *tend;
    uint32_t *tb;              // direction words, tb_pair_words per pair
    uint64_t tb_pair_words;
    uint32_t n;
    int32_t a, b, o, e;        // match, mismatch, gap_open, gap_extend
    int32_t nval;              // N_CODE & 0xF
    int32_t has_npen, npen;
    int32_t head, tail;        // semi-global skipped head / tail (enum data_source)
    int32_t packed;
    uint32_t lds_stride;       // bytes of LDS per pair slot (>= max padded target + 4)
    int32_t force_exact;       // always take the exact-N substitution path
    uint32_t one;              // 0x00010001 (opaque to the compiler, see wavefront16.hpp)
    int32_t fast16;            // wavefront16: the value range of the packed path holds (planner)
    int32_t vmin;              // wavefront16 GLOBAL/SEMI: bound on |lowest reachable value| (planner)
    uint8_t *handled;          // wavefront16: per block, 1 = aligned here, 0 = left to the int32 kernel
    const uint8_t *skip;       // int32 kernel: pairs whose packed block already aligned them
    uint32_t skip_ppb;         // pairs per packed block
    int32_t *tbfix;            // wavefront16 GLOBAL+TB: H at the traceback start cell (ql, tl), see tb_kernel
    const uint32_t *perm;      // slot -> pair (pairs sorted by step-axis length, dispatch.hip), or NULL
    uint32_t slot0;            // wavefront16 SEMI TAIL=QUERY/BOTH: first slot of this class launch (n = its end)
    uint32_t tb_q8;            // wavefront16 TB kernels: direction chunks of 8 consecutive pairs interleaved (tb_kernel)
    uint32_t kf16;             // wavefront16 LOCAL: f16-pattern keys over this many columns (0: 16-bit keys H*256 + col)
    const int32_t *stop;       // SEMI TAIL=TARGET reverse pass (start.hpp): per pair, the forward score; the
                               // last-row maximum is then taken inside the first 8-column strip holding a
                               // value >= it (the reference's early exit), else over the whole row
    // GLOBAL + traceback by band recomputation (wavefront16.hpp WF16_GLOBAL_CP, sweep then band pass):
    // per wave, the left-edge state of every lane's band window (cp: [wave][64][2R] words) and the
    // bottom-row hand-off of every lane over the window of the lane below (stm: [wave][wd+1][64]),
    // then the band's direction flags (bflags: [wave][64 lanes][wd/4 windows][R/4] uint4)
    uint32_t *cp;
    uint2 *stm;
    uint4 *bflags;
    uint32_t band_w, band_wd;  // lane lg's window: columns [max(lg*R - band_w, 0), + band_wd), band_wd % 4 == 0
    // a mixed-shape launch (wf16_mix_kernel): the second region's buffers and window width
    uint32_t *cp2;
    uint2 *stm2;
    uint4 *bflags2;
    uint32_t band_wd2;
    const uint32_t *n_dev;     // when set: the launch's pair count is *n_dev (<= n; traceback fallback list)
    uint32_t n_dev_off;        // ... less this offset (the fallback list in chunks of n slots)
    uint32_t tb_slot;          // direction words indexed by slot, not by pair (the capped fallback buffer)
    const int32_t *lstop;      // LOCAL reverse pass of WITH_START (start.hpp): per pair the forward score; the
                               // e-drift sweep stops once every pair's first cell reaching it is settled
    // LOCAL keys by step segments (wavefront16.hpp WF16_LOCAL_SEG): segment j = steps [j*2^kseg_shift,
    // (j+1)*2^kseg_shift); the keys of every finished segment, [wave][segment < kseg_n][64 lanes][R]
    uint32_t *kseg;
    uint32_t kseg_shift, kseg_n;
    // WITH_START reverse pass (start.hpp): the sequences are read backwards in place -- qlen / tlen
    // (per pair) are the reversed lengths L, position p of a reversed sequence is position L-1-p at
    // the pair's offset, positions p >= L are N (nval)
    int32_t rev;
    // rclass.hip: the slots (perm) are sorted longest first by the register-axis words, so a
    // block's first slot is its longest; 0: perm follows another key (block maximum taken)
    int32_t perm_xkey;
    // wavefront16.hpp wf16_mix_kernel: the short shape's first block and slot, its LDS bytes per slot
    uint32_t tail_b0, tail_p0, tail_lds;
    // int32 kernel after a mixed launch: slots from skip_p1 on have their flags from skip_b1 on, one
    // per skip_ppb2 slots (skip_p1 = 0xFFFFFFFF: one flag per skip_ppb slots throughout)
    uint32_t skip_p1, skip_b1, skip_ppb2;
};

// the packed launch's flag covering slot idx (wf16_mix_kernel: two block sizes)
__device__ __forceinline__ uint32_t skip_flag(const WfArgs &A, uint32_t idx) {
    return idx < A.skip_p1 ? idx / A.skip_ppb : A.skip_b1 + (idx - A.skip_p1) / A.skip_ppb2;
}

constexpr int kWavesPerBlock = 4;
constexpr int kBlock = 64 * kWavesPerBlock;
constexpr uint8_t kInvalidCode = 0xFF;

#ifndef GX_DPP_FUSE
#define GX_DPP_FUSE 1   // bound_ctrl hand-offs (no "old" init; a following subtract folds into the DPP op): +0.6 %
#endif
__device__ __forceinline__ int32_t shr_lane(int32_t v) {   // lane i <- lane i-1 (lane 0 <- 0)
    return __builtin_amdgcn_update_dpp(0, v, 0x138 /* wave_shr:1 */, 0xF, 0xF, GX_DPP_FUSE != 0);
}

__device__ __forceinline__ int32_t max3(int32_t a, int32_t b, int32_t c) {
    return max(max(a, b), c);   // -> v_max3_i32
}

template <int G>
__device__ __forceinline__ uint64_t group_max_u64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < G; m <<= 1) {
        uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
        uint32_t olo = __shfl_xor(lo, m), ohi = __shfl_xor(hi, m);
        uint64_t o = ((uint64_t)ohi << 32) | olo;
        v = o > v ? o : v;
    }
    return v;
}

// codes of the 4 bases at padded positions [4w, 4w+4) of a sequence starting at
// byte offset `off`, as 4 bytes (little-endian: byte k = position 4w+k)
__device__ __forceinline__ uint32_t load4_codes(const uint8_t *base, uint32_t off, uint32_t w, int packed) {
    if (!packed) {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(base + off + 4u * w);
        return v & 0x0F0F0F0Fu;
    }
    const uint32_t word = reinterpret_cast<const uint32_t *>(base)[(off >> 3) + (w >> 1)];
    const uint32_t half = (w & 1) ? (word & 0xFFFFu) : (word >> 16);   // 4 nibbles, first in bits 15:12
    return ((half >> 12) & 15u) | (((half >> 8) & 15u) << 8) | (((half >> 4) & 15u) << 16) |
           ((half & 15u) << 24);
}

// the same 4 positions of "the first L bases at `off`, reversed" (start.hpp), N (nval) from L on:
// position p is the original L-1-p, so the 4 bytes are the original [L-4-4w, L-4w) byte-swapped
// (sequences are padded to 8 bytes: every word read lies inside the pair's padded bytes)
__device__ __forceinline__ uint32_t load4_codes_rev(const uint8_t *base, uint32_t off, uint32_t L, uint32_t w,
                                                    int packed, uint32_t nval) {
    const int32_t st = (int32_t)L - 4 - 4 * (int32_t)w;   // original position of byte 3
    if (st <= -4) return nval * 0x01010101u;
    uint32_t x;
    if (!packed) {
        const int32_t a = st >> 2, sh = st & 3;              // floor: a >= -1
        const uint32_t *src = reinterpret_cast<const uint32_t *>(base + off);
        const uint32_t lo = a >= 0 ? src[a] : 0u, hi = sh ? src[a + 1] : 0u;
        x = sh ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)sh) : lo;   // bytes st .. st+3
        x = __builtin_bswap32(x) & 0x0F0F0F0Fu;             // byte j = position st+3-j
    } else {
        x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int32_t q = st + 3 - j;
            if (q >= 0) {
                const uint32_t wd = reinterpret_cast<const uint32_t *>(base)[(off >> 3) + ((uint32_t)q >> 3)];
                x |= ((wd >> (28 - 4 * (q & 7))) & 15u) << (8 * j);
            }
        }
    }
    if (st < 0) {                                            // bytes j >= L - 4w are past the sequence
        const uint32_t keep = L - 4 * w, m = (1u << (8 * keep)) - 1u;
        x = (x & m) | (nval * 0x01010101u & ~m);
    }
    return x;
}
__device__ __forceinline__ uint32_t load4_codes_dir(const WfArgs &A, const uint8_t *base, uint32_t off, uint32_t L,
                                                    uint32_t w) {
    return A.rev ? load4_codes_rev(base, off, L, w, A.packed, (uint32_t)A.nval) : load4_codes(base, off, w, A.packed);
}

template <int ALGO, bool KEYS, bool TB, int G, int R, bool EXACT, bool STOP>
__device__ __forceinline__ void wf_body(const WfArgs &A, const uint8_t *tcodes, const uint32_t lg,
                                        const uint32_t pair, const uint32_t tbi, const bool valid, const uint32_t ql,
                                        const uint32_t tl, const uint32_t qpad, const uint32_t tpad,
                                        const uint32_t nsteps, const uint32_t (&qc)[R], const bool (&qn)[R]) {
    const int32_t OE = A.o + A.e;
    const int32_t ext = A.e;
    const int32_t NS = A.has_npen ? -A.npen : 0;          // score of an N cell (LOCAL rule)
    const bool head_q = (A.head == 1 || A.head == 3);     // QUERY or BOTH
    const bool head_t = (A.head == 2 || A.head == 3);     // TARGET or BOTH
    const uint32_t r0 = lg * R;

    // --- per-row state ---
    int32_t Hk[R];     // LOCAL/GLOBAL: H(r, c-1).  SEMI: H(r, c-1) - OE
    int32_t Ek[R];     // LOCAL/GLOBAL: E(r, c).    SEMI: E(r, c-1)
    int32_t key[R];
    uint32_t dw[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int32_t r = (int32_t)(r0 + k);
        key[k] = INT32_MIN;
        dw[k] = 0;
        if (ALGO == WF_LOCAL) {
            Hk[k] = 0; Ek[k] = 0;                               // local_kernel_template.h:118-120
        } else if (ALGO == WF_GLOBAL) {
            Hk[k] = (r == 0) ? 0 : -(A.o + A.e * r);            // global.h:57-60 (Q2)
            Ek[k] = -32768;
        } else {
            const int32_t h = head_q ? 0 : ((r == 0) ? 0 : -(A.o + A.e * r));   // semiglobal :87-99
            Hk[k] = h - OE;
            Ek[k] = head_q ? 0 : -32768;
        }
    }
    int32_t recvH = 0, prevRecvH = 0, recvF = 0;
    if (ALGO != WF_LOCAL) {
        // the upper lane's bottom row at column -1 (its initial H)
        const int32_t rb = (int32_t)r0 - 1;
        int32_t hb;
        if (ALGO == WF_GLOBAL) hb = (rb <= 0) ? 0 : -(A.o + A.e * rb);
        else hb = (head_q ? 0 : ((rb <= 0) ? 0 : -(A.o + A.e * rb))) - OE;
        recvH = hb; prevRecvH = hb;
    }

    const uint32_t kq_lane = (ql - 1) / R;      // lane holding the last query row
    const uint32_t kq = (ql - 1) - kq_lane * R;
    const int32_t thr = (STOP && valid) ? A.stop[pair] : 0;

    for (uint32_t s = 0; s < nsteps; ++s) {
        const int32_t c = (int32_t)s - (int32_t)lg;
        // inputs arriving from the row above the lane's first row
        int32_t diag, f;
        if (lg == 0) {
            if (ALGO == WF_LOCAL) { diag = 0; f = 0; }                    // p[],f[] reset per strip
            else if (ALGO == WF_GLOBAL) {
                diag = (c <= 0) ? 0 : -(A.o + A.e * c);                    // global.h:70
                f = -32768;                                                // global.h:69
            } else {
                const int32_t hd = head_t ? 0 : ((c <= 0) ? 0 : -(A.o + A.e * c));   // :127 (p[m])
                const int32_t hu = head_t ? 0 : -(A.o + A.e * c);                    // :125 (h[m], Q3)
                diag = hd - OE;
                f = max(hu - OE, -32768 - ext);
            }
        } else {
            diag = prevRecvH;
            f = recvF;
        }
        const bool active = valid && c >= 0 && (uint32_t)c < tpad;
        if (active) {
            const uint32_t tc = tcodes[c];
            const bool tN = (int32_t)tc == A.nval;
            int32_t Mt, Xt;
            if (ALGO == WF_GLOBAL) {
                Mt = (A.has_npen && tN) ? -A.npen : A.a;
                Xt = (A.has_npen && tN) ? -A.npen : -A.b;
            } else {
                Mt = tN ? NS : A.a;
                Xt = tN ? NS : -A.b;
            }
            const int32_t NQ = (ALGO == WF_GLOBAL) ? -A.npen : NS;
            if (ALGO == WF_SEMI) { Mt += OE; Xt += OE; }
            int32_t Cc = 0;
            if (KEYS) {
                const bool in_t = (ALGO == WF_LOCAL) ? true : ((uint32_t)c < tl);
                Cc = (in_t ? (1 << 30) : -(1 << 30)) + (32767 - c);
            }
#pragma unroll
            for (int k = 0; k < R; ++k) {
                int32_t sc = (qc[k] == tc) ? Mt : Xt;
                if (EXACT && (ALGO != WF_GLOBAL || A.has_npen)) sc = qn[k] ? (ALGO == WF_SEMI ? NQ + OE : NQ) : sc;
                if (ALGO == WF_SEMI) {
                    // CORE_COMPUTE_SEMIGLOBAL (semiglobal_kernel_template.h:17-28)
                    const int32_t E = max(Hk[k], Ek[k] - ext);          // E(r,c)
                    const int32_t tmp = diag + sc;                       // H(r-1,c-1) + s
                    const int32_t H = max3(tmp, f, E);
                    Ek[k] = E;
                    diag = Hk[k];
                    Hk[k] = H - OE;
                    f = max(Hk[k], f - ext);                             // F(r+1,c)
                    if (STOP) {
                        // cells >= thr rank first: smallest strip, then largest H, then first
                        // column; the others by (H, first column); columns >= tl never
                        const int32_t kv = (uint32_t)c >= tl ? INT32_MIN
                                         : H >= thr ? (0x40000000 | ((1023 - (c >> 3)) << 19) | ((H - thr) << 3) |
                                                       (7 - (c & 7)))
                                                    : H * 16384 + (16383 - c);
                        key[k] = max(key[k], kv);
                    } else if (KEYS) key[k] = max(key[k], H * 32768 + Cc);
                } else {
                    // CORE_LOCAL_COMPUTE / CORE_GLOBAL_COMPUTE (local :19-30, global.h:4-12)
                    const int32_t tmp = diag + sc;
                    int32_t H = max3(tmp, f, Ek[k]);
                    if (ALGO == WF_LOCAL) H = max(H, 0);
                    const int32_t toe = tmp - OE;
                    const int32_t fm = f - ext;
                    const int32_t em = Ek[k] - ext;
                    if (TB) {
                        // direction nibble (local :49-56, global.h:18-25)
                        const uint32_t mx_ = (tmp >= diag) ? 0u : 1u;
                        uint32_t nib = (H == tmp) ? mx_ : ((H == f) ? 3u : 2u);
                        nib |= (toe > fm) ? 0u : 8u;
                        nib |= (toe > em) ? 0u : 4u;
                        dw[k] = (dw[k] << 4) | nib;
                    }
                    Ek[k] = max(toe, em);
                    f = max(toe, fm);
                    diag = Hk[k];
                    Hk[k] = H;
                    if (KEYS) key[k] = max(key[k], H * 32768 + Cc);
                }
            }
            if (TB && ((c & 7) == 7)) {
                uint32_t *dst = A.tb + (uint64_t)tbi * A.tb_pair_words + (uint64_t)(c >> 3) * qpad + r0;   // tbi: pair or slot
#pragma unroll
                for (int k = 0; k < R; k += 4) {
                    if (r0 + k < qpad) {
                        *reinterpret_cast<uint4 *>(dst + k) = make_uint4(dw[k], dw[k + 1], dw[k + 2], dw[k + 3]);
                    }
                }
            }
            if (ALGO == WF_GLOBAL && (uint32_t)c == tl - 1 && lg == kq_lane) {
                int32_t h = 0;
#pragma unroll
                for (int k = 0; k < R; ++k) h = (k == (int)kq) ? Hk[k] : h;
                A.score[pair] = h;                                  // global.h:98-103,299
            }
        }
        // hand the bottom row to the lane below
        prevRecvH = recvH;
        recvH = shr_lane(Hk[R - 1]);
        recvF = shr_lane(f);
    }

    // ---------------- results ----------------
    if (ALGO == WF_LOCAL) {
        // strip-major first maximum (Q1): per row (H, first column) -> order key
        uint64_t best = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint32_t r = r0 + k;
            if (r < qpad && key[k] >= 0) {
                const int32_t H = (key[k] >> 15) - 32768;
                const uint32_t col = 32767u - ((uint32_t)key[k] & 0x7FFFu);
                const uint32_t ord = (((col >> 3) * qpad + r) << 3) + (col & 7);
                const uint64_t cand = ((uint64_t)(uint32_t)(H + (1 << 20)) << 32) | (0xFFFFFFFFu - ord);
                best = cand > best ? cand : best;
            }
        }
        best = group_max_u64<G>(best);
        if (valid && lg == 0) {
            int32_t H = (int32_t)(best >> 32) - (1 << 20);
            uint32_t ord = 0xFFFFFFFFu - (uint32_t)best;
            int32_t qe = 0, te = 0;
            if (best == 0 || H <= 0) { H = 0; }
            else {
                const uint32_t col8 = ord & 7, rest = ord >> 3;
                qe = (int32_t)(rest % qpad);
                te = (int32_t)((rest / qpad) * 8 + col8);
            }
            A.score[pair] = H;                                       // local :428-430
            if (A.qend) A.qend[pair] = qe;
            if (A.tend) A.tend[pair] = te;
        }
    } else if (ALGO == WF_SEMI) {
        const bool tail_t = (A.tail == 2 || A.tail == 3);
        const bool tail_q = (A.tail == 1 || A.tail == 3);
        // TAIL TARGET: row ql-1, columns < tl, first max (semiglobal :160-178)
        uint64_t bt = 0;
        if (KEYS && lg == kq_lane) {
            int32_t kk = INT32_MIN;
#pragma unroll
            for (int k = 0; k < R; ++k) kk = (k == (int)kq) ? key[k] : kk;
            if (STOP) { if (kk != INT32_MIN) bt = (uint64_t)((uint32_t)kk ^ 0x80000000u) | (1ull << 40); }
            else if (kk >= 0) bt = ((uint64_t)(uint32_t)kk) | (1ull << 40);
        }
        // TAIL QUERY: H at the last padded column, rows < ql, first max (:185-193)
        uint64_t bq = 0;
        if (tail_q) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const uint32_t r = r0 + k;
                if (r < ql) {
                    const int32_t v = (int16_t)(Hk[k] + OE);          // short2 row buffer (Q5)
                    const uint64_t cand = ((uint64_t)(uint32_t)(v + (1 << 20)) << 32) | (0xFFFFFFFFu - r);
                    bq = cand > bq ? cand : bq;
                }
            }
        }
        bt = group_max_u64<G>(bt);
        bq = group_max_u64<G>(bq);
        if (valid && lg == 0) {
            int32_t maxHH = -32768, maxX = (int32_t)tl, maxY = (int32_t)ql;   // :49,63-64 (Q10)
            if (STOP && bt != 0) {
                const int32_t kk = (int32_t)((uint32_t)bt ^ 0x80000000u);
                int32_t H, col;
                if (kk >= 0x40000000) {
                    col = 8 * (1023 - ((kk >> 19) & 1023)) + 7 - (kk & 7);
                    H = thr + ((kk >> 3) & 0xFFFF);
                } else {
                    H = kk >> 14;                                   // floor: 16383 - c in [0, 16384)
                    col = 16383 - (kk & 16383);
                }
                maxHH = H; maxY = col;
            } else if (tail_t && bt != 0) {
                const uint32_t kk = (uint32_t)bt;
                const int32_t H = (int32_t)(kk >> 15) - 32768;
                const int32_t col = 32767 - (int32_t)(kk & 0x7FFFu);
                if (H > maxHH) { maxHH = H; maxY = col; }
            }
            if (tail_q) {
                if (bq != 0) {
                    const int32_t v = (int32_t)(bq >> 32) - (1 << 20);
                    const int32_t r = (int32_t)(0xFFFFFFFFu - (uint32_t)bq);
                    if (v > maxHH) { maxHH = v; maxX = r; }
                }
                if (maxX != (int32_t)tl) maxY = (int32_t)ql;               // :206-207
            }
            A.score[pair] = maxHH;
            if (A.qend) A.qend[pair] = maxX;
            if (A.tend) A.tend[pair] = maxY;
        }
    }
}

// One block's pairs (virtual block bx) of the int32 kernel.
template <int ALGO, bool KEYS, bool TB, int G, int R, bool STOP>
__device__ __forceinline__ void wf_block(const WfArgs &A, uint8_t *lds, const uint32_t bx) {
    constexpr int P = 64 / G;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1);
    const uint32_t slot = lane / G;
    const uint32_t pair0 = (bx * kWavesPerBlock + wave) * P;
    const uint32_t idx = pair0 + slot;   // slot; the pair is perm[slot] when sorted
    // pairs the packed kernel already aligned are skipped (dispatch.hip); its flags are per block of slots
    // (traceback fallback: a device-side count, less the chunk's offset)
    const uint32_t nn = A.n_dev ? min(*A.n_dev > A.n_dev_off ? *A.n_dev - A.n_dev_off : 0u, A.n) : A.n;
    const bool valid = idx < nn && !(A.skip && A.skip[skip_flag(A, idx)]);
    const uint32_t pair = (valid && A.perm) ? A.perm[idx] : idx;
    if (A.skip && !__syncthreads_or(valid)) return;      // block-uniform early exit

    uint32_t ql = 0, tl = 0, qo = 0, to = 0;
    if (valid) { ql = A.qlen[pair]; tl = A.tlen[pair]; qo = A.qoff[pair]; to = A.toff[pair]; }
    const uint32_t qpad = (ql + 7u) & ~7u;
    const uint32_t tpad = (tl + 7u) & ~7u;

    // ---- stage the wave's P targets as byte codes in LDS ----
    const uint32_t stride = A.lds_stride;
    uint8_t *wlds = lds + (size_t)wave * P * stride;
    const uint32_t words = stride >> 2;
    for (uint32_t base = 0; base < P * words; base += 64) {   // uniform trip count: shuffles see all lanes
        const uint32_t idx = base + lane;
        const uint32_t ps = min(idx / words, (uint32_t)P - 1), w = idx - ps * words;
        const uint32_t src_lane = ps * G;
        const uint32_t ptp = __shfl(tpad, src_lane);
        const uint32_t pto = __shfl(to, src_lane);
        const uint32_t ptl = __shfl(tl, src_lane);
        if (idx < P * words) {
            uint32_t v = 0xFFFFFFFFu;
            if (4u * w < ptp) v = load4_codes_dir(A, A.t, pto, ptl, w);
            reinterpret_cast<uint32_t *>(wlds + ps * stride)[w] = v;
        }
    }
    __syncthreads();

    // ---- the lane's query rows ----
    uint32_t qc[R];
    bool qn[R];
    bool has_n = false;
    const uint32_t r0 = lg * R;
#pragma unroll
    for (int k = 0; k < R; k += 4) {
        uint32_t v = 0xFFFFFFFFu;
        if (valid && r0 + k < qpad) v = load4_codes_dir(A, A.q, qo, ql, (r0 + k) >> 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            qc[k + j] = (v >> (8 * j)) & 0xFFu;
            qn[k + j] = ((int32_t)qc[k + j] == A.nval);
            if (r0 + k + j < ql && qn[k + j]) has_n = true;
        }
    }
    // steps: widest padded target of the wave + lanes of the group - 1
    uint32_t tmaxw = tpad;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) tmaxw = max(tmaxw, (uint32_t)__shfl_xor(tmaxw, m));
    const uint32_t nsteps = tmaxw + G - 1;
    const uint8_t *tcodes = wlds + slot * stride;

    // exact substitution only when a real query N could change a pad-free cell
    bool exact = A.force_exact != 0;
    if (ALGO != WF_GLOBAL || A.has_npen) exact = exact || __any(has_n);
    if (exact)
        wf_body<ALGO, KEYS, TB, G, R, true, STOP>(A, tcodes, lg, pair, A.tb_slot ? idx : pair, valid, ql, tl, qpad, tpad,
                                                 nsteps, qc, qn);
    else
        wf_body<ALGO, KEYS, TB, G, R, false, STOP>(A, tcodes, lg, pair, A.tb_slot ? idx : pair, valid, ql, tl, qpad, tpad,
                                                 nsteps, qc, qn);
}

// As the fallback of a packed launch (A.skip) the grid is capped (dispatch.hip wf_grid) and each
// block walks the virtual blocks bx, bx + gridDim.x, ...: a batch the packed kernel took whole
// then costs a few flag reads per block instead of a full grid of early exits.  The flags of 64
// of its virtual blocks are read at once, one per lane, and only those holding a declined pair
// are run (one flag read per virtual block in turn cost 32 us per 1 M config-2 pairs and 0.44 ms
// per 10 M config-4 pairs: a chain of dependent loads).  Every wave reads the same flags, so the
// loop is block-uniform; each wave stages into its own LDS region, so consecutive virtual blocks
// need no barrier between them beyond those of the body.
template <int ALGO, bool KEYS, bool TB, int G, int R, bool STOP = false>
__global__ __launch_bounds__(kBlock) void wf_kernel(WfArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr uint32_t PPB = kWavesPerBlock * (64 / G);
    const uint32_t nblk = (A.n + PPB - 1) / PPB;
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x; base < nblk; base += 64 * gridDim.x) {
        const uint32_t bx = base + lane * gridDim.x;
        bool run = bx < nblk;
        if (run && A.skip) {   // a declined pair: some flag over its slots is clear
            const uint32_t f0 = skip_flag(A, bx * PPB), f1 = skip_flag(A, min(bx * PPB + PPB, A.n) - 1);
            bool all = true;
            for (uint32_t f = f0; f <= f1; ++f) all &= A.skip[f] != 0;
            run = !all;
        }
        for (uint64_t m = __ballot(run); m; m &= m - 1)
            wf_block<ALGO, KEYS, TB, G, R, STOP>(A, lds, base + (uint32_t)__builtin_ctzll(m) * gridDim.x);
    }
}

}  // namespace gx
