// batched.hip — launcher of the nvbio-style batched scoring front-end (nvbio.hpp).
// Replaces BatchedAlignmentScore<stream, scheduler>::enact (NvB/nvbio/alignment/
// batched_inl.h) and the scheduler tags (batched.h:44-87): every scheduler maps to
// the same lane-group wavefront launch; there is no temporary storage.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "engine.hpp"
#include "nvbio.hpp"
#include "nvtrace.hpp"
#include "nvbio16.hpp"
#include "nvbanded.hpp"

namespace gx {

namespace {

struct NvShape { int G, R; };
// the smallest G*R >= the longest pattern: 150-bp reads take (8, 19), 152 rows
constexpr NvShape kNvShapes[] = {{8, 8}, {8, 12}, {8, 16}, {8, 19}, {8, 24}, {16, 16}, {16, 20}, {32, 16}, {64, 16}};

using NvFn = void (*)(NvArgs);

template <int ALN, int TYPE, bool MASK>
NvFn nv_pick(int G, int R) {
#define GX_CASE(g, r) if (G == g && R == r) return &nv_kernel<ALN, TYPE, g, r, MASK>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 19) GX_CASE(8, 24) GX_CASE(16, 16) GX_CASE(16, 20)
    GX_CASE(32, 16) GX_CASE(64, 16)
#undef GX_CASE
    return nullptr;
}

using Nv16Fn = void (*)(Nv16Args);
template <int ALN, int TYPE, bool SHARED>
Nv16Fn nv16_pick(int G, int R) {
#define GX_CASE(g, r) if (G == g && R == r) return &nv16_kernel<ALN, TYPE, g, r, SHARED>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 19) GX_CASE(8, 24) GX_CASE(16, 16) GX_CASE(16, 20)
    GX_CASE(32, 16) GX_CASE(64, 16)
#undef GX_CASE
    return nullptr;
}
template <int ALN, bool SHARED>
Nv16Fn nv16_lookup_t(int type, int G, int R) {
    return type == NV_GLOBAL ? nv16_pick<ALN, NV_GLOBAL, SHARED>(G, R)
         : type == NV_SEMI ? nv16_pick<ALN, NV_SEMI, SHARED>(G, R) : nv16_pick<ALN, NV_LOCAL, SHARED>(G, R);
}
Nv16Fn nv16_lookup(int aln, int type, bool shared, int G, int R) {
    if (shared)
        return aln == NV_GOTOH ? nv16_lookup_t<NV_GOTOH, true>(type, G, R) : nv16_lookup_t<NV_SW, true>(type, G, R);
    return aln == NV_GOTOH ? nv16_lookup_t<NV_GOTOH, false>(type, G, R) : nv16_lookup_t<NV_SW, false>(type, G, R);
}
// LDS of the packed kernel: one table per column of the shared text, or of every
// pair's text (two pairs per lane group, 4 waves per block)
uint32_t nv16_cols(bool shared, uint32_t max_t, int G) { return shared ? (max_t + G + 63u) & ~63u : (max_t + 3u) & ~3u; }
size_t nv16_lds(bool shared, uint32_t max_t, int G) {
    return (size_t)nv16_cols(shared, max_t, G) * 4 * (shared ? 1 : 4 * 2 * (64 / G));
}

// The packed kernel (nvbio16.hpp): 2-bit texts, gaps and (LOCAL) mismatches <= 0,
// match - mismatch in a byte, and every value (bounded by (M + N + 2) * the largest
// score magnitude) inside the 16-bit f16 window.  GASALX_NV16=0: int32 only.
bool nv16_ok(int aligner, int type, int32_t match, int32_t mismatch, int32_t go, int32_t ge, int32_t del, int32_t ins,
             bool shared_text, uint32_t text_bits, uint32_t max_p, uint32_t max_t, uint32_t *base) {
    const char *env = std::getenv("GASALX_NV16");
    if (env && std::atoi(env) == 0) return false;
    (void)shared_text;
    if (text_bits != 2) return false;
    if (match < mismatch || match - mismatch > 255) return false;
    if (aligner == NV_GOTOH ? (go > 0 || ge > 0) : (del > 0 || ins > 0)) return false;
    if (mismatch > 0 || mismatch < -255) return false;   // virtual rows score the byte |mismatch|
    const int64_t mag = std::max<int64_t>({std::abs((int64_t)match), std::abs((int64_t)mismatch), std::abs((int64_t)go),
                                           std::abs((int64_t)ge), std::abs((int64_t)del), std::abs((int64_t)ins), 1});
    if (mag > 0x200) return false;   // a gap subtracted from NEG must not borrow across the halves
    const int64_t vabs = ((int64_t)max_p + max_t + 2) * mag * 2;
    if (aligner == NV_GOTOH && type != NV_LOCAL) {
        // the drift frame (nvbio16.hpp FR): values + g*(r+c) + (go - ge) lie within the
        // all-gap path below and the diagonal above; virtual rows (r >= -G*R, G*R <=
        // 2*max_p + 64) fall by g per row, sink keys add up to g*max_t
        const int64_t g = -(int64_t)ge, gr = 2 * (int64_t)max_p + 64;
        const int64_t b = 0x400 + g * (gr + 2) + 4 * (std::abs((int64_t)go) + g) + 64;
        const int64_t top = b + std::abs((int64_t)go - ge) + std::max<int64_t>(match, 0) * max_p +
                            g * ((int64_t)max_p + 2 * (int64_t)max_t + 4) + 512;
        if (top > 0x7BFF) return false;
        *base = (uint32_t)b;
        return true;
    }
    const int64_t b = 0x400 + 2 * (std::abs((int64_t)go) + std::abs((int64_t)ge) + std::abs((int64_t)del) +
                                   std::abs((int64_t)ins)) + vabs + 64;
    if (b + vabs + 512 > 0x7BFF) return false;
    *base = (uint32_t)b;
    return true;
}

NvFn nv_lookup(bool gotoh, int type, bool mask, int G, int R) {
    if (gotoh) {
        if (type == NV_GLOBAL) return nv_pick<NV_GOTOH, NV_GLOBAL, false>(G, R);
        if (type == NV_SEMI) return nv_pick<NV_GOTOH, NV_SEMI, false>(G, R);
        return mask ? nv_pick<NV_GOTOH, NV_LOCAL, true>(G, R) : nv_pick<NV_GOTOH, NV_LOCAL, false>(G, R);
    }
    if (type == NV_GLOBAL) return nv_pick<NV_SW, NV_GLOBAL, false>(G, R);
    if (type == NV_SEMI) return nv_pick<NV_SW, NV_SEMI, false>(G, R);
    return mask ? nv_pick<NV_SW, NV_LOCAL, true>(G, R) : nv_pick<NV_SW, NV_LOCAL, false>(G, R);
}

// the lane-group shape for patterns up to max_p: the smallest G*R that covers them
// whose text slots fit in LDS (one shared slot, or one per pair)
const NvShape *nv_shape(uint32_t max_p, uint32_t stride, bool per_pair_text, size_t *lds_out) {
    for (const NvShape &sh : kNvShapes) {
        if ((uint32_t)(sh.G * sh.R) < max_p) continue;
        const size_t lds = per_pair_text ? (size_t)4 * (64 / sh.G) * stride * 2 : (size_t)stride * 2;
        if (lds > 160 * 1024) continue;
        *lds_out = lds;
        return &sh;
    }
    return nullptr;
}

}  // namespace

std::string nv_plan_name(const gasalx_nv_aligner &al, uint32_t max_p, uint32_t max_t, bool per_pair_text,
                         uint32_t text_bits) {
    static const char *an[] = {"ed", "sw", "gotoh"}, *tn[] = {"global", "local", "semi"};
    if (al.aligner < 0 || al.aligner > 2 || al.type < 0 || al.type > 2) return "none";
    size_t lds = 0;
    const NvShape *sh = nv_shape(max_p, (std::max<uint32_t>(max_t, 1) + 7u) & ~7u, per_pair_text, &lds);
    if (!sh) return "none";
    const bool ed = al.aligner == NV_ED;
    uint32_t base = 0;
    const bool pk = nv16_ok(ed ? NV_SW : al.aligner, al.type, ed ? 0 : al.match, ed ? -1 : al.mismatch, al.gap_open,
                            al.gap_ext, ed ? -1 : al.deletion, ed ? -1 : al.insertion, !per_pair_text, text_bits, max_p,
                            max_t, &base);
    const bool fits = nv16_lds(!per_pair_text, max_t, sh->G) <= 160 * 1024;
    return std::string(pk && fits ? "nvbio16_" : "nvbio_") + an[al.aligner] + "_" + tn[al.type] + (per_pair_text ? "" : "_shared") +
           "_G" + std::to_string(sh->G) + "R" + std::to_string(sh->R);
}

int nv_score_device(const gasalx_nv_aligner &al, uint32_t n, const gasalx_nv_strings &pat,
                    const gasalx_nv_strings &txt, int32_t *scores, int16_t *scores16, uint32_t max_p, uint32_t max_t,
                    hipStream_t st) {
    if (n == 0) return GASALX_OK;
    if (al.aligner < 0 || al.aligner > 2 || al.type < 0 || al.type > 2) { set_error("bad aligner"); return GASALX_EINVAL; }
    for (uint32_t b : {pat.bits, txt.bits})
        if (b != 2 && b != 4 && b != 8) { set_error("symbol bits must be 2, 4 or 8"); return GASALX_EINVAL; }
    if (!pat.words || !pat.offsets || !txt.words || (!scores && !scores16)) { set_error("null argument"); return GASALX_EINVAL; }
    NvArgs A;
    A.pw = pat.words; A.poff = pat.offsets; A.pbits = pat.bits; A.pbig = pat.big_endian;
    A.tw = txt.words; A.toff = txt.offsets; A.tbits = txt.bits; A.tbig = txt.big_endian;
    A.tlen0 = txt.offsets ? 0 : txt.length;
    if (!txt.offsets) max_t = txt.length;
    A.score = scores; A.score16 = scores16; A.n = n;
    const bool gotoh = al.aligner == NV_GOTOH;
    if (al.aligner == NV_ED) { A.match = 0; A.mismatch = -1; A.del = -1; A.ins = -1; }   // ed_utils.h:45-52
    else { A.match = al.match; A.mismatch = al.mismatch; A.del = al.deletion; A.ins = al.insertion; }
    A.go = al.gap_open; A.ge = al.gap_ext;
    // |values| stay far from the -inf stand-in (nvbio's infimum never wins either)
    int64_t mag = std::max<int64_t>({std::abs((int64_t)A.match), std::abs((int64_t)A.mismatch),
                                     std::abs((int64_t)A.go), std::abs((int64_t)A.ge), std::abs((int64_t)A.del),
                                     std::abs((int64_t)A.ins), 1});
    if ((int64_t)(max_p + max_t + 2) * mag * 2 >= (1ll << 28)) { set_error("scores out of the exact range"); return GASALX_ERANGE; }
    // LOCAL pads (pattern rows >= M, text columns >= N) never exceed a real cell when no
    // step can raise a score without a match; otherwise mask them
    const bool mask = al.type == NV_LOCAL &&
                      (A.mismatch > 0 || (gotoh ? (A.go > 0 || A.ge > 0) : (A.del > 0 || A.ins > 0)));
    const uint32_t stride = (std::max<uint32_t>(max_t, 1) + 7u) & ~7u;
    size_t lds = 0;
    const NvShape *sh = nv_shape(max_p, stride, txt.offsets != nullptr, &lds);
    uint32_t base = 0;
    if (sh && nv16_ok(gotoh ? NV_GOTOH : NV_SW, al.type, A.match, A.mismatch, A.go, A.ge, A.del, A.ins, !txt.offsets,
                      txt.bits, max_p, max_t, &base)) {
        const bool shared = !txt.offsets;
        Nv16Fn fn = nv16_lookup(gotoh ? NV_GOTOH : NV_SW, al.type, shared, sh->G, sh->R);
        if (fn) {
            Nv16Args D;
            D.pw = A.pw; D.poff = A.poff; D.pbits = A.pbits; D.pbig = A.pbig;
            D.tw = A.tw; D.toff = A.toff; D.tbig = A.tbig; D.tlen0 = A.tlen0;
            D.score = scores; D.score16 = scores16; D.n = n;
            D.match = A.match; D.mismatch = A.mismatch; D.go = A.go; D.ge = A.ge; D.del = A.del; D.ins = A.ins;
            D.base = base;
            D.lds_cols = nv16_cols(shared, shared ? A.tlen0 : max_t, sh->G);
            const size_t lds16 = nv16_lds(shared, shared ? A.tlen0 : max_t, sh->G);
            if (lds16 <= 160 * 1024) {
                if (lds16 > 64 * 1024) {
                    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)lds16);
                    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
                }
                const uint32_t per_block = 8 * (64 / sh->G);   // two pairs per lane group
                hipLaunchKernelGGL(fn, dim3((n + per_block - 1) / per_block), dim3(256), lds16, st, D);
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
                return GASALX_OK;
            }
        }
    }
    NvFn fn = sh ? nv_lookup(gotoh, al.type, mask, sh->G, sh->R) : nullptr;
    if (fn) {
        A.lds_stride = stride;
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
        }
        const uint32_t per_block = 4 * (64 / sh->G);
        hipLaunchKernelGGL(fn, dim3((n + per_block - 1) / per_block), dim3(256), lds, st, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
        return GASALX_OK;
    }
    set_error("pattern longer than 1024 or text too long for LDS (" + std::to_string(max_p) + ", " +
              std::to_string(max_t) + ")");
    return GASALX_ERANGE;
}

// ---- BatchedBandedAlignmentScore<band> (nvbanded.hpp): thread per pair, band in registers,
//      instances for bands up to 8, 16 and 32 ----
namespace {
using NvBandFn = void (*)(NvBandArgs);
template <int ALN, int TYPE>
NvBandFn nv_band_pick(uint32_t band) {
    switch (band) {
        case 8: return &nv_banded_kernel<ALN, TYPE, 8, true>;
        case 16: return &nv_banded_kernel<ALN, TYPE, 16, true>;
        case 32: return &nv_banded_kernel<ALN, TYPE, 32, true>;
        default: break;
    }
    if (band <= 8) return &nv_banded_kernel<ALN, TYPE, 8>;
    if (band <= 16) return &nv_banded_kernel<ALN, TYPE, 16>;
    if (band <= 32) return &nv_banded_kernel<ALN, TYPE, 32>;
    return nullptr;
}
template <int ALN>
NvBandFn nv_band_lookup_t(int type, uint32_t band) {
    return type == NV_GLOBAL ? nv_band_pick<ALN, NV_GLOBAL>(band)
         : type == NV_SEMI ? nv_band_pick<ALN, NV_SEMI>(band) : nv_band_pick<ALN, NV_LOCAL>(band);
}
using NvBand16Fn = void (*)(NvBand16Args);
template <int ALN, int TYPE>
NvBand16Fn nv_band16_pick(uint32_t band) {
    switch (band) {   // band lengths of an instance's own size: the slot tests fold
        case 8: return &nv_banded16_kernel<ALN, TYPE, 8, true>;
        case 16: return &nv_banded16_kernel<ALN, TYPE, 16, true>;
        case 32: return &nv_banded16_kernel<ALN, TYPE, 32, true>;
        default: break;
    }
    if (band <= 8) return &nv_banded16_kernel<ALN, TYPE, 8>;
    if (band <= 16) return &nv_banded16_kernel<ALN, TYPE, 16>;
    if (band <= 32) return &nv_banded16_kernel<ALN, TYPE, 32>;
    return nullptr;
}
template <int ALN>
NvBand16Fn nv_band16_lookup_t(int type, uint32_t band) {
    return type == NV_GLOBAL ? nv_band16_pick<ALN, NV_GLOBAL>(band)
         : type == NV_SEMI ? nv_band16_pick<ALN, NV_SEMI>(band) : nv_band16_pick<ALN, NV_LOCAL>(band);
}
// the packed banded kernel: 2-bit texts, gaps <= 0, match - mismatch in a byte, every
// value (bounded by (M + band + 2) * the largest score magnitude) inside the 16-bit f16
// window (as nv16_ok); GASALX_NVB16=0: int32 only
bool nvb16_ok(int32_t match, int32_t mismatch, int32_t go, int32_t ge, int32_t del, int32_t ins, uint32_t text_bits,
              uint32_t max_p, uint32_t band, uint32_t *base) {
    const char *env = std::getenv("GASALX_NVB16");
    if (env && std::atoi(env) == 0) return false;
    if (text_bits != 2) return false;
    if (match < mismatch || match - mismatch > 255) return false;
    if (go > 0 || ge > 0 || del > 0 || ins > 0) return false;
    const int64_t mag = std::max<int64_t>({std::abs((int64_t)match), std::abs((int64_t)mismatch), std::abs((int64_t)go),
                                           std::abs((int64_t)ge), std::abs((int64_t)del), std::abs((int64_t)ins), 1});
    if (mag > 0x200) return false;
    const int64_t vabs = ((int64_t)max_p + band + 2) * mag * 2;
    const int64_t b = 0x400 + 2 * (std::abs((int64_t)go) + std::abs((int64_t)ge) + std::abs((int64_t)del) +
                                   std::abs((int64_t)ins)) + vabs + 64;
    if (b + vabs + 512 > 0x7BFF) return false;
    *base = (uint32_t)b;
    return true;
}
}  // namespace

int nv_banded_score_device(const gasalx_nv_aligner &al, uint32_t band, uint32_t n, const gasalx_nv_strings &pat,
                           const gasalx_nv_strings &txt, int32_t *scores, hipStream_t st, uint32_t max_p) {
    if (al.aligner < 0 || al.aligner > 2 || al.type < 0 || al.type > 2) { set_error("bad aligner"); return GASALX_EINVAL; }
    if (band < 2 || band > 32) { set_error("band length must be 2..32"); return GASALX_EINVAL; }
    for (uint32_t b : {pat.bits, txt.bits})
        if (b != 2 && b != 4 && b != 8) { set_error("symbol bits must be 2, 4 or 8"); return GASALX_EINVAL; }
    if (n == 0) return GASALX_OK;
    if (!pat.words || !pat.offsets || !txt.words || !scores) { set_error("null argument"); return GASALX_EINVAL; }
    NvBandArgs A;
    A.pw = pat.words; A.poff = pat.offsets; A.pbits = pat.bits; A.pbig = pat.big_endian;
    A.tw = txt.words; A.toff = txt.offsets; A.tbits = txt.bits; A.tbig = txt.big_endian;
    A.tlen0 = txt.offsets ? 0 : txt.length;
    A.score = scores; A.n = n; A.band = band;
    if (al.aligner == NV_ED) { A.match = 0; A.mismatch = -1; A.del = -1; A.ins = -1; }   // ed_banded_inl.h:63-78
    else { A.match = al.match; A.mismatch = al.mismatch; A.del = al.deletion; A.ins = al.insertion; }
    A.go = al.gap_open; A.ge = al.gap_ext;
    uint32_t base = 0;
    if (max_p && nvb16_ok(A.match, A.mismatch, A.go, A.ge, A.del, A.ins, txt.bits, max_p, band, &base)) {
        NvBand16Args D;
        D.pw = A.pw; D.poff = A.poff; D.pbits = A.pbits; D.pbig = A.pbig;
        D.tw = A.tw; D.toff = A.toff; D.tbig = A.tbig; D.tlen0 = A.tlen0;
        D.score = scores; D.n = n; D.n_lanes = (n + 1) / 2; D.band = band;
        D.match = A.match; D.mismatch = A.mismatch; D.go = A.go; D.ge = A.ge; D.del = A.del; D.ins = A.ins;
        D.base = base;
        NvBand16Fn f16 = al.aligner == NV_GOTOH ? nv_band16_lookup_t<NV_GOTOH>(al.type, band)
                                                : nv_band16_lookup_t<NV_SW>(al.type, band);
        hipLaunchKernelGGL(f16, dim3((D.n_lanes + 255) / 256), dim3(256), 0, st, D);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
        return GASALX_OK;
    }
    NvBandFn fn = al.aligner == NV_GOTOH ? nv_band_lookup_t<NV_GOTOH>(al.type, band) : nv_band_lookup_t<NV_SW>(al.type, band);
    hipLaunchKernelGGL(fn, dim3((n + 255) / 256), dim3(256), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
    return GASALX_OK;
}


// nvbio BatchedAlignmentTraceback (nvtrace.hpp): one pair per thread, flags and the previous row in
// the caller's workspace (dir: pad8(max_p) * max_t bytes per pair, row: max_t int2 per pair)
int nv_traceback_device(const gasalx_nv_aligner &al, uint32_t n, const gasalx_nv_strings &pat,
                        const gasalx_nv_strings &txt, uint32_t max_p, uint32_t max_t, uint8_t *dir, int32_t *row,
                        int32_t *score, uint32_t *src, uint32_t *snk, uint8_t *ops, uint32_t ops_stride,
                        uint32_t *n_ops, hipStream_t st) {
    if (al.aligner != NV_GOTOH && al.aligner != NV_SW && al.aligner != NV_ED) {
        set_error("traceback: unknown aligner");
        return GASALX_EINVAL;
    }
    if (al.type < 0 || al.type > 2) { set_error("bad alignment type"); return GASALX_EINVAL; }
    for (uint32_t b : {pat.bits, txt.bits})
        if (b != 2 && b != 4 && b != 8) { set_error("symbol bits must be 2, 4 or 8"); return GASALX_EINVAL; }
    if (n == 0) return GASALX_OK;
    if (!pat.words || !pat.offsets || !txt.words || !score || !src || !snk || !ops || !n_ops || !dir || !row) {
        set_error("null argument");
        return GASALX_EINVAL;
    }
    NvTbArgs A;
    A.pw = pat.words; A.poff = pat.offsets; A.pbits = pat.bits; A.pbig = pat.big_endian;
    A.tw = txt.words; A.toff = txt.offsets; A.tlen0 = txt.offsets ? 0 : txt.length; A.tbits = txt.bits;
    A.tbig = txt.big_endian;
    A.match = al.match; A.mismatch = al.mismatch; A.go = al.gap_open; A.ge = al.gap_ext;
    A.del = al.deletion; A.ins = al.insertion;
    if (al.aligner == NV_ED) { A.match = 0; A.mismatch = -1; A.del = -1; A.ins = -1; }   // ed_inl.h:347-365
    A.n = n; A.max_m = max_p; A.max_n = max_t;
    A.dir = dir; A.row = row; A.score = score; A.src = src; A.snk = snk; A.ops = ops; A.ops_stride = ops_stride;
    A.n_ops = n_ops;
    using Fn = void (*)(NvTbArgs);
    static const Fn tab[2][3] = {{&nv_traceback_kernel<false, 0>, &nv_traceback_kernel<false, 1>, &nv_traceback_kernel<false, 2>},
                                 {&nv_traceback_kernel<true, 0>, &nv_traceback_kernel<true, 1>, &nv_traceback_kernel<true, 2>}};
    hipLaunchKernelGGL(tab[al.aligner == NV_GOTOH ? 1 : 0][al.type], dim3((n + 255) / 256), dim3(256), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
    return GASALX_OK;
}

// BatchedBandedAlignmentTraceback<band> (nvtrace.hpp nv_banded_traceback_kernel); ED runs as
// SW with EditDistanceSWScheme (ed_banded_inl.h:175-295).  The band's register arrays come in
// 8, 16 and 32 cells with the band length as a kernel argument, and exactly 7, 15 and 31 cells
// (nvBowtie's BAND_LEN values, traceback_inl.h:239-257) with the length folded in.
int nv_banded_traceback_device(const gasalx_nv_aligner &al, uint32_t band, uint32_t n, const gasalx_nv_strings &pat,
                               const gasalx_nv_strings &txt, uint32_t max_p, uint32_t *dir, int32_t *score,
                               uint32_t *src, uint32_t *snk, uint8_t *ops, uint32_t ops_stride, uint32_t *n_ops,
                               hipStream_t st) {
    if (al.aligner != NV_GOTOH && al.aligner != NV_SW && al.aligner != NV_ED) {
        set_error("banded traceback: unknown aligner");
        return GASALX_EINVAL;
    }
    if (al.type < 0 || al.type > 2) { set_error("bad alignment type"); return GASALX_EINVAL; }
    if (band < 2 || band > 32) { set_error("band length must be 2..32"); return GASALX_EINVAL; }
    for (uint32_t b : {pat.bits, txt.bits})
        if (b != 2 && b != 4 && b != 8) { set_error("symbol bits must be 2, 4 or 8"); return GASALX_EINVAL; }
    if (n == 0) return GASALX_OK;
    if (!pat.words || !pat.offsets || !txt.words || !score || !src || !snk || !ops || !n_ops || !dir) {
        set_error("null argument");
        return GASALX_EINVAL;
    }
    NvBandTbArgs A;
    A.pw = pat.words; A.poff = pat.offsets; A.pbits = pat.bits; A.pbig = pat.big_endian;
    A.tw = txt.words; A.toff = txt.offsets; A.tlen0 = txt.offsets ? 0 : txt.length; A.tbits = txt.bits;
    A.tbig = txt.big_endian;
    A.match = al.match; A.mismatch = al.mismatch; A.go = al.gap_open; A.ge = al.gap_ext;
    A.del = al.deletion; A.ins = al.insertion;
    if (al.aligner == NV_ED) { A.match = 0; A.mismatch = -1; A.del = -1; A.ins = -1; }
    A.n = n; A.band = band; A.words = (band + 3) / 4; A.max_m = max_p;
    A.dir = dir; A.score = score; A.src = src; A.snk = snk; A.ops = ops; A.ops_stride = ops_stride; A.n_ops = n_ops;
    using Fn = void (*)(NvBandTbArgs);
#define NVBT_ROW(G, T) {&nv_banded_traceback_kernel<G, T, 8>, &nv_banded_traceback_kernel<G, T, 16>, &nv_banded_traceback_kernel<G, T, 32>}
    static const Fn tab[2][3][3] = {{NVBT_ROW(false, 0), NVBT_ROW(false, 1), NVBT_ROW(false, 2)},
                                    {NVBT_ROW(true, 0), NVBT_ROW(true, 1), NVBT_ROW(true, 2)}};
#undef NVBT_ROW
#define NVBT_EX(G, T) {&nv_banded_traceback_kernel<G, T, 7, true>, &nv_banded_traceback_kernel<G, T, 15, true>, &nv_banded_traceback_kernel<G, T, 31, true>}
    static const Fn tab_ex[2][3][3] = {{NVBT_EX(false, 0), NVBT_EX(false, 1), NVBT_EX(false, 2)},
                                       {NVBT_EX(true, 0), NVBT_EX(true, 1), NVBT_EX(true, 2)}};
#undef NVBT_EX
    const int g = al.aligner == NV_GOTOH ? 1 : 0;
    const int ex = band == 7 ? 0 : band == 15 ? 1 : band == 31 ? 2 : -1;
    const Fn fn = ex >= 0 ? tab_ex[g][al.type][ex] : tab[g][al.type][band <= 8 ? 0 : band <= 16 ? 1 : 2];
    hipLaunchKernelGGL(fn, dim3((n + 255) / 256), dim3(256), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
    return GASALX_OK;
}

}  // namespace gx
