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

std::string nv_plan_name(const gasalx_nv_aligner &al, uint32_t max_p, uint32_t max_t, bool per_pair_text) {
    static const char *an[] = {"ed", "sw", "gotoh"}, *tn[] = {"global", "local", "semi"};
    if (al.aligner < 0 || al.aligner > 2 || al.type < 0 || al.type > 2) return "none";
    size_t lds = 0;
    const NvShape *sh = nv_shape(max_p, (std::max<uint32_t>(max_t, 1) + 7u) & ~7u, per_pair_text, &lds);
    if (!sh) return "none";
    return std::string("nvbio_") + an[al.aligner] + "_" + tn[al.type] + (per_pair_text ? "" : "_shared") + "_G" +
           std::to_string(sh->G) + "R" + std::to_string(sh->R);
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

}  // namespace gx
