// dispatch.hip — kernel instantiation table and the flat host dispatcher.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "banded16.hpp"
#include "local16.hpp"
#include "engine.hpp"
#include "generic.hpp"
#include "pairhmm.hpp"
#include "ksw16.hpp"
#include "start.hpp"
#include "wavefront.hpp"
#include "wavefront16.hpp"

namespace gx {

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
const char *last_error() { return g_last_error.c_str(); }

hipError_t DevBuf::reserve(size_t need) {
    if (need <= bytes && p) return hipSuccess;
    release();
    size_t cap = std::max<size_t>(need, 256);
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) { p = nullptr; bytes = 0; return e; }
    bytes = cap;
    return hipSuccess;
}
void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}
void Workspace::release_all() {
    for (DevBuf *b : {&packed_q, &packed_t, &tb, &rows_h, &rows_e, &rev, &ends_q, &ends_t, &misc, &aux,
                      &rev_meta, &sort_meta, &band_cp, &band_stm, &band_fl, &band_fb, &kseg}) b->release();
}

// ----------------------------------------------------------------------------
// (G lanes per pair, R rows per lane) shapes: query rows covered = G*R.
struct Shape { int G, R; };
static const Shape kShapes[] = {{8, 8}, {8, 12}, {8, 16}, {8, 20}, {16, 16}, {16, 20}, {32, 20}, {64, 20}};
// packed kernels (register axis = query for LOCAL/GLOBAL, target for SEMI):
// R = 19 fits 150 bp (152 padded) and R = 23 fits 182 bp (184 padded) exactly
// G = 16/32/64 shapes with few rows per lane serve small batches (make_plan)
static const Shape kShapes16[] = {{8, 8},   {8, 12},  {8, 16},  {8, 19},  {8, 20},  {8, 23},  {16, 10}, {16, 12},
                                  {16, 16}, {16, 20}, {32, 5},  {32, 6},  {32, 9},  {32, 20}, {64, 3},  {64, 5},
                                  {64, 20}};

using WfFn = void (*)(WfArgs);

template <int ALGO, bool KEYS, bool TB>
static WfFn wf_pick(int G, int R) {
#define GX_CASE(g, r) if (G == g && R == r) return &wf_kernel<ALGO, KEYS, TB, g, r>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 20)
    GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 20) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

static WfFn wf_pick_stop(int G, int R) {   // SEMI TAIL=TARGET reverse pass (start.hpp)
#define GX_CASE(g, r) if (G == g && R == r) return &wf_kernel<WF_SEMI, true, false, g, r, true>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 20)
    GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 20) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

static WfFn wf_lookup(int algo, bool keys, bool tb, int G, int R) {
    if (algo == WF_LOCAL) return tb ? wf_pick<WF_LOCAL, true, true>(G, R) : wf_pick<WF_LOCAL, true, false>(G, R);
    if (algo == WF_GLOBAL) return tb ? wf_pick<WF_GLOBAL, false, true>(G, R) : wf_pick<WF_GLOBAL, false, false>(G, R);
    return keys ? wf_pick<WF_SEMI, true, false>(G, R) : wf_pick<WF_SEMI, false, false>(G, R);
}

template <int ALGO>
static WfFn wf16_pick(int G, int R) {
#define GX_CASE(g, r) if (G == g && R == r) return &wf16_kernel<ALGO, g, r>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 19) GX_CASE(8, 20) GX_CASE(8, 23)
    GX_CASE(16, 10) GX_CASE(16, 12) GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 5) GX_CASE(32, 6) GX_CASE(32, 9)
    GX_CASE(32, 20) GX_CASE(64, 3) GX_CASE(64, 5) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

static WfFn wf16_pick_tb(int G, int R) {   // R % 4 == 0 shapes (wavefront16.hpp store groups)
#define GX_CASE(g, r) if (G == g && R == r) return &wf16_kernel<WF16_GLOBAL_TB, g, r>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 20)
    GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 20) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

template <int ALGO>
static WfFn wf16_pick_r4(int G, int R) {   // R % 4 == 0 shapes (band recomputation)
#define GX_CASE(g, r) if (G == g && R == r) return &wf16_kernel<ALGO, g, r>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 20)
    GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 20) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

static WfFn wf16_pick_local_tb(int G, int R) {   // R % 4 == 0 shapes
#define GX_CASE(g, r) if (G == g && R == r) return &wf16_kernel<WF16_LOCAL_TB, g, r>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 20)
    GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 20) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

static WfFn wf16_lookup(int algo, bool tb, int G, int R, bool key2 = false, bool stop = false, bool ku16 = false,
                        bool lrs = false, bool kseg = false, bool tbd = false) {
    if (algo == WF_LOCAL) return tb ? (tbd ? (G == 16 && R == 12 ? &wf16_kernel<WF16_LOCAL_TBD, 16, 12>
                                                                  : wf16_pick_r4<WF16_LOCAL_TBD>(G, R))
                                           : wf16_pick_local_tb(G, R))
                                    : key2 ? wf16_pick<WF16_LOCAL_K2>(G, R)
                                                               : (ku16 || lrs || kseg) ? wf16_local_lookup(G, R, ku16, lrs, kseg)
                                                                               : wf16_pick<WF_LOCAL>(G, R);
    if (algo == WF_GLOBAL) return tb ? wf16_pick_tb(G, R) : wf16_pick<WF_GLOBAL>(G, R);
    return stop ? wf16_pick<WF16_SEMI_STOP>(G, R) : wf16_pick<WF_SEMI>(G, R);
}

static inline uint32_t pad8(uint32_t x) { return (x + 7u) & ~7u; }

static bool env_flag(const char *name, bool dflt);

// packed LOCAL with the round-2 keys H*256 + (255 - column): H <= 255, 512 columns (two key
// sets above 256), 256 with traceback
static bool local_key16_ok(const gasalx_params &p, uint32_t mq, uint32_t mt) {
    const int64_t a = p.match, b = p.mismatch, oe = (int64_t)p.gap_open + p.gap_extend;
    const int64_t k = std::max<int64_t>(b, p.has_n_penalty ? p.n_penalty : 0);
    const int64_t t8 = pad8(mt);
    if (a * std::min(mq, mt) > 255 || t8 > (p.start_pos == 2 ? 256 : 512)) return false;
    return 0x400 + oe + k + 16 + 255 + a + k + 64 <= 0x7BFF;
}

// The packed kernels (wavefront16.hpp) are exact when every stored value stays
// inside [0x0400, 0x7BFF] (positive normal f16 patterns) and the score tables
// fit bytes.  Mirrors pk16_params; returns false to keep the int32 kernel.
static bool packed16_ok(const gasalx_params &p, int wf_algo, uint32_t mq, uint32_t mt, int32_t *vmin,
                        int64_t span = 0) {
    if (p.second_best || (p.start_pos == 1 && wf_algo == WF_GLOBAL)) return false;
    if (p.start_pos == 2 && wf_algo == WF_SEMI) return false;     // no traceback for SEMI (reference)
    // GLOBAL+TB reads the first pad query row, scored -K = -max(b, npen) there:
    // exact for N-vs-base cells only if that equals the reference's -npen
    if (p.start_pos == 2 && wf_algo == WF_GLOBAL && p.has_n_penalty && p.n_penalty < p.mismatch) return false;
    if (p.match < 0 || p.mismatch < 0 || p.gap_open < 0 || p.gap_extend < 0) return false;
    if (p.has_n_penalty && p.n_penalty < 0) return false;
    const int64_t a = p.match, b = p.mismatch, oe = (int64_t)p.gap_open + p.gap_extend, e = p.gap_extend;
    const int64_t npen = p.has_n_penalty ? p.n_penalty : 0;
    const int64_t q8 = pad8(mq), t8 = pad8(mt);
    if (wf_algo == WF_LOCAL) {
        const int64_t k = std::max(b, npen);
        if (a + k > 255) return false;   // table bytes
        *vmin = 0;
        // 16-bit keys H*256 + col: 256 columns each, a second key set up to 512 (not with traceback)
        if (local_key16_ok(p, mq, mt)) return true;
        // the e-drift kernels key on H*C + col (f16 patterns or u16; traceback: f16): make_plan
        // checks their frame and key range for the chosen shape
        return env_flag("GASALX_KF16", true);
    }
    int64_t k, top, drift = 0;
    if (wf_algo == WF_SEMI) {
        // TAIL=TARGET (last query row); TAIL=QUERY/BOTH score-only through the class launches
        // (the last padded column, Q11): targets up to 256 (R <= 32), rows keyed in 16 bits
        const bool tq = p.start_pos == 0 && (p.tail == 1 || p.tail == 3);
        if (p.tail != 2 && !tq) return false;
        if (tq && (t8 > 256 || q8 > 65535)) return false;
        // table offset K = OE + e (wavefront16.hpp step_semi's frame): bytes s + K >= 0
        if (oe + e < b || oe + e < npen) return false;
        k = oe + e;
    } else {
        // GLOBAL: values drift by e per anti-diagonal, table offset K = max(2*ceil(max(b,
        // npen)/2), 2e) (pk16_params, step_global).  Traceback reads the first pad query
        // row, scored -K: keep the round-2 offset there (K == 2*ceil(max(b, npen)/2))
        drift = e;
        const int64_t k0 = 2 * ((std::max(b, npen) + 1) / 2);
        k = std::max(k0, 2 * e);
        if (p.start_pos == 2 && k != k0) return false;
    }
    if (a + k > 255) return false;
    // span: largest row + column of any cell the launch computes.  Both halves of
    // a register hold the same cell of two pairs of different lengths, so one
    // pair's pad cells share 32-bit adds with the other's real cells: every
    // computed cell (register rows up to G*R, steps past the longest sequence)
    // must stay inside the window or a borrow corrupts the neighbour (SEMI keeps
    // no floor on E/F; values fall by at most e per row or column along a gap).
    // make_plan checks again with the chosen shape's span.
    if (!span) span = q8 + t8 + 2 * 64 + 8;
    const int64_t neg = 0x400 + 2 * e + 16;
    if (wf_algo == WF_SEMI) {
        // SEMI's frame (+ e per anti-diagonal): E and F never decay, every F is at least
        // its column's top boundary and every E its row's left one, so no value falls
        // below B - 3*OE whatever the span; values rise by the frame, e per row + column
        // (the tail keys add up to e*(span) more to put the last row or column in one frame)
        const int64_t v = 4 * oe + k + 64;
        top = neg + v + a * std::min(q8, t8) + a + k + oe + 64 + e * (2 * span + 1);
        if (top > 0x7BFF) return false;
        *vmin = (int32_t)v;
        return true;
    }
    const int64_t v = 4 * oe + k + e * span + 2 * drift + 64;   // below every reachable value
    top = neg + v + a * std::min(q8, t8) + a + k + oe + 64 + drift * span;
    if (top > 0x7BFF) return false;
    *vmin = (int32_t)v;
    return true;
}

// Largest |value| the DP can reach, to decide whether int32 arithmetic without
// the reference's int16 row-buffer truncation is exact.
static bool int16_safe(const gasalx_params &p, uint32_t mq, uint32_t mt) {
    const int64_t L = (int64_t)pad8(mq) + pad8(mt) + 16;
    const int64_t step = (int64_t)std::max({std::abs(p.match), std::abs(p.mismatch),
                                            p.has_n_penalty ? std::abs(p.n_penalty) : 0}) +
                         std::abs(p.gap_open) + std::abs(p.gap_extend);
    return std::abs((int64_t)p.gap_open) + L * step < 30000;
}

// A/B switch: the environment variable, read as an integer, or `dflt` when unset
static bool env_flag(const char *name, bool dflt) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) != 0 : dflt;
}
static int env_int(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}

// Packed banded kernel (banded16.hpp): stored values B + [0, Hmax] and keys
// H*8 + 7 + 0x400 inside [0x0400, 0x7BFF]; pads score -b, which needs an N score
// <= 0.  GASALX_BAND16=0 keeps every pair on the int32 kernel (A/B runs).
static uint32_t band16_base(const gasalx_params &p) { return 0x400u + (uint32_t)(p.gap_open + p.gap_extend + p.mismatch); }
static bool band16_ok(const gasalx_params &p, uint32_t q8, uint32_t t8) {
    const char *env = std::getenv("GASALX_BAND16");
    if (env && std::atoi(env) == 0) return false;
    if (p.match < 0 || p.mismatch < 0 || p.gap_open < 0 || p.gap_extend < 0) return false;
    if (p.match + p.mismatch > 255 || p.gap_open + p.gap_extend > 4096) return false;
    if (p.has_n_penalty && p.n_penalty < 0) return false;
    if (q8 > 65535) return false;   // the first-maximum row is tracked in 16 bits
    const int64_t hmax = (int64_t)p.match * std::min(q8, t8);
    return hmax + band16_base(p) <= 0x7BFF && hmax * 8 + 7 + 0x400 <= 0x7BFF;
}

// Packed LOCAL second-best kernel (local16.hpp): table bytes s + K in [0, 255]
// (K = max(0, b, N_PENALTY)), stored values B + [0, Hmax] and keys H*8 + 7 +
// 0x400 inside [0x0400, 0x7BFF].  GASALX_LOCAL16=0 keeps every pair on the int32
// kernel (A/B runs).
static int32_t local16_sn(const gasalx_params &p) { return p.has_n_penalty ? -p.n_penalty : 0; }
static uint32_t local16_k(const gasalx_params &p) { return (uint32_t)std::max({0, p.mismatch, -local16_sn(p)}); }
static uint32_t local16_base(const gasalx_params &p) { return 0x400u + (uint32_t)(p.gap_open + p.gap_extend) + local16_k(p); }
static bool local16_ok(const gasalx_params &p, uint32_t q8, uint32_t t8) {
    const char *env = std::getenv("GASALX_LOCAL16");
    if (env && std::atoi(env) == 0) return false;
    if (p.match < 0 || p.gap_open < 0 || p.gap_extend < 0 || p.gap_open + p.gap_extend > 4096) return false;
    const int64_t k = local16_k(p), sn = local16_sn(p);
    if (p.match + k > 255 || k - p.mismatch > 255 || sn + k > 255) return false;
    if (q8 > 65535 || t8 / 8 > 65535) return false;   // rows and strips are tracked in 16 bits
    // largest gain of one cell: match, a negative mismatch or a negative N penalty
    const int64_t step = std::max<int64_t>({(int64_t)p.match, -(int64_t)p.mismatch, sn});
    const int64_t hmax = step * std::min(q8, t8);
    return hmax + local16_base(p) <= 0x7BFF && hmax * 8 + 7 + 0x400 <= 0x7BFF;
}

Plan make_plan(const gasalx_params &p, const BatchShape &s, bool has_ops) {
    Plan pl;
    pl.max_q = s.max_q; pl.max_t = s.max_t;
    const uint32_t q8 = pad8(s.max_q), t8 = pad8(s.max_t);
    const bool tb = p.start_pos == 2;
    int wf_algo = -1;
    bool keys = false;
    // LOCAL WITH_START: start.hpp (its reversed query drops pad rows, exact unless N cells score > 0)
    if (p.algo == 3 /*LOCAL*/ && !p.second_best && !(p.start_pos == 1 && p.has_n_penalty && p.n_penalty < 0)) {
        wf_algo = WF_LOCAL;
        keys = true;
    }
    else if (p.algo == 1 /*GLOBAL*/) { wf_algo = WF_GLOBAL; }
    else if (p.algo == 2 /*SEMI*/ && !p.second_best && (p.start_pos != 1 || p.tail == 2)) {   // WITH_START: start.hpp
        wf_algo = WF_SEMI;
        keys = (p.tail == 2 || p.tail == 3);
    }
    // SEMI TAIL=NONE, score-only: the reference keeps maxHH = MINUS_INF and the initial ends
    // (semiglobal_kernel_template.h:49-51,63-64,206-218; neither tail block runs)
    if (p.algo == 2 && p.tail == 0 && p.start_pos == 0 && !p.second_best) {
        pl.kind = PLAN_CONST;
        pl.name = "semi_tail_none";
        return pl;
    }
    bool ok = wf_algo >= 0 && int16_safe(p, s.max_q, s.max_t) && t8 < 32000 && p.gap_extend >= 0;
    if (wf_algo == WF_SEMI && p.start_pos == 1 && t8 > 8192) ok = false;   // stop key: strips < 1024
    if (ok) {
        const Shape *pick = nullptr;
        for (const Shape &sh : kShapes)
            if ((uint32_t)(sh.G * sh.R) >= q8) { pick = &sh; break; }
        if (!pick) ok = false;
        else {
            pl.G = pick->G; pl.R = pick->R;
            pl.lds_stride = std::max<uint32_t>(t8, 8);
            pl.lds_bytes = (size_t)kWavesPerBlock * (64 / pl.G) * pl.lds_stride;
            if (pl.lds_bytes > 160 * 1024) ok = false;
        }
    }
    if (ok) {
        pl.kind = PLAN_WAVEFRONT;
        pl.wf_algo = wf_algo; pl.keys = keys; pl.tb = tb && wf_algo != WF_SEMI;
        pl.need_pack = has_ops;
        // GASALX_PACKED16=0: every block on the int32 kernel (A/B runs, the int32 probe of
        // bench.py --force-int32); read per call
        const char *pk_env = std::getenv("GASALX_PACKED16");
        pl.packed16 = !(pk_env && std::atoi(pk_env) == 0) && packed16_ok(p, wf_algo, s.max_q, s.max_t, &pl.vmin);
        if (pl.packed16) {
            const uint32_t x8 = (wf_algo == WF_SEMI) ? t8 : q8, y8 = (wf_algo == WF_SEMI) ? q8 : t8;
            pl.G16 = 0;
            // small batches: enough lanes per pair that the launch still holds about two
            // waves per SIMD (128/G pairs per wave, 1024 SIMDs); traceback keeps G = 8 up
            // GASALX_GMIN: fixed minimum G (A/B runs, parity sweeps); read per call so a
            // test process can sweep it
            const char *gmin_env = std::getenv("GASALX_GMIN");
            const int gforce = gmin_env ? std::atoi(gmin_env) : 0;
            uint32_t gmin = 8;
            if (s.n && !pl.tb)
                while (gmin < 64 && (uint64_t)s.n * gmin < 2048ull * 128) gmin *= 2;
            if (gforce > 0) gmin = (uint32_t)gforce;
            // traceback kernels store flags in groups of 4 rows and keep >= 16 rows per
            // lane (their instances, wf16_pick_tb): the other shapes are never taken,
            // forced or not -- except LOCAL+TB's G16R12 (3 waves per SIMD),
            // taken under GASALX_LTBD_G16=1 for the A/B against the 2-wave G8R20
            const bool ltbd16 = pl.tb && wf_algo == WF_LOCAL && env_flag("GASALX_LTBD_G16", false);
            if (ltbd16) gmin = std::max<uint32_t>(gmin, 16);
            for (const Shape &sh : kShapes16)
                if ((uint32_t)sh.G >= gmin && (uint32_t)(sh.G * sh.R) >= x8 &&
                    !(pl.tb && (sh.R % 4 || (sh.G > 8 && sh.R < 16)) && !(ltbd16 && sh.G == 16 && sh.R == 12))) {
                    pl.G16 = sh.G; pl.R16 = sh.R;
                    break;
                }
            // SEMI TAIL=QUERY/BOTH: G = 8 and R = padded target / 8 per class launch (the
            // last padded column at register R - 1 of lane 7); the plan names the largest
            pl.semi_tq = pl.packed16 && wf_algo == WF_SEMI && p.tail != 2;
            if (pl.semi_tq) { pl.G16 = 8; pl.R16 = (int)(x8 / 8); }
            const uint32_t words = (y8 + 2 * pl.G16 + 4 + 3) & ~3u;   // odd-step tail + prefetch
            pl.lds16_stride = words * 8;                               // uint2 per position
            pl.lds16_bytes = (size_t)kWavesPerBlock * (64 / std::max(pl.G16, 1)) * pl.lds16_stride;
            if (pl.G16 == 0 || pl.lds16_bytes > 160 * 1024) pl.packed16 = false;
            if (pl.packed16 && wf_algo != WF_LOCAL)   // the value window over the chosen shape's cells
                pl.packed16 = packed16_ok(p, wf_algo, s.max_q, s.max_t, &pl.vmin,
                                          (int64_t)pl.G16 * pl.R16 + y8 + 2 * pl.G16 + 8);
            pl.key2 = wf_algo == WF_LOCAL && y8 > 256;
            // LOCAL score kernels in the e-drift frame (wavefront16.hpp step_local_dr): keys
            // H*C + (C-1-c) with C = the padded target length, as f16 patterns 0x0400 + key
            // while (Hmax + 1) * C <= 0x7800, as u16 integers (WF16_LOCAL_U16, one more
            // instruction per two cells) up to 65536 -- either covers targets past 256 columns
            // without the second key set; values B + H + e(r + c) over the shape's span stay in
            // the window and the top lane's first diagonal B - 2e above 0x0400.  GASALX_KF16=0
            // keeps the round-2 kernel (the tests' cross-check of both key forms)
            // LOCAL + traceback takes the e-drift kernel with f16 keys (WF16_LOCAL_TBD) when they fit
            if (wf_algo == WF_LOCAL && env_flag("GASALX_KF16", true)) {
                const int64_t a = std::max(p.match, 0), e = p.gap_extend, oe = (int64_t)p.gap_open + e;
                const int64_t k = std::max<int64_t>(p.mismatch, p.has_n_penalty ? p.n_penalty : 0);
                const int64_t hmax = a * std::min(q8, t8), base = 0x400 + oe + k + 16;
                const int64_t span = (int64_t)pl.G16 * pl.R16 + y8 + 2 * pl.G16 + 8;
                const bool frame = base + hmax + e * span + a + k + 64 <= 0x7BFF && base - 2 * e >= 0x400;
                // past both, f16 keys by step segments of M = 2^m columns (WF16_LOCAL_SEG): (Hmax +
                // 1) * M <= 0x7800 for any target length.  GASALX_KSEG=0: never, 2: before u16 keys
                const char *ks = std::getenv("GASALX_KSEG");
                const int kseg_mode = ks ? std::atoi(ks) : 1;
                uint32_t mseg = 0;
                while ((hmax + 1) * (int64_t)(2u << mseg) <= 0x7800 && mseg < 12) ++mseg;   // M = 2^mseg
                const bool seg_ok = frame && kseg_mode > 0 && mseg >= 2 && y8 <= 0xFFFF;
                // key range: steps C + G (wavefront16.hpp step_local_dr: keys rank steps)
                const int64_t kc = (int64_t)y8 + pl.G16;
                // (GX_LOCAL_KA0: row k's keys carry e*k more, taken off after the sweep)
                const int64_t hk = hmax + (GX_LOCAL_KA0 && (!pl.tb || GX_LTB_KA0) ? e * (pl.R16 - 1) : 0);
                if (frame && (hk + 1) * kc <= 0x7800) {
                    pl.kf16 = y8;
                } else if (pl.tb) {
                    // (the traceback kernel has f16 keys only)
                } else if (seg_ok && kseg_mode == 2) {
                    pl.kf16 = y8;
                    pl.kseg_shift = mseg;
                } else if (frame && (hmax + 1) * kc <= 0x10000 && y8 <= 0xFFFF) {
                    pl.kf16 = y8;
                    pl.ku16 = true;
                } else if (seg_ok) {
                    pl.kf16 = y8;
                    pl.kseg_shift = mseg;
                }
                if (pl.kf16) pl.key2 = false;
            }
            // (LOCAL+TB's G16R12, GASALX_LTBD_G16: an e-drift instance only)
            if (wf_algo == WF_LOCAL && pl.tb && pl.G16 == 16 && pl.R16 == 12 && !pl.kf16) pl.packed16 = false;
            // outside both frames the round-2 keys must hold (packed16_ok admitted the drift case)
            if (wf_algo == WF_LOCAL && !pl.kf16 && !local_key16_ok(p, s.max_q, s.max_t)) pl.packed16 = false;
            pl.semi_tq = pl.semi_tq && pl.packed16;
            // GLOBAL + traceback: the score sweep stores band checkpoints, a second pass
            // recomputes each lane's band window with flags, the walk leaves the band only
            // through the full-matrix fallback (wavefront16.hpp WF16_GLOBAL_CP / _BAND).
            // GASALX_TB_BAND=0: the full-matrix flags kernel (A/B); GASALX_TB_BAND_W: the
            // band's half width w (window of lane lg: columns [max(lg*R - w, 0), + R + 2w))
            if (pl.packed16 && pl.tb && wf_algo == WF_GLOBAL && pl.R16 % 4 == 0 && env_flag("GASALX_TB_BAND", true)) {
                const char *bw = std::getenv("GASALX_TB_BAND_W");
                // w = 22: config 3's paths stray up to 20 cells from the diagonal, and any pair
                // that leaves its band costs the chain a full-matrix sweep and a second walk,
                // latency floors however few pairs they hold; w = 10 -> 22 took config 3 from
                // 2,953 to 3,647 GCUPS on one engine and 4,240 to 4,450-4,560 on three, though
                // the band pass grows by 60 % (profiles/r05/n_band_width.md)
                const int w = bw ? std::max(0, std::atoi(bw)) : 22;
                pl.tb_band = true;
                pl.band_w = (uint32_t)w;
                pl.band_wd = ((uint32_t)(pl.R16 + 2 * w) + 3u) & ~3u;
            }
        }
        const char *an = wf_algo == WF_LOCAL ? (p.start_pos == 1 ? "local_start" : "local")
                       : wf_algo == WF_GLOBAL ? "global"
                       : pl.semi_tq ? "semi_tq" : (p.start_pos == 1 ? "semi_start" : "semi");
        if (pl.packed16)
            // (_nodrift: a LOCAL score plan outside the e-drift frame's window, the round-2 kernel)
            pl.name = std::string("wavefront16_") + an + (pl.tb ? (pl.tb_band ? "_tbband" : "_tb") : "") +
                      (pl.key2 ? "_k2" : "") +
                      (wf_algo == WF_LOCAL && !pl.tb && !pl.key2 && !pl.kf16 ? "_nodrift" : "") +
                      (wf_algo == WF_LOCAL && pl.tb && pl.kf16 ? "_dr" : "") +
                      (pl.ku16 ? "_u16" : "") + (pl.kseg_shift ? "_seg" + std::to_string(1u << pl.kseg_shift) : "") + "_G" +
                      std::to_string(pl.G16) + "R" + std::to_string(pl.R16);
        else
            pl.name = std::string("wavefront_") + an + (pl.tb ? "_tb" : "") + (keys ? "_keys" : "") + "_G" +
                      std::to_string(pl.G) + "R" + std::to_string(pl.R);
    } else if (p.algo == 1 || p.algo == 2 || p.algo == 3 || p.algo == 5 || p.algo == 6) {
        pl.kind = PLAN_GENERIC;
        pl.need_pack = true;
        static const char *names[] = {"?", "global", "semi", "local", "?", "banded", "ksw"};
        pl.name = std::string("generic_") + names[p.algo];
        if (p.algo == 5 && band16_ok(p, q8, t8)) {
            pl.band16 = true;
            pl.name = "banded16_local";
        }
        if (p.algo == 3 && p.second_best && p.start_pos == 0 && local16_ok(p, q8, t8)) {
            pl.local16 = true;
            pl.name = "local16_second";
        }
    } else {
        pl.kind = PLAN_NONE;
        pl.name = "none";
    }
    return pl;
}

#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        hipError_t e__ = (x);                                                            \
        if (e__ != hipSuccess) {                                                         \
            set_error(std::string(#x) + ": " + hipGetErrorString(e__));                  \
            return GASALX_EDEVICE;                                                       \
        }                                                                                \
    } while (0)

static int grid_for(uint32_t n, uint32_t per_block) { return (int)((n + per_block - 1) / per_block); }
// the int32 wavefront kernel's grid: every block, or, as the fallback of a packed launch (A.skip:
// usually few or no declined blocks), at most 8 blocks per CU walking the rest (wavefront.hpp wf_kernel)
static int wf_grid(uint32_t n, int G, bool fallback) {
    const int g = grid_for(n, kWavesPerBlock * (64 / G));
    return fallback ? std::min(g, 8 * 256) : g;
}

// Device-to-device byte copy, 16 bytes per lane (the CIGAR buffer's start as the query batch,
// get_tb.h:94): the runtime's copy ran at ≈0.4 TB/s for the config-3 batch (30 MB, 80 us
// under the two-stream bench, profiles/r04_nw_tb_kernel_stats.csv).  Both pointers 16-byte
// aligned, else the runtime copy.
__global__ __launch_bounds__(256) void copy16_kernel(uint4 *dst, const uint4 *src, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}
static hipError_t copy_d2d(void *dst, const void *src, size_t bytes, hipStream_t st) {
    if (((uintptr_t)dst | (uintptr_t)src) & 15u || bytes < 4096)
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
    const uint64_t n16 = bytes / 16;
    copy16_kernel<<<(int)std::min<uint64_t>((n16 + 255) / 256, 8192), 256, 0, st>>>((uint4 *)dst, (const uint4 *)src, n16);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && bytes % 16)
        e = hipMemcpyAsync((uint8_t *)dst + n16 * 16, (const uint8_t *)src + n16 * 16, bytes % 16, hipMemcpyDeviceToDevice, st);
    return e;
}

// The short second shape of a packed score launch (wf16_mix_kernel): more lanes per pair and
// fewer rows per lane, a wave a third as long, over the launch's last slots.  Taken for the
// score plans it is instantiated for (LOCAL in the e-drift frame with f16 keys at G8R19, 150 bp:
// config 2; GLOBAL score at G16R20, 300 bp), when the launch holds at least two rounds of its
// waves and the value window and key range also hold for the second shape's span.  The slots
// past the last whole round of long waves (GASALX_TAIL_K more rounds: 0 by default) take it;
// GASALX_TAIL=0: one shape (A/B).
struct TailShape {
    WfFn fn = nullptr;
    int G2 = 0, R2 = 0;
    uint32_t b0 = 0, p0 = 0, ppb = 1, lds_stride = 0;
    size_t lds_bytes = 0;
    int32_t vmin = 0;   // GLOBAL: the value-window bound for the larger span of the two shapes
};
static TailShape tail_shape(const Plan &pl, const gasalx_params &p, const WfArgs &A, uint32_t n) {
    TailShape t;
    // (read per call, so a test process can compare both)
    const bool on = env_flag("GASALX_TAIL", true);
    const char *ke = std::getenv("GASALX_TAIL_K");
    const int kextra = ke ? std::atoi(ke) : 0;
    if (!on || !pl.packed16 || (pl.tb && !pl.tb_band) || pl.key2 || pl.ku16 || pl.kseg_shift || pl.semi_tq ||
        A.rev || A.n_dev || A.stop || A.lstop)
        return t;
    int G2 = 0, R2 = 0;
    WfFn fn = nullptr;
    if (pl.wf_algo == WF_LOCAL && pl.kf16 && pl.G16 == 8 && pl.R16 == 19) {
        G2 = 32; R2 = 5; fn = &wf16_mix_kernel<WF_LOCAL, 8, 19, 32, 5>;
    } else if (pl.tb_band) {
        // the band traceback's sweep + band pass (R % 4 == 0 for the band windows); GASALX_CP_TAIL=32: G32R12
        if (pl.wf_algo != WF_GLOBAL || pl.G16 != 16 || pl.R16 != 20) return t;
        if (env_int("GASALX_CP_TAIL", 64) == 32) {
            G2 = 32; R2 = 12; fn = &wf16_mix_kernel<WF16_GLOBAL_CP, 16, 20, 32, 12>;
        } else {
            G2 = 64; R2 = 8; fn = &wf16_mix_kernel<WF16_GLOBAL_CP, 16, 20, 64, 8>;
        }
    } else if (pl.wf_algo == WF_GLOBAL && pl.G16 == 16 && pl.R16 == 20) {
        G2 = 64; R2 = 5; fn = &wf16_mix_kernel<WF_GLOBAL, 16, 20, 64, 5>;
    } else {
        return t;
    }
    const int64_t q8 = pad8(pl.max_q), y8 = pad8(pl.max_t);   // LOCAL / GLOBAL: the target is the step axis
    // the second shape's span and keys must fit the value window too (make_plan checked the first's)
    const int64_t span2 = (int64_t)G2 * R2 + y8 + 2 * G2 + 8;
    if (pl.wf_algo == WF_LOCAL) {
        const int64_t a = std::max(p.match, 0), e = p.gap_extend, oe = (int64_t)p.gap_open + e;
        const int64_t k = std::max<int64_t>(p.mismatch, p.has_n_penalty ? p.n_penalty : 0);
        const int64_t hmax = a * std::min(q8, y8), base = 0x400 + oe + k + 16;
        const int64_t hk2 = hmax + (GX_LOCAL_KA0 ? e * (R2 - 1) : 0);   // (KA0 key offsets)
        if (!(base + hmax + e * span2 + a + k + 64 <= 0x7BFF && (hk2 + 1) * (y8 + G2) <= 0x7800)) return t;
        t.vmin = pl.vmin;
    } else {
        // the window offset for the larger span serves both shapes: their values then sit higher
        // in the same window, whose top packed16_ok checked for that span
        if (!packed16_ok(p, WF_GLOBAL, pl.max_q, pl.max_t, &t.vmin, std::max<int64_t>(span2, (int64_t)pl.G16 * pl.R16 + y8 + 2 * pl.G16 + 8)))
            return t;
        t.vmin = std::max(t.vmin, pl.vmin);
    }
    static int cus = 0;
    if (!cus) { int d = 0; (void)hipGetDevice(&d); (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d); }
    const uint64_t slots = (uint64_t)wf16_waves(pl.wf_algo, pl.R16) * 4 * (cus > 0 ? cus : 256);
    const uint32_t ppw = 2 * (64 / pl.G16), ppb = kWavesPerBlock * ppw;
    const uint64_t waves = (n + ppw - 1) / ppw;
    const uint64_t rounds = waves / slots;
    if (rounds < 2 + (uint64_t)std::max(kextra, 0)) return t;
    const uint64_t long_waves = (rounds - (uint64_t)std::max(kextra, 0)) * slots;
    t.b0 = (uint32_t)(long_waves / kWavesPerBlock);
    t.p0 = t.b0 * ppb;
    if (t.p0 >= n) return TailShape();
    t.ppb = kWavesPerBlock * 2 * (64 / G2);
    const uint32_t words = ((uint32_t)y8 + 2 * G2 + 4 + 3) & ~3u;   // as make_plan's, for G2
    t.lds_stride = words * 8;
    t.lds_bytes = (size_t)kWavesPerBlock * (64 / G2) * t.lds_stride;
    t.fn = fn;
    t.G2 = G2;
    t.R2 = R2;
    return t;
}

// Launch the wavefront kernel(s) of plan `pl` over one device batch: the packed
// kernel first when the plan has one (it flags the blocks it aligned), then the
// int32 kernel, which aligns exactly the pairs of the declined blocks.
static int launch_wavefront(Workspace &ws, const Plan &pl, const gasalx_params &p, const WfArgs &base,
                            hipStream_t st) {
    WfArgs A = base;
    const uint32_t n = A.n;
    A.a = p.match; A.b = p.mismatch; A.o = p.gap_open; A.e = p.gap_extend;
    A.nval = p.n_code & 0xF;
    A.has_npen = p.has_n_penalty; A.npen = p.n_penalty;
    A.head = p.head; A.tail = p.tail;
    A.lds_stride = pl.lds_stride;
    A.force_exact = (p.mismatch <= 0 || (p.has_n_penalty && p.n_penalty < 0)) ? 1 : 0;
    A.one = 0x00010001u;
    if (pl.packed16) {
        // packed kernel first; it marks every block it aligned in ws.misc ...
        WfArgs P16 = A;
        P16.lds_stride = pl.lds16_stride;
        P16.fast16 = 1;
        P16.vmin = pl.vmin;
        P16.kf16 = pl.kf16;
        const uint32_t ppb16 = kWavesPerBlock * (64 / pl.G16) * 2;
        uint32_t grid16 = grid_for(n, ppb16);
        // the launch's last slots on a shorter shape (wavefront16.hpp wf16_mix_kernel), so that its
        // end is not a fraction of a round of long waves running alone
        const TailShape tail = tail_shape(pl, p, A, n);
        size_t lds16 = pl.lds16_bytes;
        if (tail.fn) {
            P16.tail_b0 = tail.b0; P16.tail_p0 = tail.p0; P16.tail_lds = tail.lds_stride;
            P16.vmin = tail.vmin;
            grid16 = tail.b0 + grid_for(n - tail.p0, tail.ppb);
            lds16 = std::max(lds16, tail.lds_bytes);
        }
        HIPCHK(ws.misc.reserve(grid16 + 64));
        P16.handled = ws.misc.as<uint8_t>();
        ws.pk_flags = grid16; ws.pk_ppb = ppb16; ws.pk_pairs = n;
        ws.pk_p1 = tail.fn ? tail.p0 : 0xFFFFFFFFu; ws.pk_b1 = tail.b0; ws.pk_ppb2 = tail.fn ? tail.ppb : 1;
        if (pl.tb) {
            HIPCHK(ws.aux.reserve((size_t)n * 4));
            P16.tbfix = ws.aux.as<int32_t>();
        }
        WfFn f16 = pl.tb_band ? wf16_pick_r4<WF16_GLOBAL_CP>(pl.G16, pl.R16)
                              : wf16_lookup(pl.wf_algo, pl.tb, pl.G16, pl.R16, pl.key2, A.stop != nullptr, pl.ku16,
                                            A.lstop != nullptr && pl.kf16 != 0 && !pl.kseg_shift, pl.kseg_shift != 0,
                                            pl.tb && pl.kf16 != 0);
        // WITH_START reverse passes: the register axis sized per block (rclass.hip)
        const bool lrs = pl.wf_algo == WF_LOCAL && !pl.tb && !pl.key2 && A.lstop != nullptr && pl.kf16 != 0 &&
                         !pl.kseg_shift;
        if (A.rev && !pl.tb_band && (A.stop != nullptr || lrs)) {
            const int ra = A.stop ? WF16_SEMI_STOP : pl.ku16 ? WF16_LOCAL_U16_RS : WF16_LOCAL_RS;
            if (WfFn rc = wf16_rclass_lookup(ra, pl.G16, pl.R16)) f16 = rc;
        }
        if (pl.kseg_shift) {
            // the finished segments' keys per wave: saves at steps M, 2M, ... < nsteps <= C + G - 1
            const uint32_t nsave = std::max<uint32_t>(1u, (pl.kf16 + (uint32_t)pl.G16 - 2u) >> pl.kseg_shift);
            const uint64_t waves = (uint64_t)grid16 * kWavesPerBlock;
            HIPCHK(ws.kseg.reserve(waves * nsave * (uint64_t)pl.R16 * 64 * 4 + 64));
            P16.kseg = ws.kseg.as<uint32_t>();
            P16.kseg_shift = pl.kseg_shift;
            P16.kseg_n = nsave;
        }
        if (tail.fn) f16 = tail.fn;
        if (!f16) { set_error("no packed wavefront instance"); return GASALX_EUNSUPPORTED; }
        if (lds16 > 64 * 1024)
            HIPCHK(hipFuncSetAttribute((const void *)f16, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds16));
        hipLaunchKernelGGL(f16, dim3(grid16), dim3(kBlock), lds16, st, P16);
        HIPCHK(hipGetLastError());
        // ... and the int32 kernel aligns the pairs of the blocks it declined
        A.skip = ws.misc.as<uint8_t>();
        A.skip_ppb = ppb16;
        A.skip_p1 = tail.fn ? tail.p0 : 0xFFFFFFFFu;
        A.skip_b1 = tail.b0;
        A.skip_ppb2 = tail.fn ? tail.ppb : 1;
    }
    // (the band path's int32 launch aligns its declined blocks without direction words: the walk sends
    // those pairs to the fallback list, whose launch writes them into the capped buffer)
    WfFn fn = A.stop ? wf_pick_stop(pl.G, pl.R) : wf_lookup(pl.wf_algo, pl.keys, pl.tb && !pl.tb_band, pl.G, pl.R);
    if (!fn) { set_error("no wavefront instance"); return GASALX_EUNSUPPORTED; }
    if (pl.lds_bytes > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds_bytes));
    hipLaunchKernelGGL(fn, dim3(wf_grid(n, pl.G, A.skip != nullptr)), dim3(kBlock), pl.lds_bytes, st, A);
    HIPCHK(hipGetLastError());
    return GASALX_OK;
}

// SEMI TAIL=QUERY/BOTH, packed (wavefront16.hpp WF16_SEMI_TQ): one launch per class of
// pairs with the same padded target length 8R, over a slot range (slots sorted by target
// words when the batch holds more than one class; the class sizes are read back, one
// synchronisation of the stream), flags per slot; then the int32 kernel over the slots
// the packed launches declined.
static int launch_semi_tq(Workspace &ws, const Plan &pl, const gasalx_params &p, const WfArgs &base,
                          hipStream_t st, bool one_class) {
    WfArgs A = base;
    const uint32_t n = A.n;
    A.a = p.match; A.b = p.mismatch; A.o = p.gap_open; A.e = p.gap_extend;
    A.nval = p.n_code & 0xF;
    A.has_npen = p.has_n_penalty; A.npen = p.n_penalty;
    A.head = p.head; A.tail = p.tail;
    A.lds_stride = pl.lds_stride;
    A.force_exact = (p.mismatch <= 0 || (p.has_n_penalty && p.n_penalty < 0)) ? 1 : 0;
    A.one = 0x00010001u;
    const uint32_t t8w = (uint32_t)pl.R16;                  // largest class
    const size_t sh = (size_t)(t8w + 1) * 4;
    HIPCHK(ws.sort_meta.reserve((size_t)n * 4 + 2 * sh + 64));
    uint32_t *perm = ws.sort_meta.as<uint32_t>(), *hist = perm + n, *cursor = hist + t8w + 1;
    std::vector<uint32_t> h(t8w + 1, 0u);
    if (one_class) {
        h[0] = n;   // every pair in the largest class (host-side lengths, BatchShape::one_t8): no read-back
    } else {
        // the class sizes, read back: one synchronisation of the stream (gasalx.h, max_t_len)
        HIPCHK(hipMemsetAsync(hist, 0, sh, st));
        rev_hist_kernel<<<sort_grid(n), 256, sh, st>>>(REV_PLAIN, A.tlen, nullptr, n, t8w, hist);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(h.data(), hist, sh, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    int classes = 0;
    for (uint32_t b = 0; b <= t8w; b++) classes += h[b] != 0;
    A.perm = nullptr;
    if (classes > 1) {                                       // counting sort: longest targets first
        rev_scan_kernel<<<1, 256, 0, st>>>(hist, cursor, t8w + 1);
        rev_scatter_kernel<<<sort_grid(n), 256, 2 * sh, st>>>(REV_PLAIN, A.tlen, nullptr, n, t8w, cursor, perm);
        HIPCHK(hipGetLastError());
        A.perm = perm;
    }
    HIPCHK(ws.misc.reserve(n + 64));
    HIPCHK(hipMemsetAsync(ws.misc.p, 0, n, st));            // slots no class launch covers stay declined
    ws.pk_flags = n; ws.pk_ppb = 1; ws.pk_pairs = n;
    WfArgs P16 = A;
    P16.lds_stride = pl.lds16_stride;
    P16.fast16 = 1;
    P16.vmin = pl.vmin;
    P16.handled = ws.misc.as<uint8_t>();
    const uint32_t ppb16 = kWavesPerBlock * (64 / 8) * 2;
    uint32_t slot = 0;
    for (uint32_t b = 0; b <= t8w; slot += h[b], b++) {
        const uint32_t R = t8w - b;                          // bucket b: padded target of 8R
        if (!h[b] || R == 0) continue;
        Wf16Fn fn = wf16_tq_lookup((int)R);
        if (!fn) { set_error("no packed TAIL=QUERY/BOTH instance"); return GASALX_EUNSUPPORTED; }
        if (pl.lds16_bytes > 64 * 1024)
            HIPCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)pl.lds16_bytes));
        P16.slot0 = slot;
        P16.n = slot + h[b];
        hipLaunchKernelGGL(fn, dim3(grid_for(h[b], ppb16)), dim3(kBlock), pl.lds16_bytes, st, P16);
        HIPCHK(hipGetLastError());
    }
    A.skip = ws.misc.as<uint8_t>();
    A.skip_ppb = 1;
    A.skip_p1 = 0xFFFFFFFFu;
    WfFn fn = wf_lookup(pl.wf_algo, pl.keys, false, pl.G, pl.R);
    if (!fn) { set_error("no wavefront instance"); return GASALX_EUNSUPPORTED; }
    if (pl.lds_bytes > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds_bytes));
    hipLaunchKernelGGL(fn, dim3(wf_grid(n, pl.G, A.skip != nullptr)), dim3(kBlock), pl.lds_bytes, st, A);
    HIPCHK(hipGetLastError());
    return GASALX_OK;
}

// SEMI TAIL=NONE outputs (PLAN_CONST): score MINUS_INF, query_batch_end = maxXY_x =
// ref_len, target_batch_end = maxXY_y = read_len (semiglobal_kernel_template.h:49-51,63-64,
// 206-218: Q10's end conventions with no tail block run)
__global__ __launch_bounds__(256) void semi_tail_none_kernel(int32_t *score, int32_t *qend, int32_t *tend,
                                                             const uint32_t *qlen, const uint32_t *tlen, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    score[i] = -32768;
    if (qend) qend[i] = (int32_t)tlen[i];
    if (tend) tend[i] = (int32_t)qlen[i];
}

// WITH_START on the wavefront kernels (start.hpp): the same kernel reading the forward
// sequences backwards over slots sorted by reversed target length, and the map of its ends
// to the start cell.
static int start_reverse(Workspace &ws, int mode, const gasalx_params &p, const uint8_t *q, const uint8_t *t,
                         int packed, const gasalx_batch &b, const BatchShape &shape, const int32_t *score,
                         const int32_t *qend, const int32_t *tend, int32_t *qstart, int32_t *tstart, hipStream_t st) {
    const uint32_t n = b.n_alns;
    const uint32_t q8 = pad8(shape.max_q), t8 = pad8(shape.max_t), t8w = t8 / 8, q8w = q8 / 8;
    // LOCAL: slots that stop early (the drift sweep's lstop) share waves (start.hpp rev_bucket),
    // and the query words come first when the two-key histogram fits LDS
    const bool lstop = mode == REV_LOCAL;
    const bool qkey = lstop && (size_t)(q8w + 1) * (t8w + 1) * 8 <= 64 * 1024;
    const uint32_t nb = qkey ? (q8w + 1) * (t8w + 1) : t8w + 1;
    HIPCHK(ws.rev_meta.reserve((size_t)n * 4 * 6 + (size_t)nb * 8 + 64));
    uint32_t *meta = ws.rev_meta.as<uint32_t>();
    uint32_t *rqlen = meta, *rtlen = meta + n;
    int32_t *rscore = reinterpret_cast<int32_t *>(meta + 2 * (size_t)n);
    int32_t *rqend = rscore + n, *rtend = rscore + 2 * (size_t)n;
    uint32_t *perm = meta + 5 * (size_t)n;
    uint32_t *hist = meta + 6 * (size_t)n, *cursor = hist + nb;
    // counting sort of the pairs by reversed target words (longest first)
    const size_t sh = (size_t)nb * 4;
    if (2 * sh > 64 * 1024) { set_error("WITH_START: target too long for the slot sort"); return GASALX_ERANGE; }
    HIPCHK(hipMemsetAsync(hist, 0, sh, st));
    const int32_t *skey = lstop ? score : nullptr;
    const uint32_t *kql = qkey ? b.q_lens : nullptr;
    rev_hist_kernel<<<sort_grid(n), 256, sh, st>>>(mode, b.t_lens, tend, n, t8w, hist, skey, p.match, kql, qend,
                                                       q8w, nb);
    rev_scan_kernel<<<1, 256, 0, st>>>(hist, cursor, nb);
    rev_scatter_kernel<<<sort_grid(n), 256, 2 * sh, st>>>(mode, b.t_lens, tend, n, t8w, cursor, perm, nullptr,
                                                              skey, p.match, kql, qend, q8w, nb);
    rev_len_kernel<<<grid_for(n, 256), 256, 0, st>>>(mode, q, b.q_offsets, b.q_lens, b.t_lens, qend, tend, packed,
                                                      (uint32_t)(p.n_code & 0xF), n, rqlen, rtlen);
    HIPCHK(hipGetLastError());
    gasalx_params pr = p;
    pr.start_pos = 0;
    BatchShape rs; rs.max_q = q8; rs.max_t = t8; rs.n = n;
    const Plan pl = make_plan(pr, rs, false);
    if (pl.kind != PLAN_WAVEFRONT) { set_error("reverse pass has no wavefront plan"); return GASALX_EUNSUPPORTED; }
    WfArgs A;
    std::memset(&A, 0, sizeof(A));
    A.q = q; A.t = t;
    A.qoff = b.q_offsets; A.toff = b.t_offsets; A.qlen = rqlen; A.tlen = rtlen;
    A.rev = 1;
    A.perm = perm;
    A.perm_xkey = (mode == REV_SEMI || qkey) ? 1 : 0;   // sorted by the register-axis words first
    A.score = rscore; A.qend = rqend; A.tend = rtend;
    A.stop = mode == REV_SEMI ? score : nullptr;     // the forward score per pair
    A.lstop = lstop ? score : nullptr;
    A.n = n;
    A.packed = packed;
    int rc = launch_wavefront(ws, pl, pr, A, st);
    if (rc) return rc;
    start_map_kernel<<<grid_for(n, 256), 256, 0, st>>>(mode, score, b.q_lens, rqlen, b.t_lens, tend, rscore, rqend,
                                                        rtend, qstart, tstart, n);
    HIPCHK(hipGetLastError());
    return GASALX_OK;
}

// GASALX_SORT=0/1 overrides the caller's BatchShape::sort (A/B and probes)
static bool sort_wanted(const BatchShape &s) {
    static const int force = [] {
        const char *e = std::getenv("GASALX_SORT");
        return e ? std::atoi(e) : -1;
    }();
    return force < 0 ? s.sort : force != 0;
}

// Uneven lengths, two pairs per lane (banded16 / local16): pair up slots of equal
// tile geometry (QR, TR) by a counting sort on it.  *perm stays NULL (identity)
// for even batches, small ones and geometry counts whose histogram exceeds LDS.
static int geometry_perm(Workspace &ws, const gasalx_batch &b, const BatchShape &shape, uint32_t n, hipStream_t st,
                         const uint32_t **perm_out) {
    *perm_out = nullptr;
    const uint32_t trw = pad8(shape.max_t) / 8, nkeys = (pad8(shape.max_q) / 8) * trw;
    const size_t sh = (size_t)(nkeys + 1) * 4;
    if (!(sort_wanted(shape) && n >= 4096 && 2 * sh <= 64 * 1024)) return GASALX_OK;
    HIPCHK(ws.sort_meta.reserve((size_t)n * 8 + 2 * sh + 64));
    uint32_t *perm = ws.sort_meta.as<uint32_t>(), *klen = perm + n, *hist = klen + n, *cursor = hist + nkeys + 1;
    band16_key_kernel<<<grid_for(n, 256), 256, 0, st>>>(b.q_lens, b.t_lens, n, trw, klen);
    HIPCHK(hipMemsetAsync(hist, 0, sh, st));
    rev_hist_kernel<<<sort_grid(n), 256, sh, st>>>(REV_PLAIN, klen, nullptr, n, nkeys, hist);
    rev_scan_kernel<<<1, 256, 0, st>>>(hist, cursor, nkeys + 1);
    rev_scatter_kernel<<<sort_grid(n), 256, 2 * sh, st>>>(REV_PLAIN, klen, nullptr, n, nkeys, cursor, perm);
    HIPCHK(hipGetLastError());
    *perm_out = perm;
    return GASALX_OK;
}

// Everything after align_device's prologue, over the pairs of b (a whole batch or one
// chunk of it).  walk_qseq: the query codes the traceback walk reads when the CIGAR
// buffer overlays the query batch (copied once by the prologue), else NULL.
static int align_body(Workspace &ws, const gasalx_params &p, const Plan &pl, const gasalx_batch &b,
                      const gasalx_results &out, hipStream_t st, const BatchShape &shape, uint64_t cigar_cap,
                      const uint8_t *walk_qseq);

int align_device(Workspace &ws, const gasalx_params &p, const gasalx_batch &b, const gasalx_results &out,
                 hipStream_t st, const BatchShape &shape, uint64_t cigar_cap) {
    if (b.n_alns == 0 || b.q_bytes == 0 || b.t_bytes == 0) { set_error("empty batch"); return GASALX_EINVAL; }
    if ((b.q_bytes & 7) || (b.t_bytes & 7)) { set_error("batch bytes not a multiple of 8"); return GASALX_EINVAL; }
    if (!out.aln_score) { set_error("aln_score output required"); return GASALX_EINVAL; }
    if (p.algo == 6 && !b.seed_scores) { set_error("KSW needs seed_scores"); return GASALX_EINVAL; }
    if (shape.max_q == 0 || shape.max_t == 0) { set_error("zero-length sequence"); return GASALX_ERANGE; }
    const bool has_ops = b.q_ops && b.t_ops;
    // gasalx_packed_pairs reads the packed launch flags of this call only: a call that launches
    // no packed kernel (or reuses misc for other flags, the KSW / banded / local16 todo arrays)
    // must not leave the last call's count behind
    ws.pk_flags = 0;
    BatchShape sized = shape;
    sized.n = b.n_alns;
    Plan pl = make_plan(p, sized, has_ops);
    const uint32_t n = b.n_alns;
    const bool tb = p.start_pos == 2;

    // TB: the device cigar buffer starts as the unpacked query batch, as in the
    // reference where get_tb writes into unpacked_query_batch (get_tb.h:94,
    // gasal_align.cu:281); n_cigar_ops = query_batch_lens unless get_tb runs.
    if (tb && out.cigar && (const void *)out.cigar != (const void *)b.q_batch)
        HIPCHK(copy_d2d(out.cigar, b.q_batch, b.q_bytes, st));
    const bool runs_tb = tb && (p.algo == 1 || p.algo == 3) && pl.kind != PLAN_NONE;
    if (tb && out.n_cigar_ops && !runs_tb && (const void *)out.n_cigar_ops != (const void *)b.q_lens)
        HIPCHK(hipMemcpyAsync(out.n_cigar_ops, b.q_lens, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    if (pl.kind == PLAN_NONE) return GASALX_OK;   // UNKNOWN / MICROLOCAL: nothing launched

    // the walk writes CIGARs over the unpacked query batch when that is the cigar
    // buffer (get_tb.h:94) but the packed kernels' walk reads query codes from it:
    // give it a copy, taken before any walk runs
    const uint8_t *walk_qseq = nullptr;
    const bool cigar_on_query = out.cigar && (const uint8_t *)out.cigar < b.q_batch + b.q_bytes &&
                                b.q_batch < (const uint8_t *)out.cigar + (cigar_cap ? cigar_cap : b.q_bytes);
    if (runs_tb && out.cigar && out.n_cigar_ops && pl.kind == PLAN_WAVEFRONT && pl.packed16 && !pl.need_pack) {
        if (cigar_on_query) {
            HIPCHK(ws.packed_q.reserve(b.q_bytes));
            HIPCHK(hipMemcpyAsync(ws.packed_q.p, b.q_batch, b.q_bytes, hipMemcpyDeviceToDevice, st));
            walk_qseq = ws.packed_q.as<uint8_t>();
        }
    }

    // (one launch chain: the walk is latency-bound -- ~600 dependent steps whatever the batch size --
    // so splitting a call into halves whose walks overlap the next half's DP leaves the last walk
    // exposed and gained nothing; round 6 measured it, profiles/r06/)
    return align_body(ws, p, pl, b, out, st, sized, cigar_cap, walk_qseq);
}

static int align_body(Workspace &ws, const gasalx_params &p, const Plan &pl, const gasalx_batch &b,
                      const gasalx_results &out, hipStream_t st, const BatchShape &shape, uint64_t cigar_cap,
                      const uint8_t *walk_qseq) {
    const bool has_ops = b.q_ops && b.t_ops;
    const uint32_t n = b.n_alns;
    const bool tb = p.start_pos == 2;
    const bool runs_tb = tb && (p.algo == 1 || p.algo == 3) && pl.kind != PLAN_NONE;
    if (pl.kind == PLAN_CONST) {
        semi_tail_none_kernel<<<grid_for(n, 256), 256, 0, st>>>(out.aln_score, out.q_end, out.t_end, b.q_lens,
                                                                      b.t_lens, n);
        HIPCHK(hipGetLastError());
        return GASALX_OK;
    }

    const uint8_t *qsrc = b.q_batch, *tsrc = b.t_batch;
    int packed = p.is_packed ? 1 : 0;
    if (pl.need_pack) {
        const uint32_t qw = b.q_bytes / 8, tw = b.t_bytes / 8;
        HIPCHK(ws.packed_q.reserve((size_t)qw * 4 + 16));
        HIPCHK(ws.packed_t.reserve((size_t)tw * 4 + 16));
        if (p.is_packed) {
            HIPCHK(hipMemcpyAsync(ws.packed_q.p, b.q_batch, (size_t)qw * 4, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipMemcpyAsync(ws.packed_t.p, b.t_batch, (size_t)tw * 4, hipMemcpyDeviceToDevice, st));
        } else {
            pack_kernel<<<std::min(grid_for(qw, 256), 4096), 256, 0, st>>>(b.q_batch, ws.packed_q.as<uint32_t>(), qw);
            pack_kernel<<<std::min(grid_for(tw, 256), 4096), 256, 0, st>>>(b.t_batch, ws.packed_t.as<uint32_t>(), tw);
        }
        if (has_ops) {
            revcomp_kernel<<<grid_for(n, 256), 256, 0, st>>>(ws.packed_q.as<uint32_t>(), ws.packed_t.as<uint32_t>(),
                                                             b.q_lens, b.t_lens, b.q_offsets, b.t_offsets, b.q_ops,
                                                             b.t_ops, n, p.n_code);
            // with isPacked the reference's packed buffer aliases the unpacked one, so
            // the reversed words are what the cigar D2H copy sees (ctors.cpp:64-68)
            if (tb && out.cigar && p.is_packed)
                HIPCHK(hipMemcpyAsync(out.cigar, ws.packed_q.p, (size_t)qw * 4, hipMemcpyDeviceToDevice, st));
        }
        qsrc = ws.packed_q.as<uint8_t>();
        tsrc = ws.packed_t.as<uint8_t>();
        packed = 1;
    }

    // traceback storage: one word per (8-column strip, padded query row); the
    // packed traceback kernels' skewed uint16 layout needs (t8 + G + 2) / 4 windows
    // of G*R 16-bit entries instead (wavefront16.hpp)
    uint64_t tb_words = (uint64_t)pad8(shape.max_q) * (pad8(shape.max_t) / 8);
    if (pl.packed16 && pl.tb)
        tb_words = std::max<uint64_t>(tb_words, (((uint64_t)pl.G16 * pl.R16 * ((pad8(shape.max_t) + pl.G16 + 2) / 4) / 2 + 3) & ~3ull));
    int32_t *qend = out.q_end, *tend = out.t_end;
    const bool wf_start = pl.kind == PLAN_WAVEFRONT && (p.algo == 3 || p.algo == 2) && p.start_pos == 1 &&
                          (out.q_start || out.t_start);
    // (whole groups of 8 pairs: the packed kernels' interleaved layout, tb_store_window)
    // the band path's full-matrix direction words serve its fallback list only: GASALX_TB_FBCAP slots
    // (131,072 by default), the list then aligned in chunks of that many (the rest reserve every pair)
    const uint32_t fb_cap = std::max(64, env_int("GASALX_TB_FBCAP", 131072));
    const uint32_t n_tb = (pl.kind == PLAN_WAVEFRONT && pl.packed16 && pl.tb_band) ? std::min(n, fb_cap) : n;
    if (runs_tb) HIPCHK(ws.tb.reserve((size_t)((n_tb + 7) & ~7u) * tb_words * 4 + 64));
    if (runs_tb || wf_start) {
        if ((p.algo == 3 || p.algo == 2) && (!qend || !tend)) {
            HIPCHK(ws.ends_q.reserve((size_t)n * 4));
            HIPCHK(ws.ends_t.reserve((size_t)n * 4));
            if (!qend) qend = ws.ends_q.as<int32_t>();
            if (!tend) tend = ws.ends_t.as<int32_t>();
        }
    }

    const uint32_t *slot_of = nullptr;   // pair -> slot when the wavefront launch ran sorted
    uint32_t tb_q8 = 0;                  // the packed TB kernels' interleaved layout
    WfArgs A;                            // the wavefront launch (kept for the traceback fallback)
    std::memset(&A, 0, sizeof(A));
    uint32_t *fb_count = nullptr;        // band traceback: pairs handed to the full-matrix fallback
    if (pl.kind == PLAN_WAVEFRONT) {
        A.q = qsrc; A.t = tsrc;
        A.qoff = b.q_offsets; A.toff = b.t_offsets; A.qlen = b.q_lens; A.tlen = b.t_lens;
        A.score = out.aln_score;
        A.qend = (p.algo == 1) ? nullptr : qend;
        A.tend = (p.algo == 1) ? nullptr : tend;
        A.tb = ws.tb.as<uint32_t>();
        A.tb_pair_words = tb_words;
        A.n = n;
        A.packed = packed;
        // uneven lengths: a wave's step count is set by its longest step-axis
        // sequence (target; query for the transposed SEMI kernel), so run the
        // slots in length order (counting sort, longest first)
        // (semi_tq sorts by target class itself; a launch whose waves hold fewer than 8 pairs --
        // the small-batch shapes, G >= 32 -- gains nothing from the order and would pay the three
        // sort launches: a 5,000-pair batch of the reference's sample data, profiles/r06/boundary)
        const int gsort = pl.packed16 ? pl.G16 : pl.G;
        if (sort_wanted(shape) && n >= 4096 && !pl.semi_tq && 2 * (64 / std::max(gsort, 1)) >= 8) {
            const uint32_t s8w = pad8(pl.wf_algo == WF_SEMI ? shape.max_q : shape.max_t) / 8;
            const uint32_t *slen = pl.wf_algo == WF_SEMI ? b.q_lens : b.t_lens;
            const size_t sh = (size_t)(s8w + 1) * 4;
            if (2 * sh <= 64 * 1024) {
                HIPCHK(ws.sort_meta.reserve((size_t)n * 8 + (size_t)(s8w + 1) * 8 + 64));
                uint32_t *perm = ws.sort_meta.as<uint32_t>(), *inv = perm + n, *hist = inv + n, *cursor = hist + s8w + 1;
                HIPCHK(hipMemsetAsync(hist, 0, sh, st));
                rev_hist_kernel<<<sort_grid(n), 256, sh, st>>>(REV_PLAIN, slen, nullptr, n, s8w, hist);
                rev_scan_kernel<<<1, 256, 0, st>>>(hist, cursor, s8w + 1);
                rev_scatter_kernel<<<sort_grid(n), 256, 2 * sh, st>>>(REV_PLAIN, slen, nullptr, n, s8w,
                                                                          cursor, perm, inv);
                HIPCHK(hipGetLastError());
                A.perm = perm;
                slot_of = inv;
            }
        }
        // unsorted waves hold consecutive pairs: interleave their direction chunks
        A.tb_q8 = (pl.packed16 && pl.tb && !pl.tb_band && !A.perm) ? 1u : 0u;
        tb_q8 = A.tb_q8;
        if (pl.tb_band && runs_tb) {
            // band recomputation buffers per wave of the packed launch (wavefront16.hpp); a mixed-
            // shape launch (tail_shape) keeps its second region's after the first's
            const uint32_t ppb16 = kWavesPerBlock * (64 / pl.G16) * 2;
            A.n = n;
            const TailShape tail = tail_shape(pl, p, A, n);
            const uint64_t waves = (uint64_t)(tail.fn ? tail.b0 : grid_for(n, ppb16)) * kWavesPerBlock;
            const uint64_t waves2 = tail.fn ? (uint64_t)grid_for(n - tail.p0, tail.ppb) * kWavesPerBlock : 0;
            const uint32_t wd2 = tail.fn ? (((uint32_t)(tail.R2 + 2 * pl.band_w) + 3u) & ~3u) : 4u;
            const uint64_t cpw1 = waves * 2 * pl.R16 * 64, cpw2 = waves2 * 2 * tail.R2 * 64;   // words
            const uint64_t st1 = waves * 64 * band_stream_words(pl.band_wd), st2 = waves2 * 64 * band_stream_words(wd2);
            const uint64_t fl1 = waves * 64 * (pl.band_wd / 4) * (pl.R16 / 4), fl2 = waves2 * 64 * (wd2 / 4) * (tail.R2 / 4);
            HIPCHK(ws.band_cp.reserve((cpw1 + cpw2) * 4 + 64));
            HIPCHK(ws.band_stm.reserve((st1 + st2) * 8 + 64));
            HIPCHK(ws.band_fl.reserve((fl1 + fl2) * 16 + 64));
            HIPCHK(ws.band_fb.reserve((size_t)n * 4 + grid_for(n, ppb16) + 256));
            A.cp = ws.band_cp.as<uint32_t>();
            A.stm = ws.band_stm.as<uint2>();
            A.bflags = ws.band_fl.as<uint4>();
            A.band_w = pl.band_w;
            A.band_wd = pl.band_wd;
            A.cp2 = A.cp + cpw1;
            A.stm2 = A.stm + st1;
            A.bflags2 = A.bflags + fl1;
            A.band_wd2 = wd2;
            fb_count = ws.band_fb.as<uint32_t>();
        }
        int rc = pl.semi_tq ? launch_semi_tq(ws, pl, p, A, st, shape.one_t8) : launch_wavefront(ws, pl, p, A, st);
        if (rc) return rc;
        if (wf_start) {
            rc = start_reverse(ws, p.algo == 3 ? REV_LOCAL : REV_SEMI, p, qsrc, tsrc, packed, b, shape, out.aln_score,
                               qend, tend, out.q_start, out.t_start, st);
            if (rc) return rc;
        }
    } else {
        GenArgs A;
        std::memset(&A, 0, sizeof(A));
        A.qw = ws.packed_q.as<uint32_t>(); A.tw = ws.packed_t.as<uint32_t>();
        A.qoff = b.q_offsets; A.toff = b.t_offsets; A.qlen = b.q_lens; A.tlen = b.t_lens;
        A.seed = b.seed_scores;
        A.score = out.aln_score; A.qend = qend; A.tend = tend; A.qstart = out.q_start; A.tstart = out.t_start;
        A.score2 = out.aln_score2; A.qend2 = out.q_end2; A.tend2 = out.t_end2;
        A.tb = ws.tb.as<uint32_t>(); A.tb_pair_words = tb_words;
        const uint32_t q8 = pad8(shape.max_q), t8 = pad8(shape.max_t);
        uint32_t maxq = p.max_query_len > 0 ? (uint32_t)p.max_query_len : std::max(q8, t8);
        if (maxq < q8) { set_error("max_query_len smaller than a padded query"); return GASALX_ERANGE; }
        if (p.algo == 2 && p.start_pos == 1 && maxq < t8) {
            set_error("semi-global WITH_START needs max_query_len >= padded target length");
            return GASALX_ERANGE;
        }
        A.rows_cap = std::max(maxq, q8) + 8;
        A.maxq = (int32_t)maxq;
        A.rev_words = maxq / 8 + 1;
        A.n = n;
        A.a = p.match; A.b = p.mismatch; A.o = p.gap_open; A.e = p.gap_extend;
        A.nval = p.n_code & 0xF; A.has_npen = p.has_n_penalty; A.npen = p.n_penalty;
        A.start_pos = p.start_pos; A.second = p.second_best; A.head = p.head; A.tail = p.tail;
        A.kbw = p.k_band >> 3;
        const size_t rows_elems = (size_t)A.rows_cap * n;
        if (p.algo == 6) {
            const size_t ke = (size_t)(shape.max_q + 8) * n;
            HIPCHK(ws.rows_h.reserve(ke * 8));
            // 8-bit (h, e) entries, then 16-bit, then int2, each for the pairs whose score
            // bound does not fit the level before
            uint8_t *todo = nullptr;
            {
                HIPCHK(ws.misc.reserve(n));
                HIPCHK(hipMemsetAsync(ws.misc.p, 0, n, st));
                todo = ws.misc.as<uint8_t>();
                // two pairs per lane in 16-bit halves first (ksw16.hpp): the pairs it takes
                // get todo = 0xFF, the rest run the levels below (GASALX_KSW16=0: levels only)
                const int32_t nsc = p.has_n_penalty ? -p.n_penalty : 0;
                const int32_t kofs = std::max({0, p.mismatch, -nsc, -p.match});
                const bool k16 = env_flag("GASALX_KSW16", true) && p.gap_open >= 0 && p.gap_extend >= 0 &&
                                 p.gap_open + p.gap_extend <= 0x300 && p.match + kofs <= 255 &&
                                 -p.mismatch + kofs <= 255 && nsc + kofs <= 255 && shape.max_q <= 254;
                if (k16) {
                    Ksw16Args K;
                    std::memset(&K, 0, sizeof(K));
                    K.qw = A.qw; K.tw = A.tw;
                    K.qoff = b.q_offsets; K.toff = b.t_offsets; K.qlen = b.q_lens; K.tlen = b.t_lens;
                    K.seed = b.seed_scores;
                    K.score = out.aln_score; K.qend = qend; K.tend = tend;
                    K.todo = todo;
                    K.n = n; K.n_lanes = (n + 1) / 2; K.cols = (shape.max_q + 3) & ~1u;
                    K.stride = grid_for(K.n_lanes, 256) * 256;
                    K.a = p.match; K.b = p.mismatch; K.o = p.gap_open; K.e = p.gap_extend;
                    K.nval = p.n_code & 0xF; K.has_npen = p.has_n_penalty; K.npen = p.n_penalty;
                    K.kofs = kofs;
                    // the entry row in registers when the padded query fits an instance
                    // (selector words in LDS: QC / 2 words per lane), else the global array
                    int qc = 0;
                    for (int c : {64, 96, 160})
                        if (K.cols <= (uint32_t)c) { qc = c; break; }
                    if (qc) {
                        void (*fn)(Ksw16Args) = qc == 64 ? &ksw16_kernel<64> : qc == 96 ? &ksw16_kernel<96> : &ksw16_kernel<160>;
                        const size_t lds = (size_t)4 * (qc / 2) * 64 * 4;
                        if (lds > 64 * 1024)
                            HIPCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                        hipLaunchKernelGGL(fn, dim3(grid_for(K.n_lanes, 256)), dim3(256), lds, st, K);
                    } else {
                        const size_t ent_words = (size_t)K.cols * K.stride, sel_words = (size_t)(K.cols / 2) * K.stride;
                        HIPCHK(ws.rows_e.reserve((ent_words + sel_words) * 4 + 64));
                        K.ent = ws.rows_e.as<uint32_t>(); K.sel = K.ent + ent_words;
                        ksw16_kernel<0><<<grid_for(K.n_lanes, 256), 256, 0, st>>>(K);
                    }
                    HIPCHK(hipGetLastError());
                }
                // level 0 with the entries in LDS when two blocks of >= 64 threads fit
                // a CU, for batches of up to 4 waves per SIMD: LDS then holds 2 waves
                // per SIMD, and larger batches run faster on the global array with its
                // higher occupancy (200 K config-2 pairs: 806 -> 890 GCUPS; 1 M: 1,320
                // global, 1,146 LDS).  GASALX_KSW_LDS=0/1 forces either (A/B)
                const char *kl = std::getenv("GASALX_KSW_LDS");
                const bool lds_on = kl ? std::atoi(kl) != 0 : n <= 4u * 1024u * 64u;
                uint32_t tpb = 0;
                size_t lds = 0;
                if (lds_on)
                    for (uint32_t t : {256u, 128u, 64u}) {
                        lds = (size_t)t * (shape.max_q + 2) * 2;
                        if (2 * lds <= 160 * 1024) { tpb = t; break; }
                    }
                if (tpb) {
                    if (lds > 64 * 1024)
                        HIPCHK(hipFuncSetAttribute((const void *)&gen_ksw_kernel<0, true>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                    gen_ksw_kernel<0, true><<<grid_for(n, tpb), tpb, lds, st>>>(A, ws.rows_h.p, todo);
                } else {
                    gen_ksw_kernel<0><<<grid_for(n, 256), 256, 0, st>>>(A, ws.rows_h.p, todo);
                }
                gen_ksw_kernel<1><<<grid_for(n, 256), 256, 0, st>>>(A, ws.rows_h.p, todo);
            }
            gen_ksw_kernel<2><<<grid_for(n, 256), 256, 0, st>>>(A, ws.rows_h.p, todo);
        } else {
            HIPCHK(ws.rows_h.reserve(rows_elems * 2));
            HIPCHK(ws.rows_e.reserve(rows_elems * 2));
            A.rowH = ws.rows_h.as<int16_t>(); A.rowE = ws.rows_e.as<int16_t>();
            if (p.algo == 3) {
                if (pl.local16) {
                    Local16Args D;
                    std::memset(&D, 0, sizeof(D));
                    D.qw = A.qw; D.tw = A.tw;
                    D.qoff = b.q_offsets; D.toff = b.t_offsets; D.qlen = b.q_lens; D.tlen = b.t_lens;
                    D.score = out.aln_score; D.qend = qend; D.tend = tend;
                    D.score2 = out.aln_score2; D.qend2 = out.q_end2; D.tend2 = out.t_end2;
                    D.n = n; D.n_lanes = (n + 1) / 2;
                    D.a = p.match; D.b = p.mismatch; D.oe = p.gap_open + p.gap_extend; D.e = p.gap_extend;
                    D.nval = A.nval; D.sn = local16_sn(p); D.k = local16_k(p); D.base = local16_base(p);
                    HIPCHK(ws.misc.reserve(n));
                    HIPCHK(hipMemsetAsync(ws.misc.p, 0, n, st));
                    D.todo = ws.misc.as<uint8_t>();
                    D.rows_cap = q8;
                    HIPCHK(ws.aux.reserve((size_t)q8 * ((D.n_lanes + 63) / 64) * 64 * 8 + 64));
                    D.rows = ws.aux.as<uint2>();
                    {
                        const int rc = geometry_perm(ws, b, shape, n, st, &D.perm);
                        if (rc) return rc;
                    }
                    // 3 waves per SIMD (162 VGPRs): 2 waves 2 % and 4 waves (spills) 5-15 % slower
                    local2nd16_kernel<3><<<grid_for(D.n_lanes, 256), 256, 0, st>>>(D);
                    HIPCHK(hipGetLastError());
                    A.todo = D.todo;
                }
                gen_local_kernel<<<grid_for(n, 256), 256, 0, st>>>(A);
            }
            else if (p.algo == 2) {
                if (p.start_pos == 1) {
                    HIPCHK(ws.rev.reserve((size_t)2 * A.rev_words * n * 4));
                    A.rev = ws.rev.as<uint32_t>();
                }
                gen_semi_kernel<<<grid_for(n, 256), 256, 0, st>>>(A);
            } else if (p.algo == 5) {
                if (pl.band16) {
                    BandArgs D;
                    std::memset(&D, 0, sizeof(D));
                    D.qw = A.qw; D.tw = A.tw;
                    D.qoff = b.q_offsets; D.toff = b.t_offsets; D.qlen = b.q_lens; D.tlen = b.t_lens;
                    D.score = out.aln_score; D.qend = qend; D.tend = tend;
                    D.n = n; D.n_lanes = (n + 1) / 2;
                    D.a = p.match; D.b = p.mismatch; D.oe = p.gap_open + p.gap_extend; D.e = p.gap_extend;
                    D.kbw = A.kbw; D.nval = A.nval; D.base = band16_base(p);
                    HIPCHK(ws.misc.reserve(n));
                    HIPCHK(hipMemsetAsync(ws.misc.p, 0, n, st));
                    D.todo = ws.misc.as<uint8_t>();
                    HIPCHK(ws.aux.reserve((size_t)q8 * D.n_lanes * 8 + 64));
                    D.rows = ws.aux.as<uint2>();
                    {
                        const int rc = geometry_perm(ws, b, shape, n, st, &D.perm);
                        if (rc) return rc;
                    }
                    band16_kernel<<<grid_for(D.n_lanes, 256), 256, 0, st>>>(D);
                    HIPCHK(hipGetLastError());
                    A.todo = D.todo;
                }
                gen_banded_kernel<<<grid_for(n, 256), 256, 0, st>>>(A);
            }
            else gen_global_kernel<<<grid_for(n, 256), 256, 0, st>>>(A);
        }
        HIPCHK(hipGetLastError());
    }

    if (runs_tb && out.cigar && out.n_cigar_ops) {
        TbArgs T;
        T.tb = ws.tb.as<uint32_t>(); T.tb_pair_words = tb_words;
        T.qlen = b.q_lens; T.tlen = b.t_lens; T.qoff = b.q_offsets;
        T.score = out.aln_score; T.qend = qend; T.tend = tend;
        T.qstart = out.q_start; T.tstart = out.t_start;
        T.cigar = out.cigar; T.n_ops = out.n_cigar_ops; T.n = n;
        T.cigar_cap = cigar_cap ? cigar_cap : b.q_bytes;
        T.a = p.match; T.b = p.mismatch; T.o = p.gap_open; T.e = p.gap_extend;
        T.is_local = p.algo == 3;
        T.pk_flags = nullptr;
        T.pk_ppb = 1; T.pk_R = 1; T.pk_G = 1; T.pk_rmagic = 0; T.pk_q8 = 0;
        T.pk_fix = nullptr;
        T.pk_p1 = 0xFFFFFFFFu; T.pk_b1 = 0; T.pk_ppb2 = 1;
        T.band2 = nullptr; T.band_wd2 = 4; T.pk_R2 = 4; T.pk_G2 = 1; T.pk_ppw2 = 1; T.pk_rmagic2 = 0;
        T.slot_of = slot_of;
        T.sc_nn = p.has_n_penalty ? -p.n_penalty : p.match;   // GLOBAL: N == N is a match unless N_PENALTY
        T.qseq = qsrc; T.tseq = tsrc; T.toff = b.t_offsets; T.seq_packed = packed;
        if (walk_qseq) T.qseq = walk_qseq;   // align_device's copy of the query codes
        T.nval = p.n_code & 0xF; T.has_npen = p.has_n_penalty; T.npen = p.n_penalty;
        if (pl.kind == PLAN_WAVEFRONT && pl.packed16) {
            T.pk_flags = ws.misc.as<uint8_t>();
            T.pk_ppb = kWavesPerBlock * (64 / pl.G16) * 2;
            T.pk_R = pl.R16;
            T.pk_G = pl.G16;
            T.pk_rmagic = (uint32_t)((0x100000000ull + pl.R16 - 1) / pl.R16);
            T.pk_fix = ws.aux.as<int32_t>();
            T.pk_q8 = tb_q8;
            T.pk_p1 = ws.pk_p1; T.pk_b1 = ws.pk_b1; T.pk_ppb2 = ws.pk_ppb2;   // the launch's flag ranges
        }
        T.band = nullptr; T.band_w = 0; T.band_wd = 4; T.pk_ppw = 1;
        T.fb_list = T.fb_count = nullptr;
        T.list = T.n_dev = nullptr;
        T.n_dev_off = 0; T.tb_slot = 0;
        if (fb_count) {
            T.band = ws.band_fl.as<uint4>();
            T.band_w = pl.band_w; T.band_wd = pl.band_wd;
            T.pk_ppw = 2 * (64 / pl.G16);
            if (T.pk_p1 != 0xFFFFFFFFu) {   // the second region of a mixed-shape launch (tail_shape)
                const TailShape tail = tail_shape(pl, p, A, n);
                if (!tail.fn || tail.p0 != T.pk_p1) { set_error("band traceback: tail shape changed"); return GASALX_EINVAL; }
                T.band2 = A.bflags2;
                T.band_wd2 = A.band_wd2;
                T.pk_R2 = tail.R2; T.pk_G2 = tail.G2; T.pk_ppw2 = 2 * (64 / tail.G2);
                T.pk_rmagic2 = (uint32_t)((0x100000000ull + tail.R2 - 1) / tail.R2);
            }
            T.fb_count = fb_count;
            T.fb_list = fb_count + 64;
            HIPCHK(hipMemsetAsync(fb_count, 0, 4, st));
        }
        tb_kernel<<<grid_for(n, 256), 256, 0, st>>>(T);
        HIPCHK(hipGetLastError());
        if (fb_count) {
            // pairs whose path left the band (or whose block the packed launch declined): the
            // full-matrix packed traceback kernel over the list (slots = list positions; per-pair
            // flag layout at slot positions of the capped buffer), its int32 kernel for any block it
            // declines, and the walk again -- in chunks of n_tb list positions, each launch reading
            // the device-side count less its chunk's offset (empty chunks exit at once)
            Plan fp = pl;
            fp.tb_band = false;
            for (uint32_t k0 = 0; k0 < n; k0 += n_tb) {
                const uint32_t cn = std::min(n_tb, n - k0);
                WfArgs F = A;
                // the band walk has written CIGAR prefixes over the query batch when that is the
                // CIGAR buffer (get_tb.h:94): the DP reads align_device's copy of the codes then
                if (walk_qseq) F.q = walk_qseq;
                F.perm = T.fb_list + k0;
                F.n = cn;
                F.n_dev = fb_count;
                F.n_dev_off = k0;
                F.tb_slot = 1;
                F.tb_q8 = 0;
                F.cp = nullptr; F.stm = nullptr; F.bflags = nullptr;
                int rc = launch_wavefront(ws, fp, p, F, st);
                if (rc) return rc;
                TbArgs T2 = T;
                T2.band = nullptr;
                T2.list = T.fb_list + k0;
                T2.n = cn;
                T2.n_dev = fb_count;
                T2.n_dev_off = k0;
                T2.tb_slot = 1;
                T2.slot_of = nullptr;
                T2.pk_q8 = 0;
                T2.pk_p1 = 0xFFFFFFFFu;   // the fallback launch is one shape (its n_dev excludes the tail)
                T2.fb_list = T2.fb_count = nullptr;
                tb_kernel<<<grid_for(cn, 256), 256, 0, st>>>(T2);
                HIPCHK(hipGetLastError());
            }
        }
    }
    return GASALX_OK;
}

// ----------------------------------------------------------------------------
constexpr int kHmmRows = 8;   // read rows per lane
using HmmFn = void (*)(HmmArgs);
template <bool QUALS, bool ABS>
static HmmFn hmm_lookup(int G) {
    switch (G) {
        case 4: return &pairhmm_kernel<4, kHmmRows, QUALS, ABS>;
        case 8: return &pairhmm_kernel<8, kHmmRows, QUALS, ABS>;
        case 16: return &pairhmm_kernel<16, kHmmRows, QUALS, ABS>;
        case 32: return &pairhmm_kernel<32, kHmmRows, QUALS, ABS>;
        case 64: return &pairhmm_kernel<64, kHmmRows, QUALS, ABS>;
        default: return nullptr;
    }
}

// lanes per pair for a read of max_r rows: `rows` read rows per lane, G in {4, ..., 64}
static int hmm_group(uint32_t max_r, int rows) {
    for (int g : {4, 8, 16, 32, 64})
        if ((uint32_t)g * rows >= max_r) return g;
    return 0;
}
int pairhmm_group(uint32_t max_r) { return hmm_group(max_r, kHmmRows); }

// One launch over slots [slot0, slot1) of A (A.perm maps slots to pairs, or NULL).
static int pairhmm_launch(HmmArgs A, bool quals, uint32_t max_r, uint32_t slot0, uint32_t slot1, uint32_t max_h,
                          hipStream_t st) {
    const int rows = kHmmRows;
    const int G = hmm_group(max_r, rows);
    if (slot1 <= slot0) return GASALX_OK;
    if (!G) { set_error("PairHMM read longer than 512"); return GASALX_ERANGE; }
    A.slot0 = slot0;
    A.n = slot1;
    A.lds_stride = (std::max<uint32_t>(max_h, 4) + 3) & ~3u;
    // reads shorter than the group's rows: the top lane's first row is virtual and
    // absorbs the boundary (pairhmm.hpp ABS)
    const bool absorb = (uint32_t)G * rows > max_r;
    // haplotype slots, then the per-lane prior tables (pairhmm.hpp): 4 waves x 4 codes x
    // rows x 64 lanes x 4 bytes
    const size_t lds = (((size_t)4 * (64 / G) * A.lds_stride + 15) & ~(size_t)15) + (size_t)4 * 4 * rows * 64 * 4;
    if (lds > 160 * 1024) { set_error("PairHMM haplotype too long"); return GASALX_ERANGE; }
    HmmFn fn = quals ? (absorb ? hmm_lookup<true, true>(G) : hmm_lookup<true, false>(G))
                     : (absorb ? hmm_lookup<false, true>(G) : hmm_lookup<false, false>(G));
    if (lds > 64 * 1024) HIPCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(fn, dim3(grid_for(slot1 - slot0, 4 * (64 / G))), dim3(256), lds, st, A);
    HIPCHK(hipGetLastError());
    return GASALX_OK;
}

int pairhmm_device(Workspace &ws, const gasalx_hmm_batch &b, float *result, hipStream_t st, uint32_t max_r,
                   uint32_t max_h) {
    (void)ws;
    if (b.n_pairs == 0) return GASALX_OK;
    HmmArgs A;
    std::memset(&A, 0, sizeof(A));
    A.reads = b.reads; A.roff = b.read_offsets; A.rlen = b.read_lens;
    A.qm = b.qm; A.delta = b.delta; A.xiksi = b.xiksi; A.alpha = b.alpha;
    A.haps = b.haps; A.hoff = b.hap_offsets; A.hlen = b.hap_lens;
    A.result = result;
    return pairhmm_launch(A, false, max_r, 0, b.n_pairs, max_h, st);
}

int pairhmm_quals_device(Workspace &ws, const gasalx_hmm_qual_batch &b, float *result, hipStream_t st,
                         const float *ph2pr_dev, const uint32_t *perm, const HmmClass *classes, int n_classes,
                         uint32_t max_r, uint32_t max_h) {
    (void)ws;
    if (b.n_pairs == 0) return GASALX_OK;
    HmmArgs A;
    std::memset(&A, 0, sizeof(A));
    A.reads = b.reads; A.roff = b.read_offsets; A.rlen = b.read_lens;
    A.bq = b.base_quals; A.iq = b.ins_quals; A.dq = b.del_quals; A.ph2pr = ph2pr_dev;
    A.haps = b.haps; A.hoff = b.hap_offsets; A.hlen = b.hap_lens;
    A.result = result;
    A.perm = perm;
    if (!classes) return pairhmm_launch(A, true, max_r, 0, b.n_pairs, max_h, st);
    for (int c = 0; c < n_classes; c++) {
        int rc = pairhmm_launch(A, true, classes[c].max_r, classes[c].slot0, classes[c].slot1,
                                classes[c].max_h, st);
        if (rc) return rc;
    }
    return GASALX_OK;
}

}  // namespace gx
