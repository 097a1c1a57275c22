// engine.hpp — host-side dispatcher of the MI355X engine.
//
// Replaces gasal_kernel_launcher + the KERNEL_SWITCH macro tree
// (Non-CDP/GASAL2/src/gasal_align.cu:10-25, gasal_align.h:7-107) and the CDP
// launch wrappers (CDP/GASAL2/src/gasal_align.cu:27-52) by one flat planner:
// (algo, start, head, tail, secondBest, lengths) -> one kernel family + launch
// shape, all launched from the host on one hipStream_t.  No device-side enqueue.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "gasalx.h"

namespace gx {

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t reserve(size_t need);   // grow-only
    void release();
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

struct Workspace {
    int device = 0;
    DevBuf packed_q, packed_t;      // packed words (RC / generic paths)
    DevBuf tb;                      // traceback direction words
    DevBuf rows_h, rows_e, rev;     // generic kernels' row buffers
    DevBuf ends_q, ends_t;          // LOCAL WITH_TB ends when the caller did not ask for them
    DevBuf misc;                    // packed kernels: per-block "aligned here" flags
    DevBuf aux;                     // packed GLOBAL+TB: H' of the traceback start cell per pair
    DevBuf rev_meta;                // WITH_START: reversed lengths, slot order, reverse-pass results
    DevBuf sort_meta;               // length sort of the forward pass: perm, inverse, histogram
    DevBuf band_cp, band_stm, band_fl;   // GLOBAL+TB band recomputation: checkpoints, hand-offs, flags
    DevBuf band_fb;                 // its fallback: count, then the list of pairs, then the launch's flags
    DevBuf kseg;                    // packed LOCAL keys by segments: the finished segments' keys per wave
    // the last packed launch's "aligned here" flags in misc (gasalx_packed_pairs): flag count, pairs
    // per flag, pairs of the launch (0 flags: no packed launch yet)
    uint32_t pk_flags = 0, pk_ppb = 0, pk_pairs = 0;
    // a mixed-shape launch (wavefront16.hpp wf16_mix_kernel): flags from pk_b1 on cover pk_ppb2 pairs
    // each, from pair pk_p1 on (pk_p1 = 0xFFFFFFFF: one block size)
    uint32_t pk_p1 = 0xFFFFFFFFu, pk_b1 = 0, pk_ppb2 = 1;
    void release_all();
};

// PLAN_CONST: outputs that do not depend on the DP (SEMI TAIL=NONE, score-only)
enum PlanKind { PLAN_NONE = 0, PLAN_WAVEFRONT, PLAN_GENERIC, PLAN_CONST };

struct Plan {
    PlanKind kind = PLAN_NONE;
    int wf_algo = 0;        // WfAlgo
    bool keys = false, tb = false;
    bool packed16 = false;  // two pairs per lane in 16-bit halves (wavefront16.hpp), int32 fallback
    bool key2 = false;      // packed LOCAL over 257..512 target columns (second key set)
    int G16 = 0, R16 = 0;   // packed kernel shape
    uint32_t lds16_stride = 0;
    size_t lds16_bytes = 0;
    int32_t vmin = 0;       // packed GLOBAL/SEMI value-range bound
    uint32_t kf16 = 0;      // packed LOCAL: f16-pattern key columns (wavefront16.hpp step_local KU), 0 = 16-bit keys
    bool ku16 = false;      // packed LOCAL in the e-drift frame with u16 keys (WF16_LOCAL_U16)
    uint32_t kseg_shift = 0; // packed LOCAL with f16 keys by step segments of 2^kseg_shift (WF16_LOCAL_SEG), 0 = off
    int G = 0, R = 0;
    uint32_t lds_stride = 0;
    size_t lds_bytes = 0;
    bool need_pack = false; // generic kernels / reverse-complement need packed words
    bool band16 = false;    // banded: two pairs per lane in 16-bit halves (banded16.hpp), int32 fallback
    bool local16 = false;   // LOCAL second best: two pairs per lane in 16-bit halves (local16.hpp), int32 fallback
    bool semi_tq = false;   // SEMI TAIL=QUERY/BOTH: packed class launches (one per padded target length), int32 fallback
    bool tb_band = false;   // packed GLOBAL+TB by band recomputation (wavefront16.hpp WF16_GLOBAL_CP / _BAND)
    uint32_t band_w = 0, band_wd = 0;
    uint32_t max_q = 0, max_t = 0;   // the batch shape the plan was made for
    std::string name;
};

// Host-visible summary of a batch needed for planning.
struct BatchShape {
    uint32_t max_q = 0, max_t = 0;
    bool sort = false;   // lengths are uneven: run the wavefront kernels over pairs sorted by step-axis length
    uint32_t n = 0;      // pairs in the launch (0 = unknown: shapes for large batches)
    bool tb_split = true; // traceback: chunks on two streams so a chunk's walk overlaps the next DP
    bool one_t8 = false;  // host-side lengths: every padded target length is the same (SEMI TAIL=QUERY/BOTH
                          // then launches its one class without reading the class histogram back)
};

Plan make_plan(const gasalx_params &p, const BatchShape &shape, bool has_ops);

// Host-side check for BatchShape::sort: the padded lengths of the step axis
// (targets; queries for SEMI-GLOBAL, whose kernel runs transposed) spread over
// at least two 8-base words.
inline bool uneven_lengths(const gasalx_params &p, const uint32_t *q_lens, const uint32_t *t_lens, uint32_t n) {
    const uint32_t *l = p.algo == 2 ? q_lens : t_lens;
    if (!l || n == 0) return false;
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t w = (l[i] + 7) >> 3;
        lo = w < lo ? w : lo;
        hi = w > hi ? w : hi;
    }
    return hi >= lo + 2;
}

// Host-side check for BatchShape::one_t8: one padded target length in the batch, and it is the
// padded max_t the plan is sized for (a caller's max_t_len is only an upper bound, and a chunk of
// the host pipeline may hold only shorter targets: the class launch then covers no pair, so the
// histogram decides)
inline bool one_pad8(const uint32_t *t_lens, uint32_t n, uint32_t max_t) {
    if (!t_lens || n == 0) return false;
    const uint32_t w = (t_lens[0] + 7) >> 3;
    if (w != (max_t + 7) >> 3) return false;
    for (uint32_t i = 1; i < n; i++)
        if (((t_lens[i] + 7) >> 3) != w) return false;
    return true;
}

// Launch the full path for a device-resident batch on `stream`.
// Returns GASALX_OK or an error code; sets the thread's last error message.
// cigar_cap: bytes writable at out.cigar (0 = b.q_bytes)
int align_device(Workspace &ws, const gasalx_params &p, const gasalx_batch &b, const gasalx_results &out,
                 hipStream_t stream, const BatchShape &shape, uint64_t cigar_cap = 0);

int pairhmm_device(Workspace &ws, const gasalx_hmm_batch &b, float *result, hipStream_t stream, uint32_t max_r,
                   uint32_t max_h);

// PairHMM from Phred qualities.  ph2pr_dev: the 128-entry table in device memory.
// With perm/classes (host path): slots sorted by (read, haplotype) length, one launch
// per class of slots sharing a lane-group size; otherwise one launch over all pairs.
struct HmmClass { uint32_t slot0, slot1, max_r, max_h; };
int pairhmm_group(uint32_t max_r);
int pairhmm_quals_device(Workspace &ws, const gasalx_hmm_qual_batch &b, float *result, hipStream_t stream,
                         const float *ph2pr_dev, const uint32_t *perm, const HmmClass *classes, int n_classes,
                         uint32_t max_r, uint32_t max_h);

// nvbio-style batched scoring (batched.hip, nvbio.hpp)
int nv_score_device(const gasalx_nv_aligner &al, uint32_t n, const gasalx_nv_strings &pat,
                    const gasalx_nv_strings &txt, int32_t *scores, int16_t *scores16, uint32_t max_p, uint32_t max_t,
                    hipStream_t stream);
// nvbio BatchedBandedAlignmentScore<band> (batched.hip / nvbanded.hpp): BestSink score per pair
// max_p: the longest pattern (0: unknown; the packed kernel needs it for its value window)
int nv_banded_score_device(const gasalx_nv_aligner &al, uint32_t band, uint32_t n, const gasalx_nv_strings &pat,
                           const gasalx_nv_strings &txt, int32_t *scores, hipStream_t st, uint32_t max_p);
int nv_traceback_device(const gasalx_nv_aligner &al, uint32_t n, const gasalx_nv_strings &pat,
                        const gasalx_nv_strings &txt, uint32_t max_p, uint32_t max_t, uint8_t *dir, int32_t *row,
                        int32_t *score, uint32_t *src, uint32_t *snk, uint8_t *ops, uint32_t ops_stride,
                        uint32_t *n_ops, hipStream_t st);
int nv_banded_traceback_device(const gasalx_nv_aligner &al, uint32_t band, uint32_t n, const gasalx_nv_strings &pat,
                               const gasalx_nv_strings &txt, uint32_t max_p, uint32_t *dir, int32_t *score,
                               uint32_t *src, uint32_t *snk, uint8_t *ops, uint32_t ops_stride, uint32_t *n_ops,
                               hipStream_t st);
std::string nv_plan_name(const gasalx_nv_aligner &al, uint32_t max_p, uint32_t max_t, bool per_pair_text,
                         uint32_t text_bits);

// The engine's own stream (capi.cpp; gasalx_engine is opaque elsewhere).
hipStream_t engine_stream(gasalx_engine *e);

void set_error(const std::string &msg);
const char *last_error();

}  // namespace gx
