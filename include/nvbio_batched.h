/*
 * nvbio_batched.h — nvbio-shaped batched alignment scoring over libgasal (second
 * front-end).
 *
 * Replaces, for the scoring path sw-benchmark drives:
 *   nvbio::aln::BatchedAlignmentScore<stream, scheduler>   NvB/nvbio/alignment/batched.h:313-352
 *   the scheduler tags                                      batched.h:44-87
 *   SimpleSmithWatermanScheme / SimpleGotohScheme           alignment/utils.h:92-135
 *   make_{edit_distance,smith_waterman,gotoh}_aligner       alignment/alignment_base.h:180-330
 *   nvbio::aln::BatchedBandedAlignmentScore<BAND_LEN, stream, scheduler>
 *                                                           batched.h:337-352, batched_banded_inl.h:44-75
 *   nvbio::aln::BatchedAlignmentTraceback<CHECKPOINTS, stream, scheduler>
 *                                                           batched.h:436-449, batched_inl.h:612-664
 *   nvbio::aln::BatchedBandedAlignmentTraceback<BAND_LEN, CHECKPOINTS, stream, scheduler>
 *                                                           batched.h:464-478, batched_banded_inl.h:248-297
 *   sw-benchmark's AlignmentStream (reads 4-bit DNA_N big-endian, reference 2-bit,
 *   int16 scores)                                           NvB/sw-benchmark/sw-benchmark.cu:100-215
 * Every scheduler maps to the same MI355X kernel (nvbio.hpp: lane groups per pattern,
 * text in LDS; banded: nvbanded.hpp, one pair per thread with the band in registers);
 * there is no temporary storage, so max_temp_storage() is 0.  The TextBlockingTag /
 * PatternBlockingTag score semantics are provided (both give the same scores), full and
 * banded.  Traceback: BatchedAlignmentTraceback<CHECKPOINTS, stream_type> (full DP) and
 * BatchedBandedAlignmentTraceback<BAND_LEN, CHECKPOINTS, stream_type> for the edit-distance,
 * Smith-Waterman and Gotoh aligners over a TracebackStream (nvtrace.hpp: one pair per thread,
 * as the reference's DeviceThreadScheduler runs it); the warp variants are not provided.
 *
 * Header-only C++ over the flat C-ABI (gasalx.h); link with -lgasal.
 */
#ifndef NVBIO_BATCHED_H
#define NVBIO_BATCHED_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "gasalx.h"

namespace nvbio {

typedef uint8_t uint8;
typedef int16_t int16;
typedef int32_t int32;
typedef uint32_t uint32;
typedef uint64_t uint64;

namespace aln {

enum AlignmentType { GLOBAL, LOCAL, SEMI_GLOBAL };   // alignment_base.h:54

struct PatternBlockingTag {};
struct TextBlockingTag {};

// batch schedulers (batched.h:44-87): tags only; all run the same device kernel
struct HostThreadScheduler {};
template <uint32 BLOCKDIM_T, uint32 MINBLOCKS_T>
struct DeviceThreadBlockScheduler {
    static const uint32 BLOCKDIM = BLOCKDIM_T;
    static const uint32 MINBLOCKS = MINBLOCKS_T;
};
typedef DeviceThreadBlockScheduler<128, 1> DeviceThreadScheduler;
struct DeviceStagedThreadScheduler {};
struct DeviceWarpScheduler {};

struct SimpleSmithWatermanScheme {   // utils.h:92-110
    SimpleSmithWatermanScheme() {}
    SimpleSmithWatermanScheme(int32 match, int32 mm, int32 del, int32 ins)
        : m_match(match), m_mismatch(mm), m_deletion(del), m_insertion(ins) {}
    int32 match(uint8 = 0) const { return m_match; }
    int32 mismatch(uint8 = 0) const { return m_mismatch; }
    int32 deletion() const { return m_deletion; }
    int32 insertion() const { return m_insertion; }
    int32 m_match = 0, m_mismatch = 0, m_deletion = 0, m_insertion = 0;
};

struct SimpleGotohScheme {   // utils.h:114-135
    SimpleGotohScheme() {}
    SimpleGotohScheme(int32 match, int32 mm, int32 gap_open, int32 gap_ext)
        : m_match(match), m_mismatch(mm), m_gap_open(gap_open), m_gap_ext(gap_ext) {}
    int32 match(uint8 = 0) const { return m_match; }
    int32 mismatch(uint8 = 0) const { return m_mismatch; }
    int32 pattern_gap_open() const { return m_gap_open; }
    int32 pattern_gap_extension() const { return m_gap_ext; }
    int32 text_gap_open() const { return m_gap_open; }
    int32 text_gap_extension() const { return m_gap_ext; }
    int32 m_match = 0, m_mismatch = 0, m_gap_open = 0, m_gap_ext = 0;
};

template <AlignmentType T_TYPE, typename AlgorithmType = PatternBlockingTag>
struct EditDistanceAligner {
    static const AlignmentType TYPE = T_TYPE;
    gasalx_nv_aligner c_aligner() const {
        gasalx_nv_aligner a = {GASALX_NV_ED, (int32)TYPE, 0, -1, 0, 0, -1, -1};
        return a;
    }
};

template <AlignmentType T_TYPE, typename scoring_scheme_type, typename AlgorithmType = PatternBlockingTag>
struct SmithWatermanAligner {
    static const AlignmentType TYPE = T_TYPE;
    SmithWatermanAligner() {}
    explicit SmithWatermanAligner(const scoring_scheme_type s) : scheme(s) {}
    gasalx_nv_aligner c_aligner() const {
        gasalx_nv_aligner a = {GASALX_NV_SW, (int32)TYPE, scheme.match(), scheme.mismatch(), 0, 0,
                               scheme.deletion(), scheme.insertion()};
        return a;
    }
    scoring_scheme_type scheme;
};

template <AlignmentType T_TYPE, typename scoring_scheme_type, typename AlgorithmType = PatternBlockingTag>
struct GotohAligner {
    static const AlignmentType TYPE = T_TYPE;
    GotohAligner() {}
    explicit GotohAligner(const scoring_scheme_type s) : scheme(s) {}
    gasalx_nv_aligner c_aligner() const {
        gasalx_nv_aligner a = {GASALX_NV_GOTOH, (int32)TYPE, scheme.match(), scheme.mismatch(),
                               scheme.pattern_gap_open(), scheme.pattern_gap_extension(), 0, 0};
        return a;
    }
    scoring_scheme_type scheme;
};

template <AlignmentType TYPE>
EditDistanceAligner<TYPE> make_edit_distance_aligner() { return EditDistanceAligner<TYPE>(); }
template <AlignmentType TYPE, typename algorithm_tag>
EditDistanceAligner<TYPE, algorithm_tag> make_edit_distance_aligner() { return EditDistanceAligner<TYPE, algorithm_tag>(); }
template <AlignmentType TYPE, typename scheme_type>
SmithWatermanAligner<TYPE, scheme_type> make_smith_waterman_aligner(const scheme_type &s) {
    return SmithWatermanAligner<TYPE, scheme_type>(s);
}
template <AlignmentType TYPE, typename algorithm_tag, typename scheme_type>
SmithWatermanAligner<TYPE, scheme_type, algorithm_tag> make_smith_waterman_aligner(const scheme_type &s) {
    return SmithWatermanAligner<TYPE, scheme_type, algorithm_tag>(s);
}
template <AlignmentType TYPE, typename scheme_type>
GotohAligner<TYPE, scheme_type> make_gotoh_aligner(const scheme_type &s) { return GotohAligner<TYPE, scheme_type>(s); }
template <AlignmentType TYPE, typename algorithm_tag, typename scheme_type>
GotohAligner<TYPE, scheme_type, algorithm_tag> make_gotoh_aligner(const scheme_type &s) {
    return GotohAligner<TYPE, scheme_type, algorithm_tag>(s);
}

// The device string sets and score sink of one batch: sw-benchmark's AlignmentStream
// (sw-benchmark.cu:100-215) with its packing made explicit.  All pointers are device
// pointers.  Patterns: n_tasks + 1 symbol offsets; text: one string shared by every
// pattern (text_offsets NULL) or n_tasks + 1 offsets.
template <typename aligner_type_T>
struct AlignmentStream {
    typedef aligner_type_T aligner_type;
    AlignmentStream(const aligner_type aligner, const uint32 count, const uint32 *offsets, const uint32 *patterns,
                    const uint32 max_pattern_len, const uint32 total_pattern_len, const uint32 *text,
                    const uint32 text_len, int16 *scores)
        : m_aligner(aligner), m_count(count), m_max_pattern_len(max_pattern_len),
          m_total_pattern_len(total_pattern_len), m_text_len(text_len), m_offsets(offsets), m_patterns(patterns),
          m_text(text), m_scores(scores) {}

    const aligner_type &aligner() const { return m_aligner; }
    uint32 max_pattern_length() const { return m_max_pattern_len; }
    uint32 max_text_length() const { return m_text_len; }
    uint32 size() const { return m_count; }
    uint64 cells() const { return uint64(m_total_pattern_len) * uint64(m_text_len); }

    aligner_type m_aligner;
    uint32 m_count, m_max_pattern_len, m_total_pattern_len, m_text_len;
    const uint32 *m_offsets, *m_patterns, *m_text;
    int16 *m_scores;
    int32 *m_scores32 = nullptr;            // optional int32 scores
    const uint32 *m_text_offsets = nullptr; // per-pattern texts instead of the shared one
    uint32 m_pattern_bits = 4, m_pattern_big_endian = 1;   // io::SequenceDataTraits<DNA_N>
    uint32 m_text_bits = 2, m_text_big_endian = 0;         // REF_BITS / REF_BIG_ENDIAN
};

// One engine per thread for the current device (set_device, default 0).
inline int &current_device() {
    static thread_local int d = 0;
    return d;
}
inline void set_device(int d) { current_device() = d; }
inline gasalx_engine *engine() {
    static thread_local gasalx_engine *eng[64] = {};
    const int d = current_device();
    if (d < 0 || d >= 64) { fprintf(stderr, "nvbio_batched: bad device %d\n", d); exit(EXIT_FAILURE); }
    if (!eng[d] && gasalx_engine_create(d, &eng[d]) != GASALX_OK) {
        fprintf(stderr, "nvbio_batched: %s\n", gasalx_last_error());
        exit(EXIT_FAILURE);
    }
    return eng[d];
}

template <typename stream_type, typename scheduler_type>
struct BatchedAlignmentScore {
    typedef stream_type input_stream_type;
    typedef typename stream_type::aligner_type aligner_type;

    // no temporary storage: the DP state stays in registers and LDS
    static uint64 max_temp_storage(const uint32, const uint32, const uint32) { return 0; }

    // enact the batch on the engine's stream (nvbio's enact is asynchronous too; the
    // benchmark synchronises the device afterwards).  Errors exit, as nvbio's do.
    void enact(stream_type stream, uint64 temp_size = 0u, uint8 *temp = NULL, void *hip_stream = NULL) {
        (void)temp_size; (void)temp;
        const gasalx_nv_aligner a = stream.aligner().c_aligner();
        gasalx_nv_strings p = {stream.m_patterns, stream.m_offsets, 0, stream.m_pattern_bits,
                               stream.m_pattern_big_endian};
        gasalx_nv_strings t = {stream.m_text, stream.m_text_offsets, stream.m_text_len, stream.m_text_bits,
                               stream.m_text_big_endian};
        const int rc = gasalx_nv_score_device(engine(), &a, stream.size(), &p, &t, stream.m_scores32,
                                              stream.m_scores, stream.max_pattern_length(),
                                              stream.max_text_length(), hip_stream);
        if (rc != GASALX_OK) {
            fprintf(stderr, "BatchedAlignmentScore::enact: %s\n", gasalx_last_error());
            exit(EXIT_FAILURE);
        }
    }
};

// Banded scoring (batched_banded_inl.h:44-75): every pattern against the first
// pattern_length + BAND_LEN - 1 symbols of its text, cells (i, i + j) with j < BAND_LEN
// (2..32).  Scores are int32 (stream.m_scores32); a text shorter than its pattern is
// skipped and scores INT32_MIN, as nvbio's BestSink leaves it.
template <uint32 BAND_LEN, typename stream_type, typename scheduler_type = DeviceThreadScheduler>
struct BatchedBandedAlignmentScore {
    typedef stream_type input_stream_type;
    typedef typename stream_type::aligner_type aligner_type;

    static uint64 min_temp_storage(const uint32, const uint32, const uint32) { return 0; }
    static uint64 max_temp_storage(const uint32, const uint32, const uint32) { return 0; }

    void enact(stream_type stream, uint64 temp_size = 0u, uint8 *temp = NULL, void *hip_stream = NULL) {
        (void)temp_size; (void)temp;
        const gasalx_nv_aligner a = stream.aligner().c_aligner();
        gasalx_nv_strings p = {stream.m_patterns, stream.m_offsets, 0, stream.m_pattern_bits,
                               stream.m_pattern_big_endian};
        gasalx_nv_strings t = {stream.m_text, stream.m_text_offsets, stream.m_text_len, stream.m_text_bits,
                               stream.m_text_big_endian};
        if (stream.m_scores32 == NULL) {
            fprintf(stderr, "BatchedBandedAlignmentScore::enact: banded scores are int32, set m_scores32\n");
            exit(EXIT_FAILURE);
        }
        const int rc = gasalx_nv_banded_score_device(engine(), &a, BAND_LEN, stream.size(), &p, &t,
                                                     stream.m_scores32, stream.max_pattern_length(), hip_stream);
        if (rc != GASALX_OK) {
            fprintf(stderr, "BatchedBandedAlignmentScore::enact: %s\n", gasalx_last_error());
            exit(EXIT_FAILURE);
        }
    }
};

// The outputs of a traceback batch (batched_inl.h:612-664's stream.output(): the Alignment
// and the backtracer of each job), as device arrays: per pair the BestSink score, the
// Alignment's source and sink as (x = text, y = pattern) pairs, and the backtracker's pushes
// in push order (end of the alignment first; 0 SUBSTITUTION, 1 INSERTION, 2 DELETION) at
// ops + k * ops_stride, n_ops[k] of them (ops_stride >= max pattern + max text length).
enum { SUBSTITUTION = 0, INSERTION = 1, DELETION = 2 };   // alignment_base.h:139-147

template <typename aligner_type_T>
struct TracebackStream : AlignmentStream<aligner_type_T> {
    typedef aligner_type_T aligner_type;
    TracebackStream(const aligner_type aligner, const uint32 count, const uint32 *offsets, const uint32 *patterns,
                    const uint32 max_pattern_len, const uint32 total_pattern_len, const uint32 *text,
                    const uint32 text_len, int32 *scores, uint32 *sources, uint32 *sinks, uint8 *ops,
                    const uint32 ops_stride, uint32 *n_ops)
        : AlignmentStream<aligner_type_T>(aligner, count, offsets, patterns, max_pattern_len, total_pattern_len,
                                          text, text_len, nullptr),
          m_sources(sources), m_sinks(sinks), m_ops(ops), m_ops_stride(ops_stride), m_n_ops(n_ops) {
        this->m_scores32 = scores;
    }
    uint32 *m_sources, *m_sinks;
    uint8 *m_ops;
    uint32 m_ops_stride;
    uint32 *m_n_ops;
    uint32 m_max_text_len = 0;   // per-pair texts: the longest (0 = read back)
};

// Feed one job's result (host copies of the stream's outputs) to an nvbio Backtracer (push(op),
// clip(len)) in the order alignment_traceback calls it (alignment_inl.h:413-462): the end clip,
// the pushes, the start clip.
template <typename backtracer_type>
void replay(backtracer_type &bt, const uint32 pattern_len, const uint32 source_y, const uint32 sink_y,
            const uint8 *ops, const uint32 n_ops) {
    bt.clip(pattern_len - sink_y);
    for (uint32 i = 0; i < n_ops; ++i) bt.push(ops[i]);
    bt.clip(source_y);
}

template <uint32 CHECKPOINTS, typename stream_type, typename scheduler_type = DeviceThreadScheduler>
struct BatchedAlignmentTraceback {
    typedef stream_type input_stream_type;
    typedef typename stream_type::aligner_type aligner_type;

    // the workspace (flags of every cell, one DP row per pair) is the engine's, not the caller's:
    // these report what enact() reserves in it (batches past 4 GB of it run in chunks), so a
    // caller sizing its batches from them sees the device memory a call takes.
    // enact() calls sharing one engine() must be serialised: they share that workspace.
    static uint64 min_temp_storage(const uint32 max_pattern_len, const uint32 max_text_len, const uint32) {
        return gasalx_nv_traceback_workspace(max_pattern_len, max_text_len, 1);
    }
    static uint64 max_temp_storage(const uint32 max_pattern_len, const uint32 max_text_len, const uint32 n) {
        return gasalx_nv_traceback_workspace(max_pattern_len, max_text_len, n);
    }

    void enact(stream_type stream, uint64 temp_size = 0u, uint8 *temp = NULL, void *hip_stream = NULL) {
        (void)temp_size; (void)temp;
        const gasalx_nv_aligner a = stream.aligner().c_aligner();
        gasalx_nv_strings p = {stream.m_patterns, stream.m_offsets, 0, stream.m_pattern_bits,
                               stream.m_pattern_big_endian};
        gasalx_nv_strings t = {stream.m_text, stream.m_text_offsets, stream.m_text_len, stream.m_text_bits,
                               stream.m_text_big_endian};
        const int rc = gasalx_nv_traceback_device(engine(), &a, stream.size(), &p, &t, stream.max_pattern_length(),
                                                  stream.m_text_offsets ? stream.m_max_text_len : stream.m_text_len,
                                                  stream.m_scores32, stream.m_sources, stream.m_sinks, stream.m_ops,
                                                  stream.m_ops_stride, stream.m_n_ops, hip_stream);
        if (rc != GASALX_OK) {
            fprintf(stderr, "BatchedAlignmentTraceback::enact: %s\n", gasalx_last_error());
            exit(EXIT_FAILURE);
        }
    }
};

// Banded traceback (banded_inl.h:352-427): the band's cells (i, i + j), j < BAND_LEN (2..32);
// ops_stride >= 2 x max pattern length + BAND_LEN.  nvBowtie runs BAND_LEN 3 / 7 / 15 / 31
// (nvBowtie/bowtie2/cuda/traceback_inl.h:239-257).  CHECKPOINTS only sizes the reference's
// storage; the flags of every cell live in the engine's workspace here.
template <uint32 BAND_LEN, uint32 CHECKPOINTS, typename stream_type, typename scheduler_type = DeviceThreadScheduler>
struct BatchedBandedAlignmentTraceback {
    typedef stream_type input_stream_type;
    typedef typename stream_type::aligner_type aligner_type;

    // the engine's workspace a call reserves (see BatchedAlignmentTraceback)
    static uint64 min_temp_storage(const uint32 max_pattern_len, const uint32, const uint32) {
        return gasalx_nv_banded_traceback_workspace(max_pattern_len, BAND_LEN, 1);
    }
    static uint64 max_temp_storage(const uint32 max_pattern_len, const uint32, const uint32 n) {
        return gasalx_nv_banded_traceback_workspace(max_pattern_len, BAND_LEN, n);
    }

    void enact(stream_type stream, uint64 temp_size = 0u, uint8 *temp = NULL, void *hip_stream = NULL) {
        (void)temp_size; (void)temp;
        const gasalx_nv_aligner a = stream.aligner().c_aligner();
        gasalx_nv_strings p = {stream.m_patterns, stream.m_offsets, 0, stream.m_pattern_bits,
                               stream.m_pattern_big_endian};
        gasalx_nv_strings t = {stream.m_text, stream.m_text_offsets, stream.m_text_len, stream.m_text_bits,
                               stream.m_text_big_endian};
        const int rc = gasalx_nv_banded_traceback_device(engine(), &a, BAND_LEN, stream.size(), &p, &t,
                                                         stream.max_pattern_length(), stream.m_scores32,
                                                         stream.m_sources, stream.m_sinks, stream.m_ops,
                                                         stream.m_ops_stride, stream.m_n_ops, hip_stream);
        if (rc != GASALX_OK) {
            fprintf(stderr, "BatchedBandedAlignmentTraceback::enact: %s\n", gasalx_last_error());
            exit(EXIT_FAILURE);
        }
    }
};

}  // namespace aln
}  // namespace nvbio

#endif
