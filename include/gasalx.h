/*
 * gasalx.h — flat C-ABI of the MI355X GASAL2-compatible engine (FFI boundary).
 *
 * Plain pointers and sizes only; no HIP or torch types in the signatures
 * (streams are passed as void*, i.e. a hipStream_t).  The entry points are the
 * ones a ctypes / cgo / JNI binding of the reference's path would bind:
 *
 *   gasalx_align_host    <- gasal_aln(...)   (Non-CDP/GASAL2/src/__deprecated.cpp:5,
 *                                             the flat batch call, commented out in
 *                                             the reference; same argument meaning,
 *                                             plus the Parameters fields it needs)
 *   gasalx_align_device  <- gasal_aln_async(...) (gasal_align.cu:29) without the host
 *                           staging: inputs already resident in device memory
 *   gasalx_pairhmm_*     <- pairHMM<<<>>> launch (Non-CDP/PairHMM/inter_task/
 *                           Synthetic_data/tile_1/tile_1.cu:44,507-524)
 *
 * The reference's C++ API (gasal_header.h: gasal_init_streams, gasal_host_batch_fill,
 * gasal_aln_async, gasal_is_aln_async_done, ...) is provided by the same library
 * with C++ linkage.  Every call here returns 0 on success and a negative
 * GASALX_E* code on failure (the reference exits instead, gasal.h:15-22);
 * gasalx_last_error() gives the message of the calling thread's last failure.
 */
#ifndef GASALX_H
#define GASALX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GASALX_ABI_VERSION 1

enum {
    GASALX_OK = 0,
    GASALX_EINVAL = -1,      /* bad argument (sizes, alignment, enum value)          */
    GASALX_ERANGE = -2,      /* sequence length / score range the engine rejects     */
    GASALX_EDEVICE = -3,     /* HIP runtime error                                    */
    GASALX_ENOMEM = -4,      /* device or host allocation failed                     */
    GASALX_EUNSUPPORTED = -5 /* configuration not implemented                        */
};

/* Mirrors the Parameters fields the reference's boundary reads
 * plus the compile-time knobs that become run-time values here. */
typedef struct gasalx_params {
    int32_t match;          /* gasal_subst_scores.match                              */
    int32_t mismatch;       /* gasal_subst_scores.mismatch (penalty, positive)       */
    int32_t gap_open;       /* gasal_subst_scores.gap_open                           */
    int32_t gap_extend;     /* gasal_subst_scores.gap_extend                         */
    int32_t algo;           /* enum algo_type                                        */
    int32_t start_pos;      /* enum comp_start                                       */
    int32_t second_best;    /* enum Bool                                             */
    int32_t head;           /* enum data_source, semi-global skipped head            */
    int32_t tail;           /* enum data_source, semi-global skipped tail            */
    int32_t k_band;         /* BANDED band width in bases (kernel uses k_band >> 3)  */
    int32_t is_packed;      /* inputs are already 4-bit packed words                 */
    int32_t n_code;         /* reference N_CODE (0x4E for ASCII input)               */
    int32_t has_n_penalty;  /* reference N_PENALTY defined?                          */
    int32_t n_penalty;
    int32_t max_query_len;  /* reference MAX_QUERY_LEN (0 = large enough for the batch) */
} gasalx_params;

/* Batch description; the pointers are device pointers for gasalx_align_device and
 * host pointers for gasalx_align_host.  Layout as the reference's host batch:
 * sequences concatenated, each padded with N_CODE to a multiple of 8, offsets in
 * bytes including the pads, lengths without them (GASAL2 README.md:145). */
typedef struct gasalx_batch {
    const uint8_t *q_batch;
    const uint32_t *q_offsets;
    const uint32_t *q_lens;
    const uint8_t *t_batch;
    const uint32_t *t_offsets;
    const uint32_t *t_lens;
    uint32_t q_bytes;             /* multiple of 8 */
    uint32_t t_bytes;             /* multiple of 8 */
    uint32_t n_alns;
    const uint8_t *q_ops;         /* enum operation_on_seq per pair, or NULL */
    const uint8_t *t_ops;
    const uint32_t *seed_scores;  /* KSW h0 per pair, or NULL */
    uint32_t max_q_len;           /* upper bound of q_lens (0 = unknown: the engine reads   */
    uint32_t max_t_len;           /* the lengths back, which synchronises the stream).      */
                                  /* SEMI_GLOBAL with TAIL = QUERY/BOTH, score only, reads  */
                                  /* back the histogram of padded target lengths (one sync */
                                  /* of the stream) even when both are given; the host     */
                                  /* entry points skip it when every target has the same   */
                                  /* padded length                                         */
} gasalx_batch;

/* Output arrays (n_alns entries; cigar has q_bytes entries).  NULL = not wanted.
 * Fields the reference would not write for the configuration are untouched. */
typedef struct gasalx_results {
    int32_t *aln_score;
    int32_t *q_end;
    int32_t *t_end;
    int32_t *q_start;
    int32_t *t_start;
    int32_t *aln_score2;
    int32_t *q_end2;
    int32_t *t_end2;
    uint8_t *cigar;          /* reversed RLE bytes at each pair's query offset     */
    uint32_t *n_cigar_ops;
} gasalx_results;

typedef struct gasalx_engine gasalx_engine;   /* device workspace, one per thread */

int gasalx_abi_version(void);
const char *gasalx_last_error(void);

int gasalx_device_count(int *count);
int gasalx_engine_create(int device, gasalx_engine **out);
int gasalx_engine_destroy(gasalx_engine *eng);

/* Asynchronous on `stream` (a hipStream_t; NULL = the engine's own stream). */
int gasalx_align_device(gasalx_engine *eng, const gasalx_params *params, const gasalx_batch *dev_batch,
                        const gasalx_results *dev_out, void *stream);

/* Synchronous host-to-host call (H2D, kernels, D2H). */
int gasalx_align_host(gasalx_engine *eng, const gasalx_params *params, const gasalx_batch *host_batch,
                      const gasalx_results *host_out);

/* Page-locked host memory from the HIP runtime libgasal itself uses (hipHostMalloc),
 * for caller-owned input / result buffers (the reference's host pages and host_res
 * are pinned: host_batch.cpp:79-153, res.cpp:8-70).  Freed with gasalx_host_free. */
int gasalx_host_alloc(uint64_t bytes, void **out);
int gasalx_host_free(void *ptr);

/* Which kernel family the dispatcher selects for a batch (for tests/profiling):
 * writes a short NUL-terminated name into buf. */
int gasalx_describe_plan(const gasalx_params *params, uint32_t max_q_len, uint32_t max_t_len, char *buf,
                         uint32_t buf_len);

/* Diagnostics: pairs of the engine's last packed (two-pairs-per-lane) launches that the packed
 * kernel aligned itself (*handled) out of the pairs those launches covered (*total); the rest went
 * to the int32 kernel.  The engine's own workspace and its two host-pipeline stages each count
 * their last packed launch (a WITH_START call: the reverse pass) and forgets it once read.
 * Synchronises the engine's streams; 0 / 0 when no packed launch ran since the last read. */
int gasalx_packed_pairs(gasalx_engine *engine, uint64_t *handled, uint64_t *total);

/* PairHMM forward.  Per read base: read byte and the four per-base parameters
 * (qm = ph2pr[bq], delta = ph2pr[iq], xiksi = ph2pr[dq], alpha = 1 - ph2pr[(iq+dq)&127],
 * tile_1.cu:415-419) at the read's offset; haplotype bytes at hap offsets. */
typedef struct gasalx_hmm_batch {
    const uint8_t *reads;
    const uint32_t *read_offsets;
    const uint32_t *read_lens;
    const float *qm;
    const float *delta;
    const float *xiksi;
    const float *alpha;
    const uint8_t *haps;
    const uint32_t *hap_offsets;
    const uint32_t *hap_lens;
    uint32_t read_bytes;
    uint32_t hap_bytes;
    uint32_t n_pairs;
    uint32_t max_read_len;        /* upper bounds (0 = unknown, read back from the device) */
    uint32_t max_hap_len;
} gasalx_hmm_batch;

int gasalx_pairhmm_device(gasalx_engine *eng, const gasalx_hmm_batch *dev_batch, float *dev_result, void *stream);
int gasalx_pairhmm_host(gasalx_engine *eng, const gasalx_hmm_batch *host_batch, float *host_result);

/* Host-side helper: per-base PairHMM parameters from Phred qualities
 * (tile_1.cu:216-220 ph2pr table, :415-419). */
int gasalx_pairhmm_params(const uint8_t *bq, const uint8_t *iq, const uint8_t *dq, uint32_t n, float *qm,
                          float *delta, float *xiksi, float *alpha);

/* PairHMM from Phred qualities: the reference's input format (tile_1.cu:246-290,
 * Intra-task/real_data/improved_warp_based/improved_warp_based.cu:240-279).  base /
 * insertion / deletion quality bytes sit at the read offsets; the four per-base
 * parameters are formed on the device from the same ph2pr table the reference's host
 * builds (powf(10, -q/10), tile_1.cu:216-220; mapping :415-419), so the kernel's
 * input is 4 bytes per read base instead of 17. */
typedef struct gasalx_hmm_qual_batch {
    const uint8_t *reads;
    const uint32_t *read_offsets;
    const uint32_t *read_lens;
    const uint8_t *base_quals;
    const uint8_t *ins_quals;
    const uint8_t *del_quals;
    const uint8_t *haps;
    const uint32_t *hap_offsets;
    const uint32_t *hap_lens;
    uint64_t read_bytes;          /* bytes of reads (and of each quality array) */
    uint64_t hap_bytes;
    uint32_t n_pairs;
    uint32_t max_read_len;        /* upper bounds (0 = unknown) */
    uint32_t max_hap_len;
} gasalx_hmm_qual_batch;

/* Device-resident batch: one launch, lane groups sized by the longest read. */
int gasalx_pairhmm_quals_device(gasalx_engine *eng, const gasalx_hmm_qual_batch *dev_batch, float *dev_result,
                                void *stream);
/* Host arrays in, results out in input order.  Pairs run sorted by (read length,
 * haplotype length) as the reference's host sorts them (tile_1.cu:180-195,325), in
 * classes of reads that share a lane-group size (one launch each) instead of the
 * reference's 32-pair interleaved chunks (tile_1.cu:346-500). */
int gasalx_pairhmm_quals_host(gasalx_engine *eng, const gasalx_hmm_qual_batch *host_batch, float *host_result);

/* Reader of the reference's PairHMM input files: groups of `size` pairs, each pair
 * = read length, read bases, then read-length base / insertion / deletion / gcp
 * qualities, haplotype length, haplotype bases (whitespace-separated, fscanf
 * semantics of tile_1.cu:246-290; qualities stored as (char) values).  Arrays are
 * owned by the returned object (gasalx_hmm_file_free). */
typedef struct gasalx_hmm_file {
    uint32_t n_pairs;
    uint32_t n_groups;
    uint32_t *group_sizes;        /* pairs per group, in file order */
    uint8_t *reads;
    uint32_t *read_offsets;
    uint32_t *read_lens;
    uint8_t *base_quals, *ins_quals, *del_quals, *gcp_quals;
    uint8_t *haps;
    uint32_t *hap_offsets;
    uint32_t *hap_lens;
    uint64_t read_bytes;
    uint64_t hap_bytes;
} gasalx_hmm_file;

int gasalx_hmm_file_read(const char *path, gasalx_hmm_file **out);
int gasalx_hmm_file_free(gasalx_hmm_file *f);

/* Second front-end: nvbio-style batched alignment scoring (NvB/nvbio/alignment/
 * batched.h:44-87, the BatchedAlignmentScore<stream, scheduler> idiom of
 * sw-benchmark.cu:355-443; C++ wrapper in include/nvbio_batched.h).  nvbio's textbook
 * recurrences, not GASAL2's: Gotoh (gotoh/gotoh_inl.h), Smith-Waterman with linear
 * gaps (sw/sw_inl.h), edit distance (ed/ed_utils.h:45-52), each GLOBAL / LOCAL /
 * SEMI_GLOBAL (pattern fully aligned, text ends free); the output is the BestSink
 * score per pair. */
enum { GASALX_NV_ED = 0, GASALX_NV_SW = 1, GASALX_NV_GOTOH = 2 };
enum { GASALX_NV_GLOBAL = 0, GASALX_NV_LOCAL = 1, GASALX_NV_SEMI_GLOBAL = 2 };   /* nvbio AlignmentType */

typedef struct gasalx_nv_aligner {
    int32_t aligner;      /* GASALX_NV_ED / _SW / _GOTOH */
    int32_t type;         /* GASALX_NV_GLOBAL / _LOCAL / _SEMI_GLOBAL */
    int32_t match;        /* signed scores as in SimpleGotohScheme / SimpleSmithWatermanScheme */
    int32_t mismatch;     /*   (utils.h:92-135): penalties are negative                        */
    int32_t gap_open;     /* Gotoh: a gap of k symbols scores gap_open + (k-1) * gap_ext         */
    int32_t gap_ext;
    int32_t deletion;     /* Smith-Waterman: per text symbol skipped                            */
    int32_t insertion;    /* Smith-Waterman: per pattern symbol skipped                         */
} gasalx_nv_aligner;

/* A packed string set (nvbio PackedStream): symbol s of the set is field s % (32/bits)
 * of word s / (32/bits), counted from the top of the word when big_endian (nvbio reads,
 * SequenceDataTraits SEQUENCE_BIG_ENDIAN) or from bit 0 otherwise (sw-benchmark's
 * 2-bit reference, REF_BIG_ENDIAN = false). */
typedef struct gasalx_nv_strings {
    const uint32_t *words;
    const uint32_t *offsets;  /* n + 1 symbol offsets; texts: NULL = one text of `length` symbols for every pair */
    uint32_t length;
    uint32_t bits;            /* 2, 4 or 8 */
    uint32_t big_endian;
} gasalx_nv_strings;

/* scores (int32) and/or scores16 (int16, sw-benchmark's score vector) per pair.
 * Patterns up to 1024 symbols; max lengths are upper bounds (0 = read back). */
int gasalx_nv_score_device(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t n_pairs,
                           const gasalx_nv_strings *dev_patterns, const gasalx_nv_strings *dev_texts,
                           int32_t *dev_scores, int16_t *dev_scores16, uint32_t max_pattern_len,
                           uint32_t max_text_len, void *stream);
/* The kernel a gasalx_nv_score_* call with these bounds runs (e.g.
 * "nvbio16_gotoh_semi_shared_G8R19": the packed kernel, two pairs per lane group;
 * "nvbio_..." the int32 one); per_pair_texts = 0 for one shared text. */
int gasalx_nv_describe_plan(const gasalx_nv_aligner *aligner, uint32_t max_pattern_len, uint32_t max_text_len,
                            int per_pair_texts, uint32_t text_bits, char *buf, uint32_t buf_len);
/* Host arrays in and out (words: the number of words of each set). */
int gasalx_nv_score_host(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t n_pairs,
                         const gasalx_nv_strings *patterns, uint64_t pattern_words, const gasalx_nv_strings *texts,
                         uint64_t text_words, int32_t *scores, int16_t *scores16);

/* nvbio's BatchedBandedAlignmentScore<band_len> (NvB/nvbio/alignment/batched.h:337,
 * batched_banded_inl.h:44-75): the banded DP of sw_banded_inl.h / gotoh_banded_inl.h /
 * ed_banded_inl.h over cells (i, i + j), 0 <= j < band_len (2..32): two pairs per lane in
 * 16-bit halves for 2-bit texts inside the value window, else one pair per thread (int32).
 * BestSink score per pair; INT32_MIN when a text is shorter than its pattern (skipped,
 * as the reference does). */
int gasalx_nv_banded_score_device(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t band_len,
                                  uint32_t n_pairs, const gasalx_nv_strings *dev_patterns,
                                  const gasalx_nv_strings *dev_texts, int32_t *dev_scores,
                                  uint32_t max_pattern_len, void *stream);   /* max_pattern_len: 0 = read back */
int gasalx_nv_banded_score_host(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t band_len,
                                uint32_t n_pairs, const gasalx_nv_strings *patterns, uint64_t pattern_words,
                                const gasalx_nv_strings *texts, uint64_t text_words, int32_t *scores);

/* nvbio's BatchedAlignmentTraceback<CHECKPOINTS> (NvB/nvbio/alignment/batched.h:436,
 * batched_inl.h:612-664, alignment_inl.h:365-465): the full-DP traceback of the Gotoh,
 * Smith-Waterman and edit-distance aligners (ED runs as SW with 0 / -1 / -1 / -1, as
 * ed/ed_inl.h:347-365 does), GLOBAL / LOCAL /
 * SEMI_GLOBAL, one pair per thread.  Per pair: the BestSink score, the Alignment's source and
 * sink as (x, y) = (text, pattern) coordinates in sources[2k..] / sinks[2k..] (0xFFFFFFFF when no
 * cell was reported), and the backtracker's pushes in push order (end of the alignment first) at
 * ops + k * ops_stride: 0 SUBSTITUTION ('M'), 1 INSERTION ('I', a pattern symbol), 2 DELETION ('D',
 * a text symbol); n_ops[k] of them.  nvbio's Backtracer also receives clip(pattern_len - sink.y)
 * before the pushes and clip(source.y) after them (nvbio_batched.h replays both).
 * ops_stride >= max pattern + max text length; nvbio's int16 DP columns bound
 * (max pattern + max text + 2) * max |score| <= 32767, and pattern x text <= 16 M cells.
 * Workspace: pad8(pattern) x text bytes + 8 bytes per text symbol per pair, held by the engine; a
 * batch runs in chunks of at most 4 GB of it (gasalx_nv_traceback_workspace gives the bytes a
 * call reserves).  Calls that share an engine must be serialised (one workspace per engine). */
uint64_t gasalx_nv_traceback_workspace(uint32_t max_pattern_len, uint32_t max_text_len, uint32_t n_pairs);
int gasalx_nv_traceback_device(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t n_pairs,
                               const gasalx_nv_strings *dev_patterns, const gasalx_nv_strings *dev_texts,
                               uint32_t max_pattern_len, uint32_t max_text_len, int32_t *dev_scores,
                               uint32_t *dev_sources, uint32_t *dev_sinks, uint8_t *dev_ops, uint32_t ops_stride,
                               uint32_t *dev_n_ops, void *stream);   /* max lengths: 0 = read back */
int gasalx_nv_traceback_host(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t n_pairs,
                             const gasalx_nv_strings *patterns, uint64_t pattern_words,
                             const gasalx_nv_strings *texts, uint64_t text_words, int32_t *scores,
                             uint32_t *sources, uint32_t *sinks, uint8_t *ops, uint32_t ops_stride,
                             uint32_t *n_ops);
/* nvbio BatchedBandedAlignmentTraceback<BAND_LEN, CHECKPOINTS, stream> (NvB/nvbio/alignment/
 * batched.h:464-478, batched_banded_inl.h:248-297; nvBowtie's callers traceback_inl.h:239-257):
 * the banded traceback of every pair, band length 2..32 as an argument.  Outputs as
 * gasalx_nv_traceback_*: the BestSink score, source and sink (x = text, y = pattern end) and the
 * pushes in push order; INT32_MIN and (-1, -1) ends for a pair whose text is shorter than its
 * pattern.  ED, SW and Gotoh aligners.  ops_stride >= 2 x max pattern + band; nvbio's int16
 * checkpoints bound (max pattern + band + 3) * max |score| <= 32736.  Workspace: max pattern x
 * pad4(band) bytes per pair, held by the engine, in chunks of at most 4 GB
 * (gasalx_nv_banded_traceback_workspace); calls sharing an engine must be serialised.
 * max_pattern_len 0 = read back. */
uint64_t gasalx_nv_banded_traceback_workspace(uint32_t max_pattern_len, uint32_t band, uint32_t n_pairs);
int gasalx_nv_banded_traceback_device(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t band,
                                      uint32_t n_pairs, const gasalx_nv_strings *dev_patterns,
                                      const gasalx_nv_strings *dev_texts, uint32_t max_pattern_len,
                                      int32_t *dev_scores, uint32_t *dev_sources, uint32_t *dev_sinks,
                                      uint8_t *dev_ops, uint32_t ops_stride, uint32_t *dev_n_ops, void *stream);
int gasalx_nv_banded_traceback_host(gasalx_engine *eng, const gasalx_nv_aligner *aligner, uint32_t band,
                                    uint32_t n_pairs, const gasalx_nv_strings *patterns, uint64_t pattern_words,
                                    const gasalx_nv_strings *texts, uint64_t text_words, int32_t *scores,
                                    uint32_t *sources, uint32_t *sinks, uint8_t *ops, uint32_t ops_stride,
                                    uint32_t *n_ops);

/* Multi-GPU from one host process.  A group holds one engine per
 * entry of a device list (entries may repeat a device); a host batch is split into
 * contiguous ranges of pairs with equal cell counts (Σ ql·tl; gasalx_shard_bounds),
 * and one host thread per entry runs gasalx_align_host (or the PairHMM call) on its
 * range, writing into that range of the caller's result arrays.  The reference's
 * pattern is STAR's static split (Non-CDP/STAR/src/cuda-nw.cu:296-367: per-GPU
 * workload, cudaSetDevice, one stream per device, disjoint host result ranges);
 * GASAL2 itself exposes only gasal_set_device (interfaces.cpp:98-125).
 * GASALX_MULTI_RCCL: build an RCCL communicator over the list (ncclCommInitAll, when
 * the entries are distinct devices and librccl can be opened) for
 * gasalx_multi_allgather; otherwise that call uses peer copies. */
typedef struct gasalx_multi gasalx_multi;
enum { GASALX_MULTI_RCCL = 1 };

int gasalx_multi_create(const int *devices, int n_devices, uint32_t flags, gasalx_multi **out);
int gasalx_multi_destroy(gasalx_multi *m);
int gasalx_multi_info(const gasalx_multi *m, int *n_devices, int *uses_rccl);
/* The engine of entry `index` (owned by the group), e.g. for device-resident calls. */
int gasalx_multi_engine(gasalx_multi *m, int index, gasalx_engine **out);
/* Contiguous ranges [bounds[k], bounds[k+1]) (world + 1 entries) balancing Σ a[i]·b[i]:
 * boundary k is one past the first pair whose prefix sum reaches k/world of the total. */
int gasalx_shard_bounds(const uint32_t *a, const uint32_t *b, uint32_t n, int world, uint32_t *bounds);
/* Host arrays in and out, as gasalx_align_host.  WITH_TB: the shards' query byte ranges
 * must not overlap (each pair's CIGAR lands at its query offset, get_tb.h:94). */
int gasalx_multi_align_host(gasalx_multi *m, const gasalx_params *params, const gasalx_batch *host_batch,
                            const gasalx_results *host_out);
int gasalx_multi_pairhmm_host(gasalx_multi *m, const gasalx_hmm_batch *host_batch, float *host_result);
int gasalx_multi_pairhmm_quals_host(gasalx_multi *m, const gasalx_hmm_qual_batch *host_batch, float *host_result);
/* Device-resident shards (a batch already split over the entries' devices, as config 4's
 * 10 M reads would sit in HBM): entry i aligns batches[i] -- device arrays on its own device,
 * max_q_len / max_t_len set, or the lengths are read back -- into outs[i] on streams[i] (NULL:
 * the entry's engine stream), one host thread per entry.  gather (optional, NULL to skip): the
 * exchange step in the same call, every entry's aln_score (padded to gather_stride int32 per
 * entry: each aln_score buffer holds gather_stride entries) lands at gather[j] + i * gather_stride
 * on every entry j (gasalx_multi_allgather: RCCL when the group has a communicator, else peer
 * copies).  With streams given the call returns once the work is queued; with NULL it waits. */
int gasalx_multi_align_device(gasalx_multi *m, const gasalx_params *params, const gasalx_batch *batches,
                              const gasalx_results *outs, void *const *streams, int32_t *const *gather,
                              uint32_t gather_stride);
/* The same for PairHMM: entry i scores batches[i] into results[i] (float, gather_stride entries
 * when gathering), then the optional gather of the float results. */
int gasalx_multi_pairhmm_device(gasalx_multi *m, const gasalx_hmm_batch *batches, float *const *results,
                                void *const *streams, float *const *gather, uint32_t gather_stride);
/* The exchange step: entry i's `bytes` at send[i] (device memory of its device) land at
 * recv[j] + i * bytes on every entry j.  streams: one hipStream_t per entry (the call
 * is then asynchronous), or NULL for the engines' streams and a synchronous call. */
int gasalx_multi_allgather(gasalx_multi *m, const void *const *send, void *const *recv, uint64_t bytes,
                           void *const *streams);

/* Synthetic workloads of SURVEY.md §8(d) (benchmark/test data, std::mt19937_64).
 * Writes a GASAL2-layout batch (N_CODE padding) into caller buffers sized by
 * gasalx_synth_sizes.  kind: 1..4 = configs 1..4.  Pairs come in blocks of 65,536,
 * each from its own seeded generator (block 0: `seed` itself), so
 * gasalx_synth_range can write pairs [start, start + n) of a larger batch on
 * their own (one rank's shard); offsets then start at 0. */
int gasalx_synth_sizes(int kind, uint32_t n_pairs, uint64_t *q_bytes, uint64_t *t_bytes);
int gasalx_synth_spec(int kind, uint32_t *q_len, uint32_t *t_len);
int gasalx_synth_pairs(int kind, uint64_t seed, uint32_t n_pairs, uint8_t *q_batch, uint32_t *q_offsets,
                       uint32_t *q_lens, uint8_t *t_batch, uint32_t *t_offsets, uint32_t *t_lens);
int gasalx_synth_range(int kind, uint64_t seed, uint64_t start, uint32_t n_pairs, uint8_t *q_batch,
                       uint32_t *q_offsets, uint32_t *q_lens, uint8_t *t_batch, uint32_t *t_offsets,
                       uint32_t *t_lens);

#ifdef __cplusplus
}
#endif
#endif
