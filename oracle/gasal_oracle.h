/*
 * gasal_oracle.h — CPU restatement of the GASAL2 batched-alignment semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library; the product path
 * (genomics-gpu_amd/) never links or calls it.
 *
 * Parity anchor: the reference's kernels cannot be built in this image (they
 * need the CUDA runtime headers, gasal.h:9), so this restatement is pinned by
 * the known-answer vectors that SURVEY.md §8c records from the host-compiled
 * reference, plus the property tests in tests/.  Every function cites the
 * reference lines it follows (paths relative to Non-CDP/GASAL2/src).
 */
#ifndef GASAL_ORACLE_H
#define GASAL_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same numeric values as the reference enums (gasal.h:37-73). */
enum { ORC_WITHOUT_START = 0, ORC_WITH_START = 1, ORC_WITH_TB = 2 };
enum { ORC_NONE = 0, ORC_QUERY = 1, ORC_TARGET = 2, ORC_BOTH = 3 };
enum { ORC_UNKNOWN = 0, ORC_GLOBAL = 1, ORC_SEMI_GLOBAL = 2, ORC_LOCAL = 3,
       ORC_MICROLOCAL = 4, ORC_BANDED = 5, ORC_KSW = 6 };

typedef struct orc_params {
    int32_t match;          /* gasal_subst_scores.match      (_cudaMatchScore)    */
    int32_t mismatch;       /* gasal_subst_scores.mismatch   (_cudaMismatchScore) */
    int32_t gap_open;       /* _cudaGapO                                          */
    int32_t gap_extend;     /* _cudaGapExtend                                     */
    int32_t algo;           /* Parameters::algo                                   */
    int32_t start_pos;      /* Parameters::start_pos                              */
    int32_t second_best;    /* Parameters::secondBest                             */
    int32_t head, tail;     /* semiglobal_skipping_head / _tail                   */
    int32_t k_band;         /* Parameters::k_band (the kernel receives k_band>>3)  */
    int32_t is_packed;      /* Parameters::isPacked                               */
    int32_t n_code;         /* compile-time N_CODE of the reference (0x4E)        */
    int32_t has_n_penalty;  /* N_PENALTY defined?                                 */
    int32_t n_penalty;
    int32_t max_query_len;  /* compile-time MAX_QUERY_LEN of the reference        */
} orc_params;

/*
 * Batch entry that mirrors what gasal_aln_async (gasal_align.cu:29-307)
 * computes: pack -> optional reverse/complement -> alignment kernel ->
 * optional traceback.  Output arrays that the reference would not write for
 * the chosen configuration are left untouched (callers pre-fill them).
 *   cigar: qbytes bytes; initialised by this call to the device-side
 *          "unpacked_query_batch" contents, then overwritten by get_tb, exactly
 *          like the D2H copy at gasal_align.cu:281.
 * Returns 0 on success, negative on invalid arguments.
 */
int orc_aln_batch(const orc_params *p,
                  const uint8_t *q_batch, const uint32_t *q_offsets, const uint32_t *q_lens,
                  const uint8_t *t_batch, const uint32_t *t_offsets, const uint32_t *t_lens,
                  uint32_t q_bytes, uint32_t t_bytes, uint32_t n_alns,
                  const uint8_t *q_ops, const uint8_t *t_ops, const uint32_t *seed_scores,
                  int32_t *aln_score, int32_t *q_end, int32_t *t_end,
                  int32_t *q_start, int32_t *t_start,
                  int32_t *aln_score2, int32_t *q_end2, int32_t *t_end2,
                  uint8_t *cigar, uint32_t *n_cigar_ops, int n_threads);

/* gasal_pack_kernel restatement (kernels/pack_rc_seqs.h:13-53). */
void orc_pack(const uint8_t *bytes, uint32_t n_bytes, uint32_t *words);

/* gasal_reversecomplement_kernel restatement for one sequence (pack_rc_seqs.h:56-212). */
void orc_revcomp_one(uint32_t *batch_words, uint32_t word_idx, uint32_t len, uint8_t op, int32_t n_code);

/*
 * PairHMM forward, inter-task tile_1 semantics
 * (Non-CDP/PairHMM/inter_task/Synthetic_data/tile_1/tile_1.cu:44-177).
 * Per read base: read[i], and the four per-base parameters the reference
 * host code builds (tile_1.cu:415-419): qm = ph2pr[bq], delta = ph2pr[iq],
 * xiksi = ph2pr[dq], alpha = 1 - ph2pr[(iq+dq)&127].
 */
void orc_pairhmm_params(const uint8_t *bq, const uint8_t *iq, const uint8_t *dq, uint32_t n,
                        float *qm, float *delta, float *xiksi, float *alpha);
int orc_pairhmm_batch(uint32_t n_pairs,
                      const uint8_t *reads, const uint32_t *read_off, const uint32_t *read_len,
                      const float *qm, const float *delta, const float *xiksi, const float *alpha,
                      const uint8_t *haps, const uint32_t *hap_off, const uint32_t *hap_len,
                      float *result, int n_threads);

/*
 * nvbio batched alignment score (second front-end; nvbio_oracle.c).  aligner:
 * ORC_NV_ED / _SW / _GOTOH; type: nvbio AlignmentType (GLOBAL 0, LOCAL 1, SEMI_GLOBAL 2).
 * prm = {match, mismatch, gap_open, gap_ext, deletion, insertion} (signed).
 * Strings are nvbio packed sets (bits per symbol, big-endian flag); toff NULL = one
 * shared text of tlen0 symbols.  Returns the BestSink score per pair.
 */
enum { ORC_NV_ED = 0, ORC_NV_SW = 1, ORC_NV_GOTOH = 2 };
enum { ORC_NV_GLOBAL = 0, ORC_NV_LOCAL = 1, ORC_NV_SEMI_GLOBAL = 2 };
int32_t orc_nv_score_one(int aligner, int type, const int32_t prm[6], const uint32_t *pat, uint32_t M,
                         const uint32_t *txt, uint32_t N);
int orc_nv_score_batch(int aligner, int type, const int32_t prm[6], uint32_t n,
                       const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                       const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits, uint32_t tbig,
                       int32_t *scores, int n_threads);
/* nvbio banded score (BatchedBandedAlignmentScore<band>): same arguments plus the band
 * length (>= 2); BestSink score per pair, INT32_MIN when text_len < pattern_len. */
int32_t orc_nv_banded_score_one(int aligner, int type, const int32_t prm[6], uint32_t band, const uint32_t *pat,
                                uint32_t M, const uint32_t *txt, uint32_t N);
int orc_nv_banded_score_batch(int aligner, int type, const int32_t prm[6], uint32_t band, uint32_t n,
                              const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                              const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits, uint32_t tbig,
                              int32_t *scores, int n_threads);
/* nvbio full-DP traceback (nvbio_oracle.c): Gotoh, Smith-Waterman and ED (= SW with 0/-1/-1/-1) */
int32_t orc_nv_traceback_one(int aligner, int type, const int32_t prm[6], const uint32_t *pat, uint32_t M,
                             const uint32_t *txt, uint32_t N, uint32_t src[2], uint32_t snk[2], uint8_t *ops,
                             uint32_t *n_ops);
int orc_nv_traceback_batch(int aligner, int type, const int32_t prm[6], uint32_t n,
                           const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                           const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits, uint32_t tbig,
                           int32_t *scores, uint32_t *src, uint32_t *snk, uint8_t *ops, uint32_t ops_stride,
                           uint32_t *n_ops, int n_threads);
/* nvbio banded traceback (BatchedBandedAlignmentTraceback<band>): per pair the BestSink score,
 * source / sink (x = text, y = pattern) and the pushes; ED, SW and Gotoh aligners */
int32_t orc_nv_banded_traceback_one(int aligner, int type, const int32_t prm[6], uint32_t band, const uint32_t *pat,
                                    uint32_t M, const uint32_t *txt, uint32_t N, uint32_t src[2], uint32_t snk[2],
                                    uint8_t *ops, uint32_t *n_ops);
int orc_nv_banded_traceback_batch(int aligner, int type, const int32_t prm[6], uint32_t band, uint32_t n,
                                  const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                                  const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits,
                                  uint32_t tbig, int32_t *scores, uint32_t *src, uint32_t *snk, uint8_t *ops,
                                  uint32_t ops_stride, uint32_t *n_ops, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
