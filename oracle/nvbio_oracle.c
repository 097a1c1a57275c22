/*
 * nvbio_oracle.c — CPU restatement of nvbio's batched alignment scoring
 * (TEST INFRASTRUCTURE ONLY; see gasal_oracle.h for who may load liborc).
 *
 * Follows the TextBlockingTag score functions literally: 8-column text stripes,
 * pattern rows top to bottom inside a stripe, the stripe's right column carried
 * to the next one as (H, E) (paths under Non-CDP/NvB/nvbio/alignment):
 *   gotoh/gotoh_inl.h:985-1110   update_row (F from above, E from the left, max3, LOCAL clamp,
 *                                 LOCAL sink over every cell of the band)
 *   gotoh/gotoh_inl.h:1140-1260  stripe loop: first band H(-1, c) = GLOBAL ? Go + Ge*c : 0,
 *                                 F = infimum; SEMI_GLOBAL sink over the last row per stripe
 *   gotoh/gotoh_inl.h:1395-1420  last stripe: SEMI / GLOBAL sinks guarded by block + j <= N / == N
 *   gotoh/gotoh_inl.h:60-88      first column: H(i,-1) = LOCAL ? 0 : Go + Ge*i, E = LOCAL ? 0 : infimum
 *   sw/sw_inl.h:895-970, 1069-1215 and :60-80  the same for linear gaps (Del left, Ins top)
 *   ed/ed_inl.h:97, ed/ed_utils.h:45-52        edit distance = SW with (0, -1, -1, -1)
 *   sink_inl.h:38-40, 59-68      BestSink: starts at INT32_MIN, keeps the last maximum (<=)
 *   utils.h:92-135               SimpleSmithWatermanScheme / SimpleGotohScheme
 * The infimum is Field_traits<int32>::min() - min(Go, Ge) (gotoh_inl.h:1162), int32 columns.
 *
 * Banded (orc_nv_banded_*; NvB/nvbio/alignment/batched_banded_inl.h:44-75 per pair):
 *   sw/sw_banded_inl.h:44-54      row zero: band[j] = GLOBAL ? j * deletion : 0
 *   sw/sw_banded_inl.h:361-512    rows: band[j] = H(i, i + j); j = 0 has no left, j = B-1 no top;
 *                                 top = band[j+1] + deletion, left = band[j-1] + insertion;
 *                                 sinks: LOCAL every cell, GLOBAL band[B-1], SEMI band[j < m]
 *   gotoh/gotoh_banded_inl.h:44-75, 405-666  the same with F (vertical, per band slot) and E
 *                                 (horizontal, carried along the row); F[B-1] = infimum
 *   ed/ed_banded_inl.h:63-78      edit distance = the SW form with (0, -1, -1, -1)
 *   the alignment is skipped (BestSink stays INT32_MIN) when text_len < pattern_len.
 *
 * Parity status: nvbio needs CUDA + thrust to build.  The restatement is pinned by the
 * reference's own unit-test vectors (NvB/nvbio-test/alignment_test.cu:680-793 via
 * tests/golden/nvbio_reference_kats.json: CIGAR-implied optima and the banded edit-distance
 * cases) and by hand-derived known answers (tests/test_nvbio_oracle.py).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "gasal_oracle.h"

#define NV_BAND 8

static inline int32_t nmax(int32_t a, int32_t b) { return a > b ? a : b; }

/* PackedStream symbol s of a set (nvbio/basic/packedstream.h layout). */
static uint32_t nv_sym(const uint32_t *w, uint32_t bits, uint32_t big, uint64_t s) {
    const uint32_t per = 32u / bits, p = (uint32_t)(s % per);
    const uint32_t sh = big ? 32u - bits * (p + 1) : bits * p;
    return (w[s / per] >> sh) & (bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u));
}

int32_t orc_nv_score_one(int aligner, int type, const int32_t prm[6], const uint32_t *pat, uint32_t M,
                         const uint32_t *txt, uint32_t N) {
    int32_t match = prm[0], mismatch = prm[1], Go = prm[2], Ge = prm[3], Del = prm[4], Ins = prm[5];
    if (aligner == ORC_NV_ED) { match = 0; mismatch = -1; Del = -1; Ins = -1; }
    const int gotoh = aligner == ORC_NV_GOTOH;
    const int32_t infimum = INT32_MIN - (Go < Ge ? Go : Ge);
    int32_t best = INT32_MIN;                                  /* BestSink() */
    /* temp column: (H, E) of the stripe's last column per pattern row */
    int32_t *tH = (int32_t *)malloc((M + 1) * sizeof(int32_t));
    int32_t *tE = (int32_t *)malloc((M + 1) * sizeof(int32_t));
    for (uint32_t i = 0; i < M; i++) {
        if (gotoh) { tH[i] = type != ORC_NV_LOCAL ? Go + Ge * (int32_t)i : 0; tE[i] = type == ORC_NV_LOCAL ? 0 : infimum; }
        else { tH[i] = type != ORC_NV_LOCAL ? Ins * (int32_t)(i + 1) : 0; tE[i] = 0; }
    }
    const uint32_t end_block = N > NV_BAND ? (N + NV_BAND - 1) / NV_BAND * NV_BAND : NV_BAND;
    for (uint32_t block = 0; block < end_block; block += NV_BAND) {
        const int last = block + NV_BAND >= end_block;
        int32_t Hb[NV_BAND + 1], Fb[NV_BAND + 1];
        uint32_t r_cache[NV_BAND];
        for (uint32_t t = 0; t < NV_BAND; t++) r_cache[t] = block + t < N ? txt[block + t] : 0xFFFFFFFFu;
        for (uint32_t j = 0; j <= NV_BAND; j++) {
            if (gotoh) Hb[j] = type == ORC_NV_GLOBAL ? (block + j > 0 ? Go + Ge * (int32_t)(block + j - 1) : 0) : 0;
            else Hb[j] = type == ORC_NV_GLOBAL ? Del * (int32_t)(block + j) : 0;
            Fb[j] = infimum;
        }
        int32_t temp_i = Hb[0];
        for (uint32_t i = 0; i < M; i++) {
            const uint32_t q = pat[i];
            int32_t Hdiag = temp_i;
            Hb[0] = temp_i = tH[i];
            int32_t E = tE[i];
            for (uint32_t j = 1; j <= NV_BAND; j++) {
                const int32_t S = (r_cache[j - 1] == q) ? match : mismatch;
                int32_t h;
                if (gotoh) {
                    Fb[j] = nmax(Fb[j] + Ge, Hb[j] + Go);
                    E = nmax(E + Ge, Hb[j - 1] + Go);
                    h = nmax(nmax(E, Fb[j]), Hdiag + S);
                } else {
                    h = nmax(nmax(Hb[j] + Ins, Hb[j - 1] + Del), Hdiag + S);
                }
                if (type == ORC_NV_LOCAL) h = nmax(h, 0);
                Hdiag = Hb[j];
                Hb[j] = h;
                if (type == ORC_NV_LOCAL && (!last || block + j <= N) && best <= h) best = h;
            }
            tH[i] = Hb[NV_BAND];
            tE[i] = E;
        }
        for (uint32_t j = 1; j <= NV_BAND; j++) {   /* :1224-1229, :1403-1420 (Hb = the last row) */
            if (type == ORC_NV_SEMI_GLOBAL && (!last || block + j <= N) && best <= Hb[j]) best = Hb[j];
            if (type == ORC_NV_GLOBAL && last && block + j == N && best <= Hb[j]) best = Hb[j];
        }
    }
    free(tH);
    free(tE);
    return best;
}

int orc_nv_score_batch(int aligner, int type, const int32_t prm[6], uint32_t n,
                       const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                       const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits, uint32_t tbig,
                       int32_t *scores, int n_threads) {
    if (!prm || !pw || !poff || !tw || !scores) return -1;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads)
#endif
    for (long k = 0; k < (long)n; k++) {
        const uint32_t M = poff[k + 1] - poff[k];
        const uint64_t t0 = toff ? toff[k] : 0;
        const uint32_t N = toff ? toff[k + 1] - toff[k] : tlen0;
        uint32_t *p = (uint32_t *)malloc((M + 1) * sizeof(uint32_t));
        uint32_t *t = (uint32_t *)malloc((N + 1) * sizeof(uint32_t));
        for (uint32_t i = 0; i < M; i++) p[i] = nv_sym(pw, pbits, pbig, (uint64_t)poff[k] + i);
        for (uint32_t i = 0; i < N; i++) t[i] = nv_sym(tw, tbits, tbig, t0 + i);
        scores[k] = orc_nv_score_one(aligner, type, prm, p, M, t, N);
        free(p);
        free(t);
    }
    return 0;
}

/*
 * Banded score, one pair (see the header for the reference lines).  Text symbols are
 * read as 255 past text_len: the row loop's guard (sw_banded_inl.h:453,
 * gotoh_banded_inl.h:597); the reference's first-band load (:375 / :433) has no guard
 * and reads past the string only when text_len < band - 1.
 */
int32_t orc_nv_banded_score_one(int aligner, int type, const int32_t prm[6], uint32_t band, const uint32_t *pat,
                                uint32_t M, const uint32_t *txt, uint32_t N) {
    int32_t match = prm[0], mismatch = prm[1], Go = prm[2], Ge = prm[3], Del = prm[4], Ins = prm[5];
    if (aligner == ORC_NV_ED) { match = 0; mismatch = -1; Del = -1; Ins = -1; }
    int32_t best = INT32_MIN;                                  /* BestSink() */
    if (N < M || band < 2) return best;
    const uint32_t B = band;
    int32_t *H = (int32_t *)malloc(B * sizeof(int32_t)), *F = (int32_t *)malloc(B * sizeof(int32_t));
    /* gotoh_banded_inl.h:440-442: Field_traits<short>::min() - max(Go, Ge, text Go, text Ge) */
    const int32_t infimum = -32768 - (Go > Ge ? Go : Ge);
#define TXT(k) ((k) < N ? txt[k] : 255u)
    if (aligner == ORC_NV_GOTOH) {
        H[0] = 0;
        for (uint32_t j = 1; j < B; j++) H[j] = type == ORC_NV_GLOBAL ? Go + (int32_t)(j - 1) * Ge : 0;
        for (uint32_t j = 0; j < B; j++) F[j] = infimum;
        for (uint32_t i = 0; i < M; i++) {
            const uint32_t q = pat[i];
            int32_t hi;
            {   /* j == 0 */
                F[0] = nmax(F[1] + Ge, H[1] + Go);
                const int32_t diag = H[0] + (TXT(i) == q ? match : mismatch);
                hi = nmax(F[0], diag);
                if (type == ORC_NV_LOCAL) { hi = nmax(hi, 0); if (best <= hi) best = hi; }
                H[0] = hi;
            }
            int32_t E = H[0] + Go;
            for (uint32_t j = 1; j + 1 < B; j++) {
                F[j] = nmax(F[j + 1] + Ge, H[j + 1] + Go);
                const int32_t diag = H[j] + (TXT(i + j) == q ? match : mismatch);
                hi = nmax(nmax(F[j], E), diag);
                if (type == ORC_NV_LOCAL) { hi = nmax(hi, 0); if (best <= hi) best = hi; }
                H[j] = hi;
                E = nmax(hi + Go, E + Ge);
            }
            {   /* j == B-1 */
                F[B - 1] = infimum;
                const int32_t diag = H[B - 1] + (TXT(i + B - 1) == q ? match : mismatch);
                hi = nmax(E, diag);
                if (type == ORC_NV_LOCAL) { hi = nmax(hi, 0); if (best <= hi) best = hi; }
                H[B - 1] = hi;
            }
        }
    } else {
        for (uint32_t j = 0; j < B; j++) H[j] = type == ORC_NV_GLOBAL ? (int32_t)j * Del : 0;
        for (uint32_t i = 0; i < M; i++) {
            const uint32_t q = pat[i];
            int32_t hi;
            {   /* j == 0: top and diagonal */
                const int32_t diag = H[0] + (TXT(i) == q ? match : mismatch);
                hi = nmax(H[1] + Del, diag);
                if (type == ORC_NV_LOCAL) { hi = nmax(hi, 0); if (best <= hi) best = hi; }
                H[0] = hi;
            }
            for (uint32_t j = 1; j + 1 < B; j++) {
                const int32_t diag = H[j] + (TXT(i + j) == q ? match : mismatch);
                hi = nmax(nmax(H[j + 1] + Del, H[j - 1] + Ins), diag);
                if (type == ORC_NV_LOCAL) { hi = nmax(hi, 0); if (best <= hi) best = hi; }
                H[j] = hi;
            }
            {   /* j == B-1: left and diagonal */
                const int32_t diag = H[B - 1] + (TXT(i + B - 1) == q ? match : mismatch);
                hi = nmax(H[B - 2] + Ins, diag);
                if (type == ORC_NV_LOCAL) { hi = nmax(hi, 0); if (best <= hi) best = hi; }
                H[B - 1] = hi;
            }
        }
    }
#undef TXT
    if (type == ORC_NV_GLOBAL) {
        if (best <= H[B - 1]) best = H[B - 1];
    } else if (type == ORC_NV_SEMI_GLOBAL) {
        const uint32_t m = (M + B - 1 < N ? M + B - 1 : N) - (M - 1);
        if (best <= H[0]) best = H[0];
        for (uint32_t j = 1; j < B; j++)
            if (j < m && best <= H[j]) best = H[j];
    }
    free(H);
    free(F);
    return best;
}

int orc_nv_banded_score_batch(int aligner, int type, const int32_t prm[6], uint32_t band, uint32_t n,
                              const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                              const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits, uint32_t tbig,
                              int32_t *scores, int n_threads) {
    if (!prm || !pw || !poff || !tw || !scores || band < 2) return -1;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads)
#endif
    for (long k = 0; k < (long)n; k++) {
        const uint32_t M = poff[k + 1] - poff[k];
        const uint64_t t0 = toff ? toff[k] : 0;
        const uint32_t N = toff ? toff[k + 1] - toff[k] : tlen0;
        uint32_t *p = (uint32_t *)malloc((M + 1) * sizeof(uint32_t));
        uint32_t *t = (uint32_t *)malloc((N + 1) * sizeof(uint32_t));
        for (uint32_t i = 0; i < M; i++) p[i] = nv_sym(pw, pbits, pbig, (uint64_t)poff[k] + i);
        for (uint32_t i = 0; i < N; i++) t[i] = nv_sym(tw, tbits, tbig, t0 + i);
        scores[k] = orc_nv_banded_score_one(aligner, type, prm, band, p, M, t, N);
        free(p);
        free(t);
    }
    return 0;
}
