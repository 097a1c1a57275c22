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

/*
 * Full-DP traceback, one pair (nvbio alignment_traceback, NvB/nvbio/alignment):
 *   alignment_inl.h:365-465     checkpoint pass with a BestSink, then the walk back from its
 *                               sink through the checkpointed submatrices, then (SEMI_GLOBAL /
 *                               GLOBAL) the first row / column, then the clips
 *   gotoh/gotoh_inl.h:462-593   PatternBlockingTag update_row: rows i = text symbols, columns
 *                               j = pattern symbols in stripes of BAND_LEN = 8 (:1491-1495);
 *                               F from the row above (DELETION), E from the left (INSERTION),
 *                               max3, LOCAL clamp; hdir = top > left ? (top > diag ? DEL : SUB)
 *                               : (left > diag ? INS : SUB), edir / fdir = strictly greater
 *                               extension; LOCAL reports every cell (i + 1, block + j) to the sink
 *   gotoh/gotoh_inl.h:441-442   the stored flags: LOCAL and H == 0 -> SINK, | edir | fdir
 *   gotoh/gotoh_inl.h:695, 247-300  boundaries: H(-1, c) = LOCAL ? 0 : Go + Ge*c (0 at c = -1),
 *                               F(-1, c) = infimum; H(i, -1) = GLOBAL ? Go + Ge*i : 0,
 *                               E(i, -1) = LOCAL ? 0 : infimum (GotohCheckpointContext::init)
 *   gotoh/gotoh_inl.h:1806-1872 the walk: H state follows hdir (INS -> E state, DEL -> F state,
 *                               else a diagonal step), E / F states step and leave on a clear
 *                               extension bit; LOCAL stops on SINK in the H state
 *   sw/sw_inl.h:420-540, 380-400, 660-663, 243-251, 1653-1709  the same for linear gaps:
 *                               top = H(i-1, j) + deletion, left = H(i, j-1) + insertion,
 *                               H(-1, c) = LOCAL ? 0 : insertion*(c+1), H(i, -1) = GLOBAL ?
 *                               deletion*(i+1) : 0; the walk steps on the stored op
 *   utils_inl.h:273-300         SEMI_GLOBAL reports H(i, M-1) at (i + 1, M) per row of the last
 *                               stripe, GLOBAL H(N-1, M-1) at (N, M) once
 *   sink_inl.h                  BestSink keeps the last maximum (<=) in report order: for LOCAL
 *                               stripe, then row, then column
 * ops[] are the backtracker's pushes in push order (end of the alignment first): 0 SUBSTITUTION,
 * 1 INSERTION (a pattern symbol), 2 DELETION (a text symbol) -- nvbio-test's TestBacktracker
 * prints "MID"[op] (alignment_test_utils.h:628-645).  src / snk: the Alignment's source and
 * sink (x = text coordinate, y = pattern coordinate); (0xFFFFFFFF, 0xFFFFFFFF) and no ops when
 * no cell was reported.  Scores are int32 here; nvbio stores columns and checkpoints as int16
 * (utils.h:49-64), the same values while they stay within ±32767.
 */
int32_t orc_nv_traceback_one(int aligner, int type, const int32_t prm[6], const uint32_t *pat, uint32_t M,
                             const uint32_t *txt, uint32_t N, uint32_t src[2], uint32_t snk[2], uint8_t *ops,
                             uint32_t *n_ops) {
    const int32_t match = prm[0], mismatch = prm[1], Go = prm[2], Ge = prm[3], Del = prm[4], Ins = prm[5];
    const int gotoh = aligner == ORC_NV_GOTOH;
    const int32_t infimum = -32768 - (Go < Ge ? Go : Ge);
    enum { SUB = 0, INS = 1, DEL = 2, SNK = 3, INS_EXT = 4, DEL_EXT = 8 };
    *n_ops = 0;
    src[0] = src[1] = snk[0] = snk[1] = 0xFFFFFFFFu;
    if (M == 0 || N == 0) return INT32_MIN;
    if (aligner == ORC_NV_ED) {   /* ed/ed_inl.h:347-365: SW with EditDistanceSWScheme (ed_utils.h:45-52) */
        const int32_t ed[6] = {0, -1, 0, 0, -1, -1};
        return orc_nv_traceback_one(ORC_NV_SW, type, ed, pat, M, txt, N, src, snk, ops, n_ops);
    }
    uint8_t *dir = (uint8_t *)malloc((size_t)M * N);
    int32_t *Hp = (int32_t *)malloc((M + 1) * sizeof(int32_t));   /* H(i-1, c), c = -1 .. M-1 at [c + 1] */
    int32_t *Fp = (int32_t *)malloc((M + 1) * sizeof(int32_t));   /* F(i-1, c) at [c + 1] */
    for (uint32_t c = 0; c <= M; c++) {
        const int32_t cc = (int32_t)c - 1;
        Hp[c] = type == ORC_NV_LOCAL || cc < 0 ? 0 : gotoh ? Go + Ge * cc : Ins * (cc + 1);
        Fp[c] = infimum;
    }
    int32_t best = INT32_MIN;
    uint32_t bx = 0xFFFFFFFFu, by = 0xFFFFFFFFu, bblk = 0;
    for (uint32_t i = 0; i < N; i++) {
        const uint32_t r = txt[i];
        const int32_t hl0 = type == ORC_NV_GLOBAL ? (gotoh ? Go + Ge * (int32_t)i : Del * (int32_t)(i + 1)) : 0;
        int32_t diagH = Hp[0];                /* H(i-1, -1) */
        int32_t left = hl0;                   /* H(i, j-1) */
        int32_t E = type == ORC_NV_LOCAL ? 0 : infimum;
        Hp[0] = hl0;
        for (uint32_t j = 0; j < M; j++) {
            const int32_t S = r == pat[j] ? match : mismatch;
            const int32_t up = Hp[j + 1];
            int32_t h, top, lft;
            uint8_t d;
            if (gotoh) {
                const int32_t ftop = Fp[j + 1] + Ge, htop = up + Go;
                const int32_t F = nmax(ftop, htop);
                const uint8_t fdir = ftop > htop ? DEL_EXT : SUB;
                const int32_t eleft = E + Ge, hleft = left + Go;
                E = nmax(eleft, hleft);
                const uint8_t edir = eleft > hleft ? INS_EXT : SUB;
                Fp[j + 1] = F;
                top = F; lft = E;
                const int32_t diag = diagH + S;
                h = nmax(nmax(lft, top), diag);
                if (type == ORC_NV_LOCAL) h = nmax(h, 0);
                const uint8_t hdir = top > lft ? (top > diag ? DEL : SUB) : (lft > diag ? INS : SUB);
                d = (uint8_t)((type == ORC_NV_LOCAL && h == 0 ? SNK : hdir) | edir | fdir);
            } else {
                top = up + Del; lft = left + Ins;
                const int32_t diag = diagH + S;
                h = nmax(nmax(top, lft), diag);
                if (type == ORC_NV_LOCAL) h = nmax(h, 0);
                const uint8_t hdir = top > lft ? (top > diag ? DEL : SUB) : (lft > diag ? INS : SUB);
                d = (uint8_t)(type == ORC_NV_LOCAL && h == 0 ? SNK : hdir);
            }
            dir[(size_t)i * M + j] = d;
            diagH = up;
            Hp[j + 1] = h;
            left = h;
            if (type == ORC_NV_LOCAL) {   /* report order: stripe, row, column; the last maximum wins */
                const uint32_t blk = j / NV_BAND;
                if (h > best || (h == best && (blk > bblk || (blk == bblk && (i + 1 > bx || (i + 1 == bx && j + 1 >= by)))))) {
                    best = h; bx = i + 1; by = j + 1; bblk = blk;
                }
            }
        }
        if (type == ORC_NV_SEMI_GLOBAL && best <= Hp[M]) { best = Hp[M]; bx = i + 1; by = M; }
    }
    if (type == ORC_NV_GLOBAL) { best = Hp[M]; bx = N; by = M; }
    snk[0] = bx; snk[1] = by;
    /* the walk (alignment_inl.h:413-462): row = x, col = y - 1 */
    int32_t row = (int32_t)bx, col = (int32_t)by - 1;
    int state = 0;   /* HSTATE / ESTATE / FSTATE */
    uint32_t k = 0;
    while (row > 0 && col >= 0) {
        const uint8_t op = dir[(size_t)(row - 1) * M + (uint32_t)col];
        if (gotoh) {
            const uint8_t h_op = op & 3u;
            if (type == ORC_NV_LOCAL && state == 0 && h_op == SNK) break;
            if (state == 1) {
                if ((op & INS_EXT) == 0) state = 0;
                --col; ops[k++] = INS;
            } else if (state == 2) {
                if ((op & DEL_EXT) == 0) state = 0;
                --row; ops[k++] = DEL;
            } else if (h_op == INS) {
                state = 1;
            } else if (h_op == DEL) {
                state = 2;
            } else {
                --col; --row; ops[k++] = SUB;
            }
        } else {
            if (type == ORC_NV_LOCAL && op == SNK) break;
            if (op != DEL) --col;
            if (op != INS) --row;
            ops[k++] = op;
        }
    }
    uint32_t sx = (uint32_t)row, sy = (uint32_t)(col + 1);
    if (type != ORC_NV_LOCAL && sx == 0)
        for (; sy > 0; --sy) ops[k++] = INS;
    if (type == ORC_NV_GLOBAL && sy == 0)
        for (; sx > 0; --sx) ops[k++] = DEL;
    src[0] = sx; src[1] = sy;
    *n_ops = k;
    free(dir); free(Hp); free(Fp);
    return best;
}

/* n pairs; ops of pair k at ops + k * ops_stride (ops_stride >= M_k + N_k) */
int orc_nv_traceback_batch(int aligner, int type, const int32_t prm[6], uint32_t n,
                           const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                           const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits, uint32_t tbig,
                           int32_t *scores, uint32_t *src, uint32_t *snk, uint8_t *ops, uint32_t ops_stride,
                           uint32_t *n_ops, int n_threads) {
    if (!prm || !pw || !poff || !tw || !scores || !src || !snk || !ops || !n_ops) return -1;
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
        scores[k] = M + N <= ops_stride
                        ? orc_nv_traceback_one(aligner, type, prm, p, M, t, N, src + 2 * k, snk + 2 * k,
                                               ops + (size_t)k * ops_stride, n_ops + k)
                        : INT32_MIN;
        free(p);
        free(t);
    }
    return 0;
}

/*
 * Banded traceback, one pair (nvbio banded_alignment_traceback, banded_inl.h:352-427, as
 * BatchedBandedAlignmentTraceback<BAND_LEN, CHECKPOINTS> runs it, batched_banded_inl.h:248-297):
 * the checkpoint pass with a BestSink, then the walk from its sink back through the recomputed
 * band submatrices, then the clips.  Rows i = pattern symbols, band entry j = text symbol i + j
 * (the orientation of the banded score, orc_nv_banded_score_one):
 *   gotoh/gotoh_banded_inl.h:482-614  the row: j = 0 top (F) and diagonal; 0 < j < B-1 max3;
 *       j = B-1 left (E) and diagonal; F from the row above is an INSERTION (pattern symbol
 *       against a gap), E along the row a DELETION; hdir = top > left ? (top > diag ? INS : SUB)
 *       : (left > diag ? DEL : SUB) (j = 0: top > diag ? INS : SUB; j = B-1: left > diag ? DEL :
 *       SUB); fdir = F[j+1] + Ge > H[j+1] + Go ? DELETION_EXT; the E flag of cell j is the edir
 *       of cell j-1's update (INSERTION_EXT when E + Ge > H + Go; SUB for j <= 1);
 *   gotoh_banded_inl.h:323-339  stored flag: (LOCAL and H == 0 ? SINK : hdir) | edir | fdir;
 *   gotoh_banded_inl.h:895-962  the walk: entry = sink.x - sink.y, row = sink.y - 1; H state:
 *       DEL -> E state, INS -> F state, else row - 1 and push SUB; E state: entry - 1, push
 *       DELETION, leave on a clear INSERTION_EXT bit; F state: entry + 1, row - 1, push INSERTION,
 *       leave on a clear DELETION_EXT bit; LOCAL stops on SINK in the H state with source
 *       (entry + row + 1, row + 1); otherwise the walk ends past row 0 with source (entry, 0);
 *   sw/sw_banded_inl.h:392-475, 268-279, 740-798  the same for linear gaps (top + deletion,
 *       left + insertion); the SW submatrix stores hdir as is, never SINK, so the SW walk runs
 *       to row 0 in LOCAL too; ED is SW with EditDistanceSWScheme (ed_banded_inl.h:175-295);
 *   the sink (banded score pass): LOCAL every cell (i + j + 1, i + 1) in row-then-band order,
 *       SEMI_GLOBAL the last row's entries j < min(M + B - 1, N) - (M - 1) at (M + j, M),
 *       GLOBAL entry B-1 at (M + B - 1, M); BestSink keeps the last maximum (sink_inl.h:59-68).
 * nvbio recomputes each submatrix from int16 checkpoints clamped at -32736
 * (gotoh_banded_inl.h:234-239): the same flags while every score stays above it, which the
 * C-ABI's range condition ensures.  A pair with N < M keeps the BestSink's INT32_MIN and
 * (-1, -1) ends (gotoh_banded_inl.h:431-432, banded_inl.h:389-392).
 */
int32_t orc_nv_banded_traceback_one(int aligner, int type, const int32_t prm[6], uint32_t band, const uint32_t *pat,
                                    uint32_t M, const uint32_t *txt, uint32_t N, uint32_t src[2], uint32_t snk[2],
                                    uint8_t *ops, uint32_t *n_ops) {
    int32_t match = prm[0], mismatch = prm[1], Go = prm[2], Ge = prm[3], Del = prm[4], Ins = prm[5];
    if (aligner == ORC_NV_ED) { match = 0; mismatch = -1; Del = -1; Ins = -1; }
    enum { SUB = 0, INS = 1, DEL = 2, SNK = 3, INS_EXT = 4, DEL_EXT = 8 };
    const int gotoh = aligner == ORC_NV_GOTOH;
    *n_ops = 0;
    src[0] = src[1] = snk[0] = snk[1] = 0xFFFFFFFFu;
    if (N < M || band < 2) return INT32_MIN;
    const uint32_t B = band;
    const int32_t infimum = -32768 - (Go > Ge ? Go : Ge);
    int32_t *H = (int32_t *)malloc(B * sizeof(int32_t)), *F = (int32_t *)malloc(B * sizeof(int32_t));
    uint8_t *dir = (uint8_t *)malloc((size_t)M * B + 1);
    for (uint32_t j = 0; j < B; j++) {
        if (gotoh) H[j] = j == 0 ? 0 : (type == ORC_NV_GLOBAL ? Go + (int32_t)(j - 1) * Ge : 0);
        else H[j] = type == ORC_NV_GLOBAL ? (int32_t)j * Del : 0;
        F[j] = infimum;
    }
    int32_t best = INT32_MIN;
    uint32_t bx = 0xFFFFFFFFu, by = 0xFFFFFFFFu;
#define TXT(k) ((k) < N ? txt[k] : 255u)
#define REPORT(h, x, y) do { if (best <= (h)) { best = (h); bx = (x); by = (y); } } while (0)
    for (uint32_t i = 0; i < M; i++) {
        const uint32_t q = pat[i];
        uint8_t *d = dir + (size_t)i * B;
        if (gotoh) {
            int32_t E = 0;
            uint8_t edir = SUB;
            for (uint32_t j = 0; j < B; j++) {
                const int32_t diag = H[j] + (TXT(i + j) == q ? match : mismatch);
                uint8_t fdir = SUB, hdir;
                int32_t hi;
                if (j + 1 < B) {
                    const int32_t ftop = F[j + 1] + Ge, htop = H[j + 1] + Go;
                    F[j] = nmax(ftop, htop);
                    fdir = ftop > htop ? DEL_EXT : SUB;
                } else {
                    F[j] = infimum;
                }
                if (j == 0) {
                    hi = nmax(F[0], diag);
                    hdir = F[0] > diag ? INS : SUB;
                } else if (j + 1 < B) {
                    hi = nmax(nmax(F[j], E), diag);
                    hdir = F[j] > E ? (F[j] > diag ? INS : SUB) : (E > diag ? DEL : SUB);
                } else {
                    hi = nmax(E, diag);
                    hdir = E > diag ? DEL : SUB;
                }
                if (type == ORC_NV_LOCAL) {
                    hi = nmax(hi, 0);
                    if (hi == 0) hdir = SNK;
                    REPORT(hi, i + j + 1, i + 1);
                }
                d[j] = (uint8_t)(hdir | (j == 0 ? SUB : edir) | fdir);
                H[j] = hi;
                if (j == 0) { E = hi + Go; edir = SUB; }
                else {
                    const int32_t eleft = E + Ge, ediag = hi + Go;
                    edir = eleft > ediag ? INS_EXT : SUB;
                    E = nmax(ediag, eleft);
                }
            }
        } else {
            for (uint32_t j = 0; j < B; j++) {
                const int32_t diag = H[j] + (TXT(i + j) == q ? match : mismatch);
                int32_t hi;
                uint8_t hdir;
                if (j == 0) {
                    const int32_t top = H[1] + Del;
                    hi = nmax(top, diag);
                    hdir = top > diag ? INS : SUB;
                } else if (j + 1 < B) {
                    const int32_t top = H[j + 1] + Del, left = H[j - 1] + Ins;
                    hi = nmax(nmax(top, left), diag);
                    hdir = top > left ? (top > diag ? INS : SUB) : (left > diag ? DEL : SUB);
                } else {
                    const int32_t left = H[j - 1] + Ins;
                    hi = nmax(left, diag);
                    hdir = left > diag ? DEL : SUB;
                }
                if (type == ORC_NV_LOCAL) {
                    hi = nmax(hi, 0);
                    REPORT(hi, i + j + 1, i + 1);
                }
                d[j] = hdir;
                H[j] = hi;
            }
        }
    }
    if (type == ORC_NV_GLOBAL) {
        REPORT(H[B - 1], M + B - 1, M);
    } else if (type == ORC_NV_SEMI_GLOBAL) {
        const uint32_t m = (M + B - 1 < N ? M + B - 1 : N) - (M - 1u);
        REPORT(H[0], M, M);
        for (uint32_t j = 1; j < B; j++)
            if (j < m) REPORT(H[j], M + j, M);
    }
#undef REPORT
#undef TXT
    snk[0] = bx; snk[1] = by;
    uint32_t k = 0;
    if (bx != 0xFFFFFFFFu && by != 0xFFFFFFFFu) {
        int32_t e = (int32_t)bx - (int32_t)by, row = (int32_t)by - 1;
        int state = 0;   /* H / E / F */
        uint32_t sx = 0, sy = 0;
        int found = 0;
        while (row >= 0) {
            const uint8_t op = dir[(size_t)row * B + (uint32_t)e];
            if (gotoh) {
                if (type == ORC_NV_LOCAL && state == 0 && (op & 3u) == SNK) { found = 1; break; }
                if (state == 1) {
                    if ((op & INS_EXT) == 0) state = 0;
                    --e; ops[k++] = DEL;
                } else if (state == 2) {
                    if ((op & DEL_EXT) == 0) state = 0;
                    ++e; --row; ops[k++] = INS;
                } else if ((op & 3u) == DEL) {
                    state = 1;
                } else if ((op & 3u) == INS) {
                    state = 2;
                } else {
                    --row; ops[k++] = SUB;
                }
            } else {
                if (op == DEL) { --e; ops[k++] = DEL; }
                else if (op == INS) { ++e; --row; ops[k++] = INS; }
                else { --row; ops[k++] = SUB; }
            }
        }
        if (found) { sy = (uint32_t)row + 1; sx = (uint32_t)e + sy; }
        else { sy = 0; sx = (uint32_t)e; }
        src[0] = sx; src[1] = sy;
    }
    *n_ops = k;
    free(H); free(F); free(dir);
    return best;
}

/* n pairs; ops of pair k at ops + k * ops_stride (ops_stride >= 2 M_k + band: every row is one
 * SUB or INS push, and the DEL pushes are at most band - 1 plus the INS pushes) */
int orc_nv_banded_traceback_batch(int aligner, int type, const int32_t prm[6], uint32_t band, uint32_t n,
                                  const uint32_t *pw, const uint32_t *poff, uint32_t pbits, uint32_t pbig,
                                  const uint32_t *tw, const uint32_t *toff, uint32_t tlen0, uint32_t tbits,
                                  uint32_t tbig, int32_t *scores, uint32_t *src, uint32_t *snk, uint8_t *ops,
                                  uint32_t ops_stride, uint32_t *n_ops, int n_threads) {
    if (!prm || !pw || !poff || !tw || !scores || !src || !snk || !ops || !n_ops) return -1;
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
        if (2 * M + band <= ops_stride) {
            scores[k] = orc_nv_banded_traceback_one(aligner, type, prm, band, p, M, t, N, src + 2 * k, snk + 2 * k,
                                                    ops + (size_t)k * ops_stride, n_ops + k);
        } else {
            scores[k] = INT32_MIN; n_ops[k] = 0;
            src[2 * k] = src[2 * k + 1] = snk[2 * k] = snk[2 * k + 1] = 0xFFFFFFFFu;
        }
        free(p);
        free(t);
    }
    return 0;
}
