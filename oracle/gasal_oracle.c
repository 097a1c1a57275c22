/*
 * gasal_oracle.c — CPU restatement of the GASAL2 kernels (TEST INFRASTRUCTURE).
 *
 * Not part of the product.  See gasal_oracle.h for the pinning statement.
 * All line references are to /root/reference/Non-CDP/GASAL2/src unless noted.
 *
 * Conventions shared with the reference:
 *   - bases are 4-bit codes (ASCII & 0xF), eight per uint32 word, first base
 *     in bits 31:28 (kernels/pack_rc_seqs.h:24-31);
 *   - the query is the row axis ("ridx"), the target the column axis ("gidx");
 *   - the DP runs in 8-column target strips; within a strip every padded query
 *     row is visited top to bottom and the 8 columns left to right;
 *   - the row buffer that carries (H, E) between strips is int16 (short2,
 *     local_kernel_template.h:112), arithmetic inside a strip is int32.
 */
#include "gasal_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NEG_INF16 (-32768) /* MINUS_INF = SHRT_MIN, gasal_kernels.h:35 */

typedef struct {
    int32_t a, b, o, e, oe;
    int32_t nval, has_npen, npen;
} scores_t;

static inline int32_t mx(int32_t x, int32_t y) { return x > y ? x : y; }
static inline int32_t mn(int32_t x, int32_t y) { return x < y ? x : y; }

/* 32-bit shifts with PTX shl/shr clamping (amount >= 32 gives 0). */
static inline uint32_t shl32(uint32_t x, uint32_t s) { return s >= 32 ? 0u : (x << s); }
static inline uint32_t shr32(uint32_t x, uint32_t s) { return s >= 32 ? 0u : (x >> s); }

static inline uint32_t code_at(const uint32_t *w, uint32_t pos) {
    return (w[pos >> 3] >> (28 - ((pos & 7) << 2))) & 15u;
}

/* DEV_GET_SUB_SCORE_LOCAL (gasal_kernels.h:39-51): N on either side scores 0
 * (or -N_PENALTY).  Used by local, semi-global, banded and KSW. */
static inline int32_t sub_local(const scores_t *s, uint32_t q, uint32_t t) {
    int32_t v = (q == t) ? s->a : -s->b;
    if ((int32_t)q == s->nval || (int32_t)t == s->nval) v = s->has_npen ? -s->npen : 0;
    return v;
}
/* DEV_GET_SUB_SCORE_GLOBAL (gasal_kernels.h:44-54): no N rule without N_PENALTY. */
static inline int32_t sub_global(const scores_t *s, uint32_t q, uint32_t t) {
    int32_t v = (q == t) ? s->a : -s->b;
    if (s->has_npen && ((int32_t)q == s->nval || (int32_t)t == s->nval)) v = -s->npen;
    return v;
}

/* ------------------------------------------------------------------------ */
/* Direction store: one uint32 per (strip, padded row); nibble for column m of
 * the strip at bits 31-4m..28-4m (local_kernel_template.h:53-56).  The
 * reference's uint4 tiles (2 per 8x8 tile) are exactly this word sequence
 * with linear cell index strip*8*Q8 + row*8 + col (get_tb.h:50). */
typedef struct {
    uint32_t *w;   /* [T][Q8] */
    uint32_t q8, t_strips;
} dirs_t;

static inline void dir_put(dirs_t *d, uint32_t strip, uint32_t row, uint32_t word) {
    if (d && d->w) d->w[(size_t)strip * d->q8 + row] = word;
}

/* get_tb.h:50-71 addressing; cells past the pair's padded grid read as 0
 * (the reference reads unwritten memory there). */
static inline uint32_t dir_get(const dirs_t *d, int i, int j) {
    long cell = ((long)(i >> 3) * d->q8 << 3) + ((long)j << 3) + (i & 7);
    long strip = cell / (8L * d->q8);
    long rem = cell - strip * 8L * d->q8;
    long row = rem >> 3, col = rem & 7;
    if (strip < 0 || strip >= (long)d->t_strips) return 0;
    uint32_t word = d->w[strip * d->q8 + row];
    return (word >> (28 - (col << 2))) & 15u;
}

typedef struct {
    int32_t score, qend, tend, qstart, tstart, score2, qend2, tend2;
    int wrote_ends, wrote_start, wrote_second;
} res_t;

/* ------------------------------------------------------------------------ */
/* gasal_local_kernel<LOCAL, S, B> (local_kernel_template.h:71-519).          */
static void k_local(const scores_t *sc, const uint32_t *qw, uint32_t ql,
                    const uint32_t *tw, uint32_t tl, int start_pos, int second,
                    dirs_t *dirs, res_t *o) {
    const uint32_t QR = (ql >> 3) + ((ql & 7) ? 1 : 0);
    const uint32_t TR = (tl >> 3) + ((tl & 7) ? 1 : 0);
    const uint32_t Q8 = QR * 8;
    int16_t *rowH = (int16_t *)calloc(Q8 + 8, sizeof(int16_t));
    int16_t *rowE = (int16_t *)calloc(Q8 + 8, sizeof(int16_t));
    int32_t h[9], f[9], p[9];
    int32_t maxHH = 0, maxY = 0, prevMax = 0, maxX = 0;
    int32_t max2 = 0, prev2 = 0, x2 = 0, y2 = 0;

    for (uint32_t i = 0; i < TR; i++) {
        for (int m = 0; m < 9; m++) h[m] = f[m] = p[m] = 0;   /* :123-127 */
        const int32_t gidx = (int32_t)(i << 3);
        for (uint32_t r = 0; r < Q8; r++) {
            const uint32_t qb = code_at(qw, r);
            uint32_t dword = 0;
            h[0] = rowH[r];
            int32_t e = rowE[r];
            for (int m = 1; m <= 8; m++) {
                const uint32_t tb = code_at(tw, (uint32_t)(gidx + m - 1));
                const int32_t s = sub_local(sc, qb, tb);
                const int32_t tmp = p[m] + s;                     /* CORE_LOCAL_COMPUTE :22 */
                int32_t H = mx(mx(mx(tmp, f[m]), e), 0);
                if (start_pos == ORC_WITH_TB) {                   /* CORE_LOCAL_COMPUTE_TB :49-56 */
                    const int sh = 28 - ((m - 1) << 2);
                    const uint32_t m_or_x = (tmp >= p[m]) ? 0u : 1u;
                    dword |= (H == tmp) ? (m_or_x << sh) : ((H == f[m]) ? (3u << sh) : (2u << sh));
                    dword |= ((tmp - sc->oe) > (f[m] - sc->e)) ? 0u : (1u << (sh + 3));
                    dword |= ((tmp - sc->oe) > (e - sc->e)) ? 0u : (1u << (sh + 2));
                }
                f[m] = mx(tmp - sc->oe, f[m] - sc->e);
                e = mx(tmp - sc->oe, e - sc->e);
                if (maxHH < H) { maxY = gidx + m - 1; maxHH = H; }  /* :28-29 */
                if (second) {                                        /* :145-150 */
                    if (max2 < H && maxHH > H) { y2 = gidx + m - 1; max2 = H; }
                }
                h[m] = H;
                p[m] = h[m - 1];
            }
            rowH[r] = (int16_t)h[8];
            rowE[r] = (int16_t)e;
            if (start_pos == ORC_WITH_TB) dir_put(dirs, i, r, dword);
            maxX = (prevMax < maxHH) ? (int32_t)r : maxX;            /* :412 */
            if (second) {                                            /* :414-418 */
                x2 = (prev2 < maxHH) ? (int32_t)r : x2;
                prev2 = mx(max2, prev2);
            }
            prevMax = mx(maxHH, prevMax);
        }
    }
    o->score = maxHH; o->qend = maxX; o->tend = maxY; o->wrote_ends = 1;   /* :428-430 */
    if (second) { o->score2 = max2; o->qend2 = x2; o->tend2 = y2; o->wrote_second = 1; }

    if (start_pos == ORC_WITH_START) {                                /* :441-511 */
        const int32_t fwd = maxHH;
        const int32_t rend_reg = mn((maxX >> 3) + 1, (int32_t)QR);
        const int32_t gend_reg = mn((maxY >> 3) + 1, (int32_t)TR);
        const int32_t qbase = rend_reg - 1, tbase = gend_reg - 1;   /* word indices */
        int32_t mH = 0, pM = 0, sx = 0, sy = 0;
        memset(rowH, 0, (Q8 + 8) * sizeof(int16_t));
        memset(rowE, 0, (Q8 + 8) * sizeof(int16_t));
        int32_t gidx = (gend_reg << 3) + 8 - 1;
        for (int32_t i = 0; i < gend_reg && mH < fwd; i++) {
            for (int m = 0; m < 9; m++) h[m] = f[m] = p[m] = 0;
            const uint32_t gpac = tw[tbase - i];
            gidx -= 8;
            int32_t ridx = (rend_reg << 3) - 1;
            int32_t gi = 0;
            for (int32_t j = 0; j < rend_reg && mH < fwd; j++) {
                const uint32_t rpac = qw[qbase - j];
                for (int k = 0; k <= 28 && mH < fwd; k += 4) {
                    const uint32_t qb = (rpac >> k) & 15u;
                    h[0] = rowH[gi];
                    int32_t e = rowE[gi];
                    for (int l = 0, m = 1; l <= 28; l += 4, m++) {   /* CORE_LOCAL_COMPUTE_START */
                        const uint32_t tb = (gpac >> l) & 15u;
                        const int32_t s = sub_local(sc, qb, tb);
                        const int32_t tmp = p[m] + s;
                        const int32_t H = mx(mx(mx(tmp, f[m]), e), 0);
                        f[m] = mx(tmp - sc->oe, f[m] - sc->e);
                        e = mx(tmp - sc->oe, e - sc->e);
                        if (mH < H) { sy = gidx + (m - 1); mH = H; }   /* Q8 */
                        h[m] = H;
                        p[m] = h[m - 1];
                    }
                    rowH[gi] = (int16_t)h[8];
                    rowE[gi] = (int16_t)e;
                    sx = (pM < mH) ? ridx : sx;
                    pM = mx(mH, pM);
                    ridx--; gi++;
                }
            }
        }
        o->qstart = sx; o->tstart = sy; o->wrote_start = 1;
    }
    free(rowH); free(rowE);
}

/* ------------------------------------------------------------------------ */
/* gasal_global_kernel<S> (kernels/global.h:30-303).                         */
static void k_global(const scores_t *sc, const uint32_t *qw, uint32_t ql,
                     const uint32_t *tw, uint32_t tl, int start_pos, dirs_t *dirs, res_t *o) {
    const uint32_t QR = (ql >> 3) + ((ql & 7) ? 1 : 0);
    const uint32_t TR = (tl >> 3) + ((tl & 7) ? 1 : 0);
    const uint32_t Q8 = QR * 8;
    int16_t *rowH = (int16_t *)malloc((Q8 + 8) * sizeof(int16_t));
    int16_t *rowE = (int16_t *)malloc((Q8 + 8) * sizeof(int16_t));
    int32_t h[9], f[9], p[9], max_h[9];
    for (int m = 0; m < 9; m++) max_h[m] = 0;
    rowH[0] = 0; rowE[0] = NEG_INF16;                                  /* :57-60 (Q2) */
    for (uint32_t r = 1; r < Q8 + 8; r++) {
        rowH[r] = (int16_t)(-(sc->o + sc->e * (int32_t)r));
        rowE[r] = NEG_INF16;
    }
    int32_t u = 1, rr = 1;                                             /* :63-64 */
    h[0] = 0; p[0] = 0;
    for (uint32_t i = 0; i < TR; i++) {
        for (int m = 1; m < 9; m++, u++, rr++) {                       /* :67-71 */
            h[m] = -(sc->o + sc->e * u);
            f[m] = NEG_INF16;
            p[m] = (rr == 1) ? 0 : -(sc->o + sc->e * (rr - 1));
        }
        for (uint32_t r = 0; r < Q8; r++) {
            const uint32_t qb = code_at(qw, r);
            uint32_t dword = 0;
            h[0] = rowH[r];
            int32_t e = rowE[r];
            for (int m = 1; m <= 8; m++) {
                const uint32_t tb = code_at(tw, (i << 3) + (uint32_t)m - 1);
                const int32_t s = sub_global(sc, qb, tb);
                const int32_t tmp = p[m] + s;                        /* CORE_GLOBAL_COMPUTE :7-12 */
                const int32_t H = mx(mx(tmp, f[m]), e);
                if (start_pos == ORC_WITH_TB) {                      /* :18-25 */
                    const int sh = 28 - ((m - 1) << 2);
                    const uint32_t m_or_x = (tmp >= p[m]) ? 0u : 1u;
                    dword |= (H == tmp) ? (m_or_x << sh) : ((H == f[m]) ? (3u << sh) : (2u << sh));
                    dword |= ((tmp - sc->oe) > (f[m] - sc->e)) ? 0u : (1u << (sh + 3));
                    dword |= ((tmp - sc->oe) > (e - sc->e)) ? 0u : (1u << (sh + 2));
                }
                f[m] = mx(tmp - sc->oe, f[m] - sc->e);
                e = mx(tmp - sc->oe, e - sc->e);
                h[m] = H;
                p[m] = h[m - 1];
            }
            rowH[r] = (int16_t)h[8];
            rowE[r] = (int16_t)e;
            if (start_pos == ORC_WITH_TB) dir_put(dirs, i, r, dword);
            if (r + 1 == ql)                                          /* :98-103 */
                for (int m = 1; m < 9; m++) max_h[m] = h[m];
        }
    }
    o->score = max_h[8 - ((TR << 3) - tl)];                            /* :299 */
    free(rowH); free(rowE);
}

/* ------------------------------------------------------------------------ */
/* gasal_semi_global_kernel<T,S,B,HEAD,TAIL> (semiglobal_kernel_template.h:39-388). */
static inline int head_frees_query(int head) { return head == ORC_QUERY || head == ORC_BOTH; }
static inline int head_frees_target(int head) { return head == ORC_TARGET || head == ORC_BOTH; }
static inline int tail_target(int tail) { return tail == ORC_TARGET || tail == ORC_BOTH; }
static inline int tail_query(int tail) { return tail == ORC_QUERY || tail == ORC_BOTH; }

static void semi_init_rows(const scores_t *sc, int head, int16_t *rowH, int16_t *rowE, uint32_t n) {
    if (head_frees_query(head)) {                                       /* :87-92 */
        for (uint32_t r = 0; r < n; r++) { rowH[r] = 0; rowE[r] = 0; }
    } else {                                                            /* :94-98 */
        rowH[0] = 0; rowE[0] = NEG_INF16;
        for (uint32_t r = 1; r < n; r++) {
            rowH[r] = (int16_t)(-(sc->o + sc->e * (int32_t)r));
            rowE[r] = NEG_INF16;
        }
    }
}

/* One pass of the semi-global DP over strips [i0, TR) of the packed words
 * qwords/twords (forward pass: the real batch; reverse pass: the reversed
 * copies).  early_stop: stop once maxHH >= fwd (WITH_START, :301,323). */
static void semi_pass(const scores_t *sc, int head, int tail, int second,
                      const uint32_t *qwords, uint32_t QR, uint32_t ql,
                      const uint32_t *twords, uint32_t TR, uint32_t tl, int32_t i0,
                      int16_t *rowH, int16_t *rowE, int early_stop, int32_t fwd,
                      int32_t *maxHH, int32_t *maxY, int32_t *max2, int32_t *y2) {
    int32_t h[9], f[9], p[9];
    int32_t u = 0, rr = 0;
    if (head == ORC_QUERY || head == ORC_NONE) {                        /* :101-107 */
        u = 0; rr = 0; h[u++] = 0; p[rr++] = 0;
    } else {
        h[0] = 0; p[0] = 0;
    }
    for (int32_t i = i0; i < (int32_t)TR && (!early_stop || *maxHH < fwd); i++) {
        const int32_t gidx = i << 3;
        if (head_frees_target(head)) {                                  /* :114-121 */
            for (int m = 0; m < 9; m++) { h[m] = 0; f[m] = NEG_INF16; p[m] = 0; }
        } else {                                                        /* :123-128 (Q3) */
            for (int m = 1; m < 9; m++, u++, rr++) {
                h[m] = -(sc->o + sc->e * (u - 1));
                f[m] = NEG_INF16;
                p[m] = (rr == 1) ? 0 : -(sc->o + sc->e * (rr - 1));
            }
        }
        /* the WITH_START pass can start at a negative strip (gend_reg < 0 when the
         * end row lies past the target, :273); the reference then reads its
         * reverse_target_batch[] out of bounds.  Defined here as zero words. */
        const uint32_t gpac = i >= 0 ? twords[i] : 0u;
        uint32_t ridx = 0;
        for (uint32_t j = 0; j < QR && (!early_stop || *maxHH < fwd); j++) {
            const uint32_t rpac = qwords[j];
            for (int k = 28; k >= 0; k -= 4) {
                const uint32_t qb = (rpac >> k) & 15u;
                h[0] = rowH[ridx];
                int32_t e = rowE[ridx];
                int32_t prev = h[0] - sc->oe;
                for (int l = 28, m = 1; m < 9; l -= 4, m++) {           /* CORE_COMPUTE_SEMIGLOBAL :17-28 */
                    const uint32_t tb = (gpac >> l) & 15u;
                    const int32_t s = sub_local(sc, qb, tb);
                    int32_t curr = h[m] - sc->oe;
                    f[m] = mx(curr, f[m] - sc->e);
                    curr = p[m] + s;
                    curr = mx(curr, f[m]);
                    e = mx(prev, e - sc->e);
                    curr = mx(curr, e);
                    h[m] = curr;
                    p[m] = prev + sc->oe;
                    prev = curr - sc->oe;
                }
                rowH[ridx] = (int16_t)h[8];
                rowE[ridx] = (int16_t)e;
                ridx++;
                if (tail_target(tail) && ridx == ql) {                  /* :160-178 */
                    for (int m = 1; m < 9; m++) {
                        const int32_t col = gidx + m - 1;
                        if (h[m] > *maxHH && col < (int32_t)tl) { *maxY = col; *maxHH = h[m]; }
                        if (second) {
                            if (h[m] > *max2 && h[m] < *maxHH && col < (int32_t)tl) { *y2 = col; *max2 = h[m]; }
                        }
                    }
                }
            }
        }
    }
}

static void k_semiglobal(const scores_t *sc, int head, int tail, int second, int start_pos,
                         uint32_t maxq, const uint32_t *qw, uint32_t ql,
                         const uint32_t *tw, uint32_t tl, res_t *o) {
    const uint32_t QR = (ql >> 3) + ((ql & 7) ? 1 : 0);
    const uint32_t TR = (tl >> 3) + ((tl & 7) ? 1 : 0);
    uint32_t nrow = maxq;                      /* the reference buffer spans MAX_QUERY_LEN rows */
    if (nrow < QR * 8 + 8) nrow = QR * 8 + 8;
    int16_t *rowH = (int16_t *)malloc(nrow * sizeof(int16_t));
    int16_t *rowE = (int16_t *)malloc(nrow * sizeof(int16_t));
    int32_t maxHH = NEG_INF16, maxX = (int32_t)tl, maxY = (int32_t)ql;  /* :49,63-64 */
    int32_t max2 = NEG_INF16, x2 = (int32_t)tl, y2 = (int32_t)ql;       /* :71-74 */
    semi_init_rows(sc, head, rowH, rowE, nrow);
    semi_pass(sc, head, tail, second, qw, QR, ql, tw, TR, tl, 0, rowH, rowE, 0, 0,
              &maxHH, &maxY, &max2, &y2);
    if (tail_query(tail)) {                                             /* :185-214 */
        for (uint32_t m = 0; m < maxq; m++) {
            const int32_t v = rowH[m];
            if (v > maxHH && m < ql) { maxX = (int32_t)m; maxHH = v; }
            if (second) {
                if (v > max2 && v < maxHH && m < tl) { x2 = (int32_t)m; max2 = v; }   /* Q12 */
            }
        }
        if (maxX != (int32_t)tl) maxY = (int32_t)ql;
        if (second && x2 != (int32_t)tl) y2 = (int32_t)ql;
    }
    o->score = maxHH; o->tend = maxY; o->qend = maxX; o->wrote_ends = 1;   /* :216-218 */
    if (second) { o->score2 = max2; o->tend2 = y2; o->qend2 = x2; o->wrote_second = 1; }

    if (start_pos == ORC_WITH_START) {                                  /* :227-383 */
        const uint32_t nw = maxq >> 3;
        uint32_t *rq = (uint32_t *)calloc(nw + QR + TR + 2, sizeof(uint32_t));
        uint32_t *rt = (uint32_t *)calloc(nw + QR + TR + 2, sizeof(uint32_t));
        for (int32_t i = (int32_t)ql - 1, k = 0; i >= 0; i--, k++) {    /* :245-253 */
            const uint32_t sym = code_at(qw, (uint32_t)i);
            rq[k >> 3] |= sym << (28 - ((k & 7) << 2));
        }
        for (int32_t i = (int32_t)tl - 1, k = 0; i >= 0; i--, k++) {    /* :258-266 */
            const uint32_t sym = code_at(tw, (uint32_t)i);
            rt[k >> 3] |= sym << (28 - ((k & 7) << 2));
        }
        const int32_t gend_pos = maxY, fwd = maxHH;
        const int32_t d = (int32_t)TR - ((gend_pos >> 3) + 1);          /* :273 */
        const int32_t gend_reg = d > 0 ? d - 1 : d;
        int32_t rmax = NEG_INF16, ry = 0, dummy2 = 0, dummyy = 0;
        semi_init_rows(sc, head, rowH, rowE, nrow);
        semi_pass(sc, head, tail, 0, rq, QR, ql, rt, TR, tl, gend_reg, rowH, rowE, 1, fwd,
                  &rmax, &ry, &dummy2, &dummyy);
        if (tail_query(tail)) {                                         /* :362-378 */
            for (uint32_t m = 0; m < maxq; m++) {
                const int32_t v = rowH[m];
                if (v > rmax && m < ql) { maxX = (int32_t)m; rmax = v; }
            }
            if (maxX != (int32_t)tl) ry = (int32_t)ql;
        }
        o->tstart = ((int32_t)tl - 1) - ry;                             /* :380-381 */
        o->qstart = ((int32_t)ql - 1) - maxX;
        o->wrote_start = 1;
        free(rq); free(rt);
    }
    free(rowH); free(rowE);
}

/* ------------------------------------------------------------------------ */
/* gasal_banded_tiled_kernel (kernels/banded.h:10-139).                        */
static void k_banded(const scores_t *sc, int32_t kbw, const uint32_t *qw, uint32_t ql,
                     const uint32_t *tw, uint32_t tl, res_t *o) {
    const int32_t QR = (int32_t)((ql >> 3) + ((ql & 7) ? 1 : 0));
    const int32_t TR = (int32_t)((tl >> 3) + ((tl & 7) ? 1 : 0));
    int16_t *rowH = (int16_t *)calloc((size_t)QR * 8 + 8, sizeof(int16_t));
    int16_t *rowE = (int16_t *)calloc((size_t)QR * 8 + 8, sizeof(int16_t));
    int32_t h[9], f[9], p[9];
    int32_t maxHH = 0, prevMax = 0, maxX = 0, maxY = 0;
    const int32_t kother = TR - (QR - kbw);                             /* :35 */
    for (int32_t i = 0; i < TR; i++) {
        for (int m = 0; m < 9; m++) h[m] = f[m] = p[m] = 0;
        const int32_t gidx = i << 3;
        int32_t ridx = mx(0, i - kother + 1) << 3;                     /* :83-85 */
        const int32_t last_tile = mn(kbw + i, QR);
        for (int32_t j = ridx >> 3; j < last_tile; j++) {
            const uint32_t rpac = qw[j];
            for (int k = 28; k >= 0; k -= 4) {
                const uint32_t qb = (rpac >> k) & 15u;
                h[0] = rowH[ridx];
                int32_t e = rowE[ridx];
                for (int l = 28, m = 1; m < 9; l -= 4, m++) {          /* :100-115 */
                    const uint32_t tb = (tw[i] >> l) & 15u;
                    const int32_t s = sub_local(sc, qb, tb);
                    f[m] = mx(h[m] - sc->oe, f[m] - sc->e);
                    h[m] = p[m] + s;
                    h[m] = mx(h[m], f[m]);
                    h[m] = mx(h[m], 0);
                    e = mx(h[m - 1] - sc->oe, e - sc->e);
                    h[m] = mx(h[m], e);
                    if (maxHH < h[m]) { maxY = gidx + (m - 1); maxHH = h[m]; }   /* FIND_MAX */
                    p[m] = h[m - 1];
                }
                rowH[ridx] = (int16_t)h[8];
                rowE[ridx] = (int16_t)e;
                maxX = (prevMax < maxHH) ? ridx : maxX;
                prevMax = mx(maxHH, prevMax);
                ridx++;
            }
        }
    }
    o->score = maxHH; o->qend = maxX; o->tend = maxY; o->wrote_ends = 1;
    free(rowH); free(rowE);
}

/* ------------------------------------------------------------------------ */
/* gasal_ksw_kernel<B> (kernels/ksw_kernel_template.h:46-199): BWA ksw_extend
 * with zdrop = 0, no band, PEN_CLIP5 = 5. */
static void k_ksw(const scores_t *sc, uint32_t h0u, const uint32_t *qw, uint32_t qlen,
                  const uint32_t *tw, uint32_t tlen, res_t *o) {
    const uint32_t QR = (qlen >> 3) + 1, TR = (tlen >> 3) + 1;         /* :56-57 (Q16) */
    const int o_del = sc->o, o_ins = sc->o, e_del = sc->e, e_ins = sc->e;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const int zdrop = 0;
    const int nq = (int)qlen + 2 > 8 ? (int)qlen + 2 : 8;
    int32_t *eh_h = (int32_t *)calloc((size_t)nq + 8, sizeof(int32_t));
    int32_t *eh_e = (int32_t *)calloc((size_t)nq + 8, sizeof(int32_t));
    eh_h[0] = (int32_t)h0u;                                             /* :78-81 */
    eh_h[1] = (h0u > (uint32_t)oe_ins) ? (int32_t)(h0u - (uint32_t)oe_ins) : 0;
    for (int j = 2; j <= (int)qlen && eh_h[j - 1] > e_ins; ++j) eh_h[j] = eh_h[j - 1] - e_ins;
    int max = (int32_t)h0u, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = (int)qlen;
    int j = 0;
    for (uint32_t tt = 0; tt < TR; tt++) {
        const uint32_t gpac = tw[tt];
        for (uint32_t tb_id = 0; tb_id < 8; tb_id++) {
            const int i = (int)(tt * 8 + tb_id);
            if (i >= (int)tlen) break;
            const uint32_t gbase = (gpac >> (32 - (tb_id + 1) * 4)) & 0x0F;
            int t, f = 0, h1, m = 0, mj = -1;
            if (beg == 0) {
                h1 = (int32_t)(h0u - (uint32_t)(o_del + e_del * (i + 1)));
                if (h1 < 0) h1 = 0;
            } else h1 = 0;
            for (uint32_t qt = 0; qt < QR; qt++) {
                const uint32_t rpac = qw[qt];
                int brk = 0;
                for (uint32_t qb_id = 0; qb_id < 8; qb_id++) {
                    j = (int)(qt * 8 + qb_id);
                    if (j < beg) continue;
                    if (j >= end) { brk = 1; break; }
                    const uint32_t rbase = (rpac >> (32 - (qb_id + 1) * 4)) & 0x0F;
                    int h, M = eh_h[j], e = eh_e[j];
                    eh_h[j] = h1;
                    const int32_t s = sub_local(sc, rbase, gbase);
                    M = M ? M + s : 0;
                    h = M > e ? M : e;
                    h = h > f ? h : f;
                    h1 = h;
                    mj = m > h ? mj : j;
                    m = m > h ? m : h;
                    t = M - oe_del; t = t > 0 ? t : 0;
                    e -= e_del; e = e > t ? e : t;
                    eh_e[j] = e;
                    t = M - oe_ins; t = t > 0 ? t : 0;
                    f -= e_ins; f = f > t ? f : t;
                }
                (void)brk;
            }
            eh_h[end] = h1; eh_e[end] = 0;                              /* :153-154 */
            if (j == (int)qlen) {
                max_ie = gscore > h1 ? max_ie : i;
                gscore = gscore > h1 ? gscore : h1;
            }
            if (m == 0) break;   /* leaves this 8-column tile only (:159-160) */
            if (m > max) {
                max = m; max_i = i; max_j = mj;
                max_off = max_off > abs(mj - i) ? max_off : abs(mj - i);
            } else if (zdrop > 0) {
                /* zdrop is 0 in the reference (:62); branch never taken */
            }
            for (j = beg; (j < end) && eh_h[j] == 0 && eh_e[j] == 0; ++j) ;
            beg = j;
            for (j = end; (j >= beg) && eh_h[j] == 0 && eh_e[j] == 0; --j) ;
            end = j + 2 < (int)qlen ? j + 2 : (int)qlen;
        }
    }
    (void)max_off;
    if (gscore <= 0 || gscore <= max - 5) {                             /* :188-197 */
        o->score = max; o->qend = max_j + 1; o->tend = max_i + 1;
    } else {
        o->score = gscore; o->qend = (int32_t)qlen; o->tend = max_ie + 1;
    }
    o->wrote_ends = 1;
    free(eh_h); free(eh_e);
}

/* ------------------------------------------------------------------------ */
/* gasal_get_tb<T> (kernels/get_tb.h:4-149). Writes the reversed RLE bytes at
 * cigar[0..] and returns n_ops; for LOCAL also the start coordinates. */
static uint32_t k_get_tb(const scores_t *sc, int is_local, const dirs_t *d,
                         uint32_t ql, uint32_t tl, res_t *o, uint8_t *cigar) {
    int i, j;
    int total = 0, curr = 0;
    if (is_local) { i = o->tend; j = o->qend; total = o->score; curr = 0; }
    else { i = (int)tl; j = (int)ql; }
    uint32_t prev = 0, opf = 0;
    int n_ops = 0, off = 0, count = 0;
    int op_select = 3, op_shift = 0;
    while (i >= 0 && j >= 0) {
        const uint32_t cell_op = dir_get(d, i, j);
        const uint32_t op = (cell_op >> op_shift) & (uint32_t)op_select;
        opf = (op == 0 || op_select == 3) ? op : (uint32_t)op_shift;            /* :78 */
        op_select = (op == 0 || (op == 1 && op_select == 3)) ? 3 : 1;            /* :80 */
        op_shift = (op == 0 || (op == 1 && op_select == 3)) ? 0 :                /* :82 (new op_select) */
                   ((op == 2 || op == 3) ? (int)op : op_shift);
        if (count < 63 && opf == prev) {
            count++;
        } else {
            if (count > 0) { cigar[off++] = (uint8_t)(prev | (uint32_t)(count << 2)); n_ops++; }
            count = 1;
        }
        if (is_local) {                                                           /* :100-103 */
            curr += ((opf == 2 || opf == 3) && prev != opf) ? -sc->oe
                  : ((opf == 2 || opf == 3) ? -sc->e : (opf == 1 ? -sc->b : sc->a));
            if (curr == total) break;
        }
        prev = opf;
        i = (opf == 0 || opf == 1 || opf == 2) ? i - 1 : i;
        j = (opf == 0 || opf == 1 || opf == 3) ? j - 1 : j;
    }
    cigar[off++] = (uint8_t)(prev | (uint32_t)(count << 2));                     /* :113-117 */
    n_ops++;
    if (!is_local) {                                                              /* :119-139 */
        while (i >= 0) {
            const uint8_t rc = (uint8_t)((i + 1) <= 63 ? (i + 1) : 63);
            cigar[off++] = (uint8_t)(2u | (uint32_t)(rc << 2)); n_ops++; i -= 63;
        }
        while (j >= 0) {
            const uint8_t rc = (uint8_t)((j + 1) <= 63 ? (j + 1) : 63);
            cigar[off++] = (uint8_t)(3u | (uint32_t)(rc << 2)); n_ops++; j -= 63;
        }
    } else {
        o->tstart = i; o->qstart = j; o->wrote_start = 1;                        /* :142-145 */
    }
    return (uint32_t)n_ops;
}

/* ------------------------------------------------------------------------ */
void orc_pack(const uint8_t *bytes, uint32_t n_bytes, uint32_t *words) {
    for (uint32_t w = 0; w < n_bytes / 8; w++) {
        uint32_t v = 0;
        for (int k = 0; k < 8; k++) v |= ((uint32_t)bytes[w * 8 + k] & 15u) << (28 - 4 * k);
        words[w] = v;
    }
}

static uint32_t nib_reverse(uint32_t x) {
    uint32_t r = 0;
    for (int k = 28; k >= 0; k -= 4) r |= ((x >> k) & 15u) << (28 - k);
    return r;
}

void orc_revcomp_one(uint32_t *W, uint32_t base, uint32_t len, uint8_t op, int32_t n_code) {
    const uint32_t regs = (len >> 3) + ((len & 7) ? 1 : 0);
    const uint32_t swaps = (regs >> 1) + (regs & 1);
#define RD(idx) ((long)(base) + (long)(idx) >= 0 ? W[(long)(base) + (long)(idx)] : 0u)
    if (regs == 0) return;
    if (op & 1) {                                                        /* :109-167 */
        uint32_t nbr = 0;
        const uint32_t last = W[base + regs - 1];
        for (int jj = 0; jj < 32; jj += 4) nbr += ((int32_t)((last >> jj) & 15u) == n_code);
        nbr <<= 2;
        const uint32_t lowmask = shl32(1u, nbr) - 1u;
        for (uint32_t i = 0; i < swaps; i++) {
            const long a = (long)regs - 2 - (long)i, b = (long)regs - 1 - (long)i;
            const uint32_t r1 = W[base + i];
            const uint32_t r2 = shl32(RD(a), 32 - nbr) | shr32(RD(b), nbr);
            const uint32_t rv1 = nib_reverse(r1), rv2 = nib_reverse(r2);
            const uint32_t q1 = shl32(rv1, nbr) | (RD(b) & lowmask);
            const uint32_t q2 = (RD(a) & (0xFFFFFFFFu - lowmask)) | shr32(rv1, 32 - nbr);
            W[base + i] = rv2;
            W[base + b] = q1;
            if (i != swaps - 1 && (long)base + a >= 0) W[base + a] = q2;
        }
    }
    if (op & 2) {                                                        /* :169-205 */
        for (uint32_t i = 0; i < regs; i++) {
            uint32_t rp = W[base + i];
            for (int k = 28; k >= 0; k -= 4) {
                uint32_t nt = (rp >> k) & 15u;
                switch (nt) {
                    case 1: nt = 4; break;   /* A -> T */
                    case 3: nt = 7; break;   /* C -> G */
                    case 4: nt = 1; break;   /* T -> A */
                    case 7: nt = 3; break;   /* G -> C */
                    default: break;
                }
                rp = (rp & ~(15u << k)) | (nt << k);
            }
            W[base + i] = rp;
        }
    }
#undef RD
}

/* ------------------------------------------------------------------------ */
int orc_aln_batch(const orc_params *P,
                  const uint8_t *q_batch, const uint32_t *q_offsets, const uint32_t *q_lens,
                  const uint8_t *t_batch, const uint32_t *t_offsets, const uint32_t *t_lens,
                  uint32_t q_bytes, uint32_t t_bytes, uint32_t n,
                  const uint8_t *q_ops, const uint8_t *t_ops, const uint32_t *seed,
                  int32_t *score, int32_t *qend, int32_t *tend, int32_t *qstart, int32_t *tstart,
                  int32_t *score2, int32_t *qend2, int32_t *tend2,
                  uint8_t *cigar, uint32_t *n_ops, int n_threads) {
    if (!P || n == 0 || q_bytes == 0 || t_bytes == 0) return -1;        /* gasal_align.cu:32-43 */
    if ((q_bytes & 7) || (t_bytes & 7)) return -2;                      /* :45-52 */
    scores_t sc;
    sc.a = P->match; sc.b = P->mismatch; sc.o = P->gap_open; sc.e = P->gap_extend;
    sc.oe = P->gap_open + P->gap_extend;                                /* :334 */
    sc.nval = P->n_code & 0xF; sc.has_npen = P->has_n_penalty; sc.npen = P->n_penalty;

    /* device-side packed copies */
    uint32_t *qw = (uint32_t *)malloc(q_bytes / 8 * sizeof(uint32_t) + 16);
    uint32_t *tw = (uint32_t *)malloc(t_bytes / 8 * sizeof(uint32_t) + 16);
    uint8_t *unpacked_q = (uint8_t *)malloc(q_bytes);
    memcpy(unpacked_q, q_batch, q_bytes);
    if (P->is_packed) {
        /* packed_*_batch aliases the unpacked buffer (ctors.cpp:64-68) */
        memcpy(qw, q_batch, q_bytes / 8 * sizeof(uint32_t));
        memcpy(tw, t_batch, t_bytes / 8 * sizeof(uint32_t));
    } else {
        orc_pack(q_batch, q_bytes, qw);
        orc_pack(t_batch, t_bytes, tw);
    }
    if (q_ops && t_ops) {                                               /* :232-246 */
        for (uint32_t k = 0; k < n; k++) {
            if (q_ops[k] == 0 && t_ops[k] == 0) continue;
            orc_revcomp_one(qw, q_offsets[k] >> 3, q_lens[k], q_ops[k], P->n_code);
            orc_revcomp_one(tw, t_offsets[k] >> 3, t_lens[k], t_ops[k], P->n_code);
        }
        if (P->is_packed) {
            memcpy(unpacked_q, qw, q_bytes / 8 * sizeof(uint32_t));
        }
    }
    const int tb = (P->start_pos == ORC_WITH_TB);
    if (tb && cigar) memcpy(cigar, unpacked_q, q_bytes);
    const int algo = P->algo;
    const uint32_t maxq = P->max_query_len > 0 ? (uint32_t)P->max_query_len : 0;
    int rc = 0;

#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(n_threads)
#endif
    for (long kk = 0; kk < (long)n; kk++) {
        const uint32_t k = (uint32_t)kk;
        const uint32_t ql = q_lens[k], tl = t_lens[k];
        const uint32_t *qk = qw + (q_offsets[k] >> 3);
        const uint32_t *tk = tw + (t_offsets[k] >> 3);
        res_t r;
        memset(&r, 0, sizeof(r));
        dirs_t dirs = {0, 0, 0};
        const uint32_t QR = (ql >> 3) + ((ql & 7) ? 1 : 0);
        const uint32_t TR = (tl >> 3) + ((tl & 7) ? 1 : 0);
        if (tb && (algo == ORC_LOCAL || algo == ORC_GLOBAL)) {
            dirs.q8 = QR * 8; dirs.t_strips = TR;
            dirs.w = (uint32_t *)calloc((size_t)TR * QR * 8 + 1, sizeof(uint32_t));
        }
        switch (algo) {
            case ORC_LOCAL:
                k_local(&sc, qk, ql, tk, tl, P->start_pos, P->second_best, &dirs, &r);
                break;
            case ORC_GLOBAL:
                k_global(&sc, qk, ql, tk, tl, P->start_pos, &dirs, &r);
                break;
            case ORC_SEMI_GLOBAL: {
                uint32_t mq = maxq ? maxq : (QR * 8 > TR * 8 ? QR * 8 : TR * 8);
                k_semiglobal(&sc, P->head, P->tail, P->second_best, P->start_pos, mq, qk, ql, tk, tl, &r);
                break;
            }
            case ORC_BANDED:
                k_banded(&sc, P->k_band >> 3, qk, ql, tk, tl, &r);
                break;
            case ORC_KSW:
                k_ksw(&sc, seed ? seed[k] : 0u, qk, ql, tk, tl, &r);
                break;
            default:
                break;   /* UNKNOWN / MICROLOCAL: nothing launched (gasal_align.cu:20-21) */
        }
        if (tb && (algo == ORC_LOCAL || algo == ORC_GLOBAL) && cigar) {
            const uint32_t nops = k_get_tb(&sc, algo == ORC_LOCAL, &dirs, ql, tl, &r,
                                           cigar + q_offsets[k]);
            if (n_ops) n_ops[k] = nops;
        } else if (tb && n_ops) {
            n_ops[k] = ql;   /* device query_batch_lens copied back as n_cigar_ops (gasal_align.cu:282) */
        }
        free(dirs.w);
        if (score && algo != ORC_UNKNOWN && algo != ORC_MICROLOCAL) score[k] = r.score;
        if (r.wrote_ends && algo != ORC_GLOBAL) {
            if (qend) qend[k] = r.qend;
            if (tend) tend[k] = r.tend;
        }
        if (r.wrote_start && algo != ORC_GLOBAL) {
            if (qstart) qstart[k] = r.qstart;
            if (tstart) tstart[k] = r.tstart;
        }
        if (r.wrote_second) {
            if (score2) score2[k] = r.score2;
            if (qend2) qend2[k] = r.qend2;
            if (tend2) tend2[k] = r.tend2;
        }
    }
    free(qw); free(tw); free(unpacked_q);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* PairHMM (inter_task/Synthetic_data/tile_1/tile_1.cu).                       */
void orc_pairhmm_params(const uint8_t *bq, const uint8_t *iq, const uint8_t *dq, uint32_t n,
                        float *qm, float *delta, float *xiksi, float *alpha) {
    float ph2pr[128];
    for (int i = 0; i < 128; i++) ph2pr[i] = powf(10.f, -((float)i) / 10.f);   /* tile_1.cu:216-220 */
    for (uint32_t k = 0; k < n; k++) {                                         /* :415-419 */
        qm[k] = ph2pr[bq[k] & 127];
        delta[k] = ph2pr[iq[k] & 127];
        xiksi[k] = ph2pr[dq[k] & 127];
        alpha[k] = 1.0f - ph2pr[((int)(iq[k] & 127) + (int)(dq[k] & 127)) & 127];
    }
}

static float pairhmm_one(const uint8_t *rd, uint32_t R, const float *qm, const float *delta,
                         const float *xiksi, const float *alpha, const uint8_t *hp, uint32_t H,
                         float *MG, float *IG, float *DG) {
    const float c0 = 1.329228e+36f, c3 = 0.9f, c4 = 0.1f;                      /* :228-233 */
    float result = 0.0f;                                                       /* constant[5] */
    for (uint32_t i = 0; i < R; i++) {
        const float Qm0 = qm[i];
        const float d = delta[i], x = xiksi[i], al = alpha[i];
        const float Qm_1 = 1.0f - Qm0;                                         /* :101 */
        const float Qm = Qm0 / 3.0f;                                           /* fdividef, :104 */
        float Ml = 0, Dl = 0, Il = 0, MU = 0, IU = 0, DU = 0, MMID = 0;
        if (i == 0) {                                                          /* :114-118 */
            DU = c0 / (float)H;
            MMID = c3 * DU;
        }
        for (uint32_t j = 0; j < H; j++) {
            if (i > 0) { MU = MG[j]; IU = IG[j]; DU = DG[j]; }
            const float MID = IU + DU;                                         /* :149-162 */
            const float DDM = Ml * x;
            const float IIMI = IU * c4;
            const float aa = (hp[j] == rd[i]) ? Qm_1 : Qm;
            const float MIIDD = c3 * MID;
            Ml = aa * MMID;
            Il = fmaf(MU, d, IIMI);
            Dl = fmaf(Dl, c4, DDM);
            MMID = fmaf(al, MU, MIIDD);
            if (i < R - 1) { MG[j] = Ml; IG[j] = Il; DG[j] = Dl; }
            else result = result + (Ml + Il);
        }
    }
    return result;
}

int orc_pairhmm_batch(uint32_t n, const uint8_t *reads, const uint32_t *read_off, const uint32_t *read_len,
                      const float *qm, const float *delta, const float *xiksi, const float *alpha,
                      const uint8_t *haps, const uint32_t *hap_off, const uint32_t *hap_len,
                      float *result, int n_threads) {
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel num_threads(n_threads)
#endif
    {
        uint32_t cap = 0;
        float *buf = NULL;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (long kk = 0; kk < (long)n; kk++) {
            const uint32_t k = (uint32_t)kk;
            const uint32_t H = hap_len[k];
            if (H > cap) { free(buf); cap = H; buf = (float *)malloc(3 * (size_t)cap * sizeof(float)); }
            const uint32_t ro = read_off[k];
            result[k] = pairhmm_one(reads + ro, read_len[k], qm + ro, delta + ro, xiksi + ro, alpha + ro,
                                    haps + hap_off[k], H, buf, buf + cap, buf + 2 * cap);
        }
        free(buf);
    }
    return 0;
}
