// capi.cpp — extern "C" flat API (include/gasalx.h) over the engine.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "engine.hpp"
#include "gasalx.h"

// One stage of the host-staged pipeline (gasalx_align_host on large batches):
// its own stream, workspace and device copies of one chunk of pairs.
struct HostSlot {
    hipStream_t st = nullptr;
    gx::Workspace ws;
    gx::DevBuf q, t, meta, cig;
    std::vector<uint8_t> hmeta;   // host image of the chunk's per-pair region (meta)
    void release() {
        ws.release_all();
        for (gx::DevBuf *b : {&q, &t, &meta, &cig}) b->release();
        if (st) { (void)hipStreamSynchronize(st); (void)hipStreamDestroy(st); st = nullptr; }
    }
};

struct gasalx_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    gx::Workspace ws;
    HostSlot slot[2];
    // staging for the host-to-host entry points
    gx::DevBuf q, t, qo, to, ql, tl, qop, top, seed;
    gx::DevBuf o_score, o_qe, o_te, o_qs, o_ts, o_s2, o_qe2, o_te2, o_cig, o_nops, lens_max;
    gx::DevBuf h_reads, h_ro, h_rl, h_qm, h_de, h_xi, h_al, h_haps, h_ho, h_hl, h_res;
    gx::DevBuf h_bq, h_iq, h_dq, h_perm, ph2pr;   // PairHMM from qualities: staging + the ph2pr table
    gx::DevBuf nv_pw, nv_po, nv_tw, nv_to, nv_s, nv_s16;   // nvbio front-end staging
    gx::DevBuf nv_dir, nv_row, nv_src, nv_snk, nv_ops, nv_nops;   // nvbio traceback: workspace + staging
    void release() {
        ws.release_all();
        for (HostSlot &s : slot) s.release();
        for (gx::DevBuf *b : {&q, &t, &qo, &to, &ql, &tl, &qop, &top, &seed, &o_score, &o_qe, &o_te, &o_qs, &o_ts,
                              &o_s2, &o_qe2, &o_te2, &o_cig, &o_nops, &lens_max, &h_reads, &h_ro, &h_rl, &h_qm,
                              &h_de, &h_xi, &h_al, &h_haps, &h_ho, &h_hl, &h_res, &h_bq, &h_iq, &h_dq, &h_perm,
                              &ph2pr, &nv_pw, &nv_po, &nv_tw, &nv_to, &nv_s, &nv_s16, &nv_dir, &nv_row,
                              &nv_src, &nv_snk, &nv_ops, &nv_nops})
            b->release();
    }
};

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e__ = (x);                                                        \
        if (e__ != hipSuccess) {                                                     \
            gx::set_error(std::string(#x) + ": " + hipGetErrorString(e__));          \
            return e__ == hipErrorOutOfMemory ? GASALX_ENOMEM : GASALX_EDEVICE;      \
        }                                                                            \
    } while (0)

hipStream_t gx::engine_stream(gasalx_engine *e) { return e->stream; }

namespace {

__attribute__((unused)) uint32_t host_max(const uint32_t *a, uint32_t n) {
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; i++) m = std::max(m, a[i]);
    return m;
}

// Read back max(q_lens), max(t_lens) from device memory (synchronises `st`).
int device_max_lens(gasalx_engine *eng, const uint32_t *dq, const uint32_t *dt, uint32_t n, hipStream_t st,
                    uint32_t *mq, uint32_t *mt) {
    std::vector<uint32_t> hq(n), ht(n);
    CK(hipMemcpyAsync(hq.data(), dq, n * 4ull, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(ht.data(), dt, n * 4ull, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    (void)eng;
    *mq = host_max(hq.data(), n);
    *mt = host_max(ht.data(), n);
    return GASALX_OK;
}

template <class T>
int stage_in(gx::DevBuf &d, const T *h, size_t count, hipStream_t st, T **dptr) {
    *dptr = nullptr;
    if (!h) return GASALX_OK;
    CK(d.reserve(count * sizeof(T) + 16));
    CK(hipMemcpyAsync(d.p, h, count * sizeof(T), hipMemcpyHostToDevice, st));
    *dptr = d.as<T>();
    return GASALX_OK;
}

bool valid_params(const gasalx_params *p) {
    if (!p) return false;
    if (p->algo < 0 || p->algo > 6) return false;
    if (p->start_pos < 0 || p->start_pos > 2) return false;
    if (p->head < 0 || p->head > 3 || p->tail < 0 || p->tail > 3) return false;
    return true;
}

}  // namespace

extern "C" {

int gasalx_abi_version(void) { return GASALX_ABI_VERSION; }
const char *gasalx_last_error(void) { return gx::last_error(); }

int gasalx_device_count(int *count) {
    if (!count) return GASALX_EINVAL;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) { *count = 0; gx::set_error(hipGetErrorString(e)); return GASALX_EDEVICE; }
    *count = c;
    return GASALX_OK;
}

int gasalx_engine_create(int device, gasalx_engine **out) {
    if (!out) return GASALX_EINVAL;
    *out = nullptr;
    CK(hipSetDevice(device));
    gasalx_engine *e = new (std::nothrow) gasalx_engine();
    if (!e) return GASALX_ENOMEM;
    e->device = device;
    e->ws.device = device;
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) { delete e; gx::set_error(hipGetErrorString(he)); return GASALX_EDEVICE; }
    *out = e;
    return GASALX_OK;
}

int gasalx_engine_destroy(gasalx_engine *eng) {
    if (!eng) return GASALX_OK;
    (void)hipSetDevice(eng->device);
    if (eng->stream) { (void)hipStreamSynchronize(eng->stream); (void)hipStreamDestroy(eng->stream); }
    eng->release();
    delete eng;
    return GASALX_OK;
}

int gasalx_describe_plan(const gasalx_params *params, uint32_t max_q_len, uint32_t max_t_len, char *buf,
                         uint32_t buf_len) {
    if (!valid_params(params) || !buf || buf_len == 0) return GASALX_EINVAL;
    gx::BatchShape s;
    s.max_q = max_q_len; s.max_t = max_t_len;
    gx::Plan pl = gx::make_plan(*params, s, false);
    std::snprintf(buf, buf_len, "%s", pl.name.c_str());
    return GASALX_OK;
}

int gasalx_align_device(gasalx_engine *eng, const gasalx_params *params, const gasalx_batch *b,
                        const gasalx_results *out, void *stream) {
    if (!eng || !valid_params(params) || !b || !out) { gx::set_error("null argument"); return GASALX_EINVAL; }
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    gx::BatchShape shape;
    shape.max_q = b->max_q_len;
    shape.max_t = b->max_t_len;
    if ((shape.max_q == 0 || shape.max_t == 0) && b->n_alns) {
        int rc = device_max_lens(eng, b->q_lens, b->t_lens, b->n_alns, st, &shape.max_q, &shape.max_t);
        if (rc) return rc;
    }
    return gx::align_device(eng->ws, *params, *b, *out, st, shape);
}

namespace {

uint32_t pad8u(uint32_t x) { return (x + 7u) & ~7u; }


// Sequences laid out back to back from offset 0 (what gasal_host_batch_fill
// produces): chunks of pairs then own contiguous byte ranges.
bool contiguous(const uint32_t *off, const uint32_t *len, uint32_t n, uint32_t bytes) {
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (off[i] != at) return false;
        at += pad8u(len[i]);
    }
    return at == bytes;
}

// Large host batches: chunks of pairs alternate between two streams, so the
// H2D copy of chunk k+1 overlaps the kernels of chunk k (the copies run at
// PCIe speed from pageable memory on this platform, tools/h2d_probe.cpp).
// Per chunk: two sequence copies plus ONE copy of everything per-pair
// (rebased offsets, lengths, ops, seeds, the caller's output contents) and
// ONE copy back of the per-pair outputs.
int align_host_pipelined(gasalx_engine *eng, const gasalx_params *params, const gasalx_batch *hb,
                         const gasalx_results *ho, uint32_t chunk) {
    const uint32_t n = hb->n_alns;
    const bool tb = params->start_pos == 2;
    const uint32_t mq = hb->max_q_len ? hb->max_q_len : host_max(hb->q_lens, n);
    const uint32_t mt = hb->max_t_len ? hb->max_t_len : host_max(hb->t_lens, n);
    int32_t *const hout[8] = {ho->aln_score, ho->q_end, ho->t_end, ho->q_start,
                              ho->t_start, ho->aln_score2, ho->q_end2, ho->t_end2};
    uint32_t *const hnops = tb ? ho->n_cigar_ops : nullptr;
    // outputs every kernel of the algorithm writes (generic.hpp, wavefront*.hpp):
    // the score for all aligning algos, the ends for all but GLOBAL
    const bool ends = params->algo == 2 || params->algo == 3 || params->algo == 5 || params->algo == 6;
    const bool aligns = ends || params->algo == 1;   // UNKNOWN / MICROLOCAL launch nothing
    const bool written[8] = {aligns, ends, ends, false, false, false, false, false};
    for (HostSlot &s : eng->slot) {
        if (!s.st) CK(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
        s.ws.device = eng->device;
    }
    // per-pair region of a chunk of m pairs: 4-byte columns, 16-byte aligned
    auto col = [](uint32_t m) { return ((size_t)m * 4 + 15) & ~(size_t)15; };
    auto bcol = [](uint32_t m) { return ((size_t)m + 15) & ~(size_t)15; };
    struct Pending { uint32_t i0, i1; uint64_t qlo, qhi; size_t out_at, out_len; bool live; } pend[2] = {};
    auto drain = [&](int k) -> int {   // the slot's previous chunk: results back to the caller
        Pending &pp = pend[k];
        if (!pp.live) return GASALX_OK;
        HostSlot &s = eng->slot[k];
        const uint32_t m = pp.i1 - pp.i0;
        if (pp.out_len)
            CK(hipMemcpyAsync(s.hmeta.data() + pp.out_at, s.meta.as<uint8_t>() + pp.out_at, pp.out_len,
                              hipMemcpyDeviceToHost, s.st));
        if (tb && ho->cigar)
            CK(hipMemcpyAsync(ho->cigar + pp.qlo, s.cig.p, pp.qhi - pp.qlo, hipMemcpyDeviceToHost, s.st));
        CK(hipStreamSynchronize(s.st));
        size_t at = pp.out_at;
        for (int f = 0; f < 8; f++)
            if (hout[f]) { std::memcpy(hout[f] + pp.i0, s.hmeta.data() + at, m * 4ull); at += col(m); }
        if (hnops) std::memcpy(hnops + pp.i0, s.hmeta.data() + at, m * 4ull);
        pp.live = false;
        return GASALX_OK;
    };
    int rc = GASALX_OK, k = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += chunk, k ^= 1) {
        const uint32_t i1 = std::min(n, i0 + chunk), m = i1 - i0;
        HostSlot &s = eng->slot[k];
        if ((rc = drain(k))) return rc;
        const uint64_t qlo = hb->q_offsets[i0], qhi = (uint64_t)hb->q_offsets[i1 - 1] + pad8u(hb->q_lens[i1 - 1]);
        const uint64_t tlo = hb->t_offsets[i0], thi = (uint64_t)hb->t_offsets[i1 - 1] + pad8u(hb->t_lens[i1 - 1]);
        // host image of the per-pair region
        size_t at = 0;
        const size_t a_qo = at; at += col(m);
        const size_t a_to = at; at += col(m);
        const size_t a_ql = at; at += col(m);
        const size_t a_tl = at; at += col(m);
        const size_t a_qop = at; if (hb->q_ops) at += bcol(m);
        const size_t a_top = at; if (hb->t_ops) at += bcol(m);
        const size_t a_seed = at; if (hb->seed_scores) at += col(m);
        const size_t out_at = at;
        size_t a_out[8];
        for (int f = 0; f < 8; f++) { a_out[f] = at; if (hout[f]) at += col(m); }
        const size_t a_nops = at; if (hnops) at += col(m);
        const size_t total = at;
        s.hmeta.resize(total);
        uint8_t *h = s.hmeta.data();
        uint32_t *qo = reinterpret_cast<uint32_t *>(h + a_qo), *to = reinterpret_cast<uint32_t *>(h + a_to);
        for (uint32_t i = 0; i < m; i++) {
            qo[i] = hb->q_offsets[i0 + i] - (uint32_t)qlo;
            to[i] = hb->t_offsets[i0 + i] - (uint32_t)tlo;
        }
        std::memcpy(h + a_ql, hb->q_lens + i0, m * 4ull);
        std::memcpy(h + a_tl, hb->t_lens + i0, m * 4ull);
        if (hb->q_ops) std::memcpy(h + a_qop, hb->q_ops + i0, m);
        if (hb->t_ops) std::memcpy(h + a_top, hb->t_ops + i0, m);
        if (hb->seed_scores) std::memcpy(h + a_seed, hb->seed_scores + i0, m * 4ull);
        // the caller's contents, so fields the reference does not write come back
        // unchanged; fields every kernel of this algo writes need no copy in
        for (int f = 0; f < 8; f++)
            if (hout[f] && !written[f]) std::memcpy(h + a_out[f], hout[f] + i0, m * 4ull);
        if (hnops) std::memcpy(h + a_nops, hnops + i0, m * 4ull);
        CK(s.meta.reserve(total + 16));
        uint8_t *dm = s.meta.as<uint8_t>();
        uint8_t *p8;
        // isPacked (score-only): the caller's pages hold 4-bit words, half the bytes of the
        // unpacked units that offsets and q_bytes count (pack_rc_seqs.h:24-31); only those move
        const uint64_t pk = params->is_packed ? 2 : 1;
        if ((rc = stage_in(s.q, hb->q_batch + qlo / pk, (qhi - qlo) / pk, s.st, &p8))) return rc;
        gasalx_batch db = *hb;
        db.q_batch = p8;
        if ((rc = stage_in(s.t, hb->t_batch + tlo / pk, (thi - tlo) / pk, s.st, &p8))) return rc;
        db.t_batch = p8;
        CK(hipMemcpyAsync(dm, h, total, hipMemcpyHostToDevice, s.st));
        db.q_offsets = reinterpret_cast<uint32_t *>(dm + a_qo);
        db.t_offsets = reinterpret_cast<uint32_t *>(dm + a_to);
        db.q_lens = reinterpret_cast<uint32_t *>(dm + a_ql);
        db.t_lens = reinterpret_cast<uint32_t *>(dm + a_tl);
        db.q_ops = hb->q_ops ? dm + a_qop : nullptr;
        db.t_ops = hb->t_ops ? dm + a_top : nullptr;
        db.seed_scores = hb->seed_scores ? reinterpret_cast<uint32_t *>(dm + a_seed) : nullptr;
        db.q_bytes = (uint32_t)(qhi - qlo);
        db.t_bytes = (uint32_t)(thi - tlo);
        db.n_alns = m;
        db.max_q_len = mq;
        db.max_t_len = mt;
        gasalx_results dout;
        std::memset(&dout, 0, sizeof(dout));
        int32_t **dfield[8] = {&dout.aln_score, &dout.q_end, &dout.t_end, &dout.q_start,
                               &dout.t_start, &dout.aln_score2, &dout.q_end2, &dout.t_end2};
        for (int f = 0; f < 8; f++) *dfield[f] = hout[f] ? reinterpret_cast<int32_t *>(dm + a_out[f]) : nullptr;
        if (hnops) dout.n_cigar_ops = reinterpret_cast<uint32_t *>(dm + a_nops);
        if (tb && ho->cigar) {
            CK(s.cig.reserve(qhi - qlo + 16));
            dout.cigar = s.cig.as<uint8_t>();
        }
        gx::BatchShape shape;
        shape.max_q = mq;
        shape.max_t = mt;
        shape.sort = gx::uneven_lengths(*params, hb->q_lens + i0, hb->t_lens + i0, m);
        shape.one_t8 = gx::one_pad8(hb->t_lens + i0, m, shape.max_t);
        shape.tb_split = false;   // the two slots' streams already overlap one chunk's walk with the next DP
        if ((rc = gx::align_device(s.ws, *params, db, dout, s.st, shape))) {
            for (HostSlot &x : eng->slot) (void)hipStreamSynchronize(x.st);
            return rc;
        }
        pend[k] = {i0, i1, qlo, qhi, out_at, total - out_at, true};
    }
    for (int j = 0; j < 2; j++) {
        k ^= 1;
        if ((rc = drain(k))) return rc;
    }
    return GASALX_OK;
}

}  // namespace

int gasalx_align_host(gasalx_engine *eng, const gasalx_params *params, const gasalx_batch *hb,
                      const gasalx_results *ho) {
    if (!eng || !valid_params(params) || !hb || !ho) { gx::set_error("null argument"); return GASALX_EINVAL; }
    if (!hb->q_batch || !hb->t_batch || !hb->q_offsets || !hb->t_offsets || !hb->q_lens || !hb->t_lens) {
        gx::set_error("missing batch array");
        return GASALX_EINVAL;
    }
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    const uint32_t n = hb->n_alns;
    // large batches in the standard layout go through the two-stream pipeline
    // TB: the traceback walk is latency-bound per chunk whatever its size, so chunks
    // of ~5.5 G padded cells, 2 to 8 of them (1 M x 150 bp: 4, 34.0 ms pageable against
    // 50.5 with 2; 100 K x 300 bp: 2); score-only: 8
    uint32_t n_chunks = 8;
    if (params->start_pos == 2) {
        const double mq = hb->max_q_len ? hb->max_q_len : host_max(hb->q_lens, n);
        const double mt = hb->max_t_len ? hb->max_t_len : host_max(hb->t_lens, n);
        n_chunks = (uint32_t)std::min(8.0, std::max(2.0, std::round((double)n * mq * mt / 5.5e9)));
    }
    const uint32_t chunk = std::max<uint32_t>(16384, (uint32_t)(((uint64_t)n + n_chunks - 1) / n_chunks));
    const bool tb = params->start_pos == 2;
    if (n >= 2 * chunk && !(params->is_packed && tb) && contiguous(hb->q_offsets, hb->q_lens, n, hb->q_bytes) &&
        contiguous(hb->t_offsets, hb->t_lens, n, hb->t_bytes))
        return align_host_pipelined(eng, params, hb, ho, chunk);
    gasalx_batch db = *hb;
    int rc = 0;
    uint8_t *p8; uint32_t *p32;
    // isPacked without traceback: only the packed half of the pages moves (with traceback the
    // device CIGAR buffer starts as the whole query batch, gasal_align.cu:281)
    const uint32_t pk = params->is_packed && !tb ? 2 : 1;
    if ((rc = stage_in(eng->q, hb->q_batch, hb->q_bytes / pk, st, &p8))) return rc; db.q_batch = p8;
    if ((rc = stage_in(eng->t, hb->t_batch, hb->t_bytes / pk, st, &p8))) return rc; db.t_batch = p8;
    if ((rc = stage_in(eng->qo, hb->q_offsets, n, st, &p32))) return rc; db.q_offsets = p32;
    if ((rc = stage_in(eng->to, hb->t_offsets, n, st, &p32))) return rc; db.t_offsets = p32;
    if ((rc = stage_in(eng->ql, hb->q_lens, n, st, &p32))) return rc; db.q_lens = p32;
    if ((rc = stage_in(eng->tl, hb->t_lens, n, st, &p32))) return rc; db.t_lens = p32;
    if ((rc = stage_in(eng->qop, hb->q_ops, n, st, &p8))) return rc; db.q_ops = p8;
    if ((rc = stage_in(eng->top, hb->t_ops, n, st, &p8))) return rc; db.t_ops = p8;
    if ((rc = stage_in(eng->seed, hb->seed_scores, n, st, &p32))) return rc; db.seed_scores = p32;
    if (!db.max_q_len) db.max_q_len = host_max(hb->q_lens, n);
    if (!db.max_t_len) db.max_t_len = host_max(hb->t_lens, n);

    // outputs: staged in with the caller's contents so fields the reference
    // would not write come back unchanged
    gasalx_results dout;
    std::memset(&dout, 0, sizeof(dout));
    int32_t *i32;
    if ((rc = stage_in(eng->o_score, ho->aln_score, n, st, &i32))) return rc; dout.aln_score = i32;
    if ((rc = stage_in(eng->o_qe, ho->q_end, n, st, &i32))) return rc; dout.q_end = i32;
    if ((rc = stage_in(eng->o_te, ho->t_end, n, st, &i32))) return rc; dout.t_end = i32;
    if ((rc = stage_in(eng->o_qs, ho->q_start, n, st, &i32))) return rc; dout.q_start = i32;
    if ((rc = stage_in(eng->o_ts, ho->t_start, n, st, &i32))) return rc; dout.t_start = i32;
    if ((rc = stage_in(eng->o_s2, ho->aln_score2, n, st, &i32))) return rc; dout.aln_score2 = i32;
    if ((rc = stage_in(eng->o_qe2, ho->q_end2, n, st, &i32))) return rc; dout.q_end2 = i32;
    if ((rc = stage_in(eng->o_te2, ho->t_end2, n, st, &i32))) return rc; dout.t_end2 = i32;
    if ((rc = stage_in(eng->o_cig, ho->cigar, hb->q_bytes, st, &p8))) return rc; dout.cigar = p8;
    if ((rc = stage_in(eng->o_nops, ho->n_cigar_ops, n, st, &p32))) return rc; dout.n_cigar_ops = p32;

    gx::BatchShape shape;
    shape.max_q = db.max_q_len;
    shape.max_t = db.max_t_len;
    shape.sort = gx::uneven_lengths(*params, hb->q_lens, hb->t_lens, n);
    shape.one_t8 = gx::one_pad8(hb->t_lens, n, shape.max_t);
    rc = gx::align_device(eng->ws, *params, db, dout, st, shape);
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
#define BACK(h, d, cnt)                                                                             \
    if (h) CK(hipMemcpyAsync((void *)(h), (d), (size_t)(cnt) * sizeof(*(h)), hipMemcpyDeviceToHost, st));
    BACK(ho->aln_score, dout.aln_score, n)
    BACK(ho->q_end, dout.q_end, n)
    BACK(ho->t_end, dout.t_end, n)
    BACK(ho->q_start, dout.q_start, n)
    BACK(ho->t_start, dout.t_start, n)
    BACK(ho->aln_score2, dout.aln_score2, n)
    BACK(ho->q_end2, dout.q_end2, n)
    BACK(ho->t_end2, dout.t_end2, n)
    BACK(ho->cigar, dout.cigar, hb->q_bytes)
    BACK(ho->n_cigar_ops, dout.n_cigar_ops, n)
#undef BACK
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

int gasalx_pairhmm_device(gasalx_engine *eng, const gasalx_hmm_batch *b, float *res, void *stream) {
    if (!eng || !b || !res) { gx::set_error("null argument"); return GASALX_EINVAL; }
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    uint32_t mr = b->max_read_len, mh = b->max_hap_len;
    if ((!mr || !mh) && b->n_pairs) {
        int rc = device_max_lens(eng, b->read_lens, b->hap_lens, b->n_pairs, st, &mr, &mh);
        if (rc) return rc;
    }
    return gx::pairhmm_device(eng->ws, *b, res, st, mr, mh);
}

int gasalx_pairhmm_host(gasalx_engine *eng, const gasalx_hmm_batch *hb, float *hres) {
    if (!eng || !hb || !hres) { gx::set_error("null argument"); return GASALX_EINVAL; }
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    const uint32_t n = hb->n_pairs;
    gasalx_hmm_batch db = *hb;
    int rc;
    uint8_t *p8; uint32_t *p32; float *pf;
    if ((rc = stage_in(eng->h_reads, hb->reads, hb->read_bytes, st, &p8))) return rc; db.reads = p8;
    if ((rc = stage_in(eng->h_ro, hb->read_offsets, n, st, &p32))) return rc; db.read_offsets = p32;
    if ((rc = stage_in(eng->h_rl, hb->read_lens, n, st, &p32))) return rc; db.read_lens = p32;
    if ((rc = stage_in(eng->h_qm, hb->qm, hb->read_bytes, st, &pf))) return rc; db.qm = pf;
    if ((rc = stage_in(eng->h_de, hb->delta, hb->read_bytes, st, &pf))) return rc; db.delta = pf;
    if ((rc = stage_in(eng->h_xi, hb->xiksi, hb->read_bytes, st, &pf))) return rc; db.xiksi = pf;
    if ((rc = stage_in(eng->h_al, hb->alpha, hb->read_bytes, st, &pf))) return rc; db.alpha = pf;
    if ((rc = stage_in(eng->h_haps, hb->haps, hb->hap_bytes, st, &p8))) return rc; db.haps = p8;
    if ((rc = stage_in(eng->h_ho, hb->hap_offsets, n, st, &p32))) return rc; db.hap_offsets = p32;
    if ((rc = stage_in(eng->h_hl, hb->hap_lens, n, st, &p32))) return rc; db.hap_lens = p32;
    CK(eng->h_res.reserve((size_t)n * 4 + 16));
    uint32_t mr = hb->max_read_len ? hb->max_read_len : host_max(hb->read_lens, n);
    uint32_t mh = hb->max_hap_len ? hb->max_hap_len : host_max(hb->hap_lens, n);
    rc = gx::pairhmm_device(eng->ws, db, eng->h_res.as<float>(), st, mr, mh);
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
    CK(hipMemcpyAsync(hres, eng->h_res.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

}  // extern "C"

namespace {

// ph2pr[q] = powf(10, -q/10) on the host, as the reference builds it (tile_1.cu:216-220)
void ph2pr_table(float *t) {
    for (int i = 0; i < 128; i++) t[i] = powf(10.f, -((float)i) / 10.f);
}

// The engine's device copy of the table (uploaded once, synchronously).
int ph2pr_device(gasalx_engine *eng, const float **out) {
    if (!eng->ph2pr.p) {
        float t[128];
        ph2pr_table(t);
        CK(eng->ph2pr.reserve(sizeof(t)));
        CK(hipMemcpy(eng->ph2pr.p, t, sizeof(t), hipMemcpyHostToDevice));
    }
    *out = eng->ph2pr.as<float>();
    return GASALX_OK;
}

bool hmm_qual_batch_ok(const gasalx_hmm_qual_batch *b) {
    return b && (b->n_pairs == 0 || (b->reads && b->read_offsets && b->read_lens && b->base_quals && b->ins_quals &&
                                     b->del_quals && b->haps && b->hap_offsets && b->hap_lens));
}

}  // namespace

extern "C" {

int gasalx_pairhmm_quals_device(gasalx_engine *eng, const gasalx_hmm_qual_batch *b, float *res, void *stream) {
    if (!eng || !hmm_qual_batch_ok(b) || !res) { gx::set_error("null argument"); return GASALX_EINVAL; }
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    uint32_t mr = b->max_read_len, mh = b->max_hap_len;
    if ((!mr || !mh) && b->n_pairs) {
        int rc = device_max_lens(eng, b->read_lens, b->hap_lens, b->n_pairs, st, &mr, &mh);
        if (rc) return rc;
    }
    const float *tab;
    int rc = ph2pr_device(eng, &tab);
    if (rc) return rc;
    return gx::pairhmm_quals_device(eng->ws, *b, res, st, tab, nullptr, nullptr, 0, mr, mh);
}

int gasalx_pairhmm_quals_host(gasalx_engine *eng, const gasalx_hmm_qual_batch *hb, float *hres) {
    if (!eng || !hmm_qual_batch_ok(hb) || !hres) { gx::set_error("null argument"); return GASALX_EINVAL; }
    const uint32_t n = hb->n_pairs;
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    // slots in (read length, haplotype length) order (tile_1.cu:180-195 operator<, :325)
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; i++) perm[i] = i;
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t x, uint32_t y) {
        const uint32_t rx = hb->read_lens[x], ry = hb->read_lens[y];
        return rx != ry ? rx < ry : hb->hap_lens[x] < hb->hap_lens[y];
    });
    // classes: runs of slots whose reads need the same lane-group size
    std::vector<gx::HmmClass> classes;
    for (uint32_t s = 0; s < n; s++) {
        const uint32_t r = hb->read_lens[perm[s]], h = hb->hap_lens[perm[s]];
        const int g = gx::pairhmm_group(r);
        if (classes.empty() || gx::pairhmm_group(classes.back().max_r) != g) classes.push_back({s, s, 0, 0});
        gx::HmmClass &c = classes.back();
        c.slot1 = s + 1;
        c.max_r = std::max(c.max_r, r);
        c.max_h = std::max(c.max_h, h);
    }
    gasalx_hmm_qual_batch db = *hb;
    int rc;
    uint8_t *p8; uint32_t *p32;
    if ((rc = stage_in(eng->h_reads, hb->reads, hb->read_bytes, st, &p8))) return rc; db.reads = p8;
    if ((rc = stage_in(eng->h_bq, hb->base_quals, hb->read_bytes, st, &p8))) return rc; db.base_quals = p8;
    if ((rc = stage_in(eng->h_iq, hb->ins_quals, hb->read_bytes, st, &p8))) return rc; db.ins_quals = p8;
    if ((rc = stage_in(eng->h_dq, hb->del_quals, hb->read_bytes, st, &p8))) return rc; db.del_quals = p8;
    if ((rc = stage_in(eng->h_ro, hb->read_offsets, n, st, &p32))) return rc; db.read_offsets = p32;
    if ((rc = stage_in(eng->h_rl, hb->read_lens, n, st, &p32))) return rc; db.read_lens = p32;
    if ((rc = stage_in(eng->h_haps, hb->haps, hb->hap_bytes, st, &p8))) return rc; db.haps = p8;
    if ((rc = stage_in(eng->h_ho, hb->hap_offsets, n, st, &p32))) return rc; db.hap_offsets = p32;
    if ((rc = stage_in(eng->h_hl, hb->hap_lens, n, st, &p32))) return rc; db.hap_lens = p32;
    uint32_t *dperm;
    if ((rc = stage_in(eng->h_perm, perm.data(), n, st, &dperm))) return rc;
    CK(eng->h_res.reserve((size_t)n * 4 + 16));
    const float *tab;
    if ((rc = ph2pr_device(eng, &tab))) return rc;
    rc = gx::pairhmm_quals_device(eng->ws, db, eng->h_res.as<float>(), st, tab, dperm, classes.data(),
                                  (int)classes.size(), 0, 0);
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
    CK(hipMemcpyAsync(hres, eng->h_res.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

namespace {
// max over i of off[i+1] - off[i]
uint32_t max_span(const uint32_t *off, uint32_t n) {
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; i++) m = std::max(m, off[i + 1] - off[i]);
    return m;
}
}  // namespace

int gasalx_nv_score_device(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t n, const gasalx_nv_strings *pat,
                           const gasalx_nv_strings *txt, int32_t *scores, int16_t *scores16, uint32_t max_p,
                           uint32_t max_t, void *stream) {
    if (!eng || !al || !pat || !txt) { gx::set_error("null argument"); return GASALX_EINVAL; }
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    if (n && (!max_p || (txt->offsets && !max_t))) {   // read the offsets back (synchronises the stream)
        std::vector<uint32_t> po(n + 1), to(txt->offsets ? n + 1 : 0);
        CK(hipMemcpyAsync(po.data(), pat->offsets, (n + 1) * 4ull, hipMemcpyDeviceToHost, st));
        if (txt->offsets) CK(hipMemcpyAsync(to.data(), txt->offsets, (n + 1) * 4ull, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        if (!max_p) max_p = max_span(po.data(), n);
        if (txt->offsets && !max_t) max_t = max_span(to.data(), n);
    }
    return gx::nv_score_device(*al, n, *pat, *txt, scores, scores16, max_p, max_t, st);
}

int gasalx_nv_describe_plan(const gasalx_nv_aligner *al, uint32_t max_p, uint32_t max_t, int per_pair,
                            uint32_t text_bits, char *buf, uint32_t buf_len) {
    if (!al || !buf || buf_len == 0) { gx::set_error("null argument"); return GASALX_EINVAL; }
    std::snprintf(buf, buf_len, "%s", gx::nv_plan_name(*al, max_p, max_t, per_pair != 0, text_bits).c_str());
    return GASALX_OK;
}

int gasalx_nv_score_host(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t n, const gasalx_nv_strings *pat,
                         uint64_t pat_words, const gasalx_nv_strings *txt, uint64_t txt_words, int32_t *scores,
                         int16_t *scores16) {
    if (!eng || !al || !pat || !txt || !pat->words || !pat->offsets || !txt->words || (!scores && !scores16)) {
        gx::set_error("null argument");
        return GASALX_EINVAL;
    }
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    const uint32_t max_p = max_span(pat->offsets, n);
    const uint32_t max_t = txt->offsets ? max_span(txt->offsets, n) : txt->length;
    gasalx_nv_strings dp = *pat, dt = *txt;
    int rc;
    uint32_t *p32;
    if ((rc = stage_in(eng->nv_pw, pat->words, pat_words, st, &p32))) return rc; dp.words = p32;
    if ((rc = stage_in(eng->nv_po, pat->offsets, (size_t)n + 1, st, &p32))) return rc; dp.offsets = p32;
    if ((rc = stage_in(eng->nv_tw, txt->words, txt_words, st, &p32))) return rc; dt.words = p32;
    if ((rc = stage_in(eng->nv_to, txt->offsets, txt->offsets ? (size_t)n + 1 : 0, st, &p32))) return rc;
    dt.offsets = txt->offsets ? p32 : nullptr;
    int32_t *ds = nullptr;
    int16_t *ds16 = nullptr;
    if (scores) { CK(eng->nv_s.reserve((size_t)n * 4)); ds = eng->nv_s.as<int32_t>(); }
    if (scores16) { CK(eng->nv_s16.reserve((size_t)n * 2)); ds16 = eng->nv_s16.as<int16_t>(); }
    rc = gx::nv_score_device(*al, n, dp, dt, ds, ds16, max_p, max_t, st);
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
    if (scores) CK(hipMemcpyAsync(scores, ds, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    if (scores16) CK(hipMemcpyAsync(scores16, ds16, (size_t)n * 2, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

int gasalx_nv_banded_score_device(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t band, uint32_t n,
                                  const gasalx_nv_strings *pat, const gasalx_nv_strings *txt, int32_t *scores,
                                  uint32_t max_p, void *stream) {
    if (!eng || !al || !pat || !txt) { gx::set_error("null argument"); return GASALX_EINVAL; }
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    if (n && !max_p && pat->offsets) {   // read the offsets back (synchronises the stream)
        std::vector<uint32_t> po(n + 1);
        CK(hipMemcpyAsync(po.data(), pat->offsets, (n + 1) * 4ull, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        max_p = max_span(po.data(), n);
    }
    return gx::nv_banded_score_device(*al, band, n, *pat, *txt, scores, st, max_p);
}

int gasalx_nv_banded_score_host(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t band, uint32_t n,
                                const gasalx_nv_strings *pat, uint64_t pat_words, const gasalx_nv_strings *txt,
                                uint64_t txt_words, int32_t *scores) {
    if (!eng || !al || !pat || !txt || !pat->words || !pat->offsets || !txt->words || !scores) {
        gx::set_error("null argument");
        return GASALX_EINVAL;
    }
    if (band < 2 || band > 32) { gx::set_error("band length must be 2..32"); return GASALX_EINVAL; }
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    gasalx_nv_strings dp = *pat, dt = *txt;
    int rc;
    uint32_t *p32;
    if ((rc = stage_in(eng->nv_pw, pat->words, pat_words, st, &p32))) return rc; dp.words = p32;
    if ((rc = stage_in(eng->nv_po, pat->offsets, (size_t)n + 1, st, &p32))) return rc; dp.offsets = p32;
    if ((rc = stage_in(eng->nv_tw, txt->words, txt_words, st, &p32))) return rc; dt.words = p32;
    if ((rc = stage_in(eng->nv_to, txt->offsets, txt->offsets ? (size_t)n + 1 : 0, st, &p32))) return rc;
    dt.offsets = txt->offsets ? p32 : nullptr;
    CK(eng->nv_s.reserve((size_t)n * 4));
    rc = gx::nv_banded_score_device(*al, band, n, dp, dt, eng->nv_s.as<int32_t>(), st, max_span(pat->offsets, n));
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
    CK(hipMemcpyAsync(scores, eng->nv_s.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

// nvbio BatchedAlignmentTraceback (nvtrace.hpp).  nvbio keeps its DP columns and checkpoints in
// int16 (alignment/utils.h:49-64): the scores of every cell must stay within them.
static int64_t nv_score_mag(const gasalx_nv_aligner *al) {
    if (al->aligner == GASALX_NV_ED) return 1;   // ED: EditDistanceSWScheme's 0 / -1 (ed_utils.h:45-52)
    return std::max<int64_t>({std::abs((int64_t)al->match), std::abs((int64_t)al->mismatch),
                              std::abs((int64_t)al->gap_open), std::abs((int64_t)al->gap_ext),
                              std::abs((int64_t)al->deletion), std::abs((int64_t)al->insertion), 1});
}

// nvbio traceback workspace per call (the engine's: flags of every cell, one DP row per pair) and
// the chunk budget the device entry points split a batch by
static constexpr uint64_t kNvTbBudget = 4ull << 30;
uint64_t gasalx_nv_traceback_workspace(uint32_t max_p, uint32_t max_t, uint32_t n) {
    const uint64_t per = (uint64_t)((max_p + 7) / 8) * 8 * max_t + (uint64_t)max_t * 8;
    const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(n, kNvTbBudget / std::max<uint64_t>(per, 1)));
    return per * chunk + 128;
}
uint64_t gasalx_nv_banded_traceback_workspace(uint32_t max_p, uint32_t band, uint32_t n) {
    const uint64_t per = (uint64_t)max_p * ((band + 3) / 4) * 4;
    const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(n, kNvTbBudget / std::max<uint64_t>(per, 1)));
    return per * chunk + 64;
}

static int nv_tb_checks(const gasalx_nv_aligner *al, uint32_t max_p, uint32_t max_t, uint32_t ops_stride) {
    const int64_t mag = nv_score_mag(al);
    if (((int64_t)max_p + max_t + 2) * mag > 32767) {
        gx::set_error("traceback: scores would leave nvbio's int16 columns (lengths x |score|)");
        return GASALX_ERANGE;
    }
    if (ops_stride < max_p + max_t) { gx::set_error("traceback: ops_stride < max pattern + max text length"); return GASALX_EINVAL; }
    if ((uint64_t)max_p * max_t > (1ull << 24)) { gx::set_error("traceback: pattern x text above 16 M cells"); return GASALX_ERANGE; }
    return GASALX_OK;
}

int gasalx_nv_traceback_device(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t n,
                               const gasalx_nv_strings *pat, const gasalx_nv_strings *txt, uint32_t max_p,
                               uint32_t max_t, int32_t *scores, uint32_t *sources, uint32_t *sinks, uint8_t *ops,
                               uint32_t ops_stride, uint32_t *n_ops, void *stream) {
    if (!eng || !al || !pat || !txt) { gx::set_error("null argument"); return GASALX_EINVAL; }
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    if (!max_p || (txt->offsets && !max_t)) {   // read the offsets back (synchronises the stream)
        std::vector<uint32_t> po(n + 1), to(txt->offsets ? n + 1 : 0);
        CK(hipMemcpyAsync(po.data(), pat->offsets, (n + 1) * 4ull, hipMemcpyDeviceToHost, st));
        if (txt->offsets) CK(hipMemcpyAsync(to.data(), txt->offsets, (n + 1) * 4ull, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        if (!max_p) max_p = max_span(po.data(), n);
        if (txt->offsets && !max_t) max_t = max_span(to.data(), n);
    }
    if (!txt->offsets) max_t = txt->length;
    int rc = nv_tb_checks(al, max_p, max_t, ops_stride);
    if (rc) return rc;
    // the batch runs in chunks whose workspace (flags of every cell + one row per pair) stays
    // within kNvTbBudget (1 M 150 x 182 pairs would otherwise take 28 GB of HBM)
    const uint64_t per = gasalx_nv_traceback_workspace(max_p, max_t, 1);
    const uint32_t chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, kNvTbBudget / per));
    CK(eng->nv_dir.reserve((size_t)((max_p + 7) / 8) * 8 * max_t * chunk + 64));
    CK(eng->nv_row.reserve((size_t)max_t * chunk * 8 + 64));
    for (uint32_t s = 0; s < n; s += chunk) {
        const uint32_t m = std::min(chunk, n - s);
        gasalx_nv_strings p = *pat, t = *txt;
        p.offsets = pat->offsets + s;
        if (txt->offsets) t.offsets = txt->offsets + s;
        rc = gx::nv_traceback_device(*al, m, p, t, max_p, max_t, eng->nv_dir.as<uint8_t>(), eng->nv_row.as<int32_t>(),
                                     scores + s, sources + 2ull * s, sinks + 2ull * s, ops + (size_t)s * ops_stride,
                                     ops_stride, n_ops + s, st);
        if (rc) return rc;
    }
    return GASALX_OK;
}

int gasalx_nv_traceback_host(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t n, const gasalx_nv_strings *pat,
                             uint64_t pat_words, const gasalx_nv_strings *txt, uint64_t txt_words, int32_t *scores,
                             uint32_t *sources, uint32_t *sinks, uint8_t *ops, uint32_t ops_stride, uint32_t *n_ops) {
    if (!eng || !al || !pat || !txt || !pat->words || !pat->offsets || !txt->words || !scores || !sources || !sinks ||
        !ops || !n_ops) {
        gx::set_error("null argument");
        return GASALX_EINVAL;
    }
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    const uint32_t max_p = max_span(pat->offsets, n);
    const uint32_t max_t = txt->offsets ? max_span(txt->offsets, n) : txt->length;
    int rc = nv_tb_checks(al, max_p, max_t, ops_stride);
    if (rc) return rc;
    gasalx_nv_strings dp = *pat, dt = *txt;
    uint32_t *p32;
    if ((rc = stage_in(eng->nv_pw, pat->words, pat_words, st, &p32))) return rc; dp.words = p32;
    if ((rc = stage_in(eng->nv_po, pat->offsets, (size_t)n + 1, st, &p32))) return rc; dp.offsets = p32;
    if ((rc = stage_in(eng->nv_tw, txt->words, txt_words, st, &p32))) return rc; dt.words = p32;
    if ((rc = stage_in(eng->nv_to, txt->offsets, txt->offsets ? (size_t)n + 1 : 0, st, &p32))) return rc;
    dt.offsets = txt->offsets ? p32 : nullptr;
    CK(eng->nv_s.reserve((size_t)n * 4));
    CK(eng->nv_src.reserve((size_t)n * 8));
    CK(eng->nv_snk.reserve((size_t)n * 8));
    CK(eng->nv_ops.reserve((size_t)n * ops_stride + 64));
    CK(eng->nv_nops.reserve((size_t)n * 4));
    rc = gasalx_nv_traceback_device(eng, al, n, &dp, &dt, max_p, max_t, eng->nv_s.as<int32_t>(),
                                    eng->nv_src.as<uint32_t>(), eng->nv_snk.as<uint32_t>(), eng->nv_ops.as<uint8_t>(),
                                    ops_stride, eng->nv_nops.as<uint32_t>(), st);
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
    CK(hipMemcpyAsync(scores, eng->nv_s.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(sources, eng->nv_src.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(sinks, eng->nv_snk.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(ops, eng->nv_ops.p, (size_t)n * ops_stride, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(n_ops, eng->nv_nops.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

// nvbio BatchedBandedAlignmentTraceback<band> (nvtrace.hpp).  nvbio's checkpoints are int16
// pairs clamped at -32736 (gotoh_banded_inl.h:234-239): every score must stay above it.
static int nv_btb_checks(const gasalx_nv_aligner *al, uint32_t band, uint32_t max_p, uint32_t ops_stride) {
    if (band < 2 || band > 32) { gx::set_error("band length must be 2..32"); return GASALX_EINVAL; }
    if (((int64_t)max_p + band + 3) * nv_score_mag(al) > 32736) {
        gx::set_error("banded traceback: scores would leave nvbio's int16 checkpoints (lengths x |score|)");
        return GASALX_ERANGE;
    }
    if ((uint64_t)ops_stride < 2ull * max_p + band) {
        gx::set_error("banded traceback: ops_stride < 2 x max pattern length + band");
        return GASALX_EINVAL;
    }
    return GASALX_OK;
}

int gasalx_nv_banded_traceback_device(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t band, uint32_t n,
                                      const gasalx_nv_strings *pat, const gasalx_nv_strings *txt, uint32_t max_p,
                                      int32_t *scores, uint32_t *sources, uint32_t *sinks, uint8_t *ops,
                                      uint32_t ops_stride, uint32_t *n_ops, void *stream) {
    if (!eng || !al || !pat || !txt) { gx::set_error("null argument"); return GASALX_EINVAL; }
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = stream ? (hipStream_t)stream : eng->stream;
    if (!max_p) {   // read the offsets back (synchronises the stream)
        std::vector<uint32_t> po(n + 1);
        CK(hipMemcpyAsync(po.data(), pat->offsets, (n + 1) * 4ull, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        max_p = max_span(po.data(), n);
    }
    int rc = nv_btb_checks(al, band, max_p, ops_stride);
    if (rc) return rc;
    const uint64_t per = gasalx_nv_banded_traceback_workspace(max_p, band, 1);
    const uint32_t chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, kNvTbBudget / per));
    CK(eng->nv_dir.reserve((size_t)max_p * ((band + 3) / 4) * 4 * chunk + 64));
    for (uint32_t s = 0; s < n; s += chunk) {
        const uint32_t m = std::min(chunk, n - s);
        gasalx_nv_strings p = *pat, t = *txt;
        p.offsets = pat->offsets + s;
        if (txt->offsets) t.offsets = txt->offsets + s;
        rc = gx::nv_banded_traceback_device(*al, band, m, p, t, max_p, eng->nv_dir.as<uint32_t>(), scores + s,
                                            sources + 2ull * s, sinks + 2ull * s, ops + (size_t)s * ops_stride,
                                            ops_stride, n_ops + s, st);
        if (rc) return rc;
    }
    return GASALX_OK;
}

int gasalx_nv_banded_traceback_host(gasalx_engine *eng, const gasalx_nv_aligner *al, uint32_t band, uint32_t n,
                                    const gasalx_nv_strings *pat, uint64_t pat_words, const gasalx_nv_strings *txt,
                                    uint64_t txt_words, int32_t *scores, uint32_t *sources, uint32_t *sinks,
                                    uint8_t *ops, uint32_t ops_stride, uint32_t *n_ops) {
    if (!eng || !al || !pat || !txt || !pat->words || !pat->offsets || !txt->words || !scores || !sources || !sinks ||
        !ops || !n_ops) {
        gx::set_error("null argument");
        return GASALX_EINVAL;
    }
    const uint32_t max_p = n ? max_span(pat->offsets, n) : 0;
    int rc = nv_btb_checks(al, band, max_p, ops_stride);
    if (rc) return rc;
    if (n == 0) return GASALX_OK;
    CK(hipSetDevice(eng->device));
    hipStream_t st = eng->stream;
    gasalx_nv_strings dp = *pat, dt = *txt;
    uint32_t *p32;
    if ((rc = stage_in(eng->nv_pw, pat->words, pat_words, st, &p32))) return rc; dp.words = p32;
    if ((rc = stage_in(eng->nv_po, pat->offsets, (size_t)n + 1, st, &p32))) return rc; dp.offsets = p32;
    if ((rc = stage_in(eng->nv_tw, txt->words, txt_words, st, &p32))) return rc; dt.words = p32;
    if ((rc = stage_in(eng->nv_to, txt->offsets, txt->offsets ? (size_t)n + 1 : 0, st, &p32))) return rc;
    dt.offsets = txt->offsets ? p32 : nullptr;
    CK(eng->nv_s.reserve((size_t)n * 4));
    CK(eng->nv_src.reserve((size_t)n * 8));
    CK(eng->nv_snk.reserve((size_t)n * 8));
    CK(eng->nv_ops.reserve((size_t)n * ops_stride + 64));
    CK(eng->nv_nops.reserve((size_t)n * 4));
    rc = gasalx_nv_banded_traceback_device(eng, al, band, n, &dp, &dt, max_p, eng->nv_s.as<int32_t>(),
                                           eng->nv_src.as<uint32_t>(), eng->nv_snk.as<uint32_t>(),
                                           eng->nv_ops.as<uint8_t>(), ops_stride, eng->nv_nops.as<uint32_t>(), st);
    if (rc) { (void)hipStreamSynchronize(st); return rc; }
    CK(hipMemcpyAsync(scores, eng->nv_s.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(sources, eng->nv_src.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(sinks, eng->nv_snk.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(ops, eng->nv_ops.p, (size_t)n * ops_stride, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(n_ops, eng->nv_nops.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return GASALX_OK;
}

int gasalx_pairhmm_params(const uint8_t *bq, const uint8_t *iq, const uint8_t *dq, uint32_t n, float *qm,
                          float *delta, float *xiksi, float *alpha) {
    if (n && (!bq || !iq || !dq || !qm || !delta || !xiksi || !alpha)) return GASALX_EINVAL;
    float ph2pr[128];
    ph2pr_table(ph2pr);
    for (uint32_t k = 0; k < n; k++) {                                         // :415-419
        qm[k] = ph2pr[bq[k] & 127];
        delta[k] = ph2pr[iq[k] & 127];
        xiksi[k] = ph2pr[dq[k] & 127];
        alpha[k] = 1.0f - ph2pr[((int)(iq[k] & 127) + (int)(dq[k] & 127)) & 127];
    }
    return GASALX_OK;
}

int gasalx_host_alloc(uint64_t bytes, void **out) {
    if (!out) { gx::set_error("gasalx_host_alloc: null output"); return GASALX_EINVAL; }
    *out = nullptr;
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        *out = nullptr;
        gx::set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
        return GASALX_ENOMEM;
    }
    return GASALX_OK;
}

int gasalx_host_free(void *p) {
    if (!p) return GASALX_OK;
    hipError_t e = hipHostFree(p);
    if (e != hipSuccess) { gx::set_error(std::string("hipHostFree: ") + hipGetErrorString(e)); return GASALX_EDEVICE; }
    return GASALX_OK;
}

}  // extern "C"

// Diagnostics (gasalx.h): the last packed launch's "aligned here" flags of each workspace.
extern "C" int gasalx_packed_pairs(gasalx_engine *e, uint64_t *handled, uint64_t *total) {
    if (!e || !handled || !total) { gx::set_error("gasalx_packed_pairs: NULL argument"); return GASALX_EINVAL; }
    *handled = *total = 0;
    CK(hipSetDevice(e->device));
    auto one = [&](gx::Workspace &ws, hipStream_t st) -> int {
        if (st) CK(hipStreamSynchronize(st));
        if (!ws.pk_flags || !ws.misc.p) return GASALX_OK;
        std::vector<uint8_t> f(ws.pk_flags);
        CK(hipMemcpy(f.data(), ws.misc.p, f.size(), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < ws.pk_flags; i++) {
            // (a mixed-shape launch: the blocks from pk_b1 on cover pk_ppb2 pairs from pk_p1 on)
            const bool t2 = ws.pk_p1 != 0xFFFFFFFFu && i >= ws.pk_b1;
            const uint64_t lo = t2 ? (uint64_t)ws.pk_p1 + (uint64_t)(i - ws.pk_b1) * ws.pk_ppb2 : (uint64_t)i * ws.pk_ppb;
            const uint64_t hi = std::min<uint64_t>(lo + (t2 ? ws.pk_ppb2 : ws.pk_ppb), ws.pk_pairs);
            if (hi > lo && f[i]) *handled += hi - lo;
        }
        *total += ws.pk_pairs;
        ws.pk_flags = 0;   // read once: the next call counts only launches after this one
        return GASALX_OK;
    };
    int rc;
    if ((rc = one(e->ws, e->stream))) return rc;
    for (HostSlot &s : e->slot)
        if ((rc = one(s.ws, s.st))) return rc;
    return GASALX_OK;
}
