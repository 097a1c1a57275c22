// multi.cpp — one host process driving several MI355X devices (include/gasalx.h,
// gasalx_multi_*).
//
// pairs are independent, so a batch is split into contiguous
// ranges of pairs with equal cell counts (prefix sum of ql·tl), one range per
// device entry; one host thread per entry sets its device and runs the
// single-device host pipeline (gasalx_align_host: chunks of pairs on two
// streams, H2D of chunk k+1 overlapping the kernels of chunk k) into a
// disjoint range of the caller's result arrays.  This is the reference's only
// multi-GPU pattern for alignment — STAR's static split
// (Non-CDP/STAR/src/cuda-nw.cu:296-367: workload per GPU, cudaSetDevice, one
// stream per device, results into disjoint host ranges) — with the split
// balanced by cells instead of pair counts and GASAL2's per-thread storage
// (test_prog.cpp:203-231) as the per-device engine.
//
// The exchange step (optional, §8(e)): gasalx_multi_allgather gathers equal-
// size per-device buffers into every device, through RCCL (ncclCommInitAll
// over the device list, ncclAllGather in one group) when the entries name
// distinct devices and librccl is present, and through peer copies otherwise.
// librccl is opened at run time (dlopen): the library has no link dependency on
// it, and a process that already holds one (torch bundles librccl.so.1) shares
// that copy through the soname.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "gasalx.h"

namespace {

uint32_t pad8u(uint32_t x) { return (x + 7u) & ~7u; }

// RCCL entry points, resolved once per process
struct Rccl {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
};

const Rccl &rccl() {
    static const Rccl r = [] {
        Rccl x;
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
        if (!h) return x;
        x.init_all = (decltype(x.init_all))dlsym(h, "ncclCommInitAll");
        x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
        x.all_gather = (decltype(x.all_gather))dlsym(h, "ncclAllGather");
        x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
        x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        x.ok = x.init_all && x.destroy && x.all_gather && x.group_start && x.group_end && x.error_string;
        return x;
    }();
    return r;
}

// Contiguous [bounds[k], bounds[k+1]) ranges balancing Σ a[i]·b[i]: boundary k is one
// past the first pair whose inclusive prefix sum reaches k/world of the total
// (gasal_dist.shard_bounds applies the same integer rule).
void shard_rule(const uint32_t *a, const uint32_t *b, uint32_t n, int world, uint32_t *bounds) {
    std::vector<uint64_t> csum(n);
    uint64_t acc = 0;
    for (uint32_t i = 0; i < n; i++) csum[i] = (acc += (uint64_t)a[i] * b[i]);
    bounds[0] = 0;
    for (int k = 1; k < world; k++) {
        const unsigned __int128 target = (unsigned __int128)acc * (unsigned)k;
        // first i with csum[i] * world >= total * k
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if ((unsigned __int128)csum[mid] * (unsigned)world >= target) hi = mid;
            else lo = mid + 1;
        }
        bounds[k] = std::max(bounds[k - 1], n ? std::min(n, lo + 1) : 0u);
    }
    bounds[world] = n;
    for (int k = 1; k <= world; k++) bounds[k] = std::max(bounds[k], bounds[k - 1]);
}

// [lo, hi) byte range spanned by sequences [s, e) (offsets incl. pads, unpadded lengths)
void span(const uint32_t *off, const uint32_t *len, uint32_t s, uint32_t e, bool pad, uint64_t *lo,
          uint64_t *hi) {
    uint64_t a = ~0ull, z = 0;
    for (uint32_t i = s; i < e; i++) {
        a = std::min<uint64_t>(a, off[i]);
        z = std::max<uint64_t>(z, (uint64_t)off[i] + (pad ? pad8u(len[i]) : len[i]));
    }
    *lo = e > s ? a : 0;
    *hi = e > s ? z : 0;
}

std::vector<uint32_t> rebase(const uint32_t *off, uint32_t s, uint32_t e, uint64_t lo) {
    std::vector<uint32_t> r(e - s);
    for (uint32_t i = s; i < e; i++) r[i - s] = (uint32_t)(off[i] - lo);
    return r;
}

template <class T> T *at(T *p, uint64_t k) { return p ? p + k : nullptr; }

// the calling thread's current device, restored when the guard leaves scope (engine
// creation and ncclCommInitAll switch devices)
struct DeviceGuard {
    int dev = -1;
    bool had = false;
    DeviceGuard() { had = hipGetDevice(&dev) == hipSuccess; }
    ~DeviceGuard() { if (had) (void)hipSetDevice(dev); }
};

}  // namespace

struct gasalx_multi {
    std::vector<int> devices;
    std::vector<gasalx_engine *> engines;
    std::vector<ncclComm_t> comms;   // RCCL, one per entry (distinct devices only)
    void release() {
        if (!comms.empty() && rccl().ok)
            for (ncclComm_t c : comms) (void)rccl().destroy(c);
        comms.clear();
        for (gasalx_engine *e : engines) gasalx_engine_destroy(e);
        engines.clear();
    }
};

namespace {

// Run fn(i, start, end) on one host thread per device entry with a non-empty
// shard; the first failure's code and message become the caller's.
template <class F> int run_sharded(gasalx_multi *m, const std::vector<uint32_t> &bounds, F fn) {
    const int nd = (int)m->engines.size();
    std::vector<int> rc(nd, GASALX_OK);
    std::vector<std::string> msg(nd);
    std::vector<std::thread> th;
    for (int i = 0; i < nd; i++) {
        if (bounds[i + 1] <= bounds[i]) continue;
        th.emplace_back([&, i] {
            rc[i] = fn(i, bounds[i], bounds[i + 1]);
            if (rc[i]) msg[i] = gx::last_error();
        });
    }
    for (std::thread &t : th) t.join();
    for (int i = 0; i < nd; i++)
        if (rc[i]) {
            gx::set_error("device entry " + std::to_string(i) + " (device " + std::to_string(m->devices[i]) +
                          "): " + msg[i]);
            return rc[i];
        }
    return GASALX_OK;
}

}  // namespace

extern "C" {

int gasalx_shard_bounds(const uint32_t *a, const uint32_t *b, uint32_t n, int world, uint32_t *bounds) {
    if (world < 1 || !bounds || (n && (!a || !b))) { gx::set_error("gasalx_shard_bounds: bad argument"); return GASALX_EINVAL; }
    shard_rule(a, b, n, world, bounds);
    return GASALX_OK;
}

int gasalx_multi_create(const int *devices, int n_devices, uint32_t flags, gasalx_multi **out) {
    if (!out || !devices || n_devices < 1) { gx::set_error("gasalx_multi_create: bad argument"); return GASALX_EINVAL; }
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) { gx::set_error("no HIP device"); return GASALX_EDEVICE; }
    for (int i = 0; i < n_devices; i++)
        if (devices[i] < 0 || devices[i] >= count) {
            gx::set_error("gasalx_multi_create: device " + std::to_string(devices[i]) + " of " + std::to_string(count));
            return GASALX_EINVAL;
        }
    DeviceGuard guard;
    gasalx_multi *m = new (std::nothrow) gasalx_multi();
    if (!m) return GASALX_ENOMEM;
    m->devices.assign(devices, devices + n_devices);
    for (int i = 0; i < n_devices; i++) {
        gasalx_engine *e = nullptr;
        int rc = gasalx_engine_create(devices[i], &e);
        if (rc) { m->release(); delete m; return rc; }
        m->engines.push_back(e);
    }
    std::vector<int> sorted(m->devices);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if ((flags & GASALX_MULTI_RCCL) && distinct && rccl().ok) {
        m->comms.resize(n_devices);
        const ncclResult_t r = rccl().init_all(m->comms.data(), n_devices, m->devices.data());
        if (r != ncclSuccess) {   // no communicator: the gather falls back to peer copies
            m->comms.clear();
        }
    }
    *out = m;
    return GASALX_OK;
}

int gasalx_multi_destroy(gasalx_multi *m) {
    if (!m) return GASALX_OK;
    m->release();
    delete m;
    return GASALX_OK;
}

int gasalx_multi_info(const gasalx_multi *m, int *n_devices, int *uses_rccl) {
    if (!m) { gx::set_error("null argument"); return GASALX_EINVAL; }
    if (n_devices) *n_devices = (int)m->engines.size();
    if (uses_rccl) *uses_rccl = m->comms.empty() ? 0 : 1;
    return GASALX_OK;
}

int gasalx_multi_engine(gasalx_multi *m, int index, gasalx_engine **out) {
    if (!m || !out || index < 0 || index >= (int)m->engines.size()) { gx::set_error("bad argument"); return GASALX_EINVAL; }
    *out = m->engines[index];
    return GASALX_OK;
}

int gasalx_multi_align_host(gasalx_multi *m, const gasalx_params *params, const gasalx_batch *hb,
                            const gasalx_results *ho) {
    if (!m || !params || !hb || !ho) { gx::set_error("null argument"); return GASALX_EINVAL; }
    const uint32_t n = hb->n_alns;
    if (n == 0) return GASALX_OK;
    if (!hb->q_batch || !hb->t_batch || !hb->q_offsets || !hb->t_offsets || !hb->q_lens || !hb->t_lens) {
        gx::set_error("missing batch array");
        return GASALX_EINVAL;
    }
    const int nd = (int)m->engines.size();
    std::vector<uint32_t> bounds(nd + 1);
    shard_rule(hb->q_lens, hb->t_lens, n, nd, bounds.data());
    const bool tb = params->start_pos == 2 && ho->cigar;
    // CIGARs land at each pair's query offset (get_tb.h:94): shards must not share query bytes
    std::vector<std::pair<uint64_t, uint64_t>> qr(nd);
    for (int i = 0; i < nd; i++) span(hb->q_offsets, hb->q_lens, bounds[i], bounds[i + 1], true, &qr[i].first, &qr[i].second);
    if (tb)
        for (int i = 0; i < nd; i++)
            for (int j = i + 1; j < nd; j++)
                if (qr[i].first < qr[j].second && qr[j].first < qr[i].second && qr[i].second > qr[i].first &&
                    qr[j].second > qr[j].first) {
                    gx::set_error("WITH_TB across devices: shards share query bytes (one-to-many pairing); "
                                  "use one device or disjoint query slots");
                    return GASALX_EINVAL;
                }
    return run_sharded(m, bounds, [&](int i, uint32_t s, uint32_t e) -> int {
        uint64_t qlo = qr[i].first, qhi = qr[i].second, tlo, thi;
        span(hb->t_offsets, hb->t_lens, s, e, true, &tlo, &thi);
        const std::vector<uint32_t> qo = rebase(hb->q_offsets, s, e, qlo), to = rebase(hb->t_offsets, s, e, tlo);
        gasalx_batch b = *hb;
        b.q_batch = hb->q_batch + qlo;
        b.t_batch = hb->t_batch + tlo;
        b.q_offsets = qo.data();
        b.t_offsets = to.data();
        b.q_lens = hb->q_lens + s;
        b.t_lens = hb->t_lens + s;
        b.q_bytes = (uint32_t)(qhi - qlo);
        b.t_bytes = (uint32_t)(thi - tlo);
        b.n_alns = e - s;
        b.q_ops = at(hb->q_ops, s);
        b.t_ops = at(hb->t_ops, s);
        b.seed_scores = at(hb->seed_scores, s);
        gasalx_results r;
        r.aln_score = at(ho->aln_score, s);
        r.q_end = at(ho->q_end, s);
        r.t_end = at(ho->t_end, s);
        r.q_start = at(ho->q_start, s);
        r.t_start = at(ho->t_start, s);
        r.aln_score2 = at(ho->aln_score2, s);
        r.q_end2 = at(ho->q_end2, s);
        r.t_end2 = at(ho->t_end2, s);
        r.cigar = at(ho->cigar, qlo);
        r.n_cigar_ops = at(ho->n_cigar_ops, s);
        return gasalx_align_host(m->engines[i], params, &b, &r);
    });
}

int gasalx_multi_pairhmm_host(gasalx_multi *m, const gasalx_hmm_batch *hb, float *res) {
    if (!m || !hb || !res) { gx::set_error("null argument"); return GASALX_EINVAL; }
    const uint32_t n = hb->n_pairs;
    if (n == 0) return GASALX_OK;
    const int nd = (int)m->engines.size();
    std::vector<uint32_t> bounds(nd + 1);
    shard_rule(hb->read_lens, hb->hap_lens, n, nd, bounds.data());
    return run_sharded(m, bounds, [&](int i, uint32_t s, uint32_t e) -> int {
        uint64_t rlo, rhi, hlo, hhi;
        span(hb->read_offsets, hb->read_lens, s, e, false, &rlo, &rhi);
        span(hb->hap_offsets, hb->hap_lens, s, e, false, &hlo, &hhi);
        const std::vector<uint32_t> ro = rebase(hb->read_offsets, s, e, rlo), ho = rebase(hb->hap_offsets, s, e, hlo);
        gasalx_hmm_batch b = *hb;
        b.reads = hb->reads + rlo;
        b.qm = hb->qm + rlo;
        b.delta = hb->delta + rlo;
        b.xiksi = hb->xiksi + rlo;
        b.alpha = hb->alpha + rlo;
        b.read_offsets = ro.data();
        b.read_lens = hb->read_lens + s;
        b.haps = hb->haps + hlo;
        b.hap_offsets = ho.data();
        b.hap_lens = hb->hap_lens + s;
        b.read_bytes = (uint32_t)(rhi - rlo);
        b.hap_bytes = (uint32_t)(hhi - hlo);
        b.n_pairs = e - s;
        return gasalx_pairhmm_host(m->engines[i], &b, res + s);
    });
}

int gasalx_multi_pairhmm_quals_host(gasalx_multi *m, const gasalx_hmm_qual_batch *hb, float *res) {
    if (!m || !hb || !res) { gx::set_error("null argument"); return GASALX_EINVAL; }
    const uint32_t n = hb->n_pairs;
    if (n == 0) return GASALX_OK;
    const int nd = (int)m->engines.size();
    std::vector<uint32_t> bounds(nd + 1);
    shard_rule(hb->read_lens, hb->hap_lens, n, nd, bounds.data());
    return run_sharded(m, bounds, [&](int i, uint32_t s, uint32_t e) -> int {
        uint64_t rlo, rhi, hlo, hhi;
        span(hb->read_offsets, hb->read_lens, s, e, false, &rlo, &rhi);
        span(hb->hap_offsets, hb->hap_lens, s, e, false, &hlo, &hhi);
        const std::vector<uint32_t> ro = rebase(hb->read_offsets, s, e, rlo), ho = rebase(hb->hap_offsets, s, e, hlo);
        gasalx_hmm_qual_batch b = *hb;
        b.reads = hb->reads + rlo;
        b.base_quals = hb->base_quals + rlo;
        b.ins_quals = hb->ins_quals + rlo;
        b.del_quals = hb->del_quals + rlo;
        b.read_offsets = ro.data();
        b.read_lens = hb->read_lens + s;
        b.haps = hb->haps + hlo;
        b.hap_offsets = ho.data();
        b.hap_lens = hb->hap_lens + s;
        b.read_bytes = rhi - rlo;
        b.hap_bytes = hhi - hlo;
        b.n_pairs = e - s;
        b.max_read_len = 0;
        b.max_hap_len = 0;
        for (uint32_t k = s; k < e; k++) {
            b.max_read_len = std::max(b.max_read_len, hb->read_lens[k]);
            b.max_hap_len = std::max(b.max_hap_len, hb->hap_lens[k]);
        }
        return gasalx_pairhmm_quals_host(m->engines[i], &b, res + s);
    });
}

static int multi_allgather(gasalx_multi *m, const void *const *send, void *const *recv, uint64_t bytes,
                           void *const *streams);

// Device-resident shards: fn(i, stream) queues entry i's work on its stream (one host thread per
// entry with pairs: a call without max lengths reads them back, which synchronises that stream),
// then the optional gather of `elem`-byte results (gather_stride per entry), then, with no
// caller streams, the wait for every entry.
extern "C++" template <class F>
static int run_device(gasalx_multi *m, const uint32_t *counts, void *const *streams, const void *const *send,
                      void *const *gather, uint32_t gather_stride, uint32_t elem, F fn) {
    const int nd = (int)m->engines.size();
    std::vector<hipStream_t> st(nd);
    for (int i = 0; i < nd; i++) st[i] = streams && streams[i] ? (hipStream_t)streams[i] : gx::engine_stream(m->engines[i]);
    if (gather) {
        for (int i = 0; i < nd; i++)
            if (counts[i] > gather_stride || !gather[i] || (counts[i] && !send[i])) {
                gx::set_error("gather: every entry needs a result buffer of gather_stride >= its pairs and a receive buffer");
                return GASALX_EINVAL;
            }
    }
    std::vector<uint32_t> bounds(nd + 1);
    for (int i = 0; i < nd; i++) bounds[i + 1] = bounds[i] + 1;   // one "shard" per entry (run_sharded's form)
    int rc = run_sharded(m, bounds, [&](int i, uint32_t, uint32_t) -> int {
        return counts[i] ? fn(i, st[i]) : GASALX_OK;
    });
    if (rc) return rc;
    if (gather) {
        std::vector<void *> sp(nd);
        for (int i = 0; i < nd; i++) sp[i] = st[i];
        rc = multi_allgather(m, send, (void *const *)gather, (uint64_t)gather_stride * elem, sp.data());
        if (rc) return rc;
    }
    if (!streams)
        for (int i = 0; i < nd; i++) {
            (void)hipSetDevice(m->devices[i]);
            const hipError_t e = hipStreamSynchronize(st[i]);
            if (e != hipSuccess) { gx::set_error(std::string("multi device call: ") + hipGetErrorString(e)); return GASALX_EDEVICE; }
        }
    return GASALX_OK;
}

int gasalx_multi_align_device(gasalx_multi *m, const gasalx_params *params, const gasalx_batch *batches,
                              const gasalx_results *outs, void *const *streams, int32_t *const *gather,
                              uint32_t gather_stride) {
    if (!m || !params || !batches || !outs) { gx::set_error("null argument"); return GASALX_EINVAL; }
    DeviceGuard guard;
    const int nd = (int)m->engines.size();
    std::vector<uint32_t> counts(nd);
    std::vector<const void *> send(nd);
    for (int i = 0; i < nd; i++) { counts[i] = batches[i].n_alns; send[i] = outs[i].aln_score; }
    return run_device(m, counts.data(), streams, send.data(), (void *const *)gather, gather_stride, 4,
                      [&](int i, hipStream_t st) { return gasalx_align_device(m->engines[i], params, &batches[i], &outs[i], st); });
}

int gasalx_multi_pairhmm_device(gasalx_multi *m, const gasalx_hmm_batch *batches, float *const *results,
                                void *const *streams, float *const *gather, uint32_t gather_stride) {
    if (!m || !batches || !results) { gx::set_error("null argument"); return GASALX_EINVAL; }
    DeviceGuard guard;
    const int nd = (int)m->engines.size();
    std::vector<uint32_t> counts(nd);
    std::vector<const void *> send(nd);
    for (int i = 0; i < nd; i++) { counts[i] = batches[i].n_pairs; send[i] = results[i]; }
    return run_device(m, counts.data(), streams, send.data(), (void *const *)gather, gather_stride, 4,
                      [&](int i, hipStream_t st) { return gasalx_pairhmm_device(m->engines[i], &batches[i], results[i], st); });
}

// (the calling thread's current device is restored on every exit: a torch caller's
// current_device must not move to the last entry's device)
int gasalx_multi_allgather(gasalx_multi *m, const void *const *send, void *const *recv, uint64_t bytes,
                           void *const *streams) {
    DeviceGuard guard;
    return multi_allgather(m, send, recv, bytes, streams);
}

static int multi_allgather(gasalx_multi *m, const void *const *send, void *const *recv, uint64_t bytes,
                           void *const *streams) {
    if (!m || !send || !recv) { gx::set_error("null argument"); return GASALX_EINVAL; }
    const int nd = (int)m->engines.size();
    for (int i = 0; i < nd; i++)
        if (!send[i] || !recv[i]) { gx::set_error("gasalx_multi_allgather: null buffer"); return GASALX_EINVAL; }
    std::vector<hipStream_t> st(nd);
    for (int i = 0; i < nd; i++) {
        st[i] = streams && streams[i] ? (hipStream_t)streams[i] : gx::engine_stream(m->engines[i]);
    }
    if (!m->comms.empty()) {
        const Rccl &r = rccl();
        ncclResult_t res = r.group_start();
        for (int i = 0; i < nd && res == ncclSuccess; i++) {
            if (hipSetDevice(m->devices[i]) != hipSuccess) {
                (void)r.group_end();   // never leave the thread's RCCL group open
                gx::set_error("hipSetDevice");
                return GASALX_EDEVICE;
            }
            res = r.all_gather(send[i], recv[i], bytes, ncclUint8, m->comms[i], st[i]);
        }
        const ncclResult_t end = r.group_end();
        if (res == ncclSuccess) res = end;
        if (res != ncclSuccess) {
            gx::set_error(std::string("ncclAllGather: ") + r.error_string(res));
            return GASALX_EDEVICE;
        }
    } else {
        // peer copies: entry j receives every entry's buffer at j's offset i·bytes, on
        // its own stream, after the work queued on every sender's stream
        std::vector<hipEvent_t> ev(nd, nullptr);
        auto drop = [&] {
            for (hipEvent_t x : ev)
                if (x) (void)hipEventDestroy(x);
        };
        for (int i = 0; i < nd; i++) {
            (void)hipSetDevice(m->devices[i]);
            if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(ev[i], st[i]) != hipSuccess) {
                drop();
                gx::set_error("allgather: event");
                return GASALX_EDEVICE;
            }
        }
        for (int j = 0; j < nd; j++) {
            (void)hipSetDevice(m->devices[j]);
            for (int i = 0; i < nd; i++)
                if (i != j && hipStreamWaitEvent(st[j], ev[i], 0) != hipSuccess) {
                    drop();
                    gx::set_error("allgather: stream wait");
                    return GASALX_EDEVICE;
                }
        }
        drop();   // destroying a recorded event is safe; the waits are queued
        for (int j = 0; j < nd; j++) {
            if (hipSetDevice(m->devices[j]) != hipSuccess) { gx::set_error("hipSetDevice"); return GASALX_EDEVICE; }
            for (int i = 0; i < nd; i++) {
                hipError_t e = hipMemcpyPeerAsync(static_cast<uint8_t *>(recv[j]) + (uint64_t)i * bytes, m->devices[j],
                                                  send[i], m->devices[i], bytes, st[j]);
                if (e != hipSuccess) { gx::set_error(std::string("hipMemcpyPeerAsync: ") + hipGetErrorString(e)); return GASALX_EDEVICE; }
            }
        }
    }
    if (!streams)
        for (int i = 0; i < nd; i++) {
            (void)hipSetDevice(m->devices[i]);
            hipError_t e = hipStreamSynchronize(st[i]);
            if (e != hipSuccess) { gx::set_error(std::string("allgather: ") + hipGetErrorString(e)); return GASALX_EDEVICE; }
        }
    return GASALX_OK;
}

}  // extern "C"
