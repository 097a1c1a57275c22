// gasal_api.cpp — the reference's C++ host API (gasal_header.h), re-built on
// the MI355X engine.  Observable behaviour follows the reference host code
// (Non-CDP/GASAL2/src/{ctors,host_batch,res,interfaces}.cpp, gasal_align.cu):
// same buffer ownership, growth policy and warnings, is_free/-1/-2 protocol,
// exit(EXIT_FAILURE) on errors; kernels and the launch plan are this engine's.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>

#include "../../include/gasal_header.h"
#include "../../include/res.h"
#include "engine.hpp"
#include "gasalx.h"

namespace {

// Per-device scoring constants (the reference's __constant__ symbols,
// gasal_kernels.h:29-33, are per device context).
struct DeviceScores { gasal_subst_scores s; bool set; };
DeviceScores g_scores[64];
std::mutex g_mu;
std::map<const gasal_gpu_storage_t *, gx::Workspace *> g_ws;   // storage -> engine workspace

int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}

gx::Workspace *workspace_for(const gasal_gpu_storage_t *s) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_ws.find(s);
    if (it != g_ws.end()) return it->second;
    gx::Workspace *w = new gx::Workspace();
    w->device = current_device();
    g_ws[s] = w;
    return w;
}

void drop_workspace(const gasal_gpu_storage_t *s) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_ws.find(s);
    if (it == g_ws.end()) return;
    it->second->release_all();
    delete it->second;
    g_ws.erase(it);
}

template <class T> void host_alloc(T **p, size_t count) {
    CHECKHIPERROR(hipHostMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault));
}
template <class T> void dev_alloc(T **p, size_t count) {
    CHECKHIPERROR(hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T)));
    CHECKHIPERROR(hipMemset(*p, 0, std::max<size_t>(count, 1) * sizeof(T)));
}

// Arrays of one storage that travel together (the four lens/offsets arrays, the result arrays)
// live in one allocation, `cap` elements apart, so that a batch moves them with one copy instead
// of one per array (each hipMemcpyAsync is a DMA command of its own: the boundary bench's 5,000-
// pair batches spent more engine time on the small copies than on their bytes).  The arrays
// keep their own pointers (the reference's fields); the block is freed with its last array.
struct Block { void *base; size_t cap; int refs; bool dev; };
std::mutex g_bmu;
std::map<const void *, Block *> g_blk;   // every array pointer of a block -> its block

template <class T> void block_alloc(bool dev, size_t cap, std::initializer_list<T **> arrays) {
    cap = std::max<size_t>(cap, 1);
    T *base = nullptr;
    if (dev) dev_alloc(&base, cap * arrays.size());
    else host_alloc(&base, cap * arrays.size());
    Block *b = new Block{base, cap, (int)arrays.size(), dev};
    std::lock_guard<std::mutex> lk(g_bmu);
    size_t i = 0;
    for (T **a : arrays) { *a = base + cap * i++; g_blk[*a] = b; }
}
// true when p was an array of a block (released; the block freed with its last array)
bool block_release(const void *p) {
    Block *b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_bmu);
        auto it = g_blk.find(p);
        if (it == g_blk.end()) return false;
        b = it->second;
        g_blk.erase(it);
        if (--b->refs > 0) return true;
    }
    if (b->dev) CHECKHIPERROR(hipFree(b->base));
    else CHECKHIPERROR(hipHostFree(b->base));
    delete b;
    return true;
}
// elements per array when a[0..k) are consecutive arrays of one block, else 0
template <class T> size_t block_run(std::initializer_list<T *> a) {
    std::lock_guard<std::mutex> lk(g_bmu);
    const T *first = *a.begin();
    auto it = g_blk.find(first);
    if (it == g_blk.end()) return 0;
    const size_t cap = it->second->cap;
    size_t i = 0;
    for (T *p : a) {
        auto jt = g_blk.find(p);
        if (jt == g_blk.end() || jt->second != it->second || p != first + cap * i) return 0;
        ++i;
    }
    return cap;
}

template <class T> void host_free(T *&p) { if (p && !block_release(p)) CHECKHIPERROR(hipHostFree(p)); p = nullptr; }
template <class T> void dev_free(T *&p) { if (p && !block_release(p)) CHECKHIPERROR(hipFree(p)); p = nullptr; }

uint32_t pad8(uint32_t x) { return x % 8 ? x + (8 - x % 8) : x; }

}  // namespace

// ============================================================== res.cpp ====
// the result arrays in one block per side, in the order score, q_end, t_end, q_start, t_start
// (the fields res.cpp:26-67 / :115-138 allocate), so gasal_aln_async returns them with one copy
static void res_block(bool dev, uint32_t max_n_alns, Parameters *params, gasal_res_t *res) {
    const bool ends = params->algo != GLOBAL;
    const bool starts = ends && (params->start_pos == WITH_START || params->start_pos == WITH_TB);
    if (starts)
        block_alloc<int32_t>(dev, max_n_alns, {&res->aln_score, &res->query_batch_end, &res->target_batch_end,
                                               &res->query_batch_start, &res->target_batch_start});
    else if (ends)
        block_alloc<int32_t>(dev, max_n_alns, {&res->aln_score, &res->query_batch_end, &res->target_batch_end});
    else
        block_alloc<int32_t>(dev, max_n_alns, {&res->aln_score});
}

gasal_res_t *gasal_res_new_host(uint32_t max_n_alns, Parameters *params) {
    gasal_res_t *res = (gasal_res_t *)calloc(1, sizeof(gasal_res_t));
    if (!res) { fprintf(stderr, "Malloc error on res host "); exit(1); }
    res_block(false, max_n_alns, params, res);
    if (params->start_pos == WITH_TB) host_alloc(&res->n_cigar_ops, max_n_alns);   // :68-70
    return res;
}

gasal_res_t *gasal_res_new_device_cpy(uint32_t max_n_alns, Parameters *params) {
    gasal_res_t *res = (gasal_res_t *)calloc(1, sizeof(gasal_res_t));
    res_block(true, max_n_alns, params, res);
    return res;
}

gasal_res_t *gasal_res_new_device(gasal_res_t *device_cpy) {
    // a device-resident struct holding the device pointers (res.cpp:76-101)
    gasal_res_t *d = nullptr;
    CHECKHIPERROR(hipMalloc((void **)&d, sizeof(gasal_res_t)));
    gasal_res_t tmp;
    std::memset(&tmp, 0, sizeof(tmp));
    tmp.aln_score = device_cpy->aln_score;
    tmp.query_batch_start = device_cpy->query_batch_start;
    tmp.target_batch_start = device_cpy->target_batch_start;
    tmp.query_batch_end = device_cpy->query_batch_end;
    tmp.target_batch_end = device_cpy->target_batch_end;
    CHECKHIPERROR(hipMemcpy(d, &tmp, sizeof(tmp), hipMemcpyHostToDevice));
    return d;
}

void gasal_res_destroy_host(gasal_res_t *res) {
    if (!res) return;
    host_free(res->aln_score);
    host_free(res->query_batch_start);
    host_free(res->target_batch_start);
    host_free(res->query_batch_end);
    host_free(res->target_batch_end);
    host_free(res->n_cigar_ops);
    host_free(res->cigar);
    free(res);
}

void gasal_res_destroy_device(gasal_res_t *device_res, gasal_res_t *device_cpy) {
    if (!device_cpy || !device_res) return;
    dev_free(device_cpy->aln_score);
    dev_free(device_cpy->query_batch_start);
    dev_free(device_cpy->target_batch_start);
    dev_free(device_cpy->query_batch_end);
    dev_free(device_cpy->target_batch_end);
    dev_free(device_cpy->cigar);
    CHECKHIPERROR(hipFree(device_res));
    free(device_cpy);
}

// ======================================================= host_batch.cpp ====
host_batch_t *gasal_host_batch_new(uint32_t batch_bytes, uint32_t offset) {
    host_batch_t *res = (host_batch_t *)calloc(1, sizeof(host_batch_t));
    host_alloc(&res->data, batch_bytes);
    res->page_size = batch_bytes;
    res->data_size = 0;
    res->is_locked = 0;
    res->offset = offset;
    res->next = NULL;
    return res;
}

void gasal_host_batch_destroy(host_batch_t *res) {
    if (res == NULL) { fprintf(stderr, "[GASAL ERROR] Trying to free a NULL pointer\n"); exit(1); }
    while (res) {
        host_batch_t *nx = res->next;
        host_free(res->data);
        free(res);
        res = nx;
    }
}

host_batch_t *gasal_host_batch_getlast(host_batch_t *arg) {
    while (arg->next) arg = arg->next;
    return arg;
}

void gasal_host_batch_reset(gasal_gpu_storage_t *gpu_storage) {
    for (host_batch_t *p : {gpu_storage->extensible_host_unpacked_query_batch,
                            gpu_storage->extensible_host_unpacked_target_batch})
        for (; p; p = p->next) { p->data_size = 0; p->offset = 0; p->is_locked = 0; }
}

// Appends one sequence and its N_CODE padding (host_batch.cpp:79-153).
uint32_t gasal_host_batch_fill(gasal_gpu_storage_t *gpu_storage, uint32_t idx, const char *data, uint32_t size,
                               data_source SRC) {
    host_batch_t *cur = NULL;
    uint32_t *total_bytes = NULL;
    if (SRC == QUERY) { cur = gpu_storage->extensible_host_unpacked_query_batch; total_bytes = &gpu_storage->host_max_query_batch_bytes; }
    else if (SRC == TARGET) { cur = gpu_storage->extensible_host_unpacked_target_batch; total_bytes = &gpu_storage->host_max_target_batch_bytes; }
    else return idx;
    const uint32_t pads = (8 - size % 8) % 8;
    const uint32_t need = size + pads;
    while (cur->is_locked) cur = cur->next;
    if (cur->next == NULL && cur->page_size - cur->data_size < need) {
        fprintf(stderr,
                "[GASAL WARNING:] Trying to write %d bytes while only %d remain (%s) (block size %d, filled %d bytes).\n"
                "                 Allocating a new block of size %d, total size available reaches %d. Doing this "
                "repeadtedly slows down the execution.\n",
                need, cur->page_size - cur->data_size, SRC == QUERY ? "query" : "target", cur->page_size,
                cur->data_size, cur->page_size * 2, *total_bytes + cur->page_size * 2);
        host_batch_t *nx = gasal_host_batch_new(cur->page_size * 2, cur->offset + cur->data_size);
        cur->next = nx;
        cur->is_locked = 1;
        *total_bytes += cur->page_size * 2;
        cur = nx;
    }
    if (cur->next != NULL && cur->page_size - cur->data_size < need) {
        cur->next->offset = cur->offset + cur->data_size;
        cur->is_locked = 1;
        cur = cur->next;
    }
    if (cur->page_size - cur->data_size >= need) {
        std::memcpy(&cur->data[idx - cur->offset], data, size);
        std::memset(&cur->data[idx + size - cur->offset], 0x4E /* N_CODE */, pads);
        idx += need;
        cur->data_size += need;
    }
    return idx;
}

uint32_t gasal_host_batch_add(gasal_gpu_storage_t *gpu_storage, uint32_t idx, const char *data, uint32_t size,
                              data_source SRC) {
    host_batch_t *cur = NULL;
    uint32_t *total_bytes = NULL;
    if (SRC == QUERY) { cur = gpu_storage->extensible_host_unpacked_query_batch; total_bytes = &gpu_storage->host_max_query_batch_bytes; }
    else if (SRC == TARGET) { cur = gpu_storage->extensible_host_unpacked_target_batch; total_bytes = &gpu_storage->host_max_target_batch_bytes; }
    else return idx;
    for (;;) {   // host_batch.cpp:162-223
        if (*total_bytes >= idx + size && (cur->next == NULL || cur->next->offset >= idx + size)) {
            std::memcpy(&cur->data[idx - cur->offset], data, size);
            return idx + size;
        } else if (*total_bytes >= idx + size && cur->next != NULL && cur->next->offset < idx + size) {
            cur = cur->next;
        } else {
            fprintf(stderr,
                    "[GASAL WARNING:] Trying to write %d bytes at position %d on host memory (%s) while only  %d "
                    "bytes are available. Therefore, allocating %d bytes more on CPU. Repeating this many times can "
                    "provoke a degradation of performance.\n",
                    size, idx, SRC == QUERY ? "query" : "target", *total_bytes, *total_bytes * 2);
            *total_bytes += *total_bytes;
            while (*total_bytes < size) *total_bytes += *total_bytes;
            host_batch_t *nx = gasal_host_batch_new(*total_bytes, idx);
            cur->next = nx;
            cur = nx;
        }
    }
}

uint32_t gasal_host_batch_addbase(gasal_gpu_storage_t *gpu_storage, uint32_t idx, const char base, data_source SRC) {
    return gasal_host_batch_add(gpu_storage, idx, &base, 1, SRC);
}

void gasal_host_batch_print(host_batch_t *res) {
    fprintf(stderr, "[GASAL PRINT] Page data: offset=%d, next_offset=%d, data size=%d, page size=%d\n", res->offset,
            (res->next != NULL ? (int)res->next->offset : -1), res->data_size, res->page_size);
}

void gasal_host_batch_printall(host_batch_t *res) {
    for (; res; res = res->next) {
        gasal_host_batch_print(res);
        if (res->next) fprintf(stderr, "+--->");
    }
}

// ======================================================= interfaces.cpp ====
template <class T> static T *host_realloc(T *src, int new_n, int old_n) {
    if (new_n < old_n) {
        fprintf(stderr, "[GASAL ERROR] cudoHostRealloc: invalid sizes. New size < old size (%d < %d)", new_n, old_n);
        exit(EXIT_FAILURE);
    }
    T *dst = nullptr;
    host_alloc(&dst, (size_t)new_n);
    if (src) { std::memcpy(dst, src, (size_t)old_n * sizeof(T)); CHECKHIPERROR(hipHostFree(src)); }
    return dst;
}

void gasal_host_alns_resize(gasal_gpu_storage_t *gs, int new_max_alns, Parameters *params) {
    fprintf(stderr, "[GASAL WARNING] Resizing gpu_storage from %d sequences to %d sequences... ", gs->host_max_n_alns,
            new_max_alns);
    gs->host_query_op = host_realloc(gs->host_query_op, new_max_alns, gs->host_max_n_alns);
    gs->host_target_op = host_realloc(gs->host_target_op, new_max_alns, gs->host_max_n_alns);
    if (params->algo == KSW) gs->host_seed_scores = host_realloc(gs->host_seed_scores, new_max_alns, gs->host_max_n_alns);
    {
        // the four lens / offsets arrays move to a new block together (contents kept, as cudaHostRealloc)
        uint32_t *ql = gs->host_query_batch_lens, *tl = gs->host_target_batch_lens;
        uint32_t *qo = gs->host_query_batch_offsets, *to = gs->host_target_batch_offsets;
        if (new_max_alns < (int)gs->host_max_n_alns) {
            fprintf(stderr, "[GASAL ERROR] cudoHostRealloc: invalid sizes. New size < old size (%d < %d)", new_max_alns,
                    gs->host_max_n_alns);
            exit(EXIT_FAILURE);
        }
        block_alloc<uint32_t>(false, new_max_alns, {&gs->host_query_batch_lens, &gs->host_target_batch_lens,
                                                    &gs->host_query_batch_offsets, &gs->host_target_batch_offsets});
        const size_t old_bytes = (size_t)gs->host_max_n_alns * 4;
        std::memcpy(gs->host_query_batch_lens, ql, old_bytes);
        std::memcpy(gs->host_target_batch_lens, tl, old_bytes);
        std::memcpy(gs->host_query_batch_offsets, qo, old_bytes);
        std::memcpy(gs->host_target_batch_offsets, to, old_bytes);
        host_free(ql); host_free(tl); host_free(qo); host_free(to);
    }
    uint8_t *cigar = gs->host_res ? gs->host_res->cigar : nullptr;
    if (gs->host_res) gs->host_res->cigar = nullptr;
    gasal_res_destroy_host(gs->host_res);
    gs->host_res = gasal_res_new_host(new_max_alns, params);
    gs->host_res->cigar = cigar;
    gasal_res_destroy_device(gs->device_res, gs->device_cpy);
    gs->device_cpy = gasal_res_new_device_cpy(new_max_alns, params);
    gs->device_res = gasal_res_new_device(gs->device_cpy);
    if (params->secondBest) {
        gasal_res_destroy_host(gs->host_res_second);
        gasal_res_destroy_device(gs->device_res_second, gs->device_cpy_second);
        gs->host_res_second = gasal_res_new_host(new_max_alns, params);
        gs->device_cpy_second = gasal_res_new_device_cpy(new_max_alns, params);
        gs->device_res_second = gasal_res_new_device(gs->device_cpy_second);
    } else {
        gs->host_res_second = NULL;
        gs->device_cpy_second = NULL;
        gs->device_res_second = NULL;
    }
    gs->host_max_n_alns = new_max_alns;
    // device-side lens/offsets follow on the next gasal_aln_async (gpu_max_n_alns growth)
    fprintf(stderr, " done. This can harm performance.\n");
}

void gasal_op_fill(gasal_gpu_storage_t *gs, uint8_t *data, uint32_t nbr_seqs_in_stream, data_source SRC) {
    uint8_t *dst = SRC == QUERY ? gs->host_query_op : (SRC == TARGET ? gs->host_target_op : NULL);
    if (dst) std::memcpy(dst, data, nbr_seqs_in_stream);
}

void gasal_set_device(int gpu_select, bool isPrintingProp) {
    if (isPrintingProp) {
        int num = 0;
        (void)hipGetDeviceCount(&num);
        fprintf(stderr, "Found %d GPUs\n", num);
        if (gpu_select > num - 1) {
            fprintf(stderr, "Error: can't select device %d when only %d devices are selected (range from 0 to %d)\n",
                    gpu_select, num, num - 1);
            exit(EXIT_FAILURE);
        }
        if (num > 0) {
            hipDeviceProp_t prop;
            for (int d = 0; d < num; d++) {
                (void)hipGetDeviceProperties(&prop, d);
                fprintf(stderr, "\tGPU %d: %s\n", d, prop.name);
            }
            (void)hipGetDeviceProperties(&prop, gpu_select);
            fprintf(stderr, "Selected device %d : %s\n", gpu_select, prop.name);
            (void)hipSetDevice(gpu_select);
        }
    } else {
        (void)hipSetDevice(gpu_select);
    }
}

// ============================================================ ctors.cpp ====
gasal_gpu_storage_v gasal_init_gpu_storage_v(int n_streams) {
    gasal_gpu_storage_v v;
    v.a = (gasal_gpu_storage_t *)calloc(n_streams, sizeof(gasal_gpu_storage_t));
    v.n = n_streams;
    return v;
}

void gasal_init_streams(gasal_gpu_storage_v *vec, int max_query_len, int max_target_len, int max_n_alns,
                        Parameters *params) {
    const uint32_t q8 = pad8((uint32_t)max_query_len), t8 = pad8((uint32_t)max_target_len);
    const uint32_t qbytes = (uint32_t)max_n_alns * q8, tbytes = (uint32_t)max_n_alns * t8;   // ctors.cpp:33-38
    for (int i = 0; i < vec->n; i++) {
        gasal_gpu_storage_t *gs = &vec->a[i];
        gs->extensible_host_unpacked_query_batch = gasal_host_batch_new(qbytes, 0);
        gs->extensible_host_unpacked_target_batch = gasal_host_batch_new(tbytes, 0);
        dev_alloc(&gs->unpacked_query_batch, qbytes);
        dev_alloc(&gs->unpacked_target_batch, tbytes);
        host_alloc(&gs->host_query_op, max_n_alns);
        host_alloc(&gs->host_target_op, max_n_alns);
        std::memset(gs->host_query_op, 0, max_n_alns);
        std::memset(gs->host_target_op, 0, max_n_alns);
        dev_alloc(&gs->query_op, max_n_alns);
        dev_alloc(&gs->target_op, max_n_alns);
        if (params->isPacked) {                                      // ctors.cpp:64-72
            gs->packed_query_batch = (uint32_t *)gs->unpacked_query_batch;
            gs->packed_target_batch = (uint32_t *)gs->unpacked_target_batch;
        } else {
            dev_alloc(&gs->packed_query_batch, qbytes / 8);
            dev_alloc(&gs->packed_target_batch, tbytes / 8);
        }
        if (params->algo == KSW) {
            host_alloc(&gs->host_seed_scores, max_n_alns);
            dev_alloc(&gs->seed_scores, max_n_alns);
        } else {
            gs->host_seed_scores = NULL;
            gs->seed_scores = NULL;
        }
        block_alloc<uint32_t>(false, max_n_alns, {&gs->host_query_batch_lens, &gs->host_target_batch_lens,
                                                  &gs->host_query_batch_offsets, &gs->host_target_batch_offsets});
        block_alloc<uint32_t>(true, max_n_alns, {&gs->query_batch_lens, &gs->target_batch_lens,
                                                 &gs->query_batch_offsets, &gs->target_batch_offsets});
        gs->host_res = gasal_res_new_host(max_n_alns, params);
        if (params->start_pos == WITH_TB) host_alloc(&gs->host_res->cigar, qbytes);
        gs->device_cpy = gasal_res_new_device_cpy(max_n_alns, params);
        gs->device_res = gasal_res_new_device(gs->device_cpy);
        if (params->secondBest) {
            gs->host_res_second = gasal_res_new_host(max_n_alns, params);
            gs->device_cpy_second = gasal_res_new_device_cpy(max_n_alns, params);
            gs->device_res_second = gasal_res_new_device(gs->device_cpy_second);
        } else {
            gs->host_res_second = NULL;
            gs->device_cpy_second = NULL;
            gs->device_res_second = NULL;
        }
        if (params->start_pos == WITH_TB) {
            // size bookkeeping as the reference (ctors.cpp:112-115); the direction
            // words themselves live in the engine workspace, grown on demand
            gs->packed_tb_matrix_size = (uint64_t)std::ceil((double)((uint64_t)q8 * t8) / 32.0) * max_n_alns;
        }
        gs->packed_tb_matrices = NULL;
        CHECKHIPERROR(hipStreamCreate(&gs->str));
        gs->is_free = 1;
        gs->host_max_query_batch_bytes = qbytes;
        gs->host_max_target_batch_bytes = tbytes;
        gs->host_max_n_alns = max_n_alns;
        gs->gpu_max_query_batch_bytes = qbytes;
        gs->gpu_max_target_batch_bytes = tbytes;
        gs->gpu_max_n_alns = max_n_alns;
        gs->current_n_alns = 0;
        (void)workspace_for(gs);
    }
}

void gasal_destroy_streams(gasal_gpu_storage_v *vec, Parameters *params) {
    for (int i = 0; i < vec->n; i++) {
        gasal_gpu_storage_t *gs = &vec->a[i];
        if (gs->str) CHECKHIPERROR(hipStreamSynchronize(gs->str));
        gasal_host_batch_destroy(gs->extensible_host_unpacked_query_batch);
        gasal_host_batch_destroy(gs->extensible_host_unpacked_target_batch);
        gasal_res_destroy_host(gs->host_res);
        gasal_res_destroy_device(gs->device_res, gs->device_cpy);
        if (params->secondBest) {
            gasal_res_destroy_host(gs->host_res_second);
            gasal_res_destroy_device(gs->device_res_second, gs->device_cpy_second);
        }
        dev_free(gs->seed_scores);
        host_free(gs->host_seed_scores);
        dev_free(gs->query_op);
        dev_free(gs->target_op);
        host_free(gs->host_query_op);
        host_free(gs->host_target_op);
        host_free(gs->host_query_batch_offsets);
        host_free(gs->host_target_batch_offsets);
        host_free(gs->host_query_batch_lens);
        host_free(gs->host_target_batch_lens);
        if (!params->isPacked) {
            dev_free(gs->packed_query_batch);
            dev_free(gs->packed_target_batch);
        }
        dev_free(gs->unpacked_query_batch);
        dev_free(gs->unpacked_target_batch);
        dev_free(gs->query_batch_offsets);
        dev_free(gs->target_batch_offsets);
        dev_free(gs->query_batch_lens);
        dev_free(gs->target_batch_lens);
        if (gs->str) CHECKHIPERROR(hipStreamDestroy(gs->str));
        gs->str = NULL;
        drop_workspace(gs);
    }
}

void gasal_destroy_gpu_storage_v(gasal_gpu_storage_v *vec) {
    if (vec->a != NULL) free(vec->a);
    vec->a = NULL;
}

void gasal_gpu_mem_alloc(gasal_gpu_storage_t *gs, int qb, int tb, int na, Parameters *params) {
    dev_alloc(&gs->unpacked_query_batch, qb);
    dev_alloc(&gs->unpacked_target_batch, tb);
    dev_alloc(&gs->packed_query_batch, qb / 8);
    dev_alloc(&gs->packed_target_batch, tb / 8);
    block_alloc<uint32_t>(true, na, {&gs->query_batch_lens, &gs->target_batch_lens, &gs->query_batch_offsets,
                                     &gs->target_batch_offsets});
    if (!gs->device_cpy) gs->device_cpy = gasal_res_new_device_cpy(na, params);
    gs->device_res = gasal_res_new_device(gs->device_cpy);
    gs->gpu_max_query_batch_bytes = qb;
    gs->gpu_max_target_batch_bytes = tb;
    gs->gpu_max_n_alns = na;
}

void gasal_gpu_mem_free(gasal_gpu_storage_t *gs, Parameters *params) {
    dev_free(gs->unpacked_query_batch);
    dev_free(gs->unpacked_target_batch);
    dev_free(gs->packed_query_batch);
    dev_free(gs->packed_target_batch);
    dev_free(gs->query_batch_offsets);
    dev_free(gs->target_batch_offsets);
    dev_free(gs->query_batch_lens);
    dev_free(gs->target_batch_lens);
    gasal_res_destroy_device(gs->device_res, gs->device_cpy);
    gs->device_res = NULL; gs->device_cpy = NULL;
    if (params->secondBest) {
        gasal_res_destroy_device(gs->device_res_second, gs->device_cpy_second);
        gs->device_res_second = NULL; gs->device_cpy_second = NULL;
    }
}

// ====================================================== gasal_align.cu ====
void gasal_copy_subst_scores(gasal_subst_scores *subst) {
    const int d = current_device();
    if (d < 0 || d >= 64) { fprintf(stderr, "[GASAL ERROR:] device index out of range\n"); exit(EXIT_FAILURE); }
    g_scores[d].s = *subst;
    g_scores[d].set = true;
}

static void grow_or_die(uint32_t need, uint32_t &cap, const char *what) {
    uint32_t i = 2;
    while (cap * i < need) i++;
    fprintf(stderr,
            "[GASAL WARNING:] actual_%s(%d) > Allocated GPU memory (gpu_max_%s=%d). Therefore, allocating %d bytes "
            "on GPU (gpu_max_%s=%d). Performance may be lost if this is repeated many times.\n",
            what, need, what, cap, cap * i, what, cap * i);
    cap *= i;
}

void gasal_aln_async(gasal_gpu_storage_t *gs, const uint32_t qbytes, const uint32_t tbytes, const uint32_t n,
                     Parameters *params) {
    // argument checks (gasal_align.cu:32-67)
    if (n <= 0) { fprintf(stderr, "[GASAL ERROR:] actual_n_alns <= 0\n"); exit(EXIT_FAILURE); }
    if (qbytes <= 0) { fprintf(stderr, "[GASAL ERROR:] actual_query_batch_bytes <= 0\n"); exit(EXIT_FAILURE); }
    if (tbytes <= 0) { fprintf(stderr, "[GASAL ERROR:] actual_target_batch_bytes <= 0\n"); exit(EXIT_FAILURE); }
    if (qbytes % 8) { fprintf(stderr, "[GASAL ERROR:] actual_query_batch_bytes=%d is not a multiple of 8\n", qbytes); exit(EXIT_FAILURE); }
    if (tbytes % 8) { fprintf(stderr, "[GASAL ERROR:] actual_target_batch_bytes=%d is not a multiple of 8\n", tbytes); exit(EXIT_FAILURE); }
    if (qbytes > gs->host_max_query_batch_bytes) {
        fprintf(stderr, "[GASAL ERROR:] actual_query_batch_bytes(%d) > host_max_query_batch_bytes(%d)\n", qbytes, gs->host_max_query_batch_bytes);
        exit(EXIT_FAILURE);
    }
    if (tbytes > gs->host_max_target_batch_bytes) {
        fprintf(stderr, "[GASAL ERROR:] actual_target_batch_bytes(%d) > host_max_target_batch_bytes(%d)\n", tbytes, gs->host_max_target_batch_bytes);
        exit(EXIT_FAILURE);
    }
    if (n > gs->host_max_n_alns) {
        fprintf(stderr, "[GASAL ERROR:] actual_n_alns(%d) > host_max_n_alns(%d)\n", n, gs->host_max_n_alns);
        exit(EXIT_FAILURE);
    }
    // device buffer growth (:70-145)
    if (gs->gpu_max_query_batch_bytes < qbytes) {
        grow_or_die(qbytes, gs->gpu_max_query_batch_bytes, "query_batch_bytes");
        dev_free(gs->unpacked_query_batch);
        if (!params->isPacked) dev_free(gs->packed_query_batch);
        dev_alloc(&gs->unpacked_query_batch, gs->gpu_max_query_batch_bytes);
        if (params->isPacked) gs->packed_query_batch = (uint32_t *)gs->unpacked_query_batch;
        else dev_alloc(&gs->packed_query_batch, gs->gpu_max_query_batch_bytes / 8);
        if (params->start_pos == WITH_TB) {
            host_free(gs->host_res->cigar);
            host_alloc(&gs->host_res->cigar, gs->gpu_max_query_batch_bytes);
        }
    }
    if (gs->gpu_max_target_batch_bytes < tbytes) {
        grow_or_die(tbytes, gs->gpu_max_target_batch_bytes, "target_batch_bytes");
        dev_free(gs->unpacked_target_batch);
        if (!params->isPacked) dev_free(gs->packed_target_batch);
        dev_alloc(&gs->unpacked_target_batch, gs->gpu_max_target_batch_bytes);
        if (params->isPacked) gs->packed_target_batch = (uint32_t *)gs->unpacked_target_batch;
        else dev_alloc(&gs->packed_target_batch, gs->gpu_max_target_batch_bytes / 8);
    }
    if (gs->gpu_max_n_alns < n) {
        grow_or_die(n, gs->gpu_max_n_alns, "n_alns");
        for (uint32_t **p : {&gs->query_batch_offsets, &gs->target_batch_offsets, &gs->query_batch_lens,
                             &gs->target_batch_lens, &gs->seed_scores})
            dev_free(*p);
        dev_free(gs->query_op);
        dev_free(gs->target_op);
        block_alloc<uint32_t>(true, gs->gpu_max_n_alns, {&gs->query_batch_lens, &gs->target_batch_lens,
                                                         &gs->query_batch_offsets, &gs->target_batch_offsets});
        dev_alloc(&gs->seed_scores, gs->gpu_max_n_alns);
        dev_alloc(&gs->query_op, gs->gpu_max_n_alns);
        dev_alloc(&gs->target_op, gs->gpu_max_n_alns);
        gasal_res_destroy_device(gs->device_res, gs->device_cpy);
        gs->device_cpy = gasal_res_new_device_cpy(gs->gpu_max_n_alns, params);
        gs->device_res = gasal_res_new_device(gs->device_cpy);
        if (params->secondBest) {
            gasal_res_destroy_device(gs->device_res_second, gs->device_cpy_second);
            gs->device_cpy_second = gasal_res_new_device_cpy(gs->gpu_max_n_alns, params);
            gs->device_res_second = gasal_res_new_device(gs->device_cpy_second);
        }
    }
    hipStream_t st = gs->str;
    // host pages -> device (:152-175)
    for (host_batch_t *p = gs->extensible_host_unpacked_query_batch; p; p = p->next)
        if (p->data_size) CHECKHIPERROR(hipMemcpyAsync(gs->unpacked_query_batch + p->offset, p->data, p->data_size, hipMemcpyHostToDevice, st));
    for (host_batch_t *p = gs->extensible_host_unpacked_target_batch; p; p = p->next)
        if (p->data_size) CHECKHIPERROR(hipMemcpyAsync(gs->unpacked_target_batch + p->offset, p->data, p->data_size, hipMemcpyHostToDevice, st));
    // lens / offsets / seeds / ops (:207-235)
    const size_t mcap_h = block_run<uint32_t>({gs->host_query_batch_lens, gs->host_target_batch_lens,
                                               gs->host_query_batch_offsets, gs->host_target_batch_offsets});
    const size_t mcap_d = block_run<uint32_t>({gs->query_batch_lens, gs->target_batch_lens, gs->query_batch_offsets,
                                               gs->target_batch_offsets});
    if (mcap_h && mcap_h == mcap_d) {   // one copy: three whole arrays and the first n of the fourth
        CHECKHIPERROR(hipMemcpyAsync(gs->query_batch_lens, gs->host_query_batch_lens, (3 * mcap_h + n) * 4ull,
                                     hipMemcpyHostToDevice, st));
    } else {
        CHECKHIPERROR(hipMemcpyAsync(gs->query_batch_lens, gs->host_query_batch_lens, n * 4ull, hipMemcpyHostToDevice, st));
        CHECKHIPERROR(hipMemcpyAsync(gs->target_batch_lens, gs->host_target_batch_lens, n * 4ull, hipMemcpyHostToDevice, st));
        CHECKHIPERROR(hipMemcpyAsync(gs->query_batch_offsets, gs->host_query_batch_offsets, n * 4ull, hipMemcpyHostToDevice, st));
        CHECKHIPERROR(hipMemcpyAsync(gs->target_batch_offsets, gs->host_target_batch_offsets, n * 4ull, hipMemcpyHostToDevice, st));
    }
    if (params->algo == KSW) {
        if (gs->seed_scores == NULL) fprintf(stderr, "seed_scores == NULL\n");
        if (gs->host_seed_scores == NULL) fprintf(stderr, "host_seed_scores == NULL\n");
        if (gs->seed_scores == NULL || gs->host_seed_scores == NULL) exit(EXIT_FAILURE);
        CHECKHIPERROR(hipMemcpyAsync(gs->seed_scores, gs->host_seed_scores, n * 4ull, hipMemcpyHostToDevice, st));
    }
    if (params->isReverseComplement) {
        CHECKHIPERROR(hipMemcpyAsync(gs->query_op, gs->host_query_op, n, hipMemcpyHostToDevice, st));
        CHECKHIPERROR(hipMemcpyAsync(gs->target_op, gs->host_target_op, n, hipMemcpyHostToDevice, st));
    }

    // one flat dispatch in place of gasal_kernel_launcher (:249)
    const int dev = current_device();
    const gasal_subst_scores sc = g_scores[dev].set ? g_scores[dev].s : gasal_subst_scores{1, 4, 6, 1};
    gasalx_params P;
    std::memset(&P, 0, sizeof(P));
    P.match = sc.match; P.mismatch = sc.mismatch; P.gap_open = sc.gap_open; P.gap_extend = sc.gap_extend;
    P.algo = params->algo; P.start_pos = params->start_pos; P.second_best = params->secondBest;
    P.head = params->semiglobal_skipping_head; P.tail = params->semiglobal_skipping_tail;
    P.k_band = params->k_band; P.is_packed = params->isPacked ? 1 : 0;
    P.n_code = 0x4E; P.has_n_penalty = 0; P.n_penalty = 0; P.max_query_len = 0;
    gasalx_batch B;
    std::memset(&B, 0, sizeof(B));
    B.q_batch = gs->unpacked_query_batch; B.q_offsets = gs->query_batch_offsets; B.q_lens = gs->query_batch_lens;
    B.t_batch = gs->unpacked_target_batch; B.t_offsets = gs->target_batch_offsets; B.t_lens = gs->target_batch_lens;
    B.q_bytes = qbytes; B.t_bytes = tbytes; B.n_alns = n;
    B.q_ops = params->isReverseComplement ? gs->query_op : NULL;
    B.t_ops = params->isReverseComplement ? gs->target_op : NULL;
    B.seed_scores = params->algo == KSW ? gs->seed_scores : NULL;
    uint32_t mq = 0, mt = 0;
    for (uint32_t k = 0; k < n; k++) {
        mq = std::max(mq, gs->host_query_batch_lens[k]);
        mt = std::max(mt, gs->host_target_batch_lens[k]);
    }
    B.max_q_len = mq; B.max_t_len = mt;
    gasalx_results R;
    std::memset(&R, 0, sizeof(R));
    R.aln_score = gs->device_cpy->aln_score;
    R.q_end = gs->device_cpy->query_batch_end; R.t_end = gs->device_cpy->target_batch_end;
    R.q_start = gs->device_cpy->query_batch_start; R.t_start = gs->device_cpy->target_batch_start;
    if (params->secondBest && gs->device_cpy_second) {
        R.aln_score2 = gs->device_cpy_second->aln_score;
        R.q_end2 = gs->device_cpy_second->query_batch_end;
        R.t_end2 = gs->device_cpy_second->target_batch_end;
    }
    if (params->start_pos == WITH_TB) {
        R.cigar = gs->unpacked_query_batch;     // get_tb writes CIGARs here (get_tb.h:94)
        R.n_cigar_ops = gs->query_batch_lens;   // and n_ops here (get_tb.h:146)
    }
    gx::BatchShape shape;
    shape.max_q = mq; shape.max_t = mt;
    shape.sort = gx::uneven_lengths(P, gs->host_query_batch_lens, gs->host_target_batch_lens, n);
    shape.one_t8 = gx::one_pad8(gs->host_target_batch_lens, n, shape.max_t);
    gx::Workspace *ws = workspace_for(gs);
    // get_tb may run past the batch into the rest of unpacked_query_batch (Q14)
    if (gx::align_device(*ws, P, B, R, st, shape, gs->gpu_max_query_batch_bytes) != GASALX_OK) {
        fprintf(stderr, "[GASAL HIP ERROR:] %s\n", gx::last_error());
        exit(EXIT_FAILURE);
    }
    // results -> host (:266-304)
    gasal_res_t *h = gs->host_res, *d = gs->device_cpy;
#define D2H(field)                                                                                          \
    if (h->field != NULL && d->field != NULL)                                                               \
        CHECKHIPERROR(hipMemcpyAsync(h->field, d->field, n * sizeof(*h->field), hipMemcpyDeviceToHost, st));
    // one copy when both sides hold the same result arrays in one block of the same capacity
    auto res_d2h = [&](gasal_res_t *h, gasal_res_t *d) {
        const bool st5 = h->query_batch_start && d->query_batch_start, e3 = h->query_batch_end && d->query_batch_end;
        size_t ch = 0, cd = 0, k = 1;
        if (st5) {
            k = 5;
            ch = block_run<int32_t>({h->aln_score, h->query_batch_end, h->target_batch_end, h->query_batch_start, h->target_batch_start});
            cd = block_run<int32_t>({d->aln_score, d->query_batch_end, d->target_batch_end, d->query_batch_start, d->target_batch_start});
        } else if (e3 && !h->query_batch_start && !d->query_batch_start) {
            k = 3;
            ch = block_run<int32_t>({h->aln_score, h->query_batch_end, h->target_batch_end});
            cd = block_run<int32_t>({d->aln_score, d->query_batch_end, d->target_batch_end});
        } else if (!h->query_batch_end && !d->query_batch_end && !h->query_batch_start && !d->query_batch_start) {
            ch = cd = n;   // the score alone
        }
        if (ch && ch == cd && h->aln_score && d->aln_score) {
            CHECKHIPERROR(hipMemcpyAsync(h->aln_score, d->aln_score, ((k - 1) * ch + n) * 4ull, hipMemcpyDeviceToHost, st));
            return;
        }
        D2H(aln_score) D2H(query_batch_start) D2H(target_batch_start) D2H(query_batch_end) D2H(target_batch_end)
    };
    res_d2h(h, d);
    if (params->start_pos == WITH_TB) {
        CHECKHIPERROR(hipMemcpyAsync(h->cigar, gs->unpacked_query_batch, qbytes, hipMemcpyDeviceToHost, st));
        CHECKHIPERROR(hipMemcpyAsync(h->n_cigar_ops, gs->query_batch_lens, n * 4ull, hipMemcpyDeviceToHost, st));
    }
    if (params->secondBest) {
        res_d2h(gs->host_res_second, gs->device_cpy_second);
    }
#undef D2H
    gs->is_free = 0;
}

int gasal_is_aln_async_done(gasal_gpu_storage_t *gs) {
    if (gs->is_free == 1) return -2;
    hipError_t e = hipStreamQuery(gs->str);
    if (e != hipSuccess) {
        if (e == hipErrorNotReady) return -1;
        fprintf(stderr, "[GASAL HIP ERROR:] %s(HIP error no.=%d). Line no. %d in file %s\n", hipGetErrorString(e),
                (int)e, __LINE__, __FILE__);
        exit(EXIT_FAILURE);
    }
    gasal_host_batch_reset(gs);
    gs->is_free = 1;
    gs->current_n_alns = 0;
    return 0;
}
