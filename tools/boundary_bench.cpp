// boundary_bench.cpp — throughput of the drop-in boundary driven the way the reference's own
// host program drives it (Non-CDP/GASAL2/test_prog/test_prog.cpp:12,18,202-347): T OpenMP host
// threads, each with its own gasal_gpu_storage_v of NB_STREAMS storages, filling host batches of
// STREAM_BATCH_SIZE pairs with gasal_host_batch_fill, launching them with gasal_aln_async on any
// free storage and polling gasal_is_aln_async_done.  A client of the C++ API only
// (include/gasal_header.h, -lgasal), like tools/test_prog.cpp.
//
//   boundary_bench [--repl N] [--batch B] [--storages S] [--warm W] [--reps K] [--dump FILE]
//                  [--poll-us U (probe: sleep U us between polls once a thread's pairs are all launched)]
//                  <test_prog options: -y local|semi_global|global|ksw|banded, -s, -t, -n T, ...>
//                  query.fasta[.gz] target.fasta[.gz]
//
// The FASTA pairs (plain or gzip) are read in lock step and replicated N times in memory.  The
// storages are set up once (gasal_init_streams, timed apart), W untimed passes warm the GPU and
// grow the buffers, then K timed passes each align every pair.  One JSON line on stdout: pairs,
// cells, init and per-pass wall times, GCUPS of the fastest pass.  --dump writes the last pass's
// results per pair (int32 score, q_end, t_end, q_start, t_start, each n entries) for the caller's
// parity check.
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gasal_header.h"

namespace {

double now_ms() {
    timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_sec * 1e3 + tv.tv_usec / 1e3;
}

// records of a FASTA file (plain or gzip): sequences only, in order
bool read_fasta(const char *path, std::vector<std::string> &seqs) {
    gzFile f = gzopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    std::string cur;
    bool open = false;
    while (gzgets(f, buf, sizeof(buf))) {
        size_t l = strlen(buf);
        while (l && (buf[l - 1] == '\n' || buf[l - 1] == '\r')) buf[--l] = 0;
        if (l && strchr("></+", buf[0])) {
            if (open) seqs.push_back(cur);
            cur.clear();
            open = true;
        } else if (open) {
            cur += buf;
        }
    }
    if (open) seqs.push_back(cur);
    gzclose(f);
    return true;
}

struct Slot {
    gasal_gpu_storage_t *st = nullptr;
    int first = 0, n = 0;
};

}  // namespace

int main(int argc, char **argv) {
    int repl = 1, batch = 5000, storages = 2, warm = 1, reps = 3, poll_us = 0;
    const char *dump = nullptr;
    std::vector<char *> rest = {argv[0]};
    for (int i = 1; i < argc; ++i) {
        auto val = [&](const char *name) -> const char * {
            if (i + 1 >= argc) { fprintf(stderr, "%s needs a value\n", name); exit(1); }
            return argv[++i];
        };
        if (!strcmp(argv[i], "--repl")) repl = atoi(val("--repl"));
        else if (!strcmp(argv[i], "--batch")) batch = atoi(val("--batch"));
        else if (!strcmp(argv[i], "--storages")) storages = atoi(val("--storages"));
        else if (!strcmp(argv[i], "--warm")) warm = atoi(val("--warm"));
        else if (!strcmp(argv[i], "--reps")) reps = atoi(val("--reps"));
        else if (!strcmp(argv[i], "--dump")) dump = val("--dump");
        else if (!strcmp(argv[i], "--poll-us")) poll_us = atoi(val("--poll-us"));   // probe: sleep between polls
        else rest.push_back(argv[i]);
    }
    if (rest.size() < 3) { fprintf(stderr, "usage: boundary_bench [options] query.fasta target.fasta\n"); return 1; }
    // Parameters opens the FASTA files itself; the pairs are read here (gzip aware)
    Parameters *args = new Parameters((int)rest.size(), rest.data());
    args->parse();
    const char *qpath = rest[rest.size() - 2], *tpath = rest[rest.size() - 1];
    std::vector<std::string> q0, t0;
    if (!read_fasta(qpath, q0) || !read_fasta(tpath, t0) || q0.size() != t0.size() || q0.empty()) {
        fprintf(stderr, "boundary_bench: cannot read the FASTA pairs\n");
        return 1;
    }
    const int base = (int)q0.size();
    const int total = base * repl;
    size_t max_q = 0, max_len = 0;
    double cells = 0;
    for (int i = 0; i < base; ++i) {
        max_q = std::max(max_q, q0[i].size());
        max_len = std::max({max_len, q0[i].size(), t0[i].size()});
        cells += (double)q0[i].size() * t0[i].size();
    }
    cells *= repl;

    gasal_subst_scores sc;
    sc.match = args->sa; sc.mismatch = args->sb; sc.gap_open = args->gapo; sc.gap_extend = args->gape;
    gasal_copy_subst_scores(&sc);

    const int n_threads = std::max(1, args->n_threads);
    const int per_thread = (total + n_threads - 1) / n_threads;
    const double ti = now_ms();
    std::vector<gasal_gpu_storage_v> vecs(n_threads);
    for (int z = 0; z < n_threads; ++z) {
        vecs[z] = gasal_init_gpu_storage_v(storages);
        gasal_init_streams(&vecs[z], (int)max_q + 7, (int)max_len + 7, batch, args);
    }
    const double init_ms = now_ms() - ti;

    const bool starts = args->start_pos == WITH_START || args->start_pos == WITH_TB;
    std::vector<int32_t> out(dump ? (size_t)total * 5 : 0, 0);
    std::vector<double> pass_ms;
    for (int pass = 0; pass < warm + reps; ++pass) {
        const bool last = pass == warm + reps - 1;
        const double tp = now_ms();
        omp_set_num_threads(n_threads);
#pragma omp parallel
        {
            const int tid = omp_get_thread_num();
            const int begin = std::min(total, tid * per_thread);
            const int end = std::min(total, begin + per_thread);
            std::vector<Slot> slots(storages);
            for (int z = 0; z < storages; ++z) slots[z].st = &vecs[tid].a[z];
            int next = begin, in_flight = 0;
            while (next < end || in_flight > 0) {
                if (poll_us > 0 && next >= end) usleep(poll_us);
                for (Slot &s : slots) {   // launch on every free storage (test_prog.cpp:265-330)
                    if (next >= end || s.n != 0 || s.st->is_free != 1) continue;
                    const int n = std::min(batch, end - next);
                    if ((uint32_t)n > s.st->host_max_n_alns) gasal_host_alns_resize(s.st, n, args);
                    uint32_t qidx = 0, tidx = 0;
                    for (int j = 0; j < n; ++j) {
                        const int k = (next + j) % base;
                        s.st->host_query_batch_offsets[j] = qidx;
                        s.st->host_target_batch_offsets[j] = tidx;
                        qidx = gasal_host_batch_fill(s.st, qidx, q0[k].c_str(), (uint32_t)q0[k].size(), QUERY);
                        tidx = gasal_host_batch_fill(s.st, tidx, t0[k].c_str(), (uint32_t)t0[k].size(), TARGET);
                        s.st->host_query_batch_lens[j] = (uint32_t)q0[k].size();
                        s.st->host_target_batch_lens[j] = (uint32_t)t0[k].size();
                    }
                    gasal_aln_async(s.st, qidx, tidx, n, args);
                    s.first = next;
                    s.n = n;
                    next += n;
                    ++in_flight;
                }
                for (Slot &s : slots) {   // collect (test_prog.cpp:332-347)
                    if (s.n == 0 || gasal_is_aln_async_done(s.st) != 0) continue;
                    if (last && dump) {
                        const gasal_res_t *r = s.st->host_res;
                        for (int j = 0; j < s.n; ++j) {
                            const size_t p = (size_t)s.first + j;
                            out[p] = r->aln_score[j];
                            if (args->algo != GLOBAL) {
                                out[(size_t)total + p] = r->query_batch_end[j];
                                out[2 * (size_t)total + p] = r->target_batch_end[j];
                            }
                            if (starts && args->algo != GLOBAL) {
                                out[3 * (size_t)total + p] = r->query_batch_start[j];
                                out[4 * (size_t)total + p] = r->target_batch_start[j];
                            }
                        }
                    }
                    s.n = 0;
                    --in_flight;
                }
            }
        }
        if (pass >= warm) pass_ms.push_back(now_ms() - tp);
    }
    for (int z = 0; z < n_threads; ++z) {
        gasal_destroy_streams(&vecs[z], args);
        gasal_destroy_gpu_storage_v(&vecs[z]);
    }
    if (dump) {
        FILE *f = fopen(dump, "wb");
        if (!f || fwrite(out.data(), 4, out.size(), f) != out.size()) { fprintf(stderr, "dump failed\n"); return 1; }
        fclose(f);
    }
    const double best = *std::min_element(pass_ms.begin(), pass_ms.end());
    printf("{\"pairs\": %d, \"base_pairs\": %d, \"repl\": %d, \"cells\": %.0f, \"threads\": %d, \"storages\": %d, "
           "\"batch\": %d, \"init_ms\": %.3f, \"pass_ms\": [",
           total, base, repl, cells, n_threads, storages, batch, init_ms);
    for (size_t i = 0; i < pass_ms.size(); ++i) printf("%s%.3f", i ? ", " : "", pass_ms[i]);
    printf("], \"best_ms\": %.3f, \"gcups\": %.2f}\n", best, cells / best / 1e6);
    delete args;
    return 0;
}
