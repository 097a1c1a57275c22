// test_prog.cpp — command-line driver of libgasal with GASAL2's test_prog contract.
//
// Written from the documented behaviour,
// as a client of the drop-in C++ API only (include/gasal_header.h, -lgasal):
//
//   test_prog.out [-a INT] [-b INT] [-q INT] [-r INT] [-s] [-t] [-p] [-n INT]
//                 [-y local|semi_global|global|ksw|banded] [-x HEAD TAIL] [-k INT]
//                 query.fasta target.fasta
//
// * FASTA pairs are read in lockstep; a record header starts with one of
//   '>' '<' '/' '+', which selects the per-sequence operation FORWARD_NATURAL,
//   REVERSE_NATURAL, FORWARD_COMPLEMENT, REVERSE_COMPLEMENT (test_prog.cpp:79-137).
// * The pairs are split into equal contiguous ranges over -n host threads; each
//   thread owns NB_STREAMS storages and keeps them busy with batches of up to
//   BATCH_PAIRS pairs (gasal_host_batch_fill / gasal_op_fill / gasal_aln_async,
//   polled with gasal_is_aln_async_done).
// * With -p, one line per pair (order within a batch kept, batches of different
//   storages may interleave):
//     query_name=<hdr>\ttarget_name=<hdr>\tscore=<s>
//     [\tquery_batch_start=..\ttarget_batch_start=..]   start_pos WITH_START/WITH_TB and
//                                                        (SEMI_GLOBAL with head != NONE, or
//                                                         algo LOCAL/MICROLOCAL/BANDED/KSW)
//     [\tquery_batch_end=..\ttarget_batch_end=..]       algo != GLOBAL
//     [\t2nd_score=..\t2nd_query_batch_end=..\t2nd_target_batch_end=..]   secondBest
//     [\tCIGAR=<forward RLE, runs of one op merged>]     WITH_TB
//   (test_prog.cpp:349-430; the head-only test of the start condition is kept).
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>

#include <algorithm>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "gasal_header.h"

namespace {

constexpr int NB_STREAMS = 2;
constexpr int BATCH_PAIRS = 5000;

struct Pair {
    std::string qname, tname, q, t;
    uint8_t qop = 0, top = 0;
};

int header_op(char c) {
    static const char kStarts[] = "></+";
    for (int i = 0; i < 4; ++i)
        if (c == kStarts[i]) return i;
    return -1;
}

// Reads both files in lockstep; returns false on a structural mismatch.
bool read_pairs(std::istream &qf, std::istream &tf, std::vector<Pair> &out) {
    std::string ql, tl;
    Pair cur;
    bool open = false;
    while (std::getline(qf, ql) && std::getline(tf, tl)) {
        const int qo = ql.empty() ? -1 : header_op(ql[0]);
        const int to = tl.empty() ? -1 : header_op(tl[0]);
        if (qo >= 0 && to >= 0) {
            if (open) out.push_back(cur);
            cur = Pair();
            cur.qname = ql.substr(1);
            cur.tname = tl.substr(1);
            cur.qop = (uint8_t)qo;
            cur.top = (uint8_t)to;
            open = true;
        } else if (open) {
            cur.q += ql;
            cur.t += tl;
        } else {
            return false;
        }
    }
    if (open) out.push_back(cur);
    return true;
}

const char kOpChar[4] = {'M', 'X', 'D', 'I'};

// CIGAR bytes are count<<2|op in reverse order at the pair's query offset.
std::string forward_cigar(const uint8_t *bytes, uint32_t n_ops) {
    std::ostringstream s;
    if (n_ops == 0) return s.str();
    int op = bytes[n_ops - 1] & 3, count = bytes[n_ops - 1] >> 2;
    for (int u = (int)n_ops - 2; u >= 0; --u) {
        const int o = bytes[u] & 3;
        if (o == op) {
            count += bytes[u] >> 2;
        } else {
            s << count << kOpChar[op];
            op = o;
            count = bytes[u] >> 2;
        }
    }
    s << count << kOpChar[op];
    return s.str();
}

struct Slot {
    gasal_gpu_storage_t *st = nullptr;
    int first = 0;   // index of the batch's first pair
    int n = 0;       // pairs in flight (0 = idle)
};

void print_batch(const Parameters &P, const std::vector<Pair> &pairs, const Slot &s, std::ostream &os) {
    const gasal_res_t *r = s.st->host_res;
    const gasal_res_t *r2 = s.st->host_res_second;
    const bool starts = (P.start_pos == WITH_START || P.start_pos == WITH_TB) &&
                        ((P.algo == SEMI_GLOBAL && P.semiglobal_skipping_head != NONE) || P.algo > SEMI_GLOBAL);
    for (int j = 0; j < s.n; ++j) {
        const Pair &p = pairs[s.first + j];
        os << "query_name=" << p.qname << "\ttarget_name=" << p.tname << "\tscore=" << r->aln_score[j];
        if (starts)
            os << "\tquery_batch_start=" << r->query_batch_start[j] << "\ttarget_batch_start="
               << r->target_batch_start[j];
        if (P.algo != GLOBAL)
            os << "\tquery_batch_end=" << r->query_batch_end[j] << "\ttarget_batch_end=" << r->target_batch_end[j];
        if (P.secondBest)
            os << "\t2nd_score=" << r2->aln_score[j] << "\t2nd_query_batch_end=" << r2->query_batch_end[j]
               << "\t2nd_target_batch_end=" << r2->target_batch_end[j];
        if (P.start_pos == WITH_TB)
            os << "\tCIGAR="
               << forward_cigar(r->cigar + s.st->host_query_batch_offsets[j], r->n_cigar_ops[j]);
        os << "\n";
    }
}

double now_ms() {
    timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_sec * 1e3 + tv.tv_usec / 1e3;
}

}  // namespace

int main(int argc, char **argv) {
    Parameters *args = new Parameters(argc, argv);
    args->parse();
    // extension: GASALX_TEST_PROG_RC=1 applies the header modifiers (the reference's
    // parser never sets isReverseComplement, so its driver parses them but ignores them)
    if (const char *rc = getenv("GASALX_TEST_PROG_RC")) args->isReverseComplement = rc[0] == '1';
    args->print();

    gasal_subst_scores sc;
    sc.match = args->sa;
    sc.mismatch = args->sb;
    sc.gap_open = args->gapo;
    sc.gap_extend = args->gape;
    gasal_copy_subst_scores(&sc);

    std::cerr << "Loading files...." << std::endl;
    std::vector<Pair> pairs;
    if (!read_pairs(args->query_batch_fasta, args->target_batch_fasta, pairs)) {
        std::cerr << "Batch1 and target_batch files should be fasta having same number of sequences" << std::endl;
        return EXIT_FAILURE;
    }
    size_t max_q = 0, max_len = 0;
    for (const Pair &p : pairs) {
        max_q = std::max(max_q, p.q.size());
        max_len = std::max({max_len, p.q.size(), p.t.size()});
    }
    std::cerr << "Processing " << pairs.size() << " pairs (max query " << max_q << ", max length " << max_len
              << ")..." << std::endl;

    const int n_threads = std::max(1, args->n_threads);
    const int total = (int)pairs.size();
    const int per_thread = (total + n_threads - 1) / n_threads;
    const double t0 = now_ms();

    std::vector<gasal_gpu_storage_v> vecs(n_threads);
    for (int z = 0; z < n_threads; ++z) {
        vecs[z] = gasal_init_gpu_storage_v(NB_STREAMS);
        gasal_init_streams(&vecs[z], (int)max_q + 7, (int)max_len + 7, BATCH_PAIRS, args);
    }

    omp_set_num_threads(n_threads);
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        const int begin = std::min(total, tid * per_thread);
        const int end = std::min(total, begin + per_thread);
        std::vector<uint8_t> qops, tops;
        Slot slots[NB_STREAMS];
        for (int z = 0; z < NB_STREAMS; ++z) slots[z].st = &vecs[tid].a[z];
        int next = begin, in_flight = 0;
        while (next < end || in_flight > 0) {
            // launch on every idle storage
            for (Slot &s : slots) {
                if (next >= end || s.n != 0 || s.st->is_free != 1) continue;
                const int n = std::min(BATCH_PAIRS, end - next);
                if ((uint32_t)n > s.st->host_max_n_alns) gasal_host_alns_resize(s.st, n, args);
                uint32_t qidx = 0, tidx = 0;
                qops.resize(n);
                tops.resize(n);
                for (int j = 0; j < n; ++j) {
                    const Pair &p = pairs[next + j];
                    s.st->host_query_batch_offsets[j] = qidx;
                    s.st->host_target_batch_offsets[j] = tidx;
                    qidx = gasal_host_batch_fill(s.st, qidx, p.q.c_str(), (uint32_t)p.q.size(), QUERY);
                    tidx = gasal_host_batch_fill(s.st, tidx, p.t.c_str(), (uint32_t)p.t.size(), TARGET);
                    s.st->host_query_batch_lens[j] = (uint32_t)p.q.size();
                    s.st->host_target_batch_lens[j] = (uint32_t)p.t.size();
                    qops[j] = p.qop;
                    tops[j] = p.top;
                }
                s.st->current_n_alns = n;
                gasal_op_fill(s.st, qops.data(), n, QUERY);
                gasal_op_fill(s.st, tops.data(), n, TARGET);
                gasal_aln_async(s.st, qidx, tidx, n, args);
                s.st->current_n_alns = 0;
                s.first = next;
                s.n = n;
                next += n;
                ++in_flight;
            }
            // collect finished storages
            for (Slot &s : slots) {
                if (s.n == 0 || gasal_is_aln_async_done(s.st) != 0) continue;
                if (args->print_out) {
                    std::ostringstream os;
                    print_batch(*args, pairs, s, os);
#pragma omp critical
                    std::cout << os.str() << std::flush;
                }
                s.n = 0;
                --in_flight;
            }
        }
    }

    for (int z = 0; z < n_threads; ++z) {
        gasal_destroy_streams(&vecs[z], args);
        gasal_destroy_gpu_storage_v(&vecs[z]);
    }
    std::cerr << std::endl << "Done" << std::endl;
    fprintf(stderr, "Total execution time (in milliseconds): %.3f\n", now_ms() - t0);
    delete args;
    return 0;
}
