// hmm_io.cpp — reader of the reference's PairHMM input files (host ingestion).
//
// Format, as the reference's drivers scan it (Non-CDP/PairHMM/inter_task/
// Synthetic_data/tile_1/tile_1.cu:246-290; Intra-task/real_data/
// improved_warp_based/improved_warp_based.cu:217-279): a sequence of groups, each
//   size
//   size x { read_size  read_bases  read_size x base_qual  read_size x ins_qual
//            read_size x del_qual  read_size x gcp_qual  haplotype_size  haplotype_bases }
// with every field whitespace-separated (fscanf %d / %s).  Qualities are kept as
// (char)value, i.e. their low 8 bits, and the kernels use q & 127 (tile_1.cu:415-419).
// Streams the file token by token, so multi-gigabyte real-data files need no
// second copy in memory.
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "engine.hpp"
#include "gasalx.h"

namespace {

struct Tokens {
    FILE *f;
    std::string tok;
    bool next() {   // the next whitespace-separated token, false at end of file
        tok.clear();
        int c;
        while ((c = std::getc(f)) != EOF && std::isspace(c)) {}
        if (c == EOF) return false;
        do tok.push_back((char)c); while ((c = std::getc(f)) != EOF && !std::isspace(c));
        return true;
    }
    bool integer(long *v) {
        if (!next()) return false;
        char *end = nullptr;
        errno = 0;
        *v = std::strtol(tok.c_str(), &end, 10);
        return errno == 0 && end && *end == '\0';
    }
};

template <class T>
T *dup(const std::vector<T> &v) {
    T *p = static_cast<T *>(std::malloc(v.size() * sizeof(T) + 1));
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

}  // namespace

extern "C" {

int gasalx_hmm_file_free(gasalx_hmm_file *f) {
    if (!f) return GASALX_OK;
    for (void *p : {(void *)f->group_sizes, (void *)f->reads, (void *)f->read_offsets, (void *)f->read_lens,
                    (void *)f->base_quals, (void *)f->ins_quals, (void *)f->del_quals, (void *)f->gcp_quals,
                    (void *)f->haps, (void *)f->hap_offsets, (void *)f->hap_lens})
        std::free(p);
    std::free(f);
    return GASALX_OK;
}

int gasalx_hmm_file_read(const char *path, gasalx_hmm_file **out) {
    if (!path || !out) { gx::set_error("gasalx_hmm_file_read: null argument"); return GASALX_EINVAL; }
    *out = nullptr;
    FILE *fp = std::fopen(path, "r");
    if (!fp) { gx::set_error(std::string("cannot open ") + path); return GASALX_EINVAL; }
    Tokens t{fp, {}};
    std::vector<uint32_t> groups, roff, rlen, hoff, hlen;
    std::vector<uint8_t> reads, quals[4], haps;
    auto fail = [&](const std::string &what) {
        std::fclose(fp);
        gx::set_error(std::string(path) + ": " + what + " (pair " + std::to_string(rlen.size()) + ")");
        return GASALX_EINVAL;
    };
    long size;
    while (t.integer(&size)) {
        if (size < 0) return fail("negative group size");
        groups.push_back((uint32_t)size);
        for (long p = 0; p < size; p++) {
            long rl, hl, q;
            if (!t.integer(&rl) || rl <= 0) return fail("bad read length");
            if (!t.next() || (long)t.tok.size() < rl) return fail("read shorter than its length");
            // offsets are uint32 (gasalx_hmm_file): a file past 4 GiB of read (or haplotype)
            // bytes is refused rather than wrapped
            if (reads.size() + (uint64_t)rl > 0xFFFFFFFFull) return fail("more than 4 GiB of read bases");
            roff.push_back((uint32_t)reads.size());
            rlen.push_back((uint32_t)rl);
            reads.insert(reads.end(), t.tok.begin(), t.tok.begin() + rl);
            for (int k = 0; k < 4; k++)
                for (long j = 0; j < rl; j++) {
                    if (!t.integer(&q)) return fail("missing quality value");
                    quals[k].push_back((uint8_t)(char)q);
                }
            if (!t.integer(&hl) || hl <= 0) return fail("bad haplotype length");
            if (!t.next() || (long)t.tok.size() < hl) return fail("haplotype shorter than its length");
            if (haps.size() + (uint64_t)hl > 0xFFFFFFFFull) return fail("more than 4 GiB of haplotype bases");
            hoff.push_back((uint32_t)haps.size());
            hlen.push_back((uint32_t)hl);
            haps.insert(haps.end(), t.tok.begin(), t.tok.begin() + hl);
        }
    }
    if (!t.tok.empty()) return fail("trailing token '" + t.tok + "'");
    std::fclose(fp);
    gasalx_hmm_file *f = static_cast<gasalx_hmm_file *>(std::calloc(1, sizeof(gasalx_hmm_file)));
    if (!f) return GASALX_ENOMEM;
    f->n_pairs = (uint32_t)rlen.size();
    f->n_groups = (uint32_t)groups.size();
    f->group_sizes = dup(groups);
    f->reads = dup(reads); f->read_offsets = dup(roff); f->read_lens = dup(rlen);
    f->base_quals = dup(quals[0]); f->ins_quals = dup(quals[1]); f->del_quals = dup(quals[2]);
    f->gcp_quals = dup(quals[3]);
    f->haps = dup(haps); f->hap_offsets = dup(hoff); f->hap_lens = dup(hlen);
    f->read_bytes = reads.size();
    f->hap_bytes = haps.size();
    if (!f->group_sizes || !f->reads || !f->read_offsets || !f->read_lens || !f->base_quals || !f->ins_quals ||
        !f->del_quals || !f->gcp_quals || !f->haps || !f->hap_offsets || !f->hap_lens) {
        gasalx_hmm_file_free(f);
        return GASALX_ENOMEM;
    }
    *out = f;
    return GASALX_OK;
}

}  // extern "C"
