// sw_benchmark.cpp — the nvbio sw-benchmark idiom over the second front-end
// (include/nvbio_batched.h), as a client of that header and -lgasal only.
//
//   sw_benchmark [-tests gotoh:ed:sw] [-scores FILE] reads.{fa,fq} reference.fa
//
// * Reads (FASTA or FASTQ) are packed as nvbio reads: DNA_N codes (A0 C1 G2 T3, other 4),
//   4 bits per symbol, big-endian words; the reference FASTA is one text of 2-bit codes,
//   non-ACGT stored as 0 (sw-benchmark.cu:290-330 ReferenceCoder, :73-74).
// * Batches of 256K reads (sw-benchmark.cu:555); per batch and test, one
//   BatchedAlignmentScore<AlignmentStream<aligner>, DeviceThreadScheduler>::enact
//   timed to completion, GCUPS = total pattern symbols x reference length / s
//   (sw-benchmark.cu:355-380).  Tests: Gotoh (2, -1, -2, -1) global / semi-global /
//   local, edit distance semi-global (sw-benchmark.cu:585-655), and -tests sw adds
//   Smith-Waterman (2, -1, -1, -1) local.
// * -scores FILE writes every int16 score, one line per read and test, for parity
//   checks (tests/test_gpu_nvbio.py).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <fstream>
#include <string>
#include <vector>

#include "nvbio_batched.h"

using namespace nvbio;

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC_RAW, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

#define HCK(x)                                                                                 \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

static uint32 dna_n(char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 4;
    }
}

// FASTA or FASTQ records (sequence lines only)
static std::vector<std::string> read_sequences(const char *path) {
    std::ifstream in(path);
    if (!in) { fprintf(stderr, "cannot open %s\n", path); exit(1); }
    std::vector<std::string> out;
    std::string line, cur;
    bool fastq = in.peek() == '@';
    if (fastq) {
        while (std::getline(in, line)) {
            std::string seq, plus, qual;
            std::getline(in, seq);
            std::getline(in, plus);
            std::getline(in, qual);
            out.push_back(seq);
        }
        return out;
    }
    bool have = false;
    while (std::getline(in, line)) {
        if (!line.empty() && line[0] == '>') {
            if (have) out.push_back(cur);
            cur.clear();
            have = true;
        } else cur += line;
    }
    if (have) out.push_back(cur);
    return out;
}

static void pack(const std::vector<uint32> &codes, uint32 bits, bool big, std::vector<uint32> &words) {
    const uint32 per = 32 / bits;
    words.assign(codes.size() / per + 2, 0u);
    for (size_t s = 0; s < codes.size(); s++) {
        const uint32 p = (uint32)(s % per);
        const uint32 sh = big ? 32 - bits * (p + 1) : bits * p;
        words[s / per] |= codes[s] << sh;
    }
}

template <typename aligner_type>
static void profile(const char *name, const aligner_type aligner, uint32 n, const uint32 *d_off, const uint32 *d_pat,
                    uint32 max_len, uint32 total, const uint32 *d_ref, uint32 ref_len, int16 *d_scores,
                    FILE *scores_out, const char *test) {
    typedef aln::AlignmentStream<aligner_type> stream_type;
    stream_type stream(aligner, n, d_off, d_pat, max_len, total, d_ref, ref_len, d_scores);
    aln::BatchedAlignmentScore<stream_type, aln::DeviceThreadScheduler> batch;
    batch.enact(stream, 0, NULL);   // warm-up launch (code objects, engine)
    HCK(hipDeviceSynchronize());
    const double t0 = now();
    batch.enact(stream, 0, NULL);
    HCK(hipDeviceSynchronize());
    const double dt = now() - t0;
    fprintf(stderr, "    %15s :   %7.1f GCUPS\n", name, 1.0e-9 * (double)stream.cells() / dt);
    if (scores_out) {
        std::vector<int16> h(n);
        HCK(hipMemcpy(h.data(), d_scores, n * sizeof(int16), hipMemcpyDeviceToHost));
        for (uint32 i = 0; i < n; i++) fprintf(scores_out, "%s\t%s\t%u\t%d\n", test, name, i, (int)h[i]);
    }
}

int main(int argc, char **argv) {
    bool t_gotoh = true, t_ed = true, t_sw = false;
    const char *scores_path = nullptr;
    if (argc < 3) {
        fprintf(stderr, "usage: sw_benchmark [-tests gotoh:ed:sw] [-scores FILE] reads ref.fa\n");
        return 1;
    }
    for (int i = 1; i < argc - 2; i++) {
        if (!strcmp(argv[i], "-tests")) {
            const std::string s = argv[++i];
            t_gotoh = s.find("gotoh") != std::string::npos;
            t_ed = s.find("ed") != std::string::npos;
            t_sw = s.find("sw") != std::string::npos;
        } else if (!strcmp(argv[i], "-scores")) scores_path = argv[++i];
    }
    fprintf(stderr, "sw-benchmark... started\n");
    const std::vector<std::string> reads = read_sequences(argv[argc - 2]);
    const std::vector<std::string> refs = read_sequences(argv[argc - 1]);
    std::vector<uint32> ref_codes;
    for (const std::string &r : refs)
        for (char c : r) { const uint32 v = dna_n(c); ref_codes.push_back(v < 4 ? v : 0); }
    const uint32 ref_len = (uint32)ref_codes.size();
    fprintf(stderr, "  reference: %u bps\n", ref_len);
    std::vector<uint32> ref_words;
    pack(ref_codes, 2, false, ref_words);
    uint32 *d_ref;
    HCK(hipMalloc(&d_ref, ref_words.size() * 4));
    HCK(hipMemcpy(d_ref, ref_words.data(), ref_words.size() * 4, hipMemcpyHostToDevice));
    FILE *sout = scores_path ? fopen(scores_path, "w") : nullptr;

    const uint32 batch_size = 256 * 1024;
    for (size_t b0 = 0; b0 < reads.size(); b0 += batch_size) {
        const uint32 n = (uint32)std::min<size_t>(batch_size, reads.size() - b0);
        std::vector<uint32> codes, offs(1, 0);
        uint32 max_len = 0;
        for (uint32 i = 0; i < n; i++) {
            for (char c : reads[b0 + i]) codes.push_back(dna_n(c));
            offs.push_back((uint32)codes.size());
            max_len = std::max<uint32>(max_len, (uint32)reads[b0 + i].size());
        }
        const uint32 total = (uint32)codes.size();
        fprintf(stderr, "  %u reads, avg: %u bps, max: %u bps\n", n, n ? total / n : 0, max_len);
        std::vector<uint32> words;
        pack(codes, 4, true, words);
        uint32 *d_pat, *d_off;
        int16 *d_scores;
        HCK(hipMalloc(&d_pat, words.size() * 4));
        HCK(hipMalloc(&d_off, offs.size() * 4));
        HCK(hipMalloc(&d_scores, (size_t)n * 2 + 2));
        HCK(hipMemcpy(d_pat, words.data(), words.size() * 4, hipMemcpyHostToDevice));
        HCK(hipMemcpy(d_off, offs.data(), offs.size() * 4, hipMemcpyHostToDevice));
        if (t_gotoh) {
            aln::SimpleGotohScheme scoring;
            scoring.m_match = 2; scoring.m_mismatch = -1; scoring.m_gap_open = -2; scoring.m_gap_ext = -1;
            fprintf(stderr, "  testing Gotoh scoring speed...\n");
            profile("global", aln::make_gotoh_aligner<aln::GLOBAL, aln::TextBlockingTag>(scoring), n, d_off, d_pat,
                    max_len, total, d_ref, ref_len, d_scores, sout, "gotoh");
            profile("semi-global", aln::make_gotoh_aligner<aln::SEMI_GLOBAL, aln::TextBlockingTag>(scoring), n, d_off,
                    d_pat, max_len, total, d_ref, ref_len, d_scores, sout, "gotoh");
            profile("local", aln::make_gotoh_aligner<aln::LOCAL, aln::TextBlockingTag>(scoring), n, d_off, d_pat,
                    max_len, total, d_ref, ref_len, d_scores, sout, "gotoh");
        }
        if (t_ed) {
            fprintf(stderr, "  testing Edit Distance scoring speed...\n");
            profile("semi-global", aln::make_edit_distance_aligner<aln::SEMI_GLOBAL, aln::TextBlockingTag>(), n, d_off,
                    d_pat, max_len, total, d_ref, ref_len, d_scores, sout, "ed");
        }
        if (t_sw) {
            fprintf(stderr, "  testing Smith-Waterman scoring speed...\n");
            profile("local", aln::make_smith_waterman_aligner<aln::LOCAL, aln::TextBlockingTag>(
                                 aln::SimpleSmithWatermanScheme(2, -1, -1, -1)),
                    n, d_off, d_pat, max_len, total, d_ref, ref_len, d_scores, sout, "sw");
        }
        HCK(hipFree(d_pat));
        HCK(hipFree(d_off));
        HCK(hipFree(d_scores));
    }
    if (sout) fclose(sout);
    HCK(hipFree(d_ref));
    fprintf(stderr, "sw-benchmark... done\n");
    return 0;
}
