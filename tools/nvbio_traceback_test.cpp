// nvbio_traceback_test — a client of include/nvbio_batched.h's traceback templates, shaped like
// nvbio-test's SingleTest::full / ::banded checks (NvB/nvbio-test/alignment_test.cu:230-356,
// :749-904): each case runs one pattern against one text through BatchedAlignmentTraceback or
// BatchedBandedAlignmentTraceback on the GPU, replays the result into a backtracker that builds
// the run-length string the reference's test prints, and compares it with the string the
// reference asserts.  Exit status 0 when every case matches.
//
// usage: nvbio_traceback_test
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "nvbio_batched.h"

using namespace nvbio;
using namespace nvbio::aln;

#define HIP_OK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

// the test's backtracker: push() writes one op, clip() writes 'S' cells without advancing (the
// end clip comes first and the pushes overwrite it), so the string is the pushes followed by the
// start clip (alignment_test_utils.h:628-645); rle() as the test prints it (:76-99)
struct StringBacktracker {
    std::string s;
    size_t pos = 0;
    void clip(uint32 n) {
        if (s.size() < pos + n) s.resize(pos + n, 'S');
        for (uint32 i = 0; i < n; ++i) s[pos + i] = 'S';
    }
    void push(uint8 op) {
        const char c = "MID"[op];
        if (pos < s.size()) s[pos] = c; else s.push_back(c);
        ++pos;
    }
    std::string rle() const {
        std::string out;
        for (size_t i = 0; i < s.size();) {
            size_t j = i;
            while (j < s.size() && s[j] == s[i]) ++j;
            out += std::to_string(j - i) + s[i];
            i = j;
        }
        return out;
    }
};

static uint32 dna(char c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : 4; }

// 4-bit big-endian pattern words and 2-bit little-endian text words (sw-benchmark's packing)
static std::vector<uint32> pack(const char *s, uint32 bits, bool big) {
    const uint32 per = 32 / bits, n = (uint32)strlen(s);
    std::vector<uint32> w((n + per - 1) / per + 1, 0u);
    for (uint32 i = 0; i < n; ++i) {
        const uint32 p = i % per, sh = big ? 32 - bits * (p + 1) : bits * p;
        w[i / per] |= (dna(s[i]) & ((1u << bits) - 1u)) << sh;
    }
    return w;
}

template <typename T>
static T *to_dev(const std::vector<T> &v) {
    T *d = nullptr;
    HIP_OK(hipMalloc(&d, v.size() * sizeof(T) + 16));
    HIP_OK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

struct Result {
    int32 score;
    uint32 source[2], sink[2];
    std::string cigar;
};

// BAND_LEN 0: the full-DP traceback
template <uint32 BAND_LEN, typename aligner_type>
static Result run(const aligner_type aligner, const char *pattern, const char *text) {
    const uint32 M = (uint32)strlen(pattern), N = (uint32)strlen(text);
    std::vector<uint32> pw = pack(pattern, 4, true), tw = pack(text, 2, false);
    std::vector<uint32> off = {0u, M};
    uint32 *d_pw = to_dev(pw), *d_tw = to_dev(tw), *d_off = to_dev(off);
    const uint32 stride = 2 * M + N + 32;
    int32 *d_score;
    uint32 *d_src, *d_snk, *d_nops;
    uint8 *d_ops;
    HIP_OK(hipMalloc(&d_score, 4));
    HIP_OK(hipMalloc(&d_src, 8));
    HIP_OK(hipMalloc(&d_snk, 8));
    HIP_OK(hipMalloc(&d_nops, 4));
    HIP_OK(hipMalloc(&d_ops, stride));
    TracebackStream<aligner_type> stream(aligner, 1, d_off, d_pw, M, M, d_tw, N, d_score, d_src, d_snk, d_ops,
                                         stride, d_nops);
    if constexpr (BAND_LEN == 0) {
        BatchedAlignmentTraceback<32, TracebackStream<aligner_type>> batch;
        batch.enact(stream);
    } else {
        BatchedBandedAlignmentTraceback<BAND_LEN, 32, TracebackStream<aligner_type>> batch;
        batch.enact(stream);
    }
    HIP_OK(hipDeviceSynchronize());
    Result r;
    uint32 n_ops = 0;
    std::vector<uint8> ops(stride);
    HIP_OK(hipMemcpy(&r.score, d_score, 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(r.source, d_src, 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(r.sink, d_snk, 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(&n_ops, d_nops, 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(ops.data(), d_ops, stride, hipMemcpyDeviceToHost));
    StringBacktracker bt;
    replay(bt, M, r.source[1], r.sink[1], ops.data(), n_ops);
    r.cigar = bt.rle();
    for (void *p : {(void *)d_pw, (void *)d_tw, (void *)d_off, (void *)d_score, (void *)d_src, (void *)d_snk,
                    (void *)d_nops, (void *)d_ops})
        HIP_OK(hipFree(p));
    return r;
}

static int failures = 0;

static void check(const char *name, const Result &r, const char *expected) {
    const bool ok = r.cigar == expected;
    failures += !ok;
    printf("%-26s %6d  %-20s [%u:%u] x [%u:%u]  %s\n", name, r.score, r.cigar.c_str(), r.source[0], r.sink[0],
           r.source[1], r.sink[1], ok ? "ok" : "MISMATCH");
}

int main() {
    // alignment_test.cu:761-794
    const char *str = "ACAACTA", *ref = "AAACACCCTAACACACTAAA";
    const SimpleSmithWatermanScheme sw(2, -1, -1, -1);
    const SimpleGotohScheme go(2, -1, -1, -1);
    check("sw global", run<0>(make_smith_waterman_aligner<GLOBAL>(sw), str, ref), "1M2D3M1D3M10D");
    check("sw local", run<0>(make_smith_waterman_aligner<LOCAL>(sw), str, ref), "4M1D3M");
    check("sw semi-global", run<0>(make_smith_waterman_aligner<SEMI_GLOBAL>(sw), str, ref), "4M1D3M");
    check("gotoh global", run<0>(make_gotoh_aligner<GLOBAL>(go), str, ref), "1M2D3M1D3M10D");
    check("gotoh local", run<0>(make_gotoh_aligner<LOCAL>(go), str, ref), "4M1D3M");
    check("gotoh semi-global", run<0>(make_gotoh_aligner<SEMI_GLOBAL>(go), str, ref), "4M1D3M");
    check("banded-semi-global (7)", run<7>(make_gotoh_aligner<SEMI_GLOBAL>(go), str, ref), "4M1D3M");
    // :799-826
    const SimpleGotohScheme real(0, -5, -8, -3);
    check("banded-semi-global (31)",
          run<31>(make_gotoh_aligner<SEMI_GLOBAL>(real),
                  "TTATGTAGGTGGTCTGGTTTTTGCCTTTTAAGCTTCTGCAAAAAACAACAACAAACTTGTGGTATTACACTGACTCTACAGATCAATTTGGGGACAACTTCCATGTGTTCCACCACCAATACTGAATCTTTCAATCGACTGACGTGGTAT",
                  "ATCGGATTCTTTCTTACTTGTAGGTGGTCTGGTTTTTGCCTTTTAAGCTTCTGCAAAAAACAACAACAAACTTGTGGTATTACACTGACTCTACAGATCAATTTGGGGACAACTTCCATGTGTTCCACCACCAATACTGAATCTTTCAATCGACTGACGTGGTATCTCTCTCTCCATCTAT"),
          "147M2D3M");
    // :829-904
    const char *str2 =
        "TAGGAGGTAACATGTATGGAGCATTTACCATAGGCCAAGCACTGTTCTAAGAACTTCGGACATGTTATCTCACTTGTATAAGTACTTAGGTGCCTACAACATAAGCAGCACCTGGTAAATTAAGTATTGAAAAAATGCAGATCG";
    const char *ref2 =
        "CAGCACTGACCGGTGAGCATAAACCCTGGGGATGCCCAGAGCTGGTACAGCCAGGAGCTCCAGAAGCGTGGGATTCTCAGAGGGAAGTGGAGCTCACTGCTCTACAGGTCCTATTCAAGTTAGAAAGTAAGATACAATGCACACAAAGCCAAATTGTC"
        "ATCATTCAGCTCCTATTACAGGGGAACTAAGAGCTGCATTGAAAATTATTTGCAAAGCTTGTAAGTGGTTCTGCCACTTATTAGCCGTGTGAACCTTAGCAAATTACCTAGCGTCTCTGAGTTTCAACTTCCTCATCTACAAAATAGAAATGATAATAAT"
        "AACCGCATCGCAAGAGTTGTTGGAAAAATGAAAATGAGGTATCATAGGAGGTAACATGTATGGAGCATTTACCATAGGCCAAGCACTGTTCTAAGAACTTCGGACATGTTATCTCACTTGTATAAGTACTTAGGTGCCTACAACATAAACAGCACCTGGT"
        "AAATTAAGTATTGAAAAAATGC";
    check("real gotoh semi-global", run<0>(make_gotoh_aligner<SEMI_GLOBAL>(real), str2, ref2), "6I138M");
    check("real ed semi-global", run<0>(make_edit_distance_aligner<SEMI_GLOBAL>(), str2, ref2), "1I1M2I1M3I136M");
    printf("%s\n", failures ? "FAILED" : "all cases match the reference's strings");
    return failures ? 1 : 0;
}
