// synth.cpp — synthetic workloads of SURVEY.md §8(d) (std::mt19937_64, seeded).
// Benchmark / test data only; writes GASAL2-layout batches (N_CODE padding to a
// multiple of 8, offsets including pads, unpadded lengths: README.md:145).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "gasalx.h"

namespace {

const char kBases[4] = {'A', 'C', 'G', 'T'};

struct Spec { uint32_t qlen, tlen; double sub, indel; int mode; };
// mode 0: target = mutated query (config 1, 3); 1: half related / half unrelated
// (config 2); 2: read = mutated substring of a target window (config 4)
bool spec_for(int kind, Spec *s) {
    switch (kind) {
        case 1: *s = {64, 64, 0.05, 0.01, 0}; return true;
        case 2: *s = {150, 150, 0.08, 0.01, 1}; return true;
        case 3: *s = {300, 300, 0.05, 0.01, 0}; return true;
        case 4: *s = {150, 182, 0.04, 0.005, 2}; return true;
        default: return false;
    }
}

uint32_t pad8(uint32_t x) { return (x + 7u) & ~7u; }

std::string random_seq(std::mt19937_64 &g, uint32_t n) {
    std::string s(n, 'A');
    for (uint32_t i = 0; i < n; i++) s[i] = kBases[g() & 3];
    return s;
}

// substitutions with rate sub, indels (length 1-3) with rate indel, then
// trimmed or extended with random bases to exactly `len`
std::string mutate(std::mt19937_64 &g, const std::string &src, double sub, double indel, uint32_t len) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::string out;
    out.reserve(src.size() + 16);
    for (size_t i = 0; i < src.size();) {
        const double u = U(g);
        if (u < indel * 0.5) {                       // insertion
            const int k = 1 + (int)(g() % 3);
            for (int j = 0; j < k; j++) out.push_back(kBases[g() & 3]);
            out.push_back(src[i++]);
        } else if (u < indel) {                      // deletion
            i += 1 + (size_t)(g() % 3);
        } else if (u < indel + sub) {                // substitution to a different base
            const char c = src[i++];
            char d = c;
            while (d == c) d = kBases[g() & 3];
            out.push_back(d);
        } else {
            out.push_back(src[i++]);
        }
    }
    if (out.size() > len) out.resize(len);
    while (out.size() < len) out.push_back(kBases[g() & 3]);
    return out;
}

// Pairs are generated in blocks of kSynthBlock: block b draws from its own
// mt19937_64, seeded with `seed` for block 0 (so batches of up to 65,536 pairs are
// the plain sequential stream) and splitmix64(seed + b) after that.  Any range of
// a batch can therefore be generated on its own, and blocks run in parallel:
// each rank of a multi-GPU run generates exactly its shard of one global batch.
constexpr uint64_t kSynthBlock = 65536;

uint64_t block_seed(uint64_t seed, uint64_t b) {
    if (b == 0) return seed;
    uint64_t z = seed + b * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// pairs [lo, hi) of the global batch, written at slot k - first
void synth_block(const Spec &s, uint64_t seed, uint64_t b, uint64_t lo, uint64_t hi, uint64_t first, uint8_t *qbat,
                 uint32_t *qoff, uint32_t *qlen, uint8_t *tbat, uint32_t *toff, uint32_t *tlen) {
    std::mt19937_64 g(block_seed(seed, b));
    const uint32_t qp = pad8(s.qlen), tp = pad8(s.tlen);
    for (uint64_t k = b * kSynthBlock; k < hi; k++) {
        std::string q, t;
        if (s.mode == 0) {
            q = random_seq(g, s.qlen);
            t = mutate(g, q, s.sub, s.indel, s.tlen);
        } else if (s.mode == 1) {
            q = random_seq(g, s.qlen);
            t = (k & 1) ? random_seq(g, s.tlen) : mutate(g, q, s.sub, s.indel, s.tlen);
        } else {
            t = random_seq(g, s.tlen);
            const uint32_t off = (uint32_t)(g() % (s.tlen - s.qlen + 1));
            q = mutate(g, t.substr(off, s.qlen), s.sub, s.indel, s.qlen);
        }
        if (k < lo) continue;   // the block's stream is drawn from its start
        const uint64_t slot = k - first;
        const uint64_t qo = slot * qp, to = slot * tp;
        std::memcpy(qbat + qo, q.data(), s.qlen);
        std::memset(qbat + qo + s.qlen, 'N', qp - s.qlen);
        std::memcpy(tbat + to, t.data(), s.tlen);
        std::memset(tbat + to + s.tlen, 'N', tp - s.tlen);
        qoff[slot] = (uint32_t)qo; toff[slot] = (uint32_t)to;
        qlen[slot] = s.qlen; tlen[slot] = s.tlen;
    }
}

}  // namespace

extern "C" int gasalx_synth_sizes(int kind, uint32_t n, uint64_t *qb, uint64_t *tb) {
    Spec s;
    if (!spec_for(kind, &s) || !qb || !tb) return GASALX_EINVAL;
    *qb = (uint64_t)n * pad8(s.qlen);
    *tb = (uint64_t)n * pad8(s.tlen);
    return GASALX_OK;
}

extern "C" int gasalx_synth_spec(int kind, uint32_t *q_len, uint32_t *t_len) {
    Spec s;
    if (!spec_for(kind, &s) || !q_len || !t_len) return GASALX_EINVAL;
    *q_len = s.qlen;
    *t_len = s.tlen;
    return GASALX_OK;
}

extern "C" int gasalx_synth_range(int kind, uint64_t seed, uint64_t start, uint32_t n, uint8_t *qbat, uint32_t *qoff,
                                  uint32_t *qlen, uint8_t *tbat, uint32_t *toff, uint32_t *tlen) {
    Spec s;
    if (!spec_for(kind, &s) || !qbat || !qoff || !qlen || !tbat || !toff || !tlen) return GASALX_EINVAL;
    if ((uint64_t)n * pad8(std::max(s.qlen, s.tlen)) >= (1ull << 32)) return GASALX_ERANGE;   // uint32 offsets
    const uint64_t end = start + n;
    const uint64_t b0 = start / kSynthBlock, b1 = (end + kSynthBlock - 1) / kSynthBlock;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const char *env = std::getenv("OMP_NUM_THREADS");
    unsigned nt = env && std::atoi(env) > 0 ? (unsigned)std::atoi(env) : std::min(hw, 16u);
    nt = (unsigned)std::min<uint64_t>(nt, b1 - b0);
    std::atomic<uint64_t> next{b0};
    auto work = [&] {
        for (uint64_t b; (b = next.fetch_add(1)) < b1;)
            synth_block(s, seed, b, std::max(start, b * kSynthBlock), std::min(end, (b + 1) * kSynthBlock), start,
                        qbat, qoff, qlen, tbat, toff, tlen);
    };
    std::vector<std::thread> th;
    for (unsigned i = 1; i < nt; i++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    return GASALX_OK;
}

extern "C" int gasalx_synth_pairs(int kind, uint64_t seed, uint32_t n, uint8_t *qbat, uint32_t *qoff, uint32_t *qlen,
                                  uint8_t *tbat, uint32_t *toff, uint32_t *tlen) {
    return gasalx_synth_range(kind, seed, 0, n, qbat, qoff, qlen, tbat, toff, tlen);
}
