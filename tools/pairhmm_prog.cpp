// pairhmm_prog.cpp — command-line driver of the PairHMM path with the reference
// drivers' contract, as a client of the flat C-ABI only (include/gasalx.h, -lgasal).
//
//   pairhmm_prog [-fakesize N] [-print all|first|last|none] input.txt
//
// * input.txt: the reference's input format (groups of `size` pairs; read, base /
//   insertion / deletion / gcp qualities, haplotype), parsed by gasalx_hmm_file_read
//   (tile_1.cu:246-290).
// * Each group is one batch, as in the reference's while(!feof) loop.  With
//   -fakesize N, pair 0 of the group is replicated N times first
//   (inter_task/Synthetic_data/tile_1/tile_1.cu:298-313; the Intra-task synthetic
//   drivers do the same).
// * The batch runs through gasalx_pairhmm_quals_host: sorted by (read, haplotype)
//   length, ph2pr parameters formed on the device (tile_1.cu:216-220, 325, 415-419).
// * Per result line "  i=%d  %e" (tile_1.cu:530-531 prints i = 0; the Intra-task
//   synthetic driver prints the last, improved_warp_based.cu:433-434); -print picks
//   which (default first).  Then the timing line and "GCUPS: %lf" computed as the
//   reference does, from the last pair's read and haplotype lengths times the batch
//   size (tile_1.cu:552-553).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <string>
#include <vector>

#include "gasalx.h"

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC_RAW, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static int die(const char *what, int rc) {
    fprintf(stderr, "pairhmm_prog: %s failed (%d): %s\n", what, rc, gasalx_last_error());
    return 1;
}

int main(int argc, char **argv) {
    long fakesize = 0;
    std::string print = "first";
    const char *path = nullptr;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-fakesize") && i + 1 < argc) fakesize = atol(argv[++i]);
        else if (!strcmp(argv[i], "-print") && i + 1 < argc) print = argv[++i];
        else if (argv[i][0] == '-') { fprintf(stderr, "unknown option %s\n", argv[i]); return 1; }
        else path = argv[i];
    }
    if (!path) {
        fprintf(stderr, "usage: pairhmm_prog [-fakesize N] [-print all|first|last|none] input.txt\n");
        return 1;
    }
    double t0 = now();
    gasalx_hmm_file *f = nullptr;
    int rc = gasalx_hmm_file_read(path, &f);
    if (rc) return die("gasalx_hmm_file_read", rc);
    const double read_time = now() - t0;
    gasalx_engine *eng = nullptr;
    if ((rc = gasalx_engine_create(0, &eng))) return die("gasalx_engine_create", rc);

    double compute = 0, read_read = 0, hap_hap = 0;
    uint64_t last_batch = 0;
    uint32_t first = 0;
    for (uint32_t g = 0; g < f->n_groups; g++) {
        const uint32_t size = f->group_sizes[g];
        if (size == 0) continue;
        gasalx_hmm_qual_batch b;
        memset(&b, 0, sizeof(b));
        std::vector<uint32_t> ro, rl, ho, hl;
        if (fakesize > 0) {   // replicate pair 0 of the group (tile_1.cu:298-313)
            const uint32_t p = first;
            ro.assign(fakesize, f->read_offsets[p]); rl.assign(fakesize, f->read_lens[p]);
            ho.assign(fakesize, f->hap_offsets[p]); hl.assign(fakesize, f->hap_lens[p]);
            b.n_pairs = (uint32_t)fakesize;
        } else {
            ro.assign(f->read_offsets + first, f->read_offsets + first + size);
            rl.assign(f->read_lens + first, f->read_lens + first + size);
            ho.assign(f->hap_offsets + first, f->hap_offsets + first + size);
            hl.assign(f->hap_lens + first, f->hap_lens + first + size);
            b.n_pairs = size;
        }
        b.reads = f->reads; b.read_offsets = ro.data(); b.read_lens = rl.data();
        b.base_quals = f->base_quals; b.ins_quals = f->ins_quals; b.del_quals = f->del_quals;
        b.haps = f->haps; b.hap_offsets = ho.data(); b.hap_lens = hl.data();
        b.read_bytes = f->read_bytes; b.hap_bytes = f->hap_bytes;
        std::vector<float> res(b.n_pairs);
        const double t1 = now();
        if ((rc = gasalx_pairhmm_quals_host(eng, &b, res.data()))) return die("gasalx_pairhmm_quals_host", rc);
        compute += now() - t1;
        read_read = rl.back();
        hap_hap = hl.back();
        last_batch = b.n_pairs;
        if (print == "all")
            for (uint32_t i = 0; i < b.n_pairs; i++) printf("  i=%u  %e\n", i, res[i]);
        else if (print == "first") printf("  i=%d  %e\n", 0, res[0]);
        else if (print == "last") printf("  i=%u  %e\n", b.n_pairs - 1, res[b.n_pairs - 1]);
        first += size;
    }
    printf("read_time=%e  initial_time=%e  computation_time= %e total_time=%e\n", read_time, 0.0, compute,
           now() - t0);
    printf("GCUPS: %lf \n", compute > 0 ? (double)last_batch * read_read * hap_hap / compute / 1e9 : 0.0);
    gasalx_engine_destroy(eng);
    gasalx_hmm_file_free(f);
    return 0;
}
