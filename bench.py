#!/usr/bin/env python3
"""Benchmark of the hot path: batched affine-gap alignment (GASAL2 kernels) and
PairHMM on MI355X, BASELINE.json configs 1-5.  Default: config 2, SW local
score + end positions over 1M pairs x 150 bp per GPU.

A step = one pass of the HIP engine over this rank's shard of one global
synthetic batch (SURVEY.md §8(d) generator, gasalx_synth_range), already
resident in HBM, launched through the C-ABI (gasalx_align_device) on a
non-default stream; with N > 1 the step also all-gathers every rank's int32
scores (RCCL over xGMI), the exchange step of SURVEY.md §8(e).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--pairs P]

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) the ranks come
from the environment; `--gpus N` without WORLD_SIZE starts N ranks itself
(torch.distributed.run, 127.0.0.1) before any GPU call.  Timing is bracketed by
a barrier + synchronize on both sides, the max over ranks is reported.

After the timed steps every rank checks its shard's device outputs against the
CPU oracle (oracle/, the reference's kernels restated in C), bit-exactly for
integer outputs, rtol 1e-5 for PairHMM, and rank 0 checks the gathered scores;
the line carries "parity".  At N = 1 the same oracle run is timed as the CPU
baseline (the box's cores), beside a 1-core sample.
"""
import argparse
import dataclasses
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
# torch first: its bundled HIP runtime (soname libamdhip64.so.7) must be the one
# libgasal binds to; loading libgasal first would bring in /opt/rocm's copy as well,
# and two HIP runtimes in one process do not share the device
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd"))
import gasal_ffi as G  # noqa: E402
import gasal_dist as D  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SIMDS, CLOCK = 256 * 4, 2.4e9
# VALU lane throughput, MI355X_MICROARCH.md: SIMD-32, a wave64 VALU instruction every 2 cycles per
# SIMD -> 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz = 78.6 T 32-bit lane-ops/s; the FP32 vector peak
# counts an FMA as 2 flops: 157.3 TFLOPS
VALU_LANE_OPS = SIMDS * 32 * CLOCK
FP32_VECTOR_PEAK = 2 * VALU_LANE_OPS            # 157.3 TFLOPS (MI355X_MICROARCH.md MFMA table, F32 row)

MAIN_METRIC = "GCUPS on batched 150bp affine-gap SW at 1/2/4/8 MI355X; HBM-roofline %"

# name: kind (synth config), pairs, scaling ("weak": pairs per GPU; "strong": global
# pairs), params, algorithmic bytes per pair, algorithmic ops per cell, label
WORKLOADS = {
    "sw_local": dict(kind=2, pairs=1_000_000, scaling="weak", params=dict(algo=G.LOCAL), bytes=332, ops=12,
                     label="config2: SW local affine (a1 b4 o6 e1) score+ends, 1M pairs x 150bp per GPU, "
                           "seed 0x5EED0002"),
    "sw_local_start": dict(kind=2, pairs=1_000_000, scaling="weak", params=dict(algo=G.LOCAL, start_pos=G.WITH_START),
                           bytes=340, ops=12, streams=2,
                           label="config2 + WITH_START: SW local score+ends+starts, 1M pairs x 150bp per GPU"),
    "sw_local_tb": dict(kind=2, pairs=1_000_000, scaling="weak", params=dict(algo=G.LOCAL, start_pos=G.WITH_TB),
                        bytes=340 + 152, ops=16, streams=2,
                        label="config2 + WITH_TB: SW local score+ends+starts+CIGAR, 1M pairs x 150bp per GPU"),
    "sw_local_300": dict(kind=3, pairs=1_000_000, scaling="weak", params=dict(algo=G.LOCAL), bytes=632, ops=12,
                         label="config-3 data (300 x 300, target = mutated query) through SW local score+ends, "
                               "1M pairs per GPU (VERDICT r03 item 5: past the single-key window)"),
    "nw_score": dict(kind=3, pairs=100_000, scaling="weak", params=dict(algo=G.GLOBAL), bytes=624, ops=16,
                     label="config-3 data, NW global score only (no traceback), 100K pairs x 300bp per GPU: the "
                           "sweep the band traceback's first pass is built on"),
    "nw_tb": dict(kind=3, pairs=100_000, scaling="weak", params=dict(algo=G.GLOBAL, start_pos=G.WITH_TB), bytes=650,
                  ops=16, streams=3, label="config3: NW global + traceback/CIGAR, 100K pairs x 300bp per GPU, seed 0x5EED0003"),
    "semi": dict(kind=4, pairs=10_000_000, scaling="strong",
                 params=dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET), bytes=364, ops=11,
                 label="config4: semi-global TARGET/TARGET, 10M 150bp reads in 182bp windows sharded over the "
                       "GPUs, RCCL gather of scores, seed 0x5EED0004"),
    "semi_start": dict(kind=4, pairs=10_000_000, scaling="strong",
                       params=dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET, start_pos=G.WITH_START,
                                   max_query_len=192), bytes=372, ops=11, streams=2,
                       label="config4 + WITH_START: semi-global TARGET/TARGET score+ends+starts, 10M reads sharded"),
    "semi_banded": dict(kind=4, pairs=10_000_000, scaling="strong", params=dict(algo=G.BANDED, k_band=16), bytes=364,
                        ops=None, label="config4 data, banded-tiled k_band=16 (SURVEY §8(d) second run), 10M reads "
                                      "sharded; cells = full rectangle"),
    "pairhmm": dict(kind=5, pairs=100_000, scaling="weak", params=None, bytes=4762, ops=11,
                    label="config5: PairHMM fp32 forward, 100K reads x haplotypes (250 x 500) per GPU, "
                          "seed 0x5EED0005"),
    "nvbio_gotoh": dict(kind=6, pairs=262_144, scaling="weak", params=None, bytes=88, ops=9,
                        label="second front-end (nvbio BatchedAlignmentScore idiom, sw-benchmark.cu:585-615): "
                              "Gotoh (2,-1,-2,-1) semi-global, 256K 150bp reads (4-bit DNA_N) per GPU against one "
                              "1,000bp 2-bit reference, seed 0x5EED0006"),
    "nvbio_banded": dict(kind=6, band=16, pairs=1_048_576, scaling="weak", params=None, bytes=128, ops=9,
                         label="second front-end, banded (nvbio BatchedBandedAlignmentScore<16>, batched.h:337): "
                               "Gotoh (2,-1,-2,-1) semi-global, 1M 150bp reads (4-bit DNA_N) per GPU, each against "
                               "its 165bp reference window (2-bit) starting 7bp before the read's origin; cells = "
                               "the band's (150 x 16 per pair), seed 0x5EED0006"),
    "ksw": dict(kind=2, pairs=1_000_000, scaling="weak", params=dict(algo=G.KSW), bytes=340, ops=14, packed=True,
                seed_score=10,
                label="GASAL2 KSW (ksw_kernel_template.h:47-199, BWA ksw_extend semantics) on config-2 data, 1M "
                      "pairs x 150bp per GPU, seed score 10 per pair; cells = the full rectangle (the kernel "
                      "trims, as the reference does)"),
    "boundary": dict(kind=7, pairs=1_000_000, scaling="weak", params=dict(algo=G.LOCAL), bytes=None, ops=12,
                     label="the drop-in boundary driven as the reference's test_prog drives it (test_prog.cpp:12,18,"
                           "202-347): T host threads x 2 gasal_gpu_storage x 5,000-pair host batches through "
                           "gasal_host_batch_fill / gasal_aln_async / gasal_is_aln_async_done, SW local score + "
                           "ends, over the reference's 20K sample pairs (query 150 bp, target 152-277 bp) "
                           "replicated to 1M pairs; host pages to host results, PCIe included"),
    "cpu_plumbing": dict(kind=1, pairs=1024, scaling="weak", params=dict(algo=G.LOCAL), bytes=152, ops=12,
                         label="config1: 1024 pairs 64x64 SW local through the host-side CPU verify scorer "
                               "(oracle/), same batch through the GPU, seed 0x5EED0001"),
}
METRICS = {
    "pairhmm": "GCUPS of PairHMM fp32 forward (config 5, 250x500) on MI355X",
    "nvbio_gotoh": "GCUPS of nvbio-style batched Gotoh semi-global scoring (sw-benchmark idiom) on MI355X",
    "nvbio_banded": "GCUPS (band cells) of nvbio-style banded (16) Gotoh semi-global scoring on MI355X",
    "cpu_plumbing": "GCUPS of the repo's host-side CPU verify scorer (config 1, 1024 x 64x64)",
    "boundary": "GCUPS end to end through gasal_aln_async (test_prog pattern, host batches to host results) on MI355X",
    "ksw": "GCUPS of GASAL2 KSW extension (config-2 data, 1M x 150bp) on MI355X",
    "sw_local_300": "GCUPS of batched 300bp affine-gap SW local (config-3 data) on MI355X",
    "nw_score": "GCUPS of batched 300bp affine-gap NW global score (config-3 data) on MI355X",
}
SEEDS = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005, 6: 0x5EED0006}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warmup steps (default: at least 3 steps and at least --warmup-seconds of GPU "
                         "time, so the timed steps run at the clock the GPU settles at under load: a cold "
                         "MI355X ramps over the first ~30 ms, profiles/r05/clock_ramp.md)")
    ap.add_argument("--warmup-seconds", type=float, default=0.5)
    ap.add_argument("--pairs", type=int, default=0,
                    help="pairs per GPU (weak workloads) or global pairs (strong); default: the config's")
    ap.add_argument("--workload", default="sw_local", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="1-core CPU baseline sample budget")
    ap.add_argument("--parity-pairs", type=int, default=2_000_000,
                    help="per rank: check at most this many pairs of the shard against the oracle (0 = none)")
    ap.add_argument("--streams", type=int, default=None,
                    help="GASAL workloads: engines (gasal_gpu_storage) on their own streams, steps "
                         "issued round-robin as the reference's host program drives gasal_aln_async "
                         "(test_prog.cpp NB_STREAMS = 2 per host thread); 1 = every step on one stream.  Default: "
                         "2 for the traceback and WITH_START workloads (a step's walk or reverse-pass prep runs "
                         "beside the next step's DP), 3 for config 3 (profiles/r04/p_nw_tb_s*.json: 2 -> 3,860, "
                         "3 -> 4,189, 4 -> 3,727 GCUPS in one session), else 1")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline timings")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-staged (PCIe-inclusive) timing")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: leave out the all-gather of scores")
    ap.add_argument("--force-int32", action="store_true",
                    help="probe: every block on the int32 kernels (GASALX_PACKED16=0), as pairs outside the "
                         "packed kernels' 16-bit value window run")
    ap.add_argument("--scores", default="",
                    help="probe: match,mismatch,gap_open,gap_extend overriding the workload's scores "
                         "(e.g. 2,4,6,1 takes config 2 outside the 16-bit window)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1: torch.distributed backend (nccl = RCCL over xGMI; gloo stages the exchange "
                         "through host memory, so several ranks can share one GPU)")
    ap.add_argument("--threads", default="1,2,4,8",
                    help="boundary workload: host thread counts to run (test_prog -n), comma separated")
    ap.add_argument("--batch-pairs", type=int, default=5000,
                    help="boundary workload: pairs per host batch (test_prog's STREAM_BATCH_SIZE = 5,000)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's shard of the global batch as a JSON line and exit (no GPU call)")
    return ap.parse_args()


# ----------------------------------------------------------------- launch ---
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`--gpus N` outside torchrun: run this script as N ranks (one process per GPU)
    through torch.distributed.run, before this process touches the GPU, and exit
    with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.exit(subprocess.call(cmd, env=env))


# ------------------------------------------------------------------ data ----
PH_BLOCK = 8192


def synth_pairhmm(start, n, seed, rl=250, hl=500):
    """SURVEY.md 8(d) config 5, pairs [start, start + n) of the global batch: haplotype
    500 bp uniform; read = 250-bp substring with 2% mismatches; base quals U[10,40],
    insertion/deletion quals 45 (gcp ignored).  Blocks of 8,192 pairs, each from
    numpy's default_rng((seed, block)), so a rank generates only its shard."""
    alpha = np.frombuffer(b"ACGT", np.uint8)
    reads, haps, bqs = [], [], []
    b0, b1 = start // PH_BLOCK, (start + n + PH_BLOCK - 1) // PH_BLOCK
    for b in range(b0, b1):
        rng = np.random.default_rng((seed, b))
        m = PH_BLOCK
        hb = alpha[rng.integers(0, 4, (m, hl))]
        st = rng.integers(0, hl - rl + 1, m)
        rb = hb[np.arange(m)[:, None], st[:, None] + np.arange(rl)[None, :]].copy()
        flip = rng.random((m, rl)) < 0.02
        rb[flip] = alpha[(np.searchsorted(alpha, rb[flip]) + rng.integers(1, 4, int(flip.sum()))) % 4]
        bq = rng.integers(10, 41, (m, rl)).astype(np.uint8)
        lo, hi = max(start, b * PH_BLOCK) - b * PH_BLOCK, min(start + n, (b + 1) * PH_BLOCK) - b * PH_BLOCK
        reads.append(rb[lo:hi]); haps.append(hb[lo:hi]); bqs.append(bq[lo:hi])
    reads, haps, bq = np.concatenate(reads), np.concatenate(haps), np.concatenate(bqs).reshape(-1)
    iq = np.full(n * rl, 45, np.uint8)
    qm, de, xi, al = G.pairhmm_params(bq, iq, iq)
    return dict(reads=reads.reshape(-1), read_offsets=np.arange(n, dtype=np.uint32) * rl,
                read_lens=np.full(n, rl, np.uint32), qm=qm, delta=de, xiksi=xi, alpha=al, haps=haps.reshape(-1),
                hap_offsets=np.arange(n, dtype=np.uint32) * hl, hap_lens=np.full(n, hl, np.uint32), bq=bq, iq=iq)


NV_REF_LEN, NV_READ_LEN = 1000, 150
NV_ALIGNER = dict(aligner=G.NV_GOTOH, type=G.NV_SEMI_GLOBAL, match=2, mismatch=-1, gap_open=-2, gap_ext=-1)


def pack_uniform(codes, bits, big):
    """nvbio PackedStream words of a flat symbol array (fast path of G.PackedSet.pack)."""
    per = 32 // bits
    flat = np.concatenate([codes.astype(np.uint32), np.zeros((-len(codes)) % per + per, np.uint32)])
    k = np.arange(per, dtype=np.uint32)
    shift = (32 - bits * (k + 1)) if big else bits * k
    return np.bitwise_or.reduce(flat.reshape(-1, per) << shift, axis=1).astype(np.uint32)


def synth_nvbio(start, n, seed, band=0):
    """Reads of 150 bp taken from a 1,000 bp random reference at uniform offsets with
    5% substitutions (N included, as DNA_N reads carry them); blocks of 8,192 reads
    from default_rng((seed, block)) so a rank generates only its shard.  Codes:
    reads DNA_N 4-bit big-endian, reference 2-bit little-endian (sw-benchmark.cu:73-74, 290-330)."""
    ref = np.random.default_rng((seed, 1 << 40)).integers(0, 4, NV_REF_LEN).astype(np.uint32)
    reads = []
    b0, b1 = start // PH_BLOCK, (start + n + PH_BLOCK - 1) // PH_BLOCK
    for b in range(b0, b1):
        rng = np.random.default_rng((seed, b))
        st = rng.integers(0, NV_REF_LEN - NV_READ_LEN + 1, PH_BLOCK)
        rd = ref[st[:, None] + np.arange(NV_READ_LEN)[None, :]].copy()
        sub = rng.random(rd.shape) < 0.05
        rd[sub] = rng.integers(0, 5, int(sub.sum()))
        lo, hi = max(start, b * PH_BLOCK) - b * PH_BLOCK, min(start + n, (b + 1) * PH_BLOCK) - b * PH_BLOCK
        reads.append(rd[lo:hi])
    codes = np.concatenate(reads).reshape(-1)
    pat = G.PackedSet(pack_uniform(codes, 4, True), np.arange(n + 1, dtype=np.uint32) * NV_READ_LEN, 0, 4, True)
    txt = G.PackedSet(pack_uniform(ref, 2, False), None, NV_REF_LEN, 2, False)
    if band:
        # banded: each read against its own window of NV_READ_LEN + band - 1 symbols that
        # starts band // 2 before the read's origin (clamped to the reference)
        wl_ = NV_READ_LEN + band - 1
        sts = []
        for b in range(b0, b1):
            st = np.random.default_rng((seed, b)).integers(0, NV_REF_LEN - NV_READ_LEN + 1, PH_BLOCK)
            lo, hi = max(start, b * PH_BLOCK) - b * PH_BLOCK, min(start + n, (b + 1) * PH_BLOCK) - b * PH_BLOCK
            sts.append(st[lo:hi])
        w0 = np.clip(np.concatenate(sts) - band // 2, 0, NV_REF_LEN - wl_)
        tcodes = ref[w0[:, None] + np.arange(wl_)[None, :]].reshape(-1)
        txt = G.PackedSet(pack_uniform(tcodes, 2, False), np.arange(n + 1, dtype=np.uint32) * wl_, 0, 2, False)
        return dict(codes=codes, pat=pat, txt=txt, band=band, tcodes=tcodes, wlen=wl_)
    return dict(codes=codes, pat=pat, txt=txt)


def nv_oracle(O, nv, sub, n_threads, lo=0, hi=None):
    """The oracle over reads [lo, hi) of a kind-6 batch (sub: their packed patterns)."""
    al = G.NvAligner(**NV_ALIGNER)
    if not nv.get("band"):
        return O.nv_score(al, sub, nv["txt"], n_threads=n_threads)
    w = nv["wlen"]
    hi = len(nv["pat"].offsets) - 1 if hi is None else hi
    t = G.PackedSet(pack_uniform(nv["tcodes"][lo * w:hi * w], 2, False), np.arange(hi - lo + 1, dtype=np.uint32) * w,
                    0, 2, False)
    return O.nv_banded_score(al, nv["band"], sub, t, n_threads=n_threads)


def nv_subset(nv, e):
    codes = nv["codes"][:e * NV_READ_LEN]
    return G.PackedSet(pack_uniform(codes, 4, True), np.arange(e + 1, dtype=np.uint32) * NV_READ_LEN, 0, 4, True)


def ph_subset(h, e):
    """The first e pairs of a PairHMM batch (uniform lengths)."""
    rl, hl = int(h["read_lens"][0]), int(h["hap_lens"][0])
    out = {k: h[k][:e * rl] for k in ("reads", "qm", "delta", "xiksi", "alpha")}
    out.update(haps=h["haps"][:e * hl], read_offsets=h["read_offsets"][:e], read_lens=h["read_lens"][:e],
               hap_offsets=h["hap_offsets"][:e], hap_lens=h["hap_lens"][:e])
    return out


# ---------------------------------------------------------------- oracle ----
def _oracle(native=False):
    """The CPU oracle.  native: its -O3 -march=native build for this host,
    compiled here, used for the timed baseline (and the parity run that doubles as it)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    O.NATIVE_OK = O.native_available() if native else False
    return O


def lib_sha256():
    import hashlib
    h = hashlib.sha256()
    with open(G.LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def oracle_threads():
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        return env
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return min(16, n)   # one GPU's CPU share on the pool (16); the line records the host's total


def host_info():
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "NUMA node(s)", "Socket(s)", "Thread(s) per core"):
                info[k.strip().lower().replace(" ", "_").replace("(s)", "s")] = v.strip()
    except Exception:
        pass
    return info


def oracle_align(O, batch, pkw, threads, seed_score=None):
    seeds = None if seed_score is None else np.full(batch.n, seed_score, np.uint32)
    return O.align(batch, O.make_params(**pkw), seed_scores=seeds, n_threads=threads)


def oracle_pairhmm(O, h, threads):
    return O.pairhmm(h["reads"], h["read_offsets"], h["read_lens"], h["qm"], h["delta"], h["xiksi"], h["alpha"],
                     h["haps"], h["hap_offsets"], h["hap_lens"], n_threads=threads)


def cells_of(batch):
    return int(np.sum(batch.q_lens.astype(np.int64) * batch.t_lens.astype(np.int64)))


def band_cells_of(batch, k_band):
    """Cells the banded-tiled kernel computes: 64 per 8x8 tile of the band, strip i
    covering query tiles [max(0, i - kother + 1), min(k_band/8 + i, QR)) with
    kother = TR - (QR - k_band/8) (banded.h:35, :73-75)."""
    kbw = k_band >> 3
    qr = (batch.q_lens.astype(np.int64) + 7) // 8
    tr = (batch.t_lens.astype(np.int64) + 7) // 8
    total = 0
    for (a, b), cnt in zip(*np.unique(np.stack([qr, tr], 1), axis=0, return_counts=True)):
        ko = b - (a - kbw)
        a, b, ko = int(a), int(b), int(ko)
        tiles = sum(max(0, min(kbw + i, a) - max(0, i - ko + 1)) for i in range(b))
        total += int(cnt) * 64 * tiles
    return total


def single_core_rate(O, kind, data, pkw, budget_s, seed_score=None):
    """The oracle on 1 thread over a prefix of the rank-0 shard, bounded by budget_s."""
    chunk = 256 if kind in (5, 6) else 4096
    done, cells, used = 0, 0, 0.0
    n = len(data["read_lens"]) if kind == 5 else (len(data["pat"].offsets) - 1 if kind == 6 else data.n)
    while used < budget_s and done < n:
        e = min(done + chunk, n)
        if kind == 6:
            codes = data["codes"][done * NV_READ_LEN:e * NV_READ_LEN]
            sub = G.PackedSet(pack_uniform(codes, 4, True), np.arange(e - done + 1, dtype=np.uint32) * NV_READ_LEN,
                              0, 4, True)
            t0 = time.perf_counter()
            nv_oracle(O, data, sub, 1, done, e)
            used += time.perf_counter() - t0
            cells += (e - done) * NV_READ_LEN * (data.get("band") or NV_REF_LEN)
        elif kind == 5:
            sub = {k: (v[done * 250:e * 250] if k in ("reads", "qm", "delta", "xiksi", "alpha")
                       else v[done * 500:e * 500] if k == "haps" else v[done:e]) for k, v in data.items()}
            sub["read_offsets"] = sub["read_offsets"] - sub["read_offsets"][0]
            sub["hap_offsets"] = sub["hap_offsets"] - sub["hap_offsets"][0]
            t0 = time.perf_counter()
            oracle_pairhmm(O, sub, 1)
            used += time.perf_counter() - t0
            cells += int(np.sum(sub["read_lens"].astype(np.int64) * sub["hap_lens"].astype(np.int64)))
        else:
            sub = data.slice(done, e)
            t0 = time.perf_counter()
            oracle_align(O, sub, pkw, 1, seed_score)
            used += time.perf_counter() - t0
            cells += cells_of(sub)
        done = e
    return {"value": round(cells / used / 1e9, 4), "unit": "GCUPS", "cores": 1,
            "sample": f"first {done} pairs of the rank-0 shard ({cells / 1e9:.3f} G cells, {used:.1f} s)"}


# ---------------------------------------------------------------- parity ----
def compare_align(g, o, fields, batch=None, cigar=False):
    """Per-field mismatch counts between device results g and oracle results o.
    CIGAR: n_ops for every pair; bytes for every pair whose CIGAR fits its pad8(ql)
    slot and whose left neighbour's does too (an overflowing CIGAR runs
    into the next slot, order-dependent in the reference)."""
    mism = {f: int(np.count_nonzero(g[f] != o[f])) for f in fields}
    extra = {}
    if cigar:
        mism["n_ops"] = int(np.count_nonzero(g["n_ops"] != o["n_ops"]))
        slot = (batch.q_lens.astype(np.int64) + 7) // 8 * 8
        over = o["n_ops"].astype(np.int64) > slot
        ok = ~over
        ok[1:] &= ~over[:-1]
        gc, oc = g["cigar"], o["cigar"]
        bad = 0
        offs, nops = batch.q_offsets.astype(np.int64), o["n_ops"].astype(np.int64)
        # vectorised byte compare over the checked pairs' CIGAR bytes
        diff = np.flatnonzero(gc[:len(oc)] != oc)
        if diff.size:
            owner = np.searchsorted(offs, diff, side="right") - 1
            rel = diff - offs[owner]
            hit = ok[owner] & (rel < nops[owner])
            bad = int(np.unique(owner[hit]).size)
        mism["cigar_pairs"] = bad
        extra["cigar_pairs_skipped_q14"] = int((~ok).sum())
    return mism, extra


# ------------------------------------------------------------------ e2e -----
def end_to_end(eng, kind, data, params, cells, reps=5, seed_score=None):
    """PCIe-inclusive rate through the host-buffer entry point (gasalx_align_host /
    gasalx_pairhmm_host): host arrays in, H2D + kernels + D2H, results back in host
    arrays.  Reported beside `value`, never as it."""
    if kind == 6 and data.get("band"):
        call = lambda: eng.nv_banded_score_host(G.NvAligner(**NV_ALIGNER), data["band"], data["pat"], data["txt"])
        path = "gasalx_nv_banded_score_host (pageable host arrays; H2D + kernel + D2H)"
    elif kind == 6:
        call = lambda: eng.nv_score_host(G.NvAligner(**NV_ALIGNER), data["pat"], data["txt"])
        path = "gasalx_nv_score_host (pageable host arrays; H2D + kernel + D2H)"
    elif kind == 5:
        h = data
        args = (h["reads"], h["read_offsets"], h["read_lens"], h["qm"], h["delta"], h["xiksi"], h["alpha"],
                h["haps"], h["hap_offsets"], h["hap_lens"])
        call = lambda: eng.pairhmm_host(*args)
        path = "gasalx_pairhmm_host (pageable host arrays; H2D + kernel + D2H)"
    else:
        fields = ["score"] if params.algo == G.GLOBAL else ["score", "q_end", "t_end"]
        if params.start_pos == G.WITH_START:
            fields += ["q_start", "t_start"]
        seeds = None if seed_score is None else np.full(data.n, seed_score, np.uint32)
        call = lambda: eng.align_host(data, params, fields=fields, seed_scores=seeds)
        path = ("gasalx_align_host (pageable host arrays; chunks of pairs on two streams, "
                "H2D of chunk k+1 overlapping the kernels of chunk k)")

    def timed(fn):
        fn()
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            times.append(time.perf_counter() - t0)
        return float(np.median(times)), times

    dt, times = timed(call)
    res = {"value": round(cells / dt / 1e9, 2), "unit": "GCUPS", "ms_per_batch": round(dt * 1e3, 3),
           "ms_all": [round(t * 1e3, 3) for t in times], "path": path}
    if kind == 5 and "bq" in data:
        # the quality-input path (reference input terms: 4 bytes per read base instead of 17)
        h = data
        hd = G.HmmData(h["reads"], h["read_offsets"], h["read_lens"], h["bq"], h["iq"], h["iq"],
                       np.zeros(0, np.uint8), h["haps"], h["hap_offsets"], h["hap_lens"],
                       np.array([len(h["read_lens"])], np.uint32))
        dtq, _ = timed(lambda: eng.pairhmm_quals_host(hd))
        res["quals_host"] = {"value": round(cells / dtq / 1e9, 2), "ms_per_batch": round(dtq * 1e3, 3),
                             "path": "gasalx_pairhmm_quals_host (read + 3 quality bytes per base in; ph2pr "
                                     "parameters formed on the device; length-sorted classes)"}
    if kind in (5, 6):
        return res
    if params.start_pos != G.WITH_TB and not params.is_packed:
        # the reference's isPacked input (gasal_align.cu:190-201; words as pack_rc_seqs.h:24-31): the
        # caller's pages hold 4-bit codes, half the bytes move and the kernels read the words
        # directly; the outputs must equal the ASCII run's
        pb = dataclasses.replace(data, q_data=pack_host(data.q_data), t_data=pack_host(data.t_data))
        pp = G.make_params(**{**params_kwargs(params), "is_packed": 1})
        ref = eng.align_host(data, params, fields=fields, seed_scores=seeds)
        got = eng.align_host(pb, pp, fields=fields, seed_scores=seeds)
        bad = sum(int(np.count_nonzero(got[f] != ref[f])) for f in fields)
        dtk, _ = timed(lambda: eng.align_host(pb, pp, fields=fields, seed_scores=seeds))
        res["packed_input"] = {"value": round(cells / dtk / 1e9, 2), "ms_per_batch": round(dtk * 1e3, 3),
                               "h2d_bytes": int((data.q_bytes + data.t_bytes) // 2),
                               "mismatches_vs_ascii_input": bad,
                               "path": "gasalx_align_host with isPacked (4-bit words, pageable)"}
    if kind != 5 and params.start_pos == G.WITH_TB:
        host = G.PinnedHost(data.q_bytes)
        dtp, _ = timed(lambda: eng.align_host(data, params, fields=fields, seed_scores=seeds, cigar_out=host.array))
        host.close()
        res["pinned_cigar"] = {"value": round(cells / dtp / 1e9, 2), "ms_per_batch": round(dtp * 1e3, 3)}
    if True:
        # sequence bytes page-locked too, as the reference's host batch pages are
        # (host_batch.cpp:79-153 fills pinned pages), plus the CIGAR buffer for TB
        hq, ht = G.PinnedHost(data.q_bytes), G.PinnedHost(data.t_bytes)
        hq.array[:] = data.q_data
        ht.array[:] = data.t_data
        pb = dataclasses.replace(data, q_data=hq.array, t_data=ht.array)
        hc = G.PinnedHost(data.q_bytes) if params.start_pos == G.WITH_TB else None
        dtp, _ = timed(lambda: eng.align_host(pb, params, fields=fields, seed_scores=seeds,
                                              cigar_out=hc.array if hc else None))
        res["pinned_io"] = {"value": round(cells / dtp / 1e9, 2), "ms_per_batch": round(dtp * 1e3, 3),
                            "pinned": "q/t sequence bytes" + (" + CIGAR buffer" if hc else "")}
        for h in (hq, ht, hc):
            if h:
                h.close()
    return res


def pack_host(b):
    """ASCII bytes -> the reference's packed words (pack_rc_seqs.h:24-31: byte k of each 8 ->
    nibble at bits 31-4k), returned as bytes padded with zeros to the unpacked length."""
    nib = (np.asarray(b, np.uint8).reshape(-1, 8) & 0xF).astype(np.uint32)
    w = np.zeros(nib.shape[0], np.uint32)
    for k in range(8):
        w |= nib[:, k] << np.uint32(28 - 4 * k)
    out = np.zeros(len(b), np.uint8)
    out[:4 * len(w)] = w.view(np.uint8)
    return out


def params_kwargs(p):
    return dict(algo=p.algo, start_pos=p.start_pos, second_best=p.second_best, head=p.head, tail=p.tail,
                match=p.match, mismatch=p.mismatch, gap_open=p.gap_open, gap_extend=p.gap_extend, k_band=p.k_band,
                n_code=p.n_code, n_penalty=p.n_penalty if p.has_n_penalty else None,
                max_query_len=p.max_query_len)


def dtype_label(plan, kind):
    if kind == 5:
        return "fp32"
    if kind == 6:
        return "int16x2 packed (two pairs per lane group, exact value window)" if plan.startswith("nvbio16") \
            else "int32"
    if plan.startswith("wavefront16"):
        return "int16x2 packed (exact value window), int32 fallback per declined block"
    if plan.startswith("banded16"):
        return "int16x2 packed (two pairs per lane, exact value window), int32 fallback per declined pair"
    if plan.startswith("wavefront_"):
        return "int32"
    if plan == "generic_ksw":
        return ("int8 (h, e) entries, int16x2 packed arithmetic (ksw16: two pairs per lane, exact 8-bit bound), "
                "thread-per-pair 8/16/32-bit levels per declined pair")
    return "int32 (int16 row buffer, as the reference)"


# ----------------------------------------------------------------- config 1 -
def run_cpu_plumbing(args, wl):
    """Config 1: the host-side CPU verify scorer over 1024 x 64x64 (timed K passes on
    1 thread), and the same batch through the GPU, compared bit-exactly."""
    O = _oracle()
    n = args.pairs or wl["pairs"]
    batch = G.Batch.synth(1, n, SEEDS[1])
    pkw = wl["params"]
    cells = cells_of(batch)
    for _ in range(3 if args.warmup is None else args.warmup):
        oracle_align(O, batch, pkw, 1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        o = oracle_align(O, batch, pkw, 1)
    dt = time.perf_counter() - t0
    out = {"metric": METRICS["cpu_plumbing"], "value": round(cells * args.steps / dt / 1e9, 4), "unit": "GCUPS",
           "n_gpus": 1, "steps": args.steps, "warmup": 3 if args.warmup is None else args.warmup,
           "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "int32", "data": "synthetic (SURVEY.md 8(d) config 1 generator)",
           "config": {"workload": wl["label"], "pairs": n, "cells_per_step": cells, "cores": 1}}
    # this workload is the CPU path itself: its baseline is the same timing, stated like every other line's
    out["cpu_baseline"] = {"value": out["value"], "unit": "GCUPS", "cores": 1, "kind": "port",
                           "sample": f"the whole workload ({n} pairs x {args.steps} passes, 1 thread)"}
    if torch.cuda.is_available():
        eng = G.Engine(0)
        g = eng.align_host(batch, G.make_params(**pkw), fields=["score", "q_end", "t_end"])
        mism, _ = compare_align(g, o, ("score", "q_end", "t_end"))
        out["parity"] = {"pairs_checked": n, "mismatches": sum(mism.values()), "by_field": mism,
                         "against": "oracle/ (CPU restatement), same batch through gasalx_align_host",
                         "plan": G.describe_plan(G.make_params(**pkw), 64, 64)}
        eng.close()
    print(json.dumps(out), flush=True)


# --------------------------------------------------------------- boundary -
def run_boundary(args, wl):
    """The drop-in boundary the way the reference's test_prog uses it (tools/boundary_bench.cpp: T
    OpenMP threads x 2 storages x 5,000-pair batches through gasal_host_batch_fill / gasal_aln_async
    / gasal_is_aln_async_done), over the reference's own 20K sample pairs replicated to --pairs;
    every pair of the last pass checked against the oracle; beside it the flat host entry point
    (gasalx_align_host) and the device-resident call (gasalx_align_device) on the same pairs."""
    import gzip
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import read_fasta_pairs
    exe = os.path.join(ROOT, "tools", "boundary_bench")
    if not os.path.exists(exe):
        sys.exit("bench.py: tools/boundary_bench is not built (make -C tools)")
    tmp = tempfile.mkdtemp(prefix="gasal_boundary_")
    paths = []
    for name in ("query_batch.fasta.gz", "target_batch.fasta.gz"):
        dst = os.path.join(tmp, name[:-3])
        with gzip.open(os.path.join(ROOT, "tests", "golden", name), "rb") as fi, open(dst, "wb") as fo:
            fo.write(fi.read())
        paths.append(dst)
    q, t, _, _ = read_fasta_pairs()
    base = len(q)
    repl = max(1, (args.pairs or wl["pairs"]) // base)
    n = base * repl
    cells = int(sum(len(a) * len(b) for a, b in zip(q, t))) * repl
    runs, dumps = [], {}
    for T in [int(x) for x in args.threads.split(",") if x]:
        dump = os.path.join(tmp, f"res_{T}.bin")
        cmd = [exe, "--repl", str(repl), "--batch", str(args.batch_pairs),
               "--warm", str(1 if args.warmup is None else max(1, args.warmup)),
               "--reps", str(max(1, min(args.steps, 5))), "--dump", dump, "-y", "local", "-n", str(T)] + paths
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            sys.exit(f"bench.py: boundary_bench -n {T} failed: {r.stderr[-2000:]}")
        line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        runs.append(line)
        dumps[T] = dump
    best = max(runs, key=lambda x: x["gcups"])
    # parity: the oracle over the 20K sample pairs, every replica of every run against it
    O = _oracle(native=not args.no_cpu)
    batch = G.Batch.from_pairs(q, t)
    t_o = time.perf_counter()
    ref = oracle_align(O, batch, wl["params"], oracle_threads())
    oracle_s = time.perf_counter() - t_o
    mism = {}
    for T, path in dumps.items():
        got = np.fromfile(path, np.int32).reshape(5, n)
        bad = 0
        for k, f in enumerate(("score", "q_end", "t_end")):
            bad += int(np.count_nonzero(got[k].reshape(repl, base) != ref[f][None, :]))
        mism[f"threads_{T}"] = bad
    # the flat host entry point and the device-resident call on the same (tiled) pairs
    big = G.Batch(np.tile(batch.q_data, repl),
                  (batch.q_offsets[None, :].astype(np.int64) + np.arange(repl)[:, None] * batch.q_bytes)
                  .reshape(-1).astype(np.uint32), np.tile(batch.q_lens, repl),
                  np.tile(batch.t_data, repl),
                  (batch.t_offsets[None, :].astype(np.int64) + np.arange(repl)[:, None] * batch.t_bytes)
                  .reshape(-1).astype(np.uint32), np.tile(batch.t_lens, repl))
    params = G.make_params(**wl["params"])
    eng = G.Engine(0)
    fields = ["score", "q_end", "t_end"]
    eng.align_host(big, params, fields=fields)
    th = []
    for _ in range(3):
        t0 = time.perf_counter()
        gh = eng.align_host(big, params, fields=fields)
        th.append(time.perf_counter() - t0)
    host_bad = sum(int(np.count_nonzero(gh[f].reshape(repl, base) != ref[f][None, :])) for f in fields)
    dev = torch.device("cuda", 0)
    as_i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    d = {"q_batch": torch.from_numpy(big.q_data).to(dev), "t_batch": torch.from_numpy(big.t_data).to(dev),
         "q_offsets": as_i32(big.q_offsets), "t_offsets": as_i32(big.t_offsets), "q_lens": as_i32(big.q_lens),
         "t_lens": as_i32(big.t_lens), "aln_score": torch.empty(n, dtype=torch.int32, device=dev),
         "q_end": torch.empty(n, dtype=torch.int32, device=dev), "t_end": torch.empty(n, dtype=torch.int32, device=dev)}
    ptrs = {k: v.data_ptr() for k, v in d.items()}
    stream = torch.cuda.Stream(dev)
    mq, mt = int(big.q_lens.max()), int(big.t_lens.max())
    for _ in range(3):
        eng.align_device_ptrs(params, ptrs, big.q_bytes, big.t_bytes, n, mq, mt, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in evs:
        a.record(stream)
        eng.align_device_ptrs(params, ptrs, big.q_bytes, big.t_bytes, n, mq, mt, stream.cuda_stream)
        b.record(stream)
    torch.cuda.synchronize(dev)
    dev_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    dev_bad = sum(int(np.count_nonzero(d[k].cpu().numpy().reshape(repl, base) != ref[f][None, :]))
                  for k, f in (("aln_score", "score"), ("q_end", "q_end"), ("t_end", "t_end")))
    plan = G.describe_plan(params, mq, mt)
    eng.close()
    out = {"metric": METRICS["boundary"], "value": best["gcups"], "unit": "GCUPS", "n_gpus": 1,
           "steps": len(best["pass_ms"]), "warmup": 1 if args.warmup is None else max(1, args.warmup),
           "ms_per_step": best["best_ms"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": dtype_label(plan, 2),
           "data": "the reference's test_prog sample pairs (tests/golden/*_batch.fasta.gz), replicated",
           "config": {"workload": wl["label"], "pairs": n, "base_pairs": base, "replicas": repl, "cells": cells,
                      "threads_best": best["threads"], "storages_per_thread": best["storages"],
                      "batch_pairs": best["batch"], "plan_of_a_batch": G.describe_plan(params, mq, mt)},
           "runs": runs,
           "vs_reference_a100_derived": {"end_to_end_48.6": round(best["gcups"] / 48.6, 2),
                                         "kernel_window_80": round(best["gcups"] / 80.0, 2),
                                         "source": "BASELINE.md section 1 (CDP/GASAL2/test_prog/report1.sqlite)"},
           "flat_host_entry": {"value": round(cells / min(th) / 1e9, 2), "ms": round(min(th) * 1e3, 3),
                               "mismatches": host_bad,
                               "path": "gasalx_align_host on the same pairs (pageable arrays; chunks on two streams)"},
           "device_resident": {"value": round(cells / dev_ms / 1e6, 2), "ms": round(dev_ms, 3), "mismatches": dev_bad,
                               "plan": plan,
                               "path": "gasalx_align_device on the same pairs in HBM (HIP events around the call)"},
           "parity": {"pairs_checked": n * len(dumps), "mismatches": sum(mism.values()), "by_run": mism,
                      "tolerance": "bit-exact", "against": "oracle/ over the 20K sample pairs; every replica of "
                                                          "every run's last pass compared with it"}}
    if not args.no_cpu:
        out["cpu_baseline"] = {"value": round(cells / repl / oracle_s / 1e9, 4), "unit": "GCUPS",
                               "cores": oracle_threads(), "kind": "port",
                               "sample": f"the {base} sample pairs once (the parity run, {oracle_s:.2f} s)"}
    print(json.dumps(out), flush=True)
    if out["parity"]["mismatches"] or host_bad or dev_bad:
        sys.exit(3)


# ------------------------------------------------------------------ main ----
def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus and args.gpus > 1:
        spawn_ranks(args.gpus)
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    wl = WORKLOADS[args.workload]
    if args.workload == "cpu_plumbing":
        if world != 1:
            sys.exit("bench.py: cpu_plumbing is a 1-process workload")
        return run_cpu_plumbing(args, wl)
    if args.workload == "boundary":
        if world != 1:
            sys.exit("bench.py: the boundary workload runs one process (its host threads share the GPU)")
        return run_boundary(args, wl)

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    kind, pkw = wl["kind"], wl["params"]
    probe = {}
    if args.force_int32:
        os.environ["GASALX_PACKED16"] = "0"
        probe["force_int32"] = True
    if args.scores:
        a, b, o, e = (int(x) for x in args.scores.split(","))
        pkw = dict(pkw or {}, match=a, mismatch=b, gap_open=o, gap_extend=e)
        probe["scores"] = [a, b, o, e]
    per = args.pairs or wl["pairs"]
    n_global = per * world if wl["scaling"] == "weak" else per
    seed = SEEDS[kind]
    if kind == 5:
        rl, hl = 250, 500
    elif kind == 6:
        rl, hl = NV_READ_LEN, NV_REF_LEN
    else:
        rl, hl = G.synth_spec(kind)
    shards = D.all_shards(n_global, rl, hl, world)
    start, end = shards[rank]
    n = end - start
    counts = [e - s for s, e in shards]
    do_gather = world > 1 and not args.no_gather
    if args.dry_run:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "pairs_global": n_global,
                          "shard": [start, end], "gather": do_gather}), flush=True)
        return

    import torch.distributed as dist
    # ranks beyond the visible devices share them (LOCAL_RANK % device_count): with the
    # gloo backend, the exact N-rank path (spawn -> engine -> exchange -> parity) runs on
    # a box with fewer GPUs than ranks; RCCL needs one rank per device
    n_dev = torch.cuda.device_count()
    dev_index = local_rank % max(n_dev, 1)
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)
    backend = args.dist_backend
    if world > 1:
        if backend == "nccl" and world > n_dev:
            sys.exit(f"bench.py: {world} ranks over {n_dev} GPUs needs --dist-backend gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=dev)
        else:
            dist.init_process_group("gloo", init_method="env://")

    def allreduce(t, op):
        """all_reduce of a small device tensor (through host memory under gloo)."""
        if world == 1:
            return t
        if backend == "gloo":
            h = t.cpu()
            dist.all_reduce(h, op=op)
            return h.to(t.device)
        dist.all_reduce(t, op=op)
        return t

    eng = G.Engine(dev_index)
    stream = torch.cuda.Stream(dev)      # a real (non-null) stream: kernels and timing events share it
    # (engine, stream, gather) per set; GASAL workloads with --streams S > 1 hold S of them
    sets, extra_bufs = [], []
    torch.cuda.set_stream(stream)
    gather = D.ScoreGather(counts, world, dev, dtype=torch.float32 if kind == 5 else torch.int32,
                           backend=backend) if do_gather else None
    t_syn = time.perf_counter()
    if kind == 6:
        band = wl.get("band", 0)
        nv = synth_nvbio(start, n, seed, band)
        data = nv
        cells_per_step = n * rl * (band or hl)
        al = G.NvAligner(**NV_ALIGNER)
        dpw = torch.from_numpy(nv["pat"].words.view(np.int32)).to(dev)
        dpo = torch.from_numpy(nv["pat"].offsets.view(np.int32)).to(dev)
        dtw = torch.from_numpy(nv["txt"].words.view(np.int32)).to(dev)
        dto = torch.from_numpy(nv["txt"].offsets.view(np.int32)).to(dev) if band else None
        result = gather.buf if gather else torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        pat = {"words": dpw.data_ptr(), "offsets": dpo.data_ptr(), "bits": 4, "big_endian": True}
        txt = {"words": dtw.data_ptr(), "offsets": dto.data_ptr() if band else 0, "length": 0 if band else NV_REF_LEN,
               "bits": 2, "big_endian": False}
        plan = f"nvbanded16_gotoh_semi_B{band} (two pairs per lane, band in registers)" if band else \
            G.nv_describe_plan(al, rl, hl)

        def align(k=0):
            if band:
                eng.nv_banded_score_device_ptrs(al, band, n, pat, txt, result.data_ptr(), stream.cuda_stream, rl)
            else:
                eng.nv_score_device_ptrs(al, n, pat, txt, result.data_ptr(), 0, rl, hl, stream.cuda_stream)

        def results():
            return {"score": result[:n].cpu().numpy()}
    elif kind == 5:
        h = synth_pairhmm(start, n, seed)
        data = h
        cells_per_step = int(np.sum(h["read_lens"].astype(np.int64) * h["hap_lens"].astype(np.int64)))
        dh = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.int32) if v.dtype == np.uint32 else v).to(dev)
              for k, v in h.items()}
        result = gather.buf if gather else torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        hptrs = {k: v.data_ptr() for k, v in dh.items()}
        plan = f"pairhmm_wavefront (read {rl} x hap {hl})"

        def align(k=0):
            eng.pairhmm_device_ptrs(hptrs, len(h["reads"]), len(h["haps"]), n, rl, hl, result.data_ptr(),
                                    stream.cuda_stream)

        def results():
            return {"result": result[:n].cpu().numpy()}
    else:
        batch = G.Batch.synth(kind, n, seed, start=start)
        data = batch
        cells_per_step = cells_of(batch)
        params = G.make_params(**pkw)
        as_i32 = lambda a: torch.from_numpy(a.view(np.int32).copy()).to(dev)
        d = {"q_batch": torch.from_numpy(batch.q_data).to(dev), "t_batch": torch.from_numpy(batch.t_data).to(dev),
             "q_offsets": as_i32(batch.q_offsets), "t_offsets": as_i32(batch.t_offsets),
             "q_lens": as_i32(batch.q_lens), "t_lens": as_i32(batch.t_lens),
             "aln_score": gather.buf if gather else torch.empty(n, dtype=torch.int32, device=dev)}
        fields = ["score"]
        if pkw["algo"] != G.GLOBAL:
            d["q_end"] = torch.empty(n, dtype=torch.int32, device=dev)
            d["t_end"] = torch.empty(n, dtype=torch.int32, device=dev)
            fields += ["q_end", "t_end"]
        if pkw.get("start_pos") in (G.WITH_START, G.WITH_TB) and pkw["algo"] != G.GLOBAL:
            d["q_start"] = torch.empty(n, dtype=torch.int32, device=dev)
            d["t_start"] = torch.empty(n, dtype=torch.int32, device=dev)
            fields += ["q_start", "t_start"]
        if wl.get("seed_score") is not None:     # KSW: the seed score of every pair
            d["seed_scores"] = torch.full((n,), wl["seed_score"], dtype=torch.int32, device=dev)
        tb = pkw.get("start_pos") == G.WITH_TB
        if tb:
            d["cigar"] = torch.empty(batch.q_bytes, dtype=torch.uint8, device=dev)
            d["n_cigar_ops"] = torch.empty(n, dtype=torch.int32, device=dev)
        ptrs = {k: v.data_ptr() for k, v in d.items()}
        plan = G.describe_plan(params, rl, hl)
        names = {"score": "aln_score", "q_end": "q_end", "t_end": "t_end", "q_start": "q_start",
                 "t_start": "t_start"}
        # --streams S: S engines (own workspaces) on S streams, each with its own outputs
        # (and, N > 1, its own exchange buffers); step i runs on set i % S, so a step's
        # traceback walk runs beside the next step's DP.  Set 0's outputs (steps 0, S,
        # 2S, ...) are the ones checked.
        set_ptrs = [ptrs]
        sets.append((eng, stream, gather))
        inputs = ("q_batch", "t_batch", "q_offsets", "t_offsets", "q_lens", "t_lens", "seed_scores")
        for _ in range(max(1, args.streams or wl.get("streams", 1)) - 1):
            e2, s2 = G.Engine(dev_index), torch.cuda.Stream(dev)
            g2 = D.ScoreGather(counts, world, dev, dtype=torch.int32, backend=backend) if gather else None
            d2 = {k: (v if k in inputs else (g2.buf if g2 is not None and k == "aln_score" else torch.empty_like(v)))
                  for k, v in d.items()}
            sets.append((e2, s2, g2))
            set_ptrs.append({k: v.data_ptr() for k, v in d2.items()})
            extra_bufs.append(d2)

        def align(k=0):
            sets[k][0].align_device_ptrs(params, set_ptrs[k], batch.q_bytes, batch.t_bytes, n, rl, hl,
                                         sets[k][1].cuda_stream)

        def results(k=0):
            dk = d if k == 0 else extra_bufs[k - 1]
            r = {f: dk[names[f]][:n].cpu().numpy() for f in fields}
            if tb:
                r["cigar"] = dk["cigar"].cpu().numpy()
                r["n_ops"] = dk["n_cigar_ops"].cpu().numpy().view(np.uint32)
            return r
    torch.cuda.synchronize(dev)
    synth_s = time.perf_counter() - t_syn
    if not sets:
        sets.append((eng, stream, gather))
    n_sets = len(sets)

    def step(i):
        k = i % n_sets
        align(k)
        if sets[k][2] is not None:   # the exchange step of SURVEY §8(e): every rank gets all scores
            with torch.cuda.stream(sets[k][1]):
                sets[k][2]()

    if args.warmup is not None:
        for i in range(args.warmup):
            step(i)
    else:
        # time-based: every rank runs the same steps.  Each step holds a collective (the score
        # all-gather), so the decision to stop is taken together: after each step from the third
        # on, the ranks all-reduce "keep warming" (MAX over ranks) and all leave at the same step
        # (a per-rank decision could leave one rank in a step's all_gather while
        # another had moved on to the next collective)
        i, t_w = 0, time.perf_counter()
        while True:
            step(i)
            i += 1
            if i < 3:
                continue
            torch.cuda.synchronize(dev)
            keep = torch.tensor([1 if time.perf_counter() - t_w < args.warmup_seconds else 0],
                                dtype=torch.int64, device=dev)
            if world > 1:
                keep = allreduce(keep, dist.ReduceOp.MAX)
            if int(keep[0]) == 0:
                break
        args.warmup = i
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        k = (args.warmup + i) % n_sets
        st_i, g_i = sets[k][1], sets[k][2]
        ev[i][0].record(st_i)
        align(k)
        ev[i][1].record(st_i)
        if g_i is not None:
            with torch.cuda.stream(st_i):
                g_i()
        ev[i][2].record(st_i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    ev_ms = kern_ms
    gath_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    t = torch.tensor([elapsed, kern_ms, gath_ms], dtype=torch.float64, device=dev)
    if world > 1:
        t = allreduce(t, dist.ReduceOp.MAX)
    elapsed, kern_ms, gath_ms = (float(x) for x in t)
    if n_sets > 1:
        # launches of consecutive steps overlap on the two streams: a launch's own duration
        # (events, rocprof) includes the time it shares the GPU, so the kernel time of a step
        # is its share of the wall time
        kern_ms = elapsed * 1e3 / args.steps

    # ---- parity: this rank's shard against the oracle (the CPU baseline at N = 1) ----
    parity, cpu = None, None
    O = _oracle(native=world == 1 and not args.no_cpu) if (args.parity_pairs > 0 or (world == 1 and not args.no_cpu)) \
        else None
    threads = oracle_threads()
    builds = None
    if world == 1 and not args.no_cpu and O is not None:
        # the CPU baseline: both builds of the oracle on a 1-core sample (half the budget
        # each), the faster one then times the 16-thread parity run
        builds = {"portable": single_core_rate(O, kind, data, pkw, args.cpu_seconds / 2, wl.get("seed_score"))}
        if O.NATIVE_OK:
            O.use_native(True)
            builds["native"] = single_core_rate(O, kind, data, pkw, args.cpu_seconds / 2, wl.get("seed_score"))
            O.use_native(builds["native"]["value"] >= builds["portable"]["value"])
    if args.parity_pairs > 0:
        m = min(n, args.parity_pairs)
        got = results()
        t_o = time.perf_counter()
        if kind == 6:
            ref = nv_oracle(O, data, nv_subset(data, m), threads, 0, m)
            mism = {"score": int(np.count_nonzero(got["score"][:m] != ref))}
            extra = {}
            ref_scores = ref
        elif kind == 5:
            ref = oracle_pairhmm(O, ph_subset(data, m), threads)
            g_ = got["result"][:m]
            rel = np.abs(g_.astype(np.float64) - ref) / np.maximum(np.abs(ref.astype(np.float64)), 1e-30)
            mism = {"result_rtol_1e-5": int(np.count_nonzero(~(rel <= 1e-5)))}
            extra = {"max_rel_err": float(rel.max(initial=0.0))}
            ref_scores = ref
        else:
            sub = data.slice(0, m)
            ref = oracle_align(O, sub, pkw, threads, wl.get("seed_score"))
            gsub = {f: got[f][:m] for f in fields}
            if tb:
                gsub["cigar"] = got["cigar"][:sub.q_bytes]
                gsub["n_ops"] = got["n_ops"][:m]
            mism, extra = compare_align(gsub, ref, fields, batch=sub, cigar=tb)
            ref_scores = ref["score"]
            # --streams S: the other engines aligned the same inputs; their outputs must equal set 0's
            if n_sets > 1:
                other = 0
                for k in range(1, n_sets):
                    gk = results(k)
                    gks = {f: gk[f][:m] for f in fields}
                    if tb:
                        gks["cigar"] = gk["cigar"][:sub.q_bytes]
                        gks["n_ops"] = gk["n_ops"][:m]
                    other += sum(compare_align(gks, gsub, fields, batch=sub, cigar=tb)[0].values())
                mism["other_streams_vs_set0"] = other
        oracle_s = time.perf_counter() - t_o
        cells_checked = m * rl * ((data.get("band") or hl) if kind == 6 else hl)
        tot = torch.tensor([m, sum(mism.values())], dtype=torch.int64, device=dev)
        gather_bad = 0
        if gather is not None:
            # the gathered scores (timed steps' exchange) against every rank's oracle scores
            og = D.ScoreGather(counts, world, dev, dtype=gather.buf.dtype, backend=backend)
            og.buf[:m] = torch.as_tensor(np.asarray(ref_scores), device=dev)
            og()
            gfull = gather.out.cpu().numpy()
            ofull = og.out.cpu().numpy()
            mlist = [min(c, args.parity_pairs) for c in counts]
            for r in range(world):
                a, b = gfull[r, :mlist[r]], ofull[r, :mlist[r]]
                if kind == 5:
                    rr = np.abs(a.astype(np.float64) - b) / np.maximum(np.abs(b.astype(np.float64)), 1e-30)
                    gather_bad += int(np.count_nonzero(~(rr <= 1e-5)))
                else:
                    gather_bad += int(np.count_nonzero(a != b))
        if world > 1:
            tot = allreduce(tot, dist.ReduceOp.SUM)
        parity = {"pairs_checked": int(tot[0]), "mismatches": int(tot[1]),
                  "by_field_rank0": mism, **extra,
                  "tolerance": "rtol 1e-5" if kind == 5 else "bit-exact",
                  **({"oracle": "oracle/nvbio_oracle.c (nvbio semantics)"} if kind == 6 else {}),
                  "against": "oracle/ (CPU restatement of the reference kernels), on the timed steps' outputs"}
        if gather is not None:
            parity["gathered_scores_checked"] = int(sum(min(c, args.parity_pairs) for c in counts))
            parity["gathered_mismatches"] = gather_bad
        if world == 1 and not args.no_cpu:
            cpu = {"value": round(cells_checked / oracle_s / 1e9, 4), "unit": "GCUPS", "cores": threads,
                   "kind": "port",
                   "sample": f"first {m} pairs of the rank-0 batch ({cells_checked / 1e9:.2f} G cells, "
                             f"{oracle_s:.1f} s, the parity run), oracle/gasal_oracle.c OpenMP x{threads}",
                   "build": "gcc -O3 -march=native (built on this host)" if O._active
                            else "gcc -O3 (portable build: faster than -march=native on the 1-core sample, "
                                 "or the native build failed)"}
    if world == 1 and not args.no_cpu:
        if cpu is None:
            cpu = {"value": None, "unit": "GCUPS", "cores": threads, "kind": "port", "sample": "parity run skipped"}
        fast = max(builds.values(), key=lambda r: r["value"])
        cpu["single_core"] = dict(fast, builds={k: v["value"] for k, v in builds.items()})
        cpu["host"] = host_info()
        cpu["note"] = (f"cores = the OpenMP threads used (OMP_NUM_THREADS, else min(16, CPUs)): one GPU's "
                       f"CPU share on this pool, which limits a job's worker pool to it; host totals in "
                       f"'host' (the whole machine's CPUs, shared by its 8 GPUs' jobs, are not timed)")

    if rank == 0:
        # every pair of every shard (uniform lengths); the banded front-end counts its band's cells
        total_cells = n_global * rl * ((data.get("band") or hl) if kind == 6 else hl)
        gcups = total_cells * args.steps / elapsed / 1e9
        kern_s = kern_ms / 1e3
        achieved = wl["bytes"] * n / kern_s / 1e9
        pmc = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
            except Exception:
                pmc = None
        # counters only from a pass over this very build and plan (the library's sha256 changes
        # with any kernel change, so a stale file is never used); otherwise traffic is null
        sha = lib_sha256()
        same = (pmc is not None and pmc.get("pairs_per_launch") == n and pmc.get("plan") == plan and
                pmc.get("lib_sha256") == sha and not probe)
        traffic = pmc.get("hbm_bytes_per_launch") if same else None
        kcells = cells_per_step / kern_s
        # VALU roofline of the dominant kernel: its own wave-instructions (PMC SQ_INSTS_VALU of a
        # pass over this very library and plan) issued back to back at the SIMD's full rate -- one
        # wave64 instruction per 2 cycles per SIMD-32 (MI355X_MICROARCH.md), 1,024 SIMDs at 2.4
        # GHz -- is the fastest that instruction stream can run, so frac = that time / the
        # measured time <= 1.  Instructions priced above 2 cycles (VOP3P, v_perm, FMA: the
        # measured table profiles/r04_valu_issue_rates.json) keep frac below 1 at full issue.
        # Without a matching PMC file peak and frac stay null; the SURVEY 8(d) algorithmic op
        # count is reported as a rate beside it, not as a fraction (the packed kernels issue
        # fewer instructions than it counts).
        valu = {"bound": "valu issue", "achieved": round(kcells / 1e12, 4), "unit": "T cells/s",
                "peak": None, "frac": None,
                "basis": "the kernel's VALU wave-instructions per cell (PMC SQ_INSTS_VALU) at one per 2 cycles "
                         "per SIMD-32 (MI355X_MICROARCH.md), 1,024 SIMDs x 2.4 GHz"}
        if kind == 6 or wl["ops"] is None:
            bcells = band_cells_of(data, pkw.get("k_band", 0)) if kind != 6 else cells_per_step
            if kind != 6:
                valu["band_cells_per_step"] = bcells
                valu["band_fraction"] = round(bcells / cells_per_step, 4)
        ops = wl["ops"] or 12
        valu["algorithmic"] = {"ops_per_cell": ops, "achieved_t_ops": round(kcells * ops / 1e12, 3),
                               "basis": "SURVEY.md 8(d) algorithmic ops per cell (informational: a rate, not a "
                                        "fraction of the VALU ceiling)"}
        if kind == 5:
            fl = kcells * wl["ops"]
            valu["fp32"] = {"achieved_tflops": round(fl / 1e12, 2), "peak_tflops": round(FP32_VECTOR_PEAK / 1e12, 1),
                            "frac": round(fl / FP32_VECTOR_PEAK, 4),
                            "basis": "11 fp32 flops per cell (3 FMA = 6, 4 mul, 1 add; SURVEY.md 8(d)) against "
                                     "the FP32 vector peak 157.3 TFLOPS (MI355X_MICROARCH.md)"}
        if same and pmc.get("valu_insts_per_launch"):
            pk_t = pmc.get("kernel_ns", 0) / 1e9 or kern_s
            vi = float(pmc["valu_insts_per_launch"])
            cells_launch = bcells if (wl["ops"] is None and kind != 6) else cells_per_step
            t_issue = vi * 2.0 / (SIMDS * CLOCK)            # every instruction at the full rate
            peak_cells = cells_launch / t_issue
            ach = cells_launch / pk_t
            valu.update({"peak": round(peak_cells / 1e12, 4), "achieved": round(ach / 1e12, 4),
                         "frac": round(ach / peak_cells, 4),
                         "instr_per_cell": round(vi * 64 / cells_launch, 3),
                         "cycles_per_instr_per_simd": round(SIMDS * CLOCK * pk_t / vi, 3),
                         "kernel": pmc.get("kernel"), "kernel_ms_pmc": round(pk_t * 1e3, 4),
                         "source": f"profiles/pmc_{args.workload}.json (SQ_INSTS_VALU; same library sha256 and "
                                   f"plan as this run)"})
            cen = pmc.get("census")
            if cen and cen.get("cycles_per_valu"):
                # per-class issue bound: the same instruction count priced by the
                # steady loop's mix at the measured issue costs (kernel_census.py: full-rate ops 2.07
                # cycles, VOP3P / v_perm / three-input VOP3 4.1-4.25 per wave64 instruction per SIMD)
                cpv = float(cen["cycles_per_valu"])
                t_priced = vi * cpv / (SIMDS * CLOCK)
                valu["issue_priced"] = {
                    "frac": round(t_priced / pk_t, 4), "cycles_per_valu": cpv,
                    "loop_valu": cen.get("loop_valu"), "loop_issue_cycles": cen.get("loop_issue_cycles"),
                    "basis": "PMC SQ_INSTS_VALU x the steady loop's average issue cost per VALU instruction "
                             "(tools/kernel_census.py over this library, profiles/r04_valu_issue_rates.json), "
                             "against 1,024 SIMDs x 2.4 GHz: how close the kernel runs to the issue bound of its "
                             "own instruction mix ('frac' beside it prices every instruction at 2 cycles)"}
        if kind != 5 and wl["ops"]:
            # fixed ceiling: SURVEY.md 8(d)'s algorithmic ops per cell at the packed
            # 2 x 16-bit lane rate, independent of how many instructions the kernel issues
            fixed = 2 * VALU_LANE_OPS / wl["ops"]
            valu["fixed_ceiling"] = {
                "peak": round(fixed / 1e12, 4), "unit": "T cells/s", "frac": round(kcells / fixed, 4),
                "basis": f"{wl['ops']} algorithmic int ops per cell (SURVEY.md 8(d)) at 2 x 16-bit lanes per "
                         f"32-bit lane op, 78.6 T lane ops/s (MI355X_MICROARCH.md): a ceiling that does not "
                         f"move with the kernel's own instruction count"}
        out = {
            "metric": METRICS.get(args.workload, MAIN_METRIC),
            "value": round(gcups, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": None,
            "dtype": dtype_label(plan, kind),
            "data": "synthetic (SURVEY.md 8(d) generator), resident in HBM",
            "config": {"workload": wl["label"], "pairs_global": n_global, "pairs_rank0": n,
                       "cells_rank0_step": cells_per_step, "plan": plan, "lib_sha256": sha,
                       **({"probe": probe} if probe else {}),
                       "parallelism": f"dp{world} (cell-balanced contiguous shards of one global batch)" +
                                      ((", RCCL all-gather of scores in every step" if backend == "nccl" else
                                        ", gloo all-gather of scores (through host memory) in every step")
                                       if gather else ""),
                       **({"dist_backend": backend, "devices": n_dev} if world > 1 else {}),
                       **({"streams": f"{n_sets} engines on {n_sets} streams, steps round-robin "
                                      f"(gasal_aln_async per storage, test_prog.cpp's NB_STREAMS)"}
                          if n_sets > 1 else {}),
                       "synth_s_rank0": round(synth_s, 2)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "bytes_per_pair": wl["bytes"], "kernel_ms": round(kern_ms, 4),
                         "timed": ("HIP events around the align call on its stream (every kernel of the call; "
                                   "WITH_START/WITH_TB calls launch more than the dominant kernel)") if n_sets == 1 else
                                  (f"wall time per step of the {n_sets}-stream round-robin (steps overlap; "
                                   f"HIP events around one align call on its stream: {ev_ms:.4f} ms, the "
                                   f"launches sharing the GPU with the other stream's)")},
            "valu_roofline": valu,
            "kernel_gcups": round(cells_per_step / kern_s / 1e9, 2),
            "gather_ms": round(gath_ms, 4) if gather else None,
            "parity": parity,
            # the derived A100 figure is GASAL2's own kernels; PairHMM and the nvbio
            # front-end have no published number to set beside
            "vs_reference_a100_derived": None if kind in (5, 6) else round(gcups / world / 80.0, 2),
        }
        if world == 1 and not args.no_e2e:
            out["end_to_end"] = end_to_end(eng, kind, data, None if kind in (5, 6) else params, cells_per_step,
                                           seed_score=wl.get("seed_score"))
        if cpu is not None:
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    if parity and (parity["mismatches"] or parity.get("gathered_mismatches")):
        sys.exit(3)


if __name__ == "__main__":
    main()
