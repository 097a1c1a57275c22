#!/usr/bin/env python3
"""Benchmark of the hot path: batched affine-gap Smith-Waterman (GASAL2 LOCAL,
score + end positions) on MI355X, BASELINE.json config 2.

A step = one pass of the HIP engine over one batch of 1M synthetic pairs
(ql = tl = 150, SURVEY.md §8(d) generator, seed 0x5EED0002 + rank) that is
already resident in HBM, launched through the C-ABI (gasalx_align_device) on
torch's current stream.  Multi-GPU: one process per GPU, each aligns its own
batch (weak scaling, no data-path collective); timing is bracketed by a
barrier + synchronize and the max over ranks is reported.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P] [--workload sw_local|nw_tb|semi|pairhmm]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd"))
import gasal_ffi as G  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue peak: 1024 SIMDs x 2.4 GHz, one wave64 instruction per 2 cycles (full-rate ops;
# v_pk_*, max/min_32, perm, maximum3 issue at 4 — profiles/r01_valu_issue_rates.md)
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2

WORKLOADS = {
    # name: (synth kind, default pairs, params, algorithmic bytes per pair, int ops per cell, label)
    "sw_local": (2, 1_000_000, dict(algo=G.LOCAL), 332, 12,
                 "config2: SW local affine (a1 b4 o6 e1) score+ends, 1M pairs x 150bp, seed 0x5EED0002"),
    "sw_local_start": (2, 1_000_000, dict(algo=G.LOCAL, start_pos=G.WITH_START), 340, 12,
                       "config2 + WITH_START: SW local affine score+ends+starts, 1M pairs x 150bp, seed 0x5EED0002"),
    "sw_local_tb": (2, 1_000_000, dict(algo=G.LOCAL, start_pos=G.WITH_TB), 340 + 152, 16,
                    "config2 + WITH_TB: SW local affine score+ends+starts+CIGAR, 1M pairs x 150bp, seed 0x5EED0002"),
    "nw_tb": (3, 100_000, dict(algo=G.GLOBAL, start_pos=G.WITH_TB), 650, 16,
              "config3: NW global + traceback/CIGAR, 100K pairs x 300bp, seed 0x5EED0003"),
    "semi": (4, 1_250_000, dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET), 364, 12,
             "config4 shard: semi-global TARGET/TARGET, 150bp reads in 182bp windows, seed 0x5EED0004"),
    "semi_start": (4, 1_250_000, dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET, start_pos=G.WITH_START,
                                      max_query_len=192), 372, 12,
                   "config4 shard + WITH_START: semi-global TARGET/TARGET score+ends+starts, 150bp reads in 182bp "
                   "windows, seed 0x5EED0004"),
    "pairhmm": (5, 100_000, None, 4762, 11,
                "config5: PairHMM fp32 forward, 100K reads x haplotypes (250 x 500), seed 0x5EED0005"),
}
METRICS = {
    "pairhmm": "GCUPS of PairHMM fp32 forward (config 5, 250x500) on MI355X",
}


def synth_pairhmm(n, seed, rl=250, hl=500):
    """haplotype 500 bp uniform; read = 250-bp substring with
    2% mismatches; base quals U[10,40], insertion/deletion quals 45 (gcp ignored)."""
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"ACGT", np.uint8)
    haps = alpha[rng.integers(0, 4, (n, hl))]
    start = rng.integers(0, hl - rl + 1, n)
    reads = haps[np.arange(n)[:, None], start[:, None] + np.arange(rl)[None, :]].copy()
    flip = rng.random((n, rl)) < 0.02
    reads[flip] = alpha[(np.searchsorted(alpha, reads[flip]) + rng.integers(1, 4, int(flip.sum()))) % 4]
    bq = rng.integers(10, 41, n * rl).astype(np.uint8)
    iq = np.full(n * rl, 45, np.uint8)
    qm, de, xi, al = G.pairhmm_params(bq, iq, iq)
    return dict(reads=reads.reshape(-1), read_offsets=np.arange(n, dtype=np.uint32) * rl,
                read_lens=np.full(n, rl, np.uint32), qm=qm, delta=de, xiksi=xi, alpha=al, haps=haps.reshape(-1),
                hap_offsets=np.arange(n, dtype=np.uint32) * hl, hap_lens=np.full(n, hl, np.uint32))


def cpu_baseline_pairhmm(h, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n = len(h["read_lens"])
    chunk, done, cells, t_used = 2000, 0, 0, 0.0
    while t_used < budget_s and done < n:
        e = min(done + chunk, n)
        rl, hl = h["read_lens"][done:e], h["hap_lens"][done:e]
        r0, h0 = int(h["read_offsets"][done]), int(h["hap_offsets"][done])
        r1, h1 = int(h["read_offsets"][e - 1] + rl[-1]), int(h["hap_offsets"][e - 1] + hl[-1])
        t0 = time.perf_counter()
        O.pairhmm(h["reads"][r0:r1], h["read_offsets"][done:e] - r0, rl, h["qm"][r0:r1], h["delta"][r0:r1],
                  h["xiksi"][r0:r1], h["alpha"][r0:r1], h["haps"][h0:h1], h["hap_offsets"][done:e] - h0, hl,
                  n_threads=threads)
        t_used += time.perf_counter() - t0
        cells += int(np.sum(rl.astype(np.int64) * hl.astype(np.int64)))
        done = e
    return {"value": round(cells / t_used / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": f"first {done} pairs of the rank-0 batch ({cells / 1e9:.2f} G cells, {t_used:.1f} s), "
                      f"oracle/gasal_oracle.c orc_pairhmm_batch OpenMP x{threads}"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=0, help="pairs per GPU (default: the config's size)")
    ap.add_argument("--workload", default="sw_local", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-staged (PCIe-inclusive) timing")
    ap.add_argument("--gather", action="store_true",
                    help="N>1: all-gather every rank's int32 scores (RCCL) inside each timed step")
    return ap.parse_args()


def cpu_baseline(batch, params_kw, budget_s):
    """The repo's CPU restatement of the GASAL2 kernels (oracle/), timed on a
    bounded prefix of the same workload on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    op = O.make_params(**params_kw)
    chunk = 20000
    done_pairs, cells, t_used = 0, 0, 0.0
    while t_used < budget_s and done_pairs < batch.n:
        idx = np.arange(done_pairs, min(done_pairs + chunk, batch.n))
        sub = batch.subset(idx)
        t0 = time.perf_counter()
        O.align(sub, op, n_threads=threads)
        t_used += time.perf_counter() - t0
        cells += int(np.sum(sub.q_lens.astype(np.int64) * sub.t_lens.astype(np.int64)))
        done_pairs += len(idx)
    return {"value": round(cells / t_used / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": f"first {done_pairs} pairs of the rank-0 batch ({cells / 1e9:.2f} G cells, {t_used:.1f} s), "
                      f"oracle/gasal_oracle.c OpenMP x{threads}"}


def end_to_end(eng, kind, data, params, cells, reps=5):
    """PCIe-inclusive rate through the host-buffer entry point (gasalx_align_host /
    gasalx_pairhmm_host): host arrays in, H2D + kernels + D2H, results back in host
    arrays.  Reported beside `value`, never as it."""
    if kind == 5:
        h = data
        args = (h["reads"], h["read_offsets"], h["read_lens"], h["qm"], h["delta"], h["xiksi"], h["alpha"],
                h["haps"], h["hap_offsets"], h["hap_lens"])
        call = lambda: eng.pairhmm_host(*args)
        path = "gasalx_pairhmm_host (pageable host arrays; H2D + kernel + D2H)"
    else:
        fields = ["score"] if params.algo == G.GLOBAL else ["score", "q_end", "t_end"]
        if params.start_pos == G.WITH_START:
            fields += ["q_start", "t_start"]
        call = lambda: eng.align_host(data, params, fields=fields)
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
    if kind != 5 and params.start_pos == G.WITH_TB:
        # the same call with a page-locked CIGAR buffer (as the reference's own host_res,
        # res.cpp:8-70): the D2H skips the runtime's pageable staging copy
        host = G.PinnedHost(data.q_bytes)
        dtp, _ = timed(lambda: eng.align_host(data, params, fields=fields, cigar_out=host.array))
        host.close()
        res["pinned_cigar"] = {"value": round(cells / dtp / 1e9, 2), "ms_per_batch": round(dtp * 1e3, 3)}
    if kind != 5:
        # sequence bytes page-locked too, as the reference's host batch pages are
        # (host_batch.cpp:79-153 fills pinned pages), plus the CIGAR buffer for TB
        hq, ht = G.PinnedHost(data.q_bytes), G.PinnedHost(data.t_bytes)
        hq.array[:] = data.q_data
        ht.array[:] = data.t_data
        pb = dataclasses.replace(data, q_data=hq.array, t_data=ht.array)
        hc = G.PinnedHost(data.q_bytes) if params.start_pos == G.WITH_TB else None
        dtp, _ = timed(lambda: eng.align_host(pb, params, fields=fields, cigar_out=hc.array if hc else None))
        res["pinned_io"] = {"value": round(cells / dtp / 1e9, 2), "ms_per_batch": round(dtp * 1e3, 3),
                            "pinned": "q/t sequence bytes" + (" + CIGAR buffer" if hc else "")}
        for h in (hq, ht, hc):
            if h:
                h.close()
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    kind, default_pairs, pkw, bytes_per_pair, ops_per_cell, label = WORKLOADS[args.workload]
    n = args.pairs or default_pairs
    seed = {2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}[kind] + rank
    eng = G.Engine(local_rank)
    stream = torch.cuda.Stream(dev)      # a real (non-null) stream: kernels and timing events share it
    torch.cuda.set_stream(stream)
    gathered = None
    if kind == 5:
        h = synth_pairhmm(n, seed)
        cells_per_step = int(np.sum(h["read_lens"].astype(np.int64) * h["hap_lens"].astype(np.int64)))
        dh = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.int32) if v.dtype == np.uint32 else v).to(dev)
              for k, v in h.items()}
        result = torch.empty(n, dtype=torch.float32, device=dev)
        hptrs = {k: v.data_ptr() for k, v in dh.items()}
        maxr, maxh = int(h["read_lens"].max()), int(h["hap_lens"].max())
        plan = f"pairhmm_wavefront (read {maxr} x hap {maxh})"

        def step():
            eng.pairhmm_device_ptrs(hptrs, len(h["reads"]), len(h["haps"]), n, maxr, maxh, result.data_ptr(),
                                    stream.cuda_stream)
    else:
        batch = G.Batch.synth(kind, n, seed)
        cells_per_step = int(np.sum(batch.q_lens.astype(np.int64) * batch.t_lens.astype(np.int64)))
        params = G.make_params(**pkw)

        # inputs resident in HBM before the timed region
        as_i32 = lambda a: torch.from_numpy(a.view(np.int32).copy()).to(dev)
        d = {
            "q_batch": torch.from_numpy(batch.q_data).to(dev), "t_batch": torch.from_numpy(batch.t_data).to(dev),
            "q_offsets": as_i32(batch.q_offsets), "t_offsets": as_i32(batch.t_offsets),
            "q_lens": as_i32(batch.q_lens), "t_lens": as_i32(batch.t_lens),
            "aln_score": torch.empty(n, dtype=torch.int32, device=dev),
        }
        if pkw["algo"] != G.GLOBAL:
            d["q_end"] = torch.empty(n, dtype=torch.int32, device=dev)
            d["t_end"] = torch.empty(n, dtype=torch.int32, device=dev)
        if pkw.get("start_pos") in (G.WITH_START, G.WITH_TB) and pkw["algo"] != G.GLOBAL:
            d["q_start"] = torch.empty(n, dtype=torch.int32, device=dev)
            d["t_start"] = torch.empty(n, dtype=torch.int32, device=dev)
        if pkw.get("start_pos") == G.WITH_TB:
            d["cigar"] = torch.empty(batch.q_bytes, dtype=torch.uint8, device=dev)
            d["n_cigar_ops"] = torch.empty(n, dtype=torch.int32, device=dev)
        ptrs = {k: v.data_ptr() for k, v in d.items()}
        maxq, maxt = int(batch.q_lens.max()), int(batch.t_lens.max())
        plan = G.describe_plan(params, maxq, maxt)
        gathered = [torch.empty_like(d["aln_score"]) for _ in range(world)] if (args.gather and world > 1) else None

        def step():
            eng.align_device_ptrs(params, ptrs, batch.q_bytes, batch.t_bytes, n, maxq, maxt, stream.cuda_stream)
            if gathered is not None:   # optional exchange step of SURVEY §8(e): every rank gets all scores
                dist.all_gather(gathered, d["aln_score"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])

    if rank == 0:
        total_cells = cells_per_step * world * args.steps
        gcups = total_cells / elapsed / 1e9
        kern_s = kern_ms / 1e3
        achieved = bytes_per_pair * n / kern_s / 1e9
        valu_roof = None
        pmc = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
            except Exception:
                pmc = None
        traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        if pmc and pmc.get("valu_insts_per_launch") and pmc.get("pairs_per_launch", n) == n:
            # dynamic VALU wave-instructions of the dominant kernel (SQ_INSTS_VALU, same workload)
            ach = pmc["valu_insts_per_launch"] / kern_s
            valu_roof = {"bound": "valu-issue", "achieved": round(ach / 1e12, 4), "peak": VALU_PEAK_WAVE_INSTR / 1e12,
                         "unit": "T wave-instr/s", "frac": round(ach / VALU_PEAK_WAVE_INSTR, 4),
                         "valu_insts_per_launch": pmc["valu_insts_per_launch"],
                         "source": f"profiles/pmc_{args.workload}.json (SQ_INSTS_VALU)"}
        out = {
            "metric": METRICS.get(args.workload, "GCUPS on batched 150bp affine-gap SW at 1/2/4/8 MI355X; HBM-roofline %"),
            "value": round(gcups, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if kind == 5 else "int32",
            "data": "synthetic (SURVEY.md 8(d) generator, std::mt19937_64), resident in HBM",
            "config": {"workload": label, "pairs_per_gpu": n, "cells_per_gpu_step": cells_per_step,
                       "plan": plan,
                       "parallelism": f"dp{world} (pairs sharded)" + (", all-gather of scores" if gathered else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "bytes_per_pair": bytes_per_pair, "kernel_ms": round(kern_ms, 4),
                         "timed": "HIP events around the whole step on its stream (every kernel of the step; "
                                  "WITH_START/WITH_TB steps launch more than the dominant kernel)"},
            "valu_roofline": valu_roof,
            "kernel_gcups": round(cells_per_step / kern_s / 1e9, 2),
            "vs_reference_a100_derived": round(gcups / world / 80.0, 2),
        }
        if world == 1 and not args.no_e2e:
            out["end_to_end"] = end_to_end(eng, kind, h if kind == 5 else batch, None if kind == 5 else params,
                                           cells_per_step)
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = (cpu_baseline_pairhmm(h, args.cpu_seconds) if kind == 5
                                   else cpu_baseline(batch, pkw, args.cpu_seconds))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
