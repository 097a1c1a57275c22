#!/usr/bin/env python3
"""Throughput of the nvbio BatchedAlignmentTraceback and BatchedBandedAlignmentTraceback
front-ends (gasalx_nv_traceback_device / gasalx_nv_banded_traceback_device, nvtrace.hpp) on
MI355X: reads of 150 bp drawn from per-pair text windows of 150 + slack symbols
(4-bit big-endian patterns, 2-bit texts, the sw-benchmark packing), inputs resident in HBM, timed
with HIP events around the device call; the first pairs' outputs are checked against
oracle/nvbio_oracle.c (test infrastructure).  Prints one JSON line per aligner/type.

usage: nv_traceback_probe.py [pairs] [slack]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd"))
sys.path.insert(0, ROOT)
import gasal_ffi as G  # noqa: E402
import oracle.oracle as O  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    slack = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    rng = np.random.default_rng(0x5EED0077)
    m = 150
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)

    def make(tlen, max_start):
        # reads of m drawn at offsets 0..max_start of their text windows, 3 % substitutions
        texts = rng.integers(0, 4, (n, tlen))
        st = rng.integers(0, max_start + 1, n)
        pats = texts[np.arange(n)[:, None], st[:, None] + np.arange(m)[None, :]].copy()
        flip = rng.random(pats.shape) < 0.03
        pats[flip] = (pats[flip] + rng.integers(1, 4, int(flip.sum()))) % 4
        P = G.PackedSet.pack(list(pats))
        T = G.PackedSet.pack(list(texts), bits=2, big_endian=False)
        return pats, texts, (t(P.words), t(P.offsets), t(T.words), t(T.offsets))

    pats, texts, (pw, po, tw, to) = make(m + slack, slack)
    stride = m + m + slack
    outs_t = dict(score=torch.zeros(n, dtype=torch.int32, device=dev), source=torch.zeros(2 * n, dtype=torch.int32, device=dev),
                  sink=torch.zeros(2 * n, dtype=torch.int32, device=dev), ops=torch.zeros(n * stride, dtype=torch.uint8, device=dev),
                  n_ops=torch.zeros(n, dtype=torch.int32, device=dev))
    outs = {k: v.data_ptr() for k, v in outs_t.items()}
    pat = dict(words=pw.data_ptr(), offsets=po.data_ptr(), bits=4, big_endian=True)
    txt = dict(words=tw.data_ptr(), offsets=to.data_ptr(), bits=2, big_endian=False)
    eng = G.Engine(0)
    ts = torch.cuda.Stream()      # a real stream: the null stream's handle 0 would mean the engine's own
    s = ts.cuda_stream
    cells = n * m * (m + slack)
    for name, al in (("gotoh_local", G.NvAligner(G.NV_GOTOH, G.NV_LOCAL, 2, -1, -2, -1)),
                     ("gotoh_semi", G.NvAligner(G.NV_GOTOH, G.NV_SEMI_GLOBAL, 2, -1, -2, -1)),
                     ("gotoh_global", G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, 2, -1, -2, -1)),
                     ("sw_local", G.NvAligner(G.NV_SW, G.NV_LOCAL, match=2, mismatch=-1, deletion=-1, insertion=-1))):
        call = lambda: eng.nv_traceback_device_ptrs(al, n, pat, txt, outs, stride, m, m + slack, s)
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(ts)
        for _ in range(reps):
            call()
        e1.record(ts)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        k = 500
        o = O.nv_traceback(al, G.PackedSet.pack(list(pats[:k])), G.PackedSet.pack(list(texts[:k]), bits=2, big_endian=False))
        g_sc = outs_t["score"][:k].cpu().numpy()
        g_ops = outs_t["ops"][:k * stride].cpu().numpy().reshape(k, stride)
        g_n = outs_t["n_ops"][:k].cpu().numpy()
        bad = int((g_sc != o["score"]).sum()) + sum(int(not np.array_equal(g_ops[i, :g_n[i]], o["ops"][i])) for i in range(k))
        # bytes the pass moves per cell: the flag byte written, the (H, E) int2 hand-off between stripes
        # of 8 columns written and read (8 + 8 B per 8 cells); the walk reads ~(M + N) flag bytes per pair
        hbm = cells * 3 + n * (2 * m + slack)
        print(json.dumps({"probe": "nv_traceback", "aligner": name, "pairs": n, "pattern": m, "text": m + slack,
                          "ms": round(ms, 3), "gcups": round(cells / ms / 1e6, 1), "checked": k, "mismatches": bad,
                          "hbm_GBps_algorithmic": round(hbm / ms / 1e6, 1),
                          "hbm_frac": round(hbm / ms / 1e6 / 8000.0, 4),
                          "kernel": "nv_traceback_kernel (one pair per thread, full DP + walk)"}), flush=True)
    for band in (7, 15, 31):
        # nvBowtie's windows: the read's diagonal inside the band (text = read + band - 1 symbols,
        # the read starting in the band's first half)
        pats, texts, (pw, po, tw, to) = make(m + band - 1, band // 2)
        pat = dict(words=pw.data_ptr(), offsets=po.data_ptr(), bits=4, big_endian=True)
        txt = dict(words=tw.data_ptr(), offsets=to.data_ptr(), bits=2, big_endian=False)
        for name, al in (("gotoh_semi", G.NvAligner(G.NV_GOTOH, G.NV_SEMI_GLOBAL, 0, -5, -8, -3)),
                         ("gotoh_local", G.NvAligner(G.NV_GOTOH, G.NV_LOCAL, 2, -1, -2, -1)),
                         ("ed_semi", G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL))):
            bstride = 2 * m + band
            call = lambda: eng.nv_banded_traceback_device_ptrs(al, band, n, pat, txt, outs, bstride, m, s)
            for _ in range(2):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 5
            e0.record(ts)
            for _ in range(reps):
                call()
            e1.record(ts)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            k = 500
            o = O.nv_banded_traceback(al, band, G.PackedSet.pack(list(pats[:k])),
                                      G.PackedSet.pack(list(texts[:k]), bits=2, big_endian=False))
            g_sc = outs_t["score"][:k].cpu().numpy()
            g_ops = outs_t["ops"][:k * bstride].cpu().numpy().reshape(k, bstride)
            g_n = outs_t["n_ops"][:k].cpu().numpy()
            bad = int((g_sc != o["score"]).sum()) + sum(int(not np.array_equal(g_ops[i, :g_n[i]], o["ops"][i]))
                                                        for i in range(k))
            bcells = n * m * band
            flag_bytes = n * m * ((band + 3) // 4) * 4
            hbm = flag_bytes + n * (2 * m + band)   # flags written once; the walk reads ~(M + band) of them
            print(json.dumps({"probe": "nv_banded_traceback", "aligner": name, "band": band, "pairs": n, "pattern": m,
                              "text": m + band - 1, "ms": round(ms, 3), "gcups": round(bcells / ms / 1e6, 1),
                              "flag_store_GBps": round(flag_bytes / ms / 1e6, 1),
                              "hbm_frac": round(hbm / ms / 1e6 / 8000.0, 4), "checked": k, "mismatches": bad,
                              "kernel": "nv_banded_traceback_kernel (one pair per thread, band in registers + walk)"}),
                  flush=True)


if __name__ == "__main__":
    main()
