"""Kernel-time probe of every planner path on device-resident synthetic batches
(SURVEY.md §8(d) generators): which kernels run and at what GCUPS.  Not a bench
line (bench.py is); a map of where the non-headline configurations stand.

  python tools/path_probe.py [pairs]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd"))
import gasal_ffi as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
dev = torch.device("cuda", 0)
eng = G.Engine(0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)

MODES = [
    ("local", 2, dict(algo=G.LOCAL)),
    ("local_start", 2, dict(algo=G.LOCAL, start_pos=G.WITH_START)),
    ("local_tb", 2, dict(algo=G.LOCAL, start_pos=G.WITH_TB)),
    ("local_second", 2, dict(algo=G.LOCAL, second_best=1)),
    ("semi_tt", 4, dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET)),
    ("semi_tt_start", 4, dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET, start_pos=G.WITH_START,
                              max_query_len=192)),
    ("semi_both", 4, dict(algo=G.SEMI_GLOBAL, head=G.BOTH, tail=G.BOTH)),
    ("semi_query", 4, dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.QUERY)),
    ("semi_none", 4, dict(algo=G.SEMI_GLOBAL, head=G.NONE, tail=G.NONE)),
    ("global", 3, dict(algo=G.GLOBAL)),
    ("global_tb", 3, dict(algo=G.GLOBAL, start_pos=G.WITH_TB)),
    ("banded16", 2, dict(algo=G.BANDED, k_band=16)),
    ("ksw", 2, dict(algo=G.KSW)),
]
only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None
batches = {}
out = []
for name, kind, kw in MODES:
    if only and name not in only:
        continue
    m = n // 10 if kind == 3 else n
    if kind not in batches:
        batches[kind] = G.Batch.synth(kind, m, 0x5EED0000 + kind)
    b = batches[kind]
    p = G.make_params(**kw)
    as_i32 = lambda a: torch.from_numpy(a.view(np.int32).copy()).to(dev)
    d = {"q_batch": torch.from_numpy(b.q_data).to(dev), "t_batch": torch.from_numpy(b.t_data).to(dev),
         "q_offsets": as_i32(b.q_offsets), "t_offsets": as_i32(b.t_offsets),
         "q_lens": as_i32(b.q_lens), "t_lens": as_i32(b.t_lens)}
    for f in ("aln_score", "q_end", "t_end", "q_start", "t_start", "aln_score2", "q_end2", "t_end2", "n_cigar_ops"):
        d[f] = torch.empty(b.n, dtype=torch.int32, device=dev)
    d["cigar"] = torch.empty(b.q_bytes, dtype=torch.uint8, device=dev)
    if kw["algo"] == G.KSW:
        d["seed_scores"] = torch.full((b.n,), 10, dtype=torch.int32, device=dev)
    ptrs = {k: v.data_ptr() for k, v in d.items()}
    mq, mt = int(b.q_lens.max()), int(b.t_lens.max())
    cells = int(np.sum(b.q_lens.astype(np.int64) * b.t_lens.astype(np.int64)))
    call = lambda: eng.align_device_ptrs(p, ptrs, b.q_bytes, b.t_bytes, b.n, mq, mt, stream.cuda_stream)
    call()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
    for a, z in evs:
        a.record(stream)
        call()
        z.record(stream)
    torch.cuda.synchronize(dev)
    ms = float(np.median([a.elapsed_time(z) for a, z in evs]))
    rec = {"mode": name, "plan": G.describe_plan(p, mq, mt), "pairs": b.n, "ms": round(ms, 3),
           "gcups": round(cells / ms / 1e6, 1)}
    out.append(rec)
    print(json.dumps(rec), flush=True)
