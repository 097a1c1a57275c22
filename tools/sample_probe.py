"""Kernel time on the reference's own sample data: the test_prog pairs
(tests/golden/{query,target}_batch.fasta.gz, 20,000 pairs, query 150 bp, target
152-277 bp) replicated to N pairs, device-resident.  Unlike the synthetic
configs the targets vary in length (and exceed 256 bases).

  python tools/sample_probe.py [pairs] [mode,...]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gasal_ffi as G  # noqa: E402
import helpers  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["local", "local_start", "local_tb", "semi_tt", "global"]
PARAMS = {
    "local": dict(algo=G.LOCAL),
    "local_start": dict(algo=G.LOCAL, start_pos=G.WITH_START),
    "local_tb": dict(algo=G.LOCAL, start_pos=G.WITH_TB),
    "semi_tt": dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET),
    "global": dict(algo=G.GLOBAL),
}
q, t, _, _ = helpers.read_fasta_pairs()
reps = -(-n // len(q))
b = G.Batch.from_pairs((q * reps)[:n], (t * reps)[:n])
dev = torch.device("cuda", 0)
eng = G.Engine(0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
as_i32 = lambda a: torch.from_numpy(a.view(np.int32).copy()).to(dev)
d = {"q_batch": torch.from_numpy(b.q_data).to(dev), "t_batch": torch.from_numpy(b.t_data).to(dev),
     "q_offsets": as_i32(b.q_offsets), "t_offsets": as_i32(b.t_offsets),
     "q_lens": as_i32(b.q_lens), "t_lens": as_i32(b.t_lens)}
for f in ("aln_score", "q_end", "t_end", "q_start", "t_start", "n_cigar_ops"):
    d[f] = torch.empty(b.n, dtype=torch.int32, device=dev)
d["cigar"] = torch.empty(b.q_bytes, dtype=torch.uint8, device=dev)
ptrs = {k: v.data_ptr() for k, v in d.items()}
mq, mt = int(b.q_lens.max()), int(b.t_lens.max())
cells = int(np.sum(b.q_lens.astype(np.int64) * b.t_lens.astype(np.int64)))
for name in modes:
    p = G.make_params(**PARAMS[name])
    call = lambda: eng.align_device_ptrs(p, ptrs, b.q_bytes, b.t_bytes, b.n, mq, mt, stream.cuda_stream)
    call()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, z in evs:
        a.record(stream)
        call()
        z.record(stream)
    torch.cuda.synchronize(dev)
    ms = float(np.median([a.elapsed_time(z) for a, z in evs]))
    print(json.dumps({"mode": name, "data": f"test_prog sample pairs x{reps}", "plan": G.describe_plan(p, mq, mt),
                      "pairs": b.n, "mean_q": round(float(b.q_lens.mean()), 1),
                      "mean_t": round(float(b.t_lens.mean()), 1), "ms": round(ms, 3),
                      "gcups": round(cells / ms / 1e6, 1),
                      "lib": os.path.basename(os.environ.get("GASALX_LIB", "libgasal.so")),
                      "sort": os.environ.get("GASALX_SORT", "auto")}), flush=True)
