"""Triage: LOCAL WITH_START pairs whose start differs from the oracle (config-2 synth,
20K pairs, seed 0x5EED0002), printed with their forward results."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "genomics-gpu_amd"), os.path.join(ROOT, "oracle")]
import gasal_ffi as G
import oracle as O
O.build()
eng = G.Engine(0)
b = G.Batch.synth(2, 20_000, 0x5EED0002)
for kf in ("1", "0"):
    os.environ["GASALX_KF16"] = kf
    g = eng.align_host(b, G.make_params(algo=G.LOCAL, start_pos=G.WITH_START))
    o = O.align(b, O.make_params(algo=O.LOCAL, start_pos=O.WITH_START))
    for f in ("score", "q_end", "t_end", "q_start", "t_start"):
        bad = np.flatnonzero(g[f] != o[f])
        print("kf16", kf, f, bad.size, bad[:5].tolist())
    bad = np.flatnonzero((g["q_start"] != o["q_start"]) | (g["t_start"] != o["t_start"]))
    for i in bad[:3]:
        print(i, {f: (int(g[f][i]), int(o[f][i])) for f in ("score", "q_end", "t_end", "q_start", "t_start")},
              "ql", int(b.q_lens[i]), "tl", int(b.t_lens[i]))
