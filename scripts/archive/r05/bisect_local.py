"""Round 5 debug: the reference's sample pairs through LOCAL under the planner's switches, against
the oracle (which switch changes the mismatches)."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) == 1:
    for env in ({}, {"GASALX_SORT": "0"}, {}):
        r = subprocess.run([sys.executable, __file__, "x"], env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
        print(env, r.stdout.strip()[-600:], r.stderr.strip()[-400:], flush=True)
    sys.exit(0)
import numpy as np
import torch  # noqa
sys.path[:0] = [os.path.join(ROOT, "genomics-gpu_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import gasal_ffi as G, oracle as O, helpers
q, t, _, _ = helpers.read_fasta_pairs(limit=12000)
b = G.Batch.from_pairs(q, t)
eng = G.Engine(0)
o = O.align(b, O.make_params(algo=G.LOCAL))
for mode in ("host", "host_sub5000"):
    bb = b if mode == "host" else b.slice(0, 5000)
    oo = o if mode == "host" else {k: v[:5000] for k, v in o.items() if hasattr(v, "__len__")}
    g = eng.align_host(bb, G.make_params(algo=G.LOCAL), fields=["score", "q_end", "t_end"])
    bad = {f: np.flatnonzero(g[f] != oo[f]).tolist()[:5] for f in ("score", "q_end", "t_end")}
    nb = {f: int(np.count_nonzero(g[f] != oo[f])) for f in ("score", "q_end", "t_end")}
    ex = [(i, int(g["t_end"][i]), int(oo["t_end"][i]), int(bb.q_lens[i]), int(bb.t_lens[i])) for i in bad["t_end"]]
    print(mode, G.describe_plan(G.make_params(algo=G.LOCAL), int(bb.q_lens.max()), int(bb.t_lens.max())), nb, ex,
          eng.packed_pairs())
