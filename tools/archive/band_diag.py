"""Diagnostic: GLOBAL+TB band recomputation vs the oracle on one batch under several
GASALX_TB_BAND / GASALX_TB_BAND_W settings (GPU)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gasal_ffi as G, oracle as O, helpers
O.build()
eng = G.Engine(0)
rng = np.random.default_rng(33)
lo, hi, n = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (8, 64, 600)))
qs, ts = helpers.random_pairs(rng, n, lo, hi, lo, hi)
b = G.Batch.from_pairs(qs, ts)
kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
o = O.align(b, O.make_params(**kw))
keep = np.nonzero(o["n_ops"] <= (b.q_lens + 7) // 8 * 8)[0]
b = b.subset(keep); o = O.align(b, O.make_params(**kw))
for env in ({"GASALX_TB_BAND": "0"}, {"GASALX_TB_BAND_W": "12"}, {"GASALX_TB_BAND_W": "0"}, {"GASALX_TB_BAND_W": "64"}):
    for k in ("GASALX_TB_BAND", "GASALX_TB_BAND_W"): os.environ.pop(k, None)
    os.environ.update(env)
    g = eng.align_host(b, G.make_params(**kw))
    bad = np.nonzero(g["n_ops"] != o["n_ops"])[0]
    sb = np.nonzero(g["score"] != o["score"])[0]
    print(env, G.describe_plan(G.make_params(**kw), hi, hi), "n", b.n, "score bad", sb.size, "n_ops bad", bad.size,
          "first", [(int(i), int(b.q_lens[i]), int(b.t_lens[i]), int(g["n_ops"][i]), int(o["n_ops"][i])) for i in bad[:6]],
          flush=True)
eng.close()
