"""Debug probe: packed SEMI (TAIL=TARGET, with and without WITH_START; DBG_ALGO=global|local
for the others, HEAD=NONE cases) at each
forced minimum lane-group size (GASALX_GMIN), against the oracle, on the inputs
of tests/test_gpu_parity.py::test_semiglobal_with_start_wavefront.

  python tools/semi_start_debug.py            # parent: one child per G
  python tools/semi_start_debug.py child G    # one G (GASALX_GMIN already set)
"""
import json
import os
import subprocess
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "genomics-gpu_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, _p)

TMAX = int(os.environ.get("DBG_TMAX", "260"))
ALGO = os.environ.get("DBG_ALGO", "semi")   # semi | global | local
if len(sys.argv) < 3:
    for g in (8, 16, 32, 64):
        env = dict(os.environ, GASALX_GMIN=str(g))
        r = subprocess.run([sys.executable, __file__, "child", str(g)], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

import gasal_ffi as G  # noqa: E402
import helpers  # noqa: E402
import oracle as O  # noqa: E402

O.build()
eng = G.Engine(0)
FIELDS = ("score", "q_end", "t_end", "q_start", "t_start")
cases = [(h, al, sc) for h in (G.NONE, G.QUERY, G.TARGET, G.BOTH)
         for al, sc in ((b"ACGT", (1, 4, 6, 1)), (b"ACGT", (2, 3, 5, 2)), (b"ACGT", (3, 6, 0, 0)))]
for head, alphabet, scores in cases:
    a, bb, o, e = scores
    rng = np.random.default_rng(zlib.crc32(repr((head, alphabet, scores)).encode()) & 0xFFFF)
    qs, ts = helpers.random_pairs(rng, 1000, 1, 200, 1, TMAX, related=0.6, alphabet=alphabet)
    b = G.Batch.from_pairs(qs, ts)
    if ALGO != "semi" and head != G.NONE:
        continue
    for start in (0, G.WITH_START):
        if ALGO == "semi":
            kw = dict(algo=G.SEMI_GLOBAL, head=head, tail=G.TARGET, match=a, mismatch=bb,
                      gap_open=o, gap_extend=e, max_query_len=512)
        elif ALGO == "global":
            if start:
                continue
            kw = dict(algo=G.GLOBAL, match=a, mismatch=bb, gap_open=o, gap_extend=e, max_query_len=512)
        else:
            kw = dict(algo=G.LOCAL, match=a, mismatch=bb, gap_open=o, gap_extend=e, max_query_len=512)
        if start:
            kw["start_pos"] = start
        g = eng.align_host(b, G.make_params(**kw))
        r = O.align(b, O.make_params(**kw))
        bad = {f: np.nonzero(g[f] != r[f])[0] for f in FIELDS}
        bad = {f: v for f, v in bad.items() if v.size}
        idx = sorted({int(j) for v in bad.values() for j in v[:3]})[:3]
        ex = [{"i": i, "ql": int(b.q_lens[i]), "tl": int(b.t_lens[i]),
               **{f: [int(g[f][i]), int(r[f][i])] for f in FIELDS}} for i in idx]
        print(json.dumps({"algo": ALGO, "G": int(sys.argv[2]), "tmax": TMAX, "head": int(head), "scores": scores, "start": bool(start),
                          "bad": {f: int(v.size) for f, v in bad.items()}, "ex": ex}), flush=True)
