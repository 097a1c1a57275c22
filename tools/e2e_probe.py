"""Time the host-staged entry point (gasalx_align_host) on a config-2 batch; run
under rocprofv3 --kernel-trace --memory-copy-trace to see the copy/kernel overlap."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-gpu_amd"))
import gasal_ffi as G  # noqa: E402

kind = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else {2: 1000000, 3: 100000}[kind]
eng = G.Engine(0)
b = G.Batch.synth(kind, n, 0x5EED0000 + kind)
p = G.make_params(algo=G.LOCAL) if kind == 2 else G.make_params(algo=G.GLOBAL, start_pos=G.WITH_TB)
fields = ["score", "q_end", "t_end"] if kind == 2 else ["score"]
for i in range(4):
    t = time.perf_counter()
    eng.align_host(b, p, fields=fields)
    print(f"iter {i}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
