#!/usr/bin/env python3
"""Config-3 pairs whose oracle CIGAR path leaves its lane band window, per band half width w
(the wavefront16 GLOBAL_CP band: lane lg of R = 20 rows covers columns [max(lg*R - w, 0), + ((R + 2w + 3) & ~3))).
Test/analysis tool: runs the oracle (oracle/), never the product path.  profiles/r05/n_band_width.md."""
import sys, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'genomics-gpu_amd')
import oracle.oracle as O
import gasal_ffi as G
n = 100000
b = G.Batch.synth(3, n, 0x5EED0003)
r = O.align(b, O.make_params(algo=O.GLOBAL, start_pos=O.WITH_TB), n_threads=8)
cig, nops, qoff = r['cigar'], r['n_ops'], b.q_offsets
R = 20
ws = [10, 12, 16, 20, 22, 24]
cnt = {w: 0 for w in ws}
maxdev = []
for k in range(n):
    ops = cig[qoff[k]:qoff[k] + nops[k]][::-1]      # reversed RLE -> forward order
    i = j = 0   # i: target col, j: query row
    rows, cols = [], []
    for byte in ops:
        op, c = byte & 3, byte >> 2
        for _ in range(c):
            if op in (0, 1): i += 1; j += 1
            elif op == 2: i += 1
            else: j += 1
            rows.append(j); cols.append(i)
    rows = np.array(rows); cols = np.array(cols)
    maxdev.append(np.abs(cols - rows).max() if len(rows) else 0)
    lane = rows // R
    for w in ws:
        L = np.maximum(lane * R - w, 0); wd = ((R + 2 * w) + 3) & ~3
        t = cols - L
        if np.any((t < 0) | (t >= wd)): cnt[w] += 1
md = np.array(maxdev)
print('max |col-row| on path: max', md.max(), 'p99', np.percentile(md, 99), 'p999', np.percentile(md, 99.9))
print({w: cnt[w] for w in ws}, 'of', n)
