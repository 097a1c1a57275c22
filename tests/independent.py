"""Second, independent CPU restatement of the GASAL2 score kernels, in numpy,
vectorised across pairs (TEST INFRASTRUCTURE ONLY).

Why a second one: the C oracle (oracle/gasal_oracle.c) and the engine's
thread-per-pair kernels (genomics-gpu_amd/csrc/generic.hpp) were written by the
same hand and follow each other closely, so a misreading shared by both would
pass every parity test between them.  This module is written directly from the
reference kernels' loop structure, in a different form (all pairs advance
together, one numpy op per cell position; state arrays indexed like the
reference's h/f/p/e/global registers), and is used to check the C oracle on
config 1 and on random batches (tests/test_independent.py).

Reference loop structure restated (paths under Non-CDP/GASAL2/src/kernels):
  for each 8-column target strip i:            (local_kernel_template.h:122, global.h:65,
      reset h/f/p for the strip                 semiglobal_kernel_template.h:110)
      for each query row ridx (padded):
          h[0], e = global[ridx]                (short2: int16 storage)
          for m = 1..8: CORE_*_COMPUTE          (local :19-30, global.h:4-12, semi :17-28)
          global[ridx] = (h[8], e)
Pad bases (N_CODE) are scored like the reference: LOCAL rule (N scores 0, or
-N_PENALTY) for local/semi-global, no N rule for global (gasal_kernels.h:39-56).
"""
from __future__ import annotations

import numpy as np

MINUS_INF = -32768


def _codes(data, offs, lens, n_code):
    """[n, pad8(max)] 4-bit codes; positions past a pair's padded length read N."""
    pad = (lens.astype(np.int64) + 7) // 8 * 8
    width = int(pad.max(initial=8))
    idx = offs.astype(np.int64)[:, None] + np.arange(width)[None, :]
    inside = np.arange(width)[None, :] < pad[:, None]
    src = np.where(inside, np.minimum(idx, len(data) - 1), 0)
    c = (data[src].astype(np.int32) & 15)
    return np.where(inside, c, n_code & 15), pad


def _sub(rb, gb, a, b, nval, npen, n_rule):
    s = np.where(rb == gb, a, -b)
    if n_rule or npen is not None:
        s = np.where((rb == nval) | (gb == nval), -(npen or 0) if npen is not None else 0, s)
    return s


def _i16(x):
    return x.astype(np.int16).astype(np.int32)


def local(batch, a=1, b=4, o=6, e=1, n_code=0x4E, npen=None, second=False):
    """gasal_local_kernel<LOCAL, WITHOUT_START, B> (local_kernel_template.h:72-439)."""
    q, qpad = _codes(batch.q_data, batch.q_offsets, batch.q_lens, n_code)
    t, tpad = _codes(batch.t_data, batch.t_offsets, batch.t_lens, n_code)
    n, R = q.shape
    T = t.shape[1]
    nval, OE = n_code & 15, o + e
    gH = np.zeros((R + 1, n), np.int32)
    gE = np.zeros((R + 1, n), np.int32)
    maxHH = np.zeros(n, np.int32)
    maxY = np.zeros(n, np.int32)
    prev = np.zeros(n, np.int32)
    maxX = np.zeros(n, np.int32)
    m2 = np.zeros(n, np.int32); y2 = np.zeros(n, np.int32); prev2 = np.zeros(n, np.int32)
    x2 = np.zeros(n, np.int32)
    for i in range(T // 8):
        strip_ok = i * 8 < tpad
        h = np.zeros((9, n), np.int32); f = np.zeros((9, n), np.int32); p = np.zeros((9, n), np.int32)
        gb = t[:, i * 8:i * 8 + 8].T
        for r in range(R):
            ok = strip_ok & (r < qpad)
            h[0] = gH[r]; ee = gE[r].copy()
            rb = q[:, r]
            for m in range(1, 9):
                s = _sub(rb, gb[m - 1], a, b, nval, npen, True)
                tmp = p[m] + s
                H = np.maximum(np.maximum(np.maximum(tmp, f[m]), ee), 0)
                h[m] = H
                f[m] = np.maximum(tmp - OE, f[m] - e)
                ee = np.maximum(tmp - OE, ee - e)
                upd = ok & (maxHH < H)
                maxY = np.where(upd, i * 8 + m - 1, maxY)
                maxHH = np.where(upd, H, maxHH)
                if second:
                    ov = ok & (m2 < H) & (maxHH > H)
                    y2 = np.where(ov, i * 8 + m - 1, y2)
                    m2 = np.where(ov, H, m2)
                p[m] = h[m - 1]
            gH[r] = _i16(h[8]); gE[r] = _i16(ee)
            maxX = np.where(ok & (prev < maxHH), r, maxX)
            if second:
                x2 = np.where(ok & (prev2 < maxHH), r, x2)     # the reference compares maxHH here (:417)
                prev2 = np.where(ok, np.maximum(m2, prev2), prev2)
            prev = np.where(ok, np.maximum(maxHH, prev), prev)
    out = {"score": maxHH, "q_end": maxX, "t_end": maxY}
    if second:
        out.update(score2=m2, q_end2=x2, t_end2=y2)
    return out


def global_(batch, a=1, b=4, o=6, e=1, n_code=0x4E, npen=None):
    """gasal_global_kernel (global.h:31-303): score = H(ql-1, tl-1)."""
    q, qpad = _codes(batch.q_data, batch.q_offsets, batch.q_lens, n_code)
    t, tpad = _codes(batch.t_data, batch.t_offsets, batch.t_lens, n_code)
    n, R = q.shape
    T = t.shape[1]
    nval, OE = n_code & 15, o + e
    ql, tl = batch.q_lens.astype(np.int64), batch.t_lens.astype(np.int64)
    rows = np.arange(R + 1)
    gH = _i16(np.broadcast_to(np.where(rows == 0, 0, -(o + e * rows))[:, None], (R + 1, n)))   # short2 init
    gE = np.full((R + 1, n), MINUS_INF, np.int32)
    score = np.zeros(n, np.int32)
    for i in range(T // 8):
        h = np.zeros((9, n), np.int32); p = np.zeros((9, n), np.int32)
        f = np.full((9, n), MINUS_INF, np.int32)
        for m in range(1, 9):
            c = i * 8 + m - 1
            p[m] = 0 if c == 0 else -(o + e * c)
        gb = t[:, i * 8:i * 8 + 8].T
        for r in range(R):
            h[0] = gH[r]; ee = gE[r].copy()
            rb = q[:, r]
            for m in range(1, 9):
                s = _sub(rb, gb[m - 1], a, b, nval, npen, False)
                tmp = p[m] + s
                h[m] = np.maximum(np.maximum(tmp, f[m]), ee)
                f[m] = np.maximum(tmp - OE, f[m] - e)
                ee = np.maximum(tmp - OE, ee - e)
                p[m] = h[m - 1]
            gH[r] = _i16(h[8]); gE[r] = _i16(ee)
            # global.h:98-103,299: H of row ql-1 at column tl-1 (the pair's last strip)
            hit = (r == ql - 1) & (i == (tl - 1) // 8)
            col = ((tl - 1) % 8 + 1).astype(np.int64)
            score = np.where(hit, h[col, np.arange(n)], score)
    return {"score": score}


def semi(batch, head=2, tail=2, a=1, b=4, o=6, e=1, n_code=0x4E, npen=None):
    """gasal_semi_global_kernel<.., WITHOUT_START, FALSE, HEAD, TAIL>
    (semiglobal_kernel_template.h:40-225).  head/tail: 0 NONE 1 QUERY 2 TARGET 3 BOTH."""
    q, qpad = _codes(batch.q_data, batch.q_offsets, batch.q_lens, n_code)
    t, tpad = _codes(batch.t_data, batch.t_offsets, batch.t_lens, n_code)
    n, R = q.shape
    T = t.shape[1]
    nval, OE = n_code & 15, o + e
    ql, tl = batch.q_lens.astype(np.int64), batch.t_lens.astype(np.int64)
    head_q, head_t = head in (1, 3), head in (2, 3)
    tail_q, tail_t = tail in (1, 3), tail in (2, 3)
    rows = np.arange(R + 1)
    if head_q:
        gH = np.zeros((R + 1, n), np.int32); gE = np.zeros((R + 1, n), np.int32)
    else:
        gH = _i16(np.broadcast_to(np.where(rows == 0, 0, -(o + e * rows))[:, None], (R + 1, n)))   # short2 init
        gE = np.full((R + 1, n), MINUS_INF, np.int32)
    maxHH = np.full(n, MINUS_INF, np.int32)
    maxX = tl.astype(np.int32).copy()     # :63 (Q10)
    maxY = ql.astype(np.int32).copy()
    for i in range(T // 8):
        strip_ok = i * 8 < tpad
        h = np.zeros((9, n), np.int32); p = np.zeros((9, n), np.int32)
        f = np.full((9, n), MINUS_INF, np.int32)
        if not head_t:
            for m in range(1, 9):
                c = i * 8 + m - 1
                h[m] = -(o + e * c)                       # :123-128 (Q3)
                p[m] = 0 if c == 0 else -(o + e * c)
        gb = t[:, i * 8:i * 8 + 8].T
        for r in range(R):
            ok = strip_ok & (r < qpad)
            h[0] = gH[r]; ee = gE[r].copy()
            prev_d = h[0] - OE
            rb = q[:, r]
            for m in range(1, 9):
                s = _sub(rb, gb[m - 1], a, b, nval, npen, True)
                cur = h[m] - OE
                f[m] = np.maximum(cur, f[m] - e)
                cur = np.maximum(p[m] + s, f[m])
                ee = np.maximum(prev_d, ee - e)
                cur = np.maximum(cur, ee)
                h[m] = cur
                p[m] = prev_d + OE
                prev_d = cur - OE
            # a strip past the pair's own target leaves its row buffer alone (TAIL QUERY reads it)
            gH[r] = np.where(strip_ok, _i16(h[8]), gH[r]); gE[r] = np.where(strip_ok, _i16(ee), gE[r])
            if tail_t:
                last = ok & (r == ql - 1)
                for m in range(1, 9):
                    col = i * 8 + m - 1
                    upd = last & (h[m] > maxHH) & (col < tl)
                    maxY = np.where(upd, col, maxY)
                    maxHH = np.where(upd, h[m], maxHH)
    if tail_q:
        # :185-193: H at the last padded column (global[m].x), rows m < ql (Q11)
        for mrow in range(R):
            v = gH[mrow]
            upd = (v > maxHH) & (mrow < ql)
            maxX = np.where(upd, mrow, maxX)
            maxHH = np.where(upd, v, maxHH)
        maxY = np.where(maxX != tl, ql, maxY)
    return {"score": maxHH, "q_end": maxX, "t_end": maxY}
