"""Value-window edges of the packed (two pairs per lane, 16-bit) wavefront kernels.

The planner (dispatch.hip packed16_ok, and the e-drift frame conditions of make_plan)
admits a batch to a packed kernel only when every stored value provably stays inside the
positive-normal f16 window [0x0400, 0x7BFF].  These tests search, through the planner
itself (gasalx_describe_plan, host code), for the last score set or length it admits,
then align batches that push the values to that edge -- identical pairs (largest H),
unrelated pairs and long gaps (lowest values), lengths 1-40 beside full-length pairs in
one launch (two halves of one register with different lengths) -- bit-exactly against
the oracle, at the admitted edge (plan asserted packed) and one step past it (plan
asserted int32, or the non-drift packed kernel).  VERDICT r03 "What's weak" 2.
"""
import zlib

import numpy as np
import pytest

import gasal_ffi as G
import helpers
import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ("score", "q_end", "t_end", "q_start", "t_start")


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def plan(kw, ql, tl):
    return G.describe_plan(G.make_params(**kw), ql, tl)


def last_admitted(kw, key, lo, hi, ql, tl, prefix):
    """Largest value v of kw[key] in [lo, hi] whose plan at ql x tl starts with prefix,
    scanning upwards until the first refusal (the window conditions are monotone)."""
    last = None
    for v in range(lo, hi + 1):
        if plan(dict(kw, **{key: v}), ql, tl).startswith(prefix):
            last = v
        else:
            break
    return last


def edge_batch(seed, n, L, tl=None):
    """Pairs at the window's edges: identical (max score), unrelated, long gaps at the
    ends and in the middle, and short pairs (1-40) in the same launch."""
    rng = np.random.default_rng(seed)
    tl = tl or L
    qs, ts = [], []
    for i in range(n):
        kind = i % 6
        q = helpers.random_seq(rng, L)
        if kind == 0:                                   # identical: the largest H
            t = (q + helpers.random_seq(rng, tl))[:tl]
        elif kind == 1:                                 # unrelated
            t = helpers.random_seq(rng, tl)
        elif kind == 2:                                 # long leading gap in the target
            g = int(rng.integers(L // 3, L))
            t = (helpers.random_seq(rng, g) + q)[:tl]
        elif kind == 3:                                 # long gap in the middle
            h = L // 2
            t = (q[:h] + helpers.random_seq(rng, int(rng.integers(5, L // 2))) + q[h:])[:tl]
        elif kind == 4:                                 # short pairs beside full-length ones
            ql = int(rng.integers(1, 41))
            q = q[:ql]
            t = helpers.mutate(rng, q)[: int(rng.integers(1, 41))] or b"A"
        else:                                           # related
            t = (helpers.mutate(rng, q) + helpers.random_seq(rng, tl))[:tl]
        qs.append(q)
        ts.append(t)
    return G.Batch.from_pairs(qs, ts)


def check(engine, b, kw, cigar=False):
    g = engine.align_host(b, G.make_params(**kw))
    o = O.align(b, O.make_params(**kw))
    for f in FIELDS:
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, (f"{f}: {bad.size}/{b.n} mismatches; first #{bad[0]}: gpu={g[f][bad[0]]} "
                               f"oracle={o[f][bad[0]]} q={b.q_lens[bad[0]]} t={b.t_lens[bad[0]]} kw={kw}")
    if cigar:
        slot = (b.q_lens.astype(np.int64) + 7) // 8 * 8
        assert np.array_equal(g["n_ops"], o["n_ops"]), "n_cigar_ops differ"
        ok = o["n_ops"] <= slot
        ok[1:] &= o["n_ops"][:-1] <= slot[:-1]        # an overflowing CIGAR runs on
        for i in np.nonzero(ok)[0][:2000]:
            off, k = int(b.q_offsets[i]), int(o["n_ops"][i])
            assert np.array_equal(g["cigar"][off:off + k], o["cigar"][off:off + k]), f"cigar of pair {i}"


def _seed(*a):
    return zlib.crc32(repr(a).encode()) & 0xFFFF


# ---------------------------------------------------------------- LOCAL ----
@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (1, 1, 0, 1), (2, 3, 5, 2)])
def test_local_drift_frame_length_edge(engine, scores):
    # e-drift LOCAL kernel (step_local_dr): keys 0x0400 + H*C + (C-1-c) need (Hmax+1)*C <= 0x7800
    a, b, o, e = scores
    kw = dict(algo=G.LOCAL, match=a, mismatch=b, gap_open=o, gap_extend=e)
    L = None
    for cand in range(16, 520, 8):
        name = plan(kw, cand, cand)
        if name.startswith("wavefront16_local_G"):
            L = cand
        elif L is not None:
            break
    assert L is not None, plan(kw, 150, 150)
    inside = edge_batch(_seed(scores, 0), 600, L)
    check(engine, inside, kw)
    past = plan(kw, L + 8, L + 8)
    assert past.startswith(("wavefront16_local_u16_G", "wavefront16_local_seg", "wavefront16_local_nodrift_G",
                            "wavefront_local")), past
    check(engine, edge_batch(_seed(scores, 1), 600, L + 8), kw)


@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (2, 4, 6, 1), (2, 3, 5, 2)])
def test_local_u16_key_length_edge(engine, scores):
    # u16 keys (WF16_LOCAL_U16): (Hmax + 1) * C <= 65536; the first length past it takes the
    # round-2 kernel or the int32 one
    a, b, o, e = scores
    kw = dict(algo=G.LOCAL, match=a, mismatch=b, gap_open=o, gap_extend=e)
    L = None
    for cand in range(16, 600, 8):
        if plan(kw, cand, cand).startswith("wavefront16_local_u16_G"):
            L = cand
        elif L is not None:
            break
    assert L is not None
    check(engine, edge_batch(_seed("u16", scores, 0), 600, L), kw)
    past = plan(kw, L + 8, L + 8)
    assert not past.startswith("wavefront16_local_u16_G"), past
    check(engine, edge_batch(_seed("u16", scores, 1), 300, L + 8), kw)


def test_local_u16_keys_config2_match2_and_long_targets(engine):
    # config 2 at match 2 (outside the round-2 window) and 150 x 400 pairs (u16 keys instead
    # of the second key set), score + ends and WITH_START
    b = G.Batch.synth(2, 20000, 0x5EED0002)
    kw = dict(algo=G.LOCAL, match=2)
    assert plan(kw, 150, 150).startswith("wavefront16_local_u16_G")
    check(engine, b, kw)
    check(engine, b.slice(0, 6000), dict(kw, start_pos=G.WITH_START))
    rng = np.random.default_rng(77)
    qs, ts = helpers.random_pairs(rng, 3000, 100, 150, 200, 400)
    b2 = G.Batch.from_pairs(qs, ts)
    assert plan(dict(algo=G.LOCAL), 150, 400).startswith("wavefront16_local_u16_G")
    check(engine, b2, dict(algo=G.LOCAL))


@pytest.mark.parametrize("match", [1, 2, 3])
def test_local_segment_keys_300(engine, match):
    # 300 x 300 (config-3 data) past both single-key ranges: f16 keys by step segments
    # (WF16_LOCAL_SEG), score + ends, short pairs and gaps beside them
    kw = dict(algo=G.LOCAL, match=match)
    name = plan(kw, 300, 300)
    assert name.startswith("wavefront16_local_seg"), name
    check(engine, G.Batch.synth(3, 6000, 0x5EED0300 + match), kw)
    check(engine, edge_batch(_seed("seg", match), 1200, 300), kw)
    check(engine, G.Batch.synth(3, 2000, 0x5EED0310 + match), dict(kw, start_pos=G.WITH_START))


def test_local_segment_keys_match3_and_forced(engine, monkeypatch):
    # config 2 at match 3 (outside u16), and GASALX_KSEG=2 (segments before u16 keys) at match 2,
    # against the oracle; segment lengths from 8 (1 kb targets) up
    b = G.Batch.synth(2, 20000, 0x5EED0003)
    kw = dict(algo=G.LOCAL, match=3)
    assert plan(kw, 150, 150).startswith("wavefront16_local_seg64_G")
    check(engine, b, kw)
    monkeypatch.setenv("GASALX_KSEG", "2")
    assert plan(dict(algo=G.LOCAL, match=2), 150, 150).startswith("wavefront16_local_seg64_G")
    check(engine, b, dict(algo=G.LOCAL, match=2))
    monkeypatch.delenv("GASALX_KSEG")
    rng = np.random.default_rng(78)
    qs, ts = helpers.random_pairs(rng, 1500, 60, 150, 300, 500)
    kw1 = dict(algo=G.LOCAL, match=2)
    assert "_seg" in plan(kw1, 150, 500), plan(kw1, 150, 500)
    check(engine, G.Batch.from_pairs(qs, ts), kw1)


@pytest.mark.parametrize("L", [40, 150])
def test_local_packed_score_edge(engine, L):
    # packed LOCAL: a * min(ql, tl) <= 255 (16-bit keys), a + K <= 255 (table bytes)
    kw = dict(algo=G.LOCAL, mismatch=4, gap_open=6, gap_extend=1)
    a = last_admitted(kw, "match", 1, 255, L, L, "wavefront16_local")
    assert a is not None and a >= 1
    check(engine, edge_batch(_seed(L, a), 600, L), dict(kw, match=a))
    assert plan(dict(kw, match=a + 1), L, L).startswith("wavefront_local"), plan(dict(kw, match=a + 1), L, L)
    check(engine, edge_batch(_seed(L, a + 1), 300, L), dict(kw, match=a + 1))


# --------------------------------------------------------------- GLOBAL ----
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("key", ["gap_extend", "match"])
def test_global_window_edge(engine, tb, key):
    # GLOBAL (+TB): the drift frame's top, B + a*min + e*span, must stay under 0x7BFF
    kw = dict(algo=G.GLOBAL, match=1, mismatch=4, gap_open=6, gap_extend=1)
    if tb:
        kw["start_pos"] = G.WITH_TB
    L = 300
    pre = "wavefront16_global"
    v = last_admitted(kw, key, 1, 255, L, L, pre)
    assert v is not None
    kin = dict(kw, **{key: v})
    assert plan(kin, L, L).startswith(pre)
    check(engine, edge_batch(_seed(tb, key, v), 400, L), kin, cigar=tb)
    kout = dict(kw, **{key: v + 1})
    assert not plan(kout, L, L).startswith(pre), plan(kout, L, L)
    check(engine, edge_batch(_seed(tb, key, v + 1), 200, L), kout, cigar=tb)


def test_global_traceback_short_pairs_every_band(engine, monkeypatch):
    # lengths 1-40 (the r03 e-drift failure class) through the band traceback with windows
    # narrower and wider than a lane's rows
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    rng = np.random.default_rng(41)
    qs, ts = helpers.random_pairs(rng, 1500, 1, 40, 1, 40)
    b = G.Batch.from_pairs(qs, ts)
    for w in ("0", "2", "8", "24"):
        monkeypatch.setenv("GASALX_TB_BAND_W", w)
        assert "_tbband_" in plan(kw, 40, 40)
        check(engine, b, kw, cigar=True)
    # queries much longer than their targets (lanes whose band window lies past the
    # wave's widest target stop at it), the long queries' rows beyond the targets in most lanes
    qs, ts = helpers.random_pairs(rng, 1500, 200, 300, 1, 60)
    b = G.Batch.from_pairs(qs, ts)
    for w in ("2", "10"):
        monkeypatch.setenv("GASALX_TB_BAND_W", w)
        assert "_tbband_" in plan(kw, 300, 60)
        check(engine, b, kw, cigar=True)


# ---------------------------------------------------------- SEMI-GLOBAL ----
@pytest.mark.parametrize("tail", [G.TARGET, G.QUERY, G.BOTH])
@pytest.mark.parametrize("key", ["gap_extend", "match"])
def test_semiglobal_window_edge(engine, tail, key):
    # SEMI (TAIL=TARGET: transposed sweep; TAIL=QUERY/BOTH: class launches): the frame's top
    # B + a*min + e*(2*span + 1) under 0x7BFF
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=tail, match=1, mismatch=4, gap_open=6, gap_extend=1)
    ql, tl = 150, 182
    pre = "wavefront16_semi"
    v = last_admitted(kw, key, 1, 255, ql, tl, pre)
    assert v is not None
    kin = dict(kw, **{key: v})
    check(engine, edge_batch(_seed(tail, key, v), 600, ql, tl), kin)
    kout = dict(kw, **{key: v + 1})
    assert not plan(kout, ql, tl).startswith(pre), plan(kout, ql, tl)
    check(engine, edge_batch(_seed(tail, key, v + 1), 300, ql, tl), kout)


@pytest.mark.parametrize("head", [G.NONE, G.QUERY, G.TARGET, G.BOTH])
def test_semiglobal_short_pairs_every_head(engine, head):
    # lengths 1-40 beside 150 x 182 pairs in one launch, every HEAD, TAIL=TARGET
    kw = dict(algo=G.SEMI_GLOBAL, head=head, tail=G.TARGET)
    b = edge_batch(_seed("short", head), 900, 150, 182)
    assert plan(kw, 150, 182).startswith("wavefront16_semi")
    check(engine, b, kw)
