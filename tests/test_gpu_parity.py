"""GPU parity: the HIP engine (through the C-ABI, gasal_ffi) against the CPU
oracle on identical inputs.  Integer outputs must match bit-exactly; PairHMM
within 1e-5 relative (BASELINE.json north_star)."""
import os

import zlib

import numpy as np
import pytest

import gasal_ffi as G
import helpers
import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ("score", "q_end", "t_end", "q_start", "t_start", "score2", "q_end2", "t_end2")


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def _params_pair(**kw):
    return G.make_params(**kw), O.make_params(**kw)


def check(engine, batch, q_ops=None, t_ops=None, seed=None, cigar=False, **kw):
    gp, op = _params_pair(**kw)
    g = engine.align_host(batch, gp, q_ops=q_ops, t_ops=t_ops, seed_scores=seed)
    o = O.align(batch, op, q_ops=q_ops, t_ops=t_ops, seed_scores=seed)
    for f in FIELDS:
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, (f"{f}: {bad.size}/{batch.n} mismatches; first #{bad[0]}: gpu={g[f][bad[0]]} "
                               f"oracle={o[f][bad[0]]} q={batch.q_lens[bad[0]]} t={batch.t_lens[bad[0]]} kw={kw}")
    if cigar:
        assert np.array_equal(g["n_ops"], o["n_ops"]), "n_cigar_ops differ"
        assert np.array_equal(g["cigar"], o["cigar"]), "cigar bytes differ"
    return g, o


def no_cigar_overflow(batch, **kw):
    """Drop pairs whose CIGAR outgrows its pad8(ql)-byte slot (the
    reference then overwrites the neighbour's slot, order-dependent)."""
    o = O.align(batch, O.make_params(**kw))
    keep = np.nonzero(o["n_ops"] <= (batch.q_lens + 7) // 8 * 8)[0]
    return batch.subset(keep) if len(keep) < batch.n else batch


def rand_batch(seed, n, qmin, qmax, tmin, tmax, alphabet=b"ACGT", related=0.7):
    rng = np.random.default_rng(seed)
    qs, ts = helpers.random_pairs(rng, n, qmin, qmax, tmin, tmax, related=related, alphabet=alphabet)
    return G.Batch.from_pairs(qs, ts)


# ------------------------------------------------------------------ KATs ----
def test_kat_through_gpu(engine):
    kat = helpers.kat()
    b = G.Batch.from_pairs([p["q"] for p in kat["pairs"]], [p["t"] for p in kat["pairs"]])
    gp = G.make_params(algo=G.LOCAL)
    r = engine.align_host(b, gp)
    for i, p in enumerate(kat["pairs"]):
        assert (r["score"][i], r["q_end"][i], r["t_end"][i]) == (p["local"]["score"], p["local"]["q_end"],
                                                                 p["local"]["t_end"])
    r = engine.align_host(b, G.make_params(algo=G.GLOBAL, start_pos=G.WITH_TB))
    for i, p in enumerate(kat["pairs"]):
        e = p["global_tb"]
        assert r["score"][i] == e["score"] and r["n_ops"][i] == e["n_ops"]
        off = int(b.q_offsets[i])
        assert list(r["cigar"][off:off + e["n_ops"]]) == e["bytes_rev"]
    r = engine.align_host(b, G.make_params(algo=G.SEMI_GLOBAL))
    for i, p in enumerate(kat["pairs"]):
        e = p["semi_tt"]
        assert (r["score"][i], r["q_end"][i], r["t_end"][i]) == (e["score"], e["q_end"], e["t_end"])


# ----------------------------------------------------------------- local ----
@pytest.mark.parametrize("qr,tr", [((1, 40), (1, 40)), ((60, 64), (60, 64)), ((140, 160), (140, 160)),
                                   ((150, 150), (150, 150)), ((200, 320), (150, 400)), ((600, 1200), (500, 900))])
def test_local_random(engine, qr, tr):
    b = rand_batch(hash((qr, tr)) & 0xFFFF, 700, *qr, *tr)
    check(engine, b, algo=G.LOCAL)


def test_local_with_n_bases(engine):
    b = rand_batch(11, 800, 20, 150, 20, 150, alphabet=b"ACGTN")
    check(engine, b, algo=G.LOCAL)


def test_local_other_iupac_and_lowercase(engine):
    b = rand_batch(12, 500, 30, 120, 30, 120, alphabet=b"ACGTacgtRYKMSWN")
    check(engine, b, algo=G.LOCAL)


@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (2, 3, 5, 2), (5, 4, 10, 1), (1, 1, 0, 1), (3, 6, 0, 0)])
def test_local_scores(engine, scores):
    a, bb, o, e = scores
    b = rand_batch(13 + a, 500, 50, 160, 50, 160)
    check(engine, b, algo=G.LOCAL, match=a, mismatch=bb, gap_open=o, gap_extend=e)


def test_local_sample_fasta(engine):
    q, t, _, _ = helpers.read_fasta_pairs(limit=3000)
    check(engine, G.Batch.from_pairs(q, t), algo=G.LOCAL)


def test_local_traceback(engine):
    q, t, _, _ = helpers.read_fasta_pairs(limit=1500)
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_TB)
    check(engine, no_cigar_overflow(G.Batch.from_pairs(q, t), **kw), cigar=True, **kw)
    check(engine, no_cigar_overflow(rand_batch(21, 500, 10, 100, 10, 100), **kw), cigar=True, **kw)


def test_local_with_start(engine):
    q, t, _, _ = helpers.read_fasta_pairs(limit=800)
    check(engine, G.Batch.from_pairs(q, t), algo=G.LOCAL, start_pos=G.WITH_START)


@pytest.mark.parametrize("qr,tr,alphabet,scores", [
    ((1, 40), (1, 40), b"ACGT", (1, 4, 6, 1)),
    ((140, 160), (140, 160), b"ACGT", (1, 4, 6, 1)),
    ((1, 200), (1, 250), b"ACGTN", (1, 4, 6, 1)),
    ((50, 150), (50, 180), b"ACGTRYacgt", (1, 4, 6, 1)),       # declined blocks -> int32 kernel both passes
    ((60, 160), (60, 160), b"ACGT", (2, 3, 5, 2)),
    ((60, 160), (60, 160), b"ACGT", (3, 6, 0, 0)),
    ((200, 320), (150, 400), b"ACGT", (1, 4, 6, 1)),          # int32 wavefront (target > 256)
])
def test_local_with_start_wavefront(engine, qr, tr, alphabet, scores):
    # WITH_START runs the LOCAL wavefront kernel twice (forward, then on the reversed
    # end-word-aligned slots, start.hpp); local_kernel_template.h:441-511 incl. Q8
    a, bb, o, e = scores
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_START, match=a, mismatch=bb, gap_open=o, gap_extend=e)
    assert G.describe_plan(G.make_params(**kw), qr[1], tr[1]).startswith(("wavefront16_local_start",
                                                                            "wavefront_local_start"))
    b = rand_batch(zlib.crc32(repr((qr, tr, alphabet, scores)).encode()) & 0xFFFF, 1200, *qr, *tr,
                   alphabet=alphabet, related=0.5)
    check(engine, b, **kw)


def test_local_with_start_config2_sample(engine):
    engine.packed_pairs()                                    # forget earlier launches
    check(engine, G.Batch.synth(2, 20000, 0x5EED0002), algo=G.LOCAL, start_pos=G.WITH_START)
    # the reverse pass (the last packed launch) read the forward sequences backwards on the
    # packed kernel for every pair (start.hpp, WfArgs::rev)
    handled, total = engine.packed_pairs()
    assert total == 20000 and handled == total, (handled, total)


def test_local_with_start_shared_query_and_zero_scores(engine):
    # one-to-many pairing (every pair reads the same query slot) and all-mismatch pairs (score 0 -> start 0,0)
    rng = np.random.default_rng(77)
    q = helpers.random_seq(rng, 120, b"ACGT")
    ts = [helpers.random_seq(rng, int(rng.integers(1, 200)), b"ACGT") for _ in range(300)] + [b"TTTT"] * 5
    b1 = G.Batch.from_pairs([q] * len(ts), ts)
    shared = G.Batch(b1.q_data[:int(b1.q_offsets[1])].copy(), np.zeros(b1.n, np.uint32), b1.q_lens,
                     b1.t_data, b1.t_offsets, b1.t_lens)
    check(engine, shared, algo=G.LOCAL, start_pos=G.WITH_START)
    zb = G.Batch.from_pairs([b"AAAA", b"A", b"CCCCCCCCC"], [b"TTTT", b"G", b"GGG"])
    g, _ = check(engine, zb, algo=G.LOCAL, start_pos=G.WITH_START)
    assert list(g["q_start"]) == [0, 0, 0] and list(g["t_start"]) == [0, 0, 0]


@pytest.mark.parametrize("npen", [0, 2, -1])
def test_local_with_start_n_penalty(engine, npen):
    b = rand_batch(98 + npen, 800, 5, 150, 5, 170, alphabet=b"ACGTACGTN", related=0.6)
    check(engine, b, algo=G.LOCAL, start_pos=G.WITH_START, n_penalty=npen)


def test_local_with_start_packed_and_ops(engine):
    b = rand_batch(96, 600, 10, 150, 10, 150)
    rng = np.random.default_rng(97)
    qo = rng.integers(0, 4, b.n).astype(np.uint8)
    to = rng.integers(0, 4, b.n).astype(np.uint8)
    check(engine, b, q_ops=qo, t_ops=to, algo=G.LOCAL, start_pos=G.WITH_START)


@pytest.mark.parametrize("alphabet,scores", [(b"ACGT", (1, 4, 6, 1)), (b"ACGTN", (2, 3, 5, 2)),
                                             (b"ACGTRY", (1, 4, 6, 1))])
def test_local_long_targets_two_keys(engine, monkeypatch, alphabet, scores):
    # packed LOCAL over 257..512 target columns: the round-2 kernel's second key set per row
    # (GASALX_KF16=0), and the e-drift kernels the planner takes by default (u16 keys or
    # step segments), on the same pairs
    a, bb, o, e = scores
    kw = dict(algo=G.LOCAL, match=a, mismatch=bb, gap_open=o, gap_extend=e)
    default = G.describe_plan(G.make_params(**kw), 120, 512)
    assert default.startswith(("wavefront16_local_u16_G8R16", "wavefront16_local_seg")), default
    rng = np.random.default_rng(zlib.crc32(repr((alphabet, scores)).encode()) & 0xFFFF)
    qs, ts = helpers.random_pairs(rng, 1500, 1, 120, 200, 512, alphabet=alphabet, related=0.5)
    # ties across the 256-column boundary: a repeated block on both sides of it
    rep = helpers.random_seq(rng, 40)
    qs += [rep] * 20
    ts += [helpers.random_seq(rng, 230 + i) + rep + helpers.random_seq(rng, 10) + rep for i in range(20)]
    check(engine, G.Batch.from_pairs(qs, ts), **kw)
    check(engine, G.Batch.from_pairs(qs[:600], ts[:600]), start_pos=G.WITH_START, **kw)
    monkeypatch.setenv("GASALX_KF16", "0")
    assert G.describe_plan(G.make_params(**kw), 120, 512) == "wavefront16_local_k2_G8R16"
    check(engine, G.Batch.from_pairs(qs, ts), **kw)
    check(engine, G.Batch.from_pairs(qs[:600], ts[:600]), start_pos=G.WITH_START, **kw)


@pytest.mark.parametrize("kw", [dict(algo=G.LOCAL), dict(algo=G.LOCAL, start_pos=G.WITH_START),
                                dict(algo=G.LOCAL, start_pos=G.WITH_TB), dict(algo=G.GLOBAL),
                                dict(algo=G.GLOBAL, start_pos=G.WITH_TB),
                                dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET),
                                dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET, start_pos=G.WITH_START,
                                     max_query_len=512),
                                dict(algo=G.SEMI_GLOBAL, head=G.BOTH, tail=G.BOTH)])
def test_length_sorted_launch(engine, kw):
    # >= 4096 pairs of uneven lengths through the host entry: the wavefront kernels
    # run over pairs sorted by step-axis length (dispatch.hip), results in pair order
    rng = np.random.default_rng(zlib.crc32(repr(kw).encode()) & 0xFFFF)
    qs, ts = helpers.random_pairs(rng, 5000, 1, 200, 1, 300, alphabet=b"ACGTACGTACGTN", related=0.6)
    b = G.Batch.from_pairs(qs, ts)
    tb = kw.get("start_pos") == G.WITH_TB
    check(engine, no_cigar_overflow(b, **kw) if tb else b, cigar=tb, **kw)


def test_local_second_best(engine):
    check(engine, rand_batch(22, 600, 30, 150, 30, 200), algo=G.LOCAL, second_best=1)


def _with_env(name, on):
    if on:
        os.environ.pop(name, None)
    else:
        os.environ[name] = "0"


def test_local16_plan():
    p = lambda **kw: G.make_params(algo=G.LOCAL, second_best=1, **kw)
    assert G.describe_plan(p(), 150, 150) == "local16_second"
    assert G.describe_plan(p(n_penalty=-2), 150, 150) == "local16_second"
    # WITH_START / traceback, bytes outside [0, 255], values past the key window: int32
    assert G.describe_plan(p(start_pos=G.WITH_START), 150, 150) == "generic_local"
    assert G.describe_plan(p(start_pos=G.WITH_TB), 150, 150) == "generic_local"
    assert G.describe_plan(p(match=200, mismatch=60), 150, 150) == "generic_local"
    assert G.describe_plan(p(match=5), 1000, 1000) == "generic_local"


LOCAL16_SCORES = [{}, dict(match=2, mismatch=3, gap_open=5, gap_extend=2),
                  dict(match=3, mismatch=1, gap_open=1, gap_extend=1, n_penalty=2),
                  dict(match=1, mismatch=4, gap_open=6, gap_extend=1, n_penalty=-1),
                  dict(match=2, mismatch=0, gap_open=0, gap_extend=0)]


@pytest.mark.parametrize("config", [2, 4])
@pytest.mark.parametrize("scores", LOCAL16_SCORES)
def test_local16_second_best_configs(engine, config, scores):
    # one tile geometry per batch: every lane carries two pairs; an odd count leaves the
    # last lane one pair.  n_penalty=-1 scores pad cells +1: they lead both maxima
    check(engine, G.Batch.synth(config, 3001, 0x5EED0100 + config), algo=G.LOCAL, second_best=1, **scores)


def test_local16_pads_differ_per_half(engine):
    rng = np.random.default_rng(191)
    qs, ts = [], []
    for _ in range(2000):
        q = helpers.random_seq(rng, int(rng.integers(145, 153)))
        t = (helpers.mutate(rng, q) + helpers.random_seq(rng, 60))[:int(rng.integers(177, 185))]
        qs.append(q); ts.append(t)
    b = G.Batch.from_pairs(qs, ts)
    for kw in ({}, dict(n_penalty=-1), dict(n_penalty=3)):
        check(engine, b, algo=G.LOCAL, second_best=1, **kw)


@pytest.mark.parametrize("n", [4000, 9001])
def test_local16_mixed_geometry(engine, n):
    # n >= 4096 pairs slots of equal geometry by a counting sort; smaller batches decline
    # the second pair of a mismatched lane to the int32 kernel
    check(engine, rand_batch(195 + n, n, 1, 260, 1, 300), algo=G.LOCAL, second_best=1)


def test_local16_n_bases_and_iupac(engine):
    # N inside a target: N tables (packed); N in a query or another letter: the int32 kernel
    rng = np.random.default_rng(197)
    qs, ts = [], []
    for i in range(3000):
        q = bytearray(helpers.random_seq(rng, 150))
        t = bytearray((helpers.mutate(rng, bytes(q)) + helpers.random_seq(rng, 40))[:182])
        if i % 7 == 0:
            q[int(rng.integers(0, 150))] = ord("N")
        if i % 3 == 0:
            for _ in range(3):
                t[int(rng.integers(0, 182))] = ord("N")
        if i % 11 == 0:
            t[int(rng.integers(0, 182))] = b"RYa"[i % 3]
        qs.append(bytes(q)); ts.append(bytes(t))
    b = G.Batch.from_pairs(qs, ts)
    for kw in ({}, dict(n_penalty=3), dict(n_penalty=-2)):
        check(engine, b, algo=G.LOCAL, second_best=1, **kw)


def test_local16_value_window_edge(engine):
    # H up to match * 1,704 = 3,408 (the key limit is 3,455)
    rng = np.random.default_rng(199)
    qs, ts = [], []
    for _ in range(64):
        q = helpers.random_seq(rng, 1700)
        qs.append(q)
        ts.append(helpers.mutate(rng, q, sub=0.005, indel=0.0)[:1704])
    b = G.Batch.from_pairs(qs, ts)
    kw = dict(algo=G.LOCAL, second_best=1, match=2, mismatch=3, gap_open=5, gap_extend=2)
    assert G.describe_plan(G.make_params(**kw), 1700, 1704) == "local16_second"
    check(engine, b, **kw)


def test_local16_equals_int32_kernel(engine):
    b = G.Batch.synth(2, 20000, 0x5EED0002)
    p = G.make_params(algo=G.LOCAL, second_best=1)
    r16 = engine.align_host(b, p)
    try:
        _with_env("GASALX_LOCAL16", False)
        assert G.describe_plan(p, 150, 150) == "generic_local"
        r32 = engine.align_host(b, p)
    finally:
        _with_env("GASALX_LOCAL16", True)
    for f in ("score", "q_end", "t_end", "score2", "q_end2", "t_end2"):
        assert np.array_equal(r16[f], r32[f]), f


# ---------------------------------------------------------------- global ----
@pytest.mark.parametrize("qr,tr", [((1, 30), (1, 30)), ((290, 310), (290, 310)), ((300, 300), (300, 300)),
                                   ((100, 1000), (100, 1000))])
def test_global_random(engine, qr, tr):
    b = rand_batch(31 + qr[0], 600, *qr, *tr)
    check(engine, b, algo=G.GLOBAL)


@pytest.mark.parametrize("qr,tr,tb", [((1490, 1500), (1490, 1500), False), ((1490, 1500), (1490, 1500), True),
                                      ((990, 1000), (1990, 2000), False), ((990, 1000), (1990, 2000), True)])
def test_global_long_reads_thread_per_pair(engine, qr, tr, tb):
    # beyond the wavefront shapes (padded query > 1280) or the exact-int32 range
    # (q + t above ~2.7 kb at 1/4/6/1): the thread-per-pair kernel with the
    # reference's int16 row buffer (global.h:30-303), with and without traceback
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB if tb else G.WITHOUT_START)
    assert G.describe_plan(G.make_params(**kw), qr[1], tr[1]) == "generic_global"
    b = rand_batch(0x610B + qr[0] + tb, 48, *qr, *tr, related=0.8)
    check(engine, no_cigar_overflow(b, **kw) if tb else b, cigar=tb, **kw)


def test_global_int16_row_buffer_wrap(engine):
    # large scores over 3 kb: row-buffer values leave int16 and wrap as in the reference (Q5)
    kw = dict(algo=G.GLOBAL, match=9, mismatch=12, gap_open=20, gap_extend=5)
    assert G.describe_plan(G.make_params(**kw), 3000, 3000) == "generic_global"
    check(engine, rand_batch(0x610C, 16, 2900, 3000, 2900, 3000, related=0.9), **kw)


def test_global_traceback_len_not_mult8(engine):
    rng = np.random.default_rng(32)
    qs, ts = [], []
    while len(qs) < 800:
        q, t = helpers.random_pairs(rng, 1, 20, 310, 20, 310)
        if len(q[0]) % 8 and len(t[0]) % 8:
            qs += q; ts += t
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    check(engine, no_cigar_overflow(G.Batch.from_pairs(qs, ts), **kw), cigar=True, **kw)


def test_global_traceback_any_len(engine):
    # lengths = 0 mod 8 hit SURVEY Q9 (a read past the padded grid, defined as 0 here and in the oracle)
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    check(engine, no_cigar_overflow(rand_batch(33, 600, 8, 64, 8, 64), **kw), cigar=True, **kw)


def test_global_traceback_overflow_counts(engine):
    # Q14 overflow: n_cigar_ops and scores still agree even when slots collide
    b = rand_batch(34, 600, 8, 64, 8, 64)
    check(engine, b, algo=G.GLOBAL, start_pos=G.WITH_TB)


# ----------------------------------------------------------- semi-global ----
@pytest.mark.parametrize("head", [G.NONE, G.QUERY, G.TARGET, G.BOTH])
@pytest.mark.parametrize("tail", [G.NONE, G.QUERY, G.TARGET, G.BOTH])
def test_semiglobal_head_tail(engine, head, tail):
    b = rand_batch(40 + head * 4 + tail, 400, 20, 160, 20, 200)
    check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail)


@pytest.mark.parametrize("head,tail", [(G.TARGET, G.TARGET), (G.BOTH, G.BOTH), (G.NONE, G.QUERY)])
def test_semiglobal_second_best(engine, head, tail):
    b = rand_batch(50 + head, 300, 20, 150, 20, 150)
    check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail, second_best=1, max_query_len=160)


@pytest.mark.parametrize("head,tail", [(G.TARGET, G.TARGET), (G.NONE, G.NONE), (G.QUERY, G.BOTH)])
def test_semiglobal_with_start(engine, head, tail):
    b = rand_batch(60 + head, 300, 20, 150, 20, 150)
    check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail, start_pos=G.WITH_START, max_query_len=160)


@pytest.mark.parametrize("head", [G.NONE, G.QUERY, G.TARGET, G.BOTH])
@pytest.mark.parametrize("alphabet,scores", [(b"ACGT", (1, 4, 6, 1)), (b"ACGTN", (1, 4, 6, 1)),
                                             (b"ACGTRYacgt", (1, 4, 6, 1)),      # declined -> int32 stop kernel
                                             (b"ACGT", (2, 3, 5, 2)), (b"ACGT", (3, 6, 0, 0))])
def test_semiglobal_with_start_wavefront(engine, head, alphabet, scores):
    # TAIL=TARGET WITH_START: reverse pass = the same kernel on reversed slots with the
    # early-exit stop key (start.hpp; semiglobal_kernel_template.h:227-383)
    a, bb, o, e = scores
    kw = dict(algo=G.SEMI_GLOBAL, head=head, tail=G.TARGET, start_pos=G.WITH_START, match=a, mismatch=bb,
              gap_open=o, gap_extend=e, max_query_len=512)
    assert G.describe_plan(G.make_params(**kw), 200, 260).startswith(("wavefront16_semi_start", "wavefront_semi_start"))
    b = rand_batch(zlib.crc32(repr((head, alphabet, scores)).encode()) & 0xFFFF, 1000, 1, 200, 1, 260,
                   alphabet=alphabet, related=0.6)
    check(engine, b, **kw)


@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (2, 3, 5, 2)])
@pytest.mark.parametrize("head", [G.NONE, G.TARGET])
def test_semiglobal_targets_to_192(engine, head, scores):
    # padded targets of 185..192 take the G = 16, R = 12 shape (the few-row wide shapes
    # once disagreed with the oracle with HEAD=NONE, fixed: test_semiglobal_every_packed_shape)
    a, bb, o, e = scores
    kw = dict(algo=G.SEMI_GLOBAL, head=head, tail=G.TARGET, match=a, mismatch=bb, gap_open=o, gap_extend=e,
              max_query_len=512)
    assert G.describe_plan(G.make_params(**kw), 200, 190) == "wavefront16_semi_G16R12"
    b = rand_batch(0x5E32 + 7 * head + a, 1000, 1, 200, 1, 190, related=0.6)
    check(engine, b, **kw)
    check(engine, b, start_pos=G.WITH_START, **kw)


@pytest.mark.parametrize("head", [G.NONE, G.TARGET])
def test_semiglobal_long_targets_wide_groups(engine, head):
    # targets past 320 columns take the G = 32 / 64 packed shapes (R = 20)
    kw = dict(algo=G.SEMI_GLOBAL, head=head, tail=G.TARGET, match=1, mismatch=4, gap_open=6, gap_extend=1,
              max_query_len=512)
    assert G.describe_plan(G.make_params(**kw), 200, 600) == "wavefront16_semi_G32R20"
    b = rand_batch(0x5E31 + head, 600, 1, 200, 330, 600, related=0.6)
    check(engine, b, **kw)
    check(engine, b, start_pos=G.WITH_START, **kw)


def test_semiglobal_with_start_reads_in_windows(engine):
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET, start_pos=G.WITH_START, max_query_len=192)
    check(engine, G.Batch.synth(4, 20000, 0x5EED0004), **kw)
    for n in (1, 7, 33):
        check(engine, rand_batch(500 + n, n, 1, 150, 1, 190), **kw)
    b = rand_batch(510, 500, 10, 150, 10, 150)
    rng = np.random.default_rng(511)
    check(engine, b, q_ops=rng.integers(0, 4, b.n).astype(np.uint8), t_ops=rng.integers(0, 4, b.n).astype(np.uint8),
          **kw)


def test_semiglobal_reads_in_windows(engine):
    b = G.Batch.synth(4, 2000, 0x5EED0004)
    check(engine, b, algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET)


# --------------------------------------------------------- banded / KSW ----
@pytest.mark.parametrize("k_band", [8, 16, 48])
def test_banded(engine, k_band):
    check(engine, rand_batch(70 + k_band, 400, 30, 150, 30, 200), algo=G.BANDED, k_band=k_band)


def _with_band16(on):
    if on:
        os.environ.pop("GASALX_BAND16", None)
    else:
        os.environ["GASALX_BAND16"] = "0"


def test_banded16_plan():
    assert G.describe_plan(G.make_params(algo=G.BANDED, k_band=16), 150, 182).startswith("banded16")
    # N scores > 0 (pads would matter), match + mismatch > 255: the int32 kernel only
    assert G.describe_plan(G.make_params(algo=G.BANDED, k_band=16, n_penalty=-1), 150, 182) == "generic_banded"
    assert G.describe_plan(G.make_params(algo=G.BANDED, k_band=16, match=200, mismatch=60), 150, 182) == \
        "generic_banded"


@pytest.mark.parametrize("k_band", [0, 4, 8, 16, 24, 64, 400])
@pytest.mark.parametrize("scores", [{}, dict(match=2, mismatch=3, gap_open=5, gap_extend=2),
                                    dict(match=3, mismatch=1, gap_open=1, gap_extend=1, n_penalty=2)])
def test_banded16_config4_geometry(engine, k_band, scores):
    # one tile geometry (150 x 182, SURVEY config 4): every lane carries two pairs; an odd
    # count leaves the last lane one pair
    check(engine, G.Batch.synth(4, 3001, 0x5EED0004 + k_band), algo=G.BANDED, k_band=k_band, **scores)


def test_banded16_pads_differ_per_half(engine):
    # same (QR, TR) per lane, different ql / tl inside the last words: each half has its
    # own pad rows and columns
    rng = np.random.default_rng(91)
    qs, ts = [], []
    for _ in range(2000):
        q = helpers.random_seq(rng, int(rng.integers(145, 153)))
        t = (helpers.mutate(rng, q) + helpers.random_seq(rng, 60))[:int(rng.integers(177, 185))]
        qs.append(q); ts.append(t)
    for k_band in (8, 16, 40):
        check(engine, G.Batch.from_pairs(qs, ts), algo=G.BANDED, k_band=k_band)


@pytest.mark.parametrize("n", [4000, 9001])
def test_banded16_mixed_geometry(engine, n):
    # uneven lengths: n >= 4096 pairs slots of equal geometry by a counting sort, smaller
    # batches decline the second pair of a mismatched lane to the int32 kernel
    b = rand_batch(95 + n, n, 20, 260, 20, 300)
    for k_band in (16, 48):
        check(engine, b, algo=G.BANDED, k_band=k_band)


def test_banded16_n_bases_and_iupac(engine):
    # N / other letters inside a sequence take the int32 kernel (per pair); the rest stay packed
    rng = np.random.default_rng(97)
    qs, ts = [], []
    for i in range(3000):
        q = bytearray(helpers.random_seq(rng, 150))
        t = bytearray((helpers.mutate(rng, bytes(q)) + helpers.random_seq(rng, 40))[:182])
        if i % 7 == 0:
            q[int(rng.integers(0, 150))] = ord("N")
        if i % 11 == 0:
            t[int(rng.integers(0, 182))] = b"NRY"[i % 3]
        qs.append(bytes(q)); ts.append(bytes(t))
    b = G.Batch.from_pairs(qs, ts)
    for kw in ({}, dict(n_penalty=3)):
        check(engine, b, algo=G.BANDED, k_band=16, **kw)


def test_banded16_value_window_edge(engine):
    # H up to match * 1,704 = 3,408 (the key limit is 3,455): long identical-ish pairs with
    # match 2, at the top of the packed value window
    rng = np.random.default_rng(99)
    qs, ts = [], []
    for _ in range(64):
        q = helpers.random_seq(rng, 1700)
        qs.append(q)
        ts.append(helpers.mutate(rng, q, sub=0.005, indel=0.0)[:1704])
    b = G.Batch.from_pairs(qs, ts)
    kw = dict(algo=G.BANDED, k_band=64, match=2, mismatch=3, gap_open=5, gap_extend=2)
    assert G.describe_plan(G.make_params(**kw), 1700, 1704).startswith("banded16")
    check(engine, b, **kw)


def test_banded16_equals_int32_kernel(engine):
    # the packed kernel and the reference-shaped int32 kernel on the same batch
    b = G.Batch.synth(4, 20000, 0x5EED0004)
    p = G.make_params(algo=G.BANDED, k_band=16)
    r16 = engine.align_host(b, p)
    try:
        _with_band16(False)
        r32 = engine.align_host(b, p)
    finally:
        _with_band16(True)
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(r16[f], r32[f]), f


def test_ksw(engine):
    b = rand_batch(80, 500, 10, 150, 10, 150)
    seed = np.random.default_rng(81).integers(0, 60, b.n).astype(np.uint32)
    check(engine, b, seed=seed, algo=G.KSW)


@pytest.mark.parametrize("lens,seeds", [((1, 40), (0, 5)), ((8, 8), (0, 30)), ((64, 64), (0, 100)),
                                        ((100, 260), (0, 200)), ((150, 150), (10, 11)),
                                        ((100, 200), (65000, 66000)),    # 16-bit entries overflow: int2 kernel
                                        ((60, 160), (0, 300))])          # mixed 8- and 16-bit levels in one batch
def test_ksw_trimming(engine, lens, seeds):
    # beg/end trimming (ksw_kernel_template.h:181-186) tracked in registers: rows that die
    # early (small seeds), query lengths that are multiples of 8 (the gscore test after the
    # column loop, Q16), unrelated pairs (m == 0 ends a tile early)
    rng = np.random.default_rng(lens[0] * 7 + seeds[1])
    b = rand_batch(int(rng.integers(1 << 16)), 1500, *lens, *lens, related=0.6)
    seed = rng.integers(*seeds, b.n).astype(np.uint32)
    check(engine, b, seed=seed, algo=G.KSW)
    check(engine, b, seed=seed, algo=G.KSW, match=2, mismatch=3, gap_open=5, gap_extend=2)


@pytest.mark.parametrize("kw", [dict(mismatch=-1), dict(mismatch=-2, match=1), dict(n_penalty=-3),
                                dict(mismatch=-1, n_penalty=-2, match=0)])
def test_ksw_gainful_mismatch_and_n(engine, kw):
    # a negative mismatch (or N penalty) is a per-cell gain: the narrow entry levels must size
    # their bound by it, not by the match score alone (h would spill into the e field)
    rng = np.random.default_rng(len(repr(kw)))
    b = rand_batch(int(rng.integers(1 << 16)), 1200, 100, 260, 100, 260, alphabet=b"ACGTACGTN", related=0.5)
    seed = rng.integers(0, 40, b.n).astype(np.uint32)
    check(engine, b, seed=seed, algo=G.KSW, **kw)


@pytest.mark.parametrize("kw", [dict(mismatch=-1), dict(mismatch=-3, match=1), dict(n_penalty=-4),
                                dict(mismatch=-1, n_penalty=-1, match=2)])
def test_local_second_best_gainful_mismatch_and_n(engine, kw):
    # local16_ok's value window counts a negative mismatch / N penalty as the per-cell gain
    b = rand_batch(7000 + len(repr(kw)), 1500, 100, 200, 100, 240, alphabet=b"ACGTACGTN", related=0.5)
    check(engine, b, algo=G.LOCAL, second_best=1, **kw)
    check(engine, G.Batch.synth(2, 4001, 0x5EED0200), algo=G.LOCAL, second_best=1, **kw)


@pytest.mark.parametrize("lds", ["0", "1"])
@pytest.mark.parametrize("lens", [(100, 150), (400, 600), (700, 800)])
def test_ksw_entry_storage(engine, monkeypatch, lds, lens):
    # 8-bit level entries in LDS (block of 256 / 128 / 64 threads by query length; none
    # fits past ~630 bp) or in the global [column][pair] array: both against the oracle
    monkeypatch.setenv("GASALX_KSW_LDS", lds)
    rng = np.random.default_rng(lens[0] + int(lds))
    b = rand_batch(int(rng.integers(1 << 16)), 700, *lens, *lens, related=0.8)
    seed = rng.integers(0, 40, b.n).astype(np.uint32)
    check(engine, b, seed=seed, algo=G.KSW)


# ------------------------------------------------ reverse / complement ----
@pytest.mark.parametrize("algo", [G.LOCAL, G.GLOBAL, G.SEMI_GLOBAL])
def test_reverse_complement_ops(engine, algo):
    b = rand_batch(90 + algo, 500, 10, 150, 10, 150)
    rng = np.random.default_rng(91)
    qo = rng.integers(0, 4, b.n).astype(np.uint8)
    to = rng.integers(0, 4, b.n).astype(np.uint8)
    check(engine, b, q_ops=qo, t_ops=to, algo=algo)


def test_packed_input(engine):
    b = rand_batch(95, 400, 10, 150, 10, 150)
    pq = np.zeros(b.q_bytes // 8, np.uint32)
    pt = np.zeros(b.t_bytes // 8, np.uint32)
    import ctypes
    O.lib().orc_pack(O._ptr(b.q_data), ctypes.c_uint32(b.q_bytes), O._ptr(pq))
    O.lib().orc_pack(O._ptr(b.t_data), ctypes.c_uint32(b.t_bytes), O._ptr(pt))
    bp = G.Batch(pq.view(np.uint8).copy(), b.q_offsets, b.q_lens, pt.view(np.uint8).copy(), b.t_offsets, b.t_lens)
    # the packed buffer is bytes/2 long; lengths/offsets keep the unpacked units (offsets >> 3 = word index)
    bp.q_data = np.concatenate([bp.q_data, np.zeros(b.q_bytes - len(bp.q_data), np.uint8)])
    bp.t_data = np.concatenate([bp.t_data, np.zeros(b.t_bytes - len(bp.t_data), np.uint8)])
    g1 = check(engine, bp, algo=G.LOCAL, is_packed=1)[0]
    g0 = engine.align_host(b, G.make_params(algo=G.LOCAL))
    assert np.array_equal(g0["score"], g1["score"])


@pytest.mark.parametrize("algo,kw", [(G.LOCAL, {}), (G.SEMI_GLOBAL, dict(head=G.TARGET, tail=G.TARGET)),
                                     (G.GLOBAL, {})])
def test_packed_input_pipelined_host_path(engine, algo, kw):
    # isPacked through the two-stream host pipeline (n >= 2 chunks): only the packed half of
    # the pages moves H2D (capi.cpp); outputs equal the ASCII run's and the oracle's
    import ctypes
    b = G.Batch.synth(4 if algo == G.SEMI_GLOBAL else 2, 40000, 0x5EED0002)
    pq = np.zeros(b.q_bytes // 8, np.uint32)
    pt = np.zeros(b.t_bytes // 8, np.uint32)
    O.lib().orc_pack(O._ptr(b.q_data), ctypes.c_uint32(b.q_bytes), O._ptr(pq))
    O.lib().orc_pack(O._ptr(b.t_data), ctypes.c_uint32(b.t_bytes), O._ptr(pt))
    qd = np.zeros(b.q_bytes, np.uint8); qd[:b.q_bytes // 2] = pq.view(np.uint8)
    td = np.zeros(b.t_bytes, np.uint8); td[:b.t_bytes // 2] = pt.view(np.uint8)
    bp = G.Batch(qd, b.q_offsets, b.q_lens, td, b.t_offsets, b.t_lens)
    g1 = engine.align_host(bp, G.make_params(algo=algo, is_packed=1, **kw))
    g0 = engine.align_host(b, G.make_params(algo=algo, **kw))
    o = O.align(b.slice(0, 4000), O.make_params(algo=algo, **kw))
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(g0[f], g1[f]), f
        assert np.array_equal(g1[f][:4000], o[f][:4000]), f


# ----------------------------------------------------- full-size configs ----
def test_plan_is_wavefront_for_bench_configs():
    assert G.describe_plan(G.make_params(algo=G.LOCAL), 150, 150).startswith("wavefront16_local")
    assert G.describe_plan(G.make_params(algo=G.GLOBAL, start_pos=G.WITH_TB), 300, 300).startswith("wavefront16_global_tb")
    assert G.describe_plan(G.make_params(algo=G.SEMI_GLOBAL), 150, 182).startswith("wavefront16_semi")
    assert G.describe_plan(G.make_params(algo=G.GLOBAL), 300, 300).startswith("wavefront16_global")


# ------------------------------------------ packed kernels + int32 fallback ----
@pytest.mark.parametrize("algo,kw", [(G.GLOBAL, {}), (G.SEMI_GLOBAL, dict(head=G.TARGET, tail=G.TARGET)),
                                     (G.SEMI_GLOBAL, dict(head=G.NONE, tail=G.TARGET)),
                                     (G.SEMI_GLOBAL, dict(head=G.QUERY, tail=G.TARGET)),
                                     (G.LOCAL, {})])
@pytest.mark.parametrize("alphabet", [b"ACGT", b"ACGTN", b"ACGTACGTACGTACGTN", b"ACGTRYacgt"])
def test_packed_paths_with_declined_blocks(engine, algo, kw, alphabet):
    # blocks holding a code the packed kernel cannot score are re-aligned by the int32 kernel
    rng = np.random.default_rng(zlib.crc32(repr((algo, alphabet)).encode()) & 0xFFFF)
    qs, ts = helpers.random_pairs(rng, 1500, 1, 180, 1, 200, alphabet=alphabet)
    b = G.Batch.from_pairs(qs, ts)
    check(engine, b, algo=algo, **kw)


@pytest.mark.parametrize("n", [1, 2, 31, 65, 333])
@pytest.mark.parametrize("algo", [G.GLOBAL, G.SEMI_GLOBAL])
def test_packed_odd_batch_sizes(engine, n, algo):
    b = rand_batch(200 + n, n, 1, 190, 1, 190)
    check(engine, b, algo=algo, head=G.TARGET, tail=G.TARGET)


@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (2, 3, 5, 2), (5, 4, 10, 1), (1, 1, 0, 1), (3, 6, 0, 0)])
@pytest.mark.parametrize("algo", [G.GLOBAL, G.SEMI_GLOBAL])
def test_packed_scores(engine, scores, algo):
    a, bb, o, e = scores
    b = rand_batch(300 + a * 7 + bb, 500, 30, 160, 30, 190)
    check(engine, b, algo=algo, head=G.TARGET, tail=G.TARGET, match=a, mismatch=bb, gap_open=o, gap_extend=e)


@pytest.mark.parametrize("algo", [G.LOCAL, G.GLOBAL, G.SEMI_GLOBAL])
def test_packed_with_n_penalty(engine, algo):
    b = rand_batch(400 + algo, 800, 20, 150, 20, 180, alphabet=b"ACGTACGTN")
    check(engine, b, algo=algo, head=G.TARGET, tail=G.TARGET, n_penalty=2)


def test_config2_sample_exact(engine):
    b = G.Batch.synth(2, 40000, 0x5EED0002)
    check(engine, b, algo=G.LOCAL)


@pytest.mark.parametrize("n", [1, 3, 17, 63, 129, 1000])
def test_local_packed_odd_batch_sizes(engine, n):
    # two pairs per lane: odd counts leave a half-empty lane group
    b = rand_batch(100 + n, n, 1, 150, 1, 150)
    check(engine, b, algo=G.LOCAL)


def test_local_packed_mixed_lengths_and_n(engine):
    rng = np.random.default_rng(101)
    qs, ts = helpers.random_pairs(rng, 3000, 1, 200, 1, 250, alphabet=b"ACGTN")
    b = G.Batch.from_pairs(qs, ts)
    assert G.describe_plan(G.make_params(algo=G.LOCAL), int(b.q_lens.max()), int(b.t_lens.max())).startswith(
        "wavefront16")
    check(engine, b, algo=G.LOCAL)


def test_local_packed_vs_int32_paths_agree(engine):
    # match=1 uses the f16-key packed kernel; the same scores scaled by 2 the u16-key one
    b = G.Batch.synth(2, 5000, 7)
    r1 = engine.align_host(b, G.make_params(algo=G.LOCAL))
    r2 = engine.align_host(b, G.make_params(algo=G.LOCAL, match=2, mismatch=8, gap_open=12, gap_extend=2))
    assert np.array_equal(r1["score"] * 2, r2["score"])
    assert np.array_equal(r1["q_end"], r2["q_end"]) and np.array_equal(r1["t_end"], r2["t_end"])


def test_config3_sample_exact(engine):
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    check(engine, no_cigar_overflow(G.Batch.synth(3, 4000, 0x5EED0003), **kw), cigar=True, **kw)


# --------------------------------------------------------------- PairHMM ----
def _hmm_batch(pairs):
    reads = b"".join(p["read"].encode() for p in pairs)
    haps = b"".join(p["hap"].encode() for p in pairs)
    rl = np.array([len(p["read"]) for p in pairs], np.uint32)
    hl = np.array([len(p["hap"]) for p in pairs], np.uint32)
    ro = np.concatenate([[0], np.cumsum(rl)[:-1]]).astype(np.uint32)
    ho = np.concatenate([[0], np.cumsum(hl)[:-1]]).astype(np.uint32)
    bq = np.concatenate([p["bq"] for p in pairs]).astype(np.uint8)
    iq = np.concatenate([p["iq"] for p in pairs]).astype(np.uint8)
    dq = np.concatenate([p["dq"] for p in pairs]).astype(np.uint8)
    qm, de, xi, al = O.pairhmm_params(bq, iq, dq)
    return (np.frombuffer(reads, np.uint8), ro, rl, qm, de, xi, al, np.frombuffer(haps, np.uint8), ho, hl)


def test_pairhmm_reference_datasets(engine):
    d = os.path.join(helpers.GOLDEN, "pairhmm_dataset")
    pairs = [helpers.read_pairhmm_dataset(os.path.join(d, f))[0] for f in sorted(os.listdir(d))]
    args = _hmm_batch(pairs)
    g = engine.pairhmm_host(*args)
    o = O.pairhmm(*args)
    np.testing.assert_allclose(g, o, rtol=1e-5)
    kat = helpers.kat()["pairhmm_32_32"]
    i = sorted(os.listdir(d)).index(kat["file"])
    assert abs(g[i] - kat["result"]) / kat["result"] < 1e-5


def test_pairhmm_random_long(engine):
    rng = np.random.default_rng(5)
    pairs = []
    for _ in range(300):
        H = int(rng.integers(50, 520))
        R = int(rng.integers(20, min(H, 300)))
        hap = helpers.random_seq(rng, H).decode()
        st = int(rng.integers(0, H - R + 1))
        read = bytearray(hap[st:st + R].encode())
        for i in range(R):
            if rng.random() < 0.02:
                read[i] = b"ACGT"[int(rng.integers(0, 4))]
        pairs.append(dict(read=read.decode(), hap=hap, bq=rng.integers(10, 41, R), iq=np.full(R, 45),
                          dq=np.full(R, 45)))
    args = _hmm_batch(pairs)
    np.testing.assert_allclose(engine.pairhmm_host(*args), O.pairhmm(*args), rtol=1e-5)


@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (2, 3, 5, 2), (1, 1, 0, 1), (3, 6, 0, 0)])
@pytest.mark.parametrize("alphabet", [b"ACGT", b"ACGTACGTACGTN", b"ACGTRY"])
def test_packed_global_traceback(engine, scores, alphabet):
    # packed traceback words (and the int32 kernel's for declined blocks) feed the same get_tb walk
    a, bb, o, e = scores
    rng = np.random.default_rng(zlib.crc32(repr((scores, alphabet)).encode()) & 0xFFFF)
    qs, ts = helpers.random_pairs(rng, 700, 20, 310, 20, 310, alphabet=alphabet)
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB, match=a, mismatch=bb, gap_open=o, gap_extend=e)
    check(engine, no_cigar_overflow(G.Batch.from_pairs(qs, ts), **kw), cigar=True, **kw)


@pytest.mark.parametrize("w", ["0", "3", "12", "40"])
@pytest.mark.parametrize("n,lens", [(700, (20, 310, 20, 310)), (5000, (100, 300, 60, 320)), (333, (1, 40, 1, 40))])
def test_global_traceback_band_and_fallback(engine, monkeypatch, w, n, lens):
    # GLOBAL+TB by band recomputation (wavefront16.hpp WF16_GLOBAL_CP / _BAND): paths that leave
    # a lane's window go to the full-matrix fallback; w = 0 sends most pairs there, uneven
    # lengths with n >= 4096 run the length-sorted slots (slot_of in the walk)
    monkeypatch.setenv("GASALX_TB_BAND_W", w)
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    assert "_tbband_" in G.describe_plan(G.make_params(**kw), lens[1], lens[3])
    b = rand_batch(zlib.crc32(repr((w, n)).encode()) & 0xFFFF, n, *lens)
    check(engine, no_cigar_overflow(b, **kw), cigar=True, **kw)


@pytest.mark.parametrize("cap", ["64", "1000"])
@pytest.mark.parametrize("w,alphabet", [("0", b"ACGT"), ("3", b"ACGTACGTACGTNR")])
def test_global_traceback_band_capped_fallback(engine, monkeypatch, cap, w, alphabet):
    """The band path's full-matrix direction buffer holds GASALX_TB_FBCAP slots, not one per pair:
    the fallback list (paths that left the band, and pairs of blocks the packed launch declined,
    whose int32 launch now writes no direction words) runs in chunks of that many list positions,
    each launch reading the device-side count less its offset.  A narrow band sends most pairs
    there; IUPAC codes decline blocks; uneven lengths run sorted slots."""
    monkeypatch.setenv("GASALX_TB_BAND_W", w)
    monkeypatch.setenv("GASALX_TB_FBCAP", cap)
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    assert "_tbband_" in G.describe_plan(G.make_params(**kw), 300, 320)
    b = rand_batch(zlib.crc32(repr((cap, w, alphabet)).encode()) & 0xFFFF, 5000, 100, 300, 60, 320,
                   alphabet=alphabet)
    check(engine, no_cigar_overflow(b, **kw), cigar=True, **kw)


def test_global_traceback_band_equals_full_matrix(engine, monkeypatch):
    # config-3 data: the band pass + walk (+ fallback) and the full-matrix flags kernel agree
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    b = G.Batch.synth(3, 20000, 0x5EED0003)
    g1 = engine.align_host(b, G.make_params(**kw))
    monkeypatch.setenv("GASALX_TB_BAND", "0")
    assert "_tbband_" not in G.describe_plan(G.make_params(**kw), 300, 300)
    g0 = engine.align_host(b, G.make_params(**kw))
    for f in ("score", "n_ops", "cigar"):
        assert np.array_equal(g0[f], g1[f]), f


@pytest.mark.parametrize("scores", [(1, 4, 6, 1), (2, 3, 5, 2), (1, 1, 0, 1), (3, 6, 0, 0), (5, 4, 10, 1)])
@pytest.mark.parametrize("alphabet,npen", [(b"ACGT", None), (b"ACGTACGTACGTN", None), (b"ACGTACGTN", 2),
                                           (b"ACGTRY", None)])
def test_packed_local_traceback(engine, scores, alphabet, npen):
    # packed LOCAL+TB flags (and the int32 kernel's words for declined blocks) feed the
    # LOCAL get_tb walk: CIGAR bytes, n_ops and the start cell it stops at
    a, bb, o, e = scores
    rng = np.random.default_rng(zlib.crc32(repr((scores, alphabet, npen)).encode()) & 0xFFFF)
    qs, ts = helpers.random_pairs(rng, 900, 1, 200, 1, 250, alphabet=alphabet, related=0.6)
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_TB, match=a, mismatch=bb, gap_open=o, gap_extend=e, n_penalty=npen)
    assert G.describe_plan(G.make_params(**kw), 200, 250).startswith("wavefront16_local_tb") or a * 200 > 255
    check(engine, no_cigar_overflow(G.Batch.from_pairs(qs, ts), **kw), cigar=True, **kw)


def test_packed_local_traceback_config2(engine):
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_TB)
    check(engine, no_cigar_overflow(G.Batch.synth(2, 20000, 0x5EED0002), **kw), cigar=True, **kw)


@pytest.mark.parametrize("kw", [dict(algo=G.LOCAL), dict(algo=G.GLOBAL, start_pos=G.WITH_TB),
                                dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET),
                                dict(algo=G.LOCAL, start_pos=G.WITH_TB)])
def test_host_pipeline_chunks(engine, kw):
    # >= 2 x 16384 pairs in the back-to-back layout: gasalx_align_host splits the batch
    # into chunks on two streams (capi.cpp align_host_pipelined); results and CIGARs
    # must land exactly where the single-shot path puts them
    rng = np.random.default_rng(0x919E)
    qs, ts = helpers.random_pairs(rng, 40000, 8, 72, 8, 80, alphabet=b"ACGTACGTACGTN")
    batch = G.Batch.from_pairs(qs, ts)
    tb = kw.get("start_pos") == G.WITH_TB
    if tb:
        batch = no_cigar_overflow(batch, **kw)
    q_ops = rng.integers(0, 4, batch.n).astype(np.uint8) if kw["algo"] == G.LOCAL and not tb else None
    t_ops = rng.integers(0, 4, batch.n).astype(np.uint8) if q_ops is not None else None
    assert batch.n >= 2 * 16384
    check(engine, batch, q_ops=q_ops, t_ops=t_ops, cigar=tb, **kw)


def test_pairhmm_edge_lengths(engine):
    # bottom-aligned read rows (pairhmm.hpp): reads of 1 row, exact multiples of the
    # lane rows, one more / one less, haplotypes shorter than the read, varied quals
    rng = np.random.default_rng(0xE1)
    pairs = []
    for R in (1, 2, 7, 8, 9, 31, 32, 33, 64, 65, 127, 128, 129, 255, 256):
        for H in (1, 2, max(1, R - 1), R, R + 1, 500):
            hap = helpers.random_seq(rng, H).decode()
            read = helpers.random_seq(rng, R).decode() if rng.random() < 0.5 else (hap * (R // H + 1))[:R]
            pairs.append(dict(read=read, hap=hap, bq=rng.integers(0, 60, R), iq=rng.integers(10, 60, R),
                              dq=rng.integers(10, 60, R)))
    args = _hmm_batch(pairs)
    np.testing.assert_allclose(engine.pairhmm_host(*args), O.pairhmm(*args), rtol=1e-5)
    # every lane-group size with the longest read exactly filling the group's rows
    # (boundary select) and one row short of it (the top lane's first row absorbs
    # the boundary, pairhmm.hpp ABS)
    for cap in (256, 255, 129, 128, 127, 64, 63, 33, 32, 31, 9, 8, 7):
        sub = [p for p in pairs if len(p["read"]) <= cap]
        a = _hmm_batch(sub)
        np.testing.assert_allclose(engine.pairhmm_host(*a), O.pairhmm(*a), rtol=1e-5, err_msg=f"reads <= {cap}")


def test_pairhmm_prior_table_vs_compare(engine):
    # pairhmm.hpp: blocks whose bases are all A/C/G/T read the rows' priors from the
    # per-lane LDS table, blocks holding any other byte compare per row.  The same pairs
    # must give the same floats either way: pure A/C/G/T pairs alone (table), then each
    # followed by a pair with N / other bytes (every block compares)
    rng = np.random.default_rng(0xAB1E)
    pure, odd = [], []
    for i in range(96):
        H = int(rng.integers(30, 500)) if i else 500
        R = int(rng.integers(5, min(H, 250))) if i else 250
        hap = helpers.random_seq(rng, H).decode()
        read = helpers.random_seq(rng, R).decode() if i % 3 == 0 else (hap * 2)[:R]
        q = dict(bq=rng.integers(5, 50, R), iq=rng.integers(10, 60, R), dq=rng.integers(10, 60, R))
        pure.append(dict(read=read, hap=hap, **q))
        oh = bytearray(hap.encode())
        orr = bytearray(read.encode())
        for j in rng.integers(0, H, 3):
            oh[j] = b"NacgtX"[int(rng.integers(0, 6))]
        orr[int(rng.integers(0, R))] = ord("N")
        odd.append(dict(read=orr.decode(), hap=oh.decode(), **q))
    mixed = [p for ab in zip(pure, odd) for p in ab]
    a = _hmm_batch(pure)
    gp = engine.pairhmm_host(*a)
    gm = engine.pairhmm_host(*_hmm_batch(mixed))
    assert np.array_equal(gp, gm[0::2])
    np.testing.assert_allclose(gp, O.pairhmm(*a), rtol=1e-5)
    m = _hmm_batch(mixed)
    np.testing.assert_allclose(gm, O.pairhmm(*m), rtol=1e-5)


def test_host_pipeline_pinned_cigar(engine):
    # a caller-owned page-locked CIGAR buffer (bench.py end_to_end "pinned_cigar") must
    # come back byte-identical to the library-allocated one, whatever it held before
    rng = np.random.default_rng(0x919F)
    qs, ts = helpers.random_pairs(rng, 40000, 8, 72, 8, 80)
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_TB)
    batch = no_cigar_overflow(G.Batch.from_pairs(qs, ts), **kw)
    gp = G.make_params(**kw)
    ref = engine.align_host(batch, gp)
    host = G.PinnedHost(batch.q_bytes)
    pinned = host.array
    pinned[:] = 0xFF
    got = engine.align_host(batch, gp, cigar_out=pinned)
    assert got["cigar"] is pinned
    for f in ("score", "q_end", "t_end", "q_start", "t_start", "n_ops", "cigar"):
        assert np.array_equal(got[f], ref[f]), f
    host.close()
    # the handle dropped before the call: the array alone keeps the pinned memory alive
    import gc
    arr = G.PinnedHost(batch.q_bytes).array
    gc.collect()
    got = engine.align_host(batch, gp, cigar_out=arr)
    del arr
    gc.collect()
    assert np.array_equal(got["cigar"], ref["cigar"])


@pytest.mark.parametrize("algo", [G.LOCAL, G.GLOBAL])
def test_host_pipeline_tb_slot_reuse(engine, algo):
    # TB batches are chunked by padded cells (capi.cpp gasalx_align_host): one
    # 448 x 448 pair among 80 K short ones gives 80 K x 448^2 / 5.5 G -> 3 chunks, so
    # slot 0 is drained (results + CIGAR bytes back) before it takes chunk 2
    rng = np.random.default_rng(0x91A0)
    qs, ts = helpers.random_pairs(rng, 80000, 8, 72, 8, 80)
    long_seq = helpers.random_seq(rng, 448, b"ACGT")
    qs[40000], ts[40000] = long_seq, long_seq
    kw = dict(algo=algo, start_pos=G.WITH_TB)
    batch = no_cigar_overflow(G.Batch.from_pairs(qs, ts), **kw)
    mq, mt = int(batch.q_lens.max()), int(batch.t_lens.max())
    assert batch.n * mq * mt / 5.5e9 >= 2.5, (batch.n, mq, mt)
    check(engine, batch, cigar=True, **kw)


# ------------------------------------------------- every packed shape ----
# (G, R) of kShapes16 (dispatch.hip).  GASALX_GMIN forces the minimum G; the
# padded register-axis length G*R then selects exactly that shape.
SHAPES16 = [(8, 8), (8, 12), (8, 16), (8, 19), (8, 20), (8, 23), (16, 10), (16, 12), (16, 16), (16, 20),
            (32, 5), (32, 6), (32, 9), (32, 20), (64, 3), (64, 5), (64, 20)]
SEMI_SCORES = [(1, 4, 6, 1), (2, 3, 5, 2), (3, 5, 4, 3)]   # every set keeps o+e >= b (packed SEMI)


def _forced_g(monkeypatch, g):
    monkeypatch.setenv("GASALX_GMIN", str(g))


def _shape_batch(seed, n, qmax, tmax, fix_q=None, fix_t=None):
    rng = np.random.default_rng(seed)
    qs, ts = helpers.random_pairs(rng, n, 1, qmax, 1, tmax, related=0.6)
    # one pair at the full register-axis length, so the padded maximum selects the shape
    if fix_t:
        ts[0] = (ts[0] * (fix_t // max(1, len(ts[0])) + 1))[:fix_t]
    if fix_q:
        qs[1] = (qs[1] * (fix_q // max(1, len(qs[1])) + 1))[:fix_q]
    return G.Batch.from_pairs(qs, ts)


@pytest.mark.parametrize("g,r", SHAPES16)
def test_semiglobal_every_packed_shape(engine, monkeypatch, g, r):
    """Packed SEMI (registers = target columns) forced onto every (G, R) shape, all
    four HEADs x three score sets, score-only and WITH_START (TAIL=TARGET).  The few-row
    wide shapes once disagreed with the oracle with HEAD=NONE: lane 1's diagonal into
    (row 0, column R) was seeded with the wrong top-boundary value (wavefront16.hpp)."""
    _forced_g(monkeypatch, g)
    tl = g * r
    b = _shape_batch(0x5A00 + g * 31 + r, 300, 200, tl, fix_t=tl)
    for head in (G.NONE, G.QUERY, G.TARGET, G.BOTH):
        for a, bb, o, e in SEMI_SCORES:
            kw = dict(algo=G.SEMI_GLOBAL, head=head, tail=G.TARGET, match=a, mismatch=bb, gap_open=o,
                      gap_extend=e, max_query_len=max(512, tl))
            assert G.describe_plan(G.make_params(**kw), 200, tl) == f"wavefront16_semi_G{g}R{r}"
            check(engine, b, **kw)
            check(engine, b, start_pos=G.WITH_START, **kw)


def test_semiglobal_head_none_entry_at_lane_boundary(engine, monkeypatch):
    """Known answer for the fixed lane-1 seed: with HEAD=NONE the best alignment enters
    row 0 diagonally from the top boundary at column R - 1, cost -(o + e*R) (Q3/Q2
    textbook diagonal, semiglobal_kernel_template.h:123-128).  Query = target[R:R+40]."""
    rng = np.random.default_rng(0x5A11)
    for g, r in [(64, 3), (32, 5), (16, 10), (8, 19)]:
        _forced_g(monkeypatch, g)
        tl = g * r
        t = helpers.random_seq(rng, tl)
        q = t[r:r + 40]
        b = G.Batch.from_pairs([q, q], [t, t])
        kw = dict(algo=G.SEMI_GLOBAL, head=G.NONE, tail=G.TARGET, max_query_len=max(512, tl))
        assert G.describe_plan(G.make_params(**kw), 40, tl) == f"wavefront16_semi_G{g}R{r}"
        g_, o_ = check(engine, b, **kw)
        # 40 matches after a top-boundary diagonal of -(6 + 1*r)
        assert int(o_["score"][0]) == 40 - (6 + r) and int(o_["t_end"][0]) == r + 39


@pytest.mark.parametrize("g,r", SHAPES16)
@pytest.mark.parametrize("algo", [G.LOCAL, G.GLOBAL])
def test_local_global_every_packed_shape(engine, monkeypatch, algo, g, r):
    """LOCAL / GLOBAL packed kernels (registers = query rows) forced onto every shape."""
    _forced_g(monkeypatch, g)
    ql = g * r
    b = _shape_batch(0x5B00 + g * 31 + r + algo, 300, ql, 240, fix_q=ql)
    # LOCAL packs only while a * min(ql, tl) <= 255 (16-bit keys): match 1
    for a, bb, o, e in [(1, 4, 6, 1), (1, 3, 5, 2), (1, 2, 2, 1)]:
        kw = dict(algo=algo, match=a, mismatch=bb, gap_open=o, gap_extend=e)
        plan = G.describe_plan(G.make_params(**kw), ql, 240)
        # (LOCAL: f16 or u16 keys in the e-drift frame, whichever the key range allows)
        assert plan.startswith(f"wavefront16_{'local' if algo == G.LOCAL else 'global'}_") and \
            plan.endswith(f"_G{g}R{r}") and "start" not in plan, plan
        check(engine, b, **kw)


# ------------------------------------------- config 1 and the second oracle ----
def test_config1_through_gpu(engine):
    """BASELINE config 1 (1024 pairs 64x64, seed 0x5EED0001): the batch the CPU verify
    scorer runs (tests/test_independent.py) through the GPU, against both restatements."""
    import independent as I
    b = G.Batch.synth(1, 1024, 0x5EED0001)
    g, o = check(engine, b, algo=G.LOCAL)
    r = I.local(b)
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(g[f], r[f]), f


@pytest.mark.parametrize("head,tail", [(0, 0), (0, 2), (1, 3), (2, 2), (3, 1)])
def test_gpu_against_independent_restatement(engine, head, tail):
    import independent as I
    rng = np.random.default_rng(0x1D + 4 * head + tail)
    qs, ts = helpers.random_pairs(rng, 400, 1, 120, 1, 160, alphabet=b"ACGTN")
    b = G.Batch.from_pairs(qs, ts)
    g = engine.align_host(b, G.make_params(algo=G.SEMI_GLOBAL, head=head, tail=tail))
    r = I.semi(b, head, tail)
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(g[f], r[f]), f
    g = engine.align_host(b, G.make_params(algo=G.LOCAL, second_best=1))
    r = I.local(b, second=True)
    for f in ("score", "q_end", "t_end", "score2", "q_end2", "t_end2"):
        assert np.array_equal(g[f], r[f]), f
    g = engine.align_host(b, G.make_params(algo=G.GLOBAL))
    assert np.array_equal(g["score"], I.global_(b)["score"])


# ------------------------------------- PairHMM from qualities (input files) ----
def _hmm_oracle(d):
    qm, de, xi, al = O.pairhmm_params(d.base_quals, d.ins_quals, d.del_quals)
    return O.pairhmm(d.reads, d.read_offsets, d.read_lens, qm, de, xi, al, d.haps, d.hap_offsets, d.hap_lens)


def _hmm_float(engine, d):
    qm, de, xi, al = d.float_params()
    return engine.pairhmm_host(d.reads, d.read_offsets, d.read_lens, qm, de, xi, al, d.haps, d.hap_offsets,
                               d.hap_lens)


def test_pairhmm_quals_reference_files(engine):
    # every reference dataset file (Intra-task and inter_task synthetic sets) through the
    # native reader and the quality-input kernels; == the float-parameter path bit for bit
    import glob
    files = sorted(glob.glob(os.path.join(helpers.GOLDEN, "pairhmm_dataset", "*.txt")) +
                   glob.glob(os.path.join(helpers.GOLDEN, "pairhmm_inter_dataset", "*.txt")))
    for f in files:
        d = G.read_hmm_file(f)
        g = engine.pairhmm_quals_host(d)
        np.testing.assert_allclose(g, _hmm_oracle(d), rtol=1e-5, err_msg=f)
        assert np.array_equal(g.view(np.uint32), _hmm_float(engine, d).view(np.uint32)), f


def test_pairhmm_quals_sorted_classes_mixed_lengths(engine):
    # reads of 1..512 bases (all five lane-group classes) and haplotypes of 1..700 in
    # random order: sorted by length on the host (tile_1.cu:325), one launch per class,
    # results back in input order
    rng = np.random.default_rng(0x4D32)
    pairs = []
    for _ in range(3000):
        R = int(rng.integers(1, 513))
        H = int(rng.integers(1, 701))
        hap = helpers.random_seq(rng, H).decode()
        read = helpers.random_seq(rng, R).decode() if rng.random() < 0.3 else (hap * (R // H + 1))[:R]
        pairs.append(dict(read=read, hap=hap, bq=rng.integers(0, 256, R), iq=rng.integers(0, 128, R),
                          dq=rng.integers(0, 128, R)))
    d = G.HmmData.from_pairs(pairs)
    g = engine.pairhmm_quals_host(d)
    np.testing.assert_allclose(g, _hmm_oracle(d), rtol=1e-5)
    assert np.array_equal(g.view(np.uint32), _hmm_float(engine, d).view(np.uint32))


def test_pairhmm_prog_driver(tmp_path):
    # the driver binary (tools/pairhmm_prog, C-ABI client): a multi-group file, every
    # result line against the oracle; -fakesize replicates pair 0 as the reference does
    import subprocess
    from test_hmm_io import _rand_pairs, _write_groups
    rng = np.random.default_rng(0x4D33)
    groups = [_rand_pairs(rng, 40), _rand_pairs(rng, 7)]
    path = tmp_path / "in.txt"
    _write_groups(path, groups)
    prog = os.path.join(os.path.dirname(helpers.GOLDEN), "..", "tools", "pairhmm_prog")
    out = subprocess.run([prog, "-print", "all", str(path)], capture_output=True, text=True, check=True).stdout
    vals = [float(l.split()[1]) for l in out.splitlines() if l.startswith("  i=")]
    d = G.read_hmm_file(str(path))
    np.testing.assert_allclose(np.array(vals, np.float32), _hmm_oracle(d), rtol=1e-5)
    assert "GCUPS:" in out
    out = subprocess.run([prog, "-fakesize", "1000", "-print", "last", str(path)], capture_output=True, text=True,
                         check=True).stdout
    lines = [l for l in out.splitlines() if l.startswith("  i=")]
    assert len(lines) == 2 and lines[0].startswith("  i=999")
    np.testing.assert_allclose(float(lines[0].split()[1]), _hmm_oracle(d)[0], rtol=1e-5)


def test_host_pipeline_cigar_overflow_at_chunk_edge(engine):
    """SURVEY Q14 at a chunk boundary of gasalx_align_host's pipeline:
    the last pair of chunk 0 has a CIGAR longer than its slot (1 query base against 600
    target bases: ten 63-capped D runs around one M).  Scores, n_ops and every pair's own
    slot bytes match the oracle (which writes pairs in order); only the residue in the
    neighbour's slot may differ."""
    rng = np.random.default_rng(0x91A1)
    qs, ts = helpers.random_pairs(rng, 44000, 8, 72, 8, 80)
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    # no other overflowing pair (their spill into a neighbour's slot races with the
    # neighbour's own CIGAR on the GPU, in an order the reference leaves undefined too)
    o0 = O.align(G.Batch.from_pairs(qs, ts), O.make_params(**kw))
    keep = [i for i in range(len(qs)) if o0["n_ops"][i] <= (len(qs[i]) + 7) // 8 * 8][:40000]
    qs, ts = [qs[i] for i in keep], [ts[i] for i in keep]
    qs[19999], ts[19999] = b"A", helpers.random_seq(rng, 600, b"C")
    b = G.Batch.from_pairs(qs, ts)
    gp, op = _params_pair(**kw)
    g = engine.align_host(b, gp)
    o = O.align(b, op)
    assert o["n_ops"][19999] > 8
    assert np.array_equal(g["score"], o["score"]) and np.array_equal(g["n_ops"], o["n_ops"])
    slot = (b.q_lens.astype(np.int64) + 7) // 8 * 8
    for k in range(b.n):
        m = int(min(o["n_ops"][k], slot[k]))
        off = int(b.q_offsets[k])
        if not np.array_equal(g["cigar"][off:off + m], o["cigar"][off:off + m]):
            raise AssertionError(f"pair {k}: own-slot CIGAR bytes differ")


# ------------------------------------------ SEMI TAIL = QUERY / BOTH / NONE ----
# semiglobal_kernel_template.h:160-203: TAIL=QUERY reads H at the last padded target
# column (Q11) for every query row, TAIL=BOTH after the last-row maximum, and the end
# rule "t_end = ql unless q_end == tl"; TAIL=NONE writes MINUS_INF and the initial ends.
# The packed kernel (wavefront16.hpp WF16_SEMI_TQ) runs one launch per padded target
# length 8R (dispatch.hip launch_semi_tq), the pad columns scored by the N rule.
TQ_TAILS = [G.QUERY, G.BOTH]


def test_semiglobal_every_head_tail_plan():
    for head in (G.NONE, G.QUERY, G.TARGET, G.BOTH):
        for tail in (G.NONE, G.QUERY, G.TARGET, G.BOTH):
            name = G.describe_plan(G.make_params(algo=G.SEMI_GLOBAL, head=head, tail=tail), 150, 182)
            want = {G.NONE: "semi_tail_none", G.TARGET: "wavefront16_semi_G8R23"}.get(tail, "wavefront16_semi_tq_G8R23")
            assert name == want, (head, tail, name)


@pytest.mark.parametrize("tail", TQ_TAILS)
@pytest.mark.parametrize("head", [G.NONE, G.QUERY, G.TARGET, G.BOTH])
def test_semiglobal_tail_query_config4(engine, head, tail):
    # one class (182 bp windows: 184 padded, R = 23, two pad columns), every score set
    b = G.Batch.synth(4, 3000, 0x5EED0400 + 4 * head + tail)
    for a, bb, o, e in SEMI_SCORES:
        check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail, match=a, mismatch=bb, gap_open=o, gap_extend=e)


@pytest.mark.parametrize("tail", TQ_TAILS)
def test_semiglobal_tail_query_loose_max_t(engine, tail):
    # one padded target length in the batch, but a caller's max_t_len (an upper
    # bound, gasalx.h) above it -- the class launch must be the batch's class, not pad8(max_t)'s,
    # or every pair falls to the int32 kernel; results equal either way, so the packed count is
    # what this checks
    b = G.Batch.synth(4, 6000, 0x5EED0411 + tail)          # 182 bp windows: one class, R = 23
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=tail)
    o = O.align(b, O.make_params(**kw))
    for mt in (0, 184, 200, 256):
        engine.packed_pairs()                                # forget earlier launches
        g = engine.align_host(b, G.make_params(**kw), max_t_len=mt)
        for f in ("score", "q_end", "t_end"):
            assert np.array_equal(g[f], o[f]), (mt, f)
        handled, total = engine.packed_pairs()
        assert total >= b.n and handled == total, (mt, handled, total)


def test_semiglobal_tail_query_pipeline_chunks_of_shorter_targets(engine):
    # the host pipeline's chunks (16,384 pairs and up): chunks 1 and 2 hold only 100 bp
    # targets while the batch's max_t is 182 (capi.cpp per-chunk class check)
    rng = np.random.default_rng(0x0E7A)
    n = 3 * 16384
    qs, ts = [], []
    for i in range(n):
        tl = 182 if i < 16384 else 100
        t = helpers.random_seq(rng, tl)
        ts.append(t)
        qs.append(helpers.mutate(rng, t)[: (150 if tl == 182 else 90)])
    b = G.Batch.from_pairs(qs, ts)
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.QUERY)
    engine.packed_pairs()                                    # forget earlier launches
    g = engine.align_host(b, G.make_params(**kw))
    o = O.align(b, O.make_params(**kw))
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(g[f], o[f]), f
    handled, total = engine.packed_pairs()
    assert total > 0 and handled == total, (handled, total)


@pytest.mark.parametrize("tail", TQ_TAILS)
@pytest.mark.parametrize("head", [G.NONE, G.QUERY, G.TARGET, G.BOTH])
def test_semiglobal_tail_query_classes(engine, head, tail):
    # targets of 1..256 (every class R = 1..32, a length-sorted slot order), queries shorter
    # and longer than their targets (rows past tl: the q_end == tl end rule), 0..7 pad columns
    rng = np.random.default_rng(0x7A11 + 4 * head + tail)
    qs, ts = [], []
    for i in range(2500):
        tl = int(rng.integers(1, 257))
        ql = int(rng.integers(1, min(3 * tl, 400) + 1))
        t = helpers.random_seq(rng, tl)
        q = (helpers.mutate(rng, t * 3)[:ql] if i % 2 else helpers.random_seq(rng, ql))
        qs.append(q); ts.append(t)
    b = G.Batch.from_pairs(qs, ts)
    assert G.describe_plan(G.make_params(algo=G.SEMI_GLOBAL, head=head, tail=tail), 400, 256) == \
        "wavefront16_semi_tq_G8R32"
    check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail)
    check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail, match=2, mismatch=3, gap_open=5, gap_extend=2)


@pytest.mark.parametrize("tail", TQ_TAILS)
@pytest.mark.parametrize("npen", [None, 2, 0])
def test_semiglobal_tail_query_n_and_iupac(engine, tail, npen):
    # N in targets and queries (the N rule, with and without N_PENALTY), other letters:
    # blocks holding them are declined per slot to the int32 kernel
    rng = np.random.default_rng(0x7A20 + tail * 3 + (npen or 0))
    qs, ts = helpers.random_pairs(rng, 2000, 1, 200, 1, 250, alphabet=b"ACGTACGTACGTN")
    qs[7] = qs[7][:3] + b"R" + qs[7][4:]
    b = G.Batch.from_pairs(qs, ts)
    for head in (G.NONE, G.BOTH):
        check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail, n_penalty=npen)


def test_semiglobal_tail_query_ties_and_rows_past_target(engine):
    # a query that repeats the target: the last column's maximum recurs on later rows
    # (first row wins), rows at index tl and beyond, equal target-row and column maxima
    qs, ts = [], []
    for t in (b"ACGTACGTAC", b"ACGTACGT", b"AAAAAAAAAAAAAAAA", b"ACG", b"A"):
        for k in (1, 2, 3, 5):
            qs.append(t * k)
            ts.append(t)
            qs.append((t * k)[1:])
            ts.append(t)
    b = G.Batch.from_pairs(qs, ts)
    for head in (G.NONE, G.QUERY, G.TARGET, G.BOTH):
        for tail in TQ_TAILS:
            check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=tail)


def test_semiglobal_tail_none_outputs(engine):
    b = rand_batch(0x7A30, 777, 1, 300, 1, 300)
    for head in (G.NONE, G.QUERY, G.TARGET, G.BOTH):
        g, _ = check(engine, b, algo=G.SEMI_GLOBAL, head=head, tail=G.NONE)
        assert (g["score"] == -32768).all() and np.array_equal(g["q_end"], b.t_lens.astype(np.int32))


def test_semiglobal_tail_query_equals_int32_kernel(engine, monkeypatch):
    b = G.Batch.synth(4, 20000, 0x5EED0004)
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.BOTH)
    r16 = engine.align_host(b, G.make_params(**kw))
    monkeypatch.setenv("GASALX_PACKED16", "0")
    assert G.describe_plan(G.make_params(**kw), 150, 182).startswith("wavefront_semi")
    r32 = engine.align_host(b, G.make_params(**kw))
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(r16[f], r32[f]), f


@pytest.mark.parametrize("kw", [dict(), dict(match=2, mismatch=3, gap_open=5, gap_extend=2), dict(n_penalty=2)])
def test_ksw16_equals_levels(engine, monkeypatch, kw):
    # two pairs per lane (ksw16.hpp) against the thread-per-pair levels on config-2 data with
    # N in a tenth of the targets (queries with N stay on the levels), odd pair count
    b = G.Batch.synth(2, 20001, 0x5EED0216)
    rng = np.random.default_rng(216)
    for k in rng.choice(b.n, b.n // 10, replace=False):
        o = int(b.t_offsets[k]) + int(rng.integers(0, int(b.t_lens[k])))
        b.t_data[o] = ord("N")
    seed = rng.integers(0, 40, b.n).astype(np.uint32)
    p = G.make_params(algo=G.KSW, **kw)
    r16 = engine.align_host(b, p, seed_scores=seed)
    monkeypatch.setenv("GASALX_KSW16", "0")
    r32 = engine.align_host(b, p, seed_scores=seed)
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(r16[f], r32[f]), f
    o = O.align(b, O.make_params(algo=G.KSW, **kw), seed_scores=seed)
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(r16[f], o[f]), f


# ------------------------------------------------ mixed-shape (tail) launches ----
def _device_align(engine, b, algo):
    """One gasalx_align_device call over the whole batch in HBM (one packed launch: the host
    pipeline would split it into chunks), through torch device buffers."""
    import torch
    dev = torch.device("cuda", 0)
    u = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32) if a.dtype == np.uint32 else a).to(dev)
    d = {"q_batch": u(b.q_data), "t_batch": u(b.t_data), "q_offsets": u(b.q_offsets), "t_offsets": u(b.t_offsets),
         "q_lens": u(b.q_lens), "t_lens": u(b.t_lens)}
    for f in ("aln_score", "q_end", "t_end"):
        d[f] = torch.full((b.n,), -7, dtype=torch.int32, device=dev)
    engine.align_device_ptrs(G.make_params(algo=algo), {k: v.data_ptr() for k, v in d.items()}, b.q_bytes,
                             b.t_bytes, b.n, int(b.q_lens.max()), int(b.t_lens.max()))
    torch.cuda.synchronize()
    return {"score": d["aln_score"].cpu().numpy(), "q_end": d["q_end"].cpu().numpy(),
            "t_end": d["t_end"].cpu().numpy()}


@pytest.mark.parametrize("kind,n,algo", [(2, 120_000, G.LOCAL), (3, 60_000, G.GLOBAL)])
def test_tail_shape_launch(engine, monkeypatch, kind, n, algo):
    """A launch of two or more rounds of packed waves runs its last slots on a shorter shape
    (wavefront16.hpp wf16_mix_kernel; LOCAL G8R19 + G32R5 for config 2, GLOBAL G16R20 + G64R5 for
    300 bp).  Results equal the oracle and the one-shape launch's, and the packed launch takes
    every pair (its two flag ranges counted by gasalx_packed_pairs)."""
    b = G.Batch.synth(kind, n, 0x7A11 + kind)
    o = O.align(b, O.make_params(algo=algo))
    fields = ("score",) if algo == G.GLOBAL else ("score", "q_end", "t_end")
    monkeypatch.setenv("GASALX_TAIL", "1")
    engine.packed_pairs()                                    # forget earlier launches
    g = _device_align(engine, b, algo)
    handled, total = engine.packed_pairs()
    assert handled == total == n
    monkeypatch.setenv("GASALX_TAIL", "0")
    g0 = _device_align(engine, b, algo)
    for f in fields:
        assert np.array_equal(g[f], o[f]), f
        assert np.array_equal(g0[f], o[f]), f


@pytest.mark.parametrize("cp_tail", ["64", "32", "off"])
def test_tail_shape_band_traceback(engine, monkeypatch, cp_tail):
    """NW + CIGAR by band recomputation over more than two rounds of waves in one device call: the
    last slots run the second shape (wf16_mix_kernel<WF16_GLOBAL_CP, 16, 20, 64, 8> or 32 x 12,
    GASALX_CP_TAIL) with their own band buffers, and the walk (tb_kernel) reads each pair's band
    flags with its region's shape.  Scores, CIGAR bytes and n_ops as the oracle; every pair packed."""
    import torch
    n = 60_000
    b = G.Batch.synth(3, n, 0x7A31)
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    o = O.align(b, O.make_params(**kw))
    monkeypatch.setenv("GASALX_TAIL", "0" if cp_tail == "off" else "1")
    if cp_tail != "off":
        monkeypatch.setenv("GASALX_CP_TAIL", cp_tail)
    dev = torch.device("cuda", 0)
    u = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32) if a.dtype == np.uint32 else a).to(dev)
    d = {"q_batch": u(b.q_data), "t_batch": u(b.t_data), "q_offsets": u(b.q_offsets), "t_offsets": u(b.t_offsets),
         "q_lens": u(b.q_lens), "t_lens": u(b.t_lens),
         "aln_score": torch.full((n,), -7, dtype=torch.int32, device=dev),
         "cigar": torch.zeros(b.q_bytes, dtype=torch.uint8, device=dev),
         "n_cigar_ops": torch.zeros(n, dtype=torch.int32, device=dev)}
    engine.packed_pairs()                                    # forget earlier launches
    engine.align_device_ptrs(G.make_params(**kw), {k: v.data_ptr() for k, v in d.items()}, b.q_bytes, b.t_bytes,
                             n, int(b.q_lens.max()), int(b.t_lens.max()))
    torch.cuda.synchronize()
    handled, total = engine.packed_pairs()
    assert handled == total == n, (handled, total)
    assert np.array_equal(d["aln_score"].cpu().numpy(), o["score"])
    nops = d["n_cigar_ops"].cpu().numpy().view(np.uint32)
    assert np.array_equal(nops, o["n_ops"]), int((nops != o["n_ops"]).sum())
    # CIGAR bytes of the pairs whose CIGAR fits its slot (longer ones overwrite the next)
    got, ref = d["cigar"].cpu().numpy(), o["cigar"]
    fits = o["n_ops"] <= (b.q_lens + 7) // 8 * 8
    fits[1:] &= fits[:-1]                                    # and the pair before it did not run over
    for i in np.nonzero(fits)[0][:: max(1, n // 4000)]:
        s, k = int(b.q_offsets[i]), int(o["n_ops"][i])
        assert np.array_equal(got[s:s + k], ref[s:s + k]), i


@pytest.mark.parametrize("k_extra", ["0", "1"])
def test_tail_shape_declined_blocks(engine, monkeypatch, k_extra):
    """IUPAC codes in pairs of both shapes' ranges: their blocks decline to the int32 kernel, which
    reads the mixed launch's two flag ranges (wavefront.hpp skip_flag); every pair exact."""
    n = 120_000
    b = G.Batch.synth(2, n, 0x7A20)
    q = b.q_data.copy()
    picks = [5, 70_000, n - 30_000, n - 5_000, n - 1_000, n - 17, n - 1]
    for i in picks:
        q[int(b.q_offsets[i]) + 3] = ord("R")
    b = G.Batch(q, b.q_offsets, b.q_lens, b.t_data, b.t_offsets, b.t_lens)
    o = O.align(b, O.make_params(algo=O.LOCAL))
    monkeypatch.setenv("GASALX_TAIL", "1")
    monkeypatch.setenv("GASALX_TAIL_K", k_extra)
    engine.packed_pairs()
    g = _device_align(engine, b, G.LOCAL)
    handled, total = engine.packed_pairs()
    assert total == n and n - 64 * len(picks) <= handled < n
    for f in ("score", "q_end", "t_end"):
        assert np.array_equal(g[f], o[f]), f


def test_local_traceback_three_wave_shape(engine, monkeypatch):
    """LOCAL+TB on the 3-wave G16R12 instance (GASALX_LTBD_G16=1, the A/B of VERDICT r05 item 4):
    CIGAR bytes, n_ops, starts and ends as the oracle, config-2 data and ragged pairs."""
    monkeypatch.setenv("GASALX_LTBD_G16", "1")
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_TB)
    assert G.describe_plan(G.make_params(**kw), 150, 150).endswith("_G16R12")
    check(engine, no_cigar_overflow(G.Batch.synth(2, 20000, 0x5EED0002), **kw), cigar=True, **kw)
    rng = np.random.default_rng(0x16C12)
    # (lengths inside the e-drift kernel's f16 key range, (Hmax + 1) * (C + 16) <= 0x7800)
    qs, ts = helpers.random_pairs(rng, 900, 1, 150, 1, 180, alphabet=b"ACGTACGTN", related=0.6)
    check(engine, no_cigar_overflow(G.Batch.from_pairs(qs, ts), **kw), cigar=True, **kw)


def test_local_segments_in_registers(engine, monkeypatch):
    """LOCAL keys by step segments with the finished segments' best per row in registers
    (GASALX_KSEG_REG=1, WF16_LOCAL_SEGR, the A/B of VERDICT r05 item 6) on 300 x 300 pairs,
    including maxima tied across segment boundaries (a later segment wins only when higher)."""
    monkeypatch.setenv("GASALX_KSEG_REG", "1")
    kw = dict(algo=G.LOCAL)
    assert G.describe_plan(G.make_params(**kw), 300, 300) == "wavefront16_local_seg64_G16R20"
    check(engine, G.Batch.synth(3, 30000, 0x5EED0003), **kw)
    rng = np.random.default_rng(0x5E6)
    rep = helpers.random_seq(rng, 50)
    qs, ts = [], []
    for i in range(400):
        qs.append(helpers.random_seq(rng, 20 + i % 40) + rep + helpers.random_seq(rng, 30))
        gap = 10 + (i * 7) % 150
        ts.append(helpers.random_seq(rng, 5 + i % 60) + rep + helpers.random_seq(rng, gap) + rep +
                  helpers.random_seq(rng, 8))
    qs = [q[:300] for q in qs]
    ts = [t[:300] for t in ts]
    check(engine, G.Batch.from_pairs(qs, ts), **kw)
