"""The C oracle against a second, independent numpy restatement of the reference
kernels (tests/independent.py) — CPU only.  Breaks the blind spot of the oracle and
the engine's thread-per-pair kernels sharing one reading of the reference: the two
restatements here differ in form (pair-vectorised numpy vs per-pair C).

Config 1 of BASELINE.json (1024 pairs, 64x64, seed 0x5EED0001, the repo's
host-side CPU verify scorer) runs here as the CPU plumbing case."""
import numpy as np
import pytest

import gasal_ffi as G
import helpers
import independent as I
import oracle as O


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def _same(r, o, fields):
    for f in fields:
        bad = np.flatnonzero(r[f] != o[f])
        assert bad.size == 0, f"{f}: {bad.size} mismatches, first #{bad[0]}: numpy={r[f][bad[0]]} oracle={o[f][bad[0]]}"


def test_config1_cpu_plumbing():
    b = G.Batch.synth(1, 1024, 0x5EED0001)
    assert b.n == 1024 and set(b.q_lens) == {64} and set(b.t_lens) == {64}
    o = O.align(b, O.make_params(algo=O.LOCAL), n_threads=1)
    _same(I.local(b), o, ("score", "q_end", "t_end"))
    # related pairs (5% subs, 1% indels) align with high scores
    assert np.median(o["score"]) > 30


SCORES = [(1, 4, 6, 1), (2, 3, 5, 2), (3, 6, 0, 0)]


def _batch(seed, n=300, alphabet=b"ACGT"):
    rng = np.random.default_rng(seed)
    qs, ts = helpers.random_pairs(rng, n, 1, 70, 1, 90, alphabet=alphabet)
    return G.Batch.from_pairs(qs, ts)


@pytest.mark.parametrize("sc", SCORES)
@pytest.mark.parametrize("alphabet", [b"ACGT", b"ACGTN"])
def test_local_and_second_best(sc, alphabet):
    a, bb, o, e = sc
    b = _batch(11 + a, alphabet=alphabet)
    ref = O.align(b, O.make_params(algo=O.LOCAL, match=a, mismatch=bb, gap_open=o, gap_extend=e, second_best=1))
    _same(I.local(b, a, bb, o, e, second=True), ref, ("score", "q_end", "t_end", "score2", "q_end2", "t_end2"))


@pytest.mark.parametrize("sc", SCORES)
def test_global(sc):
    a, bb, o, e = sc
    b = _batch(21 + a, alphabet=b"ACGTN")
    ref = O.align(b, O.make_params(algo=O.GLOBAL, match=a, mismatch=bb, gap_open=o, gap_extend=e))
    _same(I.global_(b, a, bb, o, e), ref, ("score",))


def test_n_penalty():
    b = _batch(31, alphabet=b"ACGTN")
    for algo, fn, fields in ((O.LOCAL, I.local, ("score", "q_end", "t_end")), (O.GLOBAL, I.global_, ("score",))):
        ref = O.align(b, O.make_params(algo=algo, n_penalty=2))
        _same(fn(b, npen=2), ref, fields)


@pytest.mark.parametrize("head", [0, 1, 2, 3])
@pytest.mark.parametrize("tail", [0, 1, 2, 3])
def test_semiglobal(head, tail):
    b = _batch(41 + 4 * head + tail, n=200, alphabet=b"ACGTN")
    for a, bb, o, e in SCORES[:2]:
        ref = O.align(b, O.make_params(algo=O.SEMI_GLOBAL, head=head, tail=tail, match=a, mismatch=bb, gap_open=o,
                                       gap_extend=e))
        _same(I.semi(b, head, tail, a, bb, o, e), ref, ("score", "q_end", "t_end"))


def test_row_buffer_int16_wrap():
    # the inter-strip row buffer is short2; a long global alignment whose
    # left-boundary values fall below -32768 wraps there, in both restatements
    rng = np.random.default_rng(7)
    q = helpers.random_seq(rng, 40)
    t = helpers.random_seq(rng, 40)
    b = G.Batch.from_pairs([q], [t])
    ref = O.align(b, O.make_params(algo=O.GLOBAL, gap_open=2000, gap_extend=900))
    _same(I.global_(b, 1, 4, 2000, 900), ref, ("score",))
