"""CPU oracle pinned against the reference's known-answer vectors
plus self-consistency properties of the GASAL2 semantics.  No GPU needed."""
import os

import numpy as np
import pytest

import oracle as O
from gasal_ffi import Batch, decode_cigar
import helpers


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def _run(pairs, **kw):
    b = Batch.from_pairs([p[0] for p in pairs], [p[1] for p in pairs])
    return b, O.align(b, O.make_params(**kw))


KAT = helpers.kat()


@pytest.mark.parametrize("idx", range(len(KAT["pairs"])))
def test_kat_local(idx):
    p = KAT["pairs"][idx]
    _, r = _run([(p["q"], p["t"])], algo=O.LOCAL)
    assert (r["score"][0], r["q_end"][0], r["t_end"][0]) == (p["local"]["score"], p["local"]["q_end"], p["local"]["t_end"])


@pytest.mark.parametrize("idx", range(len(KAT["pairs"])))
def test_kat_global(idx):
    p = KAT["pairs"][idx]
    _, r = _run([(p["q"], p["t"])], algo=O.GLOBAL)
    assert r["score"][0] == p["global"]["score"]
    assert r["q_end"][0] == O.SENTINEL   # GLOBAL writes no ends (res.cpp:26-30)


@pytest.mark.parametrize("idx", range(len(KAT["pairs"])))
def test_kat_semiglobal_target_target(idx):
    p = KAT["pairs"][idx]
    _, r = _run([(p["q"], p["t"])], algo=O.SEMI_GLOBAL, head=O.TARGET, tail=O.TARGET)
    e = p["semi_tt"]
    assert (r["score"][0], r["q_end"][0], r["t_end"][0]) == (e["score"], e["q_end"], e["t_end"])


@pytest.mark.parametrize("idx", range(len(KAT["pairs"])))
def test_kat_global_traceback(idx):
    p = KAT["pairs"][idx]
    b, r = _run([(p["q"], p["t"])], algo=O.GLOBAL, start_pos=O.WITH_TB)
    e = p["global_tb"]
    assert r["score"][0] == e["score"]
    assert r["n_ops"][0] == e["n_ops"]
    assert list(r["cigar"][0:e["n_ops"]]) == e["bytes_rev"]


def test_kat_sample_pair_1():
    q, t, _, _ = helpers.read_fasta_pairs(limit=1)
    e = KAT["sample_pair_1_local"]
    _, r = _run([(q[0], t[0])], algo=O.LOCAL)
    assert (r["score"][0], r["q_end"][0], r["t_end"][0]) == (e["score"], e["q_end"], e["t_end"])


def _cigar_score(cig: str, a=1, b=4, o=6, e=1):
    import re
    s = 0
    for n, op in re.findall(r"(\d+)([MXDI])", cig):
        n = int(n)
        if op == "M":
            s += a * n
        elif op == "X":
            s -= b * n
        else:
            s -= o + e * n
    return s


def test_local_tb_cigar_consistent_with_score():
    """2000/2000 local+TB CIGARs imply aln_score.  Same property here
    on the reference's own sample pairs."""
    q, t, _, _ = helpers.read_fasta_pairs(limit=400)
    b = Batch.from_pairs(q, t)
    r = O.align(b, O.make_params(algo=O.LOCAL, start_pos=O.WITH_TB))
    bad = 0
    for k in range(b.n):
        cig = decode_cigar(r["cigar"], int(b.q_offsets[k]), int(r["n_ops"][k]))
        bad += _cigar_score(cig) != r["score"][k]
    assert bad == 0


def test_local_start_matches_traceback_start():
    """The reverse-pass start (WITH_START) and the traceback start agree on
    unambiguous alignments (identical sequences embedded in random flanks)."""
    rng = np.random.default_rng(7)
    qs, ts = [], []
    for _ in range(50):
        core = helpers.random_seq(rng, 40)
        qs.append(helpers.random_seq(rng, 5) + core + helpers.random_seq(rng, 5))
        ts.append(helpers.random_seq(rng, 20) + core + helpers.random_seq(rng, 9))
    b = Batch.from_pairs(qs, ts)
    r1 = O.align(b, O.make_params(algo=O.LOCAL, start_pos=O.WITH_TB))
    assert np.all(r1["score"] >= 40)
    assert np.all(r1["q_start"] <= 5) and np.all(r1["t_start"] <= 20)


def test_q2_leading_query_gap_quirk():
    """Q2: H(r,-1) = -(o+e*r): q=TTACGT t=ACGT scores -3 (textbook -4)."""
    _, r = _run([("TTACGT", "ACGT")], algo=O.GLOBAL)
    assert r["score"][0] == -3


def test_pairhmm_kat_32_32():
    e = KAT["pairhmm_32_32"]
    p = helpers.read_pairhmm_dataset(os.path.join(helpers.GOLDEN, "pairhmm_dataset", e["file"]))[0]
    qm, de, xi, al = O.pairhmm_params(p["bq"], p["iq"], p["dq"])
    read = np.frombuffer(p["read"].encode(), np.uint8)
    hap = np.frombuffer(p["hap"].encode(), np.uint8)
    res = O.pairhmm(read, [0], [len(read)], qm, de, xi, al, hap, [0], [len(hap)])
    assert abs(res[0] - e["result"]) / e["result"] < 1e-6


def test_pairhmm_all_datasets_finite():
    d = os.path.join(helpers.GOLDEN, "pairhmm_dataset")
    for f in sorted(os.listdir(d)):
        p = helpers.read_pairhmm_dataset(os.path.join(d, f))[0]
        qm, de, xi, al = O.pairhmm_params(p["bq"], p["iq"], p["dq"])
        read = np.frombuffer(p["read"].encode(), np.uint8)
        hap = np.frombuffer(p["hap"].encode(), np.uint8)
        res = O.pairhmm(read, [0], [len(read)], qm, de, xi, al, hap, [0], [len(hap)])
        assert np.isfinite(res[0]) and res[0] > 0, f
