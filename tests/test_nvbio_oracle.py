"""CPU checks of the nvbio front-end's oracle (oracle/nvbio_oracle.c), the checker of
the second front-end (include/nvbio_batched.h).  nvbio needs CUDA + thrust, so it
cannot run here: the restatement is pinned by hand-derived known answers (each
worked out below from the recurrences of gotoh/gotoh_inl.h, sw/sw_inl.h and
ed/ed_utils.h) and cross-checked against an independent textbook DP written here
in plain Python (full matrices, no stripes)."""
import numpy as np
import pytest

import gasal_ffi as G
import oracle as O

GOTOH = (2, -1, -2, -1)   # sw-benchmark.cu:587-591


def score(al, p, t):
    P = G.PackedSet.pack([G.dna_n_codes(p)])
    T = G.PackedSet.pack([G.ref2_codes(t)], bits=2, big_endian=False)
    return int(O.nv_score(al, P, T)[0])


def gotoh(type_, p, t, s=GOTOH):
    return score(G.NvAligner(G.NV_GOTOH, type_, *s), p, t)


# Gotoh known answers, scheme (match 2, mismatch -1, gap open -2, gap extend -1): a gap of
# k symbols scores -2 - (k - 1) (F = max(F + Ge, H + Go), gotoh_inl.h:1029-1037)
KATS = [
    # type, pattern, text, expected, derivation
    (G.NV_GLOBAL, "ACGT", "ACGT", 8, "4 matches"),
    (G.NV_GLOBAL, "ACGT", "AGT", 4, "A C- G T: 3 matches (6), one pattern gap (-2)"),
    (G.NV_GLOBAL, "AAAA", "A", -2, "1 match (2), gap of 3 (-4)"),
    (G.NV_GLOBAL, "ACGTTTTACGT", "ACGTACGT", 12, "8 matches (16), gap of 3 (-4)"),
    (G.NV_GLOBAL, "TTACGT", "ACGT", 5, "leading gap of 2 (-3), 4 matches (8): textbook boundary"),
    (G.NV_SEMI_GLOBAL, "CGT", "AACGTAA", 6, "free text ends, 3 matches"),
    (G.NV_SEMI_GLOBAL, "CGTT", "AACGTAA", 5, "CGT + T/A mismatch: 6 - 1"),
    (G.NV_LOCAL, "GGACGTGG", "TTACGTTT", 8, "ACGT, flanks mismatch"),
    (G.NV_LOCAL, "TTTT", "GGGG", 0, "no match: the 0 clamp"),
]


@pytest.mark.parametrize("type_,p,t,expected,why", KATS)
def test_gotoh_known_answers(type_, p, t, expected, why):
    assert gotoh(type_, p, t) == expected, why


def test_sw_and_ed_known_answers():
    sw = G.NvAligner(G.NV_SW, G.NV_GLOBAL, match=1, mismatch=-1, deletion=-1, insertion=-1)
    assert score(sw, "ACGT", "ACT") == 2                     # A C G- T: 3 - 1
    sw_local = G.NvAligner(G.NV_SW, G.NV_LOCAL, match=2, mismatch=-3, deletion=-5, insertion=-5)
    assert score(sw_local, "ACGT", "TTACGTTT") == 8
    ed = lambda t_: G.NvAligner(G.NV_ED, t_)
    assert score(ed(G.NV_GLOBAL), "ACGTACGT", "ACGTTCGT") == -1     # one substitution
    assert score(ed(G.NV_GLOBAL), "ACGT", "ACGTAA") == -2           # two text symbols deleted
    assert score(ed(G.NV_SEMI_GLOBAL), "GTA", "ACGTACG") == 0       # exact substring
    assert score(ed(G.NV_SEMI_GLOBAL), "GTTA", "ACGTACG") == -1     # one insertion
    assert score(ed(G.NV_LOCAL), "ACGT", "TTTT") == 0               # match 0, the 0 clamp


def test_empty_pattern_and_text():
    # M = 0: only the band initialisation reaches the sink (gotoh_inl.h:1188, 1403-1420)
    P0 = G.PackedSet.pack([np.zeros(0, np.uint32)])
    T5 = G.PackedSet.pack([G.ref2_codes("ACGTA")], bits=2, big_endian=False)
    assert int(O.nv_score(G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, *GOTOH), P0, T5)[0]) == -2 - 4
    assert int(O.nv_score(G.NvAligner(G.NV_GOTOH, G.NV_SEMI_GLOBAL, *GOTOH), P0, T5)[0]) == 0
    assert int(O.nv_score(G.NvAligner(G.NV_GOTOH, G.NV_LOCAL, *GOTOH), P0, T5)[0]) == -2 ** 31
    assert int(O.nv_score(G.NvAligner(G.NV_SW, G.NV_GLOBAL, 1, -1, 0, 0, -3, -3), P0, T5)[0]) == -15


# ---- independent textbook DP (full matrices) ----
def textbook(aligner, type_, p, t, s):
    M, N = len(p), len(t)
    NEG = -10 ** 9
    match, mism, go, ge, de, ins = s
    if aligner == G.NV_ED:
        match, mism, de, ins = 0, -1, -1, -1
    H = [[0] * (N + 1) for _ in range(M + 1)]
    E = [[NEG] * (N + 1) for _ in range(M + 1)]
    F = [[NEG] * (N + 1) for _ in range(M + 1)]
    gotoh_ = aligner == G.NV_GOTOH
    for j in range(1, N + 1):   # row -1: text prefix skipped
        H[0][j] = (go + ge * (j - 1) if gotoh_ else de * j) if type_ == G.NV_GLOBAL else 0
    for i in range(1, M + 1):   # column -1: pattern prefix skipped
        H[i][0] = (go + ge * (i - 1) if gotoh_ else ins * i) if type_ != G.NV_LOCAL else 0
    best = -2 ** 31
    for i in range(1, M + 1):
        for j in range(1, N + 1):
            sc = match if p[i - 1] == t[j - 1] else mism
            if gotoh_:
                F[i][j] = max(F[i - 1][j] + ge, H[i - 1][j] + go)
                E[i][j] = max(E[i][j - 1] + ge, H[i][j - 1] + go)
                h = max(E[i][j], F[i][j], H[i - 1][j - 1] + sc)
            else:
                h = max(H[i - 1][j] + ins, H[i][j - 1] + de, H[i - 1][j - 1] + sc)
            if type_ == G.NV_LOCAL:
                h = max(h, 0)
                best = max(best, h)
            H[i][j] = h
    if type_ == G.NV_SEMI_GLOBAL and M and N:
        best = max(H[M][1:])
    if type_ == G.NV_GLOBAL and M and N:
        best = H[M][N]
    return best


@pytest.mark.parametrize("aligner", [G.NV_ED, G.NV_SW, G.NV_GOTOH])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL])
def test_oracle_matches_textbook_dp(aligner, type_):
    rng = np.random.default_rng(1000 * aligner + type_)
    s = (2, -1, -2, -1, -1, -1) if aligner == G.NV_GOTOH else (2, -3, 0, 0, -2, -3)
    for _ in range(60):
        M, N = int(rng.integers(1, 30)), int(rng.integers(1, 40))
        p = list(rng.integers(0, 5, M))       # DNA_N codes incl. N = 4 (never matches the 2-bit text)
        t = list(rng.integers(0, 4, N))
        al = G.NvAligner(aligner, type_, *s)
        P = G.PackedSet.pack([np.array(p, np.uint32)], bits=4)
        T = G.PackedSet.pack([np.array(t, np.uint32)], bits=2, big_endian=False)
        assert int(O.nv_score(al, P, T)[0]) == textbook(aligner, type_, p, t, s)


# ---- known answers the reference's own nvbio test holds (tests/golden/nvbio_reference_kats.json,
#      made by tests/golden/make_nvbio_reference_kats.py from alignment_test.cu:680-793) ----
def _ref_kats():
    import json
    import os
    import helpers
    return json.load(open(os.path.join(helpers.GOLDEN, "nvbio_reference_kats.json")))


def ref_aligner(c):
    t = {"GLOBAL": G.NV_GLOBAL, "LOCAL": G.NV_LOCAL, "SEMI_GLOBAL": G.NV_SEMI_GLOBAL}[c["type"]]
    s = c["scheme"]
    if c["aligner"] == "ed":
        return G.NvAligner(G.NV_ED, t)
    if c["aligner"] == "sw":
        return G.NvAligner(G.NV_SW, t, match=s["match"], mismatch=s["mismatch"], deletion=s["deletion"],
                           insertion=s["insertion"])
    return G.NvAligner(G.NV_GOTOH, t, s["match"], s["mismatch"], s["gap_open"], s["gap_ext"])


def test_reference_alignment_test_cigars():
    # ACAACTA vs AAACACCCTAACACACTAAA (alignment_test.cu:749-793): the optimum each expected
    # CIGAR implies, SW and Gotoh x GLOBAL / LOCAL / SEMI_GLOBAL
    cases = _ref_kats()["alignment"]
    assert len(cases) == 6
    for c in cases:
        assert score(ref_aligner(c), c["pattern"], c["text"]) == c["score"], c


def test_reference_edit_distance_cases():
    # the banded (band 5) SEMI_GLOBAL edit-distance cases of alignment_test.cu:680-745 on the
    # full DP: every stated optimum lies inside the band, so the full DP agrees
    for c in _ref_kats()["edit_distance"]:
        assert score(G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL), c["pattern"], c["text"]) == c["score"], c


# ---- banded front-end (BatchedBandedAlignmentScore<band>, orc_nv_banded_*) ----
INT32_MIN = -(1 << 31)


def banded_textbook(aligner, type_, p, t, band, s):
    """Independent restatement of nvbio's banded DP over full-matrix cells (i, c) with
    0 <= c - i < band (sw_banded_inl.h / gotoh_banded_inl.h, written here as a 2-D
    recurrence): row -1 holds cells c = -1 .. band - 2; a cell's "top" is (i - 1, c)
    (deletion, Gotoh F) when that cell is in the band, its "left" (i, c - 1)
    (insertion, Gotoh E) when c - 1 >= i; text symbols past the end compare as 255."""
    match, mismatch, go, ge, dl, ins = s
    if aligner == G.NV_ED:
        match, mismatch, dl, ins = 0, -1, -1, -1
    M, N, B = len(p), len(t), band
    if N < M:
        return INT32_MIN
    inf = -32768 - max(go, ge)
    H, F = {}, {}
    for c in range(-1, B - 1):
        j = c + 1
        if aligner == G.NV_GOTOH:
            H[(-1, c)] = 0 if j == 0 else (go + (j - 1) * ge if type_ == G.NV_GLOBAL else 0)
        else:
            H[(-1, c)] = j * dl if type_ == G.NV_GLOBAL else 0
        F[(-1, c)] = inf
    best = INT32_MIN
    for i in range(M):
        E = None
        for c in range(i, i + B):
            sym = t[c] if c < N else 255
            diag = H[(i - 1, c - 1)] + (match if sym == p[i] else mismatch)
            has_top, has_left = c - (i - 1) < B, c - 1 >= i
            if aligner == G.NV_GOTOH:
                F[(i, c)] = max(F[(i - 1, c)] + ge, H[(i - 1, c)] + go) if has_top else inf
                cand = [diag, F[(i, c)]] + ([E] if has_left else [])
            else:
                cand = [diag] + ([H[(i - 1, c)] + dl] if has_top else []) + ([H[(i, c - 1)] + ins] if has_left else [])
            h = max(cand)
            if type_ == G.NV_LOCAL:
                h = max(h, 0)
                best = max(best, h)
            H[(i, c)] = h
            if aligner == G.NV_GOTOH:
                E = h + go if E is None else max(h + go, E + ge)
    last = M - 1
    if type_ == G.NV_GLOBAL:
        best = max(best, H[(last, last + B - 1)])
    elif type_ == G.NV_SEMI_GLOBAL:
        m = (min(M + B - 1, N) - (M - 1)) % (1 << 32)
        for j in range(B):
            if j == 0 or j < m:
                best = max(best, H[(last, last + j)])
    return best


def banded_score(al, band, p, t):
    P = G.PackedSet.pack([np.array(p, np.uint32)], bits=4)
    T = G.PackedSet.pack([np.array(t, np.uint32)], bits=2, big_endian=False)
    return int(O.nv_banded_score(al, band, P, T)[0])


def test_reference_banded_edit_distance_cases():
    # alignment_test.cu:680-745: banded_alignment_score<5>(edit distance, SEMI_GLOBAL) against
    # the stated scores, on the banded restatement itself
    for c in _ref_kats()["edit_distance"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        got = int(O.nv_banded_score(G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL), c["band"], P, T)[0])
        assert got == c["score"], c


def test_reference_banded_gotoh_case():
    # alignment_test.cu:790 and :796-826: the band-7 and band-31 Gotoh SEMI_GLOBAL runs whose
    # tracebacks are 4M1D3M and 147M2D3M; their scores are those CIGARs' best in-band
    # placements (make_nvbio_reference_kats.py)
    cases = _ref_kats()["banded"]
    assert [c["band"] for c in cases] == [7, 31]
    for c in cases:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        assert int(O.nv_banded_score(ref_aligner(c), c["band"], P, T)[0]) == c["score"]
    assert cases[0]["score"] == 10


@pytest.mark.parametrize("aligner,s", [(G.NV_GOTOH, (2, -1, -2, -1, 0, 0)), (G.NV_SW, (2, -3, 0, 0, -2, -3)),
                                       (G.NV_ED, (0, 0, 0, 0, 0, 0)), (G.NV_GOTOH, (1, -4, -6, -1, 0, 0)),
                                       (G.NV_SW, (1, 2, 0, 0, 1, -1))])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL])
def test_banded_matches_textbook(aligner, s, type_):
    rng = np.random.default_rng(1000 + 10 * aligner + type_)
    al = G.NvAligner(aligner, type_, *s)
    for band in (2, 3, 5, 7, 8, 13, 32):
        for _ in range(12):
            M = int(rng.integers(0, 24))
            N = max(0, M + int(rng.integers(-2, 3 * band)))
            p = [int(x) for x in rng.integers(0, 4, M)]
            t = [int(x) for x in rng.integers(0, 4, N)]
            for k in range(min(M, N)):
                if rng.random() < 0.7:
                    t[min(N - 1, k + band // 3)] = p[k]
            if N < band - 1:
                continue   # the reference's first-band load reads past such a text (nvbio_oracle.c)
            assert banded_score(al, band, p, t) == banded_textbook(aligner, type_, p, t, band, s), (band, p, t)


def test_banded_short_text_is_skipped():
    al = G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, 2, -1, -2, -1)
    assert banded_score(al, 5, [0, 1, 2, 3], [0, 1, 2]) == INT32_MIN


# ---- BatchedAlignmentTraceback (orc_nv_traceback_*, the checker of nvtrace.hpp) ----
def _replay_score(al, p, t, ops, src, snk):
    """The score of the alignment the pushes describe, walked from the source forwards (the
    TestBacktracker::score idea, alignment_test_utils.h:650-720): Gotoh gaps open once per run."""
    s, j, k, prev = 0, int(src[1]), int(src[0]), None
    for op in ops[::-1]:
        if op == 0:
            s += al.match if p[j] == t[k] else al.mismatch
            j += 1; k += 1
        elif op == 1:
            s += (al.gap_ext if prev == 1 else al.gap_open) if al.aligner == G.NV_GOTOH else al.insertion
            j += 1
        else:
            s += (al.gap_ext if prev == 2 else al.gap_open) if al.aligner == G.NV_GOTOH else al.deletion
            k += 1
        prev = op
    assert (k, j) == (int(snk[0]), int(snk[1]))
    return s


def test_traceback_reference_cigars():
    # alignment_test.cu:778-792: SW and Gotoh x GLOBAL / LOCAL / SEMI_GLOBAL traceback strings
    for c in _ref_kats()["alignment"]:
        al = ref_aligner(c)
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        r = O.nv_traceback(al, P, T)
        assert int(r["score"][0]) == c["score"], c
        got = O.nv_cigar_string(r["ops"][0], len(c["pattern"]), r["source"][0][1], r["sink"][0][1])
        assert got == c["cigar"], (c, got)


@pytest.mark.parametrize("aligner", [G.NV_SW, G.NV_GOTOH], ids=["sw", "gotoh"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_traceback_is_an_optimal_path(aligner, type_):
    # random pairs: the traceback's score is the score-only pass's (a different blocking of the
    # same DP), and its pushes, replayed from the source, reach the sink with that score
    rng = np.random.default_rng(11 + 3 * aligner + type_)
    s = (2, -3, -5, -2) if aligner == G.NV_GOTOH else (2, -1, 0, 0)
    al = (G.NvAligner(G.NV_GOTOH, type_, *s) if aligner == G.NV_GOTOH
          else G.NvAligner(G.NV_SW, type_, match=2, mismatch=-1, deletion=-2, insertion=-2))
    pats, texts = [], []
    for _ in range(300):
        m = int(rng.integers(1, 60))
        p = rng.integers(0, 4, m)
        t = np.concatenate([rng.integers(0, 4, int(rng.integers(0, 12))), p, rng.integers(0, 4, int(rng.integers(0, 12)))])
        t[rng.random(len(t)) < 0.1] = rng.integers(0, 4)
        pats.append(p); texts.append(t)
    P = G.PackedSet.pack(pats, bits=2, big_endian=False)
    T = G.PackedSet.pack(texts, bits=2, big_endian=False)
    r = O.nv_traceback(al, P, T)
    assert list(r["score"]) == list(O.nv_score(al, P, T))
    for k in range(len(pats)):
        assert _replay_score(al, pats[k], texts[k], r["ops"][k], r["source"][k], r["sink"][k]) == r["score"][k], k


def test_traceback_real_problems():
    # alignment_test.cu:828-904: the 144 x 500 Gotoh and edit-distance SEMI_GLOBAL tracebacks
    # (6I138M, 1I1M2I1M3I136M); ED traces back as SW with EditDistanceSWScheme
    cases = _ref_kats()["traceback_real"]
    assert [c["aligner"] for c in cases] == ["gotoh", "ed"]
    for c in cases:
        al = ref_aligner(c)
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        r = O.nv_traceback(al, P, T)
        assert int(r["score"][0]) == c["score"] == int(O.nv_score(al, P, T)[0]), c["cigar"]
        got = O.nv_cigar_string(r["ops"][0], len(c["pattern"]), r["source"][0][1], r["sink"][0][1])
        assert got == c["cigar"], got


# ---- BatchedBandedAlignmentTraceback (orc_nv_banded_traceback_*) ----
def test_banded_traceback_reference_cigars():
    # alignment_test.cu:790-793 (band 7, 4M1D3M) and :796-826 (band 31, 147M2D3M)
    for c in _ref_kats()["banded"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        r = O.nv_banded_traceback(ref_aligner(c), c["band"], P, T)
        assert int(r["score"][0]) == c["score"]
        got = O.nv_cigar_string(r["ops"][0], len(c["pattern"]), r["source"][0][1], r["sink"][0][1])
        assert got == c["cigar"], (c["band"], got)


def _banded_replay(al, band, p, t, ops, src, snk):
    """The score of the pushes replayed from the source (TestBacktracker::score's idea): the
    banded SW scores a pattern-only step (INSERTION) with the deletion penalty and a text-only
    step with the insertion penalty (sw_banded_inl.h:392-475: top + deletion, left + insertion);
    a GLOBAL source at text offset e > 0 starts from row zero's H[e] (sw_banded_inl.h:44-54,
    gotoh_banded_inl.h:48-77); text symbols past the end are nvbio's 255, a mismatch."""
    gotoh = al.aligner == G.NV_GOTOH
    sw = (0, -1, -1, -1) if al.aligner == G.NV_ED else (al.match, al.mismatch, al.deletion, al.insertion)
    match, mismatch = (al.match, al.mismatch) if gotoh else sw[:2]
    e = int(src[0])
    s = 0
    if al.type == G.NV_GLOBAL and e:
        s = al.gap_open + (e - 1) * al.gap_ext if gotoh else e * sw[2]
    j, k, prev = int(src[1]), e, None
    for op in ops[::-1]:
        if op == 0:
            s += match if k < len(t) and p[j] == t[k] else mismatch
            j += 1; k += 1
        elif op == 1:
            s += (al.gap_ext if prev == 1 else al.gap_open) if gotoh else sw[2]
            j += 1
        else:
            s += (al.gap_ext if prev == 2 else al.gap_open) if gotoh else sw[3]
            k += 1
        prev = op
    assert (k, j) == (int(snk[0]), int(snk[1]))
    assert 0 <= k - j < band
    return s


@pytest.mark.parametrize("aligner", [G.NV_ED, G.NV_SW, G.NV_GOTOH], ids=["ed", "sw", "gotoh"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_banded_traceback_is_an_optimal_path(aligner, type_):
    # random pairs and bands: the score is the banded score pass's, and the pushes replayed from
    # the source reach the sink with it -- except the SW LOCAL walk, which nvbio runs past the
    # zero cells to row 0 (the SW submatrix holds no SINK flags, sw_banded_inl.h:268-279, 776)
    rng = np.random.default_rng(77 + 3 * aligner + type_)
    al = (G.NvAligner(G.NV_GOTOH, type_, 2, -3, -5, -2) if aligner == G.NV_GOTOH
          else G.NvAligner(G.NV_SW, type_, match=2, mismatch=-1, deletion=-2, insertion=-3) if aligner == G.NV_SW
          else G.NvAligner(G.NV_ED, type_))
    for band in (2, 3, 7, 8, 16, 31, 32):
        pats, texts = [], []
        for _ in range(40):
            m = int(rng.integers(0, 50))
            p = rng.integers(0, 4, m)
            t = np.concatenate([rng.integers(0, 4, int(rng.integers(0, band))), p,
                                rng.integers(0, 4, int(rng.integers(0, band)))])[: m + int(rng.integers(-2, band + 2))]
            t = t.copy()
            t[rng.random(len(t)) < 0.1] = rng.integers(0, 4)
            pats.append(p); texts.append(t)
        P = G.PackedSet.pack(pats, bits=2, big_endian=False)
        T = G.PackedSet.pack(texts, bits=2, big_endian=False)
        r = O.nv_banded_traceback(al, band, P, T)
        assert list(r["score"]) == list(O.nv_banded_score(al, band, P, T)), band
        for k in range(len(pats)):
            if len(texts[k]) < len(pats[k]):
                assert r["score"][k] == INT32_MIN and list(r["sink"][k]) == [0xFFFFFFFF] * 2 and len(r["ops"][k]) == 0
                continue
            if aligner != G.NV_GOTOH and type_ == G.NV_LOCAL:
                continue
            if r["sink"][k][0] == 0xFFFFFFFF:
                continue
            assert _banded_replay(al, band, pats[k], texts[k], r["ops"][k], r["source"][k], r["sink"][k]) == r["score"][k], (band, k)
