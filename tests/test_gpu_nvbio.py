"""GPU parity of the second front-end (nvbio-style batched scoring, include/nvbio_batched.h
over gasalx_nv_*): the HIP kernels (nvbio.hpp) against the oracle restatement
(oracle/nvbio_oracle.c) on the same packed string sets.  Scores are integers:
bit-exact.  Covers the three aligners x three alignment types, shared and per-pair
texts, 2/4/8-bit packings in both word orders, patterns up to 1024 symbols, the
sw-benchmark driver (tools/sw_benchmark) end to end."""
import os
import subprocess

import numpy as np
import pytest

import gasal_ffi as G
import helpers
import oracle as O

pytestmark = pytest.mark.gpu

ALIGNERS = [G.NvAligner(G.NV_GOTOH, 0, 2, -1, -2, -1), G.NvAligner(G.NV_SW, 0, 2, -3, 0, 0, -2, -3),
            G.NvAligner(G.NV_ED, 0), G.NvAligner(G.NV_GOTOH, 0, 5, -4, -10, -1)]


def _al(base, type_):
    return G.NvAligner(base.aligner, type_, base.match, base.mismatch, base.gap_open, base.gap_ext, base.deletion,
                       base.insertion)


def _related(rng, text, m):
    if len(text) <= m:
        return list(rng.integers(0, 4, m))
    st = int(rng.integers(0, len(text) - m + 1))
    p = list(text[st:st + m])
    for k in range(m):
        if rng.random() < 0.06:
            p[k] = int(rng.integers(0, 5))
    return p


def _check(engine, al, P, T):
    g = engine.nv_score_host(al, P, T)
    o = O.nv_score(al, P, T)
    bad = np.nonzero(g != o)[0]
    assert bad.size == 0, f"{bad.size}/{len(g)} differ, first #{bad[0]}: gpu={g[bad[0]]} oracle={o[bad[0]]} {al}"
    return g


@pytest.mark.parametrize("base", ALIGNERS, ids=["gotoh", "sw", "ed", "gotoh_b"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_shared_text(engine, base, type_):
    # the sw-benchmark layout: every read against one reference (2-bit LE), reads 4-bit BE DNA_N
    rng = np.random.default_rng(7 * base.aligner + type_ + base.match)
    text = list(rng.integers(0, 4, 1500))
    pats = [np.array(_related(rng, text, int(rng.integers(1, 260))), np.uint32) for _ in range(700)]
    P = G.PackedSet.pack(pats, bits=4, big_endian=True)
    T = G.PackedSet.pack([np.array(text, np.uint32)], bits=2, big_endian=False, shared=True)
    _check(engine, _al(base, type_), P, T)


@pytest.mark.parametrize("base", ALIGNERS[:3], ids=["gotoh", "sw", "ed"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_per_pair_texts(engine, base, type_):
    rng = np.random.default_rng(100 + 7 * base.aligner + type_)
    pats, texts = [], []
    for _ in range(900):
        t = list(rng.integers(0, 4, int(rng.integers(1, 400))))
        texts.append(np.array(t, np.uint32))
        pats.append(np.array(_related(rng, t, int(rng.integers(1, 200))), np.uint32))
    P = G.PackedSet.pack(pats, bits=4, big_endian=True)
    T = G.PackedSet.pack(texts, bits=2, big_endian=False)
    _check(engine, _al(base, type_), P, T)


@pytest.mark.parametrize("bits,big", [(2, True), (2, False), (4, False), (8, True), (8, False)])
def test_packings(engine, bits, big):
    rng = np.random.default_rng(bits * 2 + big)
    hi = 4 if bits == 2 else (16 if bits == 4 else 256)
    pats = [rng.integers(0, hi, int(rng.integers(1, 150))).astype(np.uint32) for _ in range(400)]
    texts = [rng.integers(0, hi, int(rng.integers(1, 300))).astype(np.uint32) for _ in range(400)]
    for type_ in (G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL):
        _check(engine, _al(ALIGNERS[0], type_), G.PackedSet.pack(pats, bits, big), G.PackedSet.pack(texts, bits, big))


@pytest.mark.parametrize("m", [8, 64, 65, 96, 97, 128, 129, 152, 153, 192, 193, 256, 257, 320, 321, 512, 513, 1024])
def test_pattern_lengths_every_shape(engine, m):
    # lane-group shapes (8,8) (8,12) (8,16) (8,19) (8,24) (16,16) (16,20) (32,16) (64,16) of
    # batched.hip, at their edges
    rng = np.random.default_rng(m)
    text = list(rng.integers(0, 4, 2200))
    pats = [np.array(_related(rng, text, m - int(rng.integers(0, 3))), np.uint32) for _ in range(96)]
    T = G.PackedSet.pack([np.array(text, np.uint32)], bits=2, big_endian=False, shared=True)
    for type_ in (G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL):
        _check(engine, _al(ALIGNERS[0], type_), G.PackedSet.pack(pats), T)
    assert G.nv_describe_plan(ALIGNERS[0], m, 2200).startswith("nvbio16_gotoh_global_shared_G")


def test_empty_and_positive_scores(engine):
    # empty patterns / texts, and a scheme whose gaps score > 0 (LOCAL pads then masked)
    rng = np.random.default_rng(3)
    pats = [np.zeros(0, np.uint32), rng.integers(0, 4, 5).astype(np.uint32), np.zeros(0, np.uint32),
            rng.integers(0, 4, 30).astype(np.uint32)]
    texts = [rng.integers(0, 4, 9).astype(np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32),
             rng.integers(0, 4, 70).astype(np.uint32)]
    P, T = G.PackedSet.pack(pats, 4), G.PackedSet.pack(texts, 2, False)
    for type_ in (G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL):
        for al in ALIGNERS:
            _check(engine, _al(al, type_), P, T)
        _check(engine, G.NvAligner(G.NV_SW, type_, 1, 2, 0, 0, 1, -1), P, T)
        _check(engine, G.NvAligner(G.NV_GOTOH, type_, 1, -1, 1, 1), P, T)


def test_int16_scores(engine):
    rng = np.random.default_rng(11)
    text = list(rng.integers(0, 4, 900))
    pats = [np.array(_related(rng, text, 150), np.uint32) for _ in range(300)]
    P = G.PackedSet.pack(pats)
    T = G.PackedSet.pack([np.array(text, np.uint32)], 2, False, shared=True)
    al = _al(ALIGNERS[0], G.NV_GLOBAL)
    s32, s16 = engine.nv_score_host(al, P, T, int16=True)
    assert np.array_equal(s16, s32.astype(np.int16))
    assert np.array_equal(s32, O.nv_score(al, P, T))


def test_sw_benchmark_driver(tmp_path):
    # tools/sw_benchmark (client of include/nvbio_batched.h): FASTQ reads against a FASTA
    # reference, every int16 score of every test against the oracle
    rng = np.random.default_rng(0x5B)
    ref = helpers.random_seq(rng, 1200).decode()
    reads = []
    for _ in range(1500):
        m = int(rng.integers(50, 151))
        st = int(rng.integers(0, len(ref) - m))
        r = bytearray(ref[st:st + m].encode())
        for k in range(m):
            if rng.random() < 0.05:
                r[k] = b"ACGTN"[int(rng.integers(0, 5))]
        reads.append(r.decode())
    fq = tmp_path / "reads.fq"
    fq.write_text("".join(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n" for i, s in enumerate(reads)))
    fa = tmp_path / "ref.fa"
    fa.write_text(">ref\n" + "\n".join(ref[i:i + 60] for i in range(0, len(ref), 60)) + "\n")
    out = tmp_path / "scores.tsv"
    prog = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "sw_benchmark")
    r = subprocess.run([prog, "-tests", "gotoh:ed:sw", "-scores", str(out), str(fq), str(fa)], capture_output=True,
                       text=True, check=True)
    assert "GCUPS" in r.stderr
    got = {}
    for line in out.read_text().splitlines():
        test, name, i, v = line.split("\t")
        got.setdefault((test, name), []).append(int(v))
    P = G.PackedSet.pack([G.dna_n_codes(s) for s in reads], 4, True)
    T = G.PackedSet.pack([G.ref2_codes(ref)], 2, False, shared=True)
    cases = {("gotoh", "global"): G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, 2, -1, -2, -1),
             ("gotoh", "semi-global"): G.NvAligner(G.NV_GOTOH, G.NV_SEMI_GLOBAL, 2, -1, -2, -1),
             ("gotoh", "local"): G.NvAligner(G.NV_GOTOH, G.NV_LOCAL, 2, -1, -2, -1),
             ("ed", "semi-global"): G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL),
             ("sw", "local"): G.NvAligner(G.NV_SW, G.NV_LOCAL, 2, -1, 0, 0, -1, -1)}
    for key, al in cases.items():
        assert np.array_equal(np.array(got[key], np.int16), O.nv_score(al, P, T).astype(np.int16)), key


def _with_nv16(on):
    if on:
        os.environ.pop("GASALX_NV16", None)
    else:
        os.environ["GASALX_NV16"] = "0"


def test_packed_plan_conditions():
    # the packed kernel (nvbio16.hpp): one shared 2-bit text, gaps <= 0, LOCAL mismatch <= 0
    g = ALIGNERS[0]
    assert G.nv_describe_plan(g, 150, 1000).startswith("nvbio16_")
    assert G.nv_describe_plan(g, 150, 1000, per_pair_texts=True).startswith("nvbio_")   # tables beyond LDS
    assert G.nv_describe_plan(g, 150, 400, per_pair_texts=True).startswith("nvbio16_gotoh_global_G8R19")
    assert G.nv_describe_plan(g, 150, 1000, text_bits=4).startswith("nvbio_")
    assert G.nv_describe_plan(G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, 1, -1, 1, 1), 150, 1000).startswith("nvbio_")
    assert G.nv_describe_plan(G.NvAligner(G.NV_SW, G.NV_LOCAL, 1, 2, 0, 0, -1, -1), 150, 1000).startswith("nvbio_")
    assert G.nv_describe_plan(G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL), 150, 1000).startswith("nvbio16_ed_semi")


@pytest.mark.parametrize("base", ALIGNERS, ids=["gotoh", "sw", "ed", "gotoh_b"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_packed_equals_int32_mixed_lengths(engine, base, type_):
    # two pairs per lane group with different pattern lengths (each half has its own last
    # row), odd pair counts, N and IUPAC pattern symbols (never match the 2-bit text)
    rng = np.random.default_rng(500 + 7 * base.aligner + type_)
    text = list(rng.integers(0, 4, 700))
    pats = []
    for i in range(1001):
        p = _related(rng, text, int(rng.integers(1, 153)))
        if i % 9 == 0:
            p[int(rng.integers(0, len(p)))] = int(rng.integers(4, 16))
        pats.append(np.array(p, np.uint32))
    P = G.PackedSet.pack(pats, bits=4, big_endian=True)
    T = G.PackedSet.pack([np.array(text, np.uint32)], bits=2, big_endian=False, shared=True)
    al = _al(base, type_)
    g16 = _check(engine, al, P, T)
    try:
        _with_nv16(False)
        g32 = engine.nv_score_host(al, P, T)
    finally:
        _with_nv16(True)
    assert np.array_equal(g16, g32)


@pytest.mark.parametrize("base", ALIGNERS, ids=["gotoh", "sw", "ed", "gotoh_b"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_packed_per_pair_texts_equals_int32(engine, base, type_):
    # per-pair texts of different lengths in the two halves of a lane group (each half's
    # own sink column), empty texts and patterns, odd counts
    rng = np.random.default_rng(900 + 7 * base.aligner + type_)
    pats, texts = [], []
    for i in range(777):
        t = list(rng.integers(0, 4, int(rng.integers(0 if i % 50 == 0 else 1, 380))))
        texts.append(np.array(t, np.uint32))
        m = 0 if i % 61 == 0 else int(rng.integers(1, 140))
        pats.append(np.array(_related(rng, t, m) if t else list(rng.integers(0, 4, m)), np.uint32))
    P = G.PackedSet.pack(pats, bits=4, big_endian=True)
    T = G.PackedSet.pack(texts, bits=2, big_endian=False)
    al = _al(base, type_)
    assert G.nv_describe_plan(al, 140, 380, per_pair_texts=True).startswith("nvbio16_")
    g16 = _check(engine, al, P, T)
    try:
        _with_nv16(False)
        g32 = engine.nv_score_host(al, P, T)
    finally:
        _with_nv16(True)
    assert np.array_equal(g16, g32)


def test_packed_value_window_edge(engine):
    # patterns of 1,024 against one 6,000-symbol text: (M + N + 2) * 2 * mag = 14,052,
    # near the packed kernel's window; GLOBAL reaches about -(N + M)
    rng = np.random.default_rng(4242)
    text = list(rng.integers(0, 4, 6000))
    pats = [np.array(_related(rng, text, 1024 - int(rng.integers(0, 40))), np.uint32) for _ in range(40)]
    P = G.PackedSet.pack(pats)
    T = G.PackedSet.pack([np.array(text, np.uint32)], 2, False, shared=True)
    for type_ in (G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL):
        al = G.NvAligner(G.NV_SW, type_, 1, -1, 0, 0, -1, -1)
        assert G.nv_describe_plan(al, 1024, 6000).startswith("nvbio16_")
        _check(engine, al, P, T)


def test_reference_known_answers(engine):
    # the reference's own nvbio test vectors (alignment_test.cu:680-793, as scores in
    # tests/golden/nvbio_reference_kats.json), through the HIP kernels
    import test_nvbio_oracle as T
    kats = T._ref_kats()
    for c in kats["alignment"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        # one shared text (the sw-benchmark layout), then the same text per pair
        for shared in (True, False):
            Tx = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False, shared=shared)
            assert int(engine.nv_score_host(T.ref_aligner(c), P, Tx)[0]) == c["score"], (c, shared)
    ed = kats["edit_distance"]
    P = G.PackedSet.pack([G.dna_n_codes(c["pattern"]) for c in ed])
    Tx = G.PackedSet.pack([G.ref2_codes(c["text"]) for c in ed], bits=2, big_endian=False)
    got = engine.nv_score_host(G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL), P, Tx)
    assert list(got) == [c["score"] for c in ed]


# ---- BatchedBandedAlignmentScore<band> (gasalx_nv_banded_score_*, nvbanded.hpp) ----
def _check_banded(engine, al, band, P, T):
    g = engine.nv_banded_score_host(al, band, P, T)
    o = O.nv_banded_score(al, band, P, T)
    bad = np.nonzero(g != o)[0]
    assert bad.size == 0, f"band {band}: {bad.size}/{len(g)} differ, first #{bad[0]}: gpu={g[bad[0]]} oracle={o[bad[0]]} {al}"
    return g


@pytest.mark.parametrize("base", ALIGNERS, ids=["gotoh", "sw", "ed", "gotoh_b"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_banded_per_pair_texts(engine, base, type_):
    # reads against windows a few symbols longer (the banded use: a candidate location),
    # every band-length instance (<= 8, <= 16, <= 32) at and inside its edges
    rng = np.random.default_rng(300 + 7 * base.aligner + type_)
    pats, texts = [], []
    for _ in range(1500):
        m = int(rng.integers(0, 200))
        t = list(rng.integers(0, 4, max(0, m + int(rng.integers(-3, 40)))))
        texts.append(np.array(t, np.uint32))
        pats.append(np.array(_related(rng, t, m), np.uint32))
    P = G.PackedSet.pack(pats, bits=4, big_endian=True)
    T = G.PackedSet.pack(texts, bits=2, big_endian=False)
    for band in (2, 5, 7, 8, 9, 16, 17, 31, 32):
        _check_banded(engine, _al(base, type_), band, P, T)


@pytest.mark.parametrize("bits,big", [(2, True), (4, False), (8, True), (8, False)])
def test_banded_packings_and_shared_text(engine, bits, big):
    rng = np.random.default_rng(40 + bits + big)
    hi = 4 if bits == 2 else (16 if bits == 4 else 256)
    pats = [rng.integers(0, hi, int(rng.integers(0, 120))).astype(np.uint32) for _ in range(600)]
    texts = [rng.integers(0, hi, int(rng.integers(0, 160))).astype(np.uint32) for _ in range(600)]
    P, T = G.PackedSet.pack(pats, bits, big), G.PackedSet.pack(texts, bits, big)
    shared = G.PackedSet.pack([rng.integers(0, hi, 300).astype(np.uint32)], bits, big, shared=True)
    for type_ in (G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL):
        for band in (4, 12, 32):
            _check_banded(engine, _al(ALIGNERS[0], type_), band, P, T)
            _check_banded(engine, _al(ALIGNERS[1], type_), band, P, shared)


def test_banded_reference_known_answers(engine):
    # alignment_test.cu:680-745 (band 5 edit distance) and :790 (band 7 Gotoh semi-global)
    import test_nvbio_oracle as TN
    kats = TN._ref_kats()
    for c in kats["edit_distance"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        assert int(engine.nv_banded_score_host(G.NvAligner(G.NV_ED, G.NV_SEMI_GLOBAL), 5, P, T)[0]) == c["score"], c
    for c in kats["banded"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        assert int(engine.nv_banded_score_host(TN.ref_aligner(c), c["band"], P, T)[0]) == c["score"]


@pytest.mark.parametrize("n", [1, 2, 3, 257, 4097])
def test_banded_packed_equals_int32(engine, monkeypatch, n):
    # the two-pairs-per-lane int16 kernel (2-bit texts) against the int32 one and the oracle:
    # odd counts leave the last lane's high half empty; N pattern symbols, empty patterns,
    # texts shorter than the pattern (skipped pairs) and patterns near the 16-bit window
    rng = np.random.default_rng(900 + n)
    pats, texts = [], []
    for k in range(n):
        m = int(rng.integers(0, 1200)) if k % 7 == 3 else int(rng.integers(0, 160))
        t = list(rng.integers(0, 4, max(0, m + int(rng.integers(-4, 36)))))
        p = _related(rng, t, m)
        if k % 5 == 1 and m:
            p[int(rng.integers(0, m))] = 4   # N
        texts.append(np.array(t, np.uint32))
        pats.append(np.array(p, np.uint32))
    P = G.PackedSet.pack(pats, bits=4, big_endian=True)
    T = G.PackedSet.pack(texts, bits=2, big_endian=False)
    for base in ALIGNERS:
        for type_ in (G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL):
            for band in (3, 16, 29):
                al = _al(base, type_)
                g16 = _check_banded(engine, al, band, P, T)
                monkeypatch.setenv("GASALX_NVB16", "0")
                g32 = engine.nv_banded_score_host(al, band, P, T)
                monkeypatch.delenv("GASALX_NVB16")
                assert np.array_equal(g16, g32), (al, band)


def test_banded_rejects_bad_band(engine):
    P = G.PackedSet.pack([np.zeros(4, np.uint32)])
    with pytest.raises(RuntimeError, match="band length"):
        engine.nv_banded_score_host(ALIGNERS[0], 33, P, P)
    with pytest.raises(RuntimeError, match="band length"):
        engine.nv_banded_score_host(ALIGNERS[0], 1, P, P)


# ---- BatchedAlignmentTraceback (gasalx_nv_traceback_*, nvtrace.hpp) ----
def _check_traceback(engine, al, P, T):
    g = engine.nv_traceback_host(al, P, T)
    o = O.nv_traceback(al, P, T)
    assert np.array_equal(g["score"], o["score"]), al
    assert np.array_equal(g["source"], o["source"]) and np.array_equal(g["sink"], o["sink"]), al
    bad = [k for k in range(len(g["ops"])) if not np.array_equal(g["ops"][k], o["ops"][k])]
    assert not bad, f"{len(bad)} pairs' pushes differ, first #{bad[0]} {al}"
    return g


def test_traceback_reference_cigars(engine):
    # alignment_test.cu:778-792 through the HIP kernel: the reference's CIGAR strings
    import test_nvbio_oracle as T
    for c in T._ref_kats()["alignment"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        for shared in (True, False):
            Tx = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False, shared=shared)
            g = _check_traceback(engine, T.ref_aligner(c), P, Tx)
            assert int(g["score"][0]) == c["score"]
            assert O.nv_cigar_string(g["ops"][0], len(c["pattern"]), g["source"][0][1], g["sink"][0][1]) == c["cigar"]


@pytest.mark.parametrize("aligner", [G.NV_SW, G.NV_GOTOH], ids=["sw", "gotoh"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_traceback_random_pairs(engine, aligner, type_):
    # reads against windows around them (edits, flanks), per-pair texts and one shared text,
    # 4-bit big-endian patterns and 2-bit texts as sw-benchmark packs them; lengths 1..150
    rng = np.random.default_rng(500 + 3 * aligner + type_)
    al = (G.NvAligner(G.NV_GOTOH, type_, 2, -1, -2, -1) if aligner == G.NV_GOTOH
          else G.NvAligner(G.NV_SW, type_, match=2, mismatch=-1, deletion=-1, insertion=-1))
    pats, texts = [], []
    for _ in range(2000):
        m = int(rng.integers(1, 151))
        p = rng.integers(0, 4, m)
        t = np.concatenate([rng.integers(0, 4, int(rng.integers(0, 20))), p, rng.integers(0, 4, int(rng.integers(0, 20)))])
        t[rng.random(len(t)) < 0.05] = rng.integers(0, 4)
        pats.append(p); texts.append(t)
    P = G.PackedSet.pack(pats)
    _check_traceback(engine, al, P, G.PackedSet.pack(texts, bits=2, big_endian=False))
    _check_traceback(engine, al, P, G.PackedSet.pack([texts[0]], bits=2, big_endian=False, shared=True))


def test_traceback_rejects(engine):
    # scores beyond nvbio's int16 columns are refused
    P = G.PackedSet.pack([np.zeros(10, np.uint32)])
    T = G.PackedSet.pack([np.zeros(10, np.uint32)], bits=2, big_endian=False)
    with pytest.raises(Exception):
        engine.nv_traceback_host(G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, 2000, -1, -2, -1), P, T)


def test_traceback_real_problems(engine):
    # alignment_test.cu:828-904 through the HIP kernel: 6I138M (Gotoh) and 1I1M2I1M3I136M (ED)
    import test_nvbio_oracle as TN
    for c in TN._ref_kats()["traceback_real"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False)
        g = _check_traceback(engine, TN.ref_aligner(c), P, T)
        assert int(g["score"][0]) == c["score"]
        assert O.nv_cigar_string(g["ops"][0], len(c["pattern"]), g["source"][0][1], g["sink"][0][1]) == c["cigar"]


@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_traceback_edit_distance(engine, type_):
    # ED traces back as SW with EditDistanceSWScheme (ed/ed_inl.h:347-365)
    rng = np.random.default_rng(640 + type_)
    pats, texts = [], []
    for _ in range(1000):
        m = int(rng.integers(1, 120))
        p = rng.integers(0, 4, m)
        t = np.concatenate([rng.integers(0, 4, int(rng.integers(0, 16))), p, rng.integers(0, 4, int(rng.integers(0, 16)))])
        t[rng.random(len(t)) < 0.05] = rng.integers(0, 4)
        pats.append(p); texts.append(t)
    _check_traceback(engine, G.NvAligner(G.NV_ED, type_), G.PackedSet.pack(pats),
                     G.PackedSet.pack(texts, bits=2, big_endian=False))


# ---- BatchedBandedAlignmentTraceback (gasalx_nv_banded_traceback_*, nvtrace.hpp) ----
def _check_banded_traceback(engine, al, band, P, T):
    g = engine.nv_banded_traceback_host(al, band, P, T)
    o = O.nv_banded_traceback(al, band, P, T)
    assert np.array_equal(g["score"], o["score"]), (al, band)
    assert np.array_equal(g["source"], o["source"]) and np.array_equal(g["sink"], o["sink"]), (al, band)
    bad = [k for k in range(len(g["ops"])) if not np.array_equal(g["ops"][k], o["ops"][k])]
    assert not bad, f"{len(bad)} pairs' pushes differ, first #{bad[0]} {al} band {band}"
    return g


def test_banded_traceback_reference_cigars(engine):
    # alignment_test.cu:790-793 (band 7, 4M1D3M) and :796-826 (band 31, 147M2D3M)
    import test_nvbio_oracle as TN
    for c in TN._ref_kats()["banded"]:
        P = G.PackedSet.pack([G.dna_n_codes(c["pattern"])])
        for shared in (True, False):
            T = G.PackedSet.pack([G.ref2_codes(c["text"])], bits=2, big_endian=False, shared=shared)
            g = _check_banded_traceback(engine, TN.ref_aligner(c), c["band"], P, T)
            assert int(g["score"][0]) == c["score"]
            got = O.nv_cigar_string(g["ops"][0], len(c["pattern"]), g["source"][0][1], g["sink"][0][1])
            assert got == c["cigar"], got


@pytest.mark.parametrize("aligner", [G.NV_ED, G.NV_SW, G.NV_GOTOH], ids=["ed", "sw", "gotoh"])
@pytest.mark.parametrize("type_", [G.NV_GLOBAL, G.NV_LOCAL, G.NV_SEMI_GLOBAL], ids=["global", "local", "semi"])
def test_banded_traceback_random_pairs(engine, aligner, type_):
    # reads against windows a little longer than them, every band class (8 / 16 / 32 registers)
    # and band lengths inside each; texts shorter than the pattern (skipped), empty patterns, N
    # pattern symbols; per-pair texts and one shared text
    rng = np.random.default_rng(720 + 3 * aligner + type_)
    al = (G.NvAligner(G.NV_GOTOH, type_, 2, -3, -5, -2) if aligner == G.NV_GOTOH
          else G.NvAligner(G.NV_SW, type_, match=2, mismatch=-1, deletion=-2, insertion=-3) if aligner == G.NV_SW
          else G.NvAligner(G.NV_ED, type_))
    for band in (2, 3, 7, 8, 9, 15, 16, 17, 31, 32):
        pats, texts = [], []
        for k in range(600):
            m = int(rng.integers(0, 160))
            p = rng.integers(0, 4, m).astype(np.uint32)
            t = np.concatenate([rng.integers(0, 4, int(rng.integers(0, band))), p,
                                rng.integers(0, 4, band)])[: max(0, m + int(rng.integers(-2, band + 2)))].copy()
            t[rng.random(len(t)) < 0.06] = rng.integers(0, 4)
            if k % 9 == 4 and m:
                p[int(rng.integers(0, m))] = 4   # N
            pats.append(p); texts.append(t)
        P = G.PackedSet.pack(pats, bits=4, big_endian=True)
        _check_banded_traceback(engine, al, band, P, G.PackedSet.pack(texts, bits=2, big_endian=False))
        if band in (7, 31):
            _check_banded_traceback(engine, al, band, P, G.PackedSet.pack([texts[1]], bits=2, big_endian=False, shared=True))


def test_traceback_cpp_client():
    # tools/nvbio_traceback_test: BatchedAlignmentTraceback and BatchedBandedAlignmentTraceback of
    # include/nvbio_batched.h from C++, replayed into a backtracker, against the strings
    # alignment_test.cu asserts (:778-793, :825, :867, :903)
    prog = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "nvbio_traceback_test")
    r = subprocess.run([prog], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" ok") == 10, r.stdout


def test_banded_traceback_rejects(engine):
    P = G.PackedSet.pack([np.zeros(10, np.uint32)])
    T = G.PackedSet.pack([np.zeros(12, np.uint32)], bits=2, big_endian=False)
    al = G.NvAligner(G.NV_GOTOH, G.NV_SEMI_GLOBAL, 2, -1, -2, -1)
    for band in (1, 33):
        with pytest.raises(RuntimeError, match="band length"):
            engine.nv_banded_traceback_host(al, band, P, T)
    with pytest.raises(Exception):
        engine.nv_banded_traceback_host(G.NvAligner(G.NV_GOTOH, G.NV_GLOBAL, 3000, -1, -2, -1), 8, P, T)
