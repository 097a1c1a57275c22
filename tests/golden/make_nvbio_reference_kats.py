#!/usr/bin/env python3
"""Build tests/golden/nvbio_reference_kats.json: known answers that the reference's own
nvbio unit test holds (NvB/nvbio-test/alignment_test.cu), restated as scores.

* :749-793 aligns pattern ACAACTA against text AAACACCCTAACACACTAAA with
  Smith-Waterman (match 2, mismatch -1, deletion -1, insertion -1) and Gotoh (match 2,
  mismatch -1, gap open -1, gap extend -1), GLOBAL / LOCAL / SEMI_GLOBAL, and asserts the
  traceback's CIGAR string and that its score equals the optimum (:258-281).  The CIGAR is
  printed in the order TestBacktracker pushed the ops, sink to source
  (alignment_test_utils.h:640-643, rle :76-99), and scored source to sink by reading it
  backwards (:654-658).  The optimum each CIGAR implies is therefore the best score of the
  reversed op string over its placements in the text (the traceback's placement is one of
  them and is optimal; no placement can beat the optimum).
* :790 runs the banded (band 7) Gotoh SEMI_GLOBAL case of the same strings and asserts the
  banded traceback's CIGAR 4M1D3M and that its score equals ref_banded_sw's (:296-356): the
  banded optimum is the best score of that op string over the placements whose cells all
  lie inside the band (cell (i, c) in the band when 0 <= c - i < 7).
* :796-826 runs the banded (band 31) Gotoh SEMI_GLOBAL traceback of a 150-symbol read against
  a 181-symbol window (match 0, mismatch -5, gap open -8, gap extend -3) and asserts 147M2D3M;
  :828-868 the full-DP Gotoh SEMI_GLOBAL traceback of a 144-symbol read against a 500-symbol
  text (same scheme), 6I138M; :870-904 the full-DP edit-distance SEMI_GLOBAL traceback of the
  same strings, 1I1M2I1M3I136M.  Their scores are implied the same way.
* :680-745 holds banded (band 5) SEMI_GLOBAL edit-distance cases with stated scores.
  They are kept with the band; the test asserts them against the full-DP front-end where
  the full DP computes the same value (every case here: each optimum lies inside the band).

Data only: this script derives numbers from strings quoted from those lines; it does not
read or run the reference."""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nvbio_reference_kats.json")

PATTERN, TEXT = "ACAACTA", "AAACACCCTAACACACTAAA"          # alignment_test.cu:756-757
CIGARS = {"GLOBAL": "1M2D3M1D3M10D", "LOCAL": "4M1D3M", "SEMI_GLOBAL": "4M1D3M"}   # :771-773, :783-785
SCHEMES = {
    "sw": dict(match=2, mismatch=-1, deletion=-1, insertion=-1),           # :764-768
    "gotoh": dict(match=2, mismatch=-1, gap_open=-1, gap_ext=-1),          # :776-780
}
REAL_GOTOH = dict(match=0, mismatch=-5, gap_open=-8, gap_ext=-3)      # :813-817, :853-857
ED_SCHEME = dict(match=0, mismatch=-1, deletion=-1, insertion=-1)      # ed_utils.h:45-52
BANDED_READ = ("TTATGTAGGTGGTCTGGTTTTTGCCTTTTAAGCTTCTGCAAAAAACAACAACAAACTTGTGGTATTACACTGACTCTACAG"
               "ATCAATTTGGGGACAACTTCCATGTGTTCCACCACCAATACTGAATCTTTCAATCGACTGACGTGGTAT")    # :810
BANDED_WINDOW = ("ATCGGATTCTTTCTTACTTGTAGGTGGTCTGGTTTTTGCCTTTTAAGCTTCTGCAAAAAACAACAACAAACTTGTGGTATTA"
                 "CACTGACTCTACAGATCAATTTGGGGACAACTTCCATGTGTTCCACCACCAATACTGAATCTTTCAATCGACTGACGTGGT"
                 "ATCTCTCTCTCCATCTAT")                                                           # :811
FULL_READ = ("TAGGAGGTAACATGTATGGAGCATTTACCATAGGCCAAGCACTGTTCTAAGAACTTCGGACATGTTATCTCACTTGTATAAG"
             "TACTTAGGTGCCTACAACATAAGCAGCACCTGGTAAATTAAGTATTGAAAAAATGCAGATCG")          # :842-843
FULL_TEXT = ("CAGCACTGACCGGTGAGCATAAACCCTGGGGATGCCCAGAGCTGGTACAGCCAGGAGCTCCAGAAGCGTGGGATTCTCAGAG"
             "GGAAGTGGAGCTCACTGCTCTACAGGTCCTATTCAAGTTAGAAAGTAAGATACAATGCACACAAAGCCAAATTGTC"
             "ATCATTCAGCTCCTATTACAGGGGAACTAAGAGCTGCATTGAAAATTATTTGCAAAGCTTGTAAGTGGTTCTGCCACTTAT"
             "TAGCCGTGTGAACCTTAGCAAATTACCTAGCGTCTCTGAGTTTCAACTTCCTCATCTACAAAATAGAAATGATAATAAT"
             "AACCGCATCGCAAGAGTTGTTGGAAAAATGAAAATGAGGTATCATAGGAGGTAACATGTATGGAGCATTTACCATAGGCC"
             "AAGCACTGTTCTAAGAACTTCGGACATGTTATCTCACTTGTATAAGTACTTAGGTGCCTACAACATAAACAGCACCTGGT"
             "AAATTAAGTATTGAAAAAATGC")                                                       # :844-848
ED_CASES = [   # (test id, pattern, text, expected score): alignment_test.cu:680-745
    (1, "GGGTGCTCAA", "AAAAGGGTGCTCAA", 0),
    (2, "GGGTAAGCTC", "AAAAGGGTGCTCAA", -2),
    (3, "AAGGGTGCTC", "AAAAGGGTGCAATC", -2),
    (4, "AAAAGGGTGC", "AAAAGGGTGCTCAA", 0),
    (5, "AAAAGGGTG", "AAAAGGAAGTGCTC", -2),
    (6, "CACCGGGT", "AACAGGGTGCTC", -2),
]


def ops_of(cigar):
    out, num = [], ""
    for ch in cigar:
        if ch.isdigit():
            num += ch
        else:
            out += [ch] * int(num)
            num = ""
    return out


def cigar_score(ops, p, t, start, kind, s):
    """Score of ops (source to sink) placed at text position `start`; None if it does not fit.
    M consumes one pattern and one text symbol; D a text symbol; I a pattern symbol."""
    i = j = 0
    k = start
    total, prev = 0, None
    for op in ops:
        if op == "M":
            if i >= len(p) or k >= len(t):
                return None
            total += s["match"] if p[i] == t[k] else s["mismatch"]
            i += 1; k += 1
        else:
            if op == "D":
                if k >= len(t):
                    return None
                k += 1
            else:
                if i >= len(p):
                    return None
                i += 1
            if kind == "sw":
                total += s["deletion"] if op == "D" else s["insertion"]
            else:
                total += s["gap_open"] if prev != op else s["gap_ext"]
        prev = op
    if i != len(p):
        return None
    return total


def implied(cigar, kind, type_, p=PATTERN, t=TEXT, scheme=None):
    ops = ops_of(cigar)[::-1]                   # printed sink to source
    starts = [0] if type_ == "GLOBAL" else range(len(t))
    best = None
    for st in starts:
        sc = cigar_score(ops, p, t, st, kind, scheme or SCHEMES[kind])
        if sc is None:
            continue
        if type_ == "GLOBAL" and st + sum(op != "I" for op in ops) != len(t):
            continue
        best = sc if best is None or sc > best else best
    return best


def in_band_placements(ops, band):
    """Text starts whose path keeps every cell (i, c) at 0 <= c - i < band (leading text gaps
    are the free semi-global start and carry no cell)."""
    out = []
    for st in range(band):
        i, k, ok = 0, st, True
        for op in ops:
            if op == "M":
                cell = k - i; i += 1; k += 1
            elif op == "D":
                cell = k - (i - 1) if i > 0 else 0; k += 1
            else:
                cell = k - 1 - i; i += 1
            ok &= 0 <= cell < band
        if ok:
            out.append(st)
    return out


def implied_banded(cigar, kind, band, p=PATTERN, t=TEXT, scheme=None):
    ops = ops_of(cigar)[::-1]
    best = None
    for st in in_band_placements(ops, band):
        sc = cigar_score(ops, p, t, st, kind, scheme or SCHEMES[kind])
        if sc is not None:
            best = sc if best is None or sc > best else best
    return best


def main():
    cases = []
    for kind in ("sw", "gotoh"):
        for type_, cigar in CIGARS.items():
            cases.append(dict(aligner=kind, type=type_, scheme=SCHEMES[kind], pattern=PATTERN, text=TEXT,
                              cigar=cigar, score=implied(cigar, kind, type_),
                              source="NvB/nvbio-test/alignment_test.cu:749-793"))
    ed = [dict(test_id=i, pattern=p, text=t, score=e, band=5, type="SEMI_GLOBAL",
               source="NvB/nvbio-test/alignment_test.cu:680-745") for i, p, t, e in ED_CASES]
    banded = [dict(aligner="gotoh", type="SEMI_GLOBAL", band=7, scheme=SCHEMES["gotoh"], pattern=PATTERN, text=TEXT,
                   cigar="4M1D3M", score=implied_banded("4M1D3M", "gotoh", 7),
                   source="NvB/nvbio-test/alignment_test.cu:790 (SingleTest::banded, :296-356)")]
    banded.append(dict(aligner="gotoh", type="SEMI_GLOBAL", band=31, scheme=REAL_GOTOH, pattern=BANDED_READ,
                       text=BANDED_WINDOW, cigar="147M2D3M",
                       score=implied_banded("147M2D3M", "gotoh", 31, BANDED_READ, BANDED_WINDOW, REAL_GOTOH),
                       source="NvB/nvbio-test/alignment_test.cu:796-826"))
    real = [dict(aligner="gotoh", type="SEMI_GLOBAL", scheme=REAL_GOTOH, pattern=FULL_READ, text=FULL_TEXT,
                 cigar="6I138M", score=implied("6I138M", "gotoh", "SEMI_GLOBAL", FULL_READ, FULL_TEXT, REAL_GOTOH),
                 source="NvB/nvbio-test/alignment_test.cu:828-868"),
            dict(aligner="ed", type="SEMI_GLOBAL", scheme=ED_SCHEME, pattern=FULL_READ, text=FULL_TEXT,
                 cigar="1I1M2I1M3I136M",
                 score=implied("1I1M2I1M3I136M", "sw", "SEMI_GLOBAL", FULL_READ, FULL_TEXT, ED_SCHEME),
                 source="NvB/nvbio-test/alignment_test.cu:870-904")]
    json.dump({"alignment": cases, "edit_distance": ed, "banded": banded, "traceback_real": real},
              open(OUT, "w"), indent=1)
    print(OUT, [(c["aligner"], c["type"], c["score"]) for c in cases + banded + real])


if __name__ == "__main__":
    main()
