"""Shared test helpers: fixture readers and random batch builders."""
from __future__ import annotations

import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def kat():
    with open(os.path.join(GOLDEN, "survey_kat.json")) as f:
        return json.load(f)


def read_fasta_pairs(limit=None):
    """The reference test_prog's 20K sample pairs (test_prog/{query,target}_batch.fasta.gz),
    read in lock step like test_prog.cpp:90-137; returns (queries, targets, q_mod, t_mod)."""
    starts = "></+"

    def records(path):
        out, mods, cur = [], [], None
        with gzip.open(path, "rt") as fh:
            for line in fh:
                line = line.rstrip("\n")
                if line and line[0] in starts:
                    if cur is not None:
                        out.append(cur)
                    mods.append(starts.index(line[0]))
                    cur = ""
                    if limit is not None and len(out) >= limit:
                        break
                elif cur is not None:
                    cur += line
        if cur is not None and (limit is None or len(out) < limit):
            out.append(cur)
        return out[:limit] if limit else out, mods[:limit] if limit else mods

    q, qm = records(os.path.join(GOLDEN, "query_batch.fasta.gz"))
    t, tm = records(os.path.join(GOLDEN, "target_batch.fasta.gz"))
    n = min(len(q), len(t))
    return q[:n], t[:n], qm[:n], tm[:n]


def read_pairhmm_dataset(path):
    """Synthetic PairHMM input (Non-CDP/PairHMM/Intra-task/Synthetic_data/dataset/*.txt),
    parsed as tile_1.cu:246-290: read len, read + base/ins/del/gcp quals, hap len, hap."""
    toks = open(path).read().split()
    pos = 0
    size = int(toks[pos]); pos += 1
    pairs = []
    for _ in range(size):
        rl = int(toks[pos]); pos += 1
        read = toks[pos]; pos += 1
        quals = []
        for _q in range(4):
            quals.append([int(x) for x in toks[pos:pos + rl]]); pos += rl
        hl = int(toks[pos]); pos += 1
        hap = toks[pos]; pos += 1
        pairs.append(dict(read=read, bq=quals[0], iq=quals[1], dq=quals[2], gcp=quals[3], hap=hap[:hl]))
    return pairs


BASES = np.frombuffer(b"ACGT", np.uint8)


def random_seq(rng, n, alphabet=b"ACGT"):
    a = np.frombuffer(alphabet, np.uint8)
    return bytes(a[rng.integers(0, len(a), n)])


def mutate(rng, s: bytes, sub=0.08, indel=0.02):
    out = bytearray()
    i = 0
    while i < len(s):
        u = rng.random()
        if u < indel / 2:
            out += random_seq(rng, int(rng.integers(1, 4)))
            out.append(s[i]); i += 1
        elif u < indel:
            i += int(rng.integers(1, 4))
        elif u < indel + sub:
            out += random_seq(rng, 1); i += 1
        else:
            out.append(s[i]); i += 1
    return bytes(out) if out else b"A"


def random_pairs(rng, n, qmin, qmax, tmin, tmax, related=0.7, alphabet=b"ACGT"):
    qs, ts = [], []
    for _ in range(n):
        ql = int(rng.integers(qmin, qmax + 1))
        q = random_seq(rng, ql, alphabet)
        if rng.random() < related:
            t = mutate(rng, q)
            tl = int(rng.integers(tmin, tmax + 1))
            t = (t + random_seq(rng, max(0, tl - len(t)), alphabet))[:tl]
        else:
            t = random_seq(rng, int(rng.integers(tmin, tmax + 1)), alphabet)
        qs.append(q); ts.append(t)
    return qs, ts
