"""ctypes binding of the CPU oracle (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.  The oracle is a
C restatement of the GASAL2 kernels (see gasal_oracle.h); parity is pinned by
the SURVEY.md §8c known-answer vectors (tests/golden/survey_kat.json).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborc.so")

# enum values of the reference (gasal.h:37-73)
WITHOUT_START, WITH_START, WITH_TB = 0, 1, 2
NONE, QUERY, TARGET, BOTH = 0, 1, 2, 3
UNKNOWN, GLOBAL, SEMI_GLOBAL, LOCAL, MICROLOCAL, BANDED, KSW = 0, 1, 2, 3, 4, 5, 6


class OrcParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "match", "mismatch", "gap_open", "gap_extend", "algo", "start_pos",
        "second_best", "head", "tail", "k_band", "is_packed", "n_code",
        "has_n_penalty", "n_penalty", "max_query_len")]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_NATIVE_PATH = os.path.join(_HERE, "build", "native", "liborc.so")
_libs = {}            # path -> loaded handle
_active = None        # path lib() returns (None: the portable build)


def native_available() -> bool:
    """Build the -O3 -march=native variant (oracle/Makefile `native`) for this host's CPU:
    the timed CPU baseline of bench.py.  False if it does not build."""
    try:
        subprocess.run(["make", "-s", "-C", _HERE, "native"], check=True, capture_output=True, timeout=300)
    except Exception:
        return False
    return os.path.exists(_NATIVE_PATH)


def use_native(on: bool = True) -> bool:
    """Route the oracle calls of this process through the native (on) or the portable
    build; both stay loaded.  Returns whether the native build is now in use."""
    global _active
    if on and not native_available():
        on = False
    _active = _NATIVE_PATH if on else None
    return on


def lib():
    path = _active or _LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            build()
        h = ctypes.CDLL(path)
        h.orc_aln_batch.restype = ctypes.c_int
        h.orc_pairhmm_batch.restype = ctypes.c_int
        _libs[path] = h
    return _libs[path]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def make_params(algo=LOCAL, start_pos=WITHOUT_START, second_best=0, head=TARGET, tail=TARGET,
                match=1, mismatch=4, gap_open=6, gap_extend=1, k_band=0, is_packed=0,
                n_code=0x4E, n_penalty=None, max_query_len=0) -> OrcParams:
    return OrcParams(match, mismatch, gap_open, gap_extend, algo, start_pos, int(second_best),
                     head, tail, k_band, is_packed, n_code,
                     0 if n_penalty is None else 1, 0 if n_penalty is None else n_penalty,
                     max_query_len)


SENTINEL = -(2 ** 31) + 7


def align(batch, params: OrcParams, q_ops=None, t_ops=None, seed_scores=None, n_threads=0):
    """Run the oracle on a Batch (see tests/batch.py).  Returns dict of arrays;
    fields the reference would not write stay at SENTINEL."""
    n = batch.n
    out = {k: np.full(n, SENTINEL, np.int32) for k in
           ("score", "q_end", "t_end", "q_start", "t_start", "score2", "q_end2", "t_end2")}
    # a CIGAR longer than its slot runs into the next; slack keeps the
    # last pair's overrun inside the array
    slack = int((np.asarray(batch.q_lens, np.int64) + np.asarray(batch.t_lens, np.int64)).max(initial=0)) + 64
    cigar = np.zeros(batch.q_bytes + slack, np.uint8)
    n_ops = np.zeros(n, np.uint32)
    qo = None if q_ops is None else np.ascontiguousarray(q_ops, np.uint8)
    to = None if t_ops is None else np.ascontiguousarray(t_ops, np.uint8)
    sd = None if seed_scores is None else np.ascontiguousarray(seed_scores, np.uint32)
    rc = lib().orc_aln_batch(
        ctypes.byref(params),
        _ptr(batch.q_data), _ptr(batch.q_offsets), _ptr(batch.q_lens),
        _ptr(batch.t_data), _ptr(batch.t_offsets), _ptr(batch.t_lens),
        ctypes.c_uint32(batch.q_bytes), ctypes.c_uint32(batch.t_bytes), ctypes.c_uint32(n),
        _ptr(qo), _ptr(to), _ptr(sd),
        _ptr(out["score"]), _ptr(out["q_end"]), _ptr(out["t_end"]),
        _ptr(out["q_start"]), _ptr(out["t_start"]),
        _ptr(out["score2"]), _ptr(out["q_end2"]), _ptr(out["t_end2"]),
        _ptr(cigar), _ptr(n_ops), ctypes.c_int(n_threads))
    if rc != 0:
        raise ValueError(f"orc_aln_batch failed: {rc}")
    out["cigar"] = cigar[:batch.q_bytes]
    out["n_ops"] = n_ops
    return out


def pairhmm_params(bq, iq, dq):
    n = len(bq)
    qm, de, xi, al = (np.zeros(n, np.float32) for _ in range(4))
    lib().orc_pairhmm_params(_ptr(np.ascontiguousarray(bq, np.uint8)),
                             _ptr(np.ascontiguousarray(iq, np.uint8)),
                             _ptr(np.ascontiguousarray(dq, np.uint8)), ctypes.c_uint32(n),
                             _ptr(qm), _ptr(de), _ptr(xi), _ptr(al))
    return qm, de, xi, al


def pairhmm(reads, read_off, read_len, qm, delta, xiksi, alpha, haps, hap_off, hap_len, n_threads=0):
    n = len(read_len)
    res = np.zeros(n, np.float32)
    c = lambda a, t: np.ascontiguousarray(a, t)
    lib().orc_pairhmm_batch(ctypes.c_uint32(n), _ptr(c(reads, np.uint8)), _ptr(c(read_off, np.uint32)),
                            _ptr(c(read_len, np.uint32)), _ptr(c(qm, np.float32)), _ptr(c(delta, np.float32)),
                            _ptr(c(xiksi, np.float32)), _ptr(c(alpha, np.float32)), _ptr(c(haps, np.uint8)),
                            _ptr(c(hap_off, np.uint32)), _ptr(c(hap_len, np.uint32)), _ptr(res),
                            ctypes.c_int(n_threads))
    return res


def nv_score(aligner, patterns, texts, n_threads=0):
    """nvbio batched score restatement (nvbio_oracle.c): aligner is a gasal_ffi.NvAligner
    (or anything with aligner/type/prm()), patterns/texts gasal_ffi.PackedSet-like."""
    n = len(patterns.offsets) - 1
    out = np.zeros(n, np.int32)
    lib().orc_nv_score_batch.restype = ctypes.c_int
    rc = lib().orc_nv_score_batch(ctypes.c_int(aligner.aligner), ctypes.c_int(aligner.type), _ptr(aligner.prm()),
                                  ctypes.c_uint32(n), _ptr(patterns.words), _ptr(patterns.offsets),
                                  ctypes.c_uint32(patterns.bits), ctypes.c_uint32(int(patterns.big_endian)),
                                  _ptr(texts.words), _ptr(texts.offsets), ctypes.c_uint32(texts.length),
                                  ctypes.c_uint32(texts.bits), ctypes.c_uint32(int(texts.big_endian)), _ptr(out),
                                  ctypes.c_int(n_threads))
    if rc != 0:
        raise RuntimeError(f"orc_nv_score_batch failed ({rc})")
    return out



def nv_traceback(aligner, patterns, texts, n_threads=0):
    """nvbio full-DP traceback restatement (nvbio_oracle.c orc_nv_traceback_*): per pair the
    BestSink score, source and sink (x = text, y = pattern coordinate) and the backtracker's
    pushes in push order (0 SUBSTITUTION 'M', 1 INSERTION 'I', 2 DELETION 'D')."""
    n = len(patterns.offsets) - 1
    po = np.asarray(patterns.offsets, np.int64)
    plen = po[1:] - po[:-1]
    if texts.offsets is not None:
        to = np.asarray(texts.offsets, np.int64)
        tlen = to[1:] - to[:-1]
    else:
        tlen = np.full(n, int(texts.length), np.int64)
    stride = int((plen + tlen).max(initial=0)) + 1
    scores = np.zeros(n, np.int32)
    src = np.zeros(2 * n, np.uint32)
    snk = np.zeros(2 * n, np.uint32)
    ops = np.zeros(max(n * stride, 1), np.uint8)
    n_ops = np.zeros(n, np.uint32)
    lib().orc_nv_traceback_batch.restype = ctypes.c_int
    rc = lib().orc_nv_traceback_batch(ctypes.c_int(aligner.aligner), ctypes.c_int(aligner.type), _ptr(aligner.prm()),
                                      ctypes.c_uint32(n), _ptr(patterns.words), _ptr(patterns.offsets),
                                      ctypes.c_uint32(patterns.bits), ctypes.c_uint32(int(patterns.big_endian)),
                                      _ptr(texts.words), _ptr(texts.offsets), ctypes.c_uint32(texts.length),
                                      ctypes.c_uint32(texts.bits), ctypes.c_uint32(int(texts.big_endian)),
                                      _ptr(scores), _ptr(src), _ptr(snk), _ptr(ops), ctypes.c_uint32(stride),
                                      _ptr(n_ops), ctypes.c_int(n_threads))
    if rc != 0:
        raise RuntimeError(f"orc_nv_traceback_batch failed ({rc})")
    return dict(score=scores, source=src.reshape(n, 2), sink=snk.reshape(n, 2),
                ops=[ops[k * stride:k * stride + int(n_ops[k])].copy() for k in range(n)])


def nv_banded_traceback(aligner, band, patterns, texts, n_threads=0):
    """nvbio banded traceback restatement (nvbio_oracle.c orc_nv_banded_traceback_*):
    BatchedBandedAlignmentTraceback<band>; the dict nv_traceback returns."""
    n = len(patterns.offsets) - 1
    po = np.asarray(patterns.offsets, np.int64)
    plen = po[1:] - po[:-1]
    stride = 2 * int(plen.max(initial=0)) + int(band) + 1
    scores = np.zeros(n, np.int32)
    src = np.zeros(2 * n, np.uint32)
    snk = np.zeros(2 * n, np.uint32)
    ops = np.zeros(max(n * stride, 1), np.uint8)
    n_ops = np.zeros(n, np.uint32)
    lib().orc_nv_banded_traceback_batch.restype = ctypes.c_int
    rc = lib().orc_nv_banded_traceback_batch(
        ctypes.c_int(aligner.aligner), ctypes.c_int(aligner.type), _ptr(aligner.prm()), ctypes.c_uint32(band),
        ctypes.c_uint32(n), _ptr(patterns.words), _ptr(patterns.offsets), ctypes.c_uint32(patterns.bits),
        ctypes.c_uint32(int(patterns.big_endian)), _ptr(texts.words), _ptr(texts.offsets),
        ctypes.c_uint32(texts.length), ctypes.c_uint32(texts.bits), ctypes.c_uint32(int(texts.big_endian)),
        _ptr(scores), _ptr(src), _ptr(snk), _ptr(ops), ctypes.c_uint32(stride), _ptr(n_ops), ctypes.c_int(n_threads))
    if rc != 0:
        raise RuntimeError(f"orc_nv_banded_traceback_batch failed ({rc})")
    return dict(score=scores, source=src.reshape(n, 2), sink=snk.reshape(n, 2),
                ops=[ops[k * stride:k * stride + int(n_ops[k])].copy() for k in range(n)])


def nv_cigar_string(ops, M, source_y, sink_y):
    """nvbio-test's TestBacktracker string of one alignment, as rle() prints it: the pushes in
    push order, then the start clip (source.y 'S'; the end clip, pattern length - sink.y, is
    written first and overwritten by the pushes, alignment_test_utils.h:628-645)."""
    s = "".join("MID"[o] for o in ops) + "S" * int(source_y)
    out, prev, cnt = [], None, 0
    for ch in s:
        if ch == prev:
            cnt += 1
        else:
            if prev is not None:
                out.append(f"{cnt}{prev}")
            prev, cnt = ch, 1
    if cnt:
        out.append(f"{cnt}{prev}")
    return "".join(out)


def nv_banded_score(aligner, band, patterns, texts, n_threads=0):
    """nvbio banded score restatement (nvbio_oracle.c orc_nv_banded_*): BatchedBandedAlignmentScore<band>."""
    n = len(patterns.offsets) - 1
    out = np.zeros(n, np.int32)
    lib().orc_nv_banded_score_batch.restype = ctypes.c_int
    rc = lib().orc_nv_banded_score_batch(ctypes.c_int(aligner.aligner), ctypes.c_int(aligner.type),
                                         _ptr(aligner.prm()), ctypes.c_uint32(band), ctypes.c_uint32(n),
                                         _ptr(patterns.words), _ptr(patterns.offsets), ctypes.c_uint32(patterns.bits),
                                         ctypes.c_uint32(int(patterns.big_endian)), _ptr(texts.words),
                                         _ptr(texts.offsets), ctypes.c_uint32(texts.length),
                                         ctypes.c_uint32(texts.bits), ctypes.c_uint32(int(texts.big_endian)),
                                         _ptr(out), ctypes.c_int(n_threads))
    if rc != 0:
        raise RuntimeError(f"orc_nv_banded_score_batch failed ({rc})")
    return out
