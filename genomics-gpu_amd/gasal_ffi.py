"""ctypes binding of libgasal's flat C-ABI (include/gasalx.h).

This is the Python side of the drop-in boundary: it mirrors the reference's
host-side batch construction (gasal_host_batch_fill: sequences concatenated,
each N_CODE-padded to a multiple of 8, offsets including pads, lengths without
them — Non-CDP/GASAL2/src/host_batch.cpp:79-153, README.md:145) and calls the
HIP engine.  There is no CPU fallback: if lib/libgasal.so is missing or no GPU
is present, the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GASALX_LIB") or os.path.join(_HERE, "lib", "libgasal.so")

# enum values of the reference (gasal.h:37-73)
WITHOUT_START, WITH_START, WITH_TB = 0, 1, 2
NONE, QUERY, TARGET, BOTH = 0, 1, 2, 3
UNKNOWN, GLOBAL, SEMI_GLOBAL, LOCAL, MICROLOCAL, BANDED, KSW = 0, 1, 2, 3, 4, 5, 6
N_CODE = 0x4E

# exported symbols of include/gasalx.h
EXPORTS = (
    "gasalx_abi_version", "gasalx_last_error", "gasalx_device_count", "gasalx_engine_create",
    "gasalx_engine_destroy", "gasalx_align_device", "gasalx_align_host", "gasalx_describe_plan",
    "gasalx_pairhmm_device", "gasalx_pairhmm_host", "gasalx_pairhmm_params", "gasalx_synth_sizes",
    "gasalx_synth_spec", "gasalx_synth_pairs", "gasalx_synth_range", "gasalx_host_alloc", "gasalx_host_free",
    "gasalx_pairhmm_quals_device", "gasalx_pairhmm_quals_host", "gasalx_hmm_file_read", "gasalx_hmm_file_free",
    "gasalx_nv_score_device", "gasalx_nv_score_host", "gasalx_nv_describe_plan",
    "gasalx_nv_banded_score_device", "gasalx_nv_banded_score_host",
    "gasalx_nv_traceback_device", "gasalx_nv_traceback_host",
    "gasalx_nv_banded_traceback_device", "gasalx_nv_banded_traceback_host",
    "gasalx_multi_create", "gasalx_multi_destroy", "gasalx_multi_info", "gasalx_multi_engine",
    "gasalx_shard_bounds", "gasalx_multi_align_host", "gasalx_multi_pairhmm_host",
    "gasalx_multi_pairhmm_quals_host", "gasalx_multi_allgather", "gasalx_packed_pairs",
    "gasalx_multi_align_device", "gasalx_multi_pairhmm_device",
)
MULTI_RCCL = 1

# nvbio front-end (gasalx_nv_*): aligners and AlignmentType (nvbio/alignment/alignment_base.h:54)
NV_ED, NV_SW, NV_GOTOH = 0, 1, 2
NV_GLOBAL, NV_LOCAL, NV_SEMI_GLOBAL = 0, 1, 2


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "match", "mismatch", "gap_open", "gap_extend", "algo", "start_pos", "second_best", "head", "tail",
        "k_band", "is_packed", "n_code", "has_n_penalty", "n_penalty", "max_query_len")]


class CBatch(ctypes.Structure):
    _fields_ = [("q_batch", ctypes.c_void_p), ("q_offsets", ctypes.c_void_p), ("q_lens", ctypes.c_void_p),
                ("t_batch", ctypes.c_void_p), ("t_offsets", ctypes.c_void_p), ("t_lens", ctypes.c_void_p),
                ("q_bytes", ctypes.c_uint32), ("t_bytes", ctypes.c_uint32), ("n_alns", ctypes.c_uint32),
                ("q_ops", ctypes.c_void_p), ("t_ops", ctypes.c_void_p), ("seed_scores", ctypes.c_void_p),
                ("max_q_len", ctypes.c_uint32), ("max_t_len", ctypes.c_uint32)]


class CResults(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "aln_score", "q_end", "t_end", "q_start", "t_start", "aln_score2", "q_end2", "t_end2", "cigar",
        "n_cigar_ops")]


class CHmmBatch(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_void_p), ("read_offsets", ctypes.c_void_p), ("read_lens", ctypes.c_void_p),
                ("qm", ctypes.c_void_p), ("delta", ctypes.c_void_p), ("xiksi", ctypes.c_void_p),
                ("alpha", ctypes.c_void_p), ("haps", ctypes.c_void_p), ("hap_offsets", ctypes.c_void_p),
                ("hap_lens", ctypes.c_void_p), ("read_bytes", ctypes.c_uint32), ("hap_bytes", ctypes.c_uint32),
                ("n_pairs", ctypes.c_uint32), ("max_read_len", ctypes.c_uint32), ("max_hap_len", ctypes.c_uint32)]


class CHmmQualBatch(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_void_p), ("read_offsets", ctypes.c_void_p), ("read_lens", ctypes.c_void_p),
                ("base_quals", ctypes.c_void_p), ("ins_quals", ctypes.c_void_p), ("del_quals", ctypes.c_void_p),
                ("haps", ctypes.c_void_p), ("hap_offsets", ctypes.c_void_p), ("hap_lens", ctypes.c_void_p),
                ("read_bytes", ctypes.c_uint64), ("hap_bytes", ctypes.c_uint64), ("n_pairs", ctypes.c_uint32),
                ("max_read_len", ctypes.c_uint32), ("max_hap_len", ctypes.c_uint32)]


class CHmmFile(ctypes.Structure):
    _fields_ = [("n_pairs", ctypes.c_uint32), ("n_groups", ctypes.c_uint32), ("group_sizes", ctypes.c_void_p),
                ("reads", ctypes.c_void_p), ("read_offsets", ctypes.c_void_p), ("read_lens", ctypes.c_void_p),
                ("base_quals", ctypes.c_void_p), ("ins_quals", ctypes.c_void_p), ("del_quals", ctypes.c_void_p),
                ("gcp_quals", ctypes.c_void_p), ("haps", ctypes.c_void_p), ("hap_offsets", ctypes.c_void_p),
                ("hap_lens", ctypes.c_void_p), ("read_bytes", ctypes.c_uint64), ("hap_bytes", ctypes.c_uint64)]


class CNvAligner(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("aligner", "type", "match", "mismatch", "gap_open", "gap_ext",
                                               "deletion", "insertion")]


class CNvStrings(ctypes.Structure):
    _fields_ = [("words", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("length", ctypes.c_uint32),
                ("bits", ctypes.c_uint32), ("big_endian", ctypes.c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libgasal not built: {LIB_PATH} (run __graft_entry__.build())")
        # torch (when present) first: its bundled HIP runtime (soname libamdhip64.so.7)
        # must be the one libgasal binds to; loading libgasal first brings in /opt/rocm's
        # copy, and two HIP runtimes in one process do not share the device (torch then
        # reports no GPU).  INTEGRATION.md, "One HIP runtime per process".
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.gasalx_last_error.restype = ctypes.c_char_p
        for name in EXPORTS:
            # (an older build loaded through GASALX_LIB for an A/B run may lack the newest entry
            # points; tests/test_capi.py checks the default build exports every one)
            if name != "gasalx_last_error" and hasattr(_lib, name):
                getattr(_lib, name).restype = ctypes.c_int
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().gasalx_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def make_params(algo=LOCAL, start_pos=WITHOUT_START, second_best=0, head=TARGET, tail=TARGET, match=1, mismatch=4,
                gap_open=6, gap_extend=1, k_band=0, is_packed=0, n_code=N_CODE, n_penalty=None,
                max_query_len=0) -> Params:
    return Params(match, mismatch, gap_open, gap_extend, algo, start_pos, int(second_best), head, tail, k_band,
                  is_packed, n_code, 0 if n_penalty is None else 1, 0 if n_penalty is None else n_penalty,
                  max_query_len)


def pad8(x):
    return (x + 7) // 8 * 8


@dataclass
class Batch:
    """A GASAL2-layout batch in host memory."""
    q_data: np.ndarray
    q_offsets: np.ndarray
    q_lens: np.ndarray
    t_data: np.ndarray
    t_offsets: np.ndarray
    t_lens: np.ndarray

    @property
    def n(self):
        return len(self.q_lens)

    @property
    def q_bytes(self):
        return len(self.q_data)

    @property
    def t_bytes(self):
        return len(self.t_data)

    @staticmethod
    def _side(seqs):
        lens = np.array([len(s) for s in seqs], np.uint32)
        offs = np.zeros(len(seqs), np.uint32)
        total = int(sum(pad8(len(s)) for s in seqs))
        data = np.full(max(total, 8), N_CODE, np.uint8)
        pos = 0
        for i, s in enumerate(seqs):
            b = s.encode() if isinstance(s, str) else bytes(s)
            offs[i] = pos
            data[pos:pos + len(b)] = np.frombuffer(b, np.uint8)
            pos += pad8(len(b))
        return data, offs, lens

    @classmethod
    def from_pairs(cls, queries, targets):
        qd, qo, ql = cls._side(queries)
        td, to, tl = cls._side(targets)
        return cls(qd, qo, ql, td, to, tl)

    @classmethod
    def synth(cls, kind: int, n: int, seed: int, start: int = 0):
        """SURVEY.md §8(d) workloads (kind 1..4 = configs 1..4): pairs [start, start + n)
        of the seeded batch, via gasalx_synth_range (offsets start at 0)."""
        qb, tb = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().gasalx_synth_sizes(kind, ctypes.c_uint32(n), ctypes.byref(qb), ctypes.byref(tb)), "synth_sizes")
        qd, td = np.zeros(qb.value, np.uint8), np.zeros(tb.value, np.uint8)
        qo, ql, to, tl = (np.zeros(n, np.uint32) for _ in range(4))
        _check(lib().gasalx_synth_range(kind, ctypes.c_uint64(seed), ctypes.c_uint64(start), ctypes.c_uint32(n),
                                        _p(qd), _p(qo), _p(ql), _p(td), _p(to), _p(tl)), "synth_range")
        return cls(qd, qo, ql, td, to, tl)

    def slice(self, start: int, end: int):
        """Pairs [start, end) as a batch of their own.  When the pairs' bytes are laid out
        in order (offsets increasing, each sequence in its own padded slot, as
        gasal_host_batch_fill writes them) this is a view with rebased offsets;
        otherwise the pairs are re-packed (subset)."""
        if end <= start:
            return self.subset([])
        qo, to = self.q_offsets[start:end].astype(np.int64), self.t_offsets[start:end].astype(np.int64)
        ql, tl = self.q_lens[start:end].astype(np.int64), self.t_lens[start:end].astype(np.int64)
        qp, tp = (ql + 7) // 8 * 8, (tl + 7) // 8 * 8
        if np.array_equal(qo[1:], qo[:-1] + qp[:-1]) and np.array_equal(to[1:], to[:-1] + tp[:-1]):
            q0, t0 = int(qo[0]), int(to[0])
            q1, t1 = int(qo[-1] + qp[-1]), int(to[-1] + tp[-1])
            return Batch(self.q_data[q0:q1], (qo - q0).astype(np.uint32), self.q_lens[start:end].copy(),
                         self.t_data[t0:t1], (to - t0).astype(np.uint32), self.t_lens[start:end].copy())
        return self.subset(np.arange(start, end))

    def subset(self, idx):
        """Re-pack pairs idx into a fresh batch (keeps each pair's padded bytes)."""
        qs = [bytes(self.q_data[self.q_offsets[i]:self.q_offsets[i] + self.q_lens[i]]) for i in idx]
        ts = [bytes(self.t_data[self.t_offsets[i]:self.t_offsets[i] + self.t_lens[i]]) for i in idx]
        return Batch.from_pairs(qs, ts)


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


SENTINEL = -(2 ** 31) + 7
OUT_FIELDS = ("score", "q_end", "t_end", "q_start", "t_start", "score2", "q_end2", "t_end2")


class _PinnedArray(np.ndarray):
    """ndarray over page-locked bytes; holds the allocation's owner so the memory
    lives as long as any view of it does."""
    _owner = None


class _PinnedOwner:
    """The allocation itself: freed (gasalx_host_free) as soon as the last array
    referring to it is gone.  Nothing refers back to the arrays, so no reference
    cycle waits for the cyclic collector."""

    def __init__(self, ptr: int):
        self.ptr = ptr
        self._finalizer = weakref.finalize(self, lib().gasalx_host_free, ctypes.c_void_p(ptr))


class PinnedHost:
    """Page-locked host bytes from libgasal's own HIP runtime (gasalx_host_alloc), for
    caller-owned buffers such as align_host(cigar_out=...), as the reference's host_res
    is pinned (res.cpp:8-70).

    `array` (and every view or slice of it) keeps the allocation alive, and the memory
    is freed as soon as the last of them is gone (this handle included): close()
    drops this handle's own reference, it never frees memory an array still points at."""

    def __init__(self, nbytes: int):
        L = lib()
        self._p = ctypes.c_void_p()
        _check(L.gasalx_host_alloc(ctypes.c_uint64(max(int(nbytes), 1)), ctypes.byref(self._p)), "host_alloc")
        self.nbytes = int(nbytes)
        owner = _PinnedOwner(self._p.value)
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * max(self.nbytes, 1)).from_address(self._p.value))
        arr = raw[:self.nbytes].view(_PinnedArray)
        arr._owner = owner
        self.array = arr

    def close(self):
        self.array = None


class Engine:
    """One device workspace + stream (gasalx_engine)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().gasalx_engine_create(device, ctypes.byref(self._h)), "engine_create")

    def close(self):
        if self._h:
            lib().gasalx_engine_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def align_host(self, batch: Batch, params: Params, q_ops=None, t_ops=None, seed_scores=None, fields=None,
                   cigar_out=None, max_q_len=0, max_t_len=0):
        """fields: the result arrays to request (default all; the rest are passed as NULL).
        cigar_out: optional caller-owned uint8 array of q_bytes for the CIGAR buffer (e.g. a
        page-locked one, as the reference's own host_res, res.cpp:8-70), used as given.
        max_q_len / max_t_len: the batch's upper bounds of the lengths (gasalx.h; 0 = from the lengths)."""
        n = batch.n
        out = {k: np.full(n, SENTINEL, np.int32) for k in (OUT_FIELDS if fields is None else fields)}
        tb = params.start_pos == WITH_TB          # CIGAR buffers only when the reference fills them
        if cigar_out is not None:
            if not (tb and isinstance(cigar_out, np.ndarray) and cigar_out.dtype == np.uint8
                    and cigar_out.ndim == 1 and cigar_out.size >= batch.q_bytes and cigar_out.flags.c_contiguous):
                raise ValueError("cigar_out: contiguous uint8 array of at least q_bytes, WITH_TB only")
            cigar = cigar_out
        else:
            cigar = np.zeros(batch.q_bytes if tb else 0, np.uint8)
        n_ops = np.zeros(n if tb else 0, np.uint32)
        qo = None if q_ops is None else np.ascontiguousarray(q_ops, np.uint8)
        to = None if t_ops is None else np.ascontiguousarray(t_ops, np.uint8)
        sd = None if seed_scores is None else np.ascontiguousarray(seed_scores, np.uint32)
        cb = CBatch(_p(batch.q_data), _p(batch.q_offsets), _p(batch.q_lens), _p(batch.t_data), _p(batch.t_offsets),
                    _p(batch.t_lens), batch.q_bytes, batch.t_bytes, n, _p(qo), _p(to), _p(sd), max_q_len, max_t_len)
        cr = CResults(*(_p(out[k]) if k in out else None for k in OUT_FIELDS), _p(cigar) if tb else None,
                      _p(n_ops) if tb else None)
        _check(lib().gasalx_align_host(self._h, ctypes.byref(params), ctypes.byref(cb), ctypes.byref(cr)),
               "align_host")
        out["cigar"] = cigar
        out["n_ops"] = n_ops
        return out

    def packed_pairs(self):
        """(handled, total): pairs of the last packed launches the packed kernels aligned themselves
        (gasalx_packed_pairs); the rest went to the int32 kernel."""
        h, t = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().gasalx_packed_pairs(self._h, ctypes.byref(h), ctypes.byref(t)), "packed_pairs")
        return int(h.value), int(t.value)

    def align_device_ptrs(self, params: Params, ptrs: dict, q_bytes: int, t_bytes: int, n: int, max_q: int,
                          max_t: int, stream: int = 0):
        """Device-resident call: ptrs holds integer device addresses (e.g. torch tensor.data_ptr())."""
        g = lambda k: ptrs.get(k) or None
        cb = CBatch(g("q_batch"), g("q_offsets"), g("q_lens"), g("t_batch"), g("t_offsets"), g("t_lens"), q_bytes,
                    t_bytes, n, g("q_ops"), g("t_ops"), g("seed_scores"), max_q, max_t)
        cr = CResults(g("aln_score"), g("q_end"), g("t_end"), g("q_start"), g("t_start"), g("aln_score2"),
                      g("q_end2"), g("t_end2"), g("cigar"), g("n_cigar_ops"))
        _check(lib().gasalx_align_device(self._h, ctypes.byref(params), ctypes.byref(cb), ctypes.byref(cr),
                                         ctypes.c_void_p(stream or None)), "align_device")

    def pairhmm_host(self, reads, read_off, read_len, qm, delta, xiksi, alpha, haps, hap_off, hap_len):
        c = lambda a, t: np.ascontiguousarray(a, t)
        reads, haps = c(reads, np.uint8), c(haps, np.uint8)
        arrs = [c(read_off, np.uint32), c(read_len, np.uint32), c(qm, np.float32), c(delta, np.float32),
                c(xiksi, np.float32), c(alpha, np.float32), c(hap_off, np.uint32), c(hap_len, np.uint32)]
        n = len(arrs[1])
        res = np.zeros(n, np.float32)
        hb = CHmmBatch(_p(reads), _p(arrs[0]), _p(arrs[1]), _p(arrs[2]), _p(arrs[3]), _p(arrs[4]), _p(arrs[5]),
                       _p(haps), _p(arrs[6]), _p(arrs[7]), len(reads), len(haps), n, 0, 0)
        _check(lib().gasalx_pairhmm_host(self._h, ctypes.byref(hb), _p(res)), "pairhmm_host")
        return res

    def pairhmm_quals_host(self, hmm: "HmmData"):
        """PairHMM from Phred qualities (the reference's input files): sorted by length,
        one launch per lane-group class; results in input order."""
        res = np.zeros(hmm.n, np.float32)
        hb = hmm.cstruct()
        _check(lib().gasalx_pairhmm_quals_host(self._h, ctypes.byref(hb), _p(res)), "pairhmm_quals_host")
        return res

    def nv_score_host(self, aligner: "NvAligner", patterns: "PackedSet", texts: "PackedSet", int16=False):
        """nvbio-style batched scores (gasalx_nv_score_host): patterns[i] against texts[i]
        (or the one shared text).  int16: also return sw-benchmark's int16 score vector."""
        n = patterns.n
        sc = np.zeros(n, np.int32)
        s16 = np.zeros(n, np.int16) if int16 else None
        ca = aligner.cstruct()
        _check(lib().gasalx_nv_score_host(self._h, ctypes.byref(ca), ctypes.c_uint32(n),
                                          ctypes.byref(patterns.cstruct()), ctypes.c_uint64(len(patterns.words)),
                                          ctypes.byref(texts.cstruct()), ctypes.c_uint64(len(texts.words)), _p(sc),
                                          _p(s16)), "nv_score_host")
        return (sc, s16) if int16 else sc

    def nv_banded_score_host(self, aligner: "NvAligner", band: int, patterns: "PackedSet", texts: "PackedSet"):
        """nvbio BatchedBandedAlignmentScore<band> (gasalx_nv_banded_score_host): BestSink
        score per pair, INT32_MIN where a text is shorter than its pattern."""
        n = patterns.n
        sc = np.zeros(n, np.int32)
        ca = aligner.cstruct()
        _check(lib().gasalx_nv_banded_score_host(self._h, ctypes.byref(ca), ctypes.c_uint32(band), ctypes.c_uint32(n),
                                                 ctypes.byref(patterns.cstruct()),
                                                 ctypes.c_uint64(len(patterns.words)), ctypes.byref(texts.cstruct()),
                                                 ctypes.c_uint64(len(texts.words)), _p(sc)), "nv_banded_score_host")
        return sc

    def nv_traceback_host(self, aligner: "NvAligner", patterns: "PackedSet", texts: "PackedSet"):
        """nvbio BatchedAlignmentTraceback (gasalx_nv_traceback_host): per pair the BestSink score, the
        Alignment's source and sink ((x, y) = (text, pattern)) and the backtracker's pushes in push
        order (0 'M', 1 'I', 2 'D') -- the dict oracle.nv_traceback returns."""
        n = patterns.n
        po = np.asarray(patterns.offsets, np.int64)
        plen = po[1:] - po[:-1]
        if texts.offsets is not None:
            to = np.asarray(texts.offsets, np.int64)
            tlen = to[1:] - to[:-1]
        else:
            tlen = np.full(n, int(texts.length), np.int64)
        stride = int(plen.max(initial=0) + tlen.max(initial=0))
        sc = np.zeros(n, np.int32)
        src = np.zeros(2 * n, np.uint32)
        snk = np.zeros(2 * n, np.uint32)
        ops = np.zeros(max(n * stride, 1), np.uint8)
        nops = np.zeros(n, np.uint32)
        ca = aligner.cstruct()
        _check(lib().gasalx_nv_traceback_host(self._h, ctypes.byref(ca), ctypes.c_uint32(n),
                                              ctypes.byref(patterns.cstruct()), ctypes.c_uint64(len(patterns.words)),
                                              ctypes.byref(texts.cstruct()), ctypes.c_uint64(len(texts.words)),
                                              _p(sc), _p(src), _p(snk), _p(ops), ctypes.c_uint32(stride), _p(nops)),
               "nv_traceback_host")
        return dict(score=sc, source=src.reshape(n, 2), sink=snk.reshape(n, 2),
                    ops=[ops[k * stride:k * stride + int(nops[k])].copy() for k in range(n)])

    def nv_traceback_device_ptrs(self, aligner: "NvAligner", n: int, pat: dict, txt: dict, outs: dict,
                                 ops_stride: int, max_pattern_len: int = 0, max_text_len: int = 0, stream: int = 0):
        """Device-resident traceback (gasalx_nv_traceback_device); pat/txt as nv_score_device_ptrs, outs =
        {"score", "source", "sink", "ops", "n_ops"} device addresses."""
        mk = lambda d: CNvStrings(d["words"], d.get("offsets") or None, d.get("length", 0), d["bits"],
                                  int(d.get("big_endian", False)))
        ca = aligner.cstruct()
        v = lambda k: ctypes.c_void_p(outs[k] or None)
        _check(lib().gasalx_nv_traceback_device(self._h, ctypes.byref(ca), ctypes.c_uint32(n), ctypes.byref(mk(pat)),
                                                ctypes.byref(mk(txt)), ctypes.c_uint32(max_pattern_len),
                                                ctypes.c_uint32(max_text_len), v("score"), v("source"), v("sink"),
                                                v("ops"), ctypes.c_uint32(ops_stride), v("n_ops"),
                                                ctypes.c_void_p(stream or None)), "nv_traceback_device")

    def nv_banded_traceback_host(self, aligner: "NvAligner", band: int, patterns: "PackedSet", texts: "PackedSet"):
        """nvbio BatchedBandedAlignmentTraceback<band> (gasalx_nv_banded_traceback_host): the dict
        oracle.nv_banded_traceback returns."""
        n = patterns.n
        po = np.asarray(patterns.offsets, np.int64)
        stride = 2 * int((po[1:] - po[:-1]).max(initial=0)) + int(band)
        sc = np.zeros(n, np.int32)
        src = np.zeros(2 * n, np.uint32)
        snk = np.zeros(2 * n, np.uint32)
        ops = np.zeros(max(n * stride, 1), np.uint8)
        nops = np.zeros(n, np.uint32)
        ca = aligner.cstruct()
        _check(lib().gasalx_nv_banded_traceback_host(self._h, ctypes.byref(ca), ctypes.c_uint32(band), ctypes.c_uint32(n),
                                                     ctypes.byref(patterns.cstruct()), ctypes.c_uint64(len(patterns.words)),
                                                     ctypes.byref(texts.cstruct()), ctypes.c_uint64(len(texts.words)),
                                                     _p(sc), _p(src), _p(snk), _p(ops), ctypes.c_uint32(stride), _p(nops)),
               "nv_banded_traceback_host")
        return dict(score=sc, source=src.reshape(n, 2), sink=snk.reshape(n, 2),
                    ops=[ops[k * stride:k * stride + int(nops[k])].copy() for k in range(n)])

    def nv_banded_traceback_device_ptrs(self, aligner: "NvAligner", band: int, n: int, pat: dict, txt: dict,
                                        outs: dict, ops_stride: int, max_pattern_len: int = 0, stream: int = 0):
        """Device-resident banded traceback (gasalx_nv_banded_traceback_device); arguments as
        nv_traceback_device_ptrs."""
        mk = lambda d: CNvStrings(d["words"], d.get("offsets") or None, d.get("length", 0), d["bits"],
                                  int(d.get("big_endian", False)))
        ca = aligner.cstruct()
        v = lambda k: ctypes.c_void_p(outs[k] or None)
        _check(lib().gasalx_nv_banded_traceback_device(self._h, ctypes.byref(ca), ctypes.c_uint32(band), ctypes.c_uint32(n),
                                                       ctypes.byref(mk(pat)), ctypes.byref(mk(txt)),
                                                       ctypes.c_uint32(max_pattern_len), v("score"), v("source"),
                                                       v("sink"), v("ops"), ctypes.c_uint32(ops_stride), v("n_ops"),
                                                       ctypes.c_void_p(stream or None)), "nv_banded_traceback_device")

    def nv_banded_score_device_ptrs(self, aligner: "NvAligner", band: int, n: int, pat: dict, txt: dict,
                                    scores_ptr: int, stream: int = 0, max_pattern_len: int = 0):
        """Device-resident banded scoring (gasalx_nv_banded_score_device); pat/txt as nv_score_device_ptrs."""
        mk = lambda d: CNvStrings(d["words"], d.get("offsets") or None, d.get("length", 0), d["bits"],
                                  int(d.get("big_endian", False)))
        ca = aligner.cstruct()
        _check(lib().gasalx_nv_banded_score_device(self._h, ctypes.byref(ca), ctypes.c_uint32(band), ctypes.c_uint32(n),
                                                   ctypes.byref(mk(pat)), ctypes.byref(mk(txt)),
                                                   ctypes.c_void_p(scores_ptr or None), ctypes.c_uint32(max_pattern_len),
                                                   ctypes.c_void_p(stream or None)),
               "nv_banded_score_device")

    def nv_score_device_ptrs(self, aligner: "NvAligner", n: int, pat: dict, txt: dict, scores_ptr: int = 0,
                             scores16_ptr: int = 0, max_pattern_len: int = 0, max_text_len: int = 0, stream: int = 0):
        """Device-resident nvbio-style scoring: pat/txt = {"words": ptr, "offsets": ptr or 0, "length": int,
        "bits": int, "big_endian": bool} with device addresses."""
        mk = lambda d: CNvStrings(d["words"], d.get("offsets") or None, d.get("length", 0), d["bits"],
                                  int(d.get("big_endian", False)))
        ca = aligner.cstruct()
        _check(lib().gasalx_nv_score_device(self._h, ctypes.byref(ca), ctypes.c_uint32(n), ctypes.byref(mk(pat)),
                                            ctypes.byref(mk(txt)), ctypes.c_void_p(scores_ptr or None),
                                            ctypes.c_void_p(scores16_ptr or None), ctypes.c_uint32(max_pattern_len),
                                            ctypes.c_uint32(max_text_len), ctypes.c_void_p(stream or None)),
               "nv_score_device")

    def pairhmm_device_ptrs(self, ptrs: dict, read_bytes: int, hap_bytes: int, n: int, max_r: int, max_h: int,
                            result_ptr: int, stream: int = 0):
        g = lambda k: ptrs.get(k) or None
        hb = CHmmBatch(g("reads"), g("read_offsets"), g("read_lens"), g("qm"), g("delta"), g("xiksi"), g("alpha"),
                       g("haps"), g("hap_offsets"), g("hap_lens"), read_bytes, hap_bytes, n, max_r, max_h)
        _check(lib().gasalx_pairhmm_device(self._h, ctypes.byref(hb), ctypes.c_void_p(result_ptr),
                                           ctypes.c_void_p(stream or None)), "pairhmm_device")


def shard_bounds(a, b, world: int) -> list:
    """gasalx_shard_bounds: contiguous [start, end) ranges balancing sum(a[i] * b[i])."""
    a = np.ascontiguousarray(a, np.uint32)
    b = np.ascontiguousarray(b, np.uint32)
    out = np.zeros(world + 1, np.uint32)
    _check(lib().gasalx_shard_bounds(_p(a), _p(b), ctypes.c_uint32(len(a)), world, _p(out)), "shard_bounds")
    return [(int(out[k]), int(out[k + 1])) for k in range(world)]


class Multi:
    """A multi-GPU group (gasalx_multi): one engine per device entry, host batches split
    into cell-balanced contiguous shards with one host thread per entry."""

    def __init__(self, devices, rccl: bool = False):
        devs = (ctypes.c_int * len(devices))(*devices)
        self.devices = list(devices)
        self._h = ctypes.c_void_p()
        _check(lib().gasalx_multi_create(devs, len(devices), MULTI_RCCL if rccl else 0, ctypes.byref(self._h)),
               "multi_create")

    def close(self):
        if self._h:
            lib().gasalx_multi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def uses_rccl(self) -> bool:
        n, r = ctypes.c_int(), ctypes.c_int()
        _check(lib().gasalx_multi_info(self._h, ctypes.byref(n), ctypes.byref(r)), "multi_info")
        return bool(r.value)

    def align_host(self, batch: "Batch", params: "Params", q_ops=None, t_ops=None, seed_scores=None, fields=None):
        n = batch.n
        out = {k: np.full(n, SENTINEL, np.int32) for k in (OUT_FIELDS if fields is None else fields)}
        tb = params.start_pos == WITH_TB
        cigar = np.zeros(batch.q_bytes if tb else 0, np.uint8)
        n_ops = np.zeros(n if tb else 0, np.uint32)
        qo = None if q_ops is None else np.ascontiguousarray(q_ops, np.uint8)
        to = None if t_ops is None else np.ascontiguousarray(t_ops, np.uint8)
        sd = None if seed_scores is None else np.ascontiguousarray(seed_scores, np.uint32)
        cb = CBatch(_p(batch.q_data), _p(batch.q_offsets), _p(batch.q_lens), _p(batch.t_data), _p(batch.t_offsets),
                    _p(batch.t_lens), batch.q_bytes, batch.t_bytes, n, _p(qo), _p(to), _p(sd), 0, 0)
        cr = CResults(*(_p(out[k]) if k in out else None for k in OUT_FIELDS), _p(cigar) if tb else None,
                      _p(n_ops) if tb else None)
        _check(lib().gasalx_multi_align_host(self._h, ctypes.byref(params), ctypes.byref(cb), ctypes.byref(cr)),
               "multi_align_host")
        out["cigar"] = cigar
        out["n_ops"] = n_ops
        return out

    def pairhmm_host(self, reads, read_off, read_len, qm, delta, xiksi, alpha, haps, hap_off, hap_len):
        c = lambda a, t: np.ascontiguousarray(a, t)
        reads, haps = c(reads, np.uint8), c(haps, np.uint8)
        arrs = [c(read_off, np.uint32), c(read_len, np.uint32), c(qm, np.float32), c(delta, np.float32),
                c(xiksi, np.float32), c(alpha, np.float32), c(hap_off, np.uint32), c(hap_len, np.uint32)]
        n = len(arrs[1])
        res = np.zeros(n, np.float32)
        hb = CHmmBatch(_p(reads), _p(arrs[0]), _p(arrs[1]), _p(arrs[2]), _p(arrs[3]), _p(arrs[4]), _p(arrs[5]),
                       _p(haps), _p(arrs[6]), _p(arrs[7]), len(reads), len(haps), n, 0, 0)
        _check(lib().gasalx_multi_pairhmm_host(self._h, ctypes.byref(hb), _p(res)), "multi_pairhmm_host")
        return res

    def pairhmm_quals_host(self, hmm: "HmmData"):
        res = np.zeros(hmm.n, np.float32)
        hb = hmm.cstruct()
        _check(lib().gasalx_multi_pairhmm_quals_host(self._h, ctypes.byref(hb), _p(res)), "multi_pairhmm_quals_host")
        return res

    def align_device_ptrs(self, params: "Params", shards, streams=None, gather=None, gather_stride: int = 0):
        """Device-resident shards (gasalx_multi_align_device): shards[i] is a dict as
        Engine.align_device_ptrs takes (integer device addresses on entry i's device) plus "q_bytes",
        "t_bytes", "n", "max_q", "max_t"; gather: one receive address per entry (world x
        gather_stride int32) or None."""
        k = len(self.devices)
        if len(shards) != k:
            raise ValueError("one shard per device entry")
        g = lambda d, key: d.get(key) or None
        cbs = (CBatch * k)(*[CBatch(g(d, "q_batch"), g(d, "q_offsets"), g(d, "q_lens"), g(d, "t_batch"),
                                    g(d, "t_offsets"), g(d, "t_lens"), d["q_bytes"], d["t_bytes"], d["n"],
                                    g(d, "q_ops"), g(d, "t_ops"), g(d, "seed_scores"), d.get("max_q", 0),
                                    d.get("max_t", 0)) for d in shards])
        crs = (CResults * k)(*[CResults(g(d, "aln_score"), g(d, "q_end"), g(d, "t_end"), g(d, "q_start"),
                                        g(d, "t_start"), g(d, "aln_score2"), g(d, "q_end2"), g(d, "t_end2"),
                                        g(d, "cigar"), g(d, "n_cigar_ops")) for d in shards])
        sts = None if streams is None else (ctypes.c_void_p * k)(*streams)
        gat = None if gather is None else (ctypes.c_void_p * k)(*gather)
        _check(lib().gasalx_multi_align_device(self._h, ctypes.byref(params), cbs, crs, sts, gat,
                                               ctypes.c_uint32(gather_stride)), "multi_align_device")

    def pairhmm_device_ptrs(self, shards, streams=None, gather=None, gather_stride: int = 0):
        """Device-resident PairHMM shards (gasalx_multi_pairhmm_device): shards[i] holds the device
        addresses of Engine.pairhmm_device_ptrs's arrays plus "result", "read_bytes", "hap_bytes",
        "n", "max_r", "max_h"."""
        k = len(self.devices)
        if len(shards) != k:
            raise ValueError("one shard per device entry")
        g = lambda d, key: d.get(key) or None
        hbs = (CHmmBatch * k)(*[CHmmBatch(g(d, "reads"), g(d, "read_offsets"), g(d, "read_lens"), g(d, "qm"),
                                          g(d, "delta"), g(d, "xiksi"), g(d, "alpha"), g(d, "haps"),
                                          g(d, "hap_offsets"), g(d, "hap_lens"), d["read_bytes"], d["hap_bytes"],
                                          d["n"], d.get("max_r", 0), d.get("max_h", 0)) for d in shards])
        res = (ctypes.c_void_p * k)(*[d["result"] for d in shards])
        sts = None if streams is None else (ctypes.c_void_p * k)(*streams)
        gat = None if gather is None else (ctypes.c_void_p * k)(*gather)
        _check(lib().gasalx_multi_pairhmm_device(self._h, hbs, res, sts, gat, ctypes.c_uint32(gather_stride)),
               "multi_pairhmm_device")

    def allgather_ptrs(self, send_ptrs, recv_ptrs, nbytes: int, streams=None):
        """Device buffers (integer addresses), one send and one recv per entry."""
        k = len(self.devices)
        snd = (ctypes.c_void_p * k)(*send_ptrs)
        rcv = (ctypes.c_void_p * k)(*recv_ptrs)
        sts = None if streams is None else (ctypes.c_void_p * k)(*streams)
        _check(lib().gasalx_multi_allgather(self._h, snd, rcv, ctypes.c_uint64(nbytes), sts), "multi_allgather")


def synth_spec(kind: int):
    """(query length, target length) of a synthetic workload (all pairs alike)."""
    q, t = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().gasalx_synth_spec(kind, ctypes.byref(q), ctypes.byref(t)), "synth_spec")
    return q.value, t.value


def describe_plan(params: Params, max_q: int, max_t: int) -> str:
    buf = ctypes.create_string_buffer(128)
    _check(lib().gasalx_describe_plan(ctypes.byref(params), max_q, max_t, buf, 128), "describe_plan")
    return buf.value.decode()


def nv_describe_plan(aligner: "NvAligner", max_p: int, max_t: int, per_pair_texts: bool = False,
                     text_bits: int = 2) -> str:
    buf = ctypes.create_string_buffer(128)
    al = aligner.cstruct()
    _check(lib().gasalx_nv_describe_plan(ctypes.byref(al), max_p, max_t, int(per_pair_texts), text_bits, buf, 128),
           "nv_describe_plan")
    return buf.value.decode()


@dataclass
class HmmData:
    """PairHMM pairs in the reference's input terms: reads with base / insertion /
    deletion / gcp qualities and haplotypes (tile_1.cu:246-290)."""
    reads: np.ndarray
    read_offsets: np.ndarray
    read_lens: np.ndarray
    base_quals: np.ndarray
    ins_quals: np.ndarray
    del_quals: np.ndarray
    gcp_quals: np.ndarray
    haps: np.ndarray
    hap_offsets: np.ndarray
    hap_lens: np.ndarray
    group_sizes: np.ndarray

    @property
    def n(self):
        return len(self.read_lens)

    def cstruct(self) -> CHmmQualBatch:
        return CHmmQualBatch(_p(self.reads), _p(self.read_offsets), _p(self.read_lens), _p(self.base_quals),
                             _p(self.ins_quals), _p(self.del_quals), _p(self.haps), _p(self.hap_offsets),
                             _p(self.hap_lens), len(self.reads), len(self.haps), self.n,
                             int(self.read_lens.max(initial=0)), int(self.hap_lens.max(initial=0)))

    @classmethod
    def from_pairs(cls, pairs):
        """pairs: dicts with read, hap (str/bytes) and bq, iq, dq (, gcp) sequences."""
        enc = lambda s: s.encode() if isinstance(s, str) else bytes(s)
        reads = [enc(p["read"]) for p in pairs]
        haps = [enc(p["hap"]) for p in pairs]
        rl = np.array([len(r) for r in reads], np.uint32)
        hl = np.array([len(h) for h in haps], np.uint32)
        ro = np.concatenate([[0], np.cumsum(rl, dtype=np.uint64)[:-1]]).astype(np.uint32)
        ho = np.concatenate([[0], np.cumsum(hl, dtype=np.uint64)[:-1]]).astype(np.uint32)
        q = lambda k: np.concatenate([np.asarray(p.get(k, np.zeros(len(p["read"]))), np.int64)
                                      for p in pairs]).astype(np.uint8)
        return cls(np.frombuffer(b"".join(reads), np.uint8).copy(), ro, rl, q("bq"), q("iq"), q("dq"), q("gcp"),
                   np.frombuffer(b"".join(haps), np.uint8).copy(), ho, hl, np.array([len(pairs)], np.uint32))

    def float_params(self):
        """The reference host's four per-base parameters (tile_1.cu:415-419)."""
        return pairhmm_params(self.base_quals, self.ins_quals, self.del_quals)


@dataclass
class NvAligner:
    """nvbio aligner + scoring scheme (make_gotoh_aligner / make_smith_waterman_aligner /
    make_edit_distance_aligner; SimpleGotohScheme and SimpleSmithWatermanScheme, signed)."""
    aligner: int
    type: int
    match: int = 0
    mismatch: int = 0
    gap_open: int = 0
    gap_ext: int = 0
    deletion: int = 0
    insertion: int = 0

    def cstruct(self):
        return CNvAligner(self.aligner, self.type, self.match, self.mismatch, self.gap_open, self.gap_ext,
                          self.deletion, self.insertion)

    def prm(self):
        return np.array([self.match, self.mismatch, self.gap_open, self.gap_ext, self.deletion, self.insertion],
                        np.int32)


@dataclass
class PackedSet:
    """An nvbio packed string set: `bits` per symbol, symbol 0 in the top bits of a word
    when big_endian; offsets (n + 1 symbols) or None for one shared string of `length`."""
    words: np.ndarray
    offsets: np.ndarray | None
    length: int
    bits: int
    big_endian: bool

    @property
    def n(self):
        return 0 if self.offsets is None else len(self.offsets) - 1

    def cstruct(self):
        return CNvStrings(_p(self.words), _p(self.offsets), self.length, self.bits, int(self.big_endian))

    @classmethod
    def pack(cls, seqs, bits=4, big_endian=True, shared=False):
        """seqs: sequences of symbol codes (each < 2**bits).  shared: one string (texts)."""
        seqs = [np.asarray(s, np.uint32) for s in seqs]
        lens = np.array([len(s) for s in seqs], np.uint64)
        total = int(lens.sum())
        per = 32 // bits
        flat = np.concatenate(seqs) if seqs else np.zeros(0, np.uint32)
        if flat.size and int(flat.max()) >= (1 << bits):
            raise ValueError("symbol does not fit the packing")
        idx = np.arange(total, dtype=np.uint64)
        pos = (idx % per).astype(np.uint32)
        shift = (32 - bits * (pos + 1)) if big_endian else bits * pos
        words = np.zeros((total + per - 1) // per + 1, np.uint64)
        np.add.at(words, (idx // per).astype(np.int64), flat.astype(np.uint64) << shift.astype(np.uint64))
        words = words.astype(np.uint32)
        if shared:
            return cls(words, None, total, bits, big_endian)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
        return cls(words, offs, 0, bits, big_endian)


# sw-benchmark's encodings (sw-benchmark.cu:290-330): reads as DNA_N (A0 C1 G2 T3, other 4),
# the reference through nst_nt4_table with N (and every non-ACGT byte) stored as 0
def dna_n_codes(seq) -> np.ndarray:
    b = np.frombuffer(seq.encode() if isinstance(seq, str) else bytes(seq), np.uint8)
    lut = np.full(256, 4, np.uint32)
    for i, ch in enumerate(b"ACGT"):
        lut[ch] = i
        lut[ch + 32] = i
    return lut[b]


def ref2_codes(seq) -> np.ndarray:
    c = dna_n_codes(seq)
    return np.where(c < 4, c, 0).astype(np.uint32)


def read_hmm_file(path: str) -> HmmData:
    """Parse a reference PairHMM input file with the library's native reader
    (gasalx_hmm_file_read)."""
    h = ctypes.POINTER(CHmmFile)()
    _check(lib().gasalx_hmm_file_read(os.fsencode(path), ctypes.byref(h)), "hmm_file_read")
    try:
        f = h.contents
        n, rb, hb = f.n_pairs, f.read_bytes, f.hap_bytes
        arr = lambda ptr, cnt, t: np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(t)), (cnt,)).copy() \
            if cnt else np.zeros(0, np.dtype(t))
        u8, u32 = ctypes.c_uint8, ctypes.c_uint32
        return HmmData(arr(f.reads, rb, u8), arr(f.read_offsets, n, u32), arr(f.read_lens, n, u32),
                       arr(f.base_quals, rb, u8), arr(f.ins_quals, rb, u8), arr(f.del_quals, rb, u8),
                       arr(f.gcp_quals, rb, u8), arr(f.haps, hb, u8), arr(f.hap_offsets, n, u32),
                       arr(f.hap_lens, n, u32), arr(f.group_sizes, f.n_groups, u32))
    finally:
        lib().gasalx_hmm_file_free(h)


def pairhmm_params(bq, iq, dq):
    n = len(bq)
    out = [np.zeros(n, np.float32) for _ in range(4)]
    c = lambda a: np.ascontiguousarray(a, np.uint8)
    _check(lib().gasalx_pairhmm_params(_p(c(bq)), _p(c(iq)), _p(c(dq)), ctypes.c_uint32(n), *(_p(o) for o in out)),
           "pairhmm_params")
    return out


def decode_cigar(cigar: np.ndarray, offset: int, n_ops: int) -> str:
    """Forward CIGAR text from the reversed RLE bytes, as test_prog prints it
    (Non-CDP/GASAL2/test_prog/test_prog.cpp:382-428)."""
    if n_ops == 0:
        return ""
    ops = "MXDI"
    b = cigar[offset:offset + n_ops]
    last, count = int(b[-1]) & 3, int(b[-1]) >> 2
    out = []
    for u in range(n_ops - 2, -1, -1):
        cur = int(b[u]) & 3
        if cur == last:
            count += int(b[u]) >> 2
        else:
            out.append(f"{count}{ops[last]}")
            count = int(b[u]) >> 2
        last = cur
    out.append(f"{count}{ops[last]}")
    return "".join(out)
