"""PairHMM host ingestion (CPU only): the library's native reader of the reference's
input files (gasalx_hmm_file_read) against an independent Python parse of the same
files, multi-group files, quality values that wrap through (char) and &127, and
malformed input.  Format: tile_1.cu:246-290 (inter_task/Synthetic_data/tile_1)."""
import glob
import os

import numpy as np
import pytest

import gasal_ffi as G
import helpers

FILES = sorted(glob.glob(os.path.join(helpers.GOLDEN, "pairhmm_dataset", "*.txt")) +
               glob.glob(os.path.join(helpers.GOLDEN, "pairhmm_inter_dataset", "*.txt")))


def _write_groups(path, groups):
    """groups: list of lists of pair dicts (read, hap, bq, iq, dq, gcp)."""
    with open(path, "w") as f:
        for g in groups:
            f.write(f"{len(g)}\n")
            for p in g:
                f.write(f"{len(p['read'])}\n{p['read']} ")
                for k in ("bq", "iq", "dq", "gcp"):
                    f.write(" ".join(str(int(v)) for v in p[k]) + " ")
                f.write(f"\n{len(p['hap'])}\n{p['hap']}\n")


def _rand_pairs(rng, n):
    out = []
    for _ in range(n):
        R, H = int(rng.integers(1, 300)), int(rng.integers(1, 600))
        out.append(dict(read=helpers.random_seq(rng, R).decode(), hap=helpers.random_seq(rng, H).decode(),
                        bq=rng.integers(-20, 300, R), iq=rng.integers(0, 128, R), dq=rng.integers(0, 200, R),
                        gcp=rng.integers(0, 60, R)))
    return out


def _same(d, pairs):
    assert d.n == len(pairs)
    for i, p in enumerate(pairs):
        r0, rl = int(d.read_offsets[i]), int(d.read_lens[i])
        h0, hl = int(d.hap_offsets[i]), int(d.hap_lens[i])
        assert bytes(d.reads[r0:r0 + rl]).decode() == p["read"][:rl]
        assert bytes(d.haps[h0:h0 + hl]).decode() == p["hap"][:hl]
        for k, arr in (("bq", d.base_quals), ("iq", d.ins_quals), ("dq", d.del_quals), ("gcp", d.gcp_quals)):
            # (char)value: the low 8 bits, as the reference stores them
            assert np.array_equal(arr[r0:r0 + rl], (np.asarray(p[k], np.int64) & 0xFF).astype(np.uint8)), k


@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_native_reader_matches_python_parse(path):
    d = G.read_hmm_file(path)
    _same(d, helpers.read_pairhmm_dataset(path))
    assert list(d.group_sizes) == [d.n]


def test_multi_group_file(tmp_path):
    rng = np.random.default_rng(0x4D31)
    groups = [_rand_pairs(rng, 3), _rand_pairs(rng, 1), _rand_pairs(rng, 5)]
    path = tmp_path / "groups.txt"
    _write_groups(path, groups)
    d = G.read_hmm_file(str(path))
    assert list(d.group_sizes) == [3, 1, 5]
    _same(d, [p for g in groups for p in g])
    # the parameters the kernels form from these bytes (q & 127, tile_1.cu:415-419)
    qm, de, xi, al = d.float_params()
    ph2pr = np.array([np.float32(10.0) ** np.float32(-i / 10.0) for i in range(128)], np.float32)
    assert np.allclose(qm, ph2pr[d.base_quals & 127], rtol=1e-6)


@pytest.mark.parametrize("text,err", [("1\n4\nACGT 1 2 3\n", "missing quality"),
                                      ("1\n4\nAC 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1\n4\nACGT\n", "read shorter"),
                                      ("1\n2\nAC 1 1 1 1 1 1 1 1\n3\nAC\n", "haplotype shorter"),
                                      ("x\n", "trailing token")])
def test_malformed_files_fail_loudly(tmp_path, text, err):
    path = tmp_path / "bad.txt"
    path.write_text(text)
    with pytest.raises(RuntimeError, match=err):
        G.read_hmm_file(str(path))


def test_missing_file_fails():
    with pytest.raises(RuntimeError, match="cannot open"):
        G.read_hmm_file("/nonexistent/pairhmm.txt")
