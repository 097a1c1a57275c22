"""The test_prog-contract driver (tools/test_prog.cpp, a client of the drop-in
C++ API: include/gasal_header.h + -lgasal) against the oracle.

It exercises the whole reference-shaped host path — Parameters parsing,
gasal_init_streams, gasal_host_batch_fill, gasal_op_fill, gasal_aln_async,
gasal_is_aln_async_done, result buffers — and the printed output contract of
SURVEY.md §8(a) a19 (test_prog.cpp:349-430).  Expected lines are formatted
here from the oracle's results with the same rules."""
import os
import subprocess

import numpy as np
import pytest

import gasal_ffi as G
import helpers
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tools", "test_prog.out")
HEADS = "></+"


def _write_fasta(path, names, seqs, mods, lines=1):
    """The two files are read in lock step (test_prog.cpp:90-137), so a record
    must span the same number of lines in both; `lines` splits every sequence
    into that many lines."""
    with open(path, "w") as f:
        for n, s, m in zip(names, seqs, mods):
            f.write(f"{HEADS[m]}{n}\n")
            step = -(-len(s) // lines)
            for i in range(lines):
                f.write(s[i * step:(i + 1) * step] + "\n")


def _expected_lines(qn, tn, batch, o, algo, start_pos, head, second):
    starts = start_pos in (G.WITH_START, G.WITH_TB) and (
        (algo == G.SEMI_GLOBAL and head != G.NONE) or algo > G.SEMI_GLOBAL)
    out = []
    for i in range(batch.n):
        s = f"query_name={qn[i]}\ttarget_name={tn[i]}\tscore={o['score'][i]}"
        if starts:
            s += f"\tquery_batch_start={o['q_start'][i]}\ttarget_batch_start={o['t_start'][i]}"
        if algo != G.GLOBAL:
            s += f"\tquery_batch_end={o['q_end'][i]}\ttarget_batch_end={o['t_end'][i]}"
        if second:
            s += f"\t2nd_score={o['score2'][i]}\t2nd_query_batch_end={o['q_end2'][i]}" \
                 f"\t2nd_target_batch_end={o['t_end2'][i]}"
        if start_pos == G.WITH_TB:
            s += "\tCIGAR=" + G.decode_cigar(o["cigar"], int(batch.q_offsets[i]), int(o["n_ops"][i]))
        out.append(s)
    return out


def test_driver_built_and_linked():
    assert os.path.exists(DRIVER), "tools/test_prog.out not built (__graft_entry__.build())"
    r = subprocess.run([DRIVER, "-h"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "Usage" in r.stderr
    ldd = subprocess.run(["ldd", DRIVER], capture_output=True, text=True).stdout
    assert "libgasal.so" in ldd


def test_driver_rejects_bad_args():
    r = subprocess.run([DRIVER, "-y", "local", "nope.fa", "nope2.fa"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "File error" in r.stderr


CASES = [
    # (cli options, algo, start_pos, head, tail, second, n_pairs, threads, rc)
    (["-y", "local"], G.LOCAL, G.WITHOUT_START, G.TARGET, G.TARGET, False, 12000, 1, False),
    (["-y", "local", "-s"], G.LOCAL, G.WITH_START, G.TARGET, G.TARGET, False, 3000, 2, False),
    (["-y", "local", "-t"], G.LOCAL, G.WITH_TB, G.TARGET, G.TARGET, False, 3000, 1, False),
    (["-y", "local", "--second-best"], G.LOCAL, G.WITHOUT_START, G.TARGET, G.TARGET, True, 3000, 1, False),
    (["-y", "global"], G.GLOBAL, G.WITHOUT_START, G.TARGET, G.TARGET, False, 3000, 1, False),
    (["-y", "global", "-t"], G.GLOBAL, G.WITH_TB, G.TARGET, G.TARGET, False, 3000, 1, False),
    (["-y", "semi_global"], G.SEMI_GLOBAL, G.WITHOUT_START, G.TARGET, G.TARGET, False, 3000, 1, False),
    (["-y", "semi_global", "-s", "-x", "QUERY", "BOTH"], G.SEMI_GLOBAL, G.WITH_START, G.QUERY, G.BOTH, False,
     3000, 1, False),
    (["-y", "local", "-a", "2", "-b", "3", "-q", "5", "-r", "2"], G.LOCAL, G.WITHOUT_START, G.TARGET, G.TARGET,
     False, 3000, 1, False),
    (["-y", "local", "-s"], G.LOCAL, G.WITH_START, G.TARGET, G.TARGET, False, 3000, 1, True),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[" ".join(c[0]) + (" rc" if c[8] else "") for c in CASES])
def test_driver_output_contract(tmp_path, case):
    opts, algo, start_pos, head, tail, second, n, threads, rc = case
    O.build()
    q, t, _, _ = helpers.read_fasta_pairs(limit=n)
    n = len(q)
    rng = np.random.default_rng(7)
    qm = rng.integers(0, 4, n) if rc else np.zeros(n, int)
    tm = rng.integers(0, 4, n) if rc else np.zeros(n, int)
    qn = [f"q{i}_{len(q[i])}" for i in range(n)]
    tn = [f"t{i}_{len(t[i])}" for i in range(n)]
    _write_fasta(tmp_path / "q.fa", qn, q, qm, lines=1 + (n % 3))
    _write_fasta(tmp_path / "t.fa", tn, t, tm, lines=1 + (n % 3))
    score = dict(match=1, mismatch=4, gap_open=6, gap_extend=1)
    if "-a" in opts:
        score = dict(match=2, mismatch=3, gap_open=5, gap_extend=2)
    env = dict(os.environ)
    if rc:
        env["GASALX_TEST_PROG_RC"] = "1"
    cmd = [DRIVER, "-p", "-n", str(threads)] + opts + [str(tmp_path / "q.fa"), str(tmp_path / "t.fa")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    got = [ln for ln in r.stdout.split("\n") if ln]
    assert len(got) == n

    batch = G.Batch.from_pairs(q, t)
    kw = dict(algo=algo, start_pos=start_pos, head=head, tail=tail, second_best=int(second), **score)
    o = O.align(batch, O.make_params(**kw), q_ops=qm.astype(np.uint8) if rc else None,
                t_ops=tm.astype(np.uint8) if rc else None)
    want = _expected_lines(qn, tn, batch, o, algo, start_pos, head, second)
    if start_pos == G.WITH_TB:
        # a CIGAR longer than its pad8(ql) slot overwrites the neighbour's slot
        over = set(np.nonzero(o["n_ops"] > (batch.q_lens + 7) // 8 * 8)[0])
        skip = over | {i + 1 for i in over}
        want = [w for i, w in enumerate(want) if i not in skip]
        names = {qn[i] for i in skip}
        got = [g for g in got if g.split("\t")[0][len("query_name="):] not in names]
    # batches of different storages/threads may interleave; within a batch order is kept
    assert sorted(got) == sorted(want)


BOUNDARY = os.path.join(ROOT, "tools", "boundary_bench")


@pytest.mark.gpu
@pytest.mark.parametrize("threads,batch,repl", [(1, 5000, 1), (3, 5000, 2), (2, 1777, 1)])
def test_boundary_bench_results(tmp_path, threads, batch, repl):
    # tools/boundary_bench (bench.py --workload boundary): the reference's test_prog loop over the
    # 20K sample pairs (gzip FASTA read directly), replicated; its dump of the last pass's results
    # must equal the oracle on every replica of every pair, for any thread count and batch size
    O.build()
    assert os.path.exists(BOUNDARY), "tools/boundary_bench not built (__graft_entry__.build())"
    g = os.path.join(ROOT, "tests", "golden")
    dump = tmp_path / "res.bin"
    cmd = [BOUNDARY, "--repl", str(repl), "--warm", "1", "--reps", "1", "--batch", str(batch), "--dump", str(dump),
           "-y", "local", "-n", str(threads), os.path.join(g, "query_batch.fasta.gz"),
           os.path.join(g, "target_batch.fasta.gz")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    import json
    info = json.loads(line)
    q, t, _, _ = helpers.read_fasta_pairs()
    n = len(q)
    assert info["pairs"] == n * repl and info["threads"] == threads and info["gcups"] > 0
    o = O.align(G.Batch.from_pairs(q, t), O.make_params(algo=O.LOCAL))
    got = np.fromfile(dump, np.int32).reshape(5, n * repl)
    for k, f in enumerate(("score", "q_end", "t_end")):
        assert np.array_equal(got[k].reshape(repl, n), np.broadcast_to(o[f], (repl, n))), f
