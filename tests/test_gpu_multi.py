"""Multi-GPU as a product path, on the hardware a test box has.

* gasalx_multi_* (csrc/multi.cpp): one process, one host thread and engine per
  device entry, cell-balanced contiguous shards, results written into disjoint
  ranges of the caller's arrays — STAR's static split
  (Non-CDP/STAR/src/cuda-nw.cu:296-367) balanced by cells.  Entries may repeat a
  device, so {0, 0} runs the exact two-thread path on one GPU; checked
  bit-exactly against the oracle (PairHMM: rtol 1e-5).
* gasalx_multi_allgather: peer copies for repeated devices, RCCL
  (ncclCommInitAll / ncclAllGather) for a list of distinct devices.
* bench.py --gpus 2 --dist-backend gloo: the one-process-per-GPU path the driver
  times (spawn -> engine -> ScoreGather exchange -> parity), with both ranks on
  device 0 (LOCAL_RANK % device_count)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import gasal_dist as D
import gasal_ffi as G
import helpers
import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def _check_all(g, o, fields):
    for f in fields:
        bad = np.flatnonzero(g[f] != o[f])
        assert bad.size == 0, f"{f}: {bad.size} mismatches, first #{bad[0]}: {g[f][bad[0]]} vs {o[f][bad[0]]}"


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_align_config4_bit_exact(devices):
    # config-4 data (150 bp reads in 182 bp windows, SEMI TARGET/TARGET), sharded over the
    # entries: every pair's outputs equal the oracle's
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET)
    b = G.Batch.synth(4, 60_000, 0x5EED0004)
    m = G.Multi(devices)
    g = m.align_host(b, G.make_params(**kw), fields=["score", "q_end", "t_end"])
    m.close()
    o = O.align(b, O.make_params(**kw))
    _check_all(g, o, ("score", "q_end", "t_end"))


def test_multi_shards_follow_shard_bounds():
    # uneven lengths: each entry's range is gasalx_shard_bounds' (== gasal_dist.shard_bounds);
    # LOCAL on the reference's sample pairs, results in input order
    qs, ts, _, _ = helpers.read_fasta_pairs(limit=6000)
    b = G.Batch.from_pairs(qs, ts)
    assert G.shard_bounds(b.q_lens, b.t_lens, 3) == D.shard_bounds(D.cell_counts(b.q_lens, b.t_lens), 3)
    m = G.Multi([0, 0, 0])
    g = m.align_host(b, G.make_params(algo=G.LOCAL), fields=["score", "q_end", "t_end"])
    m.close()
    _check_all(g, O.align(b, O.make_params(algo=G.LOCAL)), ("score", "q_end", "t_end"))


def test_multi_align_traceback_and_start():
    # CIGARs land at each shard's query byte range; WITH_START through the reverse pass
    kw = dict(algo=G.GLOBAL, start_pos=G.WITH_TB)
    b = G.Batch.synth(3, 3000, 0x5EED0003)
    m = G.Multi([0, 0])
    g = m.align_host(b, G.make_params(**kw))
    o = O.align(b, O.make_params(**kw))
    assert np.array_equal(g["score"], o["score"])
    assert np.array_equal(g["n_ops"], o["n_ops"]) and np.array_equal(g["cigar"], o["cigar"])
    kw = dict(algo=G.LOCAL, start_pos=G.WITH_START)
    b = G.Batch.synth(2, 20_000, 0x5EED0002)
    g = m.align_host(b, G.make_params(**kw))
    _check_all(g, O.align(b, O.make_params(**kw)), ("score", "q_end", "t_end", "q_start", "t_start"))
    m.close()


def test_multi_align_one_to_many_traceback_rejected():
    # WITH_TB with shards sharing query bytes (every pair uses query 0) is refused, not raced
    b = G.Batch.synth(3, 64, 0x5EED0003)
    b.q_offsets[:] = 0
    b.q_lens[:] = b.q_lens[0]
    m = G.Multi([0, 0])
    with pytest.raises(RuntimeError, match="share query bytes"):
        m.align_host(b, G.make_params(algo=G.GLOBAL, start_pos=G.WITH_TB))
    # score-only is fine with one-to-many pairing
    g = m.align_host(b, G.make_params(algo=G.GLOBAL))
    assert np.array_equal(g["score"], O.align(b, O.make_params(algo=G.GLOBAL))["score"])
    m.close()


def _hmm_pairs(rng, n):
    pairs = []
    for _ in range(n):
        H = int(rng.integers(40, 500))
        R = int(rng.integers(10, min(H, 260)))
        hap = helpers.random_seq(rng, H).decode()
        st = int(rng.integers(0, H - R + 1))
        pairs.append(dict(read=hap[st:st + R], hap=hap, bq=rng.integers(10, 41, R), iq=np.full(R, 45),
                          dq=np.full(R, 45)))
    return pairs


def test_multi_pairhmm():
    d = G.HmmData.from_pairs(_hmm_pairs(np.random.default_rng(77), 900))
    qm, de, xi, al = d.float_params()
    args = (d.reads, d.read_offsets, d.read_lens, qm, de, xi, al, d.haps, d.hap_offsets, d.hap_lens)
    m = G.Multi([0, 0])
    g = m.pairhmm_host(*args)
    gq = m.pairhmm_quals_host(d)
    m.close()
    np.testing.assert_allclose(g, O.pairhmm(*args), rtol=1e-5)
    eng = G.Engine(0)
    # the quality path sorts per shard: same bits as one engine over the whole batch
    assert np.array_equal(gq.view(np.uint32), eng.pairhmm_quals_host(d).view(np.uint32))
    eng.close()


def _gather_case(devices, rccl):
    import torch
    m = G.Multi(devices, rccl=rccl)
    k, cnt = len(devices), 5001
    send = [torch.arange(cnt, dtype=torch.int32, device=f"cuda:{d}") * (i + 3) for i, d in enumerate(devices)]
    recv = [torch.full((k * cnt,), -1, dtype=torch.int32, device=f"cuda:{d}") for d in devices]
    torch.cuda.synchronize()
    m.allgather_ptrs([s.data_ptr() for s in send], [r.data_ptr() for r in recv], cnt * 4)
    want = torch.cat([s.cpu() for s in send])
    for r in recv:
        assert torch.equal(r.cpu(), want)
    used = m.uses_rccl
    m.close()
    return used


def test_multi_allgather_peer_copies():
    assert _gather_case([0, 0], rccl=True) is False     # repeated device: no communicator, peer copies


def test_multi_allgather_rccl():
    # a communicator over the distinct devices of the box (one on a 1-GPU box: the RCCL
    # code path itself — dlopen, ncclCommInitAll, grouped ncclAllGather)
    import torch
    devs = list(range(torch.cuda.device_count()))
    assert _gather_case(devs, rccl=True) is True


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_device_count() < 2, reason="needs two distinct GPUs (ADVICE r03: the distinct-device "
                                                "shard and peer-copy paths)")
def test_multi_distinct_devices_align_and_gather():
    # distinct devices: one engine per GPU (cross-device event waits, hipMemcpyPeerAsync of the
    # results) and the allgather over a communicator of distinct devices, against the oracle
    devs = list(range(min(_device_count(), 4)))
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET)
    b = G.Batch.synth(4, 40_000, 0x5EED0004)
    m = G.Multi(devs)
    g = m.align_host(b, G.make_params(**kw), fields=["score", "q_end", "t_end"])
    m.close()
    _check_all(g, O.align(b, O.make_params(**kw)), ("score", "q_end", "t_end"))
    assert _gather_case(devs, rccl=False) is False      # peer copies between distinct devices
    assert _gather_case(devs, rccl=True) is True


def _device_entries():
    # the box's distinct devices when it has several (at most 4), else entry 0 twice
    n = _device_count()
    return list(range(min(n, 4))) if n >= 2 else [0, 0]


def test_multi_align_device_resident_shards_and_gather():
    # gasalx_multi_align_device: each entry's shard already in its device's
    # memory, one stream per entry, then the score gather in the same call; every shard's outputs
    # and every entry's gathered scores against the oracle
    import torch
    devs = _device_entries()
    k = len(devs)
    kw = dict(algo=G.SEMI_GLOBAL, head=G.TARGET, tail=G.TARGET)
    b = G.Batch.synth(4, 50_001, 0x5EED0004)
    o = O.align(b, O.make_params(**kw))
    bounds = G.shard_bounds(b.q_lens, b.t_lens, k)
    stride = max(e - s for s, e in bounds)
    m = G.Multi(devs, rccl=True)
    keep, shards, gat, streams = [], [], [], []
    for (s, e), d in zip(bounds, devs):
        sb = b.slice(s, e)
        dev = f"cuda:{d}"
        t = {"q_batch": torch.from_numpy(sb.q_data).to(dev), "t_batch": torch.from_numpy(sb.t_data).to(dev)}
        for f in ("q_offsets", "t_offsets", "q_lens", "t_lens"):
            t[f] = torch.from_numpy(getattr(sb, f).view(np.int32).copy()).to(dev)
        t["aln_score"] = torch.full((stride,), -7, dtype=torch.int32, device=dev)
        t["q_end"] = torch.empty(e - s, dtype=torch.int32, device=dev)
        t["t_end"] = torch.empty(e - s, dtype=torch.int32, device=dev)
        g = torch.full((k * stride,), -1, dtype=torch.int32, device=dev)
        st = torch.cuda.Stream(dev)
        keep.append((t, g, st))
        shard = {f: v.data_ptr() for f, v in t.items()}
        shard.update(q_bytes=sb.q_bytes, t_bytes=sb.t_bytes, n=e - s, max_q=int(sb.q_lens.max()),
                     max_t=int(sb.t_lens.max()))
        shards.append(shard)
        gat.append(g.data_ptr())
        streams.append(st.cuda_stream)
    torch.cuda.synchronize()
    m.align_device_ptrs(G.make_params(**kw), shards, gather=gat, gather_stride=stride)   # synchronous
    m.align_device_ptrs(G.make_params(**kw), shards, streams=streams, gather=gat, gather_stride=stride)
    for st in streams:
        torch.cuda.ExternalStream(st).synchronize()
    want = np.full(k * stride, -7, np.int32)
    for i, (s, e) in enumerate(bounds):
        t = keep[i][0]
        for f, name in (("score", "aln_score"), ("q_end", "q_end"), ("t_end", "t_end")):
            assert np.array_equal(t[name][:e - s].cpu().numpy(), o[f][s:e]), (i, f)
        want[i * stride:i * stride + (e - s)] = o["score"][s:e]
    for i in range(k):
        assert np.array_equal(keep[i][1].cpu().numpy(), want), f"gather at entry {i}"
    m.close()


def test_multi_pairhmm_device_resident_shards_and_gather():
    import torch
    devs = _device_entries()
    k = len(devs)
    d = G.HmmData.from_pairs(_hmm_pairs(np.random.default_rng(78), 700))
    qm, de, xi, al = d.float_params()
    ref = O.pairhmm(d.reads, d.read_offsets, d.read_lens, qm, de, xi, al, d.haps, d.hap_offsets, d.hap_lens)
    bounds = G.shard_bounds(d.read_lens, d.hap_lens, k)
    stride = max(e - s for s, e in bounds)
    m = G.Multi(devs)
    keep, shards, gat = [], [], []
    for (s, e), dv in zip(bounds, devs):
        dev = f"cuda:{dv}"
        r0, r1 = int(d.read_offsets[s]), int(d.read_offsets[e - 1] + d.read_lens[e - 1])
        h0, h1 = int(d.hap_offsets[s]), int(d.hap_offsets[e - 1] + d.hap_lens[e - 1])
        u = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        t = {"reads": u(d.reads[r0:r1]), "haps": u(d.haps[h0:h1]),
             "read_offsets": u((d.read_offsets[s:e] - r0).astype(np.int32)), "read_lens": u(d.read_lens[s:e].view(np.int32)),
             "hap_offsets": u((d.hap_offsets[s:e] - h0).astype(np.int32)), "hap_lens": u(d.hap_lens[s:e].view(np.int32)),
             "qm": u(qm[r0:r1]), "delta": u(de[r0:r1]), "xiksi": u(xi[r0:r1]), "alpha": u(al[r0:r1]),
             "result": torch.full((stride,), -1.0, dtype=torch.float32, device=dev)}
        g = torch.full((k * stride,), -2.0, dtype=torch.float32, device=dev)
        keep.append((t, g))
        shard = {f: v.data_ptr() for f, v in t.items()}
        shard.update(read_bytes=r1 - r0, hap_bytes=h1 - h0, n=e - s)
        shards.append(shard)
        gat.append(g.data_ptr())
    torch.cuda.synchronize()
    m.pairhmm_device_ptrs(shards, gather=gat, gather_stride=stride)
    for i, (s, e) in enumerate(bounds):
        np.testing.assert_allclose(keep[i][0]["result"][:e - s].cpu().numpy(), ref[s:e], rtol=1e-5)
    g0 = keep[0][1].cpu().numpy()
    for i in range(k):
        assert np.array_equal(keep[i][1].cpu().numpy().view(np.uint32), g0.view(np.uint32)), f"gather at entry {i}"
        s, e = bounds[i]
        np.testing.assert_allclose(g0[i * stride:i * stride + e - s], ref[s:e], rtol=1e-5)
    m.close()


@pytest.mark.parametrize("workload,pairs,checked,world,warm", [("semi", 200_000, 200_000, 2, "1"),
                                                               ("nw_tb", 20_000, 40_000, 2, "1"),
                                                               ("pairhmm", 8_000, 16_000, 2, "1"),
                                                               ("semi", 200_000, 200_000, 4, "1"),
                                                               ("semi", 200_000, 200_000, 2, None)])
def test_bench_ranks_gloo_one_gpu(workload, pairs, checked, world, warm):
    # the exact N-rank bench path on one device: torch.distributed.run spawns the ranks, each
    # aligns its cell-balanced shard into ScoreGather.buf, the gloo exchange runs in every
    # timed step, and rank 0 checks the gathered scores of every rank against the oracle.
    # nw_tb runs several engines on their own streams per rank (its default), each with its own
    # exchange buffers; pairhmm gathers fp32 results (config 5, "1 -> 8 GPUs"); semi at world 4.
    # warm None: the default time-based warmup, whose stop decision the ranks take together
    # (each rank's own clock could leave the ranks in different collectives)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
           "--workload", workload, "--pairs", str(pairs), "--steps", "3", "--no-e2e"]
    cmd += ["--warmup", warm] if warm else ["--warmup-seconds", "0.3"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(lines[-1])
    assert out["n_gpus"] == world and out["config"]["dist_backend"] == "gloo"
    par = out["parity"]
    assert par["mismatches"] == 0 and par["pairs_checked"] == checked      # nw_tb: pairs per rank (weak)
    assert par["gathered_mismatches"] == 0 and par["gathered_scores_checked"] == checked
