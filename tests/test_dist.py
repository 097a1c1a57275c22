"""Multi-process sharding on CPU: cell-balanced contiguous
shards and the optional all-gather of per-pair results, world_size 2 over
gloo.  The per-rank aligner here is the CPU oracle (no GPU in this
container); on GPUs the same code runs with the engine and the nccl (RCCL)
backend."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import gasal_dist as D
import gasal_ffi as G
import helpers
import oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_bounds_cover_and_balance(world):
    rng = np.random.default_rng(world)
    cells = rng.integers(1, 40000, 1001).astype(np.int64)
    b = D.shard_bounds(cells, world)
    assert b[0][0] == 0 and b[-1][1] == len(cells)
    for (s0, e0), (s1, _) in zip(b, b[1:]):
        assert e0 == s1 and s0 <= e0
    share = cells.sum() / world
    for s, e in b:
        assert cells[s:e].sum() <= share + cells.max()


def test_shard_bounds_edge_cases():
    assert D.shard_bounds(np.array([], np.int64), 4) == [(0, 0)] * 4
    assert D.shard_bounds(np.array([5], np.int64), 2) in ([(0, 1), (1, 1)], [(0, 0), (0, 1)])
    with pytest.raises(ValueError):
        D.shard_bounds(np.array([1]), 0)


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(1234)
    qs, ts = helpers.random_pairs(rng, 301, 20, 160, 20, 200)
    batch = G.Batch.from_pairs(qs, ts)
    op = O.make_params(algo=O.LOCAL)
    full, s, e = D.align_sharded(lambda sub, p: O.align(sub, p, n_threads=1), batch, op, rank, world, gather=True)
    assert (s, e) == (0, batch.n)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **full)
    dist.destroy_process_group()


def test_gloo_world2_sharded_align_and_gather(tmp_path):
    O.build()
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rng = np.random.default_rng(1234)
    qs, ts = helpers.random_pairs(rng, 301, 20, 160, 20, 200)
    batch = G.Batch.from_pairs(qs, ts)
    ref = O.align(batch, O.make_params(algo=O.LOCAL))
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npz")
        for f in ("score", "q_end", "t_end"):
            assert np.array_equal(got[f], ref[f]), (r, f)


def _bench_path_worker(rank, world, port, out_dir, kind, n_global):
    """The bench's multi-GPU step on CPU: this rank's shard of one global synthetic
    batch (gasal_dist.synth_shard -> gasalx_synth_range), aligned (here by the oracle,
    on the GPU by the engine into ScoreGather.buf), then the exchange step
    (ScoreGather, the same all_gather the bench times in every step)."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ql, tl = G.synth_spec(kind)
    shards = D.all_shards(n_global, ql, tl, world)
    sub, start, end = D.synth_shard(kind, n_global, 0x5EED0000 + kind, rank, world)
    assert (start, end) == shards[rank] and sub.n == end - start
    gat = D.ScoreGather([e - s for s, e in shards], world, "cpu")
    local = O.align(sub, O.make_params(algo=O.LOCAL), n_threads=1)
    gat.buf[:sub.n] = torch.from_numpy(local["score"])
    gat()
    np.save(os.path.join(out_dir, f"g{rank}.npy"), gat.full())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,n_global", [(2, 1, 701), (3, 2, 257)])
def test_gloo_bench_shard_path(tmp_path, world, kind, n_global):
    O.build()
    mp.spawn(_bench_path_worker, args=(world, _free_port(), str(tmp_path), kind, n_global), nprocs=world, join=True)
    full = G.Batch.synth(kind, n_global, 0x5EED0000 + kind)
    ref = O.align(full, O.make_params(algo=O.LOCAL))["score"]
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"g{r}.npy"), ref), r


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_library_shard_bounds_match_python(world):
    # the multi-GPU C-ABI (gasalx_shard_bounds, csrc/multi.cpp) and gasal_dist split alike
    rng = np.random.default_rng(100 + world)
    for n in (0, 1, 7, 1000):
        ql = rng.integers(1, 400, n).astype(np.uint32)
        tl = rng.integers(1, 600, n).astype(np.uint32)
        assert G.shard_bounds(ql, tl, world) == D.shard_bounds(D.cell_counts(ql, tl), world), (n, world)
    ql = np.full(10_000_000, 150, np.uint32)
    tl = np.full(10_000_000, 182, np.uint32)
    assert G.shard_bounds(ql, tl, world) == D.all_shards(10_000_000, 150, 182, world)
