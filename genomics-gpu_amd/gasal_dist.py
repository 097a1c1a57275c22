"""Multi-GPU sharding of a GASAL2 batch.

Pairs are independent, so a batch is split into contiguous ranges of pairs
with (nearly) equal cell counts — the prefix sum of ql·tl — one range per
rank (one process per GPU).  Each rank aligns its range with its own engine;
no collective is on the data path.  The optional exchange step is one
all-gather of the per-pair int32 results (RCCL over xGMI with the "nccl"
backend on GPUs, gloo on CPU), replacing the reference's per-thread host
result buffers (test_prog.cpp:203-231) with a node-wide result array.
"""
from __future__ import annotations

import numpy as np

RESULT_FIELDS = ("score", "q_end", "t_end", "q_start", "t_start", "score2", "q_end2", "t_end2")


def cell_counts(q_lens, t_lens) -> np.ndarray:
    return np.asarray(q_lens, np.int64) * np.asarray(t_lens, np.int64)


def shard_bounds(cells: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [start, end) ranges, one per rank, balancing Σ cells.

    Boundary k is the first pair whose inclusive prefix sum reaches k/world of
    the total, so every range holds at most one pair's cells above its share."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = len(cells)
    csum = np.cumsum(np.asarray(cells, np.int64))
    total = int(csum[-1]) if n else 0
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        cuts.append(int(np.searchsorted(csum, target, side="left")) + (1 if n else 0))
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for k in range(1, len(cuts)):          # monotone (empty ranges allowed)
        cuts[k] = max(cuts[k], cuts[k - 1])
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def shard_batch(batch, rank: int, world: int):
    """This rank's pairs as a freshly packed Batch, plus its [start, end)."""
    start, end = shard_bounds(cell_counts(batch.q_lens, batch.t_lens), world)[rank]
    return batch.subset(np.arange(start, end)), start, end


def gather_results(local: dict, start: int, end: int, n_total: int, world: int, device="cpu",
                   fields=("score", "q_end", "t_end")) -> dict:
    """All-gather per-pair int32 results of every rank into full arrays.

    Shards have unequal sizes; each rank pads its slice to the largest shard
    (all_gather needs equal shapes) and the padding is dropped after."""
    import torch
    import torch.distributed as dist
    sizes = torch.tensor([end - start], dtype=torch.int64, device=device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    counts = [int(s.item()) for s in all_sizes]
    cap = max(max(counts), 1)
    nf = len(fields)
    buf = torch.zeros((nf, cap), dtype=torch.int32, device=device)
    for i, f in enumerate(fields):
        buf[i, :end - start] = torch.as_tensor(np.asarray(local[f], np.int32), device=device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    full = {f: np.empty(n_total, np.int32) for f in fields}
    pos = 0
    for r in range(world):
        part = out[r].cpu().numpy()
        for i, f in enumerate(fields):
            full[f][pos:pos + counts[r]] = part[i, :counts[r]]
        pos += counts[r]
    if pos != n_total:
        raise RuntimeError(f"gathered {pos} pairs, expected {n_total}")
    return full


def align_sharded(align_fn, batch, params, rank: int, world: int, gather: bool = True, device="cpu",
                  fields=("score", "q_end", "t_end")):
    """Shard `batch`, align this rank's part with align_fn(sub_batch, params) -> dict,
    and (optionally) all-gather the results.  align_fn is the engine's align_host
    (or align_device wrapper) in production."""
    sub, start, end = shard_batch(batch, rank, world)
    local = align_fn(sub, params) if sub.n else {f: np.zeros(0, np.int32) for f in fields}
    if not gather:
        return local, start, end
    return gather_results(local, start, end, batch.n, world, device=device, fields=fields), 0, batch.n
