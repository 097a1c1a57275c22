"""Multi-GPU sharding of a GASAL2 batch.

Pairs are independent, so a batch is split into contiguous ranges of pairs
with (nearly) equal cell counts — the prefix sum of ql·tl — one range per
rank (one process per GPU).  Each rank aligns its range with its own engine;
no collective is on the data path.  The exchange step is one all-gather of the
per-pair int32 results (RCCL over xGMI with the "nccl" backend on GPUs, gloo on
CPU for tests), replacing the reference's per-thread host result buffers
(test_prog.cpp:203-231) with a node-wide result array.

The same functions serve bench.py (engine on the GPU, RCCL) and the world-size-2
gloo test (oracle as the aligner): `rank_shard` picks the rank's range of one
global batch, `synth_shard` generates exactly those pairs (gasalx_synth_range),
`ScoreGather` is the exchange step the bench times inside every step.
"""
from __future__ import annotations

import numpy as np

RESULT_FIELDS = ("score", "q_end", "t_end", "q_start", "t_start", "score2", "q_end2", "t_end2")


def cell_counts(q_lens, t_lens) -> np.ndarray:
    return np.asarray(q_lens, np.int64) * np.asarray(t_lens, np.int64)


def shard_bounds(cells: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [start, end) ranges, one per rank, balancing Σ cells.

    Boundary k is one past the first pair whose inclusive prefix sum reaches k/world
    of the total (csum·world >= total·k, in integers), so every range holds at most
    one pair's cells above its share.  The library's gasalx_shard_bounds (the
    multi-GPU C-ABI, csrc/multi.cpp) applies the same rule."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = len(cells)
    csum = np.cumsum(np.asarray(cells, np.int64))
    total = int(csum[-1]) if n else 0
    scaled = [int(c) * world for c in csum] if n and total * world >= 2 ** 62 else csum * world
    cuts = [0]
    for k in range(1, world):
        cuts.append(int(np.searchsorted(scaled, total * k, side="left")) + (1 if n else 0))
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for k in range(1, len(cuts)):          # monotone (empty ranges allowed)
        cuts[k] = max(cuts[k], cuts[k - 1])
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def rank_shard(q_lens, t_lens, rank: int, world: int) -> tuple[int, int]:
    """This rank's [start, end) of a global batch with these lengths."""
    return shard_bounds(cell_counts(q_lens, t_lens), world)[rank]


def shard_batch(batch, rank: int, world: int):
    """This rank's pairs as a batch (a view when the layout allows), plus its [start, end)."""
    start, end = rank_shard(batch.q_lens, batch.t_lens, rank, world)
    return batch.slice(start, end), start, end


def synth_shard(kind: int, n_global: int, seed: int, rank: int, world: int):
    """This rank's shard of the seeded synthetic global batch of n_global pairs
    (SURVEY.md §8(d) configs 1-4), generated on its own: (batch, start, end)."""
    import gasal_ffi as G
    ql, tl = G.synth_spec(kind)
    start, end = rank_shard(np.full(n_global, ql), np.full(n_global, tl), rank, world)
    return G.Batch.synth(kind, end - start, seed, start=start), start, end


def all_shards(n_global: int, q_len: int, t_len: int, world: int) -> list[tuple[int, int]]:
    return shard_bounds(cell_counts(np.full(n_global, q_len), np.full(n_global, t_len)), world)


class ScoreGather:
    """The exchange step: every rank's per-pair int32 (or fp32) results, padded to the
    largest shard (all_gather needs equal shapes), gathered into one [world, cap]
    tensor on every rank.  `buf` is the rank's padded result tensor; the aligner
    writes its first n_local entries in place."""

    def __init__(self, counts: list[int], world: int, device, dtype=None, backend: str = "nccl"):
        import torch
        self.counts = list(counts)
        self.world = world
        self.cap = max(max(self.counts), 1)
        dt = dtype or torch.int32
        self.buf = torch.zeros(self.cap, dtype=dt, device=device)
        self.out = torch.zeros((world, self.cap), dtype=dt, device=device)
        self._parts = list(self.out.unbind(0))
        # gloo with device tensors: stage through host memory (ranks may share a GPU)
        self._host = backend == "gloo" and self.buf.device.type != "cpu"
        if self._host:
            self._hbuf = torch.zeros(self.cap, dtype=dt)
            self._hout = torch.zeros((world, self.cap), dtype=dt)
            self._hparts = list(self._hout.unbind(0))

    def __call__(self):
        import torch.distributed as dist
        if self._host:
            self._hbuf.copy_(self.buf)
            dist.all_gather(self._hparts, self._hbuf)
            self.out.copy_(self._hout)
            return
        dist.all_gather(self._parts, self.buf)

    def full(self) -> np.ndarray:
        """The gathered results in global pair order (padding dropped)."""
        h = self.out.cpu().numpy()
        return np.concatenate([h[r, :self.counts[r]] for r in range(self.world)])


def gather_results(local: dict, start: int, end: int, n_total: int, world: int, device="cpu",
                   fields=("score", "q_end", "t_end")) -> dict:
    """All-gather per-pair int32 results of every rank into full arrays."""
    import torch
    import torch.distributed as dist
    sizes = torch.tensor([end - start], dtype=torch.int64, device=device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    counts = [int(s.item()) for s in all_sizes]
    full = {}
    for f in fields:
        g = ScoreGather(counts, world, device)
        g.buf[:end - start] = torch.as_tensor(np.asarray(local[f], np.int32), device=device)
        g()
        full[f] = g.full()
    if len(full[fields[0]]) != n_total:
        raise RuntimeError(f"gathered {len(full[fields[0]])} pairs, expected {n_total}")
    return full


def align_sharded(align_fn, batch, params, rank: int, world: int, gather: bool = True, device="cpu",
                  fields=("score", "q_end", "t_end")):
    """Shard `batch`, align this rank's part with align_fn(sub_batch, params) -> dict,
    and (optionally) all-gather the results."""
    sub, start, end = shard_batch(batch, rank, world)
    local = align_fn(sub, params) if sub.n else {f: np.zeros(0, np.int32) for f in fields}
    if not gather:
        return local, start, end
    return gather_results(local, start, end, batch.n, world, device=device, fields=fields), 0, batch.n
