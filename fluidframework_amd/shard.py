"""Document sharding over the GPUs of one node.

Documents are independent, so the hot path has no collective: rank r owns a contiguous range of
documents and replays them on its own GPU.  The only cross-rank exchange is the final reduction of
counters and summary digests (RCCL over xGMI on the GPU box; gloo in the CPU tests).

The run digest is the sum mod 2**64 of the per-document summary hashes (FNV-1a 64 of every blob), so
it does not depend on how documents were sharded; it is reduced exactly as four 16-bit limbs.
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1


def doc_range(rank: int, world: int, docs_per_rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `docs_per_rank` documents; rank r holds [r*n, (r+1)*n)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    return rank * docs_per_rank, (rank + 1) * docs_per_rank


def strong_range(rank: int, world: int, total_docs: int) -> tuple[int, int]:
    """Strong scaling: the node's `total_docs` documents split into `world` contiguous ranges whose
    sizes differ by at most one (the LPT assignment for documents of equal cost, e.g. one synthetic
    recipe)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    base, rem = divmod(total_docs, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def doc_cost(op_counts, seg_estimate) -> np.ndarray:
    """Estimated apply cost of each document, sum over its ops of the leaves it scans (SURVEY.md 8e:
    ops x est. S): a document growing from s0 leaves by ~1 leaf per op costs ops * (s0 + ops / 2)."""
    ops = np.asarray(op_counts, dtype=np.float64)
    s0 = np.asarray(seg_estimate, dtype=np.float64)
    return ops * (s0 + ops / 2.0 + 1.0)


def lpt_assign(costs, world: int) -> list[np.ndarray]:
    """Greedy longest-processing-time assignment of documents to ranks: documents in
    decreasing cost, each to the least-loaded rank (ties: lowest rank).  Returns each rank's document
    indices in ascending order (their order in the rank's batch)."""
    import heapq

    costs = np.asarray(costs, dtype=np.float64)
    order = np.lexsort((np.arange(len(costs)), -costs))  # cost descending, index ascending
    heap = [(0.0, r) for r in range(world)]
    out: list[list[int]] = [[] for _ in range(world)]
    for d in order:
        load, r = heapq.heappop(heap)
        out[r].append(int(d))
        heapq.heappush(heap, (load + float(costs[d]), r))
    return [np.array(sorted(x), dtype=np.int64) for x in out]


def digest(hashes: np.ndarray) -> int:
    """Order- and sharding-independent digest: sum of per-document uint64 hashes mod 2**64."""
    h = np.asarray(hashes, dtype=np.uint64)
    return int(h.sum(dtype=np.uint64)) & MASK64  # numpy uint64 sums wrap mod 2**64


def digest_limbs(d: int) -> list[int]:
    return [(d >> (16 * q)) & 0xFFFF for q in range(4)]


def limbs_digest(limbs) -> int:
    return sum(int(x) << (16 * q) for q, x in enumerate(limbs)) & MASK64


def reduce_run(dist, device, elapsed: float, messages: int, bad_docs: int, run_digest: int, extra=()) -> dict:
    """Reduce one bench run over ranks: max elapsed, summed messages / bad documents / digest, and the sums
    of `extra` (integer counters, e.g. the ranks' oracle-sample counts)."""
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    extra = [int(x) for x in extra]
    s = torch.tensor([messages, bad_docs] + digest_limbs(run_digest) + extra, dtype=torch.int64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    v = s.tolist()
    return {"elapsed": float(t.item()), "messages": int(v[0]), "bad_docs": int(v[1]),
            "digest": limbs_digest(v[2:6]), "extra": [int(x) for x in v[6:]]}


def reduce_max(dist, device, values) -> list[float]:
    """Element-wise max over ranks of a few floats (e.g. the end-to-end step's phase times)."""
    import torch

    t = torch.tensor([float(x) for x in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]
