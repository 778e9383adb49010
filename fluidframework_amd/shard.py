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


def digest(hashes: np.ndarray) -> int:
    """Order- and sharding-independent digest: sum of per-document uint64 hashes mod 2**64."""
    h = np.asarray(hashes, dtype=np.uint64)
    return int(h.sum(dtype=np.uint64)) & MASK64  # numpy uint64 sums wrap mod 2**64


def digest_limbs(d: int) -> list[int]:
    return [(d >> (16 * q)) & 0xFFFF for q in range(4)]


def limbs_digest(limbs) -> int:
    return sum(int(x) << (16 * q) for q, x in enumerate(limbs)) & MASK64


def reduce_run(dist, device, elapsed: float, messages: int, bad_docs: int, run_digest: int) -> dict:
    """Reduce one bench run over ranks: max elapsed, summed messages / bad documents / digest."""
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([messages, bad_docs] + digest_limbs(run_digest), dtype=torch.int64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    v = s.tolist()
    return {"elapsed": float(t.item()), "messages": int(v[0]), "bad_docs": int(v[1]),
            "digest": limbs_digest(v[2:6])}
