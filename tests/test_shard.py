"""Document sharding and the final cross-rank reduction (bench.py --gpus N), on CPU with gloo.

Every rank replays its own document range (here with the CPU oracle standing in for the GPU, as the
checker) and the ranks reduce counters and summary digests; the result must equal a single-process
run over all documents.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fluidframework_amd import shard
from fluidframework_amd.synth import make_cfg, tables

DOCS, OPS = 3, 120


def _digests(lo, hi):
    from oracle.oracle import generate
    cfg = make_cfg(hi - lo, OPS, writers=4, max_lag=8, doc_base=lo)
    _, hashes, status = generate(cfg, tables(writers=4), 0, hi - lo, threads=2)
    return hashes, status


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.doc_range(rank, world, DOCS)
    hashes, status = _digests(lo, hi)
    r = shard.reduce_run(dist, "cpu", 1.0 + rank, (hi - lo) * OPS, int((status != 0).sum()), shard.digest(hashes))
    if rank == 0:
        out.put(r)
    dist.destroy_process_group()


def test_doc_range_partitions_documents():
    ranges = [shard.doc_range(r, 4, 10) for r in range(4)]
    assert ranges == [(0, 10), (10, 20), (20, 30), (30, 40)]
    with pytest.raises(ValueError):
        shard.doc_range(4, 4, 10)


def test_digest_is_sharding_independent():
    h = np.array([2**64 - 1, 5, 2**63, 12345], dtype=np.uint64)
    whole = shard.digest(h)
    parts = (shard.digest(h[:1]) + shard.digest(h[1:])) & shard.MASK64
    assert whole == parts
    assert shard.limbs_digest(shard.digest_limbs(whole)) == whole


def test_two_ranks_gloo_match_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    r = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hashes, status = _digests(0, world * DOCS)
    assert r["messages"] == world * DOCS * OPS
    assert r["bad_docs"] == 0 and not status.any()
    assert r["elapsed"] == float(world)  # max over ranks
    assert r["digest"] == shard.digest(hashes)


def test_strong_ranges_cover_every_document_once():
    for total in (0, 1, 7, 100_000, 100_003):
        for world in (1, 2, 3, 4, 8):
            rs = [shard.strong_range(r, world, total) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def test_lpt_assignment_balances_estimated_cost():
    """Greedy LPT over Σ(ops × est. S): every document once, and the most loaded rank
    carries at most 4/3 of the optimum's bound (max(mean load, largest document))."""
    rng = np.random.default_rng(5)
    ops = rng.integers(10, 5000, size=997)
    seg = rng.integers(0, 3000, size=997)
    costs = shard.doc_cost(ops, seg)
    for world in (1, 2, 4, 8):
        parts = shard.lpt_assign(costs, world)
        allv = np.sort(np.concatenate(parts))
        assert np.array_equal(allv, np.arange(len(costs)))
        loads = np.array([costs[p].sum() for p in parts])
        bound = max(costs.sum() / world, costs.max())
        assert loads.max() <= 4 / 3 * bound + 1e-6
    # equal costs: the assignment is the equal-size split
    parts = shard.lpt_assign(np.ones(10), 4)
    assert sorted(len(p) for p in parts) == [2, 2, 3, 3]
