"""Client.applyStashedOp (merge-tree/src/client.ts:830-856), in the shape of
merge-tree/src/test/client.applyStashedOpFarm.spec.ts:23-110: a client's unsent ops are applied by a fresh client
(same starting state) as stashed ops, which puts it in the same local state; that client then regenerates them
(regeneratePendingOp, the resubmit) and their sequenced messages reach it (acks) and an observer: every client
ends with the same text, and the stash client's pending queue is empty.

CPU: the oracle (texts and pending-group counts asserted at every stage).  -m gpu: the HIP engine replays each
session batch by batch and gives the oracle's answer at every check (texts, pending counts, leaves at the end).
"""
import random

import pytest

from clients import Clients, ann, ins, rem

WRITER, STASH, OBS = "writer", "stash", "observer"


def _random_op(rng, n, i):
    k = rng.random()
    if n == 0 or k < 0.45:
        return ins(rng.randint(0, n), rng.choice(["a", "bc", "def", "\n", "gh"]) * rng.randint(1, 2))
    a = rng.randint(0, n - 1)
    b = min(n, a + rng.randint(1, 4))
    if k < 0.85:
        return rem(a, b)
    return ann(a, b, {"k": i % 3, "c": "x" if i % 2 else None})


def farm(seed, rounds=4, ops_per_round=12, group=False):
    rng = random.Random(seed)
    s = Clients([WRITER, STASH, OBS], initial="hello stashed world")
    seq = 0
    for r in range(rounds):
        ops = []
        for i in range(ops_per_round):  # the writer's unsent local ops (its stashed ops)
            op = _random_op(rng, s.length(WRITER), i)
            if group and i % 4 == 3:  # localTransaction: one GROUP op
                n2 = s.length(WRITER) + (len(op["seg"]) if op["type"] == 0 else -(op["pos2"] - op["pos1"]) if op["type"] == 1 else 0)
                op = {"type": 3, "ops": [op, _random_op(rng, n2, i + 1)]}
                for m in op["ops"]:
                    s.logs[WRITER].local_op(m, s.it)
                s.flush()
            else:
                s.local(WRITER, op)
            ops.append(op)
        metas = [s.stash(STASH, op) for op in ops]  # applyStashedOp on the fresh client
        assert [len(m) if isinstance(m, list) else 1 for m in metas] == [len(o["ops"]) if o["type"] == 3 else 1 for o in ops]
        assert s.text(STASH) == s.text(WRITER), f"round {r}: the stash client differs after applyStashedOp"
        assert s.pending(STASH) == s.pending(WRITER) > 0
        # resubmit (the spec's regeneratedStashedOps): regeneratePendingOp of every stashed op in order -- each
        # takes the pending queue's head and queues its regenerated groups at the tail -- then the regenerated
        # messages are sequenced and reach the stash client (its acks) and the observer
        regenerated = []
        for op in ops:
            for mop in (op["ops"] if op["type"] == 3 else [op]):  # (one pending group per member op)
                regenerated.append(s.regenerate(STASH, mop))
        msgs = []
        for new in regenerated:
            seq += 1
            m = s.make(STASH, new, seq)
            s.apply(STASH, m)
            s.apply(OBS, dict(m))
            msgs.append(m)
        assert s.pending(STASH) == 0
        assert s.text(STASH) == s.text(OBS)
        # the writer's session never sent its ops (the stash client resubmitted them): it rolls them back, newest
        # first, and applies the sequenced messages as remote ones
        for op in reversed(ops):
            for mop in (list(reversed(op["ops"])) if op["type"] == 3 else [op]):
                s.rollback(WRITER, mop)
        assert s.pending(WRITER) == 0
        for m in msgs:
            s.apply(WRITER, dict(m))
        assert s.text(WRITER) == s.text(STASH) == s.text(OBS), f"round {r}"
    return s


@pytest.mark.parametrize("seed,group", [(1, False), (2, False), (3, True)])
def test_stashed_op_farm_oracle(seed, group):
    farm(seed, group=group)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,group", [(1, False), (3, True)])
def test_stashed_op_farm_engine(seed, group):
    farm(seed, group=group).replay_engine()


def test_apply_stashed_op_needs_collaboration():
    """assert 0x2db: a client that is not collaborating has no pending segment group to return"""
    from fluidframework_amd.batch import DocLog, Interner

    with pytest.raises(AssertionError, match="0x2db"):
        DocLog().apply_stashed_op(ins(0, "x"), Interner())
