"""Pending local annotates with a combiningOp other than "rewrite" (SURVEY.md 8f4): PropertiesManager.addProperties
(merge-tree/src/segmentPropertiesManager.ts:60-157) at seq = UnassignedSequenceNumber keeps each key's pending count
and sets combine(op, previousValue, undefined, seq) (properties.ts:24-69); remote annotates leave pending keys alone
unless they combine themselves (shouldModifyKey, :94-104); the ack drops the counts (ackPendingProperties, :32-58).

Known answers from those rules: a local "incr" on an absent key is defaultValue + undefined = NaN; a local
"consensus" on an absent key is {value: undefined, seq: -1}; an unknown name keeps the previous value (or
defaultValue).  A seeded farm mixes local and remote plain / combining annotates, acks and rollbacks on two writers
and an observer.  CPU: the oracle; -m gpu: the HIP engine equals the oracle at every check (properties in key order,
texts, leaves).
"""
import random

import pytest

from clients import Clients, ann, ins

A, B = "writer-a", "writer-b"


def cann(a, b, props, co):
    op = ann(a, b, props)
    op["combiningOp"] = co
    return op


def _props(s, c, pos):
    p = s.props(c, pos)
    return dict(p) if p is not None else None


def kat_local_incr_absent():
    s = Clients([A, B], initial="abcdef")
    s.local(A, cann(1, 3, {"n": 0}, {"name": "incr", "defaultValue": 1}))
    p = _props(s, A, 1)
    assert "n" in p and p["n"] is None, p  # 1 + undefined = NaN (JSON.stringify writes it as null)
    return s


def kat_local_consensus_absent():
    s = Clients([A, B], initial="abcdef")
    s.local(A, cann(0, 2, {"c": "x"}, {"name": "consensus"}))
    assert _props(s, A, 0) == {"c": {"seq": -1}}  # {value: undefined, seq: UnassignedSequenceNumber}
    return s


def kat_unknown_name_keeps_previous():
    s = Clients([A, B], initial="abcdef")
    op = s.local(A, ann(0, 4, {"k": "v1"}))
    s.apply(A, s.make(A, op, 1))
    s.local(A, cann(0, 4, {"k": "v2"}, {"name": "max", "defaultValue": 7}))
    assert _props(s, A, 0) == {"k": "v1"}  # combine's default branch returns the current value
    s.local(A, cann(4, 6, {"z": "v2"}, {"name": "max", "defaultValue": 7}))
    assert _props(s, A, 4) == {"z": 7}  # ... or defaultValue when there is none
    return s


def kat_pending_key_blocks_plain_remote():
    s = Clients([A, B], initial="abcdef")
    op = s.local(A, cann(0, 3, {"k": 0}, {"name": "incr", "defaultValue": 1}))
    # B's plain annotate of the same key, sequenced first: A keeps its pending value
    rop = s.local(B, ann(0, 3, {"k": 5}))
    m1 = s.make(B, rop, 1)
    s.apply(B, m1)
    s.apply(A, m1)
    assert _props(s, A, 0) == {"k": None}  # (NaN)
    assert s.groups(A, 0, ref=1, client=s.logs[A].short_id(A)) == 1
    # A's own message: the ack (its value stays until another change)
    m2 = s.make(A, op, 2, ref=1)
    s.apply(A, m2)
    s.apply(B, m2)
    assert s.pending(A) == 0
    # now a plain remote annotate lands
    rop = s.local(B, ann(0, 3, {"k": "b2"}))
    m3 = s.make(B, rop, 3, ref=2)
    s.apply(B, m3)
    s.apply(A, m3)
    assert _props(s, A, 0)["k"] == "b2"
    return s


def farm(seed, rounds=6, newlen=False):
    rng = random.Random(seed)
    s = Clients([A, B, "observer"], initial="the quick brown fox", newlen=newlen)
    seq = 0
    # (no "consensus" here: a second consensus on its {value, seq: -1} object mutates it in place, which the engine
    # sends back to the TypeScript client -- kat_local_consensus_absent covers the first one)
    cos = [None, None, {"name": "incr", "defaultValue": 2}, {"name": "keep", "defaultValue": 7}]
    for r in range(rounds):
        sent = {A: [], B: []}
        for w in (A, B):
            for i in range(rng.randint(2, 5)):
                n = s.length(w)
                if rng.random() < 0.3:
                    op = s.local(w, ins(rng.randint(0, n), rng.choice(["xy", "z", "\n"])))
                else:
                    a = rng.randint(0, n - 1)
                    b = min(n, a + rng.randint(1, 5))
                    co = rng.choice(cos)
                    props = {rng.choice(["k", "m"]): rng.choice([1, 2.5, None, True])}  # ("incr" of a string: a string)
                    op = s.local(w, cann(a, b, props, co) if co else ann(a, b, props))
                sent[w].append(op)
            if rng.random() < 0.3 and sent[w]:  # roll the newest back
                s.rollback(w, sent[w].pop())
        order, qa, qb = [], list(sent[A]), list(sent[B])  # a random interleaving; each writer's ops stay in order
        while qa or qb:
            w = A if qa and (not qb or rng.random() < 0.5) else B
            order.append((w, (qa if w == A else qb).pop(0)))
        refs = {w: s.cur[w] for w in (A, B)}
        for w, op in order:
            seq += 1
            m = s.make(w, op, seq, ref=refs[w])
            for c in s.names:
                s.apply(c, dict(m))
        for c in s.names:
            for pos in range(0, s.length(c), 3):
                s.props(c, pos)
        assert s.text(A) == s.text(B) == s.text("observer")
    return s


KATS = [kat_local_incr_absent, kat_local_consensus_absent, kat_unknown_name_keeps_previous,
        kat_pending_key_blocks_plain_remote]


@pytest.mark.parametrize("kat", KATS, ids=[k.__name__ for k in KATS])
def test_local_combining_kat_oracle(kat):
    kat()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_local_combining_farm_oracle(seed):
    farm(seed)


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=[k.__name__ for k in KATS])
def test_local_combining_kat_engine(kat):
    kat().replay_engine()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,newlen", [(1, False), (2, True)])
def test_local_combining_farm_engine(seed, newlen):
    farm(seed, newlen=newlen).replay_engine()
