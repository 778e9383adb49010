"""Reconnect: Client.regeneratePendingOp (client.ts:917-960) -> normalizeSegmentsOnRebase
(mergeTree.ts:2352-2381, 2231-2331) and resetPendingDeltaToOps (client.ts:708-800), SURVEY.md 8f4.

Known answers from packages/dds/merge-tree/src/test/resetPendingSegmentsToOp.spec.ts: a client
("local user") makes nested local inserts (and a remove / annotate over everything), regenerates each
pending op at the head of the pending queue, and the regenerated ops (one per segment: the nested
inserts split each other) are then acked; the original-properties regressions (:194-243) check the
regenerated insert's props.  A seeded farm in the shape of client.reconnectFarm.spec.ts: the writer's
pending ops are held back while a remote writer's messages are sequenced, then regenerated and
resubmitted; the writer and an observer that applies every sequenced message must read the same text
after every round.  CPU: the oracle; -m gpu: the HIP engine's regenerate records, texts and leaves equal
the oracle's.
"""
import random

import numpy as np
import pytest

from fluidframework_amd import regen
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, options

ME = "local user"


def ins(pos, seg):
    return {"type": 0, "pos1": pos, "seg": seg}


def rem(a, b):
    return {"type": 1, "pos1": a, "pos2": b}


def ann(a, b, props):
    return {"type": 2, "pos1": a, "pos2": b, "props": props}


class Writer:
    """A TestClient that started collaborating as ME: local ops, regeneratePendingOp, and its own
    sequenced messages (makeOpMessage -> applyMsg, an ack).  Every step flushes a batch into the oracle
    (the host reads regenerate results after the batch); the batches are kept for the engine replay."""

    def __init__(self, it, newlen=False):
        self.it = it
        self.opts = options(new_length_calc=newlen)
        self.log = DocLog()
        self.log.start_collab(ME)
        self.doc = OracleDoc(self.opts)
        self.batches = []
        self.regens = []  # per batch: {record index: [(type, pos, len, offset, props dict or None)]}
        self.seq = 0
        self.events = []     # what the writer did, for the Node shim replay
        self.regen_out = []  # the regenerated ops of each reconnect
        self.flush()

    def flush(self):
        b = build_batch([self.log], self.it)
        assert self.doc.apply(b, 0) == 0
        recs = regen.records(self.doc.deltas())
        self.batches.append(b)
        self.regens.append(decoded(recs, lambda r: self.doc.regen_props(r), self.it))
        return recs

    def text(self):
        return self.doc.text()

    def local(self, op):
        self.events.append({"local": op})
        self.log.local_op(op, self.it)
        self.flush()
        return op

    def rollback(self, op):
        """Client.rollback of the newest pending op."""
        self.events.append({"rollback": op})
        self.log.rollback(op, self.it)
        self.flush()

    def regenerate(self, ops):
        """regeneratePendingOp of each op, oldest first (each takes the queue head) -> the new ops."""
        firsts = [self.log.regenerate(op) for op in ops]
        recs = self.flush()
        out = [regen.regenerated_op(op, recs, f, lambda r: regen.props_dict(self.doc.regen_props(r), self.it))
               for op, f in zip(ops, firsts)]
        self.events.append({"regen": ops})
        self.regen_out.append(out)
        return out

    def message(self, contents, client=ME, ref=None, msn=0):
        self.seq += 1
        m = {"clientId": client, "sequenceNumber": self.seq,
             "referenceSequenceNumber": self.seq - 1 if ref is None else ref,
             "minimumSequenceNumber": msn, "type": "op", "contents": contents}
        self.events.append({"msg": m})
        self.log.message(m, self.it)
        self.flush()
        return m


def decoded(recs, props_of, it):
    return {k: [(t, p, n, o, regen.props_dict(props_of(r), it) if r >= 0 else None) for t, p, n, o, r in v]
            for k, v in recs.items()}


def count_ops(op):
    return len(op["ops"]) if op.get("type") == 3 else 1


def observer_text(msgs, it, newlen=False):
    """A client that applies `msgs` as remote messages (TestClient otherClient)."""
    log = DocLog()
    log.start_collab("other user")
    for m in msgs:
        log.message(m, it)
    doc = OracleDoc(options(new_length_calc=newlen))
    assert doc.apply(build_batch([log], it), 0) == 0
    return doc.text()


def nested_inserts(w):
    return [w.local(ins(i, "hello")) for i in range(5)]  # resetPendingSegmentsToOp.spec.ts:43-49


# (name, expected regenerated op counts): the nested-insert cases of resetPendingSegmentsToOp.spec.ts:53-191
def _kat(name):
    it = Interner()
    w = Writer(it)
    ops = nested_inserts(w)
    if name == "acked insertSegment":
        msgs = [w.message(op, ref=0) for op in ops]
        return w, msgs, []
    if name == "nacked insertSegment":
        new = w.regenerate(ops)
        return w, [w.message(op) for op in new], new
    if name in ("acked removeRange", "nacked removeRange", "acked annotateRange", "nacked annotateRange"):
        msgs = [w.message(op, ref=0) for op in ops]
        n = len(w.text())
        op = w.local(rem(0, n) if "remove" in name else ann(0, n, {"foo": "bar"}))
        if name.startswith("acked"):
            return w, msgs + [w.message(op)], []
        new = w.regenerate([op])
        return w, msgs + [w.message(x) for x in new], new
    if name in ("nacked insertSegment and removeRange", "nacked insertSegment and annotateRange"):
        n = len(w.text())
        ops.append(w.local(rem(0, n) if "remove" in name else ann(0, n, {"foo": "bar"})))
        new = w.regenerate(ops)
        return w, [w.message(op) for op in new], new
    raise KeyError(name)


KATS = [("acked insertSegment", 0), ("nacked insertSegment", 9), ("acked removeRange", 0),
        ("nacked removeRange", 9), ("nacked insertSegment and removeRange", 18), ("acked annotateRange", 0),
        ("nacked annotateRange", 9), ("nacked insertSegment and annotateRange", 18)]


@pytest.mark.parametrize("kat", KATS, ids=[k[0] for k in KATS])
def test_reset_pending_kats_oracle(kat):
    name, want = kat
    w, msgs, new = _kat(name)
    # "we expect a nack op per segment since our original ops split segments" (pendingSegments.length)
    assert sum(count_ops(op) for op in new) == want
    # every regenerated op acked without an assert; an observer of the sequenced ops reads the same text
    assert w.text() == observer_text(msgs, w.it)


def test_nested_insert_text_oracle():
    """insertTextLocal(i, "hello") for i < 5 nests each insert in the previous one."""
    it = Interner()
    w = Writer(it)
    nested_inserts(w)
    assert w.text() == "hhhhhelloelloelloelloello"


def _props_kat(kind):
    """resetPendingSegmentsToOp.spec.ts:194-243 (plus the case without props: the segment's current
    properties, createInsertSegmentOp(pos, segment))."""
    it = Interner()
    w = Writer(it)
    if kind == "marker":
        op = w.local(ins(0, {"marker": {"refType": 0}, "props": {"markerId": "id", "prop1": "foo"}}))
        w.local(ann(0, 1, {"prop2": "bar"}))  # client.annotateMarker
    elif kind == "text":
        op = w.local(ins(0, {"text": "abc", "props": {"prop1": "foo"}}))
        w.local(ann(0, 3, {"prop2": "bar"}))
    else:
        op = w.local(ins(0, "abc"))
        w.local(ann(0, 3, {"prop2": "bar"}))
    new = w.regenerate([op])[0]
    w.message(ann(0, 1 if kind == "marker" else 3, {"prop2": "bar"}), ref=0)  # the acks, in queue order
    w.message(new)
    return w, new


def _zombie_kat():
    """An annotate regenerate does not re-send (its segments were removed remotely meanwhile,
    client.ts:741-755) keeps its pending key counts (pendingKeyUpdateCount is only decremented by an ack):
    a later annotate of the key from a client that had not seen the removal leaves it alone
    (segmentPropertiesManager.ts:94-104) while it still applies the other keys."""
    it = Interner()
    w = Writer(it)
    w.message(ins(0, "abcdef"), client="A")  # seq 1
    op = w.local(ann(1, 3, {"k": "w"}))
    w.message(rem(0, 4), client="A", ref=1)  # seq 2: "abcd" removed, the annotated "bc" with it
    new = w.regenerate([op])[0]
    w.message(new)  # seq 3: an empty group
    w.message(ann(2, 4, {"k": "b", "j": 1}), client="B", ref=1)  # seq 4: B never saw the removal
    return w, new


def test_regenerate_drops_removed_annotate_oracle():
    w, new = _zombie_kat()
    assert new == {"ops": [], "type": 3}
    assert w.text() == "ef"


def test_regenerated_insert_uses_original_properties_oracle():
    _, op = _props_kat("marker")
    assert op["seg"] == {"marker": {"refType": 0}, "props": {"markerId": "id", "prop1": "foo"}}
    _, op = _props_kat("text")
    assert op["seg"] == {"text": "abc", "props": {"prop1": "foo"}}
    _, op = _props_kat("plain")
    assert op["seg"] == {"text": "abc", "props": {"prop2": "bar"}}


def _wide_kat(n=300):
    """A pending remove over more segments than 256 (the engine's former pending-group ring): remote inserts
    at MSN 0 stay separate segments, the writer removes everything locally, regenerates it (one group per
    segment, resetPendingDeltaToOps) and the regenerated removes are acked."""
    it = Interner()
    w = Writer(it)
    for k in range(n):
        w.message(ins(k, "ab"[k % 2]), client="A")
    op = w.local(rem(0, n))
    w.message(ins(0, "z"), client="A", ref=w.seq)  # the writer was disconnected: a remote op first
    new = w.regenerate([op])[0]
    w.message(new)
    return w, new


def test_regenerate_wide_remove_oracle():
    w, new = _wide_kat()
    assert new["type"] == 3 and len(new["ops"]) == 300
    assert w.text() == "z"


def _farm(seed, rounds=30, newlen=False):
    """client.reconnectFarm.spec.ts's shape with one reconnecting writer: per round the writer makes local
    edits; a remote writer's messages are sequenced first (the writer was disconnected); then the writer
    regenerates its pending ops and resubmits them (or, some rounds, its original messages go through
    as sent).  Returns the writer; its text must equal the observer's after each round."""
    rnd = random.Random(seed)
    it = Interner()
    w = Writer(it, newlen)
    seen = []  # every sequenced message, for the observer
    msn = 0
    for r in range(rounds):
        ref, pending = w.seq, []
        for _ in range(rnd.randint(1, 5)):
            t = w.text()
            x = rnd.random()
            if t and x < 0.3:
                a = rnd.randrange(len(t))
                op = rem(a, min(len(t), a + rnd.randint(1, 4)))
            elif t and x < 0.5:
                a = rnd.randrange(len(t))
                op = ann(a, min(len(t), a + rnd.randint(1, 5)), {"k": rnd.randint(0, 3), "w": "me"})
            else:
                op = ins(rnd.randint(0, len(t)), "".join(rnd.choice("ABCD") for _ in range(rnd.randint(1, 4))))
            pending.append(w.local(op))
        if len(pending) > 1 and rnd.random() < 0.25:  # the newest edit is rolled back, never sent
            w.rollback(pending.pop())
        reconnect = rnd.random() < 0.75
        if not reconnect:  # the original messages are sequenced first, at their refSeq
            for op in pending:
                seen.append(w.message(op, ref=ref, msn=msn))
        for _ in range(rnd.randint(0, 5)):  # a remote writer, always caught up (refSeq = seq - 1)
            t = observer_text(seen, it, newlen)
            x = rnd.random()
            if t and x < 0.35:
                a = rnd.randrange(len(t))
                op = rem(a, min(len(t), a + rnd.randint(1, 5)))
            elif t and x < 0.55:
                a = rnd.randrange(len(t))
                op = ann(a, min(len(t), a + rnd.randint(1, 5)), {"k": rnd.randint(0, 3), "w": "remote"})
            else:
                op = ins(rnd.randint(0, len(t)), "".join(rnd.choice("xyz") for _ in range(rnd.randint(1, 3))))
            msn = max(msn, w.seq - 6)
            seen.append(w.message(op, client="remote", msn=msn))
        if reconnect and pending:  # regenerate at currentSeq and resubmit
            cur = w.seq
            for op in w.regenerate(pending):
                seen.append(w.message(op, ref=cur, msn=msn))
        assert w.text() == observer_text(seen, it, newlen), f"seed {seed} round {r}"
        w.events.append({"check": w.text()})
    return w


@pytest.mark.parametrize("newlen", [False, True], ids=["oldlen", "newlen"])
@pytest.mark.parametrize("seed", range(4))
def test_reconnect_farm_oracle(seed, newlen):
    _farm(seed, newlen=newlen)


def _engine(n, newlen=False):
    from fluidframework_amd.engine import Engine
    return Engine(n, new_length_calc=newlen, max_segments=4096, heap_entries=4096, text_units=1 << 18, prop_words=1 << 18,
                  remover_cells=1 << 14, ops_per_launch=64)


def _replay_engine(w, newlen=False):
    """The writer's batches on the engine, one at a time: every batch's regenerate records (props
    decoded) and text equal the oracle's; at the end the leaves do."""
    eng = _engine(1, newlen)
    orc = OracleDoc(w.opts)
    for k, b in enumerate(w.batches):
        eng.apply(b)
        assert orc.apply(b, 0) == 0
        st, op = eng.status(0)
        assert st == 0, f"batch {k}: status {st:#x} at op {op}"
        got = decoded(regen.records(eng.deltas(0)), lambda r: eng.props(0, r), w.it)
        assert got == w.regens[k], f"batch {k}"
        assert eng.text(0) == orc.text(), f"batch {k}"
    ge, gh = eng.export(0)
    oe, oh = orc.export()
    assert gh == oh and np.array_equal(ge, oe)


@pytest.mark.gpu
def test_reset_pending_kats_engine():
    for name, _ in KATS:
        w, _, _ = _kat(name)
        _replay_engine(w)
    for kind in ("marker", "text", "plain"):
        w, _ = _props_kat(kind)
        _replay_engine(w)
    _replay_engine(_zombie_kat()[0])  # the removed segment's props (leaf hashes) equal the oracle's
    _replay_engine(_wide_kat()[0])    # 300 regenerated groups (more than 256 pending at once)


@pytest.mark.gpu
@pytest.mark.parametrize("newlen", [False, True], ids=["oldlen", "newlen"])
def test_reconnect_farm_engine(newlen):
    for seed in range(3):
        _replay_engine(_farm(seed, newlen=newlen), newlen)


@pytest.mark.gpu
def test_reconnect_through_node_shim(tmp_path):
    """BatchReplayClient.regeneratePendingOp / applyMsg / localTransaction (fluidframework_amd/node) on the
    farm's events: the regenerated ops and the texts at every round equal the oracle's."""
    import json
    import os
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    for seed, newlen in ((0, False), (1, True)):
        w = _farm(seed, rounds=12, newlen=newlen)
        f = tmp_path / f"events{seed}.json"
        f.write_text(json.dumps({"me": ME, "newlen": newlen, "events": w.events}))
        r = subprocess.run(["node", os.path.join(here, "node", "reconnect_engine.js"), str(f)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout)
        assert res["regens"] == w.regen_out
        assert res["texts"] == [e["check"] for e in w.events if "check" in e]
