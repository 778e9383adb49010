"""Rollback of pending local ops: Client.rollback -> MergeTree.rollback
(client.ts:421-423, mergeTree.ts:2049-2159).

Known answers transcribed from packages/dds/merge-tree/src/test/client.rollback.spec.ts: a client that
started collaborating ("localUser") makes local ops, rolls the newest back (optionally after acking
others: TestClient.makeOpMessage's messages carry the client's own id, so applyMsg acks them), and the
text must read as the test expects.  CPU: the oracle; -m gpu: the HIP engine against the same texts and
the oracle's leaves (tree levels, removal info, property hashes) and V1 summaries.  A seeded farm rolls
back random local edits among remote messages: the text must equal a client that never made them.
"""
import random

import numpy as np
import pytest

from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, options

ME = "localUser"
TEXT = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789!@#$%^&*()"


def ins(pos, text, props=None):
    return {"type": 0, "pos1": pos, "seg": {"text": text, "props": props} if props else text}


def rem(a, b):
    return {"type": 1, "pos1": a, "pos2": b}


def ann(a, b, props):
    return {"type": 2, "pos1": a, "pos2": b, "props": props}


# (name, steps, expected text); a step is ("op", op) a local op, ("rb", op) rollback of the newest
# pending op (op = its contents), ("ack", op) a local op acked at once (applyMsg(makeOpMessage(...)))
ROLLBACK_KATS = [
    ("insert on empty string", [("op", ins(0, "abcd")), ("rb", ins(0, "abcd"))], ""),
    ("insert and partial lengths",
     [("op", ins(0, "ghi")), ("op", ins(0, "def")), ("op", ins(0, "abc")), ("rb", ins(0, "abc"))], "defghi"),
    ("insert twice and partial lengths",
     [("op", ins(0, "ghi")), ("op", ins(0, "def")), ("op", ins(0, "abc")), ("rb", ins(0, "abc")),
      ("rb", ins(0, "def"))], "ghi"),
    ("multiple inserts with split segments",
     [("op", ins(0, "aefg")), ("op", ins(1, "bd")), ("op", ins(2, "c")), ("rb", ins(2, "c")), ("rb", ins(1, "bd"))],
     "aefg"),
    ("annotate causes split string",
     [("op", ins(0, "abcdefg")), ("op", ann(1, 3, {"foo": "bar"})), ("rb", ann(1, 3, {"foo": "bar"}))], "abcdefg"),
    ("annotate over split string",
     [("op", ins(0, "abfg")), ("op", ins(1, "cde")), ("op", ann(1, 6, {"foo": "bar"})),
      ("rb", ann(1, 6, {"foo": "bar"}))], "acdebfg"),
    ("annotate that later gets split",
     [("op", ins(0, "abfg")), ("op", ann(0, 4, {"foo": "bar"})), ("op", ins(1, "cde")), ("rb", ins(1, "cde")),
      ("rb", ann(0, 4, {"foo": "bar"}))], "abfg"),
    ("annotates with multiple previous property sets",
     [("op", ins(0, "acde")), ("op", ann(0, 3, {"foo": "one"})), ("op", ann(2, 4, {"foo": "two"})),
      ("op", ann(0, 3, {"foo": "three"})), ("op", ins(1, "b")), ("rb", ins(1, "b")),
      ("rb", ann(0, 3, {"foo": "three"})), ("rb", ann(2, 4, {"foo": "two"})), ("rb", ann(0, 3, {"foo": "one"}))],
     "acde"),
    ("annotate with same prop",
     [("op", ins(0, "abcde")), ("op", ann(2, 3, {"foo": "bar"})), ("op", ann(1, 4, {"foo": "bar"})),
      ("rb", ann(1, 4, {"foo": "bar"}))], "abcde"),
    ("delete on single segment", [("op", ins(0, "abcd")), ("op", rem(0, 4)), ("rb", rem(0, 4))], "abcd"),
    ("delete which causes split segments", [("op", ins(0, "abcde")), ("op", rem(1, 4)), ("rb", rem(1, 4))], "abcde"),
    ("delete across split segments",
     [("op", ins(0, "abcde")), ("op", ann(2, 3, {"foo": "bar"})), ("op", rem(1, 4)), ("rb", rem(1, 4))], "abcde"),
    ("delete and update blocks",
     [("op", ins(i, c)) for i, c in enumerate(TEXT)] + [("op", rem(1, 4)), ("rb", rem(1, 4)),
                                                       ("op", ins(len(TEXT) - 1, "+"))],
     TEXT[:-1] + "+" + TEXT[-1]),
    ("zamboni rolled back insert",
     [("op", ins(0, "aefg")), ("op", ins(1, "bcd")), ("rb", ins(1, "bcd"))]
     + [("acklen", c) for c in "hello world"], "aefghello world"),
    ("zamboni rolled back annotated segment",
     [("ackins", ins(0, "abcde", {"color": "red"})), ("op", ann(2, 3, {"foo": "bar"})),
      ("rb", ann(2, 3, {"foo": "bar"}))] + [("acklen", c) for c in "hello world"], "abcdehello world"),
    ("zamboni rolled back remove",
     [("ackins", ins(0, "abcde", {"color": "red"})), ("op", rem(1, 4)), ("rb", rem(1, 4))]
     + [("acklen", c) for c in "hello world"], "abcdehello world"),
]


class _Client:
    """TestClient's local-op + makeOpMessage pattern as DocLog records; tracks the local text length."""

    def __init__(self, it):
        self.it = it
        self.log = DocLog()
        self.log.start_collab(ME)
        self.seq = 0
        self.text = ""
        self.pending = []  # local ops not acked yet, oldest first
        self.undo = []     # the local text before each pending op (rollback restores it)

    def local(self, op):
        self.log.local_op(op, self.it)
        self.pending.append(op)
        self.undo.append(self.text)
        if op["type"] == 0:
            seg = op["seg"] if isinstance(op["seg"], str) else op["seg"]["text"]
            self.text = self.text[:op["pos1"]] + seg + self.text[op["pos1"]:]
        elif op["type"] == 1:
            self.text = self.text[:op["pos1"]] + self.text[op["pos2"]:]

    def ack_oldest(self):
        op = self.pending.pop(0)
        self.undo.pop(0)
        self.seq += 1
        self.log.message({"clientId": ME, "sequenceNumber": self.seq, "referenceSequenceNumber": self.seq - 1,
                          "minimumSequenceNumber": self.seq - 1, "type": "op", "contents": op}, self.it)

    def rollback(self, op):
        self.log.rollback(op, self.it)
        self.pending.pop()
        self.text = self.undo.pop()


def _kat_log(steps, it):
    c = _Client(it)
    for kind, op in steps:
        if kind == "op":
            c.local(op)
        elif kind == "rb":
            c.rollback(op)
        elif kind == "ack":
            while c.pending:
                c.ack_oldest()
        elif kind == "ackins":
            c.local(op)
            c.ack_oldest()
        elif kind == "acklen":  # insertTextLocal(getLength(), c) acked at once
            c.local(ins(len(c.text), op))
            c.ack_oldest()
    while c.pending:  # (ack what is left so the summary shows every segment)
        c.ack_oldest()
    return c.log


@pytest.mark.parametrize("kat", ROLLBACK_KATS, ids=[k[0] for k in ROLLBACK_KATS])
def test_rollback_kat_oracle(kat):
    name, steps, want = kat
    it = Interner()
    log = _kat_log(steps, it)
    b = build_batch([log], it)
    doc = OracleDoc(options())
    assert doc.apply(b, 0) == 0
    assert doc.text() == want


def _farm(seed, cycles=40):
    """Cycles of: remote messages (made on the remote text), then local edits at the writer's local view
    (read from the oracle as the log grows), then either a rollback of every pending edit (newest first)
    or their messages (acks for the writer, remote ops for everyone else), as
    client.rollbackFarm.spec.ts interleaves them.  Returns (interner, the writer's batches, the other
    client's batches): both texts must agree at the end."""
    rnd = random.Random(seed)
    it = Interner()
    mine, other = DocLog(), DocLog()
    mine.start_collab(ME)
    other.start_collab("other")
    view_doc, other_doc = OracleDoc(options()), OracleDoc(options())
    batches, other_batches = [], []
    seq = 0

    def flush(log, doc, out):
        b = build_batch([log], it)
        out.append(b)
        assert doc.apply(b, 0) == 0
        return doc.text()

    for _ in range(cycles):
        for _ in range(rnd.randint(0, 4)):  # a remote writer's messages, made on the observer's (sequenced) text
            t = flush(other, other_doc, other_batches)
            seq += 1
            if t and rnd.random() < 0.4:
                a = rnd.randrange(len(t))
                op = rem(a, min(len(t), a + rnd.randint(1, 4)))
            elif t and rnd.random() < 0.3:
                a = rnd.randrange(len(t))
                op = ann(a, min(len(t), a + rnd.randint(1, 5)), {"k": rnd.randint(0, 3)})
            else:
                op = ins(rnd.randint(0, len(t)), "".join(rnd.choice("xyz") for _ in range(rnd.randint(1, 3))))
            m = {"clientId": "remote", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
                 "minimumSequenceNumber": max(0, seq - 6), "type": "op", "contents": op}
            mine.message(m, it)
            other.message(m, it)
        pending, ref = [], seq
        for _ in range(rnd.randint(1, 5)):  # local edits at the writer's local view
            view = flush(mine, view_doc, batches)
            if view and rnd.random() < 0.35:
                a = rnd.randrange(len(view))
                op = rem(a, min(len(view), a + rnd.randint(1, 3)))
            elif view and rnd.random() < 0.3:
                a = rnd.randrange(len(view))
                op = ann(a, min(len(view), a + rnd.randint(1, 4)), {"k": rnd.randint(0, 3), "m": "L"})
            else:
                op = ins(rnd.randint(0, len(view)), "".join(rnd.choice("ABC") for _ in range(rnd.randint(1, 3))))
            mine.local_op(op, it)
            pending.append(op)
        if rnd.random() < 0.5:  # roll back every pending edit, newest first
            while pending:
                mine.rollback(pending.pop(), it)
        else:  # send them: acks for the writer, remote ops for the other client
            for op in pending:
                seq += 1
                m = {"clientId": ME, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                     "minimumSequenceNumber": max(0, seq - 6), "type": "op", "contents": op}
                mine.message(m, it)
                other.message(m, it)
    batches.append(build_batch([mine], it))
    other_batches.append(build_batch([other], it))
    return it, batches, other_batches


@pytest.mark.parametrize("seed", range(6))
def test_rollback_farm_oracle(seed):
    it, batches, other_batches = _farm(seed)
    doc, other = OracleDoc(options()), OracleDoc(options())
    for b in batches:
        assert doc.apply(b, 0) == 0
    for b in other_batches:
        assert other.apply(b, 0) == 0
    assert doc.text() == other.text()


def _engine(n):
    from fluidframework_amd.engine import Engine
    return Engine(n, max_segments=8192, heap_entries=8192, text_units=1 << 18, prop_words=1 << 18,
                  remover_cells=1 << 14, ops_per_launch=64)


@pytest.mark.gpu
def test_rollback_kats_engine():
    """Every KAT as one document of one engine batch: texts, leaves and V1 summaries equal the oracle's."""
    it = Interner()
    logs = [_kat_log(k[1], it) for k in ROLLBACK_KATS]
    b = build_batch(logs, it)
    eng = _engine(len(logs))
    eng.apply(b)
    eng.summarize()
    for d, (name, _, want) in enumerate(ROLLBACK_KATS):
        st, op = eng.status(d)
        assert st == 0, f"{name}: status {st:#x} at op {op}"
        assert eng.text(d) == want, name
        orc = OracleDoc(options())
        assert orc.apply(b, d) == 0
        ge, gh = eng.export(d)
        oe, oh = orc.export()
        assert gh == oh and ge.shape == oe.shape, name
        assert np.array_equal(ge, oe), name
        assert eng.summary(d) == orc.summarize(b, d), name


@pytest.mark.gpu
def test_rollback_farm_engine():
    """The seeded farms, one document each, batch by batch as the farm built them: the engine's texts
    and final leaves equal the oracle's."""
    farms = [_farm(seed) for seed in range(4)]
    for seed, (it, batches, other_batches) in enumerate(farms):
        eng = _engine(1)
        orc = OracleDoc(options())
        for b in batches:
            eng.apply(b)
            assert orc.apply(b, 0) == 0
            st, op = eng.status(0)
            assert st == 0, f"seed {seed}: status {st:#x} at op {op}"
            assert eng.text(0) == orc.text(), f"seed {seed}"
        ge, gh = eng.export(0)
        oe, oh = orc.export()
        assert gh == oh and np.array_equal(ge, oe), f"seed {seed}"
