"""Annotate known answers transcribed from the reference's merge-tree/src/test/mergeTree.annotate.spec.ts
(SURVEY.md 8a row a10 and 8f4): property results of local, remote, acked, interleaved and "rewrite"
annotates, including PropertiesManager's pending key counts (shouldModifyKey, segmentPropertiesManager.ts:
94-104) and pending rewrites (pendingRewriteCount, :72-80), asserted through getContainingSegment.

The spec drives a MergeTree directly (local client 17, remote client 35).  Here the same edits are a
client's op stream: "hello world!" inserted before collaboration, the remote client's Tile marker at 3 (seq
1), then startCollaboration(local, 1, 1); a local annotate is a pending local op, a remote one a sequenced
message, and ackPendingSegment is this client's own sequenced message.  The spec's direct
`segment.splitAt(...)` calls become a remote insert inside the segment (the same splitAt, with
copyPropertiesTo / segmentGroups.copyTo).  Every case runs on the oracle (CPU) and on the HIP engine
against the oracle (-m gpu): properties (key order included) and segmentGroups sizes.
"""
import pytest

from fluidframework_amd import regen
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, options

ME, REM = "local", "remote"
START, MARKER, END = 1, 3, 5        # annotateStart, markerPosition, annotateEnd
SPLIT = (END - START) // 2 + START  # splitPos = 3
REWRITE = {"name": "rewrite"}


def ann(a, b, props, co=None):
    op = {"type": 2, "pos1": a, "pos2": b, "props": props}
    if co is not None:
        op["combiningOp"] = co
    return op


class Tree:
    """The spec's beforeEach, as a client: every step is flushed into the oracle as its own batch (kept for
    the engine replay) and the checks read getContainingSegment at (currentSequenceNumber, local)."""

    def __init__(self, collab=True):
        self.it = Interner()
        self.log = DocLog()
        self.doc = OracleDoc(options())
        self.batches = []
        self.checks = []  # (batch index, pos, expected groups or None, the oracle's properties, currentSeq)
        self.seq = 0
        self.collab = False
        self.log.local_insert(0, "hello world!", self.it)  # insertSegments(..., UniversalSequenceNumber, LocalClientId)
        self.remote({"type": 0, "pos1": MARKER, "seg": {"marker": {"refType": 1}}})  # Marker.make(Tile), seq 1
        if collab:
            self.collab = True
            self.log.start_collab(ME, self.seq, self.seq)  # startCollaboration(local, minSeq 1, currentSeq 1)
        self.flush()

    def flush(self):
        b = build_batch([self.log], self.it)
        assert self.doc.apply(b, 0) == 0
        self.batches.append(b)

    def remote(self, op):  # annotateRange(..., refSeq = currentSequenceNumber, remote, ++currentSequenceNumber)
        self.seq += 1
        self.log.message({"clientId": REM, "sequenceNumber": self.seq, "referenceSequenceNumber": self.seq - 1,
                          "minimumSequenceNumber": 1 if self.collab else 0, "type": "op", "contents": op},
                         self.it)
        self.flush()

    def local(self, op):  # annotateRange(..., refSeq = currentSequenceNumber, local, UnassignedSequenceNumber)
        self.log.local_op(op, self.it)
        self.flush()
        return op

    def ack(self, op):  # ackPendingSegment({op, sequencedMessage: {sequenceNumber: ++currentSequenceNumber}})
        self.seq += 1
        self.log.message({"clientId": ME, "sequenceNumber": self.seq, "referenceSequenceNumber": self.seq - 1,
                          "minimumSequenceNumber": 1, "type": "op", "contents": op}, self.it)
        self.flush()

    def split_at(self, pos):  # segment.splitAt(...) -> a remote single-unit insert at pos
        self.remote({"type": 0, "pos1": pos, "seg": "X"})

    def client(self):
        return self.log.client_ix[ME] if self.collab else -1

    def props(self, pos):
        """(segmentGroups.size, properties dict or None) of getContainingSegment(pos, current, local)."""
        r = self.doc.containing_props(pos, self.seq, self.client())
        assert r is not None, f"no segment at {pos}"
        groups, pairs = r
        return groups, (None if pairs is None else regen.props_dict(pairs, self.it))

    def check(self, pos, want, groups=None):
        """assert.equal(segment.properties?.k, v) for each k, v (v None: the key is absent / falsy)."""
        g, p = self.props(pos)
        p = p or {}
        for k, v in want.items():
            assert p.get(k) == v, f"{k}: {p.get(k)!r} != {v!r} (props {p})"
        if groups is not None:
            assert g == groups, f"segmentGroups.size {g} != {groups}"
        self.checks.append((len(self.batches) - 1, pos, groups, p, self.seq))


# ---- annotateRange / not collaborating (:53-97)
def kat_not_collab_remote():
    t = Tree(collab=False)
    t.remote(ann(START, END, {"propertySource": "remote"}))
    t.check(START, {"propertySource": "remote"})
    return t


def kat_not_collab_local():
    t = Tree(collab=False)
    t.local(ann(START, END, {"propertySource": "local"}))
    t.check(START, {"propertySource": "local"})
    return t


# ---- collaborating / local first (:107-527)
LOCAL = {"propertySource": "local"}


def local_first(co=None):
    t = Tree()
    op = t.local(ann(START, END, LOCAL, co))
    return t, op


def kat_unsequenced_local():
    t, _ = local_first()
    t.check(START, {"propertySource": "local"})
    return t


def kat_unsequenced_local_after_local():
    t, _ = local_first()
    t.local(ann(START, END, {"secondProperty": "local"}))
    t.check(START, {"secondProperty": "local"})
    return t


def kat_unsequenced_local_split():
    t, _ = local_first()
    t.split_at(START + 1)  # "el" -> "e" | "l": the right half copies the properties
    t.check(START + 2, {"propertySource": "local"})
    return t


def kat_local_after_local_split():
    t, op = local_first()
    second = t.local(ann(START, END, {"secondChange": 1}))
    split_only = t.local(ann(SPLIT, END, {"splitOnly": 1}))
    t.check(START, {"propertySource": "local", "secondChange": 1, "splitOnly": None}, groups=2)
    t.check(SPLIT, {"propertySource": "local", "secondChange": 1, "splitOnly": 1}, groups=3)
    t.ack(op)
    t.check(START, {"propertySource": "local", "secondChange": 1, "splitOnly": None}, groups=1)
    t.check(SPLIT, {"propertySource": "local", "secondChange": 1, "splitOnly": 1}, groups=2)
    t.ack(second)
    t.check(START, {"propertySource": "local", "secondChange": 1, "splitOnly": None}, groups=0)
    t.check(SPLIT, {"propertySource": "local", "secondChange": 1, "splitOnly": 1}, groups=1)
    t.ack(split_only)
    t.check(START, {"propertySource": "local", "secondChange": 1, "splitOnly": None}, groups=0)
    t.check(SPLIT, {"propertySource": "local", "secondChange": 1, "splitOnly": 1}, groups=0)
    return t


def kat_unsequenced_local_before_remote():
    t, _ = local_first()
    t.remote(ann(START, END, {"propertySource": "remote", "remoteProperty": 1}))
    t.check(START, {"propertySource": "local", "remoteProperty": 1}, groups=1)
    return t


def kat_sequenced_local():
    t, op = local_first()
    t.ack(op)
    t.check(START, {"propertySource": "local"}, groups=0)
    return t


def kat_sequenced_local_before_remote():
    t, op = local_first()
    t.ack(op)
    t.remote(ann(START, END, {"propertySource": "remote", "remoteProperty": 1}))
    t.check(START, {"propertySource": "remote", "remoteProperty": 1}, groups=0)
    return t


def kat_three_local_changes():
    t, op = local_first()
    t.check(START, {"propertySource": "local"})
    op2 = t.local(ann(START, END, {"propertySource": "local2", "secondSource": 1}))
    t.check(START, {"propertySource": "local2", "secondSource": 1})
    op3 = t.local(ann(START, END, {"thirdSource": 1}))
    want = {"propertySource": "local2", "secondSource": 1, "thirdSource": 1}
    t.check(START, want)
    for o in (op, op2, op3):
        t.ack(o)
        t.check(START, want)
    return t


def kat_two_local_interleaved_remote():
    t, op = local_first()
    t.local(ann(START, END, {"secondSource": "local2"}))
    t.ack(op)
    t.remote(ann(START, END, {"propertySource": "remote", "remoteOnly": 1, "secondSource": "remote"}))
    t.check(START, {"remoteOnly": 1, "propertySource": "remote", "secondSource": "local2"})
    return t


# ---- collaborating / remote first (:528-640)
def remote_first():
    t = Tree()
    t.remote(ann(START, END, {"propertySource": "remote", "remoteProperty": 1}))
    t.check(START, {}, groups=0)  # segmentGroups.empty
    return t


def kat_remote_only():
    t = remote_first()
    t.check(START, {"propertySource": "remote", "remoteProperty": 1})
    return t


def kat_split_remote():
    t = remote_first()
    t.split_at(START + 1)  # segment.splitAt(1)
    t.check(START + 2, {"propertySource": "remote", "remoteProperty": 1})
    return t


def kat_remote_before_unsequenced_local():
    t = remote_first()
    t.local(ann(START, END, {"propertySource": "local"}))
    t.check(START, {"propertySource": "local", "remoteProperty": 1})
    return t


def kat_remote_before_sequenced_local():
    t = remote_first()
    op = t.local(ann(START, END, {"propertySource": "local"}))
    t.check(START, {}, groups=1)
    t.ack(op)
    t.check(START, {"propertySource": "local", "remoteProperty": 1}, groups=0)
    return t


# ---- collaborating / local with rewrite first (:641-808)
def kat_rewrite_local_after_local():
    t, _ = local_first(REWRITE)
    t.local(ann(START, END, {"propertySource": "local2", "secondProperty": "local"}))
    t.check(START, {"propertySource": "local2", "secondProperty": "local"})
    return t


def kat_rewrite_local_before_remote():
    t, _ = local_first(REWRITE)
    t.remote(ann(START, END, {"propertySource": "remote", "remoteProperty": 1}))
    t.check(START, {"propertySource": "local", "remoteProperty": None}, groups=1)  # every remote key blocked
    return t


def kat_rewrite_sequenced_before_remote():
    t, op = local_first(REWRITE)
    t.ack(op)
    t.remote(ann(START, END, {"propertySource": "remote", "remoteProperty": 1}))
    t.check(START, {"propertySource": "remote", "remoteProperty": 1}, groups=0)
    return t


def kat_rewrite_two_local_interleaved_remote():
    t, op = local_first(REWRITE)
    t.local(ann(START, END, {"secondSource": "local2"}, REWRITE))
    t.ack(op)
    t.remote(ann(START, END, {"propertySource": "remote", "remoteOnly": 1, "secondSource": "remote"}))
    t.check(START, {"remoteOnly": None, "propertySource": None, "secondSource": "local2"})
    return t


KATS = [kat_not_collab_remote, kat_not_collab_local, kat_unsequenced_local, kat_unsequenced_local_after_local,
        kat_unsequenced_local_split, kat_local_after_local_split, kat_unsequenced_local_before_remote,
        kat_sequenced_local, kat_sequenced_local_before_remote, kat_three_local_changes,
        kat_two_local_interleaved_remote, kat_remote_only, kat_split_remote, kat_remote_before_unsequenced_local,
        kat_remote_before_sequenced_local, kat_rewrite_local_after_local, kat_rewrite_local_before_remote,
        kat_rewrite_sequenced_before_remote, kat_rewrite_two_local_interleaved_remote]


@pytest.mark.parametrize("kat", KATS, ids=[k.__name__[4:] for k in KATS])
def test_annotate_kats_oracle(kat):
    kat()


def _rollback_rewrite_case():
    """Rollback of a local rewrite (MergeTree.rollback with PropertiesRollback.Rewrite, mergeTree.ts:2129-2152):
    the deltas -- keys the rewrite deleted, then its keys' old values -- come back as a plain annotate, so a
    deleted key returns at the end of the key order; an older pending annotate's key keeps its count."""
    t = Tree()
    t.remote(ann(START, END, {"a": 1, "b": 2, "c": 3}))
    first = t.local(ann(START, END, {"c": 9}))
    op = t.local(ann(START, END, {"b": 5, "d": 0}, REWRITE))
    t.check(START, {"a": None, "b": 5, "c": None, "d": 0}, groups=2)
    t.log.rollback(op, t.it)
    t.flush()
    t.check(START, {"a": 1, "b": 2, "c": 9, "d": None}, groups=1)
    g, p = t.props(START)
    assert list(p) == ["b", "a", "c"], p  # "a" and "c" re-added behind "b"
    t.ack(first)
    t.remote(ann(START, END, {"c": "r"}))
    t.check(START, {"c": "r"}, groups=0)
    return t


def test_rollback_rewrite_oracle():
    _rollback_rewrite_case()


def _engine():
    from fluidframework_amd.engine import Engine
    return Engine(1, max_segments=1024, heap_entries=1024, text_units=1 << 14, prop_words=1 << 14,
                  remover_cells=1 << 12, ops_per_launch=64)


def _replay_engine(t):
    """The tree's batches on the engine, one at a time; after each checked batch the engine's containing
    segment has the oracle's properties (key order included) and segmentGroups size."""
    eng = _engine()
    checks = {}
    for c in t.checks:
        checks.setdefault(c[0], []).append(c)
    for k, b in enumerate(t.batches):
        eng.apply(b)
        st, op = eng.status(0)
        assert st == 0, f"batch {k}: status {st:#x} at op {op}"
        for _, pos, groups, props, seq in checks.get(k, []):
            r = eng.containing_segment(0, pos, seq, t.client())
            assert r is not None
            got = {} if r["props"] < 0 else regen.props_dict(eng.props(0, r["props"]), t.it)
            assert list(got.items()) == list(props.items()), f"batch {k} pos {pos}: {got} != {props}"
            if groups is not None:
                assert r["groups"] == groups, f"batch {k} pos {pos}: groups {r['groups']} != {groups}"


@pytest.mark.gpu
def test_annotate_kats_engine():
    for kat in KATS + [_rollback_rewrite_case]:
        t = kat()
        _replay_engine(t)
