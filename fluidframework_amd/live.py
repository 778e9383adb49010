"""A collaborating SharedString client on the replay engine: local edits, interval collections with their own ops,
acks, and reconnect.

The reference's client is ``SharedString`` (sequence/src/sharedString.ts, sequence.ts) over a merge-tree ``Client``
and a ``DefaultMap`` of ``IntervalCollection``s (sequence/src/intervalCollection.ts).  Here the merge-tree state and
every interval endpoint live on the engine (one engine document per client); this module is the host side a
TypeScript shim would keep: the op records (``SequenceLog``), the interval collections' bookkeeping
(``fluidframework_amd.intervals``), and the calls a container runtime makes (``submit`` out, ``process`` /
``resubmit`` in).  A ``LiveSession`` drives several clients on one executor -- an ``Engine`` (``EngineExecutor``) or
any object with the same methods -- and applies every client's pending records in one batch whenever a client needs
an answer (a length, reference positions, rebased positions).
"""
from __future__ import annotations

import copy
from typing import Any, Callable

import numpy as np

from . import abi, regen
from .batch import Interner, build_batch
from .intervals import (_UNDEF, INTERVAL_ID, Collection, Interval, IntervalCollections, IntervalUnsupported,
                        UsageError, _iv_cmp, _ref_key)
from .sequence import SequenceLog


class EngineExecutor:
    """The HIP engine as a live session's executor (engine document d = client d)."""

    def __init__(self, engine):
        self.eng = engine

    def apply(self, batch) -> None:
        self.eng.apply(batch)
        for d in range(batch.n_docs):
            st, op = self.eng.status(d)
            if st != abi.MTR_OK:
                raise RuntimeError(f"engine document {d}: status {st:#x} at op {op}")

    def text(self, d: int) -> str:
        return self.eng.text(d)

    def ref_keys(self, d: int) -> list:
        return self.eng.ref_keys(d)

    def length(self, d: int, ref_seq: int, client: int) -> int:
        return self.eng.view_length(d, ref_seq, client)

    def deltas(self, d: int) -> np.ndarray:
        return self.eng.deltas(d)

    def props(self, d: int, ref: int) -> list:
        return self.eng.props(d, ref)

    def summary(self, batch, d: int) -> list[bytes]:
        self.eng.summarize()
        return self.eng.summary(d)


class LiveSession:
    """Clients of one document family on one executor: `sync()` applies every client's queued records."""

    def __init__(self, executor, interner: Interner | None = None, legacy: bool = False):
        self.ex = executor
        self.it = interner or Interner()
        self.legacy = legacy          # the legacy summary format (newMergeTreeSnapshotFormat !== true): catch-up ops
        self.clients: list[SharedStringClient] = []
        self.deltas: dict[int, np.ndarray] = {}

    def client(self, name: str | None = None) -> "SharedStringClient":
        c = SharedStringClient(self, len(self.clients), name)
        self.clients.append(c)
        return c

    def sync(self) -> None:
        if not any(c.log.ops for c in self.clients):
            return
        b = build_batch([c.log for c in self.clients], self.it)
        self.ex.apply(b)
        for c in self.clients:
            if b.docs[c.doc]["op_count"]:
                self.deltas[c.doc] = self.ex.deltas(c.doc)
                if c.log.pending:
                    c.log.resolve(self.deltas[c.doc])


    def summary(self, doc: int) -> list[bytes]:
        """Client.summarize's blobs of engine document `doc` (header, body_0, ...: SnapshotV1)."""
        self.sync()
        return self.ex.summary(build_batch([c.log for c in self.clients], self.it), doc)


class SharedStringClient:
    """One SharedString of a container (merge-tree client + interval collections) whose state lives on the
    engine.  The container runtime sets `submit_fn(contents, local_op_metadata)` and calls `process(msg, local,
    metadata)` for every sequenced message and `resubmit(contents, metadata)` after a reconnect."""

    def __init__(self, session: LiveSession, doc: int, name: str | None):
        self.session = session
        self.doc = doc
        self.name = name
        self.log = SequenceLog(legacy=session.legacy)
        self.log.intervals = IntervalCollections()
        self.submit_fn: Callable[[Any, Any], None] | None = None
        self.lseq = 0                 # collabWindow.localSeq as this host counts it (every local op, interval ops too)
        self.last_norm = 0            # Client.lastNormalizationRefSeq (client.ts:910)
        self.facades: dict[str, LiveIntervalCollection] = {}

    # ---- the executor, through the session
    @property
    def it(self) -> Interner:
        return self.session.it

    @property
    def current_seq(self) -> int:
        return self.log.current_seq

    def sync(self) -> None:
        self.session.sync()

    def get_text(self) -> str:
        self.sync()
        return self.session.ex.text(self.doc)

    def length(self) -> int:
        """getLength: the local view's length (root.cachedLength; markers count 1)"""
        self.sync()
        me = self.log.client_ix.get(self.log.observer_id, -1) if self.log.collaborating else -1
        return self.session.ex.length(self.doc, self.current_seq, me)

    get_length = length

    def ref_keys(self) -> list:
        self.sync()
        return self.session.ex.ref_keys(self.doc)

    def rebase_results(self) -> dict:
        """{record index: position} of the MTR_OP_REBASE_POS records just queued (one sync)."""
        self.sync()
        d = self.session.deltas.get(self.doc)
        out = {}
        if d is not None:
            for r in d:
                if int(r["kind"]) == abi.DELTA_REBASE:
                    out[int(r["op"])] = int(r["pos"])
        return out

    def next_local_seq(self) -> int:
        """IntervalCollection.getNextLocalSeq (intervalCollection.ts:1584-1590)."""
        self.lseq += 1
        self.log.bump_local_seq()
        return self.lseq

    def submit(self, contents: Any, metadata: Any) -> None:
        if self.submit_fn is not None:
            self.submit_fn(contents, metadata)

    # ---- connection (SharedSegmentSequence.didAttach / onConnect -> startOrUpdateCollaboration)
    def connect(self, client_id: str) -> None:
        self.log.start_collab(client_id)

    # ---- merge-tree edits (SharedSegmentSequence / SharedString local ops, sequence.ts:266-344)
    def _local(self, op: dict) -> None:
        self.log.local_op(op, self.it)
        if self.log.collaborating:
            self.lseq += 1
            self.submit(op, {"merge": True})

    def insert_text(self, pos: int, text: str, props: dict | None = None) -> None:
        seg: Any = {"text": text, "props": props} if props is not None else text
        self._local({"pos1": pos, "seg": seg, "type": 0})

    def insert_marker(self, pos: int, ref_type: int, props: dict | None = None) -> None:
        seg: Any = {"marker": {"refType": ref_type}}
        if props is not None:
            seg["props"] = props
        self._local({"pos1": pos, "seg": seg, "type": 0})

    def remove_range(self, start: int, end: int) -> None:
        self._local({"pos1": start, "pos2": end, "type": 1})

    remove_text = remove_range

    def annotate_range(self, start: int, end: int, props: dict) -> None:
        self._local({"pos1": start, "pos2": end, "props": props, "type": 2})

    # ---- interval collections
    def get_interval_collection(self, label: str) -> "LiveIntervalCollection":
        """getIntervalCollection (sequence.ts:445-447): created when absent."""
        f = self.facades.get(label)
        if f is None:
            f = self.facades[label] = LiveIntervalCollection(self, label)
        return f

    def interval_header(self) -> bytes | None:
        """The summary's `header` blob (summarizeCore, sequence.ts:467-480) of this live client."""
        from .jsjson import to_utf8

        h = self.log.intervals.serialize(self.ref_keys(), self.current_seq, live=True)
        return None if h is None else to_utf8(h)

    def summary(self) -> list[bytes]:
        """summarizeCore's merge-tree blobs (the engine's summary of this document) plus, in the legacy format, the
        ``catchupOps`` blob of the messages since the MSN (summarizeMergeTree, sequence.ts:675-695)."""
        blobs = self.session.summary(self.doc)
        cu = self.log.catchup_blob()
        return blobs + ([cu] if cu is not None else [])

    def local_reference_position(self, ref: int) -> int:
        return self.ref_keys()[ref][0]

    # ---- the runtime's calls
    def process(self, msg: dict, local: bool, metadata: Any = None) -> None:
        """SharedSegmentSequence.processCore (sequence.ts:620-646)."""
        contents = msg.get("contents")
        if isinstance(contents, dict) and contents.get("type") == "act":
            key = contents.get("key")
            if not isinstance(key, str):
                raise IntervalUnsupported("an interval op without a string key")
            c = self.log.intervals.get(key)
            value = contents.get("value") or {}
            name = value.get("opName")
            if name not in ("add", "delete", "change"):
                raise IntervalUnsupported(f"interval op {name!r}")
            c.live_process(self, name, value.get("value"), msg, local, metadata)
            return
        self.log.message(msg, self.it)

    def resubmit(self, contents: Any, metadata: Any) -> None:
        """reSubmitCore: a merge-tree op is regenerated (Client.regeneratePendingOp, client.ts:917-960, whose
        "normalize" event rebases the pending interval ops first); an interval op is rebased (DefaultMap's resubmit
        -> rebaseLocalInterval, intervalCollection.ts:1270-1279)."""
        if isinstance(contents, dict) and contents.get("type") == "act":
            c = self.log.intervals.get(contents["key"])
            value = contents["value"]
            rebased = c.rebase_local(self, value["opName"], value.get("value"), metadata["localSeq"])
            op = dict(contents)
            v = {"opName": value["opName"]}
            if rebased is not None:
                v["value"] = rebased
            op["value"] = v
            self.submit(op, metadata)
            return
        if self.current_seq != self.last_norm:  # client.ts:921-926: emit("normalize") before normalizing
            for c in self.log.intervals.data.values():
                c.on_normalize(self)
            self.last_norm = self.current_seq
        first = self.log.regenerate(contents)
        self.sync()
        recs = regen.records(self.session.deltas.get(self.doc, np.zeros(0, dtype=abi.DELTA_DTYPE)))
        op = regen.regenerated_op(contents, recs, first,
                                  lambda r: regen.props_dict(self.session.ex.props(self.doc, r), self.it))
        self.submit(op, metadata)


class LiveIntervalCollection:
    """IntervalCollection's public API (intervalCollection.ts:1428-2338) for a live client."""

    def __init__(self, client: SharedStringClient, label: str):
        self.client = client
        self.label = label
        self.coll: Collection = client.log.intervals.get(label)

    def add(self, start: int, end: int, itype: int, props: dict | None = None) -> Interval:
        return self.coll.live_add(self.client, start, end, itype, props)

    def change(self, iid: Any, start: Any = _UNDEF, end: Any = _UNDEF) -> Interval | None:
        return self.coll.live_change(self.client, iid, start, end)

    def change_properties(self, iid: Any, props: dict) -> None:
        self.coll.live_change_properties(self.client, iid, props)

    def remove_interval_by_id(self, iid: Any) -> Interval | None:
        return self.coll.live_remove(self.client, iid)

    def get_interval_by_id(self, iid: str) -> Interval | None:
        return self.coll.by_id.get(iid)

    # ---- reads
    def positions(self, iv: Interval, keys: list | None = None) -> tuple[int, int]:
        """(localReferencePositionToPosition(start), ... (end))"""
        keys = keys if keys is not None else self.client.ref_keys()
        return keys[iv.start][0], keys[iv.end][0]

    def __iter__(self):
        """[Symbol.iterator]: the start tree's in-order walk (compare order)."""
        return iter(self.coll.ordered(self.client.ref_keys()))

    def _transient_keys(self, start: int, end: int) -> tuple[list, tuple, tuple]:
        """helpers.create("transient", start, end, client, Transient) -> two Transient references at the local view
        (detached when no segment holds the position); returns the document's reference keys (one sync) and the two
        transients' compare keys.  A Transient reference is held by no segment's collection (localReference.ts:
        260-298), so once its key is read its id goes back to the host's free list with no record: queries take no
        reference slot."""
        log = self.client.log
        ts, te = log.create_ref(int(start), abi.REFTYPE_TRANSIENT), log.create_ref(int(end), abi.REFTYPE_TRANSIENT)
        keys = self.client.ref_keys()
        ks, ke = _ref_key(keys, ts), _ref_key(keys, te)
        log.release_ref(te, remove=False)
        log.release_ref(ts, remove=False)
        return keys, ks, ke

    def find_overlapping_intervals(self, start: int, end: int) -> list:
        """findOverlappingIntervals (:950-964): the intervals overlapping [start, end] (SequenceInterval.overlaps,
        :544-549), in the tree's order (RedBlackTree.gather, rbTree.ts:174-199)."""
        return self.find_overlapping_intervals_many([(start, end)])[0]

    def find_overlapping_intervals_many(self, ranges) -> list:
        """findOverlappingIntervals for each (start, end) of `ranges`, answered from one engine sync: every query's
        Transient references are created in one batch and their keys read together."""
        ranges = [(int(a), int(b)) for a, b in ranges]
        live = [k for k, (a, b) in enumerate(ranges) if b >= a and self.coll.by_id]
        out: list = [[] for _ in ranges]
        if not live:
            return out
        log = self.client.log
        refs = [(log.create_ref(ranges[k][0], abi.REFTYPE_TRANSIENT), log.create_ref(ranges[k][1], abi.REFTYPE_TRANSIENT))
                for k in live]
        keys = self.client.ref_keys()
        ordered = self.coll.ordered(keys)
        for k, (ts, te) in zip(live, refs):
            ks, ke = _ref_key(keys, ts), _ref_key(keys, te)
            out[k] = [iv for iv in ordered if _ref_key(keys, iv.start) <= ke and _ref_key(keys, iv.end) >= ks]
        for ts, te in reversed(refs):
            log.release_ref(te, remove=False)
            log.release_ref(ts, remove=False)
        return out

    def _by_end(self, keys: list) -> list:
        """the end tree's keys (compareSequenceIntervalEnds, :1168-1169): one node per end; two intervals with equal
        ends share a node, which holds the later-put one -- a history this host does not keep, so it refuses"""
        ivs = sorted(self.coll.by_id.values(), key=lambda iv: _ref_key(keys, iv.end))
        for a, b in zip(ivs, ivs[1:]):
            if _ref_key(keys, a.end) == _ref_key(keys, b.end):
                raise IntervalUnsupported("two intervals with one end: the end tree keeps one node for them")
        return ivs

    def previous_interval(self, pos: int) -> Interval | None:
        """previousInterval (:966-978): endIntervalTree.floor of a transient (pos, pos)."""
        keys, _, k = self._transient_keys(pos, pos)
        best = None
        for iv in self._by_end(keys):
            if _ref_key(keys, iv.end) <= k:
                best = iv
        return best

    def next_interval(self, pos: int) -> Interval | None:
        """nextInterval (:980-992): endIntervalTree.ceil of a transient (pos, pos)."""
        keys, _, k = self._transient_keys(pos, pos)
        for iv in self._by_end(keys):
            if _ref_key(keys, iv.end) >= k:
                return iv
        return None

    def gather(self, forward: bool = True, start: int | None = None, end: int | None = None) -> list:
        """gatherIterationResults (:864-944): every interval, or those whose start (and end) compare equal to a
        transient interval's (CreateForward/BackwardIteratorWithStart/EndPosition, :2232-2277)."""
        keys = self.client.ref_keys()
        if start is None and end is None:
            out = self.coll.ordered(keys)
            return out if forward else out[::-1]
        keys, ks, ke = self._transient_keys(start if start is not None else 0, end if end is not None else 0)
        out = self.coll.ordered(keys)
        if start is None:
            out = [iv for iv in out if _ref_key(keys, iv.end) == ke]
        elif end is None:
            out = [iv for iv in out if _ref_key(keys, iv.start) == ks]
        else:
            out = [iv for iv in out if _ref_key(keys, iv.start) == ks and _ref_key(keys, iv.end) == ke]
        return out if forward else out[::-1]
