"""SharedSegmentSequence's legacy-summary catch-up ops, host side.

In the legacy summary format (``newMergeTreeSnapshotFormat !== true``) a SharedString keeps every
sequenced message since the MSN (``messagesSinceMSNChange``, packages/dds/sequence/src/sequence.ts:185)
and writes them into the summary as the ``catchupOps`` blob (snapshotlegacy.ts:174-179).  A message
whose referenceSequenceNumber is not ``seq - 1`` is first *transformed*: the ``sequenceDelta`` events
its application raises are turned back into ops positioned in the view right after it
(``createOpsFromDelta``, sequence.ts:120-173; processMergeTreeMsg, sequence.ts:697-736), and the
stashed copy gets ``referenceSequenceNumber = seq - 1`` and those ops as contents.

The split between device and host follows the data: the engine applies the message (flagged
``MTR_F_DELTA``) and reports each delta range -- op index, position in the local view, cachedLength,
kind -- from the tree while it is in HBM/LDS (``mtr_get_deltas``); the host, which holds the message
JSON anyway, rebuilds the op objects from those ranges plus the message's own segment spec and property
set.  Nothing here applies ops: the engine is the only place merge-tree state lives.
"""
from __future__ import annotations

import copy
from typing import Any

import numpy as np

from . import abi
from .batch import DocLog, Interner, Unsupported
from .jsjson import js_key_order, js_stringify, parse, to_utf8

CATCHUP_BLOB = "catchupOps"  # SnapshotLegacy.catchupOps (snapshotlegacy.ts:43)
_GC_SPAN = 20                # sequence.ts:729-734

_UNDEF = object()  # JavaScript `undefined`


def _typeof(v: Any) -> str:
    if v is None or isinstance(v, (dict, list)):
        return "object"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    return "undefined"


def _truthy(v: Any) -> bool:
    if v is None or v is _UNDEF:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v == v and v != 0
    if isinstance(v, str):
        return len(v) > 0
    return True


def _units(s: str) -> list[str]:
    u = s.encode("utf-16-le", "surrogatepass")
    return [u[i:i + 2].decode("utf-16-le", "surrogatepass") for i in range(0, len(u), 2)]


def _for_in(v: Any) -> list[str]:
    """`for (const key in v)` over a JSON value."""
    if isinstance(v, dict):
        return js_key_order(v.keys())
    if isinstance(v, list):
        return [str(i) for i in range(len(v))]
    if isinstance(v, str):
        return [str(i) for i in range(len(_units(v)))]
    return []


def _get(v: Any, key: str) -> Any:
    if isinstance(v, dict):
        return v.get(key, _UNDEF)
    if isinstance(v, (list, str)):
        seq = v if isinstance(v, list) else _units(v)
        if key.isdigit() and str(int(key)) == key and int(key) < len(seq):
            return seq[int(key)]
    return _UNDEF


def _strict_eq(a: Any, b: Any) -> bool:
    ta, tb = _typeof(a), _typeof(b)
    if ta != tb:
        return False
    if ta == "object":
        return a is b
    return a == b


def match_properties(a: Any, b: Any) -> bool:
    """matchProperties (packages/dds/merge-tree/src/properties.ts:71-105), JavaScript truthiness,
    `typeof` and `for...in` included."""
    if _truthy(a):
        if not _truthy(b):
            return False
        for key in _for_in(a):
            bk = _get(b, key)
            if bk is _UNDEF:
                return False
            if _typeof(bk) == "object":
                if not match_properties(_get(a, key), bk):
                    return False
            elif not _strict_eq(bk, _get(a, key)):
                return False
        for key in _for_in(b):
            if _get(a, key) is _UNDEF:
                return False
    elif _truthy(b):
        return False
    return True


def _segment_json(spec: Any) -> Any:
    """segment.clone().toJSONObject() of the segment an insert op creates (TextSegment.make /
    Marker.make + addProperties: a property set exists iff the spec has props, null values are
    deletes; textSegment.ts:33-62, mergeTreeNodes.ts:385-435, 577-581)."""
    def props_of(p):
        return {k: p[k] for k in js_key_order(p.keys()) if p[k] is not None}

    if isinstance(spec, str):
        return spec
    if isinstance(spec, dict) and "text" in spec:
        if spec.get("props") is not None:
            return {"text": spec["text"], "props": props_of(spec["props"])}
        return spec["text"]
    if isinstance(spec, dict) and "marker" in spec:
        m = spec["marker"] or {}
        out: dict = {"marker": {"refType": m["refType"]} if m.get("refType") is not None else {}}
        if spec.get("props") is not None:
            out["props"] = props_of(spec["props"])
        return out
    raise Unsupported("unrecognized segment spec")


def ops_from_deltas(members: list[dict], ranges: np.ndarray, op_index: list[int]) -> list[dict]:
    """createOpsFromDelta over every sequenceDelta event of one message (sequence.ts:120-173,
    accumulated by transformOps across a group's member ops, sequence.ts:700-703).

    members:  the message's merge-tree ops; op_index[i] = the engine op index of members[i]
              (-1 when the member produced no engine op with a delta event);
    ranges:   the engine's mtr_delta records of this message's ops (abi.DELTA_DTYPE), op order."""
    ops: list[dict] = []
    by_op: dict[int, list] = {}
    for r in ranges:
        by_op.setdefault(int(r["op"]), []).append(r)
    for member, gi in zip(members, op_index):
        for r in by_op.get(gi, ()):
            kind, pos, ln = int(r["kind"]), int(r["pos"]), int(r["len"])
            last = ops[-1] if ops else None
            if kind == abi.OP_ANNOTATE:
                # propertyDeltas has every key of the op (an observer has no pending local keys,
                # segmentPropertiesManager.ts:96-151); the segment's value after the op is the op's
                op_props = member["props"]
                props = {k: op_props[k] for k in js_key_order(op_props.keys())}
                if last is not None and last.get("pos2", _UNDEF) == pos and \
                        match_properties(last.get("props", _UNDEF), props):
                    last["pos2"] += ln
                else:
                    # createAnnotateRangeOp(.., combiningOp undefined) -- JSON.stringify drops it
                    ops.append({"pos1": pos, "pos2": pos + ln, "props": props, "type": 2})
            elif kind == abi.OP_INSERT:
                ops.append({"pos1": pos, "seg": _segment_json(member["seg"]), "type": 0})
            elif kind == abi.OP_REMOVE:
                if last is not None and last.get("pos1", _UNDEF) == pos:
                    if "pos2" not in last:
                        # assert 0x3ff "pos2 should not be undefined here" (sequence.ts:155-158)
                        raise Unsupported("catch-up transform hits assert 0x3ff (remove merged into an insert)")
                    last["pos2"] += ln
                else:
                    ops.append({"pos1": pos, "pos2": pos + ln, "type": 1})
    return ops


def _is_interval_op(msg: dict) -> bool:
    c = msg.get("contents")
    if isinstance(c, str):
        c = parse(c)
    return isinstance(c, dict) and c.get("type") == "act"


class SequenceLog(DocLog):
    """A DocLog that also keeps SharedSegmentSequence's ``messagesSinceMSNChange``.

    legacy=False is the V1 format (``newMergeTreeSnapshotFormat: true``): no message is kept and no
    op is flagged.  Use: message(...) for each sequenced op, build_batch, engine apply, then
    ``resolve(engine.deltas(doc))`` before the next message; ``catchup_blob(msn)`` at summarize."""

    def __init__(self, legacy: bool = True) -> None:
        super().__init__()
        self.legacy = legacy
        self.stash: list[dict] = []
        self.pending: list[tuple[dict, list[dict], list[int]]] = []
        self.msn = 0

    def message(self, msg: dict, interner: Interner) -> None:
        if msg.get("type") == "op" and _is_interval_op(msg):
            # handled by the interval collections (sequence.ts:636-645): not a merge-tree message, not kept
            super().message(msg, interner)
            return
        self.msn = max(self.msn, int(msg["minimumSequenceNumber"]))
        if msg.get("type") != "op" or not self.legacy:
            super().message(msg, interner)
            return
        own = self.collaborating and msg.get("clientId") == self.observer_id
        if own:
            # applyMsg(msg, local = true) acks the pending segments (client.ts:858-875), which raises a
            # "maintenance" event and no "delta" event (ackPendingSegment, mergeTree.ts:1283-1323): a lagging own
            # message's transformOps listener collects nothing, so its stashed copy is createGroupOp() of no ops
            # (sequence.ts:697-725, opBuilder.ts:102-107)
            super().message(msg, interner)
            stash = copy.deepcopy(msg)
            seq = int(msg["sequenceNumber"])
            if int(msg["referenceSequenceNumber"]) != seq - 1:
                stash["referenceSequenceNumber"] = seq - 1
                stash["contents"] = {"ops": [], "type": 3}
            elif isinstance(stash.get("contents"), str):
                stash["contents"] = parse(stash["contents"])
            self._keep(stash, msg)
            return
        if int(msg["referenceSequenceNumber"]) != int(msg["sequenceNumber"]) - 1:
            c = msg["contents"]
            c = parse(c) if isinstance(c, str) else c
            for m in (c.get("ops") or []) if c.get("type") == 3 else [c]:
                # the catch-up transform needs each member's post-op values / one record per member
                if m.get("combiningOp") or m.get("relativePos1") or m.get("relativePos2"):
                    raise Unsupported("a lagging message with a combining annotate or a relative position "
                                      "in the legacy format")
        lo = len(self.ops)
        super().message(msg, interner)
        hi = len(self.ops)
        # parseHandles: the DDS sees a JSON copy with parsed contents (sequence.ts:698)
        stash = copy.deepcopy(msg)
        if isinstance(stash.get("contents"), str):
            stash["contents"] = parse(stash["contents"])
        seq = int(msg["sequenceNumber"])
        if int(msg["referenceSequenceNumber"]) != seq - 1:
            contents = stash["contents"]
            members = contents["ops"] if contents.get("type") == 3 else [contents]
            op_index = []
            k = lo
            for m in members:
                # DocLog.message emits one record per member op, in order
                rec = self.ops[k]
                if rec[0] in (abi.OP_INSERT, abi.OP_REMOVE, abi.OP_ANNOTATE):
                    self.ops[k] = (rec[0], rec[1] | abi.F_DELTA) + tuple(rec[2:])
                    op_index.append(k)
                else:
                    op_index.append(-1)
                k += 1
            assert k == hi or not members
            # {...message, referenceSequenceNumber: seq - 1, contents} keeps the key order
            stash["referenceSequenceNumber"] = seq - 1
            self.pending.append((stash, members, op_index))
        self._keep(stash, msg)

    def _keep(self, stash: dict, msg: dict) -> None:
        """messagesSinceMSNChange.push + the GC every once in a while (sequence.ts:727-735)."""
        self.stash.append(stash)
        if len(self.stash) > _GC_SPAN and self.stash[_GC_SPAN]["sequenceNumber"] < msg["minimumSequenceNumber"]:
            self.min_seq_changed(int(msg["minimumSequenceNumber"]))

    def resolve(self, deltas: np.ndarray) -> None:
        """Fill the transformed contents of the last batch's lagging messages from its delta ranges
        (engine.deltas(doc) / mtr_get_deltas; op indices are relative to this document's op list)."""
        for stash, members, op_index in self.pending:
            mine = [i for i in op_index if i >= 0]
            sel = deltas[np.isin(deltas["op"], mine)] if mine else deltas[:0]
            ops = ops_from_deltas(members, sel, op_index)
            stash["contents"] = ops[0] if len(ops) == 1 else {"ops": ops, "type": 3}
        self.pending = []

    def min_seq_changed(self, min_seq: int) -> None:
        """processMinSequenceNumberChanged (sequence.ts:738-748)."""
        i = 0
        while i < len(self.stash) and self.stash[i]["sequenceNumber"] <= min_seq:
            i += 1
        if i:
            self.stash = self.stash[i:]

    def catchup_blob(self, min_seq: int | None = None) -> bytes | None:
        """summarizeMergeTree's catch-up messages (sequence.ts:675-695) as the legacy summary's
        ``catchupOps`` blob bytes, or None when there are none (snapshotlegacy.ts:174-179)."""
        if self.pending:
            raise RuntimeError("resolve() the last batch's deltas before summarizing")
        if not self.legacy:
            return None
        min_seq = self.msn if min_seq is None else min_seq
        self.min_seq_changed(min_seq)
        for m in self.stash:
            m["minimumSequenceNumber"] = min_seq
        if not self.stash:
            return None
        return to_utf8(js_stringify(self.stash))

    def load(self, blobs: dict, long_id: str, interner: Interner, header: str | None = None) -> None:
        """SharedSegmentSequence.loadCore (sequence.ts:557-611): the interval collections' `header` blob (if
        any) populated first, Client.load of the merge-tree summary `blobs` plus the catch-up messages, each
        checked against the collab window and applied as an ordinary message, then loadFinished attaches the
        collections (their intervals' references are created after the catch-up ops, sequence.ts:750-801)."""
        if header is not None:
            from .intervals import IntervalCollections

            self.intervals = IntervalCollections()
            self._intervals_call(self.intervals.populate, header)
        self._load_merge_tree(blobs, long_id, interner)
        if self.intervals is not None:
            self._intervals_call(self.intervals.attach, self)

    def _intervals_call(self, fn, *args):
        from .intervals import IntervalUnsupported

        try:
            return fn(*args)
        except IntervalUnsupported as e:
            raise Unsupported(str(e)) from e

    def interval_collection(self, label: str):
        """SharedSegmentSequence.getIntervalCollection (sequence.ts:445-447): created when absent."""
        from .intervals import IntervalCollections

        if self.intervals is None:
            self.intervals = IntervalCollections()
        return self.intervals.get(label)

    def interval_header(self, states: list) -> bytes | None:
        """The summary's `header` blob (summarizeCore, sequence.ts:467-480): the interval collections, ordered
        from the references' states at summary time (Engine.ref_states(doc)); None when there are none."""
        if self.intervals is None:
            return None
        h = self._intervals_call(self.intervals.serialize, states, self.current_seq)
        return None if h is None else to_utf8(h)

    def _load_merge_tree(self, blobs: dict, long_id: str, interner: Interner) -> None:
        msgs = self.load_summary(blobs, long_id, interner)
        # the loaded window: minSeq / currentSeq from the header (legacy: both the summary's minSeq)
        header = blobs["header"]
        chunk = parse(header) if isinstance(header, (str, bytes)) else header
        if chunk.get("version") == "1":
            meta = chunk["headerMetadata"]
            cur = int(meta["sequenceNumber"])
            win_min = int(meta["minSequenceNumber"]) if meta.get("minSequenceNumber") is not None else cur
        else:
            cur = int(chunk["chunkSequenceNumber"])
            ms = chunk.get("chunkMinSequenceNumber")
            win_min = int(ms) if ms is not None else cur
        self.msn = max(self.msn, win_min)
        for m in msgs:
            if (m["minimumSequenceNumber"] < win_min or m["referenceSequenceNumber"] < win_min
                    or m["sequenceNumber"] <= win_min or m["sequenceNumber"] <= cur):
                raise ValueError("Invalid catchup operations in snapshot")
            cur = int(m["sequenceNumber"])
            self.message(m, interner)
