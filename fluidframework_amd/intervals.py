"""Interval collections of a SharedString on the replay engine.

The reference keeps each collection (sequence/src/intervalCollection.ts:1428 ``IntervalCollection``, :788
``LocalIntervalCollection``) as two red-black trees over ``SequenceInterval``s whose endpoints are local
references (``createSequenceInterval``, :726-767) -- ordered by ``SequenceInterval.compare`` (:505-525:
start, then end, then the id string; ``compareReferencePositions``, merge-tree/src/referencePositions.ts:113-121)
-- and summarizes a collection as the in-order walk of the start tree (``LocalIntervalCollection.serialize``,
:1105-1112).  Here the endpoints are engine references (MTR_OP_REF_CREATE records in the document's batch,
created at the op's view and slid as ``createPositionReference`` does, :697-724) and the host keeps only the
intervals and their properties: the order is computed once, when a summary is written, from the
references' positions (mtr_get_ref_states).

Why the order needs no tree: a tree keeps a collection sorted by the current comparator as long as no two
intervals change their relative order without one of them being re-inserted.  Between two references that
order only changes when one of them slides (inserts, splits and zamboni keep it; a removed segment's
references are moved by ``slideAckedRemovedSegmentReferences``, mergeTree.ts:849-884), and every slide of an
interval endpoint re-inserts that interval (``addIntervalListeners``, intervalCollection.ts:1114-1159).  So the
in-order walk is the sort by the comparator at summary time, and at that time an endpoint is either held by a
live segment -- where the comparator is the position order -- or has no segment at all (position -1, the
smallest).  Anything else (an endpoint left on a removed segment, one whose segment dropped it, duplicate
ids, transient intervals, local ops while collaborating) is reported as Unsupported: such a document falls
back.  The oracle (oracle/intervals.py) restates the trees and the slide listeners themselves; the tests
compare the two.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

from . import abi
from .jsjson import js_key_order, js_number, js_stringify, js_truthy, parse, utf16_less

VALUE_TYPE = "sharedStringIntervalCollection"  # SequenceIntervalCollectionValueType.Name, intervalCollection.ts:1195
RANGE_LABELS = "referenceRangeLabels"         # reservedRangeLabelsKey
INTERVAL_ID = "intervalId"                     # reservedIntervalIdKey
LEGACY_PREFIX = "legacy"                       # LocalIntervalCollection.legacyIdPrefix, :795

# IntervalType (intervalCollection.ts:56-77)
SIMPLE, NEST, SLIDE_ON_REMOVE, TRANSIENT = 0x0, 0x1, 0x2, 0x4


class IntervalUnsupported(Exception):
    """The document's intervals take a path this host does not restate (the caller falls back)."""


def _js_to_string(v: Any) -> str:
    """`${v}` of a JSON value (SequenceInterval.getIntervalId, :554-560)."""
    if isinstance(v, str):
        return v
    if v is True:
        return "true"
    if v is False:
        return "false"
    if v is None:
        return "null"
    if isinstance(v, (int, float)):
        return js_number(v)
    raise IntervalUnsupported("an interval id that is not a string or number")


def add_props(props: dict, new: dict) -> None:
    """PropertiesManager.addProperties without combining ops or pending keys (segmentPropertiesManager.ts:60-157):
    each key of `new` in JS key order; null deletes, anything else sets (a re-added key goes last, as in JS)."""
    for k in js_key_order(new.keys()):
        v = new[k]
        if v is None:
            props.pop(k, None)
        else:
            props[k] = v


def _ref_types(itype: int, from_op_or_snapshot: bool) -> tuple[int, int]:
    """createSequenceInterval's endpoint ReferenceTypes (:735-756)."""
    if itype == TRANSIENT:
        raise IntervalUnsupported("transient interval")
    if itype == NEST:
        b, e = abi.REFTYPE_NEST_BEGIN, abi.REFTYPE_NEST_END
    else:
        b, e = abi.REFTYPE_RANGE_BEGIN, abi.REFTYPE_RANGE_END
    f = abi.REFTYPE_SLIDE_ON_REMOVE if from_op_or_snapshot else abi.REFTYPE_STAY_ON_REMOVE
    return b | f, e | f


def _int_pos(v: Any, what: str) -> int:
    if isinstance(v, bool) or not isinstance(v, (int, float)) or v != int(v):
        raise IntervalUnsupported(f"interval {what} that is not an integer position")
    return int(v)


UNASSIGNED_SEQ = -1   # UnassignedSequenceNumber (merge-tree/src/constants.ts)
UNIVERSAL_SEQ = 0     # UniversalSequenceNumber
_UNDEF = object()     # a JS `undefined` field (dropped by JSON.stringify)


class PropertiesManager:
    """merge-tree's PropertiesManager (segmentPropertiesManager.ts:24-170) as an interval's property bag uses it
    (SequenceInterval.addProperties, intervalCollection.ts:577-585): no combining ops, so no rewrite counts.  A local
    change (seq = UnassignedSequenceNumber while collaborating) counts its keys as pending; a sequenced change from
    another client leaves a pending key alone (shouldModifyKey); the ack of the local change decrements."""

    def __init__(self):
        self.pending: dict[str, int] | None = None  # pendingKeyUpdateCount

    def ack(self, props: dict) -> None:
        """ackPendingProperties -> decrementPendingCounts (:33-58)."""
        for k in js_key_order(props.keys()):
            if self.pending is not None and k in self.pending:
                if self.pending[k] <= 0:
                    raise AssertionError("0x05c")  # "Trying to update more annotate props than do exist!"
                self.pending[k] -= 1
                if self.pending[k] == 0:
                    del self.pending[k]

    def add(self, old: dict, new: dict, seq: int | None = None, collaborating: bool = False) -> dict:
        """addProperties (:60-157) without a combining op: each key of `new` in JS key order; null deletes.
        Returns the deltas (previous values, null when absent)."""
        if self.pending is None:
            self.pending = {}
        deltas = {}
        for k in js_key_order(new.keys()):
            if collaborating:
                if seq == UNASSIGNED_SEQ:
                    self.pending[k] = self.pending.get(k, 0) + 1
                elif not (seq == UNIVERSAL_SEQ or k not in self.pending):  # shouldModifyKey
                    continue
            deltas[k] = old.get(k)
            v = new[k]
            if v is None:
                old.pop(k, None)
            else:
                old[k] = v
        return deltas

    def copy_to(self, old: dict, new: dict, mgr: "PropertiesManager") -> None:
        """copyTo (:159-180): the properties and the pending counts."""
        for k in js_key_order(old.keys()):
            new[k] = old[k]
        mgr.pending = dict(self.pending or {})


@dataclass
class Interval:
    """One SequenceInterval: its endpoint references (engine ids) and their ReferenceTypes, the intervalType and
    the property bag with its PropertiesManager."""

    start: int
    end: int
    itype: Any
    props: dict
    kind: str  # "op" (a sequenced op: a detached endpoint is allowed, :685-694), "snapshot" or "local"
    stype: int = 0  # the endpoints' ReferenceTypes as the engine holds them (ackInterval reads StayOnRemove)
    etype: int = 0
    pm: PropertiesManager = field(default_factory=PropertiesManager)

    def id(self) -> str | None:
        v = self.props.get(INTERVAL_ID)
        return None if v is None else _js_to_string(v)


@dataclass
class Collection:
    """IntervalCollection + LocalIntervalCollection of one label: LocalIntervalCollection.intervalIdMap (:791),
    which holds every interval of the collection (two intervals with one id are not restated)."""

    label: str
    saved: list | None = None          # savedSerializedIntervals until attachGraph (:1465-1470, 1559-1578)
    by_id: dict = field(default_factory=dict)

    def _create(self, log, start: int, end: int, itype: Any, view: tuple | None, kind: str) -> Interval:
        """createSequenceInterval (:726-767) -> the two MTR_OP_REF_CREATE records, start first: an op's at its
        view, slid (getSlideToSegment); a snapshot's or a local one's at the local view."""
        if isinstance(itype, bool) or not isinstance(itype, (int, float)) or itype not in (SIMPLE, NEST, SLIDE_ON_REMOVE):
            raise IntervalUnsupported(f"intervalType {itype!r}")
        bt, et = _ref_types(int(itype), kind != "local")
        s = log.create_ref(start, bt, view=view, slide=kind == "op")
        e = log.create_ref(end, et, view=view, slide=kind == "op")
        return Interval(s, e, itype, {RANGE_LABELS: [self.label]}, kind, bt, et)

    def _add(self, iv: Interval) -> None:
        """LocalIntervalCollection.add (:1078-1082): the index and the id map."""
        i = iv.id()
        if i is None:
            raise AssertionError("0x2c0")  # "ID must be created before adding interval to collection"
        if i in self.by_id or i == "":
            raise IntervalUnsupported("two intervals with one id")  # the trees' put keeps the first key
        self.by_id[i] = iv

    def _remove(self, iv: Interval) -> None:
        """removeExistingInterval (:1015-1021)."""
        del self.by_id[iv.id()]

    @staticmethod
    def _release(log, iv: Interval, keep: Interval | None = None) -> None:
        """The endpoint references of `iv` that nothing reads again -- an interval a delete dropped, or the endpoints
        a change superseded (those `keep`, the changed interval, does not share) -- go back for reuse
        (DocLog.release_ref).  The reference leaves them in their segments' collections (removeExistingInterval
        only drops the index entries and listeners, :1007-1021), where nothing observes them."""
        for r in (iv.start, iv.end):
            if keep is None or r not in (keep.start, keep.end):
                log.release_ref(r)

    def attach(self, log) -> None:
        """attachGraph (:1531-1579): the saved intervals, created from the snapshot (local view,
        SlideOnRemove endpoints), in order."""
        saved, self.saved = self.saved or [], None
        for si in saved:
            props = ensure_serialized_id(si)
            iv = self._create(log, _int_pos(si.get("start"), "start"), _int_pos(si.get("end"), "end"),
                              si.get("intervalType"), None, "snapshot")
            add_props(iv.props, props)
            self._add(iv)

    def local_add(self, log, start: int, end: int, itype: int, props: dict | None) -> Interval:
        """IntervalCollection.add (:1635-1672) on a client that is not collaborating (a detached SharedString,
        generateSharedStrings.ts:42-52): StayOnRemove endpoints at the local view; the id must be given
        (otherwise addInterval draws a uuid, :1048)."""
        if log.collaborating:
            raise IntervalUnsupported("local interval ops while collaborating")
        if isinstance(itype, int) and itype & TRANSIENT:
            raise ValueError("Can not add transient intervals")
        if not props or props.get(INTERVAL_ID) is None:
            raise IntervalUnsupported("a local interval without an id (a random uuid)")
        iv = self._create(log, int(start), int(end), itype, None, "local")
        add_props(iv.props, props)
        self._add(iv)
        return iv

    def ack_add(self, log, si: dict, msg: dict) -> None:
        """ackAdd of a remote op (:2141-2184): ensureSerializedId, addInterval(start, end, type, props, op)."""
        ensure_serialized_id(si)
        view = (int(msg["referenceSequenceNumber"]), _client(msg))
        iv = self._create(log, _int_pos(si.get("start"), "start"), _int_pos(si.get("end"), "end"),
                          si.get("intervalType"), view, "op")
        props = si.get("properties")
        if isinstance(props, dict):
            add_props(iv.props, props)
        if INTERVAL_ID not in iv.props:  # properties[reservedIntervalIdKey] ??= uuid()
            raise IntervalUnsupported("an interval without an id (a random uuid)")
        self._add(iv)

    def ack_delete(self, log, si: dict) -> None:
        """ackDelete of a remote op (:2187-2208)."""
        i = ensure_serialized_id(si).get(INTERVAL_ID)
        iv = self.by_id.get(i) if isinstance(i, str) else None  # Map.get with the raw id
        if iv is not None:
            self._remove(iv)
            self._release(log, iv)

    def ack_change(self, log, si: dict, msg: dict) -> None:
        """ackChange of a remote op (:1859-1932): changeInterval (modify, :600-656: a new reference for each
        given endpoint, the others shared) when start or end is given, then addProperties(newProps, true, seq)."""
        props = si.get("properties")
        props = props if isinstance(props, dict) else {}
        if INTERVAL_ID not in props:
            raise AssertionError("0x3fe")  # id must exist on the interval
        i = props[INTERVAL_ID]
        new_props = {k: v for k, v in props.items() if k != INTERVAL_ID}
        iv = self.by_id.get(i) if isinstance(i, str) else None
        if iv is None:
            return
        start, end = si.get("start"), si.get("end")
        if ("start" in si and start is None) or ("end" in si and end is None):
            raise IntervalUnsupported("a change op with a null endpoint")
        if start is not None or end is not None:
            if iv.kind == "local":  # createPositionReference asserts an op's references SlideOnRemove (0x2f5)
                raise IntervalUnsupported("a remote change of a local (StayOnRemove) interval")
            view = (int(msg["referenceSequenceNumber"]), _client(msg))
            s, e = iv.start, iv.end
            # modify keeps each endpoint's ReferenceType (getRefType with an op)
            st, et = _ref_types(int(iv.itype), True)
            if start is not None:
                s = log.create_ref(_int_pos(start, "start"), st, view=view, slide=True)
            if end is not None:
                e = log.create_ref(_int_pos(end, "end"), et, view=view, slide=True)
            nv = Interval(s, e, iv.itype, dict(iv.props), "op")  # propertyManager.copyTo
            self._remove(iv)
            self._add(nv)
            self._release(log, iv, keep=nv)
            iv = nv
        add_props(iv.props, new_props)

    # ---------------------------------------------------------------- a collaborating client's own ops
    # (IntervalCollection.add / change / changeProperties / removeIntervalById, :1635-1793, their acks :1859-2208 and
    # rebaseLocalInterval :1963-2029).  `live` is the client (fluidframework_amd.live.SharedStringClient): its log, the
    # executor's answers (sync, local length, reference keys, rebase results) and the op submission.
    def _pending_changes(self, end: bool) -> dict:
        name = "pending_end" if end else "pending_start"
        if not hasattr(self, name):
            setattr(self, name, {})
        return getattr(self, name)

    def _lseq_map(self, rebased: bool = False) -> dict:
        """localSeqToSerializedInterval / localSeqToRebasedInterval (:1435-1442)."""
        name = "lseq_rebased" if rebased else "lseq_serialized"
        if not hasattr(self, name):
            setattr(self, name, {})
        return getattr(self, name)

    def has_pending_change(self, iid: str, end: bool) -> bool:
        return bool(self._pending_changes(end).get(iid))

    def _add_pending_change(self, iid: str, ser: dict) -> None:
        """addPendingChange (:1795-1815)."""
        if _field(ser, "start") is not _UNDEF:
            self._pending_changes(False).setdefault(iid, []).append(ser)
        if _field(ser, "end") is not _UNDEF:
            self._pending_changes(True).setdefault(iid, []).append(ser)

    def _remove_pending_change(self, ser: dict) -> None:
        """removePendingChange (:1817-1846)."""
        props = ser.get("properties") or {}
        iid = props.get(INTERVAL_ID)
        for end, key in ((False, "start"), (True, "end")):
            if _field(ser, key) is _UNDEF:
                continue
            pm = self._pending_changes(end)
            entries = pm.get(iid)
            if entries:
                pc = entries.pop(0)
                if not entries:
                    del pm[iid]
                if _field(pc, "start") != _field(ser, "start") or _field(pc, "end") != _field(ser, "end"):
                    raise AssertionError("Mismatch in pending changes")

    def _check_position(self, live, pos: Any) -> None:
        """createPositionReference without an op or a localSeq (:697-724): getContainingSegment at the local view must
        find a segment -- 0 <= pos < the local length (nodeMap, mergeTree.ts:2526-2570) -- or createPositionReference
        FromSegoff throws (:690-692)."""
        if isinstance(pos, bool) or not isinstance(pos, int):
            raise IntervalUnsupported("a local interval endpoint that is not an integer position")
        if not 0 <= pos < live.length():
            raise UsageError("Non-transient references need segment")

    def live_add(self, live, start: int, end: int, itype: int, props: dict | None) -> Interval:
        """IntervalCollection.add (:1635-1672) while collaborating: LocalIntervalCollection.addInterval (:1032-1052)
        with StayOnRemove endpoints at the local view, then the "add" op with a new localSeq."""
        if self.saved is not None:
            raise UsageError("attach must be called prior to adding intervals")
        if isinstance(itype, int) and itype & TRANSIENT:
            raise UsageError("Can not add transient intervals")
        self._check_position(live, start)
        self._check_position(live, end)
        iv = self._create(live.log, int(start), int(end), itype, None, "local")
        if props:
            iv.pm.add(iv.props, props)
        if iv.props.get(INTERVAL_ID) is None:  # properties[reservedIntervalIdKey] ??= uuid()
            import uuid

            iv.props[INTERVAL_ID] = str(uuid.uuid4())
        self._add(iv)
        ser = {"end": end, "intervalType": itype, "properties": iv.props, "sequenceNumber": live.current_seq,
               "start": start}
        lseq = live.next_local_seq()
        self._lseq_map()[lseq] = ser
        live.submit({"key": self.label, "type": "act", "value": {"opName": "add", "value": ser}}, {"localSeq": lseq})
        return iv

    def live_remove(self, live, iid: str) -> Interval | None:
        """removeIntervalById (:1706-1715) -> deleteExistingInterval(local) (:1674-1699): the "delete" op carries
        interval.serialize() (positions from localReferencePositionToPosition, :472-487)."""
        iv = self.by_id.get(iid) if isinstance(iid, str) else None
        if iv is None:
            return None
        keys = live.ref_keys()
        self._remove(iv)
        ser = {"end": keys[iv.end][0], "intervalType": iv.itype, "sequenceNumber": live.current_seq,
               "start": keys[iv.start][0], "properties": iv.props}
        self._release(live.log, iv)
        lseq = live.next_local_seq()
        live.submit({"key": self.label, "type": "act", "value": {"opName": "delete", "value": ser}}, {"localSeq": lseq})
        return iv

    def live_change_properties(self, live, iid: Any, props: dict) -> None:
        """changeProperties (:1723-1752): pending keys, a "change" op with only the properties (and the id)."""
        if not isinstance(iid, str):
            raise UsageError("Change API requires an ID that is a string")
        if not props:
            raise UsageError("changeProperties should be called with a property set")
        iv = self.by_id.get(iid)
        if iv is None:
            return
        iv.pm.add(iv.props, props, UNASSIGNED_SEQ, True)
        props[INTERVAL_ID] = iv.id()  # (the caller's object: the op's properties)
        ser = {"intervalType": iv.itype, "sequenceNumber": live.current_seq, "properties": props}
        lseq = live.next_local_seq()
        self._lseq_map()[lseq] = ser
        live.submit({"key": self.label, "type": "act", "value": {"opName": "change", "value": ser}}, {"localSeq": lseq})

    def _change_interval(self, live, iv: Interval, start: Any, end: Any, view: tuple | None = None,
                         local_seq: int | None = None) -> Interval:
        """LocalIntervalCollection.changeInterval (:1088-1103) -> SequenceInterval.modify (:600-656): a new reference
        for each given endpoint (with an op: at its view, slid, the old ReferenceType; without: StayOnRemove at the
        local view, or at the localSeq view of a rebase), the others shared, the properties and pending counts
        copied."""
        def new_ref(pos, old_type):
            if view is not None:
                if not old_type & SLIDE_ON_REMOVE_REF:
                    raise AssertionError("0x2f5")  # "op create references must be SlideOnRemove"
                return live.log.create_ref(_int_pos(pos, "endpoint"), old_type, view=view, slide=True), old_type
            t = (old_type & ~SLIDE_ON_REMOVE_REF) | STAY_ON_REMOVE_REF
            if local_seq is not None:
                return live.log.create_ref_at(_int_pos(pos, "endpoint"), t, live.current_seq, local_seq), t
            return live.log.create_ref(_int_pos(pos, "endpoint"), t), t

        s, st, e, et = iv.start, iv.stype, iv.end, iv.etype
        if start is not _UNDEF and start is not None:
            s, st = new_ref(start, iv.stype)
        if end is not _UNDEF and end is not None:
            e, et = new_ref(end, iv.etype)
        nv = Interval(s, e, iv.itype, {}, "op" if view is not None else iv.kind, st, et)
        iv.pm.copy_to(iv.props, nv.props, nv.pm)
        self._remove(iv)
        self._add(nv)
        self._release(live.log, iv, keep=nv)
        return nv

    def live_change(self, live, iid: Any, start: Any = _UNDEF, end: Any = _UNDEF) -> Interval | None:
        """IntervalCollection.change (:1761-1793)."""
        if not isinstance(iid, str):
            raise UsageError("Change API requires an ID that is a string")
        iv = self.by_id.get(iid)
        if iv is None:
            return None
        for v in (start, end):
            if v is not _UNDEF and v is not None:
                self._check_position(live, v)
        nv = self._change_interval(live, iv, start, end)
        # interval.serialize() with start / end / properties replaced (key order end, intervalType, sequenceNumber,
        # start, properties; an undefined endpoint is no JSON field)
        ser = {} if end is _UNDEF else {"end": end}
        ser.update({"intervalType": iv.itype, "sequenceNumber": live.current_seq})
        if start is not _UNDEF:
            ser["start"] = start
        ser["properties"] = {INTERVAL_ID: iv.id()}
        lseq = live.next_local_seq()
        self._lseq_map()[lseq] = ser
        live.submit({"key": self.label, "type": "act", "value": {"opName": "change", "value": ser}}, {"localSeq": lseq})
        self._add_pending_change(iid, ser)
        return nv

    def ack_interval(self, live, iv: Interval) -> None:
        """ackInterval (:2054-2138): each StayOnRemove-era endpoint without a pending change is slid as
        getSlideToSegment says (a new reference at the slide-to segment) and becomes SlideOnRemove -- one
        MTR_OP_REF_ACK record each."""
        if not (iv.stype & STAY_ON_REMOVE_REF) and not (iv.etype & STAY_ON_REMOVE_REF):
            return
        iid = iv.props.get(INTERVAL_ID)
        if not self.has_pending_change(iid, False):
            live.log.ack_ref(iv.start)
            iv.stype = (iv.stype & ~STAY_ON_REMOVE_REF) | SLIDE_ON_REMOVE_REF
        if not self.has_pending_change(iid, True):
            live.log.ack_ref(iv.end)
            iv.etype = (iv.etype & ~STAY_ON_REMOVE_REF) | SLIDE_ON_REMOVE_REF

    def live_process(self, live, name: str, params: Any, msg: dict, local: bool, meta: dict | None) -> None:
        """The ops map's process handlers (:1281-1325) with ackAdd / ackDelete / ackChange (:1859-1932, 2141-2208)."""
        if name != "delete" and not js_truthy(params):
            return  # "if params is undefined, the interval was deleted during rebasing"
        if not isinstance(params, dict):
            raise IntervalUnsupported("interval op parameters")
        si = dict(params)
        if name == "add":
            if not local:
                return self.ack_add(live.log, si, msg)
            self._lseq_map().pop(meta["localSeq"], None)
            iv = self.by_id.get((si.get("properties") or {}).get(INTERVAL_ID))
            if iv is not None:
                self.ack_interval(live, iv)
            return
        if name == "delete":
            if not local:
                self.ack_delete(live.log, si)
            return
        # change
        if local:
            self._lseq_map().pop(meta["localSeq"], None)
            self._remove_pending_change(si)
        props = si.get("properties")
        props = props if isinstance(props, dict) else {}
        if INTERVAL_ID not in props:
            raise AssertionError("0x3fe")  # id must exist on the interval
        iid = props[INTERVAL_ID]
        new_props = {k: v for k, v in props.items() if k != INTERVAL_ID}
        iv = self.by_id.get(iid) if isinstance(iid, str) else None
        if iv is None:
            return  # the interval has been removed locally; no-op
        if local:
            iv.pm.ack(props)
            self.ack_interval(live, iv)
            return
        start = _field(si, "start") if not self.has_pending_change(iid, False) else _UNDEF
        end = _field(si, "end") if not self.has_pending_change(iid, True) else _UNDEF
        if start is None or end is None:
            raise IntervalUnsupported("a change op with a null endpoint")
        if start is not _UNDEF or end is not _UNDEF:
            view = (int(msg["referenceSequenceNumber"]), _client(msg))
            iv = self._change_interval(live, iv, start, end, view=view)
        iv.pm.add(iv.props, new_props, int(msg["sequenceNumber"]), True)

    # ---- reconnect
    def rebase_positions(self, live, lseqs: list) -> dict:
        """computeRebasedPositions (:1507-1528) of the pending ops `lseqs`: rebasePositionWithSegmentSlide of each
        given endpoint (one MTR_OP_REBASE_POS record each, answered after one sync)."""
        recs = []
        for lseq in lseqs:
            original = self._lseq_map().get(lseq)
            if original is None:
                raise AssertionError("0x551")  # "Failed to store pending serialized interval info for this localSeq."
            for key in ("start", "end"):
                v = _field(original, key)
                if v is not _UNDEF:
                    recs.append((lseq, key, live.log.rebase_position(_int_pos(v, key), int(original["sequenceNumber"]),
                                                                     lseq)))
        res = live.rebase_results() if recs else {}
        out: dict = {}
        for lseq in lseqs:
            r = dict(self._lseq_map()[lseq])
            out[lseq] = r
        for lseq, key, rec in recs:
            out[lseq][key] = res[rec]
        return out

    def on_normalize(self, live) -> None:
        """The client's "normalize" listener (attachGraph, :1542-1551)."""
        keys = list(self._lseq_map().keys())
        if keys:
            self._lseq_map(True).update(self.rebase_positions(live, keys))

    def rebase_local(self, live, name: str, ser: dict, lseq: int) -> dict | None:
        """rebaseLocalInterval (:1963-2029) -> the resubmitted op's value; None = the op is a no-op."""
        if name == "delete":
            return ser  # deletion is by id: no rebasing
        rb = self._lseq_map(True).get(lseq)
        if rb is None:
            rb = self.rebase_positions(live, [lseq])[lseq]
        props = ser.get("properties")
        iid = props.get(INTERVAL_ID) if isinstance(props, dict) else None
        local = self.by_id.get(iid) if isinstance(iid, str) else None
        rebased = {}
        for key in ("start", "end"):
            v = _field(rb, key)
            if v is not _UNDEF:
                rebased[key] = v
        rebased.update({"intervalType": ser.get("intervalType"), "sequenceNumber": live.current_seq,
                        "properties": props})
        if name == "change" and (self.has_pending_change(iid, False) or self.has_pending_change(iid, True)):
            self._remove_pending_change(ser)
            self._add_pending_change(iid, rebased)
        if _field(rebased, "start") == abi.DETACHED_POSITION or _field(rebased, "end") == abi.DETACHED_POSITION:
            if local is not None:
                self._remove(local)
            return None
        if local is not None:
            self._change_interval(live, local, _field(rebased, "start"), _field(rebased, "end"), local_seq=lseq)
        return rebased

    # ---- queries (the trees' in-order walks and searches, intervalCollection.ts:864-992)
    def ordered(self, keys: list) -> list:
        """The intervals in SequenceInterval.compare order (:505-539; compareReferencePositions,
        referencePositions.ts:113-121): the start tree's in-order walk."""
        import functools

        ivs = list(self.by_id.values())
        return sorted(ivs, key=functools.cmp_to_key(lambda a, b: _iv_cmp(keys, a, b)))

    def serialize_live(self, keys: list, current_seq: int) -> dict:
        """LocalIntervalCollection.serialize (:1105-1112) of a live client: the compare order from the references'
        keys (endpoints on removed segments included), each endpoint at localReferencePositionToPosition."""
        out = []
        for iv in self.ordered(keys):
            props = {k: v for k, v in iv.props.items() if k != RANGE_LABELS}
            out.append([keys[iv.start][0], keys[iv.end][0], current_seq, iv.itype, props])
        return {"label": self.label, "intervals": out, "version": 2}

    def serialize(self, states: list, current_seq: int) -> dict:
        """LocalIntervalCollection.serialize (:1105-1112): the intervals in compare order, each
        compressInterval(interval.serialize()) (:139-151, 472-487)."""
        keyed = []
        for iv in self.by_id.values():
            a, b = _endpoint(states, iv.start, iv.kind == "op"), _endpoint(states, iv.end, iv.kind == "op")
            keyed.append((a, b, iv))
        keyed = _sorted(keyed)
        out = []
        for a, b, iv in keyed:
            props = {k: v for k, v in iv.props.items() if k != RANGE_LABELS}
            out.append([a, b, current_seq, iv.itype, props])
        return {"label": self.label, "intervals": out, "version": 2}


def _field(d: dict, key: str) -> Any:
    """d[key], _UNDEF when the key is absent (a JS undefined field)."""
    return d[key] if key in d else _UNDEF


class UsageError(Exception):
    """The reference's UsageError / LoggingError for a bad API call (nothing changes)."""


SLIDE_ON_REMOVE_REF = abi.REFTYPE_SLIDE_ON_REMOVE
STAY_ON_REMOVE_REF = abi.REFTYPE_STAY_ON_REMOVE


def _ref_key(keys: list, ref: int) -> tuple:
    """compareReferencePositions' key of a reference from Engine.ref_keys: no segment sorts first (and equal to any
    other segment-less reference); else (segment order, offset)."""
    _, _, k, off = keys[ref]
    if k == -1:
        return (0, 0, 0)
    if k < 0:
        raise IntervalUnsupported("an interval endpoint on a segment zamboni took out of the tree")
    return (1, k, off)


def _iv_cmp(keys: list, a: Interval, b: Interval) -> int:
    """SequenceInterval.compare (:505-525)."""
    for x, y in ((_ref_key(keys, a.start), _ref_key(keys, b.start)), (_ref_key(keys, a.end), _ref_key(keys, b.end))):
        if x != y:
            return -1 if x < y else 1
    ia, ib = a.id(), b.id()
    if ia and ib:
        return 1 if utf16_less(ib, ia) else -1 if utf16_less(ia, ib) else 0
    return 0


def _endpoint(states: list, ref: int, from_op: bool) -> int:
    """An endpoint's position, where the position order is compareReferencePositions' order."""
    pos, st = states[ref]
    seg, held, removed = st & abi.REF_ST_SEGMENT, st & abi.REF_ST_HELD, st & abi.REF_ST_REMOVED
    if seg and held and not removed and pos >= 0:
        return pos
    if not seg:  # no segment (created detached by an op, or slid off the string): smaller than any
        return abi.DETACHED_POSITION  # (referencePositions.ts:119); a local creation without one throws first
    raise IntervalUnsupported("an interval endpoint on a removed segment, or dropped by its segment")


def _sorted(keyed: list) -> list:
    """Sort by (start, end, id) with SequenceInterval.compare's id rule (JS string order)."""
    import functools

    def cmp(x, y):
        if x[0] != y[0]:
            return -1 if x[0] < y[0] else 1
        if x[1] != y[1]:
            return -1 if x[1] < y[1] else 1
        a, b = x[2].id(), y[2].id()
        if a and b:
            return 1 if utf16_less(b, a) else -1 if utf16_less(a, b) else 0
        return 0

    return sorted(keyed, key=functools.cmp_to_key(cmp))


def _client(msg: dict) -> str:
    c = msg.get("clientId")
    return "null" if c is None else str(c)


def ensure_serialized_id(si: dict) -> dict:
    """LocalIntervalCollection.ensureSerializedId (:838-858): a legacy id `legacy{start}-{end}` when the
    serialized interval has none.  Returns its (possibly new) property bag."""
    props = si.get("properties")
    if not isinstance(props, dict) or props.get(INTERVAL_ID) is None:
        lid = f"{LEGACY_PREFIX}{_js_to_string(si.get('start'))}-{_js_to_string(si.get('end'))}"
        props = dict(props) if isinstance(props, dict) else {}
        props[INTERVAL_ID] = lid
        si["properties"] = props
    return props


def decompress(ci: list, label: str) -> dict:
    """decompressInterval (:122-133)."""
    props = dict(ci[4]) if len(ci) > 4 and isinstance(ci[4], dict) else {}
    props[RANGE_LABELS] = [label]
    return {"start": ci[0], "end": ci[1], "sequenceNumber": ci[2], "intervalType": ci[3], "properties": props}


class IntervalCollections:
    """SharedSegmentSequence.intervalCollections (sequence/src/sequence.ts:186, a DefaultMap of
    IntervalCollection, defaultMap.ts): populate from the summary's `header` blob, attach after the merge-tree
    load, remote "act" ops, local adds before collaboration, and the `header` blob of a summary."""

    def __init__(self):
        self.data: dict[str, Collection] = {}  # DefaultMap.data (a Map: insertion order)
        self.attached = False

    def populate(self, header: str | dict) -> None:
        """DefaultMap.populate (defaultMap.ts:254-282): Object.entries of the parsed blob (JS key order)."""
        j = parse(header) if isinstance(header, str) else header
        for key in js_key_order(j.keys()):
            ser = j[key]
            if ser.get("type") in ("Plain", "Shared"):
                continue
            if ser.get("type") != VALUE_TYPE:
                raise IntervalUnsupported(f"value type {ser.get('type')!r}")
            label = key[len("intervalCollections/"):] if key.startswith("intervalCollections/") else key
            v = ser.get("value")
            if isinstance(v, list):
                saved = [dict(x) for x in v]
            else:
                saved = [decompress(ci, v["label"]) for ci in v["intervals"]]
            c = Collection(label, saved=saved)
            # IntervalCollection.attachGraph(client, key) uses the DefaultMap key (sequence.ts:797-800)
            self.data[label] = c

    def attach(self, log) -> None:
        """SharedSegmentSequence.loadFinished -> initializeIntervalCollections (sequence.ts:750-801)."""
        for c in self.data.values():
            c.attach(log)
        self.attached = True

    def get(self, label: str) -> Collection:
        """DefaultMap.get -> createCore (defaultMap.ts:210-213, 339-349): a new, attached, empty collection."""
        c = self.data.get(label)
        if c is None:
            c = self.data[label] = Collection(label)
        return c

    def local_add(self, log, label: str, start: int, end: int, itype: int, props: dict | None) -> Interval:
        return self.get(label).local_add(log, start, end, itype, props)

    def process(self, log, contents: dict, msg: dict) -> None:
        """DefaultMap's "act" handler (defaultMap.ts:386-395) and the ops map (intervalCollection.ts:1266-1326)
        for a sequenced message of another client."""
        if _client(msg) == log.observer_id:
            raise IntervalUnsupported("acks of local interval ops")
        key = contents.get("key")
        if not isinstance(key, str):
            raise IntervalUnsupported("an interval op without a string key")
        value = contents.get("value") or {}
        name = value.get("opName")
        params = value.get("value")
        c = self.get(key)
        if name not in ("add", "delete", "change"):
            raise IntervalUnsupported(f"interval op {name!r}")  # getOpHandler throws
        if name != "delete" and not js_truthy(params):
            return  # "if params is undefined, the interval was deleted during rebasing"
        if not isinstance(params, dict):
            raise IntervalUnsupported("interval op parameters")
        params = dict(params)
        if name == "add":
            c.ack_add(log, params, msg)
        elif name == "delete":
            c.ack_delete(log, params)
        else:
            c.ack_change(log, params, msg)

    def serialize(self, states: list, current_seq: int, live: bool = False) -> str | None:
        """summarizeCore's `header` blob (sequence.ts:467-480): JSON.stringify of {key: {type, value}} over the
        collections (DefaultMap.serialize, defaultMap.ts:231-248); None when there are none.  live: `states` are a
        live client's reference keys (Engine.ref_keys)."""
        if not self.data:
            return None
        out = {}
        for key, c in self.data.items():
            if c.saved is not None:
                raise IntervalUnsupported("a collection that was never attached")
            v = c.serialize_live(states, current_seq) if live else c.serialize(states, current_seq)
            out[key] = {"type": VALUE_TYPE, "value": v}
        return js_stringify(out)
