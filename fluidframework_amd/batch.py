"""Host-side packing of ISequencedDocumentMessage streams into the engine's batch format.

This is the code a scribe-like summarizer runs before handing a batch to the engine; it mirrors the
message handling the reference does on the JS thread:

* ``Client.applyMsg`` registers ``msg.clientId`` (first-seen short ids, client.ts:858-860, 673-688),
  routes ``type == "op"`` to ``applyRemoteOp`` (client.ts:802-829) and always finishes with
  ``updateSeqNumbers(msn, seq)`` (client.ts:874-887).
* ``specToSegment`` (packages/dds/sequence/src/sequenceFactory.ts:26-38) accepts a string, a
  ``{text, props}`` object or a ``{marker: {refType}, props}`` object.
* GROUP ops (ops.ts:113) become several records with one sequence number.

Property keys/values are interned into global tables (see include/mtr_types.h).  Remote annotates
with a ``combiningOp`` are encoded per include/mtr_types.h (MTR_COMB_*); ``relativePos1/2`` become
MTR_OP_RELPOS records resolved by the engine against the marker the id maps to.  A client's own edits
while collaborating are local ops (pending until acked) and its own sequenced messages become
MTR_OP_ACK records (Client.applyMsg -> ackPendingSegment, client.ts:641-663, 866-869).  Features the
engine does not build (local combining annotates, combining results that are not plain JSON values,
marker ids whose mapping depends on block-update order) make the document ``unsupported`` (the
reference-side shim keeps such documents on the TypeScript Client).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Any, Iterable

import numpy as np

from . import abi
from .jsjson import (array_index, eq_key, js_key_order, js_string, js_stringify, js_truthy, parse, plain_value, to_utf8,
                     utf16_less)


class Unsupported(Exception):
    """A message uses a feature the engine does not implement (document must fall back)."""


# short client ids one engine document can hold (include/mtr_types.h MTR_MAX_CLIENTS): the engine
# keeps a short id in 8 bits; a document that registers more stays on the TypeScript Client
MAX_CLIENTS = 253


class Interner:
    """Global key / value / prop-op tables (ids are stable across batches)."""

    def __init__(self) -> None:
        self.keys: dict[str, int] = {}
        self.key_bytes: list[bytes] = []
        self.key_index: list[int] = []
        self.vals: dict[str, int] = {}
        self.val_bytes: list[bytes] = []
        self.val_eq: list[int] = []
        self.eq_ids: dict[str, int] = {}
        self.propops: list[list[tuple[int, int]]] = []
        self.never: dict[str, int] = {}  # never-equal values (NaN, {value: undefined, seq}) by JSON text

    def _add_value(self, s: str, eq: int) -> int:
        i = len(self.val_bytes)
        self.val_bytes.append(to_utf8(s))
        self.val_eq.append(eq)
        return i

    @staticmethod
    def value_flags(v: Any) -> int:
        """MTR_VEQ_* bits of a JSON value (include/mtr_types.h)."""
        f = 0
        if not js_truthy(v):
            f |= abi.VEQ_FALSY
        if isinstance(v, (str, list, dict)):  # value + undefined concatenates (properties.ts:39)
            f |= abi.VEQ_INCR_STR
        if isinstance(v, dict):
            sq = v.get("seq")
            if isinstance(sq, (int, float)) and not isinstance(sq, bool) and sq == -1:
                f |= abi.VEQ_CONS_MUT  # consensus would set cv.seq in place (properties.ts:56-60)
        return f

    def never_value(self, s: str) -> int:
        """A value matchProperties never matches, not even with itself (NaN -> "null"; a consensus value
        {value: undefined, seq} -> '{"seq":N}'): its own class, flagged MTR_VEQ_NEVER."""
        i = self.never.get(s)
        if i is None:
            e = len(self.eq_ids)
            self.eq_ids["never#%d" % e] = e
            i = self._add_value(s, e | abi.VEQ_NEVER)
            self.never[s] = i
        return i

    def nan(self) -> int:
        return self.never_value("null")

    def key(self, k: str) -> int:
        i = self.keys.get(k)
        if i is None:
            i = len(self.key_bytes)
            self.keys[k] = i
            self.key_bytes.append(to_utf8(js_string(k)[1:-1]))
            ix = array_index(k)
            self.key_index.append(abi.NOT_INDEX if ix is None else ix)
        return i

    def value(self, v: Any) -> int:
        if v is None:
            return abi.NULL_VALUE
        if not plain_value(v):
            raise Unsupported("property value with a nested null or an empty container")
        s = js_stringify(v)
        i = self.vals.get(s)
        if i is None:
            ek = eq_key(v)
            e = self.eq_ids.setdefault(ek, len(self.eq_ids))
            i = self._add_value(s, e | self.value_flags(v))
            self.vals[s] = i
        return i

    def propop(self, props: dict) -> int:
        pairs = [(self.key(k), self.value(props[k])) for k in js_key_order(props.keys())]
        self.propops.append(pairs)
        return len(self.propops) - 1

    def combining(self, props: dict, co: Any, seq: int) -> tuple[int, int]:
        """A remote annotate with combiningOp `co` -> (prop-op, payload2) per include/mtr_types.h."""
        if not isinstance(props, dict):
            raise Unsupported("annotate props")
        if not js_truthy(co):  # `op ? op : undefined` (segmentPropertiesManager.ts:93-94)
            return self.propop(props), abi.COMB_NONE
        if not isinstance(co, dict):
            raise Unsupported("combiningOp")
        name = co.get("name")
        if name == "rewrite":
            return self.propop(props), abi.COMB_REWRITE
        mode = {"incr": abi.COMB_INCR, "consensus": abi.COMB_CONSENSUS}.get(name, abi.COMB_KEEP)
        absent = self._value_or_null(combine_absent(co, seq))
        pairs = [(self.key(k), absent) for k in js_key_order(props.keys())]
        self.propops.append(pairs)
        return len(self.propops) - 1, mode | ((self.nan() << 3) if mode == abi.COMB_INCR else 0)

    def _value_or_null(self, r: Any) -> int:
        if r is _NAN:
            return self.nan()
        if isinstance(r, _Never):
            return self.never_value(r.json)
        if r is None:  # combine gave null: `delete oldProps[key]` (absent stays absent)
            return abi.NULL_VALUE
        return self.value(r)


class _Never:
    def __init__(self, json_text: str) -> None:
        self.json = json_text


_NAN = object()
_JS_UNDEF = object()


def combine_absent(co: dict, seq: int) -> Any:
    """combine(co, undefined, undefined, seq) (properties.ts:24-69) for a key the segment lacks: the
    value the key takes (a JSON value, None = null, _NAN, or a _Never value)."""
    cur = co.get("defaultValue", _JS_UNDEF)
    name = co.get("name")
    if name == "incr":
        if cur is _JS_UNDEF or cur is None or isinstance(cur, (bool, int, float)):
            return _NAN  # NaN < minValue is false: no clamp
        if not isinstance(cur, str):
            raise Unsupported("incr of a non-primitive default value")
        r = cur + "undefined"
        mv = co.get("minValue", _JS_UNDEF)
        if mv is not _JS_UNDEF and js_truthy(mv):
            if isinstance(mv, str):
                if utf16_less(r, mv):
                    r = mv
            elif not isinstance(mv, (int, float)) or isinstance(mv, bool):
                raise Unsupported("incr minValue comparison")
            # string < number: ToNumber("...undefined") is NaN -> false
        return r
    if name == "consensus":
        if cur is _JS_UNDEF:
            return _Never('{"seq":%d}' % seq)  # {value: undefined, seq}: JSON.stringify drops `value`
        if cur is None:
            raise Unsupported("consensus on a null default (TypeError in the reference)")
        if isinstance(cur, dict):
            sq = cur.get("seq")
            if isinstance(sq, (int, float)) and not isinstance(sq, bool) and sq == -1:
                cur = dict(cur)
                cur["seq"] = seq
        return cur
    if cur is _JS_UNDEF:
        raise Unsupported("combiningOp without a default leaves an explicit undefined property")
    return cur


def _local_comb(co: Any) -> int:
    """A local annotate's combiningOp as its ack / rollback records carry it (pos1): none, "rewrite"
    (PropertiesManager.pendingRewriteCount, segmentPropertiesManager.ts:72-80, 109-112), or another name (its
    pending key counts are kept like a plain annotate's, :126-138)."""
    if not js_truthy(co):
        return abi.COMB_NONE
    if not isinstance(co, dict):
        raise Unsupported("combiningOp")
    if co.get("name") == "rewrite":
        return abi.COMB_REWRITE
    return {"incr": abi.COMB_INCR, "consensus": abi.COMB_CONSENSUS}.get(co.get("name"), abi.COMB_KEEP)


@dataclass
class DocLog:
    """Per-document host state: client registry plus the ops/text of the batch being built."""

    observer_id: str | None = None
    clients: list[str] = field(default_factory=list)
    client_ix: dict[str, int] = field(default_factory=dict)
    ops: list[tuple] = field(default_factory=list)
    text: list[int] = field(default_factory=list)
    unsupported: str | None = None
    collaborating: bool = False
    # MergeTree.idToSegment (mergeTree.ts:549,668) as the host sees it: id key -> marker ordinal
    n_markers: int = 0
    marker_ids: dict = field(default_factory=dict)
    marker_dup: set = field(default_factory=set)  # ids mapped to two markers: block-update order decides
    marker_id_annotated: bool = False              # an annotate touched "markerId": remapped by blockUpdate
    n_refs: int = 0                                # reference ids handed out (MTR_OP_REF_CREATE ids; high-water mark)
    free_refs: list = field(default_factory=list)  # ids released for reuse (MTR_REF_SLOT), a stack
    # the merge-tree client's currentSeq (collabWindow.currentSeq) as the host sees it: interval ops do not move it
    current_seq: int = 0
    intervals: Any = None                          # fluidframework_amd.intervals.IntervalCollections, when used

    def short_id(self, long_id: str) -> int:
        """Client.getOrAddShortClientId (client.ts:673-677)."""
        i = self.client_ix.get(long_id)
        if i is None:
            i = self.add_long_id(long_id)
        return i

    def add_long_id(self, long_id: str) -> int:
        """Client.addLongClientId (client.ts:685-688): always a new short id (re-adding a known long
        id re-points it, as clientNameToIds.put does)."""
        if len(self.clients) >= MAX_CLIENTS:
            raise Unsupported(f"more than {MAX_CLIENTS} client ids in one document")
        i = len(self.clients)
        self.client_ix[long_id] = i
        self.clients.append(long_id)
        return i

    def _text(self, s: str) -> tuple[int, int]:
        u = np.frombuffer(s.encode("utf-16-le", "surrogatepass"), dtype="<u2")
        off = len(self.text)
        self.text.extend(u.tolist())
        return off, len(u)

    @staticmethod
    def _id_key(v: Any):
        """Map key of a marker id (SameValueZero; objects only match themselves: never from JSON)."""
        if isinstance(v, bool):
            return ("b", v)
        if isinstance(v, (int, float)):
            return ("n", float(v))
        if isinstance(v, str):
            return ("s", v)
        return None

    def _map_marker(self, props: Any) -> int:
        """Marker.getId (mergeTreeNodes.ts:612-617) truthy -> mapIdToSegment: the new marker ordinal + 1
        for the record's payload2 (0 = no id)."""
        if not isinstance(props, dict) or not js_truthy(props.get("markerId")):
            return 0
        k = self._id_key(props["markerId"])
        o = self.n_markers
        self.n_markers += 1
        if k is not None:
            if k in self.marker_ids:
                self.marker_dup.add(k)
            self.marker_ids[k] = o
        return o + 1

    def _relpos(self, rp: Any, which: int, short: int, seq: int, ref: int, msn: int) -> None:
        """getValidOpRange's posFromRelativePos (client.ts:527-545, mergeTree.ts:1371-1395) -> one
        MTR_OP_RELPOS record ahead of the op."""
        if not isinstance(rp, dict):
            raise Unsupported("relative position")
        rid = rp.get("id")
        k = self._id_key(rid) if js_truthy(rid) else None
        if k is None or k not in self.marker_ids:
            raise Unsupported("relative position without a mapped marker (position -1)")
        if k in self.marker_dup or self.marker_id_annotated:
            raise Unsupported("relative position on a marker id remapped by block updates")
        off = rp.get("offset", _JS_UNDEF)
        flags = abi.REL_BEFORE if js_truthy(rp.get("before")) else 0
        if off is not _JS_UNDEF:
            if off is None:  # pos += null adds 0
                off = 0
            if isinstance(off, bool) or not isinstance(off, (int, float)) or off != int(off):
                raise Unsupported("relative position offset")
            flags |= abi.REL_OFFSET
            off = int(off)
        else:
            off = 0
        self.ops.append((abi.OP_RELPOS, 0, short, seq, ref, msn, self.marker_ids[k], which, off & 0xFFFFFFFF, flags))

    def _position(self, op: dict, key: str, which: int, short: int, seq: int, ref: int, msn: int) -> int:
        """op.pos1 / op.pos2, or its relativePos (resolved by the engine): the record's field value."""
        v = op.get(key, _JS_UNDEF)
        if v is _JS_UNDEF and js_truthy(op.get("relative" + key[0].upper() + key[1:])):
            self._relpos(op["relative" + key[0].upper() + key[1:]], which, short, seq, ref, msn)
            return 0
        if v is _JS_UNDEF or v is None or isinstance(v, bool) or not isinstance(v, (int, float)):
            raise Unsupported(f"op without a usable {key}")
        return int(v)

    def _seg(self, spec: Any, interner: Interner, map_marker: bool = True) -> tuple[int, int, int, int]:
        """-> (flags, payload, payload2, propop)"""
        if isinstance(spec, str):
            off, n = self._text(spec)
            return 0, off, n, -1
        if isinstance(spec, dict) and "text" in spec:
            off, n = self._text(spec["text"])
            props = spec.get("props")
            if props is not None:  # `if (props)` in TextSegment.make: {} is truthy
                return abi.F_PROPS, off, n, interner.propop(props)
            return 0, off, n, -1
        if isinstance(spec, dict) and "marker" in spec:
            m = spec["marker"] or {}
            flags = abi.F_MARKER
            ref = m.get("refType")
            if ref is None:
                flags |= abi.F_NOREF
                ref = 0
            props = spec.get("props")
            pp = -1
            if props is not None:
                flags |= abi.F_PROPS
                pp = interner.propop(props)
            return flags, int(ref), self._map_marker(props) if map_marker else 0, pp
        raise Unsupported("unrecognized segment spec")

    # -- local edits (Client.insertSegmentLocal / removeRangeLocal / annotateRangeLocal, client.ts:225-260):
    # before collaboration they are final (pre-attach SharedString, TestClient.insertTextLocal); while
    # collaborating each is a pending op the engine keeps in a SegmentGroup until this client's sequenced
    # message for it arrives (message() turns that into MTR_OP_ACK records)
    def local_insert(self, pos: int, spec: Any, interner: Interner) -> None:
        flags, p1, p2, pp = self._seg(spec, interner)
        self.ops.append((abi.OP_LOCAL_INSERT, flags, 0, self._local_seq(), 0, 0, pos, pp, p1, p2))

    def _local_seq(self) -> int:
        """seq of a local op record: UnassignedSequenceNumber (-1) while collaborating (include/mtr_types.h)."""
        return -1 if self.collaborating else 0

    def local_remove(self, start: int, end: int) -> None:
        self.ops.append((abi.OP_LOCAL_REMOVE, 0, 0, self._local_seq(), 0, 0, start, end, 0, 0))

    def local_annotate(self, start: int, end: int, props: dict, interner: Interner, combining_op: Any = None) -> None:
        if isinstance(props, dict) and "markerId" in props:
            self.marker_id_annotated = True
        comb = _local_comb(combining_op)
        if comb in (abi.COMB_NONE, abi.COMB_REWRITE):
            pp = interner.propop(props)
        else:  # combine(op, previousValue, undefined, seq) at UnassignedSequenceNumber (while collaborating) or
            # UniversalSequenceNumber: the prop-op holds each key's absent-key result (a remote one's encoding)
            pp, comb = interner.combining(props, combining_op, -1 if self.collaborating else 0)
        self.ops.append((abi.OP_LOCAL_ANNOTATE, 0, 0, self._local_seq(), 0, 0, start, end, pp, comb))

    def rollback(self, op: dict, interner: Interner) -> None:
        """Client.rollback (client.ts:421-423 -> MergeTree.rollback, mergeTree.ts:2049-2159) of the newest
        pending local op `op` (its contents)."""
        t = op.get("type")
        pp = comb = 0
        if t == 2:
            comb = _local_comb(op.get("combiningOp"))
            pp = interner.propop(op.get("props") or {})
        elif t not in (0, 1):
            raise Unsupported(f"rollback of op type {t}")
        self.ops.append((abi.OP_ROLLBACK, 0, 0, -1, 0, 0, comb, 0, pp, t))

    def regenerate(self, op: dict) -> int:
        """Client.regeneratePendingOp (client.ts:917-960) of the oldest pending local op `op` (its contents;
        a GROUP is one record per member, in order).  Returns the index of the first record in this batch's
        op list: the MTR_DELTA_REGEN records of record k carry op = k (fluidframework_amd.regen builds the
        new op from them)."""
        members = op["ops"] if op.get("type") == 3 else [op]
        first = len(self.ops)
        for m in members:
            t = m.get("type")
            if t not in (0, 1, 2):
                raise Unsupported(f"regenerate of op type {t}")
            self.ops.append((abi.OP_REGENERATE, abi.F_DELTA, 0, -1, 0, 0, 0, 0, 0, t))
        return first

    # -- local references (localReference.ts)
    def _new_ref_id(self) -> int:
        if self.free_refs:
            return self.free_refs.pop()
        self.n_refs += 1
        return self.n_refs - 1

    def create_ref(self, pos: int, ref_type: int, view: tuple | None = None, slide: bool = False) -> int:
        """createPositionReference (sequence/src/intervalCollection.ts:697-724): Client.getContainingSegment(pos,
        view) (client.ts:1065-1078; view = (referenceSequenceNumber, long client id), None = the local view),
        Client.getSlideToSegment when `slide` (client.ts:1085-1099), then createLocalReferencePosition
        (client.ts:377-389) -- a detached reference when no segment holds pos.  Returns the reference id: a released
        one when there is one (MTR_REF_SLOT), else the next."""
        if view is None:
            short, ref, flags = 0, 0, abi.REF_LOCALVIEW
        else:
            short, ref, flags = self.short_id(str(view[1])), int(view[0]), 0
        if slide:
            flags |= abi.REF_SLIDE
        rid = self._new_ref_id()
        self.ops.append((abi.OP_REF_CREATE, 0, short, 0, ref, 0, int(pos), rid, int(ref_type), flags | abi.REF_SLOT))
        return rid

    def create_ref_at(self, pos: int, ref_type: int, ref_seq: int, local_seq: int) -> int:
        """createPositionReference with a localSeq (sequence/src/intervalCollection.ts:697-724, a rebase's
        changeInterval): getContainingSegment(pos, undefined, localSeq) -- this client's view at (ref_seq =
        currentSeq, localSeq) -- then createLocalReferencePosition; no segment = a detached reference."""
        rid = self._new_ref_id()
        self.ops.append((abi.OP_REF_CREATE, 0, 0, 0, int(ref_seq), int(local_seq), int(pos), rid, int(ref_type),
                         abi.REF_LSEQ | abi.REF_SLOT))
        return rid

    def release_ref(self, ref_id: int, remove: bool = True) -> None:
        """The host is done with reference `ref_id`; its id is reused by the next create (MTR_REF_SLOT).  remove:
        Client.removeLocalReferencePosition first (client.ts:394-396) -- a reference a segment's collection may
        hold (an interval endpoint that a change superseded or a delete dropped: nothing reads it again, and the
        reference's own left-over LocalReferencePositions are unobservable); a Transient query reference is held by
        no collection and needs no record (localReference.ts:260-298)."""
        self._check_ref(ref_id)
        if remove:
            self.ops.append((abi.OP_REF_REMOVE, 0, 0, 0, 0, 0, 0, 0, int(ref_id), 0))
        self.free_refs.append(int(ref_id))

    def _check_ref(self, ref_id: int) -> None:
        if not 0 <= ref_id < self.n_refs or ref_id in self.free_refs:
            raise ValueError(f"no local reference {ref_id}")

    def ack_ref(self, ref_id: int) -> None:
        """IntervalCollection.ackInterval for one endpoint reference (MTR_OP_REF_ACK, include/mtr_types.h)."""
        self._check_ref(ref_id)
        self.ops.append((abi.OP_REF_ACK, 0, 0, 0, 0, 0, 0, 0, int(ref_id), 0))

    def rebase_position(self, pos: int, seq_from: int, local_seq: int) -> int:
        """IntervalCollection.rebasePositionWithSegmentSlide(pos, seqNumberFrom, localSeq) (MTR_OP_REBASE_POS);
        returns the record's index in this batch (its MTR_DELTA_REBASE result carries it)."""
        self.ops.append((abi.OP_REBASE_POS, abi.F_DELTA, 0, 0, int(seq_from), int(local_seq), int(pos), 0, 0, 0))
        return len(self.ops) - 1

    def bump_local_seq(self) -> None:
        """IntervalCollection.getNextLocalSeq: ++collabWindow.localSeq (MTR_OP_LSEQ)."""
        self.ops.append((abi.OP_LSEQ, 0, 0, 0, 0, 0, 0, 0, 0, 0))

    def remove_ref(self, ref_id: int) -> None:
        """Client.removeLocalReferencePosition (client.ts:394-396)."""
        self._check_ref(ref_id)
        self.ops.append((abi.OP_REF_REMOVE, 0, 0, 0, 0, 0, 0, 0, int(ref_id), 0))

    def local_op(self, op: dict, interner: Interner) -> None:
        """A local merge-tree op (the contents this client submits): insert / remove / annotate."""
        t = op.get("type")
        if t == 0:
            self.local_insert(int(op["pos1"]), op["seg"], interner)
        elif t == 1:
            self.local_remove(int(op["pos1"]), int(op["pos2"]))
        elif t == 2:
            self.local_annotate(int(op["pos1"]), int(op["pos2"]), op.get("props") or {}, interner, op.get("combiningOp"))
        else:
            raise Unsupported(f"local op type {t}")

    def apply_stashed_op(self, op: dict, interner: Interner):
        """Client.applyStashedOp (client.ts:830-856): a stashed op of this client (its contents, from a previous
        session) applied as a local op; a GROUP applies each member.  Returns the local op metadata the reference
        returns (one token per member op: the pending SegmentGroup it made, which regeneratePendingOp later takes
        from the head of the pending queue)."""
        if op.get("type") == 3:
            return [self.apply_stashed_op(m, interner) for m in op["ops"]]
        if not self.collaborating:  # peekPendingSegmentGroups() is undefined: "Applying op must generate a pending segment"
            raise AssertionError("0x2db")
        self.local_op(op, interner)
        self.n_stashed = getattr(self, "n_stashed", 0) + 1
        return {"stashed": self.n_stashed, "type": op.get("type")}

    def start_collab(self, long_id: str | None, min_seq: int = 0, current_seq: int = 0) -> None:
        """Client.startOrUpdateCollaboration (client.ts:1133-1155): an undefined id keeps the client
        local (detached container); the first id registers a new short id (addLongClientId, even for
        a long id seen before) and starts collaboration as that client; a later id renames the
        observer (its short id now maps back to the new long id, and both long ids map to it)."""
        if long_id is None:
            return
        if self.observer_id is None:
            self.observer_id = long_id
            me = self.add_long_id(long_id)
            self.collaborating = True
            self.current_seq = current_seq
            self.ops.append((abi.OP_START_COLLAB, 0, me, current_seq, 0, min_seq, 0, 0, 0, 0))
        else:
            me = self.client_ix[self.observer_id]
            self.observer_id = long_id
            self.client_ix[long_id] = me
            self.clients[me] = long_id

    # -- loading a summary (SnapshotLoader, snapshotLoader.ts:41-257)
    def _snapshot_seg(self, spec: Any, interner: Interner, op_type: int, flags: int) -> None:
        """specToSegment with merge info (snapshotLoader.ts:88-128) -> one LOAD / APPEND record."""
        # a loaded live marker is mapped by reloadFromSegments' blockUpdate (addNodeReferences,
        # mergeTree.ts:297-306, localNetLength > 0 only); a body segment by blockInsert (:1655-1662)
        removed = isinstance(spec, dict) and "json" in spec and spec.get("removedSeq") is not None
        live = op_type != abi.OP_LOAD or not removed
        if isinstance(spec, dict) and "json" in spec:  # hasMergeInfo, snapshotChunks.ts:80-84
            f, p1, p2, pp = self._seg(spec["json"], interner, map_marker=live)
            client = self.short_id(spec["client"]) if spec.get("client") is not None else abi.CLIENT_NONCOLLAB
            seq = int(spec["seq"]) if spec.get("seq") is not None else 0
            removers = []
            if spec.get("removedClient") is not None:
                removers = [self.short_id(spec["removedClient"])]
            if spec.get("removedClientIds") is not None:
                removers = [self.short_id(x) for x in spec["removedClientIds"]]
            rseq = int(spec["removedSeq"]) if spec.get("removedSeq") is not None else -1
        else:
            f, p1, p2, pp = self._seg(spec, interner, map_marker=live)
            client, seq, removers, rseq = abi.CLIENT_NONCOLLAB, 0, [], -1
        roff = len(self.text)
        self.text.extend(removers)
        self.ops.append((op_type, f | flags, client, seq, rseq, len(removers), roff, pp, p1, p2))

    def load_summary(self, blobs: dict, long_id: str, interner: Interner) -> list:
        """Client.load from the blobs of a merge-tree summary (V1 or legacy): header segments via
        reloadFromSegments, startOrUpdateCollaboration(long_id, minSeq, seq), body segments appended.
        Returns the legacy catch-up messages (the caller applies them as ordinary messages)."""
        header = blobs["header"]
        chunk = parse(header) if isinstance(header, str) else header
        if chunk.get("version") == "1":
            segs, meta = chunk["segments"], chunk["headerMetadata"]
        else:  # toLatestVersion of a legacy chunk, snapshotChunks.ts:151-200
            segs = chunk["segmentTexts"]
            meta = chunk.get("headerMetadata") or {
                "orderedChunkMetadata": [{"id": "header"}] + (
                    [{"id": "body"}] if chunk["chunkLengthChars"] < chunk["totalLengthChars"] else []),
                "minSequenceNumber": chunk.get("chunkMinSequenceNumber"),
                "sequenceNumber": chunk["chunkSequenceNumber"]}
        for spec in segs:
            self._snapshot_seg(spec, interner, abi.OP_LOAD, 0)
        min_seq = meta.get("minSequenceNumber")
        seq = int(meta["sequenceNumber"])
        self.start_collab(long_id, int(min_seq) if min_seq is not None else seq, seq)
        for md in meta["orderedChunkMetadata"][1:]:
            body = blobs[md["id"]]
            body = parse(body) if isinstance(body, str) else body
            for spec in body.get("segments", body.get("segmentTexts", [])):
                self._snapshot_seg(spec, interner, abi.OP_INSERT, abi.F_APPEND)
        names = {"header"} | {md["id"] for md in meta["orderedChunkMetadata"]}
        extra = [k for k in blobs if k not in names]
        if extra:
            cu = blobs[extra[0]]
            return parse(cu) if isinstance(cu, str) else cu
        return []

    def seq_update(self, min_seq: int, seq: int) -> None:
        """Client.updateSeqNumbers(min, seq) outside a message (client.ts:877), e.g. summarize's catch-up."""
        self.current_seq = seq
        self.ops.append((abi.OP_SEQ, abi.F_LAST, 0, seq, seq, min_seq, 0, 0, 0, 0))

    # -- sequenced messages (Client.applyMsg)
    def message(self, msg: dict, interner: Interner) -> None:
        cid = msg.get("clientId")
        cid = "null" if cid is None else str(cid)
        short = self.short_id(cid)
        seq = int(msg["sequenceNumber"])
        ref = int(msg["referenceSequenceNumber"])
        msn = int(msg["minimumSequenceNumber"])
        if msg.get("type") != "op":
            self.current_seq = seq
            self.ops.append((abi.OP_SEQ, abi.F_LAST, short, seq, ref, msn, 0, 0, 0, 0))
            return
        contents = msg["contents"]
        if isinstance(contents, str):
            contents = parse(contents)
        if contents.get("type") == "act":  # an interval collection's op (SharedSegmentSequence.processCore,
            # sequence.ts:620-646: handled by the DefaultMap, never reaches the merge-tree client)
            from .intervals import IntervalCollections, IntervalUnsupported

            if self.intervals is None:
                self.intervals = IntervalCollections()
            try:
                self.intervals.process(self, contents, msg)
            except IntervalUnsupported as e:
                raise Unsupported(str(e)) from e
            return
        self.current_seq = seq
        members = contents["ops"] if contents.get("type") == 3 else [contents]
        if not members:
            self.ops.append((abi.OP_SEQ, abi.F_LAST, short, seq, ref, msn, 0, 0, 0, 0))
            return
        if cid == self.observer_id:  # this client's own op: ackPendingSegment per member (client.ts:641-663, 866-869)
            for i, op in enumerate(members):
                last = abi.F_LAST if i == len(members) - 1 else 0
                t = op.get("type")
                pp = comb = 0
                if t == 2:
                    comb = _local_comb(op.get("combiningOp"))
                    pp = interner.propop(op.get("props") or {})
                elif t not in (0, 1):
                    raise Unsupported(f"ack of op type {t}")
                self.ops.append((abi.OP_ACK, last, short, seq, ref, msn, comb, 0, pp, t))
            return
        for i, op in enumerate(members):
            last = abi.F_LAST if i == len(members) - 1 else 0
            t = op.get("type")
            if t == 0:
                seg = op.get("seg")
                if seg is None:
                    # applyInsertOp returns early; only updateSeqNumbers runs
                    self.ops.append((abi.OP_SEQ, last, short, seq, ref, msn, 0, 0, 0, 0))
                    continue
                n0 = len(self.ops)
                pos1 = self._position(op, "pos1", 1, short, seq, ref, msn)
                rel = abi.F_REL if len(self.ops) > n0 else 0
                flags, p1, p2, pp = self._seg(seg, interner)
                self.ops.append((abi.OP_INSERT, flags | last | rel, short, seq, ref, msn, pos1, pp, p1, p2))
            elif t == 1:
                n0 = len(self.ops)
                pos1 = self._position(op, "pos1", 1, short, seq, ref, msn)
                pos2 = self._position(op, "pos2", 2, short, seq, ref, msn)
                rel = abi.F_REL if len(self.ops) > n0 else 0
                self.ops.append((abi.OP_REMOVE, last | rel, short, seq, ref, msn, pos1, pos2, 0, 0))
            elif t == 2:
                props = op.get("props")
                if isinstance(props, dict) and "markerId" in props:
                    self.marker_id_annotated = True
                n0 = len(self.ops)
                pos1 = self._position(op, "pos1", 1, short, seq, ref, msn)
                pos2 = self._position(op, "pos2", 2, short, seq, ref, msn)
                rel = abi.F_REL if len(self.ops) > n0 else 0
                pp, comb = interner.combining(props, op.get("combiningOp"), seq)
                self.ops.append((abi.OP_ANNOTATE, last | rel, short, seq, ref, msn, pos1, pos2, pp, comb))
            else:
                raise Unsupported(f"op type {t}")


@dataclass
class MatrixLog(DocLog):
    """Host state of one SharedMatrix (SharedMatrix.processCore, matrix.ts:636-693, remote branch):
    vector ops (``contents.target`` "rows" / "cols") are merge-tree ops on that PermutationVector,
    whose segment specs are ``[length, start]`` (PermutationSegment.fromJSONObject,
    permutationvector.ts:45-48; the remote ``start`` is discarded by ``reset()`` on INSERT); a set-cell
    message becomes one MTR_OP_SETCELL record.  Both vectors share this log's client table (short ids
    are only compared for equality and mapped back to long ids in summaries).

    The client's own edits (a live SharedMatrix, matrix.ts:202-418): row / col inserts and removes are local
    merge-tree ops on that vector, pending until its own message comes back (an MTR_OP_ACK); a cell write is an
    MTR_OP_LOCAL_SETCELL record (CellMatrixLog keeps the value and the pending write)."""

    local_seq: int = 0  # the vectors' collabWindow.localSeq, kept equal by submitVectorMessage / nextLocalSeq

    def start_collab(self, long_id: str, min_seq: int = 0, current_seq: int = 0) -> None:
        """startOrUpdateCollaboration on both vectors (SharedMatrix.onConnect, matrix.ts:523-532)."""
        super().start_collab(long_id, min_seq, current_seq)

    def message(self, msg: dict, interner: Interner) -> None:
        cid = msg.get("clientId")
        cid = "null" if cid is None else str(cid)
        if msg.get("type") != "op":
            return  # SharedMatrix has no MSN handler: only its vectors' own messages move their windows
        short = self.short_id(cid)
        seq = int(msg["sequenceNumber"])
        ref = int(msg["referenceSequenceNumber"])
        msn = int(msg["minimumSequenceNumber"])
        contents = msg["contents"]
        if isinstance(contents, str):
            contents = parse(contents)
        target = contents.get("target")
        own = cid == self.observer_id
        if target is None:  # MatrixOp.set (matrix/src/ops.ts:8-12)
            if contents.get("type") != 2:
                raise Unsupported("matrix message without a target")
            if own:  # the ACK of a local write (matrix.ts:652-668): host state only
                self._own_set_ack()
                return
            self.ops.append((abi.OP_SETCELL, 0, short, seq, ref, msn, int(contents["row"]), int(contents["col"]), 0, 0))
            return
        if target not in ("rows", "cols"):
            raise Unsupported(f"matrix target {target!r}")
        tf = abi.F_COLS if target == "cols" else 0
        members = contents["ops"] if contents.get("type") == 3 else [contents]
        if not members:
            self.ops.append((abi.OP_SEQ, abi.F_LAST | tf, short, seq, ref, msn, 0, 0, 0, 0))
            return
        for i, op in enumerate(members):
            last = (abi.F_LAST if i == len(members) - 1 else 0) | tf
            t = op.get("type")
            if "relativePos1" in op or "relativePos2" in op:
                raise Unsupported("relative positions")
            if own:  # the vector's applyMsg(msg, local): ackPendingSegment per member (client.ts:866-869)
                if t not in (0, 1):
                    raise Unsupported(f"ack of vector op type {t}")
                self.ops.append((abi.OP_ACK, last, short, seq, ref, msn, 0, 0, 0, t))
                continue
            if t == 0:
                seg = op.get("seg")
                if seg is None:
                    self.ops.append((abi.OP_SEQ, last, short, seq, ref, msn, 0, 0, 0, 0))
                    continue
                if not (isinstance(seg, list) and len(seg) == 2):
                    raise Unsupported("PermutationSegment spec")
                self.ops.append((abi.OP_INSERT, last, short, seq, ref, msn, int(op["pos1"]), -1, 0, int(seg[0])))
            elif t == 1:
                self.ops.append((abi.OP_REMOVE, last, short, seq, ref, msn, int(op["pos1"]), int(op["pos2"]), 0, 0))
            else:
                raise Unsupported(f"vector op type {t}")

    # -- loading a matrix from its summary (SharedMatrix.loadCore, matrix.ts:611-631)
    def _perm_seg(self, spec: Any, op_type: int, flags: int) -> None:
        """PermutationSegment.fromJSONObject of a snapshot spec [length, start] (permutationvector.ts:45-48)
        with its merge info (SnapshotLoader.specToSegment, snapshotLoader.ts:88-128): the start is kept."""
        client, seq, removers, rseq = abi.CLIENT_NONCOLLAB, 0, [], -1
        if isinstance(spec, dict) and "json" in spec:
            client = self.short_id(spec["client"]) if spec.get("client") is not None else abi.CLIENT_NONCOLLAB
            seq = int(spec["seq"]) if spec.get("seq") is not None else 0
            if spec.get("removedClient") is not None:
                removers = [self.short_id(spec["removedClient"])]
            if spec.get("removedClientIds") is not None:
                removers = [self.short_id(x) for x in spec["removedClientIds"]]
            rseq = int(spec["removedSeq"]) if spec.get("removedSeq") is not None else -1
            spec = spec["json"]
        if not (isinstance(spec, list) and len(spec) == 2 and all(isinstance(x, (int, float)) for x in spec)):
            raise Unsupported("PermutationSegment spec")
        roff = len(self.text)
        self.text.extend(removers)
        self.ops.append((op_type, flags, client, seq, rseq, len(removers), roff, -1, int(spec[1]) & 0xFFFFFFFF,
                         int(spec[0])))

    def load_summary(self, tree: dict, long_id: str, interner: Interner) -> None:
        """rows.load then cols.load (PermutationVector.load, permutationvector.ts:327-345): the handle
        table, the V1 header segments, startOrUpdateCollaboration(long_id, minSeq, seq) from that
        vector's header, its body segments.  `tree`: {"rows" | "cols": {"segments": {blob id: blob},
        "handleTable": blob}} (cells: CellMatrixLog)."""
        me = None
        for name, tf in (("rows", 0), ("cols", abi.F_COLS)):
            vec = tree[name]
            ht = vec["handleTable"]
            ht = parse(ht.decode() if isinstance(ht, bytes) else ht) if isinstance(ht, (str, bytes)) else ht
            if not isinstance(ht, list) or not ht:
                raise Unsupported("handle table")
            off = len(self.text)
            for h in ht:
                h = int(h) & 0xFFFFFFFF
                self.text.extend((h & 0xFFFF, h >> 16))
            self.ops.append((abi.OP_HANDLES, tf, 0, 0, 0, 0, len(ht), 0, off, 0))
            segs = vec["segments"]

            def blob(k):
                x = segs[k]
                return parse(x.decode() if isinstance(x, bytes) else x) if isinstance(x, (str, bytes)) else x

            header = blob("header")
            if header.get("version") != "1":  # PermutationVector forces newMergeTreeSnapshotFormat
                raise Unsupported("matrix vector summary not in the V1 format")
            for spec in header["segments"]:
                self._perm_seg(spec, abi.OP_LOAD, tf)
            meta = header["headerMetadata"]
            seq = int(meta["sequenceNumber"])
            msn = meta.get("minSequenceNumber")
            if me is None:
                me = self.add_long_id(long_id)
            self.ops.append((abi.OP_START_COLLAB, abi.F_APPEND | tf, me, seq, 0, int(msn) if msn is not None else seq,
                             0, 0, 0, 0))
            for md in meta["orderedChunkMetadata"][1:]:
                for spec in blob(md["id"])["segments"]:
                    self._perm_seg(spec, abi.OP_INSERT, abi.F_APPEND | tf)
        self.observer_id = long_id
        self.collaborating = True

    def _own_set_ack(self) -> None:
        """A SharedMatrix observer has no pending cell writes (CellMatrixLog keeps them)."""
        raise Unsupported("ack of a cell write without the cell store")

    # -- the client's own edits (SharedMatrix.insertRows / removeRows / insertCols / removeCols, matrix.ts:363-418)
    def local_vector_op(self, target: str, op: dict, track: int = 0, ref_tid: int = -1) -> None:
        """A local insert ({type 0, pos1, seg: [count, start]}) or remove ({type 1, pos1, pos2}) on the rows or
        cols PermutationVector (PermutationVector.insert / remove -> Client.insertSegmentLocal / removeRangeLocal,
        permutationvector.ts:174-195), then submitVectorMessage's localSeq sync (matrix.ts:321-345).
        Undo (fluidframework_amd/undo.py): `track` = the tracking-group bits the op's delta segments join;
        `ref_tid` >= 0 makes an insert PermutationVector.insertRelative in front of that tracked segment, taking
        its handles and groups (include/mtr_types.h "Tracking groups")."""
        tf = abi.F_COLS if target == "cols" else 0
        t = op.get("type")
        if t == 0:
            seg = op.get("seg")
            if not (isinstance(seg, list) and len(seg) == 2):
                raise Unsupported("PermutationSegment spec")
            self.ops.append((abi.OP_LOCAL_INSERT, tf, 0, self._local_seq(), 0, 0, int(op["pos1"]), int(ref_tid),
                             int(track), int(seg[0])))
        elif t == 1 and ref_tid < 0:
            self.ops.append((abi.OP_LOCAL_REMOVE, tf, 0, self._local_seq(), 0, 0, int(op["pos1"]), int(op["pos2"]),
                             int(track), 0))
        else:
            raise Unsupported(f"local vector op type {t}")
        if self.collaborating:
            self.local_seq += 1

    def track_unlink(self, target: str, tid: int, bits: int) -> None:
        """TrackingGroup.unlink of the groups `bits` from tracked segment `tid` (-1: from all of them) on the rows or
        cols vector (MTR_OP_TRACK)."""
        tf = abi.F_COLS if target == "cols" else 0
        self.ops.append((abi.OP_TRACK, tf, 0, 0, 0, 0, int(tid), 0, int(bits), 0))

    def cols_log(self) -> DocLog:
        """The cols vector's engine document: no ops of its own, the same client table."""
        return DocLog(observer_id=self.observer_id, clients=list(self.clients), client_ix=dict(self.client_ix))


def matrix_logs(logs: list[MatrixLog]) -> list[DocLog]:
    """Engine document order for matrices: [rows 0, cols 0, rows 1, cols 1, ...]
    (declare each pair with Engine.set_matrix(2 m, 2 m + 1))."""
    out: list[DocLog] = []
    for m in logs:
        out.append(m)
        out.append(m.cols_log())
    return out


class Batch:
    """Numpy-backed arrays + the ctypes MtrBatch view of them (keeps the arrays alive)."""

    def __init__(self, docs, ops, text, propop_off, propop_kv, key_off, key_bytes, key_index,
                 val_off, val_bytes, val_eq, client_off, client_bytes):
        self.docs = np.ascontiguousarray(docs, dtype=abi.DOC_DTYPE)
        self.ops = np.ascontiguousarray(ops, dtype=abi.OP_DTYPE)
        self.text = np.ascontiguousarray(text, dtype="<u2")
        self.propop_off = np.ascontiguousarray(propop_off, dtype="<u4")
        self.propop_kv = np.ascontiguousarray(propop_kv, dtype="<u4")
        self.key_off = np.ascontiguousarray(key_off, dtype="<u4")
        self.key_bytes = np.ascontiguousarray(key_bytes, dtype="u1")
        self.key_index = np.ascontiguousarray(key_index, dtype="<u4")
        self.val_off = np.ascontiguousarray(val_off, dtype="<u4")
        self.val_bytes = np.ascontiguousarray(val_bytes, dtype="u1")
        self.val_eq = np.ascontiguousarray(val_eq, dtype="<u4")
        self.client_off = np.ascontiguousarray(client_off, dtype="<u4")
        self.client_bytes = np.ascontiguousarray(client_bytes, dtype="u1")
        # keep a non-empty allocation behind every pointer
        for name in ("text", "propop_kv", "key_bytes", "key_index", "val_bytes", "val_eq", "client_bytes"):
            a = getattr(self, name)
            if a.size == 0:
                setattr(self, name, np.zeros(1, dtype=a.dtype))
        self.c = abi.MtrBatch(
            n_docs=len(self.docs),
            n_propops=len(self.propop_off) - 1,
            n_keys=len(self.key_off) - 1,
            n_vals=len(self.val_off) - 1,
            n_ops=len(self.ops),
            n_text=len(self.text),
            docs=abi.ptr(self.docs),
            ops=abi.ptr(self.ops),
            text=abi.ptr(self.text),
            propop_off=abi.ptr(self.propop_off),
            propop_kv=abi.ptr(self.propop_kv),
            key_off=abi.ptr(self.key_off),
            key_bytes=abi.ptr(self.key_bytes),
            key_index=abi.ptr(self.key_index),
            val_off=abi.ptr(self.val_off),
            val_bytes=abi.ptr(self.val_bytes),
            val_eq=abi.ptr(self.val_eq),
            client_off=abi.ptr(self.client_off),
            client_bytes=abi.ptr(self.client_bytes),
        )

    @property
    def ref(self):
        return C.byref(self.c)

    @property
    def n_docs(self) -> int:
        return len(self.docs)


def _offsets(chunks: Iterable[bytes]) -> tuple[np.ndarray, np.ndarray]:
    chunks = list(chunks)
    off = np.zeros(len(chunks) + 1, dtype="<u4")
    if chunks:
        off[1:] = np.cumsum([len(c) for c in chunks])
    data = np.frombuffer(b"".join(chunks), dtype="u1").copy() if chunks else np.zeros(0, "u1")
    return off, data


def build_batch(logs: list[DocLog], interner: Interner) -> Batch:
    """Pack the pending ops of every DocLog (in order) into one Batch and clear them."""
    docs = np.zeros(len(logs), dtype=abi.DOC_DTYPE)
    all_ops = []
    all_text = []
    client_chunks: list[bytes] = []
    op_n = 0
    text_n = 0
    for d, log in enumerate(logs):
        docs[d]["op_begin"] = op_n
        docs[d]["op_count"] = len(log.ops)
        docs[d]["text_base"] = text_n
        docs[d]["text_count"] = len(log.text)
        docs[d]["client_base"] = len(client_chunks)
        docs[d]["n_clients"] = len(log.clients)
        for c in log.clients:
            client_chunks.append(to_utf8(js_string(c)[1:-1]))
        all_ops.extend(log.ops)
        all_text.extend(log.text)
        op_n += len(log.ops)
        text_n += len(log.text)
        log.ops = []
        log.text = []
    ops = np.array(all_ops, dtype=abi.OP_DTYPE) if all_ops else np.zeros(0, abi.OP_DTYPE)
    text = np.array(all_text, dtype="<u2")
    po = np.zeros(len(interner.propops) + 1, dtype="<u4")
    kv = []
    for i, pairs in enumerate(interner.propops):
        po[i + 1] = po[i] + len(pairs)
        for k, v in pairs:
            kv.extend((k, v))
    key_off, key_bytes = _offsets(interner.key_bytes)
    val_off, val_bytes = _offsets(interner.val_bytes)
    client_off, client_bytes = _offsets(client_chunks)
    return Batch(
        docs,
        ops,
        text,
        po,
        np.array(kv, dtype="<u4"),
        key_off,
        key_bytes,
        np.array(interner.key_index, dtype="<u4"),
        val_off,
        val_bytes,
        np.array(interner.val_eq, dtype="<u4"),
        client_off,
        client_bytes,
    )
