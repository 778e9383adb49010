"""Interval collections restated for the CPU oracle.  TEST INFRASTRUCTURE ONLY: tests/ and the bench's
cpu_baseline leg may use it as the checker; the product path (fluidframework_amd/intervals.py) never does.

A line-by-line restatement of the reference's structures, so that the product path's shortcut (it sorts at
summary time instead of keeping trees) is checked against the real thing:

* ``RedBlackTree`` -- merge-tree/src/collections/rbTree.ts:127-595 (left-leaning red-black tree: put, remove,
  removeExisting, nodeRemove, moveRedLeft/Right, balance, rotations, keys); a child the reference
  dereferences while it is undefined raises ``ReferenceThrows`` (the reference's TypeError);
* ``SequenceInterval.compare`` / ``compareReferencePositions`` -- sequence/src/intervalCollection.ts:505-539,
  merge-tree/src/referencePositions.ts:113-121, on the C++ oracle's references (oracle_doc_ref_key: the
  segment's tree-order rank stands for its ordinal);
* ``LocalIntervalCollection`` -- intervalCollection.ts:788-1166: the start tree (``IntervalTree``,
  intervalTree.ts), the end tree (``compareSequenceIntervalEnds``), the id map, and the slide listeners
  (:1114-1159), called by the C++ oracle at each reference's beforeSlide / afterSlide
  (localReference.ts:441-451, 477-484; mergeTree.ts:866-871) while a batch applies;
* ``IntervalCollection`` remote ops (ackAdd :2141, ackChange :1859, ackDelete :2187), attachGraph (:1531),
  local adds on a detached string (:1635), serializeInternal (:2213) and the DefaultMap around them
  (sequence/src/defaultMap.ts: populate, the "act" handler, serialize).

JSON is written with a small JSON.stringify restatement of its own (JS key order, JS number form).
"""
from __future__ import annotations

import json
import math
import re

from fluidframework_amd import abi
from fluidframework_amd.batch import DocLog, Interner, build_batch

from .oracle import OracleDoc, options

RED, BLACK = 0, 1
SIMPLE, NEST, SLIDE_ON_REMOVE, TRANSIENT = 0x0, 0x1, 0x2, 0x4
RANGE_LABELS, INTERVAL_ID = "referenceRangeLabels", "intervalId"


class ReferenceThrows(Exception):
    """The reference throws here (an assert, a UsageError or a TypeError)."""


class OracleUnsupported(Exception):
    """A case the restatement cannot decide (e.g. a compare against a segment no longer in the tree)."""


# ------------------------------------------------------------------ JSON, as JavaScript writes it
_INDEX = re.compile(r"^(0|[1-9][0-9]*)$")


def js_keys(d: dict) -> list:
    """Object.keys order: array-index keys ascending, then the rest in insertion order."""
    idx = sorted((k for k in d if _INDEX.match(k) and int(k) < 2 ** 32 - 1), key=int)
    return idx + [k for k in d if not (_INDEX.match(k) and int(k) < 2 ** 32 - 1)]


def js_num(v) -> str:
    f = float(v)
    if math.isnan(f) or math.isinf(f):
        return "null"
    if f == int(f) and abs(f) < 1e21:
        return str(int(f))
    r = repr(f)
    if "e" in r:
        m, e = r.split("e")
        m = m.rstrip("0").rstrip(".") if "." in m else m
        e = int(e)
        if -7 < e < 21:  # repr uses an exponent from 1e16; JS writes digits up to 1e21
            digits, _, frac = m.partition(".")
            neg = digits.startswith("-")
            digits = digits.lstrip("-") + frac
            point = len(digits.lstrip("-")) - len(frac) + e
            s = digits + "0" * max(0, point - len(digits)) if point >= len(digits) else (
                digits[:point] + "." + digits[point:] if point > 0 else "0." + "0" * (-point) + digits)
            return ("-" if neg else "") + s
        return f"{m}e{'+' if e > 0 else '-'}{abs(e)}"
    return r


def js_str(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch in "\b\f\n\r\t":
            out.append({"\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r", "\t": "\\t"}[ch])
        elif o < 0x20 or 0xD800 <= o <= 0xDFFF:
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def stringify(v) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (int, float)):
        return js_num(v)
    if isinstance(v, str):
        return js_str(v)
    if isinstance(v, list):
        return "[" + ",".join(stringify(x) for x in v) + "]"
    return "{" + ",".join(js_str(k) + ":" + stringify(v[k]) for k in js_keys(v)) + "}"


def js_parse(text: str):
    return json.loads(text, object_pairs_hook=dict, parse_int=lambda s: int(s) if abs(int(s)) < 2 ** 53 else float(s))


# ------------------------------------------------------------------ RedBlackTree (rbTree.ts)
class _Node:
    __slots__ = ("key", "data", "color", "size", "left", "right")

    def __init__(self, key, data, color, size):
        self.key, self.data, self.color, self.size = key, data, color, size
        self.left = self.right = None


def _nn(node):
    """`node!` that JavaScript then dereferences: undefined throws a TypeError."""
    if node is None:
        raise ReferenceThrows("TypeError: a red-black tree child is undefined")
    return node


class RedBlackTree:
    def __init__(self, compare):
        self.compare = compare
        self.root = None

    @staticmethod
    def is_red(n):
        return n is not None and n.color == RED

    @staticmethod
    def size_of(n):
        return n.size if n is not None else 0

    def is_empty(self):
        return self.root is None

    def get(self, key):
        n = self.root
        while n is not None:
            c = self.compare(key, n.key)
            if c < 0:
                n = n.left
            elif c > 0:
                n = n.right
            else:
                return n
        return None

    def put(self, key, data):  # (no conflict resolver: SequenceInterval collections never install one)
        self.root = self._put(self.root, key, data)
        self.root.color = BLACK

    def _put(self, n, key, data):
        if n is None:
            return _Node(key, data, RED, 1)
        c = self.compare(key, n.key)
        if c < 0:
            n.left = self._put(n.left, key, data)
        elif c > 0:
            n.right = self._put(n.right, key, data)
        else:
            n.data = data
        if self.is_red(n.right) and not self.is_red(n.left):
            n = self._rot_left(n)
        if self.is_red(n.left) and self.is_red(n.left.left):
            n = self._rot_right(n)
        if self.is_red(n.left) and self.is_red(n.right):
            self._flip(n)
        n.size = self.size_of(n.left) + self.size_of(n.right) + 1
        return n

    def _remove_min(self, n):
        if n.left is not None:
            if not self.is_red(n.left) and not self.is_red(n.left.left):
                n = self._move_red_left(n)
            n.left = self._remove_min(_nn(n.left))
            return self._balance(n)
        return None

    def remove(self, key):
        if self.get(key) is None:
            return
        self.remove_existing(key)

    def remove_existing(self, key):
        r = _nn(self.root)
        if not self.is_red(r.left) and not self.is_red(r.right):
            r.color = RED
        self.root = self._remove(r, key)

    def _remove(self, n, key):
        if self.compare(key, n.key) < 0:
            if not self.is_red(n.left) and not self.is_red(_nn(n.left).left):
                n = self._move_red_left(n)
            n.left = self._remove(_nn(n.left), key)
        else:
            if self.is_red(n.left):
                n = self._rot_right(n)
            if self.compare(key, n.key) == 0 and n.right is None:
                return None
            if not self.is_red(n.right) and not self.is_red(_nn(n.right).left):
                n = self._move_red_right(n)
            if self.compare(key, n.key) == 0:
                m = _nn(n.right)
                while m.left is not None:
                    m = m.left
                n.key, n.data = m.key, m.data
                n.right = self._remove_min(_nn(n.right))
            else:
                n.right = self._remove(_nn(n.right), key)
        return self._balance(n)

    def _rot_right(self, n):
        l = _nn(n.left)
        n.left = l.right
        l.right = n
        l.color = n.color
        n.color = RED
        l.size = n.size
        n.size = self.size_of(n.left) + self.size_of(n.right) + 1
        return l

    def _rot_left(self, n):
        r = _nn(n.right)
        n.right = r.left
        r.left = n
        r.color = n.color
        n.color = RED
        r.size = n.size
        n.size = self.size_of(n.left) + self.size_of(n.right) + 1
        return r

    @staticmethod
    def _flip(n):
        n.color ^= 1
        _nn(n.left).color ^= 1
        _nn(n.right).color ^= 1

    def _move_red_left(self, n):
        self._flip(n)
        if self.is_red(_nn(n.right).left):
            n.right = self._rot_right(n.right)
            n = self._rot_left(n)
            self._flip(n)
        return n

    def _move_red_right(self, n):
        self._flip(n)
        if self.is_red(_nn(n.left).left):
            n = self._rot_right(n)
            self._flip(n)
        return n

    def _balance(self, n):
        if self.is_red(n.right):
            n = self._rot_left(n)
        if self.is_red(n.left) and self.is_red(n.left.left):
            n = self._rot_right(n)
        if self.is_red(n.left) and self.is_red(n.right):
            self._flip(n)
        n.size = self.size_of(n.left) + self.size_of(n.right) + 1
        return n

    def floor(self, key):
        """rbTree.ts:441-462: the largest node comparing <= key (None when none)."""
        n, best = self.root, None
        while n is not None:
            c = self.compare(key, n.key)
            if c == 0:
                return n
            if c < 0:
                n = n.left
            else:
                best, n = n, n.right
        return best

    def ceil(self, key):
        """rbTree.ts:464-488: the smallest node comparing >= key (None when none)."""
        n, best = self.root, None
        while n is not None:
            c = self.compare(key, n.key)
            if c == 0:
                return n
            if c > 0:
                n = n.right
            else:
                best, n = n, n.left
        return best

    def nodes(self):
        out, stack, n = [], [], self.root
        while stack or n is not None:
            while n is not None:
                stack.append(n)
                n = n.left
            n = stack.pop()
            out.append(n)
            n = n.right
        return out

    def keys(self):
        out, stack, n = [], [], self.root
        while stack or n is not None:
            while n is not None:
                stack.append(n)
                n = n.left
            n = stack.pop()
            out.append(n.key)
            n = n.right
        return out


# ------------------------------------------------------------------ SequenceInterval
class SequenceInterval:
    __slots__ = ("start", "end", "itype", "props", "listening", "pending", "prev", "kind")

    def __init__(self, start, end, itype, props, kind):
        self.start, self.end, self.itype, self.props, self.kind = start, end, itype, props, kind
        self.listening, self.pending, self.prev = False, 0, False

    def interval_id(self):
        v = self.props.get(INTERVAL_ID)
        if v is None:
            return None
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, (int, float)):
            return js_num(v)
        if isinstance(v, str):
            return v
        raise OracleUnsupported("an interval id that is not a string or number")


def _add_props(props: dict, new: dict) -> None:
    """PropertiesManager.addProperties, no combining op and no pending key (segmentPropertiesManager.ts:60-157)."""
    for k in js_keys(new):
        if new[k] is None:
            props.pop(k, None)
        else:
            props[k] = new[k]


def _utf16(s: str) -> bytes:
    return s.encode("utf-16-be", "surrogatepass")


class _Collection:
    """IntervalCollection + LocalIntervalCollection of one label."""

    def __init__(self, owner: "OracleString", label: str, saved=None):
        self.o, self.label, self.saved = owner, label, saved
        self.tree = RedBlackTree(self.compare)
        self.end_tree = RedBlackTree(self.compare_ends)
        self.id_map: dict = {}
        self.attached = False

    # SequenceInterval.compare (:505-525)
    def compare(self, a: SequenceInterval, b: SequenceInterval) -> int:
        r = self.o.compare_refs(a.start, b.start)
        if r != 0:
            return r
        r = self.o.compare_refs(a.end, b.end)
        if r != 0:
            return r
        x = a.interval_id()
        if x:
            y = b.interval_id()
            if y:
                return 1 if _utf16(x) > _utf16(y) else -1 if _utf16(x) < _utf16(y) else 0
        return 0

    def compare_ends(self, a, b) -> int:  # compareSequenceIntervalEnds (:1168-1169)
        return self.o.compare_refs(a.end, b.end)

    # LocalIntervalCollection (:788-1166)
    def _remove_from_index(self, iv):
        self.tree.remove_existing(iv)
        self.end_tree.remove(iv)
        i = iv.interval_id()
        if i is None:
            raise ReferenceThrows("0x311")
        self.id_map.pop(i, None)

    def _add_to_index(self, iv):
        i = iv.interval_id()
        if i is None:
            raise ReferenceThrows("0x2c0")
        self.tree.put(iv, True)
        self.end_tree.put(iv, iv)
        self.id_map[i] = iv

    def add(self, iv):
        self._add_to_index(iv)
        if not iv.listening:  # addPositionChangeListeners installs once per interval
            iv.listening, iv.pending, iv.prev = True, 0, False
            self.o.ref_cb[iv.start] = (self, iv)
            self.o.ref_cb[iv.end] = (self, iv)

    def remove_existing(self, iv):
        self._remove_from_index(iv)
        if iv.listening:  # removePositionChangeListeners (:460-466)
            iv.listening = False
            self.o.ref_cb.pop(iv.start, None)
            self.o.ref_cb.pop(iv.end, None)

    def before_slide(self, iv):
        iv.pending += 1
        if not iv.prev:
            iv.prev = True
            self._remove_from_index(iv)

    def after_slide(self, iv):
        if not iv.prev:
            raise ReferenceThrows("0x3fa")
        iv.pending -= 1
        if iv.pending == 0:
            self._add_to_index(iv)
            iv.prev = False

    def create(self, start, end, itype, view, kind) -> SequenceInterval:
        """createSequenceInterval (:726-767) through the oracle's references (createPositionReference, :697-724)."""
        if isinstance(itype, bool) or not isinstance(itype, (int, float)) or itype not in (SIMPLE, NEST, SLIDE_ON_REMOVE):
            raise OracleUnsupported(f"intervalType {itype!r}")
        for p in (start, end):
            if isinstance(p, bool) or not isinstance(p, (int, float)) or p != int(p):
                raise OracleUnsupported("an endpoint that is not an integer position")
        b, e = (abi.REFTYPE_NEST_BEGIN, abi.REFTYPE_NEST_END) if itype == NEST else (abi.REFTYPE_RANGE_BEGIN,
                                                                                   abi.REFTYPE_RANGE_END)
        f = abi.REFTYPE_STAY_ON_REMOVE if kind == "local" else abi.REFTYPE_SLIDE_ON_REMOVE
        s = self.o.log.create_ref(int(start), b | f, view=view, slide=kind == "op")
        t = self.o.log.create_ref(int(end), e | f, view=view, slide=kind == "op")
        self.o.flush()
        if kind != "op":
            for r in (s, t):
                if self.o.doc.ref_key(r)[0] == -1:  # "Non-transient references need segment" (:690-692)
                    raise ReferenceThrows("UsageError: Non-transient references need segment")
        return SequenceInterval(s, t, itype, {RANGE_LABELS: [self.label]}, kind)

    def attach(self):
        """attachGraph (:1531-1579)."""
        for si in self.saved or []:
            props = ensure_serialized_id(si)
            iv = self.create(si.get("start"), si.get("end"), si.get("intervalType"), None, "snapshot")
            if props:
                _add_props(iv.props, props)
            self.add(iv)
        self.saved = None
        self.attached = True

    def ack_add(self, si, msg):
        ensure_serialized_id(si)
        view = (int(msg["referenceSequenceNumber"]), _cid(msg))
        iv = self.create(si.get("start"), si.get("end"), si.get("intervalType"), view, "op")
        p = si.get("properties")
        if p:
            _add_props(iv.props, p)
        if INTERVAL_ID not in iv.props:
            raise OracleUnsupported("uuid()")
        self.add(iv)

    def ack_delete(self, si):
        i = ensure_serialized_id(si).get(INTERVAL_ID)
        iv = self.id_map.get(i) if isinstance(i, str) else None
        if iv is not None:
            self.remove_existing(iv)

    def ack_change(self, si, msg):
        p = si.get("properties") or {}
        if INTERVAL_ID not in p:
            raise ReferenceThrows("0x3fe")
        i = p[INTERVAL_ID]
        new_props = {k: v for k, v in p.items() if k != INTERVAL_ID}
        iv = self.id_map.get(i) if isinstance(i, str) else None
        if iv is None:
            return
        start, end = si.get("start"), si.get("end")
        if ("start" in si and start is None) or ("end" in si and end is None):
            raise OracleUnsupported("a null endpoint")
        nv = iv
        if start is not None or end is not None:
            if iv.kind == "local":
                raise ReferenceThrows("0x2f5")
            view = (int(msg["referenceSequenceNumber"]), _cid(msg))
            f = abi.REFTYPE_SLIDE_ON_REMOVE
            b, e = (abi.REFTYPE_NEST_BEGIN, abi.REFTYPE_NEST_END) if iv.itype == NEST else (abi.REFTYPE_RANGE_BEGIN,
                                                                                         abi.REFTYPE_RANGE_END)
            s, t = iv.start, iv.end
            if start is not None:
                s = self.o.log.create_ref(int(start), b | f, view=view, slide=True)
            if end is not None:
                t = self.o.log.create_ref(int(end), e | f, view=view, slide=True)
            self.o.flush()
            nv = SequenceInterval(s, t, iv.itype, dict(iv.props), "op")  # modify + copyTo (:600-656)
            self.remove_existing(iv)  # changeInterval (:1088-1103)
            self.add(nv)
        _add_props(nv.props, new_props)

    def local_add(self, start, end, itype, props):
        iv = self.create(start, end, itype, None, "local")
        if props:
            _add_props(iv.props, props)
        if INTERVAL_ID not in iv.props:
            raise OracleUnsupported("uuid()")
        self.add(iv)

    # ---- queries (LocalIntervalCollection, :946-992) of a transient interval (createSequenceInterval with
    # IntervalType.Transient: Transient references at the local view)
    def transient(self, start, end) -> SequenceInterval:
        s = self.o.log.create_ref(int(start), abi.REFTYPE_TRANSIENT)
        t = self.o.log.create_ref(int(end), abi.REFTYPE_TRANSIENT)
        self.o.flush()
        return SequenceInterval(s, t, TRANSIENT, {}, "transient")

    def previous_interval(self, pos):
        """previousInterval (:966-978): endIntervalTree.floor(transient) -> its data"""
        n = self.end_tree.floor(self.transient(pos, pos))
        return None if n is None else n.data

    def next_interval(self, pos):
        """nextInterval (:980-992): endIntervalTree.ceil(transient) -> its data"""
        n = self.end_tree.ceil(self.transient(pos, pos))
        return None if n is None else n.data

    def find_overlapping(self, start, end):
        """findOverlappingIntervals (:950-964): the tree's gather of SequenceInterval.overlaps (:544-549); the
        augmentation (union of the subtree, intervalTree.ts:163-177) only prunes subtrees without a match, so the
        in-order filter gives the same list."""
        if end < start or self.tree.is_empty():
            return []
        t = self.transient(start, end)
        return [iv for iv in self.tree.keys()
                if self.o.compare_refs(iv.start, t.end) <= 0 and self.o.compare_refs(iv.end, t.start) >= 0]

    def serialize(self):
        """LocalIntervalCollection.serialize (:1105-1112) with compressInterval (:139-151)."""
        pos = self.o.doc.ref_positions()
        seq = int(self.o.doc.state()[1])
        out = []
        for iv in self.tree.keys():
            props = {k: v for k, v in iv.props.items() if k != RANGE_LABELS}
            out.append([pos[iv.start], pos[iv.end], seq, iv.itype, props])
        return {"label": self.label, "intervals": out, "version": 2}


def ensure_serialized_id(si: dict) -> dict:
    """ensureSerializedId (:838-858)."""
    p = si.get("properties")
    if not isinstance(p, dict) or p.get(INTERVAL_ID) is None:
        p = dict(p) if isinstance(p, dict) else {}
        s, e = si.get("start"), si.get("end")
        p[INTERVAL_ID] = f"legacy{js_num(s) if isinstance(s, (int, float)) else s}-" \
                         f"{js_num(e) if isinstance(e, (int, float)) else e}"
        si["properties"] = p
    return p


def _cid(msg):
    c = msg.get("clientId")
    return "null" if c is None else str(c)


class OracleString:
    """One SharedString observer on the C++ oracle with its interval collections: merge-tree records go through a
    DocLog into the oracle document; interval ops run here, between batches, and the references' slide callbacks
    run here while a batch applies."""

    def __init__(self, opts=None):
        self.doc = OracleDoc(opts or options())
        self.log = DocLog()
        self.it = Interner()
        self.data: dict = {}  # DefaultMap.data
        self.ref_cb: dict = {}  # reference id -> (collection, interval) whose listeners it carries
        self.err = None
        self.doc.set_slide_hook(self._hook)

    def close(self):
        self.doc.set_slide_hook(None)

    def _hook(self, ref, phase):
        if self.err is not None:
            return
        try:
            cb = self.ref_cb.get(ref)
            if cb is not None:
                (cb[0].before_slide if phase == 0 else cb[0].after_slide)(cb[1])
        except Exception as e:  # (an exception must not cross the C frames; re-raised after apply)
            self.err = e

    def flush(self):
        if not self.log.ops:
            return
        b = build_batch([self.log], self.it)
        rc = self.doc.apply(b, 0)
        if self.err is not None:
            e, self.err = self.err, None
            raise e
        if rc != 0:
            raise ReferenceThrows(f"oracle status {rc}")

    # compareReferencePositions (referencePositions.ts:113-121)
    def compare_refs(self, a: int, b: int) -> int:
        sa, oa = self.doc.ref_key(a)
        sb, ob = self.doc.ref_key(b)
        if sa == -2 or sb == -2:
            raise OracleUnsupported("a compare against a segment that left the tree (its stale ordinal)")
        if sa == sb:
            return oa - ob
        return -1 if sa == -1 or (sb != -1 and sa < sb) else 1

    # -- the SharedString surface
    def load(self, blobs: dict, long_id: str):
        """loadCore (sequence.ts:557-611): populate from `header`, Client.load of `content/`, then
        loadFinished -> attachGraph of each collection.  blobs: {"header": interval blob or absent,
        "content": {merge-tree blob name: text}}."""
        if "header" in blobs:
            j = js_parse(blobs["header"])
            for key in js_keys(j):
                ser = j[key]
                if ser.get("type") in ("Plain", "Shared"):
                    continue
                v = ser["value"]
                label = key[20:] if key.startswith("intervalCollections/") else key
                saved = [dict(x) for x in v] if isinstance(v, list) else [
                    {"start": c[0], "end": c[1], "sequenceNumber": c[2], "intervalType": c[3],
                     "properties": {**c[4], RANGE_LABELS: [v["label"]]}} for c in v["intervals"]]
                self.data[label] = _Collection(self, label, saved)
        catchup = self.log.load_summary(blobs["content"], long_id, self.it)
        for m in catchup or []:
            self.log.message(m, self.it)
        self.flush()
        for c in self.data.values():
            c.attach()

    def get(self, label) -> _Collection:
        c = self.data.get(label)
        if c is None:
            c = self.data[label] = _Collection(self, label)
            c.attached = True
        return c

    def message(self, msg: dict):
        contents = msg.get("contents")
        if isinstance(contents, str):
            contents = js_parse(contents)
        if msg.get("type") == "op" and isinstance(contents, dict) and contents.get("type") == "act":
            self.flush()
            if _cid(msg) == self.log.observer_id:
                raise OracleUnsupported("local interval ops")
            c = self.get(contents["key"])
            v = contents.get("value") or {}
            name, params = v.get("opName"), v.get("value")
            if name not in ("add", "delete", "change"):
                raise ReferenceThrows("Unknown type message")
            if name != "delete" and (params is None or params is False or params == 0 or params == ""):
                return
            params = dict(params)
            if name == "add":
                c.ack_add(params, msg)
            elif name == "delete":
                c.ack_delete(params)
            else:
                c.ack_change(params, msg)
            return
        self.log.message(msg, self.it)

    def summarize_header(self):
        """The `header` blob (summarizeCore, sequence.ts:467-480) or None."""
        self.flush()
        if not self.data:
            return None
        return stringify({k: {"type": "sharedStringIntervalCollection", "value": c.serialize()}
                          for k, c in self.data.items()})

    def summarize_content(self, long_id_unused=None):
        self.flush()
        b = build_batch([self.log], self.it)
        return self.doc.summarize(b, 0)

    def text(self):
        self.flush()
        return self.doc.text()
