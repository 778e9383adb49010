"""SharedMatrix undo: MatrixUndoProvider and VectorUndoProvider (matrix/src/undoprovider.ts:17-177)
with the SharedMatrix paths that feed them -- openUndo (matrix.ts:128-135), setCellCore's cellSet (:254-268),
_undoRemoveRows / _undoRemoveCols (:371-430) -- for a live matrix whose vectors run on the replay engine.

The reference links the segments a local row / col op touched into a TrackingGroup (mergeTreeTracking.ts), which
keeps them from being unlinked or merged away by zamboni, so that reverting can find them again: undoing an insert
removes each tracked segment at its current position, undoing a remove inserts a replacement in front of each
tracked (removed) segment and gives it the segment's handles -- its cells come back -- and re-sends their values.

Here the engine keeps the tracking state per segment (include/mtr_types.h "Tracking groups": a tracking id and the
bits of the groups holding it) and reports every link, split and merge of tracked segments; this host rebuilds each
group's segment list from those reports in the reference's order (link order, split-off halves appended), maps
groups to the engine's 32 bits per vector, and reads positions and handles from the vector's segment list
(mtr_get_leaves) when a revert needs them.  More than 32 groups live on one vector is an Unsupported document.

A matrix is driven through its CellMatrixLog; ``flush`` applies the queued records on the executor and resolves
the log (which hands the tracking reports back here); ``leaves(target)`` returns the executor's segment list of the
"rows" or "cols" vector; ``send(contents)`` receives every op message this client submits while attached.
"""
from __future__ import annotations

from typing import Any, Callable

from . import abi
from .batch import Unsupported

U = abi.HANDLE_UNALLOCATED
INSERT, REMOVE = 0, 1  # MergeTreeDeltaType


class _Revertible:
    """The IRevertible VectorUndoProvider.pushRevertible hands the consumer (undoprovider.ts:87-126)."""

    def __init__(self, vec: "_Vector", gid: int, kind: int) -> None:
        self.vec, self.gid, self.kind = vec, gid, kind

    def revert(self) -> None:
        self.vec.revert(self.gid, self.kind)

    def discard(self) -> None:
        self.vec.discard(self.gid)


class _CellRevertible:
    """MatrixUndoProvider.cellSet's IRevertible (undoprovider.ts:158-176); the handles and the value it replaces
    are filled in when the write's batch resolves."""

    def __init__(self, m: "UndoMatrix") -> None:
        self.m = m
        self.rh = self.ch = None
        self.old: Any = None

    def fill(self, rh: int, ch: int, old: Any) -> None:
        if rh < 1 or ch < 1:
            raise AssertionError("0x02c")  # "On cellSet(), invalid row and/or column handles!"
        self.rh, self.ch, self.old = rh, ch, old

    def revert(self) -> None:
        m = self.m
        m.flush()
        if self.rh is None:
            raise AssertionError("cellSet revertible without its cell")
        r, c = m.handle_to_position("rows", self.rh), m.handle_to_position("cols", self.ch)
        nr, nc = m.dims()
        if not (0 <= r < nr and 0 <= c < nc):  # SharedMatrix.setCell's bounds assert (matrix.ts:202-216)
            raise AssertionError("0x01a")      # "Trying to set out-of-bounds cell!"
        m.set_cell(r, c, self.old)

    def discard(self) -> None:
        pass


class _Vector:
    """VectorUndoProvider (undoprovider.ts:17-127) of the rows or the cols PermutationVector."""

    def __init__(self, m: "UndoMatrix", target: str) -> None:
        self.m, self.target = m, target
        self.groups: dict[int, list[int]] = {}  # TrackingGroup -> its segments' tracking ids, in order
        self.of: dict[int, list[int]] = {}      # tracking id -> the groups holding it (trackingCollection)
        self.bit: dict[int, int] = {}
        self.free = list(range(abi.TRACK_GROUPS))
        self.next_gid = 0
        self.op_group: dict[int, int] = {}      # record index (this batch) -> the group its delta segments join
        self.op_transfer: dict[int, int] = {}   # record index -> the segment insertRelative replaces
        self.current_group: int | None = None
        self.current_op: int | None = None
        self.live: set[int] = set()             # groups a revertible holds

    # -- groups and their engine bits
    def new_group(self) -> int:  # new TrackingGroup()
        if not self.free:
            raise Unsupported(f"more than {abi.TRACK_GROUPS} undo tracking groups live on the {self.target} vector")
        gid = self.next_gid
        self.next_gid += 1
        self.bit[gid] = self.free.pop(0)
        self.groups[gid] = []
        return gid

    def release(self, gid: int) -> None:
        self.live.discard(gid)
        if gid in self.groups:
            del self.groups[gid]
            self.free.append(self.bit.pop(gid))
            self.free.sort()

    def link(self, gid: int, tid: int) -> None:  # TrackingGroup.link (mergeTreeTracking.ts:41-46)
        g = self.groups.get(gid)
        if g is None or tid in g:  # (a group discarded before its op's reports came back)
            return
        g.append(tid)
        self.of.setdefault(tid, []).append(gid)

    def unlink(self, gid: int, tid: int) -> None:  # TrackingGroup.unlink (:47-53)
        g = self.groups.get(gid)
        if g is not None and tid in g:
            g.remove(tid)
            self.of[tid].remove(gid)

    def report(self, op: int, kind: int, a: int, b: int) -> None:
        """An engine report of this vector (in op order): a link of the op's delta segment, a split of a
        tracked segment (copyTo: every group appends the new half), a merge (the appended one leaves)."""
        if kind == abi.DELTA_TLINK:
            gid = self.op_group.get(op)
            if gid is not None:
                self.link(gid, a)
            src = self.op_transfer.get(op)
            if src is not None:  # PermutationSegment.transferToReplacement (permutationvector.ts:80-102)
                gs = list(self.of.get(src, []))
                for g in gs:
                    self.link(g, a)
                for g in gs:
                    self.unlink(g, src)
        elif kind == abi.DELTA_TSPLIT:
            for g in list(self.of.get(a, [])):
                self.link(g, b)
        elif kind == abi.DELTA_TMERGE:
            for g in list(self.of.get(a, [])):
                self.unlink(g, a)

    # -- VectorUndoProvider
    def record(self, kind: int) -> int:
        """record(operation, ranges) for an op with delta segments (undoprovider.ts:30-85): the group its segments
        join (the reverting group, else a new one); pushes the revertible once per revert."""
        gid = self.current_group if self.current_group is not None else self.new_group()
        if self.current_op is not None and self.current_op != kind:
            raise AssertionError("0x02a")  # "On vector undo, unexpected 'currentOp' type/state!"
        if self.current_op != kind:
            self.live.add(gid)
            self.m.consumer.push_to_current_operation(_Revertible(self, gid, kind))
        if self.current_group is not None:
            self.current_op = kind
        return gid

    def revert(self, gid: int, kind: int) -> None:
        if self.current_group is not None or self.current_op is not None:
            raise AssertionError("0x02b")  # "Must not nest calls to IRevertible.revert()"
        self.current_group = self.new_group()
        try:
            while True:
                self.m.flush()  # (every report in: the group's list is current -- splits append to it)
                if not self.groups.get(gid):
                    break
                tid = self.groups[gid][0]
                # unlink from the reverted group before the callback (undoprovider.ts:104-109)
                self.unlink(gid, tid)
                self.m.log.track_unlink(self.target, tid, 1 << self.bit[gid])
                if kind == INSERT:  # undoInsert: removeRows / removeCols at the segment (undoprovider.ts:138-141)
                    pos, length, _ = self.m.locate(self.target, tid)
                    self.m.remove(self.target, pos, length)
                else:               # undoRemove: SharedMatrix._undoRemoveRows / _undoRemoveCols
                    self.m.undo_remove(self.target, tid)
        finally:
            cg = self.current_group
            self.current_op = None
            self.current_group = None
            if cg is not None and cg not in self.live:
                self.release(cg)  # (nothing recorded into it)
        self.release(gid)  # every segment left it: its bit is free again

    def discard(self, gid: int) -> None:  # the revertible's discard (undoprovider.ts:116-120)
        if gid not in self.groups:
            return
        for tid in list(self.groups[gid]):
            self.unlink(gid, tid)
        self.m.log.track_unlink(self.target, -1, 1 << self.bit[gid])
        self.release(gid)


class UndoMatrix:
    """This client's SharedMatrix with an undo consumer attached (SharedMatrix.openUndo, matrix.ts:128-135):
    the local edits (insertRows / removeRows / insertCols / removeCols / setCell / setCells, matrix.ts:202-418)
    with their undo records, the provider's revert paths, and the reads a revert needs."""

    def __init__(self, log, consumer, flush: Callable[[], None], leaves: Callable[[str], Any],
                 send: Callable[[dict], None] | None = None) -> None:
        self.log = log
        log.tracker = self
        self.consumer = consumer  # IUndoConsumer: push_to_current_operation(revertible)
        self.flush = flush
        self.leaves = leaves
        self.send = send
        self.vec = {"rows": _Vector(self, "rows"), "cols": _Vector(self, "cols")}

    # -- tracker interface (CellMatrixLog.resolve)
    def report(self, target: str, op: int, kind: int, a: int, b: int) -> None:
        self.vec[target].report(op, kind, a, b)

    def batch_done(self) -> None:
        for v in self.vec.values():
            v.op_group.clear()
            v.op_transfer.clear()

    # -- reads (after a flush)
    def locate(self, target: str, tid: int) -> tuple[int, int, int]:
        """(getPosition, cachedLength, start handle) of tracked segment tid at the local view."""
        self.flush()
        pos = 0
        for ln, removed, start, t, _ in self.leaves(target):
            if t == tid:
                return pos, int(ln), int(start)
            if not removed:
                pos += int(ln)
        raise AssertionError(f"tracked segment {tid} is not in the {target} vector")

    def handle_to_position(self, target: str, h: int) -> int:
        """PermutationVector.handleToPosition (permutationvector.ts:249-300) at the current localSeq: the segment
        whose handles hold h (removed ones too), its reconnection position plus the offset."""
        pos = 0
        for ln, removed, start, _, _ in self.leaves(target):
            if start != U and start <= h < start + ln:
                return pos + (h - int(start))
            if not removed:
                pos += int(ln)
        raise AssertionError("0x029")  # "Invalid handle at start of containing segment!"

    def handles(self, target: str) -> list[int]:
        """The local view's handle per position (the handle cache, permutationvector.ts:200-230)."""
        out: list[int] = []
        for ln, removed, start, _, _ in self.leaves(target):
            if not removed:
                out.extend([U] * int(ln) if start == U else range(int(start), int(start) + int(ln)))
        return out

    def dims(self) -> tuple[int, int]:
        self.flush()
        return len(self.handles("rows")), len(self.handles("cols"))

    def grid(self) -> list[list[Any]]:
        """Every cell at the local view (SharedMatrix.getCell, matrix.ts:180-200): undefined = None."""
        self.flush()
        rows, cols = self.handles("rows"), self.handles("cols")
        return [[self.log.cells.get_cell(r, c) if r != U and c != U else None for c in cols] for r in rows]

    # -- local edits
    def _vector_op(self, target: str, contents: dict, kind: int, nonempty: bool, ref_tid: int = -1) -> None:
        v = self.vec[target]
        # VectorUndoProvider.record from the op's delta callback (permutationvector.ts:361-364); a revertible it
        # pushes may discard the redo stack first (its unlink records go ahead of the op's)
        gid = v.record(kind) if nonempty else None
        k = len(self.log.ops)
        if gid is not None:
            v.op_group[k] = gid
        if ref_tid >= 0:
            v.op_transfer[k] = ref_tid
        self.log.local_vector_op(target, contents, track=(1 << v.bit[gid]) if gid is not None else 0,
                                 ref_tid=ref_tid)
        if self.log.collaborating and self.send is not None:  # submitVectorMessage (matrix.ts:321-345)
            self.send(dict(contents, target=target))

    def insert(self, target: str, start: int, count: int) -> None:  # insertRows / insertCols
        self._vector_op(target, {"pos1": int(start), "seg": [int(count), U], "type": 0}, INSERT, count > 0)

    def remove(self, target: str, start: int, count: int) -> None:  # removeRows / removeCols
        self._vector_op(target, {"pos1": int(start), "pos2": int(start + count), "type": 1}, REMOVE, count > 0)

    def insert_rows(self, start: int, count: int) -> None:
        self.insert("rows", start, count)

    def insert_cols(self, start: int, count: int) -> None:
        self.insert("cols", start, count)

    def remove_rows(self, start: int, count: int) -> None:
        self.remove("rows", start, count)

    def remove_cols(self, start: int, count: int) -> None:
        self.remove("cols", start, count)

    def set_cell(self, row: int, col: int, value: Any, undo: bool = True) -> None:
        """setCell -> setCellCore (matrix.ts:202-268): the undo record of the value it replaces, the write, and
        while attached sendSetCellOp; undo=False is sendSetCellOp alone (a re-sent value, matrix.ts:388-400)."""
        if undo:
            r = _CellRevertible(self)
            self.consumer.push_to_current_operation(r)
            self.log.cell_undo[len(self.log.ops)] = r.fill
        self.log.local_set_cell(row, col, value)
        if self.log.collaborating and self.send is not None:
            msg = {"type": 2, "row": int(row), "col": int(col)}
            if value is not None:
                msg["value"] = value
            self.send(msg)

    def set_cells(self, row: int, col: int, col_count: int, values: list) -> None:  # setCells (matrix.ts:218-252)
        r, c = row, col
        for v in values:
            self.set_cell(r, c, v)
            c += 1
            if c == col + col_count:
                c = col
                r += 1

    def undo_remove(self, target: str, tid: int) -> None:
        """SharedMatrix._undoRemoveRows / _undoRemoveCols (matrix.ts:371-430): insertRelative in front of the
        removed segment, its handles and groups to the replacement, then a setCell op for every populated cell
        of the re-inserted rows / cols."""
        pos, length, start = self.locate(target, tid)
        self._vector_op(target, {"pos1": pos, "seg": [length, U], "type": 0}, INSERT, length > 0, ref_tid=tid)
        if not self.log.collaborating or start == U:
            return
        other = self.handles("cols" if target == "rows" else "rows")
        for i in range(length):
            h = start + i
            for j, oh in enumerate(other):
                if oh == U:
                    continue
                rh, ch = (h, oh) if target == "rows" else (oh, h)
                value = self.log.cells.get_cell(rh, ch)
                if value is not None:
                    r, c = (pos + i, j) if target == "rows" else (j, pos + i)
                    self.set_cell(r, c, value, undo=False)
