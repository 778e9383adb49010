"""SharedMatrix cell values and the ``cells`` summary blob, host side.

The engine resolves every set-cell message to a (row handle, col handle) pair on the device -- the
position adjustment, the split and the handle allocation are the hot part (rows a17/a18) -- and, for a
matrix tracked for its cells, reports in op order (``mtr_get_deltas``):

* ``MTR_DELTA_CELL`` {op, row handle, col handle}: ``cells.setCell(rowHandle, colHandle, value)``
  happened (SharedMatrix.processCore, packages/dds/matrix/src/matrix.ts:676-692);
* ``MTR_DELTA_RECYCLE`` {op, first handle, count} on a vector's document: zamboni unlinked a segment
  and its handles went back to the free list, so their row / column of cells is cleared
  (onRowHandlesRecycled / onColHandlesRecycled, matrix.ts:722-734).

The values themselves are opaque JSON the host already holds, so the cell store lives here:
:class:`SparseArray2D` restates packages/dds/matrix/src/sparsearray2d.ts -- a 4-level, 256-way
Morton-keyed trie whose *allocated levels* show in the summary (levels are never freed, cleared
cells become ``null``) -- and :class:`CellMatrixLog` pairs it with the matrix message packer.
"""
from __future__ import annotations

from typing import Any

import numpy as np

from . import abi
from .batch import Interner, MatrixLog, Unsupported
from .engine import EngineError
from .jsjson import js_stringify, parse, to_utf8

DELTA_CELL = abi.OP_SETCELL  # include/mtr_types.h MTR_DELTA_CELL
DELTA_RECYCLE = 32           # MTR_DELTA_RECYCLE


def _spread8(x: int) -> int:  # x8ToInterlacedX16 (sparsearray2d.ts:13-20)
    j = x
    j = (j | (j << 4)) & 0x0F0F
    j = (j | (j << 2)) & 0x3333
    j = (j | (j << 1)) & 0x5555
    return j


_SPREAD = [_spread8(i) for i in range(256)]


def _spread16(x: int) -> int:  # interlaceBitsX16 of the low 16 bits
    return (_SPREAD[(x >> 8) & 0xFF] << 16) | _SPREAD[x & 0xFF]


def row_bits(row: int) -> int:  # r0ToMorton16
    return (_spread16(row) << 1) & 0xFFFFFFFF


def col_bits(col: int) -> int:  # c0ToMorton16
    return _spread16(col)


def morton(row: int, col: int) -> int:  # r0c0ToMorton2x16
    return row_bits(row) | col_bits(col)


def _bytes(x: int) -> tuple[int, int, int, int]:  # byte0 .. byte3 (most significant first)
    return (x >> 24) & 0xFF, (x >> 16) & 0xFF, (x >> 8) & 0xFF, x & 0xFF


class SparseArray2D:
    """The reference's cell trie with JavaScript array semantics: ``None`` is ``undefined`` (a hole
    or a cleared cell; JSON.stringify writes both as ``null``)."""

    def __init__(self, root: list | None = None) -> None:
        self.root: list = [None] if root is None else root

    @staticmethod
    def _level(parent: list, key: int) -> list:  # getLevel: allocate a 256-entry level on first use
        if key >= len(parent):
            parent.extend([None] * (key + 1 - len(parent)))
        lv = parent[key]
        if lv is None:
            lv = parent[key] = [None] * 256
        return lv

    def set_cell(self, row: int, col: int, value: Any) -> None:
        hi = morton(row >> 16, col >> 16)
        b0, b1, b2, b3 = _bytes(morton(row, col))
        lv = self._level(self._level(self._level(self._level(self.root, hi), b0), b1), b2)
        lv[b3] = value

    def get_cell(self, row: int, col: int) -> Any:
        hi = morton(row >> 16, col >> 16)
        lv = self.root[hi] if hi < len(self.root) else None
        for b in _bytes(morton(row, col)):
            if lv is None:
                return None
            lv = lv[b]
        return lv

    def _clear(self, hi_mask: int, hi_bits: int, lo: int, mask8: int) -> None:
        """Clear every cell whose key matches `bits` on `mask` (one row: the odd Morton bits, one
        column: the even ones), walking only allocated levels (clearRows / clearCols)."""
        b = _bytes(lo)
        keys = [[k for k in range(256) if (k & mask8) == b[i]] for i in range(4)]
        for hi, l0 in enumerate(self.root):
            if l0 is None or (hi & hi_mask) != hi_bits:
                continue
            for k0 in keys[0]:
                l1 = l0[k0]
                if l1 is None:
                    continue
                for k1 in keys[1]:
                    l2 = l1[k1]
                    if l2 is None:
                        continue
                    for k2 in keys[2]:
                        l3 = l2[k2]
                        if l3 is None:
                            continue
                        for k3 in keys[3]:
                            l3[k3] = None

    def clear_rows(self, row_start: int, count: int) -> None:
        for row in range(row_start, row_start + count):
            self._clear(0xAAAAAAAA, row_bits(row >> 16), row_bits(row), 0xAA)

    def clear_cols(self, col_start: int, count: int) -> None:
        for col in range(col_start, col_start + count):
            self._clear(0x55555555, col_bits(col >> 16), col_bits(col), 0x55)

    def snapshot(self) -> list:
        return self.root


class CellMatrixLog(MatrixLog):
    """A MatrixLog that also keeps the matrix's cells: every op it packs is flagged MTR_F_DELTA (the
    engine then reports cell writes and handle recycling for this matrix), and ``resolve`` replays
    the records of the last batch into the cell store.

    Local cell writes (SharedMatrix.setCell, matrix.ts:202-310) write the cell at once and, while attached,
    enter ``pending`` (the SparseArray2D of the latest unacked local write per cell, :97, 308): a remote write
    to such a cell is skipped (it happened before, :681-690), and the ACK of the local write clears the entry
    when it is still the latest (isLatestPendingWrite, :652-668, 738-759).  The cells blob holds both tries."""

    def __init__(self) -> None:
        super().__init__()
        self.cells = SparseArray2D()
        self.pending = SparseArray2D()  # SharedMatrix.pending: localSeq of the latest unacked write per cell
        self.values: dict[int, Any] = {}
        self.local_sets: dict[int, int] = {}  # record index of a local write -> its localSeq (attached)
        self.local_meta: list = []            # (row handle, col handle, localSeq) of unacked writes, in order
        self.events: list = []                # (records before it, event): acks of local writes in this batch
        self.ops_kind: dict[int, str] = {}    # record index of a local write before attaching (no pending entry)
        self.cell_undo: dict = {}             # record index of an undoable local write -> callback(rh, ch, old value)
        self.tracker = None                   # the undo provider's tracking groups (fluidframework_amd/undo.py)
        # reconnect (reSubmitCore): per vector the last batch's MTR_DELTA_REGEN / _REGEN_X / _REBASE records
        self.reconnect: dict = {"rows": [], "cols": []}

    def local_set_cell(self, row: int, col: int, value: Any) -> None:
        """SharedMatrix.setCell(row, col, value) of this client (local positions)."""
        k = len(self.ops)
        self.ops.append((abi.OP_LOCAL_SETCELL, abi.F_DELTA, 0, 0, 0, 0, int(row), int(col), 0, 0))
        self.values[k] = value
        if self.collaborating:  # sendSetCellOp: localSeq = nextLocalSeq()
            self.local_seq += 1
            self.local_sets[k] = self.local_seq
        else:  # detached: setCellCore writes the cell and sends nothing
            self.ops_kind[k] = "local"

    def local_vector_op(self, target: str, op: dict, track: int = 0, ref_tid: int = -1) -> None:
        lo = len(self.ops)
        super().local_vector_op(target, op, track, ref_tid)
        for k in range(lo, len(self.ops)):  # (handle recycling on the vector is reported as records)
            rec = self.ops[k]
            self.ops[k] = (rec[0], rec[1] | abi.F_DELTA) + tuple(rec[2:])

    def track_unlink(self, target: str, tid: int, bits: int) -> None:
        super().track_unlink(target, tid, bits)
        rec = self.ops[-1]
        self.ops[-1] = (rec[0], rec[1] | abi.F_DELTA) + tuple(rec[2:])

    def _own_set_ack(self) -> None:
        self.events.append((len(self.ops), "ack"))

    def message(self, msg: dict, interner: Interner) -> None:
        lo = len(self.ops)
        super().message(msg, interner)
        for k in range(lo, len(self.ops)):
            rec = self.ops[k]
            self.ops[k] = (rec[0], rec[1] | abi.F_DELTA) + tuple(rec[2:])
            if rec[0] == abi.OP_SETCELL:
                contents = msg["contents"]
                if isinstance(contents, str):
                    contents = parse(contents)
                self.values[k] = contents.get("value")  # `const { value } = contents`

    def resolve(self, rows: np.ndarray, cols: np.ndarray) -> None:
        """Apply the last batch's records (engine.deltas(rows doc), engine.deltas(cols doc)) in op
        order; within one op the rows records come first (a vector op touches one vector); the acks of local
        writes in this batch come between the records at their place in the message stream."""
        self.reconnect = {"rows": [], "cols": []}
        recs = [(int(r["op"]), 0, i, r) for i, r in enumerate(rows)] + [(int(r["op"]), 1, i, r) for i, r in enumerate(cols)]
        recs += [(pos - 0.5, 2, i, None) for i, (pos, _) in enumerate(self.events)]
        recs.sort(key=lambda x: (x[0], x[1], x[2]))
        for op, which, _, r in recs:
            if which == 2:  # isLatestPendingWrite (matrix.ts:738-759) for the oldest unacked local write
                if not self.local_meta:  # the write's cell record is missing (the document stopped at or before it)
                    raise EngineError("SharedMatrix: the ACK of a local setCell has no applied write "
                                      "(check the rows document's status)")
                a, b, lseq = self.local_meta.pop(0)
                p = self.pending.get_cell(a, b)
                if p is not None and p < lseq:
                    raise AssertionError("0x023")
                if p == lseq:
                    self.pending.set_cell(a, b, None)
                continue
            kind, a, b = int(r["kind"]), int(r["pos"]), int(r["len"])
            if abi.DELTA_REGEN <= kind <= abi.DELTA_REGEN_X or kind == abi.DELTA_REBASE:  # reconnect (resubmit)
                self.reconnect["cols" if which else "rows"].append((op, kind, a, b))
                continue
            if kind in (abi.DELTA_TLINK, abi.DELTA_TSPLIT, abi.DELTA_TMERGE):  # tracking groups (undo.py)
                if self.tracker is None:
                    raise ValueError("tracking records without an undo provider")
                self.tracker.report("cols" if which else "rows", op, kind, a, b)
                continue
            if kind == DELTA_CELL:
                if op in self.cell_undo:  # MatrixUndoProvider.cellSet: the handles and the value it replaces
                    v = self.cells.get_cell(a, b)
                    self.cell_undo.pop(op)(a, b, v)
                if op in self.local_sets:  # a local write: the cell now, the pending entry until its ACK
                    self.cells.set_cell(a, b, self.values[op])
                    self.pending.set_cell(a, b, self.local_sets[op])
                    self.local_meta.append((a, b, self.local_sets[op]))
                elif self.ops_kind.get(op) == "local":
                    self.cells.set_cell(a, b, self.values[op])
                elif self.pending.get_cell(a, b) is None:  # no pending local write to the cell (:681-690)
                    self.cells.set_cell(a, b, self.values[op])
            elif kind == DELTA_RECYCLE:
                if which == 0:
                    self.cells.clear_rows(a, b)
                    self.pending.clear_rows(a, b)
                else:
                    self.cells.clear_cols(a, b)
                    self.pending.clear_cols(a, b)
            else:
                raise ValueError(f"unexpected matrix record kind {kind}")
        self.values = {}
        self.local_sets = {}
        self.events = []
        self.ops_kind = {}
        self.cell_undo = {}
        if self.tracker is not None:
            self.tracker.batch_done()

    # -- reconnect: SharedMatrix.reSubmitCore (matrix.ts:553-604)
    def regenerate_vector(self, target: str, op: dict) -> int:
        """PermutationVector.regeneratePendingOp (-> Client.regeneratePendingOp, client.ts:917-960) of the vector's
        oldest pending op `op` (its contents): one MTR_OP_REGENERATE record per member on the rows or cols vector.
        Returns the first record's index (its MTR_DELTA_REGEN records carry it)."""
        tf = abi.F_COLS if target == "cols" else 0
        members = op["ops"] if op.get("type") == 3 else [op]
        first = len(self.ops)
        for m in members:
            t = m.get("type")
            if t not in (0, 1):
                raise Unsupported(f"regenerate of vector op type {t}")
            self.ops.append((abi.OP_REGENERATE, abi.F_DELTA | tf, 0, -1, 0, 0, 0, 0, 0, t))
        return first

    def rebase_position(self, target: str, pos: int, ref_seq: int, local_seq: int) -> int:
        """SharedMatrix.rebasePosition (matrix.ts:534-551) on the rows or cols vector: getContainingSegment(pos) at
        (ref_seq, this client, local_seq), then findReconnectionPosition(segment, local_seq) + offset
        (MTR_OP_REBASE_POS with MTR_REBASE_NOSLIDE).  Returns the record's index."""
        tf = abi.F_COLS if target == "cols" else 0
        self.ops.append((abi.OP_REBASE_POS, abi.F_DELTA | tf, 0, 0, int(ref_seq), int(local_seq), int(pos), 0, 0,
                         abi.REBASE_NOSLIDE))
        return len(self.ops) - 1

    def _reconnect_records(self, target: str, first: int) -> list:
        return [r for r in self.reconnect[target] if r[0] >= first]

    def regenerated_vector_op(self, target: str, reset_op: dict, first: int) -> dict:
        """The vector op regeneratePendingOp returns (resetPendingDeltaToOps, client.ts:708-800) from the records
        of regenerate_vector's batch: a member per regenerated segment -- an insert's spec is the
        PermutationSegment clone's [length, start] (permutationvector.ts:118-120), a remove its range -- and a GROUP
        unless exactly one (createGroupOp, client.ts:959), with the op's target (submitVectorMessage,
        matrix.ts:321-345)."""
        members = reset_op["ops"] if reset_op.get("type") == 3 else [reset_op]
        recs = self._reconnect_records(target, first)
        ops = []
        k = 0
        while k < len(recs):
            op, kind, a, b = recs[k]
            if not abi.DELTA_REGEN <= kind < abi.DELTA_REGEN + 3 or k + 1 >= len(recs) or recs[k + 1][1] != abi.DELTA_REGEN_X:
                raise ValueError("MTR_DELTA_REGEN without its MTR_DELTA_REGEN_X record")
            t = kind - abi.DELTA_REGEN
            if op - first >= len(members) or t != members[op - first].get("type"):
                raise ValueError("regenerate record does not match the op")
            start = int(np.int32(np.uint32(recs[k + 1][3] & 0xFFFFFFFF)))
            ops.append({"pos1": a, "seg": [b, start], "type": 0} if t == 0 else {"pos1": a, "pos2": a + b, "type": 1})
            k += 2
        out = ops[0] if len(ops) == 1 else {"ops": ops, "type": 3}
        return dict(out, target=target)

    def rebased(self, target: str, idx: int) -> int:
        """rebase_position's answer (-1: undefined, no segment)."""
        for op, kind, a, _ in self.reconnect[target]:
            if op == idx and kind == abi.DELTA_REBASE:
                return a
        raise ValueError(f"no rebase record for record {idx}")

    def cells_blob(self) -> bytes:
        """The ``cells`` blob of SharedMatrix.summarizeCore (matrix.ts:458-462):
        JSON.stringify([cells.snapshot(), pending.snapshot()])."""
        return to_utf8(js_stringify([self.cells.snapshot(), self.pending.snapshot()]))

    def load_summary(self, tree: dict, long_id: str, interner: Interner) -> None:
        """SharedMatrix.loadCore (matrix.ts:611-631): both vectors, then the cell tries."""
        super().load_summary(tree, long_id, interner)
        self.load_cells(tree["cells"])

    def load_cells(self, blob: str | bytes) -> None:
        """SparseArray2D.load of both tries (matrix.ts:621-631; nullToUndefined)."""
        cells, pending = parse(blob.decode() if isinstance(blob, bytes) else blob)
        self.cells = SparseArray2D(cells)
        self.pending = SparseArray2D(pending)


def matrix_summary(engine, rows_doc: int, cols_doc: int, log: CellMatrixLog) -> dict:
    """SharedMatrix.summarizeCore (matrix.ts:449-464) as a nested {name: bytes | dict} tree:
    ``rows`` / ``cols`` = PermutationVector.summarize (permutationvector.ts:310-325: the V1
    ``segments`` tree and the ``handleTable`` blob), ``cells`` = the cell tries.  Call after
    engine.summarize()."""
    def vector(doc):
        blobs = engine.summary(doc)
        segs = {("header" if i == 0 else f"body_{i - 1}"): b for i, b in enumerate(blobs[:-1])}
        return {"segments": segs, "handleTable": blobs[-1]}

    return {"rows": vector(rows_doc), "cols": vector(cols_doc), "cells": log.cells_blob()}
