"""SharedMatrix known answers transcribed from the reference's own tests (VERDICT r05 Next #4):
matrix/src/test/matrix.spec.ts "Connected with two clients" / "conflict" (:309-610) and "local client" / "summarize" /
"mutate after load" (:273-307).  Every expected grid is the spec's (`extract`: one row per row, one value per column,
undefined = None).

Two SharedMatrix clients are driven by a restatement of the reference's MockContainerRuntimeFactory
(runtime/test-runtime-utils/src/mocks.ts:216-303): a submitted message carries referenceSequenceNumber = the client's
last processed sequence number; processAllMessages sequences them in submission order with minimumSequenceNumber =
the minimum over every sender's latest referenceSequenceNumber, and hands each to both clients (its author's copy is
the ACK).  The matrices' PermutationVectors and handle records run on the CPU oracle, or under -m gpu on the HIP
engine's matrix kernels, where every batch's records and both vectors' segment lists must also equal the oracle's.
"""
import itertools
import json

import numpy as np
import pytest

from fluidframework_amd.batch import Interner, build_batch
from fluidframework_amd.cells import CellMatrixLog
from oracle.oracle import OracleDoc, options

U = -2 ** 31  # Handle.unallocated (handletable.ts:11)
KINDS = [pytest.param(False, id="oracle"), pytest.param(True, id="engine", marks=pytest.mark.gpu)]


class MClient:
    """One SharedMatrix (matrix.ts) over a CellMatrixLog: its local edits pack as local vector / setCell records and,
    while attached, submit their op (submitVectorMessage / sendSetCellOp, matrix.ts:277-345)."""

    def __init__(self, s, name, k, attached=True):
        self.s, self.name, self.k = s, name, k
        self.client_id = name
        self.log = CellMatrixLog()
        if attached:
            self.log.start_collab(name)
        self.doc = OracleDoc(options(), matrix=True)
        self.seq = 0
        self.pending = []         # MockContainerRuntime's pending messages: (contents, metadata)
        self.pending_remote = []  # messages sequenced while disconnected
        self._connected = True

    def _vector(self, target, contents):
        self.log.local_vector_op(target, contents)
        if self.log.collaborating:
            self.s.submit(self, dict(contents, target=target))

    # ---- MockContainerRuntimeForReconnection (runtime/test-runtime-utils/src/mocksForReconnection.ts:18-140)
    def process(self, msg):
        if not self._connected:
            self.pending_remote.append(msg)
            return
        self.log.message(json.loads(json.dumps(msg)), self.s.it)
        self.seq = msg["sequenceNumber"]
        if msg["clientId"] == self.client_id:
            self.pending.pop(0)

    @property
    def connected(self):
        return self._connected

    @connected.setter
    def connected(self, value):
        if value == self._connected:
            return
        self._connected = value
        if not value:  # this client's unsequenced messages never reach the service
            self.s.queue = [q for q in self.s.queue if q[0] is not self]
            return
        self.s.flush()  # (the local edits so far applied: their writes' handles are known)
        for m in self.pending_remote:
            self.process(m)
        self.pending_remote = []
        self.client_id = f"reconnected-{next(self.s.ids)}"
        msgs, self.pending = self.pending, []
        for contents, meta in msgs:  # reSubmitMessages -> SharedMatrix.reSubmitCore (matrix.ts:553-604)
            self.resubmit(contents, meta)
        self.log.start_collab(self.client_id)  # setConnectionState -> both vectors' startOrUpdateCollaboration

    def resubmit(self, contents, meta):
        target = contents.get("target")
        if target is not None:  # rows / cols: regeneratePendingOp, then submitRowMessage / submitColMessage
            first = self.log.regenerate_vector(target, contents)
            self.s.flush()
            self.s.submit(self, self.log.regenerated_vector_op(target, contents, first))
            return
        lseq = meta["localSeq"]
        rh, ch = next((a, b) for a, b, q in self.log.local_meta if q == lseq)
        p = self.log.pending.get_cell(rh, ch)
        assert not (p is not None and p < lseq), "0x023"
        if p == lseq:  # isLatestPendingWrite (matrix.ts:745-762)
            ri = self.log.rebase_position("rows", contents["row"], meta["rowsRefSeq"], lseq)
            ci = self.log.rebase_position("cols", contents["col"], meta["colsRefSeq"], lseq)
            self.s.flush()
            row, col = self.log.rebased("rows", ri), self.log.rebased("cols", ci)
            if row >= 0 and col >= 0:  # sendSetCellOp with the original localSeq and refSeqs
                self.s.submit(self, dict(contents, row=row, col=col), meta)
                return
        # not re-sent: no ACK will come for this write
        self.log.local_meta = [e for e in self.log.local_meta if e[2] != lseq]

    def insert_rows(self, start, count):
        self._vector("rows", {"pos1": start, "seg": [count, U], "type": 0})

    def insert_cols(self, start, count):
        self._vector("cols", {"pos1": start, "seg": [count, U], "type": 0})

    def remove_rows(self, start, count):
        self._vector("rows", {"pos1": start, "pos2": start + count, "type": 1})

    def remove_cols(self, start, count):
        self._vector("cols", {"pos1": start, "pos2": start + count, "type": 1})

    def set_cell(self, row, col, value):
        self.log.local_set_cell(row, col, value)
        if self.log.collaborating:
            msg = {"type": 2, "row": row, "col": col}
            if value is not None:  # (an undefined value is no JSON field)
                msg["value"] = value
            # ISetOpMetadata (matrix.ts:299-305): the handles come with the write's record (CellMatrixLog.local_meta)
            self.s.submit(self, msg, {"localSeq": self.log.local_seq, "rowsRefSeq": self.seq, "colsRefSeq": self.seq})

    def set_cells(self, row, col, col_count, values):  # setCells (matrix.ts:216-252)
        r, c = row, col
        for v in values:
            self.set_cell(r, c, v)
            c += 1
            if c == col + col_count:
                c, r = col, r + 1

    def _handles(self, w):
        out = []
        for ln, removed, start, _, _ in self.s.leaves(self, w):
            if not removed:
                out.extend([U] * int(ln) if start == U else range(int(start), int(start) + int(ln)))
        return out

    def extract(self):
        """utils.ts `extract`: the cells at the local view (getCell, matrix.ts:180-200)."""
        self.s.flush()
        rows, cols = self._handles(0), self._handles(1)
        return [[self.log.cells.get_cell(r, c) if r != U and c != U else None for c in cols] for r in rows]


class MSession:
    def __init__(self, names, engine=False, attached=True):
        self.it = Interner()
        self.queue = []
        self.seq = 0
        self.min_seq = {}
        self.ids = itertools.count(1)
        self.clients = [MClient(self, n, k, attached) for k, n in enumerate(names)]
        self.eng = None
        if engine:
            from fluidframework_amd.engine import Engine

            self.eng = Engine(2 * len(names), max_segments=4096, heap_entries=4096, text_units=1 << 14,
                              prop_words=1024, remover_cells=4096, ops_per_launch=64)
            for k in range(len(names)):
                self.eng.set_matrix(2 * k, 2 * k + 1)
        self.checks = 0

    def leaves(self, c, w):
        return self.eng.leaves(2 * c.k + w) if self.eng is not None else c.doc.select(w).leaves()

    def submit(self, c, contents, meta=None):  # MockContainerRuntime.submit -> factory.pushMessage (mocks.ts:216-240)
        c.pending.append((contents, meta))
        if not c.connected:
            return
        ref = c.seq
        self.min_seq.setdefault(c.client_id, ref)
        self.queue.append((c, contents, ref, c.client_id))

    def flush(self):
        if not any(c.log.ops for c in self.clients):
            return
        cols = [c.log.cols_log() for c in self.clients]
        b = build_batch([x for c, cl in zip(self.clients, cols) for x in (c.log, cl)], self.it)
        self.last_batch = b
        if self.eng is not None:
            self.eng.apply(b)
        for c in self.clients:
            k = c.k
            assert c.doc.apply(b, 2 * k) == 0, c.name
            orows, ocols = c.doc.select(0).deltas(), c.doc.select(1).deltas()
            if self.eng is not None:
                for w in (0, 1):
                    st, op = self.eng.status(2 * k + w)
                    assert st == 0, f"{c.name}: engine status {st:#x} at op {op}"
                    assert np.array_equal(self.eng.leaves(2 * k + w), c.doc.select(w).leaves()), (c.name, w)
                assert np.array_equal(self.eng.deltas(2 * k), orows) and np.array_equal(self.eng.deltas(2 * k + 1), ocols)
                self.checks += 1
            c.log.resolve(orows, ocols)

    def process_all(self):  # processAllMessages (mocks.ts:262-303)
        self.flush()
        while self.queue:
            c, contents, ref, cid = self.queue.pop(0)
            self.min_seq[cid] = ref
            self.seq += 1
            msg = {"type": "op", "sequenceNumber": self.seq, "referenceSequenceNumber": ref,
                   "minimumSequenceNumber": min(self.min_seq.values()), "clientId": cid, "contents": contents}
            for x in self.clients:
                x.process(msg)
        self.flush()


class Two:
    """beforeEach of "Connected with two clients" (:337-347) and its `expect` (:316-335)."""

    def __init__(self, engine):
        self.s = MSession(["matrix1", "matrix2"], engine)
        self.m1, self.m2 = self.s.clients

    def expect(self, want=None):
        self.s.process_all()
        a1, a2 = self.m1.extract(), self.m2.extract()
        assert a1 == a2
        if want is not None:
            assert a1 == want


# ---------------------------------------------------------------- "Connected with two clients" / "conflict"
def set_cell(t):  # :357-366
    t.m1.insert_cols(0, 1)
    t.m1.insert_rows(0, 1)
    t.expect([[None]])
    t.m1.set_cell(0, 0, "1st")
    t.m2.set_cell(0, 0, "2nd")
    t.expect([["2nd"]])


def clear_unallocated_cell(t):  # :370-379
    t.m1.insert_cols(0, 1)
    t.m1.insert_rows(0, 1)
    t.expect([[None]])
    t.m1.set_cell(0, 0, "x")
    t.m2.set_cell(0, 0, None)
    t.expect([[None]])


def insert_and_set_in_new_row(t):  # :381-387
    t.m1.insert_cols(0, 2)
    t.expect()
    t.m1.insert_rows(0, 1)
    t.m1.set_cells(0, 1, 1, ["x"])
    t.expect([[None, "x"]])


def insert_and_set_in_new_col(t):  # :389-395
    t.m1.insert_rows(0, 2)
    t.expect([[], []])
    t.m1.insert_cols(0, 1)
    t.m1.set_cells(1, 0, 1, ["x"])
    t.expect([[None], ["x"]])


def insert_col_conflict(t):  # :397-408
    t.m1.insert_rows(0, 1)
    t.expect([[]])
    t.m1.insert_cols(0, 1)
    t.m1.set_cell(0, 0, "1st")
    t.m2.insert_cols(0, 1)
    t.m2.set_cell(0, 0, "2nd")
    t.expect([["2nd", "1st"]])


def insert_row_conflict(t):  # :410-421
    t.m1.insert_cols(0, 1)
    t.expect([])
    t.m1.insert_rows(0, 1)
    t.m1.set_cell(0, 0, "1st")
    t.m2.insert_rows(0, 1)
    t.m2.set_cell(0, 0, "2nd")
    t.expect([["2nd"], ["1st"]])


def overlapping_remove_col(t):  # :423-435
    t.m1.insert_cols(0, 3)
    t.m1.insert_rows(0, 1)
    t.m1.set_cell(0, 0, "A")
    t.m1.set_cell(0, 1, "B")
    t.m1.set_cell(0, 2, "C")
    t.expect([["A", "B", "C"]])
    t.m1.remove_cols(1, 1)
    t.m2.remove_cols(1, 1)
    t.expect([["A", "C"]])


def overlapping_remove_row(t):  # :437-449
    t.m1.insert_cols(0, 1)
    t.m1.insert_rows(0, 3)
    t.m1.set_cell(0, 0, "A")
    t.m1.set_cell(1, 0, "B")
    t.m1.set_cell(2, 0, "C")
    t.expect([["A"], ["B"], ["C"]])
    t.m1.remove_rows(1, 1)
    t.m2.remove_rows(1, 1)
    t.expect([["A"], ["C"]])


def insert_col_vs_remove_row(t):  # :451-478
    t.m1.insert_cols(0, 2)
    t.m1.insert_rows(0, 3)
    t.m1.set_cells(0, 0, 2, ["A1", "C1", "A2", "C2", "A3", "C3"])
    t.expect([["A1", "C1"], ["A2", "C2"], ["A3", "C3"]])
    t.m1.insert_cols(1, 1)
    t.m1.set_cells(0, 1, 1, ["B1", "B2", "B3"])
    t.m2.remove_rows(1, 1)
    t.expect([["A1", "B1", "C1"], ["A3", "B3", "C3"]])


def insert_row_vs_remove_col(t):  # :480-507 (and its twin :509-536)
    t.m1.insert_rows(0, 2)
    t.m1.insert_cols(0, 3)
    t.m1.set_cells(0, 0, 3, ["A1", "B1", "C1", "A3", "B3", "C3"])
    t.expect([["A1", "B1", "C1"], ["A3", "B3", "C3"]])
    t.m1.insert_rows(1, 1)
    t.m1.set_cells(1, 0, 3, ["A2", "B2", "C2"])
    t.m2.remove_cols(1, 1)
    t.expect([["A1", "C1"], ["A2", "C2"], ["A3", "C3"]])


def insert_col_vs_insert_and_remove_row(t):  # :539-553
    t.m1.insert_rows(0, 2)
    t.m1.insert_cols(0, 2)
    t.m1.set_cells(0, 0, 2, ["A1", "C1", "A2", "C2"])
    t.m1.remove_rows(1, 1)
    t.m1.insert_cols(1, 1)
    t.expect([["A1", None, "C1"]])


def insert_row_col_vs_insert_row_and_set(t):  # :556-576 (convergence only)
    t.m1.insert_rows(0, 4)
    t.m1.insert_cols(0, 4)
    t.m1.set_cells(0, 0, 4, list(range(16)))
    t.expect()
    t.m1.insert_rows(0, 1)
    t.m2.insert_rows(0, 2)
    t.m2.set_cells(0, 0, 4, ["A", "B", "C", "D"])
    t.m1.insert_cols(1, 1)
    t.expect()


def remove_rows_vs_set_cells(t):  # :579-592 (writes to deleted handles are ignored; convergence)
    t.m1.insert_rows(0, 3)
    t.m1.insert_cols(0, 2)
    t.m1.set_cells(0, 0, 2, [0, 1, 2, 3])
    t.m2.insert_rows(0, 1)
    t.expect()
    t.m1.remove_rows(1, 1)
    t.m2.set_cells(0, 0, 1, ["A", "B", "C"])
    t.expect()


def overlapping_insert_set_vs_remove_insert_set(t):  # :596-608
    t.m1.insert_rows(0, 1)
    t.m1.insert_cols(0, 4)
    t.m1.set_cells(0, 0, 4, [0, 1, 2, 3])
    t.expect([[0, 1, 2, 3]])
    t.m2.insert_cols(1, 1)
    t.m2.set_cells(0, 1, 1, ["A"])
    t.m1.remove_cols(0, 2)
    t.m1.insert_cols(0, 1)
    t.m1.set_cells(0, 0, 1, ["B"])
    t.expect([["B", "A", 2, 3]])


CONFLICT = [set_cell, clear_unallocated_cell, insert_and_set_in_new_row, insert_and_set_in_new_col, insert_col_conflict,
            insert_row_conflict, overlapping_remove_col, overlapping_remove_row, insert_col_vs_remove_row,
            insert_row_vs_remove_col, insert_col_vs_insert_and_remove_row, insert_row_col_vs_insert_row_and_set,
            remove_rows_vs_set_cells, overlapping_insert_set_vs_remove_insert_set]


@pytest.mark.parametrize("engine", KINDS)
@pytest.mark.parametrize("case", CONFLICT, ids=[c.__name__ for c in CONFLICT])
def test_connected_two_clients_conflict(case, engine):
    t = Two(engine)
    case(t)
    t.expect()  # the describe's afterEach (:350-355)
    if engine:
        assert t.s.checks > 0


# ---------------------------------------------------------------- "local client" / "summarize" (:273-307)
def _vector_tree(blobs):
    """PermutationVector.summarize's tree from [segment blobs..., handleTable] (permutationvector.ts:310-325)."""
    return {"segments": {("header" if i == 0 else f"body_{i - 1}"): b for i, b in enumerate(blobs[:-1])},
            "handleTable": blobs[-1]}


def _summary(s, c):
    """SharedMatrix.summarizeCore (matrix.ts:449-464) of client c: both vectors' trees and the cells blob."""
    s.flush()
    if s.eng is not None:
        from fluidframework_amd.cells import matrix_summary

        s.eng.summarize()
        tree = matrix_summary(s.eng, 2 * c.k, 2 * c.k + 1, c.log)
        for w, name in ((0, "rows"), (1, "cols")):  # (the oracle's summary of the same vector is the same tree)
            assert tree[name] == _vector_tree(c.doc.select(w).summarize(s.last_batch, 2 * c.k)), name
        return tree
    return {"rows": _vector_tree(c.doc.select(0).summarize(s.last_batch, 2 * c.k)),
            "cols": _vector_tree(c.doc.select(1).summarize(s.last_batch, 2 * c.k)), "cells": c.log.cells_blob()}


def _load(engine, tree):
    """summarize()'s 2nd matrix (:64-92): a new SharedMatrix loaded from the summary (SnapshotLoader starts
    collaboration as "snapshot", merge-tree snapshotLoader.ts) -- a session of one client."""
    s = MSession(["loaded"], engine, attached=False)
    c = s.clients[0]
    c.log.load_summary(tree, "snapshot", s.it)
    return s, c


@pytest.mark.parametrize("engine", KINDS)
def test_local_client_summarize_mutate_after_load(engine):  # :274-305
    s = MSession(["matrix1"], engine, attached=False)
    m = s.clients[0]
    m.insert_cols(0, 2)
    m.insert_rows(0, 2)
    m.set_cells(0, 0, 2, [0, 1, 2, 3])
    assert m.extract() == [[0, 1], [2, 3]]
    tree = _summary(s, m)
    s2, m2 = _load(engine, tree)
    assert m2.extract() == [[0, 1], [2, 3]]  # "Matrix must round-trip through summarize/load."
    assert _summary(s2, m2) == tree  # (the loaded matrix summarizes to the same tree)
    m2.insert_rows(1, 1)
    assert m2.extract() == [[0, 1], [None, None], [2, 3]]
    m2.set_cells(1, 0, 2, [10, 11])
    assert m2.extract() == [[0, 1], [10, 11], [2, 3]]
    m2.insert_cols(1, 1)
    assert m2.extract() == [[0, None, 1], [10, None, 11], [2, None, 3]]


# ---------------------------------------------------------------- "Reconnection" (:612-880)
class TwoR(Two):
    """beforeEach of "Reconnection" (:643-659): two matrices on MockContainerRuntimeFactoryForReconnection; a
    client's `connected` setter is its runtime's (disconnect drops its unsequenced messages, reconnect processes
    the messages sequenced meanwhile, takes a new client id and resubmits every pending message)."""


def resend_setcell_when_later_ops_shift(t, reconnects=1):  # :668-695 (reconnects=2: :697-729)
    t.m1.insert_rows(0, 1)
    t.m1.insert_cols(0, 1)
    t.expect([[None]])
    t.m1.set_cells(0, 0, 1, ["A"])
    t.m1.insert_cols(0, 3)
    for _ in range(reconnects):
        t.m1.connected = False
        t.m1.connected = True
    t.expect([[None, None, None, "A"]])


def resend_setcell_multiple_reconnects(t):  # :697-729
    resend_setcell_when_later_ops_shift(t, 2)


def resend_unacked_ops(t):  # :731-752
    t.m1.insert_cols(0, 1)
    t.m1.insert_rows(0, 1)
    t.m1.connected = False
    t.m1.connected = True
    t.expect([[None]])
    t.m2.set_cell(0, 0, "2nd")
    t.m2.connected = False
    t.m2.connected = True
    t.expect([["2nd"]])


def store_ops_while_disconnected(t):  # :754-779
    t.m1.connected = False
    t.m1.insert_cols(0, 1)
    t.m1.insert_rows(0, 1)
    t.m1.connected = True
    t.expect([[None]])
    t.m2.connected = False
    t.m2.set_cell(0, 0, "2nd")
    t.m2.connected = True
    t.expect([["2nd"]])


def omit_writes_to_recycled_handles(t):  # :808-825
    t.m1.insert_rows(0, 2)
    t.m1.insert_cols(0, 2)
    t.m1.set_cells(0, 0, 2, [0, 1, 2, 3])
    t.m1.remove_rows(1, 1)
    t.m1.connected = False
    t.m1.insert_rows(0, 1)
    t.m1.set_cells(0, 0, 2, [28, 49])
    t.m1.connected = True
    t.expect([[28, 49], [0, 1]])


def omit_not_yet_locally_deleted(t):  # :827-859
    t.m1.insert_rows(0, 2)
    t.m1.insert_cols(0, 4)
    t.m1.set_cells(0, 0, 4, [0, 1, 2, 3, 4, 5, 6, 7])
    t.m1.insert_rows(0, 1)
    t.m1.set_cells(0, 0, 4, [61, 57, 7, 62])
    t.m1.connected = False
    t.m1.connected = True
    t.expect([[61, 57, 7, 62], [0, 1, 2, 3], [4, 5, 6, 7]])
    t.m1.set_cells(2, 3, 1, [65])
    t.m1.connected = False
    t.m1.remove_rows(0, 1)
    t.m1.connected = True
    t.expect([[0, 1, 2, 3], [4, 5, 6, 65]])


def reset_handles_for_resubmitted_ops(t):  # :861-879
    t.m1.insert_rows(0, 1)
    t.m1.insert_cols(0, 1)
    t.m1.set_cells(0, 0, 1, [0])
    t.m2.insert_cols(0, 1)
    t.m2.insert_rows(0, 1)
    t.m2.set_cells(0, 0, 1, [90])
    t.m2.connected = False
    t.m2.connected = True
    t.expect([[90, None], [None, 0]])


RECONNECT = [resend_setcell_when_later_ops_shift, resend_setcell_multiple_reconnects, resend_unacked_ops,
             store_ops_while_disconnected, omit_writes_to_recycled_handles, omit_not_yet_locally_deleted,
             reset_handles_for_resubmitted_ops]


@pytest.mark.parametrize("engine", KINDS)
@pytest.mark.parametrize("case", RECONNECT, ids=[c.__name__ for c in RECONNECT])
def test_reconnection(case, engine):
    """The "Reconnection" cases (setCell(IFluidHandle), :781-806, compares handle objects and is not restated)."""
    t = TwoR(engine)
    case(t)
    t.expect()  # afterEach (:661-666)
    if engine:
        assert t.s.checks > 0
