"""SharedMatrix local edits: a live SharedMatrix's own row / col inserts and removes (local
merge-tree ops on its PermutationVectors, pending until their ACKs), its own cell writes
(SharedMatrix.setCell -> setCellCore -> sendSetCellOp, matrix.ts:202-310: getAllocatedHandle at the local view,
the value at once, a `pending` entry until the ACK) and the rules that keep remote writes from clobbering them
(matrix.ts:652-690, isLatestPendingWrite :738-759), with the cells blob holding both tries (:458-462).

A seeded farm: two writers make edits at their local views each round, the round's messages are sequenced in
order and applied to every client (a writer's own messages are its ACKs), an observer follows.  After the
last round (every edit acked, nothing pending) every client shows the same value at every (row, col) position
-- SharedMatrix's convergence -- although each client allocated its own handles.  CPU: the oracle drives the
clients' cell stores; -m gpu: the HIP engine's handle and recycling records equal the oracle's batch by batch,
the cell stores they drive are byte-identical, and so are both vectors' summaries.
"""
import copy
import random

import numpy as np
import pytest

from fluidframework_amd import abi
from fluidframework_amd.batch import Interner, build_batch
from fluidframework_amd.cells import CellMatrixLog
from oracle.oracle import OracleDoc, options

U = -2 ** 31  # Handle.unallocated (handletable.ts:11)


class Client:
    def __init__(self, name):
        self.name = name
        self.log = CellMatrixLog()
        self.log.start_collab(name)
        self.doc = OracleDoc(options(), matrix=True)
        self.shadow = None  # the engine-driven cell store (-m gpu)
        self.seq = 0

    def dims(self):  # the local view's row / col counts (the observer is short id 0)
        return int(self.doc.select(0).length(self.seq, 0)), int(self.doc.select(1).length(self.seq, 0))

    def value(self, r, c):
        rh, ch = self.doc.select(0).handle_at(r), self.doc.select(1).handle_at(c)
        if rh < 1 or ch < 1:
            return None
        return self.log.cells.get_cell(rh, ch)

    def grid(self):
        nr, nc = self.dims()
        return [[self.value(r, c) for c in range(nc)] for r in range(nr)]


class Session:
    def __init__(self, names, engine=False):
        self.it = Interner()
        self.clients = [Client(n) for n in names]
        self.eng = None
        if engine:
            from fluidframework_amd.engine import Engine
            self.eng = Engine(2 * len(names), max_segments=4096, heap_entries=4096, text_units=1 << 14,
                              prop_words=1024, remover_cells=4096, ops_per_launch=64)
            for m in range(len(names)):
                self.eng.set_matrix(2 * m, 2 * m + 1)
            for c in self.clients:
                c.shadow = CellMatrixLog()
        self.checks = 0

    def flush(self):
        cols = [c.log.cols_log() for c in self.clients]
        shadows = [(dict(c.log.values), dict(c.log.local_sets), list(c.log.events), dict(c.log.ops_kind))
                   for c in self.clients]
        b = build_batch([x for c, cl in zip(self.clients, cols) for x in (c.log, cl)], self.it)
        if self.eng is not None:
            self.eng.apply(b)
        for m, c in enumerate(self.clients):
            assert c.doc.apply(b, 2 * m) == 0, c.name
            orows, ocols = c.doc.select(0).deltas(), c.doc.select(1).deltas()
            c.log.resolve(orows, ocols)
            if self.eng is not None:
                assert self.eng.status(2 * m)[0] == 0 and self.eng.status(2 * m + 1)[0] == 0, c.name
                erows, ecols = self.eng.deltas(2 * m), self.eng.deltas(2 * m + 1)
                assert np.array_equal(erows, orows) and np.array_equal(ecols, ocols), c.name
                sh = c.shadow
                sh.values, sh.local_sets, sh.events, sh.ops_kind = copy.deepcopy(shadows[m])
                sh.resolve(erows, ecols)
                assert sh.cells_blob() == c.log.cells_blob(), c.name
                self.checks += 1
        return b

    def deliver(self, msgs, msn):
        for m in msgs:
            m["minimumSequenceNumber"] = msn
            for c in self.clients:
                c.log.message(m, self.it)
                c.seq = m["sequenceNumber"]


def _msg(seq, ref, client, contents):
    return {"type": "op", "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": 0,
            "clientId": client, "contents": contents}


def farm(seed, s, writers=("w1", "w2"), rounds=10, per_round=4):
    """Returns every client's final grid."""
    rnd = random.Random(seed)
    seq = [0]
    by = {c.name: c for c in s.clients}
    # a seed client grows the matrix first (remote for everyone)
    init = [{"target": "rows", "type": 0, "pos1": 0, "seg": [4, U]}, {"target": "cols", "type": 0, "pos1": 0, "seg": [3, U]}]
    msgs = []
    for op in init:
        seq[0] += 1
        msgs.append(_msg(seq[0], seq[0] - 1, "seed", op))
    s.deliver(msgs, 0)
    s.flush()
    for rd in range(rounds):
        start = seq[0]
        sent = []
        for _ in range(per_round):
            w = by[rnd.choice(writers)]
            s.flush()
            nr, nc = w.dims()
            k = rnd.random()
            if k < 0.15 or nr == 0:
                pos, cnt = rnd.randint(0, nr), rnd.randint(1, 3)
                op = {"target": "rows", "type": 0, "pos1": pos, "seg": [cnt, U]}
                w.log.local_vector_op("rows", op)
            elif k < 0.3 or nc == 0:
                pos, cnt = rnd.randint(0, nc), rnd.randint(1, 2)
                op = {"target": "cols", "type": 0, "pos1": pos, "seg": [cnt, U]}
                w.log.local_vector_op("cols", op)
            elif k < 0.4 and nr > 1:
                a = rnd.randrange(nr)
                op = {"target": "rows", "type": 1, "pos1": a, "pos2": min(nr, a + rnd.randint(1, 2))}
                w.log.local_vector_op("rows", op)
            elif k < 0.48 and nc > 1:
                a = rnd.randrange(nc)
                op = {"target": "cols", "type": 1, "pos1": a, "pos2": a + 1}
                w.log.local_vector_op("cols", op)
            else:
                r, c = rnd.randrange(nr), rnd.randrange(nc)
                v = f"{w.name}:{rd}:{rnd.randint(0, 99)}"
                op = {"type": 2, "row": r, "col": c, "value": v}
                w.log.local_set_cell(r, c, v)
            sent.append(_msg(0, w.seq, w.name, op))
        for m in sent:  # sequenced in the order they were made
            seq[0] += 1
            m["sequenceNumber"] = seq[0]
        s.deliver(sent, start)
        s.flush()
    for c in s.clients:
        assert c.log.local_meta == [], f"{c.name}: unacked local writes"
    return [c.grid() for c in s.clients]


@pytest.mark.parametrize("seed", range(8))
def test_matrix_local_farm_converges_oracle(seed):
    s = Session(["w1", "w2", "obs"])
    grids = farm(seed, s)
    assert grids[0] == grids[1] == grids[2], f"seed {seed}"
    assert any(v is not None for row in grids[0] for v in row)


def test_pending_write_masks_an_earlier_remote_write():
    """matrix.ts:681-690: a remote write sequenced before this client's own write to the same cell (but
    made before the client saw it) must not clobber the local value; the ACK then clears the pending
    entry (isLatestPendingWrite), and a later remote write lands."""
    s = Session(["me"])
    me = s.clients[0]
    s.deliver([_msg(1, 0, "other", {"target": "rows", "type": 0, "pos1": 0, "seg": [2, U]}),
               _msg(2, 1, "other", {"target": "cols", "type": 0, "pos1": 0, "seg": [2, U]})], 0)
    s.flush()
    me.log.local_set_cell(1, 1, "mine")
    s.flush()
    assert me.value(1, 1) == "mine"
    # a remote write to the same cell, sequenced first: skipped (pending local write)
    s.deliver([_msg(3, 2, "other", {"type": 2, "row": 1, "col": 1, "value": "theirs"})], 0)
    s.flush()
    assert me.value(1, 1) == "mine"
    # our ACK clears the pending entry
    s.deliver([_msg(4, 2, "me", {"type": 2, "row": 1, "col": 1, "value": "mine"})], 0)
    s.flush()
    assert me.log.pending.get_cell(me.doc.select(0).handle_at(1), me.doc.select(1).handle_at(1)) is None
    s.deliver([_msg(5, 4, "other", {"type": 2, "row": 1, "col": 1, "value": "later"})], 0)
    s.flush()
    assert me.value(1, 1) == "later"
    assert me.log.cells_blob().count(b"later") == 1


def test_two_pending_writes_keep_the_latest():
    """Two local writes to one cell: the first ACK finds a later pending localSeq and keeps the entry
    (isLatestPendingWrite false); only the second clears it."""
    s = Session(["me"])
    me = s.clients[0]
    s.deliver([_msg(1, 0, "other", {"target": "rows", "type": 0, "pos1": 0, "seg": [1, U]}),
               _msg(2, 1, "other", {"target": "cols", "type": 0, "pos1": 0, "seg": [1, U]})], 0)
    s.flush()
    me.log.local_set_cell(0, 0, "a")
    me.log.local_set_cell(0, 0, "b")
    s.flush()
    h = (me.doc.select(0).handle_at(0), me.doc.select(1).handle_at(0))
    assert me.log.pending.get_cell(*h) == 2 and me.value(0, 0) == "b"
    s.deliver([_msg(3, 2, "me", {"type": 2, "row": 0, "col": 0, "value": "a"})], 0)
    s.flush()
    assert me.log.pending.get_cell(*h) == 2
    s.deliver([_msg(4, 2, "other", {"type": 2, "row": 0, "col": 0, "value": "x"})], 0)
    s.flush()
    assert me.value(0, 0) == "b"  # still pending: the remote write happened before "b"
    s.deliver([_msg(5, 2, "me", {"type": 2, "row": 0, "col": 0, "value": "b"})], 0)
    s.flush()
    assert me.log.pending.get_cell(*h) is None


@pytest.mark.gpu
def test_matrix_local_farm_engine_matches_oracle():
    for seed in range(4):
        s = Session(["w1", "w2", "obs"], engine=True)
        grids = farm(seed, s)
        assert grids[0] == grids[1] == grids[2], f"seed {seed}"
        assert s.checks > 0
        last = s.flush()
        s.eng.summarize()
        for m, c in enumerate(s.clients):
            for w in (0, 1):
                assert s.eng.summary(2 * m + w) == c.doc.select(w).summarize(last, 2 * m), (seed, c.name, w)
