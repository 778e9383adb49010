"""SharedMatrix row/col PermutationVectors.

CPU tests pin the oracle's restatement with hand-derived known answers from the reference code
(matrix/src/matrix.ts:636-693 processCore, permutationvector.ts:209-247 getAllocatedHandle /
adjustPosition, :418-443 handle recycling on UNLINK, handletable.ts:35-60 allocate/free) and check
invariants on seeded synthetic logs.  The reference has no committed matrix summary fixtures, so
parity for matrix summaries is unpinned by the reference (oracle restatement + engine agreement);
GPU tests compare the HIP engine with the oracle vector by vector, leaf by leaf and byte by byte.
"""
from __future__ import annotations

import json

import numpy as np
import pytest

from fluidframework_amd import abi
from fluidframework_amd.batch import Interner, MatrixLog, build_batch, matrix_logs
from fluidframework_amd.synth import make_cfg, tables, with_docs
from oracle.oracle import OracleDoc, generate_matrix, options, replay_matrix_batch, summary_digest

U = abi.HANDLE_UNALLOCATED


def _msg(seq, ref, client, contents, msn=0):
    return {"type": "op", "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "clientId": client, "contents": contents}


def _kat_log():
    it = Interner()
    log = MatrixLog()
    log.start_collab("observer")
    log.message(_msg(1, 0, "A", {"target": "rows", "type": 0, "pos1": 0, "seg": [3, 7]}), it)   # insertRows(0, 3)
    log.message(_msg(2, 1, "A", {"target": "cols", "type": 0, "pos1": 0, "seg": [2, 9]}), it)   # insertCols(0, 2)
    log.message(_msg(3, 2, "B", {"type": 2, "row": 1, "col": 1, "value": "x"}), it)             # setCell(1, 1)
    log.message(_msg(4, 2, "B", {"type": 2, "row": 1, "col": 0, "value": "y"}), it)             # setCell(1, 0)
    return log, it


def _oracle(batch, doc=0):
    o = OracleDoc(options(), matrix=True)
    assert o.apply(batch, doc) == 0
    return o


def test_known_answer_handle_allocation():
    """Inserted segments start unallocated (the remote start 7/9 is reset, permutationvector.ts:354-361);
    setCell(1, 1) splits row 1 and col 1 out and gives each handle 1; setCell(1, 0) reuses row handle 1
    (cache hit) and allocates col handle 2 for col 0 (no split at position 0: `if (start)`,
    mergeTree.ts:2461)."""
    log, it = _kat_log()
    b = build_batch([log], it)
    o = _oracle(b)
    rows = o.select(0).summarize(b, 0)
    cols = o.select(1).summarize(b, 0)
    seg = lambda j: {"json": j, "seq": 1, "client": "A"}  # noqa: E731
    assert json.loads(rows[0]) == {
        "version": "1", "segmentCount": 3, "length": 3,
        "segments": [seg([1, U]), seg([1, 1]), seg([1, U])], "startIndex": 0,
        "headerMetadata": {"minSequenceNumber": 0, "sequenceNumber": 1, "orderedChunkMetadata": [{"id": "header"}],
                           "totalLength": 3, "totalSegmentCount": 3}}
    assert rows[1] == b"[2,0]"
    seg2 = lambda j: {"json": j, "seq": 2, "client": "A"}  # noqa: E731
    assert json.loads(cols[0])["segments"] == [seg2([1, 2]), seg2([1, 1])]
    assert json.loads(cols[0])["headerMetadata"]["sequenceNumber"] == 2
    assert cols[1] == b"[3,0,0]"


def test_known_answer_recycling_and_coalescing():
    """Removing an allocated row and moving the MSN past the removal unlinks it and frees its handle
    (free list head = that handle, handles[h] = old head); below-MSN segments with contiguous handles
    coalesce in the summary ([1,1] + [1,2] -> [2,1], PermutationSegment.canAppend)."""
    it = Interner()
    log = MatrixLog()
    log.start_collab("observer")
    log.message(_msg(1, 0, "A", {"target": "rows", "type": 0, "pos1": 0, "seg": [4, -1]}), it)
    log.message(_msg(2, 1, "A", {"target": "cols", "type": 0, "pos1": 0, "seg": [1, -1]}), it)
    for s, r in ((3, 0), (4, 1), (5, 2)):  # rows 0, 1, 2 get handles 1, 2, 3
        log.message(_msg(s, 2, "A", {"type": 2, "row": r, "col": 0, "value": s}), it)
    log.message(_msg(6, 5, "A", {"target": "rows", "type": 1, "pos1": 2, "pos2": 3}, msn=5), it)  # removeRows(2, 1)
    log.message(_msg(7, 6, "A", {"target": "rows", "type": 0, "pos1": 3, "seg": [1, -1]}, msn=6), it)
    b = build_batch([log], it)
    o = _oracle(b)
    rows = o.select(0).summarize(b, 0)
    head = json.loads(rows[0])
    # the removal found its block already queued for scouring (needsScour, mergeTree.ts:741-751), so
    # the scour at MSN 5 kept it (removedSeq 6 > 5); nothing has unlinked it yet
    assert head["headerMetadata"]["minSequenceNumber"] == 6
    assert head["segments"] == [[2, 1], [1, U], {"json": [1, U], "seq": 7, "client": "A"}]
    assert rows[1] == b"[4,0,0,0]"
    # MSN 7 pops the block queued by seq 7: the removed row is unlinked and handle 3 freed
    # (head -> 3 -> 4), the two unallocated rows below the MSN coalesce
    log.message(_msg(8, 7, "A", {"target": "rows", "type": 0, "pos1": 0, "seg": [1, -1]}, msn=7), it)
    b = build_batch([log], it)
    assert o.apply(b, 0) == 0
    rows = o.select(0).summarize(b, 0)
    assert json.loads(rows[0])["segments"] == [{"json": [1, U], "seq": 8, "client": "A"}, [2, 1], [2, U]]
    assert rows[1] == b"[3,0,0,4]"


def test_packer_matrix_messages():
    log, it = _kat_log()
    ops = build_batch(matrix_logs([log]), it).ops
    assert list(ops["type"]) == [abi.OP_START_COLLAB, abi.OP_INSERT, abi.OP_INSERT, abi.OP_SETCELL, abi.OP_SETCELL]
    assert list(ops["flags"]) == [0, abi.F_LAST, abi.F_LAST | abi.F_COLS, 0, 0]
    assert list(ops["payload2"][1:3]) == [3, 2]
    assert list(ops["pos1"][3:]) == [1, 1] and list(ops["pos2"][3:]) == [1, 0]


def matrix_cfg(n, ops, writers=8, max_lag=16, seed=0xfeedbed):
    # C4 mix: 20 % row/col splices (insert 12 : remove 8), 80 % setCell
    return make_cfg(n, ops, writers=writers, max_lag=max_lag, weights=(12, 8, 80), max_text=4, max_range=3,
                    seed=seed)


def handle_invariants(o, batch, doc):
    """Every live handle is covered by exactly one segment range, the free list is acyclic and holds
    exactly the handles no segment owns."""
    ex, _ = o.export()
    table = json.loads(o.summarize(batch, doc)[-1])
    owned = set()
    for r in ex:
        if r[6] >= 1:
            for h in range(int(r[6]), int(r[6]) + int(r[0])):
                assert h not in owned
                owned.add(h)
    free, h, seen = set(), table[0], 0
    while h < len(table):
        assert h not in free
        free.add(h)
        h = table[h]
        seen += 1
        assert seen <= len(table)
    assert owned.isdisjoint(free)
    assert owned | free == set(range(1, len(table)))


@pytest.mark.parametrize("writers,lag", [(8, 16), (3, 0), (16, 64)])
def test_synthetic_matrix_oracle_invariants(writers, lag):
    cfg = matrix_cfg(8, 1500, writers=writers, max_lag=lag)
    tabs = tables(writers=writers)
    b, hashes, status = generate_matrix(cfg, tabs, 0, 8, threads=4)
    assert (status == 0).all()
    for d in range(8):
        o = _oracle(b, d)
        for w in (0, 1):
            handle_invariants(o.select(w), b, d)


def expand_pairs(batch, tabs):
    """One generated document per matrix -> engine order [rows 0, cols 0, rows 1, ...]."""
    n = batch.n_docs
    docs = np.zeros(2 * n, dtype=abi.DOC_DTYPE)
    docs[0::2] = batch.docs
    docs[1::2]["op_begin"] = batch.docs["op_begin"]
    docs[1::2]["n_clients"] = batch.docs["n_clients"]
    return with_docs(tabs, docs, batch.ops, batch.text)


@pytest.mark.gpu
@pytest.mark.parametrize("writers,lag,ops,n", [(8, 16, 2000, 48), (16, 64, 1500, 48), (3, 0, 1000, 48), (8, 64, 20000, 16)],
                         ids=["w8-lag16", "w16-lag64", "w3-lag0", "c4-size"])
def test_matrix_engine_matches_oracle(writers, lag, ops, n):
    """(c4-size: config C4's matrices at full length -- 20,000 messages, 8 writers, lag <= 64.)"""
    from fluidframework_amd.engine import Engine

    cfg = matrix_cfg(n, ops, writers=writers, max_lag=lag)
    tabs = tables(writers=writers)
    gb, _, status = generate_matrix(cfg, tabs, 0, n, threads=8)
    assert (status == 0).all()
    b = expand_pairs(gb, tabs)
    eng = Engine(2 * n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=1 << 15,
                 prop_words=1024, remover_cells=4096, ops_per_launch=64)
    for m in range(n):
        eng.set_matrix(2 * m, 2 * m + 1)
    eng.apply(b)
    eng.summarize()
    for m in range(n):
        o = _oracle(gb, m)
        for w in (0, 1):
            d = 2 * m + w
            st, op = eng.status(d)
            assert st == 0, f"matrix {m} vector {w}: status {st:#x} at op {op}"
            o.select(w)
            ge, gh = eng.export(d)
            oe, oh = o.export()
            assert gh == oh and np.array_equal(ge, oe), f"matrix {m} vector {w}: leaves differ"
            assert eng.summary(d) == o.summarize(gb, m), f"matrix {m} vector {w}: summary bytes differ"


def test_oracle_matrix_replay_digests():
    """The C4 bench's CPU leg: per-vector digests of a replayed matrix equal the digests of the
    oracle's own summaries of each vector."""
    n = 6
    cfg = matrix_cfg(n, 800)
    tabs = tables(writers=8)
    b, _, status = generate_matrix(cfg, tabs, 0, n, threads=4)
    assert (status == 0).all()
    _, h, st = replay_matrix_batch(b, 0, n, 4)
    assert (st == 0).all()
    for m in range(n):
        o = _oracle(b, m)
        for w in (0, 1):
            assert int(h[2 * m + w]) == summary_digest(o.select(w).summarize(b, m)), f"matrix {m} vector {w}"


@pytest.mark.gpu
@pytest.mark.parametrize("writers,lag,ops", [(8, 64, 1500), (16, 16, 1000)])
def test_matrix_record_mode_matches_oracle_generator(writers, lag, ops):
    """Record mode for matrices (mtr_generate_matrix, the C4 bench's input): the engine draws the
    same op logs as the oracle's generator from the same seeds, and replaying them reproduces the
    oracle's per-vector summaries."""
    from fluidframework_amd.engine import Engine

    n = 32
    cfg = matrix_cfg(n, ops, writers=writers, max_lag=lag)
    tabs = tables(writers=writers)
    eng = Engine(2 * n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=1 << 12,
                 prop_words=1024, remover_cells=4096, ops_per_launch=48)
    eng.generate_matrix(cfg, tabs)
    gb = eng.download_matrix(0, n)
    ob, _, status = generate_matrix(cfg, tabs, 0, n, threads=8)
    assert (status == 0).all()
    assert np.array_equal(gb.docs["op_count"], ob.docs["op_count"])
    assert np.array_equal(gb.ops, ob.ops), "recorded matrix logs differ from the oracle generator's"
    eng.reset()
    eng.run()
    eng.summarize()
    eng.sync()
    for d in range(2 * n):
        assert eng.status(d)[0] == 0, f"document {d}: {eng.status(d)}"
    _, oh, st = replay_matrix_batch(ob, 0, n, 8)
    assert (st == 0).all()
    assert np.array_equal(eng.hashes(2 * n), oh)


# ---------------------------------------------------------------- cells

from fluidframework_amd.cells import CellMatrixLog, SparseArray2D, morton  # noqa: E402


def _morton_slow(row, col):
    """Bit-by-bit restatement of r0c0ToMorton2x16 (sparsearray2d.ts:30-31): row bit i -> 2i+1,
    col bit i -> 2i, of the low 16 bits."""
    k = 0
    for i in range(16):
        k |= ((row >> i) & 1) << (2 * i + 1)
        k |= ((col >> i) & 1) << (2 * i)
    return k


def test_sparsearray2d_morton_and_layout():
    for r, c in [(0, 0), (1, 1), (1, 2), (0x1234, 0x5678), (0xFFFF, 0), (70000, 3)]:
        assert morton(r, c) == _morton_slow(r & 0xFFFF, c & 0xFFFF)
    a = SparseArray2D()
    a.set_cell(1, 1, "x")   # key 3
    a.set_cell(1, 2, "y")   # key 6
    lvl3 = [None] * 256
    lvl3[3], lvl3[6] = "x", "y"
    pad = lambda x: [x] + [None] * 255  # noqa: E731
    assert a.snapshot() == [pad(pad(pad(lvl3)))]
    assert a.get_cell(1, 2) == "y" and a.get_cell(2, 1) is None
    # clearing keeps every allocated level (levels are never freed) and only nulls the cells
    a.set_cell(300, 5, 7)
    a.clear_rows(1, 1)
    assert a.get_cell(1, 1) is None and a.get_cell(1, 2) is None and a.get_cell(300, 5) == 7
    assert a.snapshot()[0][0][0][0] == [None] * 256
    a.clear_cols(5, 1)
    assert a.get_cell(300, 5) is None
    # a handle above 65535 lands in root[keyHi]: the root array grows with holes (JSON null)
    b = SparseArray2D()
    b.set_cell(0x10000, 0, True)
    assert len(b.snapshot()) == 3 and b.snapshot()[0] is None and b.get_cell(0x10000, 0) is True


def _cell_msgs(log, it, msgs):
    for m in msgs:
        log.message(m, it)


def test_known_answer_cells_blob():
    """The KAT matrix (test_known_answer_handle_allocation): setCell(1, 1) writes cell (row handle 1,
    col handle 1) and setCell(1, 0) writes (1, 2) -> keys 3 and 6 of one level chain; no pending
    writes -> the second trie is [null]."""
    it = Interner()
    log = CellMatrixLog()
    log.start_collab("observer")
    _cell_msgs(log, it, [
        _msg(1, 0, "A", {"target": "rows", "type": 0, "pos1": 0, "seg": [3, 7]}),
        _msg(2, 1, "A", {"target": "cols", "type": 0, "pos1": 0, "seg": [2, 9]}),
        _msg(3, 2, "B", {"type": 2, "row": 1, "col": 1, "value": "x"}),
        _msg(4, 2, "B", {"type": 2, "row": 1, "col": 0, "value": {"v": [1, 2.5]}}),
    ])
    b = build_batch([log], it)
    o = _oracle(b)
    rows, cols = o.select(0).deltas(), o.select(1).deltas()
    assert [tuple(int(x) for x in r) for r in rows] == [(3, 1, 1, abi.OP_SETCELL), (4, 1, 2, abi.OP_SETCELL)]
    assert len(cols) == 0
    log.resolve(rows, cols)
    lvl3 = ["null"] * 256
    lvl3[3], lvl3[6] = '"x"', '{"v":[1,2.5]}'
    pad = lambda x: "[" + ",".join([x] + ["null"] * 255) + "]"  # noqa: E731
    assert log.cells_blob() == ("[[" + pad(pad(pad("[" + ",".join(lvl3) + "]"))) + "],[null]]").encode()


def test_known_answer_recycled_handles_clear_cells():
    """test_known_answer_recycling_and_coalescing with values: the removed row's handle 3 is freed
    when the MSN passes its removal (seq 8) -> its cell is cleared; rows 0 and 1 keep theirs."""
    it = Interner()
    log = CellMatrixLog()
    log.start_collab("observer")
    msgs = [
        _msg(1, 0, "A", {"target": "rows", "type": 0, "pos1": 0, "seg": [4, -1]}),
        _msg(2, 1, "A", {"target": "cols", "type": 0, "pos1": 0, "seg": [1, -1]}),
    ] + [_msg(s, 2, "A", {"type": 2, "row": r, "col": 0, "value": s}) for s, r in ((3, 0), (4, 1), (5, 2))] + [
        _msg(6, 5, "A", {"target": "rows", "type": 1, "pos1": 2, "pos2": 3}, msn=5),
        _msg(7, 6, "A", {"target": "rows", "type": 0, "pos1": 3, "seg": [1, -1]}, msn=6),
    ]
    _cell_msgs(log, it, msgs)
    b = build_batch([log], it)
    o = _oracle(b)
    log.resolve(o.select(0).deltas(), o.select(1).deltas())
    assert [log.cells.get_cell(h, 1) for h in (1, 2, 3)] == [3, 4, 5]
    _cell_msgs(log, it, [_msg(8, 7, "A", {"target": "rows", "type": 0, "pos1": 0, "seg": [1, -1]}, msn=7)])
    b = build_batch([log], it)
    assert o.apply(b, 0) == 0
    rows = o.select(0).deltas()
    assert [tuple(int(x) for x in r) for r in rows] == [(0, 3, 1, 32)]
    log.resolve(rows, o.select(1).deltas())
    assert [log.cells.get_cell(h, 1) for h in (1, 2, 3)] == [3, 4, None]


def matrix_messages(batch, doc, rng):
    """Rebuild a generated matrix's messages (tests only); set-cell values are seeded JSON."""
    dd = batch.docs[doc]
    ops = batch.ops[int(dd["op_begin"]): int(dd["op_begin"]) + int(dd["op_count"])]
    names = ["observer"] + [f"client-{k}" for k in range(1, int(dd["n_clients"]))]
    msgs, group, observer = [], [], None
    for op in ops:
        t = int(op["type"])
        m = dict(seq=int(op["seq"]), ref=int(op["ref_seq"]), client=names[int(op["client"])], msn=int(op["min_seq"]))
        if t == abi.OP_START_COLLAB:
            observer = names[int(op["client"])]
            continue
        if t == abi.OP_SETCELL:
            v = [int(rng.integers(100)), "s%d" % rng.integers(10), {"k": [1, None, "z"]}, None][int(rng.integers(4))]
            msgs.append(_msg(m["seq"], m["ref"], m["client"],
                             {"type": 2, "row": int(op["pos1"]), "col": int(op["pos2"]), "value": v}, m["msn"]))
            continue
        target = "cols" if op["flags"] & abi.F_COLS else "rows"
        if t == abi.OP_INSERT:
            group.append({"pos1": int(op["pos1"]), "seg": [int(op["payload2"]), -1], "type": 0})
        elif t == abi.OP_REMOVE:
            group.append({"pos1": int(op["pos1"]), "pos2": int(op["pos2"]), "type": 1})
        else:
            raise AssertionError(t)
        if op["flags"] & abi.F_LAST:
            c = group[0] if len(group) == 1 else {"ops": group, "type": 3}
            c = dict(c, target=target) if len(group) == 1 else {"target": target, **c}
            msgs.append(_msg(m["seq"], m["ref"], m["client"], c, m["msn"]))
            group = []
    return observer, msgs


def _oracle_cells(observer, msgs, chunk):
    it = Interner()
    log = CellMatrixLog()
    log.start_collab(observer)
    o = OracleDoc(options(), matrix=True)
    for k in range(0, len(msgs), chunk):
        for m in msgs[k:k + chunk]:
            log.message(m, it)
        b = build_batch([log], it)
        assert o.apply(b, 0) == 0
        log.resolve(o.select(0).deltas(), o.select(1).deltas())
    return log, o, b


@pytest.mark.parametrize("writers,lag", [(8, 16), (16, 64)])
def test_cells_track_handle_recycling(writers, lag):
    """Seeded C4-mix matrices: the cell store never holds a value at a freed handle, every live
    cell's handles are owned by segments, and the oracle's records replayed in one batch or in
    chunks give the same cells blob."""
    cfg = matrix_cfg(4, 1500, writers=writers, max_lag=lag)
    tabs = tables(writers=writers)
    gb, _, status = generate_matrix(cfg, tabs, 0, 4, threads=4)
    assert (status == 0).all()
    n_recycled = 0
    for d in range(4):
        observer, msgs = matrix_messages(gb, d, np.random.default_rng(d))
        whole, o, b = _oracle_cells(observer, msgs, len(msgs))
        parts, _, _ = _oracle_cells(observer, msgs, 211)
        assert whole.cells_blob() == parts.cells_blob()
        owned = []
        for w in (0, 1):
            ex, _ = o.select(w).export()
            owned.append({h for r in ex if r[6] >= 1 for h in range(int(r[6]), int(r[6]) + int(r[0]))})
        root = whole.cells.snapshot()
        for k0, l1 in enumerate(root[0]):
            for k1, l2 in enumerate(l1 or []):
                for k2, l3 in enumerate(l2 or []):
                    for k3, v in enumerate(l3 or []):
                        if v is None:
                            continue
                        key = (k0 << 24) | (k1 << 16) | (k2 << 8) | k3
                        row = sum(((key >> (2 * i + 1)) & 1) << i for i in range(16))
                        col = sum(((key >> (2 * i)) & 1) << i for i in range(16))
                        assert row in owned[0] and col in owned[1]
        n_recycled += whole.cells_blob().count(b"null")
    assert n_recycled > 0


@pytest.mark.gpu
def test_matrix_cell_records_match_oracle():
    """Cell tracking on the device: per vector, the engine's MTR_DELTA_CELL / MTR_DELTA_RECYCLE records
    equal the oracle's, and the cells blobs the two drive are byte-identical."""
    from fluidframework_amd.batch import matrix_logs
    from fluidframework_amd.engine import Engine

    n, nops = 32, 2000
    cfg = matrix_cfg(n, nops, writers=8, max_lag=16)
    tabs = tables(writers=8)
    gb, _, status = generate_matrix(cfg, tabs, 0, n, threads=8)
    assert (status == 0).all()
    feeds = [matrix_messages(gb, m, np.random.default_rng(m)) for m in range(n)]
    eng = Engine(2 * n, max_segments=2 * nops + 128, heap_entries=2 * nops + 128, text_units=1 << 15,
                 prop_words=1024, remover_cells=4096, ops_per_launch=64)
    for m in range(n):
        eng.set_matrix(2 * m, 2 * m + 1)
    it = Interner()
    logs = []
    for observer, _ in feeds:
        lg = CellMatrixLog()
        lg.start_collab(observer)
        logs.append(lg)
    chunk = 617
    for k in range(0, max(len(f[1]) for f in feeds), chunk):
        for lg, (_, msgs) in zip(logs, feeds):
            for msg in msgs[k:k + chunk]:
                lg.message(msg, it)
        cols = [lg.cols_log() for lg in logs]
        b = build_batch([x for pair in zip(logs, cols) for x in pair], it)
        eng.apply(b)
        for m, lg in enumerate(logs):
            assert eng.status(2 * m)[0] == 0 and eng.status(2 * m + 1)[0] == 0
            lg.resolve(eng.deltas(2 * m), eng.deltas(2 * m + 1))
    eng.summarize()
    from fluidframework_amd.cells import matrix_summary
    for m, (observer, msgs) in enumerate(feeds):
        ref, o, rb = _oracle_cells(observer, msgs, chunk)
        assert logs[m].cells_blob() == ref.cells_blob(), f"matrix {m}: cells blob differs"
        tree = matrix_summary(eng, 2 * m, 2 * m + 1, logs[m])
        for w, name in ((0, "rows"), (1, "cols")):
            blobs = o.select(w).summarize(rb, 0)
            assert list(tree[name]["segments"].values()) + [tree[name]["handleTable"]] == blobs


# ---------------------------------------------------------------- load from a summary (f3)
def _vector_tree(blobs):
    """PermutationVector.summarize's tree from [segment blobs..., handleTable] (permutationvector.ts:310-325)."""
    return {"segments": {("header" if i == 0 else f"body_{i - 1}"): b for i, b in enumerate(blobs[:-1])},
            "handleTable": blobs[-1]}


def _oracle_matrix_tree(log, o, b):
    return {"rows": _vector_tree(o.select(0).summarize(b, 0)), "cols": _vector_tree(o.select(1).summarize(b, 0)),
            "cells": log.cells_blob()}


def _oracle_continue(tree, loader, msgs, chunk):
    """SharedMatrix.load from `tree` (the oracle), then the remaining messages in chunks."""
    it = Interner()
    lg = CellMatrixLog()
    lg.load_summary(tree, loader, it)
    o = OracleDoc(options(), matrix=True)
    b = build_batch([lg], it)
    assert o.apply(b, 0) == 0
    lg.resolve(o.select(0).deltas(), o.select(1).deltas())
    first = _oracle_matrix_tree(lg, o, b)
    for k in range(0, len(msgs), chunk):
        for m in msgs[k:k + chunk]:
            lg.message(m, it)
        b = build_batch([lg], it)
        assert o.apply(b, 0) == 0
        lg.resolve(o.select(0).deltas(), o.select(1).deltas())
    return first, _oracle_matrix_tree(lg, o, b)


@pytest.mark.parametrize("writers,lag", [(8, 16), (16, 64)])
def test_matrix_load_round_trip_oracle(writers, lag):
    """summarize -> load -> summarize is the identity (vectors' segments and handle tables, cells), and
    replay continues from the loaded matrix (C4-mix documents, split at a third)."""
    cfg = matrix_cfg(4, 1500, writers=writers, max_lag=lag)
    gb, _, status = generate_matrix(cfg, tables(writers=writers), 0, 4, threads=4)
    assert (status == 0).all()
    for d in range(4):
        observer, msgs = matrix_messages(gb, d, np.random.default_rng(d))
        cut = len(msgs) // 3
        log, o, b = _oracle_cells(observer, msgs[:cut], 211)
        tree = _oracle_matrix_tree(log, o, b)
        first, _ = _oracle_continue(tree, "loader", msgs[cut:], 173)
        assert first == tree


@pytest.mark.gpu
def test_matrix_load_round_trip_engine_matches_oracle():
    """Engine: summarize -> load -> continue for C4-mix matrices; the vectors' summaries and the cells
    blob equal the oracle doing the same from the same summary."""
    from fluidframework_amd.cells import matrix_summary
    from fluidframework_amd.engine import Engine

    n, nops = 8, 1800
    cfg = matrix_cfg(n, nops, writers=8, max_lag=32)
    gb, _, status = generate_matrix(cfg, tables(writers=8), 0, n, threads=8)
    assert (status == 0).all()
    feeds = [matrix_messages(gb, m, np.random.default_rng(m)) for m in range(n)]

    eng = Engine(2 * n, max_segments=2 * nops + 128, heap_entries=2 * nops + 128, text_units=1 << 15,
                 prop_words=1024, remover_cells=4096, ops_per_launch=64)
    eng2 = Engine(2 * n, max_segments=2 * nops + 128, heap_entries=2 * nops + 128, text_units=1 << 15,
                  prop_words=1024, remover_cells=4096, ops_per_launch=64)
    for m in range(n):
        eng.set_matrix(2 * m, 2 * m + 1)
        eng2.set_matrix(2 * m, 2 * m + 1)
    cuts = [len(f[1]) // 2 for f in feeds]
    # first half on the engine
    it = Interner()
    logs = []
    for observer, _ in feeds:
        lg = CellMatrixLog()
        lg.start_collab(observer)
        logs.append(lg)
    for k in range(0, max(cuts), 257):
        for lg, (_, msgs), c in zip(logs, feeds, cuts):
            for msg in msgs[k:min(k + 257, c)]:
                lg.message(msg, it)
        eng.apply(build_batch([x for lg in logs for x in (lg, lg.cols_log())], it))
        for m, lg in enumerate(logs):
            lg.resolve(eng.deltas(2 * m), eng.deltas(2 * m + 1))
    eng.summarize()
    trees = [matrix_summary(eng, 2 * m, 2 * m + 1, logs[m]) for m in range(n)]
    # load into a second engine and continue
    it2 = Interner()
    logs2 = []
    for m in range(n):
        lg = CellMatrixLog()
        lg.load_summary(trees[m], "loader-%d" % m, it2)
        logs2.append(lg)
    rest = [f[1][c:] for f, c in zip(feeds, cuts)]

    def apply2():
        eng2.apply(build_batch([x for lg in logs2 for x in (lg, lg.cols_log())], it2))
        for m, lg in enumerate(logs2):
            assert eng2.status(2 * m)[0] == 0 and eng2.status(2 * m + 1)[0] == 0
            lg.resolve(eng2.deltas(2 * m), eng2.deltas(2 * m + 1))

    apply2()  # the load alone: summarize reproduces the loaded tree
    eng2.summarize()
    for m in range(n):
        assert matrix_summary(eng2, 2 * m, 2 * m + 1, logs2[m]) == trees[m]
    for k in range(0, max(len(r) for r in rest), 311):
        for lg, r in zip(logs2, rest):
            for msg in r[k:k + 311]:
                lg.message(msg, it2)
        apply2()
    eng2.summarize()
    for m in range(n):
        got = matrix_summary(eng2, 2 * m, 2 * m + 1, logs2[m])
        _, exp = _oracle_continue(trees[m], "loader-%d" % m, rest[m], 311)
        assert got == exp, f"matrix {m}: round trip differs from the oracle"
