"""Legacy-summary catch-up ops: SharedSegmentSequence.processMergeTreeMsg /
createOpsFromDelta (packages/dds/sequence/src/sequence.ts:120-173, 675-748) over the engine's delta
ranges (include/mtr.h mtr_get_deltas).

The reference holds no summary fixture with a ``catchupOps`` blob (its legacyWithCatchUp snapshots are
written by a detached, non-collaborating SharedString, sequence/src/test/generateSharedStrings.ts),
so this path is pinned by hand-derived known answers from the reference code and by a
size-independent property: summarize -> load the summary (catch-up ops applied as messages) ->
summarize again gives byte-identical blobs and the same text.  The oracle's delta ranges are the
checker for the engine's, range by range.
"""
from __future__ import annotations

import json

import numpy as np
import pytest

from fluidframework_amd import abi
from fluidframework_amd.batch import Interner, build_batch
from fluidframework_amd.sequence import CATCHUP_BLOB, SequenceLog, match_properties, ops_from_deltas
from fluidframework_amd.synth import make_cfg, tables
from oracle.oracle import OracleDoc, generate, options

LEGACY = dict(snapshot_v1=False)


def _msg(seq, ref, client, contents, msn=0):
    return {"type": "op", "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "clientId": client, "contents": contents}


def test_match_properties_js_semantics():
    """properties.ts:71-105 with JavaScript truthiness: a top-level null matches 0 / "" / false
    (both take the `typeof b[key] === "object"` branch and recurse into falsy values)."""
    assert match_properties({"a": 1}, {"a": 1})
    assert not match_properties({"a": 1}, {"a": 2})
    assert not match_properties({"a": 1}, {"a": 1, "b": 2})
    assert match_properties({"a": None}, {"a": None})
    assert match_properties({"a": 0}, {"a": None})
    assert match_properties({"a": ""}, {"a": None})
    assert not match_properties({"a": 1}, {"a": None})
    assert not match_properties({"a": True}, {"a": 1})
    assert match_properties({"a": [1, 2]}, {"a": {"0": 1, "1": 2}})
    assert not match_properties(None, {"a": 1})
    assert match_properties(None, None)


def _kat():
    it = Interner()
    log = SequenceLog(legacy=True)
    log.start_collab("observer")
    msgs = [
        _msg(1, 0, "A", {"pos1": 0, "seg": "hello", "type": 0}),
        _msg(2, 1, "A", {"pos1": 0, "seg": "abc", "type": 0}),                           # abchello
        _msg(3, 1, "B", {"pos1": 2, "seg": {"text": "XY", "props": {"k": None, "b": 1}}, "type": 0}),
        _msg(4, 2, "D", {"pos1": 1, "pos2": 4, "props": {"bold": True, "1": "x"}, "type": 2}),
        _msg(5, 1, "C", {"pos1": 0, "pos2": 5, "type": 1}),
        _msg(6, 5, "A", {"pos1": 0, "seg": {"marker": {"refType": 1}, "props": {"m": 2}}, "type": 0}),
    ]
    for m in msgs:
        log.message(m, it)
    return log, it, msgs


def test_known_answer_transformed_messages():
    """Hand-derived from sequence.ts:120-173 and the merge-tree's concurrent-edit rules.

    seq 3 (B at ref 1 sees "hello") inserts XY at 2 -> local position 5 ("abc" + "he");
    seq 4 (D at ref 2 sees "abchello") annotates "bch": ranges "bc" (1, 2) and "h" (3, 1) merge;
    seq 5 (C at ref 1 sees "hello") removes h | e | llo: positions 3, 3, 5 after the removal (removed
    text counts 0), so h and e merge (same pos1) and llo starts a second remove -> a group op."""
    log, it, msgs = _kat()
    b = build_batch([log], it)
    o = OracleDoc(options(**LEGACY))
    assert o.apply(b, 0) == 0
    d = o.deltas()
    assert [tuple(int(x) for x in r) for r in d] == [
        (3, 5, 2, abi.OP_INSERT),
        (4, 1, 2, abi.OP_ANNOTATE), (4, 3, 1, abi.OP_ANNOTATE),
        (5, 3, 1, abi.OP_REMOVE), (5, 3, 1, abi.OP_REMOVE), (5, 5, 3, abi.OP_REMOVE),
    ]
    log.resolve(d)
    blob = log.catchup_blob()
    got = json.loads(blob)
    assert [m["referenceSequenceNumber"] for m in got] == [0, 1, 2, 3, 4, 5]
    assert got[0]["contents"] == msgs[0]["contents"] and got[5]["contents"] == msgs[5]["contents"]
    assert got[2]["contents"] == {"pos1": 5, "seg": {"text": "XY", "props": {"b": 1}}, "type": 0}
    assert got[3]["contents"] == {"pos1": 1, "pos2": 4, "props": {"1": "x", "bold": True}, "type": 2}
    assert got[4]["contents"] == {"ops": [{"pos1": 3, "pos2": 5, "type": 1}, {"pos1": 5, "pos2": 8, "type": 1}],
                                  "type": 3}
    # byte layout: JSON.stringify key order (message keys kept, props index keys first)
    assert b'"contents":{"pos1":1,"pos2":4,"props":{"1":"x","bold":true},"type":2}' in blob
    assert blob.startswith(b'[{"type":"op","sequenceNumber":1,"referenceSequenceNumber":0,"minimumSequenceNumber":0')


def test_stash_gc_and_summarize_trim():
    """GC once more than 20 messages are kept and the 21st is below the MSN (sequence.ts:728-734);
    summarize drops seq <= minSeq and overwrites every kept message's MSN (sequence.ts:681-687)."""
    it = Interner()
    log = SequenceLog(legacy=True)
    log.start_collab("observer")
    for s in range(1, 23):
        log.message(_msg(s, s - 1, "A", {"pos1": 0, "seg": "a", "type": 0}, msn=max(0, s - 2)), it)
    # at s = 22: len 22 > 20 and stash[20].seq = 21 < msn 20? no -> kept
    assert len(log.stash) == 22
    log.message(_msg(23, 22, "A", {"pos1": 0, "seg": "a", "type": 0}, msn=22), it)
    # stash[20].seq = 21 < 22 -> drop seq <= 22
    assert [m["sequenceNumber"] for m in log.stash] == [23]
    log.message(_msg(24, 23, "A", {"pos1": 0, "seg": "a", "type": 0}, msn=22), it)
    out = json.loads(log.catchup_blob(23))
    assert [(m["sequenceNumber"], m["minimumSequenceNumber"]) for m in out] == [(24, 23)]
    assert log.catchup_blob(24) is None


def test_v1_format_keeps_nothing():
    it = Interner()
    log = SequenceLog(legacy=False)
    log.start_collab("observer")
    log.message(_msg(1, 0, "A", {"pos1": 0, "seg": "a", "type": 0}), it)
    log.message(_msg(2, 0, "B", {"pos1": 0, "seg": "b", "type": 0}), it)
    assert not any(op[1] & abi.F_DELTA for op in log.ops)
    assert log.catchup_blob() is None


def test_remove_merging_into_an_insert_asserts():
    """lastRem.pos1 === r.position with an insert op before it: the reference asserts (0x3ff)."""
    from fluidframework_amd.batch import Unsupported
    ranges = np.array([(0, 2, 1, abi.OP_INSERT), (1, 2, 1, abi.OP_REMOVE)], dtype=abi.DELTA_DTYPE)
    members = [{"pos1": 2, "seg": "x", "type": 0}, {"pos1": 0, "pos2": 1, "type": 1}]
    with pytest.raises(Unsupported):
        ops_from_deltas(members, ranges, [0, 1])


# ---------------------------------------------------------------- synthetic round trips

def messages_from_batch(batch, doc):
    """Rebuild the ISequencedDocumentMessages of one generated document (tests only)."""
    dd = batch.docs[doc]
    ops = batch.ops[int(dd["op_begin"]): int(dd["op_begin"]) + int(dd["op_count"])]
    co, cb = batch.client_off, batch.client_bytes
    base = int(dd["client_base"])
    names = [json.loads('"' + bytes(cb[co[base + i]: co[base + i + 1]]).decode() + '"')
             for i in range(int(dd["n_clients"]))]
    text = batch.text[int(dd["text_base"]): int(dd["text_base"]) + int(dd["text_count"])]

    def props(pp):
        out = {}
        for j in range(int(batch.propop_off[pp]), int(batch.propop_off[pp + 1])):
            k, v = int(batch.propop_kv[2 * j]), int(batch.propop_kv[2 * j + 1])
            key = json.loads('"' + bytes(batch.key_bytes[batch.key_off[k]: batch.key_off[k + 1]]).decode() + '"')
            out[key] = None if v == abi.NULL_VALUE else json.loads(
                bytes(batch.val_bytes[batch.val_off[v]: batch.val_off[v + 1]]).decode())
        return out

    observer, msgs, group = None, [], []
    for op in ops:
        t = int(op["type"])
        if t == abi.OP_START_COLLAB:
            observer = names[int(op["client"])]
            continue
        if t == abi.OP_INSERT:
            s = bytes(text[int(op["payload"]): int(op["payload"]) + int(op["payload2"])]).decode("utf-16-le",
                                                                                             "surrogatepass")
            c = {"pos1": int(op["pos1"]), "seg": s, "type": 0}
        elif t == abi.OP_REMOVE:
            c = {"pos1": int(op["pos1"]), "pos2": int(op["pos2"]), "type": 1}
        elif t == abi.OP_ANNOTATE:
            c = {"pos1": int(op["pos1"]), "pos2": int(op["pos2"]), "props": props(int(op["payload"])), "type": 2}
        else:
            raise AssertionError(f"op type {t}")
        group.append(c)
        if op["flags"] & abi.F_LAST:
            contents = group[0] if len(group) == 1 else {"ops": group, "type": 3}
            msgs.append(_msg(int(op["seq"]), int(op["ref_seq"]), names[int(op["client"])], contents,
                             msn=int(op["min_seq"])))
            group = []
    return observer, msgs


class OracleReplica:
    """A SequenceLog driven by the oracle (the CPU checker of the engine-driven mirror)."""

    def __init__(self):
        self.it = Interner()
        self.log = SequenceLog(legacy=True)
        self.doc = OracleDoc(options(**LEGACY))
        self.last = None

    def flush(self):
        b = build_batch([self.log], self.it)
        assert self.doc.apply(b, 0) == 0
        self.log.resolve(self.doc.deltas())
        self.last = b

    def summary(self):
        blobs = self.doc.summarize(self.last, 0)
        cu = self.log.catchup_blob()
        return blobs + ([cu] if cu is not None else [])


def _named(blobs):
    """Legacy summary blob list -> the storage view SnapshotLoader reads (header, body..., catch-up)."""
    head = json.loads(blobs[0])
    out = {"header": blobs[0].decode()}
    rest = blobs[1:]
    names = ["body"] if head.get("chunkLengthChars", 0) < head.get("totalLengthChars", 0) else []
    for n, b in zip(names, rest):
        out[n] = b.decode()
    if len(rest) > len(names):
        out[CATCHUP_BLOB] = rest[-1].decode()
    return out


def _reload(blobs):
    r = OracleReplica()
    r.log.load(_named(blobs), "observer-2", r.it)
    r.flush()
    return r


@pytest.mark.parametrize("writers,lag", [(4, 8), (8, 32)])
def test_summarize_load_summarize_round_trip(writers, lag):
    """Loading a legacy summary and applying its catch-up ops reproduces the text and the catch-up
    blob; a second round trip is byte-stable.  The first reload's header/body can differ from the
    original where a catch-up annotate covered concurrently removed text (see
    test_annotate_over_removed_text_extends_the_catchup_op): that is the reference's behaviour."""
    cfg = make_cfg(8, 800, writers=writers, max_lag=lag)
    tabs = tables(writers=writers)
    gb, _, status = generate(cfg, tabs, 0, 8, threads=4, opts=options(**LEGACY))
    assert (status == 0).all()
    n_cu = same = 0
    for d in range(8):
        observer, msgs = messages_from_batch(gb, d)
        a = OracleReplica()
        a.log.start_collab(observer)
        for k in range(0, len(msgs), 97):
            for m in msgs[k:k + 97]:
                a.log.message(m, a.it)
            a.flush()
        s1 = a.summary()
        assert s1[-1].startswith(b'[{"type":"op"')
        n_cu += len(json.loads(s1[-1]))
        r1 = _reload(s1)
        assert r1.doc.text() == a.doc.text()
        s2 = r1.summary()
        assert s2[-1] == s1[-1]
        same += s2 == s1
        r2 = _reload(s2)
        assert r2.doc.text() == a.doc.text() and r2.summary() == s2
    assert n_cu > 0 and same >= 4


def test_annotate_over_removed_text_extends_the_catchup_op():
    """createOpsFromDelta advances pos2 by the cachedLength of every annotated segment, including one
    a concurrent op already removed (position counts it 0): C at ref 1 annotates "hell" after B's
    "el" removal, ranges h (0, 1), el (1, 2), l (1, 1) -> ops [0, 3) and [1, 2) (sequence.ts:127-146)."""
    it = Interner()
    log = SequenceLog(legacy=True)
    log.start_collab("observer")
    log.message(_msg(1, 0, "A", {"pos1": 0, "seg": "hello", "type": 0}), it)
    log.message(_msg(2, 1, "B", {"pos1": 1, "pos2": 3, "type": 1}), it)
    log.message(_msg(3, 1, "C", {"pos1": 0, "pos2": 4, "props": {"b": 1}, "type": 2}), it)
    b = build_batch([log], it)
    o = OracleDoc(options(**LEGACY))
    assert o.apply(b, 0) == 0
    d = o.deltas()
    assert [tuple(int(x) for x in r) for r in d] == [
        (3, 0, 1, abi.OP_ANNOTATE), (3, 1, 2, abi.OP_ANNOTATE), (3, 1, 1, abi.OP_ANNOTATE)]
    log.resolve(d)
    got = json.loads(log.catchup_blob())
    assert got[2]["contents"] == {"ops": [{"pos1": 0, "pos2": 3, "props": {"b": 1}, "type": 2},
                                          {"pos1": 1, "pos2": 2, "props": {"b": 1}, "type": 2}], "type": 3}


@pytest.mark.gpu
@pytest.mark.parametrize("writers,lag,ops", [(8, 32, 1500), (16, 64, 1200)])
def test_engine_deltas_match_oracle(writers, lag, ops):
    """Every op flagged MTR_F_DELTA: the engine's ranges equal the oracle's, record by record, and
    the documents end in the same state as unflagged."""
    from fluidframework_amd.engine import Engine, caps_for
    from oracle.oracle import summary_digest

    n = 64
    cfg = make_cfg(n, ops, writers=writers, max_lag=lag)
    tabs = tables(writers=writers)
    gb, hashes, status = generate(cfg, tabs, 0, n, threads=8)
    assert (status == 0).all()
    flagged = gb.ops.copy()
    kinds = np.isin(flagged["type"], [abi.OP_INSERT, abi.OP_REMOVE, abi.OP_ANNOTATE])
    flagged["flags"][kinds] |= abi.F_DELTA
    from fluidframework_amd.synth import with_docs
    b = with_docs(tabs, gb.docs, flagged, gb.text)
    eng = Engine(n, ops_per_launch=24, **caps_for(b))
    eng.apply(b)
    eng.summarize()
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
        o = OracleDoc(options())
        assert o.apply(b, d) == 0
        od, ed = o.deltas(), eng.deltas(d)
        assert len(ed) == len(od) and np.array_equal(ed, od), f"doc {d}: delta ranges differ"
        assert summary_digest(eng.summary(d)) == int(hashes[d])


@pytest.mark.gpu
def test_engine_catchup_round_trip():
    """The engine-driven mirror writes the same catch-up blob as the oracle-driven one, and the
    summarize -> load -> summarize round trip holds on the device."""
    from fluidframework_amd.engine import Engine

    cfg = make_cfg(8, 800, writers=8, max_lag=32)
    tabs = tables(writers=8)
    gb, _, status = generate(cfg, tabs, 0, 8, threads=8, opts=options(**LEGACY))
    assert (status == 0).all()
    eng = Engine(8, snapshot_v1=False, max_segments=4096, heap_entries=4096, text_units=1 << 15,
                 prop_words=1 << 14, remover_cells=2048, ops_per_launch=24)
    logs, refs, it = [], [], Interner()
    feeds = []
    for d in range(8):
        observer, msgs = messages_from_batch(gb, d)
        lg = SequenceLog(legacy=True)
        lg.start_collab(observer)
        logs.append(lg)
        feeds.append(msgs)
        r = OracleReplica()
        r.log.start_collab(observer)
        refs.append((r, msgs))
    for k in range(0, 800, 131):
        for d in range(8):
            for m in feeds[d][k:k + 131]:
                logs[d].message(m, it)
        b = build_batch(logs, it)
        eng.apply(b)
        for d in range(8):
            logs[d].resolve(eng.deltas(d))
    eng.summarize()
    for d in range(8):
        r, msgs = refs[d]
        for k in range(0, len(msgs), 131):
            for m in msgs[k:k + 131]:
                r.log.message(m, r.it)
            r.flush()
        cu = logs[d].catchup_blob()
        mine = eng.summary(d) + ([cu] if cu is not None else [])
        assert mine == r.summary(), f"doc {d}: legacy summary with catch-up differs"
    # load every summary into a fresh engine: same state as the oracle loading it, same text and
    # catch-up blob as the original
    eng2 = Engine(8, snapshot_v1=False, max_segments=4096, heap_entries=4096, text_units=1 << 15,
                  prop_words=1 << 14, remover_cells=2048, ops_per_launch=24)
    logs2, it2, full = [], Interner(), []
    for d in range(8):
        lg = SequenceLog(legacy=True)
        cu = logs[d].catchup_blob()
        full.append(eng.summary(d) + ([cu] if cu is not None else []))
        lg.load(_named(full[d]), "observer-2", it2)
        logs2.append(lg)
    b2 = build_batch(logs2, it2)
    eng2.apply(b2)
    eng2.summarize()
    for d in range(8):
        assert eng2.status(d)[0] == 0
        logs2[d].resolve(eng2.deltas(d))
        cu2 = logs2[d].catchup_blob()
        mine = eng2.summary(d) + ([cu2] if cu2 is not None else [])
        assert mine == _reload(full[d]).summary(), f"doc {d}: reloaded summary differs from the oracle's"
        assert cu2 == full[d][-1] and eng2.text(d) == eng.text(d)
