"""The local-op path: pending local inserts / removes / annotates and their acks.

Pinned by the reference's own replay test: client.replay.spec.ts:17-71 replays every committed log
(merge-tree/src/test/results) on *every* client -- each writer applies its own ops locally
(TestClient.localTransaction) as pending ops, catches up with the sequenced stream (its own messages
come back as acks, Client.applyMsg -> ackPendingSegment, client.ts:866-869) and must read the group's
resultText at the end of every group.  tests/fixtures.Perspective builds one writer's view; CPU: the
oracle, -m gpu: the HIP engine against the same expected texts and the oracle's leaves and summaries.
"""
import os

import pytest

from fixtures import Perspective, load_replay, original_summary, replay_files, replay_writers
from fluidframework_amd.batch import Interner, build_batch
from oracle.oracle import OracleDoc, options


@pytest.mark.parametrize("path", replay_files(), ids=lambda p: os.path.basename(p)[:-8])
def test_writer_perspectives_oracle(path):
    """Every writer of the log, group by group: the text after each group is resultText."""
    groups = load_replay(path)
    summary = original_summary(groups)
    it = Interner()
    views = [Perspective(w, summary, it) for w in replay_writers(groups)]
    docs = [OracleDoc(options()) for _ in views]
    for gi, g in enumerate(groups):
        for v in views:
            v.feed(g, it)
        b = build_batch([v.log for v in views], it)
        for d, (v, doc) in enumerate(zip(views, docs)):
            assert doc.apply(b, d) == 0, f"{v.writer} group {gi}"
            assert doc.text() == g["resultText"], f"{v.writer} group {gi}"


def _all_perspectives():
    """(file, groups, Perspective) for every writer of every log, with one shared Interner."""
    it = Interner()
    out = []
    for p in replay_files():
        groups = load_replay(p)
        summary = original_summary(groups)
        for w in replay_writers(groups):
            out.append((os.path.basename(p)[:-8], groups, Perspective(w, summary, it)))
    return it, out


@pytest.mark.gpu
@pytest.mark.parametrize("new_length", [False, True], ids=["oldlen", "newlen"])
def test_writer_perspectives_engine(new_length):
    """All writers of all 30 logs (110 documents) on one engine, one batch per group: the text after
    every group equals resultText, and at the end the leaves, tree levels and V1 summaries equal the
    oracle's.  (New length mode: engine vs oracle only -- the logs were recorded with the old mode.)"""
    import numpy as np

    from fluidframework_amd.engine import Engine

    it, views = _all_perspectives()
    eng = Engine(len(views), max_segments=8192, heap_entries=8192, text_units=1 << 18, prop_words=1 << 18,
                 remover_cells=1 << 14, ops_per_launch=64, new_length_calc=new_length)
    orcs = [OracleDoc(options(new_length_calc=new_length)) for _ in views]
    n_groups = max(len(g) for _, g, _ in views)
    b = None
    for gi in range(n_groups):
        # the first half of the group: mid-group states with pending local segments (the writer's
        # local view shows them) -- engine text vs the oracle's
        for _, groups, v in views:
            if gi < len(groups):
                v.feed(groups[gi], it, 0, len(groups[gi]["msgs"]) // 2, drain=False)
        b = build_batch([v.log for _, _, v in views], it)
        eng.apply(b)
        for d, (name, groups, v) in enumerate(views):
            assert orcs[d].apply(b, d) == 0, f"{name}/{v.writer} group {gi} half (oracle)"
            st, op = eng.status(d)
            assert st == 0, f"{name}/{v.writer} group {gi} half: status {st:#x} at op {op}"
            assert eng.text(d) == orcs[d].text(), f"{name}/{v.writer} group {gi} half"
        for _, groups, v in views:
            if gi < len(groups):
                v.feed(groups[gi], it, len(groups[gi]["msgs"]) // 2)
        b = build_batch([v.log for _, _, v in views], it)
        eng.apply(b)
        for d, (name, groups, v) in enumerate(views):
            assert orcs[d].apply(b, d) == 0, f"{name}/{v.writer} group {gi} (oracle)"
            st, op = eng.status(d)
            assert st == 0, f"{name}/{v.writer} group {gi}: status {st:#x} at op {op}"
            if gi < len(groups):
                want = groups[gi]["resultText"] if not new_length else orcs[d].text()
                assert eng.text(d) == want, f"{name}/{v.writer} group {gi}"
    for d, (name, _, v) in enumerate(views):
        ge, gh = eng.export(d)
        oe, oh = orcs[d].export()
        assert gh == oh and ge.shape == oe.shape, f"{name}/{v.writer}: tree shape"
        bad = np.nonzero((ge != oe).any(axis=1))[0]
        assert bad.size == 0, f"{name}/{v.writer}: leaf {bad[0]}: {ge[bad[0]].tolist()} vs {oe[bad[0]].tolist()}"
    eng.summarize()
    for d, (name, _, v) in enumerate(views):
        assert eng.summary(d) == orcs[d].summarize(b, d), f"{name}/{v.writer} summary"


@pytest.mark.gpu
def test_bulk_device_texts():
    """mtr_get_texts (one device gather for a document range) equals the per-document reads and the
    oracle's getText, for writers holding pending local segments mid-group."""
    from fluidframework_amd.engine import Engine

    it, views = _all_perspectives()
    views = views[:24]
    eng = Engine(len(views), max_segments=8192, heap_entries=8192, text_units=1 << 18, prop_words=1 << 18,
                 remover_cells=1 << 14, ops_per_launch=64)
    orcs = [OracleDoc(options()) for _ in views]
    for _, groups, v in views:
        v.feed(groups[0], it)
        v.feed(groups[1], it, 0, len(groups[1]["msgs"]) // 2, drain=False)
    b = build_batch([v.log for _, _, v in views], it)
    eng.apply(b)
    for d in range(len(views)):
        assert orcs[d].apply(b, d) == 0
    bulk = eng.texts(0, len(views))
    assert bulk == [eng.text(d) for d in range(len(views))]
    assert bulk == [o.text() for o in orcs]
    assert eng.texts(3, 3) == []
