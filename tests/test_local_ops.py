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
