"""Client.load from a summary (SnapshotLoader, snapshotLoader.ts:41-257; reloadFromSegments,
mergeTree.ts:678-728): pinned by the reference's snapshot fixtures (load -> summarize reproduces the
blob bytes, the round trips of snapshot.spec.ts / snapshotVersion.spec.ts), and by collaboration
round trips on the replay logs (summarize mid-stream, load, keep applying: text stays equal)."""
import os

import pytest

from fixtures import SNAPSHOT_VERSIONS, blob_names, load_replay, load_snapshots, replay_files, replay_log
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, options

SNAPS = load_snapshots()


def _load(blobs, v1, it=None):
    it = it or Interner()
    log = DocLog()
    catchup = log.load_summary(blobs, "snapshot", it)
    doc = OracleDoc(options(snapshot_v1=v1))
    assert doc.apply(build_batch([log], it), 0) == 0
    return doc, log, it, catchup


@pytest.mark.parametrize("key", sorted(SNAPS))
def test_load_then_summarize_reproduces_fixture(key):
    version, name = key.split("/")
    v1 = SNAPSHOT_VERSIONS[version]
    blobs = SNAPS[key]
    doc, log, it, _ = _load(blobs, v1)
    b = build_batch([log], it)
    got = doc.summarize(b, 0)
    assert dict(zip(blob_names(len(got), v1), got)) == {k: v.encode("utf-8") for k, v in blobs.items()}


@pytest.mark.parametrize("path", [p for p in replay_files() if "clients_8" in p][:5],
                         ids=lambda p: os.path.basename(p)[:-8])
def test_summarize_load_continue(path):
    """snapshot.spec.ts:156-258 style: summarize mid-collaboration, load into a new client, apply the
    remaining messages to both; the texts agree after every group."""
    groups = load_replay(path)
    cut = len(groups) // 2
    it = Interner()
    log_a = replay_log(groups, it)
    a = OracleDoc(options())
    for g in groups[:cut]:
        for m in g["msgs"]:
            log_a.message(m, it)
    last = groups[cut - 1]["msgs"][-1]
    log_a.seq_update(last["minimumSequenceNumber"], last["sequenceNumber"])
    assert a.apply(build_batch([log_a], it), 0) == 0
    blobs = a.summarize(build_batch([log_a], it), 0)
    named = dict(zip(blob_names(len(blobs), True), [x.decode("utf-8") for x in blobs]))
    b, log_b, _, _ = _load(named, True, it)
    assert b.text() == a.text() == groups[cut - 1]["resultText"]
    for g in groups[cut:]:
        for m in g["msgs"]:
            log_a.message(m, it)
            log_b.message(m, it)
        batch = build_batch([log_a, log_b], it)
        assert a.apply(batch, 0) == 0 and b.apply(batch, 1) == 0
        assert a.text() == b.text() == g["resultText"]
