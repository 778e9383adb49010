"""Fixture loaders shared by the oracle tests and the GPU parity tests.

* replay logs: tests/golden/replay/*.json.gz (converted by tests/golden/make_golden.py from
  packages/dds/merge-tree/src/test/results, replayed as in client.replay.spec.ts:17-71: observer "A"
  loads initialText non-collaboratively, starts collaboration, and applies every message as remote).
* snapshot fixtures: tests/golden/snapshots.json.gz with the recipes of
  packages/dds/sequence/src/test/generateSharedStrings.ts:42-147 restated below.
"""
from __future__ import annotations

import glob
import gzip
import json
import os

from fluidframework_amd.batch import DocLog, Interner

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SIZE_OF_FIRST_CHUNK = 10000  # SnapshotLegacy.sizeOfFirstChunk, snapshotlegacy.ts:51


def replay_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "replay", "*.json.gz")))


def load_replay(path):
    with gzip.open(path, "rt", encoding="utf-8") as fh:
        return json.load(fh)


def replay_log(groups, interner: Interner) -> DocLog:
    """DocLog primed like client.replay.spec.ts:26-36 (initial text + startOrUpdateCollaboration("A"))."""
    log = DocLog()
    if groups[0]["initialText"]:
        log.local_insert(0, groups[0]["initialText"], interner)
    log.start_collab("A")
    return log


def replay_writers(groups):
    """The authoring clients of a replay log, in first-message order."""
    seen = []
    for g in groups:
        for m in g["msgs"]:
            if m["clientId"] not in seen:
                seen.append(m["clientId"])
    return seen


def original_summary(groups):
    """client.replay.spec.ts:27-29's original client ("A": initialText inserted locally, then
    startOrUpdateCollaboration) as TestClient.createFromClientSnapshot summarizes it (SnapshotLegacy,
    test/testClient.ts:70-87): {blob name: text}.  Computed with the CPU oracle (test infrastructure);
    the legacy writer is pinned byte for byte by the snapshot fixtures."""
    from oracle.oracle import OracleDoc, options

    from fluidframework_amd.batch import build_batch

    it = Interner()
    log = replay_log(groups, it)
    b = build_batch([log], it)
    doc = OracleDoc(options(snapshot_v1=False))
    if doc.apply(b, 0) != 0:
        raise RuntimeError("original client failed to build")
    blobs = doc.summarize(b, 0)
    return {k: v.decode("utf-8") for k, v in zip(blob_names(len(blobs), False), blobs)}


class Perspective:
    """One writer client of client.replay.spec.ts:22-68 as its own document: created from the original
    client's snapshot under its long id (createFromClientSnapshot), it applies its own op locally
    (localTransaction -- a pending local op) right after catching up to the op's
    referenceSequenceNumber with the messages queued for it, and every sequenced message in order
    (its own become acks); at the end of a group it drains its queue and must read resultText."""

    def __init__(self, writer: str, summary: dict, interner: Interner):
        self.writer = writer
        self.log = DocLog()
        self.log.load_summary(summary, writer, interner)
        self.queue = []
        self.cur = 0

    def _apply(self, m, interner):
        self.log.message(m, interner)
        self.cur = int(m["sequenceNumber"])

    def feed(self, group, interner: Interner, lo: int = 0, hi: int | None = None, drain: bool = True) -> None:
        """Messages [lo, hi) of the group; drain = the group ends here (apply everything queued)."""
        for m in group["msgs"][lo:hi]:
            if m["clientId"] == self.writer:
                while self.queue and m["referenceSequenceNumber"] > self.cur:
                    self._apply(self.queue.pop(0), interner)
                self.log.local_op(m["contents"], interner)
            self.queue.append(m)
        while drain and self.queue:
            self._apply(self.queue.pop(0), interner)


def load_snapshots():
    with gzip.open(os.path.join(GOLDEN, "snapshots.json.gz"), "rt", encoding="utf-8") as fh:
        return json.load(fh)


# version -> snapshot_v1 option (generateSharedStrings.ts:23-30)
SNAPSHOT_VERSIONS = {"legacy": False, "legacyWithCatchUp": False, "v1": True, "v1Intervals": False}


def snapshot_recipe(name: str):
    """Local (non-collaborative) edits of one fixture; returns a list of tuples."""
    ins = "text"
    half = [("ins", 0, f"{ins}{i}") for i in range(int(SIZE_OF_FIRST_CHUNK / len(ins) / 2))]
    double = [("ins", 0, f"{ins}{i}") for i in range(int(SIZE_OF_FIRST_CHUNK / len(ins) * 2))]
    if name in ("headerOnly", "withIntervals", "withV1Intervals"):
        return half
    if name == "headerAndBody":
        return double
    if name == "largeBody":
        return [("ins", 0, f"{ins}-{i}") for i in range(SIZE_OF_FIRST_CHUNK)]
    if name == "withMarkers":
        ops = list(double)
        length = sum(len(o[2]) for o in ops)
        i = 0
        while i < length:  # getLength() grows by one per inserted marker
            props = {"ItemType": "Paragraph", "Properties": {"Bold": False}, "markerId": f"marker{i}",
                     "referenceTileLabels": ["Eop"]}
            ops.append(("marker", i, props))
            length += 1
            i += 70
        return ops
    if name == "withAnnotations":
        ops = list(double)
        length = sum(len(o[2]) for o in ops)
        ops += [("ann", i, i + 10, {"bold": True}) for i in range(0, length, 70)]
        return ops
    raise KeyError(name)


def snapshot_log(name: str, interner: Interner) -> DocLog:
    log = DocLog()
    for o in snapshot_recipe(name):
        if o[0] == "ins":
            log.local_insert(o[1], o[2], interner)
        elif o[0] == "marker":
            log.local_insert(o[1], {"marker": {"refType": 1}, "props": o[2]}, interner)  # ReferenceType.Tile
        else:
            log.local_annotate(o[1], o[2], o[3], interner)
    return log


def blob_names(n: int, v1: bool):
    if v1:
        return ["header"] + [f"body_{i}" for i in range(n - 1)]
    return ["header", "body"][:n]
