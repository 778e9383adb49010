"""The reference's container-runtime mocks restated for live SharedString clients (test infrastructure):
MockContainerRuntimeFactory / MockContainerRuntime (runtime/test-runtime-utils/src/mocks.ts:102-303) and their
reconnection variants (mocksForReconnection.ts:18-140), driving fluidframework_amd.live.SharedStringClient objects
on one executor -- the HIP engine (EngineExecutor) or the CPU oracle (OracleExecutor below, the checker).

* `submit` stamps clientSequenceNumber and referenceSequenceNumber = the runtime's last processed sequence number
  and queues the message at the factory (pushMessage records a new client's first referenceSequenceNumber in minSeq);
* `process_one` JSON-clones the oldest message, stores its referenceSequenceNumber as the sender's minSeq entry,
  stamps the next sequenceNumber and minimumSequenceNumber = min over minSeq (entries are never deleted), and hands it
  to every runtime (a disconnected one queues it);
* a reconnect processes the queued remote messages, takes a new client id, resubmits every pending message (the
  DDS regenerates / rebases it), then tells the DDS it is connected (startOrUpdateCollaboration: the rename).
"""
from __future__ import annotations

import itertools
import json

from fluidframework_amd.live import LiveSession

class OracleExecutor:
    """The CPU oracle as a live session's executor (one OracleDoc per client) -- the checker only."""

    def __init__(self, legacy: bool = False):
        from oracle.oracle import OracleDoc, options

        self._mk = lambda: OracleDoc(options(snapshot_v1=not legacy))
        self.docs: list = []

    def apply(self, batch) -> None:
        while len(self.docs) < batch.n_docs:
            self.docs.append(self._mk())
        for d in range(batch.n_docs):
            rc = self.docs[d].apply(batch, d)
            if rc != 0:
                raise RuntimeError(f"oracle document {d}: status {rc:#x}")

    def text(self, d):
        return self.docs[d].text()

    def ref_keys(self, d):
        return self.docs[d].ref_keys()

    def length(self, d, ref_seq, client):
        return int(self.docs[d].length(ref_seq, client))

    def deltas(self, d):
        return self.docs[d].deltas()

    def props(self, d, ref):
        return self.docs[d].regen_props(ref)

    def summary(self, batch, d):
        return self.docs[d].summarize(batch, d)


class Runtime:
    """MockContainerRuntime(ForReconnection) of one SharedString."""

    def __init__(self, factory: "Factory", name: str):
        self.factory = factory
        self.client_id = name
        self.csn = 0
        self.last_seq = 0
        self.pending: list[tuple] = []  # (contents, metadata, clientSequenceNumber)
        self.pending_remote: list[dict] = []
        self._connected = True
        self.dds = factory.session.client(name)
        self.dds.submit_fn = self.submit
        self.dds.connect(name)

    def submit(self, contents, metadata):
        if not self._connected:
            self.pending.append((contents, metadata, -1))
            return
        csn = self.csn
        self.csn += 1
        self.factory.push({"clientId": self.client_id, "clientSequenceNumber": csn, "contents": contents,
                           "referenceSequenceNumber": self.last_seq, "type": "op"})
        self.pending.append((contents, metadata, csn))

    def process(self, msg: dict) -> None:
        if not self._connected:
            self.pending_remote.append(msg)
            return
        self.last_seq = msg["sequenceNumber"]
        local = msg["clientId"] == self.client_id
        meta = None
        if local:
            contents, meta, csn = self.pending.pop(0)
            assert csn == msg["clientSequenceNumber"], "Unexpected client sequence number from message"
        self.dds.process(msg, local, meta)

    @property
    def connected(self) -> bool:
        return self._connected

    @connected.setter
    def connected(self, value: bool) -> None:
        if value == self._connected:
            return
        self._connected = value
        if value:
            for m in self.pending_remote:
                self.process(m)
            self.pending_remote = []
            self.csn = 0
            self.client_id = f"reconnected-{next(self.factory.ids)}"
            msgs, self.pending = self.pending, []
            for contents, meta, _ in msgs:
                self.dds.resubmit(contents, meta)
            self.dds.connect(self.client_id)
        else:
            self.factory.messages = [m for m in self.factory.messages if m["clientId"] != self.client_id]


class Factory:
    """MockContainerRuntimeFactory(ForReconnection): the sequencer."""

    def __init__(self, executor=None, legacy: bool = False):
        self.session = LiveSession(executor if executor is not None else OracleExecutor(legacy), legacy=legacy)
        self.seq = 0
        self.min_seq: dict[str, int] = {}
        self.messages: list[dict] = []
        self.runtimes: list[Runtime] = []
        self.ids = itertools.count(1)  # (per factory: two replays of one script name their clients alike)

    def runtime(self, name: str) -> Runtime:
        r = Runtime(self, name)
        self.runtimes.append(r)
        return r

    def push(self, msg: dict) -> None:
        if msg.get("clientId") and msg["clientId"] not in self.min_seq:
            self.min_seq[msg["clientId"]] = msg["referenceSequenceNumber"]
        self.messages.append(msg)

    @property
    def outstanding(self) -> int:
        return len(self.messages)

    def process_one(self) -> None:
        msg = json.loads(json.dumps(self.messages.pop(0)))
        self.min_seq[msg["clientId"]] = msg["referenceSequenceNumber"]
        self.seq += 1
        msg["sequenceNumber"] = self.seq
        msg["minimumSequenceNumber"] = min(self.min_seq.values()) if self.min_seq else 0
        for r in self.runtimes:
            r.process(msg)

    def process_all(self) -> None:
        while self.messages:
            self.process_one()


def positions(string, coll) -> list[tuple[int, int]]:
    """[(start, end)] of Array.from(collection), localReferencePositionToPosition of each endpoint."""
    keys = string.ref_keys()
    return [coll.positions(iv, keys) for iv in coll]


def assert_intervals(string, coll, expected, validate_overlapping: bool = True) -> None:
    """assertIntervals (intervalCollection.spec.ts:21-48)."""
    actual = list(coll)
    n = string.get_length()
    if validate_overlapping and n > 0:
        overlapping = coll.find_overlapping_intervals(0, n - 1)
        assert [id(x) for x in actual] == [id(x) for x in overlapping], "Interval search returned inconsistent results"
    got = positions(string, coll)
    assert got == [tuple(e) for e in expected], f"intervals are not as expected: {got} != {expected}"


def assert_consistent(runtimes) -> None:
    """assertConsistent (sequence/src/test/intervalUtils.ts:19-92): every connected client has the same text, the
    same collection labels and, per interval id, the same endpoint positions, intervalType and properties."""
    conn = [r for r in runtimes if r.connected]
    if len(conn) < 2:
        return
    first = conn[0].dds
    for other in (r.dds for r in conn[1:]):
        assert first.get_text() == other.get_text(), f"text {first.get_text()!r} != {other.get_text()!r}"
        la, lb = sorted(first.log.intervals.data), sorted(other.log.intervals.data)
        assert la == lb, f"labels {la} != {lb}"
        ka, kb = first.ref_keys(), other.ref_keys()
        for label in la:
            ca, cb = first.get_interval_collection(label), other.get_interval_collection(label)
            ia = list(ca)
            assert len(ia) == len(cb.coll.by_id), f"interval counts differ in {label}"
            for iv in ia:
                ov = cb.get_interval_by_id(iv.id())
                assert ov is not None, f"interval {iv.id()} missing"
                assert ca.positions(iv, ka) == cb.positions(ov, kb), (iv.id(), ca.positions(iv, ka), cb.positions(ov, kb))
                assert iv.itype == ov.itype
                assert iv.props == ov.props, (iv.props, ov.props)
