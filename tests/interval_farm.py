"""Shared by tests/test_intervals.py (CPU) and its -m gpu cases: the interval fixtures, a seeded farm of
sequenced messages that mixes merge-tree ops with interval collection ops from several writers at lagging
reference sequence numbers, and the product host (SequenceLog + fluidframework_amd.intervals) driven on
either executor (the CPU oracle's batch apply, or the HIP engine).

The farm steps a CPU-oracle observer (oracle/intervals.py, the reference's trees and slide listeners restated)
to draw every op at a position that is valid in its own view (getLength at its referenceSequenceNumber and
client), so the messages are ones a set of real clients could have sent.
"""
from __future__ import annotations

import json
import os
import random

from fixtures import GOLDEN, load_snapshots, snapshot_recipe
from fluidframework_amd.batch import Interner, build_batch
from fluidframework_amd.sequence import SequenceLog
from oracle.intervals import OracleString, js_parse

HEADERS = json.load(open(os.path.join(GOLDEN, "interval_headers.json")))
V2_HEADER = HEADERS["v1/withIntervals"]  # the three V2 headers are the same bytes
FIXTURES = ["legacy/withIntervals", "legacyWithCatchUp/withIntervals", "v1/withIntervals",
            "v1Intervals/withV1Intervals"]


def fixture_ids():
    """[(label, start, end, intervalType, intervalId)] of the generator's createIntervals calls
    (generateSharedStrings.ts:33-45), read back from the fixture (its uuids come from a seeded random-js)."""
    j = js_parse(V2_HEADER)
    return [(label, iv[0], iv[1], iv[3], iv[4]["intervalId"]) for label in j for iv in j[label]["value"]["intervals"]]


# ---------------------------------------------------------------- the product host on an executor
class HostString:
    """A SharedString observer on the product path: SequenceLog with interval collections; the merge-tree
    records run on `executor` ("oracle": the CPU oracle's batch apply -- a host-logic check; an Engine: the HIP
    path).  Everything goes into one batch; the interval header is ordered from the executor's reference states."""

    def __init__(self, executor="oracle"):
        self.log = SequenceLog(legacy=False)
        self.it = Interner()
        self.executor = executor

    def run(self):
        """-> (interval header bytes or None, content blobs, text)"""
        b = build_batch([self.log], self.it)
        if self.executor == "oracle":
            from oracle.oracle import OracleDoc, options

            doc = OracleDoc(options())
            rc = doc.apply(b, 0)
            assert rc == 0, f"oracle status {rc:#x}"
            states = doc.ref_states()
            content = doc.summarize(build_batch([self.log], self.it), 0)
            text = doc.text()
        else:
            eng = self.executor
            eng.apply(b)
            st, op = eng.status(0)
            assert st == 0, f"engine status {st:#x} at op {op}"
            states = eng.ref_states(0)
            eng.summarize()
            content = eng.summary(0)
            text = eng.text(0)
        return self.log.interval_header(states), content, text


def host_recipe(executor="oracle"):
    """generateSharedStrings.ts's withIntervals string on the product host: the local inserts of a detached
    string, then createIntervals (local adds, StayOnRemove endpoints)."""
    h = HostString(executor)
    for o in snapshot_recipe("withIntervals"):
        h.log.local_insert(o[1], o[2], h.it)
    for label, s, e, t, i in fixture_ids():
        h.log.interval_collection(label).local_add(h.log, s, e, t, {"intervalId": i})
    return h.run()


def host_load(name, executor="oracle"):
    h = HostString(executor)
    h.log.load(load_snapshots()[name], "loader", h.it, header=HEADERS[name])
    return h.run()


def oracle_recipe():
    s = OracleString()
    for o in snapshot_recipe("withIntervals"):
        s.log.local_insert(o[1], o[2], s.it)
    for label, st, e, t, i in fixture_ids():
        s.get(label).local_add(st, e, t, {"intervalId": i})
    return s


def oracle_load(name):
    s = OracleString()
    s.load({"header": HEADERS[name], "content": load_snapshots()[name]}, "loader")
    return s


# ---------------------------------------------------------------- the farm
WRITERS = ["writer-1", "writer-2", "writer-3"]
LABELS = ["comments", "7", "marks"]  # ("7" is an array index: JSON.stringify writes it first)


def farm(seed, n_msgs=160, initial="the quick brown fox jumps over the lazy dog", lag=6, p_interval=0.45):
    """-> (initial text, messages, the oracle observer after them)"""
    rng = random.Random(seed)
    obs = OracleString()
    obs.log.local_insert(0, initial, obs.it)
    obs.log.start_collab("observer")
    obs.flush()
    last_ref = {w: 0 for w in WRITERS}
    ids = {lab: [] for lab in LABELS}
    seq = 0
    msgs = []
    for i in range(n_msgs):
        w = rng.choice(WRITERS)
        ref = rng.randint(max(last_ref[w], seq - lag), seq)
        last_ref[w] = ref
        msn = min(last_ref.values())
        obs.flush()
        n = obs.doc.length(ref, obs.log.short_id(w))
        k = rng.random()
        if k < p_interval:
            lab = rng.choice(LABELS)
            kk = rng.random()
            if kk < 0.5 or not ids[lab]:
                s = rng.randint(0, max(n - 1, 0))
                e = min(n - 1, s + rng.randint(0, 6)) if rng.random() < 0.9 else n  # n: past the end (detached)
                props = {"intervalId": f"{w}:{i}", "referenceRangeLabels": [lab]}
                if rng.random() < 0.3:
                    props["color"] = rng.choice(["red", 3, 2.5, {"x": 1}])
                val = {"start": s, "end": e, "intervalType": rng.choice([2, 2, 2, 0, 1]),
                       "sequenceNumber": ref, "properties": props}
                if rng.random() < 0.05:  # an old client without ids: a legacy id (skip a repeat)
                    lid = f"legacy{s}-{e}"
                    if lid not in ids[lab]:
                        del props["intervalId"]
                        ids[lab].append(lid)
                    else:
                        ids[lab].append(props["intervalId"])
                else:
                    ids[lab].append(props["intervalId"])
                op = {"opName": "add", "value": val}
            elif kk < 0.8:
                iid = rng.choice(ids[lab])
                val = {"properties": {"intervalId": iid}, "sequenceNumber": ref, "intervalType": 2}
                r = rng.random()
                if r < 0.4:
                    val["start"] = rng.randint(0, max(n - 1, 0))
                if 0.25 < r < 0.7:
                    val["end"] = rng.randint(0, max(n - 1, 0))
                if r >= 0.6:
                    val["properties"]["color"] = rng.choice(["blue", None, 7])
                op = {"opName": "change", "value": val}
            else:
                op = {"opName": "delete", "value": {"properties": {"intervalId": rng.choice(ids[lab])},
                                                     "sequenceNumber": ref, "intervalType": 2}}
            contents = {"key": lab, "type": "act", "value": op}
        elif k < 0.75 or n < 12:
            contents = {"pos1": rng.randint(0, n), "seg": rng.choice(["ab", "xyz", "1", "long-ish text "]),
                        "type": 0}
        elif k < 0.92:
            a = rng.randint(0, n - 1)
            contents = {"pos1": a, "pos2": min(n, a + rng.randint(1, 6)), "type": 1}
        else:
            a = rng.randint(0, n - 1)
            contents = {"pos1": a, "pos2": min(n, a + rng.randint(1, 6)), "props": {"b": rng.choice([1, None])},
                        "type": 2}
        seq += 1
        m = {"clientId": w, "sequenceNumber": seq, "referenceSequenceNumber": ref,
             "minimumSequenceNumber": msn, "type": "op", "contents": contents}
        obs.message(dict(m))
        msgs.append(m)
    obs.flush()
    return initial, msgs, obs


def host_farm(initial, msgs, executor="oracle"):
    h = HostString(executor)
    h.log.local_insert(0, initial, h.it)
    h.log.start_collab("observer")
    for m in msgs:
        h.log.message(dict(m), h.it)
    return h.run()
