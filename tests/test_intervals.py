"""Interval collections (sequence/src/intervalCollection.ts:788 LocalIntervalCollection, :1428
IntervalCollection), pinned by the reference's own `header` blobs.

* The four withIntervals fixtures (sequence/src/test/snapshots/{legacy,legacyWithCatchUp,v1}/withIntervals.json
  and v1Intervals/withV1Intervals.json, the last in the V1 array format) hold the same 90 intervals: the
  oracle's restatement of the trees reproduces the V2 `header` bytes both from generateSharedStrings.ts's recipe
  (local inserts, then createIntervals' local adds) and by loading each fixture and summarizing it again
  (snapshotVersion.spec.ts loads every version; a V1 collection is written back in V2).
* The product host (fluidframework_amd/intervals.py: no trees, the order taken from the references' states when
  the summary is written) gives the same bytes; on CPU its references run on the oracle's batch apply (a check
  of the host logic), under -m gpu on the HIP engine.
* A seeded farm mixes merge-tree ops with interval add / change / delete ops of three writers at lagging
  reference sequence numbers (endpoints that slide, detach, tie): the product host's header, content blobs and
  text equal the oracle's, which re-inserts intervals from the references' slide callbacks as the reference does.
"""
import pytest

import interval_farm as F
from fluidframework_amd.batch import Unsupported
from fluidframework_amd.intervals import IntervalCollections, IntervalUnsupported
from oracle.intervals import RedBlackTree


def test_oracle_recipe_writes_the_fixture_header():
    assert F.oracle_recipe().summarize_header() == F.V2_HEADER


@pytest.mark.parametrize("name", F.FIXTURES)
def test_oracle_load_summarize_round_trip(name):
    s = F.oracle_load(name)
    assert s.summarize_header() == F.V2_HEADER
    assert len(s.text()) == 8890


def test_v1_fixture_is_the_v1_format_of_the_same_intervals():
    from oracle.intervals import js_parse

    v1, v2 = js_parse(F.HEADERS["v1Intervals/withV1Intervals"]), js_parse(F.V2_HEADER)
    assert list(v1) == list(v2) == ["collection1", "collection2"]
    for k in v1:
        assert [(x["start"], x["end"], x["properties"]["intervalId"]) for x in v1[k]["value"]] == \
               [(c[0], c[1], c[4]["intervalId"]) for c in v2[k]["value"]["intervals"]]


def test_host_recipe_writes_the_fixture_header():
    h, _, _ = F.host_recipe("oracle")
    assert h.decode() == F.V2_HEADER


@pytest.mark.parametrize("name", F.FIXTURES)
def test_host_load_summarize_round_trip(name):
    h, _, text = F.host_load(name, "oracle")
    assert h.decode() == F.V2_HEADER
    assert len(text) == 8890


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_interval_farm_host_equals_oracle(seed):
    init, msgs, obs = F.farm(seed)
    want_h, want_c, want_t = obs.summarize_header(), obs.summarize_content(), obs.text()
    got_h, got_c, got_t = F.host_farm(init, msgs, "oracle")
    assert got_t == want_t
    assert got_c == want_c
    assert got_h.decode() == want_h


def test_rbtree_restatement_orders_and_removes():
    """rbTree.ts's LLRB on integers: in-order keys sorted after puts and removes; a missing key's
    removeExisting dereferences an undefined child (the reference's TypeError)."""
    import random

    from oracle.intervals import ReferenceThrows

    rng = random.Random(5)
    t = RedBlackTree(lambda a, b: a - b)
    keys = set()
    for _ in range(400):
        k = rng.randint(0, 200)
        if rng.random() < 0.6:
            t.put(k, True)
            keys.add(k)
        elif k in keys:
            t.remove(k)
            keys.discard(k)
        assert t.keys() == sorted(keys)
    with pytest.raises(ReferenceThrows):
        t2 = RedBlackTree(lambda a, b: a - b)
        t2.put(1, True)
        t2.remove_existing(0)


def test_unsupported_paths_fall_back():
    """Local interval ops while collaborating, duplicate ids and transient intervals are reported as Unsupported
    (the document falls back), not approximated."""
    from fluidframework_amd.batch import DocLog

    log = DocLog()
    log.start_collab("me")
    ic = IntervalCollections()
    with pytest.raises(IntervalUnsupported):
        ic.local_add(log, "c", 0, 1, 2, {"intervalId": "a"})
    msg = {"clientId": "w", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
           "type": "op"}
    add = {"start": 0, "end": 0, "intervalType": 2, "properties": {"intervalId": "x"}}
    ic.process(log, {"key": "c", "type": "act", "value": {"opName": "add", "value": add}}, msg)
    with pytest.raises(IntervalUnsupported):
        ic.process(log, {"key": "c", "type": "act", "value": {"opName": "add", "value": dict(add)}}, msg)
    with pytest.raises(IntervalUnsupported):
        ic.process(log, {"key": "c", "type": "act", "value": {"opName": "add", "value": dict(add, intervalType=4)}},
                   msg)
    with pytest.raises(Unsupported):  # through DocLog.message
        log.message(dict(msg, contents={"key": "c", "type": "act", "value": {"opName": "nope", "value": {}}}), None)


@pytest.mark.gpu
def test_engine_recipe_and_loads_write_the_fixture_header():
    from fluidframework_amd.engine import Engine

    h, _, _ = F.host_recipe(Engine(1, ref_slots=4096))
    assert h.decode() == F.V2_HEADER
    for name in F.FIXTURES:
        h, content, text = F.host_load(name, Engine(1, ref_slots=4096))
        assert h.decode() == F.V2_HEADER, name
        assert len(text) == 8890


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6, 7, 8])
def test_interval_farm_engine_equals_oracle(seed):
    from fluidframework_amd.engine import Engine

    init, msgs, obs = F.farm(seed)
    want_h, want_c, want_t = obs.summarize_header(), obs.summarize_content(), obs.text()
    got_h, got_c, got_t = F.host_farm(init, msgs, Engine(1, ref_slots=4096))
    assert got_t == want_t
    assert got_c == want_c
    assert got_h.decode() == want_h
