"""Known answers of the reference's unit tests that need a live (writing) client, not an observer:

* client.rollback.spec.ts:318-360 -- "Should rollback delete and restore local references": references on two
  segments (Simple, SlideOnRemove, StayOnRemove), a local remove over both, its rollback: every reference is
  back in its segment's LocalReferenceCollection at its position;
* snapshot.spec.ts:170-184 -- "excludes un-acked segments": a writer with a pending local append summarizes
  (SnapshotV1); the summary loaded into a new client has no text, the writer keeps "0";
* snapshot.spec.ts:253-258 -- "includes segments submitted while detached": TestString("A", "starting text")
  is the writer itself (createClientsAtInitialState + startOrUpdateCollaboration), summary -> load -> text.

The oracle answers on CPU; under -m gpu the HIP engine replays each session and must give the oracle's answers
(reference positions and LocalReferenceCollection membership, texts, summary bytes).
"""
import pytest

from clients import Clients, ins, rem
from fixtures import blob_names
from fluidframework_amd import abi
from fluidframework_amd.batch import DocLog, build_batch
from oracle.oracle import OracleDoc, options

ME = "localUser"


def kat_rollback_restores_local_references():  # client.rollback.spec.ts:318-360
    # (beforeEach inserts an empty TextSegment before startOrUpdateCollaboration: it holds no position, and no
    # assert of the case reads the tree shape)
    s = Clients([ME])
    s.local(ME, ins(0, "efg"))
    s.local(ME, ins(0, "d"))
    s.local(ME, ins(0, "abc"))
    seg1 = s.containing(ME, 2)  # "abc"
    seg3 = s.containing(ME, 5)  # "efg"
    # createLocalReferencePosition(segment, offset, ...) = the segment's local position + offset
    ref1 = s.create_ref(ME, 2 - seg1[1] + 0, abi.REFTYPE_SIMPLE)
    ref_slide = s.create_ref(ME, 2 - seg1[1] + 2, abi.REFTYPE_SLIDE_ON_REMOVE)
    ref2 = s.create_ref(ME, 5 - seg3[1] + 1, abi.REFTYPE_SIMPLE)
    ref_stay = s.create_ref(ME, 5 - seg3[1] + 1, abi.REFTYPE_STAY_ON_REMOVE)
    op = s.local(ME, rem(0, 7))
    s.rollback(ME, op)
    assert s.text(ME) == "abcdefg"
    after1 = s.containing(ME, 2)
    after3 = s.containing(ME, 5)
    assert after1 is not None and after3 is not None
    for r, seg in ((ref1, after1), (ref_slide, after1), (ref2, after3), (ref_stay, after3)):
        leaf, _, _, held = s.ref_info(ME, r)
        assert leaf == seg[0] and held, f"reference {r}: segment {leaf}, held {held}"
    assert s.ref_positions(ME) == [0, 2, 5, 5]
    return s


def _summary_then_load(s, c):
    """SnapshotV1 of client c (oracle), then a new client loading it: (blobs, the loaded client's text)"""
    b = s.batches[-1]
    d = s.names.index(c)
    blobs = s.docs[c].summarize(b, d)
    log = DocLog()
    log.load_summary(dict(zip(blob_names(len(blobs), True), [x.decode() for x in blobs])), "loader", s.it)
    doc = OracleDoc(options())
    assert doc.apply(build_batch([log], s.it), 0) == 0
    return blobs, doc.text()


def kat_excludes_unacked_segments():  # snapshot.spec.ts:170-184
    s = Clients(["fakeId"], initial="")
    s.local("fakeId", ins(0, "0"))  # append("0", increaseMsn false): queued, not acked
    blobs, loaded = _summary_then_load(s, "fakeId")
    assert s.text("fakeId") == "0"
    assert loaded == ""
    return s, blobs


def kat_includes_detached_segments():  # snapshot.spec.ts:253-258
    s = Clients(["A"], initial="starting text")
    s.logs["A"].start_collab("A")  # TestString's second startOrUpdateCollaboration(id) (a no-op rename)
    s.flush()
    assert s.text("A") == "starting text"
    blobs, loaded = _summary_then_load(s, "A")
    assert loaded == "starting text"
    return s, blobs


def test_rollback_restores_local_references_oracle():
    kat_rollback_restores_local_references()


@pytest.mark.parametrize("kat", [kat_excludes_unacked_segments, kat_includes_detached_segments])
def test_local_snapshot_kat_oracle(kat):
    kat()


@pytest.mark.gpu
def test_rollback_restores_local_references_engine():
    kat_rollback_restores_local_references().replay_engine()


@pytest.mark.gpu
@pytest.mark.parametrize("kat", [kat_excludes_unacked_segments, kat_includes_detached_segments])
def test_local_snapshot_kat_engine(kat):
    s, blobs = kat()
    eng = s.replay_engine()
    eng.summarize()
    assert eng.summary(0) == blobs
