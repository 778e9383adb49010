"""Known answers of packages/dds/merge-tree/src/test/client.applyMsg.spec.ts that exercise the local-op
path: pending SegmentGroups and their acks, seq / removedSeq of the segments a local op
touched (UnassignedSequenceNumber until the sequenced message comes back), overlapping remote and local
removes, regenerating an annotate whose range was removed meanwhile, and getContainingSegment at an op's
(referenceSequenceNumber, clientId) view.  (The spec's multi-client conflict cases without local-op asserts are
observer streams in tests/test_kats.py.)

Every case runs on the oracle (CPU; each assert of the spec is asserted on the oracle's answer) and, under
-m gpu, is replayed batch by batch on the HIP engine, which must give the oracle's answer at every check.
"""
import pytest

from clients import NOT_REMOVED, UNASSIGNED, Clients, ann, ins, rem

ME = "localUser"


def _hello():
    """the spec's beforeEach (:19-27): insertTextLocal(0, "hello world") before startOrUpdateCollaboration"""
    return Clients([ME], initial="hello world")


def kat_interleaved():  # :29-121
    s = _hello()
    changes = []
    assert s.pending(ME) == 0
    for i in range(100):
        n = s.length(ME)
        p1 = n // 2
        m6 = i % 6
        if m6 in (0, 5):
            p2 = max((n - p1) // 4 - m6 + p1, p1 + 1)
            op = s.local(ME, rem(p1, p2))
        elif m6 in (1, 4):
            op = s.local(ME, ins(p1, str(i) * (m6 + 5)))
        else:
            p2 = max((n - p1) // 3 - m6 + p1, p1 + 1)
            op = s.local(ME, ann(p1, p2, {"foo": str(i)}))
        changes.append(s.make(ME, op, i + 1))
        assert s.pending(ME) == i + 1
    for i, m in enumerate(changes):
        s.apply(ME, m)
        assert s.pending(ME) == 99 - i
    assert s.pending(ME) == 0
    # every segment acked, none in a segment group (getContainingSegment at every position)
    for pos in range(s.length(ME)):
        leaf, _ = s.containing(ME, pos)
        assert s.leaf(ME, leaf)[1] != UNASSIGNED
        assert s.groups(ME, pos, ref=s.cur[ME], client=s.logs[ME].short_id(ME)) == 0
    return s


def kat_insert_text_local():  # :123-133
    s = _hello()
    op = s.local(ME, ins(0, "abc"))
    assert s.containing(ME, 0) == (0, 0)
    assert s.leaf(ME, 0)[1] == UNASSIGNED
    s.apply(ME, s.make(ME, op, 17))
    assert s.leaf(ME, 0)[1] == 17
    return s


def kat_remove_range_local():  # :135-145
    s = _hello()
    assert s.containing(ME, 0) == (0, 0)  # the "hello world" segment: its left part "h" stays at leaf 0
    op = s.local(ME, rem(0, 1))
    assert s.leaf(ME, 0)[3] == UNASSIGNED
    s.apply(ME, s.make(ME, op, 17))
    assert s.leaf(ME, 0)[3] == 17
    return s


def kat_annotate_local():  # :147-159
    s = _hello()
    op = s.local(ME, ann(0, 1, {"foo": "bar"}))
    assert s.pending(ME) == 1
    s.apply(ME, s.make(ME, op, 17))
    assert s.pending(ME) == 0
    return s


def kat_annotate_then_remove():  # :161-188
    s = _hello()
    assert s.containing(ME, 0) == (0, 0)
    end = s.length(ME)
    aop = s.local(ME, ann(0, end, {"foo": "bar"}))
    assert s.pending(ME) == 1
    rop = s.local(ME, rem(0, end))
    assert s.leaf(ME, 0)[3] == UNASSIGNED
    assert s.pending(ME) == 2
    s.apply(ME, s.make(ME, aop, 17))
    assert s.leaf(ME, 0)[3] == UNASSIGNED
    assert s.pending(ME) == 1
    s.apply(ME, s.make(ME, rop, 18))
    assert s.leaf(ME, 0)[3] == 18
    assert s.pending(ME) == 0
    return s


def kat_multiple_interleaved_annotates():  # :190-211
    s = _hello()
    end = s.length(ME)
    msgs = []
    seq = 0
    while end > 0:
        op = s.local(ME, ann(0, end, {"end": end, "foo": "bar"}))
        seq += 1
        msgs.append(s.make(ME, op, seq))
        end //= 2
    assert s.pending(ME) == len(msgs)
    for m in msgs:
        s.apply(ME, m)
    assert s.pending(ME) == 0
    return s


def kat_overlapping_deletes():  # :213-238
    s = _hello()
    assert s.containing(ME, 0) == (0, 0)
    initial = s.text(ME)
    assert s.leaf(ME, 0)[3] == NOT_REMOVED
    assert s.groups(ME, 0) == 0
    op = s.local(ME, rem(0, 5))
    assert s.leaf(ME, 0)[3] == UNASSIGNED
    assert s.groups(ME, 0) == 1
    remote = s.make(ME, op, 17, client="remoteClient")
    s.apply(ME, remote)
    assert s.leaf(ME, 0)[3] == 17
    assert s.groups(ME, 0) == 1
    s.apply(ME, s.make(ME, op, 18))
    assert s.leaf(ME, 0)[3] == 17
    assert s.groups(ME, 0) == 0
    assert s.length(ME) == len(initial) - 5
    assert s.text(ME) == initial[5:]
    return s


def kat_regenerate_annotate_over_removed_range():  # :495-522
    s = Clients(["A", "B"])
    seq = 1
    s.apply_all(s.make("A", s.local("A", ins(0, "AAA")), seq))
    aop = s.local("A", ann(0, s.length("A"), {"client": "A"}))
    seq += 1
    s.apply_all(s.make("B", s.local("B", rem(0, s.length("B"))), seq))
    new = s.regenerate("A", aop)
    assert new["type"] == 3 and len(new["ops"]) == 0, new
    return s


def kat_containing_segment_with_op():  # :524-555
    s = Clients(["A", "B"])
    seq = 1
    s.apply_all(s.make("A", s.local("A", ins(0, "ABC")), seq))
    rop = s.local("A", rem(0, 2))
    seq += 1
    remove_seq = seq
    s.apply("A", s.make("A", rop, remove_seq))
    iop = s.local("B", ins(2, "X"))
    seq += 1
    m2 = s.make("B", iop, seq)  # refSeq = B's currentSeq (1): the removed "AB" still counts
    b_on_a = s.logs["A"].short_id("B")  # getOrAddShortClientId(op.clientId)
    leaf = s.containing("A", 2, ref=m2["referenceSequenceNumber"], client=b_on_a)
    assert leaf is not None
    assert s.leaf("A", leaf[0])[0] == 1 and s.text("A") == "C"  # the segment "C"
    m3 = s.make("B", iop, seq, ref=remove_seq)
    assert s.containing("A", 2, ref=m3["referenceSequenceNumber"], client=b_on_a) is None
    return s


KATS = [kat_interleaved, kat_insert_text_local, kat_remove_range_local, kat_annotate_local, kat_annotate_then_remove,
        kat_multiple_interleaved_annotates, kat_overlapping_deletes, kat_regenerate_annotate_over_removed_range,
        kat_containing_segment_with_op]


@pytest.mark.parametrize("kat", KATS, ids=[k.__name__ for k in KATS])
def test_applymsg_local_kat_oracle(kat):
    kat()


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=[k.__name__ for k in KATS])
def test_applymsg_local_kat_engine(kat):
    kat().replay_engine()
