"""Known answers of packages/dds/merge-tree/src/test/partialLength.spec.ts:39-300.

The spec drives a MergeTree directly: "hello world!" inserted at seq 0, startCollaboration(17), then inserts and
removes by client 17 ("local") and 18 ("remote") at given (refSeq, seq), and validatePartialLengths asserts the
root's PartialSequenceLengths.getPartialLength(seq, clientId) -- and the leaf sum it must equal -- at every seq
in the window plus the listed (seq, len) answers (testUtils.ts:169-248).  Here the same edits are sequenced
messages of writers L (17) and R (18) applied by an observer client; an answer is nodeLength(root, seq, client)
of the observer's tree, which the oracle computes from the reference's PartialSequenceLengths (oracle/psl.h)
and compares with the leaf sum at every query (psl_check: no mismatch allowed).  The one case with an
unsequenced local remove (:276-300) runs on client L itself.  Under -m gpu the HIP engine must give every
length (its view scan: a segment holds position len - 1, none holds len).
"""
import pytest

from clients import Clients, ins, rem
from oracle.oracle import psl_check

OBS, L, R, R2 = "observer", "local", "remote", "remote2"
HELLO = "hello world!"


def _tree(on=OBS):
    return Clients([on], initial=HELLO)


def _msg(s, client, op, seq, ref, on=OBS):
    s.apply(on, s.make(on, op, seq, ref=ref, client=client))


def _validate(s, who, want, on=OBS):
    """validatePartialLengths(clientId, mergeTree, [{seq, len}]) at every seq of the window, then the answers"""
    c = s.logs[on].short_id(who)
    for q in range(1, s.cur[on] + 1):
        s.view_length(on, q, c)
    for q, n in want:
        got = s.view_length(on, q, c)
        assert got == n, f"{who} at seq {q}: {got} != {n}"


def kat_no_ops():  # :39-41
    s = _tree()
    _validate(s, L, [(0, 12)])
    return s


def _single_insert(author, viewer):  # :43-96
    s = _tree()
    _msg(s, author, ins(0, "more "), 1, 0)
    _validate(s, viewer, [(1, 17)])
    return s


def _single_remove(author, viewer):  # :98-158
    s = _tree()
    _msg(s, author, rem(0, 12), 1, 0)
    _validate(s, viewer, [(1, 0)])
    return s


def kat_multiple_permutations():  # :160-201
    s = _tree()
    for k, (who, text) in enumerate([(L, "1"), (R, "2"), (L, "3"), (R, "4")]):
        _msg(s, who, ins(0, text), k + 1, k)
    _validate(s, L, [(4, 16)])
    _validate(s, R, [(4, 16)])
    return s


def kat_different_heights():  # :203-221
    s = _tree()
    for i in range(100):
        _msg(s, L, ins(0, "a"), i + 1, i)
        _validate(s, L, [(i + 1, i + 13)])
        _validate(s, R, [(i + 1, i + 13)])
    _validate(s, L, [(100, 112)])
    _validate(s, R, [(100, 112)])
    return s


def kat_concurrent_remote_deletes():  # :225-249
    s = _tree()
    _msg(s, R, rem(0, 10), 1, 0)
    _msg(s, R2, rem(0, 10), 2, 0)
    _validate(s, L, [(1, 2)])
    return s


def kat_concurrent_local_and_remote_deletes():  # :250-275
    s = _tree()
    _msg(s, L, rem(0, 10), 1, 0)
    _msg(s, R, rem(0, 10), 2, 0)
    _validate(s, L, [(1, 2)])
    _validate(s, R, [(1, 2)])
    return s


def kat_unsequenced_local_and_remote_deletes():  # :276-300
    s = _tree(on=L)
    s.local(L, rem(0, 10))  # markRangeRemoved(..., clientId: local, seq: UnassignedSequenceNumber)
    _msg(s, R, rem(0, 10), 1, 0, on=L)
    _validate(s, L, [(1, 2)], on=L)
    _validate(s, R, [(1, 2)], on=L)
    return s


KATS = {
    "no_ops": kat_no_ops,
    "local_insert_local_view": lambda: _single_insert(L, L),
    "local_insert_remote_view": lambda: _single_insert(L, R),
    "remote_insert_local_view": lambda: _single_insert(R, L),
    "remote_insert_remote_view": lambda: _single_insert(R, R),
    "local_delete_local_view": lambda: _single_remove(L, L),
    "local_delete_remote_view": lambda: _single_remove(L, R),
    "remote_delete_local_view": lambda: _single_remove(R, L),
    "remote_delete_remote_view": lambda: _single_remove(R, R),
    "multiple_permutations": kat_multiple_permutations,
    "different_heights": kat_different_heights,
    "concurrent_remote_deletes": kat_concurrent_remote_deletes,
    "concurrent_local_and_remote_deletes": kat_concurrent_local_and_remote_deletes,
    "unsequenced_local_and_remote_deletes": kat_unsequenced_local_and_remote_deletes,
}


@pytest.mark.parametrize("name", list(KATS))
def test_partial_length_kat_oracle(name):
    with psl_check() as pc:
        KATS[name]()
        checks, mismatches, first = pc.stats()
    assert mismatches == 0, first


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(KATS))
def test_partial_length_kat_engine(name):
    KATS[name]().replay_engine()
