"""PartialSequenceLengths cross-check.

The reference resolves a block's length in a remote (refSeq, clientId) view with the block's
PartialSequenceLengths (mergeTree.ts:928-931 -> partialLengths.ts:698-735), maintained incrementally
where mergeTree.ts and zamboni.ts update it.  The oracle -- and the engine, whose visibility scan is
the same sum -- add up the leaves' nodeLength instead.  oracle/psl.h restates PartialSequenceLengths
(combine / fromLeaves / insertSegment / update / addSeq / zamboni / getPartialLength) and the oracle
keeps one per block at the reference's call sites; with the check on, every remote block-length query
the oracle makes (insertingWalk, nodeMap, the generator's view lengths, the legacy summary's
mapRange(minSeq, NonCollabClient) -- the one issue #1995 once broke, snapshotlegacy.ts:245-252)
compares the two.  This is the reference's own check (test/testUtils.ts:209-248, partialLength.spec.ts)
applied to every query of every op of the golden logs and of seeded synthetic documents.
"""
import pytest

from fixtures import load_replay, replay_files, replay_log
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, generate, generate_matrix, options, psl_check


def _assert_clean(pc, min_checks):
    checks, mismatches, first = pc.stats()
    assert mismatches == 0, f"{mismatches} of {checks} block lengths differ; first: {first}"
    assert checks >= min_checks, f"only {checks} block-length queries were checked"
    return checks


@pytest.mark.parametrize("v1", [True, False], ids=["v1", "legacy"])
def test_replay_logs_partial_lengths(v1):
    """All 30 golden logs, every group applied as a batch, each followed by a summary."""
    with psl_check() as pc:
        for p in replay_files():
            groups = load_replay(p)
            it = Interner()
            log = replay_log(groups, it)
            o = OracleDoc(options(snapshot_v1=v1))
            for g in groups:
                for m in g["msgs"]:
                    log.message(m, it)
                b = build_batch([log], it)
                assert o.apply(b, 0) == 0
                assert o.text() == g["resultText"]
            o.summarize(b, 0)
        _assert_clean(pc, 500_000)


@pytest.mark.parametrize("name,kw,newlen", [
    ("C3", dict(writers=8, max_lag=32), False),
    ("C2", dict(writers=16, max_lag=64), False),
    ("newlen", dict(writers=8, max_lag=32), True),
    ("long-ranges", dict(writers=8, max_lag=32, max_range=120, weights=(60, 30, 10)), False),
    ("lagless", dict(writers=3, max_lag=0), False),
])
def test_synthetic_partial_lengths(name, kw, newlen):
    """Seeded synthetic documents drawn by the oracle (the generator reads the writer's view length
    of the root before every op, the apply path every block on its walks)."""
    from fluidframework_amd.synth import make_cfg, tables

    n, ops = 24, 1500
    cfg = make_cfg(n, ops, seed=0x9510 + len(name), **kw)
    with psl_check() as pc:
        _, _, status = generate(cfg, tables(writers=kw["writers"]), 0, n, threads=8,
                                opts=options(new_length_calc=newlen))
        assert (status == 0).all()
        _assert_clean(pc, 100_000)


def test_deep_window_partial_lengths():
    """C5's shape at small size: pre-loaded segments (reloadFromSegments, then startCollaboration's
    recursive combine), 64 writers, lags up to 4096 and the MSN held back."""
    from fluidframework_amd.synth import make_cfg, tables

    n, ops, grow = 4, 1500, 3000
    cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
    with psl_check() as pc:
        _, _, status = generate(cfg, tables(writers=64), 0, n, threads=4, grow=grow)
        assert (status == 0).all()
        _assert_clean(pc, 50_000)


def test_matrix_partial_lengths():
    """PermutationVectors: setCell resolutions (getContainingSegment at the writer's view) and
    handle-allocation splits at the local view."""
    from test_matrix import matrix_cfg
    from fluidframework_amd.synth import tables

    cfg = matrix_cfg(8, 2000, writers=8, max_lag=64)
    with psl_check() as pc:
        _, _, status = generate_matrix(cfg, tables(writers=8), 0, 8, threads=8)
        assert (status == 0).all()
        _assert_clean(pc, 20_000)


def test_leaf_root_partial_lengths_lag_after_removes():
    """The modelled quirk: a root holding leaves gets no post-order update from markRangeRemoved
    (mergeTreeNodeWalk.ts:98-105), so its own partial length reads high until the next combine.
    Only nodeMap's default end (legacy extractSync) and getLength read it, and a high end changes
    nothing; the root's children -- what every walk reads -- stay exact."""
    from test_kats import ins, rem

    it = Interner()
    log = DocLog()
    log.start_collab("observer")
    for m in (ins("A", 1, 0, 0, "abc"), ins("B", 2, 1, 3, "def"), rem("A", 3, 2, 1, 4)):
        log.message(m, it)
    b = build_batch([log], it)
    with psl_check() as pc:
        o = OracleDoc(options())
        assert o.apply(b, 0) == 0
        assert o.length(3, 2) == 3  # the root at (refSeq 3, a third client): leaf sum "aef"
        checks, mismatches, _ = pc.stats()
        assert mismatches == 0 and pc.rootlag >= 1
