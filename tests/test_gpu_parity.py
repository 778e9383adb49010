"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle and the golden vectors.

Bit-exact for everything: text, leaf boundaries, tree shape (bnd levels), removal info, property
sets and summary bytes.
"""
import os

import numpy as np
import pytest

from fixtures import (SNAPSHOT_VERSIONS, blob_names, load_replay, load_snapshots, replay_files,
                      replay_log, snapshot_log)
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, options

pytestmark = pytest.mark.gpu


def _engine(n_docs, **kw):
    from fluidframework_amd.engine import Engine
    caps = dict(max_segments=8192, heap_entries=8192, text_units=1 << 18, prop_words=1 << 18, remover_cells=1 << 14)
    caps.update(kw)
    return Engine(n_docs, **caps)


def _compare_export(eng, d, orc):
    ge, gh = eng.export(d)
    oe, oh = orc.export()
    assert gh == oh, f"doc {d}: height {gh} vs oracle {oh}"
    assert ge.shape == oe.shape, f"doc {d}: {len(ge)} leaves vs oracle {len(oe)}"
    bad = np.nonzero((ge != oe).any(axis=1))[0]
    assert bad.size == 0, f"doc {d}: first differing leaf {bad[0]}: {ge[bad[0]].tolist()} vs {oe[bad[0]].tolist()}"


def test_replay_logs_group_by_group():
    """All 30 reference replay logs as 30 documents of one engine, one batch per group;
    text after every group, leaf structure and V1 summary bytes at the end."""
    files = replay_files()
    all_groups = [load_replay(p) for p in files]
    it = Interner()
    logs = [replay_log(g, it) for g in all_groups]
    orcs = [OracleDoc(options()) for _ in files]
    eng = _engine(len(files), ops_per_launch=64)
    b = build_batch(logs, it)
    eng.apply(b)
    for d, o in enumerate(orcs):
        assert o.apply(b, d) == 0
    n_groups = max(len(g) for g in all_groups)
    for gi in range(n_groups):
        for d, groups in enumerate(all_groups):
            if gi < len(groups):
                for m in groups[gi]["msgs"]:
                    logs[d].message(m, it)
        b = build_batch(logs, it)
        eng.apply(b)
        for d, groups in enumerate(all_groups):
            assert orcs[d].apply(b, d) == 0
            st, op = eng.status(d)
            assert st == 0, f"doc {d} group {gi}: status {st:#x} at op {op}"
            if gi < len(groups):
                assert eng.text(d) == groups[gi]["resultText"], f"{os.path.basename(files[d])} group {gi}"
    for d in range(len(files)):
        _compare_export(eng, d, orcs[d])
    eng.summarize()
    for d in range(len(files)):
        assert eng.summary(d) == orcs[d].summarize(b, d), f"doc {d} summary"


SNAPS = load_snapshots()


@pytest.mark.parametrize("v1", [True, False], ids=["v1", "legacy"])
def test_snapshot_fixtures(v1):
    keys = sorted(k for k in SNAPS if SNAPSHOT_VERSIONS[k.split("/")[0]] == v1)
    it = Interner()
    logs = [snapshot_log(k.split("/")[1], it) for k in keys]
    b = build_batch(logs, it)
    eng = _engine(len(keys), snapshot_v1=v1, max_segments=16384, heap_entries=256)
    eng.apply(b)
    eng.summarize()
    for d, k in enumerate(keys):
        st, op = eng.status(d)
        assert st == 0, f"{k}: status {st:#x} at op {op}"
        blobs = eng.summary(d)
        got = dict(zip(blob_names(len(blobs), v1), blobs))
        exp = {n: v.encode("utf-8") for n, v in SNAPS[k].items()}
        assert got == exp, k


@pytest.mark.parametrize("writers,max_lag", [(8, 32), (16, 64), (3, 0)])
def test_synthetic_record_mode_matches_oracle(writers, max_lag):
    """Record mode draws each op with the engine's own view length; the oracle drawing the same
    recipe must produce the identical op log, text and summary digests (C3-shaped documents)."""
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate, replay_batch, summary_digest

    n, ops = 384, 1000
    tabs = tables(writers=writers)
    cfg = make_cfg(n, ops, writers=writers, max_lag=max_lag, seed=0x5eed + writers)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=40000, prop_words=1 << 16,
                  remover_cells=4096, ops_per_launch=128)
    eng.generate(cfg, tabs)
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
    gb = eng.download(0, n)
    ob, ohash, ost = generate(cfg, tabs, 0, n, threads=16)
    assert (ost == 0).all()
    assert np.array_equal(gb.docs, ob.docs)
    assert np.array_equal(gb.ops, ob.ops), "recorded op logs differ from the oracle-driven recipe"
    assert np.array_equal(gb.text, ob.text)
    eng.summarize()
    ghash = eng.hashes(n)
    assert np.array_equal(ghash, ohash), f"{int((ghash != ohash).sum())} documents' summaries differ"
    for d in (0, 1, n - 1):
        assert summary_digest(eng.summary(d)) == int(ohash[d])
    # replaying the recorded batch from a fresh state reproduces the same summaries
    eng.reset()
    eng.run()
    eng.summarize()
    assert np.array_equal(eng.hashes(n), ohash)
    _, rhash, rst = replay_batch(ob, 0, n, 16)
    assert np.array_equal(rhash, ohash)


def test_c2_full_documents():
    """Config C2's documents at full length (5,000 messages, 16 writers, lag <= 64, up to
    ~1,300 leaves): record mode on the device equals the oracle-driven recipe op for op, and every
    summary digest equals the oracle's."""
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    n, ops, writers = 64, 5000, 16
    tabs = tables(writers=writers)
    cfg = make_cfg(n, ops, writers=writers, max_lag=64, seed=0xc2)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128,
                  text_units=2 * (int(cfg.text_cap) + 8192), prop_words=1 << 16, remover_cells=8192,
                  ops_per_launch=128)
    eng.generate(cfg, tabs)
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
    gb = eng.download(0, n)
    ob, ohash, ost = generate(cfg, tabs, 0, n, threads=16)
    assert (ost == 0).all()
    assert np.array_equal(gb.ops, ob.ops), "recorded op logs differ from the oracle-driven recipe"
    eng.summarize()
    assert np.array_equal(eng.hashes(n), ohash)
    assert eng.stats()["max_leaves"] > 600  # C2-sized documents


@pytest.mark.parametrize("v1", [True, False], ids=["v1", "legacy"])
def test_load_snapshot_fixtures(v1):
    """Client.load of every reference snapshot fixture on the device (reloadFromSegments + body
    appends), then summarize: the fixture bytes come back, and the leaf structure equals the oracle's."""
    keys = sorted(k for k in SNAPS if SNAPSHOT_VERSIONS[k.split("/")[0]] == v1)
    it = Interner()
    logs = []
    for k in keys:
        log = DocLog()
        log.load_summary(SNAPS[k], "snapshot", it)
        logs.append(log)
    b = build_batch(logs, it)
    eng = _engine(len(keys), snapshot_v1=v1, max_segments=16384, heap_entries=256)
    eng.apply(b)
    eng.summarize()
    for d, k in enumerate(keys):
        st, op = eng.status(d)
        assert st == 0, f"{k}: status {st:#x} at op {op}"
        orc = OracleDoc(options(snapshot_v1=v1))
        assert orc.apply(b, d) == 0
        _compare_export(eng, d, orc)
        blobs = eng.summary(d)
        got = dict(zip(blob_names(len(blobs), v1), blobs))
        assert got == {n: v.encode("utf-8") for n, v in SNAPS[k].items()}, k


def test_summarize_load_continue_on_device():
    """Summarize the replay logs mid-collaboration on the device, load those summaries into new
    documents, keep applying the remaining messages to both: text after every group equals
    resultText, and the loaded documents match the oracle leaf-for-leaf and byte-for-byte."""
    files = [p for p in replay_files() if "clients_8" in p]
    all_groups = [load_replay(p) for p in files]
    it = Interner()
    logs = [replay_log(g, it) for g in all_groups]
    cut = 32
    for log, groups in zip(logs, all_groups):
        for g in groups[:cut]:
            for m in g["msgs"]:
                log.message(m, it)
        last = groups[cut - 1]["msgs"][-1]
        log.seq_update(last["minimumSequenceNumber"], last["sequenceNumber"])
    n = len(files)
    eng = _engine(2 * n, ops_per_launch=64)
    b = build_batch(logs + [DocLog() for _ in range(n)], it)
    eng.apply(b)
    eng.summarize()
    loaded = []
    for d in range(n):
        blobs = eng.summary(d)
        log = DocLog()
        log.load_summary(dict(zip(blob_names(len(blobs), True), [x.decode() for x in blobs])), "snapshot", it)
        loaded.append(log)
    orcs = [OracleDoc(options()) for _ in range(n)]
    b = build_batch([DocLog() for _ in range(n)] + loaded, it)
    eng.apply(b)
    for d in range(n):
        assert orcs[d].apply(b, n + d) == 0
        assert eng.text(n + d) == all_groups[d][cut - 1]["resultText"]
    for gi in range(cut, 64):
        for d, groups in enumerate(all_groups):
            for m in groups[gi]["msgs"]:
                logs[d].message(m, it)
                loaded[d].message(m, it)
        b = build_batch(logs + loaded, it)
        eng.apply(b)
        for d, groups in enumerate(all_groups):
            assert orcs[d].apply(b, n + d) == 0
            assert eng.status(n + d)[0] == 0
            assert eng.text(d) == eng.text(n + d) == groups[gi]["resultText"], f"doc {d} group {gi}"
    eng.summarize()
    for d in range(n):
        _compare_export(eng, n + d, orcs[d])
        assert eng.summary(n + d) == orcs[d].summarize(b, n + d)


@pytest.mark.parametrize("n,grow,ops", [(8, 20000, 2000), (4, 20000, 12000), (2, 200000, 300)],
                         ids=["20k-segments", "20k-segments-long", "200k-segments"])
def test_c5_shaped_hbm_resident(n, grow, ops):
    """Config C5's shape: documents pre-grown through a summary load (20k, and C5's
    full 200k header segments, reloadFromSegments), then 64 writers with lags up to 4096 keeping the
    MSN far behind (deep collaboration window).  The documents exceed LDS, so the engine runs them
    HBM-resident (apply_kernel<true>); leaves, tree shape and summary bytes equal the oracle's.  The
    full-size case keeps the op count small: each op scans all 200k leaves."""
    import time

    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
    tabs = tables(writers=64)
    b, _, status = generate(cfg, tabs, 0, n, threads=8, grow=grow)
    assert (status == 0).all()
    eng = _engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                  text_units=2 * (int(cfg.text_cap) + 8192), ops_per_launch=256)
    t0 = time.time()
    eng.apply(b)
    eng.summarize()
    print(f"C5-shaped: {n} docs x ({grow} loaded + {ops} ops) in {time.time() - t0:.2f} s", eng.timing())
    # the documents run with hole slots (one per 16): more slots than leaves can exist
    # (a long run shrinks them under zamboni until they are respread without the dead slots)
    if ops <= 2000:
        assert eng.stats()["max_leaves"] > grow + grow // 20
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
        orc = OracleDoc(options())
        assert orc.apply(b, d) == 0
        _compare_export(eng, d, orc)
        assert eng.summary(d) == orc.summarize(b, d)


@pytest.mark.timeout(600)
def test_c5_full_documents():
    """Two of config C5's documents at full size (200k loaded segments, 20k ops from 64 writers, lag
    <= 4096): zamboni shrinks them to ~14k leaves in ~214k slots, so long runs of hole slots and
    chunks with no length in a view appear (the regime of the two fixes in DESIGN.md §2).  Summary
    digests equal the oracle's, which recorded the logs."""
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    n, grow, ops = 2, 200000, 20000
    cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
    tabs = tables(writers=64)
    b, ohash, status = generate(cfg, tabs, 0, n, threads=8, grow=grow)
    assert (status == 0).all()
    eng = _engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                  text_units=2 * (int(cfg.text_cap) + 8192), ops_per_launch=256)
    eng.apply(b)
    eng.summarize()
    for d in range(n):
        assert eng.status(d)[0] == 0, f"doc {d}: {eng.status(d)}"
    assert (eng.hashes(n) == ohash).all()


def test_long_ranges_grow_the_lds_heap():
    """Removes/annotates over up to 120 units touch many leaf blocks, each an LRU push: documents
    whose LDS heap could overflow yield before the op and are relaunched with a larger heap
    (DocHdr.heap_need).  Summaries equal the oracle's."""
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate, replay_batch

    n, ops = 256, 1200
    tabs = tables(writers=8)
    cfg = make_cfg(n, ops, writers=8, max_lag=32, max_range=120, weights=(60, 30, 10), seed=0xa11)
    b, ohash, ost = generate(cfg, tabs, 0, n, threads=16)
    assert (ost == 0).all()
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 8192,
                  prop_words=1 << 16, remover_cells=1 << 14, ops_per_launch=16)
    eng.apply(b)
    eng.summarize()
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
    assert np.array_equal(eng.hashes(n), ohash)


@pytest.mark.parametrize("newlen,v1,chunk", [(True, True, 10000), (False, True, 64), (False, False, 10000),
                                             (True, False, 256)],
                         ids=["newlen", "v1-chunk64", "legacy", "newlen-legacy-chunk256"])
def test_options_synthetic(newlen, v1, chunk):
    """IMergeTreeOptions the engine honours (mergeTree.ts:400-438): mergeTreeUseNewLengthCalculations
    (the other nodeLength branch, mergeTree.ts:935-965), SnapshotLegacy vs SnapshotV1 mid-collaboration,
    and small mergeTreeSnapshotChunkSize (many body chunks).  The oracle generates the logs under the
    same options; summaries must agree byte for byte."""
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    n, ops = 192, 1000
    opts = options(new_length_calc=newlen, snapshot_v1=v1, chunk_size=chunk)
    tabs = tables(writers=8)
    cfg = make_cfg(n, ops, writers=8, max_lag=32, seed=0xc0ffee + chunk)
    b, ohash, ost = generate(cfg, tabs, 0, n, threads=16, opts=opts)
    assert (ost == 0).all()
    eng = _engine(n, new_length_calc=newlen, snapshot_v1=v1, chunk_size=chunk, max_segments=2 * ops + 128,
                  heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 8192, prop_words=1 << 16,
                  remover_cells=4096, ops_per_launch=32)
    eng.apply(b)
    eng.summarize()
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
    ghash = eng.hashes(n)
    bad = np.nonzero(ghash != ohash)[0]
    if bad.size:
        d = int(bad[0])
        orc = OracleDoc(opts)
        assert orc.apply(b, d) == 0
        _compare_export(eng, d, orc)
        assert eng.summary(d) == orc.summarize(b, d)
    assert bad.size == 0


def test_grown_record_mode_matches_oracle_generator():
    """mtr_generate_grown (config C5's pre-grown documents drawn on the device) records the same logs
    as the oracle's generator from the same seeds, and replays to the oracle's summaries."""
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    n, grow, ops = 4, 5000, 600
    cfg = make_cfg(n, ops, writers=64, max_lag=512, text_cap=2 * grow + ops * 18 + 16)
    tabs = tables(writers=64)
    ob, ohash, ost = generate(cfg, tabs, 0, n, threads=4, grow=grow)
    assert (ost == 0).all()
    eng = _engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                  text_units=2 * (int(cfg.text_cap) + 8192), ops_per_launch=256)
    eng.generate(cfg, tabs, grow=grow)
    rec = eng.download(0, n)
    assert rec.ops.tobytes() == ob.ops.tobytes()
    eng.reset()
    eng.run()
    eng.summarize()
    assert np.array_equal(eng.hashes(n), ohash)
