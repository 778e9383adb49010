"""GPU tests of the boundary additions and of full-size documents:

* bulk summary download (mtr_get_summaries) against the per-document reads, mtr_summary_info sizing,
  the MTR_SUMMARY_TOO_SMALL answer, empty batches, the short-client-id cap;
* documents at C2 (5,000 messages, 16 writers, lag 64) and C4 (20,000 matrix messages) size against
  the oracle;
* document sharding through the real engine: two engines holding rank 0 / rank 1's document ranges
  give the same run digest as one engine holding all of them.
"""
import numpy as np
import pytest

from fluidframework_amd import abi, shard
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, generate, generate_matrix, options, replay_matrix_batch

pytestmark = pytest.mark.gpu


def _engine(n_docs, **kw):
    from fluidframework_amd.engine import Engine
    caps = dict(max_segments=8192, heap_entries=8192, text_units=1 << 18, prop_words=1 << 18, remover_cells=1 << 14)
    caps.update(kw)
    return Engine(n_docs, **caps)


@pytest.mark.parametrize("v1, chunk", [(True, 10000), (True, 300), (False, 10000), (False, 200)])
def test_summary_bodies_split_pairs_and_long_pieces(v1, chunk):
    """The summary passes' text bodies counted and written a piece (leaf) at a time: every document's blobs equal
    the oracle's (SnapshotV1 and legacy, one blob and many) for texts dense in surrogate pairs (40 % of inserts end
    with one, and splits land between the halves, so pairs straddle pieces of a coalesced spec) and inserts of up
    to 100 units (pieces longer than one lane's share, written by the wave)."""
    from oracle.oracle import OracleDoc, options
    from fluidframework_amd.synth import make_cfg, tables

    n, ops = 160, 500
    cfg = make_cfg(n, ops, writers=8, max_lag=32, max_text=100, nonbmp_permille=400, newline_permille=3,
                   seed=0x5a77 + chunk + int(v1))
    eng = _engine(n, snapshot_v1=v1, chunk_size=chunk, max_segments=2 * ops + 128, heap_entries=2 * ops + 128,
                  text_units=2 * int(cfg.text_cap) + 1024, prop_words=16384, remover_cells=4096, ops_per_launch=48)
    eng.generate(cfg, tables(writers=8))
    eng.reset()
    eng.run()
    eng.summarize()
    assert eng.stats()["bad_docs"] == 0
    hb = eng.download(0, n)
    n_multi = 0
    for d in range(n):
        orc = OracleDoc(options(snapshot_v1=v1, chunk_size=chunk))
        assert orc.apply(hb, d) == 0
        want = orc.summarize(hb, d)
        assert eng.summary(d) == want, f"doc {d}"
        n_multi += len(want) > 1
    if chunk < 1000:
        assert n_multi > 0


def test_bulk_summaries_equal_per_document_reads():
    from fluidframework_amd.engine import Engine, lib, pinned
    from fluidframework_amd.synth import make_cfg, tables

    n, ops = 64, 600
    cfg = make_cfg(n, ops, writers=8, max_lag=32, seed=0xb01c)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                  ops_per_launch=64, chunk_size=256)  # small chunks: several blobs per document
    eng.generate(cfg, tables(writers=8))
    eng.reset()
    eng.run()
    eng.summarize()
    out = pinned(eng.summary_bytes() + 64, "u1")
    buf, off = eng.summaries(0, n, out=out)
    assert int(off[-1]) == eng.summary_bytes()
    for d in range(n):
        assert Engine.split_record(buf, int(off[d]), int(off[d + 1])) == eng.summary(d)
    # a sub-range starts at offset 0
    buf2, off2 = eng.summaries(5, 9)
    for i, d in enumerate(range(5, 9)):
        assert Engine.split_record(buf2, int(off2[i]), int(off2[i + 1])) == eng.summary(d)
    # sizing: too-small buffers are refused without writing, never read as a blob count
    import ctypes as C
    nb, nbytes = C.c_int64(0), C.c_int64(0)
    assert lib().mtr_summary_info(eng.h, 3, C.byref(nb), C.byref(nbytes)) == 0
    assert nb.value == len(eng.summary(3)) and nbytes.value == sum(len(x) for x in eng.summary(3))
    small = np.zeros(max(nbytes.value - 1, 1), dtype="u1")
    lens = np.zeros(max(nb.value, 1), dtype="<i8")
    r = lib().mtr_get_summary(eng.h, 3, small.ctypes.data, small.size, lens.ctypes.data, nb.value)
    assert r == -3  # MTR_SUMMARY_TOO_SMALL
    r = lib().mtr_get_summary(eng.h, 3, small.ctypes.data, 1 << 30, lens.ctypes.data, nb.value - 1)
    assert r == -3
    need = lib().mtr_get_summaries(eng.h, 0, n, None, 0, None)
    assert need == -eng.summary_bytes()


def test_empty_batch():
    eng = _engine(4)
    b = build_batch([], Interner())
    eng.apply(b)
    eng.summarize()
    assert eng.stats()["ops"] == 0


def test_too_many_clients_is_unsupported_per_document():
    """A document with more short ids than the engine's 8-bit client field (MTR_MAX_CLIENTS) is
    marked unsupported at submit; the other documents of the batch are applied normally."""
    it = Interner()
    good, bad = DocLog(), DocLog()
    for log in (good, bad):
        log.local_insert(0, "hello", it)
        log.start_collab("observer")
    # bypass the packer's own refusal (it raises Unsupported at MAX_CLIENTS)
    bad.clients += [f"c{i}" for i in range(300)]
    b = build_batch([good, bad], it)
    eng = _engine(2)
    eng.apply(b)
    assert eng.status(0)[0] == abi.MTR_OK and eng.text(0) == "hello"
    assert eng.status(1)[0] == abi.MTR_ERR_UNSUPPORTED


def test_c2_size_documents_match_oracle():
    """C2-sized documents (5,000 messages, 16 writers, lag <= 64): up to ~1,300 leaves,
    the largest LDS classes; every summary equals the oracle's."""
    from fluidframework_amd.synth import make_cfg, tables

    n, ops = 64, 5000
    cfg = make_cfg(n, ops, writers=16, max_lag=64, seed=0xc2)
    tabs = tables(writers=16)
    b, ohash, ost = generate(cfg, tabs, 0, n, threads=16)
    assert (ost == 0).all()
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 8192,
                  prop_words=1 << 17, remover_cells=8192, ops_per_launch=48)
    eng.apply(b)
    eng.summarize()
    for d in range(n):
        st, op = eng.status(d)
        assert st == 0, f"doc {d}: status {st:#x} at op {op}"
    ghash = eng.hashes(n)
    bad = np.nonzero(ghash != ohash)[0]
    if bad.size:
        d = int(bad[0])
        orc = OracleDoc(options())
        assert orc.apply(b, d) == 0
        assert eng.summary(d) == orc.summarize(b, d)
    assert bad.size == 0
    st = eng.stats()
    assert st["max_leaves"] > 700, st  # the test reaches the large classes


def test_c4_size_matrices_match_oracle():
    """C4-sized SharedMatrix documents (20,000 messages per matrix, 20 % row/col splices,
    80 % setCell, lag <= 64): both vectors' summaries (segments + handleTable) equal the oracle's."""
    from test_matrix import expand_pairs, matrix_cfg
    from fluidframework_amd.synth import tables

    n, ops = 16, 20000
    cfg = matrix_cfg(n, ops, writers=8, max_lag=64)
    tabs = tables(writers=8)
    gb, _, status = generate_matrix(cfg, tabs, 0, n, threads=16)
    assert (status == 0).all()
    b = expand_pairs(gb, tabs)
    eng = _engine(2 * n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * ops + 1024,
                  prop_words=1024, remover_cells=8192, ops_per_launch=48)
    for m in range(n):
        eng.set_matrix(2 * m, 2 * m + 1)
    eng.apply(b)
    eng.summarize()
    for d in range(2 * n):
        st, op = eng.status(d)
        assert st == 0, f"document {d}: status {st:#x} at op {op}"
    _, oh, st = replay_matrix_batch(gb, 0, n, 16)
    assert (st == 0).all()
    assert np.array_equal(eng.hashes(2 * n), oh)


def test_two_engines_as_two_ranks_equal_one_engine():
    """Document sharding through the real engine: rank 0 / rank 1 of a strong-scaling split (two
    engines on device 0, each recording and replaying its own document range) reduce to the same run
    digest and message count as one engine holding every document."""
    from fluidframework_amd.synth import make_cfg, tables

    total, ops = 300, 500
    tabs = tables(writers=8)
    digests, msgs = [], 0
    for rank in range(2):
        lo, hi = shard.strong_range(rank, 2, total)
        cfg = make_cfg(hi - lo, ops, writers=8, max_lag=32, doc_base=lo)
        eng = _engine(hi - lo, max_segments=2 * ops + 128, heap_entries=2 * ops + 128,
                      text_units=2 * int(cfg.text_cap) + 1024, ops_per_launch=48)
        eng.generate(cfg, tabs)
        eng.reset()
        eng.run()
        eng.summarize()
        assert eng.stats()["bad_docs"] == 0
        digests.append(shard.digest(eng.hashes(hi - lo)))
        msgs += (hi - lo) * ops
        eng.close()
    cfg = make_cfg(total, ops, writers=8, max_lag=32)
    one = _engine(total, max_segments=2 * ops + 128, heap_entries=2 * ops + 128,
                  text_units=2 * int(cfg.text_cap) + 1024, ops_per_launch=48)
    one.generate(cfg, tabs)
    one.reset()
    one.run()
    one.summarize()
    assert msgs == total * ops
    assert (sum(digests) & shard.MASK64) == shard.digest(one.hashes(total))


def test_containing_segment_matches_oracle():
    """Client.getContainingSegment(pos, {referenceSequenceNumber, clientId}) on the device
    (mtr_get_containing_segment) equals the oracle's nodeMap over [pos, pos + 1) at every queried view:
    the reference replay logs stopped mid-collaboration, views from the MSN to the current seq, every
    client, every position (and one past the end)."""
    import random

    from fixtures import load_replay, replay_files, replay_log

    files = [p for p in replay_files() if "clients_8" in p][:5]
    it = Interner()
    logs, orcs = [], []
    for p in files:
        groups = load_replay(p)
        log = replay_log(groups, it)
        for g in groups[:40]:
            for m in g["msgs"]:
                log.message(m, it)
        logs.append(log)
    b = build_batch(logs, it)
    eng = _engine(len(files))
    eng.apply(b)
    rng = random.Random(7)
    n_checked = 0
    for d in range(len(files)):
        o = OracleDoc(options())
        assert o.apply(b, d) == 0
        st = o.state()
        min_seq, cur = int(st[0]), int(st[1])
        n_clients = int(b.docs["n_clients"][d])
        for _ in range(120):
            ref = rng.randint(min_seq, cur)
            client = rng.randint(0, n_clients - 1)
            L = o.length(ref, client)
            pos = rng.randint(0, max(L, 0))
            got = eng.containing_segment(d, pos, ref, client)
            exp = o.containing(pos, ref, client)
            if exp[0] < 0:
                assert got is None, (d, pos, ref, client, got)
                continue
            assert got is not None, (d, pos, ref, client, exp)
            assert (got["leaf"], got["offset"], got["length"], got["start"]) == exp, (d, pos, ref, client)
            n_checked += 1
    assert n_checked > 400


@pytest.mark.parametrize("n, parts", [(3000, 2), (3000, 64), (5000, 7), (5000, 16)])
def test_pipelined_submit_equals_serial_submit(n, parts):
    """mtr_submit_pipelined (the end-to-end hand-over with the upload overlapped): the same summaries as
    mtr_submit + mtr_run, from the recorded op logs in page-locked memory, for part counts that do not divide the
    documents evenly; a pipelined batch can be followed by an ordinary one on the same engine."""
    from fluidframework_amd.synth import make_cfg, tables

    ops = 300  # (5,000 documents: two document groups, whose parts are uploaded alternately)
    cfg = make_cfg(n, ops, writers=8, max_lag=32, seed=0x91be + parts)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                  prop_words=16384, remover_cells=4096, ops_per_launch=48)
    eng.generate(cfg, tables(writers=8))
    eng.reset()
    eng.run()
    eng.summarize()
    want = eng.hashes(n).copy()
    hb = eng.download(0, n, pinned_memory=True)
    for _ in range(2):
        eng.reset()
        eng.submit_pipelined(hb, parts)
        eng.run()
        eng.summarize()
        eng.sync()
        assert eng.stats()["bad_docs"] == 0
        assert np.array_equal(eng.hashes(n), want)
    eng.reset()
    eng.submit(hb)
    eng.run()
    eng.summarize()
    assert np.array_equal(eng.hashes(n), want)


@pytest.mark.parametrize("n, parts", [(3000, 16), (5000, 7), (5000, 64)])
def test_replay_pipelined_equals_serial_calls(n, parts, monkeypatch):
    """mtr_replay_pipelined (a range summarized and downloaded once its documents are done, while the later ranges
    still upload and apply): byte for byte the records of mtr_submit + mtr_run + mtr_summarize + mtr_get_summaries,
    the same hashes, the per-document reads still served afterwards; a buffer too small is refused.  (Ranges of any
    size: MTR_PIPE_MIN_PART_DOCS=0 -- by default ranges under 3,000 documents take the serial calls.)"""
    from fluidframework_amd.engine import EngineError, pinned
    from fluidframework_amd.synth import make_cfg, tables

    monkeypatch.setenv("MTR_PIPE_MIN_PART_DOCS", "0")

    ops = 300
    cfg = make_cfg(n, ops, writers=8, max_lag=32, seed=0x7e11 + parts)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                  prop_words=16384, remover_cells=4096, ops_per_launch=48)
    eng.generate(cfg, tables(writers=8))
    hb = eng.download(0, n, pinned_memory=True)
    eng.reset()
    eng.submit(hb)
    eng.run()
    eng.summarize()
    want_h = eng.hashes(n).copy()
    want, want_off = eng.summaries(0, n)
    want = want[:int(want_off[-1])].copy()
    out = pinned(want.size + 4096, "u1")
    for _ in range(2):
        eng.reset()
        out[:] = 0
        buf, off = eng.replay_pipelined(hb, out, parts)
        assert eng.stats()["bad_docs"] == 0
        assert np.array_equal(off, want_off)
        assert np.array_equal(buf[:int(off[-1])], want)
        assert np.array_equal(eng.hashes(n), want_h)
        for d in (0, n // 2, n - 1):
            again, again_off = eng.summaries(d, d + 1)
            assert np.array_equal(again[:int(again_off[-1])], want[int(want_off[d]):int(want_off[d + 1])])
    eng.reset()
    with pytest.raises(EngineError, match="output buffer"):
        eng.replay_pipelined(hb, pinned(want.size // 2, "u1"), parts)


@pytest.mark.parametrize("n, parts, force", [(5, 16, True), (40, 1, True), (40, 3, True), (4000, 16, False)])
def test_replay_pipelined_small_batches_and_serial_fallback(n, parts, force, monkeypatch):
    """mtr_replay_pipelined on batches the pipelined path splits into fewer ranges than asked (5 documents, 16 parts)
    or does not split at all (parts = 1; or, by default, ranges under 3,000 documents: the serial calls inside): the
    records of the serial calls."""
    from fluidframework_amd.engine import pinned
    from fluidframework_amd.synth import make_cfg, tables

    if force:
        monkeypatch.setenv("MTR_PIPE_MIN_PART_DOCS", "0")
    else:
        monkeypatch.delenv("MTR_PIPE_MIN_PART_DOCS", raising=False)

    ops = 200
    cfg = make_cfg(n, ops, writers=4, max_lag=16, seed=0x5a11 + n + parts)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                  prop_words=16384, remover_cells=4096, ops_per_launch=48)
    eng.generate(cfg, tables(writers=4))
    hb = eng.download(0, n, pinned_memory=True)
    eng.reset()
    eng.submit(hb)
    eng.run()
    eng.summarize()
    want, want_off = eng.summaries(0, n)
    want = want[:int(want_off[-1])].copy()
    eng.reset()
    buf, off = eng.replay_pipelined(hb, pinned(want.size + 64, "u1"), parts)
    assert eng.stats()["bad_docs"] == 0
    assert np.array_equal(off, want_off)
    assert np.array_equal(buf[:int(off[-1])], want)


def test_replay_pipelined_refuses_records_beyond_remote_ops(monkeypatch):
    """A range holding a record the pipelined path does not run: mtr_replay_pipelined fails with
    MTR_ERR_UNSUPPORTED's message, and after mtr_reset the serial calls apply the same batch in full."""
    from fluidframework_amd.engine import EngineError, pinned
    from fluidframework_amd.synth import make_cfg, tables, with_docs

    monkeypatch.setenv("MTR_PIPE_MIN_PART_DOCS", "0")

    n, ops = 400, 200
    cfg = make_cfg(n, ops, writers=4, max_lag=16, seed=0xbeef)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                  prop_words=16384, remover_cells=4096, ops_per_launch=48)
    eng.generate(cfg, tables(writers=8))
    eng.reset()
    eng.run()
    eng.summarize()
    want = eng.hashes(n).copy()
    hb = eng.download(0, n)
    ops_arr = hb.ops.copy()
    ops_arr["flags"][int(hb.docs["op_begin"][123]) + 7] |= abi.F_DELTA
    flagged = with_docs(tables(writers=8), hb.docs.copy(), ops_arr, hb.text)
    eng.reset()
    with pytest.raises(EngineError, match="beyond remote ops"):
        eng.replay_pipelined(flagged, pinned(1 << 24, "u1"), 4)
    eng.reset()
    eng.submit(flagged)
    eng.run()
    eng.summarize()
    assert eng.stats()["bad_docs"] == 0
    assert np.array_equal(eng.hashes(n), want)


def test_pipelined_submit_refuses_records_beyond_remote_ops():
    """A part holding a record the pipelined path does not run (here MTR_F_DELTA) is not started: mtr_run returns
    MTR_ERR_UNSUPPORTED, and after mtr_reset the same batch through mtr_submit is applied in full."""
    from fluidframework_amd.engine import EngineError
    from fluidframework_amd.synth import make_cfg, tables, with_docs

    n, ops = 400, 200
    cfg = make_cfg(n, ops, writers=4, max_lag=16, seed=0xdead)
    eng = _engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                  prop_words=16384, remover_cells=4096, ops_per_launch=48)
    eng.generate(cfg, tables(writers=8))
    eng.reset()
    eng.run()
    eng.summarize()
    want = eng.hashes(n).copy()
    hb = eng.download(0, n)
    ops_arr = hb.ops.copy()
    k = int(hb.docs["op_begin"][300]) + 5  # a message of document 300 flagged for delta reporting
    ops_arr["flags"][k] |= abi.F_DELTA
    flagged = with_docs(tables(writers=8), hb.docs.copy(), ops_arr, hb.text)
    eng.reset()
    eng.submit_pipelined(flagged, 4)
    with pytest.raises(EngineError, match="beyond remote ops"):
        eng.run()
    eng.reset()
    eng.submit(flagged)
    eng.run()
    eng.summarize()
    assert eng.stats()["bad_docs"] == 0
    assert np.array_equal(eng.hashes(n), want)  # (a delta flag reports ranges; it does not change the result)
