"""The Node host path (the reference's TypeScript side): the N-API addon over the C ABI and the JS
packer / BatchReplayClient (fluidframework_amd/node).  CPU: the addon loads, exports its entry points
and fails loudly without a GPU; the JS packer produces the same batch bytes as the Python packer.
GPU: the reference replay test through Node, text after every group + summary bytes vs the oracle."""
import base64
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from fixtures import load_replay, replay_files, replay_log
from fluidframework_amd import abi
from fluidframework_amd.batch import MAX_CLIENTS, DocLog, Interner, Unsupported, build_batch
from oracle.oracle import OracleDoc, options

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE_DIR = os.path.join(ROOT, "fluidframework_amd", "node")
ADDON = os.path.join(NODE_DIR, "mtr_napi.node")
HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.skipif(shutil.which("node") is None, reason="node is not installed")


def _addon():
    if not os.path.exists(ADDON):
        from fluidframework_amd import build
        build.build_engine()
        if build.build_node_addon() is None:
            pytest.skip("node headers missing")
    return ADDON


def _node(args, timeout=600):
    r = subprocess.run(["node"] + args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    return r.stdout


def test_addon_loads_and_fails_loudly_without_a_gpu():
    _addon()
    out = _node(["-e", "const m=require(process.argv[1]);const a=m.native();"
                 "console.log(JSON.stringify(Object.keys(a).sort()));"
                 "try{new m.BatchReplayEngine(1,{});console.log('ENGINE')}catch(e){console.log('ERR '+e.message)}",
                 NODE_DIR])
    lines = out.strip().splitlines()
    assert json.loads(lines[0]) == sorted(["createEngine", "submitRun", "summarize", "getSummary", "getText",
                                           "docStatus", "stats", "reset", "setMatrix", "getDeltas",
                                           "submitRunAsync", "summarizeAsync", "getContainingSegment", "getProps",
                                           "getRefPositions", "getRefInfo", "getRefStates", "getLeaves",
                                           "getRefKeys", "getViewLength", "replaySummaries"])
    if lines[1] != "ENGINE":  # no HIP device here: construction must throw, never fall back
        assert lines[1].startswith("ERR mtr_engine_create")


def _py_batch(paths, return_logs=False):
    it = Interner()
    logs = []
    for p in paths:
        groups = load_replay(p)
        log = replay_log(groups, it)
        for g in groups:
            for m in g["msgs"]:
                log.message(m, it)
        last = groups[-1]["msgs"][-1]
        log.seq_update(last["minimumSequenceNumber"], last["sequenceNumber"])
        logs.append(log)
    b = build_batch(logs, it)
    return (b, logs) if return_logs else b


def _py_batch_pre(paths, pre):
    """The --pre mode of tests/node/pack_batch.js: messages before startOrUpdateCollaboration, an
    undefined-id call (stays local), then a reconnect under a new id halfway (client.ts:1133-1155)."""
    it = Interner()
    logs = []
    for p in paths:
        groups = load_replay(p)
        log = DocLog()
        if groups[0]["initialText"]:
            log.local_insert(0, groups[0]["initialText"], it)
        msgs = [m for g in groups for m in g["msgs"]]
        for m in msgs[:pre]:
            log.message(m, it)
        log.start_collab(None)
        log.start_collab("A")
        half = pre + (len(msgs) - pre) // 2
        for m in msgs[pre:half]:
            log.message(m, it)
        log.start_collab("observer-2")
        for m in msgs[half:]:
            log.message(m, it)
        last = msgs[-1]
        log.seq_update(last["minimumSequenceNumber"], last["sequenceNumber"])
        logs.append(log)
    return build_batch(logs, it)


def test_start_collab_semantics():
    """addLongClientId always registers a new short id at startOrUpdateCollaboration (even for a known
    long id), an undefined id keeps the client local, a second id renames the observer."""
    it = Interner()
    log = DocLog()
    log.message({"clientId": "A", "type": "join", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                 "minimumSequenceNumber": 0}, it)
    log.start_collab(None)
    assert not log.collaborating and log.clients == ["A"]
    log.start_collab("A")
    assert log.clients == ["A", "A"] and log.client_ix["A"] == 1
    assert log.ops[-1][0] == abi.OP_START_COLLAB and log.ops[-1][2] == 1  # the op carries the new short id
    log.start_collab("B")
    assert log.clients == ["A", "B"] and log.client_ix["A"] == 1 and log.client_ix["B"] == 1
    assert log.observer_id == "B"
    n = len(log.ops)
    log.start_collab("C")  # renames again; never a second START_COLLAB record
    assert len(log.ops) == n and log.clients == ["A", "C"]


def test_client_cap_is_unsupported():
    it = Interner()
    log = DocLog()
    for i in range(MAX_CLIENTS):
        log.short_id(f"c{i}")
    with pytest.raises(Unsupported):
        log.short_id("one-too-many")


@pytest.mark.parametrize("pre", [-1, 5])
def test_js_packer_matches_python_packer(pre):
    paths = replay_files()[:6]
    _addon()
    js = json.loads(_node([os.path.join(HERE, "node", "pack_batch.js")] + (["--pre", str(pre)] if pre >= 0 else [])
                          + paths))
    raw = {k: base64.b64decode(v) for k, v in js.items()}
    py = _py_batch(paths) if pre < 0 else _py_batch_pre(paths, pre)

    def arr(name, dtype):
        return np.frombuffer(raw[name], dtype=dtype)

    assert raw["docs"] == py.docs.tobytes()
    assert raw["ops"] == py.ops.tobytes()
    n_text = int(py.docs["text_count"].sum())
    assert np.array_equal(arr("text", "<u2")[:n_text], py.text[:n_text])
    assert np.array_equal(arr("propopOff", "<u4"), py.propop_off)
    n_kv = 2 * int(py.propop_off[-1])
    assert np.array_equal(arr("propopKv", "<u4")[:n_kv], py.propop_kv[:n_kv])
    for off, data in (("keyOff", "keyBytes"), ("valOff", "valBytes"), ("clientOff", "clientBytes")):
        po = {"keyOff": py.key_off, "valOff": py.val_off, "clientOff": py.client_off}[off]
        pd = {"keyBytes": py.key_bytes, "valBytes": py.val_bytes, "clientBytes": py.client_bytes}[data]
        assert np.array_equal(arr(off, "<u4"), po)
        assert raw[data][: int(po[-1])] == pd.tobytes()[: int(po[-1])]
    n_keys, n_vals = len(py.key_off) - 1, len(py.val_off) - 1
    assert np.array_equal(arr("keyIndex", "<u4")[:n_keys], py.key_index[:n_keys])
    assert np.array_equal(arr("valEq", "<u4")[:n_vals], py.val_eq[:n_vals])


@pytest.mark.gpu
@pytest.mark.parametrize("parts, mode", [(4, "remote"), (16, "remote"), (16, "local")])
def test_replay_summaries_through_node_host(parts, mode, monkeypatch):
    """BatchReplayEngine.replaySummaries (mtr_replay_pipelined through the addon): the last group of every reference
    log applied, summarized and downloaded in one call on an engine holding the earlier groups; the records equal
    the oracle's blobs and the per-client summarize().  The remote-message batch takes the pipelined path; with a
    pending local insert queued (a record the pipelined path refuses) the addon takes the serial calls.  (30
    documents: MTR_PIPE_MIN_PART_DOCS=0 keeps the engine from taking the serial calls for ranges this small.)"""
    monkeypatch.setenv("MTR_PIPE_MIN_PART_DOCS", "0")
    paths = replay_files()
    _addon()
    res = json.loads(_node([os.path.join(HERE, "node", "replay_summaries.js"), str(parts), mode] + paths, timeout=300))
    assert res["checks"] == sum(len(load_replay(p)) for p in paths) - (mode == "local")
    assert res["pipelined"] is (mode == "remote")
    b = _py_batch(paths)
    for r in res["result"]:
        orc = OracleDoc(options())
        assert orc.apply(b, r["doc"]) == 0
        assert [base64.b64decode(x) for x in r["blobs"]] == orc.summarize(b, r["doc"]), f"doc {r['doc']}"
        assert r["same_as_summarize"]


@pytest.mark.gpu
def test_replay_logs_through_node_host():
    paths = replay_files()
    _addon()
    res = json.loads(_node([os.path.join(HERE, "node", "replay_engine.js")] + paths, timeout=300))
    assert res["checks"] == sum(len(load_replay(p)) for p in paths)
    b = _py_batch(paths)
    for r in res["result"]:
        orc = OracleDoc(options())
        assert orc.apply(b, r["doc"]) == 0
        exp = orc.summarize(b, r["doc"])
        got = [base64.b64decode(x) for x in r["blobs"]]
        assert got == exp, f"doc {r['doc']}: summary bytes differ"
        assert r["names"] == ["header"] + [f"body_{i}" for i in range(len(got) - 1)]


@pytest.mark.gpu
def test_legacy_catchup_through_node_host(tmp_path):
    """Legacy summaries with catch-up ops from BatchReplayClient (its own messages-since-MSN list,
    rebuilt from the engine's delta ranges) equal the Python mirror driven by the oracle."""
    from test_catchup import LEGACY, OracleReplica, messages_from_batch
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    _addon()
    cfg = make_cfg(6, 700, writers=8, max_lag=32)
    tabs = tables(writers=8)
    gb, _, status = generate(cfg, tabs, 0, 6, threads=6, opts=options(**LEGACY))
    assert (status == 0).all()
    docs = [dict(zip(("observer", "msgs"), messages_from_batch(gb, d))) for d in range(6)]
    f = tmp_path / "docs.json"
    f.write_text(json.dumps(docs))
    res = json.loads(_node([os.path.join(HERE, "node", "catchup_engine.js"), str(f), "113"], timeout=300))
    for d, r in enumerate(res):
        ref = OracleReplica()
        ref.log.start_collab(docs[d]["observer"])
        msgs = docs[d]["msgs"]
        for k in range(0, len(msgs), 113):
            for m in msgs[k:k + 113]:
                ref.log.message(m, ref.it)
            ref.flush()
        exp = ref.summary()
        got = [base64.b64decode(x) for x in r["blobs"]]
        assert r["names"][-1] == "catchupOps" and len(got) == len(exp)
        assert got == exp, f"doc {d}: legacy summary with catch-up differs"
        assert r["text"] == ref.doc.text()


def _compare_batch(raw, py):
    assert raw["docs"] == py.docs.tobytes()
    assert raw["ops"] == py.ops.tobytes()
    assert np.array_equal(np.frombuffer(raw["clientOff"], dtype="<u4"), py.client_off)
    n = int(py.client_off[-1])
    assert raw["clientBytes"][:n] == py.client_bytes.tobytes()[:n]


def _matrix_feeds(n, ops):
    from test_matrix import matrix_cfg, matrix_messages
    from fluidframework_amd.synth import tables
    from oracle.oracle import generate_matrix

    gb, _, status = generate_matrix(matrix_cfg(n, ops, writers=8, max_lag=16), tables(writers=8), 0, n, threads=n)
    assert (status == 0).all()
    return [dict(zip(("observer", "msgs"), matrix_messages(gb, d, np.random.default_rng(d)))) for d in range(n)]


def test_js_matrix_packer_matches_python_packer(tmp_path):
    """MatrixDocLog + matrixLogs (the Node SharedMatrix packer) produce the batch MatrixLog + matrix_logs do:
    vector ops (single and grouped) with F_COLS, set-cell records, the shared client table."""
    from fluidframework_amd.batch import MatrixLog, matrix_logs

    _addon()
    feeds = _matrix_feeds(4, 600)
    f = tmp_path / "feeds.json"
    f.write_text(json.dumps(feeds))
    raw = {k: base64.b64decode(v) for k, v in json.loads(_node([os.path.join(HERE, "node", "matrix_engine.js"),
                                                                 "--pack", str(f)])).items()}
    it = Interner()
    logs = []
    for fd in feeds:
        lg = MatrixLog()
        lg.start_collab(fd["observer"])
        for m in fd["msgs"]:
            lg.message(m, it)
        logs.append(lg)
    py = build_batch(matrix_logs(logs), it)
    assert py.n_docs == 8 and int(py.docs["op_count"][1::2].sum()) == 0
    _compare_batch(raw, py)


@pytest.mark.gpu
def test_matrix_through_node_host(tmp_path):
    """BatchMatrixClient: C4-mix matrices applied in chunks through Node; both PermutationVectors'
    summaries (segments + handleTable) equal the oracle's."""
    from oracle.oracle import OracleDoc
    from fluidframework_amd.batch import MatrixLog

    _addon()
    feeds = _matrix_feeds(6, 1500)
    f = tmp_path / "feeds.json"
    f.write_text(json.dumps(feeds))
    res = json.loads(_node([os.path.join(HERE, "node", "matrix_engine.js"), "--run", str(f), "389"], timeout=300))
    for d, fd in enumerate(feeds):
        it = Interner()
        lg = MatrixLog()
        lg.start_collab(fd["observer"])
        for m in fd["msgs"]:
            lg.message(m, it)
        b = build_batch([lg], it)
        o = OracleDoc(options(), matrix=True)
        assert o.apply(b, 0) == 0
        for w, name in ((0, "rows"), (1, "cols")):
            got = [base64.b64decode(x) for x in res[d][name]]
            assert got == o.select(w).summarize(b, 0), f"matrix {d} {name}: summary differs"


@pytest.mark.gpu
def test_async_host_and_containing_segment(tmp_path):
    """flushAsync / summarizeAsync (napi_async_work + promises): the engine is refused while a run is in
    flight, the event loop keeps turning, texts and summaries equal the oracle's; getContainingSegment
    with and without sequenceArgs equals the oracle's nodeMap at every queried (pos, refSeq, client)."""
    import random

    paths = [p for p in replay_files() if "clients_8" in p][:4] or replay_files()[:4]
    _addon()
    b, logs = _py_batch(paths, return_logs=True)
    rng = random.Random(11)
    queries, expect = [], []
    for d, log in enumerate(logs):
        o = OracleDoc(options())
        assert o.apply(b, d) == 0
        min_seq, cur = (int(x) for x in o.state()[:2])
        clients = [c for c, name in enumerate(log.clients) if log.client_ix[name] == c]
        qs, ex = [], []
        for _ in range(80):
            ref, c = rng.randint(min_seq, cur), rng.choice(clients)
            pos = rng.randint(0, max(int(o.length(ref, c)), 0))
            qs.append([pos, ref, log.clients[c]])
            ex.append(o.containing(pos, ref, c))
        me = log.client_ix[log.observer_id]
        for pos in (0, len(o.text()) // 2, len(o.text())):  # no sequenceArgs: the observer's current view
            qs.append([pos])
            ex.append(o.containing(pos, cur, me))
        queries.append(qs)
        expect.append(ex)
    f = tmp_path / "queries.json"
    f.write_text(json.dumps(queries))
    res = json.loads(_node([os.path.join(HERE, "node", "async_engine.js"), str(f)] + paths, timeout=300))
    assert res["checks"] == sum(len(load_replay(p)) for p in paths)
    assert res["busy"] > 0
    n_hit = 0
    for r, ex in zip(res["result"], expect):
        orc = OracleDoc(options())
        assert orc.apply(b, r["doc"]) == 0
        assert [base64.b64decode(x) for x in r["blobs"]] == orc.summarize(b, r["doc"])
        for got, e in zip(r["answers"], ex):
            if e[0] < 0:
                assert got is None
                continue
            assert got is not None and got[:3] == [e[0], e[1], e[2]], (r["doc"], got, e)
            assert got[3] in (-1, e[2])  # text segments carry their text
            n_hit += 1
    assert n_hit > 250


def _writer_events(groups, writer):
    """client.replay.spec.ts:41-68 from one writer's side: its op as a local op right after it caught
    up to the op's referenceSequenceNumber, every sequenced message in order (its own are acks)."""
    events, queue, cur = [], [], 0
    for g in groups:
        for m in g["msgs"]:
            if m["clientId"] == writer:
                while queue and m["referenceSequenceNumber"] > cur:
                    x = queue.pop(0)
                    events.append({"msg": x})
                    cur = x["sequenceNumber"]
                events.append({"local": m["contents"]})
            queue.append(m)
        while queue:
            x = queue.pop(0)
            events.append({"msg": x})
            cur = x["sequenceNumber"]
    return events


def test_js_local_op_packer_matches_python_packer(tmp_path):
    """Local ops while collaborating (seq = UnassignedSequenceNumber records) and acks of this client's
    own messages: the Node packer's arrays equal the Python packer's."""
    from fixtures import replay_writers

    _addon()
    feeds = []
    for p in replay_files()[3:6]:
        groups = load_replay(p)
        for w in replay_writers(groups)[:2]:
            feeds.append({"observer": w, "events": _writer_events(groups, w)})
    path = tmp_path / "feeds.json"
    path.write_text(json.dumps(feeds))
    js = json.loads(_node([os.path.join(HERE, "node", "pack_events.js"), str(path)]))
    raw = {k: base64.b64decode(v) for k, v in js.items()}
    it = Interner()
    logs = []
    for f in feeds:
        log = DocLog()
        log.start_collab(f["observer"])
        for ev in f["events"]:
            if "local" in ev:
                log.local_op(ev["local"], it)
            else:
                log.message(ev["msg"], it)
        logs.append(log)
    py = build_batch(logs, it)
    assert int((py.ops["type"] == 17).sum()) > 0 and int((py.ops["seq"] == -1).sum()) > 0
    assert raw["docs"] == py.docs.tobytes()
    assert raw["ops"] == py.ops.tobytes()
    n_kv = 2 * int(py.propop_off[-1])
    assert np.array_equal(np.frombuffer(raw["propopKv"], "<u4")[:n_kv], py.propop_kv[:n_kv])


# ---------------------------------------------------------------- Client.load in the Node host
def _load_inputs():
    """Every snapshot fixture, plus V1 summaries the oracle takes mid-collaboration of three replay logs."""
    from fixtures import SNAPSHOT_VERSIONS, blob_names, load_snapshots

    docs = [{"key": k, "blobs": v, "id": "snapshot", "v1": int(SNAPSHOT_VERSIONS[k.split("/")[0]])}
            for k, v in sorted(load_snapshots().items())]
    for p in [p for p in replay_files() if "clients_8" in p][:3]:
        groups = load_replay(p)
        it = Interner()
        log = replay_log(groups, it)
        for g in groups[: len(groups) // 2]:
            for m in g["msgs"]:
                log.message(m, it)
        orc = OracleDoc(options())
        b = build_batch([log], it)
        assert orc.apply(b, 0) == 0
        blobs = orc.summarize(b, 0)
        docs.append({"key": os.path.basename(p), "blobs": dict(zip(blob_names(len(blobs), True),
                                                                   [x.decode() for x in blobs])), "id": "loader-B", "v1": 1})
    return docs


def test_js_load_packer_matches_python_packer(tmp_path):
    """BatchReplayClient.load's records (index.js DocLog.loadSummary) equal the Python host's
    (DocLog.load_summary) for every snapshot fixture and mid-collaboration summary: the same header / body
    segment records, merge info, removedClientIds, client table and property tables."""
    _addon()
    docs = _load_inputs()
    f = tmp_path / "summaries.json"
    f.write_text(json.dumps([{"blobs": d["blobs"], "id": d["id"]} for d in docs]))
    js = json.loads(_node([os.path.join(HERE, "node", "pack_load.js"), str(f)]))
    it = Interner()
    logs, catchup = [], []
    for d in docs:
        log = DocLog()
        catchup.append(len(log.load_summary(d["blobs"], d["id"], it)))
        logs.append(log)
    py = build_batch(logs, it)
    assert js["catchup"] == catchup
    raw = {k: base64.b64decode(v) for k, v in js.items() if k != "catchup"}
    assert raw["docs"] == py.docs.tobytes()
    assert raw["ops"] == py.ops.tobytes()
    n_text = int(py.docs["text_count"].sum())
    assert np.array_equal(np.frombuffer(raw["text"], "<u2")[:n_text], py.text[:n_text])
    n_kv = 2 * int(py.propop_off[-1])
    assert np.array_equal(np.frombuffer(raw["propopKv"], "<u4")[:n_kv], py.propop_kv[:n_kv])
    assert raw["clientBytes"][: int(py.client_off[-1])] == py.client_bytes.tobytes()[: int(py.client_off[-1])]


@pytest.mark.gpu
def test_load_through_node_host(tmp_path):
    """Client.load through N-API -> C ABI -> HIP: every snapshot fixture loads and summarizes back to its own
    bytes; a V1 summary taken mid-collaboration of each of 30 replay logs loads into a second client that then
    reads resultText after every remaining group, and ends with the same summary as the oracle's replay."""
    _addon()
    from fixtures import SNAPSHOT_VERSIONS, blob_names, load_snapshots

    fx = [{"key": k, "blobs": v, "v1": int(SNAPSHOT_VERSIONS[k.split("/")[0]])}
          for k, v in sorted(load_snapshots().items())]
    f = tmp_path / "fixtures.json"
    f.write_text(json.dumps(fx))
    paths = replay_files()
    res = json.loads(_node([os.path.join(HERE, "node", "load_engine.js"), str(f)] + paths, timeout=600))
    want = {d["key"]: d for d in fx}
    assert len(res["fixtures"]) == len(fx)
    for r in res["fixtures"]:
        got = [base64.b64decode(x).decode() for x in r["blobs"]]
        assert dict(zip(r["names"], got)) == want[r["key"]]["blobs"], r["key"]
    assert res["checks"] == sum(2 * (len(g) - len(g) // 2) for g in (load_replay(p) for p in paths))
    for r, p in zip(res["logs"], paths):  # the oracle does the same: replay to the middle, summarize, load, go on
        groups = load_replay(p)
        cut = len(groups) // 2
        it = Interner()
        la = replay_log(groups, it)
        for g in groups[:cut]:
            for m in g["msgs"]:
                la.message(m, it)
        last = groups[cut - 1]["msgs"][-1]
        la.seq_update(last["minimumSequenceNumber"], last["sequenceNumber"])
        a = OracleDoc(options())
        b0 = build_batch([la], it)
        assert a.apply(b0, 0) == 0
        mid = a.summarize(b0, 0)
        assert [base64.b64decode(x) for x in r["mid"]] == mid, f"log {r['log']}: mid summary"
        lb = DocLog()
        lb.load_summary(dict(zip(blob_names(len(mid), True), [x.decode() for x in mid])), "loader-B", it)
        for g in groups[cut:]:
            for m in g["msgs"]:
                lb.message(m, it)
        last = groups[-1]["msgs"][-1]
        lb.seq_update(last["minimumSequenceNumber"], last["sequenceNumber"])
        ob = OracleDoc(options())
        bb = build_batch([lb], it)
        assert ob.apply(bb, 0) == 0
        assert [base64.b64decode(x) for x in r["b"]] == ob.summarize(bb, 0), f"log {r['log']}: loaded client's summary"


def _interval_sessions():
    """Interval sessions for the Node host: the four fixture loads, the detached recipe, and two farms."""
    import interval_farm as F
    from fixtures import load_snapshots, snapshot_recipe

    snaps = load_snapshots()
    out = []
    for name in F.FIXTURES:
        out.append({"header": F.HEADERS[name], "blobs": snaps[name], "want": F.V2_HEADER})
    out.append({"local": [[o[1], o[2]] for o in snapshot_recipe("withIntervals")],
                "adds": [list(x) for x in F.fixture_ids()], "want": F.V2_HEADER})
    for seed in (1, 2):
        init, msgs, obs = F.farm(seed)
        out.append({"initial": init, "msgs": msgs, "want": obs.summarize_header(), "text": obs.text()})
    return out


def test_js_interval_host_matches_python_host(tmp_path):
    """The Node host's interval collections (intervals.js) pack the same records as the Python host
    (fluidframework_amd/intervals.py) for the fixture loads, the detached recipe and two farms, and -- given the
    CPU oracle's reference states for those records -- write the oracle's `header` blob."""
    _addon()
    import interval_farm as F

    sessions = _interval_sessions()
    py = []
    for s in sessions:
        h = F.HostString("oracle")
        if "header" in s:
            h.log.load(s["blobs"], "loader", h.it, header=s["header"])
        for pos, text in s.get("local", []):
            h.log.local_insert(pos, text, h.it)
        for label, a, b, t, i in s.get("adds", []):
            h.log.interval_collection(label).local_add(h.log, a, b, t, {"intervalId": i})
        if "initial" in s:
            h.log.local_insert(0, s["initial"], h.it)
            h.log.start_collab("observer")
        for m in s.get("msgs", []):
            h.log.message(dict(m), h.it)
        b = build_batch([h.log], h.it)
        doc = OracleDoc(options())
        assert doc.apply(b, 0) == 0
        s["states"] = [x for st in doc.ref_states() for x in st]
        py.append((b, h.log.interval_header(doc.ref_states()).decode()))
    f = tmp_path / "sessions.json"
    f.write_text(json.dumps(sessions))
    js = json.loads(_node([os.path.join(HERE, "node", "intervals_pack.js"), str(f)]))
    for s, (b, header), j in zip(sessions, py, js):
        assert base64.b64decode(j["ops"]) == b.ops.tobytes()
        assert base64.b64decode(j["docs"]) == b.docs.tobytes()
        assert j["header"] == header == s["want"]


@pytest.mark.gpu
def test_intervals_through_node_host(tmp_path):
    """Interval collections through N-API -> C ABI -> HIP: the fixtures load and summarize back to their V2 header,
    the detached recipe writes it, and two farms' observers write the oracle's header and text."""
    _addon()
    sessions = _interval_sessions()
    f = tmp_path / "sessions.json"
    f.write_text(json.dumps(sessions))
    res = json.loads(_node([os.path.join(HERE, "node", "intervals_engine.js"), str(f)], timeout=600))
    for s, r in zip(sessions, res):
        assert r["header"] == s["want"]
        if "text" in s:
            assert r["text"] == s["text"]


@pytest.mark.gpu
def test_interval_live_ops_through_node_host():
    """A collaborating client's own interval ops (add / change / changeProperties / delete, their acks, reconnect
    rebasing) through the Node host, N-API -> C ABI -> HIP: known answers of intervalCollection.spec.ts (the same cases
    tests/test_interval_live.py runs through the Python host)."""
    _addon()
    res = json.loads(_node([os.path.join(HERE, "node", "interval_live.js")], timeout=600))
    assert res and all(v == "ok" for v in res.values()), res


@pytest.mark.gpu
def test_live_legacy_catchup_through_node_host(tmp_path):
    """Legacy-format collaborating clients (own acked messages in the catch-up list, sequence.ts:697-736 with
    local = true) through the Node host: every client's summary blobs (header, body, catchupOps) equal the
    oracle-driven Python host's on the same script (tests/test_catchup_live.py)."""
    from mock_runtime import OracleExecutor
    from test_catchup_live import farm_script, replay

    _addon()
    script = farm_script(3)
    f = tmp_path / "script.json"
    f.write_text(json.dumps(script))
    res = json.loads(_node([os.path.join(HERE, "node", "catchup_live.js"), str(f)], timeout=600))
    _, want = replay(OracleExecutor(legacy=True), script)
    assert res["texts"] == [r.dds.get_text() for r in want]
    for got, r in zip(res["summaries"], want):
        exp = r.dds.summary()
        assert got[0][0] == "header" and got[-1][0] == "catchupOps"
        assert [v.encode() for _, v in got] == exp


@pytest.mark.gpu
def test_reference_churn_through_node_host():
    """Reference-id recycling through the Node host (VERDICT r05 Next #3): tests/node/interval_churn.js runs
    test_interval_live.churn's script (same PRNG) on an engine whose reference table holds 64 ids -- 320 endpoint
    changes and 320 queries per client; every checkpoint's text and interval positions equal the oracle-driven
    Python run's, and the id high-water mark stays within the table."""
    from mock_runtime import Factory, OracleExecutor
    from test_interval_live import churn

    _addon()
    res = json.loads(_node([os.path.join(HERE, "node", "interval_churn.js"), "160"], timeout=600))
    want, _ = churn(Factory(OracleExecutor()), 160)
    assert [[t, [[list(p) for p in ps] for ps in pss]] for t, pss in want] == res["out"]
    assert max(res["nRefs"]) <= 64
