"""Combining annotate ops and relative positions.

Combining ops: PropertiesManager.addProperties (segmentPropertiesManager.ts:60-157) with the op's
combiningOp, for an observer (every key is modified: no pending local keys):

* "rewrite" deletes the old keys whose new value is absent or falsy (`!newProps[key]`, :109-123), then
  assigns as usual -- a falsy non-null value is deleted and re-added, so it moves to the end;
* any other name ignores the op's values: newValue = combine(op, previousValue, undefined, seq)
  (:145-147, properties.ts:24-69).  "incr" gives `prev + undefined` = NaN (JSON null; NaN never
  matches, so such segments never merge); "consensus" on an absent key gives {value: undefined, seq}
  (JSON {"seq":N}, never matching either) and keeps a present value; other names keep a present value
  and take the default when absent.

Relative positions: getValidOpRange -> posFromRelativePos (client.ts:527-545, mergeTree.ts:1371-1395):
the marker's getPosition at the op's (refSeq, clientId), + cachedLength + offset unless `before`
(- offset); a marker zamboni unlinked is at 0.

The expected values below are derived by hand from those lines (JavaScript semantics written next
to each case).  CPU: the oracle.  GPU: the HIP engine against the oracle (summary bytes), the same
cases plus seeded documents whose ops were rewritten to use combining ops / relative positions.
"""
import json
import random

import numpy as np
import pytest

from fluidframework_amd import abi
from fluidframework_amd.batch import DocLog, Interner, Unsupported, build_batch
from oracle.oracle import OracleDoc, options

OBS = "observer"


def msg(client, seq, ref, contents, msn=0):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


def ins(client, seq, ref, pos, seg, msn=0):
    return msg(client, seq, ref, {"type": 0, "pos1": pos, "seg": seg}, msn)


def ann(client, seq, ref, start, end, props, co=None, msn=0):
    c = {"type": 2, "pos1": start, "pos2": end, "props": props}
    if co is not None:
        c["combiningOp"] = co
    return msg(client, seq, ref, c, msn)


def noop(seq, msn):
    return {"clientId": "Z", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
            "minimumSequenceNumber": msn, "type": "noop", "contents": None}


def run_oracle(msgs, opts=None):
    it = Interner()
    log = DocLog()
    log.start_collab(OBS)
    for m in msgs:
        log.message(m, it)
    b = build_batch([log], it)
    o = OracleDoc(opts or options())
    st = o.apply(b, 0)
    return o, b, st


def segments(o, b):
    """The V1 header's segment specs (everything below the MSN: plain toJSONObject specs)."""
    blobs = o.summarize(b, 0)
    return json.loads(blobs[0])["segments"]


# (name, messages, expected segments after the MSN passed every op)
KATS = [
    ("incr makes NaN (JSON null) and NaN never merges", [
        ins("A", 1, 0, 0, "abc"),
        ann("B", 2, 1, 0, 3, {"n": 5}),
        # combine({name:"incr"}, 5, undefined) = 5 + undefined = NaN
        ann("C", 3, 2, 1, 2, {"n": 1}, {"name": "incr"}),
        noop(4, 3)],
     [{"text": "a", "props": {"n": 5}}, {"text": "b", "props": {"n": None}}, {"text": "c", "props": {"n": 5}}]),
    ("incr over a whole range: NaN neighbours stay apart", [
        ins("A", 1, 0, 0, "ab"), ins("A", 2, 1, 2, "cd"),
        ann("B", 3, 2, 0, 4, {"k": 1}, {"name": "incr", "defaultValue": 10, "minValue": 100}),
        noop(4, 3)],
     # absent: 10 + undefined = NaN (NaN < 100 is false: no clamp)
     [{"text": "ab", "props": {"k": None}}, {"text": "cd", "props": {"k": None}}]),
    ("incr of a string default concatenates", [
        ins("A", 1, 0, 0, "xy"),
        ann("B", 2, 1, 0, 2, {"s": 0}, {"name": "incr", "defaultValue": "v"}),
        noop(3, 2)],
     # "v" + undefined = "vundefined": a plain value, equal on both halves (no split here)
     [{"text": "xy", "props": {"s": "vundefined"}}]),
    ("consensus: absent -> {value: undefined, seq}, present kept", [
        ins("A", 1, 0, 0, "abcd"),
        ann("B", 2, 1, 2, 4, {"c": 7}),
        ann("C", 3, 2, 1, 3, {"c": "ignored"}, {"name": "consensus"}),
        noop(4, 3)],
     # "c" keeps 7 and merges back with "d" once below the MSN; "a" has no props: a plain string spec
     ["a", {"text": "b", "props": {"c": {"seq": 3}}}, {"text": "cd", "props": {"c": 7}}]),
    ("consensus with a default object whose seq is -1", [
        ins("A", 1, 0, 0, "ab"),
        ann("B", 2, 1, 0, 2, {"c": 0}, {"name": "consensus", "defaultValue": {"value": 4, "seq": -1}}),
        noop(3, 2)],
     # cv = defaultValue; cv.seq === -1 -> cv.seq = 2 (key order kept)
     [{"text": "ab", "props": {"c": {"value": 4, "seq": 2}}}]),
    ("other names keep present values and take the default", [
        ins("A", 1, 0, 0, "abc"),
        ann("B", 2, 1, 0, 1, {"m": 1}),
        ann("C", 3, 2, 0, 3, {"m": 99, "z": 5}, {"name": "max", "defaultValue": 3}),
        noop(4, 3)],
     [{"text": "a", "props": {"m": 1, "z": 3}}, {"text": "bc", "props": {"m": 3, "z": 3}}]),
    ("rewrite deletes absent / falsy old keys; falsy values move to the end", [
        ins("A", 1, 0, 0, "ab"),
        ann("B", 2, 1, 0, 2, {"a": 1, "b": 2, "c": 0, "e": "keep?"}),
        # old [a, b, c, e]: !newProps[a] (absent), !newProps[c] (0) and !newProps[e] (null) delete;
        # then b = 3 in place, c = 0 re-added last, d = "" added
        ann("C", 3, 2, 0, 1, {"b": 3, "c": 0, "d": "", "e": None}, {"name": "rewrite"}),
        noop(4, 3)],
     [{"text": "a", "props": {"b": 3, "c": 0, "d": ""}}, {"text": "b", "props": {"a": 1, "b": 2, "c": 0, "e": "keep?"}}]),
    ("rewrite with index-like keys keeps JS own-key order", [
        ins("A", 1, 0, 0, "q"),
        ann("B", 2, 1, 0, 1, {"x": 1, "7": 2, "2": 3}),
        ann("C", 3, 2, 0, 1, {"7": 0, "x": 5, "3": True}, {"name": "rewrite"}),
        noop(4, 3)],
     # old keys in order ["2","7","x"]: "2" absent -> deleted; "7" -> 0 falsy -> deleted then re-added
     [{"text": "q", "props": {"3": True, "7": 0, "x": 5}}]),
]


@pytest.mark.parametrize("name,msgs,expect", KATS, ids=[k[0] for k in KATS])
def test_combining_kats_oracle(name, msgs, expect):
    o, b, st = run_oracle(msgs)
    assert st == 0
    assert segments(o, b) == expect


def test_combining_unsupported_cases():
    it = Interner()
    log = DocLog()
    log.start_collab(OBS)
    with pytest.raises(Unsupported):  # a name without a default leaves an explicit undefined property
        log.message(ann("B", 1, 0, 0, 1, {"k": 1}, {"name": "whatever"}), it)
    log = DocLog()
    log.start_collab(OBS)
    with pytest.raises(Unsupported):  # consensus on a null default throws in the reference
        log.message(ann("B", 1, 0, 0, 1, {"k": 1}, {"name": "consensus", "defaultValue": None}), it)
    # incr of a present string value: the engine and the oracle mark the document unsupported
    o, b, st = run_oracle([ins("A", 1, 0, 0, "ab"), ann("B", 2, 1, 0, 2, {"s": "x"}),
                           ann("C", 3, 2, 0, 1, {"s": 1}, {"name": "incr"})])
    assert st == abi.MTR_ERR_UNSUPPORTED


def marker(mid, ref_type=1):
    return {"marker": {"refType": ref_type}, "props": {"markerId": mid}}


RELPOS_KATS = [
    ("insert after a marker with offset", [
        ins("A", 1, 0, 0, marker("m1")), ins("A", 2, 1, 1, "hello"),
        # getPosition(m1) = 0; !before: 0 + 1 (cachedLength) + 2
        msg("B", 3, 2, {"type": 0, "relativePos1": {"id": "m1", "offset": 2}, "seg": "X"})],
     "heXllo"),
    ("remove relative to markers before / after", [
        ins("A", 1, 0, 0, "abcdef"), ins("A", 2, 1, 3, marker("p")), ins("A", 3, 2, 7, marker("q")),
        # p at 3 (before -> 3 - 1 = 2), q at 7 (before, no offset -> 7): remove [2, 7) = "c" p "def"
        msg("B", 4, 3, {"type": 1, "relativePos1": {"id": "p", "before": True, "offset": 1},
                        "relativePos2": {"id": "q", "before": True}})],
     "ab"),
    ("pos1 wins over relativePos1; the view of the op's refSeq", [
        ins("A", 1, 0, 0, "abc"), ins("A", 2, 1, 1, marker("m")),
        ins("C", 3, 2, 0, "ZZ"),
        # B has not seen seq 3: m is at 1 in its view -> pos 1 + 1 = 2 -> after "a" + marker
        msg("B", 4, 2, {"type": 0, "relativePos1": {"id": "m"}, "seg": "Y"}),
        msg("B", 5, 4, {"type": 0, "pos1": 0, "relativePos1": {"id": "m"}, "seg": "W"})],
     "WZZaYbc"),
    ("annotate between two markers", [
        ins("A", 1, 0, 0, "xyz"), ins("A", 2, 1, 0, marker("s")), ins("A", 3, 2, 4, marker("e")),
        msg("B", 4, 3, {"type": 2, "relativePos1": {"id": "s"}, "relativePos2": {"id": "e", "before": True},
                        "props": {"bold": True}})],
     "xyz"),
]


@pytest.mark.parametrize("name,msgs,text", RELPOS_KATS, ids=[k[0] for k in RELPOS_KATS])
def test_relpos_kats_oracle(name, msgs, text):
    o, b, st = run_oracle(msgs)
    assert st == 0
    assert o.text() == text
    assert int((b.ops["type"] == abi.OP_RELPOS).sum()) >= 1


def test_relpos_annotate_range_props():
    o, b, st = run_oracle(RELPOS_KATS[3][1] + [noop(5, 4)])
    assert st == 0
    segs = segments(o, b)
    assert {"text": "xyz", "props": {"bold": True}} in segs


def test_relpos_unlinked_marker_is_at_zero():
    """A removed marker unlinked by zamboni keeps its idToSegment entry: getPosition walks no parent."""
    msgs = [ins("A", 1, 0, 0, "abcdef"), ins("A", 2, 1, 4, marker("m")),
            msg("A", 3, 2, {"type": 1, "pos1": 4, "pos2": 5}),
            noop(4, 3),  # MSN passes the remove: zamboni unlinks the marker
            msg("B", 5, 4, {"type": 0, "relativePos1": {"id": "m", "offset": 1}, "seg": "Q"}, msn=3)]
    o, b, st = run_oracle(msgs)
    assert st == 0
    assert o.text() == "abQcdef"  # getPosition 0, + cachedLength 1 + offset 1


def test_relpos_unsupported_cases():
    it = Interner()
    log = DocLog()
    log.start_collab(OBS)
    with pytest.raises(Unsupported):  # no marker was ever mapped to the id: position -1
        log.message(msg("B", 1, 0, {"type": 0, "relativePos1": {"id": "nope"}, "seg": "x"}), it)
    log = DocLog()
    log.start_collab(OBS)
    log.message(ins("A", 1, 0, 0, marker("d")), it)
    log.message(ins("A", 2, 1, 0, marker("d")), it)  # the same id twice: blockUpdate order decides
    with pytest.raises(Unsupported):
        log.message(msg("B", 3, 2, {"type": 0, "relativePos1": {"id": "d"}, "seg": "x"}), it)
    log = DocLog()
    log.start_collab(OBS)
    log.message(ins("A", 1, 0, 0, marker("e")), it)
    log.message(ann("A", 2, 1, 0, 1, {"markerId": "f"}), it)  # annotated ids are remapped by blockUpdate
    with pytest.raises(Unsupported):
        log.message(msg("B", 3, 2, {"type": 0, "relativePos1": {"id": "e"}, "seg": "x"}), it)


# ---------------------------------------------------------------- seeded documents
def rewritten_feed(n_ops, seed, relpos=True, combining=True):
    """A seeded C3-style document re-expressed with markers carrying ids (in place of one-unit text
    inserts), relative positions equal to the original positions (offsets from the oracle's
    getPosition at each op's view) and combining annotates.  Independent random streams per rewrite,
    so turning one off leaves the others' choices unchanged.  Returns (observer, messages)."""
    from test_catchup import messages_from_batch
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate

    cfg = make_cfg(1, n_ops, writers=6, max_lag=24, seed=seed, weights=(50, 25, 25))
    gb, _, status = generate(cfg, tables(writers=6), 0, 1, threads=1)
    assert (status == 0).all()
    observer, msgs = messages_from_batch(gb, 0)
    r_mark, r_rel, r_comb = random.Random(seed), random.Random(seed + 1000), random.Random(seed + 2000)
    out, n_mark = [], 0
    it = Interner()
    log = DocLog()
    log.start_collab(observer)
    o = OracleDoc(options())
    for m in msgs:
        c = m["contents"]
        if m.get("type") == "op" and isinstance(c, dict) and c.get("type") in (0, 1, 2):
            c = json.loads(json.dumps(c))
            if c["type"] == 0 and isinstance(c["seg"], str) and len(c["seg"]) == 1 and r_mark.random() < 0.3:
                c["seg"] = marker("k%d" % n_mark, ref_type=r_mark.choice([0, 1, 2]))
                n_mark += 1
            if relpos and n_mark and r_rel.random() < 0.3:
                b = build_batch([log], it)  # the oracle up to the previous message
                assert o.apply(b, 0) == 0
                client = log.short_id(m["clientId"])
                for key in (["pos1"] if c["type"] == 0 else ["pos1", "pos2"]):
                    k = r_rel.randrange(n_mark)
                    mp = o.marker_position(k, m["referenceSequenceNumber"], client)
                    if mp < 0:
                        continue
                    pos = c[key]
                    rel = {"id": "k%d" % k}
                    if pos >= mp + 1:
                        if pos > mp + 1 or r_rel.random() < 0.5:
                            rel["offset"] = pos - mp - 1
                    else:
                        rel["before"] = True
                        rel["offset"] = mp - pos
                    del c[key]
                    c["relative" + key[0].upper() + key[1:]] = rel
            if combining and c["type"] == 2 and r_comb.random() < 0.5:
                name = r_comb.choice(["incr", "consensus", "rewrite", "max"])
                co = {"name": name}
                if name == "incr":
                    c["props"] = {"size": 1} if r_comb.random() < 0.7 else {"size": 1, "bold": 0}
                    if r_comb.random() < 0.3:  # (a string result would make a later incr unsupported)
                        co["defaultValue"] = r_comb.choice([1, True])
                elif name == "consensus" and r_comb.random() < 0.4:
                    co["defaultValue"] = r_comb.choice([5, {"value": 1, "seq": -1}])
                elif name == "max":
                    co["defaultValue"] = r_comb.choice([1, 0, None])
                c["combiningOp"] = co
            m = dict(m, contents=c)
        log.message(m, it)
        out.append(m)
    return observer, out


def _replay(observer, msgs, chunk):
    it = Interner()
    log = DocLog()
    log.start_collab(observer)
    o = OracleDoc(options())
    batches = []
    for k in range(0, len(msgs), chunk):
        for m in msgs[k:k + chunk]:
            log.message(m, it)
        b = build_batch([log], it)
        st = o.apply(b, 0)
        batches.append(b)
        if st:
            return o, batches, st
    return o, batches, 0


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_rewritten_documents_oracle(seed):
    """Relative positions that restate the original positions change nothing: the text equals the
    replay without them; with combining annotates too the replay runs without errors."""
    observer, msgs = rewritten_feed(500, seed, combining=False)
    assert sum(1 for m in msgs if isinstance(m["contents"], dict) and
               ("relativePos1" in m["contents"] or "relativePos2" in m["contents"])) > 10
    o, _, st = _replay(observer, msgs, 97)
    assert st == 0
    obs2, msgs2 = rewritten_feed(500, seed, relpos=False, combining=False)
    o2, _, st2 = _replay(obs2, msgs2, 97)
    assert st2 == 0 and o2.text() == o.text()
    observer, msgs = rewritten_feed(500, seed)
    o3, _, st3 = _replay(observer, msgs, 97)
    assert st3 == 0


@pytest.mark.gpu
def test_combining_and_relpos_engine_matches_oracle():
    """The KATs and seeded rewritten documents through the HIP engine, in chunks: status, text and
    summary bytes equal the oracle's after every chunk."""
    from fluidframework_amd.engine import Engine

    feeds = [(OBS, k[1]) for k in KATS] + [(OBS, k[1]) for k in RELPOS_KATS]
    feeds.append((OBS, RELPOS_KATS[3][1] + [noop(5, 4)]))
    for seed in range(1, 7):
        feeds.append(rewritten_feed(500, seed))
    n = len(feeds)
    eng = Engine(n, max_segments=4096, heap_entries=4096, text_units=1 << 16, prop_words=1 << 16,
                 remover_cells=4096, ops_per_launch=16)
    it = Interner()
    logs = []
    for observer, _ in feeds:
        lg = DocLog()
        lg.start_collab(observer)
        logs.append(lg)
    orcs = [OracleDoc(options()) for _ in feeds]
    dead = [False] * n
    chunk = 61
    for k in range(0, max(len(f[1]) for f in feeds), chunk):
        for lg, (_, msgs) in zip(logs, feeds):
            for m in msgs[k:k + chunk]:
                lg.message(m, it)
        b = build_batch(logs, it)
        eng.apply(b)
        for d in range(n):
            if dead[d]:
                continue
            st = orcs[d].apply(b, d)
            est = eng.status(d)[0]
            assert est == st, f"doc {d}: engine status {est:#x}, oracle {st:#x}"
            if st:
                dead[d] = True
                continue
            assert eng.text(d) == orcs[d].text(), f"doc {d} chunk {k}"
    eng.summarize()
    for d in range(n):
        if not dead[d]:
            assert eng.summary(d) == orcs[d].summarize(b, d), f"doc {d}: summary differs"
    assert sum(dead) < n // 2


def test_js_packer_matches_python_packer(tmp_path):
    """The Node host packer encodes combining annotates, relative positions, marker ordinals and the
    value flags byte for byte like fluidframework_amd.batch."""
    import base64
    import os
    import shutil
    import subprocess

    if shutil.which("node") is None:
        pytest.skip("node is not installed")
    feeds = [(OBS, k[1]) for k in KATS] + [(OBS, k[1]) for k in RELPOS_KATS]
    feeds += [rewritten_feed(300, seed) for seed in (4, 5)]
    f = tmp_path / "feeds.json"
    f.write_text(json.dumps([{"observer": o, "msgs": m} for o, m in feeds]))
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run(["node", os.path.join(here, "node", "pack_feeds.js"), str(f)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    raw = {k: base64.b64decode(v) for k, v in json.loads(r.stdout).items()}
    it = Interner()
    logs = []
    for o, msgs in feeds:
        lg = DocLog()
        lg.start_collab(o)
        for m in msgs:
            lg.message(m, it)
        logs.append(lg)
    py = build_batch(logs, it)
    assert raw["docs"] == py.docs.tobytes()
    assert raw["ops"] == py.ops.tobytes()
    assert np.array_equal(np.frombuffer(raw["valEq"], "<u4")[:len(py.val_eq)], py.val_eq)
    assert np.array_equal(np.frombuffer(raw["valOff"], "<u4"), py.val_off)
    assert raw["valBytes"][:int(py.val_off[-1])] == py.val_bytes.tobytes()[:int(py.val_off[-1])]
    assert np.array_equal(np.frombuffer(raw["propopOff"], "<u4"), py.propop_off)
    n_kv = 2 * int(py.propop_off[-1])
    assert np.array_equal(np.frombuffer(raw["propopKv"], "<u4")[:n_kv], py.propop_kv[:n_kv])
    assert int((py.ops["type"] == abi.OP_RELPOS).sum()) > 10
    assert int(((py.ops["type"] == abi.OP_ANNOTATE) & (py.ops["payload2"] != 0)).sum()) > 10
