"""Known-answer tests transcribed from the reference's own unit tests, replayed as the observer
(summarizer) sees them: every message remote, in sequence order, to a client that authored none.

* packages/dds/merge-tree/src/test/client.applyMsg.spec.ts -- multi-client conflict cases with the
  expected final text (`logger.validate({ baseText })`).  A message's referenceSequenceNumber is its
  author's currentSeq when the op was made (TestClient.makeOpMessage, testClient.ts:286-310), its
  minimumSequenceNumber 0; initial states are built as createClientsAtInitialState does
  (testClientLogger.ts:51-78): a non-collaborating local insert, then every "-" removed locally.
* packages/dds/merge-tree/src/test/snapshot.spec.ts:156-258 -- one author appending / removing with or
  without advancing the MSN (TestString.queue: refSeq = previous seq), and after each `expect` a
  summarize -> load round trip that the following ops continue from.
* packages/dds/merge-tree/src/test/mergeTree.zamboni.spec.ts:22-74 -- the tree-shape cases, with the
  zamboni passes driven the observer's way (an MSN advance) instead of direct zamboni/packParent calls.

CPU: the oracle.  GPU (-m gpu): the HIP engine through the C ABI against the same expected texts and
the oracle's leaves, tree levels and summary bytes.
"""
import pytest

from fixtures import blob_names
from fluidframework_amd.batch import DocLog, Interner, build_batch
from oracle.oracle import OracleDoc, options

OBSERVER = "observer-O"


def msg(client, seq, ref, contents, msn=0):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


def ins(client, seq, ref, pos, text, msn=0):
    return msg(client, seq, ref, {"type": 0, "pos1": pos, "seg": text}, msn)


def rem(client, seq, ref, start, end, msn=0):
    return msg(client, seq, ref, {"type": 1, "pos1": start, "pos2": end}, msn)


def noop(client, seq, ref, msn):
    """A non-op message: only updateSeqNumbers runs (client.ts:874), which is how an observer's MSN
    advances and zamboni runs (mergeTree.ts:1025-1044)."""
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "noop", "contents": None}


def initial_state(log, it, state):
    """createClientsAtInitialState's setup (testClientLogger.ts:58-64): insert, then remove each '-'."""
    if state:
        log.local_insert(0, state, it)
    text = state
    while "-" in text:
        i = text.index("-")
        log.local_remove(i, i + 1)
        text = text[:i] + text[i + 1:]


# (name, reference test, initial state, newLengthCalc, messages, expected text)
APPLYMSG_KATS = [
    ("overlapping insert and delete", "client.applyMsg.spec.ts:240-266", "hello world", False, [
        ins("localUser", 1, 0, 0, "-"),
        ins("localUser", 2, 1, 0, "L"), rem("localUser", 3, 1, 1, 2),
        ins("remoteUser", 4, 1, 0, "R"), rem("remoteUser", 5, 1, 1, 2)], "RLhello world"),
    ("intersecting insert after local delete", "client.applyMsg.spec.ts:268-286", "", False, [
        ins("C", 1, 0, 0, "c"), rem("C", 2, 0, 0, 1), ins("B", 3, 0, 0, "b"), ins("C", 4, 0, 0, "c")], "cb"),
    ("conflicting insert after shared delete", "client.applyMsg.spec.ts:288-311", "Z", False, [
        ins("B", 1, 0, 0, "B"), rem("C", 2, 0, 0, 1), ins("C", 3, 0, 0, "C")], "CB"),
    ("local remove followed by conflicting insert", "client.applyMsg.spec.ts:313-332", "", False, [
        ins("C", 1, 0, 0, "c"), ins("B", 2, 0, 0, "b"), rem("C", 3, 0, 0, 1), ins("C", 4, 0, 0, "c")], "cb"),
    ("intersecting insert with un-acked insert and delete", "client.applyMsg.spec.ts:334-350", "", False, [
        ins("C", 1, 0, 0, "c"), ins("B", 2, 0, 0, "bb"), rem("B", 3, 0, 0, 1)], "bc"),
    ("conflicting insert over local delete", "client.applyMsg.spec.ts:352-380", "", False, [
        ins("C", 1, 0, 0, "CCC"), rem("C", 2, 0, 0, 1),
        rem("C", 3, 2, 0, 1), ins("C", 4, 2, 0, "CC"), ins("B", 5, 2, 1, "BBB")], "CCBBBC"),
    ("Local insert after acked local delete", "client.applyMsg.spec.ts:382-413", "ZZ", True, [
        rem("C", 1, 0, 0, 1), rem("B", 2, 0, 1, 2), ins("C", 3, 1, 0, "C"), ins("B", 4, 0, 1, "B")], "CB"),
    ("Remote Remove before conflicting insert", "client.applyMsg.spec.ts:415-438", "Z", False, [
        rem("B", 1, 0, 0, 1), ins("B", 2, 0, 0, "B"), ins("C", 3, 1, 0, "C")], "CB"),
    ("Conflicting inserts at deleted segment position", "client.applyMsg.spec.ts:440-462", "a----bcd-ef", False, [
        ins("B", 1, 0, 4, "B"), ins("C", 2, 0, 4, "CC"), rem("C", 3, 0, 2, 8), rem("B", 4, 2, 5, 8)], "ab"),
    ("Inconsistent shared string after pausing connection #9703", "client.applyMsg.spec.ts:464-493", "abcd", True, [
        rem("B", 1, 0, 1, 3), ins("B", 2, 1, 1, "yz"), ins("C", 3, 0, 2, "X")], "ayzXd"),
]
IDS = [k[0] for k in APPLYMSG_KATS]


def _kat_log(kat, it):
    _, _, state, _, msgs, _ = kat
    log = DocLog()
    initial_state(log, it, state)
    log.start_collab(OBSERVER)
    for m in msgs:
        log.message(m, it)
    return log


@pytest.mark.parametrize("kat", APPLYMSG_KATS, ids=IDS)
def test_applymsg_kat_oracle(kat):
    it = Interner()
    b = build_batch([_kat_log(kat, it)], it)
    o = OracleDoc(options(new_length_calc=kat[3]))
    assert o.apply(b, 0) == 0
    assert o.text() == kat[5], f"{kat[1]}: {o.text()!r} != {kat[5]!r}"


@pytest.mark.gpu
@pytest.mark.parametrize("newlen", [False, True], ids=["oldlen", "newlen"])
def test_applymsg_kats_engine(newlen):
    """Every KAT of one length mode as one document of one engine batch: the expected text, and the
    oracle's leaves / tree levels / summary bytes."""
    from fluidframework_amd.engine import Engine
    from test_gpu_parity import _compare_export

    kats = [k for k in APPLYMSG_KATS if k[3] == newlen]
    it = Interner()
    b = build_batch([_kat_log(k, it) for k in kats], it)
    eng = Engine(len(kats), new_length_calc=newlen, max_segments=256, heap_entries=256, text_units=4096,
                 prop_words=1024, remover_cells=256)
    eng.apply(b)
    eng.summarize()
    for d, k in enumerate(kats):
        assert eng.status(d)[0] == 0, k[0]
        assert eng.text(d) == k[5], f"{k[1]}: engine {eng.text(d)!r} != {k[5]!r}"
        o = OracleDoc(options(new_length_calc=newlen))
        assert o.apply(b, d) == 0
        _compare_export(eng, d, o)
        assert eng.summary(d) == o.summarize(b, d), k[0]


# ---------------------------------------------------------------- snapshot.spec.ts:156-258

class Author:
    """TestString (snapshot.spec.ts:39-147) seen from an observer: one author whose every op
    references the previous sequence number; `msn_up` sets the MSN to the op's own seq."""

    def __init__(self, initial=""):
        self.text = initial
        self.seq = 0
        self.msn = 0

    def _next(self, msn_up):
        ref = self.seq
        self.seq += 1
        if msn_up:
            self.msn = self.seq
        return ref

    def insert(self, pos, s, msn_up):
        ref = self._next(msn_up)
        self.text = self.text[:pos] + s + self.text[pos:]
        return ins("fakeId", self.seq, ref, pos, s, self.msn)

    def append(self, s, msn_up):
        return self.insert(len(self.text), s, msn_up)

    def remove(self, a, b, msn_up):
        ref = self._next(msn_up)
        self.text = self.text[:a] + self.text[b:]
        return rem("fakeId", self.seq, ref, a, b, self.msn)


def _snapshot_cases():
    """(name, initial, steps): a step is a message or ("expect", text)."""
    cases = []
    a = Author()
    cases.append(("includes segments below MSN", "", [a.append("0", True), ("expect", "0")]))
    a = Author()
    cases.append(("includes ACKed segments above the MSN", "", [a.append("0", False), ("expect", "0")]))
    a = Author()
    cases.append(("includes removals of segments above the MSN", "",
                  [a.append("0x", False), a.remove(1, 2, False), ("expect", "0")]))
    a = Author()
    cases.append(("includes removals above the MSN of segments below the MSN", "",
                  [a.append("0x", True), a.remove(1, 2, False), ("expect", "0")]))
    a = Author()
    cases.append(("can insert segments after loading removed segment", "",
                  [a.append("0x", True), a.remove(1, 2, False), ("expect", "0"), a.append("1", False),
                   ("expect", "01")]))
    a = Author()
    cases.append(("can insert segments relative to removed segment", "",
                  [a.append("0x", False), a.append("2", False), a.remove(1, 2, False), a.insert(1, "1", False),
                   a.append("3", False), ("expect", "0123")]))
    a = Author()
    cases.append(("can insert segments relative to removed segment loaded from snapshot", "",
                  [a.append("0x", False), a.append("2", False), a.remove(1, 2, False), ("expect", "02"),
                   a.insert(1, "1", False), a.append("3", False), ("expect", "0123")]))
    for up in (True, False):
        a = Author()
        steps = [a.append(str(i % 10), up) for i in range(10000 + 10)]  # SnapshotV1.chunkSize + 10
        cases.append((f"includes ACKed segments {'below' if up else 'above'} MSN in body", "",
                      steps + [("expect", a.text)]))
    a = Author("starting text")
    cases.append(("includes segments submitted while detached", "starting text", [("expect", "starting text")]))
    return cases


SNAPSHOT_CASES = _snapshot_cases()


def _run_snapshot_case_oracle(initial, steps):
    """Apply the steps to an oracle observer; at every `expect`, check the text, summarize (V1),
    load the blobs into a new observer and continue on it (TestString.checkSnapshot)."""
    it = Interner()
    log = DocLog()
    initial_state(log, it, initial)
    log.start_collab(OBSERVER)
    orc = OracleDoc(options())
    for st in steps:
        if isinstance(st, dict):
            log.message(st, it)
            continue
        b = build_batch([log], it)
        assert orc.apply(b, 0) == 0
        assert orc.text() == st[1]
        blobs = orc.summarize(b, 0)
        log = DocLog()
        log.load_summary(dict(zip(blob_names(len(blobs), True), [x.decode() for x in blobs])), OBSERVER, it)
        orc = OracleDoc(options())
        b = build_batch([log], it)
        assert orc.apply(b, 0) == 0
        assert orc.text() == st[1], "summary -> load changed the text"
        assert orc.summarize(b, 0) == blobs, "summary -> load -> summary is not byte-stable"
    return True


@pytest.mark.parametrize("case", SNAPSHOT_CASES, ids=[c[0] for c in SNAPSHOT_CASES])
def test_snapshot_kat_oracle(case):
    assert _run_snapshot_case_oracle(case[1], case[2])


@pytest.mark.gpu
def test_snapshot_kats_engine():
    """The snapshot.spec.ts cases on the device, all at once: each `expect` checks the engine's text,
    summarizes on the device, loads those blobs into a new engine document and continues there;
    summaries equal the oracle's at every step."""
    from fluidframework_amd.engine import Engine

    n = len(SNAPSHOT_CASES)
    it = Interner()
    logs, pos = [], [0] * n
    for _, initial, _ in SNAPSHOT_CASES:
        log = DocLog()
        initial_state(log, it, initial)
        log.start_collab(OBSERVER)
        logs.append(log)
    orcs = [OracleDoc(options()) for _ in range(n)]
    gen = 0
    eng = Engine(n * 4, max_segments=32768, heap_entries=32768, text_units=1 << 17, prop_words=1024,
                 remover_cells=1024, ops_per_launch=256)
    slot = list(range(n))  # engine document of each case's current observer
    nxt = n
    while True:
        active = False
        expects = {}
        for c, (_, _, steps) in enumerate(SNAPSHOT_CASES):
            while pos[c] < len(steps) and isinstance(steps[pos[c]], dict):
                logs[c].message(steps[pos[c]], it)
                pos[c] += 1
            if pos[c] < len(steps):
                expects[c] = steps[pos[c]][1]
                pos[c] += 1
                active = True
        if not active:
            break
        all_logs = [DocLog() for _ in range(n * 4)]
        for c in range(n):
            all_logs[slot[c]] = logs[c]
        b = build_batch(all_logs, it)
        eng.apply(b)
        eng.summarize()
        for c, want in expects.items():
            d = slot[c]
            assert orcs[c].apply(b, d) == 0
            assert eng.status(d)[0] == 0, SNAPSHOT_CASES[c][0]
            assert eng.text(d) == want == orcs[c].text(), SNAPSHOT_CASES[c][0]
            blobs = eng.summary(d)
            assert blobs == orcs[c].summarize(b, d), SNAPSHOT_CASES[c][0]
            logs[c] = DocLog()
            logs[c].load_summary(dict(zip(blob_names(len(blobs), True), [x.decode() for x in blobs])), OBSERVER, it)
            orcs[c] = OracleDoc(options())
            slot[c] = nxt
            nxt += 1
        gen += 1
        assert nxt <= 4 * n
    assert gen >= 2


# ---------------------------------------------------------------- mergeTree.zamboni.spec.ts:22-74

def _hello_world_observer(it):
    """beforeEach of mergeTree.zamboni.spec.ts:14-21: "hello world" one character at a time (eleven
    non-collaborating local inserts at the end), then collaboration."""
    log = DocLog()
    text = ""
    for ch in "hello world":
        log.local_insert(len(text), ch, it)
        text += ch
    log.start_collab(OBSERVER)
    return log


def _zamboni_cases():
    return [
        # packParent with no children segments (zamboni.spec.ts:22-46): remove all but the last
        # character, then the rest; zamboni (driven by the MSN) empties the tree
        ("remove all", [rem("X", 1, 0, 0, 10), rem("X", 2, 1, 0, 1, msn=1),
                        noop("X", 3, 2, 3)], ""),
        # zamboni with one segment to scour (zamboni.spec.ts:55-66)
        ("one segment", [rem("X", 1, 0, 0, 1), noop("X", 2, 1, 2)],
         "ello world"),
        # zamboni with many segments to scour (zamboni.spec.ts:67-74): the first leaf block's six
        # leaves go, and the root packs into one child
        ("many segments", [rem("X", 1, 0, 0, 6), noop("X", 2, 1, 2)],
         "world"),
    ]


ZAMBONI_CASES = _zamboni_cases()


def _zamboni_batch(case):
    it = Interner()
    log = _hello_world_observer(it)
    for m in case[1]:
        log.message(m, it)
    return build_batch([log], it)


def _root_children(exp, height):
    """Children of the root from an export (8 int32 per leaf; column 5 = bnd levels)."""
    if len(exp) == 0:
        return 0
    if height <= 1:
        return len(exp)
    return int((exp[:, 5] >= height - 1).sum())


@pytest.mark.parametrize("case", ZAMBONI_CASES, ids=[c[0] for c in ZAMBONI_CASES])
def test_zamboni_kat_oracle(case):
    b = _zamboni_batch(case)
    o = OracleDoc(options())
    assert o.apply(b, 0) == 0
    assert o.text() == case[2]
    exp, h = o.export()
    if case[0] == "many segments":
        assert _root_children(exp, h) == 1, "packParent leaves the root one child (zamboni.spec.ts:73)"


@pytest.mark.gpu
def test_zamboni_kats_engine():
    from fluidframework_amd.engine import Engine
    from test_gpu_parity import _compare_export

    for case in ZAMBONI_CASES:
        b = _zamboni_batch(case)
        eng = Engine(1, max_segments=256, heap_entries=256, text_units=4096, prop_words=1024, remover_cells=256)
        eng.apply(b)
        assert eng.status(0)[0] == 0 and eng.text(0) == case[2], case[0]
        o = OracleDoc(options())
        assert o.apply(b, 0) == 0
        _compare_export(eng, 0, o)
