"""Debug helper: apply one replay log message-by-message on the engine and the oracle and report
the first message after which the leaf structure differs (GPU box only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from fixtures import load_replay, replay_files, replay_log  # noqa: E402

from fluidframework_amd.batch import Interner, build_batch  # noqa: E402
from fluidframework_amd.engine import Engine  # noqa: E402
from oracle.oracle import OracleDoc, options  # noqa: E402

idx = int(sys.argv[1]) if len(sys.argv) > 1 else 4
path = replay_files()[idx]
groups = load_replay(path)
it = Interner()
log = replay_log(groups, it)
eng = Engine(1, max_segments=8192, heap_entries=8192, text_units=1 << 16, prop_words=1 << 16, remover_cells=1 << 12)
orc = OracleDoc(options())
b = build_batch([log], it)
eng.apply(b)
orc.apply(b, 0)
msgs = [m for g in groups for m in g["msgs"]]
print(os.path.basename(path), len(msgs), "messages")
prev_e = None
for k, m in enumerate(msgs):
    log.message(m, it)
    b = build_batch([log], it)
    eng.apply(b)
    orc.apply(b, 0)
    ge, gh = eng.export(0)
    oe, oh = orc.export()
    if gh != oh or ge.shape != oe.shape or (ge != oe).any():
        print("first divergence after message", k, "seq", m["sequenceNumber"], "msn", m["minimumSequenceNumber"],
              "contents", m["contents"])
        print("heights", gh, oh, "leaves", len(ge), len(oe), "oracle state", orc.state(), "engine", eng.stats())
        n = max(len(ge), len(oe))
        for i in range(n):
            a = ge[i].tolist() if i < len(ge) else None
            o = oe[i].tolist() if i < len(oe) else None
            mark = "  " if a == o else "!!"
            print(mark, i, a, o)
        if prev_e is not None:
            print("before (both equal):")
            for i, r in enumerate(prev_e):
                print("   ", i, r.tolist())
        break
    prev_e = oe.copy()
else:
    print("no divergence")
