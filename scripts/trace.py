"""Debug helper: zamboni trace of one replay log, message by message.
   python scripts/trace.py engine IDX N   (GPU box; MTR_TRACE=1)
   python scripts/trace.py oracle IDX N"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from fixtures import load_replay, replay_files, replay_log  # noqa: E402

from fluidframework_amd.batch import Interner, build_batch  # noqa: E402

mode, idx, upto = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
libc = ctypes.CDLL(None)
groups = load_replay(replay_files()[idx])
it = Interner()
log = replay_log(groups, it)
if mode == "engine":
    os.environ["MTR_TRACE"] = "1"
    from fluidframework_amd.engine import Engine
    doc = Engine(1, max_segments=8192, heap_entries=8192, text_units=1 << 16, prop_words=1 << 16, remover_cells=4096)
    step = lambda b: doc.apply(b)  # noqa: E731
else:
    from oracle.oracle import OracleDoc, lib, options
    lib().oracle_set_trace(1)
    doc = OracleDoc(options())
    step = lambda b: doc.apply(b, 0)  # noqa: E731
step(build_batch([log], it))
msgs = [m for g in groups for m in g["msgs"]]
for k, m in enumerate(msgs[:upto]):
    log.message(m, it)
    libc.fflush(None)
    print(f"MSG {k} seq={m['sequenceNumber']} msn={m['minimumSequenceNumber']}", flush=True)
    step(build_batch([log], it))
    libc.fflush(None)
