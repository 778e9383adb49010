"""Debug probe: C5-shaped documents (20k loaded segments), engine vs oracle per document for growing op
counts and launch sizes; prints where the first divergence appears."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.synth import make_cfg, tables  # noqa: E402
from oracle.oracle import OracleDoc, generate, options  # noqa: E402


def run(n, grow, ops, opl):
    cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
    b, _, status = generate(cfg, tables(writers=64), 0, n, threads=8, grow=grow)
    eng = Engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                 text_units=2 * (int(cfg.text_cap) + 8192), prop_words=1 << 18, remover_cells=1 << 14,
                 ops_per_launch=opl)
    t0 = time.time()
    eng.apply(b)
    out = []
    for d in range(n):
        orc = OracleDoc(options())
        orc.apply(b, d)
        ge, _ = eng.export(d)
        oe, _ = orc.export()
        st = eng.status(d)
        same = ge.shape == oe.shape and not (ge != oe).any()
        first = -1
        if not same:
            m = min(len(ge), len(oe))
            bad = np.nonzero((ge[:m] != oe[:m]).any(axis=1))[0]
            first = int(bad[0]) if bad.size else m
        out.append((d, st, len(ge), len(oe), same, first))
    nbad = sum(1 for o in out if not o[4])
    print(f"ops={ops} opl={opl}: {nbad}/{n} docs differ ({time.time() - t0:.1f}s)", flush=True)
    for o in out:
        if not o[4]:
            print("   ", o, flush=True)


CASES = [(2000, 256), (2000, 1), (500, 256), (200, 256), (100, 256), (50, 256), (20, 256)]
for ops, opl in (CASES if len(sys.argv) < 2 else CASES[:int(sys.argv[1])]):
    run(8, 20000, ops, opl)
