"""Spill experiment probe: C5-shaped documents (20k loaded segments, 64 writers) on the build MTR_LIB names, with the
op lists cut after the load (k = 0) and after k ops: per document the status, the failing op and the leaf count
against the oracle's."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.synth import make_cfg, tables, with_docs  # noqa: E402
from oracle.oracle import OracleDoc, generate, options  # noqa: E402

n, grow, ops = 8, 20000, 2000
cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
tabs = tables(writers=64)
b, _, status = generate(cfg, tabs, 0, n, threads=8, grow=grow)
base = grow + 1
for k in [int(x) for x in os.environ.get("KS", "0,1,5,50").split(",")]:
    docs = b.docs.copy()
    docs["op_count"] = base + k
    bb = with_docs(tabs, docs, b.ops, b.text)
    eng = Engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                 text_units=2 * (int(cfg.text_cap) + 8192), ops_per_launch=256)
    eng.apply(bb)
    out = []
    for d in range(n):
        st, op = eng.status(d)
        orc = OracleDoc(options())
        orc.apply(bb, d)
        ge, _ = eng.export(d)
        oe, _ = orc.export()
        same = ge.shape == oe.shape and not (ge != oe).any()
        out.append((hex(st), op, len(ge), len(oe), same))
    print("k", k, out, flush=True)
