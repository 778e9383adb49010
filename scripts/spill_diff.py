"""Spill experiment, differential probe: C5-shaped documents (20k loaded segments, 64 writers) on the build MTR_LIB
names, op lists cut after the load (k = 0) or after k ops.  Per document: status, leaf counts, and where the engine's
leaf records (mtr_export: len, seq, client, removed_seq, n_removers, bnd, is_marker, props_hash) first differ from the
oracle's, with the count of differing leaves per column -- which part of the state the failing build gets wrong."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.synth import make_cfg, tables, with_docs  # noqa: E402
from oracle.oracle import OracleDoc, generate, options  # noqa: E402

COLS = ["len", "seq", "client", "rseq", "nrem", "bnd", "marker", "props"]
n, grow, ops = int(os.environ.get("NDOCS", "8")), int(os.environ.get("GROW", "20000")), 2000
cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
tabs = tables(writers=64)
b, _, status = generate(cfg, tabs, 0, n, threads=8, grow=grow)
base = grow + 1
for k in [int(x) for x in os.environ.get("KS", "0").split(",")]:
    docs = b.docs.copy()
    docs["op_count"] = base + k
    bb = with_docs(tabs, docs, b.ops, b.text)
    eng = Engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                 text_units=2 * (int(cfg.text_cap) + 8192), ops_per_launch=int(os.environ.get("OPL", "256")))
    eng.apply(bb)
    for d in range(n):
        st, op = eng.status(d)
        orc = OracleDoc(options())
        orc.apply(bb, d)
        ge, gh = eng.export(d)
        oe, oh = orc.export()
        line = f"k {k} doc {d} status {hex(st)} op {op} leaves {len(ge)}/{len(oe)} height {gh}/{oh}"
        m = min(len(ge), len(oe))
        diff = ge[:m] != oe[:m]
        rows = np.nonzero(diff.any(axis=1))[0]
        if len(rows):
            r = int(rows[0])
            line += f" first_diff {r} eng {ge[r].tolist()} orc {oe[r].tolist()}"
            line += " per_col " + str({c: int(diff[:, i].sum()) for i, c in enumerate(COLS) if diff[:, i].any()})
            line += f" diff_rows {len(rows)} last {int(rows[-1])} rows_mod7 {np.bincount(rows % 7, minlength=7).tolist()}"
        elif len(ge) == len(oe):
            line += " same"
        print(line, flush=True)
