"""Spill experiment: replay the C5-shaped documents of c5_bisect.py up to their first divergent op on a build with
-DMTR_DEBUG_INSERT (the insert placement printed by lane 0), for the MTR_WPE_G=8 build against a spill-free one."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.synth import make_cfg, tables, with_docs  # noqa: E402
from oracle.oracle import generate  # noqa: E402

n, grow, ops = 8, 20000, 2000
cfg = make_cfg(n, ops, writers=64, max_lag=4096, text_cap=2 * grow + ops * 18 + 16)
tabs = tables(writers=64)
b, _, status = generate(cfg, tabs, 0, n, threads=8, grow=grow)
base = grow + 1
ks = [int(x) for x in os.environ.get("KS", "18,1,5,3,9,4,5,3").split(",")]
docs = b.docs.copy()
docs["op_count"] = base + np.asarray(ks)
bb = with_docs(tabs, docs, b.ops, b.text)
print("op_begin per doc:", [int(x) for x in docs["op_begin"]], flush=True)
eng = Engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
             text_units=2 * (int(cfg.text_cap) + 8192), prop_words=1 << 18, remover_cells=1 << 14, ops_per_launch=256)
eng.apply(bb)
eng.sync()
print("done", flush=True)
