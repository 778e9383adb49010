"""Phase breakdown of the apply kernel on a C3-shaped batch (needs libmtr_prof.so:
`python -m fluidframework_amd.build --prof`, run with MTR_LIB=libmtr_prof.so)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MTR_LIB", "libmtr_prof.so")

from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.synth import make_cfg, tables  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=20000)
ap.add_argument("--ops", type=int, default=1000)
ap.add_argument("--writers", type=int, default=8)
ap.add_argument("--max-lag", type=int, default=32)
ap.add_argument("--ops-per-launch", type=int, default=256)
ap.add_argument("--grow", type=int, default=0, help="C5-shaped: documents pre-grown to this many segments")
ap.add_argument("--matrix", action="store_true",
                help="C4-shaped SharedMatrix pairs (x1 = setCell messages, x2 = row/col splices)")
a = ap.parse_args()
n, ops = a.docs, a.ops
if a.matrix:
    cfg = make_cfg(n, ops, writers=a.writers, max_lag=a.max_lag, weights=(12, 8, 80), max_text=4, max_range=3,
                   text_cap=0)
    eng = Engine(2 * n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * ops + 1024,
                 prop_words=1024, remover_cells=8192, ops_per_launch=a.ops_per_launch)
    eng.generate_matrix(cfg, tables(writers=a.writers))
elif a.grow:
    g = a.grow
    cfg = make_cfg(n, ops, writers=a.writers, max_lag=a.max_lag, text_cap=2 * g + 18 * ops + 16)
    eng = Engine(n, max_segments=g + g // 14 + 2 * ops + 128, heap_entries=g + 2 * ops + 128,
                 text_units=2 * int(cfg.text_cap) + 16384, prop_words=65536, remover_cells=65536,
                 ops_per_launch=a.ops_per_launch)
    eng.generate(cfg, tables(writers=a.writers), grow=g)
else:
    cfg = make_cfg(n, ops, writers=a.writers, max_lag=a.max_lag)
    eng = Engine(n, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=2 * int(cfg.text_cap) + 1024,
                 prop_words=16384, remover_cells=4096, ops_per_launch=a.ops_per_launch)
    eng.generate(cfg, tables(writers=a.writers))
eng.profile(reset=True)
eng.reset()
eng.run()
eng.sync()
tm = eng.timing()
p = eng.profile(reset=True)
if not p:
    print(json.dumps({"docs": n, "ops": ops, "apply_ms": tm["apply_ms"]}))
    raise SystemExit(0)
tot = p["op"] or 1
rows = {k: {"cycles_per_op": v / (n * ops), "frac_of_op": v / tot} for k, v in p.items() if not k.startswith("n_")}
counts = {k: v / (n * ops) for k, v in p.items() if k.startswith("n_")}
print(json.dumps({"docs": n, "ops": ops, "apply_ms": tm["apply_ms"], "per_op_counts": counts, "phases": rows}, indent=1))
