"""Debug: engine load of a legacy summary + catch-up vs the oracle doing the same."""
import json, sys
sys.path.insert(0, ".")
import numpy as np
from tests.test_catchup import messages_from_batch, OracleReplica, _named, LEGACY
from fluidframework_amd.batch import Interner, build_batch
from fluidframework_amd.sequence import SequenceLog
from fluidframework_amd.synth import make_cfg, tables
from fluidframework_amd.engine import Engine
from oracle.oracle import generate, options

cfg = make_cfg(8, 800, writers=8, max_lag=32)
tabs = tables(writers=8)
gb, _, status = generate(cfg, tabs, 0, 8, threads=8, opts=options(**LEGACY))
sums = []
for d in range(8):
    observer, msgs = messages_from_batch(gb, d)
    a = OracleReplica(); a.log.start_collab(observer)
    for k in range(0, len(msgs), 131):
        for m in msgs[k:k + 131]:
            a.log.message(m, a.it)
        a.flush()
    sums.append(a.summary())
kw = dict(snapshot_v1=False, max_segments=4096, heap_entries=4096, text_units=1 << 15, prop_words=1 << 14,
          remover_cells=2048, ops_per_launch=24)
eng2 = Engine(8, **kw)
logs2, it2 = [], Interner()
refs = []
for d in range(8):
    lg = SequenceLog(legacy=True)
    lg.load(_named(sums[d]), "observer-2", it2)
    logs2.append(lg)
    r = OracleReplica(); r.log.load(_named(sums[d]), "observer-2", r.it); refs.append(r)
b2 = build_batch(logs2, it2)
ops = b2.ops
print("types", np.unique(ops["type"], return_counts=True), "flags", np.unique(ops["flags"], return_counts=True))
eng2.apply(b2)
eng2.summarize()
for d in range(8):
    r = refs[d]; r.flush()
    st = eng2.status(d)
    es, os_ = eng2.summary(d), r.doc.summarize(r.last, 0)
    ee, eh = eng2.export(d); oe, oh = r.doc.export()
    print(d, "status", st, "summary eq", es == os_, "orig eq", os_ == sums[d][:len(os_)], "export eq", np.array_equal(ee, oe), len(ee), len(oe), eng2.text(d) == r.doc.text())
    if es != os_:
        a, b = es[0], os_[0]
        i = next(i for i in range(min(len(a), len(b))) if a[i] != b[i]) if a[:min(len(a),len(b))] != b[:min(len(a),len(b))] else min(len(a), len(b))
        print("  first diff at", i, a[max(0,i-150):i+100]); print("  oracle     ", b[max(0,i-150):i+100])
        if len(ee) == len(oe):
            bad = np.nonzero((ee != oe).any(1))[0]
            print("  export rows differ", bad[:10], ee[bad[:3]], oe[bad[:3]])
