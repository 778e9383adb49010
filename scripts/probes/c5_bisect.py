"""Debug probe: per document, the first op after which the engine's leaves differ from the oracle's
(C5-shaped 20k-segment documents), by bisection over truncated op lists."""
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


def diff_for(ks):
    docs = b.docs.copy()
    docs["op_count"] = base + np.asarray(ks)
    bb = with_docs(tabs, docs, b.ops, b.text)
    eng = Engine(n, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                 text_units=2 * (int(cfg.text_cap) + 8192), prop_words=1 << 18, remover_cells=1 << 14,
                 ops_per_launch=256)
    eng.apply(bb)
    res = []
    for d in range(n):
        orc = OracleDoc(options())
        orc.apply(bb, d)
        ge, _ = eng.export(d)
        oe, _ = orc.export()
        res.append(not (ge.shape == oe.shape and not (ge != oe).any()))
    return res, bb, eng


import os
lo = [0] * n
hi = [ops] * n
if os.environ.get("FIXED_HI"):
    hi = [int(x) for x in os.environ["FIXED_HI"].split(",")]
    lo = [h - 1 for h in hi]
while any(h - l > 1 for l, h in zip(lo, hi)):
    mid = [(l + h) // 2 for l, h in zip(lo, hi)]
    res, _, _ = diff_for(mid)
    for d in range(n):
        if hi[d] - lo[d] <= 1:
            continue
        if res[d]:
            hi[d] = mid[d]
        else:
            lo[d] = mid[d]
print("first bad op count per doc:", hi, flush=True)
res, bb, eng = diff_for(hi)
for d in range(n):
    op = b.ops[int(b.docs["op_begin"][d]) + base + hi[d] - 1]
    print(f"doc {d}: bad={res[d]} after {hi[d]} ops; last op: {op}", flush=True)
    orc = OracleDoc(options())
    orc.apply(bb, d)
    ge, _ = eng.export(d)
    oe, _ = orc.export()
    m = min(len(ge), len(oe))
    bad = np.nonzero((ge[:m] != oe[:m]).any(axis=1))[0]
    f = int(bad[0]) if bad.size else m
    print(f"   leaves {len(ge)} vs {len(oe)}, first diff {f}", flush=True)
    for j in range(max(0, f - 2), min(m, f + 3)):
        print("   ", j, ge[j].tolist(), oe[j].tolist(), flush=True)

print("--- state before the first bad op: getContainingSegment at its pos1", flush=True)
res, bb, eng = diff_for([h - 1 for h in hi])
for d in range(n):
    op = b.ops[int(b.docs["op_begin"][d]) + base + hi[d] - 1]
    client, ref, pos1 = int(op["client"]), int(op["ref_seq"]), int(op["pos1"])
    orc = OracleDoc(options())
    orc.apply(bb, d)
    e = eng.containing_segment(d, pos1, ref, client)
    o = orc.containing(pos1, ref, client)
    print(f"doc {d}: same before={not res[d]} pos1={pos1} ref={ref} client={client}: engine "
          f"{None if e is None else (e['leaf'], e['offset'], e['length'])} oracle {o[:3]}", flush=True)

print("--- first position whose containing segment differs", flush=True)
for d in range(n):
    op = b.ops[int(b.docs["op_begin"][d]) + base + hi[d] - 1]
    client, ref, pos1 = int(op["client"]), int(op["ref_seq"]), int(op["pos1"])
    orc = OracleDoc(options())
    orc.apply(bb, d)

    def same(p):
        e = eng.containing_segment(d, p, ref, client)
        o = orc.containing(p, ref, client)
        return (e is None and o[0] < 0) or (e is not None and (e["leaf"], e["offset"]) == o[:2])

    lo_, hi_ = 0, pos1
    if same(hi_):
        print(f"doc {d}: same at pos1", flush=True)
        continue
    while hi_ - lo_ > 1:
        m = (lo_ + hi_) // 2
        if same(m):
            lo_ = m
        else:
            hi_ = m
    e = eng.containing_segment(d, hi_, ref, client)
    o = orc.containing(hi_, ref, client)
    ge, _ = eng.export(d)
    print(f"doc {d}: first differing pos {hi_}: engine leaf {e['leaf']} off {e['offset']} (seq {e['seq']} client "
          f"{e['client']} rseq {e['removed_seq']}); oracle leaf {o[0]} off {o[1]}", flush=True)
    for j in range(min(e["leaf"], o[0]) - 1, max(e["leaf"], o[0]) + 2):
        print("    ", j, ge[j].tolist(), flush=True)

print("--- remover ops and other clients' views", flush=True)
RS = {0: 29, 1: 53, 2: 68, 3: 33, 4: 27, 5: 65, 7: 305}
POS = {0: 2616, 1: 248, 2: 530, 3: 181, 4: 3051, 5: 100, 7: 2450}
for d, rs in RS.items():
    ob = int(b.docs["op_begin"][d]) + base
    seg = b.ops[ob: ob + ops]
    rem = [tuple(int(x) for x in o) for o in seg if int(o["seq"]) == rs]
    op = b.ops[ob + hi[d] - 1]
    ref = int(op["ref_seq"])
    orc = OracleDoc(options())
    orc.apply(bb, d)
    views = []
    for cl in (16, int(rem[0][2]) if rem else 0, 3, 40):
        e = eng.containing_segment(d, POS[d], ref, cl)
        o = orc.containing(POS[d], ref, cl)
        views.append((cl, (e["leaf"], e["offset"]) if e else None, o[:2]))
    print(f"doc {d}: ops with seq {rs}: {rem}; views at pos {POS[d]} ref {ref}: {views}", flush=True)
