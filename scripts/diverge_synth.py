"""Debug helper (GPU box): replay one oracle-generated synthetic document on the engine and the
oracle chunk by chunk (then op by op inside the first bad chunk) and report the first op after which
the leaf structure differs.  Usage: diverge_synth.py DOC [GROW OPS WRITERS LAG]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from fluidframework_amd import abi  # noqa: E402
from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.synth import make_cfg, tables, with_docs  # noqa: E402
from oracle.oracle import OracleDoc, generate, options  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 1
grow, ops, writers, lag = (int(x) for x in (sys.argv[2:6] + ["20000", "2000", "64", "4096"][len(sys.argv[2:6]):]))
cfg = make_cfg(d + 1, ops, writers=writers, max_lag=lag, text_cap=2 * grow + ops * 18 + 16)
tabs = tables(writers=writers)
b, _, st = generate(cfg, tabs, 0, d + 1, threads=8, grow=grow)
desc = b.docs[d]
all_ops = b.ops[int(desc["op_begin"]):int(desc["op_begin"]) + int(desc["op_count"])]
text = b.text[int(desc["text_base"]):int(desc["text_base"]) + int(desc["text_count"])]


def piece(lo, hi):
    docs = np.zeros(1, dtype=abi.DOC_DTYPE)
    docs["op_count"] = hi - lo
    docs["text_count"] = len(text)
    docs["n_clients"] = desc["n_clients"]
    return with_docs(tabs, docs, all_ops[lo:hi].copy(), text.copy())


def fresh():
    eng = Engine(1, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                 text_units=2 * (int(cfg.text_cap) + 8192), prop_words=1 << 16, remover_cells=1 << 14,
                 ops_per_launch=256)
    return eng, OracleDoc(options())


def same(eng, orc):
    ge, gh = eng.export(0)
    oe, oh = orc.export()
    return gh == oh and ge.shape == oe.shape and not (ge != oe).any(), ge, oe, gh, oh


def report(k, eng, orc):
    ok, ge, oe, gh, oh = same(eng, orc)
    op = all_ops[k]
    print("first divergence after op", k, {n: int(op[n]) for n in op.dtype.names}, "engine status", eng.status(0))
    print("heights", gh, oh, "leaves", len(ge), len(oe), "oracle state", orc.state().tolist())
    bad = [i for i in range(max(len(ge), len(oe))) if i >= len(ge) or i >= len(oe) or (ge[i] != oe[i]).any()]
    print("differing leaves:", len(bad), "first", bad[:3], "last", bad[-3:])
    seq = int(op["seq"])
    print("oracle leaves touched by this op:", [i for i in range(len(oe)) if oe[i][3] == seq or oe[i][1] == seq][:20])
    print("engine leaves touched by this op:", [i for i in range(len(ge)) if ge[i][3] == seq or ge[i][1] == seq][:20],
          "count", sum(1 for i in range(len(ge)) if ge[i][3] == seq))
    ln = orc.length(int(op["ref_seq"]), int(op["client"]))
    print("oracle view length", ln)
    import ctypes as C
    from fluidframework_amd.engine import lib
    L = lib()
    L.mtr_debug_scan.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
    L.mtr_debug_scan.restype = C.c_int64
    n = len(ge)
    buf = np.zeros(2 * n, dtype="<i4")
    if L.mtr_debug_scan(eng.h, 0, buf.ctypes.data, n) == n:
        E, V = buf[:n], buf[n:]
        for lo2, hi2 in ((bad[0] - 4, bad[0] + 4), (bad[-1] - 2, bad[-1] + 4)):
            print("E/V", [(i, int(E[i]), int(V[i])) for i in range(max(lo2, 0), min(hi2, n))])
        print("E monotone:", bool((np.diff(E) >= 0).all()), "first drop at",
              np.nonzero(np.diff(E) < 0)[0][:5].tolist())
        # probe points of lower_bound_E's first 64-ary level
        stride = (n + 63) >> 6
        print("probes", [(k, (k + 1) * stride - 1, int(E[min((k + 1) * stride - 1, n - 1)])) for k in range(40, 50)])
    lo = max(0, bad[0] - 6) if bad else 0
    for i in range(lo, min(lo + 30, max(len(ge), len(oe)))):
        a = ge[i].tolist() if i < len(ge) else None
        o = oe[i].tolist() if i < len(oe) else None
        print("  " if a == o else "!!", i, a, o)


eng, orc = fresh()
start = grow + 1
p = piece(0, start)
eng.apply(p)
assert orc.apply(p, 0) == 0
print("after load+start equal:", same(eng, orc)[0])
CH = 100
good = start
for lo in range(start, len(all_ops), CH):
    hi = min(lo + CH, len(all_ops))
    p = piece(lo, hi)
    eng.apply(p)
    rc = orc.apply(p, 0)
    if rc != 0 or not same(eng, orc)[0] or eng.status(0)[0] != 0:
        print("chunk", lo, hi, "differs; replaying op by op from", good)
        eng, orc = fresh()
        p = piece(0, good)
        eng.apply(p)
        orc.apply(p, 0)
        for k in range(good, hi):
            p = piece(k, k + 1)
            eng.apply(p)
            orc.apply(p, 0)
            if not same(eng, orc)[0] or eng.status(0)[0] != 0:
                report(k, eng, orc)
                break
        break
    good = hi
else:
    print("no divergence")
