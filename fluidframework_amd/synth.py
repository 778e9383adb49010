"""Synthetic workloads of the bench configurations.

The op-choice recipe lives in include/mtr_synth.h.  It needs the exact length of the writer's
(refSeq, clientId) view before every op, which depends on the exact B+tree placement of concurrent
inserts, so op logs are recorded by an exact simulator: on the GPU the engine itself in record mode
(:meth:`fluidframework_amd.engine.Engine.generate`), in CPU tests the oracle.  This module builds the
host tables the recipe references: the client table shared by every document and the annotate
property ops (keys {"bold": bool, "color": str, "size": int, "1": str}, ~10 % null deletes).
"""
from __future__ import annotations

import ctypes as C
import random

import numpy as np

from . import abi
from .batch import Batch, Interner, _offsets
from .jsjson import js_string, to_utf8

# name -> recipe parameters (BASELINE.json configs)
CONFIGS = {
    "C2": dict(n_docs=10_000, ops_per_doc=5_000, writers=16, max_lag=64),
    "C3": dict(n_docs=100_000, ops_per_doc=1_000, writers=8, max_lag=32),
}


class SynthCfg(C.Structure):
    """include/mtr_synth.h: mtr_synth_cfg"""
    _fields_ = [
        ("n_docs", C.c_uint32),
        ("ops_per_doc", C.c_uint32),
        ("writers", C.c_uint32),
        ("max_lag", C.c_uint32),
        ("w_insert", C.c_uint32),
        ("w_remove", C.c_uint32),
        ("w_annotate", C.c_uint32),
        ("max_text", C.c_uint32),
        ("nonbmp_permille", C.c_uint32),
        ("newline_permille", C.c_uint32),
        ("max_range", C.c_uint32),
        ("n_propops", C.c_uint32),
        ("doc_base", C.c_uint32),
        ("text_cap", C.c_uint32),
        ("seed", C.c_uint64),
    ]


def make_cfg(n_docs, ops_per_doc, writers=8, max_lag=32, weights=(45, 45, 10), max_text=16, nonbmp_permille=20,
             newline_permille=10, max_range=8, n_propops=64, doc_base=0, seed=0xfeedbed, text_cap=None) -> SynthCfg:
    if text_cap is None:
        text_cap = ops_per_doc * (max_text + 2) + 16
    return SynthCfg(n_docs, ops_per_doc, writers, max_lag, *weights, max_text, nonbmp_permille, newline_permille,
                    max_range, n_propops, doc_base, text_cap, seed)


def tables(writers=8, n_propops=64, seed=7) -> Batch:
    """A document-less batch holding the prop-op, key, value and client tables of the recipe."""
    it = Interner()
    rng = random.Random(seed)
    vals = {
        "bold": [True, False],
        "color": ["red", "green", "blue", "black"],
        "size": [10, 12, 14, 16],
        "1": ["a", "b"],
    }
    keys = list(vals)
    for _ in range(n_propops):
        chosen = rng.sample(keys, rng.choice([1, 1, 2]))
        it.propop({k: (None if rng.random() < 0.1 else rng.choice(vals[k])) for k in chosen})
    names = ["observer"] + [f"client-{k}" for k in range(1, writers + 1)]
    client_off, client_bytes = _offsets([to_utf8(js_string(c)[1:-1]) for c in names])
    po = np.zeros(len(it.propops) + 1, dtype="<u4")
    kv = []
    for i, pairs in enumerate(it.propops):
        po[i + 1] = po[i] + len(pairs)
        for k, v in pairs:
            kv.extend((k, v))
    key_off, key_bytes = _offsets(it.key_bytes)
    val_off, val_bytes = _offsets(it.val_bytes)
    return Batch(np.zeros(0, abi.DOC_DTYPE), np.zeros(0, abi.OP_DTYPE), np.zeros(0, "<u2"), po,
                 np.array(kv, dtype="<u4"), key_off, key_bytes, np.array(it.key_index, dtype="<u4"), val_off,
                 val_bytes, np.array(it.val_eq, dtype="<u4"), client_off, client_bytes)


def with_docs(tabs: Batch, docs, ops, text) -> Batch:
    """A batch of recorded documents that shares `tabs`' tables."""
    return Batch(docs, ops, text, tabs.propop_off, tabs.propop_kv, tabs.key_off, tabs.key_bytes, tabs.key_index,
                 tabs.val_off, tabs.val_bytes, tabs.val_eq, tabs.client_off, tabs.client_bytes)
