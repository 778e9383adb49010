"""ctypes / numpy mirror of include/mtr_types.h (the packed, pointer-free batch format)."""
from __future__ import annotations

import ctypes as C

import numpy as np

OP_INSERT = 0
OP_REMOVE = 1
OP_ANNOTATE = 2
OP_SEQ = 3
OP_LOCAL_INSERT = 8
OP_LOCAL_REMOVE = 9
OP_LOCAL_ANNOTATE = 10
OP_START_COLLAB = 12
OP_LOAD = 13
OP_SETCELL = 14
OP_RELPOS = 15
OP_HANDLES = 16
OP_ACK = 17
OP_ROLLBACK = 18
OP_REGENERATE = 19
OP_REF_CREATE = 20
OP_REF_REMOVE = 21
OP_LOCAL_SETCELL = 22
OP_TRACK = 23
OP_REF_ACK = 24  # an interval collection's own ops (include/mtr_types.h)
OP_REBASE_POS = 25
OP_LSEQ = 26
REF_SLIDE = 1
REF_LOCALVIEW = 2
REF_LSEQ = 4
REF_SLOT = 8  # MTR_REF_SLOT: the reference takes id pos2 (a recycled slot, include/mtr_types.h)
# ReferenceType (ops.ts:9-36)
REFTYPE_SIMPLE = 0x0
REFTYPE_TILE = 0x1
REFTYPE_NEST_BEGIN = 0x2
REFTYPE_NEST_END = 0x4
REFTYPE_RANGE_BEGIN = 0x10
REFTYPE_RANGE_END = 0x20
REFTYPE_SLIDE_ON_REMOVE = 0x40
REFTYPE_STAY_ON_REMOVE = 0x80
REFTYPE_TRANSIENT = 0x100
DETACHED_POSITION = -1
REF_ST_SEGMENT = 1  # mtr_get_ref_states bits (include/mtr.h)
REF_ST_HELD = 2
REF_ST_REMOVED = 4
DELTA_REGEN = 64
DELTA_TLINK = 96  # tracking groups (include/mtr_types.h)
DELTA_TSPLIT = 97
DELTA_TMERGE = 98
TRACK_GROUPS = 32
DELTA_REGEN_X = 72
DELTA_REBASE = 80
REBASE_NOSLIDE = 1  # MTR_OP_REBASE_POS payload2: SharedMatrix.rebasePosition (no slide)
REL_BEFORE = 1
REL_OFFSET = 2
COMB_NONE, COMB_REWRITE, COMB_INCR, COMB_CONSENSUS, COMB_KEEP = 0, 1, 2, 3, 4
VEQ_NEVER = 0x80000000
VEQ_FALSY = 0x40000000
VEQ_INCR_STR = 0x20000000
VEQ_CONS_MUT = 0x10000000
VEQ_CLASS = 0x0FFFFFFF
PROPS_NEVER = 0x80000000
HANDLE_UNALLOCATED = -0x80000000
CLIENT_NONCOLLAB = 0xFFFE

F_LAST = 1
F_MARKER = 2
F_PROPS = 4
F_NOREF = 8
F_APPEND = 16
F_COLS = 32
F_DELTA = 64
F_REL = 128

NULL_VALUE = 0xFFFFFFFF
NOT_INDEX = 0xFFFFFFFF

MTR_OK = 0
MTR_ERR_INSERT_FAILED = 1
MTR_ERR_BAD_OP = 2
MTR_ERR_CAPACITY = 3
MTR_ERR_UNSUPPORTED = 4
MTR_ERR_ASSERT = 0x1000

OP_DTYPE = np.dtype(
    [
        ("type", "u1"),
        ("flags", "u1"),
        ("client", "<u2"),
        ("seq", "<i4"),
        ("ref_seq", "<i4"),
        ("min_seq", "<i4"),
        ("pos1", "<i4"),
        ("pos2", "<i4"),
        ("payload", "<u4"),
        ("payload2", "<u4"),
    ]
)
assert OP_DTYPE.itemsize == 32

DELTA_DTYPE = np.dtype([("op", "<u4"), ("pos", "<i4"), ("len", "<i4"), ("kind", "<u4")])  # mtr_delta

DOC_DTYPE = np.dtype(
    [
        ("op_begin", "<u8"),
        ("text_base", "<u8"),
        ("op_count", "<u4"),
        ("text_count", "<u4"),
        ("client_base", "<u4"),
        ("n_clients", "<u4"),
    ]
)
assert DOC_DTYPE.itemsize == 32


class MtrOptions(C.Structure):
    _fields_ = [
        ("new_length_calc", C.c_int32),
        ("snapshot_v1", C.c_int32),
        ("chunk_size", C.c_int32),
        ("reserved", C.c_int32),
    ]


class MtrBatch(C.Structure):
    _fields_ = [
        ("n_docs", C.c_uint32),
        ("n_propops", C.c_uint32),
        ("n_keys", C.c_uint32),
        ("n_vals", C.c_uint32),
        ("n_ops", C.c_uint64),
        ("n_text", C.c_uint64),
        ("docs", C.c_void_p),
        ("ops", C.c_void_p),
        ("text", C.c_void_p),
        ("propop_off", C.c_void_p),
        ("propop_kv", C.c_void_p),
        ("key_off", C.c_void_p),
        ("key_bytes", C.c_void_p),
        ("key_index", C.c_void_p),
        ("val_off", C.c_void_p),
        ("val_bytes", C.c_void_p),
        ("val_eq", C.c_void_p),
        ("client_off", C.c_void_p),
        ("client_bytes", C.c_void_p),
    ]


def ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data if a.size else 0
