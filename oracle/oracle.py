"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by the product package (fluidframework_amd).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from fluidframework_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: run `make -C {_HERE}`")
        L = C.CDLL(path)
        L.oracle_doc_new.restype = C.c_void_p
        L.oracle_doc_new.argtypes = [C.POINTER(abi.MtrOptions)]
        L.oracle_doc_free.argtypes = [C.c_void_p]
        L.oracle_doc_new_matrix.restype = C.c_void_p
        L.oracle_doc_new_matrix.argtypes = [C.POINTER(abi.MtrOptions)]
        L.oracle_doc_select.argtypes = [C.c_void_p, C.c_int32]
        L.oracle_doc_apply.restype = C.c_int
        L.oracle_doc_apply.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]
        L.oracle_doc_text.restype = C.c_int64
        L.oracle_doc_text.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_doc_summarize.restype = C.c_int64
        L.oracle_doc_summarize.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64,
                                           C.c_void_p, C.c_int32]
        L.oracle_doc_export.restype = C.c_int64
        L.oracle_doc_export.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int32)]
        L.oracle_doc_deltas.restype = C.c_int64
        L.oracle_doc_deltas.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_doc_regen_props.restype = C.c_int64
        L.oracle_doc_regen_props.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.oracle_doc_state.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_doc_pending_groups.argtypes = [C.c_void_p]
        L.oracle_doc_pending_groups.restype = C.c_int32
        L.oracle_set_trace.argtypes = [C.c_int]
        L.oracle_generate.restype = C.c_int
        L.oracle_generate.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(abi.MtrOptions), C.c_uint32, C.c_uint32,
                                      C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_generate_grown.restype = C.c_int
        L.oracle_generate_grown.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(abi.MtrOptions), C.c_uint32,
                                            C.c_uint32, C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p]
        L.oracle_generate_matrix.restype = C.c_int
        L.oracle_generate_matrix.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(abi.MtrOptions), C.c_uint32,
                                             C.c_uint32, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_replay_batch.restype = C.c_double
        L.oracle_replay_batch.argtypes = [C.c_void_p, C.POINTER(abi.MtrOptions), C.c_uint32, C.c_uint32, C.c_int,
                                          C.c_void_p, C.c_void_p]
        L.oracle_replay_matrix_batch.restype = C.c_double
        L.oracle_replay_matrix_batch.argtypes = [C.c_void_p, C.POINTER(abi.MtrOptions), C.c_uint32, C.c_uint32,
                                                 C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_set_psl_check.argtypes = [C.c_int]
        L.oracle_psl_stats.restype = C.c_int64
        L.oracle_psl_stats.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
        L.oracle_doc_containing.restype = C.c_int32
        L.oracle_doc_containing.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
        L.oracle_doc_marker_position.restype = C.c_int32
        L.oracle_doc_marker_position.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32]
        L.oracle_doc_containing_props.restype = C.c_int64
        L.oracle_doc_containing_props.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int64]
        L.oracle_doc_length.restype = C.c_int64
        L.oracle_doc_length.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        L.oracle_doc_ref_positions.restype = C.c_int64
        L.oracle_doc_ref_positions.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_doc_handle_at.restype = C.c_int32
        L.oracle_doc_handle_at.argtypes = [C.c_void_p, C.c_int32]
        L.oracle_doc_leaves.restype = C.c_int64
        L.oracle_doc_leaves.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_doc_track_group.restype = C.c_int64
        L.oracle_doc_track_group.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64]
        L.oracle_doc_ref_states.restype = C.c_int64
        L.oracle_doc_ref_states.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_doc_ref_keys.restype = C.c_int64
        L.oracle_doc_ref_keys.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_doc_ref_key.restype = C.c_int32
        L.oracle_doc_ref_key.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.oracle_doc_set_slide_hook.restype = None
        L.oracle_doc_set_slide_hook.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_doc_ref_info.restype = C.c_int32
        L.oracle_doc_ref_info.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        _LIB = L
    return _LIB


class psl_check:
    """Context manager: oracle documents created inside keep the reference's PartialSequenceLengths
    and compare every remote block-length query with the leaf sum (oracle/psl.h).  `.stats()` ->
    (queries checked, mismatches, first mismatch); `.rootlag` = leaf-level root queries that read high
    (the reference's stale-root quirk, harmless where the reference reads it)."""

    def __enter__(self):
        lib().oracle_set_psl_check(1)
        return self

    def stats(self):
        out = np.zeros(3, dtype="<i8")
        buf = C.create_string_buffer(512)
        lib().oracle_psl_stats(out.ctypes.data, buf, 512)
        self.rootlag = int(out[2])
        return int(out[0]), int(out[1]), buf.value.decode()

    def __exit__(self, *exc):
        lib().oracle_set_psl_check(0)
        return False


class psl_answer(psl_check):
    """Context manager: oracle documents created inside answer every remote block length from their
    PartialSequenceLengths (getPartialLength, partialLengths.ts:698-735, O(log W) per block), as the
    reference does, instead of summing the block's leaves -- the reference's algorithm for bench.py's
    CPU baseline.  (No cross-check: the leaf-sum path stays the tests' checker.)"""

    def __enter__(self):
        lib().oracle_set_psl_check(2)
        return self


def options(new_length_calc=False, snapshot_v1=True, chunk_size=10000):
    return abi.MtrOptions(int(new_length_calc), int(snapshot_v1), int(chunk_size), 0)


class OracleDoc:
    def __init__(self, opts=None, matrix=False):
        self.opts = opts or options()
        self.matrix = matrix
        self.h = (lib().oracle_doc_new_matrix if matrix else lib().oracle_doc_new)(C.byref(self.opts))

    def select(self, which: int) -> "OracleDoc":
        """Matrix documents: direct queries at the rows (0) or cols (1) PermutationVector."""
        lib().oracle_doc_select(self.h, which)
        return self

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_doc_free(self.h)
            self.h = None

    def apply(self, batch, doc_index, lo=0, hi=None):
        if hi is None:
            hi = int(batch.docs[doc_index]["op_count"])
        return lib().oracle_doc_apply(self.h, C.addressof(batch.c), doc_index, lo, hi)

    def text(self) -> str:
        n = lib().oracle_doc_text(self.h, None, 0)
        buf = np.zeros(max(n, 1), dtype="<u2")
        lib().oracle_doc_text(self.h, buf.ctypes.data, n)
        return buf[:n].tobytes().decode("utf-16-le", "surrogatepass")

    def summarize(self, batch, doc_index) -> list[bytes]:
        cap = 1 << 16
        while True:
            out = np.zeros(cap, dtype="u1")
            lens = np.zeros(4096, dtype="<i8")
            r = lib().oracle_doc_summarize(self.h, C.addressof(batch.c), doc_index, out.ctypes.data, cap,
                                           lens.ctypes.data, 4096)
            if r >= 0:
                blobs = []
                off = 0
                for i in range(r):
                    blobs.append(out[off:off + lens[i]].tobytes())
                    off += lens[i]
                return blobs
            cap = -r + 16

    def export(self):
        h = C.c_int32(0)
        n = lib().oracle_doc_export(self.h, None, 0, C.byref(h))
        n = -n if n < 0 else n
        out = np.zeros((max(n, 1), 8), dtype="<i4")
        lib().oracle_doc_export(self.h, out.ctypes.data, n, C.byref(h))
        return out[:n], h.value

    def deltas(self) -> np.ndarray:
        """Delta ranges (abi.DELTA_DTYPE) of the MTR_F_DELTA ops applied since the last call."""
        n = lib().oracle_doc_deltas(self.h, None, 0)
        n = -n if n < 0 else n
        out = np.zeros(max(n, 1), dtype=abi.DELTA_DTYPE)
        lib().oracle_doc_deltas(self.h, out.ctypes.data, n)
        return out[:n]

    def regen_props(self, ref: int) -> list:
        """The properties an MTR_DELTA_REGEN_X record references: [(key id, value id), ...] in JS order."""
        n = lib().oracle_doc_regen_props(self.h, ref, None, 0)
        if n == -1:
            raise ValueError(f"no properties reference {ref}")
        n = -n if n < 0 else n
        out = np.zeros(max(n, 1), dtype="<u4")
        lib().oracle_doc_regen_props(self.h, ref, out.ctypes.data, n)
        return [(int(out[1 + 2 * k]), int(out[2 + 2 * k])) for k in range(int(out[0]))]

    def state(self):
        out = np.zeros(4, dtype="<i8")
        lib().oracle_doc_state(self.h, out.ctypes.data)
        return out

    def pending_groups(self) -> int:
        """MergeTree.pendingSegments.length"""
        return int(lib().oracle_doc_pending_groups(self.h))

    def containing(self, pos, ref_seq, client):
        """getContainingSegment -> (leaf index or -1, offset, cachedLength, segment start)."""
        out = np.zeros(4, dtype="<i4")
        lib().oracle_doc_containing(self.h, pos, ref_seq, client, out.ctypes.data)
        return tuple(int(x) for x in out) if out[0] >= 0 else (-1, 0, 0, 0)

    def containing_props(self, pos, ref_seq, client):
        """getContainingSegment's segment -> (segmentGroups.size, [(key id, value id)] or None when its
        properties are undefined); None when no segment covers pos."""
        out = np.zeros(256, dtype="<u4")
        n = lib().oracle_doc_containing_props(self.h, pos, ref_seq, client, out.ctypes.data, out.size)
        if n == -1:
            return None
        if n < -1:
            out = np.zeros(-n, dtype="<u4")
            lib().oracle_doc_containing_props(self.h, pos, ref_seq, client, out.ctypes.data, out.size)
        pairs = [(int(out[3 + 2 * k]), int(out[4 + 2 * k])) for k in range(int(out[2]))]
        return int(out[0]), (pairs if out[1] else None)

    def marker_position(self, ordinal, ref_seq, client):
        """getPosition of the marker mapped to a host marker ordinal at (refSeq, clientId); -1 if none."""
        return lib().oracle_doc_marker_position(self.h, ordinal, ref_seq, client)

    def length(self, ref_seq, client):
        return lib().oracle_doc_length(self.h, ref_seq, client)

    def handle_at(self, pos: int) -> int:
        """The handle at local position pos of the selected vector (HANDLE_UNALLOCATED, -1 = no segment)."""
        return lib().oracle_doc_handle_at(self.h, pos)

    def leaves(self) -> np.ndarray:
        """The selected vector's segments, [n, 5] int32 as Engine.leaves (mtr_get_leaves)."""
        n = lib().oracle_doc_leaves(self.h, None, 0)
        n = -n if n < 0 else n
        out = np.zeros(5 * max(n, 1), dtype="<i4")
        lib().oracle_doc_leaves(self.h, out.ctypes.data, n)
        return out[:5 * n].reshape(n, 5)

    def track_group(self, bit: int) -> list:
        """Tracking ids of the selected vector's tracking group `bit`, in the TrackingGroup's order."""
        n = lib().oracle_doc_track_group(self.h, bit, None, 0)
        n = -n if n < 0 else n
        out = np.zeros(max(n, 1), dtype="<i4")
        lib().oracle_doc_track_group(self.h, bit, out.ctypes.data, n)
        return [int(x) for x in out[:n]]

    def ref_positions(self) -> list:
        """localReferencePositionToPosition of every local reference, by id (-1 = detached)."""
        n = lib().oracle_doc_ref_positions(self.h, None, 0)
        n = -n if n < 0 else n
        out = np.zeros(max(n, 1), dtype="<i4")
        lib().oracle_doc_ref_positions(self.h, out.ctypes.data, n)
        return [int(x) for x in out[:n]]

    def ref_states(self) -> list:
        """[(position, abi.REF_ST_* bits)] of every local reference, by id (as Engine.ref_states)."""
        n = lib().oracle_doc_ref_states(self.h, None, 0)
        n = -n if n < 0 else n
        out = np.zeros(max(2 * n, 1), dtype="<i4")
        lib().oracle_doc_ref_states(self.h, out.ctypes.data, 2 * n)
        return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]

    def ref_keys(self) -> list:
        """[(position, state bits, compare key, offset)] of every local reference, by id (as Engine.ref_keys; the key
        is the segment's leaf index)."""
        n = lib().oracle_doc_ref_keys(self.h, None, 0)
        n = -n if n < 0 else n
        out = np.zeros(max(4 * n, 1), dtype="<i4")
        lib().oracle_doc_ref_keys(self.h, out.ctypes.data, 4 * n)
        return [tuple(int(x) for x in out[4 * i:4 * i + 4]) for i in range(n)]

    def ref_key(self, ref_id: int):
        """(tree-order index of the reference's segment: -1 none, -2 no longer in the tree; getOffset())"""
        out = np.zeros(2, dtype="<i4")
        if lib().oracle_doc_ref_key(self.h, ref_id, out.ctypes.data) == -3:
            raise ValueError(f"no local reference {ref_id}")
        return int(out[0]), int(out[1])

    SLIDE_HOOK = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32)

    def set_slide_hook(self, fn) -> None:
        """fn(ref_id, phase) -- phase 0 = beforeSlide, 1 = afterSlide -- during apply(); None clears."""
        self._hook = None if fn is None else self.SLIDE_HOOK(lambda ctx, r, ph: fn(r, ph))
        lib().oracle_doc_set_slide_hook(self.h, C.cast(self._hook, C.c_void_p) if self._hook else None, None)

    def ref_info(self, ref_id: int):
        """(leaf index of the reference's segment or -1, offset, refType, held by the segment's collection)"""
        out = np.zeros(4, dtype="<i4")
        lib().oracle_doc_ref_info(self.h, ref_id, out.ctypes.data)
        return tuple(int(x) for x in out[:3]) + (bool(out[3]),)


def replay_batch(batch, lo, hi, threads, opts=None):
    """Replay documents [lo, hi) on `threads` host threads -> (seconds, digests, statuses)."""
    opts = opts or options()
    n = hi - lo
    hashes = np.zeros(n, dtype="<u8")
    status = np.zeros(n, dtype="<i4")
    secs = lib().oracle_replay_batch(C.addressof(batch.c), C.byref(opts), lo, hi, threads, hashes.ctypes.data,
                                     status.ctypes.data)
    return secs, hashes, status


def replay_matrix_batch(batch, lo, hi, threads, opts=None):
    """Replay matrices [lo, hi) (one document per matrix) -> (seconds, digests [rows, cols] per
    matrix, statuses)."""
    opts = opts or options()
    n = hi - lo
    hashes = np.zeros(2 * n, dtype="<u8")
    status = np.zeros(n, dtype="<i4")
    secs = lib().oracle_replay_matrix_batch(C.addressof(batch.c), C.byref(opts), lo, hi, threads,
                                            hashes.ctypes.data, status.ctypes.data)
    return secs, hashes, status


def _mix64(z):
    M = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M
    return z ^ (z >> 31)


def summary_digest(blobs):
    """Python restatement of the summary digest (include/mtr_digest.h)."""
    M = (1 << 64) - 1
    h = _mix64(len(blobs) ^ 0x6d74723634)
    for b in blobs:
        s = 0
        for j in range(0, len(b), 8):
            w = int.from_bytes(b[j:j + 8].ljust(8, b"\0"), "little")
            s = (s + _mix64(w ^ (((j // 8 + 1) * 0x9e3779b97f4a7c15) & M))) & M
        h = _mix64(h ^ _mix64(s ^ ((len(b) * 0xd6e8feb86659fd93) & M)))
    return h


def generate(cfg, tabs, lo, hi, threads=8, opts=None, grow=0):
    """Synthetic op logs of documents [lo, hi) recorded with the oracle as the exact simulator
    -> (Batch, summary digests, statuses).  grow > 0: every document first loads `grow` two-unit
    header segments (config C5's pre-grown documents); cfg.text_cap must cover 2 * grow more units."""
    from fluidframework_amd.synth import with_docs
    opts = opts or options()
    n = hi - lo
    per = grow + cfg.ops_per_doc + 1
    ops = np.zeros(n * per, dtype=abi.OP_DTYPE)
    text = np.zeros(n * int(cfg.text_cap), dtype="<u2")
    counts = np.zeros(n, dtype="<u4")
    hashes = np.zeros(n, dtype="<u8")
    status = np.zeros(n, dtype="<i4")
    lib().oracle_generate_grown(C.byref(cfg), C.addressof(tabs.c), C.byref(opts), lo, hi, threads, grow,
                                ops.ctypes.data, text.ctypes.data, counts.ctypes.data, hashes.ctypes.data,
                                status.ctypes.data)
    docs = np.zeros(n, dtype=abi.DOC_DTYPE)
    docs["op_begin"] = np.arange(n, dtype=np.uint64) * per
    docs["op_count"] = per
    docs["text_count"] = counts
    # compact the text regions
    bases = np.zeros(n, dtype=np.uint64)
    if n:
        bases[1:] = np.cumsum(counts.astype(np.uint64))[:-1]
    docs["text_base"] = bases
    docs["client_base"] = 0
    docs["n_clients"] = cfg.writers + 1
    packed = np.concatenate([text[i * int(cfg.text_cap): i * int(cfg.text_cap) + int(counts[i])] for i in range(n)]) \
        if n else np.zeros(0, "<u2")
    return with_docs(tabs, docs, ops, packed), hashes, status


def generate_matrix(cfg, tabs, lo, hi, threads=8, opts=None):
    """SharedMatrix op logs (mtr_synth_matrix_finish) of matrices [lo, hi) recorded with the oracle
    -> (Batch with one document per matrix (the rows vector's op list), digests, statuses)."""
    from fluidframework_amd.synth import with_docs
    opts = opts or options()
    n = hi - lo
    per = cfg.ops_per_doc + 1
    ops = np.zeros(n * per, dtype=abi.OP_DTYPE)
    hashes = np.zeros(n, dtype="<u8")
    status = np.zeros(n, dtype="<i4")
    lib().oracle_generate_matrix(C.byref(cfg), C.addressof(tabs.c), C.byref(opts), lo, hi, threads,
                                 ops.ctypes.data, hashes.ctypes.data, status.ctypes.data)
    docs = np.zeros(n, dtype=abi.DOC_DTYPE)
    docs["op_begin"] = np.arange(n, dtype=np.uint64) * per
    docs["op_count"] = per
    docs["n_clients"] = cfg.writers + 1
    return with_docs(tabs, docs, ops, np.zeros(0, "<u2")), hashes, status
