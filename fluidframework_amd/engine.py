"""ctypes binding of libmtr.so (include/mtr.h) and the observer-Client mirror.

The product path: a batch packed by :mod:`fluidframework_amd.batch` goes to the HIP engine through
the C ABI.  There is no CPU fallback -- if libmtr.so (gfx950 code object) cannot be loaded or no
HIP device is present, construction fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class EngineError(RuntimeError):
    pass


class MtrCaps(C.Structure):
    _fields_ = [
        ("max_segments", C.c_uint32),
        ("heap_entries", C.c_uint32),
        ("text_units", C.c_uint32),
        ("prop_words", C.c_uint32),
        ("remover_cells", C.c_uint32),
        ("ops_per_launch", C.c_uint32),
        ("ref_slots", C.c_uint32),
    ]


class SegmentInfo(C.Structure):
    """include/mtr.h: mtr_segment_info"""
    _fields_ = [(n, C.c_int32) for n in ("leaf", "offset", "length", "seq", "client", "removed_seq", "marker",
                                         "ref_type", "props", "start", "removed", "local_seq",
                                         "local_removed_seq", "groups")]


def lib():
    """Load libmtr.so (never falls back to anything else)."""
    global _LIB
    if _LIB is None:
        # MTR_LIB=libmtr_prof.so selects the phase-timer build (python -m fluidframework_amd.build --prof)
        path = os.path.join(_HERE, os.environ.get("MTR_LIB", "libmtr.so"))
        if not os.path.exists(path):
            raise EngineError(f"{path} missing: build it with `python -m fluidframework_amd.build`")
        L = C.CDLL(path)
        L.mtr_engine_create.restype = C.c_void_p
        L.mtr_engine_create.argtypes = [C.POINTER(abi.MtrOptions), C.c_int, C.c_uint32, C.POINTER(MtrCaps)]
        L.mtr_engine_destroy.argtypes = [C.c_void_p]
        for name in ("mtr_reset", "mtr_run", "mtr_summarize", "mtr_sync"):
            getattr(L, name).argtypes = [C.c_void_p]
            getattr(L, name).restype = C.c_int
        L.mtr_submit.argtypes = [C.c_void_p, C.c_void_p]
        L.mtr_submit.restype = C.c_int
        L.mtr_submit_pipelined.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        L.mtr_submit_pipelined.restype = C.c_int
        L.mtr_replay_pipelined.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64, C.c_void_p]
        L.mtr_replay_pipelined.restype = C.c_int64
        L.mtr_get_summary.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32]
        L.mtr_get_summary.restype = C.c_int64
        L.mtr_summary_info.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.mtr_summary_info.restype = C.c_int
        L.mtr_get_summaries.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int64, C.c_void_p]
        L.mtr_get_summaries.restype = C.c_int64
        L.mtr_host_alloc.argtypes = [C.c_uint64]
        L.mtr_host_alloc.restype = C.c_void_p
        L.mtr_host_free.argtypes = [C.c_void_p]
        L.mtr_host_free.restype = C.c_int
        L.mtr_summary_hashes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        L.mtr_summary_hashes.restype = C.c_int
        L.mtr_summary_bytes.argtypes = [C.c_void_p]
        L.mtr_summary_bytes.restype = C.c_int64
        L.mtr_get_text.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_text.restype = C.c_int64
        L.mtr_get_texts.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int64, C.c_void_p]
        L.mtr_get_texts.restype = C.c_int64
        L.mtr_get_containing_segment.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_int32,
                                                 C.POINTER(SegmentInfo), C.c_void_p, C.c_int64]
        L.mtr_get_containing_segment.restype = C.c_int
        L.mtr_doc_status.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_int32)]
        L.mtr_pending_groups.argtypes = [C.c_void_p, C.c_uint32]
        L.mtr_pending_groups.restype = C.c_int32
        L.mtr_doc_status.restype = C.c_int
        L.mtr_export.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64, C.POINTER(C.c_int32)]
        L.mtr_export.restype = C.c_int64
        L.mtr_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.mtr_stats.restype = C.c_int
        L.mtr_set_matrix.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.mtr_set_matrix.restype = C.c_int
        L.mtr_get_deltas.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_deltas.restype = C.c_int64
        L.mtr_get_props.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_props.restype = C.c_int64
        L.mtr_last_timing.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.mtr_last_timing.restype = C.c_int
        L.mtr_last_error.restype = C.c_char_p
        L.mtr_profile.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]
        L.mtr_profile.restype = C.c_int
        L.mtr_generate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.mtr_generate.restype = C.c_int
        L.mtr_generate_grown.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
        L.mtr_generate_grown.restype = C.c_int
        L.mtr_generate_matrix.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.mtr_generate_matrix.restype = C.c_int
        L.mtr_download_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_uint64]
        L.mtr_download_batch.restype = C.c_int
        L.mtr_get_ref_positions.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_ref_positions.restype = C.c_int64
        L.mtr_get_ref_states.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_ref_states.restype = C.c_int64
        L.mtr_get_ref_keys.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_ref_keys.restype = C.c_int64
        L.mtr_get_leaves.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64]
        L.mtr_get_leaves.restype = C.c_int64
        L.mtr_get_ref_info.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        L.mtr_get_ref_info.restype = C.c_int32
        _LIB = L
    return _LIB


def _err() -> str:
    return (lib().mtr_last_error() or b"").decode(errors="replace")


class _Pinned:
    """Owner of one mtr_host_alloc block (freed when the last array view goes away)."""

    def __init__(self, nbytes):
        self.p = lib().mtr_host_alloc(max(int(nbytes), 1))
        if not self.p:
            raise EngineError(f"mtr_host_alloc failed: {_err()}")
        self.nbytes = max(int(nbytes), 1)

    def __del__(self):
        if getattr(self, "p", None):
            lib().mtr_host_free(self.p)
            self.p = None


def pinned(shape, dtype) -> np.ndarray:
    """A numpy array in page-locked host memory (mtr_host_alloc): op uploads and summary downloads
    from it run at full PCIe rate."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) if np.ndim(shape) else int(shape)
    owner = _Pinned(n * dt.itemsize)
    buf = (C.c_uint8 * owner.nbytes).from_address(owner.p)
    buf._owner = owner  # the array holds `buf`, `buf` holds the owner
    return np.frombuffer(buf, dtype=dt, count=n).reshape(shape)


class Engine:
    """One engine = the observer Clients of up to ``max_docs`` documents on one GPU."""

    def __init__(self, max_docs, *, device=0, new_length_calc=False, snapshot_v1=True, chunk_size=10000,
                 max_segments=0, heap_entries=0, text_units=0, prop_words=0, remover_cells=0, ops_per_launch=0,
                 ref_slots=0):
        self.opts = abi.MtrOptions(int(new_length_calc), int(snapshot_v1), int(chunk_size), 0)
        self.caps = MtrCaps(max_segments, heap_entries, text_units, prop_words, remover_cells, ops_per_launch,
                            ref_slots)
        self.max_docs = int(max_docs)
        h = lib().mtr_engine_create(C.byref(self.opts), int(device), self.max_docs, C.byref(self.caps))
        if not h:
            raise EngineError(f"mtr_engine_create failed: {_err()}")
        self.h = h
        self._batch = None

    def close(self):
        if getattr(self, "h", None):
            lib().mtr_engine_destroy(self.h)
            self.h = None

    __del__ = close

    def _check(self, rc, what):
        if rc != 0:
            raise EngineError(f"{what} failed ({rc}): {_err()}")

    def reset(self):
        self._check(lib().mtr_reset(self.h), "mtr_reset")

    def submit(self, batch):
        self._batch = batch  # keep host arrays alive until the copies completed
        self._check(lib().mtr_submit(self.h, C.addressof(batch.c)), "mtr_submit")

    def submit_pipelined(self, batch, parts=16):
        """mtr_submit_pipelined: the op records and text go over in `parts` document ranges on a copy stream and the
        next run() starts each range as soon as it has landed (remote-op batches; see include/mtr.h).  The batch's
        arrays should be page-locked (Engine.download(..., pinned_memory=True)) for the copies to overlap."""
        self._batch = batch
        self._check(lib().mtr_submit_pipelined(self.h, C.addressof(batch.c), int(parts)), "mtr_submit_pipelined")

    def replay_pipelined(self, batch, out, parts=16):
        """mtr_replay_pipelined: upload, apply, summarize and download every document's summary records into
        `out` (a u1 array, page-locked for the copies to overlap), pipelined over `parts` document ranges.
        Returns (out, doc_off) like summaries()."""
        self._batch = batch
        n = int(batch.c.n_docs)
        doc_off = np.zeros(n + 1, dtype="<i8")
        r = lib().mtr_replay_pipelined(self.h, C.addressof(batch.c), int(parts), out.ctypes.data, out.size,
                                       doc_off.ctypes.data)
        if r < 0:
            raise EngineError(f"mtr_replay_pipelined failed: {_err()}")
        return out, doc_off

    def run(self):
        self._check(lib().mtr_run(self.h), "mtr_run")

    def set_matrix(self, rows_doc, cols_doc):
        """Documents rows_doc / cols_doc are the rows / cols PermutationVectors of one SharedMatrix
        (the rows document's op list drives both; see include/mtr.h mtr_set_matrix)."""
        self._check(lib().mtr_set_matrix(self.h, int(rows_doc), int(cols_doc)), "mtr_set_matrix")

    def summarize(self):
        self._check(lib().mtr_summarize(self.h), "mtr_summarize")

    def sync(self):
        self._check(lib().mtr_sync(self.h), "mtr_sync")

    def apply(self, batch):
        self.submit(batch)
        self.run()
        self.sync()

    def generate(self, cfg, tabs, grow=0):
        """Record mode: synthesize cfg.n_docs op logs (include/mtr_synth.h) with this engine's exact
        view lengths and apply them; the recorded batch stays on the device for replays.  grow > 0:
        every document first loads `grow` two-unit snapshot segments (config C5; mtr_generate_grown)."""
        self._tabs = tabs
        self._cfg = cfg
        self._grow = grow
        self._check(lib().mtr_generate_grown(self.h, C.byref(cfg), C.addressof(tabs.c), grow), "mtr_generate")

    def generate_matrix(self, cfg, tabs):
        """Record mode for SharedMatrix logs (mtr_synth_matrix_finish): cfg.n_docs matrices, matrix m
        = engine documents (2m rows, 2m+1 cols); the recorded logs stay on the device for replays."""
        self._tabs = tabs
        self._cfg = cfg
        self._grow = 0
        self._check(lib().mtr_generate_matrix(self.h, C.byref(cfg), C.addressof(tabs.c)), "mtr_generate_matrix")

    def download_matrix(self, lo, hi):
        """The recorded op lists of matrices [lo, hi) as a host Batch with one document per matrix (the
        layout of oracle.generate_matrix)."""
        from .synth import with_docs
        n = hi - lo
        per = self._cfg.ops_per_doc + 1
        docs = np.zeros(2 * n, dtype=abi.DOC_DTYPE)
        ops = np.zeros(max(n * per, 1), dtype=abi.OP_DTYPE)
        text = np.zeros(1, dtype="<u2")
        self._check(lib().mtr_download_batch(self.h, 2 * lo, 2 * hi, docs.ctypes.data, ops.ctypes.data,
                                             text.ctypes.data, 0), "mtr_download_batch")
        return with_docs(self._tabs, docs[0::2].copy(), ops[:n * per], text)

    def download(self, lo, hi, pinned_memory=False):
        """The recorded batch of documents [lo, hi) as a host Batch (sharing the recipe tables); with
        pinned_memory the op and text arrays live in page-locked memory (full-rate uploads)."""
        from .synth import with_docs
        n = hi - lo
        per = getattr(self, "_grow", 0) + self._cfg.ops_per_doc + 1
        alloc = (lambda k, dt: pinned(k, dt)) if pinned_memory else (lambda k, dt: np.zeros(k, dtype=dt))
        docs = np.zeros(n, dtype=abi.DOC_DTYPE)
        ops = alloc(n * per, abi.OP_DTYPE)
        cap = n * int(self._cfg.text_cap)
        text = alloc(max(cap, 1), "<u2")
        self._check(lib().mtr_download_batch(self.h, lo, hi, docs.ctypes.data, ops.ctypes.data, text.ctypes.data, cap),
                    "mtr_download_batch")
        used = int(docs["text_base"][-1] + docs["text_count"][-1]) if n else 0
        text = text[:max(used, 1)] if pinned_memory else text[:max(used, 1)].copy()
        return with_docs(self._tabs, docs, ops, text)

    def summary(self, doc) -> list[bytes]:
        nb, nbytes = C.c_int64(0), C.c_int64(0)
        self._check(lib().mtr_summary_info(self.h, doc, C.byref(nb), C.byref(nbytes)), "mtr_summary_info")
        out = np.zeros(max(nbytes.value, 1), dtype="u1")
        lens = np.zeros(max(nb.value, 1), dtype="<i8")
        r = lib().mtr_get_summary(self.h, doc, out.ctypes.data, out.size, lens.ctypes.data, nb.value)
        if r < 0:
            raise EngineError(f"mtr_get_summary failed ({r}): {_err()}")
        res, off = [], 0
        for k in range(r):
            res.append(out[off:off + lens[k]].tobytes())
            off += int(lens[k])
        return res

    def summaries(self, lo=0, hi=None, out=None):
        """Every blob of documents [lo, hi) in one device-to-host copy (mtr_get_summaries).  Returns
        (buffer, doc_off): document lo + i's record is buffer[doc_off[i]:doc_off[i + 1]] = u32 blob
        count nb, nb u32 lengths, the blob bytes.  `out` (a u1 array, e.g. pinned) is reused when big
        enough."""
        hi = self._n_docs() if hi is None else hi
        doc_off = np.zeros(hi - lo + 1, dtype="<i8")
        need = lib().mtr_get_summaries(self.h, lo, hi, None, 0, doc_off.ctypes.data)
        if need == -1:
            raise EngineError(_err())
        need = -need if need < 0 else need
        if out is None or out.size < need:
            out = np.zeros(max(need, 1), dtype="u1")
        r = lib().mtr_get_summaries(self.h, lo, hi, out.ctypes.data, out.size, doc_off.ctypes.data)
        if r < 0:
            raise EngineError(f"mtr_get_summaries failed ({r}): {_err()}")
        return out, doc_off

    @staticmethod
    def split_record(buf, a, b) -> list[bytes]:
        """The blobs of one document record of :meth:`summaries`."""
        nb = int(np.frombuffer(buf[a:a + 4].tobytes(), "<u4")[0])
        lens = np.frombuffer(buf[a + 4:a + 4 + 4 * nb].tobytes(), "<u4")
        res, off = [], a + 4 + 4 * nb
        for n in lens:
            res.append(buf[off:off + int(n)].tobytes())
            off += int(n)
        assert off == b, "malformed summary record"
        return res

    def _n_docs(self):
        return int(self.stats()["docs"])

    def hashes(self, n=None) -> np.ndarray:
        n = self.max_docs if n is None else n
        out = np.zeros(n, dtype="<u8")
        self._check(lib().mtr_summary_hashes(self.h, out.ctypes.data, n), "mtr_summary_hashes")
        return out

    def summary_bytes(self) -> int:
        return int(lib().mtr_summary_bytes(self.h))

    def text(self, doc) -> str:
        n = lib().mtr_get_text(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(_err())
        buf = np.zeros(max(n, 1), dtype="<u2")
        lib().mtr_get_text(self.h, doc, buf.ctypes.data, n)
        return buf[:n].tobytes().decode("utf-16-le", "surrogatepass")

    def texts(self, lo, hi) -> list[str]:
        """Local-view texts of documents [lo, hi): one device gather, one download (mtr_get_texts)."""
        off = np.zeros(hi - lo + 1, dtype="<i8")
        n = lib().mtr_get_texts(self.h, lo, hi, None, 0, off.ctypes.data)
        if n < 0:
            raise EngineError(_err())
        buf = np.zeros(max(n, 1), dtype="<u2")
        if n and lib().mtr_get_texts(self.h, lo, hi, buf.ctypes.data, n, off.ctypes.data) != n:
            raise EngineError(f"mtr_get_texts failed: {_err()}")
        return [buf[off[i]:off[i + 1]].tobytes().decode("utf-16-le", "surrogatepass") for i in range(hi - lo)]

    def props(self, doc, ref) -> list:
        """The properties an MTR_DELTA_REGEN_X record references (mtr_get_props): [(key id, value id)]."""
        # (a first buffer of 17 words: an empty set's single word fits, so -1 can only mean an error)
        out = np.zeros(17, dtype="<u4")
        n = lib().mtr_get_props(self.h, doc, ref, out.ctypes.data, len(out))
        if n == -1:
            raise EngineError(_err())
        if n < 0:
            out = np.zeros(-n, dtype="<u4")
            if lib().mtr_get_props(self.h, doc, ref, out.ctypes.data, len(out)) != len(out):
                raise EngineError(f"mtr_get_props failed: {_err()}")
        return [(int(out[1 + 2 * k]), int(out[2 + 2 * k])) for k in range(int(out[0]))]

    def deltas(self, doc) -> np.ndarray:
        """The delta ranges (abi.DELTA_DTYPE) of the MTR_F_DELTA ops of the last batch for one document."""
        cap = 1024  # cap >= 1, so -1 can only mean an error
        while True:
            out = np.zeros(cap, dtype=abi.DELTA_DTYPE)
            n = lib().mtr_get_deltas(self.h, doc, out.ctypes.data, cap)
            if n == -1:
                raise EngineError(_err())
            if n >= 0:
                break
            cap = -n
        return out[:n]

    def containing_segment(self, doc, pos, ref_seq, client):
        """Client.getContainingSegment(pos, {referenceSequenceNumber, clientId}) on the device:
        None when no segment covers pos, else a dict of mtr_segment_info fields plus the text."""
        info = SegmentInfo()
        text = np.zeros(1 << 12, dtype="<u2")
        self._check(lib().mtr_get_containing_segment(self.h, doc, pos, ref_seq, client, C.byref(info),
                                                     text.ctypes.data, text.size), "mtr_get_containing_segment")
        if info.leaf < 0:
            return None
        if not info.marker and info.length > text.size:  # the text did not fit: ask again with room for it
            text = np.zeros(info.length, dtype="<u2")
            self._check(lib().mtr_get_containing_segment(self.h, doc, pos, ref_seq, client, C.byref(info),
                                                         text.ctypes.data, text.size), "mtr_get_containing_segment")
        r = {n: getattr(info, n) for n, _ in SegmentInfo._fields_}
        r["text"] = None if info.marker else text[:info.length].tobytes().decode("utf-16-le", "surrogatepass")
        return r

    def view_length(self, doc, ref_seq, client) -> int:
        """nodeLength(root) at the (ref_seq, client) view (mtr_get_containing_segment past the end); this client's own
        short id at its currentSeq is SharedString.getLength."""
        info = SegmentInfo()
        self._check(lib().mtr_get_containing_segment(self.h, doc, 0x7fffffff, ref_seq, client, C.byref(info), None, 0),
                    "mtr_get_containing_segment")
        return int(info.start)

    def ref_positions(self, doc) -> list:
        """Client.localReferencePositionToPosition of every local reference of `doc`, by id
        (abi.DETACHED_POSITION = -1 when it has none)."""
        n = lib().mtr_get_ref_positions(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"mtr_get_ref_positions: {_err()}")
        if n == 0:
            return []
        out = np.zeros(n, dtype="<i4")
        self._check(int(lib().mtr_get_ref_positions(self.h, doc, out.ctypes.data, n) != n), "mtr_get_ref_positions")
        return [int(x) for x in out]

    def ref_states(self, doc) -> list:
        """[(position, state bits abi.REF_ST_*)] of every local reference of `doc`, by id (mtr_get_ref_states)."""
        n = lib().mtr_get_ref_states(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"mtr_get_ref_states: {_err()}")
        if n == 0:
            return []
        out = np.zeros(2 * n, dtype="<i4")
        self._check(int(lib().mtr_get_ref_states(self.h, doc, out.ctypes.data, 2 * n) != n), "mtr_get_ref_states")
        return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]

    def ref_keys(self, doc) -> list:
        """[(position, state bits, compare key, offset)] of every local reference of `doc`, by id (mtr_get_ref_keys:
        the key increases in tree order; -1 = no segment, -2 = a segment no longer in the tree)."""
        n = lib().mtr_get_ref_keys(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"mtr_get_ref_keys: {_err()}")
        if n == 0:
            return []
        out = np.zeros(4 * n, dtype="<i4")
        self._check(int(lib().mtr_get_ref_keys(self.h, doc, out.ctypes.data, 4 * n) != n), "mtr_get_ref_keys")
        return [tuple(int(x) for x in out[4 * i:4 * i + 4]) for i in range(n)]

    def leaves(self, doc) -> np.ndarray:
        """A matrix vector's segments in tree order, [n, 5] int32: cachedLength, removed, start handle, tracking id
        (-1: none), tracking-group bits (mtr_get_leaves)."""
        n = lib().mtr_get_leaves(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"mtr_get_leaves: {_err()}")
        out = np.zeros(5 * max(n, 1), dtype="<i4")
        self._check(int(lib().mtr_get_leaves(self.h, doc, out.ctypes.data, n) != n), "mtr_get_leaves")
        return out[:5 * n].reshape(n, 5)

    def ref_info(self, doc, ref_id):
        """(leaf index of the reference's segment or -1, offset, refType, held by the segment's collection)"""
        out = np.zeros(4, dtype="<i4")
        if lib().mtr_get_ref_info(self.h, doc, ref_id, out.ctypes.data) == -2:
            raise EngineError(f"mtr_get_ref_info: {_err()}")
        return int(out[0]), int(out[1]), int(out[2]), bool(out[3])

    def pending_groups(self, doc) -> int:
        """MergeTree.pendingSegments.length of document doc (its unacked local ops' SegmentGroups)."""
        n = lib().mtr_pending_groups(self.h, doc)
        if n < 0:
            raise EngineError(f"mtr_pending_groups: bad document {doc}")
        return int(n)

    def status(self, doc):
        op = C.c_int32(-1)
        st = lib().mtr_doc_status(self.h, doc, C.byref(op))
        return st, op.value

    def export(self, doc):
        h = C.c_int32(0)
        n = lib().mtr_export(self.h, doc, None, 0, C.byref(h))
        n = -n if n < 0 else n
        out = np.zeros((max(n, 1), 8), dtype="<i4")
        lib().mtr_export(self.h, doc, out.ctypes.data, n, C.byref(h))
        return out[:n], h.value

    def stats(self) -> dict:
        out = np.zeros(10, dtype="<i8")
        self._check(lib().mtr_stats(self.h, out.ctypes.data, 10), "mtr_stats")
        keys = ["ops", "docs", "max_leaves", "sum_leaves", "bad_docs", "launches", "max_heap", "max_text",
                "sum_leaves_before_op", "text_units_inserted"]
        return dict(zip(keys, (int(x) for x in out)))

    def profile(self, reset=True) -> dict:
        """Phase timers of a -DMTR_PROF build (empty dict otherwise)."""
        out = np.zeros(len(PROFILE_KEYS), dtype="<u8")
        if lib().mtr_profile(self.h, out.ctypes.data, len(PROFILE_KEYS), int(reset)) != 0:
            return {}
        return dict(zip(PROFILE_KEYS, (int(x) for x in out)))

    def timing(self) -> dict:
        out = np.zeros(4, dtype="<f8")
        lib().mtr_last_timing(self.h, out.ctypes.data, 4)
        return {"apply_ms": float(out[0]), "summary_ms": float(out[1]), "apply_launches": int(out[2]),
                "apply_kernel_ms": float(out[3])}


PROFILE_KEYS = ["op", "prefix", "split", "shift", "insert", "range", "zamboni", "zblock", "compact", "find_uid",
                "text_gc", "loadstore", "text_copy", "update_seq", "n_zblock", "n_compact", "scour1", "pack", "nlq",
                "pmatch", "tappend", "heap", "overflow", "n_pack", "n_merge", "n_pmatch", "n_nlq", "split1", "ins1",
                "fetch", "x1", "x2", "pf_sum", "pf_dirty", "materialize", "csum", "n_chunks", "n_listed", "n_dirty", "spread", "chunk_of", "n_spread",
                "load", "pre", "view", "post", "n_sup", "n_dch", "helper", "sink",
                "ovf_bounds", "ovf_parent", "n_ovf_nowin", "n_ovf_rounds", "sup_refresh", "px_list_eval", "px_eval",
                "px_sync", "n_px_rounds", "n_walk", "n_dirty_rounds", "walk"]


def caps_for(batch, margin=1.25):
    """Per-document arena capacities that a batch can never exceed (host-side bound)."""
    ops = batch.ops
    docs = batch.docs
    n_ops = docs["op_count"].astype(np.int64)
    max_ops = int(n_ops.max()) if len(docs) else 0
    max_text = int(docs["text_count"].max()) if len(docs) else 0
    seg = 2 * max_ops + 64
    text = int(2 * max_text * margin) + 4096
    npk = np.diff(batch.propop_off.astype(np.int64)) if len(batch.propop_off) > 1 else np.zeros(1, np.int64)
    max_keys = int(npk.max()) if npk.size else 0
    prop = int((2 * max_ops) * (1 + 2 * (max_keys + 8)) * 0.25) + 4096
    rem = max_ops + 64
    return dict(max_segments=seg, heap_entries=seg, text_units=text, prop_words=prop, remover_cells=rem)
