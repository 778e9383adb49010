// mtr_napi.cc -- the thin N-API addon a Node host (the TypeScript merge-tree shim) uses to drive
// libmtr.so through its C ABI (include/mtr.h).  No engine logic lives here: arguments are Buffers /
// TypedArrays / numbers, no exception crosses the C ABI, and engine errors come back as JS Errors
// (per-document asserts are rethrown by the shim as Error("0xNNN"), common-utils assert.ts:15-21).
//
// Built against the Node headers with g++ (fluidframework_amd/build.py); links libmtr.so next to it
// through an $ORIGIN rpath.
#include <node_api.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/mtr.h"

namespace {

#define NAPI_CALL(env, call)                                          \
    do {                                                              \
        if ((call) != napi_ok) {                                      \
            napi_throw_error((env), nullptr, "N-API call failed: " #call); \
            return nullptr;                                           \
        }                                                             \
    } while (0)

napi_value throw_engine(napi_env env, const std::string& what) {
    const std::string msg = what + ": " + mtr_last_error();
    napi_throw_error(env, nullptr, msg.c_str());
    return nullptr;
}

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < want) {
        napi_throw_type_error(env, nullptr, "wrong number of arguments");
        return false;
    }
    return true;
}

// engines with an asynchronous run / summarize in flight (only the JS thread touches this set: work is
// queued and completed there); every other entry point refuses a busy engine
std::set<mtr_engine*> g_busy;

mtr_engine* engine_of(napi_env env, napi_value v) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, nullptr, "not an engine handle (destroyed?)");
        return nullptr;
    }
    if (g_busy.count(static_cast<mtr_engine*>(p))) {
        napi_throw_error(env, nullptr, "engine busy: await the pending submitRunAsync / summarizeAsync first");
        return nullptr;
    }
    return static_cast<mtr_engine*>(p);
}

int64_t num_prop(napi_env env, napi_value obj, const char* name, int64_t dflt) {
    bool has = false;
    napi_value v;
    if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return dflt;
    if (napi_get_named_property(env, obj, name, &v) != napi_ok) return dflt;
    int64_t x = dflt;
    napi_get_value_int64(env, v, &x);
    return x;
}

// pointer + element count of a Buffer or TypedArray property
template <class T>
bool arr_prop(napi_env env, napi_value obj, const char* name, const T** p, size_t* n) {
    napi_value v;
    if (napi_get_named_property(env, obj, name, &v) != napi_ok) return false;
    bool is_buf = false, is_ta = false;
    napi_is_buffer(env, v, &is_buf);
    napi_is_typedarray(env, v, &is_ta);
    void* data = nullptr;
    size_t bytes = 0;
    if (is_ta) {
        napi_typedarray_type t;
        size_t len = 0, off = 0;
        napi_value ab;
        if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok) return false;
        size_t esz = 1;
        switch (t) {
            case napi_uint16_array: case napi_int16_array: esz = 2; break;
            case napi_uint32_array: case napi_int32_array: case napi_float32_array: esz = 4; break;
            case napi_float64_array: case napi_bigint64_array: case napi_biguint64_array: esz = 8; break;
            default: esz = 1; break;
        }
        bytes = len * esz;
    } else if (is_buf) {
        if (napi_get_buffer_info(env, v, &data, &bytes) != napi_ok) return false;
    } else {
        return false;
    }
    if (bytes % sizeof(T)) return false;
    *p = static_cast<const T*>(data);
    *n = bytes / sizeof(T);
    return true;
}

// (an engine with a job in flight is never finalized: the job holds a reference to its handle)
// per engine: the page-locked buffer replaySummaries downloads into (mtr_host_alloc), grown on demand
std::map<mtr_engine*, std::pair<uint8_t*, int64_t>> g_out;

void finalize_engine(napi_env, void* data, void*) {
    if (!data) return;
    auto* e = static_cast<mtr_engine*>(data);
    auto it = g_out.find(e);
    if (it != g_out.end()) {
        mtr_host_free(it->second.first);
        g_out.erase(it);
    }
    mtr_engine_destroy(e);
}

// createEngine(maxDocs, {device, newLengthCalc, snapshotV1, chunkSize, maxSegments, heapEntries,
//                        textUnits, propWords, removerCells, opsPerLaunch, refSlots})     client.ts:107
napi_value CreateEngine(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    uint32_t max_docs = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[0], &max_docs));
    mtr_options o{};
    o.new_length_calc = int32_t(num_prop(env, argv[1], "newLengthCalc", 0));
    o.snapshot_v1 = int32_t(num_prop(env, argv[1], "snapshotV1", 1));
    o.chunk_size = int32_t(num_prop(env, argv[1], "chunkSize", 10000));
    mtr_caps c{};
    c.max_segments = uint32_t(num_prop(env, argv[1], "maxSegments", 0));
    c.heap_entries = uint32_t(num_prop(env, argv[1], "heapEntries", 0));
    c.text_units = uint32_t(num_prop(env, argv[1], "textUnits", 0));
    c.prop_words = uint32_t(num_prop(env, argv[1], "propWords", 0));
    c.remover_cells = uint32_t(num_prop(env, argv[1], "removerCells", 0));
    c.ops_per_launch = uint32_t(num_prop(env, argv[1], "opsPerLaunch", 0));
    c.ref_slots = uint32_t(num_prop(env, argv[1], "refSlots", 0));
    const int device = int(num_prop(env, argv[1], "device", 0));
    mtr_engine* e = mtr_engine_create(&o, device, max_docs, &c);
    if (!e) return throw_engine(env, "mtr_engine_create");
    napi_value h;
    NAPI_CALL(env, napi_create_external(env, e, finalize_engine, nullptr, &h));
    return h;
}

// submit(h, batch) then apply: Client.applyMsg for every packed message (client.ts:858-887).
// The batch object carries the arrays of include/mtr_types.h (see index.js buildBatch).
bool parse_batch(napi_env env, napi_value o, mtr_batch& b) {
    size_t n = 0;
    bool ok = arr_prop(env, o, "docs", &b.docs, &n);
    b.n_docs = uint32_t(n);
    ok = ok && arr_prop(env, o, "ops", &b.ops, &n);
    b.n_ops = n;
    ok = ok && arr_prop(env, o, "text", &b.text, &n);
    b.n_text = n;
    ok = ok && arr_prop(env, o, "propopOff", &b.propop_off, &n);
    b.n_propops = uint32_t(n ? n - 1 : 0);
    ok = ok && arr_prop(env, o, "propopKv", &b.propop_kv, &n);
    ok = ok && arr_prop(env, o, "keyOff", &b.key_off, &n);
    b.n_keys = uint32_t(n ? n - 1 : 0);
    ok = ok && arr_prop(env, o, "keyBytes", &b.key_bytes, &n);
    ok = ok && arr_prop(env, o, "keyIndex", &b.key_index, &n);
    ok = ok && arr_prop(env, o, "valOff", &b.val_off, &n);
    b.n_vals = uint32_t(n ? n - 1 : 0);
    ok = ok && arr_prop(env, o, "valBytes", &b.val_bytes, &n);
    ok = ok && arr_prop(env, o, "valEq", &b.val_eq, &n);
    ok = ok && arr_prop(env, o, "clientOff", &b.client_off, &n);
    ok = ok && arr_prop(env, o, "clientBytes", &b.client_bytes, &n);
    if (!ok) napi_throw_type_error(env, nullptr, "malformed batch (see include/mtr_types.h)");
    return ok;
}

napi_value SubmitRun(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    mtr_batch b{};
    if (!parse_batch(env, argv[1], b)) return nullptr;
    // the host arrays belong to the JS heap: the copy must finish before returning
    if (mtr_submit(e, &b) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_submit");
    if (mtr_run(e) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_run");
    napi_value r;
    NAPI_CALL(env, napi_get_undefined(env, &r));
    return r;
}

// replaySummaries(h, batch, parts) -> {bytes: Buffer, docOff: Float64Array}: the summarizer's whole hand-over
// (mtr_replay_pipelined): upload, apply, summarize and every document's records in host memory, pipelined at both
// ends; document d's record is bytes[docOff[d], docOff[d + 1]) = u32 blob count, u32 lengths, the blobs
// (mtr_get_summaries' layout).  The records land in a page-locked buffer of the engine's, grown when a batch needs
// more (that batch then takes the serial summarize + download), and are copied into the returned Buffer.  The
// batch's arrays are the JS heap's: the upload is not overlapped unless they are page-locked.
// whether mtr_submit_pipelined would start every range of the batch: no record its op scan refuses (op_scan_kernel
// in mtr_engine.hip -- MTR_F_DELTA, reference records, the local-op path, rare records); a refused range would be
// left unapplied while the others ran, so such a batch takes the serial calls here instead
bool pipelinable(const mtr_batch& b) {
    for (uint64_t i = 0; i < b.n_ops; i++) {
        const mtr_op& op = b.ops[i];
        const uint32_t t = op.type;
        if ((op.flags & (MTR_F_DELTA | MTR_F_REL)) || t == MTR_OP_REF_CREATE || t == MTR_OP_REF_REMOVE ||
            t == MTR_OP_REF_ACK || t == MTR_OP_REBASE_POS || t == MTR_OP_LSEQ || t == MTR_OP_ACK ||
            t == MTR_OP_ROLLBACK || t == MTR_OP_REGENERATE || t == MTR_OP_RELPOS || t == MTR_OP_HANDLES ||
            t == MTR_OP_LOCAL_SETCELL || (t >= MTR_OP_LOCAL_INSERT && t <= MTR_OP_LOCAL_ANNOTATE && op.seq == -1) ||
            (t == MTR_OP_ANNOTATE && op.payload2 != 0) ||
            ((op.flags & MTR_F_MARKER) && op.payload2 != 0 &&
             (t == MTR_OP_INSERT || t == MTR_OP_LOCAL_INSERT || t == MTR_OP_LOAD)))
            return false;
    }
    return true;
}

napi_value ReplaySummaries(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    mtr_batch b{};
    if (!parse_batch(env, argv[1], b)) return nullptr;
    uint32_t parts = 16;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &parts));
    const uint32_t n = b.n_docs;
    auto& buf = g_out[e];
    if (!buf.first) {  // a first guess (64 MiB, or the batch's text at 16 bytes a unit): a larger need takes the
        // serial download once and grows the buffer for the next call
        buf.second = std::max<int64_t>(int64_t(64) << 20, int64_t(16) * int64_t(b.n_text) + 4096 * int64_t(n));
        buf.first = static_cast<uint8_t*>(mtr_host_alloc(uint64_t(buf.second)));
        if (!buf.first) {
            g_out.erase(e);
            return throw_engine(env, "mtr_host_alloc");
        }
    }
    std::vector<int64_t> off64(size_t(n) + 1, 0);
    const bool pipe = buf.first && pipelinable(b);
    int64_t total = pipe ? mtr_replay_pipelined(e, &b, parts, buf.first, buf.second, off64.data()) : -1;
    const bool piped = total >= 0;
    if (total < 0) {
        // a batch the pipelined path refuses, or a buffer too small (the batch is applied then)
        if (pipe && std::string(mtr_last_error()).find("output buffer holds") == std::string::npos)
            return throw_engine(env, "mtr_replay_pipelined");
        if (!pipe) {
            if (mtr_submit(e, &b) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_submit");
            if (mtr_run(e) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_run");
        }
        if (mtr_summarize(e) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_summarize");
        const int64_t need = -mtr_get_summaries(e, 0, n, nullptr, 0, nullptr);
        if (need < 0) return throw_engine(env, "mtr_get_summaries");
        if (!buf.first || buf.second < need) {
            if (buf.first) mtr_host_free(buf.first);
            buf.second = need + need / 4 + 4096;
            buf.first = static_cast<uint8_t*>(mtr_host_alloc(uint64_t(buf.second)));
            if (!buf.first) {
                g_out.erase(e);
                return throw_engine(env, "mtr_host_alloc");
            }
        }
        total = mtr_get_summaries(e, 0, n, buf.first, buf.second, off64.data());
        if (total < 0) return throw_engine(env, "mtr_get_summaries");
    }
    std::vector<double> off(size_t(n) + 1, 0.0);
    for (size_t d = 0; d <= n; d++) off[d] = double(off64[d]);
    napi_value r, bytes, ab, doff, pv;
    void* data = nullptr;
    NAPI_CALL(env, napi_create_buffer_copy(env, size_t(total), buf.first, &data, &bytes));
    NAPI_CALL(env, napi_create_arraybuffer(env, off.size() * sizeof(double), &data, &ab));
    std::memcpy(data, off.data(), off.size() * sizeof(double));
    NAPI_CALL(env, napi_create_typedarray(env, napi_float64_array, off.size(), ab, 0, &doff));
    NAPI_CALL(env, napi_get_boolean(env, piped, &pv));
    NAPI_CALL(env, napi_create_object(env, &r));
    NAPI_CALL(env, napi_set_named_property(env, r, "bytes", bytes));
    NAPI_CALL(env, napi_set_named_property(env, r, "docOff", doff));
    NAPI_CALL(env, napi_set_named_property(env, r, "pipelined", pv));
    return r;
}

// ---- asynchronous forms (napi_async_work + promise): the Node event loop keeps running while the
// GPU applies a batch / builds the summaries ("mtr_run async")
struct AsyncJob {
    napi_async_work work = nullptr;
    napi_deferred deferred = nullptr;
    napi_ref keep = nullptr;  // the batch object: its arrays must outlive the host->device copies
    napi_ref eref = nullptr;  // the engine handle: its finalizer (mtr_engine_destroy) must not run mid-job
    mtr_engine* e = nullptr;
    mtr_batch b{};
    bool summarize = false;
    int rc = 0;
    std::string err;
};

void job_execute(napi_env, void* data) {  // worker thread: no N-API calls here
    AsyncJob* j = static_cast<AsyncJob*>(data);
    if (j->summarize) {
        if (mtr_summarize(j->e) != MTR_OK || mtr_sync(j->e) != MTR_OK) {
            j->rc = -1;
            j->err = std::string("mtr_summarize: ") + mtr_last_error();
        }
        return;
    }
    if (mtr_submit(j->e, &j->b) != MTR_OK || mtr_sync(j->e) != MTR_OK) {
        j->rc = -1;
        j->err = std::string("mtr_submit: ") + mtr_last_error();
    } else if (mtr_run(j->e) != MTR_OK || mtr_sync(j->e) != MTR_OK) {
        j->rc = -1;
        j->err = std::string("mtr_run: ") + mtr_last_error();
    }
}

void job_complete(napi_env env, napi_status, void* data) {  // JS thread
    AsyncJob* j = static_cast<AsyncJob*>(data);
    g_busy.erase(j->e);
    if (j->keep) napi_delete_reference(env, j->keep);
    if (j->eref) napi_delete_reference(env, j->eref);
    napi_value v;
    if (j->rc == 0) {
        napi_get_undefined(env, &v);
        napi_resolve_deferred(env, j->deferred, v);
    } else {
        napi_value msg;
        napi_create_string_utf8(env, j->err.c_str(), NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, nullptr, msg, &v);
        napi_reject_deferred(env, j->deferred, v);
    }
    napi_delete_async_work(env, j->work);
    delete j;
}

napi_value queue_job(napi_env env, AsyncJob* j, const char* name) {
    napi_value promise, res;
    if (napi_create_promise(env, &j->deferred, &promise) != napi_ok ||
        napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &res) != napi_ok ||
        napi_create_async_work(env, nullptr, res, job_execute, job_complete, j, &j->work) != napi_ok ||
        napi_queue_async_work(env, j->work) != napi_ok) {
        if (j->keep) napi_delete_reference(env, j->keep);
        if (j->eref) napi_delete_reference(env, j->eref);
        delete j;
        napi_throw_error(env, nullptr, "cannot queue asynchronous engine work");
        return nullptr;
    }
    g_busy.insert(j->e);
    return promise;
}

// submitRunAsync(h, batch) -> Promise: submitRun on a worker thread
napi_value SubmitRunAsync(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    AsyncJob* j = new AsyncJob();
    j->e = e;
    if (!parse_batch(env, argv[1], j->b) || napi_create_reference(env, argv[1], 1, &j->keep) != napi_ok) {
        delete j;
        return nullptr;
    }
    if (napi_create_reference(env, argv[0], 1, &j->eref) != napi_ok) {
        napi_delete_reference(env, j->keep);
        delete j;
        return nullptr;
    }
    return queue_job(env, j, "mtr_submit_run");
}

// summarizeAsync(h) -> Promise: summarize on a worker thread
napi_value SummarizeAsync(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    AsyncJob* j = new AsyncJob();
    j->e = e;
    j->summarize = true;
    if (napi_create_reference(env, argv[0], 1, &j->eref) != napi_ok) {
        delete j;
        return nullptr;
    }
    return queue_job(env, j, "mtr_summarize");
}

// getContainingSegment(h, doc, pos, refSeq, client) -> null | {leaf, offset, length, seq, client,
// removedSeq, marker, refType, props, start, text}   (client.ts:1065, on the device)
napi_value GetContainingSegment(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    int32_t pos = 0, ref = 0, client = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    NAPI_CALL(env, napi_get_value_int32(env, argv[2], &pos));
    NAPI_CALL(env, napi_get_value_int32(env, argv[3], &ref));
    NAPI_CALL(env, napi_get_value_int32(env, argv[4], &client));
    mtr_segment_info si{};
    std::vector<uint16_t> text(1 << 16);
    if (mtr_get_containing_segment(e, doc, pos, ref, client, &si, text.data(), int64_t(text.size())) != MTR_OK)
        return throw_engine(env, "mtr_get_containing_segment");
    if (si.leaf >= 0 && !si.marker && si.length > int32_t(text.size())) {  // a longer text: ask again with room
        text.resize(size_t(si.length));
        if (mtr_get_containing_segment(e, doc, pos, ref, client, &si, text.data(), int64_t(text.size())) != MTR_OK)
            return throw_engine(env, "mtr_get_containing_segment");
    }
    napi_value r;
    if (si.leaf < 0) {
        NAPI_CALL(env, napi_get_null(env, &r));
        return r;
    }
    NAPI_CALL(env, napi_create_object(env, &r));
    const struct {
        const char* k;
        int32_t v;
    } f[] = {{"leaf", si.leaf},   {"offset", si.offset},         {"length", si.length}, {"seq", si.seq},
             {"client", si.client}, {"removedSeq", si.removed_seq}, {"marker", si.marker}, {"refType", si.ref_type},
             {"props", si.props}, {"start", si.start}, {"removed", si.removed}, {"localSeq", si.local_seq},
             {"localRemovedSeq", si.local_removed_seq}, {"groups", si.groups}};
    for (const auto& x : f) {
        napi_value v;
        NAPI_CALL(env, napi_create_int32(env, x.v, &v));
        NAPI_CALL(env, napi_set_named_property(env, r, x.k, v));
    }
    napi_value t;
    if (!si.marker && si.length <= int32_t(text.size())) {
        NAPI_CALL(env, napi_create_string_utf16(env, reinterpret_cast<const char16_t*>(text.data()), size_t(si.length), &t));
    } else {
        NAPI_CALL(env, napi_get_null(env, &t));
    }
    NAPI_CALL(env, napi_set_named_property(env, r, "text", t));
    return r;
}

// getRefPositions(h, doc) -> Int32Array: localReferencePositionToPosition of every local reference
// (client.ts:398-403, on the device; -1 = DetachedReferencePosition)
napi_value GetRefPositions(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    const int64_t n = mtr_get_ref_positions(e, doc, nullptr, 0);
    if (n < 0) return throw_engine(env, "mtr_get_ref_positions");
    void* data = nullptr;
    napi_value ab, r;
    NAPI_CALL(env, napi_create_arraybuffer(env, size_t(n) * 4, &data, &ab));
    if (n > 0 && mtr_get_ref_positions(e, doc, static_cast<int32_t*>(data), n) != n)
        return throw_engine(env, "mtr_get_ref_positions");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, size_t(n), ab, 0, &r));
    return r;
}

// getRefStates(h, doc) -> Int32Array [position, MTR_REF_ST_* bits] per local reference (mtr_get_ref_states): what an
// interval collection's summary order needs (sequence/src/intervalCollection.ts:1105-1112)
napi_value GetRefStates(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    const int64_t n = mtr_get_ref_states(e, doc, nullptr, 0);
    if (n < 0) return throw_engine(env, "mtr_get_ref_states");
    void* data = nullptr;
    napi_value ab, r;
    NAPI_CALL(env, napi_create_arraybuffer(env, size_t(n) * 8, &data, &ab));
    if (n > 0 && mtr_get_ref_states(e, doc, static_cast<int32_t*>(data), 2 * n) != n)
        return throw_engine(env, "mtr_get_ref_states");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, size_t(2 * n), ab, 0, &r));
    return r;
}

// getLeaves(h, doc) -> Int32Array of 5 ints per segment of a SharedMatrix vector (mtr_get_leaves): cachedLength,
// removed, start handle, tracking id, tracking-group bits -- what the undo provider reads (undoprovider.ts:138-170)
napi_value GetLeaves(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    const int64_t n = mtr_get_leaves(e, doc, nullptr, 0);
    if (n < 0) return throw_engine(env, "mtr_get_leaves");
    void* data = nullptr;
    napi_value ab, r;
    NAPI_CALL(env, napi_create_arraybuffer(env, size_t(n) * 20, &data, &ab));
    if (n > 0 && mtr_get_leaves(e, doc, static_cast<int32_t*>(data), n) != n) return throw_engine(env, "mtr_get_leaves");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, size_t(5 * n), ab, 0, &r));
    return r;
}

// getRefKeys(h, doc) -> Int32Array [position, MTR_REF_ST_* bits, compare key, offset] per local reference
// (mtr_get_ref_keys): a live interval collection's order (SequenceInterval.compare, intervalCollection.ts:505-539)
napi_value GetRefKeys(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    const int64_t n = mtr_get_ref_keys(e, doc, nullptr, 0);
    if (n < 0) return throw_engine(env, "mtr_get_ref_keys");
    void* data = nullptr;
    napi_value ab, r;
    NAPI_CALL(env, napi_create_arraybuffer(env, size_t(n) * 16, &data, &ab));
    if (n > 0 && mtr_get_ref_keys(e, doc, static_cast<int32_t*>(data), 4 * n) != n)
        return throw_engine(env, "mtr_get_ref_keys");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, size_t(4 * n), ab, 0, &r));
    return r;
}

// getViewLength(h, doc, refSeq, client) -> nodeLength(root) at that view (mtr_get_containing_segment past the end);
// this client's own short id at its currentSeq is getLength (markers count 1)
napi_value GetViewLength(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    int32_t ref = 0, client = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    NAPI_CALL(env, napi_get_value_int32(env, argv[2], &ref));
    NAPI_CALL(env, napi_get_value_int32(env, argv[3], &client));
    mtr_segment_info si;
    if (mtr_get_containing_segment(e, doc, INT32_MAX, ref, client, &si, nullptr, 0) != MTR_OK)
        return throw_engine(env, "mtr_get_containing_segment");
    napi_value r;
    NAPI_CALL(env, napi_create_int32(env, si.start, &r));
    return r;
}

// getRefInfo(h, doc, id) -> [leaf, offset, refType, held] (LocalReference.getSegment/getOffset, localReference.ts:106-112)
napi_value GetRefInfo(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0, id = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &id));
    int32_t out[4];
    if (mtr_get_ref_info(e, doc, id, out) == -2) return throw_engine(env, "mtr_get_ref_info");
    napi_value r;
    NAPI_CALL(env, napi_create_array_with_length(env, 4, &r));
    for (uint32_t k = 0; k < 4; k++) {
        napi_value v;
        NAPI_CALL(env, napi_create_int32(env, out[k], &v));
        NAPI_CALL(env, napi_set_element(env, r, k, v));
    }
    return r;
}

// summarize(h): every document's blobs on the device (Client.summarize, client.ts:966)
napi_value Summarize(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    if (mtr_summarize(e) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_summarize");
    napi_value r;
    NAPI_CALL(env, napi_get_undefined(env, &r));
    return r;
}

// getSummary(h, doc) -> [Buffer blob0, Buffer blob1, ...]   (header, body / body_0, ...)
napi_value GetSummary(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    int64_t n_blobs = 0, n_bytes = 0;
    if (mtr_summary_info(e, doc, &n_blobs, &n_bytes) != MTR_OK) return throw_engine(env, "mtr_summary_info");
    std::vector<int64_t> lens(size_t(n_blobs) + 1);
    std::vector<uint8_t> buf(size_t(n_bytes) + 1);
    const int64_t nb = mtr_get_summary(e, doc, buf.data(), int64_t(buf.size()), lens.data(), int32_t(n_blobs));
    if (nb < 0) return throw_engine(env, "mtr_get_summary");
    napi_value arr;
    NAPI_CALL(env, napi_create_array_with_length(env, size_t(nb), &arr));
    int64_t off = 0;
    for (int64_t k = 0; k < nb; k++) {
        napi_value b;
        NAPI_CALL(env, napi_create_buffer_copy(env, size_t(lens[k]), buf.data() + off, nullptr, &b));
        NAPI_CALL(env, napi_set_element(env, arr, uint32_t(k), b));
        off += lens[k];
    }
    return arr;
}

// getText(h, doc) -> string (MergeTreeTextHelper.getText, MergeTreeTextHelper.ts:20)
napi_value GetText(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    const int64_t n = mtr_get_text(e, doc, nullptr, 0);
    if (n < 0) return throw_engine(env, "mtr_get_text");
    std::vector<uint16_t> u(size_t(n) + 1);
    mtr_get_text(e, doc, u.data(), n);
    napi_value s;
    NAPI_CALL(env, napi_create_string_utf16(env, reinterpret_cast<const char16_t*>(u.data()), size_t(n), &s));
    return s;
}

// docStatus(h, doc) -> [status, opIndex]   (MTR_OK or MTR_ERR_*, 0x1000 | assert id)
napi_value DocStatus(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    int32_t op = -1;
    const int st = mtr_doc_status(e, doc, &op);
    napi_value arr, a, b;
    NAPI_CALL(env, napi_create_array_with_length(env, 2, &arr));
    NAPI_CALL(env, napi_create_int32(env, st, &a));
    NAPI_CALL(env, napi_create_int32(env, op, &b));
    NAPI_CALL(env, napi_set_element(env, arr, 0, a));
    NAPI_CALL(env, napi_set_element(env, arr, 1, b));
    return arr;
}

// stats(h) -> [ops, docs, maxLeaves, sumLeaves, badDocs, launches, maxHeap, maxText, sumLeavesBeforeOp, unitsInserted]
napi_value Stats(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    int64_t v[10] = {};
    if (mtr_stats(e, v, 10) != MTR_OK) return throw_engine(env, "mtr_stats");
    napi_value arr;
    NAPI_CALL(env, napi_create_array_with_length(env, 10, &arr));
    for (uint32_t i = 0; i < 10; i++) {
        napi_value x;
        NAPI_CALL(env, napi_create_double(env, double(v[i]), &x));
        NAPI_CALL(env, napi_set_element(env, arr, i, x));
    }
    return arr;
}

// reset(h): every document back to a fresh Client
napi_value Reset(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    if (mtr_reset(e) != MTR_OK || mtr_sync(e) != MTR_OK) return throw_engine(env, "mtr_reset");
    napi_value r;
    NAPI_CALL(env, napi_get_undefined(env, &r));
    return r;
}

// setMatrix(h, rowsDoc, colsDoc): the two PermutationVectors of one SharedMatrix (mtr_set_matrix)
napi_value GetDeltas(napi_env env, napi_callback_info info) {
    // getDeltas(engine, doc) -> Int32Array of [op, pos, len, kind] records (mtr_get_deltas)
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    std::vector<mtr_delta> d(1024);
    int64_t n = mtr_get_deltas(e, doc, d.data(), int64_t(d.size()));
    if (n == -1) return throw_engine(env, "mtr_get_deltas");
    if (n < 0) {
        d.resize(size_t(-n));
        n = mtr_get_deltas(e, doc, d.data(), int64_t(d.size()));
        if (n < 0) return throw_engine(env, "mtr_get_deltas");
    }
    void* data = nullptr;
    napi_value ab, arr;
    NAPI_CALL(env, napi_create_arraybuffer(env, size_t(n) * sizeof(mtr_delta), &data, &ab));
    if (n) std::memcpy(data, d.data(), size_t(n) * sizeof(mtr_delta));
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, size_t(n) * 4, ab, 0, &arr));
    return arr;
}
// getProps(engine, doc, ref) -> Uint32Array [n, key id, value id, ...] (mtr_get_props): the properties an
// MTR_DELTA_REGEN_X record references
napi_value GetProps(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t doc = 0, ref = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &ref));
    uint32_t one = 0;  // (cap 1: an empty set's single word fits, so -1 is always an error)
    int64_t n = mtr_get_props(e, doc, ref, &one, 1);
    if (n == -1) return throw_engine(env, "mtr_get_props");
    n = n < 0 ? -n : n;
    void* data = nullptr;
    napi_value ab, arr;
    NAPI_CALL(env, napi_create_arraybuffer(env, size_t(n) * 4, &data, &ab));
    if (mtr_get_props(e, doc, ref, static_cast<uint32_t*>(data), n) != n) return throw_engine(env, "mtr_get_props");
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, size_t(n), ab, 0, &arr));
    return arr;
}
napi_value SetMatrix(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mtr_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    uint32_t rows = 0, cols = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &rows));
    NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &cols));
    if (mtr_set_matrix(e, rows, cols) != MTR_OK) return throw_engine(env, "mtr_set_matrix");
    napi_value r;
    NAPI_CALL(env, napi_get_undefined(env, &r));
    return r;
}

napi_value Init(napi_env env, napi_value exports) {
    const struct {
        const char* name;
        napi_callback cb;
    } fns[] = {{"createEngine", CreateEngine}, {"submitRun", SubmitRun}, {"summarize", Summarize},
               {"getSummary", GetSummary},     {"getText", GetText},     {"docStatus", DocStatus},
               {"stats", Stats},               {"reset", Reset},         {"setMatrix", SetMatrix},
               {"getDeltas", GetDeltas},       {"submitRunAsync", SubmitRunAsync},
               {"summarizeAsync", SummarizeAsync}, {"getContainingSegment", GetContainingSegment},
               {"getProps", GetProps}, {"getRefPositions", GetRefPositions}, {"getRefInfo", GetRefInfo},
               {"getRefStates", GetRefStates}, {"getLeaves", GetLeaves}, {"getRefKeys", GetRefKeys},
               {"getViewLength", GetViewLength}, {"replaySummaries", ReplaySummaries}};
    for (const auto& f : fns) {
        napi_value fn;
        if (napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.cb, nullptr, &fn) != napi_ok ||
            napi_set_named_property(env, exports, f.name, fn) != napi_ok)
            return nullptr;
    }
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
