/*
 * mtr.h -- C ABI of the MI355X batched merge-tree replay engine (libmtr.so).
 *
 * The engine is a drop-in for the *observer* (all-ops-remote) path of
 * @fluidframework/merge-tree's Client (packages/dds/merge-tree/src/client.ts:98):
 * a scribe-like summarizer or a replay tool hands it ISequencedDocumentMessage
 * batches for many documents at once and asks for each document's summary.
 * Paths below are relative to the reference's packages/dds/merge-tree/src/.
 *
 *   reference                                      | engine
 *   -----------------------------------------------+------------------------------------------
 *   new Client(specToSegment, logger, options)      | mtr_engine_create   (client.ts:107-131)
 *     IMergeTreeOptions (mergeTree.ts:400-438)      |   mtr_options
 *   Client.startOrUpdateCollaboration(id, min, cur) | MTR_OP_START_COLLAB record (client.ts:1133)
 *   Client.applyMsg(msg) for every message          | mtr_submit + mtr_run (client.ts:858-887)
 *   Client.updateSeqNumbers(min, seq)               | MTR_F_LAST / MTR_OP_SEQ records (client.ts:877)
 *   Client.summarize(runtime, handle, ser, [])      | mtr_summarize + mtr_get_summary (client.ts:966)
 *   createTextHelper().getText(...)                 | mtr_get_text (MergeTreeTextHelper.ts:20)
 *   assert(cond, 0xNNN) / UsageError                | mtr_doc_status (per-document status word)
 *
 * No exceptions cross the ABI; every call returns MTR_OK (0) or an error code.
 * All pointers are host pointers; device memory is owned by the engine.
 */
#ifndef MTR_H
#define MTR_H

#include <stddef.h>
#include <stdint.h>

#include "mtr_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mtr_engine mtr_engine;

/* Per-document device arena capacities (0 = engine default). */
typedef struct mtr_caps {
    uint32_t max_segments;   /* leaf records per document */
    uint32_t heap_entries;   /* zamboni LRU heap entries per document (heap.ts:11) */
    uint32_t text_units;     /* UTF-16 text arena per document */
    uint32_t prop_words;     /* property-set arena per document (u32 words) */
    uint32_t remover_cells;  /* overlapping-remove list cells per document */
    uint32_t ops_per_launch; /* ops applied per document per kernel launch (0 = all) */
    uint32_t ref_slots;      /* local references per document (allocated with the first batch that creates one) */
} mtr_caps;

/* Create an engine for up to max_docs documents on HIP device `device`. */
mtr_engine* mtr_engine_create(const mtr_options* opt, int device, uint32_t max_docs, const mtr_caps* caps);
int mtr_engine_destroy(mtr_engine* e);

/* Forget every document (all state back to a fresh Client); keeps allocations. */
int mtr_reset(mtr_engine* e);

/* Copy a batch to the device (async on the engine stream).  Document i of the batch is
 * engine document i.  The batch's host arrays may be reused after mtr_sync. */
int mtr_submit(mtr_engine* e, const mtr_batch* b);

/* mtr_submit with the hand-over pipelined (SURVEY 8d's end-to-end path: a summarizer handing over sequenced
 * remote messages).  The batch's document descriptors and tables are copied at once; its op records and text
 * go over in `parts` document ranges on a copy stream, and the next mtr_run starts each range's documents as
 * soon as their records have landed, so the upload overlaps the apply of the ranges before it.  Same results as
 * mtr_submit + mtr_run.  The batch's host arrays must stay valid (and, for an overlapped copy, page-locked:
 * mtr_host_alloc) until mtr_run returns.  Only the remote-op path is pipelined: a range holding MTR_F_DELTA,
 * local-op, local-reference or rare records (op_scan) is not started, and mtr_run then returns
 * MTR_ERR_UNSUPPORTED -- mtr_reset and submit that batch with mtr_submit.  Documents must be laid out in order
 * (each document's op records and text after the previous one's); parts <= 1 is mtr_submit. */
int mtr_submit_pipelined(mtr_engine* e, const mtr_batch* b, uint32_t parts);

/* The whole end-to-end hand-over in one call: mtr_submit_pipelined + mtr_run + mtr_summarize + mtr_get_summaries
 * over every document, pipelined at both ends -- a range whose documents have no ops left is summarized and its
 * records downloaded into `out` (cap bytes; page-locked for the copies to overlap) while the later ranges still
 * upload and apply.  Writes doc_off[0..n_docs] (as mtr_get_summaries) and returns the byte count, or -1
 * (mtr_last_error).  When cap is too small the error text starts "mtr_replay_pipelined: the output buffer holds":
 * the batch is then applied in full and mtr_summarize + mtr_get_summaries give its records.  The summaries stay
 * readable afterwards
 * (mtr_get_summary, mtr_get_summaries, mtr_hashes).  A batch the pipelined path does not take (see
 * mtr_submit_pipelined), or whose ranges would hold fewer than 3,000 documents each (MTR_PIPE_MIN_PART_DOCS), runs
 * the serial calls.  Replaces, for a summarizer, the applyMsg loop followed by
 * summarizeCore (SURVEY 8d's end-to-end row). */
int64_t mtr_replay_pipelined(mtr_engine* e, const mtr_batch* b, uint32_t parts, uint8_t* out, int64_t cap,
                             int64_t* doc_off);

/* Apply the submitted ops (Client.applyMsg for each message, in order, per document). Async. */
int mtr_run(mtr_engine* e);

/* Declare documents rows_doc and cols_doc to be the rows and cols PermutationVectors of one
 * SharedMatrix (replaces `new PermutationVector(...)` x2 in the SharedMatrix constructor,
 * matrix.ts:106-121).  The rows document's op list drives both (see MTR_OP_SETCELL / MTR_F_COLS in
 * mtr_types.h); each vector's summary is its SnapshotV1 blobs followed by its handleTable blob
 * (PermutationVector.summarize, permutationvector.ts:310-325).  Persistent across mtr_reset. */
int mtr_set_matrix(mtr_engine* e, uint32_t rows_doc, uint32_t cols_doc);

/* The delta records (mtr_delta) of the MTR_F_DELTA ops of the last submitted batch for one document,
 * in op order: for a SharedString the SequenceDeltaEvent ranges SharedSegmentSequence turns into
 * catch-up ops (sequence.ts:697-736); for a SharedMatrix vector document the MTR_DELTA_CELL /
 * MTR_DELTA_RECYCLE records of its cell tracking (include/mtr_types.h).  Returns the count, or
 * -(count) if cap is too small.  mtr_submit sizes each document's buffer by an exact bound (see
 * mtr_submit in mtr_engine.hip). */
int64_t mtr_get_deltas(mtr_engine* e, uint32_t doc, mtr_delta* out, int64_t cap);

/* The properties an MTR_DELTA_REGEN_X record references (its len field): [n, key id, value id, ...] in JS
 * own-key order, the ids of the batch tables' keys and values -- the segment's `properties` that
 * createInsertSegmentOp serializes (client.ts:763-768 -> TextSegment / Marker.toJSONObject).  Returns the
 * word count 2n + 1, -(that) when cap is too small, -1 on a bad reference (pass cap >= 1: an empty set's one
 * word then always fits, so -1 is never a size).  Replaces reading
 * segment.properties in resetPendingDeltaToOps (client.ts:708-800). */
int64_t mtr_get_props(mtr_engine* e, uint32_t doc, uint32_t ref, uint32_t* out, int64_t cap);

/* Build every document's summary blobs on the device (Client.summarize). Async except for
 * one small size read-back between the sizing and writing passes. */
int mtr_summarize(mtr_engine* e);

/* Wait for all queued work on the engine stream. */
int mtr_sync(mtr_engine* e);

/* Size of one document's summary after mtr_summarize (SnapshotV1/Legacy emit, snapshotV1.ts:122-178,
 * snapshotlegacy.ts:122-182): *n_blobs = number of blobs, *n_bytes = their total payload bytes.
 * Callers size the buffers of mtr_get_summary from it.  Returns MTR_OK or -1 (mtr_last_error). */
int mtr_summary_info(mtr_engine* e, uint32_t doc, int64_t* n_blobs, int64_t* n_bytes);

/* Blobs of one document after mtr_summarize: writes them back-to-back to out (cap bytes),
 * blob_len[k] = bytes of blob k (order: header, body / body_0, body_1, ...).
 * Returns the number of blobs (>= 1); MTR_SUMMARY_TOO_SMALL when cap or max_blobs is smaller than
 * mtr_summary_info reports (nothing written); -1 on any other error (mtr_last_error). */
#define MTR_SUMMARY_TOO_SMALL (-3)
int64_t mtr_get_summary(mtr_engine* e, uint32_t doc, uint8_t* out, int64_t cap, int64_t* blob_len,
                        int32_t max_blobs);

/* Bulk download of the summaries of documents [lo, hi) in ONE device-to-host copy (a scribe hands
 * every blob of a batch to storage at once).  Layout: per document, in order, a little-endian u32
 * blob count nb, nb u32 blob lengths, then the blob bytes.  doc_off[i] (hi - lo + 1 entries) = offset
 * of document lo + i in out; doc_off[hi - lo] = total bytes.  Returns the total bytes, or -(bytes
 * needed) when cap is too small (nothing written; a non-empty range always needs >= 8 bytes), or -1
 * on error.  `out` may be pinned memory from mtr_host_alloc for full PCIe bandwidth. */
int64_t mtr_get_summaries(mtr_engine* e, uint32_t lo, uint32_t hi, uint8_t* out, int64_t cap, int64_t* doc_off);

/* Page-locked host memory (hipHostMalloc) for op batches and summary downloads; NULL on failure. */
void* mtr_host_alloc(uint64_t bytes);
int mtr_host_free(void* p);

/* 64-bit FNV-1a of every document's summary (blob lengths + bytes), n_docs entries. */
int mtr_summary_hashes(mtr_engine* e, uint64_t* out, uint32_t n_docs);

/* Total summary bytes of all documents (after mtr_summarize). */
int64_t mtr_summary_bytes(mtr_engine* e);

/* Local-view text of one document (UTF-16 units), gathered on the device
 * (MergeTreeTextHelper.getText, MergeTreeTextHelper.ts:20-81); returns the length (writes the text only
 * when it fits in cap units), -1 on error. */
int64_t mtr_get_text(mtr_engine* e, uint32_t doc, uint16_t* out, int64_t cap);

/* Local-view texts of documents [lo, hi) in one device gather and one download: doc_off[i] = first unit
 * of document lo + i in out, doc_off[hi - lo] = total.  Returns the total units (out NULL: a size query,
 * nothing written; doc_off filled either way), -1 when cap is too small or on error. */
int64_t mtr_get_texts(mtr_engine* e, uint32_t lo, uint32_t hi, uint16_t* out, int64_t cap, int64_t* doc_off);

/* Client.getContainingSegment(pos, {referenceSequenceNumber, clientId}) (client.ts:1065-1078 ->
 * mergeTree.ts:787-813): the segment holding position pos in the (ref_seq, client) view, found on the
 * device (one wave scans the document's visibility in that view).  client: a short id, -1
 * (LocalClientId) or -2 (NonCollabClient).  text (cap units, may be NULL) receives a text segment's
 * units.  Returns MTR_OK with info->leaf = -1 when no segment covers pos; then info->start is the view's length
 * (nodeLength(root) at that view: pos = INT32_MAX is a getLength query, SharedString.getLength for this client's own
 * view). */
typedef struct mtr_segment_info {
    int32_t leaf;        /* index of the leaf in tree order, -1 = none */
    int32_t offset;      /* pos - the segment's start in the view (getContainingSegment's offset) */
    int32_t length;      /* cachedLength */
    int32_t seq;         /* segment.seq */
    int32_t client;      /* segment.clientId: short id, -1 LocalClientId, -2 NonCollabClient */
    int32_t removed_seq; /* removedSeq; -1 = UnassignedSequenceNumber (a pending local remove) when removed,
                            else not removed (undefined) */
    int32_t marker;      /* 1 = Marker (text holds nothing; ref_type holds its refType) */
    int32_t ref_type;    /* marker refType / PermutationSegment start handle / text arena offset */
    int32_t props;       /* property-set index in the document's arena, -1 = none */
    int32_t start;       /* the segment's position in the view */
    int32_t removed;     /* 1 = the segment carries removal info (acked or pending) */
    int32_t local_seq;   /* localSeq of a pending local insert (then seq = -1), else -1 */
    int32_t local_removed_seq; /* localSeq of a pending local remove (then removed_seq = -1), else -1 */
    int32_t groups;      /* segmentGroups.size: the pending local ops the segment belongs to */
} mtr_segment_info;
int mtr_get_containing_segment(mtr_engine* e, uint32_t doc, int32_t pos, int32_t ref_seq, int32_t client,
                               mtr_segment_info* info, uint16_t* text, int64_t text_cap);

/* Local references (MTR_OP_REF_CREATE / MTR_OP_REF_REMOVE records, localReference.ts): out[r] =
 * Client.localReferencePositionToPosition of reference r (client.ts:398-403 -> mergeTree.ts:1046-1062),
 * MTR_DETACHED_POSITION (-1) when it has no position.  Returns the document's reference count (out written
 * only when it fits in cap), -1 on error. */
int64_t mtr_get_ref_positions(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap);
/* Every local reference of document doc as out[2r] = its position (as mtr_get_ref_positions) and out[2r+1] = state
 * bits: MTR_REF_ST_SEGMENT (LocalReference.getSegment() is defined, localReference.ts:106), MTR_REF_ST_HELD (that
 * segment's LocalReferenceCollection holds it, :357-384), MTR_REF_ST_REMOVED (that segment is in the tree and
 * removed).  An interval collection's compare (compareReferencePositions, referencePositions.ts:113-121) agrees
 * with the position order exactly when every endpoint is held by a live segment or has no segment at all
 * (DESIGN.md section 9).  Returns the reference count (out written only when 2*count fits in cap), -1 on error. */
int64_t mtr_get_ref_states(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap);
/* Every local reference of document doc as four int32: its position and state bits (as mtr_get_ref_states), then
 * compareReferencePositions' key (referencePositions.ts:113-121): a leaf key increasing in tree order (the segment's
 * ordinal order; -1 = no segment, -2 = a segment zamboni took out of the tree, whose ordinal the engine no longer
 * knows) and LocalReference.getOffset (localReference.ts:110).  A live interval collection orders its intervals by it
 * (SequenceInterval.compare, sequence/src/intervalCollection.ts:505-539), including endpoints left on removed
 * segments.  Returns the reference count (out written only when 4*count fits in cap), -1 on error. */
int64_t mtr_get_ref_keys(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap);
/* The segments of a SharedMatrix vector document in tree order (walkAllSegments, mergeTreeNodeWalk.ts:170), five
 * int32 each: cachedLength, 1 when removed (the local view does not show it, localNetLength, mergeTree.ts:613-634),
 * PermutationSegment.start (permutationvector.ts:53-72; MTR_HANDLE_UNALLOCATED), tracking id (-1: none) and its
 * group bits (include/mtr_types.h "Tracking groups").  The SharedMatrix undo host reads getPosition,
 * handleToPosition and the column handles from it (undoprovider.ts:138-170, matrix.ts:371-430).  Returns the
 * segment count (out written only when it fits in cap segments), -1 on error. */
int64_t mtr_get_leaves(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap);
/* Reference `id` of document doc: out[0] = index (tree order) of the leaf of its segment (LocalReference.
 * getSegment, localReference.ts:106; -1 = none, or the segment is no longer in the tree), out[1] = getOffset,
 * out[2] = refType, out[3] = 1 when the segment's LocalReferenceCollection holds it (has(), :357-384).
 * Returns out[0], or -2 on error. */
int32_t mtr_get_ref_info(mtr_engine* e, uint32_t doc, uint32_t id, int32_t* out);

/* MergeTree.pendingSegments.length (mergeTree.ts:1324-1357, asserted by client.applyMsg.spec.ts): the
 * SegmentGroups of this client's local ops that no sequenced message has acked yet; -1 = bad document. */
int32_t mtr_pending_groups(mtr_engine* e, uint32_t doc);

/* Per-document status: MTR_OK or an MTR_ERR_* code; *op_index = op that failed (or -1). */
int mtr_doc_status(mtr_engine* e, uint32_t doc, int32_t* op_index);

/* Leaf records of one document in the oracle's export format (8 int32 per leaf:
 * len, seq, client, removed_seq|INT32_MIN, n_removers, bnd, is_marker, props_hash).
 * Returns #leaves or -(needed); *height = tree height. */
int64_t mtr_export(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap_leaves, int32_t* height);

/* Engine-wide counters: out[0]=ops applied, out[1]=docs, out[2]=max leaves in any doc,
 * out[3]=sum of leaves, out[4]=docs with non-OK status, out[5]=kernel launches of the last run,
 * out[6]=max heap entries, out[7]=max text units used, out[8]=sum over applied ops of the leaf count
 * before the op, out[9]=UTF-16 units inserted.  Counters accumulate from mtr_reset. */
int mtr_stats(mtr_engine* e, int64_t* out, int32_t n);

/* Device time (ms) of the last mtr_run / mtr_summarize measured with HIP events: out[0]=apply
 * (wall, engine stream), out[1]=summarize, out[2]=apply kernel launches, out[3]=sum of the apply
 * launches' own durations (a round's size-class launches overlap on up to 4 streams). */
int mtr_last_timing(mtr_engine* e, double* out, int32_t n);

/* Record mode (synthetic workloads, include/mtr_synth.h): draw cfg->n_docs documents' op logs
 * with the engine's own exact view lengths, apply them, and keep the recorded batch on the device
 * (mtr_reset + mtr_run then replays it).  `tables` supplies prop-op/key/value/client tables. */
struct mtr_synth_cfg;
int mtr_generate(mtr_engine* e, const struct mtr_synth_cfg* cfg, const mtr_batch* tables);

/* Record mode with pre-grown documents (config C5): every document first loads `grow`
 * two-unit snapshot header segments (MTR_OP_LOAD records, reloadFromSegments) and starts
 * collaboration, then draws cfg->ops_per_doc messages as mtr_generate does; per document
 * grow + 1 + ops_per_doc records and cfg->text_cap >= 2 * grow + the messages' text.  Draws the same
 * logs as the oracle's oracle_generate_grown from the same seeds. */
int mtr_generate_grown(mtr_engine* e, const struct mtr_synth_cfg* cfg, const mtr_batch* tables, uint32_t grow);

/* Record mode for SharedMatrix workloads: cfg->n_docs matrices drawn from the
 * matrix recipe (mtr_synth_matrix_finish) with the engine's exact view lengths of both vectors.
 * Matrix m is the pair (rows = engine document 2m, cols = 2m + 1; paired as by mtr_set_matrix) and
 * its op list is the rows document's; the engine needs max_docs >= 2 * n_docs.  Draws the same logs
 * as the oracle's oracle_generate_matrix from the same seeds. */
int mtr_generate_matrix(mtr_engine* e, const struct mtr_synth_cfg* cfg, const mtr_batch* tables);

/* Copy the recorded batch of documents [lo, hi) to the host (compacted: op_begin/text_base are
 * rewritten relative to the copied arrays; text_cap = capacity of `text` in UTF-16 units). */
int mtr_download_batch(mtr_engine* e, uint32_t lo, uint32_t hi, mtr_doc_desc* docs, mtr_op* ops, uint16_t* text,
                       uint64_t text_cap);

/* Apply-kernel phase timers (thread-0 clock cycles summed over documents; see apply.hip.h P_*).
 * Only a -DMTR_PROF build collects them; otherwise returns MTR_ERR_UNSUPPORTED and zeros. */
int mtr_profile(mtr_engine* e, uint64_t* out, int32_t n, int32_t reset);

/* Debug: copy the scan arrays (E = inclusive visible-length prefix, V = visible length per leaf) that
 * the last op of HBM-resident document `doc` computed: out[0..n) = E, out[n..2n) = V.  Returns n or -1. */
int64_t mtr_debug_scan(mtr_engine* e, uint32_t doc, int32_t* out, int64_t n);

/* Human-readable description of the last engine-level error (static storage). */
const char* mtr_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MTR_H */
