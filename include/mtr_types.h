/*
 * mtr_types.h -- packed, pointer-free input format shared by the HIP engine
 * (fluidframework_amd/csrc) and the CPU oracle (oracle/).
 *
 * One mtr_op is one *member op* of an ISequencedDocumentMessage
 * (common/lib/protocol-definitions/src/protocol.ts:212).  A message whose
 * contents is a GROUP op (packages/dds/merge-tree/src/ops.ts:113) becomes
 * several mtr_op records with the same seq; only the last one carries
 * MTR_F_LAST, which triggers Client.updateSeqNumbers(msn, seq)
 * (packages/dds/merge-tree/src/client.ts:858-887).  A message of any other
 * type (join/leave/noop) becomes one MTR_OP_SEQ record.
 *
 * Plain C, fixed-width fields, no torch or STL types.
 */
#ifndef MTR_TYPES_H
#define MTR_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* op.type -- MergeTreeDeltaType (ops.ts:43-48) plus engine-only records */
enum {
    MTR_OP_INSERT = 0,          /* remote insert  (client.ts:489)  */
    MTR_OP_REMOVE = 1,          /* remote remove  (client.ts:430)  */
    MTR_OP_ANNOTATE = 2,        /* remote annotate(client.ts:457)  */
    MTR_OP_SEQ = 3,             /* non-"op" message: updateSeqNumbers only */
    MTR_OP_LOCAL_INSERT = 8,    /* local insert (Client.insertSegmentLocal, client.ts:237): before collaboration
                                   seq = UniversalSequenceNumber, client = LocalClientId; while collaborating a
                                   pending op (seq = UnassignedSequenceNumber, the local client's short id, a new
                                   localSeq and SegmentGroup, mergeTree.ts:1397-1427, 1604-1637) until its ACK */
    MTR_OP_LOCAL_REMOVE = 9,    /* local remove (client.ts:227; pending: mergeTree.ts:1955-2047) */
    MTR_OP_LOCAL_ANNOTATE = 10, /* local annotate (pending keys: segmentPropertiesManager.ts:60-157); payload2 =
                                   MTR_COMB_NONE or MTR_COMB_REWRITE (a pending rewrite blocks remote changes to
                                   the segment, :72-80) */
    MTR_OP_START_COLLAB = 12,   /* Client.startOrUpdateCollaboration (client.ts:1133): seq/min_seq = currentSeq/minSeq,
                                   client = the observer's short id */
    MTR_OP_LOAD = 13,           /* a snapshot header segment (SnapshotLoader.loadHeader, snapshotLoader.ts:130-167):
                                   consecutive LOAD records are built into the tree bottom-up by
                                   MergeTree.reloadFromSegments (mergeTree.ts:678-728) before the next record */
    MTR_OP_SETCELL = 14,        /* SharedMatrix set-cell message (matrix.ts:636-693, remote branch): pos1 = row,
                                   pos2 = col at (ref_seq, client); resolves both positions
                                   (PermutationVector.adjustPosition, permutationvector.ts:232-247) and, when both
                                   are live, allocates row and col handles (getAllocatedHandle, :209-230).
                                   No updateSeqNumbers on either vector. */
    MTR_OP_HANDLES = 16,        /* PermutationVector.load's HandleTable.load (permutationvector.ts:327-345,
                                   handletable.ts:88), ahead of the vector's snapshot segments: pos1 = entry
                                   count, payload = offset of the entries in the document's text (two UTF-16
                                   units each, low half first).  Matrix documents only (MTR_F_COLS: cols). */
    MTR_OP_ACK = 17,            /* one member op of a sequenced message this client authored (Client.applyMsg,
                                   client.ts:866-869 -> ackPendingSegment, client.ts:641-663 and
                                   mergeTree.ts:1283-1322): acks the oldest pending SegmentGroup; payload2 =
                                   the member's MergeTreeDeltaType (segment.ack switches on it,
                                   mergeTreeNodes.ts:439-479), payload = its prop-op for an annotate, pos1 = its
                                   MTR_COMB_* (a local "rewrite" annotate: pendingRewriteCount) */
    MTR_OP_ROLLBACK = 18,       /* Client.rollback (client.ts:421 -> MergeTree.rollback, mergeTree.ts:2049-2159) of the
                                   newest pending local op: payload2 = its MergeTreeDeltaType, payload = its
                                   prop-op (annotate), pos1 = its MTR_COMB_* (PropertiesRollback.Rewrite) */
    MTR_OP_REGENERATE = 19,     /* Client.regeneratePendingOp (client.ts:917-960) of the oldest pending local op, for
                                   a resubmit after reconnect: normalizeSegmentsOnRebase first when currentSeq moved
                                   since the last one (mergeTree.ts:2352-2381, 2231-2331), then
                                   resetPendingDeltaToOps (client.ts:708-800): the group leaves the head of the
                                   pending queue and each member, in tree order, is re-expressed at its
                                   findReconnectionPosition (getPosition at (currentSeq, localSeq)); every member
                                   that still needs its op joins a new group of its own at the tail.  payload2 =
                                   the op's MergeTreeDeltaType.  Flag it MTR_F_DELTA: per regenerated member the
                                   engine records two mtr_delta entries, {op, position, cachedLength,
                                   MTR_DELTA_REGEN + type} then {op, offset of the member's text in the op's
                                   inserted text, properties reference, MTR_DELTA_REGEN_X} (see below). */
    MTR_OP_REF_CREATE = 20,     /* a local reference: Client.getContainingSegment(pos1, {ref_seq, client})
                                   (client.ts:1065-1078; payload2 & MTR_REF_LOCALVIEW: the local view, refSeq =
                                   currentSeq, the local client), then Client.getSlideToSegment when payload2 &
                                   MTR_REF_SLIDE (client.ts:1085-1099), then createLocalReferencePosition(segment,
                                   offset, payload = ReferenceType, client.ts:377-389 -> mergeTree.ts:2209-2226), as
                                   sequence/src/intervalCollection.ts:668-724 createPositionReference does; no
                                   segment = a detached reference (createDetachedLocalReferencePosition).  The
                                   document's references are numbered by creation, from 0; with payload2 &
                                   MTR_REF_SLOT the reference takes id pos2 instead -- a slot the host freed (one
                                   no segment's collection holds: removed, transient, or never created; else
                                   MTR_ERR_BAD_OP) or the next new id.  The host recycles ids that way: a removed
                                   reference, a transient query reference once its key was read, an interval
                                   endpoint a change superseded (nothing observable reads them again). */
    MTR_OP_REF_REMOVE = 21,     /* Client.removeLocalReferencePosition (client.ts:394-396 -> mergeTree.ts:2190-2207) of
                                   reference payload */
    MTR_OP_LOCAL_SETCELL = 22,  /* SharedMatrix.setCell of the local client (matrix.ts:202-310, setCellCore -> sendSetCellOp):
                                   pos1 = row, pos2 = col at the local view; PermutationVector.getAllocatedHandle on
                                   the rows vector, then the cols vector (permutationvector.ts:209-230: a split to the
                                   one position and a new handle when it has none); while collaborating nextLocalSeq
                                   advances both vectors' localSeq (matrix.ts:484-492).  With MTR_F_DELTA one
                                   MTR_DELTA_CELL record {op, row handle, col handle}.  A local row / col op (a local
                                   insert / remove record, MTR_F_COLS for cols) sets the other vector's localSeq to its
                                   own (submitVectorMessage, matrix.ts:321-345). */
    MTR_OP_TRACK = 23,          /* SharedMatrix undo (matrix/src/undoprovider.ts): TrackingGroup.unlink
                                   (mergeTreeTracking.ts:47-53) on a PermutationVector (MTR_F_COLS: cols) -- clear the
                                   tracking-group bits `payload` of tracked segment pos1 (-1: of every segment).
                                   See "Tracking groups" below. */
    /* An interval collection's own ops while collaborating (sequence/src/intervalCollection.ts): */
    MTR_OP_REF_ACK = 24,        /* IntervalCollection.ackInterval (:2054-2138) for endpoint reference `payload` (the
                                   host sends it only for an endpoint with no pending change): when the reference's
                                   segment holds it, getSlideToSegment (:2031-2045 -> client.ts:1085-1099) and, if that
                                   moves it, the reference is re-created there (createPositionReferenceFromSegoff with
                                   the op: no segment = a detached reference); either way its ReferenceType becomes
                                   SlideOnRemove (setSlideOnRemove, :2047-2052) */
    MTR_OP_REBASE_POS = 25,     /* IntervalCollection.rebasePositionWithSegmentSlide (:1472-1505) for a reconnect:
                                   getContainingSegment(pos1) at (ref_seq = the op's sequenceNumber, this client,
                                   localSeq = min_seq), getSlideToSegment, then findReconnectionPosition(segment,
                                   localSeq) + offset (client.ts:699-706), or DetachedReferencePosition; asserts 0x54e /
                                   0x54f.  Flag it MTR_F_DELTA: the result is one mtr_delta {op, position, 0,
                                   MTR_DELTA_REBASE} */
    /* MTR_OP_REBASE_POS with payload2 & MTR_REBASE_NOSLIDE (a SharedMatrix vector, flagged MTR_F_COLS for cols):
       SharedMatrix.rebasePosition (matrix.ts:534-551) -- no slide, no offset assert, and no segment gives
       MTR_DETACHED_POSITION (undefined: the resubmit skips the write).  MTR_OP_REGENERATE on a matrix vector
       (reSubmitCore, matrix.ts:553-570): its MTR_DELTA_REGEN_X record's second field is the segment's start
       handle (the regenerated PermutationSegment spec is [length, start]). */
    MTR_OP_LSEQ = 26,           /* IntervalCollection.getNextLocalSeq (:1584-1590): ++collabWindow.localSeq -- an
                                   interval op takes a localSeq the merge-tree's later local ops count past */
    MTR_OP_RELPOS = 15          /* a relative position of the NEXT record (getValidOpRange, client.ts:527-545 ->
                                   MergeTree.posFromRelativePos, mergeTree.ts:1371-1395), resolved at that op's
                                   (ref_seq, client) before the op runs: pos1 = marker ordinal (see below) or -1 for
                                   an id no marker was ever mapped to (position -1); pos2 = 1 or 2, the position of the
                                   next op (flagged MTR_F_REL) it replaces; payload = relativePos.offset (int32);
                                   payload2 = MTR_REL_*.
                                   Position = getPosition(marker) (+ 1 + offset unless `before`, else - offset);
                                   a marker zamboni unlinked has position 0 (its parent is gone). A resolved
                                   position < 0 makes the document MTR_ERR_UNSUPPORTED. */
};

/* MTR_OP_REBASE_POS payload2 */
enum { MTR_REBASE_NOSLIDE = 1 };

/* MTR_OP_RELPOS payload2 */
enum { MTR_REL_BEFORE = 1, MTR_REL_OFFSET = 2 };

/* MTR_OP_REF_CREATE payload2, and the ReferenceType bits (ops.ts:9-36) its payload carries.  MTR_REF_LSEQ: the
 * local client's view at (ref_seq, localSeq = min_seq) -- getContainingSegment(pos, undefined, localSeq), whose
 * lengths are localNetLength(segment, refSeq, localSeq), mergeTree.ts:636-662 (IntervalCollection.rebaseLocalInterval's
 * changeInterval, intervalCollection.ts:2019-2025 -> createPositionReference with a localSeq, :697-724) */
enum { MTR_REF_SLIDE = 1, MTR_REF_LOCALVIEW = 2, MTR_REF_LSEQ = 4, MTR_REF_SLOT = 8 };
enum {
    MTR_REFTYPE_SIMPLE = 0x0,
    MTR_REFTYPE_TILE = 0x1,
    MTR_REFTYPE_NEST_BEGIN = 0x2,
    MTR_REFTYPE_NEST_END = 0x4,
    MTR_REFTYPE_RANGE_BEGIN = 0x10,
    MTR_REFTYPE_RANGE_END = 0x20,
    MTR_REFTYPE_SLIDE_ON_REMOVE = 0x40,
    MTR_REFTYPE_STAY_ON_REMOVE = 0x80,
    MTR_REFTYPE_TRANSIENT = 0x100
};
/* localReferencePositionToPosition of a reference with no position (referencePositions.ts:103) */
#define MTR_DETACHED_POSITION (-1)
/* mtr_get_ref_states bits (include/mtr.h) */
#define MTR_REF_ST_SEGMENT 1
#define MTR_REF_ST_HELD 2
#define MTR_REF_ST_REMOVED 4

/*
 * Marker ordinals (MergeTree.idToSegment, mergeTree.ts:549,668): an insert / load record of a Marker whose
 * props carry a truthy "markerId" (Marker.getId, mergeTreeNodes.ts:612-617) has payload2 = ordinal + 1, the
 * host's per-document count of such markers; the engine maps ordinal -> segment.  The host resolves
 * relativePos.id to the latest ordinal mapped under that id.
 *
 * Remote annotate with a combiningOp (PropertiesManager.addProperties, segmentPropertiesManager.ts:60-157):
 * payload2 = MTR_COMB_* | (NaN value id << 3).  For "rewrite" the prop-op is the op's props; keys of the old
 * set whose new value is absent or falsy are deleted first (:109-123).  For the other names the op's props
 * values are ignored (combine(op, prev, undefined, seq), properties.ts:24-69): the prop-op holds, per key in
 * op order, the value the key takes when it is absent (combine of the default, computed by the host; the
 * null value = stays absent); a present value becomes NaN (incr) or stays (consensus / other names).
 */
enum { MTR_COMB_NONE = 0, MTR_COMB_REWRITE = 1, MTR_COMB_INCR = 2, MTR_COMB_CONSENSUS = 3, MTR_COMB_KEEP = 4 };

/* val_eq[v] high bits: value flags read by the combining rules and matchProperties; the low 28 bits
 * are the equivalence class */
#define MTR_VEQ_NEVER 0x80000000u   /* never equal, even to itself (NaN; {value: undefined, seq}) */
#define MTR_VEQ_FALSY 0x40000000u   /* !value (false, 0, -0, "") */
#define MTR_VEQ_INCR_STR 0x20000000u /* value + undefined is not NaN (string, object, array): unsupported */
#define MTR_VEQ_CONS_MUT 0x10000000u /* object whose "seq" is -1 (consensus mutates it in place): unsupported */
#define MTR_VEQ_CLASS 0x0fffffffu
/* engine-internal: a leaf's property-set index carries this bit when the set holds a MTR_VEQ_NEVER
 * value, so a set shared by two leaves (split halves, one annotate's memoized result) does not match
 * itself without reading it */
#define MTR_PROPS_NEVER 0x80000000u

/* op.flags */
enum {
    MTR_F_LAST = 1,    /* last member op of its message: run updateSeqNumbers(min_seq, seq) after it */
    MTR_F_MARKER = 2,  /* insert of a Marker segment (mergeTreeNodes.ts:557); payload = refType */
    MTR_F_PROPS = 4,   /* insert carries initial props: pos2 = prop-op index */
    MTR_F_NOREF = 8,   /* marker has no refType member ({"marker":{}}) */
    MTR_F_APPEND = 16, /* insert at the end of the local view with refSeq = UniversalSequenceNumber
                          (SnapshotLoader.loadBody append, snapshotLoader.ts:221-256) */
    MTR_F_COLS = 32,   /* matrix documents: the vector op targets the cols PermutationVector (contents.target
                          "cols", matrix.ts:645-651); without it, the rows vector */
    MTR_F_DELTA = 64,  /* report this op's delta ranges (mtr_get_deltas): the SequenceDeltaEvent ranges
                          SharedSegmentSequence.processMergeTreeMsg turns into catch-up ops for lagging
                          messages in the legacy format (sequence.ts:120-173, 697-736) */
    MTR_F_REL = 128    /* pos1 and/or pos2 come from the MTR_OP_RELPOS records right ahead of this op */
};

/* One delta range of an MTR_F_DELTA op (ISequenceDeltaRange, sequenceDeltaEvent.ts): the op's
 * index in its document's op list, the segment's position in the local view right after the op
 * (Client.getPosition) and its cachedLength; ranges come in tree order (SortedSegmentSet by ordinal).
 * kind: MTR_OP_INSERT (the inserted segment), MTR_OP_REMOVE (segments this op removed first),
 * MTR_OP_ANNOTATE (every annotated segment). */
/* mtr_delta.kind of a SharedMatrix document tracked for its cells (any op of the matrix flagged
 * MTR_F_DELTA): on the rows document, one MTR_DELTA_CELL record per flagged set-cell that wrote a cell
 * (pos = row handle, len = col handle; cells.setCell, matrix.ts:686-689); on each vector's document,
 * one MTR_DELTA_RECYCLE record per segment whose handles zamboni freed (pos = first handle,
 * len = count; onRowHandlesRecycled / onColHandlesRecycled, matrix.ts:722-734). */
#define MTR_DELTA_CELL MTR_OP_SETCELL
#define MTR_DELTA_RECYCLE 32
/* MTR_OP_REGENERATE results: kind MTR_DELTA_REGEN + MergeTreeDeltaType (pos = reconnection position, len =
 * cachedLength; the new op is insert(pos, segment), remove(pos, pos + len) or annotate(pos, pos + len, the op's
 * props)), followed by kind MTR_DELTA_REGEN_X: pos = the member's offset in the inserted text of the op being
 * regenerated (insert; the member's text is that text's [pos, pos + len)), len = a properties reference
 * (insert: the segment's current properties, which createInsertSegmentOp serializes when the op's own seg
 * has no props -- mtr_get_props; -1 = properties undefined). */
#define MTR_DELTA_REGEN 64
#define MTR_DELTA_REGEN_X 72
/* MTR_OP_REBASE_POS result: pos = the rebased position (MTR_DETACHED_POSITION when the segment slid off) */
#define MTR_DELTA_REBASE 80

/* Tracking groups (SharedMatrix undo: VectorUndoProvider, matrix/src/undoprovider.ts:17-127, on the merge-tree's
 * TrackingGroup, mergeTreeTracking.ts).  A PermutationVector segment a group tracks carries a tracking id (tid,
 * numbered per vector from 0 as segments become tracked, each split-off half of a tracked segment a new one; the id
 * of a segment zamboni unlinks or merges away is reused, the one freed last first, so a vector holds at most
 * prop_words / 2 ids at once) and the bit set of the groups that hold it (up to 32 groups live per vector; the host
 * maps groups to bits).  A
 * segment with a non-empty set is never unlinked by zamboni and merges only with a segment of the same set
 * (zamboni.ts:132, 156).  Records:
 *  - MTR_OP_LOCAL_INSERT / MTR_OP_LOCAL_REMOVE of a matrix vector with payload != 0: the op's delta segments (the
 *    inserted segment; the segments this remove removed first) join the groups of bits `payload`
 *    (VectorUndoProvider.record -> TrackingGroup.link, undoprovider.ts:30-85);
 *  - MTR_OP_LOCAL_INSERT of a matrix vector with pos2 >= 0: PermutationVector.insertRelative +
 *    PermutationSegment.transferToReplacement (permutationvector.ts:80-102, 184-194; matrix.ts:371-380): the new
 *    segment (at pos1, the host's getPosition of segment pos2 -- insertAtReferencePosition lands there,
 *    mergeTree.ts:1429-1530) takes segment pos2's handles and groups; payload must be != 0;
 *  - MTR_OP_TRACK: TrackingGroup.unlink, above.
 * With MTR_F_DELTA the vector's document reports, in op order: {op, tid, cachedLength, MTR_DELTA_TLINK} per
 * segment an op linked (link order), {op, tid, tid of the split-off half, MTR_DELTA_TSPLIT} when a tracked
 * segment splits (BaseSegment.splitAt -> TrackingGroupCollection.copyTo, mergeTreeNodes.ts:500), and {op, tid
 * of the appended segment, tid of the one it joined, MTR_DELTA_TMERGE} when zamboni appends one tracked segment
 * to another (zamboni.ts:158-172). */
#define MTR_DELTA_TLINK 96
#define MTR_DELTA_TSPLIT 97
#define MTR_DELTA_TMERGE 98
#define MTR_TRACK_GROUPS 32

typedef struct mtr_delta {
    uint32_t op;
    int32_t  pos;
    int32_t  len;
    uint32_t kind;
} mtr_delta;

/*
 * SharedMatrix documents: a matrix is a pair of engine documents, the rows
 * and the cols PermutationVector (permutationvector.ts:150), declared with mtr_set_matrix().  The rows
 * document's op list drives both (vector ops carry MTR_F_COLS for the cols vector; MTR_OP_SETCELL
 * touches both; MTR_OP_START_COLLAB starts both); the cols document has no ops of its own.
 * Permutation segments are [length, start] (PermutationSegment.toJSONObject, permutationvector.ts:118):
 * an insert carries its length in payload2; start is always reset to MTR_HANDLE_UNALLOCATED on
 * insert (onDelta INSERT, permutationvector.ts:354-361).
 */
#define MTR_HANDLE_UNALLOCATED ((int32_t)0x80000000) /* Handle.unallocated, handletable.ts:11 */
/* Loading a matrix from its summary (SharedMatrix.loadCore, matrix.ts:611-631): per vector (rows, then cols
 * with MTR_F_COLS) one MTR_OP_HANDLES record, its header segments as MTR_OP_LOAD records whose PermutationSegment
 * spec [length, start] keeps its start (payload = start, payload2 = length), an MTR_OP_START_COLLAB with
 * MTR_F_APPEND (that vector only, at its own header's minSeq / seq), then its body segments (MTR_F_APPEND
 * inserts). */

/*
 * Snapshot segments (MTR_OP_LOAD, and MTR_OP_INSERT with MTR_F_APPEND) carry their merge info
 * (specToSegment, snapshotLoader.ts:88-128): client = the segment's short id (0xFFFE =
 * NonCollabClient), seq = its seq (0 = UniversalSequenceNumber), ref_seq = removedSeq or -1,
 * min_seq = number of removedClientIds, pos1 = offset of those short ids (one UTF-16 unit each) in
 * the document's text, pos2 = prop-op index or -1, payload/payload2 = text (or marker refType).
 */
#define MTR_CLIENT_NONCOLLAB 0xFFFEu

/* Short client ids a document may register (the engine keeps a short id in 8 bits next to the
 * LocalClientId / NonCollabClient codes 0xff / 0xfe).  The reference's ids are unbounded
 * (client.ts:673-688); mtr_submit marks a document with more clients MTR_ERR_UNSUPPORTED (the shim
 * keeps it on the TypeScript Client) and the host packers refuse it up front. */
#define MTR_MAX_CLIENTS 253u

typedef struct mtr_op {
    uint8_t  type;     /* MTR_OP_* */
    uint8_t  flags;    /* MTR_F_* */
    uint16_t client;   /* short client id (client.ts:673-688); 0 = the observer itself */
    int32_t  seq;      /* sequenceNumber */
    int32_t  ref_seq;  /* referenceSequenceNumber */
    int32_t  min_seq;  /* minimumSequenceNumber */
    int32_t  pos1;     /* op.pos1 */
    int32_t  pos2;     /* remove/annotate: op.pos2; insert: prop-op index or -1 */
    uint32_t payload;  /* insert text: UTF-16 offset relative to doc text base; marker: refType;
                          annotate: prop-op index */
    uint32_t payload2; /* insert text: length in UTF-16 code units */
} mtr_op;

/* Per-document slice of a batch. */
typedef struct mtr_doc_desc {
    uint64_t op_begin;    /* index of the first op of this document in mtr_batch.ops */
    uint64_t text_base;   /* base index in mtr_batch.text for this document's op text */
    uint32_t op_count;
    uint32_t text_count;  /* UTF-16 units of op text in this batch for this document */
    uint32_t client_base; /* index into mtr_batch.client_off of short id 0 */
    uint32_t n_clients;   /* number of short ids registered so far (first-seen order) */
} mtr_doc_desc;

#define MTR_NULL_VALUE 0xFFFFFFFFu   /* prop-op value meaning JSON null (delete the key) */
#define MTR_NOT_INDEX  0xFFFFFFFFu   /* key_index for keys that are not JS array indices */

/*
 * A batch: flat arrays only.  Property keys and values are interned by the host:
 *   key k   : JSON-escaped key bytes key_bytes[key_off[k] .. key_off[k+1])
 *             key_index[k] = integer value if the key is a canonical JS array index
 *             (those sort first, ascending, in JS own-key order), else MTR_NOT_INDEX
 *   value v : JSON.stringify(value) bytes val_bytes[val_off[v] .. val_off[v+1]),
 *             val_eq[v] = equivalence class under matchProperties (properties.ts:71)
 *   prop-op p: ordered (key, value|MTR_NULL_VALUE) pairs
 *             propop_kv[2*propop_off[p] .. 2*propop_off[p+1]) in Object.keys order
 *   client c of doc d: JSON-escaped long id bytes
 *             client_bytes[client_off[docs[d].client_base + c] .. +1)
 */
typedef struct mtr_batch {
    uint32_t n_docs;
    uint32_t n_propops;
    uint32_t n_keys;
    uint32_t n_vals;
    uint64_t n_ops;
    uint64_t n_text;
    const mtr_doc_desc* docs;
    const mtr_op* ops;
    const uint16_t* text;
    const uint32_t* propop_off;   /* n_propops + 1 */
    const uint32_t* propop_kv;    /* 2 * propop_off[n_propops] */
    const uint32_t* key_off;      /* n_keys + 1 */
    const uint8_t*  key_bytes;
    const uint32_t* key_index;    /* n_keys */
    const uint32_t* val_off;      /* n_vals + 1 */
    const uint8_t*  val_bytes;
    const uint32_t* val_eq;       /* n_vals */
    const uint32_t* client_off;   /* total clients + 1 */
    const uint8_t*  client_bytes;
} mtr_batch;

/* Engine / oracle options: IMergeTreeOptions (mergeTree.ts:400-438) */
typedef struct mtr_options {
    int32_t new_length_calc;   /* mergeTreeUseNewLengthCalculations (default 0) */
    int32_t snapshot_v1;       /* newMergeTreeSnapshotFormat: 1 = SnapshotV1, 0 = SnapshotLegacy */
    int32_t chunk_size;        /* mergeTreeSnapshotChunkSize (default 10000) */
    int32_t reserved;
} mtr_options;

/* Status codes (a per-document status word; assert codes use the reference's hex ids) */
enum {
    MTR_OK = 0,
    MTR_ERR_INSERT_FAILED = 1,     /* UsageError("MergeTree insert failed") mergeTree.ts:1671 */
    MTR_ERR_BAD_OP = 2,            /* malformed record / unsupported op type */
    MTR_ERR_CAPACITY = 3,          /* engine-only: per-document arena exhausted */
    MTR_ERR_UNSUPPORTED = 4,       /* feature outside the observer path: caller falls back */
    MTR_ERR_ASSERT = 0x1000        /* 0x1000 | reference assert id, e.g. 0x104e for 0x04e */
};

#ifdef __cplusplus
}
#endif
#endif /* MTR_TYPES_H */
