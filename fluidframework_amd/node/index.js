'use strict';
/*
 * Node host side of the MI355X merge-tree replay engine: the observer subset of
 * @fluidframework/merge-tree's Client (packages/dds/merge-tree/src/client.ts:98) over the N-API
 * addon (mtr_napi.cc) and the C ABI (include/mtr.h).
 *
 *   reference                                          | here
 *   ---------------------------------------------------+--------------------------------------------
 *   new Client(specToSegment, logger, options)         | engine.createClient()   (one engine = many docs)
 *   client.startOrUpdateCollaboration(id, min, cur)    | same name              (client.ts:1133)
 *   client.applyMsg(msg)                               | same name              (client.ts:858)
 *   client.updateSeqNumbers(min, seq)                  | same name              (client.ts:877)
 *   client.insertTextLocal / removeRangeLocal /        | same names, before collaboration only
 *     annotateRangeLocal (non-collaborating edits)     |   (client.ts:237-285)
 *   client.summarize(runtime, handle, ser, catchUp)    | same name              (client.ts:966)
 *   client.getText() / getLength() / getCurrentSeq()   | same names
 *
 * Messages are packed on the JS thread exactly as the reference reads them (short client ids in
 * first-seen order, GROUP ops flattened, JSON.stringify / Object.keys for property values and key
 * order) and applied on the GPU in batches: applyMsg only queues, and the queue is flushed -- for
 * every document of the engine at once -- before anything is read back.  Results are identical to
 * applying each message synchronously because nothing observable happens in between.
 * Written for Node >= 12 (no optional chaining).
 */
const path = require('path');
const { IntervalCollections, IntervalUnsupported, refKey, cmpKey } = require('./intervals.js');

let addon = null;
function native() {
    if (addon === null) addon = require(path.join(__dirname, 'mtr_napi.node'));
    return addon;
}

// include/mtr_types.h
const OP = { INSERT: 0, REMOVE: 1, ANNOTATE: 2, SEQ: 3, LOCAL_INSERT: 8, LOCAL_REMOVE: 9, LOCAL_ANNOTATE: 10,
    START_COLLAB: 12, LOAD: 13, SETCELL: 14, RELPOS: 15, ACK: 17, ROLLBACK: 18, REGENERATE: 19, REF_CREATE: 20, REF_REMOVE: 21,
    REF_ACK: 24, REBASE_POS: 25, LSEQ: 26 };
const REF = { SLIDE: 1, LOCALVIEW: 2, LSEQ: 4, SLOT: 8 };  // MTR_OP_REF_CREATE payload2
const DELTA_REBASE = 80;
const DetachedReferencePosition = -1;   // referencePositions.ts:103
const DELTA_REGEN = 64, DELTA_REGEN_X = 72;
const REL = { BEFORE: 1, OFFSET: 2 };
const COMB = { NONE: 0, REWRITE: 1, INCR: 2, CONSENSUS: 3, KEEP: 4 };
const VEQ = { NEVER: 0x80000000, FALSY: 0x40000000, INCR_STR: 0x20000000, CONS_MUT: 0x10000000 };
const F = { LAST: 1, MARKER: 2, PROPS: 4, NOREF: 8, APPEND: 16, COLS: 32, DELTA: 64, REL: 128 };
const CLIENT_NONCOLLAB = 0xFFFE;  // include/mtr_types.h MTR_CLIENT_NONCOLLAB
const NULL_VALUE = 0xFFFFFFFF;
const MAX_CLIENTS = 253;  // include/mtr_types.h MTR_MAX_CLIENTS: short ids per engine document
const NOT_INDEX = 0xFFFFFFFF;
const STATUS = { OK: 0, INSERT_FAILED: 1, BAD_OP: 2, CAPACITY: 3, UNSUPPORTED: 4, ASSERT: 0x1000 };
// protocol-definitions SummaryType
const SummaryType = { Tree: 1, Blob: 2 };

class UnsupportedError extends Error {
    constructor(msg) {
        super(msg);
        this.name = 'UnsupportedError';
        this.fallback = true;  // the document must stay on the TypeScript Client
    }
}

function arrayIndex(key) {
    if (/^(0|[1-9][0-9]*)$/.test(key)) {
        const v = Number(key);
        if (v < 4294967295) return v;
    }
    return null;
}

/*
 * matchProperties (properties.ts:71-105) compares values by strict equality and recurses into any
 * `typeof === "object"` value through `for...in`, so arrays and index-keyed objects compare equal.
 * That is an equivalence -- and interning equivalence classes is exact -- for values without
 * nested nulls and empty containers; documents with such values stay on the TypeScript Client.
 */
let nanCounter = 0;
function eqKey(v) {
    if (typeof v === 'boolean') return v ? 'true' : 'false';
    if (typeof v === 'number') return Number.isNaN(v) ? 'NaN#' + (nanCounter++) : 'n' + String(v === 0 ? 0 : v);
    if (typeof v === 'string') return 's' + JSON.stringify(v);
    return '{' + Object.keys(v).sort().map((k) => JSON.stringify(k) + ':' + eqKey(v[k])).join(',') + '}';
}
function plainValue(v, nested) {
    if (v === null) return !nested;  // a top-level null deletes the key
    if (typeof v !== 'object') return true;
    const keys = Object.keys(v);
    if (keys.length === 0) return false;
    return keys.every((k) => plainValue(v[k], true));
}

const utf8 = (s) => Buffer.from(s, 'utf8');

// MTR_VEQ_* bits of a JSON value (include/mtr_types.h)
function valueFlags(v) {
    let f = 0;
    if (!v) f |= VEQ.FALSY;
    if (typeof v === 'string' || (v !== null && typeof v === 'object')) f |= VEQ.INCR_STR;  // v + undefined concatenates
    if (v !== null && typeof v === 'object' && !Array.isArray(v) && v.seq === -1) f |= VEQ.CONS_MUT;
    return f >>> 0;
}

const NAN = { nan: true };  // combine results that are not JSON values
class Never { constructor(json) { this.json = json; } }

// combine(co, undefined, undefined, seq) (properties.ts:24-69) for a key the segment lacks
function combineAbsent(co, seq) {
    const cur = co.defaultValue;
    if (co.name === 'incr') {
        if (cur === undefined || cur === null || typeof cur === 'number' || typeof cur === 'boolean') return NAN;
        if (typeof cur !== 'string') throw new UnsupportedError('incr of a non-primitive default value');
        let r = cur + 'undefined';
        const mv = co.minValue;
        if (mv) {
            if (typeof mv === 'string') { if (r < mv) r = mv; } else if (typeof mv !== 'number') {
                throw new UnsupportedError('incr minValue comparison');
            }
        }
        return r;
    }
    if (co.name === 'consensus') {
        if (cur === undefined) return new Never('{"seq":' + seq + '}');  // {value: undefined, seq}
        if (cur === null) throw new UnsupportedError('consensus on a null default (TypeError in the reference)');
        if (typeof cur === 'object' && !Array.isArray(cur) && cur.seq === -1) return Object.assign({}, cur, { seq });
        return cur;
    }
    if (cur === undefined) throw new UnsupportedError('combiningOp without a default leaves an explicit undefined property');
    return cur;
}

/** Global key / value / prop-op tables (ids stable across batches). */
class Interner {
    constructor() {
        this.keys = new Map(); this.keyBytes = []; this.keyIndex = [];
        this.vals = new Map(); this.valBytes = []; this.valEq = []; this.eqIds = new Map();
        this.propops = []; this.never = new Map();
    }
    _addValue(s, eq) {
        const i = this.valBytes.length;
        this.valBytes.push(utf8(s));
        this.valEq.push(eq >>> 0);
        return i;
    }
    neverValue(s) {  // matchProperties never matches it, not even with itself
        let i = this.never.get(s);
        if (i === undefined) {
            const e = this.eqIds.size;
            this.eqIds.set('never#' + e, e);
            i = this._addValue(s, (e | VEQ.NEVER) >>> 0);
            this.never.set(s, i);
        }
        return i;
    }
    nan() { return this.neverValue('null'); }
    _valueOrNull(r) {
        if (r === NAN) return this.nan();
        if (r instanceof Never) return this.neverValue(r.json);
        if (r === null) return NULL_VALUE;
        return this.value(r);
    }
    // a remote annotate with combiningOp co -> [propop, payload2] (include/mtr_types.h MTR_COMB_*)
    combining(props, co, seq) {
        if (props === null || typeof props !== 'object' || Array.isArray(props)) throw new UnsupportedError('annotate props');
        if (!co) return [this.propop(props), COMB.NONE];
        if (typeof co !== 'object' || Array.isArray(co)) throw new UnsupportedError('combiningOp');
        if (co.name === 'rewrite') return [this.propop(props), COMB.REWRITE];
        const mode = co.name === 'incr' ? COMB.INCR : (co.name === 'consensus' ? COMB.CONSENSUS : COMB.KEEP);
        const absent = this._valueOrNull(combineAbsent(co, seq));
        this.propops.push(Object.keys(props).map((k) => [this.key(k), absent]));
        return [this.propops.length - 1, mode === COMB.INCR ? (mode | (this.nan() << 3)) >>> 0 : mode];
    }
    key(k) {
        let i = this.keys.get(k);
        if (i === undefined) {
            i = this.keyBytes.length;
            this.keys.set(k, i);
            this.keyBytes.push(utf8(JSON.stringify(k).slice(1, -1)));
            const ix = arrayIndex(k);
            this.keyIndex.push(ix === null ? NOT_INDEX : ix);
        }
        return i;
    }
    value(v) {
        if (v === null) return NULL_VALUE;
        if (!plainValue(v, false)) throw new UnsupportedError('property value with nested null or empty container');
        const s = JSON.stringify(v);
        let i = this.vals.get(s);
        if (i === undefined) {
            const ek = eqKey(v);
            let e = this.eqIds.get(ek);
            if (e === undefined) { e = this.eqIds.size; this.eqIds.set(ek, e); }
            i = this._addValue(s, (e | valueFlags(v)) >>> 0);
            this.vals.set(s, i);
        }
        return i;
    }
    propop(props) {  // Object.keys order = JS own-key order
        this.propops.push(Object.keys(props).map((k) => [this.key(k), this.value(props[k])]));
        return this.propops.length - 1;
    }
}

/** Per-document host state: client registry plus the queued ops/text of the next batch. */
class DocLog {
    constructor() {
        this.observerId = undefined; this.clients = []; this.clientIx = new Map();
        this.ops = []; this.text = []; this.collaborating = false;
        // MergeTree.idToSegment (mergeTree.ts:549,668) as the host sees it: id key -> marker ordinal
        this.nMarkers = 0; this.markerIds = new Map(); this.markerDup = new Set(); this.markerIdAnnotated = false;
        this.nRefs = 0;  // reference ids handed out (MTR_OP_REF_CREATE ids; high-water mark)
        this.freeRefs = [];  // ids released for reuse (MTR_REF_SLOT), a stack
        this.currentSeq = 0;  // collabWindow.currentSeq as the host sees it (interval ops do not move it)
        this.intervals = undefined;  // ./intervals.js IntervalCollections, when used
    }
    _intervals(fn) {  // an interval path this host does not restate is an UnsupportedError (the document falls back)
        try {
            return fn();
        } catch (e) {
            if (e instanceof IntervalUnsupported) throw new UnsupportedError(e.message);
            throw e;
        }
    }
    static _idKey(v) {  // SameValueZero keys; objects only match themselves (never from JSON)
        if (typeof v === 'boolean') return 'b' + v;
        if (typeof v === 'number') return 'n' + String(v === 0 ? 0 : v);
        if (typeof v === 'string') return 's' + v;
        return null;
    }
    _mapMarker(props) {  // Marker.getId truthy -> mapIdToSegment: ordinal + 1 (0 = no id)
        if (!props || typeof props !== 'object' || !props.markerId) return 0;
        const k = DocLog._idKey(props.markerId);
        const o = this.nMarkers++;
        if (k !== null) {
            if (this.markerIds.has(k)) this.markerDup.add(k);
            this.markerIds.set(k, o);
        }
        return o + 1;
    }
    _relpos(rp, which, short, seq, ref, msn) {  // posFromRelativePos, mergeTree.ts:1371-1395
        if (!rp || typeof rp !== 'object') throw new UnsupportedError('relative position');
        const k = rp.id ? DocLog._idKey(rp.id) : null;
        if (k === null || !this.markerIds.has(k)) throw new UnsupportedError('relative position without a mapped marker (position -1)');
        if (this.markerDup.has(k) || this.markerIdAnnotated) {
            throw new UnsupportedError('relative position on a marker id remapped by block updates');
        }
        let off = rp.offset, flags = rp.before ? REL.BEFORE : 0;
        if (off !== undefined) {
            if (off === null) off = 0;  // pos += null adds 0
            if (typeof off !== 'number' || !Number.isInteger(off)) throw new UnsupportedError('relative position offset');
            flags |= REL.OFFSET;
        } else {
            off = 0;
        }
        this.push(OP.RELPOS, 0, short, seq, ref, msn, this.markerIds.get(k), which, off >>> 0, flags);
    }
    _position(op, key, which, short, seq, ref, msn) {  // op.pos1 / op.pos2, or its relativePos (client.ts:527-545)
        const v = op[key], rk = 'relative' + key[0].toUpperCase() + key.slice(1);
        if (v === undefined && op[rk]) {
            this._relpos(op[rk], which, short, seq, ref, msn);
            return 0;
        }
        if (typeof v !== 'number') throw new UnsupportedError('op without a usable ' + key);
        return Math.trunc(v);
    }
    shortId(longId) {  // Client.getOrAddShortClientId, client.ts:673-677
        const i = this.clientIx.get(longId);
        return i === undefined ? this.addLongId(longId) : i;
    }
    addLongId(longId) {  // Client.addLongClientId, client.ts:685-688: always a new short id
        if (this.clients.length >= MAX_CLIENTS) throw new UnsupportedError('more than ' + MAX_CLIENTS + ' client ids');
        const i = this.clients.length;
        this.clientIx.set(longId, i);
        this.clients.push(longId);
        return i;
    }
    _text(s) {
        const off = this.text.length;
        for (let i = 0; i < s.length; i++) this.text.push(s.charCodeAt(i));
        return [off, s.length];
    }
    _seg(spec, it, mapMarker = true) {  // specToSegment, sequence/src/sequenceFactory.ts:26-38 -> [flags, payload, payload2, propop]
        if (typeof spec === 'string') { const t = this._text(spec); return [0, t[0], t[1], -1]; }
        if (spec && typeof spec === 'object' && 'text' in spec) {
            const t = this._text(spec.text);
            if (spec.props !== undefined && spec.props !== null) return [F.PROPS, t[0], t[1], it.propop(spec.props)];
            return [0, t[0], t[1], -1];
        }
        if (spec && typeof spec === 'object' && 'marker' in spec) {
            const m = spec.marker || {};
            let flags = F.MARKER, ref = m.refType;
            if (ref === undefined || ref === null) { flags |= F.NOREF; ref = 0; }
            let pp = -1;
            if (spec.props !== undefined && spec.props !== null) { flags |= F.PROPS; pp = it.propop(spec.props); }
            return [flags, ref >>> 0, mapMarker ? this._mapMarker(spec.props) : 0, pp];
        }
        throw new UnsupportedError('unrecognized segment spec');
    }
    push(type, flags, client, seq, ref, msn, pos1, pos2, payload, payload2) {
        this.ops.push([type, flags, client, seq, ref, msn, pos1, pos2, payload, payload2]);
        this.nPushed = (this.nPushed || 0) + 1;  // (a stamp: getContainingSegment -> createLocalReferencePosition)
    }
    // local edits (client.ts:225-260): final before collaboration; while collaborating a pending op
    // (record seq = UnassignedSequenceNumber) until this client's sequenced message acks it
    localSeq() { return this.collaborating ? -1 : 0; }
    localInsert(pos, spec, it) {
        const s = this._seg(spec, it);
        this.push(OP.LOCAL_INSERT, s[0], 0, this.localSeq(), 0, 0, pos, s[3], s[1], s[2]);
    }
    localRemove(start, end) { this.push(OP.LOCAL_REMOVE, 0, 0, this.localSeq(), 0, 0, start, end, 0, 0); }
    // a local reference (localReference.ts): getContainingSegment(pos, view) [+ getSlideToSegment], then
    // createLocalReferencePosition -- view = {referenceSequenceNumber, clientId} or undefined (the local view)
    createRef(pos, refType, view, slide) {
        let short = 0, ref = 0, flags = REF.LOCALVIEW;
        if (view !== undefined) {
            const cid = view.clientId === null || view.clientId === undefined ? 'null' : String(view.clientId);
            short = this.shortId(cid);
            ref = view.referenceSequenceNumber;
            flags = 0;
        }
        if (slide) flags |= REF.SLIDE;
        const id = this._newRefId();
        this.push(OP.REF_CREATE, 0, short, 0, ref, 0, pos, id, refType, flags | REF.SLOT);
        return id;
    }
    _newRefId() { return this.freeRefs.length ? this.freeRefs.pop() : this.nRefs++; }
    removeRef(id) { this.push(OP.REF_REMOVE, 0, 0, 0, 0, 0, 0, 0, id, 0); }
    // the host is done with reference `id`: its id is reused by the next create (MTR_REF_SLOT); remove: a reference a
    // segment's collection may hold (a superseded or deleted interval endpoint) is removed first, a Transient query
    // reference needs no record (fluidframework_amd/batch.py DocLog.release_ref)
    releaseRef(id, remove = true) {
        if (!(id >= 0 && id < this.nRefs) || this.freeRefs.includes(id)) throw new Error('no local reference ' + id);
        if (remove) this.removeRef(id);
        this.freeRefs.push(id);
    }
    // createPositionReference with a localSeq (a rebase's changeInterval): getContainingSegment(pos, undefined,
    // localSeq) -- this client's view at (refSeq, localSeq) -- then createLocalReferencePosition
    createRefAt(pos, refType, refSeq, localSeq) {
        const id = this._newRefId();
        this.push(OP.REF_CREATE, 0, 0, 0, refSeq, localSeq, pos, id, refType, REF.LSEQ | REF.SLOT);
        return id;
    }
    ackRef(id) { this.push(OP.REF_ACK, 0, 0, 0, 0, 0, 0, 0, id, 0); }  // IntervalCollection.ackInterval, one endpoint
    // rebasePositionWithSegmentSlide(pos, seqNumberFrom, localSeq): returns the record index its result names
    rebasePosition(pos, seqFrom, localSeq) {
        this.push(OP.REBASE_POS, F.DELTA, 0, 0, seqFrom, localSeq, pos, 0, 0, 0);
        return this.ops.length - 1;
    }
    bumpLocalSeq() { this.push(OP.LSEQ, 0, 0, 0, 0, 0, 0, 0, 0, 0); }  // IntervalCollection.getNextLocalSeq
    localAnnotate(start, end, props, it, combiningOp) {
        if (props && typeof props === 'object' && 'markerId' in props) this.markerIdAnnotated = true;
        let comb = localComb(combiningOp), pp;
        if (comb === COMB.NONE || comb === COMB.REWRITE) {
            pp = it.propop(props);
        } else {  // combine(op, previousValue, undefined, seq): each key's absent-key result, as for a remote one
            const c = it.combining(props, combiningOp, this.collaborating ? -1 : 0);
            pp = c[0];
            comb = c[1];
        }
        this.push(OP.LOCAL_ANNOTATE, 0, 0, this.localSeq(), 0, 0, start, end, pp, comb);
    }
    rollback(op, it) {  // Client.rollback (client.ts:421-423 -> MergeTree.rollback, mergeTree.ts:2049-2159)
        let pp = 0, comb = 0;
        if (op.type === 2) {
            comb = localComb(op.combiningOp);
            pp = it.propop(op.props || {});
        } else if (op.type !== 0 && op.type !== 1) {
            throw new UnsupportedError('rollback of op type ' + op.type);
        }
        this.push(OP.ROLLBACK, 0, 0, -1, 0, 0, comb, 0, pp, op.type);
    }
    // Client.regeneratePendingOp (client.ts:917-960): one record per member op; returns the first record's
    // index in this batch (the op field of its MTR_DELTA_REGEN records)
    regenerate(op) {
        const members = op.type === 3 ? op.ops : [op];
        const first = this.ops.length;
        for (const m of members) {
            if (m.type !== 0 && m.type !== 1 && m.type !== 2) throw new UnsupportedError('regenerate of op type ' + m.type);
            this.push(OP.REGENERATE, F.DELTA, 0, -1, 0, 0, 0, 0, 0, m.type);
        }
        return first;
    }
    localOp(op, it) {  // Client.localTransaction member (client.ts:1029-1048)
        if (op.type === 0) this.localInsert(op.pos1, op.seg, it);
        else if (op.type === 1) this.localRemove(op.pos1, op.pos2);
        else if (op.type === 2) this.localAnnotate(op.pos1, op.pos2, op.props || {}, it, op.combiningOp);
        else throw new UnsupportedError('local op type ' + op.type);
    }
    startCollab(longId, minSeq, currentSeq) {  // client.ts:1133-1155
        if (longId === undefined) return;  // detached: stay local until attached
        if (this.observerId === undefined) {
            this.observerId = longId;
            const me = this.addLongId(longId);
            this.collaborating = true;
            this.currentSeq = currentSeq;
            this.push(OP.START_COLLAB, 0, me, currentSeq, 0, minSeq, 0, 0, 0, 0);
        } else {  // reconnect under a new id: the observer's short id is renamed
            const me = this.clientIx.get(this.observerId);
            this.observerId = longId;
            this.clientIx.set(longId, me);
            this.clients[me] = longId;
        }
    }
    seqUpdate(min, seq) { this.currentSeq = seq; this.push(OP.SEQ, F.LAST, 0, seq, seq, min, 0, 0, 0, 0); }
    // SnapshotLoader.specToSegment (snapshotLoader.ts:88-128): one LOAD (header) / APPEND (body) record whose
    // removedClientIds (short ids) ride in the text arena
    _snapshotSeg(spec, it, opType, flags) {
        // a loaded live marker is mapped by reloadFromSegments' blockUpdate (addNodeReferences, mergeTree.ts:297-306,
        // localNetLength > 0 only); a body segment by blockInsert (:1655-1662)
        const withInfo = spec !== null && typeof spec === 'object' && 'json' in spec;  // hasMergeInfo, snapshotChunks.ts:80-84
        const removed = withInfo && spec.removedSeq !== undefined && spec.removedSeq !== null;
        const live = opType !== OP.LOAD || !removed;
        let s, client = CLIENT_NONCOLLAB, seq = 0, removers = [], rseq = -1;
        if (withInfo) {
            s = this._seg(spec.json, it, live);
            if (spec.client !== undefined && spec.client !== null) client = this.shortId(spec.client);
            if (spec.seq !== undefined && spec.seq !== null) seq = spec.seq;
            if (spec.removedClient !== undefined && spec.removedClient !== null) removers = [this.shortId(spec.removedClient)];
            if (spec.removedClientIds !== undefined && spec.removedClientIds !== null) {
                removers = spec.removedClientIds.map((x) => this.shortId(x));
            }
            if (removed) rseq = spec.removedSeq;
        } else {
            s = this._seg(spec, it, live);
        }
        const roff = this.text.length;
        for (const r of removers) this.text.push(r);
        this.push(opType, s[0] | flags, client, seq, rseq, removers.length, roff, s[3], s[1], s[2]);
    }
    // Client.load -> SnapshotLoader.initialize (snapshotLoader.ts:41-257) from a summary's blobs {name: JSON text}:
    // header segments as reloadFromSegments records, startOrUpdateCollaboration(longId, minSeq, seq) (longId
    // undefined: a detached load stays local), body segments appended.  Returns the catch-up messages of a legacy
    // summary (the caller applies them as ordinary messages), [] otherwise.  Mirrors batch.py DocLog.load_summary.
    loadSummary(blobs, longId, it) {
        const chunk = JSON.parse(blobs.header);
        let segs, meta;
        if (chunk.version === '1') {
            segs = chunk.segments;
            meta = chunk.headerMetadata;
        } else {  // toLatestVersion of a legacy chunk, snapshotChunks.ts:151-200
            segs = chunk.segmentTexts;
            meta = chunk.headerMetadata || {
                orderedChunkMetadata: [{ id: 'header' }].concat(chunk.chunkLengthChars < chunk.totalLengthChars ? [{ id: 'body' }] : []),
                minSequenceNumber: chunk.chunkMinSequenceNumber,
                sequenceNumber: chunk.chunkSequenceNumber,
            };
        }
        if (meta === undefined) throw new Error('header metadata not available');
        for (const spec of segs) this._snapshotSeg(spec, it, OP.LOAD, 0);
        const minSeq = meta.minSequenceNumber;
        const seq = meta.sequenceNumber;
        this.startCollab(longId, minSeq !== undefined && minSeq !== null ? minSeq : seq, seq);
        for (const md of meta.orderedChunkMetadata.slice(1)) {
            if (blobs[md.id] === undefined) throw new Error('missing summary blob ' + md.id);
            const body = JSON.parse(blobs[md.id]);
            for (const spec of (body.segments !== undefined ? body.segments : (body.segmentTexts || []))) {
                this._snapshotSeg(spec, it, OP.INSERT, F.APPEND);
            }
        }
        const names = new Set(['header'].concat(meta.orderedChunkMetadata.map((md) => md.id)));
        const extra = Object.keys(blobs).filter((k) => !names.has(k));
        if (extra.length > 1) throw new Error('0x060');  // "There should be only one blob with catch up ops"
        return extra.length ? JSON.parse(blobs[extra[0]]) : [];
    }
    message(msg, it, local) {  // Client.applyMsg, client.ts:858-887
        const cid = msg.clientId === null || msg.clientId === undefined ? 'null' : String(msg.clientId);
        const short = this.shortId(cid);
        const seq = msg.sequenceNumber, ref = msg.referenceSequenceNumber, msn = msg.minimumSequenceNumber;
        if (msg.type !== 'op') { this.currentSeq = seq; this.push(OP.SEQ, F.LAST, short, seq, ref, msn, 0, 0, 0, 0); return; }
        let contents = msg.contents;
        if (typeof contents === 'string') contents = JSON.parse(contents);
        if (contents && contents.type === 'act') {  // an interval collection's op (sequence.ts:620-646): not a merge-tree op
            if (this.intervals === undefined) this.intervals = new IntervalCollections();
            this._intervals(() => this.intervals.process(this, contents, msg));
            return;
        }
        this.currentSeq = seq;
        const members = contents.type === 3 ? contents.ops : [contents];  // MergeTreeDeltaType.GROUP
        if (members.length === 0) { this.push(OP.SEQ, F.LAST, short, seq, ref, msn, 0, 0, 0, 0); return; }
        if (cid === this.observerId || local) {  // ackPendingSegment per member (client.ts:641-663, 866-869)
            members.forEach((op, i) => {
                const last = i === members.length - 1 ? F.LAST : 0;
                let pp = 0, comb = 0;
                if (op.type === 2) {
                    comb = localComb(op.combiningOp);
                    pp = it.propop(op.props || {});
                } else if (op.type !== 0 && op.type !== 1) {
                    throw new UnsupportedError('ack of op type ' + op.type);
                }
                this.push(OP.ACK, last, short, seq, ref, msn, comb, 0, pp, op.type);
            });
            return;
        }
        members.forEach((op, i) => {
            const last = i === members.length - 1 ? F.LAST : 0;
            if (op.type === 0) {
                if (op.seg === undefined || op.seg === null) {  // applyInsertOp returns early
                    this.push(OP.SEQ, last, short, seq, ref, msn, 0, 0, 0, 0);
                    return;
                }
                const n0 = this.ops.length;
                const pos1 = this._position(op, 'pos1', 1, short, seq, ref, msn);
                const rel = this.ops.length > n0 ? F.REL : 0;
                const s = this._seg(op.seg, it);
                this.push(OP.INSERT, s[0] | last | rel, short, seq, ref, msn, pos1, s[3], s[1], s[2]);
            } else if (op.type === 1) {
                const n0 = this.ops.length;
                const pos1 = this._position(op, 'pos1', 1, short, seq, ref, msn);
                const pos2 = this._position(op, 'pos2', 2, short, seq, ref, msn);
                const rel = this.ops.length > n0 ? F.REL : 0;
                this.push(OP.REMOVE, last | rel, short, seq, ref, msn, pos1, pos2, 0, 0);
            } else if (op.type === 2) {
                if (op.props && typeof op.props === 'object' && 'markerId' in op.props) this.markerIdAnnotated = true;
                const n0 = this.ops.length;
                const pos1 = this._position(op, 'pos1', 1, short, seq, ref, msn);
                const pos2 = this._position(op, 'pos2', 2, short, seq, ref, msn);
                const rel = this.ops.length > n0 ? F.REL : 0;
                const c = it.combining(op.props, op.combiningOp, seq);
                this.push(OP.ANNOTATE, last | rel, short, seq, ref, msn, pos1, pos2, c[0], c[1]);
            } else {
                throw new UnsupportedError('op type ' + op.type);
            }
        });
    }
}

/*
 * SharedMatrix (SharedMatrix.processCore, matrix/src/matrix.ts:636-693, remote branch): vector ops
 * (contents.target "rows" / "cols") are merge-tree ops on that PermutationVector, whose segment specs
 * are [length, start] (permutationvector.ts:45-48; the remote start is discarded on INSERT); a set-cell
 * message is one SETCELL record.  Both vectors share the rows log's client table.  Mirrors
 * fluidframework_amd/batch.py MatrixLog record for record.
 */
class MatrixDocLog extends DocLog {
    message(msg, it) {
        const cid = msg.clientId === null || msg.clientId === undefined ? 'null' : String(msg.clientId);
        if (msg.type !== 'op') return;  // SharedMatrix has no MSN handler of its own
        if (cid === this.observerId) throw new UnsupportedError('message authored by the observer (local ack path)');
        const short = this.shortId(cid);
        const seq = msg.sequenceNumber, ref = msg.referenceSequenceNumber, msn = msg.minimumSequenceNumber;
        let contents = msg.contents;
        if (typeof contents === 'string') contents = JSON.parse(contents);
        const target = contents.target;
        if (target === undefined || target === null) {  // MatrixOp.set (matrix/src/ops.ts:8-12)
            if (contents.type !== 2) throw new UnsupportedError('matrix message without a target');
            this.push(OP.SETCELL, 0, short, seq, ref, msn, contents.row, contents.col, 0, 0);
            return;
        }
        if (target !== 'rows' && target !== 'cols') throw new UnsupportedError('matrix target ' + target);
        const tf = target === 'cols' ? F.COLS : 0;
        const members = contents.type === 3 ? contents.ops : [contents];
        if (members.length === 0) { this.push(OP.SEQ, F.LAST | tf, short, seq, ref, msn, 0, 0, 0, 0); return; }
        members.forEach((op, i) => {
            const last = (i === members.length - 1 ? F.LAST : 0) | tf;
            if ('relativePos1' in op || 'relativePos2' in op) throw new UnsupportedError('relative positions');
            if (op.type === 0) {
                const seg = op.seg;
                if (seg === undefined || seg === null) { this.push(OP.SEQ, last, short, seq, ref, msn, 0, 0, 0, 0); return; }
                if (!Array.isArray(seg) || seg.length !== 2) throw new UnsupportedError('PermutationSegment spec');
                this.push(OP.INSERT, last, short, seq, ref, msn, op.pos1, -1, 0, seg[0]);
            } else if (op.type === 1) {
                this.push(OP.REMOVE, last, short, seq, ref, msn, op.pos1, op.pos2, 0, 0);
            } else {
                throw new UnsupportedError('vector op type ' + op.type);
            }
        });
    }
    colsLog() {  // the cols vector's engine document: no ops of its own, the same client table
        const c = new DocLog();
        c.observerId = this.observerId;
        c.clients = this.clients.slice();
        c.clientIx = new Map(this.clientIx);
        return c;
    }
}
/** Engine document order for matrices: [rows 0, cols 0, rows 1, cols 1, ...] (pair 2m / 2m+1). */
function matrixLogs(logs) {
    const out = [];
    for (const m of logs) { out.push(m); out.push(m.colsLog()); }
    return out;
}

function offsets(chunks) {
    const off = new Uint32Array(chunks.length + 1);
    for (let i = 0; i < chunks.length; i++) off[i + 1] = off[i] + chunks[i].length;
    return [off, Buffer.concat(chunks.concat([Buffer.alloc(1)]))];
}

/** Pack the queued ops of every DocLog (in order) into the arrays of include/mtr_types.h and clear them. */
function buildBatch(logs, it) {
    const nOps = logs.reduce((a, l) => a + l.ops.length, 0);
    const nText = logs.reduce((a, l) => a + l.text.length, 0);
    const docs = Buffer.alloc(32 * logs.length);
    const ops = Buffer.alloc(32 * nOps);
    const text = new Uint16Array(Math.max(1, nText));
    const clientChunks = [];
    let o = 0, t = 0;
    logs.forEach((log, d) => {
        const b = 32 * d;
        docs.writeUInt32LE(o >>> 0, b); docs.writeUInt32LE(Math.floor(o / 4294967296), b + 4);
        docs.writeUInt32LE(t >>> 0, b + 8); docs.writeUInt32LE(Math.floor(t / 4294967296), b + 12);
        docs.writeUInt32LE(log.ops.length, b + 16);
        docs.writeUInt32LE(log.text.length, b + 20);
        docs.writeUInt32LE(clientChunks.length, b + 24);
        docs.writeUInt32LE(log.clients.length, b + 28);
        log.clients.forEach((c) => clientChunks.push(utf8(JSON.stringify(c).slice(1, -1))));
        for (const r of log.ops) {
            const q = 32 * o;
            ops.writeUInt8(r[0], q); ops.writeUInt8(r[1], q + 1); ops.writeUInt16LE(r[2], q + 2);
            ops.writeInt32LE(r[3], q + 4); ops.writeInt32LE(r[4], q + 8); ops.writeInt32LE(r[5], q + 12);
            ops.writeInt32LE(r[6], q + 16); ops.writeInt32LE(r[7], q + 20);
            ops.writeUInt32LE(r[8] >>> 0, q + 24); ops.writeUInt32LE(r[9] >>> 0, q + 28);
            o++;
        }
        text.set(log.text, t);
        t += log.text.length;
        log.ops = []; log.text = [];
    });
    const po = new Uint32Array(it.propops.length + 1);
    const kv = [];
    it.propops.forEach((pairs, i) => { po[i + 1] = po[i] + pairs.length; pairs.forEach((p) => kv.push(p[0], p[1])); });
    const k = offsets(it.keyBytes), v = offsets(it.valBytes), c = offsets(clientChunks);
    return {
        docs, ops, text, propopOff: po, propopKv: Uint32Array.from(kv.length ? kv : [0]),
        keyOff: k[0], keyBytes: k[1], keyIndex: Uint32Array.from(it.keyIndex.length ? it.keyIndex : [0]),
        valOff: v[0], valBytes: v[1], valEq: Uint32Array.from(it.valEq.length ? it.valEq : [0]),
        clientOff: c[0], clientBytes: c[1],
    };
}

/*
 * Legacy-format catch-up messages (SURVEY.md §8 row f2).  SharedSegmentSequence keeps the messages
 * since the MSN and rewrites each lagging one (refSeq != seq - 1) from the sequenceDelta events its
 * application raised (createOpsFromDelta / processMergeTreeMsg, sequence.ts:120-173, 697-736).  The
 * engine applies messages in batches and raises no events, so the shim keeps that list itself: the
 * lagging message's ops are flagged F.DELTA, the engine reports each delta range (op, position in the
 * local view, cachedLength, kind; mtr_get_deltas) and the ops are rebuilt here after the batch.
 */
function sameProps(a, b) {  // matchProperties, properties.ts:71-105 (JS semantics, written out)
    if (!a) return !b;
    if (!b) return false;
    for (const k in a) {
        const y = b[k];
        if (y === undefined) return false;
        if (typeof y === 'object' ? !sameProps(a[k], y) : y !== a[k]) return false;
    }
    for (const k in b) if (a[k] === undefined) return false;
    return true;
}
function insertedSegmentJson(spec) {  // segment.clone().toJSONObject() of the segment an insert creates
    const kept = (p) => { const o = {}; Object.keys(p).forEach((k) => { if (p[k] !== null) o[k] = p[k]; }); return o; };
    if (typeof spec === 'string') return spec;
    const hasProps = spec.props !== undefined && spec.props !== null;
    if ('text' in spec) return hasProps ? { text: spec.text, props: kept(spec.props) } : spec.text;
    const m = spec.marker || {};
    const out = { marker: m.refType === undefined || m.refType === null ? {} : { refType: m.refType } };
    if (hasProps) out.props = kept(spec.props);
    return out;
}
function opsFromDeltas(members, opIndex, byOp) {
    const ops = [];
    members.forEach((member, i) => {
        for (const r of byOp.get(opIndex[i]) || []) {
            const pos = r[1], len = r[2], last = ops.length ? ops[ops.length - 1] : undefined;
            if (r[3] === OP.ANNOTATE) {  // an observer's propertyDeltas hold every key of the op
                const props = {};
                Object.keys(member.props).forEach((k) => { props[k] = member.props[k]; });
                if (last && last.pos2 === pos && sameProps(last.props, props)) last.pos2 += len;
                else ops.push({ pos1: pos, pos2: pos + len, props, type: 2 });
            } else if (r[3] === OP.INSERT) {
                ops.push({ pos1: pos, seg: insertedSegmentJson(member.seg), type: 0 });
            } else if (r[3] === OP.REMOVE) {
                if (last && last.pos1 === pos) {
                    if (last.pos2 === undefined) throw new Error('0x3ff');  // sequence.ts:155-158
                    last.pos2 += len;
                } else {
                    ops.push({ pos1: pos, pos2: pos + len, type: 1 });
                }
            }
        }
    });
    return ops;
}
class CatchUpLog {
    constructor() { this.stash = []; this.pending = []; }
    /** After log.message(msg) queued the message's records from op index `lo` on. */
    add(msg, log, lo, own) {
        const copy = JSON.parse(JSON.stringify(msg));  // parseHandles (sequence.ts:698)
        if (typeof copy.contents === 'string') copy.contents = JSON.parse(copy.contents);
        if (own && copy.referenceSequenceNumber !== copy.sequenceNumber - 1) {
            // an ack raises no "delta" event (ackPendingSegment, mergeTree.ts:1283-1323): transformOps collects
            // nothing and the stashed copy is createGroupOp() of no ops (sequence.ts:697-725, opBuilder.ts:102-107)
            copy.referenceSequenceNumber = copy.sequenceNumber - 1;
            copy.contents = { ops: [], type: 3 };
        } else if (copy.referenceSequenceNumber !== copy.sequenceNumber - 1) {
            const members = copy.contents.type === 3 ? copy.contents.ops : [copy.contents];
            const opIndex = members.map((_, i) => {
                const r = log.ops[lo + i];
                if (r[0] !== OP.INSERT && r[0] !== OP.REMOVE && r[0] !== OP.ANNOTATE) return -1;
                r[1] |= F.DELTA;
                return lo + i;
            });
            copy.referenceSequenceNumber = copy.sequenceNumber - 1;
            this.pending.push({ msg: copy, members, opIndex });
        }
        this.stash.push(copy);
        if (this.stash.length > 20 && this.stash[20].sequenceNumber < msg.minimumSequenceNumber) {
            this.trim(msg.minimumSequenceNumber);  // sequence.ts:728-734
        }
    }
    resolve(deltas) {  // Int32Array of [op, pos, len, kind] records of the batch just applied
        const byOp = new Map();
        for (let i = 0; i < deltas.length; i += 4) {
            const r = [deltas[i], deltas[i + 1], deltas[i + 2], deltas[i + 3]];
            if (!byOp.has(r[0])) byOp.set(r[0], []);
            byOp.get(r[0]).push(r);
        }
        for (const p of this.pending) {
            const ops = opsFromDeltas(p.members, p.opIndex, byOp);
            p.msg.contents = ops.length === 1 ? ops[0] : { ops, type: 3 };  // createGroupOp
        }
        this.pending = [];
    }
    trim(minSeq) {  // processMinSequenceNumberChanged, sequence.ts:738-748
        let i = 0;
        while (i < this.stash.length && this.stash[i].sequenceNumber <= minSeq) i++;
        if (i) this.stash = this.stash.slice(i);
    }
    forSummary(minSeq) {  // summarizeMergeTree, sequence.ts:675-695
        this.trim(minSeq);
        this.stash.forEach((m) => { m.minimumSequenceNumber = minSeq; });
        return this.stash;
    }
}

/** The observer Clients of many documents on one GPU. */
/*
 * resetPendingDeltaToOps (client.ts:708-800) from the engine's MTR_DELTA_REGEN / _X record pairs
 * (include/mtr_types.h): per member of the pending group, in tree order, the op to resubmit --
 * createInsertSegmentOp (the member's piece of the text, the op's own seg.props or else the segment's
 * current properties), createRemoveRangeOp, createAnnotateRangeOp -- and a GROUP unless exactly one.
 * The Python mirror is fluidframework_amd/regen.py.
 */
function regenRecords(d) {  // Int32Array of [op, pos, len, kind] -> Map(record index -> [[type, pos, len, off, ref]])
    const out = new Map();
    for (let i = 0; i < d.length; i += 4) {
        const kind = d[i + 3] >>> 0;
        if (kind < DELTA_REGEN || kind >= DELTA_REGEN + 3) continue;
        if (i + 4 >= d.length || (d[i + 7] >>> 0) !== DELTA_REGEN_X) throw new Error('MTR_DELTA_REGEN without its _X record');
        const op = d[i] >>> 0;
        if (!out.has(op)) out.set(op, []);
        out.get(op).push([kind - DELTA_REGEN, d[i + 1], d[i + 2], d[i + 5], d[i + 6]]);
        i += 4;
    }
    return out;
}
function regenMember(op, r, propsOf) {
    const [t, pos, n, off, ref] = r;
    if (t !== op.type) throw new Error('regenerate record does not match the op');
    if (t === 1) return { pos1: pos, pos2: pos + n, type: 1 };
    if (t === 2) {
        const o = { pos1: pos, pos2: pos + n, props: op.props, type: 2 };
        if (op.combiningOp !== undefined) o.combiningOp = op.combiningOp;
        return o;
    }
    const seg = op.seg;
    const own = seg !== null && typeof seg === 'object' && seg.props !== undefined;  // client.ts:763-767
    const props = own ? seg.props : (ref >= 0 ? propsOf(ref) : undefined);
    let spec;
    if (seg !== null && typeof seg === 'object' && 'marker' in seg) {
        spec = { marker: seg.marker };
        if (props !== undefined && props !== null) spec.props = props;
    } else {
        const text = (typeof seg === 'string' ? seg : seg.text).substring(off, off + n);  // UTF-16 units
        spec = props !== undefined && props !== null ? { text, props } : text;
    }
    return { pos1: pos, seg: spec, type: 0 };
}
function regeneratedOp(resetOp, recs, first, propsOf) {
    const members = resetOp.type === 3 ? resetOp.ops : [resetOp];
    const ops = [];
    members.forEach((m, k) => { for (const r of recs.get(first + k) || []) ops.push(regenMember(m, r, propsOf)); });
    return ops.length === 1 ? ops[0] : { ops, type: 3 };
}

// a local annotate's combiningOp: none or "rewrite" (pendingRewriteCount, segmentPropertiesManager.ts:72-80); its
// ack and rollback records carry the same code (pos1)
function localComb(co) {  // a local annotate's combiningOp as its ack / rollback records carry it (batch.py _local_comb)
    if (!co) return COMB.NONE;
    if (typeof co !== 'object') throw new UnsupportedError('combiningOp');
    if (co.name === 'rewrite') return COMB.REWRITE;
    return co.name === 'incr' ? COMB.INCR : co.name === 'consensus' ? COMB.CONSENSUS : COMB.KEEP;
}

class BatchReplayEngine {
    constructor(maxDocs, options) {
        this.options = Object.assign({ newLengthCalc: 0, snapshotV1: 1, chunkSize: 10000, device: 0 }, options || {});
        this.maxDocs = maxDocs;
        this.h = native().createEngine(maxDocs, this.options);
        this.interner = new Interner();
        this.logs = [];
        this.catchUps = [];
        this.dirty = false;
        this.summarized = false;
        this.inFlight = false;  // an async run / summarize holds the engine (its batch was taken from the logs)
    }
    _assertIdle() {
        if (this.inFlight) throw new Error('engine busy: await the pending flushAsync / summarizeAllAsync first');
    }
    createClient() {
        if (this.logs.length >= this.maxDocs) throw new Error('engine is full');
        this.logs.push(new DocLog());
        this.catchUps.push(new CatchUpLog());
        return new BatchReplayClient(this, this.logs.length - 1);
    }
    createMatrix() {  // a SharedMatrix: its rows and cols PermutationVectors as engine documents 2k, 2k+1
        if (this.logs.length + 2 > this.maxDocs) throw new Error('engine is full');
        const rows = this.logs.length;
        const log = new MatrixDocLog();
        this.logs.push(log, log.colsLog());
        this.catchUps.push(new CatchUpLog(), new CatchUpLog());
        native().setMatrix(this.h, rows, rows + 1);
        return new BatchMatrixClient(this, rows);
    }
    _batch() {
        this.logs.forEach((l, d) => {  // cols vectors share their rows log's client table
            if (l instanceof MatrixDocLog) this.logs[d + 1] = l.colsLog();
        });
        return buildBatch(this.logs, this.interner);
    }
    _afterRun() {
        this.catchUps.forEach((c, d) => { if (c.pending.length) c.resolve(native().getDeltas(this.h, d)); });
        this.dirty = false;
        this.summarized = false;
    }
    flush() {  // apply every queued message of every document
        this._assertIdle();
        if (!this.dirty) return;
        native().submitRun(this.h, this._batch());
        this._afterRun();
    }
    /**
     * The asynchronous flush: the batch is applied on a worker thread (N-API async work) and the
     * returned promise settles when the GPU is done, so the event loop keeps serving meanwhile.  Every
     * other call on this engine or its clients throws until it settles (await it): the batch has already
     * been taken from the logs, so nothing may be queued behind it.
     */
    async flushAsync() {
        this._assertIdle();
        if (!this.dirty) return;
        const batch = this._batch();
        this.inFlight = true;
        try {
            await native().submitRunAsync(this.h, batch);
        } finally {
            this.inFlight = false;
        }
        this._afterRun();
    }
    /**
     * The summarizer's hand-over in one call (mtr_replay_pipelined through the addon's replaySummaries): every
     * queued message applied, every document summarized and its records in host memory -- document d's record is
     * bytes[docOff[d], docOff[d + 1]) = u32 blob count, u32 blob lengths, the blobs.  A batch of remote messages
     * goes through the pipelined path (ranges applied as they land, summarized and downloaded as they finish;
     * `pipelined` true), any other the serial calls.
     */
    replaySummaries(parts = 16) {
        this._assertIdle();
        const r = native().replaySummaries(this.h, this._batch(), parts);
        this._afterRun();
        this.summarized = true;
        return r;
    }
    async summarizeAllAsync() {  // every document's blobs, built on a worker thread
        await this.flushAsync();
        if (!this.summarized) {
            this._assertIdle();
            this.inFlight = true;
            try {
                await native().summarizeAsync(this.h);
            } finally {
                this.inFlight = false;
            }
            this.summarized = true;
        }
    }
}

/** Client (client.ts:98) restricted to the observer path, backed by one engine document. */
class BatchReplayClient {
    constructor(engine, doc) {
        this.engine = engine; this.doc = doc; this.log = engine.logs[doc];
        this.currentSeq = 0;
        this.localSeq = 0;          // collabWindow.localSeq as this host counts it (interval ops too)
        this.lastNormalization = 0; // Client.lastNormalizationRefSeq (client.ts:910)
        this.emitters = new Map();  // label -> the collection's op emitter (IValueOpEmitter)
    }
    _queue(fn) { this.engine._assertIdle(); fn(); this.engine.dirty = true; }
    _check() {
        const st = native().docStatus(this.engine.h, this.doc);
        if (st[0] === STATUS.OK) return;
        if (st[0] >= STATUS.ASSERT) {  // assert(cond, 0xNNN) throws Error("0xNNN"), common-utils assert.ts:15-21
            throw new Error('0x' + (st[0] - STATUS.ASSERT).toString(16).padStart(3, '0'));
        }
        if (st[0] === STATUS.INSERT_FAILED) throw new Error('MergeTree insert failed');  // mergeTree.ts:1671
        if (st[0] === STATUS.UNSUPPORTED) throw new UnsupportedError('unsupported op at ' + st[1]);
        throw new Error('engine status ' + st[0] + ' at op ' + st[1]);
    }
    startOrUpdateCollaboration(longClientId, minSeq, currentSeq) {
        this._queue(() => this.log.startCollab(longClientId, minSeq || 0, currentSeq || 0));
        this.currentSeq = currentSeq || 0;
    }
    /**
     * Client.load (client.ts:1007-1019 -> SnapshotLoader.initialize, snapshotLoader.ts:41-257): the document
     * resumes from a merge-tree summary read through `storage` (IChannelStorageService: readBlob(path) ->
     * Buffer / Uint8Array, list(path) -> blob names).  A runtime that is not Detached starts collaboration as
     * runtime.clientId ?? "snapshot".  Resolves to {catchupOpsP}: the legacy format's catch-up messages, which
     * the caller applies with applyMsg (SharedSegmentSequence.loadCore does), [] for V1.
     */
    async load(runtime, storage, serializer) {
        const names = await storage.list('');
        const blobs = {};
        for (const n of names) {
            const b = await storage.readBlob(n);
            blobs[n] = typeof b === 'string' ? b : Buffer.from(b.buffer, b.byteOffset, b.byteLength).toString('utf8');
        }
        if (blobs.header === undefined) throw new Error('0x05f');  // "Missing blob header on legacy snapshot!"
        const detached = runtime && runtime.attachState === 'Detached';
        const longId = detached ? undefined : ((runtime && runtime.clientId) || 'snapshot');
        let catchup = [];
        this._queue(() => { catchup = this.log.loadSummary(blobs, longId, this.engine.interner); });
        const meta = JSON.parse(blobs.header);
        this.currentSeq = meta.version === '1' ? meta.headerMetadata.sequenceNumber
            : (meta.headerMetadata ? meta.headerMetadata.sequenceNumber : meta.chunkSequenceNumber);
        if (serializer && typeof serializer.parse === 'function' && catchup.length) {
            catchup = serializer.parse(JSON.stringify(catchup));
        }
        return { catchupOpsP: Promise.resolve(catchup) };
    }
    /** load from an ISummaryTree this shim (or the reference) produced: {type: Tree, tree: {name: {content}}}. */
    loadSummaryTree(summary, longClientId) {
        const blobs = {};
        for (const k of Object.keys(summary.tree)) {
            const c = summary.tree[k].content;
            blobs[k] = typeof c === 'string' ? c : Buffer.from(c).toString('utf8');
        }
        let catchup = [];
        this._queue(() => { catchup = this.log.loadSummary(blobs, longClientId, this.engine.interner); });
        return catchup;
    }
    applyMsg(msg, local, localOpMetadata) {
        const own = local || (msg.type === 'op' && String(msg.clientId) === this.log.observerId);
        if (msg.type === 'op' && this.log.collaborating && this.log.intervals !== undefined) {
            const c = typeof msg.contents === 'string' ? JSON.parse(msg.contents) : msg.contents;
            if (c && c.type === 'act' && (own || this.log.intervals.live)) {  // a live client's interval op
                this.processIntervalOp(msg, !!own, localOpMetadata);
                this.currentSeq = this.log.currentSeq;
                return;
            }
        }
        this._queue(() => {
            if (!this.engine.options.snapshotV1 && msg.type === 'op' && !own &&
                msg.referenceSequenceNumber !== msg.sequenceNumber - 1) {
                let c = msg.contents;
                if (typeof c === 'string') c = JSON.parse(c);
                for (const m of c.type === 3 ? (c.ops || []) : [c]) {
                    // the catch-up transform needs each member's post-op values / one record per member
                    if (m.combiningOp || m.relativePos1 || m.relativePos2) {
                        throw new UnsupportedError('a lagging message with a combining annotate or a relative position ' +
                            'in the legacy format');
                    }
                }
            }
            const lo = this.log.ops.length;
            this.log.message(msg, this.engine.interner, local);
            // (an interval op is handled by the collections and kept by no catch-up list, sequence.ts:636-645)
            if (!this.engine.options.snapshotV1 && msg.type === 'op' && this.log.currentSeq === msg.sequenceNumber) {
                this.engine.catchUps[this.doc].add(msg, this.log, lo, !!own);
            }
        });
        this.currentSeq = this.log.currentSeq;
    }
    updateSeqNumbers(min, seq) {
        this._queue(() => this.log.seqUpdate(min, seq));
        this.currentSeq = seq;
    }
    insertTextLocal(pos, text, props) {
        this._queue(() => { this.log.localInsert(pos, props ? { text, props } : text, this.engine.interner); this._countLocal(); });
    }
    insertMarkerLocal(pos, refType, props) {
        this._queue(() => {
            this.log.localInsert(pos, props ? { marker: { refType }, props } : { marker: { refType } }, this.engine.interner);
            this._countLocal();
        });
    }
    removeRangeLocal(start, end) { this._queue(() => { this.log.localRemove(start, end); this._countLocal(); }); }
    _countLocal() { if (this.log.collaborating) this.localSeq++; }  // a pending local op takes a localSeq
    /** Client.localTransaction (client.ts:1029-1048): every member op as a local (pending) op. */
    /**
     * Client.applyStashedOp(op) (client.ts:830-856): a stashed op of this client applied as a local op (GROUP: each
     * member); returns the local op metadata (one token per member: its pending SegmentGroup, which
     * regeneratePendingOp takes from the head of the pending queue).
     */
    applyStashedOp(op) {
        if (op.type === 3) return op.ops.map((o) => this.applyStashedOp(o));
        if (!this.log.collaborating) throw new Error('0x2db');  // "Applying op must generate a pending segment"
        this._queue(() => { this.log.localOp(op, this.engine.interner); this._countLocal(); });
        this.nStashed = (this.nStashed || 0) + 1;
        return { stashed: this.nStashed, type: op.type };
    }
    localTransaction(groupOp) {
        this._queue(() => { for (const op of groupOp.ops) { this.log.localOp(op, this.engine.interner); this._countLocal(); } });
    }
    annotateRangeLocal(start, end, props, combiningOp) {  // client.ts:245-260
        this._queue(() => { this.log.localAnnotate(start, end, props, this.engine.interner, combiningOp); this._countLocal(); });
    }
    /** Client.rollback(op, localOpMetadata) (client.ts:421-423) of the newest pending local op `op`. */
    rollback(op) { this._queue(() => this.log.rollback(op, this.engine.interner)); }
    /**
     * Client.regeneratePendingOp(resetOp, segmentGroup) (client.ts:917-960) for the oldest pending op
     * (`resetOp`, the op that was submitted): flushes the engine and returns the op to resubmit.
     */
    regeneratePendingOp(resetOp) {
        if (this.log.intervals !== undefined && this.log.currentSeq !== this.lastNormalization) {
            // client.ts:921-926: the "normalize" event (the interval collections rebase their pending ops) comes first
            for (const c of this.log.intervals.data.values()) this.log._intervals(() => c.onNormalize(this));
        }
        this.lastNormalization = this.log.currentSeq;
        let first = 0;
        this._queue(() => { first = this.log.regenerate(resetOp); });
        this.engine.flush();
        this._check();
        const recs = regenRecords(native().getDeltas(this.engine.h, this.doc));
        return regeneratedOp(resetOp, recs, first, (ref) => this._props(ref));
    }
    _props(ref) {  // a property set of this document's arena -> the properties object
        const w = native().getProps(this.engine.h, this.doc, ref);
        const it = this.engine.interner;
        const names = Array.from(it.keys.keys());  // ids are insertion order
        const out = {};
        for (let k = 0; k < w[0]; k++) out[names[w[1 + 2 * k]]] = JSON.parse(it.valBytes[w[2 + 2 * k]].toString('utf8'));
        return out;
    }
    /**
     * createPositionReference (sequence/src/intervalCollection.ts:697-724): a local reference at pos of the view
     * sequenceArgs = {referenceSequenceNumber, clientId} (default: this client's local view), slid off a
     * removed-and-acked segment when `slide` (Client.getSlideToSegment, client.ts:1085-1099), then
     * createLocalReferencePosition (client.ts:377-389).  -> a reference handle for the calls below.
     */
    createPositionReference(pos, refType, sequenceArgs, slide) {
        let id = 0;
        this._queue(() => { id = this.log.createRef(pos, refType, sequenceArgs, !!slide); });
        return { id, refType, client: this };
    }
    /**
     * Client.createLocalReferencePosition(segment, offset, refType) (client.ts:377-389) for a segment this
     * client's getContainingSegment returned, before any later edit: the same view and position.
     */
    createLocalReferencePosition(segment, offset, refType) {
        if (!segment || segment._at === undefined || segment._at.stamp !== this.log.nPushed) {
            throw new UnsupportedError('createLocalReferencePosition on a segment from before the last edit');
        }
        return this.createPositionReference(segment._at.start + (offset || 0), refType, segment._at.view, false);
    }
    /** Client.removeLocalReferencePosition (client.ts:394-396). */
    removeLocalReferencePosition(lref) { this._queue(() => this.log.removeRef(lref.id)); return lref; }
    /** Client.localReferencePositionToPosition (client.ts:398-403), on the device. */
    localReferencePositionToPosition(lref) {
        this.engine.flush();
        this._check();
        const p = native().getRefPositions(this.engine.h, this.doc);
        return lref.id < p.length ? p[lref.id] : DetachedReferencePosition;
    }
    /** LocalReference.getOffset (localReference.ts:110) and its segment's leaf index (-1: none / gone). */
    localReferenceSegment(lref) {
        this.engine.flush();
        this._check();
        const r = native().getRefInfo(this.engine.h, this.doc, lref.id);
        return { leafIndex: r[0], offset: r[1], held: r[3] === 1 };
    }
    getCurrentSeq() { return this.currentSeq; }
    // ---- interval collections (sequence/src/intervalCollection.ts; SharedSegmentSequence, sequence.ts:445-801)
    /** DefaultMap.populate of the SharedString summary's `header` blob, before load(). */
    loadIntervals(header) {
        this._queue(() => {
            this.log.intervals = new IntervalCollections();
            this.log._intervals(() => this.log.intervals.populate(header));
        });
    }
    /** loadFinished (sequence.ts:750-801): after load() and its catch-up messages, the collections attach. */
    loadFinished() {
        if (this.log.intervals !== undefined) this._queue(() => this.log._intervals(() => this.log.intervals.attach(this.log)));
    }
    /** getIntervalCollection(label) (sequence.ts:445-447): add(start, end, intervalType, props) on a string
     * that is not collaborating yet (a detached SharedString); remote ops arrive through applyMsg. */
    getIntervalCollection(label, emitter) {
        if (this.log.intervals === undefined) this.log.intervals = new IntervalCollections();
        const c = this.log.intervals.get(label);
        if (!this.log.collaborating) {
            return { add: (start, end, intervalType, props) => {
                this._queue(() => this.log._intervals(() => c.add(this.log, start, end, intervalType, props)));
            } };
        }
        // a collaborating client: IntervalCollection's API (intervalCollection.ts:1620-2338); emitter(opName, value,
        // localOpMetadata) receives each op to submit
        if (emitter) this.emitters.set(label, emitter);
        this.log.intervals.live = true;
        const run = (fn) => { const r = this.log._intervals(fn); this.engine.dirty = true; return r; };
        const self = this;
        // helpers.create("transient", ...): two Transient references at the local view; their compare keys are read
        // with the document's (one sync), then the ids go back to the free list -- a Transient reference is held by no
        // segment's collection (localReference.ts:260-298), so queries take no reference slot
        const transientKeys = (ranges) => {
            const ids = ranges.map(([a, b]) => [self.log.createRef(a, 0x100, undefined, false),
                self.log.createRef(b, 0x100, undefined, false)]);
            self.engine.dirty = true;
            const keys = self.refKeys();
            const out = self.log._intervals(() => ids.map(([ts, te]) => [refKey(keys, ts), refKey(keys, te)]));
            for (let k = ids.length - 1; k >= 0; k--) {
                self.log.releaseRef(ids[k][1], false);
                self.log.releaseRef(ids[k][0], false);
            }
            return [keys, out];
        };
        // the end tree (compareSequenceIntervalEnds, :1168-1169): one node per end; two intervals with equal ends
        // share a node that holds the later-put one -- a history this host does not keep, so it refuses
        const byEnd = (keys) => {
            const ivs = [...c.byId.values()].map((iv) => [refKey(keys, iv.end), iv]).sort((x, y) => cmpKey(x[0], y[0]));
            for (let k = 1; k < ivs.length; k++) {
                if (cmpKey(ivs[k - 1][0], ivs[k][0]) === 0) throw new IntervalUnsupported('two intervals with one end: the end tree keeps one node for them');
            }
            return ivs;
        };
        return {
            add: (start, end, intervalType, props) => run(() => c.liveAdd(self, start, end, intervalType, props)),
            change: (id, start, end) => run(() => c.liveChange(self, id, start, end)),
            changeProperties: (id, props) => run(() => c.liveChangeProperties(self, id, props)),
            removeIntervalById: (id) => run(() => c.liveRemove(self, id)),
            getIntervalById: (id) => c.byId.get(id),
            /** [start, end] positions (localReferencePositionToPosition of the endpoints) */
            positions(iv, keys) { const k = keys || self.refKeys(); return [k[4 * iv.start], k[4 * iv.end]]; },
            [Symbol.iterator]() { return self.log._intervals(() => c.ordered(self.refKeys()))[Symbol.iterator](); },
            findOverlappingIntervals(start, end) {  // :950-964 (SequenceInterval.overlaps in tree order)
                return this.findOverlappingIntervalsMany([[start, end]])[0];
            },
            /** findOverlappingIntervals for each [start, end] of `ranges`, from one engine sync */
            findOverlappingIntervalsMany(ranges) {
                const live = ranges.map((r, k) => k).filter((k) => ranges[k][1] >= ranges[k][0] && c.byId.size > 0);
                const out = ranges.map(() => []);
                if (live.length === 0) return out;
                const [keys, tk] = transientKeys(live.map((k) => ranges[k]));
                return self.log._intervals(() => {
                    const ordered = c.ordered(keys);
                    live.forEach((k, q) => {
                        const [ks, ke] = tk[q];
                        out[k] = ordered.filter((iv) => cmpKey(refKey(keys, iv.start), ke) <= 0 && cmpKey(refKey(keys, iv.end), ks) >= 0);
                    });
                    return out;
                });
            },
            previousInterval(pos) {  // :966-978: endIntervalTree.floor of a transient (pos, pos)
                const [keys, tk] = transientKeys([[pos, pos]]);
                return self.log._intervals(() => {
                    const k = tk[0][1];
                    let best;
                    for (const [e, iv] of byEnd(keys)) if (cmpKey(e, k) <= 0) best = iv;
                    return best;
                });
            },
            nextInterval(pos) {  // :980-992: endIntervalTree.ceil of a transient (pos, pos)
                const [keys, tk] = transientKeys([[pos, pos]]);
                return self.log._intervals(() => {
                    const k = tk[0][1];
                    for (const [e, iv] of byEnd(keys)) if (cmpKey(e, k) >= 0) return iv;
                    return undefined;
                });
            },
            // the positional iterators (:2232-2331, gatherIterationResults :864-944): the intervals whose start (and
            // end) compare equal to a transient interval's, forward or backward in the tree's order
            gather(forward = true, start, end) {
                if (start === undefined && end === undefined) {
                    const out = self.log._intervals(() => c.ordered(self.refKeys()));
                    return forward ? out : out.reverse();
                }
                const [keys, tk] = transientKeys([[start !== undefined ? start : 0, end !== undefined ? end : 0]]);
                const [ks, ke] = tk[0];
                let out = self.log._intervals(() => c.ordered(keys));
                if (start === undefined) out = out.filter((iv) => cmpKey(refKey(keys, iv.end), ke) === 0);
                else if (end === undefined) out = out.filter((iv) => cmpKey(refKey(keys, iv.start), ks) === 0);
                else out = out.filter((iv) => cmpKey(refKey(keys, iv.start), ks) === 0 && cmpKey(refKey(keys, iv.end), ke) === 0);
                return forward ? out : out.reverse();
            },
            CreateForwardIteratorWithStartPosition(pos) { return this.gather(true, pos, undefined)[Symbol.iterator](); },
            CreateBackwardIteratorWithStartPosition(pos) { return this.gather(false, pos, undefined)[Symbol.iterator](); },
            CreateForwardIteratorWithEndPosition(pos) { return this.gather(true, undefined, pos)[Symbol.iterator](); },
            CreateBackwardIteratorWithEndPosition(pos) { return this.gather(false, undefined, pos)[Symbol.iterator](); },
        };
    }
    /** The summary's `header` blob (summarizeCore, sequence.ts:467-480), undefined when there are no collections. */
    summarizeIntervals() {
        if (this.log.intervals === undefined) return undefined;
        this.engine.flush();
        this._check();
        const st = native().getRefStates(this.engine.h, this.doc);
        return this.log._intervals(() => this.log.intervals.serialize(st, this.log.currentSeq));
    }
    getText() {
        this.engine.flush();
        this._check();
        return native().getText(this.engine.h, this.doc);
    }
    /** getLength: the local view's length (root.cachedLength; a marker counts 1). */
    getLength() {
        this.engine.flush();
        this._check();
        const me = this.log.collaborating ? this.log.clientIx.get(this.log.observerId) : -1;
        return native().getViewLength(this.engine.h, this.doc, this.log.currentSeq, me);
    }
    // ---- a live client's interval collections (what IntervalCollection needs from its Client and emitter)
    refKeys() { this.engine.flush(); this._check(); return native().getRefKeys(this.engine.h, this.doc); }
    rebaseResults() {  // {record index -> position} of the MTR_OP_REBASE_POS records just queued
        this.engine.flush();
        this._check();
        const d = native().getDeltas(this.engine.h, this.doc);
        const out = new Map();
        for (let i = 0; i < d.length; i += 4) if (d[i + 3] === DELTA_REBASE) out.set(d[i], d[i + 1]);
        return out;
    }
    nextLocalSeq() {  // IntervalCollection.getNextLocalSeq (intervalCollection.ts:1584-1590)
        this._queue(() => this.log.bumpLocalSeq());
        return ++this.localSeq;
    }
    emit(label, opName, value, localOpMetadata) {  // the collection's IValueOpEmitter: an "act" op to submit
        const em = this.emitters.get(label);
        if (em) em(opName, value, localOpMetadata);
    }
    /**
     * SharedSegmentSequence.processCore's interval branch (sequence.ts:636-645) for a live client: `local` with the
     * op's localOpMetadata for this client's own ops (their acks).
     */
    processIntervalOp(msg, local, localOpMetadata) {
        let contents = msg.contents;
        if (typeof contents === 'string') contents = JSON.parse(contents);
        if (this.log.intervals === undefined) this.log.intervals = new IntervalCollections();
        this.engine._assertIdle();
        this.log._intervals(() => this.log.intervals.liveProcess(this, contents, msg, local, localOpMetadata));
        this.engine.dirty = true;
    }
    /** DefaultMap's resubmit of an interval op (rebaseLocalInterval, intervalCollection.ts:1270-1279) -> the op to send. */
    rebaseIntervalOp(contents, localOpMetadata) {
        const c = this.log.intervals.get(contents.key);
        const v = contents.value;
        const rebased = this.log._intervals(() => c.rebaseLocal(this, v.opName, v.value, localOpMetadata.localSeq));
        this.engine.dirty = true;
        return Object.assign({}, contents, { value: { opName: v.opName, value: rebased } });
    }
    /**
     * Client.getContainingSegment(pos, sequenceArgs) (client.ts:1065-1078): the segment holding pos in
     * the view of sequenceArgs = {referenceSequenceNumber, clientId} (default: this client's current
     * view), found on the device.  -> {segment: {text | marker, cachedLength, seq, clientId, removedSeq,
     * properties index}, offset} with both undefined when no segment covers pos.
     */
    getContainingSegment(pos, sequenceArgs) {
        this.engine.flush();
        this._check();
        let ref, client;
        if (sequenceArgs === undefined) {  // getClientSequenceArgsForMessage, client.ts:598-630
            ref = this.currentSeq;
            client = this.log.collaborating ? this.log.clientIx.get(this.log.observerId) : -1;
        } else {
            ref = sequenceArgs.referenceSequenceNumber;
            const cid = sequenceArgs.clientId === null || sequenceArgs.clientId === undefined ? 'null'
                : String(sequenceArgs.clientId);
            client = this.log.shortId(cid);  // getOrAddShortClientId
        }
        const r = native().getContainingSegment(this.engine.h, this.doc, pos, ref, client);
        if (r === null) return { segment: undefined, offset: undefined };
        const longId = (c) => (c >= 0 ? this.log.clients[c] : 'original');
        // (a pending local segment: seq / removedSeq = UnassignedSequenceNumber with its localSeq, as
        // mergeTree.ts:1397-1427 / 1955-2047 leave them)
        const segment = { cachedLength: r.length, seq: r.seq, clientId: longId(r.client), leafIndex: r.leaf,
            removedSeq: r.removed ? r.removedSeq : undefined, propertySet: r.props < 0 ? undefined : r.props };
        // (where createLocalReferencePosition finds it again while no edit intervened)
        Object.defineProperty(segment, '_at', { value: { start: r.start, view: sequenceArgs,
            stamp: this.log.nPushed }, enumerable: false });
        if (r.localSeq >= 0) segment.localSeq = r.localSeq;
        if (r.localRemovedSeq >= 0) segment.localRemovedSeq = r.localRemovedSeq;
        if (r.marker) segment.marker = { refType: r.refType };
        else segment.text = r.text;
        return { segment, offset: r.offset };
    }
    /**
     * Client.summarize (client.ts:966-1000) -> ISummaryTreeWithStats.  In the legacy format the
     * catch-up messages are the shim's own transformed list (CatchUpLog): the caller's list was built
     * without sequenceDelta events, so it is superseded.
     */
    summarize(runtime, handle, serializer, catchUpMsgs) {
        const dm = runtime.deltaManager;
        this.updateSeqNumbers(dm.minimumSequenceNumber, dm.lastSequenceNumber);
        const v1 = !!this.engine.options.snapshotV1;
        if (v1 && catchUpMsgs !== undefined && catchUpMsgs.length > 0) throw new Error('0x03f');
        this.engine.flush();
        this._check();
        if (!this.engine.summarized) { native().summarize(this.engine.h); this.engine.summarized = true; }
        return this._summaryTree(catchUpMsgs, dm, handle, serializer, v1);
    }
    /** summarize on a worker thread: resolves to the same ISummaryTreeWithStats. */
    async summarizeAsync(runtime, handle, serializer, catchUpMsgs) {
        const dm = runtime.deltaManager;
        this.updateSeqNumbers(dm.minimumSequenceNumber, dm.lastSequenceNumber);
        const v1 = !!this.engine.options.snapshotV1;
        if (v1 && catchUpMsgs !== undefined && catchUpMsgs.length > 0) throw new Error('0x03f');
        await this.engine.summarizeAllAsync();
        this._check();
        return this._summaryTree(catchUpMsgs, dm, handle, serializer, v1);
    }
    _summaryTree(catchUpMsgs, dm, handle, serializer, v1) {
        const blobs = native().getSummary(this.engine.h, this.doc);
        if (!v1) catchUpMsgs = this.engine.catchUps[this.doc].forSummary(dm.minimumSequenceNumber);
        const names = v1 ? blobs.map((_, i) => (i === 0 ? 'header' : 'body_' + (i - 1))) : ['header', 'body'];
        const tree = {};
        let total = 0;
        blobs.forEach((b, i) => { tree[names[i]] = { type: SummaryType.Blob, content: b.toString('utf8') }; total += b.length; });
        if (!v1 && catchUpMsgs !== undefined && catchUpMsgs.length > 0) {  // snapshotlegacy.ts:174-179
            const s = serializer ? serializer.stringify(catchUpMsgs, handle) : JSON.stringify(catchUpMsgs);
            tree[this.engine.options.catchUpBlobName || 'catchupOps'] = { type: SummaryType.Blob, content: s };
            total += Buffer.byteLength(s, 'utf8');
        }
        return {
            stats: { treeNodeCount: 1, blobNodeCount: Object.keys(tree).length, handleNodeCount: 0,
                totalBlobSize: total, unreferencedBlobSize: 0 },
            summary: { type: SummaryType.Tree, tree },
        };
    }
}

/**
 * A SharedMatrix observer (matrix/src/matrix.ts:636-693, remote branch) on a pair of engine documents:
 * applyMsg queues vector / set-cell messages; summarizeVectors returns each PermutationVector's summary
 * (V1 segments blobs + handleTable, permutationvector.ts:310-325).  (Cell values are host-side state;
 * the Python mirror fluidframework_amd/cells.py builds the cells blob from the engine's cell records.)
 */
class BatchMatrixClient {
    constructor(engine, rowsDoc) { this.engine = engine; this.doc = rowsDoc; this.log = engine.logs[rowsDoc]; }
    startOrUpdateCollaboration(longClientId, minSeq, currentSeq) {
        this.engine._assertIdle();
        this.log.startCollab(longClientId, minSeq || 0, currentSeq || 0);
        this.engine.dirty = true;
    }
    applyMsg(msg) { this.engine._assertIdle(); this.log.message(msg, this.engine.interner); this.engine.dirty = true; }
    summarizeVectors() {
        this.engine.flush();
        for (const d of [this.doc, this.doc + 1]) {
            const st = native().docStatus(this.engine.h, d);
            if (st[0] !== STATUS.OK) throw new Error('engine status ' + st[0] + ' at op ' + st[1]);
        }
        if (!this.engine.summarized) { native().summarize(this.engine.h); this.engine.summarized = true; }
        const vec = (d) => native().getSummary(this.engine.h, d).map((b) => b.toString('utf8'));
        return { rows: vec(this.doc), cols: vec(this.doc + 1) };
    }
}

module.exports = { BatchReplayEngine, BatchReplayClient, BatchMatrixClient, Interner, DocLog, MatrixDocLog, matrixLogs,
    regenRecords, regeneratedOp,
    buildBatch, UnsupportedError, OP, F, SummaryType, native };
