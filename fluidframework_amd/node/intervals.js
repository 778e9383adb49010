'use strict';
/*
 * Interval collections of a SharedString on the replay engine, for the Node host (mirrors
 * fluidframework_amd/intervals.py record for record and byte for byte; SURVEY.md 8f4).
 *
 * The reference keeps a collection (sequence/src/intervalCollection.ts:1428 IntervalCollection, :788
 * LocalIntervalCollection) in red-black trees ordered by SequenceInterval.compare (:505-525) and summarizes it as
 * the start tree's in-order walk (:1105-1112).  Here the endpoints are engine references (MTR_OP_REF_CREATE
 * records created as createPositionReference does, :697-724) and the order is computed when the summary is
 * written, from the references' positions and states (mtr_get_ref_states): a tree's order only changes when an
 * endpoint slides, and every slide re-inserts its interval (:1114-1159), so the in-order walk is the sort by the
 * comparator at summary time -- the position order for endpoints held by live segments, -1 (smallest) for
 * endpoints without a segment.  Everything else is an UnsupportedError (the document falls back).
 */

const REFTYPE = { RANGE_BEGIN: 0x10, RANGE_END: 0x20, NEST_BEGIN: 0x2, NEST_END: 0x4, SLIDE_ON_REMOVE: 0x40,
    STAY_ON_REMOVE: 0x80 };
const REF_ST = { SEGMENT: 1, HELD: 2, REMOVED: 4 };  // include/mtr_types.h MTR_REF_ST_*
const IntervalType = { Simple: 0, Nest: 1, SlideOnRemove: 2, Transient: 4 };
const VALUE_TYPE = 'sharedStringIntervalCollection';  // SequenceIntervalCollectionValueType.Name, :1195
const RANGE_LABELS = 'referenceRangeLabels';
const INTERVAL_ID = 'intervalId';

class IntervalUnsupported extends Error {
    constructor(msg) { super(msg); this.name = 'UnsupportedError'; }
}

function addProps(props, newProps) {  // PropertiesManager.addProperties, no combining op (segmentPropertiesManager.ts:60-157)
    for (const k of Object.keys(newProps)) {
        if (newProps[k] === null) delete props[k];
        else props[k] = newProps[k];
    }
}

function refTypes(itype, slideOnRemove) {  // createSequenceInterval (:735-756)
    if (itype === IntervalType.Transient) throw new IntervalUnsupported('transient interval');
    const b = itype === IntervalType.Nest ? REFTYPE.NEST_BEGIN : REFTYPE.RANGE_BEGIN;
    const e = itype === IntervalType.Nest ? REFTYPE.NEST_END : REFTYPE.RANGE_END;
    const f = slideOnRemove ? REFTYPE.SLIDE_ON_REMOVE : REFTYPE.STAY_ON_REMOVE;
    return [b | f, e | f];
}

function intPos(v, what) {
    if (typeof v !== 'number' || !Number.isInteger(v)) throw new IntervalUnsupported('interval ' + what + ' that is not an integer position');
    return v;
}

function ensureSerializedId(si) {  // LocalIntervalCollection.ensureSerializedId (:838-858)
    let props = si.properties;
    if (props === null || typeof props !== 'object' || props[INTERVAL_ID] === undefined || props[INTERVAL_ID] === null) {
        props = Object.assign({}, props && typeof props === 'object' ? props : {});
        props[INTERVAL_ID] = `legacy${si.start}-${si.end}`;
        si.properties = props;
    }
    return props;
}

function decompress(ci, label) {  // decompressInterval (:122-133)
    return { start: ci[0], end: ci[1], sequenceNumber: ci[2], intervalType: ci[3],
        properties: Object.assign({}, ci[4], { [RANGE_LABELS]: [label] }) };
}

const UnassignedSequenceNumber = -1, UniversalSequenceNumber = 0;  // merge-tree/src/constants.ts

class UsageError extends Error {  // the reference's UsageError / LoggingError for a bad API call (nothing changes)
    constructor(msg) { super(msg); this.name = 'UsageError'; }
}

/** PropertiesManager (segmentPropertiesManager.ts:24-170) as an interval's property bag uses it: no combining ops. */
class PropertiesManager {
    constructor() { this.pending = undefined; }  // pendingKeyUpdateCount
    ack(props) {  // ackPendingProperties -> decrementPendingCounts (:33-58)
        for (const k of Object.keys(props)) {
            if (this.pending !== undefined && this.pending[k] !== undefined) {
                if (!(this.pending[k] > 0)) throw new Error('0x05c');
                this.pending[k]--;
                if (this.pending[k] === 0) delete this.pending[k];
            }
        }
    }
    add(old, newProps, seq, collaborating) {  // addProperties (:60-157) without a combining op
        if (this.pending === undefined) this.pending = Object.create(null);
        const deltas = {};
        for (const k of Object.keys(newProps)) {
            if (collaborating) {
                if (seq === UnassignedSequenceNumber) {
                    this.pending[k] = (this.pending[k] || 0) + 1;
                } else if (!(seq === UniversalSequenceNumber || this.pending[k] === undefined)) {
                    continue;  // shouldModifyKey
                }
            }
            deltas[k] = old[k] === undefined ? null : old[k];
            if (newProps[k] === null) delete old[k];
            else old[k] = newProps[k];
        }
        return deltas;
    }
    copyTo(old, newProps, mgr) {  // copyTo (:159-180)
        for (const k of Object.keys(old)) newProps[k] = old[k];
        mgr.pending = Object.assign(Object.create(null), this.pending || {});
    }
}

class Interval {
    constructor(start, end, itype, props, kind, stype, etype) {
        this.start = start; this.end = end; this.itype = itype; this.props = props; this.kind = kind;
        this.stype = stype || 0; this.etype = etype || 0;  // the endpoints' ReferenceTypes as the engine holds them
        this.pm = new PropertiesManager();
    }
    id() {  // getIntervalId (:554-560)
        const v = this.props[INTERVAL_ID];
        return v === undefined || v === null ? undefined : `${v}`;
    }
}

// compareReferencePositions' key of a reference (referencePositions.ts:113-121) from getRefKeys: no segment sorts
// first (equal to any other segment-less reference), else (segment order, offset)
function refKey(keys, ref) {
    const k = keys[4 * ref + 2];
    if (k === -1) return [0, 0, 0];
    if (k < 0) throw new IntervalUnsupported('an interval endpoint on a segment zamboni took out of the tree');
    return [1, k, keys[4 * ref + 3]];
}
function cmpKey(a, b) {
    for (let i = 0; i < 3; i++) if (a[i] !== b[i]) return a[i] < b[i] ? -1 : 1;
    return 0;
}
function ivCmp(keys, a, b) {  // SequenceInterval.compare (:505-525)
    const c = cmpKey(refKey(keys, a.start), refKey(keys, b.start)) || cmpKey(refKey(keys, a.end), refKey(keys, b.end));
    if (c) return c;
    const ia = a.id(), ib = b.id();
    return ia && ib ? (ia > ib ? 1 : ia < ib ? -1 : 0) : 0;
}

class Collection {
    constructor(label, saved) { this.label = label; this.saved = saved; this.byId = new Map(); }
    _create(log, start, end, itype, view, kind) {
        if (itype !== IntervalType.Simple && itype !== IntervalType.Nest && itype !== IntervalType.SlideOnRemove) {
            throw new IntervalUnsupported('intervalType ' + itype);
        }
        const [bt, et] = refTypes(itype, kind !== 'local');
        const s = log.createRef(start, bt, view, kind === 'op');
        const e = log.createRef(end, et, view, kind === 'op');
        return new Interval(s, e, itype, { [RANGE_LABELS]: [this.label] }, kind, bt, et);
    }
    _add(iv) {
        const i = iv.id();
        if (i === undefined) throw new Error('0x2c0');
        if (this.byId.has(i) || i === '') throw new IntervalUnsupported('two intervals with one id');
        this.byId.set(i, iv);
    }
    _remove(iv) { this.byId.delete(iv.id()); }
    // the endpoint references nothing reads again (a deleted interval's, those a change superseded) go back for reuse
    static _release(log, iv, keep) {
        for (const r of [iv.start, iv.end]) if (!keep || (r !== keep.start && r !== keep.end)) log.releaseRef(r);
    }
    attach(log) {  // attachGraph (:1531-1579)
        const saved = this.saved || [];
        this.saved = undefined;
        for (const si of saved) {
            const props = ensureSerializedId(si);
            const iv = this._create(log, intPos(si.start, 'start'), intPos(si.end, 'end'), si.intervalType, undefined, 'snapshot');
            addProps(iv.props, props);
            this._add(iv);
        }
    }
    add(log, start, end, itype, props) {  // IntervalCollection.add (:1635-1672) on a string that is not collaborating
        if (log.collaborating) throw new IntervalUnsupported('local interval ops while collaborating');
        if (itype & IntervalType.Transient) throw new Error('Can not add transient intervals');
        if (!props || props[INTERVAL_ID] === undefined || props[INTERVAL_ID] === null) {
            throw new IntervalUnsupported('a local interval without an id (a random uuid)');
        }
        const iv = this._create(log, start, end, itype, undefined, 'local');
        addProps(iv.props, props);
        this._add(iv);
        return iv;
    }
    ackAdd(log, si, msg) {  // :2141-2184
        ensureSerializedId(si);
        const view = { referenceSequenceNumber: msg.referenceSequenceNumber, clientId: msg.clientId };
        const iv = this._create(log, intPos(si.start, 'start'), intPos(si.end, 'end'), si.intervalType, view, 'op');
        if (si.properties && typeof si.properties === 'object') addProps(iv.props, si.properties);
        if (iv.props[INTERVAL_ID] === undefined) throw new IntervalUnsupported('an interval without an id (a random uuid)');
        this._add(iv);
    }
    ackDelete(log, si) {  // :2187-2208
        const i = ensureSerializedId(si)[INTERVAL_ID];
        const iv = typeof i === 'string' ? this.byId.get(i) : undefined;
        if (iv !== undefined) {
            this._remove(iv);
            Collection._release(log, iv);
        }
    }
    ackChange(log, si, msg) {  // :1859-1932
        const props = si.properties && typeof si.properties === 'object' ? si.properties : {};
        if (!(INTERVAL_ID in props)) throw new Error('0x3fe');
        const { [INTERVAL_ID]: i, ...newProps } = props;
        let iv = typeof i === 'string' ? this.byId.get(i) : undefined;
        if (iv === undefined) return;
        const { start, end } = si;
        if (start === null || end === null) throw new IntervalUnsupported('a change op with a null endpoint');
        if (start !== undefined || end !== undefined) {
            if (iv.kind === 'local') throw new IntervalUnsupported('a remote change of a local (StayOnRemove) interval');
            const view = { referenceSequenceNumber: msg.referenceSequenceNumber, clientId: msg.clientId };
            const [st, et] = refTypes(iv.itype, true);
            const s = start !== undefined ? log.createRef(intPos(start, 'start'), st, view, true) : iv.start;
            const e = end !== undefined ? log.createRef(intPos(end, 'end'), et, view, true) : iv.end;
            const nv = new Interval(s, e, iv.itype, Object.assign({}, iv.props), 'op');  // modify + copyTo (:600-656)
            this._remove(iv);
            this._add(nv);
            Collection._release(log, iv, nv);
            iv = nv;
        }
        addProps(iv.props, newProps);
    }
    // ---- a collaborating client's own ops (IntervalCollection.add / change / changeProperties / removeIntervalById,
    // :1635-1793, their acks :1859-2208, rebaseLocalInterval :1963-2029); `live` is the BatchReplayClient (its log,
    // the engine's answers and the collection's op emitter).  Mirrors fluidframework_amd/intervals.py.
    _pc(end) { const n = end ? 'pendingEnd' : 'pendingStart'; if (!this[n]) this[n] = new Map(); return this[n]; }
    _lseqMap(rebased) { const n = rebased ? 'lseqRebased' : 'lseqSerialized'; if (!this[n]) this[n] = new Map(); return this[n]; }
    hasPendingChange(id, end) { const e = this._pc(end).get(id); return !!(e && e.length); }
    _addPendingChange(id, ser) {  // addPendingChange (:1795-1815)
        if (ser.start !== undefined) { if (!this._pc(false).has(id)) this._pc(false).set(id, []); this._pc(false).get(id).push(ser); }
        if (ser.end !== undefined) { if (!this._pc(true).has(id)) this._pc(true).set(id, []); this._pc(true).get(id).push(ser); }
    }
    _removePendingChange(ser) {  // removePendingChange (:1817-1846)
        const id = ser.properties ? ser.properties[INTERVAL_ID] : undefined;
        for (const [end, key] of [[false, 'start'], [true, 'end']]) {
            if (ser[key] === undefined) continue;
            const entries = this._pc(end).get(id);
            if (entries) {
                const pc = entries.shift();
                if (entries.length === 0) this._pc(end).delete(id);
                if (!pc || pc.start !== ser.start || pc.end !== ser.end) throw new Error('Mismatch in pending changes');
            }
        }
    }
    _checkPosition(live, pos) {  // createPositionReference without an op: a segment must hold pos (:690-692)
        if (typeof pos !== 'number' || !Number.isInteger(pos)) throw new IntervalUnsupported('a local interval endpoint that is not an integer position');
        if (!(pos >= 0 && pos < live.getLength())) throw new UsageError('Non-transient references need segment');
    }
    liveAdd(live, start, end, itype, props) {  // IntervalCollection.add (:1635-1672)
        if (this.saved !== undefined) throw new UsageError('attach must be called prior to adding intervals');
        if (itype & IntervalType.Transient) throw new UsageError('Can not add transient intervals');
        this._checkPosition(live, start);
        this._checkPosition(live, end);
        const iv = this._create(live.log, start, end, itype, undefined, 'local');
        if (props) iv.pm.add(iv.props, props);
        if (iv.props[INTERVAL_ID] === undefined || iv.props[INTERVAL_ID] === null) {
            iv.props[INTERVAL_ID] = require('crypto').randomBytes(16).toString('hex');  // (the reference draws a uuid)
        }
        this._add(iv);
        const ser = { end, intervalType: itype, properties: iv.props, sequenceNumber: live.currentSeq, start };
        const localSeq = live.nextLocalSeq();
        this._lseqMap(false).set(localSeq, ser);
        live.emit(this.label, 'add', ser, { localSeq });
        return iv;
    }
    liveRemove(live, id) {  // removeIntervalById (:1706-1715) -> deleteExistingInterval(local) (:1674-1699)
        const iv = typeof id === 'string' ? this.byId.get(id) : undefined;
        if (iv === undefined) return undefined;
        const keys = live.refKeys();
        this._remove(iv);
        const ser = { end: keys[4 * iv.end], intervalType: iv.itype, sequenceNumber: live.currentSeq,
            start: keys[4 * iv.start], properties: iv.props };
        Collection._release(live.log, iv);
        live.emit(this.label, 'delete', ser, { localSeq: live.nextLocalSeq() });
        return iv;
    }
    liveChangeProperties(live, id, props) {  // changeProperties (:1723-1752)
        if (typeof id !== 'string') throw new UsageError('Change API requires an ID that is a string');
        if (!props) throw new UsageError('changeProperties should be called with a property set');
        const iv = this.byId.get(id);
        if (iv === undefined) return;
        iv.pm.add(iv.props, props, UnassignedSequenceNumber, true);
        props[INTERVAL_ID] = iv.id();
        const ser = { intervalType: iv.itype, sequenceNumber: live.currentSeq, properties: props };
        const localSeq = live.nextLocalSeq();
        this._lseqMap(false).set(localSeq, ser);
        live.emit(this.label, 'change', ser, { localSeq });
    }
    // LocalIntervalCollection.changeInterval (:1088-1103) -> SequenceInterval.modify (:600-656)
    _changeInterval(live, iv, start, end, view, localSeq) {
        const newRef = (pos, oldType) => {
            if (view !== undefined) {
                if (!(oldType & REFTYPE.SLIDE_ON_REMOVE)) throw new Error('0x2f5');
                return [live.log.createRef(intPos(pos, 'endpoint'), oldType, view, true), oldType];
            }
            const t = (oldType & ~REFTYPE.SLIDE_ON_REMOVE) | REFTYPE.STAY_ON_REMOVE;
            if (localSeq !== undefined) return [live.log.createRefAt(intPos(pos, 'endpoint'), t, live.currentSeq, localSeq), t];
            return [live.log.createRef(intPos(pos, 'endpoint'), t, undefined, false), t];
        };
        let [s, st, e, et] = [iv.start, iv.stype, iv.end, iv.etype];
        if (start !== undefined && start !== null) [s, st] = newRef(start, iv.stype);
        if (end !== undefined && end !== null) [e, et] = newRef(end, iv.etype);
        const nv = new Interval(s, e, iv.itype, {}, view !== undefined ? 'op' : iv.kind, st, et);
        iv.pm.copyTo(iv.props, nv.props, nv.pm);
        this._remove(iv);
        this._add(nv);
        Collection._release(live.log, iv, nv);
        return nv;
    }
    liveChange(live, id, start, end) {  // IntervalCollection.change (:1761-1793)
        if (typeof id !== 'string') throw new UsageError('Change API requires an ID that is a string');
        const iv = this.byId.get(id);
        if (iv === undefined) return undefined;
        for (const v of [start, end]) if (v !== undefined && v !== null) this._checkPosition(live, v);
        const nv = this._changeInterval(live, iv, start, end);
        const ser = { end, intervalType: iv.itype, sequenceNumber: live.currentSeq, start, properties: { [INTERVAL_ID]: iv.id() } };
        const localSeq = live.nextLocalSeq();
        this._lseqMap(false).set(localSeq, ser);
        live.emit(this.label, 'change', ser, { localSeq });
        this._addPendingChange(id, ser);
        return nv;
    }
    ackInterval(live, iv) {  // ackInterval (:2054-2138): one MTR_OP_REF_ACK per endpoint without a pending change
        if (!(iv.stype & REFTYPE.STAY_ON_REMOVE) && !(iv.etype & REFTYPE.STAY_ON_REMOVE)) return;
        const id = iv.props[INTERVAL_ID];
        if (!this.hasPendingChange(id, false)) {
            live.log.ackRef(iv.start);
            iv.stype = (iv.stype & ~REFTYPE.STAY_ON_REMOVE) | REFTYPE.SLIDE_ON_REMOVE;
        }
        if (!this.hasPendingChange(id, true)) {
            live.log.ackRef(iv.end);
            iv.etype = (iv.etype & ~REFTYPE.STAY_ON_REMOVE) | REFTYPE.SLIDE_ON_REMOVE;
        }
    }
    liveProcess(live, name, params, msg, local, meta) {  // the ops map (:1281-1325), ackAdd/ackDelete/ackChange
        if (name !== 'delete' && !params) return;
        if (!params || typeof params !== 'object') throw new IntervalUnsupported('interval op parameters');
        const si = Object.assign({}, params);
        if (name === 'add') {
            if (!local) return this.ackAdd(live.log, si, msg);
            this._lseqMap(false).delete(meta.localSeq);
            const iv = this.byId.get((si.properties || {})[INTERVAL_ID]);
            if (iv !== undefined) this.ackInterval(live, iv);
            return undefined;
        }
        if (name === 'delete') { if (!local) this.ackDelete(live.log, si); return undefined; }
        if (local) {
            this._lseqMap(false).delete(meta.localSeq);
            this._removePendingChange(si);
        }
        const props = si.properties && typeof si.properties === 'object' ? si.properties : {};
        if (!(INTERVAL_ID in props)) throw new Error('0x3fe');
        const { [INTERVAL_ID]: id, ...newProps } = props;
        let iv = typeof id === 'string' ? this.byId.get(id) : undefined;
        if (iv === undefined) return undefined;
        if (local) { iv.pm.ack(props); this.ackInterval(live, iv); return undefined; }
        const start = this.hasPendingChange(id, false) ? undefined : si.start;
        const end = this.hasPendingChange(id, true) ? undefined : si.end;
        if (start === null || end === null) throw new IntervalUnsupported('a change op with a null endpoint');
        if (start !== undefined || end !== undefined) {
            const view = { referenceSequenceNumber: msg.referenceSequenceNumber, clientId: msg.clientId };
            iv = this._changeInterval(live, iv, start, end, view);
        }
        iv.pm.add(iv.props, newProps, msg.sequenceNumber, true);
        return undefined;
    }
    rebasePositions(live, lseqs) {  // computeRebasedPositions (:1507-1528): one MTR_OP_REBASE_POS per endpoint
        const recs = [];
        for (const lseq of lseqs) {
            const original = this._lseqMap(false).get(lseq);
            if (original === undefined) throw new Error('0x551');
            for (const key of ['start', 'end']) {
                if (original[key] !== undefined) {
                    recs.push([lseq, key, live.log.rebasePosition(intPos(original[key], key), original.sequenceNumber, lseq)]);
                }
            }
        }
        const res = recs.length ? live.rebaseResults() : new Map();
        const out = new Map();
        for (const lseq of lseqs) out.set(lseq, Object.assign({}, this._lseqMap(false).get(lseq)));
        for (const [lseq, key, rec] of recs) out.get(lseq)[key] = res.get(rec);
        return out;
    }
    onNormalize(live) {  // the client's "normalize" listener (attachGraph, :1542-1551)
        const keys = Array.from(this._lseqMap(false).keys());
        if (keys.length) for (const [k, v] of this.rebasePositions(live, keys)) this._lseqMap(true).set(k, v);
    }
    rebaseLocal(live, name, ser, localSeq) {  // rebaseLocalInterval (:1963-2029); undefined = the op is a no-op
        if (name === 'delete') return ser;
        let rb = this._lseqMap(true).get(localSeq);
        if (rb === undefined) rb = this.rebasePositions(live, [localSeq]).get(localSeq);
        const props = ser.properties;
        const id = props ? props[INTERVAL_ID] : undefined;
        const local = typeof id === 'string' ? this.byId.get(id) : undefined;
        const rebased = { start: rb.start, end: rb.end, intervalType: ser.intervalType, sequenceNumber: live.currentSeq,
            properties: props };
        if (name === 'change' && (this.hasPendingChange(id, false) || this.hasPendingChange(id, true))) {
            this._removePendingChange(ser);
            this._addPendingChange(id, rebased);
        }
        if (rebased.start === -1 || rebased.end === -1) {
            if (local !== undefined) this._remove(local);
            return undefined;
        }
        if (local !== undefined) this._changeInterval(live, local, rebased.start, rebased.end, undefined, localSeq);
        return rebased;
    }
    ordered(keys) {  // the start tree's in-order walk: SequenceInterval.compare order
        return Array.from(this.byId.values()).sort((a, b) => ivCmp(keys, a, b));
    }
    serialize(states, currentSeq) {  // LocalIntervalCollection.serialize (:1105-1112) + compressInterval (:139-151)
        const pos = (ref, fromOp) => {
            const p = states[2 * ref], st = states[2 * ref + 1];
            if ((st & REF_ST.SEGMENT) && (st & REF_ST.HELD) && !(st & REF_ST.REMOVED) && p >= 0) return p;
            if (!(st & REF_ST.SEGMENT)) return -1;  // no segment (an op's detached endpoint, or slid off): first
            throw new IntervalUnsupported('an interval endpoint on a removed segment, or dropped by its segment');
        };
        const keyed = Array.from(this.byId.values(), (iv) => [pos(iv.start, iv.kind === 'op'), pos(iv.end, iv.kind === 'op'), iv]);
        keyed.sort((x, y) => {
            if (x[0] !== y[0]) return x[0] - y[0];
            if (x[1] !== y[1]) return x[1] - y[1];
            const a = x[2].id(), b = y[2].id();
            return a && b ? (a > b ? 1 : a < b ? -1 : 0) : 0;
        });
        return { label: this.label,
            intervals: keyed.map(([a, b, iv]) => [a, b, currentSeq, iv.itype, { ...iv.props, [RANGE_LABELS]: undefined }]),
            version: 2 };
    }
}

/** SharedSegmentSequence.intervalCollections (sequence.ts:186, a DefaultMap of IntervalCollection). */
class IntervalCollections {
    constructor() { this.data = new Map(); }
    populate(header) {  // DefaultMap.populate (defaultMap.ts:254-282)
        const j = typeof header === 'string' ? JSON.parse(header) : header;
        for (const [key, ser] of Object.entries(j)) {
            if (ser.type === 'Plain' || ser.type === 'Shared') continue;
            if (ser.type !== VALUE_TYPE) throw new IntervalUnsupported('value type ' + ser.type);
            const label = key.startsWith('intervalCollections/') ? key.substring(20) : key;
            const v = ser.value;
            const saved = Array.isArray(v) ? v.map((x) => Object.assign({}, x)) : v.intervals.map((ci) => decompress(ci, v.label));
            this.data.set(label, new Collection(label, saved));
        }
    }
    attach(log) { for (const c of this.data.values()) c.attach(log); }  // loadFinished (sequence.ts:750-801)
    get(label) {  // DefaultMap.get -> createCore (defaultMap.ts:210-213, 339-349)
        let c = this.data.get(label);
        if (c === undefined) { c = new Collection(label, undefined); this.data.set(label, c); }
        return c;
    }
    liveProcess(live, contents, msg, local, meta) {  // a live client's "act" handler: its own acks too
        if (typeof contents.key !== 'string') throw new IntervalUnsupported('an interval op without a string key');
        const value = contents.value || {};
        const name = value.opName;
        if (name !== 'add' && name !== 'delete' && name !== 'change') throw new IntervalUnsupported('interval op ' + name);
        this.get(contents.key).liveProcess(live, name, value.value, msg, local, meta);
    }
    process(log, contents, msg) {  // DefaultMap's "act" handler (defaultMap.ts:386-395), the ops map (:1266-1326)
        const cid = msg.clientId === null || msg.clientId === undefined ? 'null' : String(msg.clientId);
        if (cid === log.observerId) throw new IntervalUnsupported('acks of local interval ops');
        if (typeof contents.key !== 'string') throw new IntervalUnsupported('an interval op without a string key');
        const value = contents.value || {};
        const c = this.get(contents.key);
        const name = value.opName;
        if (name !== 'add' && name !== 'delete' && name !== 'change') throw new IntervalUnsupported('interval op ' + name);
        const params = value.value;
        if (name !== 'delete' && !params) return;
        if (!params || typeof params !== 'object') throw new IntervalUnsupported('interval op parameters');
        const si = Object.assign({}, params);
        if (name === 'add') c.ackAdd(log, si, msg);
        else if (name === 'delete') c.ackDelete(log, si);
        else c.ackChange(log, si, msg);
    }
    serialize(states, currentSeq) {  // summarizeCore's header blob (sequence.ts:467-480); undefined when none
        if (this.data.size === 0) return undefined;
        const out = {};
        for (const [key, c] of this.data) {
            if (c.saved !== undefined) throw new IntervalUnsupported('a collection that was never attached');
            out[key] = { type: VALUE_TYPE, value: c.serialize(states, currentSeq) };
        }
        return JSON.stringify(out);
    }
}

module.exports = { IntervalCollections, IntervalUnsupported, IntervalType, UsageError, refKey, cmpKey };
