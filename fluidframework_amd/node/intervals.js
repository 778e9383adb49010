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

class Interval {
    constructor(start, end, itype, props, kind) {
        this.start = start; this.end = end; this.itype = itype; this.props = props; this.kind = kind;
    }
    id() {  // getIntervalId (:554-560)
        const v = this.props[INTERVAL_ID];
        return v === undefined || v === null ? undefined : `${v}`;
    }
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
        return new Interval(s, e, itype, { [RANGE_LABELS]: [this.label] }, kind);
    }
    _add(iv) {
        const i = iv.id();
        if (i === undefined) throw new Error('0x2c0');
        if (this.byId.has(i) || i === '') throw new IntervalUnsupported('two intervals with one id');
        this.byId.set(i, iv);
    }
    _remove(iv) { this.byId.delete(iv.id()); }
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
    ackDelete(si) {  // :2187-2208
        const i = ensureSerializedId(si)[INTERVAL_ID];
        const iv = typeof i === 'string' ? this.byId.get(i) : undefined;
        if (iv !== undefined) this._remove(iv);
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
            iv = nv;
        }
        addProps(iv.props, newProps);
    }
    serialize(states, currentSeq) {  // LocalIntervalCollection.serialize (:1105-1112) + compressInterval (:139-151)
        const pos = (ref, fromOp) => {
            const p = states[2 * ref], st = states[2 * ref + 1];
            if ((st & REF_ST.SEGMENT) && (st & REF_ST.HELD) && !(st & REF_ST.REMOVED) && p >= 0) return p;
            if (!(st & REF_ST.SEGMENT) && fromOp) return -1;
            if (!(st & REF_ST.SEGMENT)) throw new IntervalUnsupported('an endpoint created without an op has no segment');
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
        else if (name === 'delete') c.ackDelete(si);
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

module.exports = { IntervalCollections, IntervalUnsupported, IntervalType };
