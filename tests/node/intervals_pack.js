'use strict';
// Interval collections through the Node host packer (fluidframework_amd/node/index.js + intervals.js): each input
// session (an initial text, or a loaded summary with its interval `header`, then sequenced messages, or the detached
// recipe's local adds) becomes one DocLog; prints every session's records (base64 batch arrays) and the `header`
// blob the host writes from the reference states the Python test supplies (the CPU oracle's, for the same records).
// usage: node intervals_pack.js <sessions.json>
const fs = require('fs');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const sessions = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const out = [];
for (const s of sessions) {
    const it = new m.Interner();
    const log = new m.DocLog();
    if (s.header !== undefined) {
        const { IntervalCollections } = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'intervals.js'));
        log.intervals = new IntervalCollections();
        log.intervals.populate(s.header);
        log.loadSummary(s.blobs, 'loader', it);
        log.intervals.attach(log);
    }
    for (const o of s.local || []) log.localInsert(o[0], o[1], it);
    for (const a of s.adds || []) {
        if (log.intervals === undefined) {
            const { IntervalCollections } = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'intervals.js'));
            log.intervals = new IntervalCollections();
        }
        log.intervals.get(a[0]).add(log, a[1], a[2], a[3], { intervalId: a[4] });
    }
    if (s.initial !== undefined) {
        log.localInsert(0, s.initial, it);
        log.startCollab('observer', 0, 0);
    }
    for (const msg of s.msgs || []) log.message(msg, it);
    const b = m.buildBatch([log], it);
    const rec = {};
    for (const k of ['docs', 'ops', 'text']) rec[k] = Buffer.from(b[k].buffer, b[k].byteOffset, b[k].byteLength).toString('base64');
    rec.header = log.intervals.serialize(Int32Array.from(s.states), log.currentSeq);
    out.push(rec);
}
process.stdout.write(JSON.stringify(out));
