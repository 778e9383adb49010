'use strict';
// Pack local-op feeds with the Node host packer and print the batch arrays (base64), for comparison
// with fluidframework_amd.batch.  usage: node pack_events.js <feeds.json>
// ([{observer, events: [{local: op} | {msg: message}]}, ...]: a writer's local ops and the sequenced
// stream it applies, its own messages included -- they become acks)
const fs = require('fs');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const feeds = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const it = new m.Interner();
const logs = feeds.map((f) => {
    const log = new m.DocLog();
    log.startCollab(f.observer, 0, 0);
    for (const ev of f.events) {
        if (ev.local !== undefined) log.localOp(ev.local, it);
        else log.message(ev.msg, it);
    }
    return log;
});
const b = m.buildBatch(logs, it);
const out = {};
for (const k of Object.keys(b)) out[k] = Buffer.from(b[k].buffer, b[k].byteOffset, b[k].byteLength).toString('base64');
process.stdout.write(JSON.stringify(out));
