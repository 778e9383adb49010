'use strict';
// Pack reference replay logs with the Node host packer (fluidframework_amd/node/index.js) and print
// the batch arrays (base64) so the Python test can compare them with fluidframework_amd.batch.
// usage: node pack_batch.js <replay.json.gz> [...]
const fs = require('fs');
const zlib = require('zlib');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const it = new m.Interner();
const logs = process.argv.slice(2).map((f) => {
    const groups = JSON.parse(zlib.gunzipSync(fs.readFileSync(f)).toString('utf8'));
    const log = new m.DocLog();
    if (groups[0].initialText) log.localInsert(0, groups[0].initialText, it);
    log.startCollab('A', 0, 0);
    for (const g of groups) for (const msg of g.msgs) log.message(msg, it);
    log.seqUpdate(groups[groups.length - 1].msgs.slice(-1)[0].minimumSequenceNumber,
        groups[groups.length - 1].msgs.slice(-1)[0].sequenceNumber);
    return log;
});
const b = m.buildBatch(logs, it);
const out = {};
for (const k of Object.keys(b)) out[k] = Buffer.from(b[k].buffer, b[k].byteOffset, b[k].byteLength).toString('base64');
process.stdout.write(JSON.stringify(out));
