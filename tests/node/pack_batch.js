'use strict';
// Pack reference replay logs with the Node host packer (fluidframework_amd/node/index.js) and print
// the batch arrays (base64) so the Python test can compare them with fluidframework_amd.batch.
// usage: node pack_batch.js [--pre N] <replay.json.gz> [...]
//   --pre N: the first N messages arrive before startOrUpdateCollaboration (after an undefined-id call,
//            which must keep the client local), and the observer reconnects as 'observer-2' halfway
const fs = require('fs');
const zlib = require('zlib');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const it = new m.Interner();
let args = process.argv.slice(2);
let pre = -1;
if (args[0] === '--pre') { pre = Number(args[1]); args = args.slice(2); }
const logs = args.map((f) => {
    const groups = JSON.parse(zlib.gunzipSync(fs.readFileSync(f)).toString('utf8'));
    const log = new m.DocLog();
    if (groups[0].initialText) log.localInsert(0, groups[0].initialText, it);
    const msgs = [];
    for (const g of groups) for (const msg of g.msgs) msgs.push(msg);
    if (pre < 0) {
        log.startCollab('A', 0, 0);
        for (const msg of msgs) log.message(msg, it);
    } else {
        msgs.slice(0, pre).forEach((msg) => log.message(msg, it));
        log.startCollab(undefined, 0, 0);
        log.startCollab('A', 0, 0);
        const half = pre + Math.floor((msgs.length - pre) / 2);
        msgs.slice(pre, half).forEach((msg) => log.message(msg, it));
        log.startCollab('observer-2', 0, 0);
        msgs.slice(half).forEach((msg) => log.message(msg, it));
    }
    log.seqUpdate(groups[groups.length - 1].msgs.slice(-1)[0].minimumSequenceNumber,
        groups[groups.length - 1].msgs.slice(-1)[0].sequenceNumber);
    return log;
});
const b = m.buildBatch(logs, it);
const out = {};
for (const k of Object.keys(b)) out[k] = Buffer.from(b[k].buffer, b[k].byteOffset, b[k].byteLength).toString('base64');
process.stdout.write(JSON.stringify(out));
