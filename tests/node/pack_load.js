'use strict';
// Client.load through the Node host packer (fluidframework_amd/node/index.js DocLog.loadSummary): every summary of
// the input file becomes one document's records; prints the batch arrays (base64) and each document's catch-up
// message count, so the Python test can compare them with fluidframework_amd.batch's DocLog.load_summary.
// usage: node pack_load.js <summaries.json>   ([{blobs: {name: text}, id: long client id or null}, ...])
const fs = require('fs');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const it = new m.Interner();
const docs = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const catchup = [];
const logs = docs.map((d) => {
    const log = new m.DocLog();
    catchup.push(log.loadSummary(d.blobs, d.id === null ? undefined : d.id, it).length);
    return log;
});
const b = m.buildBatch(logs, it);
const out = { catchup };
for (const k of Object.keys(b)) out[k] = Buffer.from(b[k].buffer, b[k].byteOffset, b[k].byteLength).toString('base64');
process.stdout.write(JSON.stringify(out));
