'use strict';
// Legacy-format summaries with catch-up ops through the Node host path (SURVEY.md §8 row f2):
// BatchReplayClient keeps the transformed messages-since-MSN list from the engine's delta ranges.
// Input: a JSON file [{observer, msgs: [ISequencedDocumentMessage...]}...]; messages are applied in
// chunks of `chunk` (a getText() after each chunk flushes the batch).  Output: per document the
// summary tree's blob names and contents (base64) and the final text.
// usage: node catchup_engine.js <docs.json> <chunk>
const fs = require('fs');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const docs = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const chunk = Number(process.argv[3]);
const engine = new m.BatchReplayEngine(docs.length, { snapshotV1: 0, maxSegments: 4096, heapEntries: 4096,
    textUnits: 1 << 15, propWords: 1 << 14, removerCells: 2048, opsPerLaunch: 24 });
const clients = docs.map((d) => {
    const c = engine.createClient();
    c.startOrUpdateCollaboration(d.observer);
    return c;
});
const n = Math.max(...docs.map((d) => d.msgs.length));
for (let k = 0; k < n; k += chunk) {
    docs.forEach((d, i) => { for (const msg of d.msgs.slice(k, k + chunk)) clients[i].applyMsg(msg); });
    clients[0].getText();
}
const result = docs.map((d, i) => {
    const last = d.msgs[d.msgs.length - 1];
    const s = clients[i].summarize({ deltaManager: { minimumSequenceNumber: last.minimumSequenceNumber,
        lastSequenceNumber: last.sequenceNumber } }, undefined, undefined, undefined);
    return { doc: i, names: Object.keys(s.summary.tree), text: clients[i].getText(),
        blobs: Object.values(s.summary.tree).map((b) => Buffer.from(b.content, 'utf8').toString('base64')) };
});
process.stdout.write(JSON.stringify(result));
