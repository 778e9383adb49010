'use strict';
// The summarizer's hand-over from the Node host (BatchReplayEngine.replaySummaries -> the addon's
// replaySummaries -> mtr_replay_pipelined): the reference replay logs (client.replay.spec.ts:17-71), every group
// but the last flushed as usual (texts checked against resultText), the last applied, summarized and downloaded in
// one call.  Prints each document's record (u32 blob count, u32 lengths, blobs) as base64 blobs, whether the
// pipelined path ran, and the texts checked afterwards, for the Python test to compare with the CPU oracle.
// mode "local": document 0 also queues a pending local insert before the call, so the batch holds a record the
// pipelined path refuses and the addon takes the serial calls (V1 summaries leave the unacked insert out).
// usage: node replay_summaries.js <parts> <remote|local> <replay.json.gz> [...]
const fs = require('fs');
const zlib = require('zlib');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const parts = Number(process.argv[2]);
const mode = process.argv[3];
const files = process.argv.slice(4);
const all = files.map((f) => JSON.parse(zlib.gunzipSync(fs.readFileSync(f)).toString('utf8')));
const engine = new m.BatchReplayEngine(files.length, { snapshotV1: 1, maxSegments: 8192, heapEntries: 8192,
    textUnits: 1 << 18, propWords: 1 << 18, removerCells: 1 << 14, opsPerLaunch: 64 });
const clients = all.map((groups) => {
    const c = engine.createClient();
    if (groups[0].initialText) c.insertTextLocal(0, groups[0].initialText);
    c.startOrUpdateCollaboration('A');
    return c;
});
const nGroups = Math.max(...all.map((g) => g.length));
let checks = 0;
let rec = null;
for (let gi = 0; gi < nGroups; gi++) {
    all.forEach((groups, d) => { if (gi < groups.length) for (const msg of groups[gi].msgs) clients[d].applyMsg(msg); });
    if (gi === nGroups - 1) {
        if (mode === 'local') clients[0].insertTextLocal(0, 'xyz');
        rec = engine.replaySummaries(parts);
    }
    all.forEach((groups, d) => {
        if (gi >= groups.length || (mode === 'local' && d === 0 && gi === nGroups - 1)) return;
        if (clients[d].getText() !== groups[gi].resultText) throw new Error(`doc ${d} group ${gi}: text differs`);
        checks++;
    });
}
const result = all.map((groups, d) => {
    const r = rec.bytes.subarray(rec.docOff[d], rec.docOff[d + 1]);
    const nb = r.readUInt32LE(0);
    const blobs = [];
    let at = 4 + 4 * nb;
    for (let k = 0; k < nb; k++) {
        const len = r.readUInt32LE(4 + 4 * k);
        blobs.push(r.subarray(at, at + len).toString('base64'));
        at += len;
    }
    if (at !== r.length) throw new Error(`doc ${d}: record length ${r.length}, blobs end at ${at}`);
    // the per-client summarize() still reads the same blobs
    const last = groups[groups.length - 1].msgs.slice(-1)[0];
    const s = clients[d].summarize({ deltaManager: { minimumSequenceNumber: last.minimumSequenceNumber,
        lastSequenceNumber: last.sequenceNumber } }, undefined, undefined, []);
    const again = Object.values(s.summary.tree).map((b) => Buffer.from(b.content, 'utf8').toString('base64'));
    return { doc: d, blobs, same_as_summarize: JSON.stringify(again) === JSON.stringify(blobs) };
});
process.stdout.write(JSON.stringify({ checks, pipelined: rec.pipelined, result }));
