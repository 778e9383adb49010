'use strict';
// The asynchronous Node host path: the reference replay test (client.replay.spec.ts:17-71) with every
// group applied by BatchReplayEngine.flushAsync (N-API async work on a worker thread) and the summaries
// built by summarizeAsync, then Client.getContainingSegment queries (client.ts:1065) answered on the
// device.  Prints the summary blobs (base64) and the query answers for the Python test to compare with
// the CPU oracle.
// usage: node async_engine.js <queries.json> <replay.json.gz> [...]
//   queries.json: per document a list of [pos, refSeq, longClientId]; [pos] alone = no sequenceArgs
const fs = require('fs');
const zlib = require('zlib');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

async function main() {
    const queries = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
    const files = process.argv.slice(3);
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
    let checks = 0, busy = 0, ticks = 0;
    for (let gi = 0; gi < nGroups; gi++) {
        all.forEach((groups, d) => { if (gi < groups.length) for (const msg of groups[gi].msgs) clients[d].applyMsg(msg); });
        const p = engine.flushAsync();
        if (engine.dirty) {  // the run is in flight: the addon refuses the engine until it settles
            try { m.native().docStatus(engine.h, 0); } catch (e) { if (/engine busy/.test(e.message)) busy++; }
        }
        const timer = setImmediate(() => { ticks++; });  // the event loop is not blocked meanwhile
        await p;
        clearImmediate(timer);
        all.forEach((groups, d) => {
            if (gi >= groups.length) return;
            if (clients[d].getText() !== groups[gi].resultText) throw new Error(`doc ${d} group ${gi}: text differs`);
            checks++;
        });
    }
    const result = [];
    for (let d = 0; d < all.length; d++) {
        const groups = all[d];
        const last = groups[groups.length - 1].msgs.slice(-1)[0];
        const s = await clients[d].summarizeAsync({ deltaManager: { minimumSequenceNumber: last.minimumSequenceNumber,
            lastSequenceNumber: last.sequenceNumber } }, undefined, undefined, []);
        const answers = queries[d].map((q) => {
            const r = q.length === 1 ? clients[d].getContainingSegment(q[0])
                : clients[d].getContainingSegment(q[0], { referenceSequenceNumber: q[1], clientId: q[2] });
            if (r.segment === undefined) return null;
            const seg = r.segment;
            return [seg.leafIndex, r.offset, seg.cachedLength, seg.text === undefined ? -1 : seg.text.length, seg.seq,
                seg.clientId];
        });
        result.push({ doc: d, names: Object.keys(s.summary.tree), answers,
            blobs: Object.values(s.summary.tree).map((b) => Buffer.from(b.content, 'utf8').toString('base64')) });
    }
    process.stdout.write(JSON.stringify({ checks, busy, ticks, result }));
}
main().catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
