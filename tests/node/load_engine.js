'use strict';
// Client.load through the Node host path on the GPU (BatchReplayClient.load -> N-API -> C ABI -> HIP engine):
//  * every snapshot fixture is loaded through an IChannelStorageService stand-in and summarized again (the
//    Python test compares the bytes with the fixture's);
//  * each replay log is applied up to its middle group, summarized, loaded into a second client of the same
//    engine, and both clients apply the remaining groups: both must read resultText after every group, and
//    their final summaries are printed for the Python test.
// usage: node load_engine.js <fixtures.json> <replay.json.gz> [...]
const fs = require('fs');
const zlib = require('zlib');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

function storage(blobs) {  // IChannelStorageService
    return {
        list: async () => Object.keys(blobs),
        readBlob: async (n) => Buffer.from(blobs[n], 'utf8'),
        contains: async (n) => n in blobs,
    };
}
const runtime = (clientId) => ({ clientId, attachState: 'Attached' });
function dm(msn, seq) { return { deltaManager: { minimumSequenceNumber: msn, lastSequenceNumber: seq } }; }
const b64 = (s) => Object.values(s.summary.tree).map((x) => Buffer.from(x.content, 'utf8').toString('base64'));

async function main() {
    const fixtures = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
    const files = process.argv.slice(3);
    const logs = files.map((f) => JSON.parse(zlib.gunzipSync(fs.readFileSync(f)).toString('utf8')));
    const out = { fixtures: [], logs: [], checks: 0 };
    for (const v1 of [1, 0]) {  // one engine per summary format (the option is per engine)
        const keys = fixtures.filter((f) => f.v1 === v1);
        if (!keys.length) continue;
        const eng = new m.BatchReplayEngine(keys.length, { snapshotV1: v1, maxSegments: 16384, heapEntries: 16384,
            textUnits: 1 << 20, propWords: 1 << 18, removerCells: 1 << 14, opsPerLaunch: 64 });
        const clients = keys.map(() => eng.createClient());
        for (let i = 0; i < keys.length; i++) {
            const { catchupOpsP } = await clients[i].load(runtime('snapshot'), storage(keys[i].blobs));
            for (const msg of await catchupOpsP) clients[i].applyMsg(msg);
        }
        keys.forEach((k, i) => {
            const meta = JSON.parse(k.blobs.header);
            const hm = meta.headerMetadata || { minimumSequenceNumber: 0, sequenceNumber: meta.chunkSequenceNumber };
            const s = clients[i].summarize(dm(hm.minimumSequenceNumber || 0, hm.sequenceNumber), undefined, undefined, []);
            out.fixtures.push({ key: k.key, names: Object.keys(s.summary.tree), blobs: b64(s) });
        });
    }
    const eng = new m.BatchReplayEngine(2 * logs.length, { snapshotV1: 1, maxSegments: 8192, heapEntries: 8192,
        textUnits: 1 << 18, propWords: 1 << 18, removerCells: 1 << 14, opsPerLaunch: 64 });
    const a = logs.map((groups) => {
        const c = eng.createClient();
        if (groups[0].initialText) c.insertTextLocal(0, groups[0].initialText);
        c.startOrUpdateCollaboration('A');
        return c;
    });
    const cut = logs.map((g) => Math.floor(g.length / 2));
    logs.forEach((groups, d) => { for (let gi = 0; gi < cut[d]; gi++) for (const msg of groups[gi].msgs) a[d].applyMsg(msg); });
    const mid = logs.map((groups, d) => {
        const last = groups[cut[d] - 1].msgs.slice(-1)[0];
        return a[d].summarize(dm(last.minimumSequenceNumber, last.sequenceNumber), undefined, undefined, []);
    });
    const b = [];
    for (let d = 0; d < logs.length; d++) {
        const c = eng.createClient();
        const blobs = {};
        for (const k of Object.keys(mid[d].summary.tree)) blobs[k] = mid[d].summary.tree[k].content;
        await c.load(runtime('loader-B'), storage(blobs));
        b.push(c);
    }
    logs.forEach((groups, d) => {
        if (b[d].getText() !== groups[cut[d] - 1].resultText) throw new Error(`log ${d}: loaded text differs`);
    });
    const nGroups = Math.max(...logs.map((g) => g.length));
    for (let gi = 0; gi < nGroups; gi++) {
        logs.forEach((groups, d) => {
            if (gi < cut[d] || gi >= groups.length) return;
            for (const msg of groups[gi].msgs) { a[d].applyMsg(msg); b[d].applyMsg(msg); }
        });
        logs.forEach((groups, d) => {
            if (gi < cut[d] || gi >= groups.length) return;
            for (const c of [a[d], b[d]]) {
                if (c.getText() !== groups[gi].resultText) throw new Error(`log ${d} group ${gi}: text differs`);
                out.checks++;
            }
        });
    }
    logs.forEach((groups, d) => {
        const last = groups[groups.length - 1].msgs.slice(-1)[0];
        out.logs.push({ log: d, mid: b64(mid[d]),
            b: b64(b[d].summarize(dm(last.minimumSequenceNumber, last.sequenceNumber), undefined, undefined, [])) });
    });
    process.stdout.write(JSON.stringify(out));
}
main().catch((e) => { console.error(e.stack || e); process.exit(1); });
