'use strict';
// SharedMatrix observers through the Node host (MatrixDocLog / BatchMatrixClient).
// usage: node matrix_engine.js --pack <feeds.json>   -> the packed batch arrays (base64), matrixLogs order
//        node matrix_engine.js --run <feeds.json> <chunk> -> per matrix {rows, cols} summary blobs
//   feeds.json: [{observer, msgs}, ...], one entry per matrix
const fs = require('fs');
const path = require('path');
const m = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const mode = process.argv[2];
const feeds = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
if (mode === '--pack') {
    const it = new m.Interner();
    const logs = feeds.map((f) => {
        const log = new m.MatrixDocLog();
        log.startCollab(f.observer, 0, 0);
        for (const msg of f.msgs) log.message(msg, it);
        return log;
    });
    const b = m.buildBatch(m.matrixLogs(logs), it);
    const out = {};
    for (const k of Object.keys(b)) out[k] = Buffer.from(b[k].buffer, b[k].byteOffset, b[k].byteLength).toString('base64');
    process.stdout.write(JSON.stringify(out));
} else {
    const chunk = Number(process.argv[4]);
    const engine = new m.BatchReplayEngine(2 * feeds.length, { maxSegments: 8192, heapEntries: 8192, textUnits: 1 << 15,
        propWords: 1024, removerCells: 4096, opsPerLaunch: 64 });
    const mats = feeds.map((f) => {
        const c = engine.createMatrix();
        c.startOrUpdateCollaboration(f.observer);
        return c;
    });
    const longest = Math.max(...feeds.map((f) => f.msgs.length));
    for (let k = 0; k < longest; k += chunk) {
        feeds.forEach((f, i) => { for (const msg of f.msgs.slice(k, k + chunk)) mats[i].applyMsg(msg); });
        engine.flush();
    }
    const out = mats.map((c) => {
        const v = c.summarizeVectors();
        return { rows: v.rows.map((x) => Buffer.from(x, 'utf8').toString('base64')),
            cols: v.cols.map((x) => Buffer.from(x, 'utf8').toString('base64')) };
    });
    process.stdout.write(JSON.stringify(out));
}
