'use strict';
/*
 * Legacy-format catch-up ops of collaborating clients through the Node host (tests/test_catchup_live.py, -m gpu):
 * replays a script of edits / interval adds / reconnects (made by the Python test from its oracle-driven run) on
 * three BatchReplayClients in the legacy summary format, then prints each client's text and summary blobs
 * (header, body, catchupOps) as JSON.
 */
const fs = require('fs');
const { Factory } = require('./mock_runtime.js');

const SLIDE = 2;
const script = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const f = new Factory({ snapshotV1: 0 });
const rts = [f.runtime('0'), f.runtime('1'), f.runtime('2')];

for (const a of script) {
    const r = rts[a[1]];
    switch (a[0]) {
        case 'ins': r.insertText(a[2], a[3]); break;
        case 'rem': r.removeRange(a[2], a[3]); break;
        case 'ann': r.annotateRange(a[2], a[3], a[4]); break;
        case 'iv': r.coll('c').add(a[2], a[3], SLIDE); break;
        case 'conn':
            if (r.connected !== a[2]) {
                r.connected = a[2];
                if (a[2]) f.processAll();  // as the Python script's replay does
            }
            break;
        case 'proc': for (let i = 0; i < a[1] && f.messages.length; i++) f.processOne(); break;
        case 'procall': f.processAll(); break;
        default: throw new Error('action ' + a[0]);
    }
}
const dm = { deltaManager: { minimumSequenceNumber: f.lastMsn, lastSequenceNumber: f.seq } };
const out = { texts: rts.map((r) => r.getText()), summaries: [] };
for (const r of rts) {
    const tree = r.client.summarize(dm).summary.tree;
    out.summaries.push(Object.keys(tree).map((k) => [k, tree[k].content]));
}
process.stdout.write(JSON.stringify(out) + '\n');
