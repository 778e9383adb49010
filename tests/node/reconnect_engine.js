'use strict';
// A reconnecting writer through the Node shim (BatchReplayClient): local ops, sequenced messages (its own
// are acks), rollback and regeneratePendingOp, from the events tests/test_regenerate.py recorded on the oracle.
// Prints {regens: [[regenerated op per pending op] per reconnect], texts: [getText() at every check]}.
const fs = require('fs');
const path = require('path');
const { BatchReplayEngine } = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

const spec = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const engine = new BatchReplayEngine(1, { newLengthCalc: spec.newlen ? 1 : 0 });
const client = engine.createClient();
client.startOrUpdateCollaboration(spec.me);
const regens = [], texts = [];
for (const e of spec.events) {
    if (e.local) client.localTransaction({ ops: [e.local], type: 3 });
    else if (e.msg) client.applyMsg(e.msg);
    else if (e.rollback) client.rollback(e.rollback);
    else if (e.regen) regens.push(e.regen.map((op) => client.regeneratePendingOp(op)));
    else if (e.check) texts.push(client.getText());
}
console.log(JSON.stringify({ regens, texts }));
