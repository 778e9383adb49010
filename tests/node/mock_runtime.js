'use strict';
/*
 * The reference's container-runtime mocks restated for the Node host's live clients (test infrastructure; the Python
 * twin is tests/mock_runtime.py): MockContainerRuntimeFactory / MockContainerRuntime (runtime/test-runtime-utils/src/
 * mocks.ts:102-303) and their reconnection variants (mocksForReconnection.ts:18-140), each runtime holding the
 * SharedString around one BatchReplayClient of one engine.
 */
const path = require('path');
const { BatchReplayEngine } = require(path.join(__dirname, '..', '..', 'fluidframework_amd', 'node', 'index.js'));

class Runtime {  // MockContainerRuntime(ForReconnection) + the SharedString around one BatchReplayClient
    constructor(factory, name) {
        this.factory = factory; this.clientId = name; this.csn = 0; this.lastSeq = 0;
        this.pending = []; this.pendingRemote = []; this._connected = true;
        this.client = factory.engine.createClient();
        this.client.startOrUpdateCollaboration(name, 0, 0);
        this.colls = new Map();
    }
    submit(contents, meta) {
        if (!this._connected) { this.pending.push([contents, meta, -1]); return; }
        const csn = this.csn++;
        this.factory.push({ clientId: this.clientId, clientSequenceNumber: csn, contents,
            referenceSequenceNumber: this.lastSeq, type: 'op' });
        this.pending.push([contents, meta, csn]);
    }
    process(msg) {
        if (!this._connected) { this.pendingRemote.push(msg); return; }
        this.lastSeq = msg.sequenceNumber;
        const local = msg.clientId === this.clientId;
        let meta;
        if (local) {
            const p = this.pending.shift();
            if (p[2] !== msg.clientSequenceNumber) throw new Error('Unexpected client sequence number from message');
            meta = p[1];
        }
        this.client.applyMsg(msg, local, meta);
    }
    get connected() { return this._connected; }
    set connected(v) {
        if (v === this._connected) return;
        this._connected = v;
        if (v) {
            for (const m of this.pendingRemote) this.process(m);
            this.pendingRemote = [];
            this.csn = 0;
            this.clientId = 'reconnected-' + (++this.factory.reconnects);
            const msgs = this.pending;
            this.pending = [];
            for (const [contents, meta] of msgs) {
                if (contents.type === 'act') this.submit(this.client.rebaseIntervalOp(contents, meta), meta);
                else this.submit(this.client.regeneratePendingOp(contents), meta);
            }
            this.client.startOrUpdateCollaboration(this.clientId);
        } else {
            this.factory.messages = this.factory.messages.filter((m) => m.clientId !== this.clientId);
        }
    }
    // the SharedString API the cases use
    insertText(pos, text) { this.client.insertTextLocal(pos, text); this.submit({ pos1: pos, seg: text, type: 0 }, {}); }
    removeRange(a, b) { this.client.removeRangeLocal(a, b); this.submit({ pos1: a, pos2: b, type: 1 }, {}); }
    annotateRange(a, b, props) { this.client.annotateRangeLocal(a, b, props); this.submit({ pos1: a, pos2: b, props, type: 2 }, {}); }
    getText() { return this.client.getText(); }
    coll(label) {
        if (!this.colls.has(label)) {
            this.colls.set(label, this.client.getIntervalCollection(label, (opName, value, meta) => {
                this.submit({ key: label, type: 'act', value: { opName, value } }, meta);
            }));
        }
        return this.colls.get(label);
    }
}

class Factory {  // MockContainerRuntimeFactory(ForReconnection)
    constructor(options) { this.engine = new BatchReplayEngine(4, options); this.lastMsn = 0; this.reconnects = 0; this.seq = 0; this.minSeq = new Map(); this.messages = []; this.rts = []; }
    runtime(name) { const r = new Runtime(this, name); this.rts.push(r); return r; }
    push(msg) {
        if (msg.clientId && !this.minSeq.has(msg.clientId)) this.minSeq.set(msg.clientId, msg.referenceSequenceNumber);
        this.messages.push(msg);
    }
    processOne() {
        const msg = JSON.parse(JSON.stringify(this.messages.shift()));
        this.minSeq.set(msg.clientId, msg.referenceSequenceNumber);
        msg.sequenceNumber = ++this.seq;
        msg.minimumSequenceNumber = Math.min(...this.minSeq.values());
        this.lastMsn = msg.minimumSequenceNumber;
        for (const r of this.rts) r.process(msg);
    }
    processAll() { while (this.messages.length) this.processOne(); }
}

module.exports = { Runtime, Factory };
