'use strict';
/*
 * Reference-id recycling through the Node host (tests/test_node.py, -m gpu): the twin of tests/test_interval_live.py's
 * `churn` -- two clients change interval endpoints, query (findOverlappingIntervals, the start-position iterator) and
 * edit text every round with the same PRNG, on an engine whose reference table holds 64 ids.  Prints
 * {out: [[text, [[start, end]...]] per checkpoint], nRefs: [...], status: [...]}.
 */
const { Factory } = require('./mock_runtime.js');

const SLIDE = 2;
class Lcg {
    constructor(seed) { this.x = seed & 0x7fffffff; }
    next(n) { this.x = Number((BigInt(this.x) * 1103515245n + 12345n) & 0x7fffffffn); return (this.x >> 8) % n; }
}

const rounds = Number(process.argv[2] || 160);
const f = new Factory({ refSlots: 64 });
const s1 = f.runtime('1'), s2 = f.runtime('2');
s1.insertText(0, 'abcdefghijklmnopqrstuvwxyz'.repeat(3));
f.processAll();
const ca = s1.coll('t'), cb = s2.coll('t');
const ids = [];
for (let i = 0; i < 60; i += 12) ids.push(ca.add(i, i + 4, SLIDE).id());
f.processAll();
const g = new Lcg(20240611);
const out = [];
const positions = (rt, c) => { const keys = rt.client.refKeys(); return Array.from(c).map((iv) => c.positions(iv, keys)); };
for (let rd = 0; rd < rounds; rd++) {
    for (const [s, c] of [[s1, ca], [s2, cb]]) {
        const n = s.client.getLength();
        const lo = g.next(n);
        c.change(ids[g.next(ids.length)], lo, lo + g.next(n - lo));
        const q = g.next(n);
        for (const iv of c.findOverlappingIntervals(q, q + 3)) if (iv.id() === undefined) throw new Error('no id');
        c.gather(true, q, undefined);
        if (g.next(10) < 3) s.insertText(g.next(n), 'xy');
        if (g.next(10) < 3 && s.client.getLength() > 20) {
            const p = g.next(s.client.getLength() - 2);
            s.removeRange(p, p + 2);
        }
    }
    if (rd % 3 === 2 || rd === rounds - 1) {
        f.processAll();
        out.push([s1.getText(), [positions(s1, ca)]]);
    }
}
s1.client._check();  // (throws on a document the engine failed, e.g. MTR_ERR_CAPACITY)
s2.client._check();
process.stdout.write(JSON.stringify({ out, nRefs: [s1.client.log.nRefs, s2.client.log.nRefs] }) + '\n');
