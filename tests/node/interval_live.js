'use strict';
/*
 * A collaborating client's own interval ops through the Node host (tests/test_node.py, -m gpu): a few of
 * sequence/src/test/intervalCollection.spec.ts's known answers (the same cases tests/test_interval_live.py runs on
 * the Python host), with the reference's mock container runtime restated (runtime/test-runtime-utils/src/mocks.ts,
 * mocksForReconnection.ts) over BatchReplayClient documents of one engine.  Prints {case: "ok" | error}.
 */
const { Runtime, Factory } = require('./mock_runtime.js');

const SLIDE = 2;

function eq(a, b, what) {
    if (JSON.stringify(a) !== JSON.stringify(b)) throw new Error(what + ': ' + JSON.stringify(a) + ' != ' + JSON.stringify(b));
}
function assertIntervals(rt, c, expected, validateOverlapping = true) {  // intervalCollection.spec.ts:21-48
    const actual = Array.from(c);
    const n = rt.client.getLength();
    if (validateOverlapping && n > 0) eq(c.findOverlappingIntervals(0, n - 1).map((iv) => iv.id()), actual.map((iv) => iv.id()), 'overlapping');
    const keys = rt.client.refKeys();
    eq(actual.map((iv) => c.positions(iv, keys)), expected, 'intervals');
}
function two() { const f = new Factory(); const a = f.runtime('1'), b = f.runtime('2'); return [f, a, b]; }

const cases = {
    slide_on_remove_ack() {  // :386-409
        const [f, s1, s2] = two();
        const c1 = s1.coll('test');
        s1.insertText(0, 'ABCD');
        f.processAll();
        const c2 = s2.coll('test');
        c1.add(1, 3, SLIDE);
        f.processAll();
        s1.insertText(2, 'X');
        eq(s1.getText(), 'ABXCD', 'text');
        assertIntervals(s1, c1, [[1, 4]]);
        s2.removeRange(1, 2);
        assertIntervals(s2, c2, [[1, 2]]);
        f.processAll();
        eq(s1.getText(), 'AXCD', 'text');
        assertIntervals(s1, c1, [[1, 3]]);
        assertIntervals(s2, c2, [[1, 3]]);
    },
    slide_on_create_ack() {  // :432-472
        const f = new Factory();
        const s1 = f.runtime('1'), s2 = f.runtime('2'), s3 = f.runtime('3');
        const c1 = s1.coll('test');
        s1.insertText(0, 'ABCD');
        f.processAll();
        const c2 = s2.coll('test'), c3 = s3.coll('test');
        s1.removeRange(1, 2);
        s2.insertText(2, 'X');
        c3.add(1, 3, SLIDE);
        f.processAll();
        for (const [s, c] of [[s1, c1], [s2, c2], [s3, c3]]) { eq(s.getText(), 'AXCD', 'text'); assertIntervals(s, c, [[1, 3]]); }
    },
    double_delete_backward() {  // :182-189
        const [f, s1, s2] = two();
        s1.insertText(0, '01234');
        const c = s1.coll('test'), c2 = s2.coll('test');
        f.processAll();
        s2.removeRange(2, 3);
        c.add(2, 2, SLIDE);
        s1.removeRange(2, 5);
        f.processAll();
        assertIntervals(s1, c, [[1, 1]]);
        assertIntervals(s2, c2, [[1, 1]]);
    },
    slide_intervals_nearer() {  // :235-293
        const [f, s1, s2] = two();
        const c1 = s1.coll('test');
        s1.insertText(0, 'ABCD');
        f.processAll();
        const c2 = s2.coll('test');
        c1.add(1, 3, SLIDE);
        s2.removeRange(3, 4);
        f.processAll();
        assertIntervals(s1, c1, [[1, 2]]);
        s1.removeRange(2, 3);
        assertIntervals(s1, c1, [[1, 2]]);
        f.processAll();
        assertIntervals(s1, c1, [[1, 1]]);
        s1.removeRange(1, 2);
        assertIntervals(s1, c1, [[1, 1]], false);
        f.processAll();
        assertIntervals(s1, c1, [[0, 0]]);
        s1.removeRange(0, 1);
        f.processAll();
        assertIntervals(s1, c1, [[-1, -1]], false);
        assertIntervals(s2, c2, [[-1, -1]], false);
    },
    coherency_end_comparison() {  // :829-854
        const [f, s1] = two();
        s1.insertText(0, 'ABCDEFG');
        const c = s1.coll('test');
        c.add(1, 6, SLIDE);
        c.add(2, 5, SLIDE);
        const largest = c.add(3, 4, SLIDE);
        s1.removeRange(1, 4);
        assertIntervals(s1, c, [[1, 3], [1, 2], [1, 1]]);
        c.removeIntervalById(largest.id());
        assertIntervals(s1, c, [[1, 3], [1, 2]]);
        f.processAll();
        assertIntervals(s1, c, [[1, 2], [1, 3]]);
    },
    pending_property_sets() {  // :1111-1127
        const [f, s1, s2] = two();
        s1.insertText(0, 'ABC');
        const c1 = s1.coll('test'), c2 = s2.coll('test');
        const iv = c1.add(0, 0, SLIDE);
        f.processAll();
        const id = iv.id();
        c1.change(id, 1, 1);
        c1.changeProperties(id, { propName: 'losing value' });
        c2.changeProperties(id, { propName: 'winning value' });
        f.processAll();
        eq(c1.getIntervalById(id).props.propName, 'winning value', 'c1 prop');
        eq(c2.getIntervalById(id).props.propName, 'winning value', 'c2 prop');
    },
    reconnect_add_with_concurrent_insert() {  // :1178-1190
        const [f, s1, s2] = two();
        s1.insertText(0, 'hello friend');
        const c1 = s1.coll('test');
        f.processAll();
        const c2 = s2.coll('test');
        f.processAll();
        c1.add(6, 8, SLIDE);
        s1.connected = false;
        s2.insertText(7, 'amily its my f');
        f.processAll();
        s1.connected = true;
        f.processAll();
        eq(s2.getText(), 'hello family its my friend', 'text');
        assertIntervals(s2, c2, [[6, 22]]);
        assertIntervals(s1, c1, [[6, 22]]);
    },
    reconnect_change_with_concurrent_delete() {  // :1374-1390
        const [f, s1, s2] = two();
        s1.insertText(0, 'hello friend');
        const c1 = s1.coll('test');
        f.processAll();
        const c2 = s2.coll('test');
        f.processAll();
        const iv = c1.add(6, 8, SLIDE);
        f.processAll();
        s1.connected = false;
        c1.change(iv.id(), 5, 9);
        s2.removeRange(8, 10);
        f.processAll();
        s1.connected = true;
        f.processAll();
        eq(s2.getText(), 'hello frnd', 'text');
        assertIntervals(s2, c2, [[5, 8]]);
        assertIntervals(s1, c1, [[5, 8]]);
    },
    reconnect_add_and_string_ops() {  // :1192-1208
        const [f, s1, s2] = two();
        s1.insertText(0, 'hello friend');
        const c1 = s1.coll('test');
        f.processAll();
        const c2 = s2.coll('test');
        f.processAll();
        c1.add(6, 8, SLIDE);
        s1.connected = false;
        s2.insertText(7, 'amily its my f');
        s1.removeRange(0, 5);
        s1.insertText(0, 'hi');
        f.processAll();
        s1.connected = true;
        f.processAll();
        eq(s2.getText(), 'hi family its my friend', 'text');
        assertIntervals(s2, c2, [[3, 19]]);
        assertIntervals(s1, c1, [[3, 19]]);
    },
};

const out = {};
for (const [name, fn] of Object.entries(cases)) {
    try { fn(); out[name] = 'ok'; } catch (e) { out[name] = String(e && e.stack ? e.stack : e); }
}
process.stdout.write(JSON.stringify(out) + '\n');
