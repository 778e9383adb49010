// mtr_oracle.cpp -- CPU oracle: scalar restatement of the merge-tree observer path.
//
// TEST INFRASTRUCTURE ONLY (see mtr_oracle.h).  Every function below names the
// reference file:line it restates; paths are relative to
// packages/dds/merge-tree/src/ of the reference unless stated otherwise.
//
// Differences from the reference that are deliberate and behaviour-neutral:
//  * Block lengths seen by a remote (refSeq, clientId) view are the sum of the
//    leaves' nodeLength (undefined counted as 0) instead of
//    PartialSequenceLengths.getPartialLength (partialLengths.ts:698).  psl.h
//    restates PartialSequenceLengths and, with oracle_set_psl_check on, the oracle
//    maintains it at the reference's call sites and compares the two at every
//    query (tests/test_partial_lengths.py: all golden logs and seeded sets agree;
//    the one modelled quirk, a leaf-level root's stale own length, is documented
//    at Tree::pslCheck).
//  * Ordinals, tiles/range stacks, attribution and maintenance events are not
//    modelled: none of them change the observer's text, segment boundaries or
//    summary bytes.  Local references (localReference.ts) are restated with their
//    per-offset lists, since they are what localReferencePositionToPosition reads.
#include "mtr_oracle.h"
#include "../include/mtr_synth.h"
#include "../include/mtr_digest.h"

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <unordered_map>
#include <memory>
#include <mutex>
#include <string>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

namespace {

constexpr int kMaxNodesInBlock = 8;          // mergeTreeNodes.ts:330
constexpr int kTextSegmentGranularity = 256; // textSegment.ts:35
constexpr int kZamboniSegmentsMax = 2;       // zamboni.ts:14
constexpr int kUniversalSeq = 0;             // constants.ts:11
constexpr int kUnassignedSeq = -1;           // constants.ts:12
constexpr int kTreeMaintenanceSeq = -2;      // constants.ts:13
constexpr int kLocalClientId = -1;           // constants.ts:14
constexpr int kNonCollabClient = -2;         // constants.ts:15
constexpr int kUndef = -1;                   // "undefined" node length
constexpr int64_t kMaxSafe = 9007199254740991LL;
int g_trace = 0;
int g_trace_seq = -1;
// PartialSequenceLengths (psl.h): 0 off; 1 maintained and cross-checked against leaf sums (tests);
// 2 maintained and answering every remote block length, as the reference does (bench.py's CPU baseline)
int g_psl = 0;
std::atomic<long long> g_psl_checks{0}, g_psl_mismatch{0}, g_psl_rootlag{0};
std::mutex g_psl_mu;
std::string g_psl_first;
#define OTRACE(...)                          \
    do {                                     \
        if (g_trace) printf(__VA_ARGS__);    \
    } while (0)

struct Block;

struct PropMap {
    std::vector<std::pair<uint32_t, uint32_t>> kv;  // (key id, value id) in JS own-key order
};

struct Node {
    Block* parent = nullptr;
    int index = 0;
    bool leaf = true;
};

struct Seg : Node {
    bool marker = false;
    bool perm = false;                      // PermutationSegment (matrix/src/permutationvector.ts:41)
    int start = MTR_HANDLE_UNALLOCATED;     // PermutationSegment._start
    bool noRef = false;
    int refType = 0;
    std::u16string text;
    int len = 0;                     // cachedLength
    int seq = kUniversalSeq;         // BaseSegment.seq  mergeTreeNodes.ts:368
    int clientId = kLocalClientId;   // BaseSegment.clientId
    bool removed = false;
    int removedSeq = 0;
    std::vector<int> removedClientIds;
    bool hasProps = false;           // properties !== undefined
    bool hasPropMgr = false;         // propertyManager !== undefined
    PropMap props;
    uint32_t markerOrdinal = 0;      // host marker ordinal + 1 of a Marker with a truthy markerId (0 = none)
    // the local-op path: segmentGroups (segmentGroupCollection.ts), in enqueue order, and
    // PropertiesManager.pendingKeyUpdateCount (segmentPropertiesManager.ts:25): key id -> count > 0
    std::deque<struct SegGroup*> groups;
    std::vector<std::pair<uint32_t, int>> pendingKeys;
    int pendingRewrite = 0;  // PropertiesManager.pendingRewriteCount (segmentPropertiesManager.ts:26)
    // BaseSegment.localSeq / localRemovedSeq (mergeTreeNodes.ts:382-383): the local op that inserted /
    // removed it while unacked (-1 = undefined); cleared by the ack (:460, 469)
    int localSeq = -1;
    int localRemovedSeq = -1;
    struct LocalRefs* localRefs = nullptr;  // BaseSegment.localRefs (mergeTreeNodes.ts:380)
    // BaseSegment.trackingCollection (mergeTreeNodes.ts:373; mergeTreeTracking.ts:62-112): the TrackingGroups
    // holding the segment, and the id the engine's records and reports name it by (-1: never tracked)
    std::vector<struct TGroup*> tgroups;
    int tid = -1;
};

// TrackingGroup (mergeTreeTracking.ts:12-60): its segments in link order (split-off halves appended); one per
// group bit of a vector (the host maps the SharedMatrix undo provider's groups to bits)
struct TGroup {
    std::vector<Seg*> segs;
};

// LocalReferenceCollection (localReference.ts:142-571): per offset of its segment the before / at / after
// lists of reference ids (IRefsAtOffset, :129-133; an absent entry or list is a null pointer / has = false)
struct RefsAtOffset {
    std::list<int> lst[3];  // 0 before, 1 at, 2 after
    bool has[3] = {false, false, false};
};
struct LocalRefs {
    Seg* segment = nullptr;
    std::vector<std::unique_ptr<RefsAtOffset>> byOffset;  // refsByOffset (its length tracks cachedLength)
    int refCount = 0;
};
// LocalReference (localReference.ts:54-121): its ReferenceType, the segment and offset it is linked to, and
// the list of that offset holding it (its listNode; -1 = undefined)
struct LRef {
    int refType = 0;
    Seg* segment = nullptr;
    int offset = 0;
    int list = -1;
};

// SegmentGroup (mergeTreeNodes.ts:57-62): the segments one pending local op touched, in the order they
// joined it (walk order, then split-off halves as splitAt copies them, segmentGroupCollection.ts:47-62)
struct SegGroup {
    std::vector<Seg*> segments;
    int localSeq = 0;
    // a local annotate's previousProps (mergeTree.ts:1330-1351): each member's properties before the op
    // (the deltas of the op's keys derive from them), parallel to `segments`
    bool hasPrevious = false;
    std::vector<std::pair<bool, PropMap>> previousProps;
};

struct PSL;
struct Block : Node {
    int childCount = 0;
    Node* children[kMaxNodesInBlock] = {};
    int needsScour = -1;  // -1 undefined, 0 false, 1 true
    std::shared_ptr<PSL> pl;  // partialLengths (maintained only with the psl.h cross-check on)
    Block() { leaf = false; }
};

struct LRUEntry {
    Seg* segment;
    int maxSeq;
};

// Binary heap with the exact sift rules of collections/heap.ts:11-67
struct Heap {
    std::vector<LRUEntry> L{{nullptr, -2}};  // L[0] = comp.min (mergeTree.ts:112-115)
    int count() const { return int(L.size()) - 1; }
    const LRUEntry* peek() const { return count() > 0 ? &L[1] : nullptr; }
    LRUEntry get() {
        LRUEntry x = L[1];
        L[1] = L[count()];
        L.pop_back();
        fixDown(1);
        return x;
    }
    void add(LRUEntry x) {
        L.push_back(x);
        fixup(count());
    }
    static int cmp(const LRUEntry& a, const LRUEntry& b) { return a.maxSeq - b.maxSeq; }
    void fixup(int k) {
        while (k > 1 && cmp(L[k >> 1], L[k]) > 0) {
            std::swap(L[k >> 1], L[k]);
            k >>= 1;
        }
    }
    void fixDown(int k) {
        while ((k << 1) <= count()) {
            int j = k << 1;
            if (j < count() && cmp(L[j], L[j + 1]) > 0) j++;
            if (cmp(L[k], L[j]) <= 0) break;
            std::swap(L[k], L[j]);
            k = j;
        }
    }
};

#include "psl.h"

struct Tables {
    const mtr_batch* b = nullptr;
    bool keyIsIndex(uint32_t k) const { return b->key_index[k] != MTR_NOT_INDEX; }
    uint32_t keyIndex(uint32_t k) const { return b->key_index[k]; }
};

// JS own-key insertion: integer-like keys first in ascending order, others in insertion order.
void propSet(PropMap& m, uint32_t key, uint32_t val, const Tables& t) {
    for (auto& kv : m.kv)
        if (kv.first == key) {
            kv.second = val;
            return;
        }
    if (t.keyIsIndex(key)) {
        uint32_t ix = t.keyIndex(key);
        size_t pos = 0;
        while (pos < m.kv.size() && t.keyIsIndex(m.kv[pos].first) && t.keyIndex(m.kv[pos].first) < ix) pos++;
        m.kv.insert(m.kv.begin() + pos, {key, val});
    } else {
        m.kv.push_back({key, val});
    }
}

void propDelete(PropMap& m, uint32_t key) {
    for (size_t i = 0; i < m.kv.size(); i++)
        if (m.kv[i].first == key) {
            m.kv.erase(m.kv.begin() + i);
            return;
        }
}

// matchProperties (properties.ts:71-105) with values compared by equivalence class.
bool matchProperties(const Seg* a, const Seg* b, const mtr_batch* bt) {
    if (a->hasProps) {
        if (!b->hasProps) return false;
        if (a->props.kv.size() != b->props.kv.size()) return false;
        for (auto& ka : a->props.kv) {
            bool found = false;
            for (auto& kb : b->props.kv)
                if (kb.first == ka.first) {
                    // never-equal values (NaN, {value: undefined, seq}) fail `b[key] !== a[key]` / the
                    // recursive b[key] === undefined test even against themselves
                    if (bt->val_eq[kb.second] != bt->val_eq[ka.second] || (bt->val_eq[ka.second] & MTR_VEQ_NEVER))
                        return false;
                    found = true;
                    break;
                }
            if (!found) return false;
        }
        return true;
    }
    return !b->hasProps;
}

struct OpCtx {
    int refSeq;
    int clientId;
    int seq;
};

class Tree {
  public:
    explicit Tree(const mtr_options& o) : opt(o) { root = makeBlock(); }

    mtr_options opt;
    Block* root;
    // LocalReferencePosition.callbacks (localReference.ts:43-46): the interval collection's beforeSlide /
    // afterSlide listeners (sequence/src/intervalCollection.ts:1114-1159), one hook for every reference
    oracle_slide_hook slideHook = nullptr;
    void* slideCtx = nullptr;
    void slideEvent(int id, int phase) {
        if (slideHook) slideHook(slideCtx, id, phase);
    }
    // CollaborationWindow (mergeTreeNodes.ts:656)
    int localClientId = kLocalClientId;
    bool collaborating = false;
    int minSeq = 0;
    int currentSeq = 0;
    Heap heap;
    std::deque<Seg> segPool;
    std::deque<Block> blockPool;
    Tables tabs;
    int status = MTR_OK;
    // pending local ops: collabWindow.localSeq (mergeTreeNodes.ts:656) and MergeTree.pendingSegments
    int localSeqCounter = 0;
    std::deque<SegGroup*> pendingSegments;
    std::deque<SegGroup> groupPool;
    // tracking groups (SharedMatrix undo: matrix/src/undoprovider.ts) by bit, and the next tracking id
    TGroup tgroup[MTR_TRACK_GROUPS];
    int ntid = 0;
    std::vector<int> freeTids;  // tracking ids of segments zamboni unlinked or merged away (the engine's free stack)

    Block* makeBlock() {
        blockPool.emplace_back();
        return &blockPool.back();
    }
    Seg* makeSeg() {
        segPool.emplace_back();
        return &segPool.back();
    }

    static void assignChild(Block* b, Node* child, int index) {  // mergeTreeNodes.ts:355-362
        child->parent = b;
        child->index = index;
        b->children[index] = child;
    }

    // ---------------------------------------------------------------- lengths
    // localNetLength, mergeTree.ts:613-634 (localSeq undefined)
    int localNetLength(const Seg* s) const {
        if (s->removed) {
            if (!opt.new_length_calc) {
                int64_t rs = s->removedSeq == kUnassignedSeq ? kMaxSafe : s->removedSeq;
                if (rs > minSeq) return 0;
                return kUndef;
            }
            return 0;
        }
        return s->len;
    }

    int blockLocalLength(const Block* b) const {  // cachedLength via blockUpdate, mergeTree.ts:2387
        int len = 0;
        for (int i = 0; i < b->childCount; i++) {
            const Node* c = b->children[i];
            int l = c->leaf ? localNetLength(static_cast<const Seg*>(c)) : blockLocalLength(static_cast<const Block*>(c));
            if (l > 0) len += l;
        }
        return len;
    }

    // Remote leaf visibility, mergeTree.ts:928-1003
    int leafRemoteLength(const Seg* s, int refSeq, int clientId) const {
        bool isRemoved = s->removed;
        if (opt.new_length_calc) {  // mergeTree.ts:935-965
            int64_t seq = s->seq == kUnassignedSeq ? kMaxSafe - 1 : s->seq;
            if (isRemoved) {
                int64_t rs = s->removedSeq == kUnassignedSeq ? kMaxSafe : s->removedSeq;
                if (rs <= minSeq) return kUndef;
                if (rs <= refSeq || std::find(s->removedClientIds.begin(), s->removedClientIds.end(), clientId) !=
                                        s->removedClientIds.end())
                    return 0;
            }
            return (seq <= refSeq || s->clientId == clientId) ? s->len : 0;
        }
        if (isRemoved && s->removedSeq != kUnassignedSeq && s->removedSeq <= refSeq) return kUndef;  // :967-976
        if (s->clientId == clientId || (s->seq != kUnassignedSeq && s->seq <= refSeq)) {            // :977-988
            if (isRemoved) {
                return std::find(s->removedClientIds.begin(), s->removedClientIds.end(), clientId) !=
                               s->removedClientIds.end()
                           ? 0
                           : s->len;
            }
            return s->len;
        }
        if (isRemoved && s->removedSeq != kUnassignedSeq) return kUndef;  // :993-998
        return 0;
    }

    int blockRemoteLength(const Block* b, int refSeq, int clientId) const {
        int len = 0;
        for (int i = 0; i < b->childCount; i++) {
            const Node* c = b->children[i];
            int l = c->leaf ? leafRemoteLength(static_cast<const Seg*>(c), refSeq, clientId)
                            : blockRemoteLength(static_cast<const Block*>(c), refSeq, clientId);
            if (l > 0) len += l;
        }
        return len;
    }

    // nodeLength, mergeTree.ts:916-1004 (localSeq undefined)
    int nodeLength(const Node* n, int refSeq, int clientId) const {
        if (!collaborating || localClientId == clientId) {
            if (n->leaf) return localNetLength(static_cast<const Seg*>(n));
            return blockLocalLength(static_cast<const Block*>(n));
        }
        if (!n->leaf) {
            const Block* b = static_cast<const Block*>(n);
            // the reference's answer, partialLengths.getPartialLength (mergeTree.ts:928-931): O(log W) per
            // block instead of the leaf sum (a leaf-level root keeps the leaf sum: its own partial length
            // can read stale-high, see pslCheck; it has at most 7 leaves)
            if (pslAnswer && b->pl && !(b == root && b->childCount > 0 && b->children[0]->leaf))
                return int(b->pl->getPartialLength(refSeq, clientId));
            const int l = blockRemoteLength(b, refSeq, clientId);
            if (pslOn && !pslAnswer) pslCheck(b, refSeq, clientId, l);
            return l;
        }
        return leafRemoteLength(static_cast<const Seg*>(n), refSeq, clientId);
    }

    // ---------------------------------------------------------------- PartialSequenceLengths (psl.h)
    // The reference's block length at a remote view is partialLengths.getPartialLength
    // (mergeTree.ts:928-931); the oracle's is the sum of its leaves.  With the cross-check on, every
    // block keeps its PartialSequenceLengths, updated where mergeTree.ts / zamboni.ts update it, and
    // every remote block-length query compares the two (test/testUtils.ts:209-248).
    bool pslOn = g_psl != 0;
    bool pslAnswer = g_psl == 2;
    //
    // One reference quirk is modelled, not flagged: a root whose children are leaves never receives
    // markRangeRemoved's post-order update (depthFirstNodeWalk's first block result is undefined,
    // mergeTreeNodeWalk.ts:98-105), so its partialLengths miss removes until the next combine and
    // read high.  The reference reads a root's own partial length only as nodeMap's default end
    // (legacy extractSync's mapRange, where a high end changes nothing: the walk ends with the leaves)
    // and in getLength; such queries pass when partial length >= leaf sum (counted in rootlag).
    void pslCheck(const Block* b, int refSeq, int clientId, int leafSum) const {
        g_psl_checks++;
        const bool have = b->pl != nullptr;
        const int64_t v = have ? b->pl->getPartialLength(refSeq, clientId) : -1;
        const bool leafRoot = b == root && b->childCount > 0 && b->children[0]->leaf;
        if (have && leafRoot && v > int64_t(leafSum)) {
            g_psl_rootlag++;
            return;
        }
        if (!have || v != int64_t(leafSum)) {
            if (g_psl_mismatch++ == 0) {
                std::lock_guard<std::mutex> g(g_psl_mu);
                char buf[256];
                snprintf(buf, sizeof buf, "op seq %d: %s of %d children at (refSeq %d, client %d): partial length %lld, "
                         "leaf sum %d%s", curOpSeq, b == root ? "root" : "block", b->childCount, refSeq, clientId,
                         (long long)v, leafSum, have ? "" : " (no partialLengths)");
                g_psl_first = buf;
            }
        }
    }
    // nodeUpdateLengthNewStructure, mergeTree.ts:2183-2189
    void nodeUpdateLengthNewStructure(Block* b, bool recur = false) {
        if (pslOn && collaborating) b->pl = pslCombine(b, minSeq, recur);
    }
    // blockUpdateLength, mergeTree.ts:2431-2449 (MergeTree.options.incrementalUpdate = true)
    void blockUpdateLength(Block* b, int seq, int clientId) {
        if (!pslOn || !collaborating || seq == kUnassignedSeq || seq == kTreeMaintenanceSeq) return;
        if (b->pl && clientId != kNonCollabClient) pslUpdate(*b->pl, b, seq, clientId, minSeq);
        else b->pl = pslCombine(b, minSeq, false);
    }
    // blockUpdatePathLengths(block, UnassignedSequenceNumber, -1, newStructure = true), mergeTree.ts:2414-2429
    void blockUpdatePathLengthsNew(Block* b) {
        for (; b; b = b->parent) nodeUpdateLengthNewStructure(b);
    }

    // ------------------------------------------------------------ segments
    // TextSegment.canAppend, textSegment.ts:86-93; Marker.canAppend -> false;
    // PermutationSegment.canAppend, permutationvector.ts:131-137 (handle ranges stay contiguous)
    static bool canAppend(const Seg* a, const Seg* b) {
        if (a->perm)
            return a->start == MTR_HANDLE_UNALLOCATED ? b->start == MTR_HANDLE_UNALLOCATED
                                                      : int64_t(b->start) == int64_t(a->start) + a->len;
        if (a->marker || b->marker) return false;
        if (!a->text.empty() && a->text.back() == u'\n') return false;
        return a->len <= kTextSegmentGranularity || b->len <= kTextSegmentGranularity;
    }

    // BaseSegment.splitAt + TextSegment.createSplitSegmentAt, mergeTreeNodes.ts:481-510, textSegment.ts:121-129
    Seg* splitAt(Seg* s, int pos) {
        if (pos <= 0 || s->marker) return nullptr;
        Seg* r = makeSeg();
        if (s->perm) {  // PermutationSegment.createSplitSegmentAt, permutationvector.ts:139-154
            r->perm = true;
            r->start = s->start == MTR_HANDLE_UNALLOCATED ? MTR_HANDLE_UNALLOCATED : s->start + pos;
            r->len = s->len - pos;
            s->len = pos;
        } else {
            r->text = s->text.substr(pos);
            s->text.resize(pos);
            s->len = int(s->text.size());
            r->len = int(r->text.size());
        }
        if (s->hasPropMgr && s->hasProps) {  // copyPropertiesTo, mergeTreeNodes.ts:512-522
            r->hasPropMgr = true;
            r->hasProps = true;
            r->props = s->props;
            r->pendingKeys = s->pendingKeys;  // PropertiesManager.copyTo, segmentPropertiesManager.ts:160-184
            r->pendingRewrite = s->pendingRewrite;
        }
        r->parent = s->parent;
        r->removedClientIds = s->removedClientIds;
        r->removed = s->removed;
        r->removedSeq = s->removedSeq;
        r->seq = s->seq;
        r->clientId = s->clientId;
        r->localSeq = s->localSeq;  // mergeTreeNodes.ts:495-497
        r->localRemovedSeq = s->localRemovedSeq;
        if (s->localRefs) refsSplit(s->localRefs, pos, r);  // mergeTreeNodes.ts:501-503
        if (!s->tgroups.empty()) {  // trackingCollection.copyTo (mergeTreeNodes.ts:500; mergeTreeTracking.ts:86-92)
            r->tid = newTid();
            for (TGroup* g : s->tgroups) tlink(g, r);
            if (recycleLog) deltas.push_back({curOpIndex, s->tid, r->tid, MTR_DELTA_TSPLIT});
        }
        for (SegGroup* g : s->groups) {  // segmentGroups.copyTo -> enqueueOnCopy (segmentGroupCollection.ts:47-62)
            if (g->hasPrevious)  // previousProps of the source segment, duplicated for the copy
                for (size_t k = 0; k < g->segments.size(); k++)
                    if (g->segments[k] == s) {
                        g->previousProps.push_back(g->previousProps[k]);
                        break;
                    }
            r->groups.push_back(g);
            g->segments.push_back(r);
        }
        return r;
    }

    // ------------------------------------------------------------ tracking groups (mergeTreeTracking.ts)
    static void tlink(TGroup* g, Seg* s) {  // TrackingGroup.link (:41-46): once per segment
        if (std::find(g->segs.begin(), g->segs.end(), s) != g->segs.end()) return;
        g->segs.push_back(s);
        s->tgroups.push_back(g);
    }
    static void tunlink(TGroup* g, Seg* s) {  // TrackingGroup.unlink (:47-53)
        auto it = std::find(g->segs.begin(), g->segs.end(), s);
        if (it == g->segs.end()) return;
        g->segs.erase(it);
        s->tgroups.erase(std::find(s->tgroups.begin(), s->tgroups.end(), g));
    }
    // TrackingGroupCollection.matches (:98-110): the same groups
    static bool sameGroups(const Seg* a, const Seg* b) {
        if (a->tgroups.size() != b->tgroups.size()) return false;
        for (TGroup* g : a->tgroups)
            if (std::find(b->tgroups.begin(), b->tgroups.end(), g) == b->tgroups.end()) return false;
        return true;
    }
    uint32_t tbits(const Seg* s) const {
        uint32_t b = 0;
        for (TGroup* g : s->tgroups) b |= 1u << int(g - tgroup);
        return b;
    }
    // VectorUndoProvider.record (undoprovider.ts:30-85): an op's delta segment joins the groups of `bits`
    // tracking ids are an engine artifact the reports and leaf lists carry (include/mtr_types.h "Tracking groups"):
    // the one freed last is reused first, as the engine's free stack does (Eng::tid_new / tid_free)
    int newTid() {
        if (freeTids.empty()) return ntid++;
        const int t = freeTids.back();
        freeTids.pop_back();
        return t;
    }
    void trackLink(Seg* s, uint32_t bits) {
        if (s->tid < 0) s->tid = newTid();
        for (int b = 0; b < MTR_TRACK_GROUPS; b++)
            if (bits >> b & 1u) tlink(&tgroup[b], s);
        if (recycleLog) deltas.push_back({curOpIndex, s->tid, s->len, MTR_DELTA_TLINK});
    }
    Seg* findTid(int t) {
        std::vector<Seg*> lv;
        leaves(root, lv);
        for (Seg* x : lv)
            if (x->tid == t) return x;
        return nullptr;
    }
    // MergeTree.insertChildNode (mergeTree.ts:1582-1592)
    static void insertChildNode(Block* b, Node* child, int idx) {
        for (int i = b->childCount; i > idx; i--) {
            b->children[i] = b->children[i - 1];
            b->children[i]->index = i;
        }
        b->childCount++;
        assignChild(b, child, idx);
    }
    // MergeTree.insertAtReferencePosition (mergeTree.ts:1429-1538) at offset 0 of `ref`, for a local segment:
    // in front of the run of zero-length segments that ends at ref (breakTie against UnassignedSequenceNumber,
    // segments zamboni may drop skipped), then rebalanceTree
    void insertAtReferencePosition(Seg* ref, Seg* seg) {
        if (seg->len == 0) return;
        std::vector<Seg*> lv;
        leaves(root, lv);
        int k = int(std::find(lv.begin(), lv.end(), ref) - lv.begin());
        Seg* start = ref;
        for (int j = k - 1; j >= 0; j--) {  // backwardExcursion (:1491-1508)
            const int bl = nodeLength(lv[size_t(j)], currentSeq, localClientId);
            if (bl == kUndef) continue;
            if (bl == 0) {
                if (breakTie(0, lv[size_t(j)], kUnassignedSeq)) start = lv[size_t(j)];
                continue;
            }
            break;
        }
        if (collaborating) {
            seg->localSeq = ++localSeqCounter;
            seg->seq = kUnassignedSeq;
        } else {
            seg->seq = kUniversalSeq;
        }
        seg->clientId = localClientId;
        insertChildNode(start->parent, seg, start->index);
        for (Block* block = seg->parent; block; block = block->parent) {  // rebalanceTree (:1445-1475)
            if (block->childCount >= kMaxNodesInBlock) {
                Block* sn = split(block);
                if (block == root) updateRoot(sn);
                else insertChildNode(block->parent, sn, block->index + 1);
            } else {
                blockUpdateLength(block, kUnassignedSeq, localClientId);
            }
        }
        recordDeltas({seg}, MTR_OP_INSERT);  // mergeTreeDeltaCallback (:1530-1533)
        if (collaborating) addToPendingList(seg, nullptr, seg->localSeq);  // (:1535-1537)
    }
    // PermutationSegment.transferToReplacement (permutationvector.ts:80-102)
    static void transferToReplacement(Seg* from, Seg* to) {
        const std::vector<TGroup*> gs = from->tgroups;
        for (TGroup* g : gs) tlink(g, to);
        for (TGroup* g : gs) tunlink(g, from);
        to->start = from->start;
        from->start = MTR_HANDLE_UNALLOCATED;
    }

    // addToPendingList, mergeTree.ts:1324-1357 (previousProps are kept only for rollback: not modelled)
    SegGroup* addToPendingList(Seg* s, SegGroup* g, int localSeq) {
        if (!g) {
            groupPool.emplace_back();
            g = &groupPool.back();
            g->localSeq = localSeq;
            pendingSegments.push_back(g);
        }
        s->groups.push_back(g);  // segment.segmentGroups.enqueue (segmentGroupCollection.ts:24-27)
        g->segments.push_back(s);
        return g;
    }

    static int* pendingCount(Seg* s, uint32_t key) {
        for (auto& kc : s->pendingKeys)
            if (kc.first == key) return &kc.second;
        return nullptr;
    }

    // findRollbackPosition (mergeTree.ts:2164-2181): the cachedLengths of the segments ahead that are not
    // removed (a pending local remove counts as removed)
    int findRollbackPosition(Seg* seg) {
        std::vector<Seg*> lv;
        leaves(root, lv);
        int pos = 0;
        for (Seg* x : lv) {
            if (x == seg) break;
            if (!x->removed) pos += x->len;
        }
        return pos;
    }

    // MergeTree.rollback (mergeTree.ts:2049-2159): revert the newest pending local op (type = its
    // MergeTreeDeltaType; propop = its props for an annotate)
    void rollback(int type, uint32_t propop, uint32_t comb = 0) {
        if (pendingSegments.empty()) {
            status = MTR_ERR_BAD_OP;  // "Rollback op doesn't match last edit"
            return;
        }
        SegGroup* g = pendingSegments.back();
        if (type == MTR_OP_ANNOTATE && !g->hasPrevious) {
            status = MTR_ERR_BAD_OP;
            return;
        }
        pendingSegments.pop_back();
        for (size_t k = 0; k < g->segments.size(); k++) {
            Seg* s = g->segments[k];
            if (s->groups.empty() || s->groups.back() != g) {  // segmentGroups.pop()
                status = MTR_ERR_ASSERT | (type == MTR_OP_REMOVE ? 0x3ee : 0x3ef);
                return;
            }
            s->groups.pop_back();
            if (type == MTR_OP_REMOVE) {
                if (!s->removed || s->removedClientIds.empty() || s->removedClientIds[0] != localClientId) {
                    status = MTR_ERR_ASSERT | 0x39d;
                    return;
                }
                s->removed = false;
                s->removedSeq = 0;
                s->removedClientIds.clear();
                s->localRemovedSeq = -1;
            } else if (type == MTR_OP_INSERT) {
                const int start = findRollbackPosition(s);
                s->seq = kUniversalSeq;
                s->localSeq = -1;
                markRangeRemoved(start, start + s->len, kUniversalSeq, localClientId, kUniversalSeq);
            } else if (type == MTR_OP_ANNOTATE) {
                // annotateRange(start, start + cachedLength, previousProps[k], ..., UniversalSequenceNumber,
                // PropertiesRollback.Rollback): the walk at the segment's own local-view range reaches only
                // it; addProperties then drops the op keys' pending counts and restores their values
                const mtr_batch* b = tabs.b;
                const auto& prev = g->previousProps[k];
                s->hasPropMgr = true;
                s->hasProps = true;
                if ((comb & 7u) == MTR_COMB_REWRITE) {  // PropertiesRollback.Rewrite
                    rollbackRewrite(s, propop, prev);
                    continue;
                }
                for (uint32_t q = b->propop_off[propop]; q < b->propop_off[propop + 1]; q++) {
                    const uint32_t key = b->propop_kv[2 * q];
                    if (int* c = pendingCount(s, key)) {  // decrementPendingCounts (:37-58)
                        if (--*c == 0)
                            for (size_t j = 0; j < s->pendingKeys.size(); j++)
                                if (s->pendingKeys[j].first == key) {
                                    s->pendingKeys.erase(s->pendingKeys.begin() + j);
                                    break;
                                }
                    }
                    const std::pair<uint32_t, uint32_t>* pv = nullptr;
                    if (prev.first)
                        for (auto& kv : prev.second.kv)
                            if (kv.first == key) pv = &kv;
                    if (pv) propSet(s->props, key, pv->second, tabs);
                    else propDelete(s->props, key);
                }
            } else {
                status = MTR_ERR_BAD_OP;
                return;
            }
        }
    }

    // The rollback of a local rewrite annotate on segment s (mergeTree.ts:2129-2152 with
    // PropertiesRollback.Rewrite): decrementPendingCounts(true, oldProps) runs over the segment's *current*
    // keys (segmentPropertiesManager.ts:84-89), then the op's deltas -- the previousProps addProperties
    // returned (:106-147): the old keys the rewrite deleted (old values, old order), then its non-null keys
    // (old value, or null) -- are applied as a plain annotate: null deletes, a value sets (appended when new)
    void rollbackRewrite(Seg* s, uint32_t propop, const std::pair<bool, PropMap>& prev) {
        const mtr_batch* b = tabs.b;
        const uint32_t lo = b->propop_off[propop], hi = b->propop_off[propop + 1];
        s->pendingRewrite--;
        for (auto& kv : std::vector<std::pair<uint32_t, uint32_t>>(s->props.kv))
            if (int* c = pendingCount(s, kv.first))
                if (--*c == 0)
                    for (size_t j = 0; j < s->pendingKeys.size(); j++)
                        if (s->pendingKeys[j].first == kv.first) {
                            s->pendingKeys.erase(s->pendingKeys.begin() + j);
                            break;
                        }
        const PropMap old = prev.first ? prev.second : PropMap{};
        auto oldVal = [&](uint32_t key) -> uint32_t {
            for (auto& kv : old.kv)
                if (kv.first == key) return kv.second;
            return MTR_NULL_VALUE;
        };
        std::vector<std::pair<uint32_t, uint32_t>> deltas;
        auto put = [&](uint32_t key, uint32_t v) {
            for (auto& d : deltas)
                if (d.first == key) {
                    d.second = v;
                    return;
                }
            deltas.push_back({key, v});
        };
        for (auto& kv : old.kv) {  // the delete pass: old keys whose new value is absent or falsy
            bool truthy = false;
            for (uint32_t i = lo; i < hi; i++)
                if (b->propop_kv[2 * i] == kv.first) {
                    const uint32_t v = b->propop_kv[2 * i + 1];
                    truthy = v != MTR_NULL_VALUE && !(b->val_eq[v] & MTR_VEQ_FALSY);
                    break;
                }
            if (!truthy) put(kv.first, kv.second);
        }
        for (uint32_t i = lo; i < hi; i++)  // the op's keys (a null one was handled by the delete pass)
            if (b->propop_kv[2 * i + 1] != MTR_NULL_VALUE) put(b->propop_kv[2 * i], oldVal(b->propop_kv[2 * i]));
        for (auto& d : deltas) {
            if (d.second == MTR_NULL_VALUE) propDelete(s->props, d.first);
            else propSet(s->props, d.first, d.second, tabs);
        }
    }

    // MergeTree.ackPendingSegment (mergeTree.ts:1283-1322) for one member op of this client's sequenced
    // message; opType = that member's MergeTreeDeltaType, propop = its props (annotate)
    void ackPendingSegment(int opType, uint32_t propop, int seq, uint32_t comb = 0) {
        if (!pendingSegments.empty()) {
            SegGroup* g = pendingSegments.front();
            pendingSegments.pop_front();
            for (Seg* s : g->segments) {
                // BaseSegment.ack, mergeTreeNodes.ts:439-479
                if (s->groups.empty() || s->groups.front() != g) {
                    status = MTR_ERR_ASSERT | 0x043;  // "On ack, unexpected segmentGroup!"
                    return;
                }
                s->groups.pop_front();
                if (opType == MTR_OP_ANNOTATE) {  // ackPendingProperties -> decrementPendingCounts (:32-58)
                    const mtr_batch* b = tabs.b;
                    const bool rewrite = (comb & 7u) == MTR_COMB_REWRITE;
                    if (rewrite) s->pendingRewrite--;
                    for (uint32_t i = b->propop_off[propop]; i < b->propop_off[propop + 1]; i++) {
                        const uint32_t k = b->propop_kv[2 * i];
                        int* c = pendingCount(s, k);
                        if (!c) continue;
                        if (rewrite && b->propop_kv[2 * i + 1] == MTR_NULL_VALUE) continue;  // not tracked
                        if (*c <= 0) {
                            status = MTR_ERR_ASSERT | 0x05c;
                            return;
                        }
                        if (--*c == 0)
                            for (size_t j = 0; j < s->pendingKeys.size(); j++)
                                if (s->pendingKeys[j].first == k) {
                                    s->pendingKeys.erase(s->pendingKeys.begin() + j);
                                    break;
                                }
                    }
                } else if (opType == MTR_OP_INSERT) {
                    if (s->seq != kUnassignedSeq) {
                        status = MTR_ERR_ASSERT | 0x045;  // "On insert, seq number already assigned!"
                        return;
                    }
                    s->seq = seq;
                    s->localSeq = -1;
                } else if (opType == MTR_OP_REMOVE) {
                    if (!s->removed) {
                        status = MTR_ERR_ASSERT | 0x046;  // "On remove ack, missing removal info!"
                        return;
                    }
                    s->localRemovedSeq = -1;
                    if (s->removedSeq == kUnassignedSeq) {  // ack() is true: no overlapping remove
                        s->removedSeq = seq;
                        slideAckedRemovedSegmentReferences(s);  // mergeTree.ts:1294-1296
                    }
                } else {
                    status = MTR_ERR_BAD_OP;
                    return;
                }
                addToLRUSet(s, seq);  // mergeTree.ts:1299-1301
            }
        }
        zamboniSegments();  // mergeTree.ts:1318-1320
    }

    // ------------------------------------------------------------ local references
    std::vector<LRef> refs;  // every reference by creation (the host's reference ids)
    std::deque<LocalRefs> refPool;
    static constexpr int kSlide = MTR_REFTYPE_SLIDE_ON_REMOVE, kStay = MTR_REFTYPE_STAY_ON_REMOVE,
                         kTransient = MTR_REFTYPE_TRANSIENT;
    LocalRefs* newLocalRefs(Seg* s, size_t len) {  // new LocalReferenceCollection(segment), localReference.ts:172-181
        refPool.emplace_back();
        LocalRefs* c = &refPool.back();
        c->segment = s;
        c->byOffset.resize(len);
        return c;
    }
    RefsAtOffset& refSlot(LocalRefs* c, int offset) {  // refsByOffset[offset] ??= {} (a JS array grows on assignment)
        if (size_t(offset) >= c->byOffset.size()) c->byOffset.resize(size_t(offset) + 1);
        if (!c->byOffset[size_t(offset)]) c->byOffset[size_t(offset)].reset(new RefsAtOffset());
        return *c->byOffset[size_t(offset)];
    }
    // LocalReferenceCollection.has (localReference.ts:357-384)
    bool refsHas(const LocalRefs* c, int id) const {
        const LRef& r = refs[size_t(id)];
        return !(r.refType & kTransient) && r.segment == c->segment && r.list >= 0;
    }
    // removeLocalRef (localReference.ts:304-318)
    void refsRemove(LocalRefs* c, int id) {
        if (!c || !refsHas(c, id)) return;
        LRef& r = refs[size_t(id)];
        refSlot(c, r.offset).lst[r.list].remove(id);
        r.list = -1;
        c->refCount--;
    }
    // the collection's references in iteration order ([Symbol.iterator], localReference.ts:187-221): by offset,
    // then before / at / after
    static std::vector<int> refsOf(const LocalRefs* c) {
        std::vector<int> out;
        for (const auto& slot : c->byOffset)
            if (slot)
                for (int k = 0; k < 3; k++)
                    if (slot->has[k]) out.insert(out.end(), slot->lst[k].begin(), slot->lst[k].end());
        return out;
    }
    // MergeTree.createLocalReferencePosition (mergeTree.ts:2209-2226) -> createLocalRef / addLocalRef
    // (localReference.ts:260-298); a null segment is createDetachedLocalReferencePosition (:123-127)
    // slot >= 0: the id the host recycles (MTR_REF_SLOT, include/mtr_types.h) -- one no collection holds, or the next
    int createRef(Seg* seg, int offset, int refType, int slot = -1) {
        const int excl = !!(refType & kTransient) + !!(refType & kSlide) + !!(refType & kStay);
        if (excl > 1) return MTR_ERR_BAD_OP;  // _validateReferenceType's UsageError (:23-39)
        LRef r;
        r.refType = refType;
        const int id = slot >= 0 ? slot : int(refs.size());
        if (id > int(refs.size())) return MTR_ERR_BAD_OP;
        if (id < int(refs.size())) {
            const LRef& o = refs[size_t(id)];
            if (o.segment && o.segment->localRefs && refsHas(o.segment->localRefs, id)) return MTR_ERR_BAD_OP;
        }
        auto put = [&](const LRef& x) {
            if (id == int(refs.size())) refs.push_back(x);
            else refs[size_t(id)] = x;
        };
        if (!seg) {
            put(r);
            return status;
        }
        if (removedAndAcked(seg) && !(refType & (kSlide | kTransient))) return MTR_ERR_BAD_OP;  // UsageError
        if (!seg->localRefs) seg->localRefs = newLocalRefs(seg, size_t(seg->len));
        r.segment = seg;
        r.offset = offset;
        put(r);
        if (!(refType & kTransient)) {
            if (offset >= seg->len) return MTR_ERR_ASSERT | 0x348;  // "offset cannot be beyond segment length"
            RefsAtOffset& slot = refSlot(seg->localRefs, offset);
            slot.has[1] = true;
            slot.lst[1].push_back(id);
            refs[size_t(id)].list = 1;
            seg->localRefs->refCount++;
        }
        return status;
    }
    // LocalReferenceCollection.split (localReference.ts:398-420): the references at offsets >= pos go to the
    // split-off segment r
    void refsSplit(LocalRefs* c, int pos, Seg* r) {
        if (c->refCount) {
            LocalRefs* rc = newLocalRefs(r, 0);
            for (size_t k = size_t(pos); k < c->byOffset.size(); k++) rc->byOffset.push_back(std::move(c->byOffset[k]));
            if (size_t(pos) < c->byOffset.size()) c->byOffset.resize(size_t(pos));
            r->localRefs = rc;
            for (int id : refsOf(rc)) {
                refs[size_t(id)].segment = r;
                refs[size_t(id)].offset -= pos;
                c->refCount--;
                rc->refCount++;
            }
        } else {
            c->byOffset.resize(size_t(pos));  // refsByOffset.length = offset
        }
    }
    // LocalReferenceCollection.append (static :143-158, instance :332-350): b's references move to a behind
    // a's refsByOffset (called before a's cachedLength grows)
    void refsAppend(Seg* a, Seg* b) {
        if (b->localRefs && b->localRefs->refCount) {
            if (!a->localRefs) a->localRefs = newLocalRefs(a, size_t(a->len));
            LocalRefs* c = a->localRefs;
            LocalRefs* o = b->localRefs;
            if (int(c->byOffset.size()) != a->len) status = MTR_ERR_ASSERT | 0x2be;  // "contains a gap"
            c->refCount += o->refCount;
            o->refCount = 0;
            const int base = int(c->byOffset.size());
            for (int id : refsOf(o)) {
                refs[size_t(id)].segment = a;
                refs[size_t(id)].offset += base;
            }
            for (auto& p : o->byOffset) c->byOffset.push_back(std::move(p));
            o->byOffset.clear();
        } else if (a->localRefs) {
            a->localRefs->byOffset.resize(a->localRefs->byOffset.size() + size_t(b->len));
        }
    }
    // MergeTree._getSlideToSegment (mergeTree.ts:821-840): the first segment after s (forwardExcursion) that is
    // acked and not removed-and-acked, else the last such before it (backwardExcursion), else none
    Seg* getSlideToSegment(Seg* s) {
        if (!s || !removedAndAcked(s)) return s;
        std::vector<Seg*> lv;
        leaves(root, lv);
        const auto it = std::find(lv.begin(), lv.end(), s);
        if (it == lv.end()) return nullptr;  // unlinked: the excursions visit nothing
        auto ok = [](const Seg* x) { return x->seq != kUnassignedSeq && !removedAndAcked(x); };
        for (auto j = it + 1; j != lv.end(); ++j)
            if (ok(*j)) return *j;
        for (auto j = it; j != lv.begin();)
            if (ok(*--j)) return *j;
        return nullptr;
    }
    // MergeTree.slideAckedRemovedSegmentReferences (mergeTree.ts:849-884) with addBeforeTombstones /
    // addAfterTombstones (localReference.ts:426-490)
    void slideAckedRemovedSegmentReferences(Seg* s) {
        if (!s->localRefs || s->localRefs->refCount == 0) return;
        Seg* ns = getSlideToSegment(s);
        const std::vector<int> ids = refsOf(s->localRefs);
        if (!ns) {
            for (int id : ids)
                if (!(refs[size_t(id)].refType & kStay)) {
                    slideEvent(id, 0);  // ref.callbacks?.beforeSlide (mergeTree.ts:866-871)
                    refsRemove(s->localRefs, id);
                    slideEvent(id, 1);
                }
            return;
        }
        if (!ns->localRefs) ns->localRefs = newLocalRefs(ns, size_t(ns->len));
        LocalRefs* c = ns->localRefs;
        const bool after = leafIndex(ns) < leafIndex(s);  // newSegment.ordinal < segment.ordinal
        const int off = after ? ns->len - 1 : 0;
        RefsAtOffset& slot = refSlot(c, off);
        const int k = after ? 2 : 0;
        slot.has[k] = true;
        std::list<int>& dst = slot.lst[k];
        auto at = dst.begin();  // before-tombstones: in order at the front of the `before` list
        for (int id : ids) {
            LRef& r = refs[size_t(id)];
            if (r.refType & kStay) continue;
            if (r.refType & kSlide) slideEvent(id, 0);  // lref.callbacks?.beforeSlide (localReference.ts:441,477)
            refsRemove(r.segment->localRefs, id);  // link() with a new list node leaves the old collection
            if (r.refType & kSlide) {
                if (after) dst.push_back(id);
                else at = std::next(dst.insert(at, id));
                r.segment = ns;
                r.offset = off;
                r.list = k;
                c->refCount++;
                slideEvent(id, 1);  // afterSlide (:451,484)
            } else {
                r.segment = nullptr;  // lref.link(undefined, 0, undefined)
                r.offset = 0;
            }
        }
    }
    // MergeTree.referencePositionToLocalPosition (mergeTree.ts:1046-1062) at the local view
    // (Client.localReferencePositionToPosition, client.ts:398-403)
    int refPosition(int id) {
        const LRef& r = refs[size_t(id)];
        Seg* s = r.segment;
        if (!s || !s->parent) return MTR_DETACHED_POSITION;
        if ((r.refType & kTransient) || (s->localRefs && refsHas(s->localRefs, id)))
            return (s->removed ? 0 : r.offset) + getPosition(s, currentSeq, localClientId);
        return MTR_DETACHED_POSITION;
    }

    // ------------------------------------------------------------ reconnect
    static bool removedAndAcked(const Seg* s) { return s->removed && s->removedSeq != kUnassignedSeq; }
    // localNetLength(segment, refSeq, localSeq), mergeTree.ts:613-662: the local client's view at localSeq
    static int localNetLengthAt(const Seg* s, int refSeq, int lseq) {
        if (s->seq != kUnassignedSeq) {  // inserted remotely (or acked)
            if (s->seq > refSeq || (removedAndAcked(s) && s->removedSeq <= refSeq) ||
                (s->localRemovedSeq >= 0 && s->localRemovedSeq <= lseq))
                return 0;
            return s->len;
        }
        if (s->localSeq > lseq || (s->localRemovedSeq >= 0 && s->localRemovedSeq <= lseq)) return 0;
        return s->len;
    }

    // normalizeAdjacentSegments, mergeTree.ts:2231-2331: within a run of removed / unacked segments, acked
    // removed segments slide past the local ones, and each locally removed segment slides past the
    // unacked inserts newer than its removal; the run's segments then take the run's (parent, index)
    // places in the new order
    void normalizeAdjacent(const std::vector<Seg*>& run) {
        std::list<Seg*> lst(run.begin(), run.end());
        std::vector<std::pair<Block*, int>> places;
        for (Seg* x : run) places.push_back({x->parent, x->index});
        auto last = lst.end();  // the last segment not removed-and-acked
        for (auto it = lst.end(); it != lst.begin();) {
            --it;
            if (!removedAndAcked(*it)) {
                last = it;
                break;
            }
        }
        if (last == lst.end()) return;
        for (auto slide = last;;) {
            const bool first = slide == lst.begin();
            const auto nearer = first ? lst.end() : std::prev(slide);
            Seg* x = *slide;
            if (removedAndAcked(x)) {  // past every segment that is not also remotely removed
                lst.erase(slide);
                lst.insert(std::next(last), x);
            } else if (x->removed) {
                if (x->localRemovedSeq < 0) {
                    status = MTR_ERR_ASSERT | 0x54d;
                    return;
                }
                auto cur = slide;
                for (auto scan = std::next(slide); scan != lst.end() && !removedAndAcked(*scan) &&
                                                   (*scan)->localSeq >= 0 && (*scan)->localSeq > x->localRemovedSeq;
                     ++scan)
                    cur = scan;
                if (cur != slide) {
                    const auto after = std::next(cur);
                    lst.erase(slide);
                    lst.insert(after, x);
                }
            }
            if (first) break;
            slide = nearer;
        }
        size_t i = 0;
        std::vector<std::pair<int, Block*>> touched;
        for (Seg* x : lst) {
            Block* p = places[i].first;
            const int ix = places[i].second;
            i++;
            p->children[ix] = x;
            x->parent = p;
            x->index = ix;
        }
        // nodeUpdateLengthNewStructure on the ancestors, deepest first
        for (auto& pl : places) {
            int depth = 0;
            for (Block* b = pl.first; b; b = b->parent) depth++;
            for (Block* b = pl.first; b; b = b->parent) touched.push_back({depth--, b});
        }
        std::sort(touched.begin(), touched.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
        for (size_t k = 0; k < touched.size(); k++)
            if (k == 0 || touched[k].second != touched[k - 1].second) nodeUpdateLengthNewStructure(touched[k].second);
    }
    // normalizeSegmentsOnRebase, mergeTree.ts:2352-2381
    void normalizeSegmentsOnRebase() {
        std::vector<Seg*> lv;
        leaves(root, lv);
        std::vector<Seg*> run;
        bool local = false, acked = false;
        auto flush = [&]() {
            if (local && acked && run.size() > 1) normalizeAdjacent(run);
            run.clear();
            local = acked = false;
        };
        for (Seg* x : lv) {
            if (x->removed || x->seq == kUnassignedSeq) {
                if (removedAndAcked(x)) acked = true;
                if (x->seq == kUnassignedSeq) local = true;
                run.push_back(x);
            } else {
                flush();
            }
        }
        flush();
    }
    // Client.regeneratePendingOp (client.ts:917-960) of the oldest pending op (type: its MergeTreeDeltaType)
    // -> resetPendingDeltaToOps (client.ts:708-800); results as MTR_DELTA_REGEN / _X records
    int lastNormalizationRefSeq = 0;
    std::vector<std::pair<bool, PropMap>> regenProps;  // properties references of the MTR_DELTA_REGEN_X records
    void regenerate(int type) {
        if (currentSeq != lastNormalizationRefSeq) {
            normalizeSegmentsOnRebase();
            lastNormalizationRefSeq = currentSeq;
            if (status != MTR_OK) return;
        }
        if (pendingSegments.empty()) {
            status = MTR_ERR_ASSERT | 0x034;  // "Segment group not at head of merge tree pending queue"
            return;
        }
        SegGroup* g = pendingSegments.front();
        pendingSegments.pop_front();
        std::vector<Seg*> lv;
        leaves(root, lv);
        // findReconnectionPosition (client.ts:699-706): getPosition at (currentSeq, local client, localSeq)
        std::vector<int> before(lv.size() + 1, 0);
        for (size_t k = 0; k < lv.size(); k++) before[k + 1] = before[k] + localNetLengthAt(lv[k], currentSeq, g->localSeq);
        int off = 0;  // the member's offset in the inserted text: the members are its pieces, in order
        size_t seen = 0;
        for (size_t k = 0; k < lv.size() && seen < g->segments.size(); k++) {  // sorted by ordinal
            Seg* s = lv[k];
            if (std::find(g->segments.begin(), g->segments.end(), s) == g->segments.end()) continue;
            seen++;
            if (s->groups.empty() || s->groups.front() != g) {
                status = MTR_ERR_ASSERT | 0x035;  // "Segment group not at head of segment pending queue"
                return;
            }
            s->groups.pop_front();
            bool emit = false;
            if (type == MTR_OP_ANNOTATE) {
                emit = !s->removed || (s->localRemovedSeq >= 0 && s->removedSeq == kUnassignedSeq);
            } else if (type == MTR_OP_INSERT) {
                if (s->seq != kUnassignedSeq) {
                    status = MTR_ERR_ASSERT | 0x037;  // "Segment already has assigned sequence number"
                    return;
                }
                emit = true;
            } else if (type == MTR_OP_REMOVE) {
                emit = s->localRemovedSeq >= 0 && s->removed && s->removedSeq == kUnassignedSeq;
            } else {
                status = MTR_ERR_BAD_OP;
                return;
            }
            const int here = off;
            off += s->len;
            if (!emit) continue;
            uint32_t ref = 0xffffffffu;
            if (s->perm) {  // a PermutationSegment's clone keeps its start handle (the spec is [length, start])
                if (type == MTR_OP_INSERT) ref = uint32_t(s->start);
            } else if (type == MTR_OP_INSERT && s->hasProps) {
                ref = uint32_t(regenProps.size());
                regenProps.push_back({true, s->props});
            }
            deltas.push_back({curOpIndex, before[k], s->len, uint32_t(MTR_DELTA_REGEN + type)});
            deltas.push_back({curOpIndex, type == MTR_OP_INSERT ? here : 0, int32_t(ref), MTR_DELTA_REGEN_X});
            groupPool.emplace_back();  // a group of its own, at the tail (client.ts:787-795)
            SegGroup* ng = &groupPool.back();
            ng->localSeq = g->localSeq;
            pendingSegments.push_back(ng);
            s->groups.push_back(ng);
            ng->segments.push_back(s);
        }
    }

    // ------------------------------------------------------------ walking
    enum class LeafMode { Insert, Split };
    struct InsertContext {
        LeafMode mode;
        Seg* candidate = nullptr;
        bool hasContinue = false;
    };
    struct SegChanges {
        Node* replaceCurrent = nullptr;
        Node* next = nullptr;
    };
    static Block* unfinished() {
        static Block u;
        return &u;
    }

    SegChanges leafAction(InsertContext& ctx, Seg* segment, int pos) {
        SegChanges ch;
        if (ctx.mode == LeafMode::Insert) {  // onLeaf, mergeTree.ts:1638-1648
            if (segment) {
                ch.replaceCurrent = ctx.candidate;
                ch.next = segment;
            } else {
                ch.next = ctx.candidate;
            }
        } else {  // splitLeafSegment, mergeTree.ts:1686-1704
            if (!(pos > 0 && segment)) return ch;
            ch.next = splitAt(segment, pos);
        }
        return ch;
    }

    // breakTie, mergeTree.ts:1719-1738
    static bool breakTie(int pos, const Node* node, int seq) {
        if (node->leaf) {
            if (pos == 0) {
                int64_t newSeq = seq == kUnassignedSeq ? kMaxSafe : seq;
                const Seg* s = static_cast<const Seg*>(node);
                int64_t segSeq = s->seq == kUnassignedSeq ? kMaxSafe - 1 : s->seq;
                return newSeq > segSeq;
            }
            return false;
        }
        return true;
    }

    // first leaf after `node` in tree order (forwardExcursion, mergeTreeNodeWalk.ts:121)
    Seg* firstLeafAfter(Node* node) {
        Node* cur = node;
        while (cur->parent) {
            Block* p = cur->parent;
            for (int i = cur->index + 1; i < p->childCount; i++) {
                Node* c = p->children[i];
                while (c && !c->leaf) {
                    Block* cb = static_cast<Block*>(c);
                    c = cb->childCount > 0 ? cb->children[0] : nullptr;
                }
                if (c) return static_cast<Seg*>(c);
            }
            cur = p;
        }
        return nullptr;
    }
    // continueFrom, mergeTree.ts:1611-1615
    bool continuePredicate(Block* block) {
        Seg* s = firstLeafAfter(block);
        return s != nullptr && s->seq == kUnassignedSeq;
    }

    int leafIndex(Seg* x) {
        std::vector<Seg*> lv;
        leaves(root, lv);
        for (size_t i = 0; i < lv.size(); i++)
            if (lv[i] == x) return int(i);
        return -1;
    }
    // split, mergeTree.ts:1858-1871
    Block* split(Block* node) {
        const int half = kMaxNodesInBlock / 2;
        Block* nb = makeBlock();
        nb->childCount = half;
        node->childCount = half;
        for (int i = 0; i < half; i++) {
            assignChild(nb, node->children[half + i], i);
            node->children[half + i] = nullptr;
        }
        nodeUpdateLengthNewStructure(node);
        nodeUpdateLengthNewStructure(nb);
        return nb;
    }

    // insertingWalk, mergeTree.ts:1740-1856
    Block* insertingWalk(Block* block, int pos, int refSeq, int clientId, int seq, InsertContext& ctx) {
        int _pos = pos;
        int childIndex;
        Node* newNode = nullptr;
        for (childIndex = 0; childIndex < block->childCount; childIndex++) {
            Node* child = block->children[childIndex];
            int len = nodeLength(child, refSeq, clientId);
            if (len == kUndef) continue;
            if (_pos < len || (_pos == len && breakTie(_pos, child, seq))) {
                if (!child->leaf) {
                    Block* splitNode = insertingWalk(static_cast<Block*>(child), _pos, refSeq, clientId, seq, ctx);
                    if (splitNode == nullptr) {  // mergeTree.ts:1778-1784
                        blockUpdateLength(block, seq, clientId);
                        return nullptr;
                    }
                    if (splitNode == unfinished()) {
                        _pos -= len;
                        continue;
                    }
                    newNode = splitNode;
                    childIndex++;
                } else {
                    SegChanges ch = leafAction(ctx, static_cast<Seg*>(child), _pos);
                    if (ch.replaceCurrent) assignChild(block, ch.replaceCurrent, childIndex);
                    if (ch.next) {
                        newNode = ch.next;
                        childIndex++;
                    } else {
                        return nullptr;
                    }
                }
                break;
            } else {
                _pos -= len;
            }
        }
        if (!newNode && _pos == 0) {
            if (seq != kUnassignedSeq && ctx.hasContinue && continuePredicate(block)) return unfinished();
            newNode = leafAction(ctx, nullptr, _pos).next;
        }
        if (newNode) {
            for (int i = block->childCount; i > childIndex; i--) {
                block->children[i] = block->children[i - 1];
                block->children[i]->index = i;
            }
            assignChild(block, newNode, childIndex);
            block->childCount++;
            if (block->childCount < kMaxNodesInBlock) {  // mergeTree.ts:1837-1848
                blockUpdateLength(block, seq, clientId);
                return nullptr;
            }
            return split(block);
        }
        return nullptr;
    }

    // updateRoot, mergeTree.ts:1268-1277
    void updateRoot(Block* splitNode) {
        if (splitNode && splitNode != unfinished()) {
            Block* nr = makeBlock();
            nr->childCount = 2;
            assignChild(nr, root, 0);
            assignChild(nr, splitNode, 1);
            root = nr;
            nodeUpdateLengthNewStructure(root);
        }
    }

    // ensureIntervalBoundary, mergeTree.ts:1706-1716
    void ensureIntervalBoundary(int pos, int refSeq, int clientId) {
        InsertContext ctx{LeafMode::Split};
        Block* s = insertingWalk(root, pos, refSeq, clientId, kTreeMaintenanceSeq, ctx);
        updateRoot(s);
    }

    // addToLRUSet, mergeTree.ts:741-751
    void addToLRUSet(Seg* s, int seq) {
        if (s->parent->needsScour != 1 && seq > currentSeq) {
            s->parent->needsScour = 1;
            heap.add({s, seq});
        }
    }

    // nodeMap, mergeTree.ts:2526-2577 over depthFirstNodeWalk, mergeTreeNodeWalk.ts:35-115.  Leaf
    // actions run in walk order (they never change a length the walk reads later: the leaf was
    // passed, sibling and ancestor lengths were read before).  `post` is the walk's upAction: after
    // every block the walk descended into (downAction Continue), and on the way up for its ancestors
    // -- the root included when it holds blocks; a root holding leaves never gets it (the walk's
    // first block result is undefined, mergeTreeNodeWalk.ts:98-105).
    struct NoPost {
        void operator()(Block*) const {}
    };
    template <class F, class Post = NoPost>
    void nodeMap(int refSeq, int clientId, F&& leaf, int start, int end, Post post = Post()) {
        int endPos = end >= 0 ? end : std::max(0, nodeLength(root, refSeq, clientId));
        if (endPos == start) return;
        int pos = 0;
        bool exit = false;
        walkMap(root, refSeq, clientId, start, endPos, pos, exit, leaf, post);
        if (root->childCount > 0 && !root->children[0]->leaf) post(root);
    }
    template <class F, class Post>
    void walkMap(Block* b, int refSeq, int clientId, int start, int endPos, int& pos, bool& exit, F& leaf,
                 Post& post) {
        for (int i = 0; i < b->childCount && !exit; i++) {
            Node* n = b->children[i];
            if (endPos <= pos) {
                exit = true;
                return;
            }
            int len = nodeLength(n, refSeq, clientId);
            if (len == kUndef || len == 0) continue;
            int nextPos = pos + len;
            if (start >= nextPos) {
                pos = nextPos;
                continue;
            }
            if (n->leaf) {
                leaf(static_cast<Seg*>(n));
                pos = nextPos;
            } else {
                walkMap(static_cast<Block*>(n), refSeq, clientId, start, endPos, pos, exit, leaf, post);
                post(static_cast<Block*>(n));
            }
        }
    }

    // ------------------------------------------------------------ zamboni
    // scourNode, zamboni.ts:122-193
    void scourNode(Block* node, std::vector<Node*>& hold) {
        Seg* prev = nullptr;
        for (int k = 0; k < node->childCount; k++) {
            Node* child = node->children[k];
            if (child->leaf) {
                Seg* s = static_cast<Seg*>(child);
                if (!s->groups.empty()) {  // a segment of a pending local op is held (zamboni.ts:128, 185-188)
                    hold.push_back(s);
                    prev = nullptr;
                } else if (s->removed) {
                    if (s->removedSeq > minSeq || !s->tgroups.empty()) {  // (tracked: held, zamboni.ts:132)
                        hold.push_back(s);
                    } else {
                        // UNLINK; a PermutationVector frees the segment's handles in order
                        // (onMaintenance, permutationvector.ts:418-443)
                        if (s->perm && s->start >= 1) {
                            if (recycleLog)  // onRowHandlesRecycled / onColHandlesRecycled, matrix.ts:722-734
                                deltas.push_back({curOpIndex, s->start, s->len, MTR_DELTA_RECYCLE});
                            for (int h = 0; h < s->len; h++) freeHandle(s->start + h);
                        }
                        if (s->tid >= 0) freeTids.push_back(s->tid);
                        s->parent = nullptr;
                    }
                    prev = nullptr;
                } else {
                    if (s->seq <= minSeq) {
                        int ln = localNetLength(s);
                        bool ok = prev && canAppend(prev, s) && matchProperties(prev, s, tabs.b) &&
                                  sameGroups(prev, s) && (ln > 0);
                        if (ok) {
                            if (!s->tgroups.empty()) {  // it leaves its tracking groups (zamboni.ts:171-173)
                                if (recycleLog) deltas.push_back({curOpIndex, s->tid, prev->tid, MTR_DELTA_TMERGE});
                                const std::vector<TGroup*> gs = s->tgroups;
                                for (TGroup* g : gs) tunlink(g, s);
                            }
                            if (s->tid >= 0) freeTids.push_back(s->tid);
                            refsAppend(prev, s);    // BaseSegment.append, mergeTreeNodes.ts:527-530 (before lengths)
                            prev->text += s->text;  // TextSegment.append textSegment.ts:99-103 (BaseSegment.append for perm)
                            prev->len += s->len;
                            s->parent = nullptr;
                        } else {
                            hold.push_back(s);
                            prev = ln > 0 ? s : nullptr;
                        }
                    } else {
                        hold.push_back(s);
                        prev = nullptr;
                    }
                }
            } else {
                hold.push_back(child);
                prev = nullptr;
            }
        }
    }

    static bool underflow(const Block* b) { return b->childCount < kMaxNodesInBlock / 2; }

    // packParent, zamboni.ts:63-120
    void packParent(Block* parent) {
        std::vector<Node*> hold;
        for (int ci = 0; ci < parent->childCount; ci++) {
            Block* cb = static_cast<Block*>(parent->children[ci]);
            scourNode(cb, hold);
            cb->parent = nullptr;
        }
        OTRACE("PACK items=%d\n", int(hold.size()));
        if (!hold.empty()) {
            int total = int(hold.size());
            const int halfMax = kMaxNodesInBlock / 2;
            int childCount = std::min(kMaxNodesInBlock - 1, total / halfMax);
            if (childCount < 1) childCount = 1;
            int base = total / childCount;
            int rem = total % childCount;
            int packed = 0;
            std::vector<Block*> blocks;
            for (int ni = 0; ni < childCount; ni++) {
                int nc = base;
                if (rem > 0) {
                    nc++;
                    rem--;
                }
                Block* pb = makeBlock();
                pb->childCount = nc;
                for (int pi = 0; pi < nc; pi++) assignChild(pb, hold[packed++], pi);
                pb->parent = parent;
                blocks.push_back(pb);
                nodeUpdateLengthNewStructure(pb);  // zamboni.ts:103
            }
            for (int j = 0; j < kMaxNodesInBlock; j++) parent->children[j] = nullptr;
            for (int j = 0; j < childCount; j++) assignChild(parent, blocks[j], j);
            parent->childCount = childCount;
        } else {
            for (int j = 0; j < kMaxNodesInBlock; j++) parent->children[j] = nullptr;
            parent->childCount = 0;
        }
        if (underflow(parent) && parent->parent) packParent(parent->parent);
        else blockUpdatePathLengthsNew(parent);  // zamboni.ts:114-119
    }

    // zamboniSegments, zamboni.ts:19-60
    void dumpLeaves(const char* tag) {
        std::vector<Seg*> lv;
        leaves(root, lv);
        for (size_t i = 0; i < lv.size(); i++) {
            Seg* s = lv[i];
            int bnd = 0;
            const Node* n = s;
            while (n->parent && n->index == 0) { bnd++; n = n->parent; }
            printf("%s %zu len=%d seq=%d rs=%d bnd=%d\n", tag, i, s->len, s->seq, s->removed ? s->removedSeq : -1, bnd);
        }
    }
    int curOpSeq = -1;
    void zamboniSegments() {
        if (!collaborating) return;
        if (g_trace && curOpSeq == g_trace_seq) dumpLeaves("DUMP");
        for (int i = 0; i < kZamboniSegmentsMax; i++) {
            const LRUEntry* top = heap.peek();
            if (!top || top->maxSeq > minSeq) break;
            LRUEntry e = heap.get();
            Seg* s = e.segment;
            OTRACE("ZPOP seq=%d linked=%d ns=%d leaf=%d\n", e.maxSeq, s->parent ? 1 : 0,
                   s->parent ? s->parent->needsScour : -9, leafIndex(s));
            if (s->parent && s->parent->needsScour != 0) {
                Block* block = s->parent;
                std::vector<Node*> copy;
                scourNode(block, copy);
                block->needsScour = 0;
                int newCount = int(copy.size());
                OTRACE("SCOUR n=%d kept=%d\n", block->childCount, newCount);
                if (newCount < block->childCount) {
                    for (int j = 0; j < kMaxNodesInBlock; j++) block->children[j] = nullptr;
                    block->childCount = newCount;
                    for (int j = 0; j < newCount; j++) assignChild(block, copy[j], j);
                    if (underflow(block) && block->parent) packParent(block->parent);
                    else blockUpdatePathLengthsNew(block);  // zamboni.ts:52-56
                }
            }
        }
    }

    // setMinSeq, mergeTree.ts:1025-1044
    void setMinSeq(int ms) {
        if (ms > currentSeq) {
            status = MTR_ERR_ASSERT | 0x04e;
            return;
        }
        if (minSeq > ms) {
            status = MTR_ERR_ASSERT | 0x04f;
            return;
        }
        if (ms > minSeq) {
            minSeq = ms;
            zamboniSegments();
        }
    }
    // updateSeqNumbers, client.ts:877-887
    void updateSeqNumbers(int ms, int seq) {
        if (currentSeq > seq) {
            status = MTR_ERR_ASSERT | 0x038;
            return;
        }
        currentSeq = seq;
        if (ms > seq) {
            status = MTR_ERR_ASSERT | 0x039;
            return;
        }
        setMinSeq(ms);
    }

    // ------------------------------------------------------------ ops
    // properties: PropertiesManager.addProperties (segmentPropertiesManager.ts:60-157) for an observer
    // (no pending local keys: shouldModifyKey is always true), BaseSegment.addProperties
    // (mergeTreeNodes.ts:385-406).  comb = MTR_COMB_* | NaN value id << 3 (include/mtr_types.h).
    // seq: the op's seq (kUnassignedSeq for a pending local annotate); collab: collabWindow.collaborating as
    // BaseSegment.addProperties passes it (false for a new segment's initial props, sequenceFactory.ts)
    void addProperties(Seg* s, uint32_t propop, uint32_t comb = 0, int seq = kUniversalSeq, bool collab = false) {
        const mtr_batch* b = tabs.b;
        const uint32_t mode = comb & 7u, nanv = comb >> 3;
        s->hasPropMgr = true;
        s->hasProps = true;
        const uint32_t lo = b->propop_off[propop], hi = b->propop_off[propop + 1];
        // shouldModifyKey (:94-104): a remote op leaves keys with pending local updates alone unless it
        // has a (non-rewrite) combiningOp
        const bool remote = seq != kUnassignedSeq && seq != kUniversalSeq;
        // outstanding local rewrites block every remote change (:72-80)
        if (s->pendingRewrite > 0 && remote && collab) return;
        auto modify = [&](uint32_t key) {
            return !remote || mode >= MTR_COMB_INCR || pendingCount(s, key) == nullptr;
        };
        if (mode == MTR_COMB_REWRITE) {  // delete old keys whose new value is falsy (:109-123)
            if (collab && seq == kUnassignedSeq) s->pendingRewrite++;
            std::vector<std::pair<uint32_t, uint32_t>> kept;
            for (auto& kv : s->props.kv) {
                bool truthy = false;
                for (uint32_t i = lo; i < hi; i++)
                    if (b->propop_kv[2 * i] == kv.first) {
                        const uint32_t v = b->propop_kv[2 * i + 1];
                        truthy = v != MTR_NULL_VALUE && !(b->val_eq[v] & MTR_VEQ_FALSY);
                        break;
                    }
                if (truthy || !modify(kv.first)) kept.push_back(kv);
            }
            s->props.kv.swap(kept);
        }
        for (uint32_t i = lo; i < hi; i++) {
            uint32_t k = b->propop_kv[2 * i], v = b->propop_kv[2 * i + 1];
            if (collab) {  // :126-138
                if (seq == kUnassignedSeq) {
                    if (mode == MTR_COMB_REWRITE && v == MTR_NULL_VALUE) continue;  // (handled by the delete pass)
                    if (int* c = pendingCount(s, k)) ++*c;
                    else s->pendingKeys.push_back({k, 1});
                } else if (!modify(k)) {
                    continue;
                }
            }
            if (mode >= MTR_COMB_INCR) {  // newValue = combine(op, previousValue, undefined, seq), :145-147
                const std::pair<uint32_t, uint32_t>* prev = nullptr;
                for (auto& kv : s->props.kv)
                    if (kv.first == k) prev = &kv;
                if (prev) {
                    const uint32_t f = b->val_eq[prev->second];
                    if (mode == MTR_COMB_INCR) {
                        if (f & MTR_VEQ_INCR_STR) {  // string / object + undefined: a new string
                            status = MTR_ERR_UNSUPPORTED;
                            return;
                        }
                        v = nanv;  // number + undefined
                    } else {
                        if (mode == MTR_COMB_CONSENSUS && (f & MTR_VEQ_CONS_MUT)) {  // cv.seq = seq in place
                            status = MTR_ERR_UNSUPPORTED;
                            return;
                        }
                        v = prev->second;
                    }
                }  // absent: the host's combine of the default (or null: stays absent)
            }
            if (v == MTR_NULL_VALUE)
                propDelete(s->props, k);
            else
                propSet(s->props, k, v, tabs);
        }
    }

    Seg* segmentFromSpec(const mtr_op& op, const mtr_doc_desc& dd) {  // sequenceFactory.ts:26-38
        Seg* s = makeSeg();
        if (permMode) {  // PermutationSegment.fromJSONObject + reset() on INSERT (permutationvector.ts:45-48, 354-361)
            s->perm = true;
            s->len = int(op.payload2);
            // a snapshot segment keeps its start: loading fires no delta callback (mergeTree.ts:1410-1418)
            const bool snap = op.type == MTR_OP_LOAD || (op.flags & MTR_F_APPEND);
            s->start = snap ? int(op.payload) : MTR_HANDLE_UNALLOCATED;
            return s;
        }
        if (op.flags & MTR_F_MARKER) {
            s->marker = true;
            s->refType = int(op.payload);
            s->noRef = (op.flags & MTR_F_NOREF) != 0;
            s->len = 1;
            s->markerOrdinal = op.payload2;
        } else {
            const uint16_t* t = tabs.b->text + dd.text_base + op.payload;
            s->text.assign(reinterpret_cast<const char16_t*>(t), op.payload2);
            s->len = int(op.payload2);
        }
        if ((op.flags & MTR_F_PROPS) && op.pos2 >= 0) addProperties(s, uint32_t(op.pos2));
        return s;
    }

    // SequenceDeltaEvent ranges of MTR_F_DELTA ops (sequenceDeltaEvent.ts: position = getPosition
    // at the local view when the delta callback fires, before zamboni; tree order)
    bool deltaOn = false;
    bool trackCollect = false;
    std::vector<Seg*> trackFresh;
    bool recycleLog = false;  // a matrix vector tracked for its cells (MTR_DELTA_RECYCLE records)
    uint32_t curOpIndex = 0;
    std::vector<mtr_delta> deltas;
    void recordDeltas(const std::vector<Seg*>& segs, uint32_t kind) {
        if (!deltaOn) return;
        for (Seg* x : segs) deltas.push_back({curOpIndex, localPosition(x), x->len, kind});
    }

    // insertSegments + blockInsert, mergeTree.ts:1397-1427,1594-1685
    void insertSegments(int pos, Seg* seg, int refSeq, int clientId, int seq) {
        ensureIntervalBoundary(pos, refSeq, clientId);
        const int localSeq = seq == kUnassignedSeq ? ++localSeqCounter : 0;  // mergeTree.ts:1407-1408
        if (seg->len > 0) {
            seg->seq = seq;
            seg->clientId = clientId;
            seg->localSeq = seq == kUnassignedSeq ? localSeq : -1;  // blockInsert, mergeTree.ts:1656
            if (seg->markerOrdinal) idToSegment[seg->markerOrdinal - 1] = seg;  // blockInsert, mergeTree.ts:1655-1662
            InsertContext ctx{LeafMode::Insert, seg, true};
            Block* splitNode = insertingWalk(root, pos, refSeq, clientId, seq, ctx);
            if (seg->parent == nullptr) {
                status = MTR_ERR_INSERT_FAILED;
                return;
            }
            updateRoot(splitNode);
            recordDeltas({seg}, MTR_OP_INSERT);  // mergeTree.ts:1414-1418
            if (collaborating) {  // saveIfLocal, mergeTree.ts:1618-1637
                if (seg->seq == kUnassignedSeq && clientId == localClientId) addToPendingList(seg, nullptr, localSeq);
                else if (seg->seq > minSeq) addToLRUSet(seg, seg->seq);
            }
        }
        if (collaborating && seq != kUnassignedSeq) zamboniSegments();
    }

    // markRangeRemoved, mergeTree.ts:1955-2047
    void markRangeRemoved(int start, int end, int refSeq, int clientId, int seq) {
        ensureIntervalBoundary(start, refSeq, clientId);
        ensureIntervalBoundary(end, refSeq, clientId);
        std::vector<Seg*> fresh;  // removedSegments (mergeTree.ts:1975-2000)
        bool overwrite = false;   // _overwrite: an overlapping remove rebuilds lengths (mergeTree.ts:1966,2012-2019)
        const int localSeq = seq == kUnassignedSeq ? ++localSeqCounter : 0;  // mergeTree.ts:1970-1971
        SegGroup* group = nullptr;
        std::vector<Seg*> localOverlapWithRefs;  // mergeTree.ts:1965, 1984-1986
        nodeMap(
            refSeq, clientId,
            [&](Seg* s) {
                if (s->removed) {
                    overwrite = true;
                    if (s->removedSeq == kUnassignedSeq) {
                        s->removedClientIds.insert(s->removedClientIds.begin(), clientId);
                        s->removedSeq = seq;
                        if (s->localRefs && s->localRefs->refCount) localOverlapWithRefs.push_back(s);
                    } else {
                        s->removedClientIds.push_back(clientId);
                    }
                } else {
                    s->removed = true;
                    s->removedClientIds.assign(1, clientId);
                    s->removedSeq = seq;
                    s->localRemovedSeq = seq == kUnassignedSeq ? localSeq : -1;  // mergeTree.ts:1994
                    fresh.push_back(s);
                }
                if (collaborating) {  // mergeTree.ts:2000-2010
                    if (s->removedSeq == kUnassignedSeq && clientId == localClientId)
                        group = addToPendingList(s, group, localSeq);
                    else
                        addToLRUSet(s, seq);
                }
            },
            start, end,
            [&](Block* b) {  // afterMarkRemoved, mergeTree.ts:2012-2019
                if (overwrite) nodeUpdateLengthNewStructure(b);
                else blockUpdateLength(b, seq, clientId);
            });
        // already removed locally, so no event: their sliding references slide now (mergeTree.ts:2023-2025)
        for (Seg* s : localOverlapWithRefs) slideAckedRemovedSegmentReferences(s);
        recordDeltas(fresh, MTR_OP_REMOVE);  // mergeTree.ts:2026-2031
        if (trackCollect) trackFresh = fresh;  // (the delta segments VectorUndoProvider.record links)
        // newly removed by someone else (or before collaboration): slide after the event (mergeTree.ts:2032-2040)
        if (!collaborating || clientId != localClientId)
            for (Seg* s : fresh) slideAckedRemovedSegmentReferences(s);
        if (collaborating && seq != kUnassignedSeq) zamboniSegments();
    }

    // annotateRange, mergeTree.ts:1895-1953
    void annotateRange(int start, int end, uint32_t propop, int refSeq, int clientId, int seq, uint32_t comb = 0) {
        ensureIntervalBoundary(start, refSeq, clientId);
        ensureIntervalBoundary(end, refSeq, clientId);
        std::vector<Seg*> touched;
        const int localSeq = seq == kUnassignedSeq ? ++localSeqCounter : 0;  // mergeTree.ts:1909-1910
        SegGroup* group = nullptr;
        nodeMap(
            refSeq, clientId,
            [&](Seg* s) {
                const std::pair<bool, PropMap> before{s->hasProps, s->props};
                addProperties(s, propop, comb, seq, collaborating);
                touched.push_back(s);
                if (collaborating) {  // mergeTree.ts:1921-1935
                    if (seq == kUnassignedSeq) {
                        group = addToPendingList(s, group, localSeq);
                        group->hasPrevious = true;  // addToPendingList's previousProps (:1330-1351)
                        group->previousProps.push_back(before);
                    } else {
                        addToLRUSet(s, seq);
                    }
                }
            },
            start, end);
        recordDeltas(touched, MTR_OP_ANNOTATE);  // mergeTree.ts:1941-1946
        if (collaborating && seq != kUnassignedSeq) zamboniSegments();
    }

    // ------------------------------------------------------------ snapshot load
    // merge info of a snapshot segment, SnapshotLoader.specToSegment (snapshotLoader.ts:88-128)
    static int opClient(const mtr_op& op) { return int(int16_t(op.client)); }
    void setMergeInfo(Seg* s, const mtr_op& op, const mtr_doc_desc& dd) {
        s->clientId = opClient(op);
        s->seq = op.seq;
        if (op.ref_seq >= 0) {
            s->removed = true;
            s->removedSeq = op.ref_seq;
        }
        s->removedClientIds.clear();
        for (int k = 0; k < op.min_seq; k++) s->removedClientIds.push_back(int(tabs.b->text[dd.text_base + op.pos1 + k]));
    }

    // MergeTree.reloadFromSegments (mergeTree.ts:678-728): blocks of MaxNodesInBlock - 1 children,
    // built bottom-up layer by layer
    std::vector<Seg*> pendingLoad;
    void reloadFromSegments() {
        const int maxChildren = kMaxNodesInBlock - 1;
        if (pendingLoad.empty()) {
            root = makeBlock();
            return;
        }
        std::vector<Node*> nodes(pendingLoad.begin(), pendingLoad.end());
        pendingLoad.clear();
        for (;;) {
            const size_t blockCount = (nodes.size() + maxChildren - 1) / maxChildren;
            std::vector<Node*> blocks;
            for (size_t ni = 0, bi = 0; bi < blockCount; bi++) {
                Block* b = makeBlock();
                for (int ci = 0; ci < maxChildren && ni < nodes.size(); ci++, ni++) assignChild(b, nodes[ni], b->childCount++);
                blocks.push_back(b);
            }
            if (blocks.size() == 1) {
                root = static_cast<Block*>(blocks[0]);
                root->parent = nullptr;
                return;
            }
            nodes.swap(blocks);
        }
    }

    int apply(const mtr_op& op, const mtr_doc_desc& dd) {
        curOpSeq = op.seq;
        if (op.type == MTR_OP_LOAD) {  // SnapshotLoader.loadHeader segments (snapshotLoader.ts:130-141)
            if (collaborating) return MTR_ERR_ASSERT | 0x049;  // "Trying to reload from segments while collaborating!"
            Seg* s = segmentFromSpec(op, dd);
            setMergeInfo(s, op, dd);
            // reloadFromSegments' blockUpdate maps live markers (addNodeReferences, mergeTree.ts:297-306);
            // the host gives a removed one no ordinal
            if (s->markerOrdinal) idToSegment[s->markerOrdinal - 1] = s;
            pendingLoad.push_back(s);
            return status;
        }
        if (!pendingLoad.empty()) reloadFromSegments();
        int pos1 = op.pos1, pos2 = op.pos2;
        if (op.type == MTR_OP_RELPOS) {  // getValidOpRange -> posFromRelativePos (client.ts:527-545, mergeTree.ts:1371-1395)
            int p = -1;
            auto it = idToSegment.find(uint32_t(op.pos1));
            if (it != idToSegment.end()) {
                p = getPosition(it->second, op.ref_seq, op.client);
                const int off = (op.payload2 & MTR_REL_OFFSET) ? int(op.payload) : 0;
                p = (op.payload2 & MTR_REL_BEFORE) ? p - off : p + it->second->len + off;
            }
            if (p < 0) return MTR_ERR_UNSUPPORTED;  // the reference goes on with position -1
            relPos[op.pos2 == 2 ? 1 : 0] = p;
            relMask |= op.pos2 == 2 ? 2 : 1;
            return status;
        }
        if (op.flags & MTR_F_REL) {  // the positions the MTR_OP_RELPOS records ahead resolved
            if (relMask & 1) pos1 = relPos[0];
            if ((relMask & 2) && op.type != MTR_OP_INSERT) pos2 = relPos[1];
            relMask = 0;
        }
        switch (op.type) {
            case MTR_OP_INSERT: {
                Seg* s = segmentFromSpec(op, dd);
                if (op.flags & MTR_F_APPEND) {  // SnapshotLoader.loadBody append (snapshotLoader.ts:221-256)
                    setMergeInfo(s, op, dd);
                    insertSegments(blockLocalLength(root), s, kUniversalSeq, opClient(op), op.seq);
                    return status;
                }
                insertSegments(pos1, s, op.ref_seq, op.client, op.seq);
                break;
            }
            case MTR_OP_REMOVE:
                markRangeRemoved(pos1, pos2, op.ref_seq, op.client, op.seq);
                break;
            case MTR_OP_ANNOTATE:
                annotateRange(pos1, pos2, op.payload, op.ref_seq, op.client, op.seq, op.payload2);
                break;
            case MTR_OP_SEQ:
                break;
            case MTR_OP_HANDLES: {  // HandleTable.load (handletable.ts:88), PermutationVector.load (permutationvector.ts:327-345)
                if (!permMode || collaborating || op.pos1 < 1) return MTR_ERR_BAD_OP;
                const uint16_t* t = tabs.b->text + dd.text_base + op.payload;
                handles.assign(size_t(op.pos1), 0);
                for (int k = 0; k < op.pos1; k++) handles[size_t(k)] = int32_t(uint32_t(t[2 * k]) | (uint32_t(t[2 * k + 1]) << 16));
                return status;
            }
            // local ops (Client.insertSegmentLocal / removeRangeLocal / annotateRangeLocal -> applyInsertOp /
            // applyRemoveRangeOp / applyAnnotateRangeOp without a sequenced message, client.ts:430-520):
            // refSeq = currentSeq, the local client id, seq = UnassignedSequenceNumber while collaborating
            // (a pending op until its ack), UniversalSequenceNumber before
            case MTR_OP_LOCAL_INSERT: {
                Seg* s = segmentFromSpec(op, dd);
                if (permMode && op.pos2 >= 0) {  // SharedMatrix._undoRemoveRows / _undoRemoveCols (matrix.ts:371-430)
                    Seg* ref = findTid(op.pos2);
                    // insertRelative's op position: referencePositionToLocalPosition (client.ts:252-270)
                    if (!ref || !op.payload || localPosition(ref) != op.pos1) return MTR_ERR_BAD_OP;
                    insertAtReferencePosition(ref, s);
                    trackLink(s, op.payload);
                    transferToReplacement(ref, s);
                    return status;
                }
                insertSegments(op.pos1, s, currentSeq, localClientId, collaborating ? kUnassignedSeq : kUniversalSeq);
                if (permMode && op.payload && s->parent && status == MTR_OK) trackLink(s, op.payload);
                return status;
            }
            case MTR_OP_LOCAL_REMOVE: {
                std::vector<Seg*>* fresh = permMode && op.payload ? &trackFresh : nullptr;
                trackFresh.clear();
                trackCollect = fresh != nullptr;
                markRangeRemoved(op.pos1, op.pos2, currentSeq, localClientId,
                                 collaborating ? kUnassignedSeq : kUniversalSeq);
                trackCollect = false;
                if (fresh && status == MTR_OK)
                    for (Seg* x : trackFresh) trackLink(x, op.payload);
                return status;
            }
            case MTR_OP_TRACK: {  // TrackingGroup.unlink (the undo provider's revert / discard)
                if (!permMode) return MTR_ERR_BAD_OP;
                Seg* one = op.pos1 >= 0 ? findTid(op.pos1) : nullptr;
                for (int b = 0; b < MTR_TRACK_GROUPS; b++) {
                    if (!(op.payload >> b & 1u)) continue;
                    TGroup* g = &tgroup[b];
                    if (op.pos1 < 0) {
                        while (!g->segs.empty()) tunlink(g, g->segs.front());
                    } else if (one) {
                        tunlink(g, one);
                    }
                }
                return status;
            }
            case MTR_OP_LOCAL_ANNOTATE:
                // (a combining annotate: payload2 = MTR_COMB_* | NaN value id << 3, its prop-op the host's combine of
                // each key's default as for a remote one -- combine(op, undefined, undefined, UnassignedSequenceNumber))
                annotateRange(op.pos1, op.pos2, op.payload, currentSeq, localClientId,
                              collaborating ? kUnassignedSeq : kUniversalSeq, op.payload2);
                return status;
            case MTR_OP_ROLLBACK:  // Client.rollback (client.ts:421-423) of the newest pending local op
                if (!collaborating) return MTR_ERR_BAD_OP;
                rollback(int(op.payload2), op.payload, uint32_t(op.pos1));
                return status;
            case MTR_OP_REGENERATE:  // Client.regeneratePendingOp (client.ts:917-960) of the oldest pending op
                if (!collaborating) return MTR_ERR_BAD_OP;
                regenerate(int(op.payload2));
                return status;
            case MTR_OP_ACK:  // Client.applyMsg of this client's own message (client.ts:866-869)
                if (!collaborating) return MTR_ERR_BAD_OP;
                ackPendingSegment(int(op.payload2), op.payload, op.seq, uint32_t(op.pos1));
                break;
            case MTR_OP_REF_CREATE: {  // createPositionReference, sequence/src/intervalCollection.ts:697-724
                const bool lv = (op.payload2 & MTR_REF_LOCALVIEW) != 0;
                int off = 0;
                Seg* s = (op.payload2 & MTR_REF_LSEQ)
                             ? containingSegmentAt(op.pos1, op.ref_seq, op.min_seq, off)
                             : containingSegment(op.pos1, lv ? currentSeq : op.ref_seq, lv ? localClientId : int(op.client), off);
                if (s && (op.payload2 & MTR_REF_SLIDE)) {  // Client.getSlideToSegment, client.ts:1085-1099
                    Seg* t = getSlideToSegment(s);
                    if (t != s) {
                        off = (t && leafIndex(t) < leafIndex(s)) ? t->len - 1 : 0;
                        s = t;
                    }
                }
                return createRef(s, off, int(op.payload), (op.payload2 & MTR_REF_SLOT) ? (op.pos2 < 0 ? INT32_MAX : op.pos2) : -1);
            }
            case MTR_OP_REF_REMOVE: {  // MergeTree.removeLocalReferencePosition, mergeTree.ts:2190-2207
                if (op.payload >= refs.size()) return MTR_ERR_BAD_OP;
                Seg* s = refs[op.payload].segment;
                if (s) refsRemove(s->localRefs, int(op.payload));
                return status;
            }
            case MTR_OP_REF_ACK: {  // IntervalCollection.ackInterval (intervalCollection.ts:2054-2138), one endpoint
                if (op.payload >= refs.size()) return MTR_ERR_BAD_OP;
                const int id = int(op.payload);
                const int nt = (refs[size_t(id)].refType & ~kStay) | kSlide;  // setSlideOnRemove (:2047-2052)
                Seg* s = refs[size_t(id)].segment;
                if (s && s->localRefs && refsHas(s->localRefs, id)) {  // getSlideToSegment(lref) (:2031-2045)
                    Seg* t = getSlideToSegment(s);
                    if (t != s) {  // createPositionReferenceFromSegoff(newStart, refType, op) (:2101-2117)
                        const int off = (t && leafIndex(t) < leafIndex(s)) ? t->len - 1 : 0;
                        refsRemove(s->localRefs, id);  // removeLocalReferencePosition(oldInterval.start)
                        LRef& r = refs[size_t(id)];
                        r.segment = nullptr;
                        r.offset = 0;
                        r.list = -1;
                        if (t) {
                            if (!t->localRefs) t->localRefs = newLocalRefs(t, size_t(t->len));
                            r.segment = t;
                            r.offset = off;
                            RefsAtOffset& slot = refSlot(t->localRefs, off);
                            slot.has[1] = true;
                            slot.lst[1].push_back(id);
                            r.list = 1;
                            t->localRefs->refCount++;
                        }
                    }
                }
                refs[size_t(id)].refType = nt;
                return status;
            }
            case MTR_OP_REBASE_POS: {  // IntervalCollection.rebasePositionWithSegmentSlide (intervalCollection.ts:1472-1505)
                if (!collaborating) return MTR_ERR_BAD_OP;
                int off = 0;
                Seg* s = containingSegmentAt(op.pos1, op.ref_seq, op.min_seq, off);
                if (op.payload2 & MTR_REBASE_NOSLIDE) {  // SharedMatrix.rebasePosition (matrix.ts:534-551)
                    int res = MTR_DETACHED_POSITION;     // (no segment: undefined)
                    if (s && op.pos1 >= 0) {  // findReconnectionPosition(segment, localSeq) + offset, no slide
                        std::vector<Seg*> lv;
                        leaves(root, lv);
                        int before = 0;
                        for (Seg* x : lv) {
                            if (x == s) break;
                            before += localNetLengthAt(x, currentSeq, op.min_seq);
                        }
                        res = before + off;
                    }
                    deltas.push_back({curOpIndex, res, 0, MTR_DELTA_REBASE});
                    return status;
                }
                if (!s) return status = MTR_ERR_ASSERT | 0x54e;  // "No segment found"
                Seg* t = getSlideToSegment(s);
                int toff = off;
                if (t != s) toff = (t && leafIndex(t) < leafIndex(s)) ? t->len - 1 : 0;
                int res = MTR_DETACHED_POSITION;
                if (t) {
                    if (off < 0 || off >= s->len) return status = MTR_ERR_ASSERT | 0x54f;  // "Invalid offset"
                    // findReconnectionPosition(segment, localSeq), client.ts:699-706
                    std::vector<Seg*> lv;
                    leaves(root, lv);
                    int before = 0;
                    for (Seg* x : lv) {
                        if (x == t) break;
                        before += localNetLengthAt(x, currentSeq, op.min_seq);
                    }
                    res = before + toff;
                }
                deltas.push_back({curOpIndex, res, 0, MTR_DELTA_REBASE});
                return status;
            }
            case MTR_OP_LSEQ:  // IntervalCollection.getNextLocalSeq (intervalCollection.ts:1584-1590)
                ++localSeqCounter;
                return status;
            case MTR_OP_START_COLLAB:  // startOrUpdateCollaboration -> startCollaboration, client.ts:1133, mergeTree.ts:731
                if (collaborating) return MTR_OK;
                localClientId = opClient(op);
                minSeq = op.min_seq;
                currentSeq = op.seq;
                collaborating = true;
                heap = Heap();
                nodeUpdateLengthNewStructure(root, true);  // mergeTree.ts:738
                return status;
            default:
                return MTR_ERR_BAD_OP;
        }
        if (status == MTR_OK && (op.flags & MTR_F_LAST)) updateSeqNumbers(op.min_seq, op.seq);
        return status;
    }

    // ------------------------------------------------------------ PermutationVector (matrix)
    bool permMode = false;
    // HandleTable (matrix/src/handletable.ts:19-91): handles[0] = head of the free list
    std::vector<int64_t> handles{1};
    int allocateHandle() {  // handletable.ts:37-42
        const int64_t fr = handles[0];
        handles[0] = size_t(fr) < handles.size() ? handles[size_t(fr)] : fr + 1;
        if (size_t(fr) == handles.size()) handles.push_back(0);
        else handles[size_t(fr)] = 0;
        return int(fr);
    }
    void freeHandle(int h) {  // handletable.ts:57-60
        if (size_t(h) >= handles.size()) handles.resize(size_t(h) + 1, 0);
        handles[size_t(h)] = handles[0];
        handles[0] = h;
    }
    // getContainingSegment, mergeTree.ts:795-813: the leaf holding pos at (refSeq, clientId)
    Seg* containingSegment(int pos, int refSeq, int clientId, int& offset) {
        Seg* found = nullptr;
        offset = 0;
        int p = 0;
        bool exit = false;
        std::vector<Seg*> visit;
        auto collect = [&](Seg* x) { visit.push_back(x); };
        NoPost none;
        walkMap(root, refSeq, clientId, pos, pos + 1, p, exit, collect, none);
        if (!visit.empty()) {
            found = visit[0];
            // position of the leaf in this view: sum of the lengths of the leaves before it
            int before = 0;
            std::vector<Seg*> lv;
            leaves(root, lv);
            for (Seg* x : lv) {
                if (x == found) break;
                const int l = nodeLength(x, refSeq, clientId);
                if (l > 0) before += l;
            }
            offset = pos - before;
        }
        return found;
    }
    // getContainingSegment(pos, {refSeq, this client}, localSeq) (mergeTree.ts:795-813): nodeMap over
    // localNetLength(segment, refSeq, localSeq) (mergeTree.ts:636-662; a block's local partial length is the sum of
    // its leaves')
    Seg* containingSegmentAt(int pos, int refSeq, int lseq, int& offset) {
        std::vector<Seg*> lv;
        leaves(root, lv);
        int p = 0;
        offset = 0;
        for (Seg* x : lv) {
            const int l = localNetLengthAt(x, refSeq, lseq);
            if (l <= 0) continue;
            if (pos < p + l) {
                offset = pos - p;
                return x;
            }
            p += l;
        }
        return nullptr;
    }
    // MergeTree.idToSegment (mergeTree.ts:549,668) by host marker ordinal; never unmapped
    std::unordered_map<uint32_t, Seg*> idToSegment;
    int relPos[2] = {0, 0};
    int relMask = 0;
    // getPosition, mergeTree.ts:768-785: the preceding siblings' nodeLength (undefined = 0) up the
    // parent chain; an unlinked segment (parent undefined, zamboni.ts:146,170) is at 0
    int getPosition(Seg* seg, int refSeq, int clientId) {
        int total = 0;
        Node* prev = seg;
        for (Block* parent = seg->parent; parent; prev = parent, parent = parent->parent) {
            for (int i = 0; i < parent->childCount; i++) {
                Node* child = parent->children[i];
                if (child == prev) break;
                const int l = nodeLength(child, refSeq, clientId);
                if (l > 0) total += l;
            }
        }
        return total;
    }
    // getPosition at the local view, mergeTree.ts:768-785
    int localPosition(Seg* seg) {
        std::vector<Seg*> lv;
        leaves(root, lv);
        int before = 0;
        for (Seg* x : lv) {
            if (x == seg) break;
            const int l = localNetLength(x);
            if (l > 0) before += l;
        }
        return before;
    }
    // PermutationVector.adjustPosition, permutationvector.ts:232-247 (-1 = undefined)
    int adjustPosition(int pos, int refSeq, int clientId) {
        int off = 0;
        Seg* s = containingSegment(pos, refSeq, clientId, off);
        if (!s || s->removed) return -1;
        return localPosition(s) + off;
    }
    // PermutationVector.getAllocatedHandle, permutationvector.ts:209-230: a miss splits out the
    // one-position segment (Client.walkSegments with splitRange -> MergeTree.mapRange,
    // mergeTree.ts:2451-2469, whose `if (start)` skips the split at 0) and allocates its handle
    int getAllocatedHandle(int pos) {
        int off = 0;
        Seg* s = containingSegment(pos, currentSeq, localClientId, off);
        if (s && s->start >= 1) return s->start + off;
        if (pos) ensureIntervalBoundary(pos, currentSeq, localClientId);
        ensureIntervalBoundary(pos + 1, currentSeq, localClientId);
        int h = MTR_HANDLE_UNALLOCATED;
        nodeMap(currentSeq, localClientId, [&](Seg* x) { x->start = h = allocateHandle(); }, pos, pos + 1);
        return h;
    }

    // ------------------------------------------------------------ text
    void gatherText(Block* b, std::u16string& out) {
        for (int i = 0; i < b->childCount; i++) {
            Node* n = b->children[i];
            if (n->leaf) {
                Seg* s = static_cast<Seg*>(n);
                int l = localNetLength(s);
                if (l > 0 && !s->marker) out += s->text;
            } else {
                gatherText(static_cast<Block*>(n), out);
            }
        }
    }

    void leaves(Block* b, std::vector<Seg*>& out) {  // walkAllChildSegments, mergeTreeNodeWalk.ts:170
        for (int i = 0; i < b->childCount; i++) {
            Node* n = b->children[i];
            if (n->leaf)
                out.push_back(static_cast<Seg*>(n));
            else
                leaves(static_cast<Block*>(n), out);
        }
    }
    int height() const {
        int h = 1;
        const Block* b = root;
        while (b->childCount > 0 && !b->children[0]->leaf) {
            b = static_cast<const Block*>(b->children[0]);
            h++;
        }
        return h;
    }
};

// ---------------------------------------------------------------- JSON writer
// JSON.stringify of strings (ES2019 well-formed): escapes, lone surrogates as \udXXX.
struct Out {
    std::string s;
    void raw(const char* p) { s += p; }
    void raw(const std::string& p) { s += p; }
    void bytes(const uint8_t* p, size_t n) { s.append(reinterpret_cast<const char*>(p), n); }
    void num(int64_t v) { s += std::to_string(v); }
    void hex4(unsigned u) {
        static const char* hx = "0123456789abcdef";
        s += "\\u";
        s += hx[(u >> 12) & 15];
        s += hx[(u >> 8) & 15];
        s += hx[(u >> 4) & 15];
        s += hx[u & 15];
    }
    void utf8(uint32_t cp) {
        if (cp < 0x80) {
            s += char(cp);
        } else if (cp < 0x800) {
            s += char(0xC0 | (cp >> 6));
            s += char(0x80 | (cp & 63));
        } else if (cp < 0x10000) {
            s += char(0xE0 | (cp >> 12));
            s += char(0x80 | ((cp >> 6) & 63));
            s += char(0x80 | (cp & 63));
        } else {
            s += char(0xF0 | (cp >> 18));
            s += char(0x80 | ((cp >> 12) & 63));
            s += char(0x80 | ((cp >> 6) & 63));
            s += char(0x80 | (cp & 63));
        }
    }
    void str16(const std::u16string& t) {
        s += '"';
        for (size_t i = 0; i < t.size(); i++) {
            unsigned u = t[i];
            switch (u) {
                case '"': s += "\\\""; continue;
                case '\\': s += "\\\\"; continue;
                case '\b': s += "\\b"; continue;
                case '\f': s += "\\f"; continue;
                case '\n': s += "\\n"; continue;
                case '\r': s += "\\r"; continue;
                case '\t': s += "\\t"; continue;
                default: break;
            }
            if (u < 0x20) {
                hex4(u);
            } else if (u >= 0xD800 && u <= 0xDBFF) {
                if (i + 1 < t.size() && t[i + 1] >= 0xDC00 && t[i + 1] <= 0xDFFF) {
                    uint32_t cp = 0x10000 + ((u - 0xD800) << 10) + (t[i + 1] - 0xDC00);
                    utf8(cp);
                    i++;
                } else {
                    hex4(u);
                }
            } else if (u >= 0xDC00 && u <= 0xDFFF) {
                hex4(u);
            } else {
                utf8(u);
            }
        }
        s += '"';
    }
};

struct Emitter {
    const mtr_batch* b;
    const mtr_doc_desc* dd;
    void longClientId(Out& o, int id) const {  // Client.getLongClientId, client.ts:682-684
        o.raw("\"");
        if (id < 0 || uint32_t(id) >= dd->n_clients) {
            o.raw("original");
        } else {
            uint32_t ix = dd->client_base + uint32_t(id);
            o.bytes(b->client_bytes + b->client_off[ix], b->client_off[ix + 1] - b->client_off[ix]);
        }
        o.raw("\"");
    }
    void props(Out& o, const PropMap& p) const {
        o.raw("{");
        bool first = true;
        for (auto& kv : p.kv) {
            if (!first) o.raw(",");
            first = false;
            o.raw("\"");
            o.bytes(b->key_bytes + b->key_off[kv.first], b->key_off[kv.first + 1] - b->key_off[kv.first]);
            o.raw("\":");
            o.bytes(b->val_bytes + b->val_off[kv.second], b->val_off[kv.second + 1] - b->val_off[kv.second]);
        }
        o.raw("}");
    }
    // toJSONObject: textSegment.ts:73-77, mergeTreeNodes.ts:577-581
    void segJson(Out& o, const Seg* s) const {
        if (s->perm) {  // PermutationSegment.toJSONObject, permutationvector.ts:118-120
            o.raw("[");
            o.num(s->len);
            o.raw(",");
            o.num(s->start);
            o.raw("]");
            return;
        }
        if (s->marker) {
            o.raw("{\"marker\":{");
            if (!s->noRef) {
                o.raw("\"refType\":");
                o.num(s->refType);
            }
            o.raw("}");
            if (s->hasProps) {
                o.raw(",\"props\":");
                props(o, s->props);
            }
            o.raw("}");
        } else if (s->hasProps) {
            o.raw("{\"text\":");
            o.str16(s->text);
            o.raw(",\"props\":");
            props(o, s->props);
            o.raw("}");
        } else {
            o.str16(s->text);
        }
    }
};

struct SpecOut {
    std::string json;
    int len;
};

}  // namespace

// A SharedString document is one Tree.  A SharedMatrix document holds its two PermutationVectors
// (matrix.ts:106-121): rows in `tree`, cols in `cols`; queries read the selected one.
struct oracle_doc {
    Tree tree;
    Tree cols;
    bool matrix = false;
    int sel = 0;
    explicit oracle_doc(const mtr_options& o) : tree(o), cols(o) {}
    Tree& view() { return sel ? cols : tree; }
    // SharedMatrix.processCore, remote branch (matrix.ts:636-693)
    int applyMatrix(const mtr_op& op, const mtr_doc_desc& dd) {
        if (op.type == MTR_OP_START_COLLAB && !(op.flags & MTR_F_APPEND)) {  // didAttach/onConnect start both vectors, matrix.ts:514-532
            int st = tree.apply(op, dd);
            return st != MTR_OK ? st : cols.apply(op, dd);
        }  // (with MTR_F_APPEND: one vector's SnapshotLoader start, routed by MTR_F_COLS below)
        if (op.type == MTR_OP_SETCELL) {
            if (!tree.pendingLoad.empty()) tree.reloadFromSegments();
            if (!cols.pendingLoad.empty()) cols.reloadFromSegments();
            const int client = int(int16_t(op.client));
            const int r = tree.adjustPosition(op.pos1, op.ref_seq, client);
            if (r < 0) return MTR_OK;
            const int c = cols.adjustPosition(op.pos2, op.ref_seq, client);
            if (c < 0) return MTR_OK;
            const int rh = tree.getAllocatedHandle(r);
            const int ch = cols.getAllocatedHandle(c);
            if (rh < 1 || ch < 1) return MTR_ERR_ASSERT | 0x022;  // "row and/or col handles are invalid"
            if (op.flags & MTR_F_DELTA)  // cells.setCell(rowHandle, colHandle, value), matrix.ts:686-689
                tree.deltas.push_back({tree.curOpIndex, rh, ch, MTR_DELTA_CELL});
            return tree.status != MTR_OK ? tree.status : cols.status;
        }
        if (op.type == MTR_OP_LOCAL_SETCELL) {  // setCellCore -> sendSetCellOp (matrix.ts:254-310), this client
            if (!tree.pendingLoad.empty()) tree.reloadFromSegments();
            if (!cols.pendingLoad.empty()) cols.reloadFromSegments();
            if (op.pos1 < 0 || op.pos1 >= tree.blockLocalLength(tree.root) || op.pos2 < 0 ||
                op.pos2 >= cols.blockLocalLength(cols.root))
                return MTR_ERR_ASSERT | 0x01a;  // "Trying to set out-of-bounds cell!"
            const int rh = tree.getAllocatedHandle(op.pos1);
            const int ch = cols.getAllocatedHandle(op.pos2);
            if (tree.collaborating) {  // nextLocalSeq (matrix.ts:484-492): both windows' localSeq advance
                cols.localSeqCounter++;
                tree.localSeqCounter++;
            }
            if (op.flags & MTR_F_DELTA) tree.deltas.push_back({tree.curOpIndex, rh, ch, MTR_DELTA_CELL});
            return tree.status != MTR_OK ? tree.status : cols.status;
        }
        Tree& t = (op.flags & MTR_F_COLS) ? cols : tree;
        const int st = t.apply(op, dd);
        // submitVectorMessage (matrix.ts:321-345): a local row / col op brings the other vector's localSeq along
        if (st == MTR_OK && t.collaborating && op.type >= MTR_OP_LOCAL_INSERT && op.type <= MTR_OP_LOCAL_ANNOTATE) {
            Tree& o = (op.flags & MTR_F_COLS) ? tree : cols;
            if (t.localSeqCounter < o.localSeqCounter) return MTR_ERR_ASSERT | 0x01c;
            o.localSeqCounter = t.localSeqCounter;
        }
        return st;
    }
};

extern "C" {

void oracle_set_psl_check(int on) {
    g_psl = on;
    g_psl_checks = 0;
    g_psl_mismatch = 0;
    g_psl_rootlag = 0;
    std::lock_guard<std::mutex> g(g_psl_mu);
    g_psl_first.clear();
}

int64_t oracle_psl_stats(int64_t* out, char* first, int64_t cap) {
    out[0] = g_psl_checks.load();
    out[1] = g_psl_mismatch.load();
    out[2] = g_psl_rootlag.load();
    std::lock_guard<std::mutex> g(g_psl_mu);
    if (first && cap > 0) {
        const size_t n = std::min<size_t>(size_t(cap) - 1, g_psl_first.size());
        std::memcpy(first, g_psl_first.data(), n);
        first[n] = 0;
    }
    return out[1];
}

void oracle_set_trace(int on) {
    g_trace = on;
    const char* ts = getenv("MTR_TRACE_SEQ");
    g_trace_seq = ts ? atoi(ts) : -1;
}

oracle_doc* oracle_doc_new(const mtr_options* opt) {
    mtr_options o{0, 1, 10000, 0};
    if (opt) o = *opt;
    if (o.chunk_size <= 0) o.chunk_size = 10000;
    return new oracle_doc(o);
}

void oracle_doc_free(oracle_doc* d) { delete d; }

oracle_doc* oracle_doc_new_matrix(const mtr_options* opt) {
    oracle_doc* d = oracle_doc_new(opt);
    d->matrix = true;
    d->tree.permMode = true;
    d->cols.permMode = true;
    return d;
}

void oracle_doc_select(oracle_doc* d, int32_t which) { d->sel = d->matrix && which ? 1 : 0; }

int oracle_doc_apply(oracle_doc* d, const mtr_batch* b, uint32_t doc_index, uint32_t op_lo, uint32_t op_hi) {
    Tree& t = d->tree;
    t.tabs.b = b;
    d->cols.tabs.b = b;
    const mtr_doc_desc& dd = b->docs[doc_index];
    if (op_hi > dd.op_count) op_hi = dd.op_count;
    if (d->matrix) {  // the engine tracks a matrix's cells in a batch with any flagged op
        bool any = false;
        for (uint32_t i = op_lo; i < op_hi; i++) any = any || (b->ops[dd.op_begin + i].flags & MTR_F_DELTA);
        t.recycleLog = d->cols.recycleLog = any;
    }
    for (uint32_t i = op_lo; i < op_hi; i++) {
        const mtr_op& op = b->ops[dd.op_begin + i];
        t.curOpIndex = i;
        d->cols.curOpIndex = i;
        t.deltaOn = !d->matrix && (op.flags & MTR_F_DELTA) != 0;
        int st = d->matrix ? d->applyMatrix(op, dd) : t.apply(op, dd);
        t.deltaOn = false;
        if (st != MTR_OK) return st;
    }
    return d->matrix ? (t.status != MTR_OK ? t.status : d->cols.status) : t.status;
}

// the properties of an MTR_DELTA_REGEN_X record's reference as [n, key, value, ...] (n = 2n + 1 words)
int64_t oracle_doc_regen_props(oracle_doc* d, uint32_t ref, uint32_t* out, int64_t cap) {
    Tree& t = d->view();
    if (ref >= t.regenProps.size()) return -1;
    const PropMap& m = t.regenProps[ref].second;
    const int64_t n = 1 + 2 * int64_t(m.kv.size());
    if (n > cap) return -n;
    out[0] = uint32_t(m.kv.size());
    for (size_t k = 0; k < m.kv.size(); k++) {
        out[1 + 2 * k] = m.kv[k].first;
        out[2 + 2 * k] = m.kv[k].second;
    }
    return n;
}

int64_t oracle_doc_deltas(oracle_doc* d, mtr_delta* out, int64_t cap) {
    std::vector<mtr_delta>& v = d->view().deltas;
    const int64_t n = int64_t(v.size());
    if (n > cap) return -n;
    if (n) std::memcpy(out, v.data(), size_t(n) * sizeof(mtr_delta));
    v.clear();
    return n;
}

int64_t oracle_doc_text(oracle_doc* d, uint16_t* out, int64_t cap) {
    if (!d->view().pendingLoad.empty()) d->view().reloadFromSegments();
    std::u16string s;
    d->view().gatherText(d->view().root, s);
    int64_t n = int64_t(s.size());
    if (out) std::memcpy(out, s.data(), size_t(std::min(n, cap)) * 2);
    return n;
}

int32_t oracle_doc_pending_groups(oracle_doc* d) { return int32_t(d->view().pendingSegments.size()); }

int32_t oracle_doc_containing(oracle_doc* d, int32_t pos, int32_t ref_seq, int32_t client, int32_t* out) {
    Tree& t = d->view();
    int off = 0;
    Seg* s = t.containingSegment(pos, ref_seq, client, off);
    if (!s) {
        out[0] = -1;
        return -1;
    }
    out[0] = t.leafIndex(s);
    out[1] = off;
    out[2] = s->len;
    out[3] = pos - off;
    return out[0];
}

int64_t oracle_doc_containing_props(oracle_doc* d, int32_t pos, int32_t ref_seq, int32_t client, uint32_t* out,
                                    int64_t cap) {
    Tree& t = d->view();
    int off = 0;
    Seg* s = t.containingSegment(pos, ref_seq, client, off);
    if (!s) return -1;
    const int64_t n = 3 + 2 * int64_t(s->props.kv.size());
    if (n > cap) return -n;
    out[0] = uint32_t(s->groups.size());
    out[1] = s->hasProps ? 1u : 0u;
    out[2] = uint32_t(s->props.kv.size());
    for (size_t k = 0; k < s->props.kv.size(); k++) {
        out[3 + 2 * k] = s->props.kv[k].first;
        out[4 + 2 * k] = s->props.kv[k].second;
    }
    return n;
}

int64_t oracle_doc_ref_positions(oracle_doc* d, int32_t* out, int64_t cap) {
    Tree& t = d->view();
    if (!t.pendingLoad.empty()) t.reloadFromSegments();
    const int64_t n = int64_t(t.refs.size());
    if (n > cap) return -n;
    for (int64_t i = 0; i < n; i++) out[i] = t.refPosition(int(i));
    return n;
}

int32_t oracle_doc_ref_info(oracle_doc* d, uint32_t id, int32_t* out) {
    Tree& t = d->view();
    if (id >= t.refs.size()) return -1;
    const LRef& r = t.refs[id];
    Seg* s = r.segment;
    out[0] = s && s->parent ? t.leafIndex(s) : -1;
    out[1] = r.offset;
    out[2] = r.refType;
    out[3] = (s && s->localRefs && t.refsHas(s->localRefs, int(id))) ? 1 : 0;
    return out[0];
}

int64_t oracle_doc_ref_states(oracle_doc* d, int32_t* out, int64_t cap) {
    Tree& t = d->view();
    if (!t.pendingLoad.empty()) t.reloadFromSegments();
    const int64_t n = int64_t(t.refs.size());
    if (2 * n > cap) return -n;
    for (int64_t i = 0; i < n; i++) {
        const LRef& r = t.refs[size_t(i)];
        Seg* s = r.segment;
        const bool held = s && s->localRefs && t.refsHas(s->localRefs, int(i));
        const bool live = held || (r.refType & MTR_REFTYPE_TRANSIENT);
        out[2 * i] = t.refPosition(int(i));
        out[2 * i + 1] = (s ? MTR_REF_ST_SEGMENT : 0) | (held ? MTR_REF_ST_HELD : 0) |
                         (live && s && s->parent && s->removed ? MTR_REF_ST_REMOVED : 0);
    }
    return n;
}

// every reference as {position, state, compare key (leaf index; -1 no segment, -2 unlinked), offset}: mtr_get_ref_keys
int64_t oracle_doc_ref_keys(oracle_doc* d, int32_t* out, int64_t cap) {
    Tree& t = d->view();
    if (!t.pendingLoad.empty()) t.reloadFromSegments();
    const int64_t n = int64_t(t.refs.size());
    if (4 * n > cap) return -n;
    std::vector<int32_t> st(size_t(2 * n));
    oracle_doc_ref_states(d, st.data(), 2 * n);
    for (int64_t i = 0; i < n; i++) {
        const LRef& r = t.refs[size_t(i)];
        Seg* s = r.segment;
        out[4 * i] = st[size_t(2 * i)];
        out[4 * i + 1] = st[size_t(2 * i + 1)];
        out[4 * i + 2] = !s ? -1 : s->parent ? t.leafIndex(s) : -2;
        out[4 * i + 3] = r.offset;
    }
    return n;
}

int32_t oracle_doc_ref_key(oracle_doc* d, uint32_t id, int32_t* out) {
    Tree& t = d->view();
    if (id >= t.refs.size()) return -3;
    const LRef& r = t.refs[id];
    Seg* s = r.segment;
    out[0] = !s ? -1 : s->parent ? t.leafIndex(s) : -2;
    out[1] = r.offset;
    return out[0];
}

void oracle_doc_set_slide_hook(oracle_doc* d, oracle_slide_hook hook, void* ctx) {
    d->tree.slideHook = d->cols.slideHook = hook;
    d->tree.slideCtx = d->cols.slideCtx = ctx;
}

int32_t oracle_doc_handle_at(oracle_doc* d, int32_t pos) {
    Tree& t = d->view();
    if (!t.pendingLoad.empty()) t.reloadFromSegments();
    int off = 0;
    Seg* s = t.containingSegment(pos, t.currentSeq, t.localClientId, off);
    if (!s) return -1;
    return s->start >= 1 ? s->start + off : MTR_HANDLE_UNALLOCATED;
}

// the selected vector's segments in tree order, five int32 each, as mtr_get_leaves (include/mtr.h)
int64_t oracle_doc_leaves(oracle_doc* d, int32_t* out, int64_t cap) {
    Tree& t = d->view();
    if (!t.pendingLoad.empty()) t.reloadFromSegments();
    std::vector<Seg*> lv;
    t.leaves(t.root, lv);
    if (int64_t(lv.size()) > cap) return -int64_t(lv.size());
    for (size_t i = 0; i < lv.size(); i++) {
        const Seg* x = lv[i];
        int32_t* r = out + 5 * i;
        r[0] = x->len;
        r[1] = x->removed ? 1 : 0;
        r[2] = x->start;
        r[3] = x->tid;
        r[4] = int32_t(t.tbits(x));
    }
    return int64_t(lv.size());
}

// the tracking ids of group `bit`'s segments in the TrackingGroup's order (test check of the host's lists)
int64_t oracle_doc_track_group(oracle_doc* d, int32_t bit, int32_t* out, int64_t cap) {
    Tree& t = d->view();
    if (bit < 0 || bit >= MTR_TRACK_GROUPS) return -1;
    const std::vector<Seg*>& g = t.tgroup[bit].segs;
    if (int64_t(g.size()) > cap) return -int64_t(g.size());
    for (size_t i = 0; i < g.size(); i++) out[i] = g[i]->tid;
    return int64_t(g.size());
}

int32_t oracle_doc_marker_position(oracle_doc* d, uint32_t ordinal, int32_t ref_seq, int32_t client) {
    if (!d->view().pendingLoad.empty()) d->view().reloadFromSegments();
    Tree& t = d->view();
    auto it = t.idToSegment.find(ordinal);
    return it == t.idToSegment.end() ? -1 : t.getPosition(it->second, ref_seq, client);
}

int64_t oracle_doc_length(oracle_doc* d, int32_t ref_seq, int32_t client) {
    if (!d->view().pendingLoad.empty()) d->view().reloadFromSegments();
    return d->view().nodeLength(d->view().root, ref_seq, client);
}

void oracle_doc_state(oracle_doc* d, int64_t* out) {
    if (!d->view().pendingLoad.empty()) d->view().reloadFromSegments();
    Tree& t = d->view();
    std::vector<Seg*> lv;
    t.leaves(t.root, lv);
    out[0] = t.minSeq;
    out[1] = t.currentSeq;
    out[2] = t.heap.count();
    out[3] = int64_t(lv.size());
}

int64_t oracle_doc_export(oracle_doc* d, int32_t* out, int64_t cap, int32_t* height) {
    if (!d->view().pendingLoad.empty()) d->view().reloadFromSegments();
    Tree& t = d->view();
    std::vector<Seg*> lv;
    t.leaves(t.root, lv);
    if (height) *height = t.height();
    if (int64_t(lv.size()) > cap) return -int64_t(lv.size());
    for (size_t i = 0; i < lv.size(); i++) {
        Seg* s = lv[i];
        int bnd = 0;
        const Node* n = s;
        while (n->parent && n->index == 0) {
            bnd++;
            n = n->parent;
        }
        if (!n->parent) {
            // reached the root through first children: counts every level
        }
        uint32_t h = 2166136261u;
        if (s->hasProps) {
            h ^= 1u;
            for (auto& kv : s->props.kv) {
                h = (h ^ kv.first) * 16777619u;
                h = (h ^ t.tabs.b->val_eq[kv.second]) * 16777619u;
            }
        }
        int32_t* r = out + 8 * i;
        r[0] = s->len;
        r[1] = s->seq;
        r[2] = s->clientId;
        r[3] = s->removed ? s->removedSeq : INT32_MIN;
        r[4] = int32_t(s->removedClientIds.size());
        r[5] = bnd;
        r[6] = s->perm ? s->start : (s->marker ? 1 : 0);  // PermutationSegment: its start handle
        r[7] = int32_t(s->hasProps ? h : 0);
    }
    return int64_t(lv.size());
}

// Client.summarize (client.ts:966-1000) with SnapshotV1 (snapshotV1.ts:122-298) or
// SnapshotLegacy (snapshotlegacy.ts:122-255) and the chunk serializers (snapshotChunks.ts:86-149).
int64_t oracle_doc_summarize(oracle_doc* d, const mtr_batch* b, uint32_t doc_index, uint8_t* out, int64_t cap,
                             int64_t* blob_len, int32_t max_blobs) {
    if (!d->view().pendingLoad.empty()) d->view().reloadFromSegments();
    Tree& t = d->view();
    t.tabs.b = b;
    Emitter em{b, &b->docs[doc_index]};
    const int minSeq = t.minSeq;
    const int chunk = t.opt.chunk_size;
    std::vector<Seg*> lv;
    t.leaves(t.root, lv);
    std::vector<std::string> blobs;

    // coalesce helper state: prev is a (clone of a) segment, text accumulated in prevText
    struct Prev {
        bool has = false;
        Seg seg;  // clone
    } prev;
    std::vector<SpecOut> specs;
    auto pushPrev = [&]() {
        if (prev.has) {
            Out o;
            em.segJson(o, &prev.seg);
            specs.push_back({o.s, prev.seg.len});
        }
    };
    auto takePrev = [&](Seg* s) {
        prev.has = true;
        prev.seg = *s;
    };

    if (t.opt.snapshot_v1) {
        for (Seg* s : lv) {  // extractSync, snapshotV1.ts:180-298
            if (s->seq == kUnassignedSeq || (s->removed && s->removedSeq <= minSeq)) continue;
            if (s->seq <= minSeq && (!s->removed || s->removedSeq == kUnassignedSeq)) {
                if (!prev.has) {
                    takePrev(s);
                } else if (Tree::canAppend(&prev.seg, s) && matchProperties(&prev.seg, s, b)) {
                    prev.seg.text += s->text;
                    prev.seg.len += s->len;
                } else {
                    pushPrev();
                    takePrev(s);
                }
            } else {
                pushPrev();
                prev.has = false;
                Out o;
                o.raw("{\"json\":");
                em.segJson(o, s);
                if (s->seq > minSeq) {
                    o.raw(",\"seq\":");
                    o.num(s->seq);
                    o.raw(",\"client\":");
                    em.longClientId(o, s->clientId);
                }
                if (s->removed) {
                    o.raw(",\"removedSeq\":");
                    o.num(s->removedSeq);
                    o.raw(",\"removedClient\":");
                    em.longClientId(o, s->removedClientIds[0]);
                    o.raw(",\"removedClientIds\":[");
                    for (size_t k = 0; k < s->removedClientIds.size(); k++) {
                        if (k) o.raw(",");
                        em.longClientId(o, s->removedClientIds[k]);
                    }
                    o.raw("]");
                }
                o.raw("}");
                specs.push_back({o.s, s->len});
            }
        }
        pushPrev();
        // emit, snapshotV1.ts:122-178
        struct Chunk {
            size_t start, count;
            int64_t length;
        };
        std::vector<Chunk> chunks;
        size_t total = 0;
        int64_t totalLen = 0;
        do {
            Chunk c{total, 0, 0};
            while (c.length < chunk && c.start + c.count < specs.size()) {
                c.length += specs[c.start + c.count].len;
                c.count++;
            }
            chunks.push_back(c);
            total += c.count;
            totalLen += c.length;
        } while (total < specs.size());
        auto segList = [&](Out& o, const Chunk& c) {
            o.raw("[");
            for (size_t k = 0; k < c.count; k++) {
                if (k) o.raw(",");
                o.raw(specs[c.start + k].json);
            }
            o.raw("]");
        };
        auto chunkHead = [&](Out& o, const Chunk& c) {
            o.raw("{\"version\":\"1\",\"segmentCount\":");
            o.num(int64_t(c.count));
            o.raw(",\"length\":");
            o.num(c.length);
            o.raw(",\"segments\":");
            segList(o, c);
            o.raw(",\"startIndex\":");
            o.num(int64_t(c.start));
        };
        Out h;
        chunkHead(h, chunks[0]);
        h.raw(",\"headerMetadata\":{\"minSequenceNumber\":");
        h.num(minSeq);
        h.raw(",\"sequenceNumber\":");
        h.num(t.currentSeq);
        h.raw(",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
        for (size_t k = 1; k < chunks.size(); k++) {
            h.raw(",{\"id\":\"body_");
            h.num(int64_t(k - 1));
            h.raw("\"}");
        }
        h.raw("],\"totalLength\":");
        h.num(totalLen);
        h.raw(",\"totalSegmentCount\":");
        h.num(int64_t(total));
        h.raw("}}");
        blobs.push_back(h.s);
        for (size_t k = 1; k < chunks.size(); k++) {
            Out o;
            chunkHead(o, chunks[k]);
            o.raw("}");
            blobs.push_back(o.s);
        }
    } else {
        // extractSync, snapshotlegacy.ts:184-255: mapRange(minSeq, NonCollabClient)
        // (nodeMap with the default end: the root's own length at (minSeq, NonCollabClient))
        std::vector<SpecOut> segs;
        const int cid = kNonCollabClient;
        t.nodeMap(
            minSeq, cid,
            [&](Seg* s) {
                if (s->seq != kUnassignedSeq && s->seq <= minSeq &&
                    (!s->removed || s->removedSeq == kUnassignedSeq || s->removedSeq > minSeq)) {
                    if (prev.has && Tree::canAppend(&prev.seg, s) && matchProperties(&prev.seg, s, b)) {
                        prev.seg.text += s->text;
                        prev.seg.len += s->len;
                    } else {
                        pushPrev();
                        takePrev(s);
                    }
                }
            },
            0, -1);
        pushPrev();
        int64_t totalLen = 0;
        for (auto& sp : specs) totalLen += sp.len;
        auto getChunk = [&](int64_t approx, size_t start, size_t& count, int64_t& length) {
            count = 0;
            length = 0;
            while (length < approx && start + count < specs.size()) {
                length += specs[start + count].len;
                count++;
            }
        };
        auto body = [&](Out& o, size_t start, size_t count, int64_t length) {
            o.raw("{\"chunkStartSegmentIndex\":");
            o.num(int64_t(start));
            o.raw(",\"chunkSegmentCount\":");
            o.num(int64_t(count));
            o.raw(",\"chunkLengthChars\":");
            o.num(length);
            o.raw(",\"totalLengthChars\":");
            o.num(totalLen);
            o.raw(",\"totalSegmentCount\":");
            o.num(int64_t(specs.size()));
            o.raw(",\"chunkSequenceNumber\":");
            o.num(minSeq);
            o.raw(",\"segmentTexts\":[");
            for (size_t k = 0; k < count; k++) {
                if (k) o.raw(",");
                o.raw(specs[start + k].json);
            }
            o.raw("]");
        };
        size_t c1n;
        int64_t c1l;
        getChunk(chunk, 0, c1n, c1l);
        Out h;
        body(h, 0, c1n, c1l);
        h.raw(",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}");
        if (c1l < totalLen) h.raw(",{\"id\":\"body\"}");
        h.raw("],\"sequenceNumber\":");
        h.num(minSeq);
        h.raw(",\"totalLength\":");
        h.num(totalLen);
        h.raw(",\"totalSegmentCount\":");
        h.num(int64_t(specs.size()));
        h.raw("}}");
        blobs.push_back(h.s);
        if (c1n < specs.size()) {
            size_t c2n;
            int64_t c2l;
            getChunk(totalLen, c1n, c2n, c2l);
            Out o;
            body(o, c1n, c2n, c2l);
            o.raw("}");
            blobs.push_back(o.s);
        }
    }
    if (d->matrix) {  // PermutationVector.summarize, permutationvector.ts:310-325: + the handleTable blob
        Out o;
        o.raw("[");
        for (size_t k = 0; k < t.handles.size(); k++) {
            if (k) o.raw(",");
            o.num(t.handles[k]);
        }
        o.raw("]");
        blobs.push_back(o.s);
    }
    int64_t need = 0;
    for (auto& s : blobs) need += int64_t(s.size());
    if (need > cap || int32_t(blobs.size()) > max_blobs) return -need;
    int64_t off = 0;
    for (size_t k = 0; k < blobs.size(); k++) {
        std::memcpy(out + off, blobs[k].data(), blobs[k].size());
        blob_len[k] = int64_t(blobs[k].size());
        off += int64_t(blobs[k].size());
    }
    return int64_t(blobs.size());
}


// Summary digest of include/mtr_digest.h over nblobs and every blob (the same value the engine's
// summary_write_kernel computes).
static uint64_t summary_hash(const std::vector<std::string>& blobs) {
    uint64_t h = mtr_dg_begin(uint64_t(blobs.size()));
    for (auto& b : blobs) h = mtr_dg_next(h, mtr_dg_blob_bytes((const uint8_t*)b.data(), uint64_t(b.size())));
    return h;
}

// Replay documents [lo, hi) of a batch on `nthreads` host threads (one document per task),
// summarize each and record its digest; returns wall-clock seconds.
double oracle_replay_batch(const mtr_batch* b, const mtr_options* opt, uint32_t lo, uint32_t hi, int nthreads,
                           uint64_t* hashes, int32_t* status) {
    std::atomic<uint32_t> next{lo};
    auto t0 = std::chrono::steady_clock::now();
    auto work = [&]() {
        std::vector<uint8_t> out(1 << 16);
        std::vector<int64_t> lens(4096);
        for (;;) {
            uint32_t d = next.fetch_add(1);
            if (d >= hi) break;
            oracle_doc* doc = oracle_doc_new(opt);
            int st = oracle_doc_apply(doc, b, d, 0, b->docs[d].op_count);
            uint64_t h = 0;
            if (st == MTR_OK) {
                int64_t r;
                while ((r = oracle_doc_summarize(doc, b, d, out.data(), int64_t(out.size()), lens.data(), 4096)) < 0)
                    out.resize(size_t(-r) + 16);
                std::vector<std::string> blobs;
                int64_t off = 0;
                for (int64_t k = 0; k < r; k++) {
                    blobs.emplace_back(reinterpret_cast<const char*>(out.data() + off), size_t(lens[k]));
                    off += lens[k];
                }
                h = summary_hash(blobs);
            }
            if (hashes) hashes[d - lo] = h;
            if (status) status[d - lo] = st;
            oracle_doc_free(doc);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, nthreads); t++) th.emplace_back(work);
    for (auto& t : th) t.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// SharedMatrix replay (the CPU leg of the C4 bench and its parity check): matrices [lo, hi) of a
// batch with one document per matrix (its rows vector's op list, as oracle_generate_matrix writes
// it), each applied to a fresh matrix observer (SharedMatrix.processCore, matrix.ts:636-693) and
// summarized per vector (PermutationVector.summarize, permutationvector.ts:310-325).  hashes[2m] /
// hashes[2m + 1] = digest of the rows / cols vector's blobs; returns wall-clock seconds.
double oracle_replay_matrix_batch(const mtr_batch* b, const mtr_options* opt, uint32_t lo, uint32_t hi,
                                  int nthreads, uint64_t* hashes, int32_t* status) {
    std::atomic<uint32_t> next{lo};
    auto t0 = std::chrono::steady_clock::now();
    auto work = [&]() {
        std::vector<uint8_t> out(1 << 16);
        std::vector<int64_t> lens(4096);
        for (;;) {
            const uint32_t d = next.fetch_add(1);
            if (d >= hi) break;
            oracle_doc* doc = oracle_doc_new_matrix(opt);
            const int st = oracle_doc_apply(doc, b, d, 0, b->docs[d].op_count);
            for (int w = 0; w < 2; w++) {
                uint64_t h = 0;
                if (st == MTR_OK) {
                    oracle_doc_select(doc, w);
                    int64_t r;
                    while ((r = oracle_doc_summarize(doc, b, d, out.data(), int64_t(out.size()), lens.data(), 4096)) < 0)
                        out.resize(size_t(-r) + 16);
                    std::vector<std::string> blobs;
                    int64_t off = 0;
                    for (int64_t k = 0; k < r; k++) {
                        blobs.emplace_back(reinterpret_cast<const char*>(out.data() + off), size_t(lens[k]));
                        off += lens[k];
                    }
                    h = summary_hash(blobs);
                }
                if (hashes) hashes[2 * size_t(d - lo) + w] = h;
            }
            if (status) status[d - lo] = st;
            oracle_doc_free(doc);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, nthreads); t++) th.emplace_back(work);
    for (auto& t : th) t.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Synthetic op logs (include/mtr_synth.h) with the oracle as the exact simulator.
// SharedMatrix op logs from the matrix recipe (mtr_synth_matrix_finish), one document per task;
// per document: ops_per_doc + 1 records (START_COLLAB first); no text.  Digests are over the rows
// vector's blobs followed by the cols vector's.
int oracle_generate_matrix(const mtr_synth_cfg* cfg, const mtr_batch* tables, const mtr_options* opt, uint32_t lo,
                           uint32_t hi, int nthreads, mtr_op* ops_out, uint64_t* hashes, int32_t* status) {
    std::atomic<uint32_t> next{lo};
    const uint32_t per = cfg->ops_per_doc + 1;
    auto work = [&]() {
        std::vector<uint8_t> out(1 << 16);
        std::vector<int64_t> lens(4096);
        uint16_t dummy_text[1] = {0};
        for (;;) {
            const uint32_t d = next.fetch_add(1);
            if (d >= hi) break;
            const uint32_t r = d - lo;
            mtr_op* ops = ops_out + size_t(r) * per;
            mtr_batch b = *tables;
            mtr_doc_desc dd{};
            dd.op_count = per;
            dd.n_clients = cfg->writers + 1;
            b.n_docs = 1;
            b.docs = &dd;
            b.ops = ops;
            b.text = dummy_text;
            oracle_doc* doc = oracle_doc_new_matrix(opt);
            doc->tree.tabs.b = &b;
            doc->cols.tabs.b = &b;
            mtr_synth_state st;
            mtr_synth_init(cfg, d, &st);
            std::memset(ops, 0, sizeof(mtr_op) * per);
            ops[0].type = MTR_OP_START_COLLAB;
            int rc = doc->applyMatrix(ops[0], dd);
            for (uint32_t k = 1; k < per && rc == MTR_OK; k++) {
                mtr_op& op = ops[k];
                mtr_synth_begin(cfg, &st, int32_t(k), &op);
                const int Lr = std::max(0, doc->tree.nodeLength(doc->tree.root, op.ref_seq, op.client));
                const int Lc = std::max(0, doc->cols.nodeLength(doc->cols.root, op.ref_seq, op.client));
                mtr_synth_matrix_finish(cfg, &st, Lr, Lc, &op);
                rc = doc->applyMatrix(op, dd);
            }
            uint64_t h = 0;
            if (rc == MTR_OK && hashes) {
                std::vector<std::string> blobs;
                for (int w = 0; w < 2; w++) {
                    oracle_doc_select(doc, w);
                    int64_t nb;
                    while ((nb = oracle_doc_summarize(doc, &b, 0, out.data(), int64_t(out.size()), lens.data(), 4096)) < 0)
                        out.resize(size_t(-nb) + 16);
                    int64_t off = 0;
                    for (int64_t k = 0; k < nb; k++) {
                        blobs.emplace_back(reinterpret_cast<const char*>(out.data() + off), size_t(lens[k]));
                        off += lens[k];
                    }
                }
                h = summary_hash(blobs);
            }
            if (hashes) hashes[r] = h;
            if (status) status[r] = rc;
            oracle_doc_free(doc);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, nthreads); t++) th.emplace_back(work);
    for (auto& x : th) x.join();
    return MTR_OK;
}

// The recipe of include/mtr_synth.h driven by this oracle.  With grow > 0 every document first
// loads `grow` two-unit segments as a summary header (MTR_OP_LOAD, reloadFromSegments) before
// collaboration starts: the pre-grown documents of config C5.  Per document:
// grow + 1 + ops_per_doc records; text capacity cfg->text_cap units (>= 2 * grow + inserts).
static int generate_impl(const mtr_synth_cfg* cfg, const mtr_batch* tables, const mtr_options* opt, uint32_t lo,
                         uint32_t hi, int nthreads, uint32_t grow, mtr_op* ops_out, uint16_t* text_out,
                         uint32_t* text_counts, uint64_t* hashes, int32_t* status) {
    std::atomic<uint32_t> next{lo};
    const uint32_t per = grow + cfg->ops_per_doc + 1;
    auto work = [&]() {
        std::vector<uint8_t> out(1 << 16);
        std::vector<int64_t> lens(4096);
        for (;;) {
            const uint32_t d = next.fetch_add(1);
            if (d >= hi) break;
            const uint32_t r = d - lo;
            mtr_op* ops = ops_out + size_t(r) * per;
            uint16_t* text = text_out + size_t(r) * cfg->text_cap;
            mtr_batch b = *tables;
            mtr_doc_desc dd{};
            dd.op_begin = 0;
            dd.op_count = per;
            dd.text_base = 0;
            dd.client_base = 0;
            dd.n_clients = cfg->writers + 1;
            b.n_docs = 1;
            b.docs = &dd;
            b.ops = ops;
            b.text = text;
            oracle_doc* doc = oracle_doc_new(opt);
            doc->tree.tabs.b = &b;
            mtr_synth_state st;
            mtr_synth_init(cfg, d, &st);
            std::memset(ops, 0, sizeof(mtr_op) * per);
            int rc = MTR_OK;
            for (uint32_t k = 0; k < grow && rc == MTR_OK; k++) {  // snapshot header segments
                mtr_op& op = ops[k];
                op.type = MTR_OP_LOAD;
                op.client = uint16_t(MTR_CLIENT_NONCOLLAB);
                op.ref_seq = -1;
                op.pos2 = -1;
                op.payload = 2 * k;
                op.payload2 = 2;
                text[2 * k] = uint16_t('a' + k % 26);
                text[2 * k + 1] = uint16_t('A' + (k / 26) % 26);
                rc = doc->tree.apply(op, dd);
            }
            st.text_used = 2 * grow;
            ops[grow].type = MTR_OP_START_COLLAB;
            if (rc == MTR_OK) rc = doc->tree.apply(ops[grow], dd);
            for (uint32_t k = 1; k <= cfg->ops_per_doc && rc == MTR_OK; k++) {
                mtr_op& op = ops[grow + k];
                mtr_synth_begin(cfg, &st, int32_t(k), &op);
                const int L = std::max(0, doc->tree.nodeLength(doc->tree.root, op.ref_seq, op.client));
                mtr_synth_finish(cfg, &st, L, &op, text);
                rc = doc->tree.apply(op, dd);
            }
            dd.text_count = st.text_used;
            if (text_counts) text_counts[r] = st.text_used;
            uint64_t h = 0;
            if (rc == MTR_OK && hashes) {
                int64_t nb;
                while ((nb = oracle_doc_summarize(doc, &b, 0, out.data(), int64_t(out.size()), lens.data(), 4096)) < 0)
                    out.resize(size_t(-nb) + 16);
                std::vector<std::string> blobs;
                int64_t off = 0;
                for (int64_t k = 0; k < nb; k++) {
                    blobs.emplace_back(reinterpret_cast<const char*>(out.data() + off), size_t(lens[k]));
                    off += lens[k];
                }
                h = summary_hash(blobs);
            }
            if (hashes) hashes[r] = h;
            if (status) status[r] = rc;
            oracle_doc_free(doc);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, nthreads); t++) th.emplace_back(work);
    for (auto& t : th) t.join();
    return 0;
}

int oracle_generate(const mtr_synth_cfg* cfg, const mtr_batch* tables, const mtr_options* opt, uint32_t lo,
                    uint32_t hi, int nthreads, mtr_op* ops_out, uint16_t* text_out, uint32_t* text_counts,
                    uint64_t* hashes, int32_t* status) {
    return generate_impl(cfg, tables, opt, lo, hi, nthreads, 0, ops_out, text_out, text_counts, hashes, status);
}

int oracle_generate_grown(const mtr_synth_cfg* cfg, const mtr_batch* tables, const mtr_options* opt, uint32_t lo,
                          uint32_t hi, int nthreads, uint32_t grow, mtr_op* ops_out, uint16_t* text_out,
                          uint32_t* text_counts, uint64_t* hashes, int32_t* status) {
    return generate_impl(cfg, tables, opt, lo, hi, nthreads, grow, ops_out, text_out, text_counts, hashes, status);
}

}  // extern "C"
