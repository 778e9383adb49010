// psl.h -- PartialSequenceLengths restated for the oracle (TEST INFRASTRUCTURE ONLY, included by
// mtr_oracle.cpp after the Seg / Block definitions).
//
// The oracle answers a block's length in a remote (refSeq, clientId) view with the sum of its
// leaves' nodeLength.  The reference answers it with the block's PartialSequenceLengths
// (mergeTree.ts:928-931 -> partialLengths.ts:698-735), maintained incrementally at the call sites of
// mergeTree.ts / zamboni.ts.  This file restates that structure rule for rule so the oracle can keep
// one per block, update it where the reference does, and assert at every block-length query that
// the two answers agree (the reference's own check is test/testUtils.ts:209-248).
// Paths are relative to packages/dds/merge-tree/src/.  Local (unacked) records are not modelled: an
// observer has none.
#pragma once

#include <map>
#include <memory>
#include <vector>

// PartialSequenceLength (partialLengths.ts:105-150).  Sets own their entries (the reference never
// shares an entry object between two sets: mergePartialLengths and addClientSeqNumber copy).
struct PSLEntry {
    int seq = 0;
    int64_t len = 0;
    int64_t seglen = 0;
    int clientId = 0;
    bool hasClient = false;
    bool hasOverlap = false;
    std::map<int, int64_t> overlap;  // overlapRemoveClients: RedBlackTree<clientId, {clientId, seglen}>
};

// overlapRemoveClients helpers (partialLengths.ts:977-998)
inline void combineOverlapClients(PSLEntry& a, const PSLEntry& b) {
    if (a.hasOverlap) {
        if (b.hasOverlap)
            for (const auto& kv : b.overlap) a.overlap[kv.first] += kv.second;  // get(..) ? += : put(copy)
    } else if (b.hasOverlap) {
        a.hasOverlap = true;
        a.overlap = b.overlap;  // cloneOverlapRemoveClients
    }
}

// SortedSet (sortedSet.ts:6-80) keyed by seq + PartialSequenceLengthsSet (partialLengths.ts:19-95)
struct PSLSet {
    std::vector<PSLEntry> items;

    struct Pos {
        bool exists;
        int index;
    };
    // SortedSet.findItemPosition, sortedSet.ts:46-76 (its exact binary-search exits)
    Pos find(int key) const {
        if (items.empty()) return {false, 0};
        int start = 0, end = int(items.size()) - 1, index = -1;
        while (start <= end) {
            index = start + (end - start) / 2;
            const int k = items[size_t(index)].seq;
            if (k > key) {
                if (start == index) return {false, index};
                end = index - 1;
            } else if (k < key) {
                if (index == end) return {false, index + 1};
                start = index + 1;
            } else {
                return {true, index};
            }
        }
        return {false, index};
    }
    int latestLeqIndex(int key) const {  // partialLengths.ts:71-74
        const Pos p = find(key);
        return p.exists ? p.index : p.index - 1;
    }
    PSLEntry* latestLeq(int key) {  // partialLengths.ts:57-59
        const int i = latestLeqIndex(key);
        return i >= 0 && i < int(items.size()) ? &items[size_t(i)] : nullptr;
    }
    PSLEntry* firstGte(int key) {  // partialLengths.ts:66-69
        const Pos p = find(key);
        return p.index >= 0 && p.index < int(items.size()) ? &items[size_t(p.index)] : nullptr;
    }
    // PartialSequenceLengthsSet.addOrUpdate, partialLengths.ts:24-50
    void addOrUpdate(PSLEntry n) {
        PSLEntry* prev = latestLeq(n.seq);
        if (!(prev && prev->seq == n.seq)) n.len = (prev ? prev->len : 0) + n.seglen;
        for (int i = int(items.size()) - 1; i >= 0; i--) {  // following elements
            PSLEntry& e = items[size_t(i)];
            if (e.seq <= n.seq) break;
            e.len += n.seglen;
        }
        const Pos p = find(n.seq);
        if (p.exists) {
            PSLEntry& cur = items[size_t(p.index)];
            cur.seglen += n.seglen;
            cur.len += n.seglen;
            combineOverlapClients(cur, n);
        } else {
            items.insert(items.begin() + p.index, std::move(n));
        }
    }
    // copyDown, partialLengths.ts:76-94
    int64_t copyDown(int minSeq) {
        const int mindex = latestLeqIndex(minSeq);
        int64_t minLength = 0;
        if (mindex >= 0) {
            minLength = items[size_t(mindex)].len;
            const int seqCount = int(items.size());
            if (mindex <= seqCount - 1) {
                const int remaining = seqCount - mindex - 1;
                for (int i = 0; i < remaining; i++) {
                    items[size_t(i)] = items[size_t(i + mindex + 1)];
                    items[size_t(i)].len -= minLength;
                }
                items.resize(size_t(remaining));
            }
        }
        return minLength;
    }
};

// PartialSequenceLengths (partialLengths.ts:239-850), sequenced records only
struct PSL {
    int minSeq = 0;
    int64_t minLength = 0;
    int segmentCount = 0;
    PSLSet partialLengths;
    std::map<int, PSLSet> clientSeqNumbers;  // clientSeqNumbers[clientId] (negative ids are JS properties)

    explicit PSL(int ms) : minSeq(ms) {}

    // addClientSeqNumber / addClientSeqNumberFromPartial, partialLengths.ts:824-845
    void addClientSeqNumber(int clientId, int seq, int64_t seglen) {
        PSLEntry e;
        e.seq = seq;
        e.seglen = seglen;
        clientSeqNumbers[clientId].addOrUpdate(std::move(e));
    }
    void addClientSeqNumberFromPartial(const PSLEntry& p) {
        addClientSeqNumber(p.clientId, p.seq, p.seglen);
        if (p.hasOverlap)
            for (const auto& kv : p.overlap)  // RB-tree map order: ascending client id
                if (p.clientId != kv.first) addClientSeqNumber(kv.first, p.seq, kv.second);
    }
    // zamboni, partialLengths.ts:809-819
    void zamboni(int windowMinSeq) {
        minLength += partialLengths.copyDown(windowMinSeq);
        minSeq = windowMinSeq;
        for (auto& kv : clientSeqNumbers) kv.second.copyDown(windowMinSeq);
    }
    // getPartialLength, partialLengths.ts:698-735 (localSeq undefined)
    int64_t getPartialLength(int refSeq, int clientId) {
        int64_t pLen = minLength;
        auto it = clientSeqNumbers.find(clientId);
        PSLSet* cli = it == clientSeqNumbers.end() ? nullptr : &it->second;
        const int cliLatestIndex = cli && !cli->items.empty() ? int(cli->items.size()) - 1 : -1;
        if (PSLEntry* e = partialLengths.latestLeq(refSeq)) pLen += e->len;
        if (cliLatestIndex >= 0) {
            const PSLEntry& cliLatest = cli->items[size_t(cliLatestIndex)];
            if (cliLatest.seq > refSeq) {
                pLen += cliLatest.len;
                if (PSLEntry* preceding = cli->latestLeq(refSeq)) pLen -= preceding->len;
            }
        }
        return pLen;
    }
    // addSeq, partialLengths.ts:543-578
    static void addSeq(PSLSet& set, int seq, int64_t seqSeglen, bool hasClient, int clientId) {
        PSLEntry* seqPartialLen = nullptr;
        PSLEntry* penult = nullptr;
        PSLEntry* p = set.latestLeq(seq);
        if (p) {
            if (p->seq == seq) {
                seqPartialLen = p;
                p = set.latestLeq(seq - 1);
                if (p) penult = p;
            } else {
                penult = p;
            }
        }
        const int64_t len = penult ? penult->len + seqSeglen : seqSeglen;
        if (!seqPartialLen) {
            PSLEntry e;
            e.clientId = clientId;
            e.hasClient = hasClient;
            e.len = len;
            e.seglen = seqSeglen;
            e.seq = seq;
            set.addOrUpdate(std::move(e));
        } else {
            seqPartialLen->seglen = seqSeglen;
            seqPartialLen->len = len;
        }
    }
};

// the parts of Seg / Block this restatement reads
inline bool pslSeqLTE(int seq, int minSeq) { return seq != -1 /*Unassigned*/ && seq <= minSeq; }  // :361-363

// PartialSequenceLengths.insertSegment, partialLengths.ts:440-536 (sequenced segments)
inline void pslInsertSegment(PSL& c, const Seg* s, bool removal) {
    int seq = s->seq;
    int64_t segmentLen = s->len;
    int clientId = s->clientId;
    const std::vector<int>* overlapIds = nullptr;
    if (removal) {
        seq = s->removedSeq;
        segmentLen = -segmentLen;
        clientId = s->removedClientIds[0];
        if (s->removedClientIds.size() > 1) overlapIds = &s->removedClientIds;
    }
    PSLEntry* firstGte = c.partialLengths.firstGte(seq);
    if (firstGte && firstGte->seq == seq) {
        firstGte->seglen += segmentLen;
        if (overlapIds) {  // accumulateRemoveClientOverlap, partialLengths.ts:420-438
            if (firstGte->hasOverlap) {
                for (int id : *overlapIds) firstGte->overlap[id] += segmentLen;
            } else {
                firstGte->hasOverlap = true;
                for (int id : *overlapIds) firstGte->overlap[id] = segmentLen;  // getOverlapClients
            }
        }
    } else {
        PSLEntry e;
        e.seq = seq;
        e.clientId = clientId;
        e.hasClient = true;
        e.seglen = segmentLen;
        if (overlapIds) {
            e.hasOverlap = true;
            for (int id : *overlapIds) e.overlap[id] = segmentLen;
        }
        c.partialLengths.addOrUpdate(std::move(e));
    }
}

// PartialSequenceLengths.fromLeaves, partialLengths.ts:344-403
inline std::shared_ptr<PSL> pslFromLeaves(const Block* block, int minSeq) {
    auto c = std::make_shared<PSL>(minSeq);
    c->segmentCount = block->childCount;
    for (int i = 0; i < block->childCount; i++) {
        const Node* child = block->children[i];
        if (!child->leaf) continue;
        const Seg* s = static_cast<const Seg*>(child);
        if (pslSeqLTE(s->seq, minSeq)) c->minLength += s->len;
        else pslInsertSegment(*c, s, false);
        if (s->removed && pslSeqLTE(s->removedSeq, minSeq)) c->minLength -= s->len;
        else if (s->removed) pslInsertSegment(*c, s, true);
    }
    int64_t prevLen = 0;
    for (PSLEntry& p : c->partialLengths.items) {
        p.len = prevLen + p.seglen;
        prevLen = p.len;
        c->addClientSeqNumberFromPartial(p);
    }
    return c;
}

// PartialSequenceLengths.combine, partialLengths.ts:256-338 (computeLocalPartials false)
inline std::shared_ptr<PSL> pslCombine(Block* block, int minSeq, bool recur) {
    std::shared_ptr<PSL> leaf = pslFromLeaves(block, minSeq);
    bool hasInternalChild = false;
    std::vector<PSL*> childPartials;
    for (int i = 0; i < block->childCount; i++) {
        Node* child = block->children[i];
        if (!child->leaf) {
            hasInternalChild = true;
            Block* cb = static_cast<Block*>(child);
            if (recur) cb->pl = pslCombine(cb, minSeq, true);
            childPartials.push_back(cb->pl.get());
        }
    }
    std::shared_ptr<PSL> combined = hasInternalChild ? std::make_shared<PSL>(minSeq) : leaf;
    if (hasInternalChild) {
        if (!leaf->partialLengths.items.empty()) childPartials.push_back(leaf.get());
        std::vector<const std::vector<PSLEntry>*> lists;
        for (PSL* cp : childPartials) {
            combined->segmentCount += cp->segmentCount;
            combined->minLength += cp->minLength;
            lists.push_back(&cp->partialLengths.items);
        }
        // mergePartialLengths + mergeSortedListsBySeq, partialLengths.ts:1013-1074: repeatedly the
        // smallest seq at the lists' heads (the earliest list wins ties); each entry copied in
        std::vector<size_t> next(lists.size(), 0);
        for (;;) {
            int best = -1;
            for (size_t i = 0; i < lists.size(); i++)
                if (next[i] < lists[i]->size() &&
                    (best < 0 || (*lists[i])[next[i]].seq < (*lists[size_t(best)])[next[size_t(best)]].seq))
                    best = int(i);
            if (best < 0) break;
            combined->partialLengths.addOrUpdate((*lists[size_t(best)])[next[size_t(best)]++]);
        }
        for (const PSLEntry& p : combined->partialLengths.items) combined->addClientSeqNumberFromPartial(p);
    }
    combined->zamboni(minSeq);  // PartialSequenceLengths.options.zamboni (default true)
    return combined;
}

// PartialSequenceLengths.update, partialLengths.ts:636-686
inline void pslUpdate(PSL& pl, const Block* node, int seq, int clientId, int windowMinSeq) {
    int64_t seqSeglen = 0;
    int segCount = 0;
    for (int i = 0; i < node->childCount; i++) {
        const Node* child = node->children[i];
        if (!child->leaf) {
            const Block* cb = static_cast<const Block*>(child);
            PSL& branch = *cb->pl;
            if (PSLEntry* leq = branch.partialLengths.latestLeq(seq))
                if (leq->seq == seq) seqSeglen += leq->seglen;
            segCount += branch.segmentCount;
        } else {
            const Seg* s = static_cast<const Seg*>(child);
            const bool removedAt = s->removed && s->removedSeq == seq;
            if (s->seq == seq) {
                if (!removedAt) seqSeglen += s->len;
            } else if (removedAt) {
                seqSeglen -= s->len;
            }
            segCount++;
        }
    }
    pl.segmentCount = segCount;
    PSL::addSeq(pl.partialLengths, seq, seqSeglen, true, clientId);
    PSL::addSeq(pl.clientSeqNumbers[clientId], seq, seqSeglen, false, 0);
    pl.zamboni(windowMinSeq);
}
