// apply.hip.h -- the op-apply kernel of the MI355X merge-tree replay engine.
//
// One workgroup (256 threads = 4 wave64) owns one document for the whole launch and
// applies that document's ops strictly in order (ops never cross documents).  The
// document's leaves live in LDS as flat structure-of-arrays records in tree order; the
// reference's B+tree (MaxNodesInBlock = 8, mergeTreeNodes.ts:330) is kept exactly, encoded
// per leaf as `bnd` = number of tree levels at which the leaf starts a block.
//
// O(S) passes run on all 256 lanes: the visibility prefix scan that replaces
// PartialSequenceLengths (partialLengths.ts:698) + insertingWalk (mergeTree.ts:1740), the
// shift that makes room for a split/insert (mergeTree.ts:1831-1838), the uid search for
// LRU entries and the stream compaction after zamboni (zamboni.ts:19-120).  The O(1)
// control (tie-break, block splits, heap, scour decisions) runs on lane 0.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtr_types.h"
#include "../../include/mtr_synth.h"

namespace mtr {

constexpr int NT = 256;
constexpr int NWAVES = NT / 64;
constexpr int32_t RNONE = 0x7fffffff;  // removedSeq of a live leaf
constexpr uint32_t NONE32 = 0xffffffffu;
constexpr int kMaxNodesInBlock = 8;
constexpr int kGranularity = 256;  // TextSegmentGranularity, textSegment.ts:35

// meta word layout
constexpr uint32_t M_CLIENT_MASK = 0xffu;
constexpr int M_FREM_SHIFT = 8;
constexpr int M_BND_SHIFT = 16;
constexpr uint32_t M_BND_MASK = 0xfu << M_BND_SHIFT;
constexpr uint32_t M_MARKER = 1u << 20;
constexpr uint32_t M_OVERLAP = 1u << 21;
constexpr int M_NS_SHIFT = 22;  // needsScour of the leaf block this leaf starts: 0 undef, 1 false, 2 true
constexpr uint32_t M_NS_MASK = 3u << M_NS_SHIFT;
constexpr uint32_t M_NOREF = 1u << 24;
constexpr uint32_t M_DEL = 1u << 25;
constexpr uint32_t NS_UNDEF = 0, NS_FALSE = 1, NS_TRUE = 2;

constexpr uint32_t CL_LOCAL = 0xffu;     // LocalClientId (-1)
constexpr uint32_t CL_NONCOLLAB = 0xfeu; // NonCollabClient (-2)

__host__ __device__ inline uint32_t enc_client(int c) {
    return c >= 0 ? uint32_t(c) & 0xffu : (c == -1 ? CL_LOCAL : CL_NONCOLLAB);
}
__host__ __device__ inline int dec_client(uint32_t e) {
    return e == CL_LOCAL ? -1 : (e == CL_NONCOLLAB ? -2 : int(e));
}

// Per-document header in HBM (64 bytes)
struct DocHdr {
    int32_t nseg, height, minseq, curseq;
    int32_t collab, local, heapn, uidnext;
    int32_t textused, propused, rmused, status;
    int32_t op_cursor, fail_op, max_heap, texthalf;  // texthalf: active half of the text arena
};

// number of 32-bit SoA fields per leaf kept in HBM and LDS
constexpr int NF = 8;
enum { F_LEN = 0, F_SEQ, F_RSEQ, F_META, F_TEXT, F_PROPS, F_RM, F_UID };

struct KParams {
    DocHdr* hdr;
    uint32_t* seg;       // [doc][NF][segcap]
    uint32_t* heap;      // [doc][2][hcap]   (seq, uid), 1-based
    uint16_t* text;      // [doc][tcap]
    uint32_t* prop;      // [doc][pcap]
    uint32_t* rm;        // [doc][rcap]
    int32_t segcap, hcap, tcap, pcap, rcap;
    int32_t cap;         // LDS leaf capacity of this launch
    int32_t lhcap;       // LDS heap capacity of this launch
    int32_t global_mode; // 1: leaves/heap stay in HBM (documents larger than LDS)
    uint32_t* scratch;   // [doc][2][segcap] E/V arrays for global mode
    int32_t ops_this_launch;
    int32_t new_length_calc;
    uint32_t n_docs;
    const mtr_op* ops;
    const mtr_doc_desc* docs;
    const uint16_t* btext;
    const uint32_t* propop_off;
    const uint32_t* propop_kv;
    const uint32_t* key_index;
    const uint32_t* val_eq;
    unsigned long long* stat_ops;  // ops applied (atomic)
    // record mode (synthetic workloads): ops are drawn from include/mtr_synth.h with this
    // engine's own exact view lengths, written to gen_ops/gen_text, then applied
    int32_t gen;
    mtr_synth_cfg gen_cfg;
    mtr_synth_state* gen_state;   // [doc]
    mtr_op* gen_ops;              // == ops, writable
    uint16_t* gen_text;           // == btext, writable
    int32_t trace;                 // debug: printf zamboni decisions of document 0
    int32_t trace_seq;             // debug: dump leaves at zamboni of this op seq
};

// scalar document state + broadcast slots, in LDS
struct Sc {
    int nseg, height, minseq, curseq;
    int collab, local, heapn, uidnext;
    int textused, propused, rmused, status;
    int b0, b1, b2, b3;
    int b4, b5, b6, b7;
    int red[2 * NWAVES];
    int fail_op, max_heap, ops_done, texthalf;
    unsigned long long sum_s, sum_l;  // sum over ops of the leaf count before the op / inserted text units
};

struct View {
    int ref;
    uint32_t client;  // encoded
    int local;        // local-view rules (mergeTree.ts:613-634)
};

struct Lds {
    int* len;
    int* seq;
    int* rseq;
    uint32_t* meta;
    uint32_t* text;
    uint32_t* props;
    uint32_t* rm;
    uint32_t* uid;
    int* E;   // inclusive prefix of visible length
    int* V;   // visible length (-1 = undefined)
    int* hseq;
    uint32_t* huid;
    Sc* sc;
    mtr_synth_state* gst;
    // document slabs in HBM
    uint16_t* gtext;
    uint32_t* gprop;
    uint32_t* grm;
    int cap, lhcap;
};

__device__ inline int bnd_of(uint32_t m) { return int((m & M_BND_MASK) >> M_BND_SHIFT); }
__device__ inline uint32_t set_bnd(uint32_t m, int b) { return (m & ~M_BND_MASK) | (uint32_t(b) << M_BND_SHIFT); }
__device__ inline uint32_t ns_of(uint32_t m) { return (m & M_NS_MASK) >> M_NS_SHIFT; }
__device__ inline uint32_t set_ns(uint32_t m, uint32_t ns) { return (m & ~M_NS_MASK) | (ns << M_NS_SHIFT); }

// ------------------------------------------------------------------ block primitives
__device__ inline int wave_incl_scan(int x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}
__device__ inline int wave_sum(int x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ inline int wave_max(int x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x = max(x, __shfl_xor(x, d, 64));
    return x;
}

// exclusive block scan; also returns the block total in *total
__device__ inline int block_excl_scan(Sc* sc, int x, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = wave_incl_scan(x);
    if (lane == 63) sc->red[w] = inc;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NWAVES; k++) {
        int r = sc->red[k];
        if (k < w) base += r;
        tot += r;
    }
    __syncthreads();
    *total = tot;
    return base + inc - x;
}
__device__ inline int block_max(Sc* sc, int x) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int m = wave_max(x);
    if (lane == 0) sc->red[w] = m;
    __syncthreads();
    int r = sc->red[0];
#pragma unroll
    for (int k = 1; k < NWAVES; k++) r = max(r, sc->red[k]);
    __syncthreads();
    return r;
}

// ------------------------------------------------------------------ visibility
__device__ bool in_removers(const Lds& L, int i, uint32_t c) {
    uint32_t m = L.meta[i];
    if (((m >> M_FREM_SHIFT) & 0xffu) == c) return true;
    if (!(m & M_OVERLAP)) return false;
    uint32_t cell = L.rm[i];
    while (cell != NONE32) {
        uint32_t v = L.grm[cell];
        if ((v >> 24) == c) return true;
        cell = v & 0xffffffu;
        if (cell == 0xffffffu) break;
    }
    return false;
}

// nodeLength for a leaf (mergeTree.ts:916-1004): -1 = undefined
__device__ int vis_len(const Lds& L, int i, const View& v, int newlen) {
    int len = L.len[i];
    int rseq = L.rseq[i];
    bool removed = rseq != RNONE;
    int minseq = L.sc->minseq;
    if (v.local) {  // localNetLength, mergeTree.ts:613-634
        if (removed) {
            if (!newlen) return rseq > minseq ? 0 : -1;
            return 0;
        }
        return len;
    }
    uint32_t cl = L.meta[i] & M_CLIENT_MASK;
    int seq = L.seq[i];
    if (newlen) {  // mergeTree.ts:935-965
        if (removed) {
            if (rseq <= minseq) return -1;
            if (rseq <= v.ref || in_removers(L, i, v.client)) return 0;
        }
        return (seq <= v.ref || cl == v.client) ? len : 0;
    }
    if (removed && rseq <= v.ref) return -1;  // mergeTree.ts:967-976
    if (cl == v.client || seq <= v.ref) {
        if (removed) return in_removers(L, i, v.client) ? 0 : len;
        return len;
    }
    if (removed) return -1;
    return 0;
}

// V[i] = visible length, E[i] = inclusive prefix of max(V,0).  Contiguous chunk per thread.
__device__ void prefix(Lds& L, const View& v, int newlen) {
    const int S = L.sc->nseg;
    const int per = (S + NT - 1) / NT;
    const int lo = min(S, int(threadIdx.x) * per), hi = min(S, lo + per);
    int sum = 0;
    for (int i = lo; i < hi; i++) {
        int x = vis_len(L, i, v, newlen);
        L.V[i] = x;
        sum += max(x, 0);
    }
    int tot;
    int run = block_excl_scan(L.sc, sum, &tot);
    for (int i = lo; i < hi; i++) {
        run += max(L.V[i], 0);
        L.E[i] = run;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ data movement
__device__ inline void copy_rec(Lds& L, int dst, int src) {
    L.len[dst] = L.len[src];
    L.seq[dst] = L.seq[src];
    L.rseq[dst] = L.rseq[src];
    L.meta[dst] = L.meta[src];
    L.text[dst] = L.text[src];
    L.props[dst] = L.props[src];
    L.rm[dst] = L.rm[src];
    L.uid[dst] = L.uid[src];
}

// move leaves [at, S) to [at+1, S+1).  Rounds of NT from the top: each round reads its
// NT records into registers, barrier, writes them one slot up.
__device__ void shift_right1(Lds& L, int at) {
    const int S = L.sc->nseg;
    for (int hi = S; hi > at; hi -= NT) {
        const int lo = max(at, hi - NT);
        const int i = lo + int(threadIdx.x);
        int a0 = 0, a1 = 0, a2 = 0;
        uint32_t a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
        const bool act = i < hi;
        if (act) {
            a0 = L.len[i]; a1 = L.seq[i]; a2 = L.rseq[i]; a3 = L.meta[i];
            a4 = L.text[i]; a5 = L.props[i]; a6 = L.rm[i]; a7 = L.uid[i];
        }
        __syncthreads();
        if (act) {
            L.len[i + 1] = a0; L.seq[i + 1] = a1; L.rseq[i + 1] = a2; L.meta[i + 1] = a3;
            L.text[i + 1] = a4; L.props[i + 1] = a5; L.rm[i + 1] = a6; L.uid[i + 1] = a7;
        }
        __syncthreads();
    }
}

// stream compaction of leaves without M_DEL (zamboni unlink / append); rounds of NT from
// the bottom; destinations never exceed sources.
__device__ void compact(Lds& L) {
    const int S = L.sc->nseg;
    int base = 0;
    for (int lo = 0; lo < S; lo += NT) {
        const int i = lo + int(threadIdx.x);
        const bool act = i < S;
        int a0 = 0, a1 = 0, a2 = 0;
        uint32_t a3 = M_DEL, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
        if (act) {
            a0 = L.len[i]; a1 = L.seq[i]; a2 = L.rseq[i]; a3 = L.meta[i];
            a4 = L.text[i]; a5 = L.props[i]; a6 = L.rm[i]; a7 = L.uid[i];
        }
        int keep = (act && !(a3 & M_DEL)) ? 1 : 0;
        int tot;
        int off = block_excl_scan(L.sc, keep, &tot);  // contains barriers: reads done before writes
        if (keep) {
            int d = base + off;
            L.len[d] = a0; L.seq[d] = a1; L.rseq[d] = a2; L.meta[d] = a3;
            L.text[d] = a4; L.props[d] = a5; L.rm[d] = a6; L.uid[d] = a7;
        }
        base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        L.sc->nseg = base;
        if (base == 0) L.sc->height = 1;
    }
    __syncthreads();
}

// index of the leaf with this uid, -1 if unlinked
__device__ int find_uid(Lds& L, uint32_t u) {
    const int S = L.sc->nseg;
    int found = -1;
    for (int i = threadIdx.x; i < S; i += NT)
        if (L.uid[i] == u) found = i;
    return block_max(L.sc, found);
}

// ------------------------------------------------------------------ lane-0 helpers
__device__ inline int block_start(const Lds& L, int x, int level) {
    while (x > 0 && bnd_of(L.meta[x]) < level) x--;
    return x;
}
__device__ inline int block_end(const Lds& L, int x, int level) {
    const int S = L.sc->nseg;
    x++;
    while (x < S && bnd_of(L.meta[x]) < level) x++;
    return x;
}
__device__ inline int lower_bound_E(const Lds& L, int pos) {  // first i with E[i] >= pos
    int lo = 0, hi = L.sc->nseg;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (L.E[mid] >= pos) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// Block overflow after a leaf was added next to x (insertingWalk split + updateRoot,
// mergeTree.ts:1831-1871, 1268-1277).
__device__ void overflow_fix(Lds& L, int x) {
    Sc* sc = L.sc;
    int level = 1;
    int bs = block_start(L, x, 1), be = block_end(L, x, 1);
    int cnt = be - bs;
    while (cnt >= kMaxNodesInBlock) {
        int c5;
        if (level == 1) {
            c5 = bs + kMaxNodesInBlock / 2;
        } else {
            int k = 0;
            c5 = bs;
            for (int i = bs; i < be; i++)
                if (bnd_of(L.meta[i]) >= level - 1) {
                    if (k == kMaxNodesInBlock / 2) { c5 = i; break; }
                    k++;
                }
        }
        uint32_t m = set_bnd(L.meta[c5], level);
        if (level == 1) m = set_ns(m, NS_UNDEF);
        L.meta[c5] = m;
        if (level == sc->height) {  // root split
            sc->height++;
            L.meta[0] = set_bnd(L.meta[0], sc->height);
            break;
        }
        level++;
        bs = block_start(L, bs, level);
        be = block_end(L, bs, level);
        cnt = 0;
        for (int i = bs; i < be; i++)
            if (bnd_of(L.meta[i]) >= level - 1) cnt++;
    }
}

// ---- LRU heap (collections/heap.ts:11-67), 1-based in LDS, lane 0 only
__device__ void heap_push(Lds& L, uint32_t u, int s) {
    Sc* sc = L.sc;
    if (sc->heapn + 1 >= L.lhcap) {
        sc->status = MTR_ERR_CAPACITY;
        return;
    }
    int k = ++sc->heapn;
    L.hseq[k] = s;
    L.huid[k] = u;
    while (k > 1 && L.hseq[k >> 1] - L.hseq[k] > 0) {
        int ts = L.hseq[k >> 1]; uint32_t tu = L.huid[k >> 1];
        L.hseq[k >> 1] = L.hseq[k]; L.huid[k >> 1] = L.huid[k];
        L.hseq[k] = ts; L.huid[k] = tu;
        k >>= 1;
    }
    if (sc->heapn > sc->max_heap) sc->max_heap = sc->heapn;
}
__device__ uint32_t heap_pop(Lds& L) {
    Sc* sc = L.sc;
    uint32_t x = L.huid[1];
    int n = sc->heapn;
    L.hseq[1] = L.hseq[n];
    L.huid[1] = L.huid[n];
    n--;
    sc->heapn = n;
    int k = 1;
    while ((k << 1) <= n) {
        int j = k << 1;
        if (j < n && L.hseq[j] - L.hseq[j + 1] > 0) j++;
        if (L.hseq[k] - L.hseq[j] <= 0) break;
        int ts = L.hseq[k]; uint32_t tu = L.huid[k];
        L.hseq[k] = L.hseq[j]; L.huid[k] = L.huid[j];
        L.hseq[j] = ts; L.huid[j] = tu;
        k = j;
    }
    return x;
}

// addToLRUSet, mergeTree.ts:741-751
__device__ void add_lru(Lds& L, int i, int s) {
    Sc* sc = L.sc;
    int bs = block_start(L, i, 1);
    uint32_t m = L.meta[bs];
    if (ns_of(m) != NS_TRUE && s > sc->curseq) {
        L.meta[bs] = set_ns(m, NS_TRUE);
        heap_push(L, L.uid[i], s);
    }
}

// ---- properties (PropertiesManager.addProperties without combining ops,
//      segmentPropertiesManager.ts:60-157; JS own-key order)
// prop arena entry at offset p: [n, k0, v0, k1, v1, ...]
__device__ uint32_t props_apply(Lds& L, const KParams& P, uint32_t old, uint32_t pp) {
    Sc* sc = L.sc;
    uint32_t n_old = old == NONE32 ? 0 : L.gprop[old];
    uint32_t lo = P.propop_off[pp], hi = P.propop_off[pp + 1];
    uint32_t need = 1 + 2 * (n_old + (hi - lo));
    if (uint32_t(sc->propused) + need > uint32_t(P.pcap)) {
        sc->status = MTR_ERR_CAPACITY;
        return old;
    }
    uint32_t dst = uint32_t(sc->propused);
    uint32_t* e = L.gprop + dst;
    uint32_t n = n_old;
    for (uint32_t k = 0; k < 2 * n_old; k++) e[1 + k] = L.gprop[old + 1 + k];
    for (uint32_t q = lo; q < hi; q++) {
        uint32_t key = P.propop_kv[2 * q], val = P.propop_kv[2 * q + 1];
        int at = -1;
        for (uint32_t k = 0; k < n; k++)
            if (e[1 + 2 * k] == key) { at = int(k); break; }
        if (val == MTR_NULL_VALUE) {
            if (at >= 0) {
                for (uint32_t k = uint32_t(at); k + 1 < n; k++) {
                    e[1 + 2 * k] = e[1 + 2 * (k + 1)];
                    e[2 + 2 * k] = e[2 + 2 * (k + 1)];
                }
                n--;
            }
        } else if (at >= 0) {
            e[2 + 2 * at] = val;
        } else {
            uint32_t ix = P.key_index[key];
            uint32_t pos = n;
            if (ix != MTR_NOT_INDEX) {
                pos = 0;
                while (pos < n && P.key_index[e[1 + 2 * pos]] != MTR_NOT_INDEX && P.key_index[e[1 + 2 * pos]] < ix) pos++;
                for (uint32_t k = n; k > pos; k--) {
                    e[1 + 2 * k] = e[1 + 2 * (k - 1)];
                    e[2 + 2 * k] = e[2 + 2 * (k - 1)];
                }
            }
            e[1 + 2 * pos] = key;
            e[2 + 2 * pos] = val;
            n++;
        }
    }
    e[0] = n;
    sc->propused += int(1 + 2 * n);
    return dst;
}

// matchProperties (properties.ts:71-105) with values compared by equivalence class
__device__ bool props_match(const uint32_t* gprop, const uint32_t* val_eq, uint32_t a, uint32_t b) {
    if (a == b) return true;
    if (a == NONE32 || b == NONE32) return false;
    uint32_t na = gprop[a], nb = gprop[b];
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
        uint32_t k = gprop[a + 1 + 2 * i];
        bool found = false;
        for (uint32_t j = 0; j < nb; j++)
            if (gprop[b + 1 + 2 * j] == k) {
                if (val_eq[gprop[a + 2 + 2 * i]] != val_eq[gprop[b + 2 + 2 * j]]) return false;
                found = true;
                break;
            }
        if (!found) return false;
    }
    return true;
}

// ---- text
__device__ inline bool can_append(const Lds& L, int a, int b) {  // TextSegment.canAppend textSegment.ts:86-93
    if ((L.meta[a] | L.meta[b]) & M_MARKER) return false;
    int la = L.len[a];
    if (la > 0 && L.gtext[L.text[a] + la - 1] == u'\n') return false;
    return la <= kGranularity || L.len[b] <= kGranularity;
}

// prev.append(seg) (textSegment.ts:99-103): text of b follows text of a
__device__ inline int text_end(const Sc* sc, const KParams& P) { return (P.tcap / 2) * (sc->texthalf + 1); }

__device__ void text_append(Lds& L, const KParams& P, int a, int b) {
    Sc* sc = L.sc;
    const int tend = text_end(sc, P);
    uint32_t oa = L.text[a], ob = L.text[b];
    int la = L.len[a], lb = L.len[b];
    if (oa + uint32_t(la) == ob) {
        L.len[a] = la + lb;
        return;
    }
    if (oa + uint32_t(la) == uint32_t(sc->textused)) {
        if (sc->textused + lb > tend) { sc->status = MTR_ERR_CAPACITY; return; }
        for (int k = 0; k < lb; k++) L.gtext[sc->textused + k] = L.gtext[ob + k];
        sc->textused += lb;
        L.len[a] = la + lb;
        return;
    }
    if (sc->textused + la + lb > tend) { sc->status = MTR_ERR_CAPACITY; return; }
    uint32_t d = uint32_t(sc->textused);
    for (int k = 0; k < la; k++) L.gtext[d + k] = L.gtext[oa + k];
    for (int k = 0; k < lb; k++) L.gtext[d + la + k] = L.gtext[ob + k];
    sc->textused += la + lb;
    L.text[a] = d;
    L.len[a] = la + lb;
}

// Semi-space compaction of the text arena: copy every leaf's text into the other half in leaf
// order (block prefix scan of lengths), then switch halves.  Dead text (removed/merged leaves)
// is dropped; split halves that shared text get their own copies.
__device__ void text_gc(Lds& L, const KParams& P) {
    Sc* sc = L.sc;
    const int S = sc->nseg;
    const int per = (S + NT - 1) / NT;
    const int lo = min(S, int(threadIdx.x) * per), hi = min(S, lo + per);
    int sum = 0;
    for (int i = lo; i < hi; i++)
        if (!(L.meta[i] & M_MARKER)) sum += L.len[i];
    int tot;
    int run = block_excl_scan(sc, sum, &tot);
    const int half = P.tcap / 2;
    const int dst0 = sc->texthalf ? 0 : half;
    for (int i = lo; i < hi; i++) {
        if (L.meta[i] & M_MARKER) continue;
        const uint32_t src = L.text[i];
        const int n = L.len[i];
        for (int k = 0; k < n; k++) L.gtext[dst0 + run + k] = L.gtext[src + k];
        L.text[i] = uint32_t(dst0 + run);
        run += n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        sc->texthalf ^= 1;
        sc->textused = dst0 + tot;
        if (tot > half) sc->status = MTR_ERR_CAPACITY;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ zamboni
// scourNode over one leaf block [cs, ce) (zamboni.ts:122-193); marks M_DEL; returns #kept
__device__ int scour_leaf_block(Lds& L, const KParams& P, int cs, int ce) {
    Sc* sc = L.sc;
    int prev = -1, kept = 0;
    for (int k = cs; k < ce; k++) {
        uint32_t m = L.meta[k];
        if (m & M_DEL) continue;
        if (L.rseq[k] != RNONE) {
            if (L.rseq[k] > sc->minseq) kept++;
            else L.meta[k] = m | M_DEL;  // UNLINK
            prev = -1;
        } else if (L.seq[k] <= sc->minseq) {
            if (prev >= 0 && can_append(L, prev, k) && props_match(L.gprop, P.val_eq, L.props[prev], L.props[k]) &&
                L.len[k] > 0) {
                text_append(L, P, prev, k);
                L.meta[k] = m | M_DEL;
            } else {
                kept++;
                prev = L.len[k] > 0 ? k : -1;
            }
        } else {
            kept++;
            prev = -1;
        }
    }
    return kept;
}

constexpr int MAXH = 16;

// zamboniSegments body for one popped LRU entry whose segment is leaf x
// (zamboni.ts:33-58 + packParent zamboni.ts:63-120).  Lane 0.  Returns 1 if leaves
// were marked for deletion (caller compacts).
__device__ int zamboni_block(Lds& L, const KParams& P, int x) {
    Sc* sc = L.sc;
    const int H = sc->height;
    int rs[MAXH + 1], re[MAXH + 1], topb[MAXH + 1];
    rs[1] = block_start(L, x, 1);
    re[1] = block_end(L, x, 1);
    if (ns_of(L.meta[rs[1]]) == NS_FALSE) return 0;
    for (int l = 1; l <= H; l++) {
        if (l > 1) {
            rs[l] = block_start(L, rs[l - 1], l);
            re[l] = block_end(L, rs[l - 1], l);
        }
        topb[l] = bnd_of(L.meta[rs[l]]);
    }
    const int before = re[1] - rs[1];
    const int kept = scour_leaf_block(L, P, rs[1], re[1]);
    if (P.trace && blockIdx.x == 0) printf("SCOUR n=%d kept=%d\n", before, kept);
    // block.needsScour = false (on the block's first surviving leaf)
    int first = -1;
    for (int k = rs[1]; k < re[1]; k++)
        if (!(L.meta[k] & M_DEL)) { first = k; break; }
    if (first >= 0) {
        uint32_t m = set_bnd(L.meta[first], topb[1]);
        L.meta[first] = set_ns(m, NS_FALSE);
    }
    if (kept >= before) return 0;
    if (kept < kMaxNodesInBlock / 2 && H > 1) {
        // packParent chain
        for (int l = 2; l <= H; l++) {
            if (l == 2) {
                // packParent scours every child of P again -- including the block just scoured:
                // scourNode is not idempotent (a dropped tombstone no longer resets the merge
                // candidate), zamboni.ts:68-73,122-193.
                for (int cs = rs[2]; cs < re[2];) {
                    int ce = cs + 1;
                    while (ce < re[2] && bnd_of(L.meta[ce]) < 1) ce++;
                    scour_leaf_block(L, P, cs, ce);
                    cs = ce;
                }
            }
            // items: surviving leaves (l == 2) or surviving level-(l-2) block starts
            int T = 0;
            for (int k = rs[l]; k < re[l]; k++) {
                uint32_t m = L.meta[k];
                if (m & M_DEL) continue;
                if (l == 2 || bnd_of(m) >= l - 2) T++;
            }
            int c = 0;
            if (P.trace && blockIdx.x == 0) printf("PACK items=%d\n", T);
            if (T > 0) {
                c = min(kMaxNodesInBlock - 1, T / (kMaxNodesInBlock / 2));
                if (c < 1) c = 1;
                const int base = T / c;
                int rem = T % c;
                int item = 0, nextStart = 0, blk = 0;
                for (int k = rs[l]; k < re[l]; k++) {
                    uint32_t m = L.meta[k];
                    if (m & M_DEL) continue;
                    if (!(l == 2 || bnd_of(m) >= l - 2)) continue;
                    int nb;
                    bool isStart = item == nextStart;
                    if (isStart) {
                        int sz = base + (blk < rem ? 1 : 0);
                        nextStart += sz;
                        blk++;
                    }
                    if (item == 0) nb = topb[l];
                    else if (isStart) nb = l - 1;
                    else nb = l == 2 ? 0 : l - 2;
                    m = set_bnd(m, nb);
                    if (l == 2 && isStart) m = set_ns(m, NS_UNDEF);
                    L.meta[k] = m;
                    item++;
                }
            }
            if (!(c < kMaxNodesInBlock / 2 && l < H)) break;
        }
    }
    return 1;
}

// zamboniSegments (zamboni.ts:19-60): all threads
__device__ void zamboni(Lds& L, const KParams& P) {
    Sc* sc = L.sc;
    if (!sc->collab) return;
    if (P.trace && blockIdx.x == 0 && threadIdx.x == 0 && sc->b3 == P.trace_seq) {
        for (int i = 0; i < sc->nseg; i++)
            printf("DUMP %d len=%d seq=%d rs=%d bnd=%d\n", i, L.len[i], L.seq[i],
                   L.rseq[i] == RNONE ? -1 : L.rseq[i], bnd_of(L.meta[i]));
    }
    for (int it = 0; it < 2; it++) {
        __syncthreads();
        if (sc->heapn == 0 || sc->status != MTR_OK) return;
        if (L.hseq[1] > sc->minseq) return;
        __syncthreads();
        if (threadIdx.x == 0) {
            sc->b7 = L.hseq[1];
            sc->b4 = int(heap_pop(L));
        }
        __syncthreads();
        int x = find_uid(L, uint32_t(sc->b4));
        if (P.trace && blockIdx.x == 0 && threadIdx.x == 0)
            printf("ZPOP seq=%d linked=%d ns=%d leaf=%d\n", sc->b7, x >= 0 ? 1 : 0,
                   x >= 0 ? int(ns_of(L.meta[block_start(L, x, 1)])) : -9, x);
        if (x < 0) continue;
        if (threadIdx.x == 0) sc->b5 = zamboni_block(L, P, x);
        __syncthreads();
        if (sc->b5) compact(L);
    }
    __syncthreads();
}

// updateSeqNumbers + setMinSeq, client.ts:877-887 / mergeTree.ts:1025-1044
__device__ void update_seq(Lds& L, const KParams& P, int msn, int seq) {
    Sc* sc = L.sc;
    __syncthreads();
    int run = 0;
    if (threadIdx.x == 0) {
        if (sc->curseq > seq) sc->status = MTR_ERR_ASSERT | 0x038;
        else {
            sc->curseq = seq;
            if (msn > seq) sc->status = MTR_ERR_ASSERT | 0x039;
            else if (msn > sc->curseq) sc->status = MTR_ERR_ASSERT | 0x04e;
            else if (sc->minseq > msn) sc->status = MTR_ERR_ASSERT | 0x04f;
            else if (msn > sc->minseq) {
                sc->minseq = msn;
                run = 1;
            }
        }
        sc->b6 = run;
    }
    __syncthreads();
    if (sc->b6) zamboni(L, P);
}

// ------------------------------------------------------------------ boundary / insert
// ensureIntervalBoundary (mergeTree.ts:1706-1716): split the leaf holding pos at offset > 0
__device__ void ensure_boundary(Lds& L, const KParams& P, const View& v, int pos) {
    Sc* sc = L.sc;
    prefix(L, v, P.new_length_calc);
    if (threadIdx.x == 0) {
        sc->b0 = -1;
        const int S = sc->nseg;
        int i = lower_bound_E(L, pos);
        if (i < S) {
            const int be = block_end(L, i, 1);
            for (int j = i; j < be; j++) {
                if (L.V[j] < 0) continue;
                if (pos < L.E[j]) {
                    int off = pos - (L.E[j] - L.V[j]);
                    if (off > 0 && !(L.meta[j] & M_MARKER)) {
                        sc->b0 = j;
                        sc->b1 = off;
                    }
                    break;
                }
            }
        }
    }
    __syncthreads();
    const int j = sc->b0;
    if (j < 0) return;
    shift_right1(L, j + 1);
    if (threadIdx.x == 0) {  // BaseSegment.splitAt, mergeTreeNodes.ts:481-510
        const int off = sc->b1;
        const int r = j + 1;
        L.len[r] = L.len[j] - off;
        L.len[j] = off;
        L.seq[r] = L.seq[j];
        L.rseq[r] = L.rseq[j];
        L.meta[r] = set_ns(set_bnd(L.meta[j], 0), NS_UNDEF);
        L.text[r] = L.text[j] + uint32_t(off);
        L.props[r] = L.props[j];
        L.rm[r] = L.rm[j];
        L.uid[r] = uint32_t(sc->uidnext++);
        sc->nseg++;
        overflow_fix(L, r);
    }
    __syncthreads();
}

// insertSegments/blockInsert/insertingWalk with onLeaf (mergeTree.ts:1397-1427, 1594-1685)
__device__ void insert_segment(Lds& L, const KParams& P, const View& v, const mtr_op& op, int seq,
                               uint32_t client, const mtr_doc_desc& dd, int tie_seq) {
    Sc* sc = L.sc;
    const bool marker = (op.flags & MTR_F_MARKER) != 0;
    const int len = marker ? 1 : int(op.payload2);
    if (len <= 0) return;  // blockInsert skips empty segments
    // copy the op's text into the document arena (all lanes)
    const int t0 = sc->textused;
    if (!marker) {
        if (t0 + len > text_end(sc, P)) {
            __syncthreads();
            if (threadIdx.x == 0) sc->status = MTR_ERR_CAPACITY;
            __syncthreads();
            return;
        }
        const uint16_t* src = P.btext + dd.text_base + op.payload;
        for (int k = threadIdx.x; k < len; k += NT) L.gtext[t0 + k] = src[k];
    }
    prefix(L, v, P.new_length_calc);
    const int pos = op.pos1;
    if (threadIdx.x == 0) {
        const int S = sc->nseg;
        int slot = -1, inherit = 0;
        if (S == 0) {
            if (pos == 0) slot = 0;
            else sc->status = MTR_ERR_INSERT_FAILED;
        } else {
            int i = lower_bound_E(L, pos);
            if (i >= S) {
                sc->status = MTR_ERR_INSERT_FAILED;
            } else {
                const int bs = block_start(L, i, 1), be = block_end(L, i, 1);
                slot = be;
                for (int j = i; j < be; j++) {
                    int vj = L.V[j];
                    if (vj < 0) continue;
                    if (L.E[j] > pos || (vj == 0 && tie_seq > L.seq[j])) {  // breakTie, mergeTree.ts:1719-1738
                        slot = j;
                        break;
                    }
                }
                inherit = slot == bs ? 1 : 0;
            }
        }
        sc->b0 = slot;
        sc->b1 = inherit;
    }
    __syncthreads();
    const int slot = sc->b0;
    if (slot < 0) return;
    shift_right1(L, slot);
    if (threadIdx.x == 0) {
        const int S = sc->nseg;
        uint32_t m = client & M_CLIENT_MASK;
        if (marker) m |= M_MARKER;
        if (op.flags & MTR_F_NOREF) m |= M_NOREF;
        if (S == 0) {
            sc->height = 1;
            m = set_bnd(m, 1);
        } else if (sc->b1) {
            uint32_t om = L.meta[slot + 1];
            m = set_bnd(m, bnd_of(om));
            m = set_ns(m, ns_of(om));
            L.meta[slot + 1] = set_ns(set_bnd(om, 0), NS_UNDEF);
        }
        L.len[slot] = len;
        L.seq[slot] = seq;
        L.rseq[slot] = RNONE;
        L.meta[slot] = m;
        L.text[slot] = marker ? op.payload : uint32_t(t0);
        if (!marker) sc->textused = t0 + len;
        uint32_t pr = NONE32;
        if ((op.flags & MTR_F_PROPS) && op.pos2 >= 0) pr = props_apply(L, P, NONE32, uint32_t(op.pos2));
        L.props[slot] = pr;
        L.rm[slot] = NONE32;
        L.uid[slot] = uint32_t(sc->uidnext++);
        sc->nseg = S + 1;
        overflow_fix(L, slot);
        // saveIfLocal (mergeTree.ts:1618-1637): remote segments above minSeq go to the LRU
        if (sc->collab && !v.local && seq > sc->minseq) add_lru(L, slot, seq);
    }
    __syncthreads();
}

// markRangeRemoved / annotateRange walk (mergeTree.ts:1955-2047, 1895-1953): leaves with
// visible length > 0 inside [start, end).
__device__ void range_op(Lds& L, const KParams& P, const View& v, int start, int end, int seq, uint32_t client,
                         int is_remove, uint32_t pp) {
    Sc* sc = L.sc;
    ensure_boundary(L, P, v, start);
    ensure_boundary(L, P, v, end);
    prefix(L, v, P.new_length_calc);
    if (threadIdx.x == 0 && end != start) {
        const int S = sc->nseg;
        uint32_t memo_old[4], memo_new[4];
        int nmemo = 0;
        for (int j = lower_bound_E(L, start + 1); j < S; j++) {
            int vj = L.V[j];
            if (L.E[j] - max(vj, 0) >= end) break;
            if (vj <= 0) continue;
            if (is_remove) {
                if (L.rseq[j] != RNONE) {  // overlapping remove: removedClientIds.push
                    if (sc->rmused + 1 > P.rcap) { sc->status = MTR_ERR_CAPACITY; break; }
                    uint32_t cell = uint32_t(sc->rmused++);
                    uint32_t nxt = (L.meta[j] & M_OVERLAP) ? L.rm[j] : 0xffffffu;
                    L.grm[cell] = (client << 24) | (nxt & 0xffffffu);
                    L.rm[j] = cell;
                    L.meta[j] |= M_OVERLAP;
                } else {
                    L.rseq[j] = seq;
                    L.meta[j] = (L.meta[j] & ~(0xffu << M_FREM_SHIFT) & ~M_OVERLAP) | (client << M_FREM_SHIFT);
                    L.rm[j] = NONE32;
                }
            } else {
                uint32_t old = L.props[j], nw = NONE32;
                int hit = -1;
                for (int q = 0; q < nmemo; q++)
                    if (memo_old[q] == old) { hit = q; break; }
                if (hit >= 0) {
                    nw = memo_new[hit];
                } else {
                    nw = props_apply(L, P, old, pp);
                    if (nmemo < 4) { memo_old[nmemo] = old; memo_new[nmemo] = nw; nmemo++; }
                    else { memo_old[3] = old; memo_new[3] = nw; }
                }
                L.props[j] = nw;
            }
            if (sc->collab && !v.local) add_lru(L, j, seq);
        }
    }
    __syncthreads();
}

// ------------------------------------------------------------------ state load/store
__device__ void load_doc(Lds& L, const KParams& P, uint32_t d) {
    const DocHdr& h = P.hdr[d];
    Sc* sc = L.sc;
    if (threadIdx.x == 0) {
        sc->nseg = h.nseg; sc->height = h.height; sc->minseq = h.minseq; sc->curseq = h.curseq;
        sc->collab = h.collab; sc->local = h.local; sc->heapn = h.heapn; sc->uidnext = h.uidnext;
        sc->textused = h.textused; sc->propused = h.propused; sc->rmused = h.rmused; sc->status = h.status;
        sc->fail_op = h.fail_op; sc->max_heap = h.max_heap; sc->ops_done = 0;
        sc->sum_s = 0; sc->sum_l = 0;
        sc->texthalf = h.texthalf;
    }
    __syncthreads();
    if (P.global_mode) return;
    const int S = sc->nseg;
    const uint32_t* g = P.seg + size_t(d) * NF * P.segcap;
    for (int i = threadIdx.x; i < S; i += NT) {
        L.len[i] = int(g[F_LEN * P.segcap + i]);
        L.seq[i] = int(g[F_SEQ * P.segcap + i]);
        L.rseq[i] = int(g[F_RSEQ * P.segcap + i]);
        L.meta[i] = g[F_META * P.segcap + i];
        L.text[i] = g[F_TEXT * P.segcap + i];
        L.props[i] = g[F_PROPS * P.segcap + i];
        L.rm[i] = g[F_RM * P.segcap + i];
        L.uid[i] = g[F_UID * P.segcap + i];
    }
    const int hn = sc->heapn;
    const uint32_t* gh = P.heap + size_t(d) * 2 * P.hcap;
    for (int i = threadIdx.x; i <= hn; i += NT) {
        L.hseq[i] = int(gh[i]);
        L.huid[i] = gh[P.hcap + i];
    }
    __syncthreads();
}

__device__ void store_doc(Lds& L, const KParams& P, uint32_t d) {
    __syncthreads();
    Sc* sc = L.sc;
    const int S = P.global_mode ? 0 : sc->nseg;
    uint32_t* g = P.seg + size_t(d) * NF * P.segcap;
    for (int i = threadIdx.x; i < S; i += NT) {
        g[F_LEN * P.segcap + i] = uint32_t(L.len[i]);
        g[F_SEQ * P.segcap + i] = uint32_t(L.seq[i]);
        g[F_RSEQ * P.segcap + i] = uint32_t(L.rseq[i]);
        g[F_META * P.segcap + i] = L.meta[i];
        g[F_TEXT * P.segcap + i] = L.text[i];
        g[F_PROPS * P.segcap + i] = L.props[i];
        g[F_RM * P.segcap + i] = L.rm[i];
        g[F_UID * P.segcap + i] = L.uid[i];
    }
    const int hn = P.global_mode ? -1 : sc->heapn;
    uint32_t* gh = P.heap + size_t(d) * 2 * P.hcap;
    for (int i = threadIdx.x; i <= hn; i += NT) {
        gh[i] = uint32_t(L.hseq[i]);
        gh[P.hcap + i] = L.huid[i];
    }
    if (threadIdx.x == 0) {
        DocHdr& h = P.hdr[d];
        h.nseg = sc->nseg; h.height = sc->height; h.minseq = sc->minseq; h.curseq = sc->curseq;
        h.collab = sc->collab; h.local = sc->local; h.heapn = sc->heapn; h.uidnext = sc->uidnext;
        h.textused = sc->textused; h.propused = sc->propused; h.rmused = sc->rmused; h.status = sc->status;
        h.op_cursor += sc->ops_done;
        h.fail_op = sc->fail_op;
        h.max_heap = sc->max_heap;
        h.texthalf = sc->texthalf;
        if (sc->ops_done) {
            atomicAdd(P.stat_ops, (unsigned long long)sc->ops_done);
            atomicAdd(P.stat_ops + 1, sc->sum_s);
            atomicAdd(P.stat_ops + 2, sc->sum_l);
        }
    }
}

// LDS bytes needed for a launch of capacity cap (leaves) / lhcap (heap slots)
constexpr size_t kScBytes = ((sizeof(Sc) + 15) & ~size_t(15)) + ((sizeof(mtr_synth_state) + 15) & ~size_t(15));
__host__ __device__ inline size_t lds_bytes(int cap, int lhcap) {
    return size_t(cap) * 4 * 10 + size_t(lhcap) * 4 * 2 + kScBytes;
}
__host__ __device__ inline size_t lds_bytes_global_mode() { return kScBytes; }

// global mode: every array lives in the document's HBM slab
__device__ inline void carve_global(Lds& L, char* smem, const KParams& P, uint32_t d) {
    uint32_t* g = P.seg + size_t(d) * NF * P.segcap;
    L.len = reinterpret_cast<int*>(g + F_LEN * P.segcap);
    L.seq = reinterpret_cast<int*>(g + F_SEQ * P.segcap);
    L.rseq = reinterpret_cast<int*>(g + F_RSEQ * P.segcap);
    L.meta = g + F_META * P.segcap;
    L.text = g + F_TEXT * P.segcap;
    L.props = g + F_PROPS * P.segcap;
    L.rm = g + F_RM * P.segcap;
    L.uid = g + F_UID * P.segcap;
    uint32_t* sx = P.scratch + size_t(d) * 2 * P.segcap;
    L.E = reinterpret_cast<int*>(sx);
    L.V = reinterpret_cast<int*>(sx + P.segcap);
    uint32_t* gh = P.heap + size_t(d) * 2 * P.hcap;
    L.hseq = reinterpret_cast<int*>(gh);
    L.huid = gh + P.hcap;
    L.sc = reinterpret_cast<Sc*>(smem);
    L.gst = reinterpret_cast<mtr_synth_state*>(smem + ((sizeof(Sc) + 15) & ~size_t(15)));
    L.cap = P.segcap;
    L.lhcap = P.hcap;
}

__device__ inline void carve(Lds& L, char* smem, int cap, int lhcap) {
    char* p = smem;
    auto take = [&](size_t n) { char* r = p; p += (n + 15) & ~size_t(15); return r; };
    L.len = reinterpret_cast<int*>(take(4 * size_t(cap)));
    L.seq = reinterpret_cast<int*>(take(4 * size_t(cap)));
    L.rseq = reinterpret_cast<int*>(take(4 * size_t(cap)));
    L.meta = reinterpret_cast<uint32_t*>(take(4 * size_t(cap)));
    L.text = reinterpret_cast<uint32_t*>(take(4 * size_t(cap)));
    L.props = reinterpret_cast<uint32_t*>(take(4 * size_t(cap)));
    L.rm = reinterpret_cast<uint32_t*>(take(4 * size_t(cap)));
    L.uid = reinterpret_cast<uint32_t*>(take(4 * size_t(cap)));
    L.E = reinterpret_cast<int*>(take(4 * size_t(cap)));
    L.V = reinterpret_cast<int*>(take(4 * size_t(cap)));
    L.hseq = reinterpret_cast<int*>(take(4 * size_t(lhcap)));
    L.huid = reinterpret_cast<uint32_t*>(take(4 * size_t(lhcap)));
    L.sc = reinterpret_cast<Sc*>(take(sizeof(Sc)));
    L.gst = reinterpret_cast<mtr_synth_state*>(take(sizeof(mtr_synth_state)));
    L.cap = cap;
    L.lhcap = lhcap;
}

// record mode: draw op `idx` of document d from the synthetic recipe using this engine's exact
// view length, write it (and its text) into the batch buffers
__device__ void gen_op(Lds& L, const KParams& P, uint32_t d, const mtr_doc_desc& dd, int idx) {
    Sc* sc = L.sc;
    mtr_op* rec = P.gen_ops + dd.op_begin + idx;
    if (idx == 0) {
        if (threadIdx.x == 0) {
            mtr_op z{};
            z.type = MTR_OP_START_COLLAB;
            *rec = z;
        }
        __syncthreads();
        return;
    }
    if (threadIdx.x == 0) {
        mtr_op op;
        mtr_synth_begin(&P.gen_cfg, L.gst, idx, &op);
        sc->b2 = op.ref_seq;
        sc->b3 = op.client;
        *rec = op;
    }
    __syncthreads();
    View v;
    v.ref = sc->b2;
    v.client = enc_client(sc->b3);
    v.local = 0;
    prefix(L, v, P.new_length_calc);
    if (threadIdx.x == 0) {
        const int S = sc->nseg;
        const int len = S > 0 ? L.E[S - 1] : 0;
        mtr_op op = *rec;
        mtr_synth_finish(&P.gen_cfg, L.gst, len, &op, P.gen_text + dd.text_base);
        *rec = op;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ the kernel
__global__ void __launch_bounds__(NT) apply_kernel(KParams P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t d = blockIdx.x;
    if (d >= P.n_docs) return;
    const mtr_doc_desc dd = P.docs[d];
    const int cursor = P.hdr[d].op_cursor;
    const int n_ops = min(int(dd.op_count) - cursor, P.ops_this_launch);
    if (n_ops <= 0 || P.hdr[d].status != MTR_OK) return;
    Lds L;
    if (P.global_mode) carve_global(L, smem, P, d);
    else carve(L, smem, P.cap, P.lhcap);
    L.gtext = P.text + size_t(d) * P.tcap;
    L.gprop = P.prop + size_t(d) * P.pcap;
    L.grm = P.rm + size_t(d) * P.rcap;
    load_doc(L, P, d);
    Sc* sc = L.sc;
    if (P.gen && threadIdx.x == 0) *L.gst = P.gen_state[d];
    for (int k = 0; k < n_ops; k++) {
        if (P.gen) gen_op(L, P, d, dd, cursor + k);
        const mtr_op op = P.ops[dd.op_begin + cursor + k];
        if (threadIdx.x == 0) {
            sc->b3 = op.seq;  // (debug trace only)
            sc->sum_s += (unsigned long long)sc->nseg;
            if (op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT)
                sc->sum_l += (op.flags & MTR_F_MARKER) ? 0ull : (unsigned long long)op.payload2;
        }
        // text arena: keep room for this op's text plus zamboni merge copies
        {
            const int need = int(op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT ? op.payload2 : 0) + 4096;
            if (sc->textused + need > text_end(sc, P)) text_gc(L, P);
        }
        // capacity guard: every op adds at most two leaves
        if (sc->nseg + 2 >= L.cap) {
            if (threadIdx.x == 0) sc->status = MTR_ERR_CAPACITY;
            __syncthreads();
        }
        if (sc->status != MTR_OK) break;
        const bool local_op = op.type >= MTR_OP_LOCAL_INSERT && op.type <= MTR_OP_LOCAL_ANNOTATE;
        View v;
        int seq = op.seq;
        uint32_t client = enc_client(op.client);
        if (local_op) {
            if (sc->collab) {
                if (threadIdx.x == 0) sc->status = MTR_ERR_UNSUPPORTED;
                __syncthreads();
                break;
            }
            v.ref = sc->curseq;
            v.client = CL_LOCAL;
            v.local = 1;
            seq = 0;
            client = CL_LOCAL;
        } else {
            v.ref = op.ref_seq;
            v.client = client;
            v.local = (!sc->collab || uint32_t(sc->local) == client) ? 1 : 0;
        }
        const int tie_seq = seq;  // breakTie newSeq (never unassigned on this path)
        switch (op.type) {
            case MTR_OP_INSERT:
            case MTR_OP_LOCAL_INSERT:
                ensure_boundary(L, P, v, op.pos1);
                insert_segment(L, P, v, op, seq, client, dd, tie_seq);
                if (sc->collab && seq != -1) zamboni(L, P);
                break;
            case MTR_OP_REMOVE:
            case MTR_OP_LOCAL_REMOVE:
                range_op(L, P, v, op.pos1, op.pos2, seq, client, 1, 0);
                if (sc->collab && seq != -1) zamboni(L, P);
                break;
            case MTR_OP_ANNOTATE:
            case MTR_OP_LOCAL_ANNOTATE:
                range_op(L, P, v, op.pos1, op.pos2, seq, client, 0, op.payload);
                if (sc->collab && seq != -1) zamboni(L, P);
                break;
            case MTR_OP_SEQ:
                break;
            case MTR_OP_START_COLLAB:
                if (threadIdx.x == 0 && !sc->collab) {
                    sc->collab = 1;
                    sc->local = 0;
                    sc->minseq = op.min_seq;
                    sc->curseq = op.seq;
                    sc->heapn = 0;
                }
                __syncthreads();
                break;
            default:
                if (threadIdx.x == 0) sc->status = MTR_ERR_BAD_OP;
                __syncthreads();
                break;
        }
        if (!local_op && op.type != MTR_OP_START_COLLAB && (op.flags & MTR_F_LAST) && sc->status == MTR_OK)
            update_seq(L, P, op.min_seq, op.seq);
        __syncthreads();
        if (threadIdx.x == 0) {
            if (sc->status != MTR_OK) sc->fail_op = cursor + k;
            else sc->ops_done = k + 1;
        }
        __syncthreads();
        if (sc->status != MTR_OK) break;
    }
    if (P.gen && threadIdx.x == 0) P.gen_state[d] = *L.gst;
    store_doc(L, P, d);
}

}  // namespace mtr
