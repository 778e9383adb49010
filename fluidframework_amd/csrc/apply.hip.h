// apply.hip.h -- the op-apply kernel of the MI355X merge-tree replay engine.
//
// One workgroup (256 threads = 4 wave64) owns one document for the whole launch and applies
// that document's ops strictly in order (ops never cross documents).  The document's leaves
// live as flat structure-of-arrays records in tree order -- in LDS when they fit, otherwise in
// the document's HBM slab (Doc<true>, same code) -- and the reference's B+tree
// (MaxNodesInBlock = 8, mergeTreeNodes.ts:330) is kept exactly, encoded per leaf as `bnd` =
// number of tree levels at which the leaf starts a block.
//
// Per op, the O(S) work runs on all lanes: one visibility prefix scan for the op's
// (refSeq, clientId) view, which replaces PartialSequenceLengths (partialLengths.ts:698) and the
// length queries of insertingWalk / nodeMap (mergeTree.ts:1740, 2526); the one-slot shift that
// makes room for a split or an insert (mergeTree.ts:1831-1838); the uid search for popped LRU
// entries; and the stream compaction after zamboni (zamboni.ts:19-120).  The scan arrays stay
// valid across the op's splits, so an op scans once.  The sequential control (tie-break, block
// splits, heap, zamboni scour/pack decisions) runs as uniform code on wave 0, whose 64 lanes turn
// every walk over leaves (block bounds, binary search, child counts, pack relabelling) into ballots
// and every HBM access (text copies, property sets) into one coalesced round trip; waves 1-3 wait
// at the next barrier.
//
// Memory spaces are explicit: LDS arrays are address_space(3) pointers (ds_read/ds_write),
// HBM arrays address_space(1) (global_load/store) -- never generic flat accesses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mtr_synth.h"
#include "../../include/mtr_types.h"

namespace mtr {

constexpr int NT = 64;
constexpr int NWAVES = NT / 64;
constexpr int32_t RNONE = 0x7fffffff;  // removedSeq of a live leaf
constexpr uint32_t NONE32 = 0xffffffffu;
constexpr int kMaxNodesInBlock = 8;
constexpr int kGranularity = 256;  // TextSegmentGranularity, textSegment.ts:35
constexpr int MAXH = 16;           // max tree height

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
constexpr uint32_t M_NL = 1u << 26;   // text leaf whose last unit is '\n' (TextSegment.canAppend)
constexpr uint32_t M_NLQ = 1u << 27;  // M_NL not known yet (left half of a split): read lazily by scour
constexpr uint32_t NS_UNDEF = 0, NS_FALSE = 1, NS_TRUE = 2;

constexpr uint32_t CL_LOCAL = 0xffu;      // LocalClientId (-1)
constexpr uint32_t CL_NONCOLLAB = 0xfeu;  // NonCollabClient (-2)

__host__ __device__ inline uint32_t enc_client(int c) {
    return c >= 0 ? uint32_t(c) & 0xffu : (c == -1 ? CL_LOCAL : CL_NONCOLLAB);
}
__host__ __device__ inline int dec_client(uint32_t e) { return e == CL_LOCAL ? -1 : (e == CL_NONCOLLAB ? -2 : int(e)); }

template <class T>
using lptr = __attribute__((address_space(3))) T*;
template <class T>
using gptr = __attribute__((address_space(1))) T*;
template <class T>
__device__ inline gptr<T> gp(T* p) {
    return (gptr<T>)(p);
}

// Whole-struct copies through address-space-qualified pointers (C++ copy operations expect
// generic `this`), done word by word so they stay global_/ds_ accesses.
template <class T, class Q>
__device__ inline T ld_struct(Q p) {
    static_assert(sizeof(T) % 4 == 0, "word-sized struct");
    typedef typename std::conditional<std::is_same<Q, lptr<T>>::value || std::is_same<Q, lptr<const T>>::value,
                                      lptr<const uint32_t>, gptr<const uint32_t>>::type W;
    const W w = (W)p;
    uint32_t v[sizeof(T) / 4];
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; i++) v[i] = w[i];
    T t;
    __builtin_memcpy(&t, v, sizeof(T));
    return t;
}
template <class T, class Q>
__device__ inline void st_struct(Q p, const T& t) {
    static_assert(sizeof(T) % 4 == 0, "word-sized struct");
    typedef typename std::conditional<std::is_same<Q, lptr<T>>::value, lptr<uint32_t>, gptr<uint32_t>>::type W;
    const W w = (W)p;
    uint32_t v[sizeof(T) / 4];
    __builtin_memcpy(v, &t, sizeof(T));
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; i++) w[i] = v[i];
}

// Per-document header in HBM (64 bytes)
struct DocHdr {
    int32_t nseg, height, minseq, curseq;
    int32_t collab, local, heapn, uidnext;
    int32_t textused, propused, rmused, status;
    int32_t op_cursor, fail_op, max_heap, texthalf;  // texthalf: active half of the text arena
};

// 32-bit SoA fields per leaf kept in HBM and LDS
constexpr int NF = 8;
enum { F_LEN = 0, F_SEQ, F_RSEQ, F_META, F_TEXT, F_PROPS, F_RM, F_UID };

struct KParams {
    DocHdr* hdr;
    uint32_t* seg;   // [doc][NF][segcap]
    uint32_t* heap;  // [doc][2][hcap]   (seq, uid), 1-based
    uint16_t* text;  // [doc][tcap]
    uint32_t* prop;  // [doc][pcap]
    uint32_t* rm;    // [doc][rcap]
    int32_t segcap, hcap, tcap, pcap, rcap;
    int32_t cap;          // leaf capacity of this launch (LDS mode)
    int32_t lhcap;        // heap capacity of this launch (LDS mode)
    int32_t global_mode;  // 1: leaves/heap stay in HBM (documents larger than LDS)
    uint32_t* scratch;    // [doc][2][segcap] E/V arrays for global mode
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
    unsigned long long* stat_ops;  // [0] ops applied, [1] sum of leaves before ops, [2] inserted units
    // record mode (synthetic workloads): ops are drawn from include/mtr_synth.h with this
    // engine's own exact view lengths, written to gen_ops/gen_text, then applied
    int32_t gen;
    mtr_synth_cfg gen_cfg;
    mtr_synth_state* gen_state;  // [doc]
    mtr_op* gen_ops;             // == ops, writable
    uint16_t* gen_text;          // == btext, writable
};

// phase-timer slots (-DMTR_PROF builds)
enum { P_OP = 0, P_PREFIX, P_SPLIT, P_SHIFT, P_INSERT, P_RANGE, P_ZAMBONI, P_ZBLOCK, P_COMPACT, P_FINDUID,
       P_TEXTGC, P_LOADSTORE, P_TEXTCOPY, P_UPDSEQ, P_NZBLOCK, P_NCOMPACT, P_SCOUR1, P_PACK, P_NLQ, P_PMATCH,
       P_TAPPEND, P_HEAP, P_OVERFLOW, P_NPACK, P_NMERGE, P_NPMATCH, P_NNLQ, P_SPLIT1, P_INS1, P_FETCH, P_X1, P_X2,
       P_COUNT };

// scalar document state, broadcast slots and lane-0 scratch, in LDS
struct Sc {
    int nseg, height, minseq, curseq;
    int collab, local, heapn, uidnext;
    int textused, propused, rmused, status;
    int b0, b1, b2, b3;
    int b4, b5, b6, b7;
    int red[2 * NWAVES];
    int fail_op, max_heap, ops_done, texthalf;
    unsigned long long sum_s, sum_l;  // sum over ops of the leaf count before the op / inserted units
    int rs[MAXH + 1], re[MAXH + 1], topb[MAXH + 1];
    uint32_t memo_old[4], memo_new[4];
#ifdef MTR_PROF
    unsigned long long prof[P_COUNT];
#endif
};

struct View {
    int ref;
    uint32_t client;  // encoded
    int local;        // local-view rules (mergeTree.ts:613-634)
};

template <bool G>
struct Doc {
    template <class T>
    using A = typename std::conditional<G, gptr<T>, lptr<T>>::type;
    A<int> len, seq, rseq, E, V, hseq;
    A<uint32_t> meta, text, props, rm, uid, huid;
    lptr<Sc> sc;
    lptr<mtr_synth_state> gst;
    gptr<uint16_t> gtext;
    gptr<uint32_t> gprop, grm;
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
__device__ inline int lane_id() { return int(threadIdx.x & 63); }
__device__ inline uint64_t lanes_below() { return (uint64_t(1) << lane_id()) - 1; }
__device__ inline int first_lane(uint64_t m) { return __ffsll((long long)m) - 1; }
template <class T>
__device__ inline T rdlane(T x, int l) {  // v_readlane with a wave-uniform lane index
    return T(__builtin_amdgcn_readlane(int(x), l));
}
// order this wave's LDS/HBM writes before its later reads (other lanes' addresses included)
__device__ inline void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}
__device__ inline bool wave0() { return threadIdx.x < 64; }
__device__ inline int wave_max(int x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x = max(x, __shfl_xor(x, d, 64));
    return x;
}

// exclusive block scan; also returns the block total in *total
__device__ inline int block_excl_scan(lptr<Sc> sc, int x, int* total) {
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
__device__ inline int block_max(lptr<Sc> sc, int x) {
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

// matchProperties (properties.ts:71-105) with values compared by equivalence class
template <class PA, class PB>
__device__ bool props_match(PA gprop, PB val_eq, uint32_t a, uint32_t b) {
    if (a == b) return true;
    if (a == NONE32 || b == NONE32) return false;
    const uint32_t na = gprop[a], nb = gprop[b];
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
        const uint32_t k = gprop[a + 1 + 2 * i];
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

constexpr size_t kScBytes = ((sizeof(Sc) + 15) & ~size_t(15)) + ((sizeof(mtr_synth_state) + 15) & ~size_t(15));
// LDS bytes of a launch with leaf capacity cap and heap capacity lhcap (10 leaf arrays + heap)
__host__ __device__ inline size_t lds_bytes(int cap, int lhcap) {
    return size_t(cap) * 4 * 10 + size_t(lhcap) * 4 * 2 + kScBytes;
}
__host__ __device__ inline size_t lds_bytes_global_mode() { return kScBytes; }

// Phase timers (builds with -DMTR_PROF only): thread-0 clock cycles per phase, summed over
// documents into g_prof (mtr_profile()).

#ifdef MTR_PROF
__device__ unsigned long long g_prof[P_COUNT];
struct ProfScope {
    lptr<Sc> sc;
    int id;
    long long t;
    __device__ ProfScope(lptr<Sc> s, int i) : sc(s), id(i), t(threadIdx.x == 0 ? clock64() : 0) {}
    __device__ ~ProfScope() {
        if (threadIdx.x == 0) sc->prof[id] += (unsigned long long)(clock64() - t);
    }
};
#define PROF(id) ProfScope _prof_scope(L.sc, id)
#define PROF_COUNT(id) \
    if (threadIdx.x == 0) L.sc->prof[id]++
#else
#define PROF(id)
#define PROF_COUNT(id)
#endif

template <bool G>
struct Eng {
    using D = Doc<G>;
    template <class T>
    using A = typename D::template A<T>;

    // ------------------------------------------------------------ visibility
    static __device__ bool in_removers(const D& L, int i, uint32_t c) {
        const uint32_t m = L.meta[i];
        if (((m >> M_FREM_SHIFT) & 0xffu) == c) return true;
        if (!(m & M_OVERLAP)) return false;
        uint32_t cell = L.rm[i];
        while (cell != 0xffffffu) {
            const uint32_t v = L.grm[cell];
            if ((v >> 24) == c) return true;
            cell = v & 0xffffffu;
        }
        return false;
    }

    // nodeLength for a leaf (mergeTree.ts:916-1004): -1 = undefined
    static __device__ int vis_len(const D& L, int i, const View& v, int newlen, int minseq) {
        const int len = L.len[i];
        const int rseq = L.rseq[i];
        const bool removed = rseq != RNONE;
        if (v.local) {  // localNetLength, mergeTree.ts:613-634
            if (removed) return newlen ? 0 : (rseq > minseq ? 0 : -1);
            return len;
        }
        const uint32_t m = L.meta[i];
        const uint32_t cl = m & M_CLIENT_MASK;
        const int seq = L.seq[i];
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
    static __device__ void prefix(D& L, const View& v, int newlen) {
        PROF(P_PREFIX);
        const int S = L.sc->nseg;
        const int minseq = L.sc->minseq;
        const int per = (S + NT - 1) / NT;
        const int lo = min(S, int(threadIdx.x) * per), hi = min(S, lo + per);
        int sum = 0;
        for (int i = lo; i < hi; i++) {
            const int x = vis_len(L, i, v, newlen, minseq);
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

    // ------------------------------------------------------------ data movement
    // move leaves [at, S) (with their scan entries) to [at+1, S+1); rounds of NT from the top
    static __device__ void shift_right1(D& L, int at) {
        PROF(P_SHIFT);
        const int S = L.sc->nseg;
        for (int hi = S; hi > at; hi -= NT) {
            const int lo = max(at, hi - NT);
            const int i = lo + int(threadIdx.x);
            const bool act = i < hi;
            int a0 = 0, a1 = 0, a2 = 0, a8 = 0, a9 = 0;
            uint32_t a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
            if (act) {
                a0 = L.len[i]; a1 = L.seq[i]; a2 = L.rseq[i]; a3 = L.meta[i]; a4 = L.text[i];
                a5 = L.props[i]; a6 = L.rm[i]; a7 = L.uid[i]; a8 = L.E[i]; a9 = L.V[i];
            }
            __syncthreads();
            if (act) {
                L.len[i + 1] = a0; L.seq[i + 1] = a1; L.rseq[i + 1] = a2; L.meta[i + 1] = a3; L.text[i + 1] = a4;
                L.props[i + 1] = a5; L.rm[i + 1] = a6; L.uid[i + 1] = a7; L.E[i + 1] = a8; L.V[i + 1] = a9;
            }
            __syncthreads();
        }
    }

    // stream compaction of leaves without M_DEL (zamboni unlink / append); rounds of NT from
    // the bottom; destinations never exceed sources
    static __device__ void compact(D& L) {
        PROF(P_COMPACT);
        PROF_COUNT(P_NCOMPACT);
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
            const int keep = (act && !(a3 & M_DEL)) ? 1 : 0;
            int tot;
            const int off = block_excl_scan(L.sc, keep, &tot);  // its barriers order reads before writes
            if (keep) {
                const int d = base + off;
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
    static __device__ int find_uid(D& L, uint32_t u) {
        PROF(P_FINDUID);
        const int S = L.sc->nseg;
        int found = -1;
        for (int i = threadIdx.x; i < S; i += NT)
            if (L.uid[i] == u) found = i;
        return block_max(L.sc, found);
    }

    // ------------------------------------------------------------ wave-0 helpers
    // (uniform code on wave 0: every lane holds the same scalars; the searches are ballots)

    // start of the level-`level` block holding leaf x: last i <= x with i == 0 or bnd >= level
    static __device__ int block_start(const D& L, int x, int level) {
        for (int base = x;; base -= 64) {
            const int i = base - lane_id();
            const uint64_t m = __ballot(i <= 0 || bnd_of(L.meta[i]) >= level);
            if (m) return max(0, base - first_lane(m));
        }
    }
    // end (exclusive) of the level-`level` block holding leaf x
    static __device__ int block_end(const D& L, int x, int level) {
        const int S = L.sc->nseg;
        for (int base = x + 1;; base += 64) {
            const int i = base + lane_id();
            const uint64_t m = __ballot(i >= S || bnd_of(L.meta[i]) >= level);
            if (m) return base + first_lane(m);
        }
    }
    // first i with E[i] >= pos (S if none): 64-ary search
    static __device__ int lower_bound_E(const D& L, int pos) {
        int lo = 0, hi = L.sc->nseg;  // answer in [lo, hi]
        const int ln = lane_id();
        while (hi - lo > 64) {
            const int stride = (hi - lo + 63) >> 6;
            const int idx = lo + (ln + 1) * stride - 1;
            const uint64_t m = __ballot(idx >= hi || L.E[idx] >= pos);
            const int k = first_lane(m);  // lane 63 always qualifies
            const int nlo = lo + k * stride;
            hi = min(hi, lo + (k + 1) * stride - 1);
            lo = nlo;
        }
        const int i = lo + ln;
        const uint64_t m = __ballot(i < hi && L.E[i] >= pos);
        return m ? lo + first_lane(m) : hi;
    }
    // number of leaves in [bs, be) with bnd >= minb
    static __device__ int count_bnd(const D& L, int bs, int be, int minb) {
        int c = 0;
        for (int base = bs; base < be; base += 64) {
            const int i = base + lane_id();
            c += __popcll(__ballot(i < be && bnd_of(L.meta[i]) >= minb));
        }
        return c;
    }
    // index of the n-th (0-based) leaf in [bs, be) with bnd >= minb, -1 if none
    static __device__ int nth_bnd(const D& L, int bs, int be, int minb, int n) {
        for (int base = bs; base < be; base += 64) {
            const int i = base + lane_id();
            const bool t = i < be && bnd_of(L.meta[i]) >= minb;
            const uint64_t m = __ballot(t);
            const int pc = __popcll(m);
            if (n < pc) return base + first_lane(__ballot(t && __popcll(m & lanes_below()) == n));
            n -= pc;
        }
        return -1;
    }

    // Block overflow after a leaf was added next to x (insertingWalk split + updateRoot,
    // mergeTree.ts:1831-1871, 1268-1277).
    static __device__ void overflow_fix(D& L, int x) {
        PROF(P_OVERFLOW);
        lptr<Sc> sc = L.sc;
        int level = 1;
        int bs = block_start(L, x, 1), be = block_end(L, x, 1);
        int cnt = be - bs;
        while (cnt >= kMaxNodesInBlock) {
            int c5 = bs + kMaxNodesInBlock / 2;
            if (level > 1) c5 = nth_bnd(L, bs, be, level - 1, kMaxNodesInBlock / 2);
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
            cnt = count_bnd(L, bs, be, level - 1);
        }
    }

    // ---- LRU heap (collections/heap.ts:11-67), 1-based, lane 0 only
    static __device__ void heap_push(D& L, uint32_t u, int s) {
        lptr<Sc> sc = L.sc;
        if (sc->heapn + 1 >= L.lhcap) {
            sc->status = MTR_ERR_CAPACITY;
            return;
        }
        int k = ++sc->heapn;
        L.hseq[k] = s;
        L.huid[k] = u;
        while (k > 1 && L.hseq[k >> 1] - L.hseq[k] > 0) {
            const int ts = L.hseq[k >> 1];
            const uint32_t tu = L.huid[k >> 1];
            L.hseq[k >> 1] = L.hseq[k];
            L.huid[k >> 1] = L.huid[k];
            L.hseq[k] = ts;
            L.huid[k] = tu;
            k >>= 1;
        }
        if (sc->heapn > sc->max_heap) sc->max_heap = sc->heapn;
    }
    static __device__ uint32_t heap_pop(D& L) {
        PROF(P_HEAP);
        lptr<Sc> sc = L.sc;
        const uint32_t x = L.huid[1];
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
            const int ts = L.hseq[k];
            const uint32_t tu = L.huid[k];
            L.hseq[k] = L.hseq[j];
            L.huid[k] = L.huid[j];
            L.hseq[j] = ts;
            L.huid[j] = tu;
            k = j;
        }
        return x;
    }

    // addToLRUSet, mergeTree.ts:741-751
    static __device__ void add_lru(D& L, int i, int s) {
        lptr<Sc> sc = L.sc;
        const int bs = block_start(L, i, 1);
        const uint32_t m = L.meta[bs];
        if (ns_of(m) != NS_TRUE && s > sc->curseq) {
            L.meta[bs] = set_ns(m, NS_TRUE);
            heap_push(L, L.uid[i], s);
        }
    }

    // ---- properties (PropertiesManager.addProperties without combining ops,
    //      segmentPropertiesManager.ts:60-157; JS own-key order).  Entry: [n, k0, v0, k1, v1, ...]
    static __device__ uint32_t props_apply_serial(D& L, const KParams& P, uint32_t old, uint32_t pp) {
        lptr<Sc> sc = L.sc;
        const gptr<const uint32_t> poff = gp(P.propop_off), pkv = gp(P.propop_kv), kix = gp(P.key_index);
        const uint32_t n_old = old == NONE32 ? 0 : L.gprop[old];
        const uint32_t lo = poff[pp], hi = poff[pp + 1];
        const uint32_t need = 1 + 2 * (n_old + (hi - lo));
        if (uint32_t(sc->propused) + need > uint32_t(P.pcap)) {
            sc->status = MTR_ERR_CAPACITY;
            return old;
        }
        const uint32_t dst = uint32_t(sc->propused);
        const gptr<uint32_t> e = L.gprop + dst;
        uint32_t n = n_old;
        for (uint32_t k = 0; k < 2 * n_old; k++) e[1 + k] = L.gprop[old + 1 + k];
        for (uint32_t q = lo; q < hi; q++) {
            const uint32_t key = pkv[2 * q], val = pkv[2 * q + 1];
            int at = -1;
            for (uint32_t k = 0; k < n; k++)
                if (e[1 + 2 * k] == key) {
                    at = int(k);
                    break;
                }
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
                const uint32_t ix = kix[key];
                uint32_t pos = n;
                if (ix != MTR_NOT_INDEX) {
                    pos = 0;
                    while (pos < n && kix[e[1 + 2 * pos]] != MTR_NOT_INDEX && kix[e[1 + 2 * pos]] < ix) pos++;
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

    // Wave version: the old set and the op's keys are fetched once (one lane per entry) and the
    // set is edited in registers (lane t = entry t); falls back to the serial form above 64 keys.
    static __device__ uint32_t props_apply(D& L, const KParams& P, uint32_t old, uint32_t pp) {
        lptr<Sc> sc = L.sc;
        const gptr<const uint32_t> poff = gp(P.propop_off), pkv = gp(P.propop_kv), kix = gp(P.key_index);
        const int n_old = old == NONE32 ? 0 : int(L.gprop[old]);
        const int lo = int(poff[pp]), nq = int(poff[pp + 1]) - lo;
        if (n_old + nq > 64) return props_apply_serial(L, P, old, pp);
        const uint32_t need = 1 + 2 * uint32_t(n_old + nq);
        if (uint32_t(sc->propused) + need > uint32_t(P.pcap)) {
            sc->status = MTR_ERR_CAPACITY;
            return old;
        }
        const int ln = lane_id();
        uint32_t wk = 0, wv = 0, wx = MTR_NOT_INDEX, qk = 0, qv = 0, qx = MTR_NOT_INDEX;
        if (ln < n_old) {
            wk = L.gprop[old + 1 + 2 * ln];
            wv = L.gprop[old + 2 + 2 * ln];
        }
        if (ln < nq) {
            qk = pkv[2 * (lo + ln)];
            qv = pkv[2 * (lo + ln) + 1];
        }
        if (ln < n_old) wx = kix[wk];
        if (ln < nq) qx = kix[qk];
        int n = n_old;
        for (int q = 0; q < nq; q++) {
            const uint32_t key = rdlane(qk, q), val = rdlane(qv, q), ix = rdlane(qx, q);
            const uint64_t hit = __ballot(ln < n && wk == key);
            if (val == MTR_NULL_VALUE) {
                if (hit) {  // delete entry `at`: lanes above it move down one
                    const int at = first_lane(hit);
                    const uint32_t dk = __shfl(wk, min(ln + 1, 63)), dv = __shfl(wv, min(ln + 1, 63)),
                                   dx = __shfl(wx, min(ln + 1, 63));
                    if (ln >= at) {
                        wk = dk;
                        wv = dv;
                        wx = dx;
                    }
                    n--;
                }
            } else if (hit) {
                if (ln == first_lane(hit)) wv = val;
            } else {
                int pos = n;
                if (ix != MTR_NOT_INDEX) {  // index-like keys sort first (JS own-key order)
                    const uint64_t ge = __ballot(ln < n && !(wx != MTR_NOT_INDEX && wx < ix));
                    pos = ge ? first_lane(ge) : n;
                }
                const uint32_t uk = __shfl(wk, max(ln - 1, 0)), uv = __shfl(wv, max(ln - 1, 0)),
                               ux = __shfl(wx, max(ln - 1, 0));
                if (ln > pos) {
                    wk = uk;
                    wv = uv;
                    wx = ux;
                } else if (ln == pos) {
                    wk = key;
                    wv = val;
                    wx = ix;
                }
                n++;
            }
        }
        const uint32_t dst = uint32_t(sc->propused);
        const gptr<uint32_t> e = L.gprop + dst;
        if (ln < n) {
            e[1 + 2 * ln] = wk;
            e[2 + 2 * ln] = wv;
        }
        e[0] = uint32_t(n);
        sc->propused += 1 + 2 * n;
        wave_fence();
        return dst;
    }

    // matchProperties on wave 0: one lane per key of `a`, `b`'s keys broadcast by readlane
    static __device__ bool props_match_w(const D& L, const KParams& P, uint32_t a, uint32_t b) {
        if (a == b) return true;
        if (a == NONE32 || b == NONE32) return false;
        const int na = int(L.gprop[a]), nb = int(L.gprop[b]);
        if (na != nb) return false;
        const gptr<const uint32_t> veq = gp(P.val_eq);
        if (na > 64) return props_match(L.gprop, veq, a, b);
        PROF(P_PMATCH);
        PROF_COUNT(P_NPMATCH);
        const int ln = lane_id();
        uint32_t ka = 0, kb = 0, ea = 0, eb = 0;
        if (ln < na) {
            ka = L.gprop[a + 1 + 2 * ln];
            kb = L.gprop[b + 1 + 2 * ln];
            ea = veq[L.gprop[a + 2 + 2 * ln]];
            eb = veq[L.gprop[b + 2 + 2 * ln]];
        }
        bool ok = ln >= na;
        for (int j = 0; j < nb; j++) {
            const uint32_t kj = rdlane(kb, j), ej = rdlane(eb, j);
            if (ka == kj && ln < na) ok = ea == ej;
        }
        return __ballot(!ok) == 0;
    }

    // ---- text
    static __device__ bool can_append(uint32_t ma, int la, uint32_t mb, int lb) {  // TextSegment.canAppend, textSegment.ts:86-93
        if ((ma | mb) & M_MARKER) return false;
        if (la > 0 && (ma & M_NL)) return false;
        return la <= kGranularity || lb <= kGranularity;
    }
    static __device__ void copy_text(const D& L, uint32_t dst, uint32_t src, int n) {  // wave 0
        for (int k = lane_id(); k < n; k += 64) L.gtext[dst + k] = L.gtext[src + k];
    }
    static __device__ int text_end(lptr<Sc> sc, const KParams& P) { return (P.tcap / 2) * (sc->texthalf + 1); }

    // prev.append(seg) (textSegment.ts:99-103): text of b follows text of a
    // (wave 0; returns false on arena overflow).  Updates L.len/L.text of a; the caller keeps M_NL.
    static __device__ void text_append(D& L, const KParams& P, int a, int b) {
        PROF(P_TAPPEND);
        PROF_COUNT(P_NMERGE);
        lptr<Sc> sc = L.sc;
        const int tend = text_end(sc, P);
        const uint32_t oa = L.text[a], ob = L.text[b];
        const int la = L.len[a], lb = L.len[b];
        if (oa + uint32_t(la) == ob) {
            L.len[a] = la + lb;
            return;
        }
        if (oa + uint32_t(la) == uint32_t(sc->textused)) {
            if (sc->textused + lb > tend) {
                sc->status = MTR_ERR_CAPACITY;
                return;
            }
            copy_text(L, uint32_t(sc->textused), ob, lb);
            sc->textused += lb;
            L.len[a] = la + lb;
            return;
        }
        if (sc->textused + la + lb > tend) {
            sc->status = MTR_ERR_CAPACITY;
            return;
        }
        const uint32_t d = uint32_t(sc->textused);
        copy_text(L, d, oa, la);
        copy_text(L, d + uint32_t(la), ob, lb);
        sc->textused += la + lb;
        L.text[a] = d;
        L.len[a] = la + lb;
    }

    // Semi-space compaction of the text arena: copy every leaf's text into the other half in
    // leaf order (block prefix scan of lengths), then switch halves.
    static __device__ void text_gc(D& L, const KParams& P) {
        PROF(P_TEXTGC);
        lptr<Sc> sc = L.sc;
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

    // ------------------------------------------------------------ zamboni
    // scourNode (zamboni.ts:122-193) over the child blocks in [cs, ce): a new child block starts at
    // every leaf with bnd >= 1.  Marks M_DEL; returns #kept (used for a single block).  Wave 0:
    // the leaves are read 64 at a time into registers and visited in order by readlane.
    static __device__ int scour_range(D& L, const KParams& P, int cs, int ce) {
        lptr<Sc> sc = L.sc;
        const int minseq = sc->minseq;
        int prev = -1, kept = 0, plen = 0;
        uint32_t pmeta = 0, pprops = 0;
        for (int base = cs; base < ce; base += 64) {
            const int i = base + lane_id();
            uint32_t vm = M_DEL, vp = 0;
            int vr = 0, vs = 0, vl = 0;
            if (i < ce) {
                vm = L.meta[i];
                vr = L.rseq[i];
                vs = L.seq[i];
                vl = L.len[i];
                vp = L.props[i];
            }
            {  // merge candidates whose trailing-newline bit is unknown: one HBM round trip
                const bool q = (vm & (M_NLQ | M_DEL | M_MARKER)) == M_NLQ && vl > 0 && vr == RNONE && vs <= minseq;
                if (__ballot(q)) {
                    PROF(P_NLQ);
                    PROF_COUNT(P_NNLQ);
                    if (q) {
                        const uint16_t u = L.gtext[L.text[i] + uint32_t(vl) - 1];
                        vm = (vm & ~(M_NLQ | M_NL)) | (u == u'\n' ? M_NL : 0u);
                        L.meta[i] = vm;
                    }
                }
            }
            const int nk = min(64, ce - base);
            for (int t = 0; t < nk; t++) {
                const int k = base + t;
                const uint32_t m = rdlane(vm, t);
                if (k > cs && bnd_of(m) >= 1) prev = -1;  // next child block
                if (m & M_DEL) continue;
                const int rs = rdlane(vr, t);
                if (rs != RNONE) {
                    if (rs > minseq) kept++;
                    else L.meta[k] = m | M_DEL;  // UNLINK
                    prev = -1;
                } else if (rdlane(vs, t) <= minseq) {
                    const int lk = rdlane(vl, t);
                    const uint32_t pk = rdlane(vp, t);
                    if (prev >= 0 && lk > 0 && can_append(pmeta, plen, m, lk) && props_match_w(L, P, pprops, pk)) {
                        text_append(L, P, prev, k);
                        plen += lk;
                        pmeta = (pmeta & ~(M_NL | M_NLQ)) | (m & (M_NL | M_NLQ));
                        L.meta[prev] = pmeta;
                        L.meta[k] = m | M_DEL;
                    } else {
                        kept++;
                        if (lk > 0) {
                            prev = k;
                            pmeta = m;
                            plen = lk;
                            pprops = pk;
                        } else {
                            prev = -1;
                        }
                    }
                } else {
                    kept++;
                    prev = -1;
                }
            }
        }
        return kept;
    }

    // zamboniSegments body for one popped LRU entry whose segment is leaf x
    // (zamboni.ts:33-58 + packParent zamboni.ts:63-120).  Lane 0.  Returns 1 if leaves were
    // marked for deletion (the caller compacts).
    static __device__ int zamboni_block(D& L, const KParams& P, int x) {
        PROF(P_ZBLOCK);
        PROF_COUNT(P_NZBLOCK);
        lptr<Sc> sc = L.sc;
        const int H = sc->height;
        sc->rs[1] = block_start(L, x, 1);
        sc->re[1] = block_end(L, x, 1);
        if (ns_of(L.meta[sc->rs[1]]) == NS_FALSE) return 0;
        for (int l = 1; l <= H; l++) {
            if (l > 1) {
                sc->rs[l] = block_start(L, sc->rs[l - 1], l);
                sc->re[l] = block_end(L, sc->rs[l - 1], l);
            }
            sc->topb[l] = bnd_of(L.meta[sc->rs[l]]);
        }
        const int rs1 = sc->rs[1], re1 = sc->re[1];
        const int before = re1 - rs1;
        int kept;
        {
            PROF(P_SCOUR1);
            kept = scour_range(L, P, rs1, re1);
        }
        int first = -1;  // block.needsScour = false, kept on the block's first surviving leaf
        {
            const int i = rs1 + lane_id();
            const uint64_t m = __ballot(i < re1 && !(L.meta[i] & M_DEL));
            if (m) first = rs1 + first_lane(m);
        }
        if (first >= 0) L.meta[first] = set_ns(set_bnd(L.meta[first], sc->topb[1]), NS_FALSE);
        if (kept >= before) return 0;
        if (kept < kMaxNodesInBlock / 2 && H > 1) {
            PROF(P_PACK);
            PROF_COUNT(P_NPACK);
            for (int l = 2; l <= H; l++) {  // packParent chain
                const int ps = sc->rs[l], pe = sc->re[l];
                if (l == 2) {
                    // packParent scours every child of P again -- including the block just
                    // scoured: scourNode is not idempotent (a dropped tombstone no longer resets
                    // the merge candidate), zamboni.ts:68-73,122-193.
                    scour_range(L, P, ps, pe);
                }
                // items: surviving leaves (l == 2) or surviving level-(l-2) block starts
                int T = 0;
                for (int wb = ps; wb < pe; wb += 64) {
                    const int i = wb + lane_id();
                    const uint32_t m = i < pe ? L.meta[i] : M_DEL;
                    T += __popcll(__ballot(!(m & M_DEL) && (l == 2 || bnd_of(m) >= l - 2)));
                }
                int c = 0;
                if (T > 0) {  // rebalance into c blocks: the first `rem` get base+1 items
                    c = min(kMaxNodesInBlock - 1, T / (kMaxNodesInBlock / 2));
                    if (c < 1) c = 1;
                    const int base = T / c;
                    const int rem = T % c;
                    const int big = rem * (base + 1);
                    const int top = sc->topb[l];
                    int item0 = 0;
                    for (int wb = ps; wb < pe; wb += 64) {
                        const int i = wb + lane_id();
                        uint32_t m = i < pe ? L.meta[i] : M_DEL;
                        const bool it = !(m & M_DEL) && (l == 2 || bnd_of(m) >= l - 2);
                        const uint64_t mask = __ballot(it);
                        if (it) {
                            const int item = item0 + __popcll(mask & lanes_below());
                            const bool isStart = item < big ? item % (base + 1) == 0 : (item - big) % base == 0;
                            const int nb = item == 0 ? top : (isStart ? l - 1 : (l == 2 ? 0 : l - 2));
                            m = set_bnd(m, nb);
                            if (l == 2 && isStart) m = set_ns(m, NS_UNDEF);
                            L.meta[i] = m;
                        }
                        item0 += __popcll(mask);
                    }
                    wave_fence();
                }
                if (!(c < kMaxNodesInBlock / 2 && l < H)) break;
            }
        }
        return 1;
    }

    // zamboniSegments (zamboni.ts:19-60): all threads
    static __device__ void zamboni(D& L, const KParams& P) {
        PROF(P_ZAMBONI);
        lptr<Sc> sc = L.sc;
        if (!sc->collab) return;
        for (int it = 0; it < 2; it++) {
            __syncthreads();
            if (sc->heapn == 0 || sc->status != MTR_OK) return;
            if (L.hseq[1] > sc->minseq) return;
            __syncthreads();
            if (wave0()) sc->b4 = int(heap_pop(L));
            __syncthreads();
            const int x = find_uid(L, uint32_t(sc->b4));
            if (x < 0) continue;
            if (wave0()) sc->b5 = zamboni_block(L, P, x);
            __syncthreads();
            if (sc->b5) compact(L);
        }
        __syncthreads();
    }

    // updateSeqNumbers + setMinSeq, client.ts:877-887 / mergeTree.ts:1025-1044
    static __device__ void update_seq(D& L, const KParams& P, int msn, int seq) {
        PROF(P_UPDSEQ);
        lptr<Sc> sc = L.sc;
        __syncthreads();
        if (threadIdx.x == 0) {
            int run = 0;
            if (sc->curseq > seq) {
                sc->status = MTR_ERR_ASSERT | 0x038;
            } else {
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

    // ------------------------------------------------------------ boundary / insert
    // ensureIntervalBoundary (mergeTree.ts:1706-1716) on the current scan arrays: split the leaf
    // holding pos at an offset > 0; the two halves' scan entries are set in place.
    static __device__ void split_at(D& L, int pos) {
        PROF(P_SPLIT);
        lptr<Sc> sc = L.sc;
        if (wave0()) {
            PROF(P_SPLIT1);
            sc->b0 = -1;
            const int S = sc->nseg;
            const int i = lower_bound_E(L, pos);
            if (i < S) {
                const int be = block_end(L, i, 1);
                for (int j = i; j < be; j++) {
                    if (L.V[j] < 0) continue;
                    if (pos < L.E[j]) {
                        const int off = pos - (L.E[j] - L.V[j]);
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
        if (wave0()) {  // BaseSegment.splitAt, mergeTreeNodes.ts:481-510
            const int off = sc->b1;
            const int r = j + 1;
            const uint32_t mj = L.meta[j];
            L.len[r] = L.len[j] - off;
            L.len[j] = off;
            L.seq[r] = L.seq[j];
            L.rseq[r] = L.rseq[j];
            L.meta[r] = set_ns(set_bnd(mj, 0), NS_UNDEF);
            L.meta[j] = (mj & ~M_NL) | M_NLQ;
            L.text[r] = L.text[j] + uint32_t(off);
            L.props[r] = L.props[j];
            L.rm[r] = L.rm[j];
            L.uid[r] = uint32_t(sc->uidnext++);
            const int v = L.V[j], e = L.E[j];  // split leaves are fully visible in this view
            L.V[j] = off;
            L.E[j] = e - v + off;
            L.V[r] = v - off;
            L.E[r] = e;
            sc->nseg++;
            overflow_fix(L, r);
        }
        __syncthreads();
    }

    // insertSegments/blockInsert/insertingWalk with onLeaf (mergeTree.ts:1397-1427, 1594-1685),
    // on the current scan arrays
    // `pre`: lane t holds unit t of the op's text in `pf` (prefetched during the previous op)
    static __device__ void insert_at(D& L, const KParams& P, const View& v, const mtr_op& op, int seq,
                                     uint32_t client, const mtr_doc_desc& dd, bool pre, uint32_t pf) {
        PROF(P_INSERT);
        lptr<Sc> sc = L.sc;
        const bool marker = (op.flags & MTR_F_MARKER) != 0;
        const int len = marker ? 1 : int(op.payload2);
        if (len <= 0) return;  // blockInsert skips empty segments
        const int t0 = sc->textused;
        if (!marker) {  // copy the op's text into the document arena (all lanes)
            if (t0 + len > text_end(sc, P)) {
                __syncthreads();
                if (threadIdx.x == 0) sc->status = MTR_ERR_CAPACITY;
                __syncthreads();
                return;
            }
            PROF(P_TEXTCOPY);
            if (pre) {
                if (lane_id() < len) L.gtext[t0 + lane_id()] = uint16_t(pf);
            } else {
                const gptr<const uint16_t> src = gp(P.btext) + dd.text_base + op.payload;
                for (int k = threadIdx.x; k < len; k += NT) L.gtext[t0 + k] = src[k];
            }
        }
        const bool nl = pre && __ballot(lane_id() == len - 1 && pf == u'\n') != 0;
        const int pos = op.pos1;
        if (wave0()) {
            PROF(P_INS1);
            const int S = sc->nseg;
            int slot = -1, inherit = 0;
            if (S == 0) {
                if (pos == 0) slot = 0;
                else sc->status = MTR_ERR_INSERT_FAILED;
            } else {
                const int i = lower_bound_E(L, pos);
                if (i >= S) {
                    sc->status = MTR_ERR_INSERT_FAILED;
                } else {
                    const int bs = block_start(L, i, 1), be = block_end(L, i, 1);
                    slot = be;
                    for (int j = i; j < be; j++) {
                        const int vj = L.V[j];
                        if (vj < 0) continue;
                        if (L.E[j] > pos || (vj == 0 && seq > L.seq[j])) {  // breakTie, mergeTree.ts:1719-1738
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
        if (wave0()) {
            const int S = sc->nseg;
            uint32_t m = client & M_CLIENT_MASK;
            if (marker) m |= M_MARKER;
            else m |= pre ? (nl ? M_NL : 0u) : M_NLQ;
            if (op.flags & MTR_F_NOREF) m |= M_NOREF;
            if (S == 0) {
                sc->height = 1;
                m = set_bnd(m, 1);
            } else if (sc->b1) {
                const uint32_t om = L.meta[slot + 1];
                m = set_ns(set_bnd(m, bnd_of(om)), ns_of(om));
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
    // visible length > 0 inside [start, end), on the current scan arrays.  Lane 0.
    static __device__ void range_walk(D& L, const KParams& P, const View& v, int start, int end, int seq,
                                      uint32_t client, int is_remove, uint32_t pp) {
        PROF(P_RANGE);
        lptr<Sc> sc = L.sc;
        if (wave0() && end != start) {
            const int S = sc->nseg;
            int nmemo = 0;
            for (int j = lower_bound_E(L, start + 1); j < S; j++) {
                const int vj = L.V[j];
                if (L.E[j] - max(vj, 0) >= end) break;
                if (vj <= 0) continue;
                if (is_remove) {
                    if (L.rseq[j] != RNONE) {  // overlapping remove: removedClientIds.push
                        if (sc->rmused + 1 > P.rcap) {
                            sc->status = MTR_ERR_CAPACITY;
                            break;
                        }
                        const uint32_t cell = uint32_t(sc->rmused++);
                        const uint32_t nxt = (L.meta[j] & M_OVERLAP) ? L.rm[j] : 0xffffffu;
                        L.grm[cell] = (client << 24) | (nxt & 0xffffffu);
                        L.rm[j] = cell;
                        L.meta[j] |= M_OVERLAP;
                    } else {
                        L.rseq[j] = seq;
                        L.meta[j] = (L.meta[j] & ~(0xffu << M_FREM_SHIFT) & ~M_OVERLAP) | (client << M_FREM_SHIFT);
                        L.rm[j] = NONE32;
                    }
                } else {
                    const uint32_t old = L.props[j];
                    uint32_t nw = NONE32;
                    int hit = -1;
                    for (int q = 0; q < nmemo; q++)
                        if (sc->memo_old[q] == old) {
                            hit = q;
                            break;
                        }
                    if (hit >= 0) {
                        nw = sc->memo_new[hit];
                    } else {
                        nw = props_apply(L, P, old, pp);
                        const int q = nmemo < 4 ? nmemo++ : 3;
                        sc->memo_old[q] = old;
                        sc->memo_new[q] = nw;
                    }
                    L.props[j] = nw;
                }
                if (sc->collab && !v.local) add_lru(L, j, seq);
            }
        }
        __syncthreads();
    }

    // ------------------------------------------------------------ record mode
    // draw op `idx` of document d from the synthetic recipe using this engine's exact view length
    static __device__ void gen_op(D& L, const KParams& P, const mtr_doc_desc& dd, int idx) {
        lptr<Sc> sc = L.sc;
        const gptr<mtr_op> rec = gp(P.gen_ops) + dd.op_begin + idx;
        if (idx == 0) {
            if (threadIdx.x == 0) {
                mtr_op z{};
                z.type = MTR_OP_START_COLLAB;
                st_struct(rec, z);
            }
            __syncthreads();
            return;
        }
        if (threadIdx.x == 0) {
            mtr_op op;
            mtr_synth_state st = ld_struct<mtr_synth_state>(L.gst);
            mtr_synth_begin(&P.gen_cfg, &st, idx, &op);
            st_struct(L.gst, st);
            sc->b2 = op.ref_seq;
            sc->b3 = op.client;
            st_struct(rec, op);
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
            mtr_op op = ld_struct<mtr_op>(rec);
            mtr_synth_state st = ld_struct<mtr_synth_state>(L.gst);
            mtr_synth_finish(&P.gen_cfg, &st, len, &op, P.gen_text + dd.text_base);
            st_struct(L.gst, st);
            st_struct(rec, op);
        }
        __syncthreads();
    }

    // ------------------------------------------------------------ state load/store
    static __device__ void load_doc(D& L, const KParams& P, uint32_t d) {
        const gptr<const DocHdr> hp = gp((const DocHdr*)P.hdr) + d;
        lptr<Sc> sc = L.sc;
        if (threadIdx.x == 0) {
            const DocHdr h = ld_struct<DocHdr>(hp);
            sc->nseg = h.nseg; sc->height = h.height; sc->minseq = h.minseq; sc->curseq = h.curseq;
            sc->collab = h.collab; sc->local = h.local; sc->heapn = h.heapn; sc->uidnext = h.uidnext;
            sc->textused = h.textused; sc->propused = h.propused; sc->rmused = h.rmused; sc->status = h.status;
            sc->fail_op = h.fail_op; sc->max_heap = h.max_heap; sc->ops_done = 0; sc->texthalf = h.texthalf;
            sc->sum_s = 0;
            sc->sum_l = 0;
#ifdef MTR_PROF
            for (int q = 0; q < P_COUNT; q++) sc->prof[q] = 0;
#endif
            if (P.gen) st_struct(L.gst, ld_struct<mtr_synth_state>(gp(P.gen_state) + d));
        }
        __syncthreads();
        if (G) return;  // HBM-resident: nothing to stage
        const int S = sc->nseg;
        const int cs = P.segcap;
        const gptr<const uint32_t> g = gp((const uint32_t*)P.seg) + size_t(d) * NF * cs;
        for (int i = threadIdx.x; i < S; i += NT) {
            L.len[i] = int(g[F_LEN * cs + i]);
            L.seq[i] = int(g[F_SEQ * cs + i]);
            L.rseq[i] = int(g[F_RSEQ * cs + i]);
            L.meta[i] = g[F_META * cs + i];
            L.text[i] = g[F_TEXT * cs + i];
            L.props[i] = g[F_PROPS * cs + i];
            L.rm[i] = g[F_RM * cs + i];
            L.uid[i] = g[F_UID * cs + i];
        }
        const int hn = sc->heapn;
        const gptr<const uint32_t> gh = gp((const uint32_t*)P.heap) + size_t(d) * 2 * P.hcap;
        for (int i = threadIdx.x; i <= hn; i += NT) {
            L.hseq[i] = int(gh[i]);
            L.huid[i] = gh[P.hcap + i];
        }
        __syncthreads();
    }

    static __device__ void store_doc(D& L, const KParams& P, uint32_t d) {
        __syncthreads();
        lptr<Sc> sc = L.sc;
        if (!G) {
            const int S = sc->nseg;
            const int cs = P.segcap;
            const gptr<uint32_t> g = gp(P.seg) + size_t(d) * NF * cs;
            for (int i = threadIdx.x; i < S; i += NT) {
                g[F_LEN * cs + i] = uint32_t(L.len[i]);
                g[F_SEQ * cs + i] = uint32_t(L.seq[i]);
                g[F_RSEQ * cs + i] = uint32_t(L.rseq[i]);
                g[F_META * cs + i] = L.meta[i];
                g[F_TEXT * cs + i] = L.text[i];
                g[F_PROPS * cs + i] = L.props[i];
                g[F_RM * cs + i] = L.rm[i];
                g[F_UID * cs + i] = L.uid[i];
            }
            const int hn = sc->heapn;
            const gptr<uint32_t> gh = gp(P.heap) + size_t(d) * 2 * P.hcap;
            for (int i = threadIdx.x; i <= hn; i += NT) {
                gh[i] = uint32_t(L.hseq[i]);
                gh[P.hcap + i] = L.huid[i];
            }
        }
        if (threadIdx.x == 0) {
            const gptr<DocHdr> hp = gp(P.hdr) + d;
            DocHdr h = ld_struct<DocHdr>(hp);
            h.nseg = sc->nseg; h.height = sc->height; h.minseq = sc->minseq; h.curseq = sc->curseq;
            h.collab = sc->collab; h.local = sc->local; h.heapn = sc->heapn; h.uidnext = sc->uidnext;
            h.textused = sc->textused; h.propused = sc->propused; h.rmused = sc->rmused; h.status = sc->status;
            h.op_cursor += sc->ops_done;
            h.fail_op = sc->fail_op;
            h.max_heap = sc->max_heap;
            h.texthalf = sc->texthalf;
            st_struct(hp, h);
            if (P.gen) st_struct(gp(P.gen_state) + d, ld_struct<mtr_synth_state>(L.gst));
#ifdef MTR_PROF
            for (int q = 0; q < P_COUNT; q++) atomicAdd(&g_prof[q], sc->prof[q]);
#endif
            if (sc->ops_done) {
                atomicAdd(P.stat_ops, (unsigned long long)sc->ops_done);
                atomicAdd(P.stat_ops + 1, sc->sum_s);
                atomicAdd(P.stat_ops + 2, sc->sum_l);
            }
        }
    }

    static __device__ void carve(D& L, char* smem, const KParams& P, uint32_t d) {
        if (G) {  // every array lives in the document's HBM slab
            const gptr<uint32_t> g = gp(P.seg) + size_t(d) * NF * P.segcap;
            L.len = (A<int>)(g + F_LEN * P.segcap);
            L.seq = (A<int>)(g + F_SEQ * P.segcap);
            L.rseq = (A<int>)(g + F_RSEQ * P.segcap);
            L.meta = (A<uint32_t>)(g + F_META * P.segcap);
            L.text = (A<uint32_t>)(g + F_TEXT * P.segcap);
            L.props = (A<uint32_t>)(g + F_PROPS * P.segcap);
            L.rm = (A<uint32_t>)(g + F_RM * P.segcap);
            L.uid = (A<uint32_t>)(g + F_UID * P.segcap);
            const gptr<uint32_t> sx = gp(P.scratch) + size_t(d) * 2 * P.segcap;
            L.E = (A<int>)(sx);
            L.V = (A<int>)(sx + P.segcap);
            const gptr<uint32_t> gh = gp(P.heap) + size_t(d) * 2 * P.hcap;
            L.hseq = (A<int>)(gh);
            L.huid = (A<uint32_t>)(gh + P.hcap);
            L.cap = P.segcap;
            L.lhcap = P.hcap;
            L.sc = (lptr<Sc>)(smem);
            L.gst = (lptr<mtr_synth_state>)(smem + ((sizeof(Sc) + 15) & ~size_t(15)));
        } else {
            const int cap = P.cap, lhcap = P.lhcap;
            char* p = smem;
            auto take = [&](size_t n) {
                char* r = p;
                p += (n + 15) & ~size_t(15);
                return r;
            };
            L.len = (A<int>)(take(4 * size_t(cap)));
            L.seq = (A<int>)(take(4 * size_t(cap)));
            L.rseq = (A<int>)(take(4 * size_t(cap)));
            L.meta = (A<uint32_t>)(take(4 * size_t(cap)));
            L.text = (A<uint32_t>)(take(4 * size_t(cap)));
            L.props = (A<uint32_t>)(take(4 * size_t(cap)));
            L.rm = (A<uint32_t>)(take(4 * size_t(cap)));
            L.uid = (A<uint32_t>)(take(4 * size_t(cap)));
            L.E = (A<int>)(take(4 * size_t(cap)));
            L.V = (A<int>)(take(4 * size_t(cap)));
            L.hseq = (A<int>)(take(4 * size_t(lhcap)));
            L.huid = (A<uint32_t>)(take(4 * size_t(lhcap)));
            L.sc = (lptr<Sc>)(take(sizeof(Sc)));
            L.gst = (lptr<mtr_synth_state>)(take(sizeof(mtr_synth_state)));
            L.cap = cap;
            L.lhcap = lhcap;
        }
        L.gtext = gp(P.text) + size_t(d) * P.tcap;
        L.gprop = gp(P.prop) + size_t(d) * P.pcap;
        L.grm = gp(P.rm) + size_t(d) * P.rcap;
    }

    // ------------------------------------------------------------ per-document driver
    static __device__ void run(char* smem, const KParams& P, uint32_t d) {
        const mtr_doc_desc dd = ld_struct<mtr_doc_desc>(gp(P.docs) + d);
        const int cursor = gp(P.hdr)[d].op_cursor;
        const int n_ops = min(int(dd.op_count) - cursor, P.ops_this_launch);
        if (n_ops <= 0 || gp(P.hdr)[d].status != MTR_OK) return;
        D L;
        carve(L, smem, P, d);
        load_doc(L, P, d);
        lptr<Sc> sc = L.sc;
        const gptr<const mtr_op> ops = gp(P.ops) + dd.op_begin + cursor;
        const gptr<const uint16_t> btext = gp(P.btext) + dd.text_base;
        const int ln = lane_id();
        // lane t holds the 8 words of op (chunk + t); the next op's text is prefetched into `pf`
        uint32_t ow[8];
        uint32_t pf = 0, npf = 0;
        bool pre = false, npre = false;
        for (int k = 0; k < n_ops; k++) {
            PROF(P_OP);
            mtr_op op;
            if (P.gen) {
                gen_op(L, P, dd, cursor + k);
                op = ld_struct<mtr_op>(ops + k);
                pre = false;
            } else {
                if ((k & 63) == 0) {
                    const gptr<const uint32_t> w = (gptr<const uint32_t>)(ops + k + ln);
#pragma unroll
                    for (int q = 0; q < 8; q++) ow[q] = k + ln < n_ops ? w[q] : 0u;
                    npre = false;
                }
                uint32_t wv[8];
#pragma unroll
                for (int q = 0; q < 8; q++) wv[q] = rdlane(ow[q], k & 63);
                __builtin_memcpy(&op, wv, sizeof(op));
                pre = npre;
                pf = npf;
                npre = false;
                const int t1 = (k + 1) & 63;
                if (t1 != 0 && k + 1 < n_ops) {  // issue the next insert's text loads now
                    const uint32_t w0 = rdlane(ow[0], t1), len1 = rdlane(ow[7], t1), off1 = rdlane(ow[6], t1);
                    const uint32_t ty = w0 & 0xffu, fl = (w0 >> 8) & 0xffu;
                    if ((ty == MTR_OP_INSERT || ty == MTR_OP_LOCAL_INSERT) && !(fl & MTR_F_MARKER) && len1 <= 64) {
                        npre = true;
                        npf = uint32_t(ln) < len1 ? uint32_t(btext[off1 + ln]) : 0u;
                    }
                }
            }
            if (threadIdx.x == 0) {
                sc->sum_s += (unsigned long long)sc->nseg;
                if ((op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT) && !(op.flags & MTR_F_MARKER))
                    sc->sum_l += (unsigned long long)op.payload2;
            }
            {  // text arena: keep room for this op's text plus zamboni merge copies
                const int need =
                    int(op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT ? op.payload2 : 0) + 4096;
                if (sc->textused + need > text_end(sc, P)) text_gc(L, P);
            }
            if (sc->nseg + 2 >= L.cap) {  // every op adds at most two leaves
                __syncthreads();
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
                    __syncthreads();
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
            switch (op.type) {
                case MTR_OP_INSERT:
                case MTR_OP_LOCAL_INSERT:
                    prefix(L, v, P.new_length_calc);
                    split_at(L, op.pos1);
                    insert_at(L, P, v, op, seq, client, dd, pre, pf);
                    if (sc->collab) zamboni(L, P);
                    break;
                case MTR_OP_REMOVE:
                case MTR_OP_LOCAL_REMOVE:
                case MTR_OP_ANNOTATE:
                case MTR_OP_LOCAL_ANNOTATE: {
                    const int is_remove = op.type == MTR_OP_REMOVE || op.type == MTR_OP_LOCAL_REMOVE;
                    prefix(L, v, P.new_length_calc);
                    split_at(L, op.pos1);
                    split_at(L, op.pos2);
                    range_walk(L, P, v, op.pos1, op.pos2, seq, client, is_remove, op.payload);
                    if (sc->collab) zamboni(L, P);
                    break;
                }
                case MTR_OP_SEQ:
                    break;
                case MTR_OP_START_COLLAB:
                    __syncthreads();
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
                    __syncthreads();
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
        store_doc(L, P, d);
    }
};

template <bool G>
__global__ void __launch_bounds__(NT) apply_kernel(KParams P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t d = blockIdx.x;
    if (d >= P.n_docs) return;
    Eng<G>::run(smem, P, d);
}

}  // namespace mtr
