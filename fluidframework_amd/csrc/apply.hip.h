// apply.hip.h -- the op-apply kernel of the MI355X merge-tree replay engine.
//
// One wave64 (the whole workgroup) owns one document for the whole launch and applies that
// document's ops strictly in order (ops never cross documents).  The document's leaves live as
// flat structure-of-arrays records in tree order -- in LDS when they fit, otherwise in the
// document's HBM slab (Doc<true>, same code) -- and the reference's B+tree (MaxNodesInBlock = 8,
// mergeTreeNodes.ts:330) is kept exactly, encoded per leaf as `bnd` = number of tree levels at
// which the leaf starts a block.
//
// Single-wave program:
//  * the document's scalar state (St: leaf count, tree height, seq window, heap size, arena
//    cursors, status) is register-resident and wave-uniform (SGPRs); values read from LDS/HBM at
//    a uniform address are made uniform with readfirstlane;
//  * there are no workgroup barriers: one wave's LDS and vector-memory operations are performed in
//    order and are coherent across its lanes (LLVM AMDGPU memory model, wavefront scope), so a
//    phase boundary is only a compiler ordering point (wsync);
//  * the O(S) work runs on all lanes: the visibility prefix scan for the op's (refSeq, clientId)
//    view (replaces PartialSequenceLengths, partialLengths.ts:698, and the length queries of
//    insertingWalk / nodeMap, mergeTree.ts:1740, 2526), the one-slot shift that makes room for a
//    split or an insert (mergeTree.ts:1831-1838), the uid search for popped LRU entries, the range
//    walk of remove/annotate, and the stream compaction after zamboni (zamboni.ts:19-120);
//  * the sequential control (tie-break, block splits, heap, zamboni scour/pack decisions) is
//    uniform code whose walks over leaves are ballots over 64 leaves at a time.
//
// Memory spaces are explicit: LDS arrays are address_space(3) pointers (ds_read/ds_write),
// HBM arrays address_space(1) (global_load/store) -- never generic flat accesses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mtr_synth.h"
#include "../../include/mtr_types.h"

#define MTR_DI __device__ __forceinline__
// Rare, large paths (text-arena collection, snapshot loads, the scour fallback) as out-of-line calls: an experiment
// switch, off -- the calls take the document structs by reference, which puts them on the scratch stack (r05: 644
// scratch accesses in the CAP-224 kernel against 221 -> 44 SGPRs spilled)
#ifndef MTR_COLD_NOINLINE
#define MTR_COLD_NOINLINE 0
#endif
#if MTR_COLD_NOINLINE
#define MTR_COLD __device__ __attribute__((noinline))
#else
#define MTR_COLD MTR_DI
#endif
#ifndef MTR_UNSWITCH
#define MTR_UNSWITCH 1
#endif

namespace mtr {

constexpr int NT = 64;                  // one wave per document
constexpr int32_t RNONE = 0x7fffffff;   // removedSeq of a live leaf
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
constexpr uint32_t M_NONL = 1u << 28; // the leaf's text holds no '\n' at all (so neither does any split half)
constexpr uint32_t M_TOUCH = 1u << 29;  // transient: a delta segment of the current MTR_F_DELTA op
constexpr uint32_t M_PEND = 1u << 30;   // the leaf belongs to pending local SegmentGroups (a list of cells by uid)
constexpr uint32_t M_ZOMB = 1u << 31;   // ... or its list holds key cells of an annotate regenerate did not re-send
constexpr uint32_t ZOMBIE_SLOT = 0xffffu;  // ring-slot field of such a cell (its word 2 = the annotate's prop-op)
constexpr uint32_t NS_UNDEF = 0, NS_FALSE = 1, NS_TRUE = 2;

// The local-op path: a pending local insert keeps seq = LOCAL_BASE + localSeq and a pending
// local remove removedSeq = LOCAL_BASE + localSeq -- above every sequence number (UnassignedSequenceNumber
// is newer than anything sequenced: nodeLength / breakTie compare it that way, mergeTree.ts:935-1003,
// 1719-1738), below RNONE.  Pending SegmentGroups live in a per-document ring of kPendRing entries
// {localSeq, members so far, kind, prop-op}; a leaf's memberships are 2-word cells {next | kind << 24,
// ring slot << 16 | ordinal in the group} in the remover arena, listed under key PEND_KEY | uid.
constexpr int LOCAL_BASE = 0x40000000;
constexpr int TIE_LOCAL = 0x7ffffffe;   // breakTie's newSeq of a local insert (Number.MAX_SAFE_INTEGER)
// (a regenerate re-sends each member of a wide pending remove / annotate as its own group,
// resetPendingDeltaToOps: the ring must hold one group per segment such an op spans; 16-bit slot field)
constexpr int kPendRing = 4096;
// HBM-resident documents of at least kGapMin leaves keep one hole slot per kGapEvery (Eng::spread), so a
// split or an insert moves the leaves up to the next hole instead of the rest of the document; a shift
// looks for a hole within kHoleWindow slots
constexpr int kGapMin = 8192;
constexpr int kGapEvery = 16;
constexpr int kHoleWindow = 1024;
constexpr uint32_t PEND_KEY = 0x40000000u;
// chunk summaries of HBM-resident documents (Eng::csum_update): per 64-slot chunk its local length, newest
// event, the length of its leaves whose visibility no view in the collaboration window can change, and
// the slots of the other leaves (up to kChunkList; more = the chunk is scanned whole)
constexpr int kChunkList = 12;  // (a multiple of 4: the record's slot list is read 16 bytes at a time)
constexpr int kCsumRows = 4 + 5 * kChunkList;  // ints per chunk record (Eng::csum_update)
// superchunks (64 chunks) whose chunk lengths one round of loads fetches; prefix2's list capacity
constexpr int kDirtyBatch = 4;
constexpr int kListCap = 256;
__host__ __device__ constexpr int sup_rows(int segcap) { return segcap / 4096 + 2; }
// ints of one document's chunk summaries: the chunk records, then its superchunks' lengths and newest events
// (a multiple of 4: every document's records stay 16-byte aligned)
__host__ __device__ constexpr size_t csum_ints(int segcap) {
    return (size_t(kCsumRows) * size_t(segcap / 64 + 1) + 2 * size_t(sup_rows(segcap)) + 3) & ~size_t(3);
}
typedef int v4i __attribute__((ext_vector_type(4), may_alias));
enum { PK_INSERT = 1, PK_REMOVE = 2, PK_ANNOTATE = 3 };
// a pending local "rewrite" annotate's cells and ring entry carry PK_REWRITE beside PK_ANNOTATE: while one is
// pending, remote changes to the segment are blocked (pendingRewriteCount, segmentPropertiesManager.ts:72-80)
constexpr int PK_REWRITE = 0x80;
constexpr int PK_KIND = 0x7f;

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
MTR_DI T ld_struct(Q p) {
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
// a struct read at a wave-uniform address, made wave-uniform (SGPRs)
template <class T>
MTR_DI T uni_struct(const T& x) {
    static_assert(sizeof(T) % 4 == 0, "word-sized struct");
    uint32_t v[sizeof(T) / 4];
    __builtin_memcpy(v, &x, sizeof(T));
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; i++) v[i] = uint32_t(__builtin_amdgcn_readfirstlane(int(v[i])));
    T t;
    __builtin_memcpy(&t, v, sizeof(T));
    return t;
}
template <class T, class Q>
MTR_DI void st_struct(Q p, const T& t) {
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
    int32_t heap_need;  // LRU heap capacity the next launch must give this document (0 = none)
    int32_t dused;      // delta ranges recorded for the current batch
    int32_t lseq;       // collabWindow.localSeq (mergeTreeNodes.ts:656)
    int32_t phead, ptail;  // pending SegmentGroups: ring entries [phead, ptail) (MergeTree.pendingSegments)
    int32_t holes;         // HBM-resident documents: hole slots among the nseg leaf slots (see Eng::spread)
    int32_t chunked;       // ... and their per-64-slot chunk summaries are valid (two-level view scan)
    int32_t pfree;         // free list of pending-membership cells (first cell + 1, 0 = empty)
    int32_t lastnorm;      // Client.lastNormalizationRefSeq (client.ts:910): currentSeq of the last normalization
    int32_t nrefs;         // local references created (Eng::ref_create): ids 0 .. nrefs - 1
    int32_t tfree;         // matrix vectors: tracking ids on the free stack (Eng::tid_free)
};

// 32-bit SoA fields per leaf kept in HBM and LDS
constexpr int NF = 7;
enum { F_LEN = 0, F_SEQ, F_RSEQ, F_META, F_TEXT, F_PROPS, F_UID };

// Remover lists (removedClientIds[1..]) are cons cells in the document's remover arena; the head
// of a leaf's list is found by its uid in an open-addressing table after the cells (key = uid + 1,
// 0 = empty; cleared by mtr_reset), so leaves carry no per-slot list field: only leaves with
// M_OVERLAP have an entry.  rm slab per document: [rcap cells][2 * rtab words].
__host__ __device__ inline uint32_t rtab_hash(uint32_t uid) { return uid * 2654435761u; }

struct KParams {
    DocHdr* hdr;
    uint32_t* seg;   // [doc][NF][segcap]
    uint32_t* heap;  // [doc][2][hcap]   (seq, uid), 1-based
    uint16_t* text;  // [doc][tcap]
    uint32_t* prop;  // [doc][pcap]
    uint32_t* rm;    // [doc][rcap + 2 * rtab]: remover cells, then the uid -> list head table
    int32_t segcap, hcap, tcap, pcap, rcap;
    int32_t rtab;         // remover-head table entries (power of two)
    int32_t cap;          // leaf capacity of this launch (LDS mode)
    int32_t lhcap;        // heap capacity of this launch (LDS mode)
    int32_t global_mode;  // 1: leaves/heap stay in HBM (documents larger than LDS)
    uint32_t* scratch;    // [doc][2][segcap] E/V arrays for global mode
    int32_t ops_this_launch;
    int32_t new_length_calc;
    uint32_t n_docs;
    const uint32_t* doc_list;  // documents of this launch (one size class): block b applies doc_list[b]
    uint32_t n_launch;
    const mtr_op* ops;
    const mtr_doc_desc* docs;
    const uint16_t* btext;
    const uint32_t* propop_off;
    const uint32_t* propop_kv;
    const uint32_t* key_index;
    const uint32_t* val_eq;
    unsigned long long* stat_ops;  // [doc][4]: ops applied, sum of leaves before ops, inserted units
    uint32_t* delta;               // delta ranges of MTR_F_DELTA ops (mtr_delta records)
    const uint64_t* doff;          // [doc + 1]: document d's records are [doff[d], doff[d+1])
    // SharedMatrix pairs (mtr_set_matrix): dkind[doc] 0 = SharedString, 1 = rows PermutationVector
    // (drives the pair; dpart[doc] = its cols document), 2 = cols PermutationVector
    const uint32_t* dkind;
    const uint32_t* dpart;
    // record mode (synthetic workloads): ops are drawn from include/mtr_synth.h with this
    // engine's own exact view lengths, written to gen_ops/gen_text, then applied
    int32_t gen;
    int32_t gen_grow;  // record mode: the first gen_grow records (pre-grown snapshot segments) + START_COLLAB
                       // are written before the run; messages are records gen_grow + 1 ...
    mtr_synth_cfg gen_cfg;
    mtr_synth_state* gen_state;  // [doc]
    mtr_op* gen_ops;             // == ops, writable
    uint16_t* gen_text;          // == btext, writable
    unsigned long long* prof;    // [P_COUNT] phase-timer sums (-DMTR_PROF builds)
    uint32_t* pend;              // [doc][kPendRing][4] pending SegmentGroups (batches with local ops only)
    int32_t* csum;               // [doc][2][segcap / 64 + 1] chunk summaries of HBM-resident documents
    int32_t* umap;               // [doc][2 * segcap] uid -> slot hints of HBM-resident documents
    uint32_t* refs;              // [doc][3][refcap] local references (batches with reference records only)
    int32_t refcap;
};

// phase-timer slots (-DMTR_PROF builds)
enum { P_OP = 0, P_PREFIX, P_SPLIT, P_SHIFT, P_INSERT, P_RANGE, P_ZAMBONI, P_ZBLOCK, P_COMPACT, P_FINDUID,
       P_TEXTGC, P_LOADSTORE, P_TEXTCOPY, P_UPDSEQ, P_NZBLOCK, P_NCOMPACT, P_SCOUR1, P_PACK, P_NLQ, P_PMATCH,
       P_TAPPEND, P_HEAP, P_OVERFLOW, P_NPACK, P_NMERGE, P_NPMATCH, P_NNLQ, P_SPLIT1, P_INS1, P_FETCH, P_X1, P_X2,
       // two-level view scan (HBM-resident documents): chunk-summary rounds, dirty-chunk full scans, the scan
       // array of the op's region, summary upkeep; counts: chunks visited, listed chunks, dirty unlisted chunks
       P_PFSUM, P_PFDIRTY, P_MAT, P_CSUM, P_NCH, P_NLISTED, P_NDIRTY,
       P_SPREAD, P_CHUNKOF, P_NSPREAD,
       // snapshot-load records + the tree build, apply_op's prologue (to the dispatch), whole view scans,
       // the tail (deltas, zamboni, updateSeqNumbers)
       P_LOAD, P_PRE, P_VIEW, P_POST,
       P_NSUP, P_NDCH,  // counts: superchunks with events after refSeq, their chunks with such events
       P_HELPER,        // the team's helper waves: cycles in the passes handed to them
       P_SINK,          // (a slot nothing reads)
       P_OVB, P_OVPB, P_NOVFB, P_NOVL,  // overflow_fix: the leaf block's bounds and count, the parent walks; counts:
                                        // bounds outside the one-ballot window, loop rounds
       P_SUPREF, P_PXLIST, P_PXEVAL, P_PXSYNC, P_NPXR,  // prefix2 (wave 0): stale superchunk figures, listing,
                                                        // evaluation, barrier waits; count: team rounds
       P_NWALK, P_NDRND, P_WALK,  // counts: remover-list walks (vis_leaf), dirty-chunk rounds; cycles in the walks
       P_COUNT };

// Per-document pointers the op loop needs only now and then (text / property / remover arenas, delta
// records, the batch's property tables), kept in LDS and read where used, so they never hold SGPRs
// across the whole op loop (the loop's scalar state otherwise spills into VGPR lanes)
enum { CP_TEXT = 0, CP_PROP, CP_RM, CP_RT, CP_DELTA, CP_POFF, CP_PKV, CP_KIX, CP_VEQ, CP_HDR, CP_PEND, CP_CSUM, CP_UMAP,
       CP_REFS, CP_N };

// LDS-side scratch of one document: record-mode broadcast, cold pointers, phase timers
struct Sc {
    unsigned long long cp[CP_N];
    int gen_ref, gen_client;
    int rel[2];   // positions resolved by MTR_OP_RELPOS records for the next (MTR_F_REL) op
    int relmask;  // which of rel[] are pending: bit 0 pos1, bit 1 pos2
    int nrefs, refcap;  // local references of the document (DocHdr.nrefs) and the table's capacity
    int fail_op, max_heap, heap_need;  // DocHdr's, for this launch
    int sepoch;  // view scans of this launch (HBM-resident documents: Eng::prefix2's fill epochs)
    int vref;    // the last two-level view's refSeq (INT32_MAX: a local view)
    unsigned long long sum_s, sum_l;   // B_op counters: leaves before each op, inserted units
#ifdef MTR_PROF
    unsigned long long prof[P_COUNT];
#endif
};

// Register-resident, wave-uniform scalar state of the document being applied.
struct St {
    int nseg, height, minseq, curseq;
    int collab, local, heapn, uidnext;
    int textused, propused, rmused, status;  // textused: handle-table length for permutation vectors
    int texthalf;
    int htop;  // seq of the LRU heap's top entry (valid while heapn > 0)
    int dused;   // (delta-reporting instantiations only)
    int holes;   // hole slots (HBM-resident documents only)
    int chunked; // chunk summaries valid (HBM-resident documents with holes)
    int cur_op;  // index of the op being applied (delta-reporting instantiations only)
    // (the failing op, the heap-size high-water mark, the heap a yield asks for and the B_op counters live in
    // Sc: they change rarely, and every field here is an SGPR held across the whole op loop)
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
    A<int> len, seq, rseq, E, hseq;  // E: scan array (see Eng::prefix)
    A<uint32_t> meta, text, props, uid, huid;
    lptr<Sc> sc;
    lptr<mtr_synth_state> gst;
    lptr<int> sx;  // HBM-resident documents: superchunk rows and the dirty-chunk list (Eng::prefix2)
    int dcap;  // capacity of this document's delta records in this batch
    int cap, lhcap, rtmask;
    // cold pointers (read from LDS at the use site, made wave-uniform)
    MTR_DI unsigned long long cold(int k) const {
        const unsigned long long v = sc->cp[k];
        return (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane(int(uint32_t(v))) |
               ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))) << 32);
    }
    MTR_DI gptr<uint16_t> gtext() const { return (gptr<uint16_t>)cold(CP_TEXT); }
    MTR_DI gptr<uint32_t> gprop() const { return (gptr<uint32_t>)cold(CP_PROP); }
    MTR_DI gptr<uint32_t> grm() const { return (gptr<uint32_t>)cold(CP_RM); }
    MTR_DI gptr<uint32_t> grt() const { return (gptr<uint32_t>)cold(CP_RT); }  // remover-head table
    MTR_DI gptr<uint32_t> gdelta() const { return (gptr<uint32_t>)cold(CP_DELTA); }  // mtr_delta records
    MTR_DI gptr<const uint32_t> tab(int k) const { return (gptr<const uint32_t>)cold(k); }
    MTR_DI gptr<DocHdr> ghdr() const { return (gptr<DocHdr>)cold(CP_HDR); }      // this document's header
    MTR_DI gptr<uint32_t> gpend() const { return (gptr<uint32_t>)cold(CP_PEND); }  // its pending-group ring
    MTR_DI gptr<int> gcsum() const { return (gptr<int>)cold(CP_CSUM); }          // chunk summaries (len, then ev)
    MTR_DI gptr<int> gumap() const { return (gptr<int>)cold(CP_UMAP); }          // uid -> slot hints
    // a merge chain's text copy whose load is in flight (Eng::copy_chain): lane l stores unit pc_val at pc_dst when
    // pc_on; pc_any (uniform) when any lane has one.  The store waits for the next reader of the text arena
    // (Eng::text_flush), so the load's HBM latency overlaps the work between two zamboni passes.
    uint32_t pc_dst = 0, pc_val = 0;
    int pc_on = 0, pc_any = 0;
    int rlo = 0, rhi = 0;  // the op's view-scan region (slots) when the scan was two-level (E valid there)
    int shi = 0;           // end of the slots the last shift_right1 moved (chunk-summary upkeep)
    int wlo = 0, whi = 0;  // slots the last range walk touched
};

MTR_DI int bnd_of(uint32_t m) { return int((m & M_BND_MASK) >> M_BND_SHIFT); }
MTR_DI uint32_t set_bnd(uint32_t m, int b) { return (m & ~M_BND_MASK) | (uint32_t(b) << M_BND_SHIFT); }
MTR_DI uint32_t ns_of(uint32_t m) { return (m & M_NS_MASK) >> M_NS_SHIFT; }
MTR_DI uint32_t set_ns(uint32_t m, uint32_t ns) { return (m & ~M_NS_MASK) | (ns << M_NS_SHIFT); }

// ------------------------------------------------------------------ wave primitives
// (a wave's own lane: apply_pair2_kernel runs two waves per workgroup; with 64-thread launch bounds the mask
// folds away)
MTR_DI int lane_id() { return int(threadIdx.x & 63u); }
constexpr uint64_t LO32 = 0x00000000ffffffffull, HI32 = 0xffffffff00000000ull;  // lanes 0-31, 32-63
MTR_DI uint64_t lanes_below() { return (uint64_t(1) << lane_id()) - 1; }
MTR_DI int first_lane(uint64_t m) { return __ffsll((long long)m) - 1; }
MTR_DI int last_lane(uint64_t m) { return 63 - __clzll((long long)m); }
MTR_DI int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
MTR_DI uint32_t uniu(uint32_t x) { return uint32_t(__builtin_amdgcn_readfirstlane(int(x))); }
template <class T>
MTR_DI T rdlane(T x, int l) {  // v_readlane with a wave-uniform lane index
    return T(__builtin_amdgcn_readlane(int(x), l));
}
// Phase boundary inside one wave: orders the compiler's memory operations (the hardware already
// performs one wave's LDS and vector-memory operations in order; wavefront scope needs no waits).
MTR_DI void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// inclusive add-scan over the 64 lanes: DPP row shifts within rows of 16, then row broadcasts
MTR_DI int wave_incl_scan(int x) {
    // (bound_ctrl: lanes shifted in from outside the row read 0 -- the same sums as a 0 old value,
    // but each step folds into one v_add_u32_dpp even while x stays live)
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Lane predicates as 0 / -1 words computed on the VALU: a compare into VCC and a select, combined with
// v_and / v_or.  Written as plain C++ booleans the compiler keeps them as 64-bit lane masks and combines those
// with s_and_b64 / s_or_b64 on the CU's one scalar unit -- the unit that binds the C3 kernel (SALU ~60 % busy
// against ~27 % of the VALU issue slots: a wave64 VALU op takes 2 of a SIMD-32's cycles, 4 SIMDs per CU).
// (asm, so the compiler cannot fold two such selects back into one select of a combined lane mask)
MTR_DI int vp_lt(int a, int b) {
    int r;
    asm("v_cmp_lt_i32_e32 vcc, %1, %2\n\tv_cndmask_b32_e64 %0, 0, -1, vcc" : "=v"(r) : "v"(a), "v"(b) : "vcc");
    return r;
}
MTR_DI int vp_le(int a, int b) {
    int r;
    asm("v_cmp_le_i32_e32 vcc, %1, %2\n\tv_cndmask_b32_e64 %0, 0, -1, vcc" : "=v"(r) : "v"(a), "v"(b) : "vcc");
    return r;
}
MTR_DI int vp_eq(uint32_t a, uint32_t b) {
    int r;
    asm("v_cmp_eq_u32_e32 vcc, %1, %2\n\tv_cndmask_b32_e64 %0, 0, -1, vcc" : "=v"(r) : "v"(a), "v"(b) : "vcc");
    return r;
}
MTR_DI int vp_bit(uint32_t m, int bit) { return -int((m >> bit) & 1u); }  // -1 when bit `bit` of m is set
MTR_DI int vp_sel(int mask, int a, int b) { return (a & mask) | (b & ~mask); }  // mask ? a : b (v_bfi_b32)

// matchProperties (properties.ts:71-105) with values compared by equivalence class; a value flagged
// MTR_VEQ_NEVER (NaN, a consensus {value: undefined, seq}) matches nothing, not even itself, so a set
// holding one -- its leaf-side index carries MTR_PROPS_NEVER -- does not match itself either
constexpr uint32_t PN_MASK = ~MTR_PROPS_NEVER;
MTR_DI bool pset_never(uint32_t a) { return a != NONE32 && (a & MTR_PROPS_NEVER) != 0; }
template <class PA, class PB>
__device__ bool props_match(PA gprop, PB val_eq, uint32_t a, uint32_t b) {
    if (a == b) return !pset_never(a);
    if (a == NONE32 || b == NONE32) return false;
    a &= PN_MASK;
    b &= PN_MASK;
    const uint32_t na = gprop[a], nb = gprop[b];
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
        const uint32_t k = gprop[a + 1 + 2 * i];
        bool found = false;
        for (uint32_t j = 0; j < nb; j++)
            if (gprop[b + 1 + 2 * j] == k) {
                const uint32_t ea = val_eq[gprop[a + 2 + 2 * i]];
                if (ea != val_eq[gprop[b + 2 + 2 * j]] || (ea & MTR_VEQ_NEVER)) return false;
                found = true;
                break;
            }
        if (!found) return false;
    }
    return true;
}

// LDS scratch: Sc, plus the generator state in record-mode launches only
constexpr size_t kScOnly = (sizeof(Sc) + 15) & ~size_t(15);
constexpr size_t kScBytes = kScOnly + ((sizeof(mtr_synth_state) + 15) & ~size_t(15));
// LDS bytes of a launch with leaf capacity cap and heap capacity lhcap (8 leaf arrays + heap; 7 for a matrix vector
// of apply_pair2_kernel, which keeps no props array: Eng::NOPROPS)
__host__ __device__ inline size_t lds_bytes(int cap, int lhcap, bool gen = true, int arrays = 8) {
    return size_t(cap) * 4 * size_t(arrays) + size_t(lhcap) * 4 * 2 + (gen ? kScBytes : kScOnly);
}
// HBM-resident documents run on a team of MTR_GW waves (one workgroup per document): wave 0 applies the ops, the
// others wait at the workgroup barrier for the passes it hands out (Eng::team_*).  The team's mailbox: the task and
// its arguments, then one result slot per wave.
#ifndef MTR_GW
#define MTR_GW 2
#endif
constexpr int kTeamInts = 64;  // (task + 15 argument words, then two step-parity rows of 4 result words per wave)
constexpr size_t kTeamBytes = 4 * kTeamInts;
// (HBM-resident documents: Sc, the generator state, the team's mailbox, six superchunk rows, prefix2's chunk list
// and two words per 64 slots)
__host__ __device__ inline size_t lds_bytes_global_mode(int segcap) {
    return kScBytes + kTeamBytes +
           ((size_t(4) * (6 * sup_rows(segcap) + kListCap + 2 * (segcap / 64 + 1)) + 15) & ~size_t(15));
}

// Phase timers (builds with -DMTR_PROF only): lane-0 clock cycles per phase, summed over
// documents into g_prof (mtr_profile()).
#ifdef MTR_PROF
struct ProfScope {
    lptr<Sc> sc;
    int id;
    long long t;
    __device__ ProfScope(lptr<Sc> s, int i) : sc(s), id(i), t(clock64()) {}
    __device__ ~ProfScope() {
        const long long d = clock64() - t;
        if (lane_id() == 0) sc->prof[id] += (unsigned long long)d;
    }
};
#define PROF(id) ProfScope _prof_scope(L.sc, id)
#define PROF_T0(v) const long long v = clock64()
#define PROF_ADD(id, v) \
    if (lane_id() == 0) L.sc->prof[id] += (unsigned long long)(clock64() - (v))
#define PROF_COUNT(id) \
    if (lane_id() == 0) L.sc->prof[id]++
#else
#define PROF(id)
#define PROF_COUNT(id)
#define PROF_T0(v)
#define PROF_ADD(id, v)
#endif

// G: leaves in HBM (documents larger than LDS); PM: PermutationVector documents (SharedMatrix
// rows/cols, permutationvector.ts) -- a separate instantiation so the SharedString kernel carries
// no permutation code; CAP: the launch's LDS leaf capacity as a compile-time constant (0 = runtime, with the
// rare records compiled in; -1 = runtime, without them: the replay kernels of documents above the largest
// fixed class and of HBM-resident documents),
// which puts every leaf array at a constant LDS offset (ds_read/ds_write immediate offsets from one
// per-lane address instead of a base register and an address add per array)
template <bool G, bool PM = false, int CAP = 0, bool DL = false, bool GN = false>
struct Eng {
    using D = Doc<G>;
    // the rare records (MTR_OP_RELPOS / MTR_F_REL, MTR_OP_HANDLES, combining annotates, marker ordinals)
    // are compiled into the runtime-capacity and matrix instantiations only; the host launches those for a
    // batch holding any (mtr_submit's op scan), so the fixed-capacity replay kernels carry none of it
    static constexpr bool X = CAP == 0 || PM;
    // a matrix vector in an LDS launch of apply_pair2_kernel (remote messages only: no tracking ids, every props
    // field NONE32) keeps no props array in LDS -- 28 bytes a leaf instead of 32
    static constexpr bool NOPROPS = PM && CAP == -2;
    static MTR_DI uint32_t pget(const Doc<G>& L, int i) {
        if constexpr (NOPROPS) return NONE32;
        else return L.props[i];
    }
    static MTR_DI void pset(const Doc<G>& L, int i, uint32_t v) {
        if constexpr (!NOPROPS) L.props[i] = v;
    }
    template <class T>
    using A = typename D::template A<T>;

    // ------------------------------------------------------------ visibility
    // ---- remover-list heads by uid (per-lane probes; only M_OVERLAP leaves have entries)
    static MTR_DI uint32_t rm_get(const D& L, uint32_t uid) {
        uint32_t h = rtab_hash(uid) & uint32_t(L.rtmask);
        for (int n = 0; n <= L.rtmask; n++) {
            const uint32_t k = L.grt()[2 * h];
            if (k == uid + 1) return L.grt()[2 * h + 1];
            if (k == 0) break;
            h = (h + 1) & uint32_t(L.rtmask);
        }
        return 0xffffffu;
    }
    // set uid's head (lanes may insert concurrently: empty keys are claimed with a CAS); false = full
    static MTR_DI bool rm_set(const D& L, uint32_t uid, uint32_t head) {
        uint32_t h = rtab_hash(uid) & uint32_t(L.rtmask);
        for (int n = 0; n <= L.rtmask; n++) {
            uint32_t k = L.grt()[2 * h];
            if (k == 0) k = atomicCAS((uint32_t*)&L.grt()[2 * h], 0u, uid + 1);
            if (k == 0 || k == uid + 1) {
                L.grt()[2 * h + 1] = head;
                return true;
            }
            h = (h + 1) & uint32_t(L.rtmask);
        }
        return false;
    }

    // MergeTree.idToSegment (mergeTree.ts:549,668): marker ordinal -> the marker's uid, kept in the
    // remover-head table under key 0x80000000 | ordinal (uids stay below 2^31).  Out of line: rare.
    static MTR_DI bool mk_put(gptr<uint32_t> rt, uint32_t rtmask, uint32_t ordinal,
                                                           uint32_t uid) {
        const uint32_t key = 0x80000000u | ordinal;
        uint32_t h = rtab_hash(key) & rtmask;
        for (uint32_t n = 0; n <= rtmask; n++) {
            uint32_t k = rt[2 * h];
            if (k == 0) k = atomicCAS((uint32_t*)&rt[2 * h], 0u, key + 1);
            if (k == 0 || k == key + 1) {
                rt[2 * h + 1] = uid;
                return true;
            }
            h = (h + 1) & rtmask;
        }
        return false;
    }
    static MTR_DI bool mk_set(const D& L, uint32_t ordinal, uint32_t uid) {
        return mk_put(L.grt(), uint32_t(L.rtmask), ordinal, uid);
    }
    // -> uid | 1 << 32 when mapped, 0 when not
    static MTR_DI uint64_t mk_look(gptr<const uint32_t> rt, uint32_t rtmask,
                                                                uint32_t ordinal) {
        const uint32_t key = 0x80000000u | ordinal;
        uint32_t h = rtab_hash(key) & rtmask;
        for (uint32_t n = 0; n <= rtmask; n++) {
            const uint32_t k = uniu(rt[2 * h]);
            if (k == key + 1) return uint64_t(uniu(rt[2 * h + 1])) | (uint64_t(1) << 32);
            if (k == 0) break;
            h = (h + 1) & rtmask;
        }
        return 0;
    }

    static MTR_DI bool in_removers(const D& L, int i, uint32_t m, uint32_t c) {
        if (((m >> M_FREM_SHIFT) & 0xffu) == c) return true;
        if (!(m & M_OVERLAP)) return false;
        uint32_t cell = rm_get(L, L.uid[i]);
        while (cell != 0xffffffu) {
            const uint32_t v = L.grm()[cell];
            if ((v >> 24) == c) return true;
            cell = v & 0xffffffu;
        }
        return false;
    }

    // nodeLength for a leaf (mergeTree.ts:916-1004): -1 = undefined.  Every lane evaluates the
    // same select chain (no divergent branches); only lanes whose answer depends on a later
    // remover in the overlap list walk it, behind one ballot.
    // the fields a visibility test reads (loaded apart from the test so scans can issue the next
    // round's loads early)
    struct Hot {
        int len, rseq, seq;
        uint32_t meta;
    };
    static MTR_DI Hot ld_hot(const D& L, int i) { return Hot{L.len[i], L.rseq[i], L.seq[i], L.meta[i]}; }
    static MTR_DI int vis_len(const D& L, int i, const View& v, int newlen, int minseq, bool valid = true) {
        return vis_hot(L, ld_hot(L, i), i, v, newlen, minseq, valid);
    }
    template <int LOC = -1, int NL = -1>
    static MTR_DI int vis_hot(const D& L, const Hot& h, int i, const View& v, int newlen, int minseq, bool valid,
                              gptr<const int> slotp = nullptr) {
        const int r = vis_leaf<LOC, NL>(L, h, i, v, newlen, minseq, valid, slotp);
        if constexpr (G) return r | vp_bit(h.meta, 25);  // a hole slot (M_DEL) is no leaf (Eng::spread)
        return r;
    }
    // (LOC / NL >= 0: v.local / newlen known at compile time -- the remote view's scans carry no local branch)
    // (slotp: where the leaf's slot is read when its remover list must be walked -- a chunk record's slot list --
    // instead of i)
    template <int LOC = -1, int NL = -1>
    static MTR_DI int vis_leaf(const D& L, const Hot& h, int i, const View& v, int newlen_, int minseq, bool valid,
                               gptr<const int> slotp = nullptr) {
        static_assert(M_DEL == 1u << 25 && M_OVERLAP == 1u << 21, "vis_hot / vis_leaf bit positions");
        const int len = h.len;
        const int rseq = h.rseq;
        const uint32_t m = h.meta;
        const int seq = h.seq;
        const int newlen = NL >= 0 ? NL : newlen_;
        if (LOC >= 0 ? LOC != 0 : v.local != 0) {  // localNetLength, mergeTree.ts:613-634 (a uniform branch)
            const bool removed = rseq != RNONE;
            const int rl = newlen ? 0 : (rseq > minseq ? 0 : -1);
            return removed ? rl : len;
        }
        // Every lane evaluates the same chain of 0 / -1 predicate words (vp_*: VALU only, no lane masks and
        // no divergent branches); only lanes whose answer depends on a later remover in the overlap list walk
        // it, behind one ballot.
        const int rem = ~vp_eq(uint32_t(rseq), uint32_t(RNONE));
        const int vis = vp_eq(m & M_CLIENT_MASK, v.client) | vp_le(seq, v.ref);
        const int first = rem & vp_eq((m >> M_FREM_SHIFT) & 0xffu, v.client);
        const int after = vp_lt(v.ref, rseq);  // removed after the view's refSeq
        // lanes whose result still depends on removedClientIds[1..] (mergeTree.ts:935-1003)
        const int walk = (valid ? -1 : 0) & rem & ~first & vp_bit(m, 21) & after &
                         (newlen ? vp_lt(minseq, rseq) : vis);
        int inr = first;
        if (__ballot(walk != 0)) {
#ifdef MTR_PROF
            PROF_COUNT(P_NWALK);
            ProfScope _prof_walk(L.sc, P_WALK);
#endif
            const int iw = slotp ? (walk != 0 ? *slotp : 0) : i;
            inr |= -later_remover(L, iw, walk != 0, v.client);
        }
        if (newlen) {  // mergeTree.ts:935-965
            const int live = vis & len;
            const int gone = live & ~(~after | inr);
            return vp_sel(rem, vp_le(rseq, minseq) | gone, live);
        }
        // mergeTree.ts:967-1003
        const int seen = len & ~(rem & inr);
        // (a pending local remove is no removal here: removedSeq !== UnassignedSequenceNumber, :993-998)
        const int r = vp_sel(vis, seen, rem & (X ? vp_lt(rseq, LOCAL_BASE) : -1));
        return r | (rem & ~after);
    }
    // 1 when client c is in leaf i's removedClientIds[1..] (the overlap list), for the lanes in `walk`
    static MTR_DI int later_remover(const D& L, int i, bool walk, uint32_t c) {
        int inr = 0;
        if (walk) {
            uint32_t cell = rm_get(L, L.uid[i]);
            while (cell != 0xffffffu) {
                const uint32_t w = L.grm()[cell];
                if ((w >> 24) == c) {
                    inr = 1;
                    break;
                }
                cell = w & 0xffffffu;
            }
        }
        return inr;
    }

    // root.cachedLength: the local view's length (removed leaves count 0), mergeTree.ts:613-634
    static MTR_DI int local_length(const D& L, const St& s) {
        int sum = 0;
        for (int base = 0; base < s.nseg; base += 64) {
            const int i = base + lane_id();
            int x = 0;
            if (i < s.nseg && L.rseq[i] == RNONE) x = L.len[i];
            sum += rdlane(wave_incl_scan(x), 63);
        }
        return sum;
    }

    // The scan array: E[i] = inclusive prefix of the leaves' visible lengths in the op's view, with
    // bit 31 set when leaf i's length is undefined (nodeLength === undefined).  A leaf's visible
    // length is E[i] - E[i-1] (masked), -1 if flagged.  Rounds of 64 leaves.
    static constexpr int EMASK = 0x7fffffff;
    static MTR_DI int ev(int e, int eprev) { return e < 0 ? -1 : e - (eprev & EMASK); }
    // HBM-resident documents (G): the O(S) passes issue the loads of GK rounds of 64 leaves before
    // using any of them, so a pass exposes HBM latency once per 64 * GK leaves (HBM bandwidth is not
    // what bounds them: one wave per document walks its leaves in order)
#ifndef MTR_GK
#define MTR_GK 4
#endif
    static constexpr int GK = MTR_GK;

    static MTR_DI void prefix(D& L, const St& s, const View& v, int newlen) {
        PROF(P_PREFIX);
        const int S = s.nseg;
        const int ln = lane_id();
        int carry = 0;
        if constexpr (G) {
            for (int base = 0; base < S; base += 64 * GK) {
                Hot hk[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) hk[q] = ld_hot(L, min(base + 64 * q + ln, S - 1));
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    if (base + 64 * q >= S) break;
                    const int i = base + 64 * q + ln;
                    const int x0 = vis_hot(L, hk[q], i, v, newlen, s.minseq, i < S);
                    const int in = vp_lt(i, S);
                    const int x = x0 & in;
                    const int inc = wave_incl_scan(max(x, 0));
                    L.E[vp_sel(in, i, S)] = (carry + inc) | (x & int(0x80000000u));  // (lanes past the end: slot S)
                    carry += rdlane(inc, 63);
                }
            }
            wsync();
            return;
        }
        // (the remote view with the default length rules -- every sequenced op of another client -- gets a loop
        // without the uniform local / new-length branches)
        if (MTR_UNSWITCH && !v.local && !newlen) prefix_lds<0, 0>(L, s, v, 0);
        else prefix_lds<-1, -1>(L, s, v, newlen);
        wsync();
    }
    template <int LOC, int NL>
    static MTR_DI void prefix_lds(D& L, const St& s, const View& v, int newlen) {
        const int S = s.nseg;
        const int ln = lane_id();
        int carry = 0;
        Hot h = S > 0 ? ld_hot(L, ln) : Hot{};  // software-pipelined: loaded one round ahead
        for (int base = 0; base < S; base += 64) {
            // every lane evaluates (reads past the last leaf stay inside the LDS allocation);
            // lanes past the last leaf contribute 0 and store nothing (capacities are multiples
            // of 32, so the round's top slots may belong to the next array)
            const int i = base + ln;
            const Hot cur = h;
            if (base + 64 < S) h = ld_hot(L, i + 64);
            const int x0 = vis_hot<LOC, NL>(L, cur, i, v, newlen, s.minseq, i < S);
            const int in = vp_lt(i, S);
            const int x = x0 & in;
            const int inc = wave_incl_scan(max(x, 0));
            // (no exec-mask block around the store: lanes past the last leaf write slot S, which holds no leaf --
            // an op starts with nseg + 2 < cap)
            L.E[vp_sel(in, i, S)] = (carry + inc) | (x & int(0x80000000u));
            carry += rdlane(inc, 63);
        }
    }

    // ---- two-level view scan (HBM-resident documents with hole slots, s.chunked)
    // The slots form chunks of 64.  Per chunk the document keeps its local length (the leaves that are
    // not removed) and its newest event (the largest seq, and removedSeq of a removed leaf, over its
    // leaves).  A chunk whose newest event is <= the view's refSeq looks the same to every client at that
    // refSeq -- each leaf was inserted by then, and removed by then or not at all -- so its view length
    // is its local length; only the other chunks are evaluated leaf by leaf.  This restates what
    // PartialSequenceLengths does per block (partialLengths.ts:698-735) for chunks of the flat leaf order.
    // 64 chunks form a superchunk with the same two figures (the chunks' sum and max), so a view reads one
    // pair per 4096 slots plus the newest events of the chunks of the superchunks with later events.
    // A chunk's record: kCsumRows ints (16-byte aligned) -- {local length, newest event, the length of its
    // leaves whose visibility no view in the collaboration window can change, the count of the other
    // leaves}, then those leaves' visibility fields {len, removedSeq, seq, meta} (up to kChunkList; more =
    // the chunk is scanned whole) and their slots (for the remover lists of overlapping removes).  A view
    // evaluates a chunk with later events from its record alone: one round of loads for 64 such chunks.
    static MTR_DI int nsup(const D& L) { return sup_rows(L.cap); }
    static MTR_DI int nchr(const D& L) { return L.cap / 64 + 1; }
    static MTR_DI gptr<int> cs_rec(const D& L, int c) { return L.gcsum() + c * kCsumRows; }
    static MTR_DI gptr<int> cs_sl(const D& L) { return L.gcsum() + kCsumRows * nchr(L); }
    static MTR_DI gptr<int> cs_se(const D& L) { return cs_sl(L) + nsup(L); }
    // LDS rows (Doc::sx, lds_bytes_global_mode): per superchunk a view's inclusive prefix, the view epoch
    // that filled its chunk-prefix row, "figures stale" marks, its local length and newest event (the
    // launch's copy of the HBM rows), a view's length change from its chunks with later events; prefix2's
    // list of those chunks; per chunk its newest event (the launch's copy of the records'), and a view's
    // length of the chunk (a chunk with later events), then its inclusive prefix within its superchunk
    static MTR_DI lptr<int> sup_pre(const D& L) { return L.sx; }
    static MTR_DI lptr<int> sup_fill(const D& L) { return L.sx + nsup(L); }
    static MTR_DI lptr<int> sup_mark(const D& L) { return L.sx + 2 * nsup(L); }
    static MTR_DI lptr<int> sup_len(const D& L) { return L.sx + 3 * nsup(L); }
    static MTR_DI lptr<int> sup_ev(const D& L) { return L.sx + 4 * nsup(L); }
    static MTR_DI lptr<int> sup_dlen(const D& L) { return L.sx + 5 * nsup(L); }
    static MTR_DI lptr<int> dlist(const D& L) { return L.sx + 6 * nsup(L); }
    static MTR_DI lptr<int> ch_ev(const D& L) { return dlist(L) + kListCap; }
    static MTR_DI lptr<int> ch_x(const D& L) { return ch_ev(L) + nchr(L); }
    static MTR_DI v4i ld4(gptr<const int> p) { return *(gptr<const v4i>)p; }
    // recompute the records of the chunks covering slots [lo, hi); their superchunks go stale
    static MTR_DI void csum_update(D& L, const St& s, int lo, int hi) {
        PROF(P_CSUM);
        if constexpr (G) {
            if (!s.chunked) return;
            hi = min(hi, s.nseg);
            if (lo >= hi) return;
            const int c0 = max(lo, 0) >> 6, c1 = (hi - 1) >> 6;
            for (int cb = c0; cb <= c1; cb += GK) {  // GK chunks' leaf fields in flight per step
                uint32_t mq[GK];
                int lq[GK], sqq[GK], rq[GK];
#pragma unroll
                for (int g = 0; g < GK; g++) {
                    const int ic = min((cb + g) * 64 + lane_id(), s.nseg - 1);
                    mq[g] = L.meta[ic];
                    lq[g] = L.len[ic];
                    sqq[g] = L.seq[ic];
                    rq[g] = L.rseq[ic];
                }
#pragma unroll
                for (int g = 0; g < GK; g++) {
                    const int c = cb + g;
                    if (c > c1) break;
                    const int i = c * 64 + lane_id();
                    const bool in = i < s.nseg;
                    const uint32_t m = mq[g];
                    const int len = lq[g], sq = sqq[g], rs = rq[g];
                    const bool live = in && !(m & M_DEL);
                    const bool rem = rs != RNONE;
                    // in the window: an event after minSeq (a pending local one included), so views differ on it
                    const bool win = live && (sq > s.minseq || (rem && rs > s.minseq));
                    const uint64_t wm = __ballot(win);
                    const int nw = __popcll(wm);
                    int x = (live && !rem) ? len : 0;
                    int fx = (live && !rem && !win) ? len : 0;  // removed at or before minSeq: in no view
                    int ev = live ? max(sq, rem ? rs : 0) : 0;
                    x = rdlane(wave_incl_scan(x), 63);
                    fx = rdlane(wave_incl_scan(fx), 63);
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) ev = max(ev, __shfl_xor(ev, o));
                    const gptr<int> r = cs_rec(L, c);
                    if (win && nw <= kChunkList) {
                        const int k = __popcll(wm & lanes_below());
                        *(gptr<v4i>)(r + 4 + 4 * k) = v4i{len, rs, sq, int(m)};  // Hot's field order
                        r[4 + 4 * kChunkList + k] = i;
                    }
                    if (lane_id() == 0) {
                        *(gptr<v4i>)r = v4i{x, ev, fx, min(nw, kChunkList + 1)};
                        ch_ev(L)[c] = ev;
                    }
                }
            }
            for (int q = (c0 >> 6) + lane_id(); q <= (c1 >> 6); q += 64) sup_mark(L)[q] = 1;
            wsync();
        }
    }
    // the figures of the superchunks marked stale (before a view reads them, and before the launch ends)
    static MTR_DI void sup_refresh(D& L, const St& s) {
        if constexpr (G) {
            if (!s.chunked || s.nseg <= 0) return;
            const int nch = (s.nseg + 63) >> 6, ns = (nch + 63) >> 6, ln = lane_id();
            const lptr<int> mk = sup_mark(L), sl = sup_len(L), se = sup_ev(L), ce = ch_ev(L);
            for (int b = 0; b < ns; b += 64) {
                uint64_t m = __ballot(b + ln < ns && mk[min(b + ln, ns - 1)] != 0);
                while (m) {  // kDirtyBatch superchunks' chunk lengths in flight together
                    int q[kDirtyBatch], x[kDirtyBatch];
#pragma unroll
                    for (int k = 0; k < kDirtyBatch; k++) {
                        q[k] = m ? b + first_lane(m) : -1;
                        m &= m - 1;
                        x[k] = cs_rec(L, min(max(q[k], 0) * 64 + ln, nch - 1))[0];
                    }
#pragma unroll
                    for (int k = 0; k < kDirtyBatch; k++) {
                        if (q[k] < 0) break;
                        const int c = q[k] * 64 + ln;
                        const bool ok = c < nch;
                        const int sum = rdlane(wave_incl_scan(ok ? x[k] : 0), 63);
                        int ev = ok ? ce[min(c, nch - 1)] : 0;
#pragma unroll
                        for (int o = 1; o < 64; o <<= 1) ev = max(ev, __shfl_xor(ev, o));
                        if (ln == 0) {
                            sl[q[k]] = sum;
                            se[q[k]] = ev;
                            mk[q[k]] = 0;
                        }
                    }
                }
            }
            wsync();
        }
    }
    // the superchunk rows and chunk newest events between launches: read at launch start, refreshed and
    // written back at its end (the records themselves live in HBM)
    static MTR_DI void sup_load(D& L, const St& s) {
        if constexpr (G) {
            if (!s.chunked || s.nseg <= 0 || !L.gcsum()) return;  // (query kernels carry no summaries)
            const int nch = (s.nseg + 63) >> 6, ns = (nch + 63) >> 6;
            const gptr<int> gl = cs_sl(L), ge = cs_se(L);
            for (int q = lane_id(); q < ns; q += 64) {
                sup_len(L)[q] = gl[q];
                sup_ev(L)[q] = ge[q];
            }
            for (int c = lane_id(); c < nch; c += 64) ch_ev(L)[c] = cs_rec(L, c)[1];
            wsync();
        }
    }
    static MTR_DI void sup_flush(D& L, const St& s) {
        if constexpr (G) {
            if (!s.chunked || s.nseg <= 0 || !L.gcsum()) return;
            sup_refresh(L, s);
            const int ns = (((s.nseg + 63) >> 6) + 63) >> 6;
            const gptr<int> gl = cs_sl(L), ge = cs_se(L);
            for (int q = lane_id(); q < ns; q += 64) {
                gl[q] = sup_len(L)[q];
                ge[q] = sup_ev(L)[q];
            }
            wsync();
        }
    }
    // ---- the team: an HBM-resident document's workgroup of MTR_GW waves.  Wave 0 runs the document; a pass it
    // hands out is posted in the mailbox (task word + arguments), and the waves meet at the workgroup barrier
    // twice: once to start (the helpers wait there between passes) and once when every wave's share is done.
    enum { T_EXIT = 1, T_DIRTY = 2, T_PARENT = 3, T_PREFIX = 4, T_PACK = 5 };
    static_assert(16 + 2 * 4 * MTR_GW <= kTeamInts, "the team's mailbox holds two rows of results per wave");
    static MTR_DI int team_n() {
        if constexpr (G) return int(blockDim.x) >> 6;
        return 1;
    }
    static MTR_DI lptr<int> tbox(const D& L) { return L.sx - kTeamInts; }
    // wave 0: post task `t` (the arguments were written by lane 0 before) and start the team
    static MTR_DI void team_start(const D& L, int t) {
        if (lane_id() == 0) tbox(L)[0] = t;
        __syncthreads();
    }
    // the helper waves (w >= 1): wait for passes until wave 0 posts T_EXIT
    static MTR_DI void team_helper(char* smem, const KParams& P, uint32_t d, int w) {
        if constexpr (G) {
            D L;
            carve_ptrs(L, smem, P, d);
            const int W = team_n();
            for (;;) {
                __syncthreads();
                const lptr<int> b = tbox(L);
                const int t = uni(b[0]);
                if (t != T_DIRTY && t != T_PREFIX && t != T_PARENT && t != T_PACK) break;  // T_EXIT
                {
#ifdef MTR_PROF
                    ProfScope _prof_helper(L.sc, P_HELPER);  // (the pass, not the wait at its end)
#endif
                    View v;
                    v.ref = uni(b[2]);
                    v.client = uniu(uint32_t(b[3]));
                    v.local = uni(b[4]);
                    if (t == T_DIRTY) {
                        dirty_part(L, v, uni(b[5]), uni(b[6]), uni(b[7]), uni(b[1]), w, W, dlist(L), true);
                    } else if (t == T_PREFIX) {
                        (void)prefix2_part(L, v, uni(b[5]), uni(b[6]), uni(b[7]), uni(b[1]), w, W);
                    } else if (t == T_PARENT) {
                        int ps, pe, cnt;
                        parent_part(L, uni(b[1]), uni(b[8]), uni(b[2]), uni(b[3]), w, W, ps, pe, cnt);
                    } else {
                        (void)pack_part(L, uni(b[1]), uni(b[2]), uni(b[3]), uni(b[4]), w, W);
                    }
                }
                __syncthreads();
            }
        }
    }
    static MTR_DI void team_exit(char* smem) {
        if constexpr (G) {
            if (team_n() > 1) {
                if (lane_id() == 0) ((lptr<int>)(smem + kScBytes))[0] = T_EXIT;
                __syncthreads();
            }
        }
    }
    // view lengths of the listed chunks (dlist[0, n)) into ch_x, their change from the local lengths into
    // their superchunks' sup_dlen (a team of waves takes the rounds of 64 chunks in turn)
    static MTR_DI void dirty_chunks(D& L, const St& s, const View& v, int newlen, int n) {
        PROF(P_PFSUM);  // (the listed chunks' evaluation; P_PFDIRTY: the unlisted ones inside it)
        const int W = team_n();
        if (W > 1 && n > 64) {
            const lptr<int> b = tbox(L);
            if (lane_id() == 0) {
                b[1] = n;
                b[2] = v.ref;
                b[3] = int(v.client);
                b[4] = v.local;
                b[5] = newlen;
                b[6] = s.minseq;
                b[7] = s.nseg;
            }
            team_start(L, T_DIRTY);
            dirty_part(L, v, newlen, s.minseq, s.nseg, n, 0, W, dlist(L), true);
            __syncthreads();
            return;
        }
        dirty_part(L, v, newlen, s.minseq, s.nseg, n, 0, 1, dlist(L), false);
        wsync();
    }
    // wave w of W: rounds w, w + W, ... of the listed chunks
    static MTR_DI void dirty_part(D& L, const View& v, int newlen, int minseq, int S, int n, int w, int W,
                                  lptr<int> lst, bool atomic) {
        const int ln = lane_id();
        const lptr<int> cx = ch_x(L), sd = sup_dlen(L);
        // one lane per chunk: its record's head and visibility fields in one round of loads, issued a round ahead
        // (the slot list is read only by a lane whose leaf needs its remover list walked)
        int cn = 0;
        v4i hn = v4i{0, 0, 0, 0}, hvn[kChunkList];
        if (64 * w < n) {
            cn = lst[min(64 * w + ln, n - 1)];
            const gptr<int> r = cs_rec(L, cn);
            hn = ld4(r);
#pragma unroll
            for (int j = 0; j < kChunkList; j++) hvn[j] = ld4(r + 4 + 4 * j);
        }
        for (int e0 = 64 * w; e0 < n; e0 += 64 * W) {
#ifdef MTR_PROF
            if ((threadIdx.x >> 6) == 0) PROF_COUNT(P_NDRND);
#endif
            const int e = e0 + ln;
            const int c = cn;
            const gptr<int> r = cs_rec(L, c);
            const v4i h = hn;
            v4i hv[kChunkList];
#pragma unroll
            for (int j = 0; j < kChunkList; j++) hv[j] = hvn[j];
            if (e0 + 64 * W < n) {  // (uniform) the next round's records
                cn = lst[min(e0 + 64 * W + ln, n - 1)];
                const gptr<int> rn = cs_rec(L, cn);
                hn = ld4(rn);
#pragma unroll
                for (int j = 0; j < kChunkList; j++) hvn[j] = ld4(rn + 4 + 4 * j);
            }
            const bool listed = e < n && h.w <= kChunkList;
            int sum = h.z;
            // (the wave's longest list bounds the tests: a chunk holds a few window leaves, its record up to 12)
            int jm = listed ? h.w : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) jm = max(jm, __shfl_xor(jm, o));
            jm = __builtin_amdgcn_readfirstlane(jm);
#pragma unroll
            for (int j = 0; j < kChunkList; j++) {
                if (j < jm) {  // (a uniform skip; no break: the record stays in registers)
                    const bool on = listed && j < h.w;
                    const Hot hj{hv[j].x, hv[j].y, hv[j].z, uint32_t(hv[j].w)};
                    const int x0 =
                        vis_hot(L, hj, 0, v, newlen, minseq, on, (gptr<const int>)(r + 4 + 4 * kChunkList + j));
                    sum += on ? max(x0, 0) : 0;
                }
            }
            int vl = sum;
            uint64_t um = __ballot(e < n && !listed);
#ifdef MTR_PROF
            const bool lead = (threadIdx.x >> 6) == 0;  // (wave 0; the helpers' time is P_HELPER)
            if (ln == 0 && lead) L.sc->prof[P_NDIRTY] += (unsigned long long)__popcll(um);
            ProfScope _prof_dirty(L.sc, lead ? P_PFDIRTY : P_SINK);
#endif
            while (um) {  // more than kChunkList leaves in the window: the chunk's leaves, GK chunks at a time
                int lq[GK];
                Hot hw[GK];
#pragma unroll
                for (int g = 0; g < GK; g++) {
                    lq[g] = um ? first_lane(um) : -1;
                    um &= um - 1;
                    const int i = rdlane(c, max(lq[g], 0)) * 64 + ln;
                    hw[g] = ld_hot(L, min(i, S - 1));
                }
#pragma unroll
                for (int g = 0; g < GK; g++) {
                    if (lq[g] < 0) break;
                    const int i = rdlane(c, lq[g]) * 64 + ln;
                    const int x0 = vis_hot(L, hw[g], i, v, newlen, minseq, i < S);
                    const int tot = rdlane(wave_incl_scan(i < S ? max(x0, 0) : 0), 63);
                    if (ln == lq[g]) vl = tot;
                }
            }
            if (e < n) cx[c] = vl;
            // each superchunk's change: the listed chunks come superchunk by superchunk, so lanes of one
            // superchunk are contiguous -- a segmented sum (one scan, one shuffle) and one plain add by the
            // segment's last lane, instead of 64 same-address LDS atomics that serialize
            const int key = e < n ? (c >> 6) : -1;
            const int dv = e < n ? vl - h.x : 0;
            const int inc = wave_incl_scan(dv);
            const int kprev = __shfl(key, max(ln - 1, 0)), knext = __shfl(key, min(ln + 1, 63));
            const uint64_t starts = __ballot(ln == 0 || key != kprev);
            const int first = last_lane(starts & ((uint64_t(2) << ln) - 1));
            const int base = __shfl(inc, first) - __shfl(dv, first);
            if (e < n && (ln == 63 || knext != key)) {
                if (atomic)  // (another wave may hold chunks of the same superchunk)
                    __hip_atomic_fetch_add(&sd[key], inc - base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    sd[key] += inc - base;
            }
        }
    }
    // the view's superchunk lengths and their inclusive prefix in sup_pre; returns the view's total length.
    // need < INT32_MAX: the caller reads the view only up to position need - 1 (its searches stop at the first
    // superchunk whose prefix reaches need, and its windows reach at most one superchunk further), so the scan
    // stops once the superchunk after the one reaching need is complete -- the dirty chunks of later
    // superchunks are not evaluated, sup_pre is valid up to there and the returned length is partial.
    static MTR_DI int prefix2(D& L, const St& s, const View& v, int newlen, int need = INT32_MAX) {
        PROF(P_PREFIX);
        {
#ifdef MTR_PROF
            ProfScope _prof_sr(L.sc, P_SUPREF);
#endif
            sup_refresh(L, s);
        }
        const int nch = (s.nseg + 63) >> 6, ns = (nch + 63) >> 6, ln = lane_id();
        const int ep = uni(L.sc->sepoch) + 1;
        if (ln == 0) {
            L.sc->sepoch = ep;
            L.sc->vref = v.local ? INT32_MAX : v.ref;  // (a local view: every chunk shows its local length)
        }
        if (team_n() > 1 && !v.local) {  // the team lists and evaluates the superchunks' chunks with later events
            const lptr<int> b = tbox(L);
            if (ln == 0) {
                b[1] = need;
                b[2] = v.ref;
                b[3] = int(v.client);
                b[4] = v.local;
                b[5] = newlen;
                b[6] = s.minseq;
                b[7] = s.nseg;
            }
            team_start(L, T_PREFIX);
            const int total = prefix2_part(L, v, newlen, s.minseq, s.nseg, need, 0, team_n());
            __syncthreads();
            return total;
        }
        const lptr<int> sl = sup_len(L), se = sup_ev(L), sd = sup_dlen(L), spre = sup_pre(L), ce = ch_ev(L),
                        lst = dlist(L);
        int carry = 0;
        for (int b = 0; b < ns; b += 64) {
            const int q = b + ln, qc = min(q, ns - 1);
            const int sl0 = sl[qc], se0 = se[qc];
            const uint64_t dq0 = __ballot(q < ns && !v.local && se0 > v.ref);
            if ((dq0 >> ln) & 1) sd[q] = 0;
            wsync();
#ifdef MTR_PROF
            if (ln == 0) {
                L.sc->prof[P_NCH] += (unsigned long long)min(64, ns - b);
                L.sc->prof[P_NSUP] += (unsigned long long)__popcll(dq0);
            }
#endif
            int n = 0;
            for (uint64_t dq = dq0; dq;) {  // their chunks with later events, listed from the LDS newest events
                const int c = (b + first_lane(dq)) * 64 + ln;
                dq &= dq - 1;
                const bool dirty = c < nch && ce[min(c, nch - 1)] > v.ref;
                const uint64_t dm = __ballot(dirty);
                if (dirty) lst[n + __popcll(dm & lanes_below())] = c;
                n += __popcll(dm);
                // (a bounded scan evaluates the list every 128+ entries, so it can stop within a few superchunks
                // of need)
                if (n > kListCap - 64 || !dq || (need != INT32_MAX && n >= 128)) {
                    wsync();
#ifdef MTR_PROF
                    if (ln == 0) L.sc->prof[P_NDCH] += (unsigned long long)n;
#endif
                    dirty_chunks(L, s, v, newlen, n);
                    n = 0;
                    if (need != INT32_MAX && dq) {
                        // superchunks [b, b + lim) are complete (the next dirty one not listed yet): stop when one
                        // of them starts at or after need -- the one before it reached need
                        const int lim = first_lane(dq);
                        const bool in = q < ns && ln < lim;
                        const int slen = in ? sl0 + (((dq0 >> ln) & 1) ? sd[q] : 0) : 0;
                        const int inc = wave_incl_scan(slen);
                        if (__ballot(in && carry + inc - slen >= need)) {
                            if (in) spre[q] = carry + inc;
                            wsync();
                            return carry + rdlane(inc, 63);
                        }
                    }
                }
            }
            const int slen = q < ns ? sl0 + (((dq0 >> ln) & 1) ? sd[q] : 0) : 0;
            const int inc = wave_incl_scan(slen);
            if (q < ns) spre[q] = carry + inc;
            const bool reached = __ballot(q < ns && carry + inc - slen >= need) != 0;
            carry += rdlane(inc, 63);
            if (reached) break;  // (the whole batch is complete)
        }
        wsync();
        return carry;
    }
    // prefix2 on a team of W waves (wave w): the superchunks with later events go in rounds of kTeamSup per wave
    // -- wave w lists the dirty chunks of its kTeamSup consecutive ones (in rank order) into its own part of the
    // list and evaluates them -- and after each round every wave checks, from the same LDS words, whether the
    // superchunks done so far reach `need` (the bounded scan's stop, as prefix2's).  Returns the view's total
    // (partial when bounded) on every wave; wave 0 writes sup_pre.
#ifndef MTR_TEAM_SUP
#define MTR_TEAM_SUP 12
#endif
    static constexpr int kTeamSup = MTR_TEAM_SUP;
    // the index of the r-th set bit of m (m has more than r)
    static MTR_DI int nth_set(uint64_t m, int r) {
        const int ln = lane_id();
        const bool mine = ((m >> ln) & 1) && __popcll(m & lanes_below()) == r;
        return first_lane(__ballot(mine));
    }
    static MTR_DI int prefix2_part(D& L, const View& v, int newlen, int minseq, int S, int need, int w, int W) {
        const int nch = (S + 63) >> 6, ns = (nch + 63) >> 6, ln = lane_id();
        const lptr<int> sl = sup_len(L), se = sup_ev(L), sd = sup_dlen(L), spre = sup_pre(L), ce = ch_ev(L);
        const int lcap = kListCap / W;
        const lptr<int> lst = dlist(L) + w * lcap;
        int carry = 0;
        for (int b = 0; b < ns; b += 64) {
            const int q = b + ln, qc = min(q, ns - 1);
            const int sl0 = sl[qc], se0 = se[qc];
            const uint64_t dq0 = __ballot(q < ns && se0 > v.ref);
            if (w == 0 && ((dq0 >> ln) & 1)) sd[q] = 0;
            __syncthreads();  // (the zeros before any wave adds)
            const int nd = __popcll(dq0);
            for (int r0 = 0; r0 < nd; r0 += kTeamSup * W) {
                int n = 0;
                const int r1 = min(r0 + (w + 1) * kTeamSup, nd);
#ifdef MTR_PROF
                const bool lead = w == 0 && (threadIdx.x >> 6) == 0;
                const long long _t_l = clock64();
                if (lead) PROF_COUNT(P_NPXR);
#endif
                for (int r = r0 + w * kTeamSup; r < r1; r += 4) {  // four superchunks' newest events per LDS round
                    int cq[4], eq[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        cq[k] = (b + nth_set(dq0, min(r + k, r1 - 1))) * 64 + ln;
                        eq[k] = ce[min(cq[k], nch - 1)];
                    }
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (r + k >= r1) break;
                        const bool dirty = cq[k] < nch && eq[k] > v.ref;
                        const uint64_t dm = __ballot(dirty);
                        if (dirty) lst[n + __popcll(dm & lanes_below())] = cq[k];
                        n += __popcll(dm);
                        if (n > lcap - 64) {
                            wsync();
                            // (a superchunk's chunks are this wave's alone: plain adds)
#ifdef MTR_PROF
                            ProfScope _prof_ev(L.sc, lead ? P_PXEVAL : P_SINK);
#endif
                            dirty_part(L, v, newlen, minseq, S, n, 0, 1, lst, false);
                            n = 0;
                        }
                    }
                }
                if (n) {
                    wsync();
#ifdef MTR_PROF
                    ProfScope _prof_ev(L.sc, lead ? P_PXEVAL : P_SINK);
#endif
                    dirty_part(L, v, newlen, minseq, S, n, 0, 1, lst, false);
                }
#ifdef MTR_PROF
                if (lead) PROF_ADD(P_PXLIST, _t_l);  // (listing + evaluation; P_PXEVAL the latter)
                const long long _t_s = clock64();
#endif
                __syncthreads();
#ifdef MTR_PROF
                if (lead) PROF_ADD(P_PXSYNC, _t_s);
#endif
                const int rn = r0 + kTeamSup * W;
                if (need != INT32_MAX && rn < nd) {
                    // superchunks [b, b + lim) are complete: stop when one of them starts at or after need
                    const int lim = nth_set(dq0, rn);
                    const bool in = q < ns && ln < lim;
                    const int slen = in ? sl0 + (((dq0 >> ln) & 1) ? sd[q] : 0) : 0;
                    const int inc = wave_incl_scan(slen);
                    if (__ballot(in && carry + inc - slen >= need)) {
                        if (w == 0 && in) spre[q] = carry + inc;
                        wsync();
                        return carry + rdlane(inc, 63);
                    }
                }
            }
            const int slen = q < ns ? sl0 + (((dq0 >> ln) & 1) ? sd[q] : 0) : 0;
            const int inc = wave_incl_scan(slen);
            if (w == 0 && q < ns) spre[q] = carry + inc;
            const bool reached = __ballot(q < ns && carry + inc - slen >= need) != 0;
            carry += rdlane(inc, 63);
            if (reached) break;
        }
        wsync();
        return carry;
    }
    // lane l: the inclusive prefix of chunk 64 q + l within superchunk q in the current view (the row is
    // filled on first use: chunks with later events from ch_x, the others' local lengths from their records)
    static MTR_DI int sup_row(D& L, const St& s, int q) {
        const int nch = (s.nseg + 63) >> 6, c = q * 64 + lane_id(), cc = min(c, nch - 1);
        const int ep = uni(L.sc->sepoch);
        if (uni(sup_fill(L)[q]) == ep) return ch_x(L)[cc];
        const int vref = uni(L.sc->vref);
        const int cl = cs_rec(L, cc)[0];
        const int x = ch_ev(L)[cc] > vref ? ch_x(L)[cc] : cl;
        const int inc = wave_incl_scan(c < nch ? x : 0);
        if (c < nch) ch_x(L)[c] = inc;
        if (lane_id() == 0) sup_fill(L)[q] = ep;
        wsync();
        return inc;
    }
    // the scan array E of chunks [c0, c1] from the chunk prefix
    static MTR_DI void materialize(D& L, const St& s, const View& v, int newlen, int c0, int c1) {
        PROF(P_MAT);
        const int S = s.nseg, ln = lane_id();
        const lptr<int> spre = sup_pre(L);
        int qcur = -1, rel = 0;
        for (int cb = c0; cb <= c1; cb += GK) {
            Hot h[GK];
#pragma unroll
            for (int k = 0; k < GK; k++) h[k] = ld_hot(L, min(min(cb + k, c1) * 64 + ln, S - 1));
#pragma unroll
            for (int k = 0; k < GK; k++) {
                const int c = cb + k;
                if (c > c1) break;
                const int q = c >> 6;
                if (q != qcur && (c & 63)) {
                    rel = sup_row(L, s, q);
                    qcur = q;
                }
                const int base = (q > 0 ? uni(spre[q - 1]) : 0) + ((c & 63) ? rdlane(rel, (c & 63) - 1) : 0);
                const int i = c * 64 + ln;
                const int x0 = vis_hot(L, h[k], i, v, newlen, s.minseq, i < S);
                const int x = i < S ? x0 : 0;
                const int inc = wave_incl_scan(max(x, 0));
                if (i < S) L.E[i] = (base + inc) | (x < 0 ? int(0x80000000u) : 0);
            }
        }
        wsync();
    }
    // first chunk whose inclusive prefix reaches pos (the last chunk if none)
    static MTR_DI int chunk_of(D& L, const St& s, int nch, int pos) {
        PROF(P_CHUNKOF);
        const int ns = (nch + 63) >> 6, ln = lane_id();
        const lptr<int> spre = sup_pre(L);
        int q = -1;
        for (int b = 0; b < ns; b += 64) {
            const uint64_t m = __ballot(b + ln < ns && spre[min(b + ln, ns - 1)] >= pos);
            if (m) {
                q = b + first_lane(m);
                break;
            }
        }
        if (q < 0) return nch - 1;
        const int rel = sup_row(L, s, q);
        const int base = q > 0 ? uni(spre[q - 1]) : 0;
        const uint64_t m = __ballot(q * 64 + ln < nch && base + rel >= pos);
        return m ? q * 64 + first_lane(m) : nch - 1;
    }
    // The op's view scan: flat (prefix) or two-level, with E valid over the chunks around positions
    // [p_lo, p_hi] (one chunk before, two after: the searches' windows and the walk's reach).  Returns
    // the view's total length.
    static MTR_DI int view_scan(D& L, St& s, const View& v, int newlen, int p_lo, int p_hi, bool bounded = false) {
        PROF(P_VIEW);
        if constexpr (G) {
            L.rhi = 0;
            if (s.chunked && s.nseg > 0) {
                // (a bounded scan only when the caller reads no total: the region's searches stop at need)
                const int total = prefix2(L, s, v, newlen, bounded ? p_hi + 1 : INT32_MAX);
                const int nch = (s.nseg + 63) >> 6;
                const int c0 = max(0, chunk_of(L, s, nch, p_lo) - 1);
                // (to the chunk of the first leaf past p_hi: chunks with no length in the view -- runs of
                // holes, leaves removed for it -- may lie between, and breakTie's candidates reach that leaf)
                const int c1 = min(nch - 1, chunk_of(L, s, nch, p_hi + 1) + 2);
                materialize(L, s, v, newlen, c0, c1);
                L.rlo = c0 * 64;
                L.rhi = (c1 + 1) * 64;
                return total;
            }
        }
        prefix(L, s, v, newlen);
        return s.nseg > 0 ? (uni(L.E[s.nseg - 1]) & EMASK) : 0;
    }

    // getContainingSegment of one document (mergeTree.ts:787-813: nodeMap over [pos, pos + 1)): i = the
    // first leaf whose inclusive visible prefix exceeds pos (S if none), before = the visible length
    // ahead of it.  Writes no scan array.
    static MTR_DI void find1(const D& L, const St& s, const View& v, int pos, int& i_out, int& before, int newlen) {
        const int S = s.nseg;
        const int ln = lane_id();
        int c = 0;
        i_out = S;
        before = 0;
        for (int base = 0; base < S; base += 64) {
            const int i = base + ln;
            const Hot h = ld_hot(L, min(i, S - 1));
            const int x0 = vis_hot(L, h, i, v, newlen, s.minseq, i < S);
            const int x = (i < S) ? max(x0, 0) : 0;
            const int inc = wave_incl_scan(x);
            const uint64_t m = __ballot((i < S) & (c + inc > pos));
            if (m) {
                const int l = first_lane(m);
                i_out = base + l;
                before = c + rdlane(inc - x, l);
                return;
            }
            c += rdlane(inc, 63);
        }
        before = c;
    }

    // Client.getContainingSegment(pos, {referenceSequenceNumber, clientId}) (client.ts:1065-1078) on a
    // document's HBM state: out = mtr_segment_info (include/mtr.h) of the leaf holding pos, leaf -1
    // when no segment covers pos in that view
    static MTR_DI void containing(char* smem, const KParams& P, uint32_t d, int pos, int ref, int client, int32_t* out) {
        D L;
        carve(L, smem, P, d);
        St s;
        load_doc(L, P, s, d);
        View v;
        v.ref = ref;
        v.client = enc_client(client);
        v.local = (!s.collab || uint32_t(s.local) == v.client) ? 1 : 0;
        int i, before;
        find1(L, s, v, pos, i, before, P.new_length_calc);
        const int li = (G && s.holes && i < s.nseg) ? count_live(L, 0, i) : i;  // the leaf's ordinal
        if (lane_id() == 0) {
            if (i >= s.nseg || pos < 0) {
                out[0] = -1;
                out[9] = before;  // (no segment: the view's whole length when pos is past it)
            } else {
                const uint32_t m = L.meta[i];
                out[0] = li;
                out[1] = pos - before;
                out[2] = L.len[i];
                out[3] = L.seq[i];
                out[4] = dec_client(m & M_CLIENT_MASK);
                out[5] = L.rseq[i] == RNONE ? -1 : L.rseq[i];
                out[6] = (m & M_MARKER) ? 1 : 0;
                out[7] = int(L.text[i]);
                out[8] = pget(L, i) == NONE32 ? -1 : int(pget(L, i) & PN_MASK);
                out[9] = before;
                int groups = 0;  // segmentGroups.size: the leaf's pending cells (key cells are no group)
                if (m & M_PEND)
                    for (uint32_t c = pd_get(L, L.uid[i]); c != 0xffffffu; c = L.grm()[c] & 0xffffffu)
                        groups += (L.grm()[c + 1] >> 16) != ZOMBIE_SLOT;
                out[10] = groups;
            }
        }
    }

    // Client.localReferencePositionToPosition (client.ts:398-403 -> mergeTree.ts:1046-1062) of every local
    // reference of a document on its HBM state: out[r] = DetachedReferencePosition when the reference has no
    // segment, its segment is gone (unlinked, merged away) or no longer holds it (a Transient one is never held),
    // else its offset (0 on a removed segment) plus the segment's local-view position.  info_id >= 0: out =
    // {leaf ordinal of its segment (-1: none or gone), offset, ReferenceType, held} of that reference instead.
    // info_id == -2: two words per reference, {that position, state bits}: MTR_REF_ST_SEGMENT (it has a segment),
    // MTR_REF_ST_HELD (that segment's LocalReferenceCollection holds it), MTR_REF_ST_REMOVED (its leaf, found in the
    // tree, is removed) -- what an interval collection's compare needs beside the position.
    static MTR_DI void ref_query(char* smem, const KParams& P, uint32_t d, int32_t* out, int info_id) {
        D L;
        carve(L, smem, P, d);
        St s;
        load_doc(L, P, s, d);
        const int n = rf_uid(L) ? nrefs(L) : 0;
        const int S = s.nseg;
        if (info_id >= 0) {
            int o4[4] = {-1, 0, 0, 0};
            if (info_id < n) {
                const uint32_t u = uniu(rf_uid(L)[info_id]), t = uniu(rf_ty(L)[info_id]);
                const int x = u == NONE32 ? -1 : find_uid(L, s, u);
                o4[0] = (x >= 0 && G && s.holes) ? count_live(L, 0, x) : x;
                o4[1] = int(uniu(rf_off(L)[info_id]));
                o4[2] = int(t & ~RF_HELD);
                o4[3] = (t & RF_HELD) ? 1 : 0;
            }
            if (lane_id() == 0)
                for (int q = 0; q < 4; q++) out[q] = o4[q];
            return;
        }
        for (int rb = 0; rb < n; rb += 64) {
            const int r = rb + lane_id();
            const int rc = min(r, n - 1);
            const uint32_t u = rf_uid(L)[rc], o = rf_off(L)[rc], t = rf_ty(L)[rc];
            const bool live = (r < n) & (u != NONE32) & ((t & (RF_HELD | RT_TRANSIENT)) != 0);
            // (info_id -3: every reference that names a segment is looked for: its leaf is the compare key)
            const bool want = info_id == -3 ? (r < n) & (u != NONE32) : live;
            int res = MTR_DETACHED_POSITION, key = -1;
            bool found = false, onrm = false;
            int carry = 0;
            for (int base = 0; base < S && __ballot(want & !found); base += 64) {
                const int i = base + lane_id();
                const int ic = min(i, S - 1);
                const uint32_t m = L.meta[ic];
                const int rs = L.rseq[ic];
                const bool leaf = (i < S) & !(m & M_DEL);
                const int x = (leaf & (rs == RNONE)) ? L.len[ic] : 0;  // local view: removed leaves count 0
                const int inc = wave_incl_scan(x);
                const int excl = carry + inc - x;
                const uint32_t ui = leaf ? L.uid[ic] : NONE32;
                const int rm = rs != RNONE ? 1 : 0;  // isRemoved: acked or pending
                for (int l = 0; l < 64; l++) {  // every reference lane looks for its leaf in this round
                    const uint32_t ul = rdlane(ui, l);
                    const int el = rdlane(excl, l), rl = rdlane(rm, l);
                    const bool hit = want & !found & (ul == u);
                    res = (hit & live) ? (rl ? 0 : int(o)) + el : res;
                    key = hit ? base + l : key;
                    onrm = onrm | (hit & live & (rl != 0));
                    found = found | hit;
                }
                carry += rdlane(inc, 63);
            }
            if (info_id == -3) {
                if (r < n) {
                    out[4 * r] = res;
                    out[4 * r + 1] = (u != NONE32 ? MTR_REF_ST_SEGMENT : 0) | ((t & RF_HELD) ? MTR_REF_ST_HELD : 0) |
                                     (onrm ? MTR_REF_ST_REMOVED : 0);
                    out[4 * r + 2] = u == NONE32 ? -1 : (found ? key : -2);
                    out[4 * r + 3] = int(o);
                }
            } else if (info_id == -2) {
                if (r < n) {
                    out[2 * r] = res;
                    out[2 * r + 1] = (u != NONE32 ? MTR_REF_ST_SEGMENT : 0) | ((t & RF_HELD) ? MTR_REF_ST_HELD : 0) |
                                     (onrm ? MTR_REF_ST_REMOVED : 0);
                }
            } else if (r < n) {
                out[r] = res;
            }
        }
    }

    // getContainingSegment for two vectors at once (a setCell's row and col): two visibility scans
    // interleaved round by round (independent chains of LDS reads and DPP scans that overlap), each
    // stopping at the round that reaches its position.  ia / ib = first leaf whose inclusive
    // visible prefix exceeds pa / pb (S if none, as lower_bound_E(pos + 1)); bfa / bfb = the
    // visible length before it.  Writes no scan array.
    static MTR_DI void find2(const D& La, const St& sa, const View& va, int pa, int& ia, int& bfa, const D& Lb,
                             const St& sb, const View& vb, int pb, int& ib, int& bfb, int newlen) {
#ifdef MTR_PROF
        ProfScope _prof_scope(La.sc, P_PREFIX);
#endif
        const int Sa = sa.nseg, Sb = sb.nseg;
        const int ln = lane_id();
        int ca = 0, cb = 0;
        ia = -1;
        ib = -1;
        // software-pipelined: each round's leaf fields were loaded during the previous round
        Hot ha = Sa > 0 ? ld_hot(La, ln) : Hot{}, hb = Sb > 0 ? ld_hot(Lb, ln) : Hot{};
        for (int base = 0;; base += 64) {
            const bool ga = ia < 0 && base < Sa, gb = ib < 0 && base < Sb;  // uniform
            if (!ga && ia < 0) { ia = Sa; bfa = ca; }
            if (!gb && ib < 0) { ib = Sb; bfb = cb; }
            if (!ga && !gb) break;
            const int i = base + ln;
            const Hot ca_h = ha, cb_h = hb;
            if (ga && base + 64 < Sa) ha = ld_hot(La, i + 64);
            if (gb && base + 64 < Sb) hb = ld_hot(Lb, i + 64);
            int xa = 0, xb = 0;
            if (ga) {
                const int x0 = vis_hot(La, ca_h, i, va, newlen, sa.minseq, i < Sa);
                xa = i < Sa ? max(x0, 0) : 0;
            }
            if (gb) {
                const int x0 = vis_hot(Lb, cb_h, i, vb, newlen, sb.minseq, i < Sb);
                xb = i < Sb ? max(x0, 0) : 0;
            }
            const int sa_ = wave_incl_scan(xa);
            const int sb_ = wave_incl_scan(xb);
            if (ga) {
                const uint64_t m = __ballot(i < Sa && ca + sa_ > pa);
                if (m) {
                    const int l = first_lane(m);
                    ia = base + l;
                    bfa = ca + rdlane(sa_ - xa, l);
                } else {
                    ca += rdlane(sa_, 63);
                }
            }
            if (gb) {
                const uint64_t m = __ballot(i < Sb && cb + sb_ > pb);
                if (m) {
                    const int l = first_lane(m);
                    ib = base + l;
                    bfb = cb + rdlane(sb_ - xb, l);
                } else {
                    cb += rdlane(sb_, 63);
                }
            }
        }
    }

    // ------------------------------------------------------------ data movement
    // move leaves [at, S) (with their scan entries) to [at+1, S+1); rounds of 64 from the top.
    // HBM-resident documents with hole slots (Eng::spread) only move [at, h) into the first hole h at
    // or after `at`.  Returns whether the slot count grew (no hole was taken).
    static MTR_DI bool shift_right1(D& L, St& s, int at) {
        PROF(P_SHIFT);
        int S = s.nseg;
        bool grew = true;
        if constexpr (G) {  // GK rounds per group: every load of the group before its stores (a round's
                            // stores land above every slot the group's lower rounds read)
            if (s.holes > 0) {  // the first hole at or after `at`, within a bounded window (GK rounds of loads
                                // in flight per step)
                const int lim = min(S, at + kHoleWindow);
                bool found = false;
                for (int base = at; base < lim && !found; base += 64 * GK) {
                    uint32_t mq[GK];
#pragma unroll
                    for (int q = 0; q < GK; q++) mq[q] = L.meta[min(base + 64 * q + lane_id(), S - 1)];
#pragma unroll
                    for (int q = 0; q < GK; q++) {
                        const int i = base + 64 * q + lane_id();
                        const uint64_t hm = __ballot(i < lim && (mq[q] & M_DEL));
                        if (hm) {
                            S = base + 64 * q + first_lane(hm);  // move [at, hole) up into the hole
                            grew = false;
                            s.holes--;
                            found = true;
                            break;
                        }
                    }
                }
            }
            L.shi = S + 1;  // slots [at, S + 1) changed
            for (int hi = S; hi > at; hi -= 64 * GK) {
                int a0[GK], a1[GK], a2[GK], a8[GK];
                uint32_t a3[GK], a4[GK], a5[GK], a7[GK];
                bool act[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int hq = hi - 64 * q;
                    const int i = max(at, hq - 64) + lane_id();
                    act[q] = hq > at && i < hq;
                    const int ic = max(min(i, S - 1), 0);
                    a0[q] = L.len[ic]; a1[q] = L.seq[ic]; a2[q] = L.rseq[ic]; a8[q] = L.E[ic];
                    a3[q] = L.meta[ic]; a4[q] = L.text[ic]; a5[q] = pget(L, ic); a7[q] = L.uid[ic];
                }
                wsync();
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = max(at, hi - 64 * q - 64) + lane_id();
                    if (act[q]) {
                        L.len[i + 1] = a0[q]; L.seq[i + 1] = a1[q]; L.rseq[i + 1] = a2[q]; L.meta[i + 1] = a3[q];
                        L.text[i + 1] = a4[q]; pset(L, i + 1, a5[q]); L.uid[i + 1] = a7[q]; L.E[i + 1] = a8[q];
                        if (s.chunked) hint(L, a7[q], i + 1);
                    }
                }
                wsync();
            }
            return grew;
        }
        for (int hi = S; hi > at; hi -= 64) {
            const int lo = max(at, hi - 64);
            const int i = lo + lane_id();
            const bool act = i < hi;
            const int ic = min(i, S - 1);  // (unconditional loads: no divergent branch around them)
            const int a0 = L.len[ic], a1 = L.seq[ic], a2 = L.rseq[ic], a8 = L.E[ic];
            const uint32_t a3 = L.meta[ic], a4 = L.text[ic], a5 = pget(L, ic), a7 = L.uid[ic];
            wsync();
            if (act) {
                L.len[i + 1] = a0; L.seq[i + 1] = a1; L.rseq[i + 1] = a2; L.meta[i + 1] = a3; L.text[i + 1] = a4;
                pset(L, i + 1, a5); L.uid[i + 1] = a7; L.E[i + 1] = a8;
            }
            wsync();
        }
        return grew;
    }

    // stream compaction of leaves without M_DEL (zamboni unlink / append); rounds of 64 from the
    // bottom; destinations never exceed sources
    static MTR_DI void compact(D& L, St& s, int from) {
        PROF(P_COMPACT);
        PROF_COUNT(P_NCOMPACT);
        const int S = s.nseg;
        int base = from;
        if constexpr (G) {  // GK rounds per group, loads first (destinations never pass the group's sources)
            for (int lo = from; lo < S; lo += 64 * GK) {
                int a0[GK], a1[GK], a2[GK];
                uint32_t a3[GK], a4[GK], a5[GK], a7[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int ic = min(lo + 64 * q + lane_id(), S - 1);
                    a0[q] = L.len[ic]; a1[q] = L.seq[ic]; a2[q] = L.rseq[ic];
                    a3[q] = L.meta[ic]; a4[q] = L.text[ic]; a5[q] = pget(L, ic); a7[q] = L.uid[ic];
                }
                wsync();
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = lo + 64 * q + lane_id();
                    const bool keep = i < S && !(a3[q] & M_DEL);
                    const uint64_t km = __ballot(keep);
                    if (keep) {
                        const int d = base + __popcll(km & lanes_below());
                        L.len[d] = a0[q]; L.seq[d] = a1[q]; L.rseq[d] = a2[q]; L.meta[d] = a3[q];
                        L.text[d] = a4[q]; pset(L, d, a5[q]); L.uid[d] = a7[q];
                    }
                    base += __popcll(km);
                }
                wsync();
            }
            s.nseg = base;
            if (base == 0) s.height = 1;
            return;
        }
        for (int lo = from; lo < S; lo += 64) {
            const int i = lo + lane_id();
            const bool act = i < S;
            const int ic = min(i, S - 1);
            const int a0 = L.len[ic], a1 = L.seq[ic], a2 = L.rseq[ic];
            const uint32_t a3 = L.meta[ic], a4 = L.text[ic], a5 = pget(L, ic), a7 = L.uid[ic];
            const bool keep = act & !(a3 & M_DEL);
            const uint64_t km = __ballot(keep);
            wsync();
            if (keep) {
                const int d = base + __popcll(km & lanes_below());
                L.len[d] = a0; L.seq[d] = a1; L.rseq[d] = a2; L.meta[d] = a3;
                L.text[d] = a4; pset(L, d, a5); L.uid[d] = a7;
            }
            base += __popcll(km);
            wsync();
        }
        s.nseg = base;
        if (base == 0) s.height = 1;
    }

    // uid -> slot hint of a chunked document (find_uid checks it before scanning; a stale hint only costs
    // the scan)
    static MTR_DI void hint(const D& L, uint32_t u, int i) {
        if constexpr (G) {
            if (u < uint32_t(2 * L.cap)) L.gumap()[u] = i;
        }
    }

    // ---- hole slots (HBM-resident documents of >= kGapMin leaves): a hole is a slot with M_DEL, no
    // length, no uid and removedSeq 0 -- undefined in every view (vis_hot), skipped by every walk,
    // scour and summary; shifts take the next hole (shift_right1), zamboni leaves its deleted leaves
    // as holes (holeify) instead of compacting the rest of the document
    static MTR_DI void hole_fields(D& L, int i) {
        L.meta[i] = M_DEL;
        L.len[i] = 0;
        L.seq[i] = 0;
        L.rseq[i] = 0;
        L.uid[i] = NONE32;
        pset(L, i, NONE32);
        L.text[i] = uint32_t(MTR_HANDLE_UNALLOCATED);
    }
    static MTR_DI void holeify(D& L, St& s, int from, int to) {
        int made = 0;
        for (int base = from; base < to; base += 64) {
            const int i = base + lane_id();
            const bool in = i < to;
            const uint32_t m = L.meta[min(i, to - 1)];
            const uint32_t u = L.uid[min(i, to - 1)];
            const bool h = in && (m & M_DEL) && u != NONE32;  // newly deleted
            if (h && s.chunked && u < uint32_t(2 * L.cap)) L.gumap()[u] = -2;  // the uid is gone for good
            if (h) hole_fields(L, i);
            made += __popcll(__ballot(h));
        }
        wsync();
        s.holes += made;
        if (s.holes >= s.nseg) {  // nothing left
            s.nseg = 0;
            s.holes = 0;
            s.height = 1;
            s.chunked = 0;
        }
    }
    // Lay the leaves out with one hole per kGapEvery slots (all holes squeezed out first): leaf k goes
    // to slot k + k / (kGapEvery - 1).  Moves run from the top down, so no leaf is overwritten before it
    // is read.  Only between ops (no leaf index is held).
    static MTR_DI void spread(D& L, St& s, int cap) {
        PROF(P_SPREAD);
        PROF_COUNT(P_NSPREAD);
        s.chunked = 0;
        if (s.holes) {
            compact(L, s, 0);
            s.holes = 0;
        }
        const int S = s.nseg;
        const int n_new = S + (S - 1) / (kGapEvery - 1) + 1;
        if (S < kGapMin || n_new > cap) return;
        for (int top = S; top > 0; top -= 64) {
            const int i = top - 64 + lane_id();
            const bool in = i >= 0;
            const int ic = max(i, 0);
            const int a0 = L.len[ic], a1 = L.seq[ic], a2 = L.rseq[ic];
            const uint32_t a3 = L.meta[ic], a4 = L.text[ic], a5 = pget(L, ic), a7 = L.uid[ic];
            wsync();
            if (in) {
                const int d = i + i / (kGapEvery - 1);
                L.len[d] = a0; L.seq[d] = a1; L.rseq[d] = a2; L.meta[d] = a3;
                L.text[d] = a4; pset(L, d, a5); L.uid[d] = a7;
                if (L.gumap()) hint(L, a7, d);
            }
            wsync();
        }
        const int last = (S - 1) + (S - 1) / (kGapEvery - 1);  // slot of the last leaf
        for (int i = lane_id(); i <= last; i += 64)
            if (i % kGapEvery == kGapEvery - 1) hole_fields(L, i);
        wsync();
        s.nseg = last + 1;
        s.holes = s.nseg - S;
        s.chunked = L.gcsum() ? 1 : 0;  // chunk summaries for the two-level view scan
        csum_update(L, s, 0, s.nseg);
    }

    // index of the leaf with this uid, -1 if unlinked (uids are unique)
    static MTR_DI int find_uid(const D& L, const St& s, uint32_t u) {
        PROF(P_FINDUID);
        const int S = s.nseg;
        if constexpr (G) {  // one word per leaf: 4 * GK rounds of loads in flight
            if (s.chunked && u < uint32_t(2 * L.cap)) {  // the slot hint, verified
                const int h = uni(L.gumap()[u]);
                if (h == -2) return -1;  // merged away or unlinked (holeify): uids are never reused
                if (h >= 0 && h < S && uniu(L.uid[h]) == u) return h;
            }
            constexpr int FK = 4 * GK;
            for (int base = 0; base < S; base += 64 * FK) {
                uint32_t uk[FK];
#pragma unroll
                for (int q = 0; q < FK; q++) uk[q] = L.uid[min(base + 64 * q + lane_id(), S - 1)];
#pragma unroll
                for (int q = 0; q < FK; q++) {
                    const uint64_t m = __ballot((base + 64 * q + lane_id() < S) & (uk[q] == u));
                    if (m) return base + 64 * q + first_lane(m);
                }
            }
            return -1;
        }
        for (int base = 0; base < S; base += 64) {
            const int i = base + lane_id();
            const uint32_t ui = L.uid[min(i, S - 1)];  // unconditional (clamped) load: no divergent branch
            const uint64_t m = __ballot((i < S) & (ui == u));
            if (m) return base + first_lane(m);
        }
        return -1;
    }

    // ------------------------------------------------------------ searches (ballots)
    // start of the level-`level` block holding leaf x: last i <= x with i == 0 or bnd >= level
    static MTR_DI int block_start(const D& L, int x, int level) {
        if constexpr (G) {  // HBM: GK rounds of loads in flight per step
            for (int base = x;; base -= 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[max(base - 64 * q - lane_id(), 0)];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = base - 64 * q - lane_id();
                    const uint64_t m = __ballot((i <= 0) | (bnd_of(mq[q]) >= level));
                    if (m) return max(0, base - 64 * q - first_lane(m));
                }
            }
        }
        for (int base = x;; base -= 64) {
            const int i = base - lane_id();
            const uint32_t mi = L.meta[max(i, 0)];
            const uint64_t m = __ballot((i <= 0) | (bnd_of(mi) >= level));
            if (m) return max(0, base - first_lane(m));
        }
    }
    // end (exclusive) of the level-`level` block holding leaf x
    static MTR_DI int block_end(const D& L, const St& s, int x, int level) {
        const int S = s.nseg;
        if constexpr (G) {
            for (int base = x + 1;; base += 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[max(min(base + 64 * q + lane_id(), S - 1), 0)];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = base + 64 * q + lane_id();
                    const uint64_t m = __ballot((i >= S) | (bnd_of(mq[q]) >= level));
                    if (m) return base + 64 * q + first_lane(m);
                }
            }
        }
        for (int base = x + 1;; base += 64) {
            const int i = base + lane_id();
            const uint32_t mi = L.meta[max(min(i, S - 1), 0)];
            const uint64_t m = __ballot((i >= S) | (bnd_of(mi) >= level));
            if (m) return base + first_lane(m);
        }
    }
    // first i with E[i] >= pos (S if none): 64-ary search
    static MTR_DI int lower_bound_E(const D& L, const St& s, int pos) {
        int lo = 0, hi = s.nseg;  // answer in [lo, hi]; hi qualifies (or is S)
        if (G && L.rhi > 0) {  // a two-level scan: E holds only the op's region
            lo = min(L.rlo, s.nseg);
            hi = min(L.rhi, s.nseg);
        }
        const int ln = lane_id();
        while (hi - lo > 64) {
            // the hi - lo + 1 candidates in 64 strides: lane 63's probe reaches hi, which qualifies
            const int stride = (hi - lo + 64) >> 6;
            const int idx = lo + (ln + 1) * stride - 1;
            const int ei = L.E[min(idx, hi - 1)];
            const uint64_t m = __ballot((idx >= hi) | ((ei & EMASK) >= pos));
            const int k = first_lane(m);  // lane 63 always qualifies
            const int nlo = lo + k * stride;
            hi = min(hi, lo + (k + 1) * stride - 1);
            lo = nlo;
        }
        const int i = lo + ln;
        const int ei = L.E[min(i, max(hi - 1, 0))];
        const uint64_t m = __ballot((i < hi) & ((ei & EMASK) >= pos));
        return m ? lo + first_lane(m) : hi;
    }
    // The level-`level` block around slot x (the start of a level-(level - 1) block) and its child count (slots
    // with bnd >= level - 1): block_start + block_end + count_bnd in one pass that walks both ways at once --
    // GK rounds of loads in flight per direction -- instead of three passes one after the other (HBM-resident
    // documents, whose upper blocks can span thousands of slots).  The block's end is the first bnd >= level
    // after x: none lies between its start and x.
    static MTR_DI void parent_block(const D& L, const St& s, int x, int level, int& ps, int& pe, int& cnt) {
        if (team_n() > 1) {  // the team walks W * GK rounds per direction per step
            team_bounds(L, s, x, x + 1, level, ps, pe, cnt);
            return;
        }
        parent_walk(L, s, x, level, ps, pe, cnt);
    }
    // the team's walk: the last slot <= xb and the first slot >= xf with bnd >= level (ps, pe), and the slots
    // with bnd >= level - 1 in [ps, pe) -- xf > xb, no such slot in (xb, xf) -- counted in cnt
    static MTR_DI void team_bounds(const D& L, const St& s, int xb, int xf, int level, int& ps, int& pe, int& cnt) {
        const lptr<int> b = tbox(L);
        if (lane_id() == 0) {
            b[1] = xb;
            b[2] = level;
            b[3] = s.nseg;
            b[8] = xf;
        }
        team_start(L, T_PARENT);
        parent_part(L, xb, xf, level, s.nseg, 0, team_n(), ps, pe, cnt);
        __syncthreads();
    }
    // wave w of a team of W: step t covers slots x - (t W + w) 64 GK - [0, 64 GK) backwards and x + 1 + (t W + w)
    // 64 GK + [0, 64 GK) forwards; each wave posts {stop slot or -1, children up to it} per direction, and every
    // wave combines the posts in wave order (the nearest stop wins) -- the same answers parent_walk gives
    static MTR_DI void parent_part(const D& L, int x, int xf0, int level, int S, int w, int W, int& ps, int& pe,
                                   int& cnt) {
        const int ln = lane_id();
        const lptr<int> b = tbox(L);
        int c = 0;
        bool bdone = false, fdone = false;
        ps = 0;
        pe = S;
        for (int t = 0; !bdone || !fdone; t++) {
            const int bb = x - (t * W + w) * 64 * GK, fb = xf0 + (t * W + w) * 64 * GK;
            uint32_t mb[GK], mf[GK];
#pragma unroll
            for (int q = 0; q < GK; q++) {
                mb[q] = L.meta[max(bb - 64 * q - ln, 0)];
                mf[q] = L.meta[max(min(fb + 64 * q + ln, S - 1), 0)];
            }
            int bs = -1, bc = 0, fs = -1, fc = 0;
            if (!bdone) {
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = bb - 64 * q - ln;
                    const bool child = bnd_of(mb[q]) >= level - 1;
                    const uint64_t stop = __ballot((i <= 0) | (bnd_of(mb[q]) >= level));
                    if (stop) {
                        const int k = first_lane(stop);
                        bs = max(0, bb - 64 * q - k);
                        bc += __popcll(__ballot(child) & ((uint64_t(2) << k) - 1));
                        break;
                    }
                    bc += __popcll(__ballot(child));
                }
            }
            if (!fdone) {
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = fb + 64 * q + ln;
                    const uint64_t stop = __ballot((i >= S) | (bnd_of(mf[q]) >= level));
                    const uint64_t ch = __ballot((i < S) & (bnd_of(mf[q]) >= level - 1));
                    if (stop) {
                        const int k = first_lane(stop);
                        fs = fb + 64 * q + k;
                        fc += __popcll(ch & ((uint64_t(1) << k) - 1));
                        break;
                    }
                    fc += __popcll(ch);
                }
            }
            // (rows alternate by step parity: a wave posts step t + 1 while another may still read step t)
            const lptr<int> row = b + 16 + 4 * W * (t & 1);
            if (ln == 0) {
                row[4 * w] = bs;
                row[4 * w + 1] = bc;
                row[4 * w + 2] = fs;
                row[4 * w + 3] = fc;
            }
            __syncthreads();
            for (int u = 0; u < W; u++) {
                if (!bdone) {
                    const int s0 = uni(row[4 * u]);
                    c += uni(row[4 * u + 1]);
                    if (s0 >= 0) {
                        ps = s0;
                        bdone = true;
                    }
                }
            }
            for (int u = 0; u < W; u++) {
                if (!fdone) {
                    const int s0 = uni(row[4 * u + 2]);
                    c += uni(row[4 * u + 3]);
                    if (s0 >= 0) {
                        pe = s0;
                        fdone = true;
                    }
                }
            }
        }
        cnt = c;
    }
    static MTR_DI void parent_walk(const D& L, const St& s, int x, int level, int& ps, int& pe, int& cnt) {
        const int S = s.nseg, ln = lane_id();
        int c = 0;
        bool bdone = false, fdone = false;
        ps = 0;
        pe = S;
        for (int bb = x, fb = x + 1; !bdone || !fdone; bb -= 64 * GK, fb += 64 * GK) {
            uint32_t mb[GK], mf[GK];
#pragma unroll
            for (int q = 0; q < GK; q++) {
                mb[q] = L.meta[max(bb - 64 * q - ln, 0)];
                mf[q] = L.meta[max(min(fb + 64 * q + ln, S - 1), 0)];
            }
            if (!bdone) {
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = bb - 64 * q - ln;
                    const bool child = bnd_of(mb[q]) >= level - 1;
                    const uint64_t stop = __ballot((i <= 0) | (bnd_of(mb[q]) >= level));
                    if (stop) {  // slots bb - 64 q down to the block's start (lanes 0 .. k)
                        const int k = first_lane(stop);
                        ps = max(0, bb - 64 * q - k);
                        c += __popcll(__ballot(child) & ((uint64_t(2) << k) - 1));
                        bdone = true;
                        break;
                    }
                    c += __popcll(__ballot(child));
                }
            }
            if (!fdone) {
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = fb + 64 * q + ln;
                    const uint64_t stop = __ballot((i >= S) | (bnd_of(mf[q]) >= level));
                    const uint64_t ch = __ballot((i < S) & (bnd_of(mf[q]) >= level - 1));
                    if (stop) {  // slots fb + 64 q up to the block's end (lanes below k)
                        const int k = first_lane(stop);
                        pe = fb + 64 * q + k;
                        c += __popcll(ch & ((uint64_t(1) << k) - 1));
                        fdone = true;
                        break;
                    }
                    c += __popcll(ch);
                }
            }
        }
        cnt = c;
    }
    // number of leaves in [bs, be) with bnd >= minb
    static MTR_DI int count_bnd(const D& L, int bs, int be, int minb) {
        int c = 0;
        if constexpr (G) {
            for (int base = bs; base < be; base += 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[min(base + 64 * q + lane_id(), be - 1)];
#pragma unroll
                for (int q = 0; q < GK; q++)
                    c += __popcll(__ballot((base + 64 * q + lane_id() < be) & (bnd_of(mq[q]) >= minb)));
            }
            return c;
        }
        for (int base = bs; base < be; base += 64) {
            const int i = base + lane_id();
            const uint32_t mi = L.meta[min(i, be - 1)];
            c += __popcll(__ballot((i < be) & (bnd_of(mi) >= minb)));
        }
        return c;
    }
    // index of the n-th (0-based) leaf in [bs, be) with bnd >= minb, -1 if none
    static MTR_DI int nth_bnd(const D& L, int bs, int be, int minb, int n) {
        if constexpr (G) {  // HBM: GK rounds of loads in flight per step
            for (int base = bs; base < be; base += 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[min(base + 64 * q + lane_id(), be - 1)];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const bool t = (base + 64 * q + lane_id() < be) & (bnd_of(mq[q]) >= minb);
                    const uint64_t m = __ballot(t);
                    const int pc = __popcll(m);
                    if (n < pc) return base + 64 * q + first_lane(__ballot(t && __popcll(m & lanes_below()) == n));
                    n -= pc;
                }
            }
            return -1;
        }
        for (int base = bs; base < be; base += 64) {
            const int i = base + lane_id();
            const uint32_t mi = L.meta[min(i, be - 1)];
            const bool t = (i < be) & (bnd_of(mi) >= minb);
            const uint64_t m = __ballot(t);
            const int pc = __popcll(m);
            if (n < pc) return base + first_lane(__ballot(t && __popcll(m & lanes_below()) == n));
            n -= pc;
        }
        return -1;
    }

    // leaves of [bs, be) that are not hole slots; the index of the n-th (0-based) of them
    static MTR_DI int count_live(const D& L, int bs, int be) {
        int c = 0;
        if constexpr (G) {
            for (int base = bs; base < be; base += 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[min(base + 64 * q + lane_id(), be - 1)];
#pragma unroll
                for (int q = 0; q < GK; q++) c += __popcll(__ballot((base + 64 * q + lane_id() < be) & !(mq[q] & M_DEL)));
            }
            return c;
        }
        for (int base = bs; base < be; base += 64) {
            const int i = base + lane_id();
            c += __popcll(__ballot((i < be) & !(L.meta[min(i, be - 1)] & M_DEL)));
        }
        return c;
    }
    static MTR_DI int nth_live(const D& L, int bs, int be, int n) {
        if constexpr (G) {  // HBM: GK rounds of loads in flight per step
            for (int base = bs; base < be; base += 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[min(base + 64 * q + lane_id(), be - 1)];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const bool t = (base + 64 * q + lane_id() < be) & !(mq[q] & M_DEL);
                    const uint64_t m = __ballot(t);
                    const int pc = __popcll(m);
                    if (n < pc) return base + 64 * q + first_lane(__ballot(t && __popcll(m & lanes_below()) == n));
                    n -= pc;
                }
            }
            return -1;
        }
        for (int base = bs; base < be; base += 64) {
            const int i = base + lane_id();
            const bool t = (i < be) & !(L.meta[min(i, be - 1)] & M_DEL);
            const uint64_t m = __ballot(t);
            const int pc = __popcll(m);
            if (n < pc) return base + first_lane(__ballot(t && __popcll(m & lanes_below()) == n));
            n -= pc;
        }
        return -1;
    }

    // [bs, be) = the leaf block holding leaf x, from one ballot over leaves x-31 .. x+32 (leaf
    // blocks hold at most 7 leaves); the loops above take over only if a bound lies outside
    // (live: the block's slots that are not holes, when both bounds came from this one ballot; else -1)
    static MTR_DI void block_bounds1(const D& L, const St& s, int x, int& bs, int& be) {
        int live;
        block_bounds1_live(L, s, x, bs, be, live);
    }
    static MTR_DI void block_bounds1_live(const D& L, const St& s, int x, int& bs, int& be, int& live) {
        const int S = s.nseg;
        const int ln = lane_id();
        const int i = x - 31 + ln;
        const bool in = (i >= 0) & (i < S);
        const uint32_t mi = L.meta[in ? i : 0];
        const bool b = in & (bnd_of(mi) >= 1);
        const uint64_t sm = __ballot((i <= 0) | b) & LO32;
        const uint64_t em = __ballot((i >= S) | b) & HI32;
        bs = sm ? max(0, x - 31 + last_lane(sm)) : block_start(L, x - 32, 1);
        be = em ? x - 31 + first_lane(em) : block_end(L, s, x + 32, 1);
        live = (sm && em) ? __popcll(__ballot(in & (i >= bs) & (i < be) & !(mi & M_DEL))) : -1;
    }

    // Block overflow after a leaf was added next to x (insertingWalk split + updateRoot,
    // mergeTree.ts:1831-1871, 1268-1277).  [hbs, hbe) = x's leaf block when the caller knows it.
    // Returns the start of x's leaf block afterwards.
    static MTR_DI int overflow_fix(D& L, St& s, int x, int hbs = -1, int hbe = -1) {
        PROF(P_OVERFLOW);
        int level = 1;
        int bs = hbs, be = hbe, cnt = -1;
        {
#ifdef MTR_PROF
            ProfScope _prof_ovb(L.sc, P_OVB);
#endif
            if (bs < 0) block_bounds1_live(L, s, x, bs, be, cnt);
            if (!(G && s.holes)) cnt = be - bs;
            else if (cnt < 0) cnt = count_live(L, bs, be);  // (holes are no children)
#ifdef MTR_PROF
            if (cnt < 0 || hbs < 0) PROF_COUNT(P_NOVFB);
#endif
        }
        int xbs = bs;
        while (cnt >= kMaxNodesInBlock) {
            PROF_COUNT(P_NOVL);
            int c5 = bs + kMaxNodesInBlock / 2;
            if (G && s.holes && level == 1) c5 = nth_live(L, bs, be, kMaxNodesInBlock / 2);
            if (level == 1 && x >= c5) xbs = c5;
            if (level > 1) c5 = nth_bnd(L, bs, be, level - 1, kMaxNodesInBlock / 2);
            uint32_t m = set_bnd(uniu(L.meta[c5]), level);
            if (level == 1) m = set_ns(m, NS_UNDEF);
            L.meta[c5] = m;
            wsync();
            if (level == s.height) {  // root split
                s.height++;
                L.meta[0] = set_bnd(uniu(L.meta[0]), s.height);
                wsync();
                break;
            }
            level++;
            if constexpr (G) {
                int nbs, nbe;
#ifdef MTR_PROF
                ProfScope _prof_ovpb(L.sc, P_OVPB);
#endif
                parent_block(L, s, bs, level, nbs, nbe, cnt);
                bs = nbs;
                be = nbe;
            } else {
                bs = block_start(L, bs, level);
                be = block_end(L, s, bs, level);
                cnt = count_bnd(L, bs, be, level - 1);
            }
        }
        return xbs;
    }

    // ---- LRU heap (collections/heap.ts:11-67), 1-based, hole-based sifts (same order as swaps)
    static MTR_DI void heap_push(D& L, St& s, uint32_t u, int sq) {
        if (s.heapn + 1 >= L.lhcap) {
            s.status = MTR_ERR_CAPACITY;
            return;
        }
        int k = ++s.heapn;
        while (k > 1) {
            const int ps = uni(L.hseq[k >> 1]);
            const uint32_t pu = uniu(L.huid[k >> 1]);  // loaded with the seq: one round per level
            if (!(ps - sq > 0)) break;
            L.hseq[k] = ps;
            L.huid[k] = pu;
            k >>= 1;
        }
        L.hseq[k] = sq;
        L.huid[k] = u;
        wsync();
        if (k == 1) s.htop = sq;
        {
            const int mh = L.sc->max_heap;  // (every lane: the same value to the same word)
            L.sc->max_heap = max(mh, s.heapn);
        }
    }
    static MTR_DI uint32_t heap_pop(D& L, St& s) {
        PROF(P_HEAP);
        const uint32_t x = uniu(L.huid[1]);
        int n = s.heapn;
        const int ls = uni(L.hseq[n]);
        const uint32_t lu = uniu(L.huid[n]);
        n--;
        s.heapn = n;
        int k = 1;
        s.htop = ls;
        while ((k << 1) <= n) {
            // both children's (seq, uid) in one round of loads (slot n + 1 may be stale: unused)
            int j = k << 1;
            int sj = uni(L.hseq[j]);
            const int sj1 = uni(L.hseq[j + 1]);
            uint32_t uj = uniu(L.huid[j]);
            const uint32_t uj1 = uniu(L.huid[j + 1]);
            if (j < n && sj - sj1 > 0) {
                j++;
                sj = sj1;
                uj = uj1;
            }
            if (ls - sj <= 0) break;
            if (k == 1) s.htop = sj;
            L.hseq[k] = sj;
            L.huid[k] = uj;
            k = j;
        }
        L.hseq[k] = ls;
        L.huid[k] = lu;
        wsync();
        return x;
    }

    // addToLRUSet, mergeTree.ts:741-751, for a leaf whose leaf-block starts at bs
    static MTR_DI void add_lru_block(D& L, St& s, int bs, uint32_t u, int sq) {
        const uint32_t m = uniu(L.meta[bs]);
        if (ns_of(m) != NS_TRUE && sq > s.curseq) {
            L.meta[bs] = set_ns(m, NS_TRUE);
            wsync();
            heap_push(L, s, u, sq);
        }
    }

    // ---- the local-op path (X instantiations only)
    // head of leaf uid's pending-cell list (0xffffff = none); lane-parallel like rm_get / rm_set
    static MTR_DI uint32_t pd_get(const D& L, uint32_t uid) { return rm_get(L, PEND_KEY | uid); }
    static MTR_DI bool pd_set(const D& L, uint32_t uid, uint32_t head) { return rm_set(L, PEND_KEY | uid, head); }

    // addToPendingList (mergeTree.ts:1324-1357) for leaf i (wave-uniform): a new SegmentGroup at the ring's
    // tail when `slot` < 0, then the leaf joins it (segmentGroups.enqueue) with the group's next ordinal
    static MTR_DI int pend_add(D& L, const KParams& P, St& s, int i, int slot, int kind, uint32_t pp, int lseq,
                               uint32_t oldp = NONE32) {
        const gptr<DocHdr> h = L.ghdr();
        const gptr<uint32_t> ring = L.gpend();
        if (!ring) {
            s.status = MTR_ERR_CAPACITY;
            return -1;
        }
        if (slot < 0) {
            const int head = uni(h->phead), tail = uni(h->ptail);
            if (tail - head >= kPendRing) {
                s.status = MTR_ERR_CAPACITY;
                return -1;
            }
            slot = tail % kPendRing;
            if (lane_id() == 0) {
                ring[4 * slot] = uint32_t(lseq);
                ring[4 * slot + 1] = 0;
                ring[4 * slot + 2] = uint32_t(kind);
                ring[4 * slot + 3] = pp;
                h->ptail = tail + 1;
            }
            wsync();
        }
        const int ord = int(uniu(ring[4 * slot + 1]));
        const int fr = uni(h->pfree);  // a cell an ack or a rollback freed, else a new one
        if ((!fr && s.rmused + 3 > P.rcap) || ord > 0xffff) {
            s.status = MTR_ERR_CAPACITY;
            return slot;
        }
        const uint32_t u = uniu(L.uid[i]);
        const uint32_t m = uniu(L.meta[i]);
        const uint32_t c = fr ? uint32_t(fr - 1) : uint32_t(s.rmused);
        if (fr) {
            const uint32_t nf = uniu(L.grm()[c]) & 0xffffffu;
            if (lane_id() == 0) h->pfree = nf == 0xffffffu ? 0 : int(nf + 1);
        }
        bool ok = true;
        if (lane_id() == 0) {
            const uint32_t nxt = (m & (M_PEND | M_ZOMB)) ? pd_get(L, u) : 0xffffffu;
            L.grm()[c] = (nxt & 0xffffffu) | (uint32_t(kind) << 24);
            L.grm()[c + 1] = (uint32_t(slot) << 16) | uint32_t(ord);
            L.grm()[c + 2] = oldp;  // a local annotate's previousProps (the set before the op)
            ring[4 * slot + 1] = uint32_t(ord + 1);
            ok = pd_set(L, u, c);
            L.meta[i] = m | M_PEND;
        }
        if (__ballot(!ok)) s.status = MTR_ERR_CAPACITY;
        if (!fr) s.rmused += 3;
        wsync();
        return slot;
    }

    // unlink the cell of ring slot `slot` from leaf i's membership list and put it on the free list
    // (wave-uniform); returns the cell's previousProps word; clears M_PEND when no cell is left
    static MTR_DI uint32_t pend_drop(D& L, int i, int slot) {
        const gptr<DocHdr> h = L.ghdr();
        const uint32_t u = uniu(L.uid[i]);
        uint32_t c = uniu(pd_get(L, u)), prev = 0xffffffu, oldp = NONE32;
        int left = 0;
        while (c != 0xffffffu) {
            const uint32_t w0 = uniu(L.grm()[c]), w1 = uniu(L.grm()[c + 1]);
            const uint32_t nx = w0 & 0xffffffu;
            if (int(w1 >> 16) == slot) {
                oldp = uniu(L.grm()[c + 2]);
                const int fr = uni(h->pfree);
                if (lane_id() == 0) {
                    if (prev == 0xffffffu) pd_set(L, u, nx);
                    else L.grm()[prev] = (L.grm()[prev] & 0xff000000u) | nx;
                    L.grm()[c] = fr ? uint32_t(fr - 1) : 0xffffffu;  // push on the free list
                    h->pfree = int(c + 1);
                }
            } else {
                prev = c;
                left += int(w1 >> 16) != int(ZOMBIE_SLOT);
            }
            wsync();
            c = nx;
        }
        if (!left && lane_id() == 0) L.meta[i] = L.meta[i] & ~M_PEND;
        wsync();
        return oldp;
    }

    // the leaves a local remove / annotate touched (marked M_TOUCH by range_walk), in leaf (= walk)
    // order, join one new group (none when no leaf was touched: no group is created)
    static MTR_DI void pend_touched(D& L, const KParams& P, St& s, int kind, uint32_t pp, int lseq) {
        int slot = -1;
        for (int base = 0; base < s.nseg && s.status == MTR_OK; base += 64) {
            const int i = base + lane_id();
            const uint32_t m = L.meta[min(i, s.nseg - 1)];
            const bool t = i < s.nseg && (m & M_TOUCH);
            uint64_t tm = __ballot(t);
            if (t) L.meta[i] = m & ~M_TOUCH;
            wsync();
            for (; tm && s.status == MTR_OK; tm &= tm - 1)
                slot = pend_add(L, P, s, base + first_lane(tm), slot, kind, pp, lseq);
        }
    }

    // splitAt's segmentGroups.copyTo (segmentGroupCollection.ts:47-62): the right half r (a copy of the
    // left half's meta, M_PEND included) joins every group of the left half, each with its next ordinal
    static MTR_DI void pend_copy(D& L, const KParams& P, St& s, uint32_t left_uid, int r) {
        uint32_t c = uniu(lane_id() == 0 ? pd_get(L, left_uid) : 0u);
        c = uniu(c);
        if (lane_id() == 0) L.meta[r] = L.meta[r] & ~(M_PEND | M_ZOMB);
        wsync();
        while (c != 0xffffffu && s.status == MTR_OK) {
            const uint32_t w0 = uniu(L.grm()[c]), w1 = uniu(L.grm()[c + 1]), w2 = uniu(L.grm()[c + 2]);
            if ((w1 >> 16) == ZOMBIE_SLOT) zomb_add(L, P, s, r, w2, int(w0 >> 24) & PK_REWRITE);  // copyTo's counts
            else pend_add(L, P, s, r, int(w1 >> 16), int(w0 >> 24), 0, 0, w2);  // (previousProps duplicated)
            c = w0 & 0xffffffu;
        }
    }
    // a key cell for leaf i (wave-uniform): the pending key counts of annotate prop-op pp outlive its group
    // (pendingKeyUpdateCount, segmentPropertiesManager.ts:25, when resetPendingDeltaToOps does not re-send
    // the annotate to a segment removed meanwhile, client.ts:741-755)
    static MTR_DI void zomb_add(D& L, const KParams& P, St& s, int i, uint32_t pp, int rw = 0) {
        const gptr<DocHdr> h = L.ghdr();
        const int fr = uni(h->pfree);
        if (!fr && s.rmused + 3 > P.rcap) {
            s.status = MTR_ERR_CAPACITY;
            return;
        }
        const uint32_t u = uniu(L.uid[i]);
        const uint32_t m = uniu(L.meta[i]);
        const uint32_t c = fr ? uint32_t(fr - 1) : uint32_t(s.rmused);
        if (fr) {
            const uint32_t nf = uniu(L.grm()[c]) & 0xffffffu;
            if (lane_id() == 0) h->pfree = nf == 0xffffffu ? 0 : int(nf + 1);
        }
        bool ok = true;
        if (lane_id() == 0) {
            const uint32_t nxt = (m & (M_PEND | M_ZOMB)) ? pd_get(L, u) : 0xffffffu;
            L.grm()[c] = (nxt & 0xffffffu) | (uint32_t(PK_ANNOTATE | rw) << 24);
            L.grm()[c + 1] = ZOMBIE_SLOT << 16;
            L.grm()[c + 2] = pp;
            ok = pd_set(L, u, c);
            L.meta[i] = m | M_ZOMB;
        }
        if (__ballot(!ok)) s.status = MTR_ERR_CAPACITY;
        if (!fr) s.rmused += 3;
        wsync();
    }

    // one of a leaf's pending annotates holds `key` (PropertiesManager.pendingKeyUpdateCount[key] defined); a
    // rewrite's null keys are not counted (segmentPropertiesManager.ts:127-131)
    static MTR_DI bool key_pending(const D& L, uint32_t c, uint32_t key) {
        const gptr<const uint32_t> poff = L.tab(CP_POFF), pkv = L.tab(CP_PKV);
        const gptr<uint32_t> ring = L.gpend();
        while (c != 0xffffffu) {
            const uint32_t w0 = L.grm()[c], w1 = L.grm()[c + 1];
            if (((w0 >> 24) & PK_KIND) == PK_ANNOTATE) {
                const bool rw = ((w0 >> 24) & PK_REWRITE) != 0;
                const uint32_t pp = (w1 >> 16) == ZOMBIE_SLOT ? L.grm()[c + 2] : ring[4 * (w1 >> 16) + 3];
                for (uint32_t q = poff[pp]; q < poff[pp + 1]; q++)
                    if (pkv[2 * q] == key && !(rw && pkv[2 * q + 1] == MTR_NULL_VALUE)) return true;
            }
            c = w0 & 0xffffffu;
        }
        return false;
    }
    // a pending local rewrite on the leaf (pendingRewriteCount > 0): remote annotates leave it alone
    static MTR_DI bool rewrite_pending(const D& L, uint32_t c) {
        while (c != 0xffffffu) {
            const uint32_t w0 = L.grm()[c];
            if ((w0 >> 24) == uint32_t(PK_ANNOTATE | PK_REWRITE)) return true;
            c = w0 & 0xffffffu;
        }
        return false;
    }

    // ---- local references (X instantiations, documents with references only)
    // A per-document table of refcap entries, ids by creation (DocHdr.nrefs, kept in Sc during a launch):
    // {uid of the reference's segment (NONE32: none -- a detached reference), offset, ReferenceType | RF_HELD}.
    // RF_HELD: the segment's LocalReferenceCollection holds it (has(), localReference.ts:357-384).  Keyed by
    // uid, a reference follows its leaf through shifts, compactions, spreads and normalization; splits
    // (ref_split), scour's appends (ref_append) and acked removals (ref_slide) move it as the collection does.
    static constexpr uint32_t RF_HELD = 0x80000000u;
    static constexpr uint32_t RT_SLIDE = MTR_REFTYPE_SLIDE_ON_REMOVE, RT_STAY = MTR_REFTYPE_STAY_ON_REMOVE,
                              RT_TRANSIENT = MTR_REFTYPE_TRANSIENT;
    static MTR_DI int nrefs(const D& L) { return uni(L.sc->nrefs); }
    static MTR_DI gptr<uint32_t> rf_uid(const D& L) { return (gptr<uint32_t>)L.cold(CP_REFS); }
    static MTR_DI gptr<uint32_t> rf_off(const D& L) { return rf_uid(L) + uni(L.sc->refcap); }
    static MTR_DI gptr<uint32_t> rf_ty(const D& L) { return rf_uid(L) + 2 * uni(L.sc->refcap); }
    static MTR_DI bool removed_acked(int rs) { return rs != RNONE && rs < LOCAL_BASE; }

    // LocalReferenceCollection.split (localReference.ts:398-420): the references held at offsets >= off of the
    // leaf with uid ul go to the split-off leaf ur, at offset - off
    static MTR_DI void ref_split(const D& L, uint32_t ul, int off, uint32_t ur) {
        const int n = nrefs(L);
        const gptr<uint32_t> U = rf_uid(L), O = rf_off(L), T = rf_ty(L);
        for (int b = 0; b < n; b += 64) {
            const int r = b + lane_id();
            const int rc = min(r, n - 1);
            const uint32_t u = U[rc], o = O[rc], t = T[rc];
            if (r < n && u == ul && (t & RF_HELD) && int(o) >= off) {
                U[r] = ur;
                O[r] = o - uint32_t(off);
            }
        }
        wsync();
    }
    // LocalReferenceCollection.append (localReference.ts:143-158, 332-350): the references held by the leaf with
    // uid um go to the chain head uh, behind its `shift` units (its refsByOffset before the append)
    static MTR_DI void ref_append(const D& L, uint32_t um, uint32_t uh, int shift) {
        const int n = nrefs(L);
        const gptr<uint32_t> U = rf_uid(L), O = rf_off(L), T = rf_ty(L);
        for (int b = 0; b < n; b += 64) {
            const int r = b + lane_id();
            const int rc = min(r, n - 1);
            const uint32_t u = U[rc], o = O[rc], t = T[rc];
            if (r < n && u == um && (t & RF_HELD)) {
                U[r] = uh;
                O[r] = o + uint32_t(shift);
            }
        }
        wsync();
    }
    // _getSlideToSegment's leaf predicate (mergeTree.ts:827-832): acked (seq is not UnassignedSequenceNumber) and
    // not removed-and-acked; hole slots are no leaves
    static MTR_DI bool slide_ok(uint32_t m, int sq, int rs) {
        return !(m & M_DEL) && sq < LOCAL_BASE && !removed_acked(rs);
    }
    // MergeTree._getSlideToSegment (mergeTree.ts:821-840) of leaf x: the first such leaf after it
    // (forwardExcursion), else the last before it (backwardExcursion); -1 if none
    static MTR_DI int slide_target(const D& L, const St& s, int x) {
        const int S = s.nseg;
        for (int base = x + 1; base < S; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, S - 1);
            const uint64_t m = __ballot((i < S) & slide_ok(L.meta[ic], L.seq[ic], L.rseq[ic]));
            if (m) return base + first_lane(m);
        }
        for (int top = x - 1; top >= 0; top -= 64) {
            const int i = top - lane_id();
            const int ic = max(i, 0);
            const uint64_t m = __ballot((i >= 0) & slide_ok(L.meta[ic], L.seq[ic], L.rseq[ic]));
            if (m) return top - first_lane(m);
        }
        return -1;
    }
    // MergeTree.slideAckedRemovedSegmentReferences (mergeTree.ts:849-884) of leaf x, removed and acked
    // (wave-uniform): held SlideOnRemove references go to the slide-to leaf -- offset 0 when it follows x
    // (addBeforeTombstones), its last unit when it precedes x (addAfterTombstones, localReference.ts:426-490);
    // other held references leave the collection (and their segment, when there is a slide-to leaf);
    // StayOnRemove references stay
    static MTR_DI void ref_slide(const D& L, const St& s, int x) {
        const int n = nrefs(L);
        if (!n) return;
        const gptr<uint32_t> U = rf_uid(L), O = rf_off(L), T = rf_ty(L);
        const uint32_t ux = uniu(L.uid[x]);
        bool any = false;
        for (int b = 0; b < n; b += 64) {
            const int r = b + lane_id();
            const int rc = min(r, n - 1);
            const uint32_t t = T[rc];
            any = any || ((r < n) & (U[rc] == ux) & ((t & RF_HELD) != 0) & !(t & RT_STAY));
        }
        if (!__ballot(any)) return;
        const int tg = slide_target(L, s, x);
        const uint32_t ut = tg >= 0 ? uniu(L.uid[tg]) : NONE32;
        const uint32_t toff = (tg >= 0 && tg < x) ? uint32_t(uni(L.len[tg]) - 1) : 0u;
        for (int b = 0; b < n; b += 64) {
            const int r = b + lane_id();
            const int rc = min(r, n - 1);
            const uint32_t u = U[rc], t = T[rc];
            if ((r < n) & (u == ux) & ((t & RF_HELD) != 0) & !(t & RT_STAY)) {
                if (tg < 0) {
                    T[r] = t & ~RF_HELD;  // removeLocalRef: the reference keeps its (removed) segment
                } else if (t & RT_SLIDE) {
                    U[r] = ut;
                    O[r] = toff;
                } else {  // lref.link(undefined, 0, undefined)
                    U[r] = NONE32;
                    O[r] = 0;
                    T[r] = t & ~RF_HELD;
                }
            }
        }
        wsync();
    }
    // createPositionReference (sequence/src/intervalCollection.ts:697-724): getContainingSegment(pos1) at the
    // record's view (client.ts:1065-1078), getSlideToSegment (client.ts:1085-1099), then
    // createLocalReferencePosition (mergeTree.ts:2209-2226, localReference.ts:260-298) -- a detached reference
    // when no segment holds the position
    static MTR_DI void ref_create(D& L, const KParams& P, St& s, const mtr_op& op) {
        const int n = nrefs(L);
        int id = n;  // numbered by creation, or (MTR_REF_SLOT) a slot the host recycles
        if (op.payload2 & MTR_REF_SLOT) {
            id = op.pos2;
            if (id < 0 || id > n || (id < n && rf_uid(L) && (uniu(rf_ty(L)[id]) & RF_HELD))) {
                s.status = MTR_ERR_BAD_OP;  // (a slot some segment's collection still holds)
                return;
            }
        }
        if (!rf_uid(L) || id >= uni(L.sc->refcap)) {
            s.status = MTR_ERR_CAPACITY;
            return;
        }
        const uint32_t ty = op.payload;
        if (int((ty & RT_SLIDE) != 0) + int((ty & RT_STAY) != 0) + int((ty & RT_TRANSIENT) != 0) > 1) {
            s.status = MTR_ERR_BAD_OP;  // _validateReferenceType's UsageError (localReference.ts:23-39)
            return;
        }
        View v;
        if (op.payload2 & MTR_REF_LOCALVIEW) {
            v.ref = s.curseq;
            v.client = s.collab ? uint32_t(s.local) : CL_LOCAL;
            v.local = 1;
        } else {
            v.ref = op.ref_seq;
            v.client = enc_client(int(int16_t(op.client)));
            v.local = (!s.collab || uint32_t(s.local) == v.client) ? 1 : 0;
        }
        int i = 0, before = 0;
        if (op.payload2 & MTR_REF_LSEQ) find1_at(L, s, op.ref_seq, op.min_seq, op.pos1, i, before);
        else find1(L, s, v, op.pos1, i, before, P.new_length_calc);
        int off = op.pos1 - before;
        if (i >= s.nseg || op.pos1 < 0) i = -1;
        if (i >= 0 && (op.payload2 & MTR_REF_SLIDE) && removed_acked(uni(L.rseq[i]))) {
            const int tg = slide_target(L, s, i);
            off = (tg >= 0 && tg < i) ? uni(L.len[tg]) - 1 : 0;
            i = tg;
        }
        uint32_t u = NONE32, tw = ty;
        if (i >= 0) {
            if (removed_acked(uni(L.rseq[i])) && !(ty & (RT_SLIDE | RT_TRANSIENT))) {
                s.status = MTR_ERR_BAD_OP;  // "Can only create SlideOnRemove or Transient ... on a removed segment"
                return;
            }
            u = uniu(L.uid[i]);
            if (!(ty & RT_TRANSIENT)) {
                if (off >= uni(L.len[i])) {
                    s.status = MTR_ERR_ASSERT | 0x348;  // "offset cannot be beyond segment length"
                    return;
                }
                tw |= RF_HELD;
            }
        }
        if (lane_id() == 0) {
            rf_uid(L)[id] = u;
            rf_off(L)[id] = uint32_t(off);
            rf_ty(L)[id] = tw;
            if (id == n) L.sc->nrefs = n + 1;
        }
        wsync();
    }
    // MergeTree.removeLocalReferencePosition (mergeTree.ts:2190-2207) of reference r
    static MTR_DI void ref_remove(D& L, St& s, uint32_t r) {
        if (!rf_uid(L) || int(r) >= nrefs(L)) {
            s.status = MTR_ERR_BAD_OP;
            return;
        }
        if (lane_id() == 0) rf_ty(L)[r] = rf_ty(L)[r] & ~RF_HELD;
        wsync();
    }
    // after a remove walk that was no pending local op: every leaf this op removed first, or whose pending local
    // remove it overtook, is now removed and acked (removedSeq = this seq) and slides its references
    // (mergeTree.ts:2023-2040).  Leaves an earlier member of the same GROUP removed hold only StayOnRemove
    // references by now, so sliding them again changes nothing.
    static MTR_DI void ref_slide_walk(const D& L, const St& s, int seq) {
        for (int base = L.wlo; base < L.whi; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, L.whi - 1);
            for (uint64_t m = __ballot((i < L.whi) & (L.rseq[ic] == seq)); m; m &= m - 1)
                ref_slide(L, s, base + first_lane(m));
        }
    }

    // ---- an interval collection's own ops (sequence/src/intervalCollection.ts)
    // localRemovedSeq of a leaf whose pending local remove a remote remove overtook (removedSeq is the remote one's):
    // the localSeq of its pending-remove membership cell; -1 = none (per lane, rare)
    static MTR_DI int pend_lrs(const D& L, uint32_t u) {
        const gptr<uint32_t> ring = L.gpend();
        if (!ring) return -1;
        for (uint32_t c = pd_get(L, u); c != 0xffffffu;) {
            const uint32_t w0 = L.grm()[c], w1 = L.grm()[c + 1];
            const uint32_t sl = w1 >> 16;
            if (((w0 >> 24) & PK_KIND) == PK_REMOVE && sl != ZOMBIE_SLOT) return int(ring[4 * sl]);
            c = w0 & 0xffffffu;
        }
        return -1;
    }
    // localNetLength(segment, refSeq, localSeq) (mergeTree.ts:636-662): this client's view at localSeq lseq -- an
    // acked leaf shows when seq <= ref and it is not removed-and-acked by ref; a pending local insert (seq =
    // LOCAL_BASE + localSeq) when its localSeq <= lseq; either hides once removed by a local op whose localSeq <= lseq
    static MTR_DI int lnl_at(const D& L, uint32_t m, int sq, int rs, int ln, uint32_t u, int ref, int lseq) {
        if (m & M_DEL) return 0;  // a hole slot
        int lrs = -1;
        if (rs != RNONE && rs >= LOCAL_BASE) lrs = rs - LOCAL_BASE;
        else if (rs != RNONE && (m & M_PEND)) lrs = pend_lrs(L, u);
        bool zero = sq < LOCAL_BASE ? (sq > ref || (rs != RNONE && rs < LOCAL_BASE && rs <= ref)) : sq - LOCAL_BASE > lseq;
        zero = zero || (lrs >= 0 && lrs <= lseq);
        return zero ? 0 : ln;
    }
    // getContainingSegment(pos, {ref, this client}, lseq) (mergeTree.ts:795-813 with nodeMap's localSeq lengths): the
    // first leaf whose inclusive prefix exceeds pos (S if none) and the view length before it
    static MTR_DI void find1_at(const D& L, const St& s, int ref, int lseq, int pos, int& i_out, int& before) {
        const int S = s.nseg;
        int c = 0;
        i_out = S;
        before = 0;
        for (int base = 0; base < S; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, S - 1);
            const int x = i < S ? lnl_at(L, L.meta[ic], L.seq[ic], L.rseq[ic], L.len[ic], L.uid[ic], ref, lseq) : 0;
            const int inc = wave_incl_scan(x);
            const uint64_t mm = __ballot((i < S) & (c + inc > pos));
            if (mm) {
                const int l = first_lane(mm);
                i_out = base + l;
                before = c + rdlane(inc - x, l);
                return;
            }
            c += rdlane(inc, 63);
        }
        before = c;
    }
    // getPosition(leaf t, ref, this client, lseq) (mergeTree.ts:768-785): findReconnectionPosition (client.ts:699-706)
    static MTR_DI int pos_at(const D& L, const St& s, int t, int ref, int lseq) {
        int c = 0;
        for (int base = 0; base < t; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, s.nseg - 1);
            const int x = i < t ? lnl_at(L, L.meta[ic], L.seq[ic], L.rseq[ic], L.len[ic], L.uid[ic], ref, lseq) : 0;
            c += rdlane(wave_incl_scan(x), 63);
        }
        return c;
    }
    // IntervalCollection.ackInterval (intervalCollection.ts:2054-2138) for one endpoint: a reference its segment
    // holds is re-created at getSlideToSegment's segment and offset when that differs (none: a detached reference,
    // createPositionReferenceFromSegoff with an op); its ReferenceType becomes SlideOnRemove (setSlideOnRemove)
    static MTR_DI void ref_ack(D& L, St& s, uint32_t r) {
        if (!rf_uid(L) || int(r) >= nrefs(L)) {
            s.status = MTR_ERR_BAD_OP;
            return;
        }
        const uint32_t u = uniu(rf_uid(L)[r]), t = uniu(rf_ty(L)[r]);
        uint32_t nu = u, no = uniu(rf_off(L)[r]), nt = (t & ~RT_STAY) | RT_SLIDE;
        if (u != NONE32 && (t & RF_HELD)) {
            const int x = find_uid(L, s, u);
            // (a segment zamboni unlinked: the excursions from it find nothing)
            const int tg = x < 0 ? -1 : (removed_acked(uni(L.rseq[x])) ? slide_target(L, s, x) : x);
            if (tg < 0) {
                nu = NONE32;
                no = 0;
                nt &= ~RF_HELD;
            } else if (tg != x) {
                nu = uniu(L.uid[tg]);
                no = tg < x ? uint32_t(uni(L.len[tg]) - 1) : 0u;
            }
        }
        if (lane_id() == 0) {
            rf_uid(L)[r] = nu;
            rf_off(L)[r] = no;
            rf_ty(L)[r] = nt;
        }
        wsync();
    }
    // IntervalCollection.rebasePositionWithSegmentSlide (intervalCollection.ts:1472-1505): the position an endpoint
    // created at op.pos1 in the view (op.ref_seq, this client, localSeq op.min_seq) has after a reconnect
    // With MTR_REBASE_NOSLIDE it is SharedMatrix.rebasePosition (matrix.ts:534-551): the same getContainingSegment,
    // then findReconnectionPosition(segment, localSeq) + offset with no slide; no segment = undefined (the
    // detached position), which the resubmit skips
    static MTR_DI void rebase_pos(D& L, St& s, const mtr_op& op, int gidx) {
        int i = 0, before = 0;
        const bool noslide = (op.payload2 & MTR_REBASE_NOSLIDE) != 0;
        find1_at(L, s, op.ref_seq, op.min_seq, op.pos1, i, before);
        if (op.pos1 < 0 || i >= s.nseg) {
            if (noslide) {
                if constexpr (DL) put_record(L, s, gidx, MTR_DETACHED_POSITION, 0, MTR_DELTA_REBASE);
                return;
            }
            s.status = MTR_ERR_ASSERT | 0x54e;  // "No segment found"
            return;
        }
        const int off = op.pos1 - before;
        int t = i, toff = off;
        if (noslide) {
            if constexpr (DL) put_record(L, s, gidx, pos_at(L, s, i, s.curseq, op.min_seq) + off, 0, MTR_DELTA_REBASE);
            return;
        }
        if (removed_acked(uni(L.rseq[i]))) {  // getSlideToSegment (client.ts:1085-1099)
            t = slide_target(L, s, i);
            toff = (t >= 0 && t < i) ? uni(L.len[t]) - 1 : 0;
        }
        int res = MTR_DETACHED_POSITION;
        if (t >= 0) {
            if (off < 0 || off >= uni(L.len[i])) {
                s.status = MTR_ERR_ASSERT | 0x54f;  // "Invalid offset"
                return;
            }
            res = pos_at(L, s, t, s.curseq, op.min_seq) + toff;
        }
        if constexpr (DL) put_record(L, s, gidx, res, 0, MTR_DELTA_REBASE);
    }

    // MergeTree.ackPendingSegment (mergeTree.ts:1283-1322) with BaseSegment.ack (mergeTreeNodes.ts:439-479)
    // for one member op of this client's sequenced message (type: its MergeTreeDeltaType)
    static MTR_DI void ack(D& L, St& s, int type, int seq) {
        const gptr<DocHdr> h = L.ghdr();
        const gptr<uint32_t> ring = L.gpend();
        const int head = uni(h->phead), tail = uni(h->ptail);
        if (head == tail || !ring) return;  // pendingSegments.shift() is undefined
        const int slot = head % kPendRing;
        const int cnt = int(uniu(ring[4 * slot + 1]));
        if (lane_id() == 0) h->phead = head + 1;
        // the group's members: E[ordinal] = leaf
        for (int base = 0; base < s.nseg; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, s.nseg - 1);
            const uint32_t m = L.meta[ic];
            if (i < s.nseg && (m & M_PEND)) {
                for (uint32_t c = pd_get(L, L.uid[i]); c != 0xffffffu; c = L.grm()[c] & 0xffffffu) {
                    const uint32_t w1 = L.grm()[c + 1];
                    if (int(w1 >> 16) == slot) L.E[int(w1 & 0xffffu)] = i;
                }
            }
        }
        wsync();
        for (int o = 0; o < cnt && s.status == MTR_OK; o++) {  // in group order: drop the cell, then ack
            const int i = uni(L.E[o]);
            pend_drop(L, i, slot);
            bool slid = false;
            if (type == MTR_OP_INSERT) {
                if (uni(L.seq[i]) < LOCAL_BASE) s.status = MTR_ERR_ASSERT | 0x045;  // seq already assigned
                else if (lane_id() == 0) L.seq[i] = seq;
            } else if (type == MTR_OP_REMOVE) {
                const int rs = uni(L.rseq[i]);
                if (rs == RNONE) s.status = MTR_ERR_ASSERT | 0x046;  // missing removal info
                else if (rs >= LOCAL_BASE && lane_id() == 0) L.rseq[i] = seq;
                slid = rs != RNONE && rs >= LOCAL_BASE;  // ack() is true: no overlapping remove
            } else if (type != MTR_OP_ANNOTATE) {
                s.status = MTR_ERR_BAD_OP;
            }
            wsync();
            if (slid) ref_slide(L, s, i);  // mergeTree.ts:1294-1296
            if (G) csum_update(L, s, i, i + 1);
            int bs, be;
            block_bounds1(L, s, i, bs, be);
            add_lru_block(L, s, bs, uniu(L.uid[i]), seq);  // mergeTree.ts:1299-1301
        }
    }

    // a copy of set `cur` with each key of prop-op pp set to its value in set `old`, or deleted where
    // `old` lacks it (annotate rollback: the op's previousProps, mergeTree.ts:2129-2152); out of line (rare)
    // rw: a rewrite's rollback (PropertiesRollback.Rewrite): its deltas are the old keys it deleted (old values,
    // old order), then its non-null keys (old value or null), applied as a plain annotate (segmentPropertiesManager.ts
    // :106-147; the pending counts go with the op's cells)
    static __device__ __attribute__((noinline)) uint32_t props_restore(const D& L, const KParams& P, St& s,
                                                                      uint32_t cur, uint32_t old, uint32_t pp,
                                                                      bool rw = false) {
        const gptr<uint32_t> gprop = L.gprop();
        const gptr<const uint32_t> poff = L.tab(CP_POFF), pkv = L.tab(CP_PKV), kix = L.tab(CP_KIX),
                                   veq = L.tab(CP_VEQ);
        cur = cur == NONE32 ? cur : (cur & PN_MASK);
        old = old == NONE32 ? old : (old & PN_MASK);
        const uint32_t n_cur = cur == NONE32 ? 0u : uniu(gprop[cur]);
        const uint32_t n_old = old == NONE32 ? 0u : uniu(gprop[old]);
        const uint32_t lo = uniu(poff[pp]), hi = uniu(poff[pp + 1]);
        const uint32_t need = 1 + 2 * (n_cur + (hi - lo) + n_old);
        if (uint32_t(s.propused) + need > uint32_t(P.pcap)) {
            s.status = MTR_ERR_CAPACITY;
            return cur;
        }
        const uint32_t dst = uint32_t(s.propused);
        const gptr<uint32_t> e = gprop + dst;
        uint32_t n = n_cur;
        for (uint32_t k = 0; k < 2 * n_cur; k++) e[1 + k] = uniu(gprop[cur + 1 + k]);
        // delta steps: (rw) the old keys whose new value is absent or falsy, then the op's keys
        const uint32_t n_del = rw ? n_old : 0u;
        for (uint32_t q = 0; q < n_del + (hi - lo); q++) {
            uint32_t key, val = MTR_NULL_VALUE;
            if (q < n_del) {
                key = uniu(gprop[old + 1 + 2 * q]);
                bool truthy = false;
                for (uint32_t j = lo; j < hi; j++)
                    if (uniu(pkv[2 * j]) == key) {
                        const uint32_t nv = uniu(pkv[2 * j + 1]);
                        truthy = nv != MTR_NULL_VALUE && !(uniu(veq[nv]) & MTR_VEQ_FALSY);
                        break;
                    }
                if (truthy) continue;
                val = uniu(gprop[old + 2 + 2 * q]);
            } else {
                key = uniu(pkv[2 * (lo + q - n_del)]);
                if (rw && uniu(pkv[2 * (lo + q - n_del) + 1]) == MTR_NULL_VALUE) continue;  // (the delete pass's)
                for (uint32_t k = 0; k < n_old; k++)
                    if (uniu(gprop[old + 1 + 2 * k]) == key) {
                        val = uniu(gprop[old + 2 + 2 * k]);
                        break;
                    }
            }
            int at = -1;
            for (uint32_t k = 0; k < n; k++)
                if (uniu(e[1 + 2 * k]) == key) {
                    at = int(k);
                    break;
                }
            if (val == MTR_NULL_VALUE) {
                if (at >= 0) {
                    for (uint32_t k = uint32_t(at); k + 1 < n; k++) {
                        e[1 + 2 * k] = uniu(e[1 + 2 * (k + 1)]);
                        e[2 + 2 * k] = uniu(e[2 + 2 * (k + 1)]);
                    }
                    n--;
                }
            } else if (at >= 0) {
                e[2 + 2 * at] = val;
            } else {  // a new key in JS own-key order
                const uint32_t ix = uniu(kix[key]);
                uint32_t pos = n;
                if (ix != MTR_NOT_INDEX) {
                    pos = 0;
                    while (pos < n && uniu(kix[uniu(e[1 + 2 * pos])]) != MTR_NOT_INDEX &&
                           uniu(kix[uniu(e[1 + 2 * pos])]) < ix)
                        pos++;
                    for (uint32_t k = n; k > pos; k--) {
                        e[1 + 2 * k] = uniu(e[1 + 2 * (k - 1)]);
                        e[2 + 2 * k] = uniu(e[2 + 2 * (k - 1)]);
                    }
                }
                e[1 + 2 * pos] = key;
                e[2 + 2 * pos] = val;
                n++;
            }
        }
        uint32_t never = 0;
        for (uint32_t k = 0; k < n; k++)
            if (uniu(veq[uniu(e[2 + 2 * k])]) & MTR_VEQ_NEVER) never = MTR_PROPS_NEVER;
        e[0] = n;
        s.propused += int(1 + 2 * n);
        wsync();
        return dst | never;
    }

    // MergeTree.rollback (mergeTree.ts:2049-2159): revert the newest pending local op (type: its
    // MergeTreeDeltaType; pp: its prop-op for an annotate).  The group leaves the ring's tail; each member
    // (in group order) drops its cell and is reverted: a remove is undone, an insert becomes a segment
    // removed at UniversalSequenceNumber by this client (markRangeRemoved, :2117-2131), an annotate's keys
    // get their previous values back
    static MTR_DI void rollback(D& L, const KParams& P, St& s, int type, uint32_t pp, uint32_t comb = 0) {
        const gptr<DocHdr> h = L.ghdr();
        const gptr<uint32_t> ring = L.gpend();
        const int head = uni(h->phead), tail = uni(h->ptail);
        if (head == tail || !ring) {  // "Rollback op doesn't match last edit"
            s.status = MTR_ERR_BAD_OP;
            return;
        }
        const int slot = (tail - 1) % kPendRing;
        const int cnt = int(uniu(ring[4 * slot + 1]));
        if (lane_id() == 0) h->ptail = tail - 1;
        for (int base = 0; base < s.nseg; base += 64) {  // E[ordinal] = member leaf
            const int i = base + lane_id();
            const uint32_t m = L.meta[min(i, s.nseg - 1)];
            if (i < s.nseg && (m & M_PEND)) {
                for (uint32_t c = pd_get(L, L.uid[i]); c != 0xffffffu; c = L.grm()[c] & 0xffffffu) {
                    const uint32_t w1 = L.grm()[c + 1];
                    if (int(w1 >> 16) == slot) L.E[int(w1 & 0xffffu)] = i;
                }
            }
        }
        wsync();
        for (int o = 0; o < cnt && s.status == MTR_OK; o++) {
            const int i = uni(L.E[o]);
            const uint32_t oldp = pend_drop(L, i, slot);  // segmentGroups.pop()
            uint32_t m = uniu(L.meta[i]);
            if (type == MTR_OP_REMOVE) {
                const int rs = uni(L.rseq[i]);
                if (rs == RNONE || rs < LOCAL_BASE || ((m >> M_FREM_SHIFT) & 0xffu) != uint32_t(s.local)) {
                    s.status = MTR_ERR_ASSERT | 0x39d;  // the removal is not (only) this client's pending one
                    break;
                }
                m &= ~((0xffu << M_FREM_SHIFT) | M_OVERLAP);
                if (lane_id() == 0) L.rseq[i] = RNONE;
            } else if (type == MTR_OP_INSERT) {
                const bool live = uni(L.rseq[i]) == RNONE;  // (a removed one is not walked again)
                if (live) m = (m & ~((0xffu << M_FREM_SHIFT) | M_OVERLAP)) | (uint32_t(s.local) << M_FREM_SHIFT);
                if (lane_id() == 0) {
                    L.seq[i] = 0;
                    if (live) L.rseq[i] = 0;
                }
            } else if (type == MTR_OP_ANNOTATE) {
                const uint32_t np = props_restore(L, P, s, uniu(pget(L, i)), oldp, pp, (comb & 7u) == MTR_COMB_REWRITE);
                if (lane_id() == 0) pset(L, i, np);
            } else {
                s.status = MTR_ERR_BAD_OP;
                break;
            }
            if (lane_id() == 0) L.meta[i] = m;
            wsync();
            if (G) csum_update(L, s, i, i + 1);
        }
    }

    // ---- reconnect: Client.regeneratePendingOp (client.ts:917-960); X + DL instantiations only
    struct LeafRec {
        int len, seq, rseq;
        uint32_t meta, text, props, uid;
    };
    static MTR_DI LeafRec leaf_ld(const D& L, int i) {
        return LeafRec{L.len[i], L.seq[i], L.rseq[i], L.meta[i], L.text[i], pget(L, i), L.uid[i]};
    }
    // a leaf's data into slot i; the slot keeps its tree-structure bits (leaf-block bounds, needsScour):
    // assignChild puts the segment at the (parent, index) place (mergeTree.ts:2303-2308)
    static MTR_DI void leaf_st(D& L, int i, const LeafRec& x) {
        constexpr uint32_t kPlace = M_BND_MASK | M_NS_MASK;
        L.len[i] = x.len;
        L.seq[i] = x.seq;
        L.rseq[i] = x.rseq;
        L.meta[i] = (x.meta & ~kPlace) | (L.meta[i] & kPlace);
        L.text[i] = x.text;
        pset(L, i, x.props);
        L.uid[i] = x.uid;
    }
    // normalizeAdjacentSegments (mergeTree.ts:2231-2331) on the run of leaves in slots [a, b) (holes
    // skipped): removed-and-acked segments slide past every local one (keeping their order), each locally
    // removed segment slides past the unacked inserts newer than its removal, and the run's leaves take
    // the run's slots in the new order.  Serial (lane 0): runs are short and reconnects rare.
    static __device__ __attribute__((noinline)) void normalize_run(D& L, const KParams& P, St& s, int a, int b) {
        int n = 0;
        for (int base = a; base < b; base += 64) {  // the run's slots -> E[0, n)
            const int i = base + lane_id();
            const bool in = i < b && !(L.meta[min(i, b - 1)] & M_DEL);
            const uint64_t m = __ballot(in);
            if (in) L.E[n + __popcll(m & lanes_below())] = i;
            n += __popcll(m);
        }
        wsync();
        if (s.rmused + n > P.rcap) {  // scratch for the order: the remover arena's free tail
            s.status = MTR_ERR_CAPACITY;
            return;
        }
        const gptr<uint32_t> T = L.grm() + s.rmused;
        if (lane_id() == 0) {
            auto acked = [&](int k) {
                const int rs = L.rseq[L.E[k]];
                return rs != RNONE && rs < LOCAL_BASE;
            };
            int last = -1;  // the last segment that is not removed-and-acked
            for (int k = n - 1; k >= 0 && last < 0; k--)
                if (!acked(k)) last = k;
            if (last >= 0) {
                // walking back from `last`: T[p, n) holds the other segments of (j, last] in their new order
                // (the acked ones have all moved behind `last`)
                int p = n;
                for (int j = last; j >= 0; j--) {
                    if (acked(j)) continue;
                    const int rs = L.rseq[L.E[j]];
                    int k = 0;
                    if (rs != RNONE) {  // a local removal: past unacked inserts with localSeq > localRemovedSeq
                        const int lr = rs - LOCAL_BASE;
                        while (p + k < n) {
                            const int sq = L.seq[L.E[int(T[p + k])]];
                            if (!(sq >= LOCAL_BASE && sq - LOCAL_BASE > lr)) break;
                            k++;
                        }
                    }
                    for (int q = 0; q < k; q++) T[p - 1 + q] = T[p + q];
                    T[p - 1 + k] = uint32_t(j);
                    p--;
                }
                int w = 0;
                for (int q = p; q < n; q++) T[w++] = T[q];
                for (int k = 0; k < n; k++)
                    if (acked(k)) T[w++] = uint32_t(k);
                // slot E[k] takes the leaf of slot E[T[k]]: cycle by cycle, one leaf in registers
                for (int k = 0; k < n; k++) {
                    if (T[k] & 0x80000000u) continue;
                    if (int(T[k]) == k) {
                        T[k] |= 0x80000000u;
                        continue;
                    }
                    const LeafRec tmp = leaf_ld(L, L.E[k]);
                    int cur = k;
                    for (;;) {
                        const int src = int(T[cur] & 0x7fffffffu);
                        T[cur] |= 0x80000000u;
                        if (src == k) {
                            leaf_st(L, L.E[cur], tmp);
                            break;
                        }
                        leaf_st(L, L.E[cur], leaf_ld(L, L.E[src]));
                        cur = src;
                    }
                }
            }
        }
        wsync();
        if (G) csum_update(L, s, a, b);
    }
    // normalizeSegmentsOnRebase (mergeTree.ts:2352-2381): runs of removed / unacked leaves that hold both an
    // unacked insert and an acked removal are normalized
    static __device__ __attribute__((noinline)) void normalize(D& L, const KParams& P, St& s) {
        const int S = s.nseg;
        int a = -1, end = 0, cnt = 0;
        bool loc = false, ack = false;
        for (int base = 0; base < S && s.status == MTR_OK; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, S - 1);
            const uint32_t m = L.meta[ic];
            const int sq = L.seq[ic], rs = L.rseq[ic];
            const bool leaf = i < S && !(m & M_DEL);
            const bool run = leaf && (rs != RNONE || sq >= LOCAL_BASE);
            const uint64_t rm = __ballot(run), bm = __ballot(leaf && !run);
            const uint64_t lm = __ballot(run && sq >= LOCAL_BASE), am = __ballot(run && rs != RNONE && rs < LOCAL_BASE);
            if (!rm) {  // no run leaf here: at most the open run ends
                if (bm && a >= 0) {
                    if (loc && ack && cnt > 1) normalize_run(L, P, s, a, end);
                    a = -1;
                    cnt = 0;
                    loc = ack = false;
                }
                continue;
            }
            for (uint64_t ev = rm | bm; ev && s.status == MTR_OK; ev &= ev - 1) {
                const int l = first_lane(ev);
                const uint64_t bit = 1ull << l;
                if (rm & bit) {
                    if (a < 0) a = base + l;
                    cnt++;
                    loc = loc || (lm & bit) != 0;
                    ack = ack || (am & bit) != 0;
                    end = base + l + 1;
                } else if (a >= 0) {
                    if (loc && ack && cnt > 1) normalize_run(L, P, s, a, end);
                    a = -1;
                    cnt = 0;
                    loc = ack = false;
                }
            }
        }
        if (s.status == MTR_OK && a >= 0 && loc && ack && cnt > 1) normalize_run(L, P, s, a, end);
    }
    // regeneratePendingOp -> resetPendingDeltaToOps (client.ts:708-800) for the oldest pending group (type: the
    // op's MergeTreeDeltaType); gidx: the record's index (the MTR_DELTA_REGEN records' op field)
    static __device__ __attribute__((noinline)) void regenerate(D& L, const KParams& P, St& s, int type, int gidx) {
        const gptr<DocHdr> h = L.ghdr();
        const gptr<uint32_t> ring = L.gpend();
        if (uni(h->lastnorm) != s.curseq) {  // client.ts:921-926
            normalize(L, P, s);
            if (lane_id() == 0) h->lastnorm = s.curseq;
            wsync();
            if (s.status != MTR_OK) return;
        }
        const int head = uni(h->phead), tail = uni(h->ptail);
        if (head == tail || !ring) {
            s.status = MTR_ERR_ASSERT | 0x034;  // "Segment group not at head of merge tree pending queue"
            return;
        }
        const int slot = head % kPendRing;
        const int lseq = int(uniu(ring[4 * slot])), cnt = int(uniu(ring[4 * slot + 1]));
        const uint32_t ppo = uniu(ring[4 * slot + 3]);
        const int rw = int(uniu(ring[4 * slot + 2])) & PK_REWRITE;
        if (lane_id() == 0) h->phead = head + 1;  // pendingSegments.shift()
        wsync();
        const int S = s.nseg;
        // findReconnectionPosition (client.ts:699-706): getPosition at (currentSeq, this client, localSeq) --
        // the inclusive prefix of localNetLength(leaf, currentSeq, localSeq) (mergeTree.ts:613-662) in E
        int carry = 0;
        for (int base = 0; base < S; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, S - 1);
            const uint32_t m = L.meta[ic];
            const int sq = L.seq[ic], rs = L.rseq[ic], ln = L.len[ic];
            const bool lrem = rs != RNONE && rs >= LOCAL_BASE;  // localRemovedSeq = rs - LOCAL_BASE
            bool zero = (m & M_DEL) || (lrem && rs - LOCAL_BASE <= lseq);
            zero = zero || (sq >= LOCAL_BASE ? sq - LOCAL_BASE > lseq : (rs != RNONE && !lrem));
            const int inc = wave_incl_scan(i < S && !zero ? ln : 0);
            if (i < S) L.E[i] = carry + inc;
            carry += rdlane(inc, 63);
        }
        wsync();
        const int kind = type == MTR_OP_INSERT ? PK_INSERT : (type == MTR_OP_REMOVE ? PK_REMOVE : PK_ANNOTATE);
        int off = 0, seen = 0;  // off: the member's offset in the inserted text (its pieces, in tree order)
        for (int base = 0; base < S && seen < cnt && s.status == MTR_OK; base += 64) {
            const int i = base + lane_id();
            bool mem = false;
            if (i < S && (L.meta[i] & M_PEND))
                for (uint32_t c = pd_get(L, L.uid[i]); c != 0xffffffu; c = L.grm()[c] & 0xffffffu)
                    mem = mem || int(L.grm()[c + 1] >> 16) == slot;
            for (uint64_t mm = __ballot(mem); mm && s.status == MTR_OK; mm &= mm - 1) {  // ordinal order
                const int j = base + first_lane(mm);
                seen++;
                const int sq = uni(L.seq[j]), rs = uni(L.rseq[j]), ln = uni(L.len[j]);
                const int before = j > 0 ? uni(L.E[j - 1]) : 0;
                bool emit = false;
                if (type == MTR_OP_ANNOTATE) {  // not removed, or removed by a pending local op (client.ts:741-755)
                    emit = rs == RNONE || rs >= LOCAL_BASE;
                } else if (type == MTR_OP_INSERT) {
                    if (sq < LOCAL_BASE) {
                        s.status = MTR_ERR_ASSERT | 0x037;  // "Segment already has assigned sequence number"
                        break;
                    }
                    emit = true;
                } else if (type == MTR_OP_REMOVE) {  // still removed by this client only (client.ts:771-780)
                    emit = rs != RNONE && rs >= LOCAL_BASE;
                } else {
                    s.status = MTR_ERR_BAD_OP;
                    break;
                }
                pend_drop(L, j, slot);  // segment.segmentGroups.dequeue()
                // an annotate not re-sent keeps its pending key counts on the segment (they are never acked)
                if (type == MTR_OP_ANNOTATE && !emit) zomb_add(L, P, s, j, ppo, rw);
                const int here = off;
                off += ln;
                if (!emit) continue;
                if constexpr (DL) {
                    // (a PermutationSegment's clone keeps its start handle: the regenerated spec is [length, start])
                    const uint32_t pr = PM ? uniu(L.text[j]) : uniu(pget(L, j));
                    const int ref = PM ? (type == MTR_OP_INSERT ? int(pr) : -1)
                                       : ((type == MTR_OP_INSERT && pr != NONE32) ? int(pr & PN_MASK) : -1);
                    put_record(L, s, gidx, before, ln, uint32_t(MTR_DELTA_REGEN + type));
                    put_record(L, s, gidx, type == MTR_OP_INSERT ? here : 0, ref, MTR_DELTA_REGEN_X);
                }
                // a new group of its own at the tail, same localSeq (client.ts:787-795)
                pend_add(L, P, s, j, -1, kind | (type == MTR_OP_ANNOTATE ? rw : 0), type == MTR_OP_ANNOTATE ? ppo : 0u,
                         lseq);
            }
        }
    }

    // ---- properties (PropertiesManager.addProperties without combining ops,
    //      segmentPropertiesManager.ts:60-157; JS own-key order).  Entry: [n, k0, v0, k1, v1, ...]
    struct PropRes {
        uint32_t dst;
        int propused, status;
    };
        // (out of line: rare, and inlining it costs the replay kernels 2.5 % at C3)
    // pl: the leaf's pending-cell list (0xffffff = none): keys a pending local annotate holds are left
    // alone unless a combining op other than rewrite applies (shouldModifyKey, segmentPropertiesManager.ts:94-104)
    static __device__ __attribute__((noinline)) PropRes props_apply_serial(const D& L, const KParams& P, int propused,
                                                                         uint32_t old, uint32_t pp,
                                             uint32_t comb, uint32_t pl = 0xffffffu) {
        PropRes r{old, propused, MTR_OK};
        if (pl != 0xffffffu && rewrite_pending(L, pl)) return r;  // outstanding local rewrites block remote changes
        const gptr<uint32_t> gprop = L.gprop();
        const gptr<const uint32_t> poff = L.tab(CP_POFF), pkv = L.tab(CP_PKV), kix = L.tab(CP_KIX),
                                   veq = L.tab(CP_VEQ);
        const uint32_t mode = comb & 7u, nanv = comb >> 3;
        const bool never_old = pset_never(old);
        old &= PN_MASK;
        const uint32_t n_old = old == (NONE32 & PN_MASK) ? 0u : uniu(gprop[old]);
        const uint32_t lo = uniu(poff[pp]), hi = uniu(poff[pp + 1]);
        const uint32_t need = 1 + 2 * (n_old + (hi - lo));
        if (uint32_t(propused) + need > uint32_t(P.pcap)) {
            r.status = MTR_ERR_CAPACITY;
            return r;
        }
        const uint32_t dst = uint32_t(propused);
        const gptr<uint32_t> e = gprop + dst;
        uint32_t n = n_old;
        for (uint32_t k = 0; k < 2 * n_old; k++) e[1 + k] = gprop[old + 1 + k];
        if (mode == MTR_COMB_REWRITE) {  // old keys whose new value is absent or falsy go first (:109-123)
            uint32_t w = 0;
            for (uint32_t k = 0; k < n; k++) {
                const uint32_t key = uniu(e[1 + 2 * k]), val = uniu(e[2 + 2 * k]);
                bool keep = false;
                for (uint32_t q = lo; q < hi; q++)
                    if (uniu(pkv[2 * q]) == key) {
                        const uint32_t nv = uniu(pkv[2 * q + 1]);
                        keep = nv != MTR_NULL_VALUE && !(uniu(veq[nv]) & MTR_VEQ_FALSY);
                        break;
                    }
                if (keep || (pl != 0xffffffu && key_pending(L, pl, key))) {
                    e[1 + 2 * w] = key;
                    e[2 + 2 * w] = val;
                    w++;
                }
            }
            n = w;
        }
        for (uint32_t q = lo; q < hi; q++) {
            const uint32_t key = uniu(pkv[2 * q]);
            uint32_t val = uniu(pkv[2 * q + 1]);
            if (pl != 0xffffffu && mode < MTR_COMB_INCR && key_pending(L, pl, key)) continue;
            int at = -1;
            for (uint32_t k = 0; k < n; k++)
                if (uniu(e[1 + 2 * k]) == key) {
                    at = int(k);
                    break;
                }
            if (mode >= MTR_COMB_INCR && at >= 0) {  // combine(op, prev, undefined, seq), properties.ts:24-69
                const uint32_t prev = uniu(e[2 + 2 * at]), f = uniu(veq[prev]);
                if ((mode == MTR_COMB_INCR && (f & MTR_VEQ_INCR_STR)) ||
                    (mode == MTR_COMB_CONSENSUS && (f & MTR_VEQ_CONS_MUT))) {
                    r.status = MTR_ERR_UNSUPPORTED;
                    return r;
                }
                val = mode == MTR_COMB_INCR ? nanv : prev;
            }
            if (val == MTR_NULL_VALUE) {
                if (at >= 0) {
                    for (uint32_t k = uint32_t(at); k + 1 < n; k++) {
                        e[1 + 2 * k] = uniu(e[1 + 2 * (k + 1)]);
                        e[2 + 2 * k] = uniu(e[2 + 2 * (k + 1)]);
                    }
                    n--;
                }
            } else if (at >= 0) {
                e[2 + 2 * at] = val;
            } else {
                const uint32_t ix = uniu(kix[key]);
                uint32_t pos = n;
                if (ix != MTR_NOT_INDEX) {
                    pos = 0;
                    while (pos < n && uniu(kix[uniu(e[1 + 2 * pos])]) != MTR_NOT_INDEX &&
                           uniu(kix[uniu(e[1 + 2 * pos])]) < ix)
                        pos++;
                    for (uint32_t k = n; k > pos; k--) {
                        e[1 + 2 * k] = uniu(e[1 + 2 * (k - 1)]);
                        e[2 + 2 * k] = uniu(e[2 + 2 * (k - 1)]);
                    }
                }
                e[1 + 2 * pos] = key;
                e[2 + 2 * pos] = val;
                n++;
            }
        }
        uint32_t never = 0;
        if (mode >= MTR_COMB_INCR || never_old)
            for (uint32_t k = 0; k < n; k++)
                if (uniu(veq[uniu(e[2 + 2 * k])]) & MTR_VEQ_NEVER) never = MTR_PROPS_NEVER;
        e[0] = n;
        r.propused = propused + int(1 + 2 * n);
        r.dst = dst | never;
        return r;
    }

    // Wave version: the old set and the op's keys are fetched once (one lane per entry) and the
    // set is edited in registers (lane t = entry t).  Combining annotates (comb: MTR_COMB_* | NaN id << 3),
    // sets holding a never-equal value and sets above 64 keys take the out-of-line serial form.
    static MTR_DI uint32_t props_apply(D& L, const KParams& P, St& s, uint32_t old, uint32_t pp, uint32_t comb = 0) {
        const gptr<const uint32_t> poff = L.tab(CP_POFF), pkv = L.tab(CP_PKV), kix = L.tab(CP_KIX);
        const int n_old = old == NONE32 ? 0 : int(uniu(L.gprop()[old & PN_MASK]));
        const int lo = int(uniu(poff[pp])), nq = int(uniu(poff[pp + 1])) - lo;
        if (n_old + nq > 64 || (X && comb != 0) || pset_never(old)) {
            const PropRes r = props_apply_serial(L, P, s.propused, old, pp, comb);
            s.propused = uni(r.propused);
            if (uni(r.status) != MTR_OK) s.status = uni(r.status);
            wsync();
            return uniu(r.dst);
        }
        const uint32_t need = 1 + 2 * uint32_t(n_old + nq);
        if (uint32_t(s.propused) + need > uint32_t(P.pcap)) {
            s.status = MTR_ERR_CAPACITY;
            return old;
        }
        const int ln = lane_id();
        uint32_t wk = 0, wv = 0, wx = MTR_NOT_INDEX, qk = 0, qv = 0, qx = MTR_NOT_INDEX;
        if (ln < n_old) {
            wk = L.gprop()[old + 1 + 2 * ln];
            wv = L.gprop()[old + 2 + 2 * ln];
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
        const uint32_t dst = uint32_t(s.propused);
        const gptr<uint32_t> e = L.gprop() + dst;
        if (ln < n) {
            e[1 + 2 * ln] = wk;
            e[2 + 2 * ln] = wv;
        }
        e[0] = uint32_t(n);
        s.propused += 1 + 2 * n;
        wsync();
        return dst;
    }

    // matchProperties on the wave: one lane per key of `a`, `b`'s keys broadcast by readlane
    static MTR_DI bool props_match_w(const D& L, const KParams& P, uint32_t a, uint32_t b) {
        if (a == b) return !pset_never(a);
        if (a == NONE32 || b == NONE32) return false;
        a &= PN_MASK;
        b &= PN_MASK;
        const int na = int(uniu(L.gprop()[a])), nb = int(uniu(L.gprop()[b]));
        if (na != nb) return false;
        const gptr<const uint32_t> veq = L.tab(CP_VEQ);
        if (na > 64) return __ballot(!props_match(L.gprop(), veq, a, b)) == 0;
        PROF(P_PMATCH);
        PROF_COUNT(P_NPMATCH);
        const int ln = lane_id();
        uint32_t ka = 0, kb = 0, ea = 0, eb = 0;
        if (ln < na) {
            ka = L.gprop()[a + 1 + 2 * ln];
            kb = L.gprop()[b + 1 + 2 * ln];
            ea = veq[L.gprop()[a + 2 + 2 * ln]];
            eb = veq[L.gprop()[b + 2 + 2 * ln]];
        }
        bool found = ln >= na, ok = true;
        for (int j = 0; j < nb; j++) {
            const uint32_t kj = rdlane(kb, j), ej = rdlane(eb, j);
            if (ka == kj && ln < na) {
                found = true;
                ok = ea == ej && !(ea & MTR_VEQ_NEVER);
            }
        }
        return __ballot(!(found && ok)) == 0;
    }

    // ---- text
    static MTR_DI bool can_append(uint32_t ma, int la, uint32_t mb, int lb) {  // TextSegment.canAppend, textSegment.ts:86-93
        if ((ma | mb) & M_MARKER) return false;
        if (la > 0 && (ma & M_NL)) return false;
        return la <= kGranularity || lb <= kGranularity;
    }
    static MTR_DI void copy_text(const D& L, uint32_t dst, uint32_t src, int n) {
        const gptr<uint16_t> t = L.gtext();
        for (int k = lane_id(); k < n; k += 64) t[dst + k] = t[src + k];
    }
    static MTR_DI int text_end(const St& s, const KParams& P) { return (P.tcap / 2) * (s.texthalf + 1); }
    // one lane's copy of n units: 8 loads in flight, then 8 stores
    static MTR_DI void copy_units(const D& L, uint32_t dst, uint32_t src, int n) {
        const gptr<uint16_t> t = L.gtext();
        for (int u0 = 0; u0 < n; u0 += 8) {
            uint16_t b[8];
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (u0 + q < n) b[q] = t[src + u0 + q];
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (u0 + q < n) t[dst + u0 + q] = b[q];
        }
    }

    // Concatenation of a merge chain's texts: chain units [c0, total) go to dst + p, unit p taken
    // from the piece (a lane in `pieces`, chain offset `off`, arena offset `vt`) that covers it.
    // Every lane copies units c0 + lane, c0 + lane + 64, ...: the loads of a batch of 8 rounds
    // are all in flight before its stores (one HBM round trip per 512 units, not per 8 units of
    // one lane's piece).
    // the deferred store of copy_chain's last short chain: before anything reads the text arena, and at the
    // end of the launch
    static MTR_DI void text_flush(D& L) {
        if (L.pc_any) {
            if (L.pc_on) L.gtext()[L.pc_dst] = uint16_t(L.pc_val);
            L.pc_on = 0;
            L.pc_any = 0;
            wsync();
        }
    }
    static MTR_DI void copy_chain(D& L, uint32_t dst, int c0, int total, uint64_t pieces, uint32_t vt, int off) {
        const int ln = lane_id();
        text_flush(L);  // (its sources may be the last chain's destination)
        const gptr<uint16_t> t = L.gtext();
        if (total - c0 <= 64) {  // the common chain: one round; its load now, its store at the next text_flush
            const int pos = c0 + ln;
            uint32_t src = 0;
            for (uint64_t pm = pieces; pm; pm &= pm - 1) {
                const int j = first_lane(pm);
                const int pj = rdlane(off, j);
                src = vp_sel(vp_le(pj, pos), int(rdlane(vt, j) + uint32_t(pos - pj)), int(src));
            }
            L.pc_on = pos < total;
            L.pc_dst = dst + uint32_t(pos);
            // (lanes past the chain's end load unit 0 of this document's arena: their computed source can lie past
            // the last document's allocation)
            L.pc_val = t[uint32_t(vp_sel(vp_lt(pos, total), int(src), 0))];
            L.pc_any = 1;
            return;
        }
        for (int b0 = c0; b0 < total; b0 += 8 * 64) {
            uint16_t u[8];
            uint32_t src[8];
#pragma unroll
            for (int q = 0; q < 8; q++) src[q] = NONE32;
            for (uint64_t pm = pieces; pm; pm &= pm - 1) {  // pieces in chain order: the last start <= p wins
                const int j = first_lane(pm);
                const int pj = rdlane(off, j);
                const uint32_t tj = rdlane(vt, j);
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int pos = b0 + 64 * q + ln;
                    if (pos >= pj) src[q] = tj + uint32_t(pos - pj);
                }
            }
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (b0 + 64 * q + ln < total) u[q] = t[src[q]];
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (b0 + 64 * q + ln < total) t[dst + uint32_t(b0 + 64 * q + ln)] = u[q];
        }
    }

    // prev.append(seg) (textSegment.ts:99-103): text of b follows text of a.  Updates L.len/L.text
    // of a; the caller keeps M_NL.
    static MTR_DI void text_append(D& L, const KParams& P, St& s, int a, int b) {
        PROF(P_TAPPEND);
        text_flush(L);
        PROF_COUNT(P_NMERGE);
        const int tend = text_end(s, P);
        const uint32_t oa = uniu(L.text[a]), ob = uniu(L.text[b]);
        const int la = uni(L.len[a]), lb = uni(L.len[b]);
        if (oa + uint32_t(la) == ob) {
            L.len[a] = la + lb;
            wsync();
            return;
        }
        if (oa + uint32_t(la) == uint32_t(s.textused)) {
            if (s.textused + lb > tend) {
                s.status = MTR_ERR_CAPACITY;
                return;
            }
            copy_text(L, uint32_t(s.textused), ob, lb);
            s.textused += lb;
            L.len[a] = la + lb;
            wsync();
            return;
        }
        if (s.textused + la + lb > tend) {
            s.status = MTR_ERR_CAPACITY;
            return;
        }
        const uint32_t d = uint32_t(s.textused);
        copy_text(L, d, oa, la);
        copy_text(L, d + uint32_t(la), ob, lb);
        s.textused += la + lb;
        L.text[a] = d;
        L.len[a] = la + lb;
        wsync();
    }

    // Semi-space compaction of the text arena: copy every leaf's text into the other half in
    // leaf order (prefix scan of lengths), then switch halves.
    static MTR_COLD void text_gc(D& L, const KParams& P, St& s) {
        PROF(P_TEXTGC);
        text_flush(L);
        const int S = s.nseg;
        const int half = P.tcap / 2;
        const int dst0 = s.texthalf ? 0 : half;
        int carry = 0;
        constexpr int ZK = G ? GK : 1;  // (HBM: GK rounds of leaf fields in flight)
        for (int base = 0; base < S; base += 64 * ZK) {
            uint32_t mq[ZK], tq[ZK];
            int lq[ZK];
#pragma unroll
            for (int q = 0; q < ZK; q++) {
                const int ic = min(base + 64 * q + lane_id(), S - 1);
                mq[q] = L.meta[ic];
                lq[q] = L.len[ic];
                tq[q] = L.text[ic];
            }
#pragma unroll
            for (int q = 0; q < ZK; q++) {
                const int i = base + 64 * q + lane_id();
                const bool t = i < S && !(mq[q] & M_MARKER);
                const int n = t ? lq[q] : 0;
                const int inc = wave_incl_scan(n);
                const int off = dst0 + carry + inc - n;
                if (t) {
                    copy_units(L, uint32_t(off), tq[q], n);
                    L.text[i] = uint32_t(off);
                }
                carry += rdlane(inc, 63);
            }
        }
        wsync();
        s.texthalf ^= 1;
        s.textused = dst0 + carry;
        if (carry > half) s.status = MTR_ERR_CAPACITY;
    }

    // ------------------------------------------------------------ HandleTable (matrix/src/handletable.ts)
    // A permutation vector keeps its HandleTable in its (otherwise unused) text arena as int32
    // words; handles[0] is the head of the free list, s.textused the array length.
    static MTR_DI gptr<int32_t> handles(const D& L) { return (gptr<int32_t>)L.gtext(); }
    // HandleTable.load's entries (two UTF-16 units each, low half first), out of line (rare)
    static MTR_DI void load_handles(gptr<const uint16_t> src, gptr<int32_t> dst, int n) {
        for (int k = lane_id(); k < n; k += 64) dst[k] = int32_t(uint32_t(src[2 * k]) | (uint32_t(src[2 * k + 1]) << 16));
    }
    static MTR_DI int handle_cap(const KParams& P) { return P.tcap / 2; }
    // HandleTable.allocate, handletable.ts:37-42
    static MTR_DI int alloc_handle(D& L, const KParams& P, St& s) {
        const gptr<int32_t> h = handles(L);
        const int fr = uni(h[0]);
        const int hlen = s.textused;
        int nx;
        if (fr < hlen) {
            nx = uni(h[fr]);
        } else {  // handles[free] === undefined: the array grows by one
            if (hlen + 1 > handle_cap(P)) {
                s.status = MTR_ERR_CAPACITY;
                return MTR_HANDLE_UNALLOCATED;
            }
            nx = fr + 1;
            s.textused = hlen + 1;
        }
        if (lane_id() == 0) {
            h[fr] = 0;
            h[0] = nx;
        }
        wsync();
        return fr;
    }
    // HandleTable.free of handles a, a+1, ..., a+n-1 in that order (onMaintenance UNLINK frees a
    // segment's handles in ascending order, permutationvector.ts:418-443): handles[a] = old head,
    // handles[a+q] = a+q-1, head = a+n-1
    static MTR_DI void free_handles(D& L, St& s, int a, int n) {
        // a matrix tracked for its cells: the host clears the recycled handles' rows / cols
        // (onRowHandlesRecycled / onColHandlesRecycled, matrix.ts:722-734)
        if (DL && L.dcap > 0) put_record(L, s, s.cur_op, a, n, MTR_DELTA_RECYCLE);
        const gptr<int32_t> h = handles(L);
        const int head = uni(h[0]);
        for (int q = lane_id(); q < n; q += 64) h[a + q] = q == 0 ? head : a + q - 1;
        wsync();
        if (lane_id() == 0) h[0] = a + n - 1;
        wsync();
    }
    // PermutationSegment.canAppend (permutationvector.ts:131-137) of a chain whose head starts at
    // handle pt with accumulated length pl, and a segment starting at handle t
    static MTR_DI bool perm_contig(uint32_t pt, int pl, uint32_t t) {
        return pt == uint32_t(MTR_HANDLE_UNALLOCATED) ? t == uint32_t(MTR_HANDLE_UNALLOCATED)
                                                      : t == pt + uint32_t(pl);
    }

    // ---- tracking groups of PermutationVector segments (SharedMatrix undo, include/mtr_types.h "Tracking
    // groups"): a vector's leaves keep their tracking id in the props field (NONE32: never tracked; a permutation
    // segment has no properties) and the document's property arena holds the group bits per id (propused = ids)
    static MTR_DI uint32_t tbits(const D& L, uint32_t tid) { return tid == NONE32 ? 0u : uniu(L.gprop()[tid]); }
    // a fresh id holding `bits` (wave-uniform; NONE32 when the arena is full: s.status): the id freed last, else a
    // new one.  The free stack grows down from the arena's top and a new id reserves its slot there, so a free
    // always fits (ids: propused <= pcap / 2).
    static MTR_DI uint32_t tid_new(const D& L, const KParams& P, St& s, uint32_t bits) {
        const int nf = uni(L.ghdr()->tfree);
        uint32_t t;
        if (nf > 0) {
            t = uniu(L.gprop()[uint32_t(P.pcap) - uint32_t(nf)]);
            if (lane_id() == 0) L.ghdr()->tfree = nf - 1;
        } else if (2 * (uint32_t(s.propused) + 1u) > uint32_t(P.pcap)) {
            s.status = MTR_ERR_CAPACITY;
            return NONE32;
        } else {
            t = uint32_t(s.propused++);
        }
        if (lane_id() == 0) L.gprop()[t] = bits;
        wsync();
        return t;
    }
    // the id of a segment zamboni unlinked or merged away goes back on the free stack (no leaf names it any more,
    // and the host's groups dropped it: an unlinked segment was in none, a merged one's report unlinked it)
    static MTR_DI void tid_free(const D& L, const KParams& P, uint32_t t) {
        const int nf = uni(L.ghdr()->tfree);
        if (lane_id() == 0) {
            L.gprop()[uint32_t(P.pcap) - 1u - uint32_t(nf)] = t;
            L.gprop()[t] = 0u;
            L.ghdr()->tfree = nf + 1;
        }
        wsync();
    }
    // TrackingGroup.link (mergeTreeTracking.ts:41-46) of leaf i into the groups `bits`, reported in link order
    static MTR_DI void track_link(D& L, const KParams& P, St& s, int i, uint32_t bits) {
        uint32_t t = uniu(pget(L, i));
        if (t == NONE32) {
            t = tid_new(L, P, s, bits);
            if (t == NONE32) return;
            if (lane_id() == 0) pset(L, i, t);
        } else if (lane_id() == 0) {
            L.gprop()[t] = L.gprop()[t] | bits;
        }
        wsync();
        if (DL && L.dcap > 0) put_record(L, s, s.cur_op, int(t), uni(L.len[i]), MTR_DELTA_TLINK);
    }
    // the delta segments of a local remove (range_walk marked them M_TOUCH), in leaf order; `clear`: drop the
    // marks (a pending remove leaves them to pend_touched)
    static MTR_DI void track_touched(D& L, const KParams& P, St& s, uint32_t bits, bool clear) {
        for (int base = 0; base < s.nseg && s.status == MTR_OK; base += 64) {
            const int i = base + lane_id();
            const uint32_t m = L.meta[min(i, s.nseg - 1)];
            const bool t = i < s.nseg && (m & M_TOUCH);
            uint64_t tm = __ballot(t);
            if (t && clear) L.meta[i] = m & ~M_TOUCH;
            wsync();
            for (; tm && s.status == MTR_OK; tm &= tm - 1) track_link(L, P, s, base + first_lane(tm), bits);
        }
    }
    // BaseSegment.splitAt's trackingCollection.copyTo (mergeTreeNodes.ts:500): the right half of a split of a
    // tracked leaf (id t) joins its groups under an id of its own; an untracked half keeps none
    static MTR_DI uint32_t track_split(D& L, const KParams& P, St& s, uint32_t t) {
        const uint32_t b = tbits(L, t);
        if (!b) return NONE32;
        const uint32_t r = tid_new(L, P, s, b);
        if (r != NONE32 && DL && L.dcap > 0) put_record(L, s, s.cur_op, int(t), int(r), MTR_DELTA_TSPLIT);
        return r;
    }
    // PermutationSegment.transferToReplacement (permutationvector.ts:80-102) from the leaf with id `src` to the
    // new leaf dst (already linked, so it has an id): the handles and the groups move, the source keeps neither
    static MTR_DI void track_transfer(D& L, const KParams& P, St& s, int dst, uint32_t src) {
        int at = -1;
        for (int base = 0; base < s.nseg && at < 0; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, s.nseg - 1);
            const uint64_t hit = __ballot(i < s.nseg && !(L.meta[ic] & M_DEL) && pget(L, ic) == src);
            if (hit) at = base + first_lane(hit);
        }
        const uint32_t dt = uniu(pget(L, dst));
        if (at < 0 || at == dst || dt == NONE32) {
            s.status = MTR_ERR_BAD_OP;
            return;
        }
        if (lane_id() == 0) {
            L.text[dst] = L.text[at];
            L.text[at] = uint32_t(MTR_HANDLE_UNALLOCATED);
            L.gprop()[dt] = L.gprop()[dt] | L.gprop()[src];
            L.gprop()[src] = 0u;
        }
        wsync();
    }
    // MergeTree.insertAtReferencePosition (mergeTree.ts:1429-1530) at offset 0 of the leaf with id t: the slot in
    // front of the run of zero-length leaves that ends at it (backwardExcursion with breakTie against
    // UnassignedSequenceNumber, which every leaf loses; leaves zamboni may drop -- undefined length -- are skipped
    // over), -1 when no leaf has the id
    static MTR_DI int track_ref_slot(const D& L, const KParams& P, const St& s, uint32_t t) {
        int at = -1;
        for (int base = 0; base < s.nseg && at < 0; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, s.nseg - 1);
            const uint64_t hit = __ballot(i < s.nseg && !(L.meta[ic] & M_DEL) && pget(L, ic) == t);
            if (hit) at = base + first_lane(hit);
        }
        if (at < 0) return -1;
        int start = at;
        for (int j = at - 1; j >= 0; j--) {
            if (uniu(L.meta[j]) & M_DEL) continue;  // (a hole slot)
            const int rs = uni(L.rseq[j]);
            if (rs == RNONE) break;  // a segment the local view shows: positive length
            if (P.new_length_calc || rs >= LOCAL_BASE || rs > s.minseq) start = j;  // length 0, not undefined
        }
        return start;
    }
    // MTR_OP_TRACK: TrackingGroup.unlink of the groups `bits` from the leaf with id t (NONE32: from every leaf)
    static MTR_DI void track_clear(D& L, St& s, uint32_t t, uint32_t bits) {
        if (t != NONE32) {
            if (t >= uint32_t(s.propused)) {
                s.status = MTR_ERR_BAD_OP;
                return;
            }
            if (lane_id() == 0) L.gprop()[t] = L.gprop()[t] & ~bits;
        } else {
            for (int q = lane_id(); q < s.propused; q += 64) L.gprop()[q] = L.gprop()[q] & ~bits;
        }
        wsync();
    }

    // ------------------------------------------------------------ zamboni
    // scourNode (zamboni.ts:122-193) over the child blocks in [cs, ce): a new child block starts at
    // every leaf with bnd >= 1.  Marks M_DEL; returns #kept (used for a single block).  The leaves
    // are read 64 at a time into registers and visited in order by readlane.
    static MTR_COLD int scour_range(D& L, const KParams& P, St& s, int cs, int ce) {
        const int minseq = s.minseq;
        int prev = -1, kept = 0, plen = 0;
        uint32_t pmeta = 0, pprops = 0, ptext = 0;
        for (int base = cs; base < ce; base += 64) {
            const int i = base + lane_id();
            const int ic = min(i, ce - 1);
            uint32_t vm = L.meta[ic];
            const uint32_t vp = pget(L, ic), vt = L.text[ic];
            const int vr = L.rseq[ic], vs = L.seq[ic], vl = L.len[ic];
            if (i >= ce) vm = M_DEL;
            {  // merge candidates whose trailing-newline bit is unknown: one HBM round trip
                const bool q = !PM && (vm & (M_NLQ | M_DEL | M_MARKER)) == M_NLQ && vl > 0 && vr == RNONE &&
                               vs <= minseq;
                if (__ballot(q)) {
                    PROF(P_NLQ);
                    PROF_COUNT(P_NNLQ);
                    text_flush(L);
                    if (q) {
                        const uint16_t u = L.gtext()[L.text[i] + uint32_t(vl) - 1];
                        vm = (vm & ~(M_NLQ | M_NL)) | (u == u'\n' ? M_NL : 0u);
                        L.meta[i] = vm;
                    }
                    wsync();
                }
            }
            const int nk = min(64, ce - base);
            for (int t = 0; t < nk; t++) {
                const int k = base + t;
                const uint32_t m = rdlane(vm, t);
                if (k > cs && bnd_of(m) >= 1) prev = -1;  // next child block
                if (m & M_DEL) continue;
                if (X && (m & M_PEND)) {  // segmentGroups not empty: held (zamboni.ts:128, 185-188)
                    kept++;
                    prev = -1;
                    continue;
                }
                const int rs = rdlane(vr, t);
                if (rs != RNONE) {
                    if (rs > minseq || (PM && tbits(L, rdlane(vp, t)))) {  // (a tracked segment is held, zamboni.ts:132)
                        kept++;
                    } else {
                        L.meta[k] = m | M_DEL;  // UNLINK
                        wsync();
                        const uint32_t tk = rdlane(vt, t);
                        if (PM && tk != uint32_t(MTR_HANDLE_UNALLOCATED)) free_handles(L, s, int(tk), rdlane(vl, t));
                        if (PM && rdlane(vp, t) != NONE32) tid_free(L, P, rdlane(vp, t));
                    }
                    prev = -1;
                } else if (rdlane(vs, t) <= minseq) {
                    const int lk = rdlane(vl, t);
                    const uint32_t pk = rdlane(vp, t);
                    const uint32_t tk = rdlane(vt, t);
                    const bool ca = PM ? perm_contig(ptext, plen, tk) : can_append(pmeta, plen, m, lk);
                    // (a matrix vector: the same tracking groups, trackingCollection.matches, zamboni.ts:156)
                    if (prev >= 0 && lk > 0 && ca &&
                        (PM ? tbits(L, pprops) == tbits(L, pk) : props_match_w(L, P, pprops, pk))) {
                        if constexpr (X && !PM) {  // BaseSegment.append (mergeTreeNodes.ts:527-530)
                            if (nrefs(L)) ref_append(L, uniu(L.uid[k]), uniu(L.uid[prev]), plen);
                        }
                        if (PM && DL && L.dcap > 0 && tbits(L, pk))  // the appended segment leaves its groups
                            put_record(L, s, s.cur_op, int(pk), int(pprops), MTR_DELTA_TMERGE);
                        if (PM && pk != NONE32) tid_free(L, P, pk);
                        if (PM) {
                            L.len[prev] = plen + lk;
                            wsync();
                        } else {
                            text_append(L, P, s, prev, k);
                        }
                        plen += lk;
                        pmeta = (pmeta & ~(M_NL | M_NLQ | (m & M_NONL ? 0u : M_NONL))) | (m & (M_NL | M_NLQ));
                        L.meta[prev] = pmeta;
                        L.meta[k] = m | M_DEL;
                        wsync();
                    } else {
                        kept++;
                        if (lk > 0) {
                            prev = k;
                            pmeta = m;
                            plen = lk;
                            pprops = pk;
                            ptext = tk;
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

    // scourNode over [cs, ce) with all leaves classified at once (ce - cs <= 64).  For a leaf k
    // that was not already unlinked, the serial walk's merge candidate `prev` is the nearest
    // earlier such leaf p when no child-block boundary lies in (p, k] and p is a live leaf below
    // minSeq with positive length (p is then the chain head or its last merged member; merged
    // members matched the head, and matchProperties is an equivalence).  Leaf k merges into the
    // chain iff it is such a leaf too and canAppend/matchProperties hold against p.  The
    // TextSegmentGranularity clause of canAppend depends on the accumulated chain length, so a
    // range where a leaf longer than 256 units would link falls back to the serial walk.
    // Returns #kept, or -1 when the caller must run the serial walk (nothing was modified).
    static MTR_DI int scour_par(D& L, const KParams& P, St& s, int cs, int ce) {
        return scour_lanes(L, P, s, cs, cs + lane_id(), cs + lane_id() < ce, ce - 1);
    }
    // HBM-resident documents: a range of more than 64 slots whose leaves (hole slots aside) fit in 64
    // lanes -- each lane takes one of them in slot order; -1 when more than 64 remain
    static MTR_DI int scour_gather(D& L, const KParams& P, St& s, int cs, int ce) {
        if constexpr (G) {
            const lptr<int> slot = dlist(L);  // (prefix2's chunk list: not in use during zamboni)
            int n = 0;
            for (int b = cs; b < ce; b += 64 * GK) {
                uint32_t mq[GK];
#pragma unroll
                for (int q = 0; q < GK; q++) mq[q] = L.meta[min(b + 64 * q + lane_id(), ce - 1)];
#pragma unroll
                for (int q = 0; q < GK; q++) {
                    const int i = b + 64 * q + lane_id();
                    // a hole slot (M_DEL, no block start) takes no part in the scour's chains or boundaries
                    const bool keep = i < ce && !((mq[q] & M_DEL) && bnd_of(mq[q]) == 0);
                    const uint64_t km = __ballot(keep);
                    const int at = n + __popcll(km & lanes_below());
                    if (keep && at < 64) slot[at] = i;
                    n += __popcll(km);
                }
                if (n > 64) return -1;
            }
            wsync();
            const bool in = lane_id() < n;
            const int mine = in ? slot[lane_id()] : cs;
            wsync();
            return scour_lanes(L, P, s, cs, mine, in, ce - 1);
        }
        return -1;
    }
    // the lane-parallel scour over the leaves lanes hold (slot i, in = the lane holds one), in slot order
    static MTR_DI int scour_lanes(D& L, const KParams& P, St& s, int cs, int i, bool in, int clamp) {
        const int minseq = s.minseq;
        const int ln = lane_id();
        const int ic = in ? i : min(cs, clamp);
        const uint32_t vm0 = L.meta[ic], vp = pget(L, ic), vt = L.text[ic];
        const int vr0 = L.rseq[ic], vs = L.seq[ic], vl0 = L.len[ic];
        const uint32_t vu = X ? L.uid[ic] : 0u;  // (local references follow appends)
        uint32_t vm = in ? vm0 : M_DEL;
        const int vr = in ? vr0 : RNONE, vl = in ? vl0 : 0;
        const bool pre = (vm & M_DEL) != 0;
        const bool removed = vr != RNONE;
        const bool held = X && (vm & M_PEND) != 0;  // in a pending SegmentGroup: kept (zamboni.ts:128, 185-188)
        const bool cand = !pre & !removed & !held & (vs <= minseq) & (vl > 0);
        {  // merge candidates whose trailing-newline bit is unknown: one HBM round trip
            const bool q = cand & !PM & ((vm & (M_NLQ | M_MARKER)) == M_NLQ);
            if (__ballot(q)) {
                PROF(P_NLQ);
                PROF_COUNT(P_NNLQ);
                text_flush(L);
                if (q) {
                    const uint16_t u = L.gtext()[vt + uint32_t(vl) - 1];
                    vm = (vm & ~(M_NLQ | M_NL)) | (u == u'\n' ? M_NL : 0u);
                    L.meta[i] = vm;
                }
                wsync();
            }
        }
        const uint64_t nd = __ballot(in & !pre);
        const uint64_t bm = __ballot(in & (i > cs) & (bnd_of(vm) >= 1));
        const uint64_t below = nd & lanes_below();
        const int p = below ? last_lane(below) : -1;
        const int ps = p < 0 ? 0 : p;
        // the previous leaf's meta word with its candidacy in the top bit (M_ZOMB's place: only the marker
        // and newline bits are read from it): one shuffle
        const uint32_t pmc = uint32_t(__shfl(int((vm & ~M_ZOMB) | (cand ? 0x80000000u : 0u)), ps));
        const bool pc = (pmc >> 31) != 0;
        const uint32_t pm = pmc & 0x7fffffffu;
        const uint32_t pp = uint32_t(__shfl(int(vp), ps));
        const uint64_t upto = (uint64_t(2) << ln) - 1;  // lanes <= ln
        const uint64_t after_p = p < 0 ? ~uint64_t(0) : ~((uint64_t(2) << p) - 1);
        bool link = cand & (p >= 0) & pc & ((bm & upto & after_p) == 0);
        if (PM) {  // handle contiguity with the previous chain member (permutationvector.ts:131-137)
            const uint32_t pt = uint32_t(__shfl(int(vt), ps));
            const int pl = __shfl(vl, ps);
            link = link & perm_contig(pt, pl, vt);
        } else {
            link = link & !((vm | pm) & M_MARKER) & !(pm & M_NL);
        }
        // a matrix vector's props field is a tracking id: its group bits (0: none) -- trackingCollection.matches
        // (zamboni.ts:156) for a merge; a tracked removed segment is held (zamboni.ts:132)
        uint32_t vb = 0;
        if (PM && __ballot(in & (vp != NONE32))) vb = (in & (vp != NONE32)) ? L.gprop()[vp] : 0u;
        if (PM) {
            link = link & (uint32_t(__shfl(int(vb), ps)) == vb);
        } else {
            if (__ballot(link & (vp != pp))) {
                PROF(P_X1);
                if (link & (vp != pp)) link = props_match(L.gprop(), L.tab(CP_VEQ), pp, vp);
            }
            link = link & !((vp == pp) & pset_never(vp));  // a shared set holding a never-equal value
            if (__ballot(link & (vl > kGranularity))) return -1;
        }
        const bool unlink = !pre & removed & !held & (vr <= minseq) & (vb == 0u);
        const uint64_t lm = __ballot(link);
        if (unlink | link) L.meta[i] = vm | M_DEL;
        if (PM) {  // UNLINK frees the segment's handles, in leaf order
            for (uint64_t um = __ballot(unlink && vt != uint32_t(MTR_HANDLE_UNALLOCATED)); um; um &= um - 1) {
                const int l = first_lane(um);
                free_handles(L, s, int(rdlane(vt, l)), rdlane(vl, l));
            }
            // the tracking ids of the unlinked and the merged-away segments, in leaf order (their bits were read
            // into vb above)
            for (uint64_t fm = __ballot((unlink | link) && vp != NONE32); fm; fm &= fm - 1)
                tid_free(L, P, rdlane(vp, first_lane(fm)));
        }
        const int kept = __popcll(__ballot(in & !pre & !unlink & !link));
        if (lm) {  // concatenate each chain's text behind its head (prev.append, textSegment.ts:99-103)
            const uint64_t hm = __ballot(in & !pre & !link);  // chain heads and unmerged leaves
            // lane offsets inside its chain: inclusive scan of lengths restarted at every head
            const int hd = (hm & upto) ? last_lane(hm & upto) : 0;  // this lane's chain head (chain lanes)
            const int incl = wave_incl_scan((in & !pre) ? vl : 0);
            const int hbase = __shfl(incl - vl, hd);       // exclusive prefix at the head
            const int off = incl - vl - hbase;             // offset of this piece inside its chain
            uint64_t todo = lm;
            wsync();
            while (todo) {
                const int k0 = first_lane(todo);                   // first member of the next chain
                const int h = last_lane(hm & ((uint64_t(1) << k0) - 1));
                const uint64_t rest = hm & ~((uint64_t(2) << h) - 1);  // heads after h
                const uint64_t chain_end = rest ? ((uint64_t(1) << first_lane(rest)) - 1) : ~uint64_t(0);
                const uint64_t mem = lm & chain_end & ~((uint64_t(2) << h) - 1);
                todo &= ~mem;
                const int e = last_lane(mem);
                const int total = rdlane(incl, e) - rdlane(incl - vl, h);
                if constexpr (X && !PM) {  // BaseSegment.append (mergeTreeNodes.ts:527-530), member by member
                    if (nrefs(L))
                        for (uint64_t mm = mem; mm; mm &= mm - 1) {
                            const int l = first_lane(mm);
                            ref_append(L, rdlane(vu, l), rdlane(vu, h), rdlane(off, l));
                        }
                }
                if (PM) {  // BaseSegment.append: lengths only
                    const int hs = rdlane(i, h);  // (read with the whole wave active, as below)
                    if (DL && L.dcap > 0 && rdlane(vb, h))  // the appended segments leave their groups
                        for (uint64_t mm = mem; mm; mm &= mm - 1)
                            put_record(L, s, s.cur_op, int(rdlane(vp, first_lane(mm))), int(rdlane(vp, h)), MTR_DELTA_TMERGE);
                    if (ln == 0) L.len[hs] = total;
                    PROF_COUNT(P_NMERGE);
                    wsync();
                    continue;
                }
                PROF(P_X2);
                const uint32_t th = rdlane(vt, h);
                const int lh = rdlane(vl, h);
                const bool mine = ((mem >> ln) & 1) != 0;
                const bool inplace = __ballot(mine && vt != th + uint32_t(off)) == 0;
                uint32_t base = th;
                if (!inplace) {
                    const bool tail = th + uint32_t(lh) == uint32_t(s.textused);
                    base = tail ? th : uint32_t(s.textused);
                    const int need = int(base + uint32_t(total)) - s.textused;
                    if (s.textused + need > text_end(s, P)) {
                        s.status = MTR_ERR_CAPACITY;
                        return kept;
                    }
                    // the copied pieces: the members, and the head unless its text already ends
                    // the arena; all 64 lanes copy the chain's units [c0, total) together
                    copy_chain(L, base, tail ? lh : 0, total, (tail ? 0 : (uint64_t(1) << h)) | mem, vt, off);
                    s.textused = int(base) + total;
                }
                const uint32_t me = rdlane(vm, e), mh = rdlane(vm, h);
                const bool nonl = __ballot(mine && !(vm & M_NONL)) == 0 && (mh & M_NONL);
                // (lane h's slot is read with the whole wave active: inside `if (ln == 0)` only lane 0 is
                // active, and a value the compiler spills and reloads there holds lane 0's bits only)
                const int hs = rdlane(i, h);
                if (ln == 0) {
                    L.len[hs] = total;
                    L.text[hs] = base;
                    L.meta[hs] = (mh & ~(M_NL | M_NLQ | M_NONL)) | (me & (M_NL | M_NLQ)) | (nonl ? M_NONL : 0u);
                }
                PROF_COUNT(P_NMERGE);
                wsync();
            }
        }
        wsync();
        return kept;
    }

    // packParent's rebalancing of the level-l block [ps, pe) on an HBM-resident document (wave w of W): the
    // wave lists the items of its part of the range (surviving leaves at l == 2, else surviving level-(l-2) block
    // starts; at most 64), the waves post their counts, and each wave gives its items their new bnd marks -- the
    // first `rem` of the c blocks get base + 1 items, item 0 keeps `top`.  Returns c, or -1 (nothing written)
    // when a part holds more than 64 items: the caller's two passes take over.
    static MTR_DI int pack_part(const D& L, int ps, int pe, int l, int top, int w, int W) {
        const int ln = lane_id();
        const int part = ((pe - ps + W - 1) / W + 63) & ~63;
        const int lo = min(pe, ps + w * part), hi = min(pe, lo + part);
        // the list: prefix2's chunk list (HBM-resident documents), else the scan array E, which is dead between
        // the op's work and the next op's view scan
        lptr<int> lst;
        if constexpr (G) lst = dlist(L) + 64 * w;
        else lst = L.E;
        constexpr int ZK = G ? GK : 1;
        int n = 0;
        for (int wb = lo; wb < hi; wb += 64 * ZK) {
            uint32_t mq[ZK];
#pragma unroll
            for (int q = 0; q < ZK; q++) mq[q] = L.meta[min(wb + 64 * q + ln, hi - 1)];
#pragma unroll
            for (int q = 0; q < ZK; q++) {
                const int i = wb + 64 * q + ln;
                const bool it = i < hi && !(mq[q] & M_DEL) && (l == 2 || bnd_of(mq[q]) >= l - 2);
                const uint64_t mask = __ballot(it);
                const int k = n + __popcll(mask & lanes_below());
                if (it && k < 64) lst[k] = i;
                n += __popcll(mask);
            }
        }
        int T = n, off = 0;
        if (W > 1) {
            const lptr<int> row = tbox(L) + 16;
            if (ln == 0) row[w] = n;
            __syncthreads();
            T = 0;
            for (int u = 0; u < W; u++) {
                const int nu = uni(row[u]);
                if (u < w) off += nu;
                T += nu;
                if (nu > 64) T = -(1 << 20);
            }
        } else if (n > 64) {
            T = -1;
        }
        if (T < 0) return -1;
        if (T == 0) return 0;
        const int c = max(1, min(kMaxNodesInBlock - 1, T / (kMaxNodesInBlock / 2)));
        const int base = T / c;
        const int rem = T % c;
        const int big = rem * (base + 1);
        wsync();
        if (ln < n) {
            const int i = lst[ln];
            uint32_t m = L.meta[i];
            const int item = off + ln;
            const bool isStart = item < big ? item % (base + 1) == 0 : (item - big) % base == 0;
            const int nb = item == 0 ? top : (isStart ? l - 1 : (l == 2 ? 0 : l - 2));
            m = set_bnd(m, nb);
            if (l == 2 && isStart) m = set_ns(m, NS_UNDEF);
            L.meta[i] = m;
        }
        wsync();
        return c;
    }

    // zamboniSegments body for one popped LRU entry whose segment is leaf x
    // (zamboni.ts:33-58 + packParent zamboni.ts:63-120).  Returns the first leaf index at or
    // after which leaves may be marked for deletion (the caller compacts from there), or -1.
    static MTR_DI int zamboni_block(D& L, const KParams& P, St& s, int x, int& to) {
        PROF(P_ZBLOCK);
        PROF_COUNT(P_NZBLOCK);
        const int H = s.height;
        int rs1, re1;
        block_bounds1(L, s, x, rs1, re1);
        const uint32_t m1 = uniu(L.meta[rs1]);
        if (ns_of(m1) == NS_FALSE) return -1;
        const int topb1 = bnd_of(m1);
        const int before = G && s.holes ? count_live(L, rs1, re1) : re1 - rs1;
        to = re1;  // leaves marked for deletion lie in [from, to)
        int kept;
        {
            PROF(P_SCOUR1);
            kept = re1 - rs1 <= 64 ? scour_par(L, P, s, rs1, re1) : scour_gather(L, P, s, rs1, re1);
            if (kept < 0) kept = scour_range(L, P, s, rs1, re1);
        }
        // block.needsScour = false, kept on the block's first surviving leaf (a block of an HBM-resident
        // document can span more than 64 slots: holes)
        for (int b = rs1; b < re1; b += 64) {
            const int i = b + lane_id();
            const uint64_t m = __ballot(i < re1 && !(L.meta[min(i, re1 - 1)] & M_DEL));
            if (m) {
                const int first = b + first_lane(m);
                L.meta[first] = set_ns(set_bnd(uniu(L.meta[first]), topb1), NS_FALSE);
                wsync();
                break;
            }
        }
        if (kept >= before) return -1;
        int from = rs1;
        if (kept < kMaxNodesInBlock / 2 && H > 1) {
            PROF(P_PACK);
            PROF_COUNT(P_NPACK);
            // The level-l block around the level-(l-1) block [cs, ce): its start is found scanning
            // back from cs and its end scanning on from ce -- leaves whose bnd the scour and the
            // rebalancing below never change (they touch [cs, ce) only, where the first
            // surviving leaf may now repeat its block's start marker).
            int cs = rs1, ce = re1;
            for (int l = 2; l <= H; l++) {  // packParent chain
                int ps, pe;
                {
                    PROF(P_FETCH);
                    if (G && team_n() > 1) {
                        int cnt;
                        team_bounds(L, s, cs, ce, l, ps, pe, cnt);
                    } else {
                        ps = block_start(L, cs, l);
                        pe = block_end(L, s, ce - 1, l);
                    }
                }
                const int top = bnd_of(uniu(L.meta[ps]));
                cs = ps;
                ce = pe;
                if (l == 2) {
                    from = ps;
                    to = max(to, pe);
                    // packParent scours every child of P again -- including the block just
                    // scoured: scourNode is not idempotent (a dropped tombstone no longer resets
                    // the merge candidate), zamboni.ts:68-73,122-193.
                    PROF(P_SPLIT1);
                    if ((pe - ps <= 64 ? scour_par(L, P, s, ps, pe) : scour_gather(L, P, s, ps, pe)) < 0)
                        scour_range(L, P, s, ps, pe);
                }
                // items: surviving leaves (l == 2) or surviving level-(l-2) block starts
                {  // one pass lists them (at most 64 per wave), one round rebalances
                    int c = -1;
                    if (G && team_n() > 1) {
                        const lptr<int> b = tbox(L);
                        if (lane_id() == 0) {
                            b[1] = ps;
                            b[2] = pe;
                            b[3] = l;
                            b[4] = top;
                        }
                        team_start(L, T_PACK);
                        c = pack_part(L, ps, pe, l, top, 0, team_n());
                        __syncthreads();
                    } else {
                        c = pack_part(L, ps, pe, l, top, 0, 1);
                    }
                    if (c >= 0) {
                        if (!(c < kMaxNodesInBlock / 2 && l < H)) break;
                        continue;
                    }
                }
                constexpr int ZK = G ? GK : 1;  // (HBM: GK rounds of loads in flight)
                int T = 0;
                uint32_t m1r = M_DEL;  // a one-round range keeps its meta words in registers
                for (int wb = ps; wb < pe; wb += 64 * ZK) {
                    uint32_t mq[ZK];
#pragma unroll
                    for (int q = 0; q < ZK; q++) {
                        const int i = wb + 64 * q + lane_id();
                        mq[q] = L.meta[min(i, pe - 1)];
                        if (i >= pe) mq[q] = M_DEL;
                    }
                    if (wb == ps) m1r = mq[0];
#pragma unroll
                    for (int q = 0; q < ZK; q++)
                        T += __popcll(__ballot(!(mq[q] & M_DEL) && (l == 2 || bnd_of(mq[q]) >= l - 2)));
                }
                int c = 0;
                if (T > 0) {  // rebalance into c blocks: the first `rem` get base+1 items
                    c = min(kMaxNodesInBlock - 1, T / (kMaxNodesInBlock / 2));
                    if (c < 1) c = 1;
                    const int base = T / c;
                    const int rem = T % c;
                    const int big = rem * (base + 1);
                    int item0 = 0;
                    for (int wb = ps; wb < pe; wb += 64 * ZK) {
                        uint32_t mq[ZK];
#pragma unroll
                        for (int q = 0; q < ZK; q++) {
                            const int i = wb + 64 * q + lane_id();
                            mq[q] = pe - ps <= 64 ? m1r : L.meta[min(i, pe - 1)];
                            if (i >= pe) mq[q] = M_DEL;
                        }
#pragma unroll
                        for (int q = 0; q < ZK; q++) {
                            const int i = wb + 64 * q + lane_id();
                            uint32_t m = mq[q];
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
                    }
                    wsync();
                }
                if (!(c < kMaxNodesInBlock / 2 && l < H)) break;
            }
        }
        return from;
    }

    // zamboniSegments (zamboni.ts:19-60)
    static MTR_DI void zamboni(D& L, const KParams& P, St& s) {
        PROF(P_ZAMBONI);
        if (!s.collab) return;
        for (int it = 0; it < 2; it++) {
            if (s.heapn == 0 || s.status != MTR_OK) return;
            if (s.htop > s.minseq) return;
            const uint32_t u = heap_pop(L, s);
            const int x = find_uid(L, s, u);
            if (x < 0) continue;
            int to = 0;
            const int from = zamboni_block(L, P, s, x, to);
            if (from >= 0) {
                if (G && s.holes) {  // deleted leaves stay as hole slots
                    holeify(L, s, from, to);
                    csum_update(L, s, from, to);
                } else {
                    compact(L, s, from);
                    s.chunked = 0;
                }
            }
        }
    }

    // updateSeqNumbers + setMinSeq, client.ts:877-887 / mergeTree.ts:1025-1044; returns 1 when
    // minSeq advanced (the caller then runs zamboniSegments)
    static MTR_DI int update_seq(St& s, int msn, int seq) {
        int run = 0;
        if (s.curseq > seq) {
            s.status = MTR_ERR_ASSERT | 0x038;
        } else {
            s.curseq = seq;
            if (msn > seq) s.status = MTR_ERR_ASSERT | 0x039;
            else if (msn > s.curseq) s.status = MTR_ERR_ASSERT | 0x04e;
            else if (s.minseq > msn) s.status = MTR_ERR_ASSERT | 0x04f;
            else if (msn > s.minseq) {
                s.minseq = msn;
                run = 1;
            }
        }
        return run;
    }

    // ------------------------------------------------------------ boundary / insert
    // ensureIntervalBoundary (mergeTree.ts:1706-1716) on the current scan arrays: split the leaf
    // holding pos at an offset > 0; the two halves' scan entries are set in place.
    static MTR_DI void split_at(D& L, const KParams& P, St& s, int pos) {
        PROF(P_SPLIT);
        const int S = s.nseg;
        const int i = lower_bound_E(L, s, pos);
        if (i >= S) return;
        // one batch of loads for leaves i .. i+63: the leaf block's end, the leaf to split and
        // every field the split copies (a leaf block holds at most 7 leaves)
        const int ln = lane_id();
        const int jj = i + ln;
        const bool in = jj < S;
        const int jc = min(jj, S - 1);  // unconditional (clamped) loads
        const int ej0 = L.E[jc], ep = L.E[max(jc - 1, 0)];
        const uint32_t mj = L.meta[jc], tj = L.text[jc], pj = pget(L, jc), uj = L.uid[jc];
        const int lj = L.len[jc], sqj = L.seq[jc], rsj = L.rseq[jc];
        const int vj = ev(ej0, jc > 0 ? ep : 0);
        const int ej = ej0 & EMASK;
        const uint64_t em = __ballot(!in | (bnd_of(mj) >= 1)) & ~uint64_t(1);
        const int be = em ? i + first_lane(em) : block_end(L, s, i + 63, 1);
        const uint64_t cm = __ballot((jj < be) & (vj >= 0) & (pos < ej));
        if (!cm) return;
        const int jl = first_lane(cm);
        const int j = i + jl;
        const int v = rdlane(vj, jl), e = rdlane(ej, jl);
        const uint32_t m0 = rdlane(mj, jl);
        const int off = pos - (e - v);
        if (!(off > 0 && !(m0 & M_MARKER))) return;
        const bool grew = shift_right1(L, s, j + 1);
        {  // BaseSegment.splitAt, mergeTreeNodes.ts:481-510
            const int r = j + 1;
            L.len[r] = rdlane(lj, jl) - off;
            L.len[j] = off;
            L.seq[r] = rdlane(sqj, jl);
            L.rseq[r] = rdlane(rsj, jl);
            L.meta[r] = set_ns(set_bnd(m0, 0), NS_UNDEF);
            L.meta[j] = (m0 & M_NONL) ? (m0 & ~M_NL) : ((m0 & ~M_NL) | M_NLQ);
            {  // TextSegment: text offset; PermutationSegment: start + pos unless unallocated
                const uint32_t t0 = rdlane(tj, jl);
                L.text[r] = t0 == uint32_t(MTR_HANDLE_UNALLOCATED) ? t0 : t0 + uint32_t(off);
            }
            // (a matrix vector's props field is a tracking id: a tracked leaf's right half gets one of its own)
            pset(L, r, (PM && rdlane(pj, jl) != NONE32) ? track_split(L, P, s, rdlane(pj, jl)) : rdlane(pj, jl));
            const uint32_t ur = uint32_t(s.uidnext++);
            L.uid[r] = ur;
            if (G && s.chunked && lane_id() == 0) hint(L, ur, r);
            if constexpr (X) {  // mergeTreeNodes.ts:501-503
                if (nrefs(L)) {
                    wsync();
                    ref_split(L, uniu(rdlane(uj, jl)), off, ur);
                }
            }
            if (m0 & M_OVERLAP) {  // the right half shares the remover list
                if (lane_id() == 0 && !rm_set(L, ur, rm_get(L, rdlane(uj, jl)))) s.status = MTR_ERR_CAPACITY;
                s.status = uni(s.status);
            }
            // split leaves are fully visible in this view
            L.E[j] = e - v + off;
            L.E[r] = e;
            wsync();
            if (X && (m0 & (M_PEND | M_ZOMB))) pend_copy(L, P, s, uniu(rdlane(uj, jl)), r);
            if (grew) s.nseg++;
            if (G) csum_update(L, s, j, max(L.shi, r + 1));
            overflow_fix(L, s, r);
        }
    }

    // insertSegments/blockInsert/insertingWalk with onLeaf (mergeTree.ts:1397-1427, 1594-1685),
    // on the current scan arrays.  `pre`: lane t holds unit t of the op's text in `pf`
    // (prefetched during the previous op).
    // seq: breakTie's newSeq; sseq: the seq the new leaf keeps (LOCAL_BASE + localSeq for a pending local
    // insert, which passes lseq > 0 and joins a new SegmentGroup)
    static MTR_DI int insert_at(D& L, const KParams& P, St& s, const View& v, const mtr_op& op, int pos, int seq,
                                uint32_t client, const mtr_doc_desc& dd, bool pre, uint32_t pf, int sseq, int lseq,
                                int force = -1) {
        PROF(P_INSERT);
        const bool marker = (op.flags & MTR_F_MARKER) != 0;
        const int len = marker ? 1 : int(op.payload2);
        if (len <= 0) return -1;  // blockInsert skips empty segments
        const int t0 = s.textused;
        const int ln = lane_id();
        if (!marker && !PM) {  // copy the op's text into the document arena
            if (t0 + len > text_end(s, P)) {
                s.status = MTR_ERR_CAPACITY;
                return -1;
            }
            PROF(P_TEXTCOPY);
        }
        // the trailing-newline bit (TextSegment.canAppend) and "no newline at all" are known
        // here for every text insert, so scour never has to read them back from the arena
        bool nl = false, nonl = false;
        if (!marker && !PM) {
            bool any = false, last = false;
            if (pre) {
                if (ln < len) {
                    L.gtext()[t0 + ln] = uint16_t(pf);
                    any = pf == u'\n';
                    last = any && ln == len - 1;
                }
            } else {
                const gptr<const uint16_t> src = gp(P.btext) + dd.text_base + op.payload;
                for (int k = ln; k < len; k += 64) {
                    const uint16_t u = src[k];
                    L.gtext()[t0 + k] = u;
                    if (u == u'\n') {
                        any = true;
                        last = last || k == len - 1;
                    }
                }
            }
            nonl = __ballot(any) == 0;
            nl = __ballot(last) != 0;
        }
        const int S = s.nseg;
        int slot = -1, inherit = 0;
        bool nocand = false;  // no leaf of the block took the insert: it goes at the block's end
        uint32_t om = 0;  // meta of the leaf that starts the block when the new leaf takes its place
        bool om_known = false;
        int wbs = -1, wbe = -1;  // the leaf block around the slot, when the window saw both ends
        if (force >= 0) {  // insertAtReferencePosition: in front of leaf `force`, in its leaf block
            slot = force;
            inherit = slot == block_start(L, slot, 1) ? 1 : 0;
        } else {
            PROF(P_INS1);
            if (S == 0) {
                if (pos == 0) slot = 0;
                else s.status = MTR_ERR_INSERT_FAILED;
            } else {
                const int i = lower_bound_E(L, s, pos);
                if (i >= S) {
                    s.status = MTR_ERR_INSERT_FAILED;
                } else {
                    // one batch of loads over leaves i-31 .. i+32: the leaf block's bounds and the
                    // breakTie candidates (mergeTree.ts:1719-1738) in [i, be)
                    const int w = i - 31 + ln;
                    const bool inw = (w >= 0) & (w < S);
                    const int wc = min(max(w, 0), S - 1);  // unconditional (clamped) loads
                    const int ew0 = L.E[wc], ewp = L.E[max(wc - 1, 0)], sw = L.seq[wc];
                    const uint32_t mw = L.meta[wc];
                    const int vw = ev(ew0, wc > 0 ? ewp : 0);
                    const int ew = ew0 & EMASK;
                    const bool bw = inw & (bnd_of(mw) >= 1);
                    const uint64_t sm = __ballot((w <= 0) | bw) & LO32;
                    const uint64_t em = __ballot((w >= S) | bw) & HI32;
#ifdef MTR_DEBUG_INSERT  // (spill experiment: bw against a fresh load of the same meta words)
                    {
                        const uint32_t mw2 = __atomic_load_n((uint32_t*)&L.meta[wc], __ATOMIC_RELAXED);
                        const uint64_t b1 = __ballot(bw), b2 = __ballot(inw & (bnd_of(mw2) >= 1));
                        const uint64_t dm = __ballot(mw != mw2);
                        if (b1 != b2 && lane_id() == 0)
                            printf("MISMATCH op_begin %llu i %d ballot(bw) %llx fresh %llx meta-differs %llx\n",
                                   (unsigned long long)dd.op_begin, i, (unsigned long long)b1, (unsigned long long)b2,
                                   (unsigned long long)dm);
                    }
#endif
                    if (sm && em) {
                        const int bs = max(0, i - 31 + last_lane(sm));
                        const int be = i - 31 + first_lane(em);
                        const uint64_t cm = (HI32 | (uint64_t(1) << 31)) & __ballot((w < be) & (vw >= 0) &
                                                     ((ew > pos) | ((vw == 0) & (seq > sw))));
                        slot = cm ? i - 31 + first_lane(cm) : be;
                        nocand = !cm;
                        inherit = slot == bs ? 1 : 0;
                        wbs = bs;
                        wbe = be + 1;  // the block after the insert
                        if (inherit) {
                            om = uint32_t(rdlane(int(mw), bs - i + 31));
                            om_known = true;
                        }
                    } else {  // a bound outside the window (a block can span more than 64 slots: holes)
                        const int bs = block_start(L, i, 1), be = block_end(L, s, i, 1);
                        slot = be;
                        nocand = true;
                        for (int jb = i; jb < be; jb += 64) {
                            const int j = jb + ln;
                            bool c = false;
                            if (j < be) {
                                const int ej = L.E[j];
                                const int vj = ev(ej, j > 0 ? L.E[j - 1] : 0);
                                c = vj >= 0 && ((ej & EMASK) > pos || (vj == 0 && seq > L.seq[j]));
                            }
                            const uint64_t cm = __ballot(c);
                            if (cm) {
                                slot = jb + first_lane(cm);
                                nocand = false;
                                break;
                            }
                        }
                        inherit = slot == bs ? 1 : 0;
                    }
                }
            }
        }
        if (X && nocand && slot >= 0 && slot < S && s.collab && !v.local && uni(L.seq[slot]) >= LOCAL_BASE) {
            // insertingWalk's continuePredicate (mergeTree.ts:1611-1615, 1815-1828): the first segment after
            // the block is an unacked local one, so a remote insert walks on into the following leaf
            // blocks at position 0 (pending segments are 0 long and lose breakTie to it)
            int b0 = slot;
            for (;;) {
                const int b1 = block_end(L, s, b0, 1);
                int found = -1;
                for (int jb = b0; jb < b1 && found < 0; jb += 64) {
                    const int j = jb + ln;
                    bool c = false;
                    if (j < b1) {
                        const int ej = L.E[j];
                        const int vj = ev(ej, j > 0 ? L.E[j - 1] : 0);
                        c = vj >= 0 && ((ej & EMASK) > pos || (vj == 0 && seq > L.seq[j]));
                    }
                    const uint64_t cm = __ballot(c);
                    if (cm) found = jb + first_lane(cm);
                }
                if (found >= 0) {
                    slot = found;
                    inherit = slot == b0 ? 1 : 0;
                    break;
                }
                if (b1 < S && uni(L.seq[b1]) >= LOCAL_BASE && uni(L.seq[b1]) != RNONE) {
                    b0 = b1;
                    continue;
                }
                slot = b1;
                inherit = 0;
                break;
            }
            om_known = false;
            wbs = wbe = -1;
        }
#ifdef MTR_DEBUG_INSERT  // (spill experiment: the insert placement of HBM-resident documents, lane 0)
        if (G && lane_id() == 0 && S > 0)
            printf("ins op_begin %llu pos %d slot %d inherit %d nocand %d wbs %d wbe %d E[slot-1] %d E[slot] %d rlo %d rhi %d\n",
                   (unsigned long long)dd.op_begin, pos, slot, inherit, int(nocand), wbs, wbe, slot > 0 ? int(L.E[slot - 1]) : -9,
                   slot < S ? int(L.E[slot]) : -9, int(L.rlo), int(L.rhi));
#endif
        if (slot < 0) return -1;
        const bool grew = shift_right1(L, s, slot);
        if (G && !grew) wbs = wbe = -1;  // a hole was taken: overflow_fix finds the block itself
        uint32_t m = client & M_CLIENT_MASK;
        if (marker) m |= M_MARKER;
        else m |= (nl ? M_NL : 0u) | (nonl ? M_NONL : 0u);
        if (op.flags & MTR_F_NOREF) m |= M_NOREF;
        if (DL && !PM && (op.flags & MTR_F_DELTA)) m |= M_TOUCH;
        if (S == 0) {
            s.height = 1;
            m = set_bnd(m, 1);
        } else if (inherit) {
            if (!om_known) om = uniu(L.meta[slot + 1]);
            m = set_ns(set_bnd(m, bnd_of(om)), ns_of(om));
            L.meta[slot + 1] = set_ns(set_bnd(om, 0), NS_UNDEF);
        }
        L.len[slot] = len;
        L.seq[slot] = sseq;
        L.rseq[slot] = RNONE;
        L.meta[slot] = m;
        // PermutationSegment: start reset to unallocated on INSERT (permutationvector.ts:354-361) -- not for a
        // snapshot body segment (no delta callback while loading, mergeTree.ts:1410-1418)
        L.text[slot] = marker ? op.payload
                              : (PM ? ((op.flags & MTR_F_APPEND) ? op.payload : uint32_t(MTR_HANDLE_UNALLOCATED))
                                    : uint32_t(t0));
        if (!marker && !PM) s.textused = t0 + len;
        uint32_t pr = NONE32;
        if ((op.flags & MTR_F_PROPS) && op.pos2 >= 0) pr = props_apply(L, P, s, NONE32, uint32_t(op.pos2));
        pset(L, slot, pr);
        L.uid[slot] = uint32_t(s.uidnext++);
        if (G && s.chunked && lane_id() == 0) hint(L, uint32_t(s.uidnext - 1), slot);
        if (X && marker && op.payload2 != 0) {  // mapIdToSegment (mergeTree.ts:1655-1662)
            if (lane_id() == 0 && !mk_set(L, op.payload2 - 1, uint32_t(s.uidnext - 1))) s.status = MTR_ERR_CAPACITY;
            s.status = uni(s.status);
        }
        wsync();
        s.nseg = S + (grew ? 1 : 0);
        const int xbs = S == 0 ? 0 : overflow_fix(L, s, slot, wbs, wbe);
        // saveIfLocal (mergeTree.ts:1618-1637): remote segments above minSeq go to the LRU
        if (op.flags & MTR_F_APPEND) set_merge_info(L, P, s, slot, op, dd);
        if (s.collab && !v.local && seq > s.minseq) add_lru_block(L, s, xbs, uint32_t(s.uidnext - 1), seq);
        if (X && lseq > 0) pend_add(L, P, s, slot, -1, PK_INSERT, 0, lseq);  // saveIfLocal, mergeTree.ts:1618-1626
        if (G) csum_update(L, s, slot, max(L.shi, slot + 1));
        return slot;
    }

    // ------------------------------------------------------------ snapshot load
    // merge info of a snapshot segment on leaf i (SnapshotLoader.specToSegment, snapshotLoader.ts:88-128):
    // removedSeq, and removedClientIds as first remover + newest-first cons list of the others
    static MTR_COLD void set_merge_info(D& L, const KParams& P, St& s, int i, const mtr_op& op, const mtr_doc_desc& dd) {
        if (op.ref_seq >= 0) L.rseq[i] = op.ref_seq;
        const int nrem = op.min_seq;
        if (nrem > 0) {
            const gptr<const uint16_t> rl = gp(P.btext) + dd.text_base + uint32_t(op.pos1);
            uint32_t m = uniu(L.meta[i]);
            m = (m & ~(0xffu << M_FREM_SHIFT) & ~M_OVERLAP) | (enc_client(int(uniu(rl[0]))) << M_FREM_SHIFT);
            if (nrem > 1) {
                if (s.rmused + nrem - 1 > P.rcap) {
                    s.status = MTR_ERR_CAPACITY;
                    return;
                }
                uint32_t head = 0xffffffu;
                for (int k = 1; k < nrem; k++) {
                    const uint32_t cell = uint32_t(s.rmused++);
                    L.grm()[cell] = (enc_client(int(uniu(rl[k]))) << 24) | head;
                    head = cell;
                }
                m |= M_OVERLAP;
                if (lane_id() == 0 && !rm_set(L, uniu(L.uid[i]), head)) s.status = MTR_ERR_CAPACITY;
                s.status = uni(s.status);
            }
            L.meta[i] = m;
        }
        wsync();
    }

    // one header segment appended in order; the block structure is built by finish_load
    static MTR_COLD void load_leaf(D& L, const KParams& P, St& s, const mtr_op& op, const mtr_doc_desc& dd) {
        if (s.collab) {  // "Trying to reload from segments while collaborating!"
            s.status = MTR_ERR_ASSERT | 0x049;
            return;
        }
        if (s.height != 0) {  // reloadFromSegments replaces the whole tree
            s.nseg = 0;
            s.height = 0;
            s.holes = 0;
        }
        const bool marker = !PM && (op.flags & MTR_F_MARKER) != 0;
        const int len = marker ? 1 : int(op.payload2);
        const int i = s.nseg;
        const int t0 = s.textused;
        if (!marker && !PM) {
            if (t0 + len > text_end(s, P)) {
                s.status = MTR_ERR_CAPACITY;
                return;
            }
            const gptr<const uint16_t> src = gp(P.btext) + dd.text_base + op.payload;
            for (int k = lane_id(); k < len; k += 64) L.gtext()[t0 + k] = src[k];
            s.textused = t0 + len;
        }
        uint32_t m = enc_client(int(int16_t(op.client)));
        if (marker) m |= M_MARKER;
        else if (!PM) m |= M_NLQ;
        if (op.flags & MTR_F_NOREF) m |= M_NOREF;
        L.len[i] = len;
        L.seq[i] = op.seq;
        L.rseq[i] = RNONE;
        L.meta[i] = m;
        // PermutationSegment: the start handle of the spec [length, start] is kept (no reset on load)
        L.text[i] = (marker || PM) ? op.payload : uint32_t(t0);
        uint32_t pr = NONE32;
        if ((op.flags & MTR_F_PROPS) && op.pos2 >= 0) pr = props_apply(L, P, s, NONE32, uint32_t(op.pos2));
        pset(L, i, pr);
        L.uid[i] = uint32_t(s.uidnext++);
        if (X && marker && op.payload2 != 0) {  // reloadFromSegments' blockUpdate maps live markers (mergeTree.ts:297-306)
            if (lane_id() == 0 && !mk_set(L, op.payload2 - 1, uint32_t(s.uidnext - 1))) s.status = MTR_ERR_CAPACITY;
            s.status = uni(s.status);
        }
        wsync();
        s.nseg = i + 1;
        set_merge_info(L, P, s, i, op, dd);
    }

    // A run of plain header segments (text, no props, no removers) from the records lanes [t0, tend) of
    // the loop's 64-record window hold (lane t: the 8 words of record t): one lane per segment, as
    // load_leaf + set_merge_info would append them one by one.  Returns how many were appended (0: the
    // record at t0 takes the one-by-one path: a marker, props, removers, or room running short).
    static MTR_COLD int load_run(D& L, const KParams& P, St& s, const uint32_t (&ow)[8], int t0, int tend,
                               gptr<const uint16_t> btext) {
        PROF(P_LOAD);
        const int ln = lane_id();
        const uint32_t ty = ow[0] & 0xffu, fl = (ow[0] >> 8) & 0xffu;
        const bool el = ln >= t0 && ln < tend && ty == MTR_OP_LOAD &&
                        !(fl & (MTR_F_MARKER | MTR_F_PROPS | MTR_F_REL)) && int(ow[3]) <= 0;
        const uint64_t bad = __ballot(!el) & ~((uint64_t(1) << t0) - 1);
        const int cnt = (bad ? first_lane(bad) : 64) - t0;
        if (cnt <= 0) return 0;
        const bool act = ln >= t0 && ln < t0 + cnt;
        const int len = act ? int(ow[7]) : 0;
        const int incl = wave_incl_scan(len);
        const int tot = rdlane(incl, 63);
        // (the one-by-one path would neither yield for leaf room nor collect the text arena on the way)
        if (s.nseg + cnt + 3 > L.cap || s.textused + tot + 4096 > text_end(s, P)) return 0;
        if (act) {
            const int i = s.nseg + (ln - t0);
            const uint32_t t = uint32_t(s.textused + incl - len);
            const gptr<const uint16_t> src = btext + ow[6];
            for (int q = 0; q < len; q++) L.gtext()[t + q] = src[q];
            L.len[i] = len;
            L.seq[i] = int(ow[1]);
            L.rseq[i] = int(ow[2]) >= 0 ? int(ow[2]) : RNONE;
            L.meta[i] = enc_client(int(int16_t(ow[0] >> 16))) | M_NLQ | ((fl & MTR_F_NOREF) ? M_NOREF : 0u);
            L.text[i] = t;
            pset(L, i, NONE32);
            L.uid[i] = uint32_t(s.uidnext + (ln - t0));
        }
        wsync();
        s.nseg += cnt;
        s.uidnext += cnt;
        s.textused += tot;
        return cnt;
    }

    // MergeTree.reloadFromSegments (mergeTree.ts:678-728): MaxNodesInBlock - 1 = 7 children per block,
    // built bottom-up, so leaf i starts a level-l block iff 7^l divides i; leaf 0 starts every level
    static MTR_COLD void finish_load(D& L, St& s) {
        PROF(P_LOAD);
        const int S = s.nseg;
        int H = 1;
        for (int n = S; n > kMaxNodesInBlock - 1; n = (n + kMaxNodesInBlock - 2) / (kMaxNodesInBlock - 1)) H++;
        for (int i = lane_id(); i < S; i += 64) {
            int b = 0;
            if (i == 0) {
                b = H;
            } else {
                for (int64_t p = kMaxNodesInBlock - 1; b + 1 < H && i % p == 0; p *= kMaxNodesInBlock - 1) b++;
            }
            L.meta[i] = set_ns(set_bnd(L.meta[i], b), NS_UNDEF);
        }
        wsync();
        s.height = H;
        if (G && !PM && S >= kGapMin) spread(L, s, L.cap);
    }

    // markRangeRemoved / annotateRange walk (mergeTree.ts:1955-2047, 1895-1953): leaves with
    // visible length > 0 inside [start, end), on the current scan arrays, 64 leaves per round.
    // The walk stops at the first leaf whose view start (E - max(V,0), nondecreasing) is >= end.
    static MTR_DI void range_walk(D& L, const KParams& P, St& s, const View& v, int start, int end, int seq,
                                  uint32_t client, int is_remove, uint32_t pp, uint32_t comb, bool dl,
                                  bool pending = false, int plseq = 0) {
        // (pending: a local op while collaborating -- its leaves are marked M_TOUCH for pend_touched and
        // every key applies; remote ops leave keys with pending local updates alone)
        PROF(P_RANGE);
        if (end == start) return;
        const int S = s.nseg;
        const int ln = lane_id();
        const bool lru = s.collab && !v.local;
        int last_blk = -1;  // leaf-block start of the last touched leaf
        int pslot = -1;     // the pending annotate's group (created with its first segment)
        L.wlo = lower_bound_E(L, s, start + 1);
        L.whi = L.wlo;
        for (int base = L.wlo; base < S; base += 64) {
            L.whi = min(base + 64, S);
            const int j = base + ln;
            const bool in = j < S;
            const int jc = min(j, S - 1);  // unconditional (clamped) loads
            const int ej0 = L.E[jc], ep = L.E[max(jc - 1, 0)], rj = L.rseq[jc];
            uint32_t mj = L.meta[jc];
            const int vj = ev(ej0, jc > 0 ? ep : 0);
            const int ej = ej0 & EMASK;
            const uint64_t stop = __ballot(!in | (ej - max(vj, 0) >= end));
            const int lim = stop ? first_lane(stop) : 64;
            const bool act = (ln < lim) & (vj > 0);
            const uint64_t am = __ballot(act);
            if (am) {
                if (is_remove) {
                    const int rs = act ? rj : RNONE;
                    // a pending local remove a remote remove overtakes: removedClientIds.unshift(client),
                    // removedSeq = seq (mergeTree.ts:1976-1987)
                    const bool pr = X && act && rs != RNONE && rs >= LOCAL_BASE;
                    const bool ov = act && rs != RNONE && !pr;  // overlapping remove: removedClientIds.push
                    const uint64_t om = __ballot(ov | pr);
                    const int nov = __popcll(om);
                    if (s.rmused + nov > P.rcap) {
                        s.status = MTR_ERR_CAPACITY;
                        return;
                    }
                    bool full = false;
                    if (ov) {
                        const uint32_t cell = uint32_t(s.rmused + __popcll(om & lanes_below()));
                        const uint32_t uj = L.uid[j];
                        const uint32_t nxt = (mj & M_OVERLAP) ? rm_get(L, uj) : 0xffffffu;
                        L.grm()[cell] = (client << 24) | (nxt & 0xffffffu);
                        full = !rm_set(L, uj, cell);
                        mj |= M_OVERLAP;
                        L.meta[j] = mj;
                    } else if (pr) {  // the old first remover becomes removedClientIds[1]: the oldest cell
                        const uint32_t cell = uint32_t(s.rmused + __popcll(om & lanes_below()));
                        const uint32_t uj = L.uid[j];
                        L.grm()[cell] = (((mj >> M_FREM_SHIFT) & 0xffu) << 24) | 0xffffffu;
                        uint32_t t = (mj & M_OVERLAP) ? rm_get(L, uj) : 0xffffffu;
                        if (t == 0xffffffu) {
                            full = !rm_set(L, uj, cell);
                        } else {
                            while ((L.grm()[t] & 0xffffffu) != 0xffffffu) t = L.grm()[t] & 0xffffffu;
                            L.grm()[t] = (L.grm()[t] & 0xff000000u) | cell;
                        }
                        L.rseq[j] = seq;
                        mj = (mj & ~(0xffu << M_FREM_SHIFT)) | (client << M_FREM_SHIFT) | M_OVERLAP;
                        L.meta[j] = mj;
                    } else if (act) {
                        L.rseq[j] = seq;
                        mj = (mj & ~(0xffu << M_FREM_SHIFT) & ~M_OVERLAP) | (client << M_FREM_SHIFT);
                        if (dl) mj |= M_TOUCH;  // removedSegments: first removals only (mergeTree.ts:1975-2000)
                        L.meta[j] = mj;
                    }
                    if (__ballot(full)) s.status = MTR_ERR_CAPACITY;
                    s.rmused += nov;
                } else {
                    // one new property set per distinct old set in the round (memoized addProperties)
                    const uint32_t old = act ? pget(L, j) : 0u;
                    uint64_t pend = am;
                    if (X && !pending) {  // leaves with pending local annotates: one filtered set each
                        uint64_t pm = __ballot(act && (mj & (M_PEND | M_ZOMB)));
                        pend &= ~pm;
                        for (; pm; pm &= pm - 1) {
                            const int l = first_lane(pm);
                            const uint32_t pl = uniu(pd_get(L, uniu(L.uid[base + l])));
                            const PropRes r = props_apply_serial(L, P, s.propused, rdlane(old, l), pp, comb, pl);
                            s.propused = uni(r.propused);
                            if (uni(r.status) != MTR_OK) s.status = uni(r.status);
                            if (ln == l) pset(L, j, uniu(r.dst));
                            wsync();
                        }
                    }
                    while (pend) {
                        const uint32_t o = rdlane(old, first_lane(pend));
                        const bool mine = act && old == o && (!X || ((pend >> ln) & 1));
                        const uint64_t sel = __ballot(mine);
                        const uint32_t nw = props_apply(L, P, s, o, pp, comb);
                        if (mine) pset(L, j, nw);
                        pend &= ~sel;
                    }
                    if (dl && act) {  // every annotated segment is a delta segment
                        mj |= M_TOUCH;
                        L.meta[j] = mj;
                    }
                    if (X && pending) {  // addToPendingList with previousProps, in walk order (mergeTree.ts:1921-1930)
                        wsync();
                        for (uint64_t t = am; t && s.status == MTR_OK; t &= t - 1) {
                            const int l = first_lane(t);
                            pslot = pend_add(L, P, s, base + l, pslot,
                                             PK_ANNOTATE | ((comb & 7u) == MTR_COMB_REWRITE ? PK_REWRITE : 0), pp,
                                             plseq, rdlane(old, l));
                        }
                        mj = L.meta[jc];
                    }
                }
                wsync();
                if (lru) {  // addToLRUSet for every touched leaf, in leaf order: one step per leaf block (its
                    // first touched leaf), the block's other touched leaves skipped by mask
                    const uint64_t fm = __ballot(in && bnd_of(mj) >= 1);
                    uint64_t todo = am;
                    while (todo) {
                        const int l = first_lane(todo);
                        const uint64_t below = fm & ((uint64_t(2) << l) - 1);
                        const int b = below ? base + last_lane(below) : block_start(L, base, 1);
                        if (b != last_blk) {
                            last_blk = b;
                            add_lru_block(L, s, b, uniu(L.uid[base + l]), seq);
                        }
                        // the next block starts at the first block-start lane above l
                        const uint64_t above = l == 63 ? 0 : (fm & (~uint64_t(0) << (l + 1)));
                        todo = above ? (todo & (~uint64_t(0) << first_lane(above))) : 0;
                    }
                }
            }
            if (s.status != MTR_OK || stop) break;
        }
    }

    // ------------------------------------------------------------ record mode
    // draw op `idx` of document d from the synthetic recipe using this engine's exact view length
    static MTR_DI void gen_op(D& L, const KParams& P, St& s, const mtr_doc_desc& dd, int idx) {
        const gptr<mtr_op> rec = gp(P.gen_ops) + dd.op_begin + idx;
        if (idx < P.gen_grow) return;  // a pre-grown snapshot segment, written by synth_grow_kernel
        if (idx == P.gen_grow) {
            if (lane_id() == 0) {
                mtr_op z{};
                z.type = MTR_OP_START_COLLAB;
                st_struct(rec, z);
            }
            wsync();
            return;
        }
        if (lane_id() == 0) {
            mtr_op op;
            mtr_synth_state st = ld_struct<mtr_synth_state>(L.gst);
            mtr_synth_begin(&P.gen_cfg, &st, idx - P.gen_grow, &op);
            st_struct(L.gst, st);
            L.sc->gen_ref = op.ref_seq;
            L.sc->gen_client = op.client;
            st_struct(rec, op);
        }
        wsync();
        View v;
        v.ref = uni(L.sc->gen_ref);
        v.client = enc_client(uni(L.sc->gen_client));
        v.local = 0;
        const int len = view_scan(L, s, v, P.new_length_calc, 0, 0);
        if (lane_id() == 0) {
            mtr_op op = ld_struct<mtr_op>(rec);
            mtr_synth_state st = ld_struct<mtr_synth_state>(L.gst);
            mtr_synth_finish(&P.gen_cfg, &st, len, &op, P.gen_text + dd.text_base);
            st_struct(L.gst, st);
            st_struct(rec, op);
        }
        wsync();
    }

    // ------------------------------------------------------------ state load/store
    static MTR_DI void load_doc(D& L, const KParams& P, St& s, uint32_t d) {
        const gptr<const DocHdr> hp = gp((const DocHdr*)P.hdr) + d;
        {
            const DocHdr h = uni_struct(ld_struct<DocHdr>(hp));
            s.nseg = h.nseg; s.height = h.height; s.minseq = h.minseq; s.curseq = h.curseq;
            s.collab = h.collab; s.local = h.local; s.heapn = h.heapn; s.uidnext = h.uidnext;
            s.textused = h.textused; s.propused = h.propused; s.rmused = h.rmused;
            s.status = h.status;
            s.texthalf = h.texthalf;
            s.dused = DL ? h.dused : 0;
            s.holes = G ? h.holes : 0;
            s.chunked = G ? h.chunked : 0;
        }
        if (PM && s.textused == 0) {  // new HandleTable: handles = [1] (handletable.ts:24)
            if (lane_id() == 0) handles(L)[0] = 1;
            s.textused = 1;
        }
        if (lane_id() == 0) {
            L.sc->relmask = 0;
            L.sc->nrefs = gp((const DocHdr*)P.hdr)[d].nrefs;
            L.sc->fail_op = gp((const DocHdr*)P.hdr)[d].fail_op;
            L.sc->max_heap = gp((const DocHdr*)P.hdr)[d].max_heap;
            L.sc->heap_need = 0;
            L.sc->sum_s = 0;
            L.sc->sum_l = 0;
#ifdef MTR_PROF
            for (int q = 0; q < P_COUNT; q++) L.sc->prof[q] = 0;
#endif
            if (GN) st_struct(L.gst, ld_struct<mtr_synth_state>(gp(P.gen_state) + d));
        }
        if (!G) {  // stage the leaves and the heap into LDS
            const int S = s.nseg;
            const int cs = P.segcap;
            const gptr<const uint32_t> g = gp((const uint32_t*)P.seg) + size_t(d) * NF * cs;
            for (int i = lane_id(); i < S; i += 64) {
                L.len[i] = int(g[F_LEN * cs + i]);
                L.seq[i] = int(g[F_SEQ * cs + i]);
                L.rseq[i] = int(g[F_RSEQ * cs + i]);
                L.meta[i] = g[F_META * cs + i];
                L.text[i] = g[F_TEXT * cs + i];
                pset(L, i, g[F_PROPS * cs + i]);
                L.uid[i] = g[F_UID * cs + i];
            }
            const int hn = s.heapn;
            const gptr<const uint32_t> gh = gp((const uint32_t*)P.heap) + size_t(d) * 2 * P.hcap;
            for (int i = lane_id(); i <= hn; i += 64) {
                L.hseq[i] = int(gh[i]);
                L.huid[i] = gh[P.hcap + i];
            }
        }
        wsync();
        s.htop = s.heapn > 0 ? uni(L.hseq[1]) : 0;
        sup_load(L, s);
    }

    static MTR_DI void store_doc(D& L, const KParams& P, const St& s, uint32_t d, int ops_done) {
        wsync();
        if (!G) {
            const int S = s.nseg;
            const int cs = P.segcap;
            const gptr<uint32_t> g = gp(P.seg) + size_t(d) * NF * cs;
            for (int i = lane_id(); i < S; i += 64) {
                g[F_LEN * cs + i] = uint32_t(L.len[i]);
                g[F_SEQ * cs + i] = uint32_t(L.seq[i]);
                g[F_RSEQ * cs + i] = uint32_t(L.rseq[i]);
                g[F_META * cs + i] = L.meta[i];
                g[F_TEXT * cs + i] = L.text[i];
                g[F_PROPS * cs + i] = pget(L, i);
                g[F_UID * cs + i] = L.uid[i];
            }
            const int hn = s.heapn;
            const gptr<uint32_t> gh = gp(P.heap) + size_t(d) * 2 * P.hcap;
            for (int i = lane_id(); i <= hn; i += 64) {
                gh[i] = uint32_t(L.hseq[i]);
                gh[P.hcap + i] = L.huid[i];
            }
        }
        if (lane_id() == 0) {
            const gptr<DocHdr> hp = gp(P.hdr) + d;
            DocHdr h = ld_struct<DocHdr>(hp);
            h.nseg = s.nseg; h.height = s.height; h.minseq = s.minseq; h.curseq = s.curseq;
            h.collab = s.collab; h.local = s.local; h.heapn = s.heapn; h.uidnext = s.uidnext;
            h.textused = s.textused; h.propused = s.propused; h.rmused = s.rmused; h.status = s.status;
            h.op_cursor += ops_done;
            h.fail_op = L.sc->fail_op;
            h.max_heap = L.sc->max_heap;
            h.texthalf = s.texthalf;
            h.heap_need = L.sc->heap_need;
            if (DL) h.dused = s.dused;
            h.nrefs = L.sc->nrefs;
            if (G) {
                h.holes = s.holes;
                h.chunked = s.chunked;
            }
            st_struct(hp, h);
            if (GN) st_struct(gp(P.gen_state) + d, ld_struct<mtr_synth_state>(L.gst));
#ifdef MTR_PROF
            // (a buffer, not a __device__ symbol: the kernels live in several code objects)
            if (P.prof)
                for (int q = 0; q < P_COUNT; q++) atomicAdd(&P.prof[q], L.sc->prof[q]);
#endif
            if (ops_done) {  // this document's counters (no cross-document atomics)
                const gptr<unsigned long long> st = gp(P.stat_ops) + size_t(d) * 4;
                st[0] += (unsigned long long)ops_done;
                st[1] += L.sc->sum_s;
                st[2] += L.sc->sum_l;
            }
        }
    }

    // the HBM-resident layout's pointers alone (the team's helper waves: they write nothing carve sets up)
    static MTR_DI void carve_ptrs(D& L, char* smem, const KParams& P, uint32_t d) {
        if constexpr (G) {
            const gptr<uint32_t> g = gp(P.seg) + size_t(d) * NF * P.segcap;
            L.len = (A<int>)(g + F_LEN * P.segcap);
            L.seq = (A<int>)(g + F_SEQ * P.segcap);
            L.rseq = (A<int>)(g + F_RSEQ * P.segcap);
            L.meta = (A<uint32_t>)(g + F_META * P.segcap);
            L.text = (A<uint32_t>)(g + F_TEXT * P.segcap);
            L.props = (A<uint32_t>)(g + F_PROPS * P.segcap);
            L.uid = (A<uint32_t>)(g + F_UID * P.segcap);
            const gptr<uint32_t> sx = gp(P.scratch) + size_t(d) * 2 * P.segcap;
            L.E = (A<int>)(sx);
            const gptr<uint32_t> gh = gp(P.heap) + size_t(d) * 2 * P.hcap;
            L.hseq = (A<int>)(gh);
            L.huid = (A<uint32_t>)(gh + P.hcap);
            L.cap = P.segcap;
            L.lhcap = P.hcap;
            L.sc = (lptr<Sc>)(smem);
            L.gst = (lptr<mtr_synth_state>)(smem + ((sizeof(Sc) + 15) & ~size_t(15)));
            L.sx = (lptr<int>)(smem + kScBytes + kTeamBytes);
            L.rtmask = P.rtab - 1;
            L.dcap = 0;
        }
    }
    static MTR_DI void carve(D& L, char* smem, const KParams& P, uint32_t d) {
        if (G) {  // every array lives in the document's HBM slab
            const gptr<uint32_t> g = gp(P.seg) + size_t(d) * NF * P.segcap;
            L.len = (A<int>)(g + F_LEN * P.segcap);
            L.seq = (A<int>)(g + F_SEQ * P.segcap);
            L.rseq = (A<int>)(g + F_RSEQ * P.segcap);
            L.meta = (A<uint32_t>)(g + F_META * P.segcap);
            L.text = (A<uint32_t>)(g + F_TEXT * P.segcap);
            L.props = (A<uint32_t>)(g + F_PROPS * P.segcap);
            L.uid = (A<uint32_t>)(g + F_UID * P.segcap);
            const gptr<uint32_t> sx = gp(P.scratch) + size_t(d) * 2 * P.segcap;
            L.E = (A<int>)(sx);
            const gptr<uint32_t> gh = gp(P.heap) + size_t(d) * 2 * P.hcap;
            L.hseq = (A<int>)(gh);
            L.huid = (A<uint32_t>)(gh + P.hcap);
            L.cap = P.segcap;
            L.lhcap = P.hcap;
            L.sc = (lptr<Sc>)(smem);
            L.gst = (lptr<mtr_synth_state>)(smem + ((sizeof(Sc) + 15) & ~size_t(15)));
            L.sx = (lptr<int>)(smem + kScBytes + kTeamBytes);
            for (int q = lane_id(); q < 2 * sup_rows(L.cap); q += 64) L.sx[sup_rows(L.cap) + q] = 0;  // fills, marks
            if (lane_id() == 0) L.sc->sepoch = 0;
        } else {
            const int cap = CAP > 0 ? CAP : P.cap, lhcap = P.lhcap;
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
            if constexpr (NOPROPS) L.props = (A<uint32_t>)(p);  // (never read: pget / pset)
            else L.props = (A<uint32_t>)(take(4 * size_t(cap)));
            L.uid = (A<uint32_t>)(take(4 * size_t(cap)));
            L.E = (A<int>)(take(4 * size_t(cap)));
            // (Sc ahead of the heap: with a compile-time capacity its address is a constant, not an SGPR)
            L.sc = (lptr<Sc>)(take(sizeof(Sc)));
            L.gst = (lptr<mtr_synth_state>)(GN ? take(sizeof(mtr_synth_state)) : p);
            L.hseq = (A<int>)(take(4 * size_t(lhcap)));
            L.huid = (A<uint32_t>)(take(4 * size_t(lhcap)));
            L.sx = (lptr<int>)(p);
            L.cap = cap;
            L.lhcap = lhcap;
        }
        L.rtmask = P.rtab - 1;
        unsigned long long delta = (unsigned long long)P.delta;
        L.dcap = 0;
        if (P.doff) {
            const uint64_t o = gp(P.doff)[d];
            delta = (unsigned long long)(P.delta + o * 4);
            L.dcap = int(gp(P.doff)[d + 1] - o);
        }
        if (lane_id() == 0) {
            const unsigned long long rm = (unsigned long long)(P.rm + size_t(d) * (size_t(P.rcap) + 2 * size_t(P.rtab)));
            L.sc->cp[CP_TEXT] = (unsigned long long)(P.text + size_t(d) * P.tcap);
            L.sc->cp[CP_PROP] = (unsigned long long)(P.prop + size_t(d) * P.pcap);
            L.sc->cp[CP_RM] = rm;
            L.sc->cp[CP_RT] = rm + 4ull * uint32_t(P.rcap);
            L.sc->cp[CP_DELTA] = delta;
            L.sc->cp[CP_POFF] = (unsigned long long)P.propop_off;
            L.sc->cp[CP_PKV] = (unsigned long long)P.propop_kv;
            L.sc->cp[CP_KIX] = (unsigned long long)P.key_index;
            L.sc->cp[CP_VEQ] = (unsigned long long)P.val_eq;
            L.sc->cp[CP_HDR] = (unsigned long long)(P.hdr + d);
            L.sc->cp[CP_PEND] = (unsigned long long)(P.pend ? P.pend + size_t(d) * kPendRing * 4 : nullptr);
            L.sc->cp[CP_CSUM] = (unsigned long long)(P.csum ? P.csum + size_t(d) * csum_ints(P.segcap) : nullptr);
            L.sc->cp[CP_UMAP] = (unsigned long long)(P.umap ? P.umap + size_t(d) * 2 * P.segcap : nullptr);
            L.sc->cp[CP_REFS] = (unsigned long long)(P.refs ? P.refs + size_t(d) * 3 * size_t(P.refcap) : nullptr);
            L.sc->refcap = P.refs ? P.refcap : 0;
        }
        wsync();
    }

    // ------------------------------------------------------------ delta ranges
    // The ranges of a SequenceDeltaEvent (sequenceDeltaEvent.ts): every M_TOUCH leaf in tree order
    // with its position in the local view (Client.getPosition: removed segments count 0) and its
    // cachedLength; clears the marks.
    // one mtr_delta record written by lane 0 (wave-uniform bookkeeping)
    static MTR_DI void put_record(D& L, St& s, int op, int a, int b, uint32_t kind) {
        if (s.dused >= L.dcap) {
            s.status = MTR_ERR_CAPACITY;
            return;
        }
        if (lane_id() == 0) {
            const gptr<uint32_t> r = L.gdelta() + 4 * size_t(s.dused);
            r[0] = uint32_t(op);
            r[1] = uint32_t(a);
            r[2] = uint32_t(b);
            r[3] = kind;
        }
        s.dused++;
    }

    static MTR_DI void emit_deltas(D& L, const KParams& P, St& s, int gidx, uint32_t kind) {
        const int S = s.nseg;
        const int ln = lane_id();
        int carry = 0;
        for (int base = 0; base < S; base += 64) {
            const int i = base + ln;
            const bool in = i < S;
            uint32_t m = 0;
            int len = 0, rs = RNONE;
            if (in) {
                m = L.meta[i];
                len = L.len[i];
                rs = L.rseq[i];
            }
            const int loc = in && rs == RNONE ? len : 0;
            const int inc = wave_incl_scan(loc);
            const bool t = in && (m & M_TOUCH);
            const uint64_t tm = __ballot(t);
            if (tm) {
                const int n = __popcll(tm);
                if (s.dused + n > L.dcap) {
                    s.status = MTR_ERR_CAPACITY;
                    return;
                }
                if (t) {
                    const gptr<uint32_t> r = L.gdelta() + 4 * size_t(s.dused + __popcll(tm & lanes_below()));
                    r[0] = uint32_t(gidx);
                    r[1] = uint32_t(carry + inc - loc);
                    r[2] = uint32_t(len);
                    r[3] = kind;
                    L.meta[i] = m & ~M_TOUCH;
                }
                s.dused += n;
            }
            carry += rdlane(inc, 63);
        }
        wsync();
    }

    // ------------------------------------------------------------ one op
    // the B_op model's counters: every op but snapshot-load appends and relative-position /
    // handle-table records is a flat pass over the leaves present before it; text inserts add their units
    static MTR_DI bool counts_s(const mtr_op& op) {
        return op.type != MTR_OP_LOAD && op.type != MTR_OP_RELPOS && op.type != MTR_OP_HANDLES;
    }
    static MTR_DI bool counts_l(const mtr_op& op) {
        return (op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT) && !(op.flags & MTR_F_MARKER) && !PM &&
               !(op.flags & MTR_F_APPEND);
    }
    // the document stops at op gidx (DocHdr.fail_op)
    static MTR_DI void set_fail(D& L, int gidx) {
        if (lane_id() == 0) L.sc->fail_op = gidx;
    }
    // Client.applyMsg for one member op (client.ts:858-887): dispatch, zamboni after the op, then
    // updateSeqNumbers on the message's last member op.  Returns false when the document stops
    // (s.status != MTR_OK; s.fail_op = gidx).
    static MTR_DI bool apply_op(D& L, const KParams& P, St& s, const mtr_op& op, const mtr_doc_desc& dd, bool pre,
                                uint32_t pf, int gidx) {
        PROF_T0(_t_pre);
        if (DL) s.cur_op = gidx;
        // positions resolved by the MTR_OP_RELPOS records ahead of this op (getValidOpRange, client.ts:527-545)
        int pos1 = op.pos1, pos2 = op.pos2;
        if (X && (op.flags & MTR_F_REL)) {
            const int rm = uni(L.sc->relmask);
            if (rm & 1) pos1 = uni(L.sc->rel[0]);
            if ((rm & 2) && op.type != MTR_OP_INSERT) pos2 = uni(L.sc->rel[1]);
        }
        // (record mode never yields: ops are drawn once; matrix pairs never do: their launches have
        // room for every op)
        if (!G && !GN && !PM && s.nseg + 2 >= L.cap && L.cap < P.segcap) return false;  // yield: more leaf room
        if (!G && !GN && s.collab && L.lhcap < P.hcap) {
            // LRU pushes this op can make (one per touched leaf block): if the launch's LDS heap
            // could overflow, stop before the op and ask the next launch for a larger heap
            int need = 0;
            if (op.type == MTR_OP_INSERT) need = 1;
            else if (op.type == MTR_OP_REMOVE || op.type == MTR_OP_ANNOTATE) need = min(max(pos2 - pos1, 0), s.nseg + 2);
            else if (X && op.type == MTR_OP_ACK && L.gpend()) {  // one push per member at most
                const int hd = uni(L.ghdr()->phead);
                if (hd != uni(L.ghdr()->ptail)) need = min(int(uniu(L.gpend()[4 * (hd % kPendRing) + 1])), s.nseg + 2);
            }
            if (need && s.heapn + need + 1 >= L.lhcap) {
                L.sc->heap_need = s.heapn + need + 2;
                return false;
            }
        }
        if (!PM) {  // text arena: keep room for this op's text plus zamboni merge copies
            const int need = int(op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT ? op.payload2 : 0) + 4096;
            if (s.textused + need > text_end(s, P)) text_gc(L, P, s);
        }
        if (s.nseg + 2 >= L.cap) s.status = MTR_ERR_CAPACITY;  // every op adds at most two leaves
        if (s.status != MTR_OK) {
            set_fail(L, gidx);
            return false;
        }
        if (X && (op.flags & MTR_F_REL)) {  // consumed
            if (lane_id() == 0) L.sc->relmask = 0;
            wsync();
        }
        if (op.type == MTR_OP_LOAD) {  // SnapshotLoader.loadHeader segment
            PROF(P_LOAD);
            load_leaf(L, P, s, op, dd);
            if (s.status != MTR_OK) {
                set_fail(L, gidx);
                return false;
            }
            return true;
        }
        if (s.height == 0) finish_load(L, s);
        // holes ran low, or the slots fill the slab while holes remain, or zamboni shrank the document so
        // far that holes outnumber its leaves threefold (every slot-order pass -- view scans, block bounds,
        // scour -- would step over them: C5's documents keep ~14k of 200k leaves)
        if (G && !PM && s.nseg >= kGapMin &&
            (s.holes * 64 < s.nseg || (s.holes && s.nseg + 2 >= L.cap) || s.holes > 3 * (s.nseg - s.holes)))
            spread(L, s, L.cap);
        const bool local_op = op.type >= MTR_OP_LOCAL_INSERT && op.type <= MTR_OP_LOCAL_ANNOTATE;
        int zop = 0;
        View v;
        int seq = op.seq;
        int sseq = 0, lseq = 0;  // the seq an inserted leaf keeps; localSeq of a pending local op
        uint32_t client = enc_client(int(int16_t(op.client)));
        if (local_op) {
            v.ref = s.curseq;
            v.local = 1;
            if (s.collab) {  // a pending local op (seq = UnassignedSequenceNumber, the local client)
                if (!X) {  // (the local-op path lives in the X instantiations only)
                    s.status = MTR_ERR_UNSUPPORTED;
                    set_fail(L, gidx);
                    return false;
                }
                lseq = uni(L.ghdr()->lseq) + 1;  // ++collabWindow.localSeq (mergeTree.ts:1407, 1909, 1970)
                if (lane_id() == 0) L.ghdr()->lseq = lseq;
                v.client = uint32_t(s.local);
                client = uint32_t(s.local);
                seq = TIE_LOCAL;
                sseq = LOCAL_BASE + lseq;
            } else {
                v.client = CL_LOCAL;
                seq = 0;
                client = CL_LOCAL;
            }
        } else {
            // a snapshot body append walks at (UniversalSequenceNumber, segment client)
            v.ref = (op.flags & MTR_F_APPEND) ? 0 : op.ref_seq;
            v.client = client;
            v.local = (!s.collab || uint32_t(s.local) == client) ? 1 : 0;
        }
        PROF_ADD(P_PRE, _t_pre);
        // (each op type calls the view scan itself: one hoisted call site measured 2.5 % slower at C3)
        if (X && op.type == MTR_OP_RELPOS) view_scan(L, s, v, P.new_length_calc, 0, 0);
        switch (op.type) {
            case MTR_OP_INSERT:
            case MTR_OP_LOCAL_INSERT: {
                int pos = pos1;
                if (op.flags & MTR_F_APPEND) pos = local_length(L, s);
                view_scan(L, s, v, P.new_length_calc, pos, pos, true);
                int force = -1;  // PermutationVector.insertRelative (SharedMatrix undo): in front of tracked leaf pos2
                if (PM && local_op && op.pos2 >= 0) {
                    force = track_ref_slot(L, P, s, uint32_t(op.pos2));
                    if (force < 0) {
                        s.status = MTR_ERR_BAD_OP;
                        break;
                    }
                } else {
                    split_at(L, P, s, pos);
                }
                const int at = insert_at(L, P, s, v, op, pos, seq, client, dd, pre, pf, lseq ? sseq : seq, lseq, force);
                if (PM && local_op && at >= 0 && s.status == MTR_OK) {  // tracking groups (SharedMatrix undo)
                    if (op.payload) track_link(L, P, s, at, op.payload);      // VectorUndoProvider.record
                    if (op.pos2 >= 0 && s.status == MTR_OK) {                 // insertRelative's replacement
                        if (!op.payload) s.status = MTR_ERR_BAD_OP;
                        else track_transfer(L, P, s, at, uint32_t(op.pos2));
                    }
                }
                zop = s.collab && !local_op;
                break;
            }
            case MTR_OP_REMOVE:
            case MTR_OP_LOCAL_REMOVE:
            case MTR_OP_ANNOTATE:
            case MTR_OP_LOCAL_ANNOTATE: {
                const int is_remove = op.type == MTR_OP_REMOVE || op.type == MTR_OP_LOCAL_REMOVE;
                view_scan(L, s, v, P.new_length_calc, min(pos1, pos2), max(pos1, pos2), true);
                split_at(L, P, s, pos1);
                split_at(L, P, s, pos2);
                // a matrix vector's local remove with tracking bits: its delta segments join those groups
                const bool track = PM && op.type == MTR_OP_LOCAL_REMOVE && op.payload != 0;
                if (X && lseq) {  // pending: removedSeq = LOCAL_BASE + localSeq; the touched leaves join a group
                    range_walk(L, P, s, v, pos1, pos2, sseq, client, is_remove, op.payload, is_remove ? 0u : op.payload2,
                               is_remove != 0, true, lseq);
                    if (track && s.status == MTR_OK) track_touched(L, P, s, op.payload, false);
                    if (s.status == MTR_OK && is_remove) pend_touched(L, P, s, PK_REMOVE, 0u, lseq);
                } else {
                    range_walk(L, P, s, v, pos1, pos2, seq, client, is_remove, op.payload,
                               (op.type == MTR_OP_ANNOTATE || (X && op.type == MTR_OP_LOCAL_ANNOTATE)) ? op.payload2 : 0u,
                               (DL && !PM && (op.flags & MTR_F_DELTA) != 0) || track);
                    if (track && s.status == MTR_OK) track_touched(L, P, s, op.payload, true);
                }
                if (X && is_remove && !lseq && s.status == MTR_OK && nrefs(L)) ref_slide_walk(L, s, seq);
                if (G && is_remove) csum_update(L, s, L.wlo, L.whi);
                zop = s.collab && !local_op;
                break;
            }
            case MTR_OP_SEQ:
                break;
            case MTR_OP_ROLLBACK:  // Client.rollback (client.ts:421-423) of the newest pending local op
                if (!X || !s.collab) {
                    s.status = MTR_ERR_BAD_OP;
                    break;
                }
                rollback(L, P, s, int(op.payload2), op.payload, uint32_t(op.pos1));
                break;
            case MTR_OP_REGENERATE:  // Client.regeneratePendingOp (client.ts:917-960) of the oldest pending op
                // (a matrix vector too: SharedMatrix.reSubmitCore, matrix.ts:553-570)
                if (!X || !DL || !s.collab) {
                    s.status = MTR_ERR_BAD_OP;
                    break;
                }
                regenerate(L, P, s, int(op.payload2), gidx);
                break;
            case MTR_OP_ACK:  // Client.applyMsg of this client's own message (client.ts:866-869)
                if (!X || !s.collab) {
                    s.status = MTR_ERR_BAD_OP;
                    break;
                }
                ack(L, s, int(op.payload2), op.seq);
                zop = 1;  // ackPendingSegment ends with zamboniSegments (mergeTree.ts:1318-1320)
                break;
            case MTR_OP_HANDLES: {  // HandleTable.load (handletable.ts:88): handles = the summary's array
                const int n = op.pos1;
                if (!X || !PM || s.collab || n < 1) {
                    s.status = MTR_ERR_BAD_OP;
                } else if (n > handle_cap(P)) {
                    s.status = MTR_ERR_CAPACITY;
                } else {
                    load_handles(gp(P.btext) + dd.text_base + op.payload, handles(L), n);
                    s.textused = n;
                    wsync();
                }
                break;
            }
            case MTR_OP_RELPOS: {  // posFromRelativePos, mergeTree.ts:1371-1395, for the next (MTR_F_REL) op
                // the marker's getPosition (mergeTree.ts:768-785) at the op's view: the view lengths of the
                // leaves ahead of it, 0 once zamboni unlinked it; then + cachedLength (1) + offset, or
                // - offset when `before`; -1 when no marker is mapped to the ordinal
                const uint64_t mu = X ? mk_look(L.grt(), uint32_t(L.rtmask), uint32_t(op.pos1)) : 0;
                int p = -1;
                if (mu >> 32) {
                    const int x = find_uid(L, s, uint32_t(mu));
                    if (G && L.rhi > 0 && x > 0) materialize(L, s, v, P.new_length_calc, (x - 1) >> 6, (x - 1) >> 6);
                    p = x > 0 ? (uni(L.E[x - 1]) & EMASK) : 0;
                    const int off = (op.payload2 & MTR_REL_OFFSET) ? int(op.payload) : 0;
                    p = (op.payload2 & MTR_REL_BEFORE) ? p - off : p + 1 + off;
                }
                if (p < 0) {
                    s.status = MTR_ERR_UNSUPPORTED;  // the reference goes on with position -1
                } else {
                    const int w = op.pos2 == 2 ? 1 : 0;
                    if (lane_id() == 0) {
                        L.sc->rel[w] = p;
                        L.sc->relmask |= 1 << w;
                    }
                    wsync();
                }
                break;
            }
            case MTR_OP_TRACK:  // TrackingGroup.unlink (SharedMatrix undo; include/mtr_types.h "Tracking groups")
                if (!X || !PM) s.status = MTR_ERR_BAD_OP;
                else track_clear(L, s, op.pos1 < 0 ? NONE32 : uint32_t(op.pos1), op.payload);
                break;
            case MTR_OP_REF_CREATE:  // a local reference
                if (!X || PM) s.status = MTR_ERR_BAD_OP;
                else ref_create(L, P, s, op);
                break;
            case MTR_OP_REF_REMOVE:
                if (!X || PM) s.status = MTR_ERR_BAD_OP;
                else ref_remove(L, s, op.payload);
                break;
            case MTR_OP_REF_ACK:  // IntervalCollection.ackInterval of one endpoint
                if (!X || PM) s.status = MTR_ERR_BAD_OP;
                else ref_ack(L, s, op.payload);
                break;
            case MTR_OP_REBASE_POS:  // IntervalCollection.rebasePositionWithSegmentSlide / SharedMatrix.rebasePosition
                if (!X || !DL || !s.collab) s.status = MTR_ERR_BAD_OP;
                else rebase_pos(L, s, op, gidx);
                break;
            case MTR_OP_LSEQ:  // IntervalCollection.getNextLocalSeq: ++collabWindow.localSeq
                if (!X || PM) {
                    s.status = MTR_ERR_BAD_OP;
                } else {
                    const int ls = uni(L.ghdr()->lseq);
                    if (lane_id() == 0) L.ghdr()->lseq = ls + 1;
                    wsync();
                }
                break;
            case MTR_OP_START_COLLAB:
                if (!s.collab) {
                    s.collab = 1;
                    s.local = int(enc_client(int(int16_t(op.client))));
                    s.minseq = op.min_seq;
                    s.curseq = op.seq;
                    s.heapn = 0;
                }
                break;
            default:
                s.status = MTR_ERR_BAD_OP;
                break;
        }
        PROF_T0(_t_post);
        // mergeTreeDeltaCallback (mergeTree.ts:1414, 1943, 2028) fires before zamboni
        if (DL && !PM && (op.flags & MTR_F_DELTA) && s.status == MTR_OK &&
            (op.type == MTR_OP_INSERT || op.type == MTR_OP_REMOVE || op.type == MTR_OP_ANNOTATE))
            emit_deltas(L, P, s, gidx, op.type);
        // zamboniSegments after the op (mergeTree.ts:1420-1426, 1948-1952, 2042-2046), then
        // updateSeqNumbers, whose minSeq advance runs it again (mergeTree.ts:1037-1042)
        const bool upd = !local_op && op.type != MTR_OP_START_COLLAB && (op.flags & MTR_F_LAST);
        for (int phase = 0; phase < 2; phase++) {
            int zrun = zop;
            if (phase == 1) {
                if (!upd || s.status != MTR_OK) break;
                PROF(P_UPDSEQ);
                zrun = update_seq(s, op.min_seq, op.seq);
            }
            if (zrun) zamboni(L, P, s);
        }
        PROF_ADD(P_POST, _t_post);
        if (s.status != MTR_OK) {
            set_fail(L, gidx);
            return false;
        }
        return true;
    }

    // ------------------------------------------------------------ per-document driver
    static MTR_DI void run(char* smem, const KParams& P, uint32_t d) {
        const mtr_doc_desc dd = uni_struct(ld_struct<mtr_doc_desc>(gp(P.docs) + d));
        const int cursor = uni(gp(P.hdr)[d].op_cursor);
        int n_ops = min(int(dd.op_count) - cursor, P.ops_this_launch);
        if (n_ops <= 0 || uni(gp(P.hdr)[d].status) != MTR_OK) return;
        // a document loading header segments (one lane each, load_run) takes 64 launches' worth of records
        if (!GN && !PM && (uniu(((gptr<const uint32_t>)(gp(P.ops) + dd.op_begin + cursor))[0]) & 0xffu) == MTR_OP_LOAD)
            n_ops = min(int(dd.op_count) - cursor, 64 * P.ops_this_launch);
        if (P.dkind && uniu(gp(P.dkind)[d]) != 0) {  // a cols vector has no op list of its own
            if (lane_id() == 0) {
                gp(P.hdr)[d].status = MTR_ERR_BAD_OP;
                gp(P.hdr)[d].fail_op = cursor;
            }
            return;
        }
        D L;
        carve(L, smem, P, d);
        St s;
        load_doc(L, P, s, d);
        const gptr<const mtr_op> ops = gp(P.ops) + dd.op_begin + cursor;
        const gptr<const uint16_t> btext = gp(P.btext) + dd.text_base;
        const int ln = lane_id();
        // lane t holds the 8 words of op (chunk + t); the next op's text is prefetched into `pf`
        uint32_t ow[8];
        uint32_t pf = 0, npf = 0;
        int pre = 0, npre = 0;  // (ints, not bools: a bool live across the loop is a 64-bit lane mask)
        // the B_op counters accumulate in VGPRs (the scalar unit is the bottleneck), Sc at the end
        uint32_t acc_s = 0, acc_l = 0;
        int done = 0;
        for (int k = 0; k < n_ops; k++) {
            PROF(P_OP);
            mtr_op op;
            if (GN) {
                gen_op(L, P, s, dd, cursor + k);
                op = uni_struct(ld_struct<mtr_op>(ops + k));
                pre = 0;
            } else {
                if ((k & 63) == 0) {  // (unconditional, clamped loads: no exec-mask blocks around them)
                    const gptr<const uint32_t> w = (gptr<const uint32_t>)(ops + min(k + ln, n_ops - 1));
#pragma unroll
                    for (int q = 0; q < 8; q++) ow[q] = w[q];
                    npre = 0;
                }
                uint32_t wv[8];
#pragma unroll
                for (int q = 0; q < 8; q++) wv[q] = rdlane(ow[q], k & 63);
                __builtin_memcpy(&op, wv, sizeof(op));
                pre = npre;
                pf = npf;
                npre = 0;
                const int t1 = (k + 1) & 63;
                if (t1 != 0 && k + 1 < n_ops) {  // issue the next insert's text loads now
                    const uint32_t w0 = rdlane(ow[0], t1), len1 = rdlane(ow[7], t1), off1 = rdlane(ow[6], t1);
                    const uint32_t ty = w0 & 0xffu, fl = (w0 >> 8) & 0xffu;
                    if ((ty == MTR_OP_INSERT || ty == MTR_OP_LOCAL_INSERT) && !(fl & MTR_F_MARKER) && len1 <= 64) {
                        npre = 1;
                        npf = uint32_t(ln) < len1 ? uint32_t(btext[off1 + ln]) : 0u;
                    }
                }
            }
            if (!GN && !PM && op.type == MTR_OP_LOAD && s.height == 0 && !s.collab && s.status == MTR_OK) {
                // a run of header segments: one lane each
                const int w0 = k - (k & 63);
                const int cnt = load_run(L, P, s, ow, k & 63, min(64, n_ops - w0), btext);
                if (cnt > 0) {
                    k += cnt - 1;
                    done = k + 1;
                    npre = 0;
                    continue;
                }
            }
            const uint32_t nseg0 = uint32_t(s.nseg);
            if (!apply_op(L, P, s, op, dd, pre != 0, pf, cursor + k)) break;
            done = k + 1;
            const uint32_t cs = counts_s(op) ? nseg0 : 0u, cl = counts_l(op) ? op.payload2 : 0u;
            acc_s += cs;
            acc_l += cl;
            asm("" : "+v"(acc_s), "+v"(acc_l));
        }
        if (lane_id() == 0) {
            L.sc->sum_s += acc_s;
            L.sc->sum_l += acc_l;
        }
        // a launch never ends between MTR_OP_RELPOS records and their op: the next one re-runs them
        if (X) done -= __popc(uint32_t(uni(L.sc->relmask)));
        // a batch that ends with header segments: build the tree now (queries read it next)
        if (s.height == 0 && s.status == MTR_OK && cursor + done >= int(dd.op_count)) finish_load(L, s);
        text_flush(L);    // the last merge chain's text
        sup_flush(L, s);  // the superchunk figures the launch's ops left stale, back to HBM
        store_doc(L, P, s, d, done);
    }

    // ------------------------------------------------------------ SharedMatrix
    // one op of vector La (its partner Lo): the merge-tree op; a local row / col op then brings the partner's
    // localSeq along (submitVectorMessage, matrix.ts:321-345; assert 0x01c: this vector's is never behind)
    static MTR_DI bool vector_op(D& La, D& Lo, const KParams& P, St& sa, const mtr_op& op, const mtr_doc_desc& dd,
                                 int gidx, unsigned long long& acc_s) {
        const int n0 = sa.nseg;
        bool ok = apply_op(La, P, sa, op, dd, false, 0, gidx);
        if (ok && counts_s(op)) acc_s += (unsigned long long)n0;
        if (ok && sa.collab && op.type >= MTR_OP_LOCAL_INSERT && op.type <= MTR_OP_LOCAL_ANNOTATE) {
            const int la = uni(La.ghdr()->lseq), lo = uni(Lo.ghdr()->lseq);
            if (la < lo) {
                sa.status = MTR_ERR_ASSERT | 0x01c;
                set_fail(La, gidx);
                ok = false;
            } else if (lane_id() == 0) {
                Lo.ghdr()->lseq = la;
            }
            wsync();
        }
        return ok;
    }
    // PermutationVector.adjustPosition (permutationvector.ts:232-247): getContainingSegment at the
    // op's (refSeq, clientId) view (mergeTree.ts:795-813), undefined for a removed segment, else
    // its local-view position (getPosition, mergeTree.ts:768-785) plus the offset.  -1 = undefined.
    // Returns the leaf index (-1 = undefined) and the offset in it; handle_at finishes the job.
    static MTR_DI View local_view(const St& s) {
        View v;
        v.ref = s.curseq;
        v.client = uint32_t(s.local);
        v.local = 1;
        return v;
    }
    // (i, before: the leaf whose view range holds pos and the view length before it, from find2)
    static MTR_DI int adjust_position(D& L, St& s, int pos, int i, int before, int& off) {
        if (i >= s.nseg) return -1;
        if (uni(L.rseq[i]) != RNONE) return -1;
        off = pos - before;
        return i;
    }
    // getAllocatedHandle of the adjusted position (leaf i, offset off): at the local view that
    // position lies in the same (not removed, visible) leaf at the same offset, so a leaf that has
    // a handle answers start + off without a local-view scan; otherwise the local position is the
    // local-view length of the leaves before i (every leaf is acked: those not removed) plus off
    static MTR_DI int handle_at(D& L, const KParams& P, St& s, int i, int off) {
        const uint32_t t = uniu(L.text[i]);
        if (t != uint32_t(MTR_HANDLE_UNALLOCATED)) return int(t) + off;
        prefix(L, s, local_view(s), P.new_length_calc);
        return allocated_handle(L, P, s, (i > 0 ? (uni(L.E[i - 1]) & EMASK) : 0) + off, true);
    }
    // PermutationVector.getAllocatedHandle (permutationvector.ts:209-230) at the local view: a
    // segment without a handle is split to [pos, pos + 1) (walkSegments with splitRange ->
    // MergeTree.mapRange, mergeTree.ts:2451-2469: `if (start)` skips the split at 0) and that
    // one-position segment gets the next handle (HandleTable.allocate)
    static MTR_DI int allocated_handle(D& L, const KParams& P, St& s, int pos, bool scanned) {
        if (!scanned) prefix(L, s, local_view(s), P.new_length_calc);
        {
            const int i = lower_bound_E(L, s, pos + 1);
            if (i >= s.nseg) {  // "Trying to get handle of out-of-bounds position!"
                s.status = MTR_ERR_ASSERT | 0x027;
                return -1;
            }
            const uint32_t t = uniu(L.text[i]);
            if (t != uint32_t(MTR_HANDLE_UNALLOCATED))  // already has a handle: segment.start + offset
                return int(t) + pos - (i > 0 ? (uni(L.E[i - 1]) & EMASK) : 0);
        }
        if (pos) split_at(L, P, s, pos);
        split_at(L, P, s, pos + 1);
        const int i = lower_bound_E(L, s, pos + 1);
        const int h = alloc_handle(L, P, s);
        if (s.status != MTR_OK) return -1;
        L.text[i] = uint32_t(h);
        wsync();
        return h;
    }

    // record mode for a matrix pair: draw op `idx` from the SharedMatrix recipe
    // (mtr_synth_matrix_finish) with the writer's exact view lengths of both vectors -- the same
    // lengths the oracle's generator takes from nodeLength(root, refSeq, clientId)
    static MTR_DI void gen_pair_op(D& L0, D& L1, const KParams& P, St& s0, St& s1, const mtr_doc_desc& dd, int idx) {
        const gptr<mtr_op> rec = gp(P.gen_ops) + dd.op_begin + idx;
        if (idx == 0) {
            if (lane_id() == 0) {
                mtr_op z{};
                z.type = MTR_OP_START_COLLAB;
                st_struct(rec, z);
            }
            wsync();
            return;
        }
        if (lane_id() == 0) {
            mtr_op op;
            mtr_synth_state st = ld_struct<mtr_synth_state>(L0.gst);
            mtr_synth_begin(&P.gen_cfg, &st, idx, &op);
            st_struct(L0.gst, st);
            L0.sc->gen_ref = op.ref_seq;
            L0.sc->gen_client = op.client;
            st_struct(rec, op);
        }
        wsync();
        View v;
        v.ref = uni(L0.sc->gen_ref);
        v.client = enc_client(uni(L0.sc->gen_client));
        v.local = 0;
        prefix(L0, s0, v, P.new_length_calc);
        const int lr = s0.nseg > 0 ? (uni(L0.E[s0.nseg - 1]) & EMASK) : 0;
        prefix(L1, s1, v, P.new_length_calc);
        const int lc = s1.nseg > 0 ? (uni(L1.E[s1.nseg - 1]) & EMASK) : 0;
        if (lane_id() == 0) {
            mtr_op op = ld_struct<mtr_op>(rec);
            mtr_synth_state st = ld_struct<mtr_synth_state>(L0.gst);
            mtr_synth_matrix_finish(&P.gen_cfg, &st, lr, lc, &op);
            st_struct(L0.gst, st);
            st_struct(rec, op);
        }
        wsync();
    }

    // A matrix pair: the rows vector's op list drives the rows (L0, s0) and cols (L1, s1)
    // PermutationVectors (SharedMatrix.processCore, matrix.ts:636-693, remote branch).
    static MTR_DI void run_pair(char* smem, size_t region, const KParams& P, uint32_t d) {
        const uint32_t d1 = uniu(gp(P.dpart)[d]);
        const mtr_doc_desc dd = uni_struct(ld_struct<mtr_doc_desc>(gp(P.docs) + d));
        const int cursor = uni(gp(P.hdr)[d].op_cursor);
        const int n_ops = min(int(dd.op_count) - cursor, P.ops_this_launch);
        if (n_ops <= 0 || uni(gp(P.hdr)[d].status) != MTR_OK || uni(gp(P.hdr)[d1].status) != MTR_OK) return;
        D L0, L1;
        carve(L0, smem, P, d);
        carve(L1, smem + region, P, d1);
        St s0, s1;
        load_doc(L0, P, s0, d);
        load_doc(L1, P, s1, d1);
        int done = 0;
        unsigned long long acc_s = 0, acc_l = 0;
        const gptr<const mtr_op> ops = gp(P.ops) + dd.op_begin + cursor;
        for (int k = 0; k < n_ops; k++) {
            if (GN) gen_pair_op(L0, L1, P, s0, s1, dd, cursor + k);
            const mtr_op op = uni_struct(ld_struct<mtr_op>(ops + k));
            if (DL) s0.cur_op = s1.cur_op = cursor + k;  // (set-cell records split outside apply_op: their reports)
#ifdef MTR_PROF  // P_X1 = setCell messages, P_X2 = row/col splices
            ProfScope _prof_op(L0.sc, P_OP);
            ProfScope _prof_kind(L0.sc, op.type == MTR_OP_SETCELL ? P_X1 : P_X2);
#endif
            bool ok = true;
            if (op.type == MTR_OP_START_COLLAB && !(op.flags & MTR_F_APPEND)) {
                // didAttach / onConnect start both vectors (matrix.ts:514-532); with MTR_F_APPEND, one
                // vector's SnapshotLoader start (below, by MTR_F_COLS)
                ok = apply_op(L0, P, s0, op, dd, false, 0, cursor + k) && apply_op(L1, P, s1, op, dd, false, 0, cursor + k);
            } else if (op.type == MTR_OP_SETCELL) {
                acc_s += (unsigned long long)(s0.nseg + s1.nseg);  // both vectors are resolved
                View v;
                v.ref = op.ref_seq;
                v.client = enc_client(int(int16_t(op.client)));
                v.local = 0;
                View v1 = v;
                v.local = (!s0.collab || uint32_t(s0.local) == v.client) ? 1 : 0;
                v1.local = (!s1.collab || uint32_t(s1.local) == v1.client) ? 1 : 0;
                int roff = 0, coff = 0;
                // both vectors at the op's view in one pass (the cols result is unused when the row
                // is undefined)
                int fr, br, fc, bc;
                find2(L0, s0, v, op.pos1, fr, br, L1, s1, v1, op.pos2, fc, bc, P.new_length_calc);
                const int ri = adjust_position(L0, s0, op.pos1, fr, br, roff);
                if (ri >= 0) {
                    const int ci = adjust_position(L1, s1, op.pos2, fc, bc, coff);
                    if (ci >= 0) {
                        const int rh = handle_at(L0, P, s0, ri, roff);
                        const int ch = handle_at(L1, P, s1, ci, coff);
                        // the cell write (cells.setCell(rowHandle, colHandle, value), matrix.ts:686-689)
                        if (DL && (op.flags & MTR_F_DELTA) && s0.status == MTR_OK && s1.status == MTR_OK)
                            put_record(L0, s0, cursor + k, rh, ch, MTR_DELTA_CELL);
                    }
                }
                if (s0.status != MTR_OK) set_fail(L0, cursor + k);
                if (s1.status != MTR_OK) set_fail(L1, cursor + k);
                ok = s0.status == MTR_OK && s1.status == MTR_OK;
            } else if (op.type == MTR_OP_LOCAL_SETCELL) {  // setCellCore -> sendSetCellOp (matrix.ts:254-310)
                acc_s += (unsigned long long)(s0.nseg + s1.nseg);
                const int rh = allocated_handle(L0, P, s0, op.pos1, false);
                const int ch = s0.status == MTR_OK ? allocated_handle(L1, P, s1, op.pos2, false) : -1;
                if (s0.status == MTR_OK && s1.status == MTR_OK) {
                    if (s0.collab && lane_id() == 0) {  // nextLocalSeq (matrix.ts:484-492): both windows advance
                        L0.ghdr()->lseq = L0.ghdr()->lseq + 1;
                        L1.ghdr()->lseq = L1.ghdr()->lseq + 1;
                    }
                    wsync();
                    if (DL && (op.flags & MTR_F_DELTA)) put_record(L0, s0, cursor + k, rh, ch, MTR_DELTA_CELL);
                }
                if (s0.status != MTR_OK) set_fail(L0, cursor + k);
                if (s1.status != MTR_OK) set_fail(L1, cursor + k);
                ok = s0.status == MTR_OK && s1.status == MTR_OK;
            } else if (op.flags & MTR_F_COLS) {
                ok = vector_op(L1, L0, P, s1, op, dd, cursor + k, acc_s);
            } else {
                ok = vector_op(L0, L1, P, s0, op, dd, cursor + k, acc_s);
            }
            if (!ok) break;
            done = k + 1;
        }
        if (lane_id() == 0) {  // the matrix's counters are kept with its rows document
            L0.sc->sum_s += acc_s;
            L0.sc->sum_l += acc_l;
        }
        store_doc(L0, P, s0, d, done);
        store_doc(L1, P, s1, d1, 0);  // the cols vector's op cursor stays at 0 (it has no op list of its own)
    }

    // A matrix pair on two waves (apply_pair2_kernel): wave w owns vector w (0 = rows, 1 = cols), each in its own
    // LDS region, and both walk the pair's op list.  The two PermutationVectors share nothing but that list: a
    // setCell resolves the row on wave 0 and the col on wave 1 at the same time (the single-wave kernel's find2,
    // split across waves), and each allocates its own handle once both positions are defined (matrix.ts:669-689);
    // a row / col op runs on its own vector's wave.  The waves meet at a workgroup barrier after every op (and
    // between a setCell's resolution and its allocations), exchanging `defined` / `ok` words in LDS, so both stop
    // at the same op.  Replay only: local ops (partner localSeq), delta records and record mode keep run_pair.
    static MTR_DI void run_pair2(char* smem, size_t region, const KParams& P, uint32_t d) {
        const int w = int(threadIdx.x >> 6);  // this wave's vector
        const uint32_t d1 = uniu(gp(P.dpart)[d]);
        const uint32_t dw = w ? d1 : d;
        const mtr_doc_desc dd = uni_struct(ld_struct<mtr_doc_desc>(gp(P.docs) + d));
        const int cursor = uni(gp(P.hdr)[d].op_cursor);
        const int n_ops = min(int(dd.op_count) - cursor, P.ops_this_launch);
        // (both waves read the same words: they take the same branch)
        if (n_ops <= 0 || uni(gp(P.hdr)[d].status) != MTR_OK || uni(gp(P.hdr)[d1].status) != MTR_OK) return;
        // the exchange words sit behind the two regions: [0..1] defined, [2..5] ok (by op parity), [6..7] counters
        const lptr<int> xch = (lptr<int>)(smem + 2 * region);
        D L;
        carve(L, smem + (w ? region : 0), P, dw);
        St s;
        load_doc(L, P, s, dw);
        int done = 0;
        unsigned long long acc_s = 0;
        const gptr<const mtr_op> ops = gp(P.ops) + dd.op_begin + cursor;
        for (int k = 0; k < n_ops; k++) {
            const mtr_op op = uni_struct(ld_struct<mtr_op>(ops + k));
            bool ok = true;
            if (op.type == MTR_OP_START_COLLAB && !(op.flags & MTR_F_APPEND)) {  // both vectors (matrix.ts:514-532)
                ok = apply_op(L, P, s, op, dd, false, 0, cursor + k);
            } else if (op.type == MTR_OP_SETCELL) {
                acc_s += (unsigned long long)s.nseg;  // (each wave counts its own vector's leaves)
                View v;
                v.ref = op.ref_seq;
                v.client = enc_client(int(int16_t(op.client)));
                v.local = (!s.collab || uint32_t(s.local) == v.client) ? 1 : 0;
                const int pos = w ? op.pos2 : op.pos1;
                int f, b, off = 0;
                find1(L, s, v, pos, f, b, P.new_length_calc);
                const int idx = adjust_position(L, s, pos, f, b, off);
                if (lane_id() == 0) xch[w] = idx >= 0 ? 1 : 0;
                __syncthreads();
                const bool both = xch[0] != 0 && xch[1] != 0;  // (the row undefined: the col is not allocated)
                if (both) (void)handle_at(L, P, s, idx, off);
                if (s.status != MTR_OK) set_fail(L, cursor + k);
                ok = s.status == MTR_OK;
            } else if (((op.flags & MTR_F_COLS) != 0) == (w == 1)) {
                const int n0 = s.nseg;
                ok = apply_op(L, P, s, op, dd, false, 0, cursor + k);
                if (ok && counts_s(op)) acc_s += (unsigned long long)n0;
            }
            // (the ok words alternate by op parity: a wave writes op k + 1's word while the other may still be
            // reading op k's, never op k - 1's -- it passed this barrier of op k only after reading that)
            const int q = 2 + 2 * (k & 1);
            if (lane_id() == 0) xch[q + w] = ok ? 1 : 0;
            __syncthreads();
            if (xch[q] == 0 || xch[q + 1] == 0) break;
            done = k + 1;
        }
        if (w == 1 && lane_id() == 0) {
            xch[6] = int(acc_s & 0xffffffffull);
            xch[7] = int(acc_s >> 32);
        }
        __syncthreads();
        if (w == 0 && lane_id() == 0)  // the matrix's counters are kept with its rows document
            L.sc->sum_s += acc_s + (unsigned long long)uint32_t(xch[6]) + ((unsigned long long)uint32_t(xch[7]) << 32);
        store_doc(L, P, s, dw, w ? 0 : done);
    }
};

// GN: record mode (synthetic workloads, untimed) as its own instantiation, so the replay kernels
// carry no generator code or generator state
#ifndef MTR_WPE
#define MTR_WPE 5
#endif
// (HBM-resident documents are few per CU -- C5 puts about one per SIMD -- so their kernels may take a
// whole SIMD's registers instead of spilling: a spilling build of the lean one produced wrong views)
#ifndef MTR_WPE_G
#define MTR_WPE_G 1
#endif
// (the LDS-resident kernels with the rare records compiled in -- CAP = 0: local ops, references, intervals,
// reconnect, record mode -- run small batches of live clients: they take a SIMD's registers too, so their extra
// state stays in registers (AGPRs when it must) instead of spilling to scratch)
#ifndef MTR_WPE_X
#define MTR_WPE_X 1
#endif
template <bool G, int CAP = 0, bool DL = false, bool GN = false>
__global__ void __launch_bounds__(G ? NT * MTR_GW : NT)
    __attribute__((amdgpu_waves_per_eu(G ? MTR_WPE_G : (CAP == 0 ? MTR_WPE_X : MTR_WPE)))) apply_kernel(KParams P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (blockIdx.x >= P.n_launch) return;
    const uint32_t d = P.doc_list[blockIdx.x];
    using E = Eng<G, false, CAP, DL, GN>;
    if constexpr (G) {  // an HBM-resident document's team (launched with MTR_GW waves, or one)
        const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));  // (wave-uniform)
        if (w > 0) {
            E::team_helper(smem, P, d, w);
            return;
        }
        E::run(smem, P, d);
        E::team_exit(smem);
        return;
    }
    E::run(smem, P, d);
}

// leaf capacities with a compile-time LDS layout (apply_kernel<false, CAP>, instantiated in
// apply_caps.hip, kCapParts translation units); other capacities use the runtime layout (CAP = -1, or 0 for a
// batch with rare records)
constexpr int kCapParts = 3;
bool launch_fixed_cap_p0(int cap, uint32_t grid, size_t lds, hipStream_t st, const KParams& P);
bool launch_fixed_cap_p1(int cap, uint32_t grid, size_t lds, hipStream_t st, const KParams& P);
bool launch_fixed_cap_p2(int cap, uint32_t grid, size_t lds, hipStream_t st, const KParams& P);
#define MTR_FIXED_CAPS(X) \
    X(64) X(96) X(128) X(160) X(192) X(224) X(256) X(288) X(320) X(352) X(384) X(416) X(448) X(480) X(512) X(544) \
    X(576) X(608) X(640) X(672) X(704) X(736) X(768) X(800) X(832) X(864) X(896) X(928) X(960) X(992) X(1024) X(1088) \
    X(1152) X(1216) X(1280) X(1344) X(1408) X(1472) X(1536)
// (above 1,024 leaves the fixed capacities step by 64: a yielding launch's capacity is rounded up to one of them,
// mtr_engine.hip's class loop)

// SharedMatrix pairs: one wave applies a matrix's op list to its two PermutationVectors, each with
// its own LDS region of `pair_region` bytes (HBM-resident arrays in global mode)
template <bool G, bool DL = false, bool GN = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, G ? 1 : 8))) apply_pair_kernel(KParams P, uint32_t pair_region) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (blockIdx.x >= P.n_launch) return;
    const uint32_t d = P.doc_list[blockIdx.x];
    Eng<G, true, 0, DL, GN>::run_pair(smem, pair_region, P, d);
}

// SharedMatrix pairs on two waves (run_pair2): a 128-thread workgroup, one wave per vector
template <bool G>
__global__ void __launch_bounds__(2 * NT) __attribute__((amdgpu_waves_per_eu(1, G ? 1 : 8))) apply_pair2_kernel(KParams P, uint32_t pair_region) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (blockIdx.x >= P.n_launch) return;
    const uint32_t d = P.doc_list[blockIdx.x];
    Eng<G, true, G ? 0 : -2, false, false>::run_pair2(smem, pair_region, P, d);
}
constexpr size_t kPair2Xch = 64;  // bytes behind the two regions: run_pair2's exchange words

// the runtime-layout instantiations, launched by name from mtr_engine.hip and compiled in kVariantParts
// translation units (apply_variants.hip): X = the rare records compiled in, LEAN = without them, DL = delta
// reporting, GN = record mode; PAIR = SharedMatrix pairs
enum ApplyVariant {
    AV_LDS_X = 0, AV_HBM_X, AV_LDS_LEAN, AV_HBM_LEAN, AV_LDS_DL, AV_HBM_DL, AV_LDS_GN, AV_HBM_GN,
    AV_PAIR_LDS, AV_PAIR_HBM, AV_PAIR_LDS_DL, AV_PAIR_HBM_DL, AV_PAIR_LDS_GN, AV_PAIR_HBM_GN, AV_PAIR2_LDS,
    AV_PAIR2_HBM, AV_COUNT
};
constexpr int kVariantParts = 16;  // (one variant per part: the HBM-resident ones take many minutes each)
bool launch_variant_p0(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p1(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p2(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p3(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p4(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p5(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p6(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p7(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p8(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p9(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p10(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p11(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p12(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p13(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p14(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
bool launch_variant_p15(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region);
inline bool launch_variant(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region = 0) {
    return launch_variant_p0(v, grid, lds, st, P, region) ||
           launch_variant_p1(v, grid, lds, st, P, region) ||
           launch_variant_p2(v, grid, lds, st, P, region) ||
           launch_variant_p3(v, grid, lds, st, P, region) ||
           launch_variant_p4(v, grid, lds, st, P, region) ||
           launch_variant_p5(v, grid, lds, st, P, region) ||
           launch_variant_p6(v, grid, lds, st, P, region) ||
           launch_variant_p7(v, grid, lds, st, P, region) ||
           launch_variant_p8(v, grid, lds, st, P, region) ||
           launch_variant_p9(v, grid, lds, st, P, region) ||
           launch_variant_p10(v, grid, lds, st, P, region) ||
           launch_variant_p11(v, grid, lds, st, P, region) ||
           launch_variant_p12(v, grid, lds, st, P, region) ||
           launch_variant_p13(v, grid, lds, st, P, region) ||
           launch_variant_p14(v, grid, lds, st, P, region) ||
           launch_variant_p15(v, grid, lds, st, P, region);
}

}  // namespace mtr
