// mtr_engine.hip -- host side of the MI355X merge-tree replay engine: the C ABI of
// include/mtr.h, device memory management and kernel launches.
//
// Memory layout in HBM (one slab per document, sized by mtr_caps):
//   DocHdr                      64 B                  (collaboration window + arena cursors)
//   leaves  [NF][segcap] u32    len seq rseq meta text props uid   (SoA, tree order)
//   heap    [2][hcap]    u32    zamboni LRU heap (seq, uid), 1-based
//   text    [tcap]       u16    UTF-16 text arena (segments hold offsets)
//   props   [pcap]       u32    immutable property-set entries [n, k0, v0, ...]
//   removers[rcap]       u32    cons cells of overlapping removers (client<<24 | next), then the
//           [2*rtab]     u32    uid -> list head table (open addressing, key uid+1)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/mtr.h"
#include "../../include/mtr_synth.h"
#include "apply.hip.h"
#include "summary.hip.h"

using namespace mtr;

namespace {

thread_local std::string g_err;

void set_err(const std::string& s) { g_err = s; }

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t _e = (x);                                                       \
        if (_e != hipSuccess) {                                                    \
            set_err(std::string(#x) + ": " + hipGetErrorString(_e));               \
            return -1;                                                             \
        }                                                                          \
    } while (0)

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int ensure(size_t want) {
        if (want <= n && p) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t bytes = std::max<size_t>(want, 1) * sizeof(T);
        if (hipMalloc(&p, bytes) != hipSuccess) {
            set_err("hipMalloc failed for " + std::to_string(bytes) + " bytes");
            return -1;
        }
        n = std::max<size_t>(want, 1);
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

int round64(int x) { return std::max(64, (x + 63) & ~63); }
int round32(int x) { return std::max(64, (x + 31) & ~31); }

}  // namespace

struct mtr_engine {
    mtr_options opt{};
    mtr_caps caps{};
    int32_t rtab = 64;  // remover-head table entries per document (power of two >= 2 * remover_cells)
    int device = 0;
    uint32_t max_docs = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {};
    // size-class launches of one apply round run concurrently: class i on lane[i % kLanes]
    // (lane 0 = `stream`), joined back into `stream` before the next round
    static constexpr int kLanes = 4;
    hipStream_t aux[kLanes - 1] = {};
    hipEvent_t lane_done[kLanes] = {};
    hipEvent_t grp_fork[kLanes] = {}, grp_cls[kLanes] = {};  // per document group: round start, class counts read
    std::vector<hipEvent_t> kev;  // per-launch start/stop events (kernel durations)
    // persistent document state
    DevBuf<DocHdr> hdr;
    DevBuf<uint32_t> seg, heap, prop, rm;
    DevBuf<uint16_t> text;
    // current batch (device copies)
    uint32_t n_docs = 0;
    uint32_t max_ops_per_doc = 0;
    DevBuf<mtr_doc_desc> docs;
    DevBuf<mtr_op> ops;
    DevBuf<uint16_t> btext;
    DevBuf<uint32_t> propop_off, propop_kv, key_off, key_index, val_off, val_eq, client_off;
    DevBuf<uint8_t> key_bytes, val_bytes, client_bytes;
    DevBuf<unsigned long long> stat;  // [0] ops applied
    DevBuf<uint32_t> delta;           // delta ranges of the MTR_F_DELTA ops of the current batch
    DevBuf<uint64_t> doff;            // [doc + 1] record offsets into delta (exact per-batch bound)
    std::vector<uint64_t> h_doff;
    bool has_delta = false;
    bool has_ext = false;             // the batch holds rare records (op_scan_kernel): no fixed-capacity kernels
    bool pend_seen = false;           // a batch since mtr_reset held local ops while collaborating or acks:
                                      // documents may hold pending segments, so every launch is an X kernel
    DevBuf<uint32_t> pend;            // [doc][kPendRing][4] pending SegmentGroups (allocated on first use)
    int dev_lds = 0;                  // the device's LDS per workgroup (bytes; 0 = unknown)
    bool refs_seen = false;           // a batch since mtr_reset created local references: they follow splits,
                                      // appends and removals in the X kernels only, so every launch is one
    DevBuf<uint32_t> refs;            // [doc][3][ref_slots] local references (allocated on first use)
    DevBuf<int32_t> qbuf;             // query results (reference positions)
    DevBuf<int32_t> csum;             // [doc][csum_ints(segcap)] chunk records + superchunk rows (first HBM-resident launch)
    DevBuf<int32_t> umap;             // [doc][2 * segcap] uid -> slot hints (with csum)
    DevBuf<int32_t> red;              // small reduction / query-result buffer
    DevBuf<unsigned long long> prof;  // phase-timer sums (-DMTR_PROF builds)
    DevBuf<int32_t> cls;              // size-class counters of one apply round (classify_kernel)
    DevBuf<uint32_t> dlist;           // [class][n_docs] document lists of one apply round
    int32_t* h_cls = nullptr;         // page-locked, mapped host copy of cls (written by words_kernel)
    int32_t* d_cls = nullptr;         // (its device address)
    DevBuf<uint32_t> scratch;         // E/V arrays for HBM-resident (global-mode) launches
    DevBuf<mtr_synth_state> gstate;   // record mode generator state
    // SharedMatrix pairs (mtr_set_matrix): per document kind (0 SharedString, 1 rows vector, 2 cols
    // vector) and partner; they survive mtr_reset
    DevBuf<uint32_t> dkind, dpart;
    std::vector<uint32_t> h_kind, h_part;
    mtr_synth_cfg gcfg{};
    uint32_t ggrow = 0;  // pre-grown records of the record-mode run in progress
    // summaries
    DevBuf<int64_t> out_size, out_off;
    DevBuf<uint8_t> s_kind;                       // summary scratch (size pass -> write pass)
    DevBuf<uint32_t> s_start, s_len, s_bytes, s_lb, s_fl, s_sid, s_bb;
    DevBuf<int32_t> s_blob;
    DevBuf<unsigned long long> out_hash;
    DevBuf<uint8_t> out;
    std::vector<int64_t> h_off, h_size;
    std::vector<uint32_t> h_val_eq;  // host copy for export hashes
    int64_t out_total = 0;
    bool summarized = false;
    // pipelined hand-over (mtr_submit_pipelined): the copy stream, per part its landing event, document range and
    // op-scan bits (device, then page-locked host copy)
    hipStream_t copy = nullptr;  // (= aux[kLanes - 2]: the last launch lane)
    std::vector<hipEvent_t> part_ev;
    std::vector<uint32_t> part_lo;
    uint32_t pipe_parts = 0;
    uint32_t pipe_groups = 1;
    uint32_t pipe_last = 0;    // the part uploaded last  // document groups of the pipelined run (their parts are uploaded alternately)
    DevBuf<int32_t> pflags;
    int32_t* h_pflags = nullptr;
    uint32_t h_pflags_n = 0;
    DevBuf<mtr_doc_desc> pdocs;  // the descriptors as uploaded (part_ready_kernel enables them)
    // pipelined summaries (mtr_replay_pipelined): a part is summarized and downloaded once its documents are done
    uint8_t* pipe_out = nullptr;
    bool pipe_one_group = false;  // (set by mtr_replay_pipelined around its mtr_submit_pipelined)
    int64_t pipe_cap = 0;
    DevBuf<int32_t> pleft;                     // per part: documents with ops left (classify_kernel)
    DevBuf<uint32_t> dpart_lo;                 // the parts' first documents (+ n_docs), for classify_kernel
    int32_t *h_pleft = nullptr, *d_pleft = nullptr;   // (mapped page-locked copy, its device address)
    int64_t *h_psize = nullptr, *d_psize = nullptr;   // per document: summary sizes read back, then offsets
    uint32_t h_pleft_n = 0, h_psize_n = 0;
    std::vector<hipEvent_t> pdone_ev, psize_ev, pwrite_ev;  // per part: documents done, sizes read back, written
    // timing
    double t_apply = 0, t_summary = 0;
    double t_kernels = 0;  // sum of the apply launches' own durations (they overlap across lanes)
    int launches = 0;
};

// ------------------------------------------------------------------ small kernels
__global__ void reset_kernel(DocHdr* h, uint32_t n) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n) return;
    DocHdr z{};
    z.height = 1;
    z.local = -1;
    z.fail_op = -1;
    h[d] = z;
}

__global__ void cursor_reset_kernel(DocHdr* h, const mtr_doc_desc* docs, uint32_t n) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n) {
        h[d].op_cursor = 0;
        h[d].dused = 0;  // delta ranges are per batch
        // more short client ids than the engine's 8-bit client field holds: the document stays on
        // the TypeScript Client (MTR_MAX_CLIENTS)
        if (docs[d].n_clients > MTR_MAX_CLIENTS && h[d].status == MTR_OK) {
            h[d].status = MTR_ERR_UNSUPPORTED;
            h[d].fail_op = 0;
        }
    }
}

// dst[i] = src ? src[i] : 0 for i < n (one block): zeroing and reading back small counters without a DMA copy
__global__ void words_kernel(int32_t* dst, const int32_t* src, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src ? src[i] : 0;
    __threadfence_system();
}

// dst[i] = src[i] for i < n, 64-bit words (summary sizes to mapped host memory, offsets back)
__global__ void words64_kernel(int64_t* dst, const int64_t* src, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
    __threadfence_system();
}

// mtr_submit_pipelined: the documents [lo, hi) of part p have landed; enable them (copy the descriptor, op_count
// last, after a fence: classify_kernel reads op_count and a launch the rest) unless the part's op scan found
// records the pipelined path does not run (they then never start; mtr_run reports MTR_ERR_UNSUPPORTED)
__global__ void part_ready_kernel(DocHdr* h, mtr_doc_desc* docs, const mtr_doc_desc* src, uint32_t lo, uint32_t hi,
                                  const int32_t* flags) {
    const uint32_t d = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= hi || *flags != 0) return;
    mtr_doc_desc x = src[d];
    h[d].op_cursor = 0;
    h[d].dused = 0;
    if (x.n_clients > MTR_MAX_CLIENTS && h[d].status == MTR_OK) {  // (cursor_reset_kernel's check)
        h[d].status = MTR_ERR_UNSUPPORTED;
        h[d].fail_op = 0;
    }
    const uint32_t cnt = x.op_count;
    x.op_count = 0;
    docs[d] = x;
    __threadfence();
    docs[d].op_count = cnt;
}

// bit 3: local-reference records (MTR_OP_REF_*, and an interval collection's MTR_OP_REBASE_POS / MTR_OP_LSEQ)
// bit 0: an op flagged MTR_F_DELTA (the host sizes delta buffers only then); bit 1: a rare record the
// fixed-capacity kernels do not carry (Eng::X: relative positions, handle-table loads, combining
// annotates, marker ordinals); bit 2: the local-op path (MTR_OP_ACK, or a local op recorded while
// collaborating: seq = UnassignedSequenceNumber)
__global__ void op_scan_kernel(const mtr_op* ops, uint64_t n, int32_t* out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    bool any = false, ext = false, pend = false, refs = false;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const mtr_op op = ops[i];
        any = any || (op.flags & MTR_F_DELTA) != 0;
        refs = refs || op.type == MTR_OP_REF_CREATE || op.type == MTR_OP_REF_REMOVE || op.type == MTR_OP_REF_ACK ||
               op.type == MTR_OP_REBASE_POS || op.type == MTR_OP_LSEQ;
        pend = pend || op.type == MTR_OP_ACK || op.type == MTR_OP_ROLLBACK || op.type == MTR_OP_REGENERATE ||
               (op.type >= MTR_OP_LOCAL_INSERT && op.type <= MTR_OP_LOCAL_ANNOTATE && op.seq == -1);
        ext = ext || op.type == MTR_OP_RELPOS || op.type == MTR_OP_HANDLES || (op.flags & MTR_F_REL) ||
              op.type == MTR_OP_LOCAL_SETCELL ||
              (op.type == MTR_OP_ANNOTATE && op.payload2 != 0) ||
              ((op.flags & MTR_F_MARKER) && op.payload2 != 0 &&
               (op.type == MTR_OP_INSERT || op.type == MTR_OP_LOCAL_INSERT || op.type == MTR_OP_LOAD));
    }
    const int bits = (__ballot(any) ? 1 : 0) | (__ballot(ext) ? 2 : 0) | (__ballot(pend) ? 4 : 0) |
                     (__ballot(refs) ? 8 : 0);
    if (bits && (threadIdx.x & 63) == 0) atomicOr(out, bits);
}

// out[0] = max nseg, out[1] = max remaining ops, out[2] = max heapn
__global__ void scan_state_kernel(const DocHdr* h, const mtr_doc_desc* docs, uint32_t n, int32_t* out) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n) return;
    const DocHdr x = h[d];
    atomicMax(&out[0], x.nseg);
    int rem = x.status == MTR_OK ? int(docs[d].op_count) - x.op_cursor : 0;
    atomicMax(&out[1], rem);
    atomicMax(&out[2], x.heapn);
}

// Size classes for one apply round: documents with ops left are bucketed by leaf count (64-leaf
// classes) so that each class launch sizes its LDS by its own largest document.
// cls layout: [0] max remaining ops, then per class c: cnt[c] at 1+3c, max nseg at 2+3c, max heapn at 3+3c.
// Classes [kClasses, 2 kClasses) hold matrix pairs (rows vector documents), classed by the larger
// of the two vectors; they launch apply_pair_kernel with two LDS regions.
constexpr int kClasses = 64;
constexpr int kAllClasses = 2 * kClasses;
__global__ void __launch_bounds__(256) classify_kernel(const DocHdr* h, const mtr_doc_desc* docs, uint32_t lo,
                                                      uint32_t hi, const uint32_t* dkind, const uint32_t* dpart,
                                                      int32_t* cls, uint32_t* list, int class_leaves,
                                                      int32_t* pleft = nullptr, const uint32_t* plo = nullptr,
                                                      uint32_t pparts = 0) {
    // block-local histogram in LDS, then one global atomic per (block, class): the per-document
    // atomics on a handful of addresses would serialise at the memory side
    __shared__ int lcnt[kAllClasses], lmax[kAllClasses], lheap[kAllClasses], lbase[kAllClasses];
    __shared__ int lrem;
    const int t = threadIdx.x;
    if (t < kAllClasses) lcnt[t] = lmax[t] = lheap[t] = 0;
    if (t == 0) lrem = 0;
    __syncthreads();
    // (documents [lo, hi): one group of the round loop; its class lists are [class][hi - lo])
    const uint32_t n = hi - lo;
    const uint32_t d = lo + blockIdx.x * blockDim.x + t;
    int c = -1, rank = 0;
    if (d < hi) {
        const DocHdr x = h[d];
        const int rem = x.status == MTR_OK ? int(docs[d].op_count) - x.op_cursor : 0;
        if (rem > 0) {
            int nseg = x.nseg, heapn = max(x.heapn, x.heap_need), base = 0;
            if (dkind[d] == 1) {
                const DocHdr y = h[dpart[d]];
                nseg = max(nseg, y.nseg);
                heapn = max(heapn, max(y.heapn, y.heap_need));
                base = kClasses;
            }
            c = base + min(kClasses - 1, nseg / class_leaves);
            rank = atomicAdd(&lcnt[c], 1);
            atomicMax(&lmax[c], nseg);
            atomicMax(&lheap[c], heapn);
            atomicMax(&lrem, rem);
            if (pleft) {  // (a pipelined run: this document's part still has ops left)
                uint32_t pp = 0;  // the last part whose first document is <= d
                for (uint32_t step = 1u << (31 - __clz(int(pparts))); step > 0; step >>= 1)
                    if (pp + step < pparts && plo[pp + step] <= d) pp += step;
                if (!pleft[pp]) atomicOr(&pleft[pp], 1);
            }
        }
    }
    __syncthreads();
    if (t < kAllClasses && lcnt[t]) {
        lbase[t] = atomicAdd(&cls[1 + 3 * t], lcnt[t]);
        atomicMax(&cls[2 + 3 * t], lmax[t]);
        atomicMax(&cls[3 + 3 * t], lheap[t]);
    }
    if (t == 0 && lrem) atomicMax(&cls[0], lrem);
    __syncthreads();
    if (c >= 0) list[size_t(c) * n + lbase[c] + rank] = d;
}

// local-reference positions (or one reference's info) of a document's HBM state (mtr_get_ref_positions / _info)
__global__ void __launch_bounds__(NT) refs_kernel(KParams P, uint32_t d, int32_t* out, int info_id) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Eng<true>::ref_query(smem, P, d, out, info_id);
}

// one getContainingSegment query on a document's HBM state (mtr_get_containing_segment)
__global__ void __launch_bounds__(NT) containing_kernel(KParams P, uint32_t d, int pos, int ref, int client,
                                                        int32_t* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Eng<true>::containing(smem, P, d, pos, ref, client, out);
}

template <class T>
static int upload(mtr_engine* e, DevBuf<T>& dst, const T* src, size_t n) {
    if (dst.ensure(n)) return -1;
    if (n) HIPCHK(hipMemcpyAsync(dst.p, src, n * sizeof(T), hipMemcpyHostToDevice, e->stream));
    return 0;
}

extern "C" {

const char* mtr_last_error(void) { return g_err.c_str(); }

mtr_engine* mtr_engine_create(const mtr_options* opt, int device, uint32_t max_docs, const mtr_caps* caps) {
    auto* e = new mtr_engine();
    e->opt = opt ? *opt : mtr_options{0, 1, 10000, 0};
    if (e->opt.chunk_size <= 0) e->opt.chunk_size = 10000;
    mtr_caps c{4096, 2048, 65536, 16384, 4096, 256, 1024};
    if (caps) {
        if (caps->max_segments) c.max_segments = caps->max_segments;
        if (caps->heap_entries) c.heap_entries = caps->heap_entries;
        if (caps->text_units) c.text_units = caps->text_units;
        if (caps->prop_words) c.prop_words = caps->prop_words;
        if (caps->remover_cells) c.remover_cells = caps->remover_cells;
        if (caps->ops_per_launch) c.ops_per_launch = caps->ops_per_launch;
        if (caps->ref_slots) c.ref_slots = caps->ref_slots;
    }
    c.max_segments = (c.max_segments + 63) & ~63u;
    c.heap_entries = (c.heap_entries + 63) & ~63u;
    if (c.remover_cells > 0xfffffe) c.remover_cells = 0xfffffe;
    e->caps = c;
    while (e->rtab < 2 * int32_t(c.remover_cells)) e->rtab *= 2;
    e->device = device;
    e->max_docs = max_docs;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        set_err("cannot open HIP device " + std::to_string(device));
        delete e;
        return nullptr;
    }
    {  // HBM-resident launches (and the query kernels) still keep per-chunk rows in LDS: about segcap / 8
       // bytes (twice for a matrix pair: mtr_set_matrix checks that) -- a capacity whose rows exceed the device's
       // LDS is refused here rather than failing every later launch with a generic HIP error
        int dev_lds = 0;
        if (hipDeviceGetAttribute(&dev_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess) dev_lds = 0;
        e->dev_lds = dev_lds;
        const size_t need = (lds_bytes_global_mode(int(c.max_segments)) + 15) & ~size_t(15);
        if (dev_lds > 0 && need > size_t(dev_lds)) {
            set_err("mtr_engine_create: max_segments " + std::to_string(c.max_segments) + " needs " +
                    std::to_string(need) + " bytes of LDS in HBM-resident mode (device: " + std::to_string(dev_lds) + ")");
            (void)hipStreamDestroy(e->stream);
            delete e;
            return nullptr;
        }
    }
    for (auto& x : e->ev) (void)hipEventCreate(&x);
    for (auto& x : e->aux) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    for (auto& x : e->lane_done) (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
    for (auto& x : e->grp_fork) (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
    for (auto& x : e->grp_cls) (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
    const size_t D = std::max<uint32_t>(max_docs, 1);
    e->h_kind.assign(D, 0);
    e->h_part.assign(D, 0);
    if (e->dkind.ensure(D) || e->dpart.ensure(D) ||
        hipMemset(e->dkind.p, 0, D * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(e->dpart.p, 0, D * sizeof(uint32_t)) != hipSuccess) {
        mtr_engine_destroy(e);
        return nullptr;
    }
    if (e->hdr.ensure(D) || e->seg.ensure(D * NF * c.max_segments) || e->heap.ensure(D * 2 * c.heap_entries) ||
        e->text.ensure(D * c.text_units) || e->prop.ensure(D * c.prop_words) || e->rm.ensure(D * (c.remover_cells + 2 * size_t(e->rtab))) ||
        e->stat.ensure(D * 4) || e->red.ensure(16)) {
        mtr_engine_destroy(e);
        return nullptr;
    }
    if (mtr_reset(e) != MTR_OK) {
        mtr_engine_destroy(e);
        return nullptr;
    }
    return e;
}

int mtr_engine_destroy(mtr_engine* e) {
    if (!e) return 0;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (auto* b : {&e->seg, &e->heap, &e->prop, &e->rm, &e->propop_off, &e->propop_kv, &e->key_off, &e->key_index,
                    &e->val_off, &e->val_eq, &e->client_off})
        b->release();
    e->hdr.release();
    e->pend.release();
    e->refs.release();
    e->qbuf.release();
    e->csum.release();
    e->umap.release();
    e->text.release();
    e->btext.release();
    e->docs.release();
    e->ops.release();
    e->key_bytes.release();
    e->val_bytes.release();
    e->client_bytes.release();
    e->stat.release();
    e->delta.release();
    e->doff.release();
    e->red.release();
    e->cls.release();
    if (e->h_cls) (void)hipHostFree(e->h_cls);
    e->dlist.release();
    e->dkind.release();
    e->dpart.release();
    e->scratch.release();
    e->out_size.release();
    e->s_kind.release();
    e->s_start.release();
    e->s_len.release();
    e->s_bytes.release();
    e->s_lb.release();
    e->s_fl.release();
    e->s_sid.release();
    e->s_bb.release();
    e->s_blob.release();
    e->out_off.release();
    e->out_hash.release();
    e->out.release();
    for (auto& x : e->ev)
        if (x) (void)hipEventDestroy(x);
    for (auto& x : e->kev)
        if (x) (void)hipEventDestroy(x);
    for (auto& x : e->lane_done)
        if (x) (void)hipEventDestroy(x);
    for (auto& x : e->grp_fork)
        if (x) (void)hipEventDestroy(x);
    for (auto& x : e->grp_cls)
        if (x) (void)hipEventDestroy(x);
    for (auto& x : e->aux)
        if (x) {
            (void)hipStreamSynchronize(x);
            (void)hipStreamDestroy(x);
        }
    for (auto& x : e->part_ev)
        if (x) (void)hipEventDestroy(x);
    for (auto* v : {&e->pdone_ev, &e->psize_ev, &e->pwrite_ev})
        for (auto& x : *v)
            if (x) (void)hipEventDestroy(x);
    e->pleft.release();
    e->dpart_lo.release();
    if (e->h_pleft) (void)hipHostFree(e->h_pleft);
    if (e->h_psize) (void)hipHostFree(e->h_psize);
    e->pflags.release();
    e->pdocs.release();
    if (e->h_pflags) (void)hipHostFree(e->h_pflags);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return 0;
}

int mtr_reset(mtr_engine* e) {
    HIPCHK(hipSetDevice(e->device));
    const uint32_t n = std::max<uint32_t>(e->max_docs, 1);
    reset_kernel<<<(n + 255) / 256, 256, 0, e->stream>>>(e->hdr.p, n);
    // remover-head tables start empty (their keys are uids, which restart at 0)
    HIPCHK(hipMemsetAsync(e->rm.p, 0, e->rm.n * sizeof(uint32_t), e->stream));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemsetAsync(e->stat.p, 0, e->stat.n * sizeof(unsigned long long), e->stream));
    e->summarized = false;
    e->pend_seen = false;
    e->refs_seen = false;
    return MTR_OK;
}

int mtr_submit(mtr_engine* e, const mtr_batch* b) {
    HIPCHK(hipSetDevice(e->device));
    if (b->n_docs > e->max_docs) {
        set_err("batch has more documents than the engine was created for");
        return MTR_ERR_BAD_OP;
    }
    e->n_docs = b->n_docs;
    uint32_t mx = 0;
    for (uint32_t d = 0; d < b->n_docs; d++) mx = std::max(mx, b->docs[d].op_count);
    e->max_ops_per_doc = mx;
    const size_t nkv = b->n_propops ? size_t(b->propop_off[b->n_propops]) * 2 : 0;
    const size_t ncl = 1 + [&] {
        size_t m = 0;
        for (uint32_t d = 0; d < b->n_docs; d++) m = std::max<size_t>(m, size_t(b->docs[d].client_base) + b->docs[d].n_clients);
        return m;
    }();
    if (upload(e, e->docs, b->docs, b->n_docs) || upload(e, e->ops, b->ops, b->n_ops) ||
        upload(e, e->btext, b->text, b->n_text) || upload(e, e->propop_off, b->propop_off, size_t(b->n_propops) + 1) ||
        upload(e, e->propop_kv, b->propop_kv, nkv) || upload(e, e->key_off, b->key_off, size_t(b->n_keys) + 1) ||
        upload(e, e->key_bytes, b->key_bytes, b->n_keys ? size_t(b->key_off[b->n_keys]) : 0) ||
        upload(e, e->key_index, b->key_index, b->n_keys) || upload(e, e->val_off, b->val_off, size_t(b->n_vals) + 1) ||
        upload(e, e->val_bytes, b->val_bytes, b->n_vals ? size_t(b->val_off[b->n_vals]) : 0) ||
        upload(e, e->val_eq, b->val_eq, b->n_vals) || upload(e, e->client_off, b->client_off, ncl) ||
        upload(e, e->client_bytes, b->client_bytes, size_t(b->client_off[ncl - 1])))
        return -1;
    e->h_val_eq.assign(b->val_eq, b->val_eq + b->n_vals);
    // delta records (MTR_F_DELTA): per-document slices sized by an exact bound of this batch's records.
    // SharedString: an insert reports its one segment; a remove / annotate at most one range per unit
    // of its range and per segment.  SharedMatrix tracked for its cells (any flagged op): one record
    // per flagged set-cell, and per vector one per unlinked segment -- at most the segments present
    // at the batch start plus two per op (split + insert / load)
    e->has_delta = false;
    e->has_ext = false;
    e->h_doff.assign(size_t(b->n_docs) + 1, 0);
    bool any = false;
    if (b->n_ops) {  // one pass over the uploaded ops on the device instead of the host
        HIPCHK(hipMemsetAsync(e->red.p, 0, sizeof(int32_t), e->stream));
        const uint64_t blocks = std::min<uint64_t>((b->n_ops + 255) / 256, 4096);
        op_scan_kernel<<<uint32_t(blocks), 256, 0, e->stream>>>(e->ops.p, b->n_ops, e->red.p);
        HIPCHK(hipGetLastError());
        int32_t flag = 0;
        HIPCHK(hipMemcpyAsync(&flag, e->red.p, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        any = (flag & 1) != 0;
        e->has_ext = (flag & 2) != 0;
        if (flag & 4) {
            if (!e->pend.p) {
                if (e->pend.ensure(size_t(std::max<uint32_t>(e->max_docs, 1)) * kPendRing * 4)) return -1;
            }
            e->pend_seen = true;
        }
        if (flag & 8) {
            if (!e->refs.p &&
                e->refs.ensure(size_t(std::max<uint32_t>(e->max_docs, 1)) * 3 * size_t(e->caps.ref_slots)))
                return -1;
            e->refs_seen = true;
        }
    }
    e->has_ext = e->has_ext || e->pend_seen || e->refs_seen;
    if (any) {
        std::vector<uint64_t> need(b->n_docs, 0);
        for (uint32_t d = 0; d < b->n_docs; d++) {
            const mtr_doc_desc& dd = b->docs[d];
            const uint32_t kind = d < e->h_kind.size() ? e->h_kind[d] : 0;
            if (kind == 2) continue;  // a cols vector: sized with its rows document
            // (record mode submits op lists that are only written on the device: n_ops bounds the scan)
            const uint64_t end = std::min<uint64_t>(dd.op_begin + dd.op_count, b->n_ops);
            bool flagged = false;
            for (uint64_t i = dd.op_begin; i < end; i++) {
                const mtr_op& op = b->ops[i];
                if (!(op.flags & MTR_F_DELTA)) continue;
                flagged = true;
                if (kind == 1) {
                    if (op.type == MTR_OP_SETCELL || op.type == MTR_OP_LOCAL_SETCELL) need[d] += 1;
                    // (a vector's reconnect records: regenerate, two per member; rebasePosition, one)
                    const uint32_t dv = (op.flags & MTR_F_COLS) && e->h_part[d] < b->n_docs ? e->h_part[d] : d;
                    if (op.type == MTR_OP_REGENERATE) need[dv] += 2 * uint64_t(e->caps.max_segments);
                    if (op.type == MTR_OP_REBASE_POS) need[dv] += 1;
                } else if (op.type == MTR_OP_INSERT) {
                    need[d] += 1;
                } else if (op.type == MTR_OP_REMOVE || op.type == MTR_OP_ANNOTATE) {
                    need[d] += uint64_t(std::min<int64_t>(std::max<int64_t>(int64_t(op.pos2) - op.pos1, 0),
                                                          int64_t(e->caps.max_segments)));
                } else if (op.type == MTR_OP_REGENERATE) {  // two records per member of the group
                    need[d] += 2 * uint64_t(e->caps.max_segments);
                } else if (op.type == MTR_OP_REBASE_POS) {
                    need[d] += 1;
                }
            }
            if (kind == 1 && flagged) {
                // (+ undo tracking reports: a link per delta segment of a local vector op, a split-off half per
                // split, a merge per appended segment)
                const uint64_t recycle = 3 * uint64_t(e->caps.max_segments) + 6 * uint64_t(dd.op_count);
                need[d] += recycle;
                const uint32_t d1 = e->h_part[d];
                if (d1 < b->n_docs) need[d1] += recycle;
            }
        }
        for (uint32_t d = 0; d < b->n_docs; d++) e->h_doff[d + 1] = e->h_doff[d] + need[d];
    }
    if (e->h_doff[b->n_docs]) {
        e->has_delta = true;
        if (e->delta.ensure(size_t(e->h_doff[b->n_docs]) * 4) || e->doff.ensure(size_t(b->n_docs) + 1)) return -1;
        HIPCHK(hipMemcpyAsync(e->doff.p, e->h_doff.data(), (size_t(b->n_docs) + 1) * sizeof(uint64_t),
                              hipMemcpyHostToDevice, e->stream));
    }
    if (b->n_docs) {  // (an empty batch launches nothing: a 0-block grid is an invalid launch)
        cursor_reset_kernel<<<(b->n_docs + 255) / 256, 256, 0, e->stream>>>(e->hdr.p, e->docs.p, b->n_docs);
        HIPCHK(hipGetLastError());
    }
    e->summarized = false;
    return MTR_OK;
}

int mtr_submit_pipelined(mtr_engine* e, const mtr_batch* b, uint32_t parts) {
    HIPCHK(hipSetDevice(e->device));
    const uint32_t n = b->n_docs;
    parts = std::min(parts, n);
    // documents laid out in order (each one's records and text after the previous one's), no matrix pairs
    bool plain = parts > 1 && n <= e->max_docs;
    for (uint32_t d = 1; d < n && plain; d++)
        plain = b->docs[d].op_begin >= b->docs[d - 1].op_begin + b->docs[d - 1].op_count &&
                b->docs[d].text_base >= b->docs[d - 1].text_base + b->docs[d - 1].text_count;
    for (uint32_t d = 0; d < n && plain && d < e->h_kind.size(); d++) plain = e->h_kind[d] == 0;
    if (!plain) return mtr_submit(e, b);
    e->n_docs = n;
    uint32_t mx = 0;
    for (uint32_t d = 0; d < n; d++) mx = std::max(mx, b->docs[d].op_count);
    e->max_ops_per_doc = mx;
    // the tables, as mtr_submit (small)
    const size_t nkv = b->n_propops ? size_t(b->propop_off[b->n_propops]) * 2 : 0;
    size_t ncl = 0;
    for (uint32_t d = 0; d < n; d++) ncl = std::max<size_t>(ncl, size_t(b->docs[d].client_base) + b->docs[d].n_clients);
    ncl += 1;
    if (upload(e, e->propop_off, b->propop_off, size_t(b->n_propops) + 1) || upload(e, e->propop_kv, b->propop_kv, nkv) ||
        upload(e, e->key_off, b->key_off, size_t(b->n_keys) + 1) ||
        upload(e, e->key_bytes, b->key_bytes, b->n_keys ? size_t(b->key_off[b->n_keys]) : 0) ||
        upload(e, e->key_index, b->key_index, b->n_keys) || upload(e, e->val_off, b->val_off, size_t(b->n_vals) + 1) ||
        upload(e, e->val_bytes, b->val_bytes, b->n_vals ? size_t(b->val_off[b->n_vals]) : 0) ||
        upload(e, e->val_eq, b->val_eq, b->n_vals) || upload(e, e->client_off, b->client_off, ncl) ||
        upload(e, e->client_bytes, b->client_bytes, size_t(b->client_off[ncl - 1])) || upload(e, e->pdocs, b->docs, n))
        return -1;
    e->h_val_eq.assign(b->val_eq, b->val_eq + b->n_vals);
    e->has_delta = false;
    e->has_ext = e->pend_seen || e->refs_seen;
    e->h_doff.assign(size_t(n) + 1, 0);
    if (e->ops.ensure(b->n_ops) || e->btext.ensure(b->n_text) || e->docs.ensure(n) || e->pflags.ensure(parts)) return -1;
    // every document starts disabled (op_count 0: classify_kernel passes it over) until its part has landed
    HIPCHK(hipMemsetAsync(e->docs.p, 0, size_t(n) * sizeof(mtr_doc_desc), e->stream));
    HIPCHK(hipMemsetAsync(e->pflags.p, 0, size_t(parts) * sizeof(int32_t), e->stream));
    // the copy stream is the last launch lane, which mtr_run leaves idle while parts are landing: a stream of its
    // own would share a hardware queue with the engine stream (GPU_MAX_HW_QUEUES = 4 = the launch lanes), and the
    // copies would then hold back every launch queued behind them there
    e->copy = e->aux[mtr_engine::kLanes - 2];
    while (e->part_ev.size() < parts) {
        hipEvent_t x;
        HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        e->part_ev.push_back(x);
    }
    if (e->h_pflags_n < parts) {
        if (e->h_pflags) HIPCHK(hipHostFree(e->h_pflags));
        HIPCHK(hipHostMalloc((void**)&e->h_pflags, size_t(parts) * sizeof(int32_t), hipHostMallocDefault));
        e->h_pflags_n = parts;
    }
    HIPCHK(hipEventRecord(e->ev[0], e->stream));  // (the copy stream starts after the tables)
    HIPCHK(hipStreamWaitEvent(e->copy, e->ev[0], 0));
    e->part_lo.assign(size_t(parts) + 1, 0);
    for (uint32_t p = 0; p <= parts; p++) e->part_lo[p] = uint32_t(uint64_t(n) * p / parts);
    // two document groups (mtr_run's default above 4,096 documents), each with half the parts: the upload
    // alternates between them, so both start within the first two parts
    // (mtr_replay_pipelined: one group unless MTR_PIPE_GROUPS=2 -- the group's documents run their rounds in
    // lockstep, so its parts finish in the order they landed, a part's width apart, and their summaries and
    // downloads stream out behind them; two groups finish at two times, the second's parts all together)
    int pg = (n >= 4096u && parts >= 2) ? 2 : 1;
    if (e->pipe_one_group) {
        const char* v = std::getenv("MTR_PIPE_GROUPS");
        pg = std::min(pg, v && *v ? std::max(1, std::atoi(v)) : 1);
    }
    e->pipe_groups = uint32_t(pg);
    // (a ramp -- the first two parts a quarter and a half of the others' size -- measured slower end to end:
    // 263.5 against 260.9 ms on C3, profiles/r06_e2e_sweep.json)
    if (e->dpart_lo.ensure(size_t(parts) + 1)) return -1;
    HIPCHK(hipMemcpyAsync(e->dpart_lo.p, e->part_lo.data(), (size_t(parts) + 1) * sizeof(uint32_t),
                          hipMemcpyHostToDevice, e->stream));
    const uint32_t half = (parts + 1) / 2;
    for (uint32_t q = 0; q < parts; q++) {
        const uint32_t p = e->pipe_groups == 2 ? ((q & 1) ? half + q / 2 : q / 2) : q;
        const uint32_t lo = e->part_lo[p], hi = e->part_lo[p + 1];
        const mtr_doc_desc &a = b->docs[lo], &z = b->docs[hi - 1];
        const uint64_t o0 = a.op_begin, o1 = std::min<uint64_t>(z.op_begin + z.op_count, b->n_ops);
        const uint64_t t0 = a.text_base, t1 = std::min<uint64_t>(z.text_base + z.text_count, b->n_text);
        if (o1 > o0) {
            HIPCHK(hipMemcpyAsync(e->ops.p + o0, b->ops + o0, (o1 - o0) * sizeof(mtr_op), hipMemcpyHostToDevice, e->copy));
            const uint64_t blocks = std::min<uint64_t>((o1 - o0 + 255) / 256, 4096);
            op_scan_kernel<<<uint32_t(blocks), 256, 0, e->copy>>>(e->ops.p + o0, o1 - o0, e->pflags.p + p);
        }
        if (t1 > t0)
            HIPCHK(hipMemcpyAsync(e->btext.p + t0, b->text + t0, (t1 - t0) * sizeof(uint16_t), hipMemcpyHostToDevice, e->copy));
        part_ready_kernel<<<(hi - lo + 255) / 256, 256, 0, e->copy>>>(e->hdr.p, e->docs.p, e->pdocs.p, lo, hi, e->pflags.p + p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(e->h_pflags + p, e->pflags.p + p, sizeof(int32_t), hipMemcpyDeviceToHost, e->copy));
        HIPCHK(hipEventRecord(e->part_ev[p], e->copy));
    }
    e->pipe_parts = parts;
    e->pipe_last = e->pipe_groups == 2 ? ((parts & 1) ? half - 1 : parts - 1) : parts - 1;  // (uploaded last)
    e->summarized = false;
    return MTR_OK;
}

static int run_impl(mtr_engine* e, int gen);
static int summary_params(mtr_engine* e, SParams& P);

int mtr_run(mtr_engine* e) { return run_impl(e, 0); }

int64_t mtr_get_deltas(mtr_engine* e, uint32_t doc, mtr_delta* out, int64_t cap) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (doc >= e->max_docs) {
        set_err("mtr_get_deltas: bad document");
        return -1;
    }
    DocHdr h;
    HIPCHK(hipMemcpy(&h, e->hdr.p + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
    const int64_t n = h.dused;
    if (n > cap) return -n;
    if (n && e->has_delta && doc < e->n_docs)
        HIPCHK(hipMemcpy(out, e->delta.p + e->h_doff[doc] * 4, size_t(n) * sizeof(mtr_delta),
                         hipMemcpyDeviceToHost));
    return n;
}

int64_t mtr_get_props(mtr_engine* e, uint32_t doc, uint32_t ref, uint32_t* out, int64_t cap) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const uint64_t pw = e->caps.prop_words;
    if (doc >= e->max_docs || ref >= pw) {
        set_err("mtr_get_props: bad document or properties reference");
        return -1;
    }
    const uint32_t* base = e->prop.p + size_t(doc) * pw;
    uint32_t n = 0;
    HIPCHK(hipMemcpy(&n, base + ref, 4, hipMemcpyDeviceToHost));
    const int64_t words = 1 + 2 * int64_t(n);
    if (uint64_t(ref) + uint64_t(words) > pw) {
        set_err("mtr_get_props: reference outside the property arena");
        return -1;
    }
    if (words > cap) return -words;
    HIPCHK(hipMemcpy(out, base + ref, size_t(words) * 4, hipMemcpyDeviceToHost));
    return words;
}

int mtr_set_matrix(mtr_engine* e, uint32_t rows_doc, uint32_t cols_doc) {
    HIPCHK(hipSetDevice(e->device));
    if (rows_doc >= e->h_kind.size() || cols_doc >= e->h_kind.size() || rows_doc == cols_doc ||
        e->h_kind[rows_doc] || e->h_kind[cols_doc]) {
        set_err("mtr_set_matrix: bad or already paired documents");
        return MTR_ERR_BAD_OP;
    }
    {  // a pair's HBM-resident launches hold two documents' chunk rows in LDS
        const size_t need = 2 * ((lds_bytes_global_mode(int(e->caps.max_segments)) + 15) & ~size_t(15));
        if (e->dev_lds > 0 && need > size_t(e->dev_lds)) {
            set_err("mtr_set_matrix: max_segments " + std::to_string(e->caps.max_segments) + " needs " +
                    std::to_string(need) + " bytes of LDS for a matrix pair in HBM-resident mode (device: " +
                    std::to_string(e->dev_lds) + ")");
            return MTR_ERR_CAPACITY;
        }
    }
    e->h_kind[rows_doc] = 1;
    e->h_kind[cols_doc] = 2;
    e->h_part[rows_doc] = cols_doc;
    e->h_part[cols_doc] = rows_doc;
    HIPCHK(hipMemcpyAsync(e->dkind.p, e->h_kind.data(), e->h_kind.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          e->stream));
    HIPCHK(hipMemcpyAsync(e->dpart.p, e->h_part.data(), e->h_part.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return MTR_OK;
}

static int run_impl(mtr_engine* e, int gen) {
    HIPCHK(hipSetDevice(e->device));
    if (e->n_docs == 0) return MTR_OK;
    const int K = int(e->caps.ops_per_launch ? e->caps.ops_per_launch : 0x7fffffff);
    e->launches = 0;
    e->t_apply = 0;
    e->t_kernels = 0;
    KParams P{};
    P.hdr = e->hdr.p;
    P.seg = e->seg.p;
    P.heap = e->heap.p;
    P.text = e->text.p;
    P.prop = e->prop.p;
    P.rm = e->rm.p;
    P.segcap = int(e->caps.max_segments);
    P.hcap = int(e->caps.heap_entries);
    P.tcap = int(e->caps.text_units);
    P.pcap = int(e->caps.prop_words);
    P.rcap = int(e->caps.remover_cells);
    P.rtab = e->rtab;
    P.new_length_calc = e->opt.new_length_calc;
    P.n_docs = e->n_docs;
    P.ops = e->ops.p;
    P.docs = e->docs.p;
    P.btext = e->btext.p;
    P.propop_off = e->propop_off.p;
    P.propop_kv = e->propop_kv.p;
    P.key_index = e->key_index.p;
    P.val_eq = e->val_eq.p;
    P.stat_ops = e->stat.p;
    P.delta = e->delta.p;
    P.doff = e->has_delta ? e->doff.p : nullptr;
    P.dkind = e->dkind.p;
    P.dpart = e->dpart.p;
    P.pend = e->pend.p;
    P.refs = e->refs.p;
    P.refcap = int(e->caps.ref_slots);
    P.gen = gen;
#ifdef MTR_PROF
    if (!e->prof.p) {
        if (e->prof.ensure(64)) return -1;
        HIPCHK(hipMemset(e->prof.p, 0, 64 * sizeof(unsigned long long)));
    }
    P.prof = e->prof.p;
#endif
    if (gen) {
        P.gen_cfg = e->gcfg;
        P.gen_grow = int32_t(e->ggrow);
        P.gen_state = e->gstate.p;
        P.gen_ops = e->ops.p;
        P.gen_text = e->btext.p;
    }
    int dev_lds = 0;
    HIPCHK(hipDeviceGetAttribute(&dev_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, e->device));
    // documents whose class needs more LDS than this stay HBM-resident (MTR_LDS_LIMIT, bytes; tuning knob)
    static const size_t lds_limit = [] {
        const char* v = std::getenv("MTR_LDS_LIMIT");
        return v ? std::min<size_t>(size_t(std::atoll(v)), 160 * 1024) : size_t(160 * 1024);
    }();
    // Size classes of `class_leaves` leaves (SharedString classes: LDS sized to the class's largest
    // document plus `slack` leaves; a document that runs out of room yields before the op and is
    // classed again next round).  Tuning knobs: MTR_CLASS_LEAVES, MTR_SLACK.
    static const int class_env = [] {
        const char* v = std::getenv("MTR_CLASS_LEAVES");
        return v ? std::max(16, std::atoi(v)) : 0;
    }();
    // concurrent launch lanes (1..kLanes) and whether the fixed-capacity kernels are used (tuning knobs:
    // MTR_LANES, MTR_NO_FIXED_CAP)
    static const int nlanes = [] {
        const char* v = std::getenv("MTR_LANES");
        return v ? std::max(1, std::min(int(mtr_engine::kLanes), std::atoi(v))) : int(mtr_engine::kLanes);
    }();
    static const bool no_fixed_cap = std::getenv("MTR_NO_FIXED_CAP") != nullptr;
    // matrix pairs on one wave even when two could run them (tuning knob MTR_PAIR1)
    static const bool pair1 = std::getenv("MTR_PAIR1") != nullptr;
    static const bool ptrace = std::getenv("MTR_PIPE_TRACE") != nullptr;  // (host timeline of a pipelined run)
    const auto tr0 = std::chrono::steady_clock::now();
    auto trace = [&](const char* what, int a, int b) {
        if (ptrace)
            std::fprintf(stderr, "pipe %8.3f ms %s %d %d\n",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count(),
                         what, a, b);
    };
    static const int slack_env = [] {
        const char* v = std::getenv("MTR_SLACK");
        return v ? std::max(0, std::atoi(v)) : -1;
    }();
    // the LRU heap's floor in a yielding (tight) launch: cap / heap_div entries (tuning knob MTR_HEAP_DIV)
    static const int heap_div = [] {
        const char* v = std::getenv("MTR_HEAP_DIV");
        return v ? std::max(1, std::atoi(v)) : 8;
    }();
    // Independent document groups (tuning knob MTR_GROUPS, 1..kLanes): each group runs its own round loop
    // (classify -> one launch per size class -> classify ...) on its own streams, so one group's launches fill
    // the device while another's last documents of a round finish (a round is quantised by how many of its
    // documents the device holds at once).  SharedMatrix pairs keep one group.
    // Default: two groups for batches of 4,096 to 60,000 documents -- the 2- to 8-GPU shares of
    // C3 gain 5-10 % (profiles/r04_groups.json); above that one group (a round already fills the device), and
    // more than two leave each group too few lanes.
    static const int groups_env = [] {
        const char* v = std::getenv("MTR_GROUPS");
        return v ? std::max(1, std::min(int(mtr_engine::kLanes), std::atoi(v))) : 0;
    }();
    int n_cu = 0;
    HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, e->device));
    const bool few_docs = e->n_docs <= uint32_t(std::max(n_cu, 1));
    bool any_pair = false;
    for (uint32_t d = 0; d < e->n_docs && d < e->h_kind.size(); d++) any_pair = any_pair || e->h_kind[d] != 0;
    // (round 6: two groups at 100,000 documents too -- 424.4 M against 418.5 M ops/s on one box; the per-launch
    // roofline figure that kept one group there is no longer the headline, the step span is; a pipelined hand-over
    // keeps one group, whose lanes take the landing parts in order)
    const int g_want = groups_env > 0 ? groups_env : (e->n_docs >= 4096u && !e->pipe_parts ? 2 : 1);
    // Default class width: 128 leaves for the batches that run two groups (4,096 to 60,000 documents) -- half the
    // launches per round of 64-leaf classes, which at those sizes cost more than the wider classes' LDS spread
    // (profiles/r04_class_sweep.json: 12,500 documents 379.0 M vs 341.4 M ops/s, 25,000 395.5 M vs 385.0 M);
    // 64 above (100,000: 407.7 M vs 400.5 M) and below; 128 for matrix pairs too (C4: 46.7 M vs 38.9 M ops/s,
    // profiles/r04_sched_sweep.json)
    const int class_leaves = class_env > 0 ? class_env
                                           : (any_pair || (e->n_docs >= 4096u && e->n_docs <= 60000u) ? 128 : 64);
    // (a pipelined hand-over: its parts still landing; a group takes whole parts)
    const uint32_t PP = gen ? 0u : e->pipe_parts;
    const bool psum = PP && e->pipe_out;  // (mtr_replay_pipelined)
    // ops per launch of a pipelined run: twice the engine's -- while parts are landing a round holds few documents,
    // so its fixed costs (the launches' ramp and tail, the class read-back) weigh more per op; C3 end-to-end
    // 270.1 -> 264.3 ms at 96 against 48, the device-resident rate unchanged (profiles/r06_e2e_sweep.json)
    static const int pipe_k_env = [] {
        const char* v = std::getenv("MTR_PIPE_K");
        return v ? std::atoi(v) : 0;
    }();
    const int Kr = !PP ? K : pipe_k_env > 0 ? pipe_k_env : int(std::min<int64_t>(2 * int64_t(K), 0x7fffffff));
    int G = any_pair ? 1 : std::max(1, std::min<int>(g_want, int(e->n_docs)));
    if (PP) G = std::min<int>(int(e->pipe_groups), int(PP));
    const int L = std::max(1, nlanes / G);  // lanes (streams) per group
    const size_t ncls = 1 + 3 * kAllClasses;
    if (e->cls.ensure(ncls * mtr_engine::kLanes) || e->dlist.ensure(size_t(kAllClasses) * e->n_docs)) return -1;
    if (!e->h_cls) {
        HIPCHK(hipHostMalloc((void**)&e->h_cls, ncls * mtr_engine::kLanes * sizeof(int32_t),
                             hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&e->d_cls, e->h_cls, 0));
    }
    // stream index of group g's lane l.  A pipelined run uses all four streams whatever MTR_LANES says: the last
    // one is the copy stream, a launch lane again once every part has landed -- group 0's lanes are streams 0 (and 1
    // with two groups), group 1's stream 2 and then 3; one group: streams 0-2, then 3
    auto lane_si = [&](int g, int l) -> int {
        if (PP && G == 2) return g == 0 ? l : 2 + l;
        return PP ? l : g * L + l;
    };
    auto lane_stream = [&](int g, int l) -> hipStream_t {
        const int si = lane_si(g, l);
        return si == 0 ? e->stream : e->aux[si - 1];
    };
    // the lanes group g launches on this round
    auto lanes_of = [&](int g) -> int {
        if (!PP) return L;
        const int base = G == 2 ? (g == 0 ? 2 : 1) : int(mtr_engine::kLanes) - 1;
        if ((G == 2 && g == 0) || psum) return base;  // (the copy stream: group 1's second lane; summaries' stream)
        const hipError_t q = hipEventQuery(e->part_ev[e->pipe_last]);
        return q == hipSuccess ? base + 1 : base;
    };
    struct Grp {
        uint32_t lo = 0, hi = 0;
        bool done = false;
        uint32_t p_lo = 0, p_hi = 0, waited = 0;  // pipelined: its parts [p_lo, p_hi), [waited, p_hi) not waited for
    };
    std::vector<Grp> grp(static_cast<size_t>(G));
    for (int g = 0; g < G; g++) {
        Grp& gr = grp[size_t(g)];
        if (PP) {  // (mtr_submit_pipelined's split: two groups take [0, half) and [half, PP))
            const uint32_t half = (PP + 1) / 2;
            gr.waited = G == 2 && g == 1 ? half : 0u;
            gr.p_lo = gr.waited;
            gr.p_hi = G == 2 && g == 0 ? half : PP;
            gr.lo = e->part_lo[gr.waited];
            gr.hi = e->part_lo[gr.p_hi];
        } else {
            gr.lo = uint32_t(uint64_t(e->n_docs) * uint64_t(g) / uint64_t(G));
            gr.hi = uint32_t(uint64_t(e->n_docs) * uint64_t(g + 1) / uint64_t(G));
        }
    }
    // the groups' lanes start after everything queued on the engine stream (the batch upload)
    HIPCHK(hipEventRecord(e->ev[0], e->stream));
    if (PP) {
        for (int si = 1; si < int(mtr_engine::kLanes); si++) HIPCHK(hipStreamWaitEvent(e->aux[si - 1], e->ev[0], 0));
    } else {
        for (int g = 0; g < G; g++)
            for (int l = 0; l < L; l++)
                if (g * L + l > 0) HIPCHK(hipStreamWaitEvent(lane_stream(g, l), e->ev[0], 0));
    }
    // classify group g (on its first lane) and read its class counts back
    auto classify = [&](int g) -> int {
        Grp& gr = grp[size_t(g)];
        // (pipelined summaries: the parts that have landed by now count as waited for -- this classify sees all
        // of their documents, so a part it finds with no ops left is done)
        if (psum)
            while (gr.waited < gr.p_hi && hipEventQuery(e->part_ev[gr.waited]) == hipSuccess) gr.waited++;
        hipStream_t st = lane_stream(g, 0);
        int32_t* dcls = e->cls.p + size_t(g) * ncls;
        // (the counters are zeroed and read back by kernels, the read-back into mapped page-locked memory: a DMA
        // copy would queue behind mtr_submit_pipelined's uploads on the copy engine)
        words_kernel<<<1, 256, 0, st>>>(dcls, nullptr, int(ncls));
        if (psum) words_kernel<<<1, 256, 0, st>>>(e->pleft.p + gr.p_lo, nullptr, int(gr.p_hi - gr.p_lo));
        const uint32_t n = gr.hi - gr.lo;
        classify_kernel<<<(n + 255) / 256, 256, 0, st>>>(e->hdr.p, e->docs.p, gr.lo, gr.hi, e->dkind.p, e->dpart.p,
                                                         dcls, e->dlist.p + size_t(kAllClasses) * gr.lo, class_leaves,
                                                         psum ? e->pleft.p : nullptr, e->dpart_lo.p, PP);
        words_kernel<<<1, 256, 0, st>>>(e->d_cls + size_t(g) * ncls, dcls, int(ncls));
        if (psum) words_kernel<<<1, 256, 0, st>>>(e->d_pleft + gr.p_lo, e->pleft.p + gr.p_lo, int(gr.p_hi - gr.p_lo));
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e->grp_cls[g], st));
        return 0;
    };
    // HBM-resident launches need the scratch / chunk-record buffers: allocated by the first such launch
    auto ensure_global = [&]() -> int {
        if (e->scratch.ensure(size_t(e->n_docs) * 2 * P.segcap)) return -1;
        if (!e->csum.p) {  // for every document the engine may hold: it must never move
            const size_t n = size_t(std::max<uint32_t>(e->max_docs, 1)) * csum_ints(int(P.segcap));
            if (e->csum.ensure(n)) return -1;
            if (e->umap.ensure(size_t(std::max<uint32_t>(e->max_docs, 1)) * 2 * size_t(P.segcap))) return -1;
            HIPCHK(hipMemsetAsync(e->umap.p, 0xff, e->umap.n * sizeof(int32_t), e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
        }
        return 0;
    };
    // one round of group g: a launch per size class, spread over the group's lanes, joined on its first lane
    auto issue_round = [&](int g, bool& stuck) -> int {
        Grp& gr = grp[size_t(g)];
        const int Lr = lanes_of(g);
        const int32_t* cls = e->h_cls + size_t(g) * ncls;
        const uint32_t n = gr.hi - gr.lo;
        const int k = std::min(Kr, cls[0]);
        hipStream_t st0 = lane_stream(g, 0);
        HIPCHK(hipEventRecord(e->grp_fork[g], st0));
        int nl = 0;  // launches of this round
        for (int c = kAllClasses - 1; c >= 0; c--) {  // one launch per size class: matrix pairs, then the
            const bool pair = c >= kClasses;              // SharedString classes, largest documents first
            const int cnt = cls[1 + 3 * c], maxseg = cls[2 + 3 * c], maxheap = cls[3 + 3 * c];
            if (cnt <= 0) continue;
            // replay launches of SharedString documents yield when their leaves or LRU heap could
            // overflow the launch's LDS, so they get `slack` leaves of room; matrix pairs (setCell
            // splits) and record mode (ops drawn once) keep room for every op of the launch
            const bool tight = !pair && !P.gen;
            // (a batch of fewer documents than CUs has LDS to spare: room for the whole launch, so a document
            // does not yield and wait for a round of its own)
            const int slack = slack_env >= 0 ? slack_env : (few_docs ? k + 8 : 8);
            int cap = tight ? round32(maxseg + slack + 8) : round64(maxseg + 2 * k + 8);
            // (a yielding launch above 1,024 leaves: the next multiple of 64, a capacity with a compile-time layout)
            if (tight && cap > 1024 && cap <= 1536) cap = round64(cap);
            if (cap > P.segcap) cap = P.segcap;
            // LRU heap: what the class holds now plus room for this launch's pushes; a document that
            // could overflow it stops before the op and asks for more (DocHdr.heap_need)
            // (matrix pairs replaying remote messages: a smaller floor -- a document whose op could overflow the heap
            // yields before it like any other, and two matrices of the larger classes then fit one CU's LDS)
            int lhcap = std::min<int>(P.hcap, pair && !P.gen ? std::max(cap / 16, round32(maxheap + 2 * k + 8))
                                               : std::max(cap / (tight ? heap_div : 8),
                                                          tight ? round32(maxheap + slack + 8)
                                                                : round64(maxheap + 2 * k + 8)));
            size_t lds = lds_bytes(cap, lhcap, P.gen != 0);
            if (pair) lds = 2 * ((lds + 15) & ~size_t(15));
            KParams Q = P;
            Q.global_mode = 0;
            if (lds > lds_limit) {
                // documents larger than LDS: leaves, heap and scan arrays stay in the HBM slab
                if (ensure_global()) return -1;
                Q.csum = e->csum.p;
                Q.umap = e->umap.p;
                Q.global_mode = 1;
                Q.scratch = e->scratch.p;
                cap = Q.segcap;
                lhcap = Q.hcap;
                lds = lds_bytes_global_mode(int(Q.segcap));
                if (pair) lds = 2 * ((lds + 15) & ~size_t(15));
            }
            const int kk = tight && !Q.global_mode ? k : std::max(1, std::min(k, (cap - maxseg - 8) / 2));
            if (cap - maxseg - 8 < 2 && cap >= Q.segcap) stuck = true;  // no room and no larger LDS class
            Q.cap = cap;
            Q.lhcap = lhcap;
            Q.ops_this_launch = kk;
            Q.doc_list = e->dlist.p + size_t(kAllClasses) * gr.lo + size_t(c) * n;
            Q.n_launch = uint32_t(cnt);
            const int lane = nl % Lr;
            hipStream_t st = lane_stream(g, lane);
            if (lane != 0 && nl < Lr) HIPCHK(hipStreamWaitEvent(st, e->grp_fork[g], 0));
            const size_t q = size_t(e->launches);
            while (e->kev.size() < 2 * (q + 1)) {
                hipEvent_t x;
                HIPCHK(hipEventCreate(&x));
                e->kev.push_back(x);
            }
            HIPCHK(hipEventRecord(e->kev[2 * q], st));
            int av = -1;
            if (pair) {
                av = Q.gen ? (Q.global_mode ? AV_PAIR_HBM_GN : AV_PAIR_LDS_GN)  // record mode (mtr_generate_matrix)
                     : Q.doff ? (Q.global_mode ? AV_PAIR_HBM_DL : AV_PAIR_LDS_DL)  // a matrix tracked for its cells
                     : (Q.global_mode ? AV_PAIR_HBM : AV_PAIR_LDS);
                // replaying remote messages only: a wave per vector (run_pair2), if its exchange words fit
                if (!Q.gen && !Q.doff && !e->has_ext && !e->pend_seen && !pair1 &&
                    lds + kPair2Xch <= size_t(std::max(dev_lds, 0))) {
                    av = Q.global_mode ? AV_PAIR2_HBM : AV_PAIR2_LDS;
                    // (an LDS pair2 launch keeps no props arrays: remote messages only, Eng::NOPROPS)
                    if (!Q.global_mode) lds = 2 * ((lds_bytes(cap, lhcap, false, 7) + 15) & ~size_t(15));
                    lds += kPair2Xch;
                }
            } else if (Q.gen) {  // record mode: the generating instantiation
                av = Q.global_mode ? AV_HBM_GN : AV_LDS_GN;
            } else if (Q.doff) {  // a batch with MTR_F_DELTA ops: the delta-reporting instantiation
                av = Q.global_mode ? AV_HBM_DL : AV_LDS_DL;
            } else if (Q.global_mode) {  // HBM-resident: the lean instantiation unless the batch has rare records
                av = e->has_ext ? AV_HBM_X : AV_HBM_LEAN;
            } else if (e->has_ext) {
                av = AV_LDS_X;
            } else if (no_fixed_cap || (!launch_fixed_cap_p0(cap, uint32_t(cnt), lds, st, Q) &&
                       !launch_fixed_cap_p1(cap, uint32_t(cnt), lds, st, Q) &&
                       !launch_fixed_cap_p2(cap, uint32_t(cnt), lds, st, Q))) {
                av = AV_LDS_LEAN;  // above the fixed classes: runtime layout, lean
            }
            const uint32_t region = !pair ? 0u : uint32_t((av == AV_PAIR2_LDS || av == AV_PAIR2_HBM ? lds - kPair2Xch : lds) / 2);
            if (av >= 0 && !launch_variant(av, uint32_t(cnt), lds, st, Q, region)) {
                set_err("no apply kernel variant " + std::to_string(av));
                return -1;
            }
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(e->kev[2 * q + 1], st));
            e->launches++;
            nl++;
        }
        for (int l = 1; l < std::min(nl, Lr); l++) {  // join the lanes
            const int si = lane_si(g, l);
            HIPCHK(hipEventRecord(e->lane_done[si], lane_stream(g, l)));
            HIPCHK(hipStreamWaitEvent(st0, e->lane_done[si], 0));
        }
        return 0;
    };
    // pipelined summaries (mtr_replay_pipelined): a part whose documents have no ops left is summarized on the copy
    // stream -- the size pass, its sizes read back into mapped memory, the offsets (parts in order), the write pass
    // and the blobs' download into the caller's buffer -- while the other parts still apply
    SParams SP{};
    std::vector<int> pstate;  // per part: 0 applying, 1 done (pdone_ev recorded), 2 sizing, 3 downloading
    uint32_t next_size = 0, next_dl = 0;
    int64_t pbase = 0;
    int prc = 0;  // a summary pass's error: no more passes, the apply runs out, then run_impl returns it
    if (psum) {
        e->summarized = false;
        if (summary_params(e, SP) || e->out.ensure(size_t(e->pipe_cap) + 16) || e->pleft.ensure(PP)) return -1;
        SP.out = e->out.p;
        if (e->h_pleft_n < PP) {
            if (e->h_pleft) HIPCHK(hipHostFree(e->h_pleft));
            HIPCHK(hipHostMalloc((void**)&e->h_pleft, size_t(PP) * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(hipHostGetDevicePointer((void**)&e->d_pleft, e->h_pleft, 0));
            e->h_pleft_n = PP;
        }
        if (e->h_psize_n < e->n_docs) {
            if (e->h_psize) HIPCHK(hipHostFree(e->h_psize));
            HIPCHK(hipHostMalloc((void**)&e->h_psize, size_t(e->n_docs) * sizeof(int64_t),
                                 hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(hipHostGetDevicePointer((void**)&e->d_psize, e->h_psize, 0));
            e->h_psize_n = e->n_docs;
        }
        for (auto* v : {&e->pdone_ev, &e->psize_ev, &e->pwrite_ev})
            while (v->size() < PP) {
                hipEvent_t x;
                HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
                v->push_back(x);
            }
        pstate.assign(PP, 0);
        e->h_size.assign(e->n_docs, 0);
        e->h_off.assign(e->n_docs, 0);
    }
    int left = G;  // groups still applying
    // (the summary kernels run on the copy stream while the apply runs, on the idle engine stream once it is done,
    // so the last parts' passes do not queue behind the downloads)
    auto pump = [&]() -> int {
        if (prc) return 0;
        hipStream_t ks = left == 0 ? e->stream : e->copy;
        while (next_size < PP && pstate[next_size] == 1) {  // size passes, parts in order
            const uint32_t p = next_size++, lo = e->part_lo[p], hi = e->part_lo[p + 1];
            HIPCHK(hipStreamWaitEvent(ks, e->pdone_ev[p], 0));
            SP.doc_base = lo;
            summary_size_kernel<<<hi - lo, 64, 0, ks>>>(SP);
            words64_kernel<<<(hi - lo + 255) / 256, 256, 0, ks>>>(e->d_psize + lo, e->out_size.p + lo, hi - lo);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(e->psize_ev[p], ks));
            pstate[p] = 2;
            trace("size", int(p), 0);
        }
        while (next_dl < next_size) {  // offsets, write pass, download, parts in order
            const hipError_t q = hipEventQuery(e->psize_ev[next_dl]);
            if (q == hipErrorNotReady) break;
            HIPCHK(q);
            const uint32_t p = next_dl++, lo = e->part_lo[p], hi = e->part_lo[p + 1];
            const int64_t base = pbase;
            for (uint32_t d = lo; d < hi; d++) {
                const int64_t z = e->h_psize[d];
                if (z < 0) {
                    set_err("document " + std::to_string(d) + " has more summary chunks than the engine's blob table");
                    return MTR_ERR_CAPACITY;
                }
                e->h_size[d] = z;
                e->h_off[d] = pbase;
                e->h_psize[d] = pbase;  // (the offsets go back through the same mapped words)
                pbase += z;
            }
            if (pbase > e->pipe_cap) {
                set_err("mtr_replay_pipelined: the output buffer holds " + std::to_string(e->pipe_cap) + " bytes, the "
                        "summaries need more");
                return MTR_ERR_CAPACITY;
            }
            words64_kernel<<<(hi - lo + 255) / 256, 256, 0, ks>>>(e->out_off.p + lo, e->d_psize + lo, hi - lo);
            SP.doc_base = lo;
            summary_write_kernel<<<hi - lo, 64, 0, ks>>>(SP);
            HIPCHK(hipGetLastError());
            if (ks != e->copy) {
                HIPCHK(hipEventRecord(e->pwrite_ev[p], ks));
                HIPCHK(hipStreamWaitEvent(e->copy, e->pwrite_ev[p], 0));
            }
            if (pbase > base)
                HIPCHK(hipMemcpyAsync(e->pipe_out + base, e->out.p + base, size_t(pbase - base), hipMemcpyDeviceToHost,
                                      e->copy));
            pstate[p] = 3;
            trace("download", int(p), int((pbase - base) >> 20));
        }
        return 0;
    };
    // pipelined: a group classifies again once the next of its parts has landed (its lane 0 waits for it)
    auto wait_part = [&](int g) -> int {
        Grp& gr = grp[size_t(g)];
        HIPCHK(hipStreamWaitEvent(lane_stream(g, 0), e->part_ev[gr.waited], 0));
        gr.waited++;
        return 0;
    };
    const size_t launches0 = size_t(e->launches);
    HIPCHK(hipEventRecord(e->ev[1], e->stream));  // (timing start: after the forks above)
    for (int g = 0; g < G; g++)
        if ((PP && wait_part(g)) || classify(g)) return -1;
    bool stuck = false;
    while (left > 0) {
        bool progressed = false;
        for (int g = 0; g < G; g++) {
            Grp& gr = grp[size_t(g)];
            if (gr.done) continue;
            const hipError_t q = hipEventQuery(e->grp_cls[g]);
            if (q == hipErrorNotReady) continue;
            HIPCHK(q);
            progressed = true;
            const int32_t* cls = e->h_cls + size_t(g) * ncls;
            if (psum) {  // parts classified after they landed with no ops left: done (before this round's launches)
                for (uint32_t p = gr.p_lo; p < gr.waited; p++)
                    if (pstate[p] == 0 && e->h_pleft[p] == 0) {
                        HIPCHK(hipEventRecord(e->pdone_ev[p], lane_stream(g, 0)));
                        pstate[p] = 1;
                        trace("done", int(p), g);
                    }
            }
            if (cls[0] <= 0) {
                if (PP && gr.waited < gr.p_hi) {  // more of the group's documents are still landing
                    if (wait_part(g) || classify(g)) return -1;
                    continue;
                }
                gr.done = true;
                trace("group-done", g, 0);
                left--;
                continue;
            }
            trace("round", g, cls[0]);
            if (issue_round(g, stuck)) return -1;
            if (stuck) break;
            if (classify(g)) return -1;  // queued behind the round's launches
        }
        if (stuck) break;
        if (psum) prc = pump();
        if (!progressed) std::this_thread::yield();
    }
    while (psum && !stuck && !prc && next_dl < PP) {  // the last parts' summaries
        prc = pump();
        if (next_dl < PP) std::this_thread::yield();
    }
    for (int g = 0; g < G; g++)
        if (g > 0) {  // join every group into the engine stream
            HIPCHK(hipEventRecord(e->lane_done[lane_si(g, 0)], lane_stream(g, 0)));
            HIPCHK(hipStreamWaitEvent(e->stream, e->lane_done[lane_si(g, 0)], 0));
        }
    HIPCHK(hipEventRecord(e->ev[2], e->stream));
    HIPCHK(hipEventSynchronize(e->ev[2]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[1], e->ev[2]));
    e->t_apply += ms;
    for (size_t q = launches0; q < size_t(e->launches); q++) {
        float kms = 0;
        HIPCHK(hipEventElapsedTime(&kms, e->kev[2 * q], e->kev[2 * q + 1]));
        e->t_kernels += kms;
    }
    if (PP) {  // the parts' op-scan bits: a part holding records the pipelined path does not run was not started
        e->pipe_parts = 0;
        HIPCHK(hipStreamSynchronize(e->copy));
        trace("end", int(prc), 0);
        for (uint32_t p = 0; p < PP; p++)
            if (e->h_pflags[p]) {
                set_err("mtr_submit_pipelined: documents " + std::to_string(e->part_lo[p]) + ".." +
                        std::to_string(e->part_lo[p + 1]) + " hold records beyond remote ops (MTR_F_DELTA, local ops, "
                        "local references or rare records); mtr_reset and submit the batch with mtr_submit");
                return MTR_ERR_UNSUPPORTED;
            }
        if (prc) return prc;  // (a summary pass's error: the batch is applied, the summaries are not built)
        if (psum && !stuck) {
            e->out_total = pbase;
            e->summarized = true;
        }
    }
    if (stuck) {
        set_err("document exceeds the leaf capacity");
        return MTR_ERR_CAPACITY;
    }
    if (!psum) e->summarized = false;
    return MTR_OK;
}

int64_t mtr_replay_pipelined(mtr_engine* e, const mtr_batch* b, uint32_t parts, uint8_t* out, int64_t cap,
                             int64_t* doc_off) {
    const uint32_t n = b->n_docs;
    // a range of fewer than ~3,000 documents keeps too few in flight while the ranges land (one document group, every
    // round small): C2's 10,000 documents in 2 / 4 / 8 / 16 ranges measured 490 / 472 / 482 / 476 ms end to end
    // against 464 ms for the serial calls, C3's 100,000 in 16 ranges 258 against 322 ms (profiles/r06_e2e_sweep.json)
    const char* mpd = std::getenv("MTR_PIPE_MIN_PART_DOCS");
    const uint32_t min_part_docs = mpd ? uint32_t(std::max(0, std::atoi(mpd))) : 3000u;
    if (parts > 1 && n / parts < min_part_docs) parts = 1;  // (mtr_submit_pipelined: parts <= 1 is mtr_submit)
    e->pipe_one_group = true;
    int rc = mtr_submit_pipelined(e, b, parts);
    e->pipe_one_group = false;
    if (rc != MTR_OK) return -1;
    if (e->pipe_parts) {
        e->pipe_out = out;
        e->pipe_cap = cap;
        rc = run_impl(e, 0);
        e->pipe_out = nullptr;
        if (rc != MTR_OK) return -1;
        if (doc_off) {
            for (uint32_t d = 0; d < n; d++) doc_off[d] = e->h_off[d];
            doc_off[n] = e->out_total;
        }
        return e->out_total;
    }
    // (a batch the pipelined path does not take: mtr_submit's, then the ordinary summarize and download)
    if (mtr_run(e) != MTR_OK || mtr_summarize(e) != MTR_OK) return -1;
    const int64_t r = mtr_get_summaries(e, 0, n, out, cap, doc_off);
    if (r < -1) set_err("mtr_replay_pipelined: the output buffer holds " + std::to_string(cap) + " bytes, the summaries "
                        "need " + std::to_string(-r));
    return r < 0 ? -1 : r;
}

__global__ void synth_init_kernel(mtr_synth_cfg cfg, mtr_synth_state* st, uint32_t n) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n) mtr_synth_init(&cfg, d, &st[d]);
}
__global__ void synth_text_count_kernel(const mtr_synth_state* st, mtr_doc_desc* docs, uint32_t n) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n) docs[d].text_count = st[d].text_used;
}

// the pre-grown documents' snapshot header segments (the oracle's generate_impl writes the same records):
// segment k of every document is the two units ('a' + k % 26, 'A' + k / 26 % 26), NonCollabClient, no merge info
__global__ void synth_grow_kernel(mtr_op* ops, uint16_t* text, mtr_synth_state* st, uint32_t n, uint32_t per,
                                  uint32_t text_cap, uint32_t grow) {
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= uint64_t(n) * (grow + 1)) return;
    const uint32_t d = uint32_t(t / (grow + 1)), k = uint32_t(t % (grow + 1));
    mtr_op op{};
    if (k < grow) {
        op.type = MTR_OP_LOAD;
        op.client = uint16_t(MTR_CLIENT_NONCOLLAB);
        op.ref_seq = -1;
        op.pos2 = -1;
        op.payload = 2 * k;
        op.payload2 = 2;
        text[uint64_t(d) * text_cap + 2 * k] = uint16_t('a' + k % 26);
        text[uint64_t(d) * text_cap + 2 * k + 1] = uint16_t('A' + (k / 26) % 26);
    } else {
        op.type = MTR_OP_START_COLLAB;
        st[d].text_used = 2 * grow;
    }
    ops[uint64_t(d) * per + k] = op;
}

int mtr_generate(mtr_engine* e, const mtr_synth_cfg* cfg, const mtr_batch* tables) {
    return mtr_generate_grown(e, cfg, tables, 0);
}

int mtr_generate_grown(mtr_engine* e, const mtr_synth_cfg* cfg, const mtr_batch* tables, uint32_t grow) {
    HIPCHK(hipSetDevice(e->device));
    if (cfg->n_docs > e->max_docs || cfg->writers > MTR_SYNTH_MAX_WRITERS || cfg->writers + 1 > 0xfd ||
        uint64_t(cfg->text_cap) < 2ull * grow) {
        set_err("mtr_generate: bad configuration");
        return MTR_ERR_BAD_OP;
    }
    const uint32_t n = cfg->n_docs, per = grow + cfg->ops_per_doc + 1;
    if (n == 0) return mtr_reset(e);
    std::vector<mtr_doc_desc> docs(n);
    for (uint32_t d = 0; d < n; d++) {
        docs[d].op_begin = uint64_t(d) * per;
        docs[d].op_count = per;
        docs[d].text_base = uint64_t(d) * cfg->text_cap;
        docs[d].text_count = 0;
        docs[d].client_base = 0;
        docs[d].n_clients = cfg->writers + 1;
    }
    mtr_batch b = *tables;
    b.n_docs = n;
    b.docs = docs.data();
    b.n_ops = 0;
    b.n_text = 0;
    if (mtr_reset(e) != MTR_OK || mtr_submit(e, &b) != MTR_OK) return -1;
    if (e->ops.ensure(size_t(n) * per) || e->btext.ensure(size_t(n) * cfg->text_cap) || e->gstate.ensure(n)) return -1;
    e->gcfg = *cfg;
    e->ggrow = grow;
    synth_init_kernel<<<(n + 255) / 256, 256, 0, e->stream>>>(*cfg, e->gstate.p, n);
    HIPCHK(hipGetLastError());
    if (grow) {
        const uint64_t total = uint64_t(n) * (grow + 1);
        synth_grow_kernel<<<uint32_t((total + 255) / 256), 256, 0, e->stream>>>(e->ops.p, e->btext.p, e->gstate.p, n,
                                                                               per, cfg->text_cap, grow);
        HIPCHK(hipGetLastError());
    }
    const int rc = run_impl(e, 1);
    e->ggrow = 0;
    if (rc != MTR_OK) return -1;
    synth_text_count_kernel<<<(n + 255) / 256, 256, 0, e->stream>>>(e->gstate.p, e->docs.p, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    return MTR_OK;
}

// matrix m's generator state lives with its rows vector (engine document 2m), seeded as matrix m
__global__ void synth_init_matrix_kernel(mtr_synth_cfg cfg, mtr_synth_state* st, uint32_t n) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < 2 * n) mtr_synth_init(&cfg, d / 2, &st[d]);
}

int mtr_generate_matrix(mtr_engine* e, const mtr_synth_cfg* cfg, const mtr_batch* tables) {
    HIPCHK(hipSetDevice(e->device));
    const uint32_t n = cfg->n_docs, per = cfg->ops_per_doc + 1;
    if (2ull * n > e->max_docs || cfg->writers > MTR_SYNTH_MAX_WRITERS || cfg->writers + 1 > 0xfd) {
        set_err("mtr_generate_matrix: bad configuration");
        return MTR_ERR_BAD_OP;
    }
    if (n == 0) return mtr_reset(e);
    for (uint32_t m = 0; m < n; m++) {  // pair the vectors (mtr_set_matrix) unless already paired so
        const uint32_t r = 2 * m, c = 2 * m + 1;
        if (e->h_kind[r] == 1 && e->h_part[r] == c) continue;
        if (e->h_kind[r] || e->h_kind[c]) {
            set_err("mtr_generate_matrix: documents 2m, 2m+1 are paired otherwise");
            return MTR_ERR_BAD_OP;
        }
        e->h_kind[r] = 1;
        e->h_kind[c] = 2;
        e->h_part[r] = c;
        e->h_part[c] = r;
    }
    HIPCHK(hipMemcpyAsync(e->dkind.p, e->h_kind.data(), e->h_kind.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          e->stream));
    HIPCHK(hipMemcpyAsync(e->dpart.p, e->h_part.data(), e->h_part.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          e->stream));
    std::vector<mtr_doc_desc> docs(2 * size_t(n));
    for (uint32_t m = 0; m < n; m++) {
        for (uint32_t w = 0; w < 2; w++) {
            mtr_doc_desc& x = docs[2 * m + w];
            x.op_begin = uint64_t(m) * per;
            x.op_count = w == 0 ? per : 0;  // the cols vector has no op list of its own
            x.text_base = 0;
            x.text_count = 0;
            x.client_base = 0;
            x.n_clients = cfg->writers + 1;
        }
    }
    mtr_batch b = *tables;
    b.n_docs = 2 * n;
    b.docs = docs.data();
    b.n_ops = 0;
    b.n_text = 0;
    if (mtr_reset(e) != MTR_OK || mtr_submit(e, &b) != MTR_OK) return -1;
    if (e->ops.ensure(size_t(n) * per) || e->btext.ensure(1) || e->gstate.ensure(2 * size_t(n))) return -1;
    e->gcfg = *cfg;
    e->gcfg.text_cap = 0;  // the matrix recipe draws no text
    synth_init_matrix_kernel<<<(2 * n + 255) / 256, 256, 0, e->stream>>>(*cfg, e->gstate.p, n);
    HIPCHK(hipGetLastError());
    if (run_impl(e, 1) != MTR_OK) return -1;
    HIPCHK(hipStreamSynchronize(e->stream));
    return MTR_OK;
}

int mtr_download_batch(mtr_engine* e, uint32_t lo, uint32_t hi, mtr_doc_desc* docs, mtr_op* ops, uint16_t* text,
                       uint64_t text_cap) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (hi > e->n_docs || lo > hi) {
        set_err("mtr_download_batch: bad range");
        return -1;
    }
    std::vector<mtr_doc_desc> dd(hi - lo);
    if (hi > lo) HIPCHK(hipMemcpy(dd.data(), e->docs.p + lo, (hi - lo) * sizeof(mtr_doc_desc), hipMemcpyDeviceToHost));
    // op lists: one copy per run of documents whose lists are adjacent on the device (a recorded
    // batch is one run); empty lists (matrix cols vectors) never break a run
    uint64_t op_at = 0, text_at = 0, text_need = 0;
    if (ops) {
        uint64_t run_src = 0, run_dst = 0, run_n = 0;
        for (uint32_t i = 0; i < hi - lo; i++) {
            const mtr_doc_desc& x = dd[i];
            if (x.op_count == 0) continue;
            if (run_n && x.op_begin != run_src + run_n) {
                HIPCHK(hipMemcpy(ops + run_dst, e->ops.p + run_src, run_n * sizeof(mtr_op), hipMemcpyDeviceToHost));
                run_n = 0;
            }
            if (!run_n) {
                run_src = x.op_begin;
                run_dst = op_at;
            }
            run_n += x.op_count;
            op_at += x.op_count;
        }
        if (run_n) HIPCHK(hipMemcpy(ops + run_dst, e->ops.p + run_src, run_n * sizeof(mtr_op), hipMemcpyDeviceToHost));
    }
    for (uint32_t i = 0; i < hi - lo; i++) text_need += dd[i].text_count;
    if (text && text_need && text_need <= text_cap) {
        // texts: one copy of the span when the gaps between documents are small, then compacted
        uint64_t t0 = UINT64_MAX, t1 = 0;
        for (uint32_t i = 0; i < hi - lo; i++)
            if (dd[i].text_count) {
                t0 = std::min<uint64_t>(t0, dd[i].text_base);
                t1 = std::max<uint64_t>(t1, dd[i].text_base + dd[i].text_count);
            }
        if (t1 - t0 <= 4 * text_need + (1u << 20)) {
            std::vector<uint16_t> span(t1 - t0);
            HIPCHK(hipMemcpy(span.data(), e->btext.p + t0, span.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < hi - lo; i++) {
                std::memcpy(text + text_at, span.data() + (dd[i].text_base - t0), dd[i].text_count * sizeof(uint16_t));
                text_at += dd[i].text_count;
            }
        } else {
            for (uint32_t i = 0; i < hi - lo; i++) {
                if (dd[i].text_count)
                    HIPCHK(hipMemcpy(text + text_at, e->btext.p + dd[i].text_base, dd[i].text_count * sizeof(uint16_t),
                                     hipMemcpyDeviceToHost));
                text_at += dd[i].text_count;
            }
        }
    }
    op_at = 0;
    text_at = 0;
    for (uint32_t i = 0; i < hi - lo; i++) {
        mtr_doc_desc x = dd[i];
        x.op_begin = op_at;
        x.text_base = text_at;
        op_at += x.op_count;
        text_at += x.text_count;
        if (docs) docs[i] = x;
    }
    return MTR_OK;
}

// the summary kernels' parameters for every document of the batch (scratch buffers sized)
static int summary_params(mtr_engine* e, SParams& P) {
    const uint32_t n = e->n_docs;
    if (e->out_size.ensure(n) || e->out_off.ensure(n) || e->out_hash.ensure(n)) return -1;
    P = SParams{};
    P.hdr = e->hdr.p;
    P.seg = e->seg.p;
    P.text = e->text.p;
    P.prop = e->prop.p;
    P.rm = e->rm.p;
    P.segcap = int(e->caps.max_segments);
    P.tcap = int(e->caps.text_units);
    P.pcap = int(e->caps.prop_words);
    P.rcap = int(e->caps.remover_cells);
    P.rtab = e->rtab;
    P.snapshot_v1 = e->opt.snapshot_v1;
    P.chunk_size = e->opt.chunk_size;
    P.new_length_calc = e->opt.new_length_calc;
    P.n_docs = n;
    P.docs = e->docs.p;
    P.key_off = e->key_off.p;
    P.key_bytes = e->key_bytes.p;
    P.val_off = e->val_off.p;
    P.val_bytes = e->val_bytes.p;
    P.val_eq = e->val_eq.p;
    P.client_off = e->client_off.p;
    P.client_bytes = e->client_bytes.p;
    P.dkind = e->dkind.p;
    P.out_size = e->out_size.p;
    P.out_off = e->out_off.p;
    P.out_hash = e->out_hash.p;
    {
        const size_t sc = size_t(P.segcap);
        P.maxb = int(std::min<int64_t>(int64_t(sc) + 1, std::max<int64_t>(int64_t(P.tcap) / std::max(1, P.chunk_size) + 4, 64)));
        if (e->s_kind.ensure(n * sc) || e->s_start.ensure(n * (sc + 1)) || e->s_len.ensure(n * sc) ||
            e->s_bytes.ensure(n * sc) || e->s_blob.ensure(n * (4 + 4 * size_t(P.maxb))) || e->s_lb.ensure(n * sc) ||
            e->s_fl.ensure(n * sc) || e->s_sid.ensure(n * sc) || e->s_bb.ensure(n * sc))
            return -1;
        P.s_kind = e->s_kind.p;
        P.s_start = e->s_start.p;
        P.s_len = e->s_len.p;
        P.s_bytes = e->s_bytes.p;
        P.s_lb = e->s_lb.p;
        P.s_fl = e->s_fl.p;
        P.s_sid = e->s_sid.p;
        P.s_bb = e->s_bb.p;
        P.s_blob = e->s_blob.p;
    }
    return 0;
}

int mtr_summarize(mtr_engine* e) {
    HIPCHK(hipSetDevice(e->device));
    const uint32_t n = e->n_docs;
    if (n == 0) return MTR_OK;
    SParams P;
    if (summary_params(e, P)) return -1;
    {  // (timing probes: MTR_SUM_DEBUG, summary.hip.h g_sdbg)
        const char* v = std::getenv("MTR_SUM_DEBUG");
        const int dbg = v ? std::atoi(v) : 0;
        static int last = 0;
        if (dbg != last) {
            HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_sdbg), &dbg, sizeof(int)));
            last = dbg;
        }
    }
    HIPCHK(hipEventRecord(e->ev[2], e->stream));
    summary_size_kernel<<<n, 64, 0, e->stream>>>(P);
    HIPCHK(hipGetLastError());
    e->h_size.resize(n);
    e->h_off.resize(n);
    HIPCHK(hipMemcpyAsync(e->h_size.data(), e->out_size.p, n * sizeof(int64_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    int64_t tot = 0;
    for (uint32_t d = 0; d < n; d++) {
        if (e->h_size[d] < 0) {
            set_err("document " + std::to_string(d) + " has more summary chunks than the engine's blob table");
            return MTR_ERR_CAPACITY;
        }
        e->h_off[d] = tot;
        tot += e->h_size[d];
    }
    e->out_total = tot;
    if (e->out.ensure(size_t(tot) + 16)) return -1;
    HIPCHK(hipMemcpyAsync(e->out_off.p, e->h_off.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, e->stream));
    P.out = e->out.p;
    summary_write_kernel<<<n, 64, 0, e->stream>>>(P);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e->ev[3], e->stream));
    HIPCHK(hipEventSynchronize(e->ev[3]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
    e->t_summary = ms;
    e->summarized = true;
    return MTR_OK;
}

int mtr_sync(mtr_engine* e) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    return MTR_OK;
}

// one document's summary record in the output buffer: u32 nb, u32 len[nb], blob bytes
static int summary_record(mtr_engine* e, uint32_t doc, std::vector<uint8_t>& buf) {
    if (!e->summarized || doc >= e->n_docs) {
        set_err("no summary for this document (call mtr_summarize first)");
        return -1;
    }
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    buf.resize(size_t(e->h_size[doc]));
    HIPCHK(hipMemcpy(buf.data(), e->out.p + e->h_off[doc], buf.size(), hipMemcpyDeviceToHost));
    return 0;
}

int mtr_summary_info(mtr_engine* e, uint32_t doc, int64_t* n_blobs, int64_t* n_bytes) {
    if (!e->summarized || doc >= e->n_docs) {
        set_err("no summary for this document (call mtr_summarize first)");
        return -1;
    }
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint32_t nb = 0;
    HIPCHK(hipMemcpy(&nb, e->out.p + e->h_off[doc], 4, hipMemcpyDeviceToHost));
    if (n_blobs) *n_blobs = nb;
    if (n_bytes) *n_bytes = e->h_size[doc] - 4 - 4 * int64_t(nb);
    return MTR_OK;
}

int64_t mtr_get_summary(mtr_engine* e, uint32_t doc, uint8_t* out, int64_t cap, int64_t* blob_len, int32_t max_blobs) {
    std::vector<uint8_t> buf;
    if (summary_record(e, doc, buf)) return -1;
    uint32_t nb;
    std::memcpy(&nb, buf.data(), 4);
    const int64_t payload = int64_t(buf.size()) - 4 - 4 * int64_t(nb);
    if (payload > cap || int64_t(nb) > int64_t(max_blobs) || (payload > 0 && !out) || !blob_len) {
        set_err("mtr_get_summary: buffers smaller than mtr_summary_info reports");
        return MTR_SUMMARY_TOO_SMALL;
    }
    int64_t off = 4 + 4 * int64_t(nb);
    int64_t w = 0;
    for (uint32_t k = 0; k < nb; k++) {
        uint32_t len;
        std::memcpy(&len, buf.data() + 4 + 4 * k, 4);
        blob_len[k] = len;
        std::memcpy(out + w, buf.data() + off, len);
        off += len;
        w += len;
    }
    return int64_t(nb);
}

int64_t mtr_get_summaries(mtr_engine* e, uint32_t lo, uint32_t hi, uint8_t* out, int64_t cap, int64_t* doc_off) {
    if (!e->summarized || hi > e->n_docs || lo > hi) {
        set_err("mtr_get_summaries: bad range or no summary (call mtr_summarize first)");
        return -1;
    }
    if (lo == hi) {
        if (doc_off) doc_off[0] = 0;
        return 0;
    }
    const int64_t base = e->h_off[lo];
    const int64_t total = e->h_off[hi - 1] + e->h_size[hi - 1] - base;  // documents are laid out in order
    if (total > cap) return -total;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(out, e->out.p + base, size_t(total), hipMemcpyDeviceToHost));
    if (doc_off) {
        for (uint32_t d = lo; d < hi; d++) doc_off[d - lo] = e->h_off[d] - base;
        doc_off[hi - lo] = total;
    }
    return total;
}

void* mtr_host_alloc(uint64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<uint64_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        set_err("hipHostMalloc failed for " + std::to_string(bytes) + " bytes");
        return nullptr;
    }
    return p;
}

int mtr_host_free(void* p) {
    if (p && hipHostFree(p) != hipSuccess) return -1;
    return MTR_OK;
}

int mtr_summary_hashes(mtr_engine* e, uint64_t* out, uint32_t n_docs) {
    if (!e->summarized) return -1;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpy(out, e->out_hash.p, std::min(n_docs, e->n_docs) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return MTR_OK;
}

int64_t mtr_summary_bytes(mtr_engine* e) { return e->summarized ? e->out_total : -1; }

// ---- host-side decoding of one document's slabs (parity checks, getText)
struct HostDoc {
    DocHdr h;
    std::vector<uint32_t> seg;
    std::vector<uint16_t> text;
    std::vector<uint32_t> prop, rm, rt;
    // head of leaf i's later-removers list (the device's uid table)
    uint32_t rm_head(uint32_t uid) const {
        const uint32_t mask = uint32_t(rt.size() / 2 - 1);
        uint32_t h = rtab_hash(uid) & mask;
        for (size_t n = 0; n <= mask; n++) {
            if (rt[2 * h] == uid + 1) return rt[2 * h + 1];
            if (rt[2 * h] == 0) break;
            h = (h + 1) & mask;
        }
        return 0xffffffu;
    }
};

static int fetch_doc(mtr_engine* e, uint32_t doc, HostDoc& hd) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(&hd.h, e->hdr.p + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
    const size_t sc = e->caps.max_segments;
    hd.seg.resize(NF * sc);
    HIPCHK(hipMemcpy(hd.seg.data(), e->seg.p + size_t(doc) * NF * sc, NF * sc * 4, hipMemcpyDeviceToHost));
    hd.text.resize(std::max(hd.h.textused, 1));
    HIPCHK(hipMemcpy(hd.text.data(), e->text.p + size_t(doc) * e->caps.text_units, hd.text.size() * 2,
                     hipMemcpyDeviceToHost));
    hd.prop.resize(std::max(hd.h.propused, 1));
    HIPCHK(hipMemcpy(hd.prop.data(), e->prop.p + size_t(doc) * e->caps.prop_words, hd.prop.size() * 4,
                     hipMemcpyDeviceToHost));
    const size_t rs = e->caps.remover_cells + 2 * size_t(e->rtab);
    hd.rm.resize(std::max(hd.h.rmused, 1));
    HIPCHK(hipMemcpy(hd.rm.data(), e->rm.p + size_t(doc) * rs, hd.rm.size() * 4, hipMemcpyDeviceToHost));
    hd.rt.resize(2 * size_t(e->rtab));
    HIPCHK(hipMemcpy(hd.rt.data(), e->rm.p + size_t(doc) * rs + e->caps.remover_cells, hd.rt.size() * 4,
                     hipMemcpyDeviceToHost));
    return 0;
}

// MergeTreeTextHelper.getText (MergeTreeTextHelper.ts:20-81) at the local view, on the device: one wave
// per document [lo, lo + gridDim.x) walks its leaves 64 at a time (text segments that are not removed;
// markers add nothing), an add-scan places each leaf's units, and the wave copies them leaf by leaf
// (coalesced runs from the document's text arena).  Pass 1 (out == nullptr) writes the lengths to
// lens[doc - lo]; pass 2 writes the units at off[doc - lo].
__global__ void __launch_bounds__(NT) text_kernel(const DocHdr* hdr, const uint32_t* seg, const uint16_t* text,
                                                  int segcap, int tcap, uint32_t lo, int64_t* lens,
                                                  const int64_t* off, uint16_t* out) {
    const uint32_t d = lo + blockIdx.x;
    const int S = __builtin_amdgcn_readfirstlane(hdr[d].nseg);
    const int ln = threadIdx.x;
    const uint32_t* g = seg + size_t(d) * NF * segcap;
    const uint16_t* tx = text + size_t(d) * tcap;
    int64_t carry = out ? off[blockIdx.x] : 0;
    for (int base = 0; base < S; base += 64) {
        const int i = base + ln;
        int len = 0;
        uint32_t t = 0;
        if (i < S && int(g[F_RSEQ * segcap + i]) == RNONE && !(g[F_META * segcap + i] & M_MARKER)) {
            len = int(g[F_LEN * segcap + i]);
            t = g[F_TEXT * segcap + i];
        }
        const int inc = wave_incl_scan(len);
        if (out) {
            const int n = min(64, S - base);
            for (int l = 0; l < n; l++) {
                const int ll = __builtin_amdgcn_readlane(len, l);
                const uint32_t tl = uint32_t(__builtin_amdgcn_readlane(int(t), l));
                const int64_t o = carry + __builtin_amdgcn_readlane(inc, l) - ll;
                for (int k = ln; k < ll; k += 64) out[o + k] = tx[tl + k];
            }
        }
        carry += __builtin_amdgcn_readlane(inc, 63);
    }
    if (!out && ln == 0) lens[blockIdx.x] = carry;
}

// texts of documents [lo, hi): out = the concatenated units, doc_off[i] = start of document lo + i
// (doc_off[hi - lo] = total); returns the total (nothing written when out is NULL), -1 when cap is
// too small or on error
int64_t mtr_get_texts(mtr_engine* e, uint32_t lo, uint32_t hi, uint16_t* out, int64_t cap, int64_t* doc_off) {
    HIPCHK(hipSetDevice(e->device));
    if (hi > e->max_docs || lo > hi) {
        set_err("mtr_get_texts: bad document range");
        return -1;
    }
    const uint32_t n = hi - lo;
    if (doc_off) doc_off[0] = 0;
    if (n == 0) return 0;
    DevBuf<int64_t> lens, offs;
    if (lens.ensure(n) || offs.ensure(size_t(n) + 1)) return -1;
    text_kernel<<<n, NT, 0, e->stream>>>(e->hdr.p, e->seg.p, e->text.p, int(e->caps.max_segments),
                                         int(e->caps.text_units), lo, lens.p, nullptr, nullptr);
    HIPCHK(hipGetLastError());
    std::vector<int64_t> hl(n), ho(size_t(n) + 1, 0);
    HIPCHK(hipMemcpyAsync(hl.data(), lens.p, n * sizeof(int64_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < n; i++) ho[i + 1] = ho[i] + hl[i];
    const int64_t total = ho[n];
    if (doc_off) std::copy(ho.begin(), ho.end(), doc_off);
    if (!out || total == 0) return total;
    if (total > cap) {
        set_err("mtr_get_texts: output buffer too small");
        return -1;
    }
    DevBuf<uint16_t> dev;
    if (dev.ensure(size_t(total))) return -1;
    HIPCHK(hipMemcpyAsync(offs.p, ho.data(), (size_t(n) + 1) * sizeof(int64_t), hipMemcpyHostToDevice, e->stream));
    text_kernel<<<n, NT, 0, e->stream>>>(e->hdr.p, e->seg.p, e->text.p, int(e->caps.max_segments),
                                         int(e->caps.text_units), lo, lens.p, offs.p, dev.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, dev.p, size_t(total) * sizeof(uint16_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return total;
}

int64_t mtr_get_text(mtr_engine* e, uint32_t doc, uint16_t* out, int64_t cap) {
    if (doc >= e->max_docs) {
        set_err("mtr_get_text: bad document");
        return -1;
    }
    int64_t off[2];
    const int64_t n = mtr_get_texts(e, doc, doc + 1, nullptr, 0, off);
    if (n <= 0 || !out || n > cap) return n;
    return mtr_get_texts(e, doc, doc + 1, out, cap, off);
}

int mtr_get_containing_segment(mtr_engine* e, uint32_t doc, int32_t pos, int32_t ref_seq, int32_t client,
                               mtr_segment_info* info, uint16_t* text, int64_t text_cap) {
    HIPCHK(hipSetDevice(e->device));
    if (doc >= e->max_docs || !info) {
        set_err("mtr_get_containing_segment: bad document");
        return -1;
    }
    KParams P{};
    P.hdr = e->hdr.p;
    P.seg = e->seg.p;
    P.heap = e->heap.p;
    P.text = e->text.p;
    P.prop = e->prop.p;
    P.rm = e->rm.p;
    P.segcap = int(e->caps.max_segments);
    P.hcap = int(e->caps.heap_entries);
    P.tcap = int(e->caps.text_units);
    P.pcap = int(e->caps.prop_words);
    P.rcap = int(e->caps.remover_cells);
    P.rtab = e->rtab;
    P.new_length_calc = e->opt.new_length_calc;
    P.n_docs = e->n_docs;
    if (e->red.ensure(16)) return -1;
    containing_kernel<<<1, NT, lds_bytes_global_mode(int(P.segcap)), e->stream>>>(P, doc, pos, ref_seq, client, e->red.p);
    HIPCHK(hipGetLastError());
    int32_t r[11];
    HIPCHK(hipMemcpyAsync(r, e->red.p, sizeof(r), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    std::memset(info, 0, sizeof(*info));
    info->leaf = r[0];
    if (r[0] < 0) {
        info->start = pos >= 0 ? r[9] : 0;  // the view's length (getLength at that view) when pos is past its end
        return MTR_OK;
    }
    info->offset = r[1];
    info->length = r[2];
    // pending local values are kept above every sequence number (LOCAL_BASE + localSeq, apply.hip.h):
    // report them as the reference holds them, UnassignedSequenceNumber plus the localSeq
    info->seq = r[3] >= LOCAL_BASE ? -1 : r[3];
    info->local_seq = r[3] >= LOCAL_BASE ? r[3] - LOCAL_BASE : -1;
    info->client = r[4];
    info->removed = r[5] != -1;
    info->removed_seq = r[5] >= LOCAL_BASE ? -1 : r[5];
    info->local_removed_seq = r[5] >= LOCAL_BASE ? r[5] - LOCAL_BASE : -1;
    info->marker = r[6];
    info->ref_type = r[7];
    info->props = r[8];
    info->start = r[9];
    info->groups = r[10];
    const bool has_text = !info->marker && e->h_kind[doc] == 0;
    if (text && has_text && info->length > 0 && text_cap >= info->length)
        HIPCHK(hipMemcpy(text, e->text.p + size_t(doc) * e->caps.text_units + uint32_t(r[7]),
                         size_t(info->length) * sizeof(uint16_t), hipMemcpyDeviceToHost));
    return MTR_OK;
}

static int ref_query(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap, int info_id) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (doc >= e->max_docs) {
        set_err("local references: bad document");
        return -1;
    }
    DocHdr h;
    HIPCHK(hipMemcpy(&h, e->hdr.p + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
    const int64_t n = e->refs.p ? h.nrefs : 0;
    const int64_t words = info_id >= 0 ? 4 : info_id == -3 ? 4 * n : info_id == -2 ? 2 * n : n;
    if (info_id < 0 && (words > cap || n == 0 || !out)) return int(n);
    KParams P{};
    P.hdr = e->hdr.p;
    P.seg = e->seg.p;
    P.heap = e->heap.p;
    P.text = e->text.p;
    P.prop = e->prop.p;
    P.rm = e->rm.p;
    P.segcap = int(e->caps.max_segments);
    P.hcap = int(e->caps.heap_entries);
    P.tcap = int(e->caps.text_units);
    P.pcap = int(e->caps.prop_words);
    P.rcap = int(e->caps.remover_cells);
    P.rtab = e->rtab;
    P.new_length_calc = e->opt.new_length_calc;
    P.n_docs = e->n_docs;
    P.refs = e->refs.p;
    P.refcap = int(e->caps.ref_slots);
    if (e->qbuf.ensure(size_t(std::max<int64_t>(words, 4)))) return -1;
    refs_kernel<<<1, NT, lds_bytes_global_mode(int(P.segcap)), e->stream>>>(P, doc, e->qbuf.p, info_id);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, e->qbuf.p, size_t(words) * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return int(n);
}

int64_t mtr_get_ref_positions(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap) {
    return ref_query(e, doc, out, cap, -1);
}

int64_t mtr_get_ref_states(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap) {
    return ref_query(e, doc, out, cap, -2);
}

int64_t mtr_get_ref_keys(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap) {
    return ref_query(e, doc, out, cap, -3);
}

int32_t mtr_get_ref_info(mtr_engine* e, uint32_t doc, uint32_t id, int32_t* out) {
    if (!out) return -2;
    out[0] = -1;
    out[1] = out[2] = out[3] = 0;
    if (id > uint32_t(INT32_MAX)) {  // (a negative id would run the positions query instead)
        set_err("mtr_get_ref_info: reference id out of range");
        return -2;
    }
    if (ref_query(e, doc, out, 4, int(id)) < 0) return -2;
    return out[0];
}

int32_t mtr_pending_groups(mtr_engine* e, uint32_t doc) {
    if (doc >= e->max_docs) return -1;
    DocHdr h;
    (void)hipSetDevice(e->device);
    if (hipStreamSynchronize(e->stream) != hipSuccess ||
        hipMemcpy(&h, e->hdr.p + doc, sizeof(DocHdr), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return h.ptail - h.phead;  // (ring entries [phead, ptail): one per pending SegmentGroup)
}

int mtr_doc_status(mtr_engine* e, uint32_t doc, int32_t* op_index) {
    if (doc >= e->max_docs) return -1;
    DocHdr h;
    (void)hipSetDevice(e->device);
    if (hipStreamSynchronize(e->stream) != hipSuccess ||
        hipMemcpy(&h, e->hdr.p + doc, sizeof(DocHdr), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    if (op_index) *op_index = h.fail_op;
    return h.status;
}

int64_t mtr_export(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap, int32_t* height) {
    HostDoc hd;
    if (doc >= e->max_docs || fetch_doc(e, doc, hd)) return -1;
    const size_t sc = e->caps.max_segments;
    if (height) *height = hd.h.height;
    if (hd.h.nseg - hd.h.holes > cap) return -int64_t(hd.h.nseg - hd.h.holes);
    int k = 0;  // leaf ordinal (hole slots of HBM-resident documents are skipped)
    for (int i = 0; i < hd.h.nseg; i++) {
        const uint32_t m = hd.seg[F_META * sc + i];
        if (hd.h.holes && (m & M_DEL)) continue;
        const int32_t rs = int32_t(hd.seg[F_RSEQ * sc + i]);
        int nrem = 0;
        if (rs != RNONE) {
            nrem = 1;
            if (m & M_OVERLAP) {
                uint32_t c = hd.rm_head(hd.seg[F_UID * sc + i]);
                while (c != 0xffffffu) {
                    nrem++;
                    c = hd.rm[c] & 0xffffffu;
                }
            }
        }
        uint32_t h = 0;
        const uint32_t pr = hd.seg[F_PROPS * sc + i] & ~MTR_PROPS_NEVER;  // (index flag)
        if (hd.seg[F_PROPS * sc + i] != NONE32 && !e->h_kind[doc]) {  // (a matrix vector's: a tracking id)
            h = 2166136261u ^ 1u;
            for (uint32_t q = 0; q < hd.prop[pr]; q++) {  // same hash as the oracle export
                const uint32_t v = hd.prop[pr + 2 + 2 * q];
                h = (h ^ hd.prop[pr + 1 + 2 * q]) * 16777619u;
                h = (h ^ (v < e->h_val_eq.size() ? e->h_val_eq[v] : v)) * 16777619u;
            }
        }
        int32_t* r = out + 8 * k++;
        // (pending local values are kept above every sequence number, LOCAL_BASE + localSeq: reported as the
        // reference holds them, UnassignedSequenceNumber, as the oracle export does)
        const int32_t sq = int32_t(hd.seg[F_SEQ * sc + i]);
        r[0] = int32_t(hd.seg[F_LEN * sc + i]);
        r[1] = sq >= LOCAL_BASE ? -1 : sq;
        r[2] = dec_client(m & M_CLIENT_MASK);
        r[3] = rs == RNONE ? INT32_MIN : (rs >= LOCAL_BASE ? -1 : rs);
        r[4] = nrem;
        r[5] = int32_t((m & M_BND_MASK) >> M_BND_SHIFT);
        // PermutationSegment: its start handle (the oracle export does the same)
        r[6] = e->h_kind[doc] ? int32_t(hd.seg[F_TEXT * sc + i]) : ((m & M_MARKER) ? 1 : 0);
        r[7] = int32_t(h);
    }
    return k;
}

int64_t mtr_get_leaves(mtr_engine* e, uint32_t doc, int32_t* out, int64_t cap) {
    HostDoc hd;
    if (doc >= e->max_docs || !e->h_kind[doc]) {
        set_err("mtr_get_leaves: not a matrix vector document");
        return -1;
    }
    if (fetch_doc(e, doc, hd)) return -1;
    const size_t sc = e->caps.max_segments;
    if (!out || hd.h.nseg - hd.h.holes > cap) return hd.h.nseg - hd.h.holes;  // (a size query)
    int k = 0;
    for (int i = 0; i < hd.h.nseg; i++) {
        const uint32_t m = hd.seg[F_META * sc + i];
        if (hd.h.holes && (m & M_DEL)) continue;
        const uint32_t t = hd.seg[F_PROPS * sc + i];
        int32_t* r = out + 5 * k++;
        r[0] = int32_t(hd.seg[F_LEN * sc + i]);
        r[1] = int32_t(hd.seg[F_RSEQ * sc + i]) != RNONE ? 1 : 0;
        r[2] = int32_t(hd.seg[F_TEXT * sc + i]);
        r[3] = t == NONE32 ? -1 : int32_t(t);
        r[4] = t == NONE32 || t >= hd.prop.size() ? 0 : int32_t(hd.prop[t]);
    }
    return k;
}

// debug: the scan arrays (E, V) an HBM-resident document's last op left in the scratch slab
int64_t mtr_debug_scan(mtr_engine* e, uint32_t doc, int32_t* out, int64_t n) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const size_t sc = e->caps.max_segments;
    if (!e->scratch.p || doc >= e->n_docs || n > int64_t(sc)) return -1;
    HIPCHK(hipMemcpy(out, e->scratch.p + size_t(doc) * 2 * sc, size_t(n) * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) {  // the scan array keeps the undefined flag in bit 31
        const int32_t ei = out[i], ep = i ? (out[i - 1] & 0x7fffffff) : 0;
        out[n + i] = ei < 0 ? -1 : ei - ep;
    }
    for (int64_t i = 0; i < n; i++) out[i] &= 0x7fffffff;
    return n;
}

int mtr_stats(mtr_engine* e, int64_t* out, int32_t n) {
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    std::vector<DocHdr> h(e->n_docs);
    if (e->n_docs) HIPCHK(hipMemcpy(h.data(), e->hdr.p, e->n_docs * sizeof(DocHdr), hipMemcpyDeviceToHost));
    unsigned long long st[3] = {0, 0, 0};
    {  // per-document counters [doc][4]: ops applied, sum of leaves before ops, inserted units
        std::vector<unsigned long long> sd(size_t(e->n_docs) * 4);
        if (e->n_docs) HIPCHK(hipMemcpy(sd.data(), e->stat.p, sd.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (uint32_t d = 0; d < e->n_docs; d++)
            for (int q = 0; q < 3; q++) st[q] += sd[size_t(d) * 4 + q];
    }
    int64_t v[10] = {int64_t(st[0]), e->n_docs, 0, 0, 0, e->launches, 0, 0, int64_t(st[1]), int64_t(st[2])};
    for (auto& x : h) {
        v[2] = std::max<int64_t>(v[2], x.nseg);
        v[3] += x.nseg;
        v[4] += x.status != MTR_OK;
        v[6] = std::max<int64_t>(v[6], x.max_heap);
        v[7] = std::max<int64_t>(v[7], x.textused);
    }
    for (int i = 0; i < n && i < 10; i++) out[i] = v[i];
    return MTR_OK;
}

int mtr_last_timing(mtr_engine* e, double* out, int32_t n) {
    double v[4] = {e->t_apply, e->t_summary, double(e->launches), e->t_kernels};
    for (int i = 0; i < n && i < 4; i++) out[i] = v[i];
    return MTR_OK;
}

int mtr_profile(mtr_engine* e, uint64_t* out, int32_t n, int32_t reset) {
    if (!e || !out) return MTR_ERR_BAD_OP;
    unsigned long long v[64] = {0};
#ifdef MTR_PROF
    if (hipStreamSynchronize(e->stream) != hipSuccess) return MTR_ERR_ASSERT;
    if (!e->prof.p) {
        if (e->prof.ensure(64) || hipMemset(e->prof.p, 0, sizeof(v)) != hipSuccess) return MTR_ERR_ASSERT;
    }
    if (hipMemcpy(v, e->prof.p, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return MTR_ERR_ASSERT;
    if (reset && hipMemset(e->prof.p, 0, sizeof(v)) != hipSuccess) return MTR_ERR_ASSERT;
#else
    (void)reset;
#endif
    for (int i = 0; i < n && i < 64; i++) out[i] = v[i];
#ifdef MTR_PROF
    return MTR_OK;
#else
    return MTR_ERR_UNSUPPORTED;
#endif
}

}  // extern "C"
