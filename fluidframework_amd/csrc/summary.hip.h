// summary.hip.h -- Client.summarize on the device (client.ts:966-1000) as a gather.
//
// SnapshotV1.extractSync/emit (snapshotV1.ts:122-298) and SnapshotLegacy.extractSync/emit
// (snapshotlegacy.ts:122-255) with the chunk layouts of snapshotChunks.ts:86-149, written as exact
// JSON.stringify bytes.  One wave per document, all lanes working:
//
//   size pass  (summary_size_kernel)
//     A. extract: classify every leaf (skip / coalescable / merge-info), decide for every
//        coalescable leaf whether it appends to the previous one (canAppend + matchProperties,
//        textSegment.ts:86-93, properties.ts:71-105) by ballots over 64 leaves with a carried
//        state, and compact the spec starts into a spec list;
//     B. one lane per spec: its length in UTF-16 units and its JSON byte size;
//     C. greedy chunking of the specs into blobs (>= chunk_size chars each) and blob sizes.
//   host: exclusive scan of the per-document sizes -> output offsets.
//   write pass (summary_write_kernel)
//     blob headers/trailers by lane 0, specs by one lane each at scanned offsets, then the
//     document digest (include/mtr_digest.h) by all lanes.
//
// Output per document: [u32 nblobs][u32 blob_len x nblobs][blob bytes ...]
#pragma once
#include "../../include/mtr_digest.h"
#include "apply.hip.h"

namespace mtr {

struct SParams {
    const DocHdr* hdr;
    const uint32_t* seg;
    const uint16_t* text;
    const uint32_t* prop;
    const uint32_t* rm;
    int32_t segcap, tcap, pcap, rcap, rtab;
    int32_t snapshot_v1, chunk_size, new_length_calc;
    uint32_t n_docs;
    uint32_t doc_base;  // the launch's blocks are documents doc_base + blockIdx.x (< n_docs)
    const mtr_doc_desc* docs;
    const uint32_t* key_off;
    const uint8_t* key_bytes;
    const uint32_t* val_off;
    const uint8_t* val_bytes;
    const uint32_t* val_eq;
    const uint32_t* client_off;
    const uint8_t* client_bytes;
    const uint32_t* dkind;  // non-zero: a PermutationVector of a SharedMatrix (mtr_set_matrix)
    // scratch handed from the size pass to the write pass
    uint8_t* s_kind;    // [doc][segcap]      leaf kind: 0 skip, 1 coalescable, 2 merge-info (V1)
    uint32_t* s_start;  // [doc][segcap + 1]  first leaf of every spec (+ sentinel)
    uint32_t* s_len;    // [doc][segcap]      spec length (UTF-16 units)
    uint32_t* s_bytes;  // [doc][segcap]      spec JSON bytes
    uint32_t* s_lb;     // [doc][segcap]      per leaf: its text's JSON string-body bytes, as a string of its own
    uint32_t* s_fl;     // [doc][segcap]      per leaf: first unit | last unit << 16 (pairing across pieces)
    uint32_t* s_sid;    // [doc][segcap]      per leaf: the spec it belongs to (non-skipped leaves)
    uint32_t* s_bb;     // [doc][segcap]      per spec: its text body's bytes (NONE32: no text body); the write
                        //                    pass keeps the body's offset in s_len
    int32_t* s_blob;    // [doc][4 + 4 * maxb]: nspec, nblob, totalLength, ok; per blob start, count, length, bytes
    int32_t maxb;
    int64_t* out_size;       // size pass output
    const int64_t* out_off;  // write pass input
    uint8_t* out;
    unsigned long long* out_hash;
};

// (timing probes only, MTR_SUM_DEBUG: bit 0 / 1 skip the size / write pass's lane-serial text, bit 2 the wave's
// long bodies, bit 3 the blob digests, bit 4 the write pass, bit 5 its bodies, bit 6 the size pass's per-leaf text
// counts, bit 7 its per-spec pass, bit 8 the write pass's property sets -- the summaries are then wrong; bits 6 and 7
// only with bit 4)
__device__ int g_sdbg = 0;

// ------------------------------------------------------------------ one lane's JSON writer
template <bool W>
struct LW {
    gptr<uint8_t> p;  // document output base (write pass)
    int64_t n;        // position
    // a long text body written by the whole wave (wave_body): skip > = 0 leaves that many bytes
    // for it and records where it starts
    int64_t skip = -1;
    int64_t body_at = -1;
    MTR_DI void put(uint32_t c) {
        if (W) p[n] = uint8_t(c);
        n++;
    }
    template <size_t N>
    MTR_DI void lit(const char (&s)[N]) {
        if (W) {  // a rolled loop: unrolled, every literal's stores held their addresses in VGPRs
#pragma unroll 1
            for (size_t i = 0; i + 1 < N; i++) p[n + int64_t(i)] = uint8_t(s[i]);
        }
        n += int64_t(N - 1);
    }
    MTR_DI void bytes(gptr<const uint8_t> s, uint32_t k) {
        if (W)
            for (uint32_t i0 = 0; i0 < k; i0 += 8) {  // 8 loads in flight, then their stores
                uint8_t b[8];
#pragma unroll
                for (uint32_t q = 0; q < 8; q++) b[q] = i0 + q < k ? s[i0 + q] : 0;
#pragma unroll
                for (uint32_t q = 0; q < 8; q++)
                    if (i0 + q < k) p[n + i0 + q] = b[q];
            }
        n += k;
    }
    MTR_DI void num(int64_t v) {
        const bool neg = v < 0;
        uint64_t u = neg ? uint64_t(-v) : uint64_t(v);
        int k = 1;
        for (uint64_t t = u; t >= 10; t /= 10) k++;
        if (neg) put('-');
        if (W)
            for (int q = k - 1; q >= 0; q--) {
                p[n + q] = uint8_t('0' + (u % 10));
                u /= 10;
            }
        n += k;
    }
    MTR_DI void hex4(uint32_t u) {
        if (W) {
            p[n] = '\\';
            p[n + 1] = 'u';
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t x = (u >> (12 - 4 * q)) & 15;
                p[n + 2 + q] = uint8_t(x < 10 ? '0' + x : 'a' + x - 10);
            }
        }
        n += 6;
    }
    MTR_DI void utf8(uint32_t cp) {
        if (cp < 0x80) {
            put(cp);
        } else if (cp < 0x800) {
            put(0xC0 | (cp >> 6));
            put(0x80 | (cp & 63));
        } else if (cp < 0x10000) {
            put(0xE0 | (cp >> 12));
            put(0x80 | ((cp >> 6) & 63));
            put(0x80 | (cp & 63));
        } else {
            put(0xF0 | (cp >> 18));
            put(0x80 | ((cp >> 12) & 63));
            put(0x80 | ((cp >> 6) & 63));
            put(0x80 | (cp & 63));
        }
    }
    // one UTF-16 unit of a JSON string body (ES2019 well-formed JSON.stringify); `hi` carries a
    // pending high surrogate across units and across the pieces of a coalesced segment
    MTR_DI void unit(uint32_t u, int& hi) {
        if (hi >= 0) {
            if (u >= 0xDC00 && u <= 0xDFFF) {
                utf8(0x10000 + ((uint32_t(hi) - 0xD800) << 10) + (u - 0xDC00));
                hi = -1;
                return;
            }
            hex4(uint32_t(hi));
            hi = -1;
        }
        if (u >= 0x20 && u < 0x80 && u != '"' && u != '\\') {
            put(u);
            return;
        }
        switch (u) {
            case '"': put('\\'); put('"'); return;
            case '\\': put('\\'); put('\\'); return;
            case '\b': put('\\'); put('b'); return;
            case '\f': put('\\'); put('f'); return;
            case '\n': put('\\'); put('n'); return;
            case '\r': put('\\'); put('r'); return;
            case '\t': put('\\'); put('t'); return;
            default: break;
        }
        if (u < 0x20) hex4(u);
        else if (u >= 0xD800 && u <= 0xDBFF) hi = int(u);
        else if (u >= 0xDC00 && u <= 0xDFFF) hex4(u);
        else utf8(u);
    }
    MTR_DI void flush_hi(int& hi) {
        if (hi >= 0) hex4(uint32_t(hi));
        hi = -1;
    }
};

// one document's arrays in HBM
struct SDoc {
    gptr<const uint32_t> len, seq, rseq, meta, text, props, uid;
    gptr<const uint16_t> gtext;
    gptr<const uint32_t> gprop, grm, grt;
    int rtmask;
    gptr<uint8_t> kind;
    gptr<uint32_t> start, slen, sbytes, lb, fl, sid, bb;
    gptr<int32_t> blob;
    int S, minseq, curseq, collab, local, newlen;
    int perm, hlen;  // PermutationVector: [length, start] specs, HandleTable of hlen words in the arena
};

MTR_DI SDoc sdoc(const SParams& P, uint32_t d, const DocHdr& h) {
    SDoc D;
    const gptr<const uint32_t> g = gp(P.seg) + size_t(d) * NF * P.segcap;
    D.len = g + F_LEN * P.segcap;
    D.seq = g + F_SEQ * P.segcap;
    D.rseq = g + F_RSEQ * P.segcap;
    D.meta = g + F_META * P.segcap;
    D.text = g + F_TEXT * P.segcap;
    D.props = g + F_PROPS * P.segcap;
    D.uid = g + F_UID * P.segcap;
    D.gtext = gp(P.text) + size_t(d) * P.tcap;
    D.gprop = gp(P.prop) + size_t(d) * P.pcap;
    D.grm = gp(P.rm) + size_t(d) * (size_t(P.rcap) + 2 * size_t(P.rtab));
    D.grt = D.grm + P.rcap;
    D.rtmask = P.rtab - 1;
    D.kind = gp(P.s_kind) + size_t(d) * P.segcap;
    D.start = gp(P.s_start) + size_t(d) * (P.segcap + 1);
    D.slen = gp(P.s_len) + size_t(d) * P.segcap;
    D.sbytes = gp(P.s_bytes) + size_t(d) * P.segcap;
    D.lb = gp(P.s_lb) + size_t(d) * P.segcap;
    D.fl = gp(P.s_fl) + size_t(d) * P.segcap;
    D.sid = gp(P.s_sid) + size_t(d) * P.segcap;
    D.bb = gp(P.s_bb) + size_t(d) * P.segcap;
    D.blob = gp(P.s_blob) + size_t(d) * (4 + 4 * P.maxb);
    D.S = h.nseg;
    D.minseq = h.minseq;
    D.curseq = h.curseq;
    D.collab = h.collab;
    D.local = h.collab ? h.local : int(CL_LOCAL);
    D.newlen = P.new_length_calc;
    D.perm = P.dkind ? int(uniu(gp(P.dkind)[d]) != 0) : 0;
    D.hlen = h.textused;
    return D;
}

// head of leaf s's later-removers list (the uid table of apply.hip.h)
MTR_DI uint32_t rm_head(const SDoc& D, int s) {
    const uint32_t uid = D.uid[s];
    uint32_t h = rtab_hash(uid) & uint32_t(D.rtmask);
    for (int n = 0; n <= D.rtmask; n++) {
        const uint32_t k = D.grt[2 * h];
        if (k == uid + 1) return D.grt[2 * h + 1];
        if (k == 0) break;
        h = (h + 1) & uint32_t(D.rtmask);
    }
    return 0xffffffu;
}

// visible length in the (minSeq, NonCollabClient) view for SnapshotLegacy's mapRange
MTR_DI int legacy_vis(const SDoc& D, int len, int rs, uint32_t m, int sq) {
    const bool rem = rs != RNONE;
    if (!D.collab || uint32_t(D.local) == CL_NONCOLLAB) {
        if (rem) return D.newlen ? 0 : (rs > D.minseq ? 0 : -1);
        return len;
    }
    const int ref = D.minseq;
    const uint32_t cl = m & M_CLIENT_MASK;
    if (D.newlen) {
        if (rem) {
            if (rs <= D.minseq) return -1;
            if (rs <= ref) return 0;
        }
        return (sq <= ref || cl == CL_NONCOLLAB) ? len : 0;
    }
    if (rem && rs <= ref) return -1;
    if (cl == CL_NONCOLLAB || sq <= ref) return len;
    if (rem && rs < LOCAL_BASE) return -1;  // a pending local remove: removedSeq === Unassigned (:993-998)
    return 0;
}

// kind of a leaf for extractSync: 0 = skip, 1 = coalescable, 2 = with merge info (V1 only)
MTR_DI int leaf_kind(const SDoc& D, int v1, int len, int rs, uint32_t m, int sq) {
    const bool rem = rs != RNONE;
    if (v1) {  // snapshotV1.ts:180-298
        // unacked inserts are elided, and so are pending removes (removedSeq -1 <= minSeq, :211)
        if ((rem && (rs <= D.minseq || rs >= LOCAL_BASE)) || sq >= LOCAL_BASE) return 0;
        if (sq <= D.minseq && !rem) return 1;
        return 2;
    }
    if (legacy_vis(D, len, rs, m, sq) <= 0) return 0;  // snapshotlegacy.ts:184-255
    if (sq <= D.minseq && (!rem || rs > D.minseq)) return 1;
    return 0;
}

template <bool W>
MTR_DI void w_client(LW<W>& w, const SParams& P, const mtr_doc_desc& dd, uint32_t enc) {
    const int id = dec_client(enc);
    w.put('"');
    if (id < 0 || uint32_t(id) >= dd.n_clients) {
        w.lit("original");
    } else {
        const uint32_t ix = dd.client_base + uint32_t(id);
        const uint32_t a = gp(P.client_off)[ix], b = gp(P.client_off)[ix + 1];
        w.bytes(gp(P.client_bytes) + a, b - a);
    }
    w.put('"');
}

template <bool W>
MTR_DI void w_props(LW<W>& w, const SDoc& D, const SParams& P, uint32_t pr) {
    if (W && (g_sdbg & 256)) return;  // (probe: the write pass's property sets; positions then drift)
    w.put('{');
    pr &= PN_MASK;  // (the index may carry MTR_PROPS_NEVER)
    const uint32_t n = D.gprop[pr];
    for (uint32_t i = 0; i < n; i++) {
        if (i) w.put(',');
        const uint32_t k = D.gprop[pr + 1 + 2 * i], v = D.gprop[pr + 2 + 2 * i];
        const uint32_t ka = gp(P.key_off)[k], kb = gp(P.key_off)[k + 1];
        const uint32_t va = gp(P.val_off)[v], vb = gp(P.val_off)[v + 1];
        w.put('"');
        w.bytes(gp(P.key_bytes) + ka, kb - ka);
        w.put('"');
        w.put(':');
        w.bytes(gp(P.val_bytes) + va, vb - va);
    }
    w.put('}');
}


// the text of one leaf, 8 units per round of loads
template <bool W>
MTR_DI void w_units(LW<W>& w, const SDoc& D, uint32_t t, int n, int& hi) {
    if (g_sdbg & (W ? 2 : 1)) {
        w.n += n;
        return;
    }
    for (int u0 = 0; u0 < n; u0 += 8) {
        uint32_t b[8];
#pragma unroll
        for (int q = 0; q < 8; q++) b[q] = u0 + q < n ? uint32_t(D.gtext[t + uint32_t(u0 + q)]) : 0u;
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (u0 + q < n) w.unit(b[q], hi);
    }
}

// toJSONObject of the spec [s, e): textSegment.ts:73-77, mergeTreeNodes.ts:577-581; the text of
// a coalesced group is the concatenation of its kind-1 leaves
template <bool W>
MTR_DI void w_segjson(LW<W>& w, const SDoc& D, const SParams& P, int s, int e) {
    if (D.perm) {  // PermutationSegment.toJSONObject (permutationvector.ts:118-120) of the coalesced group
        int length = 0;
        for (int k = s; k < e; k++)
            if (k == s || D.kind[k] == 1) length += int(D.len[k]);
        w.put('[');
        w.num(length);
        w.put(',');
        w.num(int64_t(int32_t(D.text[s])));
        w.put(']');
        return;
    }
    const uint32_t m = D.meta[s];
    const uint32_t pr = D.props[s];
    if (m & M_MARKER) {
        w.lit("{\"marker\":{");
        if (!(m & M_NOREF)) {
            w.lit("\"refType\":");
            w.num(int64_t(D.text[s]));
        }
        w.put('}');
        if (pr != NONE32) {
            w.lit(",\"props\":");
            w_props(w, D, P, pr);
        }
        w.put('}');
        return;
    }
    if (pr != NONE32) w.lit("{\"text\":");
    w.put('"');
    if (w.skip >= 0) {  // the body is the wave's (wave_body)
        w.body_at = w.n;
        w.n += w.skip;
    } else {
        int hi = -1;
        for (int k = s; k < e; k++)
            if (k == s || D.kind[k] == 1) w_units(w, D, D.text[k], int(D.len[k]), hi);
        w.flush_hi(hi);
    }
    w.put('"');
    if (pr != NONE32) {
        w.lit(",\"props\":");
        w_props(w, D, P, pr);
        w.put('}');
    }
}

// one spec: a coalesced group, or IJSONSegmentWithMergeInfo (snapshotChunks.ts:64-75) in
// SnapshotV1 key order (snapshotV1.ts:251-276)
template <bool W>
MTR_DI void w_spec(LW<W>& w, const SDoc& D, const SParams& P, const mtr_doc_desc& dd, int s, int e) {
    if (D.kind[s] != 2) {
        w_segjson(w, D, P, s, e);
        return;
    }
    w.lit("{\"json\":");
    w_segjson(w, D, P, s, s + 1);
    const int sq = int(D.seq[s]);
    const uint32_t m = D.meta[s];
    if (sq > D.minseq) {
        w.lit(",\"seq\":");
        w.num(sq);
        w.lit(",\"client\":");
        w_client(w, P, dd, m & M_CLIENT_MASK);
    }
    const int rs = int(D.rseq[s]);
    if (rs != RNONE) {
        w.lit(",\"removedSeq\":");
        w.num(rs);
        const uint32_t first = (m >> M_FREM_SHIFT) & 0xffu;
        w.lit(",\"removedClient\":");
        w_client(w, P, dd, first);
        w.lit(",\"removedClientIds\":[");
        w_client(w, P, dd, first);
        if (m & M_OVERLAP) {
            // the cons list holds later removers newest-first: emit oldest-first
            int nc = 0;
            const uint32_t head = rm_head(D, s);
            for (uint32_t c = head; c != 0xffffffu; c = D.grm[c] & 0xffffffu) nc++;
            for (int q = nc - 1; q >= 0; q--) {
                uint32_t c = head;
                for (int t = 0; t < q; t++) c = D.grm[c] & 0xffffffu;
                w.put(',');
                w_client(w, P, dd, D.grm[c] >> 24);
            }
        }
        w.put(']');
    }
    w.put('}');
}

// ------------------------------------------------------------------ wave-parallel text bodies
// JSON.stringify bytes of one UTF-16 unit c of a string body given its neighbours in the body
// (NOU = none): the greedy surrogate pairing of LW::unit is local -- a low surrogate pairs iff the
// unit before it is a high surrogate, a high one iff the unit after it is a low surrogate.
constexpr uint32_t NOU = 0xffffffffu;
MTR_DI bool is_hi(uint32_t u) { return u >= 0xD800 && u <= 0xDBFF; }
MTR_DI bool is_lo(uint32_t u) { return u >= 0xDC00 && u <= 0xDFFF; }
MTR_DI int unit_bytes(uint32_t p, uint32_t c, uint32_t n) {
    if (c >= 0x20 && c < 0x80) return (c == '"' || c == '\\') ? 2 : 1;
    if (c < 0x20) return (c == '\b' || c == '\f' || c == '\n' || c == '\r' || c == '\t') ? 2 : 6;
    if (is_lo(c)) return (p != NOU && is_hi(p)) ? 0 : 6;
    if (is_hi(c)) return (n != NOU && is_lo(n)) ? 4 : 6;
    return c < 0x800 ? 2 : 3;
}
MTR_DI void unit_write(gptr<uint8_t> o, uint32_t p, uint32_t c, uint32_t n) {
    LW<true> w{o, 0};
    if (is_lo(c) && p != NOU && is_hi(p)) return;
    if (is_hi(c) && n != NOU && is_lo(n)) {
        w.utf8(0x10000 + ((c - 0xD800) << 10) + (n - 0xDC00));
        return;
    }
    if (is_hi(c) || is_lo(c)) {
        w.hex4(c);
        return;
    }
    int hi = -1;
    w.unit(c, hi);
}
// the body of spec [s, e) (pieces: leaf s and the kind-1 leaves after it, concatenated) by all
// 64 lanes, one unit per lane per round over the concatenation -- a round spans pieces, which are
// short (a few units each after the splits), so a round per piece left most lanes idle: byte
// counts, a wave scan for offsets, then each lane writes its unit (W).  The pieces are taken 64 at
// a time, one per lane; a unit's piece is found by a binary search over the lanes' piece starts.
// Returns the body's byte count.
template <bool W>
MTR_DI int64_t wave_body(const SDoc& D, int s, int e, gptr<uint8_t> out) {
    if (g_sdbg & 4) return 0;
    const int ln = lane_id();
    int64_t nb = 0;
    uint32_t prev = NOU;  // last unit of the body so far
    for (int g0 = s; g0 < e; g0 += 64) {
        const int k = g0 + ln;
        int L = 0;
        uint32_t t = 0;
        if (k < e && (k == s || D.kind[k] == 1)) {
            L = max(int(D.len[k]), 0);
            t = D.text[k];
        }
        const int incl = wave_incl_scan(L);
        const int T = rdlane(incl, 63);  // units of this group of pieces
        if (T == 0) continue;
        const int start = incl - L;
        const uint64_t nz = __ballot(L > 0);
        uint32_t after = NOU;  // first unit after this group's pieces
        for (int k2 = g0 + 64; k2 < e; k2++)
            if (D.kind[k2] == 1 && uni(int(D.len[k2])) > 0) {
                after = uniu(uint32_t(D.gtext[uniu(D.text[k2])]));
                break;
            }
        for (int u0 = 0; u0 < T; u0 += 64) {
            const int i = u0 + ln;
            const bool in = i < T;
            // unit i's piece: the last lane whose start is <= i (an empty piece shares the next one's start)
            int j = 0;
#pragma unroll
            for (int step = 32; step > 0; step >>= 1) {
                const int sc = __shfl(start, j + step);
                if (sc <= i) j += step;
            }
            const int off = i - __shfl(start, j);
            const uint32_t tj = uint32_t(__shfl(int(t), j));
            const int Lj = __shfl(L, j);
            const uint32_t c = in ? uint32_t(D.gtext[tj + uint32_t(off)]) : NOU;
            // the unit after i when it is in the next piece of the group: that piece's first unit
            const uint64_t up = j >= 63 ? 0ull : (nz & (~0ull << (j + 1)));
            const uint32_t tn = uint32_t(__shfl(int(t), up ? first_lane(up) : 0));
            uint32_t pu = uint32_t(__shfl(int(c), max(ln - 1, 0)));
            if (ln == 0) pu = prev;
            uint32_t nu = uint32_t(__shfl(int(c), min(ln + 1, 63)));
            if (i + 1 >= T) nu = after;
            else if (ln == 63) nu = off + 1 < Lj ? uint32_t(D.gtext[tj + uint32_t(off + 1)]) : uint32_t(D.gtext[tn]);
            const int bts = in ? unit_bytes(pu, c, nu) : 0;
            const int bi = wave_incl_scan(bts);
            if (W && in && bts) unit_write(out + (nb + bi - bts), pu, c, nu);
            nb += rdlane(bi, 63);
            prev = uint32_t(rdlane(int(c), min(63, T - 1 - u0)));
        }
    }
    return nb;
}
// a spec whose body the wave writes: a text segment (not a marker) longer than one round
MTR_DI bool long_body(const SDoc& D, int s, uint32_t slen) {
    return !D.perm && slen > 64u && !(D.meta[s] & M_MARKER);
}

// blob wrappers.  V1: snapshotV1.ts:122-178 + serializeAsMaxSupportedVersion; legacy:
// snapshotlegacy.ts:122-182 + serializeAsMinSupportedVersion / buildHeaderMetadataForLegacyChunk.
template <bool W>
MTR_DI void w_blob_head(LW<W>& w, const SDoc& D, int v1, int start, int count, int length, int total_len, int nspec) {
    if (v1) {
        w.lit("{\"version\":\"1\",\"segmentCount\":");
        w.num(count);
        w.lit(",\"length\":");
        w.num(length);
        w.lit(",\"segments\":[");
    } else {
        w.lit("{\"chunkStartSegmentIndex\":");
        w.num(start);
        w.lit(",\"chunkSegmentCount\":");
        w.num(count);
        w.lit(",\"chunkLengthChars\":");
        w.num(length);
        w.lit(",\"totalLengthChars\":");
        w.num(total_len);
        w.lit(",\"totalSegmentCount\":");
        w.num(nspec);
        w.lit(",\"chunkSequenceNumber\":");
        w.num(D.minseq);
        w.lit(",\"segmentTexts\":[");
    }
}
template <bool W>
MTR_DI void w_blob_tail(LW<W>& w, const SDoc& D, int v1, int c, int nblob, int start, int first_len, int total_len,
                        int nspec) {
    if (v1) {
        w.lit("],\"startIndex\":");
        w.num(start);
        if (c == 0) {
            w.lit(",\"headerMetadata\":{\"minSequenceNumber\":");
            w.num(D.minseq);
            w.lit(",\"sequenceNumber\":");
            w.num(D.curseq);
            w.lit(",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
            for (int q = 1; q < nblob; q++) {
                w.lit(",{\"id\":\"body_");
                w.num(q - 1);
                w.lit("\"}");
            }
            w.lit("],\"totalLength\":");
            w.num(total_len);
            w.lit(",\"totalSegmentCount\":");
            w.num(nspec);
            w.put('}');
        }
        w.put('}');
    } else {
        w.put(']');
        if (c == 0) {
            w.lit(",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}");
            if (first_len < total_len) w.lit(",{\"id\":\"body\"}");
            w.lit("],\"sequenceNumber\":");
            w.num(D.minseq);
            w.lit(",\"totalLength\":");
            w.num(total_len);
            w.lit(",\"totalSegmentCount\":");
            w.num(nspec);
            w.put('}');
        }
        w.put('}');
    }
}

// ------------------------------------------------------------------ size pass
constexpr int kLaneText = 32;  // a leaf's text up to this many units is counted by its lane, longer by the wave
MTR_DI void summary_size_doc(const SParams& P, uint32_t d) {
    const DocHdr h = uni_struct(ld_struct<DocHdr>(gp(P.hdr) + d));
    const mtr_doc_desc dd = uni_struct(ld_struct<mtr_doc_desc>(gp(P.docs) + d));
    SDoc D = sdoc(P, d, h);
    const int v1 = D.perm ? 1 : P.snapshot_v1;  // PermutationVector forces newMergeTreeSnapshotFormat
    const int S = D.S;
    const int ln = lane_id();
    const gptr<const uint32_t> veq = gp(P.val_eq);

    // A. extract: kinds, appends and spec starts (carry = the last non-skipped leaf so far)
    bool c_valid = false, c_k1 = false, c_mk = false, c_nl = false;
    uint32_t c_pr = NONE32, c_tx = 0;
    int c_acc = 0;  // chars of the open group (TextSegmentGranularity rule)
    int c_len = 0;  // length of the last non-skipped leaf (PermutationSegment contiguity)
    int nspec = 0;
    for (int base = 0; base < S; base += 64) {
        const int i = base + ln;
        const bool in = i < S;
        int len = 0, rs = RNONE, sq = 0;
        uint32_t m = 0, pr = NONE32, tx = 0;
        if (in) {
            len = int(D.len[i]);
            rs = int(D.rseq[i]);
            sq = int(D.seq[i]);
            m = D.meta[i];
            pr = D.perm ? NONE32 : D.props[i];  // (a permutation segment's props field is its tracking id)
            tx = D.text[i];
        }
        const int kd = in ? leaf_kind(D, v1, len, rs, m, sq) : 0;
        if (in) D.kind[i] = uint8_t(kd);
        const bool mk = (m & M_MARKER) != 0;
        bool nl = false;  // last unit is '\n'
        if (kd == 1 && !mk && len > 0 && !D.perm)
            nl = (m & M_NLQ) ? D.gtext[tx + uint32_t(len) - 1] == u'\n' : (m & M_NL) != 0;
        {  // the leaf's text as a JSON string body of its own (unit_bytes: a surrogate pairs with its neighbour
            // inside the leaf; a pair split across two pieces of a spec is corrected in B), first and last unit.
            // Short leaves one lane each, 8 units per round of loads; longer ones by the whole wave.
            const bool tl = kd != 0 && !mk && len > 0 && !D.perm && !(g_sdbg & 64);
            uint32_t lbv = 0, flv = 0;
            if (tl && len <= kLaneText) {
                uint32_t prev = NOU;
                for (int u0 = 0; u0 < len; u0 += 8) {
                    uint32_t b[9];
#pragma unroll
                    for (int q = 0; q < 9; q++) b[q] = u0 + q < len ? uint32_t(D.gtext[tx + uint32_t(u0 + q)]) : NOU;
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (u0 + q < len) lbv += uint32_t(unit_bytes(q ? b[q - 1] : prev, b[q], b[q + 1]));
                    if (u0 == 0) flv = b[0];
                    prev = b[7];
                }
                flv |= uint32_t(D.gtext[tx + uint32_t(len) - 1]) << 16;
            }
            for (uint64_t lm = __ballot(tl && len > kLaneText); lm; lm &= lm - 1) {
                const int l = first_lane(lm);
                const int L = rdlane(len, l);
                const uint32_t t = uint32_t(rdlane(int(tx), l));
                int64_t nb = 0;
                uint32_t prev = NOU;
                for (int u0 = 0; u0 < L; u0 += 64) {
                    const int u = u0 + ln;
                    const uint32_t c = u < L ? uint32_t(D.gtext[t + uint32_t(u)]) : NOU;
                    uint32_t pu = uint32_t(__shfl(int(c), max(ln - 1, 0)));
                    if (ln == 0) pu = prev;
                    uint32_t nu = uint32_t(__shfl(int(c), min(ln + 1, 63)));
                    if (u + 1 >= L) nu = NOU;
                    else if (ln == 63) nu = uint32_t(D.gtext[t + uint32_t(u + 1)]);
                    nb += rdlane(wave_incl_scan(u < L ? unit_bytes(pu, c, nu) : 0), 63);
                    prev = uint32_t(rdlane(int(c), min(63, L - 1 - u0)));
                }
                if (ln == l) {
                    lbv = uint32_t(nb);
                    flv = uint32_t(D.gtext[t]) | (prev << 16);
                }
            }
            if (in) {
                D.lb[i] = lbv;
                D.fl[i] = flv;
            }
        }
        const uint64_t ns = __ballot(kd != 0);
        const uint64_t below = ns & lanes_below();
        const int p = below ? last_lane(below) : -1;
        const int ps = p < 0 ? 0 : p;
        bool p_k1 = __shfl(int(kd == 1), ps) != 0, p_mk = __shfl(int(mk), ps) != 0, p_nl = __shfl(int(nl), ps) != 0;
        uint32_t p_pr = uint32_t(__shfl(int(pr), ps)), p_tx = uint32_t(__shfl(int(tx), ps));
        int p_len = __shfl(len, ps);
        if (p < 0) {
            p_k1 = c_valid && c_k1;
            p_mk = c_mk;
            p_nl = c_nl;
            p_pr = c_pr;
            p_tx = c_tx;
            p_len = c_len;
        }
        bool link = kd == 1 && p_k1 && !p_mk && !mk && !p_nl;
        if (D.perm)  // PermutationSegment.canAppend: contiguous handles (permutationvector.ts:131-137)
            link = link && (p_tx == uint32_t(MTR_HANDLE_UNALLOCATED) ? tx == uint32_t(MTR_HANDLE_UNALLOCATED)
                                                                     : tx == p_tx + uint32_t(p_len));
        if (link && pr != p_pr) link = props_match(D.gprop, veq, p_pr, pr);
        if (link && pr == p_pr) link = !pset_never(pr);
        if (!D.perm && __ballot(link && len > kGranularity)) {  // accumulated-length clause, in order
            uint64_t lm = __ballot(link);
            int acc = c_valid && c_k1 ? c_acc : 0;
            for (uint64_t t = ns; t; t &= t - 1) {
                const int l = first_lane(t);
                const int lk = rdlane(len, l), kk = rdlane(kd, l);
                if (kk != 1) {
                    acc = 0;
                } else if ((lm >> l) & 1) {
                    if (acc > kGranularity && lk > kGranularity) {
                        lm &= ~(uint64_t(1) << l);
                        acc = lk;
                    } else {
                        acc += lk;
                    }
                } else {
                    acc = lk;
                }
            }
            link = (lm >> ln) & 1;
        }
        const bool st = kd == 2 || (kd == 1 && !link);
        const uint64_t sm = __ballot(st);
        if (st) D.start[nspec + __popcll(sm & lanes_below())] = uint32_t(i);
        if (kd != 0) D.sid[i] = uint32_t(nspec + __popcll(sm & ((uint64_t(2) << ln) - 1)) - 1);
        nspec += __popcll(sm);
        if (ns) {  // carry: the last non-skipped leaf of this round
            const int q = last_lane(ns);
            const int incl = wave_incl_scan(kd != 0 ? len : 0);
            const uint64_t sq_m = sm & ((uint64_t(2) << q) - 1);
            const bool k1 = rdlane(int(kd == 1), q) != 0;
            int acc = 0;
            if (k1) {
                if (sq_m) {
                    const int hs = last_lane(sq_m);
                    acc = rdlane(incl, q) - rdlane(incl, hs) + rdlane(len, hs);
                } else {
                    acc = c_acc + rdlane(incl, q);
                }
            }
            c_valid = true;
            c_k1 = k1;
            c_mk = rdlane(int(mk), q) != 0;
            c_nl = rdlane(int(nl), q) != 0;
            c_pr = rdlane(pr, q);
            c_tx = rdlane(tx, q);
            c_len = rdlane(len, q);
            c_acc = acc;
        }
    }
    if (ln == 0) D.start[nspec] = uint32_t(S);
    wsync();

    wsync();
    // B. one lane per spec: length and JSON bytes -- a text body from its pieces' byte counts (A), less 8 bytes
    // for each surrogate pair split across two pieces (two escaped halves, 12 bytes, become one 4-byte character)
    for (int g0 = 0; g0 < nspec && !(g_sdbg & 128); g0 += 64) {
        const int g = g0 + ln;
        if (g < nspec) {
            const int s = int(D.start[g]), e = int(D.start[g + 1]);
            const bool txt = !D.perm && !(D.meta[s] & M_MARKER);
            int length = 0;
            int64_t body = 0;
            if (D.kind[s] == 2) {
                length = int(D.len[s]);
                if (txt) body = D.lb[s];
            } else {
                uint32_t lastu = NOU;  // last unit of the previous non-empty piece
                for (int k = s; k < e; k++)
                    if (k == s || D.kind[k] == 1) {
                        const int lk = int(D.len[k]);
                        length += lk;
                        if (txt && lk > 0) {
                            const uint32_t f = D.fl[k];
                            body += D.lb[k];
                            if (lastu != NOU && is_hi(lastu) && is_lo(f & 0xffffu)) body -= 8;
                            lastu = f >> 16;
                        }
                    }
            }
            LW<false> w{(gptr<uint8_t>)nullptr, 0};
            if (txt) w.skip = body;
            w_spec(w, D, P, dd, s, e);
            D.slen[g] = uint32_t(length);
            D.sbytes[g] = uint32_t(w.n);
            D.bb[g] = txt ? uint32_t(body) : NONE32;
        }
    }
    wsync();

    // C. greedy chunking (snapshotV1.ts:70-116 getSeqLengthSegs; legacy: header chunk, then body)
    int total_len = 0;
    for (int g0 = 0; g0 < nspec; g0 += 64) {
        const int g = g0 + ln;
        total_len += rdlane(wave_incl_scan(g < nspec ? int(D.slen[min(g, nspec - 1)]) : 0), 63);
    }
    int nblob = 0, b_start = 0, b_cnt = 0, b_len = 0;
    int64_t b_bytes = 0, doc_bytes = 0;
    int first_len = 0;
    bool ok = true;
    auto close_blob = [&]() {
        if (nblob >= P.maxb) {
            ok = false;
            return;
        }
        if (nblob == 0) first_len = b_len;
        if (ln == 0) {
            D.blob[4 + 4 * nblob + 0] = b_start;
            D.blob[4 + 4 * nblob + 1] = b_cnt;
            D.blob[4 + 4 * nblob + 2] = b_len;
        }
        nblob++;
        b_start += b_cnt;
        b_cnt = 0;
        b_len = 0;
        b_bytes = 0;
    };
    for (int g0 = 0; g0 < nspec; g0 += 64) {
        const int g = g0 + ln;
        const uint32_t lv = g < nspec ? D.slen[g] : 0u;
        const int nk = min(64, nspec - g0);
        for (int t = 0; t < nk; t++) {
            b_len += int(rdlane(lv, t));
            b_cnt++;
            const bool closes = v1 ? b_len >= P.chunk_size : (nblob == 0 && b_len >= P.chunk_size);
            if (closes && (v1 || g0 + t + 1 < nspec)) close_blob();
        }
    }
    if (b_cnt > 0 || nblob == 0) close_blob();
    // blob bytes: wrappers (lane 0) + specs + commas
    for (int c = 0; c < nblob && ok; c++) {
        const int bs = uni(D.blob[4 + 4 * c + 0]), bc = uni(D.blob[4 + 4 * c + 1]), bl = uni(D.blob[4 + 4 * c + 2]);
        int64_t sb = 0;
        for (int g0 = bs; g0 < bs + bc; g0 += 64) {
            const int g = g0 + ln;
            const int x = g < bs + bc ? int(D.sbytes[g]) : 0;
            sb += rdlane(wave_incl_scan(x), 63);
        }
        LW<false> w{(gptr<uint8_t>)nullptr, 0};
        w_blob_head(w, D, v1, bs, bc, bl, total_len, nspec);
        w_blob_tail(w, D, v1, c, nblob, bs, first_len, total_len, nspec);
        const int64_t bytes = w.n + sb + (bc > 0 ? bc - 1 : 0);
        if (ln == 0) D.blob[4 + 4 * c + 3] = int32_t(bytes);
        doc_bytes += bytes;
    }
    int hbytes = 0;  // PermutationVector: the handleTable blob, JSON.stringify(handles)
    if (D.perm) {
        const gptr<const int32_t> ht = (gptr<const int32_t>)D.gtext;
        int digits = 0;
        for (int g0 = 0; g0 < D.hlen; g0 += 64) {
            const int g = g0 + ln;
            int x = 0;
            if (g < D.hlen) {
                LW<false> w{(gptr<uint8_t>)nullptr, 0};
                w.num(ht[g]);
                x = int(w.n);
            }
            digits += rdlane(wave_incl_scan(x), 63);
        }
        hbytes = 2 + digits + max(D.hlen - 1, 0);
    }
    if (ln == 0) {
        D.blob[0] = nspec;
        D.blob[1] = nblob;
        D.blob[2] = total_len;
        D.blob[3] = ok ? 1 : 0;
        P.out_size[d] = ok ? 4 + 4 * int64_t(nblob + D.perm) + doc_bytes + hbytes : -1;
    }
}

typedef uint64_t u64_ua __attribute__((aligned(1)));
// digest of one written blob (include/mtr_digest.h): one 8-byte word per lane per round
MTR_DI uint64_t blob_digest(gptr<uint8_t> base, int64_t b0, int64_t blen) {
    if (g_sdbg & 8) return 0;
    const int ln = lane_id();
    uint64_t sum = 0;
    const int64_t nw = (blen + 7) / 8;
    for (int64_t j0 = 0; j0 < nw; j0 += 64) {
        const int64_t j = j0 + ln;
        if (j < nw) {
            uint64_t wv = 0;
            if (8 * j + 8 <= blen) {  // (one unaligned 8-byte load: the engine's code runs in unaligned access mode)
                wv = *(gptr<const u64_ua>)(base + (b0 + 8 * j));
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (8 * j + q < blen) wv |= uint64_t(base[b0 + 8 * j + q]) << (8 * q);
            }
            sum += mtr_dg_word(wv, uint64_t(j));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = uint32_t(sum), hi = uint32_t(sum >> 32);
        sum += uint64_t(uint32_t(__shfl_xor(int(lo), o))) | (uint64_t(uint32_t(__shfl_xor(int(hi), o))) << 32);
    }
    return mtr_dg_blob(uni_struct(sum), uint64_t(blen));
}

// ------------------------------------------------------------------ write pass
// one unit of a string body at w's position given its neighbours in the body (unit_bytes' bytes)
MTR_DI void emit_unit(LW<true>& w, uint32_t p, uint32_t c, uint32_t n) {
    if (is_lo(c) && p != NOU && is_hi(p)) return;
    if (is_hi(c) && n != NOU && is_lo(n)) {
        w.utf8(0x10000 + ((c - 0xD800) << 10) + (n - 0xDC00));
        return;
    }
    if (is_hi(c) || is_lo(c)) {
        w.hex4(c);
        return;
    }
    int hi = -1;
    w.unit(c, hi);
}

// the text bodies of every spec, one leaf (piece) a lane: a piece's place is its spec's body offset (kept in
// D.slen by the wrapper pass) plus the bytes of the spec's earlier pieces -- the pieces' own counts (D.lb) less
// the 2 / 6 bytes a surrogate pair split across two pieces saves at its high / low half
MTR_DI void write_bodies(const SDoc& D, gptr<uint8_t> base) {
    if (g_sdbg & 32) return;
    const int ln = lane_id();
    const int S = D.S;
    int cspec = -1;          // the spec of the last piece so far
    int coff = 0;            // bytes of that spec's body written so far
    uint32_t clast = NOU;    // the last unit of the last piece so far
    for (int b0 = 0; b0 < S; b0 += 64) {
        const int i = b0 + ln;
        const bool in = i < S;
        const int ic = min(i, S - 1);
        const uint32_t kd = D.kind[ic];
        const uint32_t m = D.meta[ic];
        const int len = int(D.len[ic]);
        const bool piece = in && kd != 0 && !(m & M_MARKER);
        const int sid = piece ? int(D.sid[ic]) : -1;
        const bool tl = piece && len > 0;  // (an empty piece writes nothing and breaks no pair)
        const uint32_t f = tl ? D.fl[ic] : 0u;
        const uint32_t first = tl ? (f & 0xffffu) : NOU, last = tl ? (f >> 16) : NOU;
        const uint64_t pm = __ballot(tl);
        if (!pm) continue;
        // neighbours in the same spec: the previous / next text piece
        const uint64_t pb = pm & lanes_below();
        const int pl = pb ? last_lane(pb) : -1;
        const int psid = __shfl(sid, max(pl, 0));
        const uint32_t plast = uint32_t(__shfl(int(last), max(pl, 0)));
        uint32_t prevu = NOU;
        if (pl >= 0) prevu = psid == sid ? plast : NOU;
        else prevu = cspec == sid ? clast : NOU;
        const uint64_t pa = ln == 63 ? 0ull : (pm & (~uint64_t(0) << (ln + 1)));
        const int nl = pa ? first_lane(pa) : 0;
        const int nsid = __shfl(sid, nl);
        const uint32_t nfirst = uint32_t(__shfl(int(first), nl));
        uint32_t nextu = NOU;
        if (pa) {
            nextu = nsid == sid ? nfirst : NOU;
        } else if (tl) {  // the window's last piece: the next text piece after the window, if in the same spec
            for (int k = b0 + 64; k < S; k++) {
                if (D.kind[k] == 0 || int(D.len[k]) <= 0) continue;
                if ((D.meta[k] & M_MARKER) || int(D.sid[k]) != sid) break;
                nextu = D.fl[k] & 0xffffu;
                break;
            }
        }
        const int ab = tl ? int(D.lb[ic]) - (is_hi(last) && nextu != NOU && is_lo(nextu) ? 2 : 0) -
                                (is_lo(first) && prevu != NOU && is_hi(prevu) ? 6 : 0)
                          : 0;
        // the bytes of the spec's earlier pieces: a scan restarted at each spec's first piece in the window
        const int incl = wave_incl_scan(ab);
        const uint64_t heads = __ballot(tl && (pl < 0 ? true : psid != sid));  // a spec's first piece here
        const uint64_t hu = heads & ((uint64_t(2) << ln) - 1);
        const int hl = hu ? last_lane(hu) : 0;
        const int hbase = __shfl(incl - ab, hl);
        const int hsid = __shfl(sid, hl);
        const int off = incl - ab - hbase + (hsid == cspec ? coff : 0);
        if (tl && len <= kLaneText) {
            LW<true> w{base, int64_t(D.slen[sid]) + off};
            uint32_t p = prevu;
            const uint32_t t = D.text[ic];
            for (int u0 = 0; u0 < len; u0 += 8) {
                uint32_t bu[9];
#pragma unroll
                for (int q = 0; q < 9; q++) bu[q] = u0 + q < len ? uint32_t(D.gtext[t + uint32_t(u0 + q)]) : nextu;
                bool plain = u0 + 8 <= len;  // eight plain ASCII units: one unaligned 8-byte store
                uint64_t x = 0;
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    plain = plain && bu[q] >= 0x20u && bu[q] < 0x80u && bu[q] != '"' && bu[q] != '\\';
                    x |= uint64_t(bu[q] & 0xffu) << (8 * q);
                }
                if (plain) {
                    *(gptr<u64_ua>)(w.p + w.n) = x;
                    w.n += 8;
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (u0 + q < len) emit_unit(w, q ? bu[q - 1] : p, bu[q], bu[q + 1]);
                }
                p = bu[7];
            }
        }
        for (uint64_t lm = __ballot(tl && len > kLaneText); lm; lm &= lm - 1) {  // long pieces: the wave
            const int l = first_lane(lm);
            const int L = rdlane(len, l);
            const uint32_t t = uniu(D.text[b0 + l]);
            const int64_t at = int64_t(uniu(D.slen[rdlane(sid, l)])) + rdlane(off, l);
            const uint32_t pv = uint32_t(rdlane(int(prevu), l)), nx = uint32_t(rdlane(int(nextu), l));
            uint32_t prev = pv;
            int64_t nb = 0;
            for (int u0 = 0; u0 < L; u0 += 64) {
                const int u = u0 + ln;
                const bool uin = u < L;
                const uint32_t c = uin ? uint32_t(D.gtext[t + uint32_t(u)]) : NOU;
                uint32_t pu = uint32_t(__shfl(int(c), max(ln - 1, 0)));
                if (ln == 0) pu = prev;
                uint32_t nu = uint32_t(__shfl(int(c), min(ln + 1, 63)));
                if (u + 1 >= L) nu = nx;
                else if (ln == 63) nu = uint32_t(D.gtext[t + uint32_t(u + 1)]);
                const int bts = uin ? unit_bytes(pu, c, nu) : 0;
                const int bi = wave_incl_scan(bts);
                if (uin && bts) unit_write(base + (at + nb + bi - bts), pu, c, nu);
                nb += rdlane(bi, 63);
                prev = uint32_t(rdlane(int(c), min(63, L - 1 - u0)));
            }
        }
        // carry: the window's last text piece
        const int q = last_lane(pm);
        cspec = rdlane(sid, q);
        coff = rdlane(off, q) + rdlane(ab, q);
        clast = uint32_t(rdlane(int(last), q));
    }
}

MTR_DI void summary_write_doc(const SParams& P, uint32_t d) {
    if (g_sdbg & 16) return;
    const DocHdr h = uni_struct(ld_struct<DocHdr>(gp(P.hdr) + d));
    const mtr_doc_desc dd = uni_struct(ld_struct<mtr_doc_desc>(gp(P.docs) + d));
    SDoc D = sdoc(P, d, h);
    const int v1 = D.perm ? 1 : P.snapshot_v1;
    const int ln = lane_id();
    const int nspec = uni(D.blob[0]), nblob = uni(D.blob[1]), total_len = uni(D.blob[2]);
    if (!uni(D.blob[3])) return;
    const int first_len = uni(D.blob[4 + 2]);
    const int64_t off0 = gp(P.out_off)[d];
    const gptr<uint8_t> base = gp(P.out) + uni_struct(off0);
    const int nall = nblob + D.perm;  // + the handleTable blob of a PermutationVector
    if (ln == 0) {
        base[0] = uint8_t(nall);
        base[1] = uint8_t(nall >> 8);
        base[2] = uint8_t(nall >> 16);
        base[3] = uint8_t(nall >> 24);
    }
    const int64_t pos0 = 4 + 4 * int64_t(nall);
    int64_t pos = pos0;
    // the blobs' wrappers and specs, each spec's text body left as a gap (its offset kept in D.slen)
    for (int c = 0; c < nblob; c++) {
        const int bs = uni(D.blob[4 + 4 * c + 0]), bc = uni(D.blob[4 + 4 * c + 1]), bl = uni(D.blob[4 + 4 * c + 2]);
        const int64_t b0 = pos;
        {
            LW<true> w{base, pos};
            if (ln == 0) w_blob_head(w, D, v1, bs, bc, bl, total_len, nspec);
            pos = uni_struct(w.n);
        }
        for (int g0 = bs; g0 < bs + bc; g0 += 64) {
            const int g = g0 + ln;
            const bool act = g < bs + bc;
            const int x = act ? int(D.sbytes[g]) + (g > bs ? 1 : 0) : 0;
            const int incl = wave_incl_scan(x);
            if (act) {
                LW<true> w{base, pos + incl - x};
                if (g > bs) w.put(',');
                const int s = int(D.start[g]), e = int(D.start[g + 1]);
                const uint32_t bb = D.bb[g];
                if (bb != NONE32) w.skip = int64_t(bb);
                w_spec(w, D, P, dd, s, e);
                if (bb != NONE32) D.slen[g] = uint32_t(w.body_at);
            }
            pos += rdlane(incl, 63);
        }
        {
            LW<true> w{base, pos};
            if (ln == 0) w_blob_tail(w, D, v1, c, nblob, bs, first_len, total_len, nspec);
            pos = uni_struct(w.n);
        }
        const int64_t blen = pos - b0;
        if (ln == 0) {
            base[4 + 4 * c + 0] = uint8_t(blen);
            base[4 + 4 * c + 1] = uint8_t(blen >> 8);
            base[4 + 4 * c + 2] = uint8_t(blen >> 16);
            base[4 + 4 * c + 3] = uint8_t(blen >> 24);
            D.blob[4 + 4 * c + 3] = int32_t(blen);
        }
    }
    wsync();
    if (!D.perm) write_bodies(D, base);
    wsync();
    uint64_t hsh = mtr_dg_begin(uint64_t(nall));
    {
        int64_t b0 = pos0;
        for (int c = 0; c < nblob; c++) {
            const int64_t blen = uni(D.blob[4 + 4 * c + 3]);
            hsh = mtr_dg_next(hsh, blob_digest(base, b0, blen));
            b0 += blen;
        }
    }
    if (D.perm) {  // handleTable blob: "[h0,h1,...]" (HandleTable.getSummaryContent, handletable.ts:84)
        const gptr<const int32_t> ht = (gptr<const int32_t>)D.gtext;
        const int64_t b0 = pos;
        if (ln == 0) base[pos] = '[';
        pos++;
        for (int g0 = 0; g0 < D.hlen; g0 += 64) {
            const int g = g0 + ln;
            const bool act = g < D.hlen;
            int x = 0;
            int32_t v = 0;
            if (act) {
                v = ht[g];
                LW<false> w{(gptr<uint8_t>)nullptr, 0};
                w.num(v);
                x = int(w.n) + (g > 0 ? 1 : 0);
            }
            const int incl = wave_incl_scan(x);
            if (act) {
                LW<true> w{base, pos + incl - x};
                if (g > 0) w.put(',');
                w.num(v);
            }
            pos += rdlane(incl, 63);
        }
        if (ln == 0) base[pos] = ']';
        pos++;
        const int64_t blen = pos - b0;
        if (ln == 0) {
            base[4 + 4 * nblob + 0] = uint8_t(blen);
            base[4 + 4 * nblob + 1] = uint8_t(blen >> 8);
            base[4 + 4 * nblob + 2] = uint8_t(blen >> 16);
            base[4 + 4 * nblob + 3] = uint8_t(blen >> 24);
        }
        wsync();
        hsh = mtr_dg_next(hsh, blob_digest(base, b0, blen));
    }
    if (ln == 0) P.out_hash[d] = hsh;
}

#ifndef MTR_SWPE
#define MTR_SWPE 8
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MTR_SWPE))) summary_size_kernel(SParams P) {
    const uint32_t d = P.doc_base + blockIdx.x;
    if (d >= P.n_docs) return;
    summary_size_doc(P, d);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MTR_SWPE))) summary_write_kernel(SParams P) {
    const uint32_t d = P.doc_base + blockIdx.x;
    if (d >= P.n_docs) return;
    summary_write_doc(P, d);
}

}  // namespace mtr
