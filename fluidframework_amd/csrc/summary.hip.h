// summary.hip.h -- Client.summarize on the device (client.ts:966-1000).
//
// SnapshotV1.extractSync/emit (snapshotV1.ts:122-298) and SnapshotLegacy.extractSync/emit
// (snapshotlegacy.ts:122-255) with the chunk layouts of snapshotChunks.ts:86-149, written as
// exact JSON.stringify bytes.  One wave per document; a sizing pass and a writing pass share
// the same code (Writer<false> / Writer<true>).  Output per document:
//     [u32 nblobs][u32 blob_len x nblobs][blob bytes ...]
#pragma once
#include "apply.hip.h"

namespace mtr {

struct SParams {
    const DocHdr* hdr;
    const uint32_t* seg;
    const uint16_t* text;
    const uint32_t* prop;
    const uint32_t* rm;
    int32_t segcap, tcap, pcap, rcap;
    int32_t snapshot_v1, chunk_size, new_length_calc;
    uint32_t n_docs;
    const mtr_doc_desc* docs;
    const uint32_t* key_off;
    const uint8_t* key_bytes;
    const uint32_t* val_off;
    const uint8_t* val_bytes;
    const uint32_t* val_eq;
    const uint32_t* client_off;
    const uint8_t* client_bytes;
    int64_t* out_size;        // sizing pass output
    const int64_t* out_off;   // writing pass input
    uint8_t* out;
    unsigned long long* out_hash;
};

template <bool W>
struct Writer {
    uint8_t* p;
    int64_t n;
    unsigned long long h;
    __device__ void put(uint8_t c) {
        if (W) {
            p[n] = c;
            h = (h ^ c) * 1099511628211ull;
        }
        n++;
    }
    __device__ void str(const char* s) {
        while (*s) put(uint8_t(*s++));
    }
    __device__ void bytes(const uint8_t* s, uint32_t k) {
        for (uint32_t i = 0; i < k; i++) put(s[i]);
    }
    __device__ void num(int64_t v) {
        char buf[24];
        int k = 0;
        bool neg = v < 0;
        uint64_t u = neg ? uint64_t(-v) : uint64_t(v);
        do {
            buf[k++] = char('0' + (u % 10));
            u /= 10;
        } while (u);
        if (neg) put('-');
        while (k) put(uint8_t(buf[--k]));
    }
    __device__ void hex4(uint32_t u) {
        const char* hx = "0123456789abcdef";
        put('\\');
        put('u');
        put(uint8_t(hx[(u >> 12) & 15]));
        put(uint8_t(hx[(u >> 8) & 15]));
        put(uint8_t(hx[(u >> 4) & 15]));
        put(uint8_t(hx[u & 15]));
    }
    __device__ void utf8(uint32_t cp) {
        if (cp < 0x80) {
            put(uint8_t(cp));
        } else if (cp < 0x800) {
            put(uint8_t(0xC0 | (cp >> 6)));
            put(uint8_t(0x80 | (cp & 63)));
        } else if (cp < 0x10000) {
            put(uint8_t(0xE0 | (cp >> 12)));
            put(uint8_t(0x80 | ((cp >> 6) & 63)));
            put(uint8_t(0x80 | (cp & 63)));
        } else {
            put(uint8_t(0xF0 | (cp >> 18)));
            put(uint8_t(0x80 | ((cp >> 12) & 63)));
            put(uint8_t(0x80 | ((cp >> 6) & 63)));
            put(uint8_t(0x80 | (cp & 63)));
        }
    }
    // JSON string body over a stream of UTF-16 units (ES2019 well-formed JSON.stringify);
    // `hi` carries a pending high surrogate across pieces of a coalesced segment.
    __device__ void units(const uint16_t* t, int k, int& hi) {
        for (int i = 0; i < k; i++) {
            uint32_t u = t[i];
            if (hi >= 0) {
                if (u >= 0xDC00 && u <= 0xDFFF) {
                    utf8(0x10000 + ((uint32_t(hi) - 0xD800) << 10) + (u - 0xDC00));
                    hi = -1;
                    continue;
                }
                hex4(uint32_t(hi));
                hi = -1;
            }
            switch (u) {
                case '"': put('\\'); put('"'); continue;
                case '\\': put('\\'); put('\\'); continue;
                case '\b': put('\\'); put('b'); continue;
                case '\f': put('\\'); put('f'); continue;
                case '\n': put('\\'); put('n'); continue;
                case '\r': put('\\'); put('r'); continue;
                case '\t': put('\\'); put('t'); continue;
                default: break;
            }
            if (u < 0x20) hex4(u);
            else if (u >= 0xD800 && u <= 0xDBFF) hi = int(u);
            else if (u >= 0xDC00 && u <= 0xDFFF) hex4(u);
            else utf8(u);
        }
    }
    __device__ void flush_hi(int& hi) {
        if (hi >= 0) hex4(uint32_t(hi));
        hi = -1;
    }
};

struct DocView {
    const uint32_t *len, *seq, *rseq, *meta, *text, *props, *rm;
    const uint16_t* gtext;
    const uint32_t* gprop;
    const uint32_t* grm;
    int S, minseq, curseq, collab, local, newlen;
};

__device__ inline bool removed(const DocView& D, int k) { return int(D.rseq[k]) != RNONE; }

__device__ inline bool sv_can_append(const DocView& D, int acc_len, uint16_t acc_last, bool acc_marker, int k) {
    if (acc_marker || (D.meta[k] & M_MARKER)) return false;
    if (acc_len > 0 && acc_last == u'\n') return false;
    return acc_len <= kGranularity || int(D.len[k]) <= kGranularity;
}

// visible length in the (minSeq, NonCollabClient) view for SnapshotLegacy's mapRange
__device__ int legacy_vis(const DocView& D, int k) {
    int len = int(D.len[k]);
    int rs = int(D.rseq[k]);
    bool rem = rs != RNONE;
    if (!D.collab || uint32_t(D.local) == CL_NONCOLLAB) {
        if (rem) return D.newlen ? 0 : (rs > D.minseq ? 0 : -1);
        return len;
    }
    int ref = D.minseq;
    uint32_t cl = D.meta[k] & M_CLIENT_MASK;
    int sq = int(D.seq[k]);
    if (D.newlen) {
        if (rem) {
            if (rs <= D.minseq) return -1;
            if (rs <= ref) return 0;
        }
        return (sq <= ref || cl == CL_NONCOLLAB) ? len : 0;
    }
    if (rem && rs <= ref) return -1;
    if (cl == CL_NONCOLLAB || sq <= ref) return len;
    if (rem) return -1;
    return 0;
}

// kind of leaf k for extraction: 0 = skip, 1 = coalescable member, 2 = merge-info (V1 only)
__device__ int leaf_kind(const DocView& D, int k, int v1) {
    if (v1) {
        if (removed(D, k) && int(D.rseq[k]) <= D.minseq) return 0;
        if (int(D.seq[k]) <= D.minseq && !removed(D, k)) return 1;
        return 2;
    }
    int l = legacy_vis(D, k);
    if (l <= 0) return 0;
    if (int(D.seq[k]) <= D.minseq && (!removed(D, k) || int(D.rseq[k]) > D.minseq)) return 1;
    return 0;
}

struct Spec {
    int start, end;  // leaves [start, end]; end == start for merge-info specs
    int kind;        // 1 group, 2 merge-info
    int length;
};

// next spec starting at leaf *k (extractSync coalescing loops)
__device__ bool next_spec(const DocView& D, const SParams& P, int v1, int* k, Spec* sp) {
    int start = -1, end = -1, acc = 0;
    uint16_t last = 0;
    bool accm = false;
    uint32_t pr = NONE32;
    while (*k < D.S) {
        const int i = *k;
        const int kind = leaf_kind(D, i, v1);
        if (kind == 0) {
            (*k)++;
            continue;
        }
        if (kind == 1) {
            if (start < 0) {
                start = end = i;
                acc = int(D.len[i]);
                accm = (D.meta[i] & M_MARKER) != 0;
                last = (!accm && acc > 0) ? D.gtext[D.text[i] + acc - 1] : 0;
                pr = D.props[i];
                (*k)++;
                continue;
            }
            if (sv_can_append(D, acc, last, accm, i) && props_match(D.gprop, P.val_eq, pr, D.props[i])) {
                end = i;
                acc += int(D.len[i]);
                last = D.gtext[D.text[i] + D.len[i] - 1];
                (*k)++;
                continue;
            }
            break;
        }
        // merge-info
        if (start >= 0) break;
        sp->start = sp->end = i;
        sp->kind = 2;
        sp->length = int(D.len[i]);
        (*k)++;
        return true;
    }
    if (start < 0) return false;
    sp->start = start;
    sp->end = end;
    sp->kind = 1;
    sp->length = acc;
    return true;
}

template <bool W>
__device__ void w_client(Writer<W>& w, const SParams& P, const mtr_doc_desc& dd, uint32_t enc) {
    int id = dec_client(enc);
    w.put('"');
    if (id < 0 || uint32_t(id) >= dd.n_clients) {
        w.str("original");
    } else {
        uint32_t ix = dd.client_base + uint32_t(id);
        w.bytes(P.client_bytes + P.client_off[ix], P.client_off[ix + 1] - P.client_off[ix]);
    }
    w.put('"');
}

template <bool W>
__device__ void w_props(Writer<W>& w, const DocView& D, const SParams& P, uint32_t pr) {
    w.put('{');
    uint32_t n = D.gprop[pr];
    for (uint32_t i = 0; i < n; i++) {
        if (i) w.put(',');
        uint32_t k = D.gprop[pr + 1 + 2 * i], v = D.gprop[pr + 2 + 2 * i];
        w.put('"');
        w.bytes(P.key_bytes + P.key_off[k], P.key_off[k + 1] - P.key_off[k]);
        w.put('"');
        w.put(':');
        w.bytes(P.val_bytes + P.val_off[v], P.val_off[v + 1] - P.val_off[v]);
    }
    w.put('}');
}

// toJSONObject of a (possibly coalesced) segment: textSegment.ts:73-77, mergeTreeNodes.ts:577-581
template <bool W>
__device__ void w_segjson(Writer<W>& w, const DocView& D, const SParams& P, const Spec& s, int v1) {
    const int f = s.start;
    const uint32_t m = D.meta[f];
    const uint32_t pr = D.props[f];
    if (m & M_MARKER) {
        w.str("{\"marker\":{");
        if (!(m & M_NOREF)) {
            w.str("\"refType\":");
            w.num(int64_t(D.text[f]));
        }
        w.put('}');
        if (pr != NONE32) {
            w.str(",\"props\":");
            w_props(w, D, P, pr);
        }
        w.put('}');
        return;
    }
    if (pr != NONE32) w.str("{\"text\":");
    w.put('"');
    int hi = -1;
    if (s.kind == 2) {
        w.units(D.gtext + D.text[f], int(D.len[f]), hi);
    } else {
        for (int k = s.start; k <= s.end; k++)
            if (leaf_kind(D, k, v1) == 1) w.units(D.gtext + D.text[k], int(D.len[k]), hi);
    }
    w.flush_hi(hi);
    w.put('"');
    if (pr != NONE32) {
        w.str(",\"props\":");
        w_props(w, D, P, pr);
        w.put('}');
    }
}

// IJSONSegmentWithMergeInfo (snapshotChunks.ts:64-75) in SnapshotV1 key order (snapshotV1.ts:251-276)
template <bool W>
__device__ void w_spec(Writer<W>& w, const DocView& D, const SParams& P, const mtr_doc_desc& dd, const Spec& s,
                       int v1) {
    if (s.kind == 1) {
        w_segjson(w, D, P, s, v1);
        return;
    }
    const int k = s.start;
    w.str("{\"json\":");
    w_segjson(w, D, P, s, v1);
    if (int(D.seq[k]) > D.minseq) {
        w.str(",\"seq\":");
        w.num(int(D.seq[k]));
        w.str(",\"client\":");
        w_client(w, P, dd, D.meta[k] & M_CLIENT_MASK);
    }
    if (removed(D, k)) {
        w.str(",\"removedSeq\":");
        w.num(int(D.rseq[k]));
        const uint32_t first = (D.meta[k] >> M_FREM_SHIFT) & 0xffu;
        w.str(",\"removedClient\":");
        w_client(w, P, dd, first);
        w.str(",\"removedClientIds\":[");
        w_client(w, P, dd, first);
        if (D.meta[k] & M_OVERLAP) {
            // cons list holds later removers newest-first; emit oldest-first
            uint32_t cells[64];
            int nc = 0;
            uint32_t c = D.rm[k];
            while (c != 0xffffffu && nc < 64) {
                cells[nc++] = c;
                c = D.grm[c] & 0xffffffu;
            }
            for (int q = nc - 1; q >= 0; q--) {
                w.put(',');
                w_client(w, P, dd, D.grm[cells[q]] >> 24);
            }
        }
        w.put(']');
    }
    w.put('}');
}

template <bool W>
__device__ void w_blob_len(Writer<W>& w, int64_t at, uint32_t len) {
    if (W) {
        w.h = (w.h ^ uint64_t(len)) * 1099511628211ull;  // blob boundary in the hash
        w.p[at + 0] = uint8_t(len);
        w.p[at + 1] = uint8_t(len >> 8);
        w.p[at + 2] = uint8_t(len >> 16);
        w.p[at + 3] = uint8_t(len >> 24);
    }
}

template <bool W>
__device__ void summarize_doc(const SParams& P, uint32_t d, Writer<W>& w) {
    const DocHdr h = P.hdr[d];
    const mtr_doc_desc dd = P.docs[d];
    DocView D;
    const uint32_t* g = P.seg + size_t(d) * NF * P.segcap;
    D.len = g + F_LEN * P.segcap;
    D.seq = g + F_SEQ * P.segcap;
    D.rseq = g + F_RSEQ * P.segcap;
    D.meta = g + F_META * P.segcap;
    D.text = g + F_TEXT * P.segcap;
    D.props = g + F_PROPS * P.segcap;
    D.rm = g + F_RM * P.segcap;
    D.gtext = P.text + size_t(d) * P.tcap;
    D.gprop = P.prop + size_t(d) * P.pcap;
    D.grm = P.rm + size_t(d) * P.rcap;
    D.S = h.nseg;
    D.minseq = h.minseq;
    D.curseq = h.curseq;
    D.collab = h.collab;
    D.local = h.collab ? h.local : int(CL_LOCAL);
    D.newlen = P.new_length_calc;
    const int v1 = P.snapshot_v1;
    const int chunk = P.chunk_size;

    // pass A: totals and number of chunks
    int64_t totalLen = 0, totalCount = 0, nChunks = 0;
    {
        int k = 0;
        Spec sp;
        int64_t clen = 0, ccnt = 0;
        bool open = false;
        while (next_spec(D, P, v1, &k, &sp)) {
            if (!open) { open = true; clen = 0; ccnt = 0; nChunks++; }
            clen += sp.length;
            ccnt++;
            totalLen += sp.length;
            totalCount++;
            if (clen >= chunk) open = false;
        }
        if (nChunks == 0) nChunks = 1;
    }
    int nblobs;
    if (v1) nblobs = int(nChunks);
    else nblobs = 1;  // legacy: header + optional body, decided below
    // legacy: chunk1 = first chunk (length >= chunk); body = everything else
    int64_t c1cnt = 0, c1len = 0;
    if (!v1) {
        int k = 0;
        Spec sp;
        while (c1len < chunk && next_spec(D, P, v1, &k, &sp)) {
            c1len += sp.length;
            c1cnt++;
        }
        if (c1cnt < totalCount) nblobs = 2;
    }
    const int64_t table = 4 + 4 * int64_t(nblobs);
    const int64_t base = w.n;
    if (W) w_blob_len(w, base, uint32_t(nblobs));  // hashes nblobs
    w.n += table;
    int k = 0;
    Spec sp;
    if (v1) {
        // emit, snapshotV1.ts:122-178
        int64_t specsBefore = 0;
        for (int c = 0; c < nblobs; c++) {
            const int64_t b0 = w.n;
            // look-ahead: this chunk's count and length
            int kk = k;
            int64_t clen = 0, ccnt = 0;
            Spec t;
            while (clen < chunk && next_spec(D, P, v1, &kk, &t)) {
                clen += t.length;
                ccnt++;
            }
            w.str("{\"version\":\"1\",\"segmentCount\":");
            w.num(ccnt);
            w.str(",\"length\":");
            w.num(clen);
            w.str(",\"segments\":[");
            int64_t emitted = 0;
            while (emitted < ccnt && next_spec(D, P, v1, &k, &sp)) {
                if (emitted) w.put(',');
                w_spec(w, D, P, dd, sp, v1);
                emitted++;
            }
            w.str("],\"startIndex\":");
            w.num(specsBefore);
            specsBefore += ccnt;
            if (c == 0) {
                w.str(",\"headerMetadata\":{\"minSequenceNumber\":");
                w.num(D.minseq);
                w.str(",\"sequenceNumber\":");
                w.num(D.curseq);
                w.str(",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
                for (int q = 1; q < nblobs; q++) {
                    w.str(",{\"id\":\"body_");
                    w.num(q - 1);
                    w.str("\"}");
                }
                w.str("],\"totalLength\":");
                w.num(totalLen);
                w.str(",\"totalSegmentCount\":");
                w.num(totalCount);
                w.put('}');
            }
            w.put('}');
            w_blob_len(w, base + 4 + 4 * c, uint32_t(w.n - b0));
        }
    } else {
        // emit, snapshotlegacy.ts:122-182 + serializeAsMinSupportedVersion / buildHeaderMetadataForLegacyChunk
        for (int c = 0; c < nblobs; c++) {
            const int64_t b0 = w.n;
            const int64_t cstart = c == 0 ? 0 : c1cnt;
            const int64_t ccnt = c == 0 ? c1cnt : totalCount - c1cnt;
            const int64_t clen = c == 0 ? c1len : totalLen - c1len;
            w.str("{\"chunkStartSegmentIndex\":");
            w.num(cstart);
            w.str(",\"chunkSegmentCount\":");
            w.num(ccnt);
            w.str(",\"chunkLengthChars\":");
            w.num(clen);
            w.str(",\"totalLengthChars\":");
            w.num(totalLen);
            w.str(",\"totalSegmentCount\":");
            w.num(totalCount);
            w.str(",\"chunkSequenceNumber\":");
            w.num(D.minseq);
            w.str(",\"segmentTexts\":[");
            for (int64_t e = 0; e < ccnt && next_spec(D, P, v1, &k, &sp); e++) {
                if (e) w.put(',');
                w_spec(w, D, P, dd, sp, v1);
            }
            w.put(']');
            if (c == 0) {
                w.str(",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}");
                if (c1len < totalLen) w.str(",{\"id\":\"body\"}");
                w.str("],\"sequenceNumber\":");
                w.num(D.minseq);
                w.str(",\"totalLength\":");
                w.num(totalLen);
                w.str(",\"totalSegmentCount\":");
                w.num(totalCount);
                w.put('}');
            }
            w.put('}');
            w_blob_len(w, base + 4 + 4 * c, uint32_t(w.n - b0));
        }
    }
}

__global__ void __launch_bounds__(64) summary_size_kernel(SParams P) {
    const uint32_t d = blockIdx.x;
    if (d >= P.n_docs || threadIdx.x != 0) return;
    Writer<false> w{nullptr, 0, 0};
    summarize_doc<false>(P, d, w);
    P.out_size[d] = w.n;
}

__global__ void __launch_bounds__(64) summary_write_kernel(SParams P) {
    const uint32_t d = blockIdx.x;
    if (d >= P.n_docs || threadIdx.x != 0) return;
    Writer<true> w{P.out + P.out_off[d], 0, 14695981039346656037ull};
    summarize_doc<true>(P, d, w);
    P.out_hash[d] = w.h;
}

}  // namespace mtr
