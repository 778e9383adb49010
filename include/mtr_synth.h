/*
 * mtr_synth.h -- the seeded synthetic op-log recipe of the bench configurations.
 *
 * It restates runMergeTreeOperationRunner (packages/dds/merge-tree/src/test/
 * mergeTreeOperationRunner.ts:200-352) with the MockContainerRuntimeFactory ordering rule
 * (packages/runtime/test-runtime-utils/src/mocks.ts:216-258): a uniformly chosen writer submits an
 * op at its reference sequence number (which lags the head by at most max_lag), messages are
 * sequenced in generation order, and the MSN is the minimum over writers of their reference
 * sequence numbers.
 *
 * Positions must be valid in the writer's (refSeq, clientId) view, and which segments that view
 * covers depends on the exact B+tree placement of concurrent inserts (mergeTree.ts:1754-1830), so
 * the recipe is driven by an exact simulator: the CPU oracle (tests) or the HIP engine itself in
 * record mode (bench).  Both call the same functions below with the view length they computed;
 * equal seeds therefore give bit-identical op logs whenever the two simulators agree.
 *
 * Header-only, usable from host C/C++ and HIP device code.
 */
#ifndef MTR_SYNTH_H
#define MTR_SYNTH_H

#include <stdint.h>

#include "mtr_types.h"

#ifdef __HIPCC__
#define MTR_HD __host__ __device__
#else
#define MTR_HD
#endif

#define MTR_SYNTH_MAX_WRITERS 64

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mtr_synth_cfg {
    uint32_t n_docs;
    uint32_t ops_per_doc;      /* sequenced messages per document */
    uint32_t writers;          /* writer clients, short ids 1..writers (0 = the observer) */
    uint32_t max_lag;          /* seq - 1 - refSeq <= max_lag */
    uint32_t w_insert, w_remove, w_annotate;
    uint32_t max_text;         /* inserted text: 1..max_text UTF-16 units ... */
    uint32_t nonbmp_permille;  /* ... plus a trailing surrogate pair with this chance */
    uint32_t newline_permille; /* per-unit chance of '\n' */
    uint32_t max_range;        /* remove/annotate length 1..max_range */
    uint32_t n_propops;        /* annotate prop-op index 0..n_propops-1 */
    uint32_t doc_base;         /* global index of document 0 (seeds) */
    uint32_t text_cap;         /* per-document text capacity of the recorded batch */
    uint64_t seed;
} mtr_synth_cfg;

/* Per-document generator state (persists across record-mode launches). */
typedef struct mtr_synth_state {
    uint64_t rng;
    int32_t msn;
    uint32_t text_used;
    int32_t refs[MTR_SYNTH_MAX_WRITERS + 1];
} mtr_synth_state;

MTR_HD static inline uint64_t mtr_rng_next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
MTR_HD static inline uint32_t mtr_rng_below(uint64_t* s, uint32_t n) {
    return n ? (uint32_t)(mtr_rng_next(s) % n) : 0u;
}

MTR_HD static inline void mtr_synth_init(const mtr_synth_cfg* cfg, uint32_t doc, mtr_synth_state* st) {
    st->rng = (cfg->seed ^ ((uint64_t)(cfg->doc_base + doc) << 20) ^ 0xdeadbeefull) * 0x9E3779B97F4A7C15ull;
    st->msn = 0;
    st->text_used = 0;
    for (int i = 0; i <= MTR_SYNTH_MAX_WRITERS; i++) st->refs[i] = 0;
}

/* Step 1 of message `seq` (1-based): choose the writer and its reference sequence number and
 * advance the MSN.  Writes op->client/seq/ref_seq/min_seq/flags. */
MTR_HD static inline void mtr_synth_begin(const mtr_synth_cfg* cfg, mtr_synth_state* st, int32_t seq, mtr_op* op) {
    const uint32_t c = 1u + mtr_rng_below(&st->rng, cfg->writers);
    const int32_t lag = (int32_t)mtr_rng_below(&st->rng, cfg->max_lag + 1u);
    int32_t want = seq - 1 - lag;
    if (want < 0) want = 0;
    if (want > st->refs[c]) st->refs[c] = want;
    int32_t m = 0x7fffffff;
    for (uint32_t w = 1; w <= cfg->writers; w++)
        if (st->refs[w] < m) m = st->refs[w];
    if (m > st->msn) st->msn = m;
    op->type = MTR_OP_SEQ;
    op->flags = MTR_F_LAST;
    op->client = (uint16_t)c;
    op->seq = seq;
    op->ref_seq = st->refs[c];
    op->min_seq = st->msn;
    op->pos1 = 0;
    op->pos2 = -1;
    op->payload = 0;
    op->payload2 = 0;
}

/* Step 2: given the view length L of (op->ref_seq, op->client), choose the op.  Inserted text is
 * written to text[st->text_used ...] (capacity cfg->text_cap; on overflow the op degrades to a
 * remove of nothing-new so the log stays valid). */
MTR_HD static inline void mtr_synth_finish(const mtr_synth_cfg* cfg, mtr_synth_state* st, int32_t L, mtr_op* op,
                                           uint16_t* text) {
    const uint32_t tot = cfg->w_insert + cfg->w_remove + cfg->w_annotate;
    const uint32_t pick = mtr_rng_below(&st->rng, tot);
    int kind = pick < cfg->w_insert ? 0 : (pick < cfg->w_insert + cfg->w_remove ? 1 : 2);
    if (L <= 0) kind = 0;
    if (kind == 0) {
        const int32_t pos = (int32_t)mtr_rng_below(&st->rng, (uint32_t)L + 1u);
        uint32_t n = 1u + mtr_rng_below(&st->rng, cfg->max_text);
        const uint32_t pair = mtr_rng_below(&st->rng, 1000u) < cfg->nonbmp_permille ? 2u : 0u;
        const uint32_t off = st->text_used;
        if (off + n + pair > cfg->text_cap) { /* out of recording space: insert one unit if possible */
            n = off < cfg->text_cap ? 1u : 0u;
        }
        for (uint32_t q = 0; q < n; q++) {
            const int nl = mtr_rng_below(&st->rng, 1000u) < cfg->newline_permille;
            const uint16_t u = nl ? (uint16_t)'\n' : (uint16_t)('a' + mtr_rng_below(&st->rng, 26u));
            text[off + q] = u;
        }
        uint32_t total = n;
        if (pair && off + n + 2 <= cfg->text_cap) {
            const uint32_t cp = 0x1F600u + mtr_rng_below(&st->rng, 64u) - 0x10000u;
            text[off + n] = (uint16_t)(0xD800u + (cp >> 10));
            text[off + n + 1] = (uint16_t)(0xDC00u + (cp & 0x3FFu));
            total += 2;
        }
        st->text_used = off + total;
        op->type = total ? MTR_OP_INSERT : MTR_OP_SEQ;
        op->pos1 = pos;
        op->payload = off;
        op->payload2 = total;
    } else {
        const int32_t start = (int32_t)mtr_rng_below(&st->rng, (uint32_t)L);
        uint32_t room = (uint32_t)(L - start);
        if (room > cfg->max_range) room = cfg->max_range;
        const int32_t len = 1 + (int32_t)mtr_rng_below(&st->rng, room);
        op->pos1 = start;
        op->pos2 = start + len;
        if (kind == 1) {
            op->type = MTR_OP_REMOVE;
        } else {
            op->type = MTR_OP_ANNOTATE;
            op->payload = mtr_rng_below(&st->rng, cfg->n_propops ? cfg->n_propops : 1u);
        }
    }
}

/* SharedMatrix recipe: after mtr_synth_begin, given the writer's view lengths of
 * the rows and cols vectors, choose a row/col splice (insertRows/removeRows/insertCols/removeCols,
 * matrix.ts:363-372) with weights w_insert / w_remove, or a setCell (weight w_annotate) at a row and
 * col inside the writer's view.  Splices insert 1..max_text positions and remove 1..max_range. */
MTR_HD static inline void mtr_synth_matrix_finish(const mtr_synth_cfg* cfg, mtr_synth_state* st, int32_t Lr,
                                                  int32_t Lc, mtr_op* op) {
    const uint32_t tot = cfg->w_insert + cfg->w_remove + cfg->w_annotate;
    const uint32_t pick = mtr_rng_below(&st->rng, tot);
    int kind = pick < cfg->w_insert ? 0 : (pick < cfg->w_insert + cfg->w_remove ? 1 : 2);
    const int cols = (int)mtr_rng_below(&st->rng, 2u);
    if (kind == 2 && (Lr <= 0 || Lc <= 0)) kind = 0;
    const int32_t L = cols ? Lc : Lr;
    if (kind == 1 && L <= 0) kind = 0;
    op->payload = 0;
    op->payload2 = 0;
    if (kind == 2) {
        op->type = MTR_OP_SETCELL;
        op->flags = 0;
        op->pos1 = (int32_t)mtr_rng_below(&st->rng, (uint32_t)Lr);
        op->pos2 = (int32_t)mtr_rng_below(&st->rng, (uint32_t)Lc);
        return;
    }
    op->flags = (uint8_t)(MTR_F_LAST | (cols ? MTR_F_COLS : 0));
    if (kind == 0) {
        op->type = MTR_OP_INSERT;
        op->pos1 = (int32_t)mtr_rng_below(&st->rng, (uint32_t)L + 1u);
        op->pos2 = -1;
        op->payload2 = 1u + mtr_rng_below(&st->rng, cfg->max_text);
    } else {
        const int32_t start = (int32_t)mtr_rng_below(&st->rng, (uint32_t)L);
        uint32_t room = (uint32_t)(L - start);
        if (room > cfg->max_range) room = cfg->max_range;
        op->type = MTR_OP_REMOVE;
        op->pos1 = start;
        op->pos2 = start + 1 + (int32_t)mtr_rng_below(&st->rng, room);
    }
}

#ifdef __cplusplus
}
#endif
#endif /* MTR_SYNTH_H */
