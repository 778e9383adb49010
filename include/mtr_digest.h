/*
 * mtr_digest.h -- the 64-bit summary digest shared by the engine (summary_write_kernel), the CPU
 * oracle and the Python tests.  It only checks bit-exactness between implementations; it is not a
 * reference-visible value.
 *
 * Per blob of n bytes: 8-byte little-endian words w_j (the last one zero-padded) each contribute
 * mix(w_j ^ (j + 1) * G) to a sum mod 2**64 -- position-sensitive and computable by all lanes of a
 * wave at once -- finished with the length.  Per document: nblobs, then every blob's value in
 * order, folded through mix.  Plain C, header-only, usable from host code and HIP device code.
 */
#ifndef MTR_DIGEST_H
#define MTR_DIGEST_H

#include <stdint.h>

#ifdef __HIPCC__
#define MTR_DG_HD __host__ __device__
#else
#define MTR_DG_HD
#endif

#define MTR_DG_GOLDEN 0x9e3779b97f4a7c15ULL
#define MTR_DG_LEN 0xd6e8feb86659fd93ULL
#define MTR_DG_SEED 0x6d74723634ULL

static inline MTR_DG_HD uint64_t mtr_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/* term of word j (0-based) of a blob */
static inline MTR_DG_HD uint64_t mtr_dg_word(uint64_t w, uint64_t j) { return mtr_mix64(w ^ ((j + 1) * MTR_DG_GOLDEN)); }

/* value of a blob from the sum of its word terms and its length in bytes */
static inline MTR_DG_HD uint64_t mtr_dg_blob(uint64_t sum, uint64_t len) { return mtr_mix64(sum ^ (len * MTR_DG_LEN)); }

static inline MTR_DG_HD uint64_t mtr_dg_begin(uint64_t nblobs) { return mtr_mix64(nblobs ^ MTR_DG_SEED); }
static inline MTR_DG_HD uint64_t mtr_dg_next(uint64_t h, uint64_t blob_value) { return mtr_mix64(h ^ blob_value); }

/* host convenience: value of one blob */
static inline uint64_t mtr_dg_blob_bytes(const uint8_t* p, uint64_t n) {
    uint64_t sum = 0;
    for (uint64_t j = 0; 8 * j < n; j++) {
        uint64_t w = 0;
        for (uint64_t b = 0; b < 8 && 8 * j + b < n; b++) w |= (uint64_t)p[8 * j + b] << (8 * b);
        sum += mtr_dg_word(w, j);
    }
    return mtr_dg_blob(sum, n);
}

#endif /* MTR_DIGEST_H */
