/*
 * bsm_synth.h -- deterministic synthetic-input generator shared by the HIP
 * kernels (device) and the CPU oracle / host code (gcc).
 *
 * Why it exists: the reference bench builds its inputs with rand 0.8.5's
 * StdRng (benches/sparse_dense_mul.rs:16-28), which is not vendored, so the
 * exact bench matrices are unreproducible ("parity unpinned", SURVEY.md
 * §8c). Instead every input of the parity suites and of bench.py comes from
 * this counter-based SplitMix64 hash, keyed by (seed, row, j). Because every
 * draw is a pure function of its key, a row can be generated independently
 * on the GPU (one workgroup per row) and on the host, and both produce the
 * same integers bit for bit. No floating-point transcendental is used, so
 * host and device cannot disagree on rounding.
 *
 * Matrix recipe: per row r, nnz_r column draws
 *   c_j = (hash(seed,r,j) >> 32) * n_cols >> 32           (Lemire range map)
 * sorted ascending, then made strictly increasing by the "bump" pass
 *   c'_j = max(c_j, c'_{j-1} + 1)      (forward)
 *   c''_j = min(c'_j, c''_{j+1} - 1)   (backward, c''_last <= n_cols-1)
 * which is a prefix-max / suffix-min and therefore also computable in
 * parallel (see spmm.hip gen kernels). Values are uniform in [0.5, 1.5).
 */
#ifndef BSM_SYNTH_H
#define BSM_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define BSM_HD __host__ __device__ __forceinline__
#else
#define BSM_HD static inline
#endif

/* SplitMix64 finaliser (Steele, Lea, Flood 2014). */
BSM_HD uint64_t bsm_mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/* Counter-based hash of a (seed, a, b, salt) key. */
BSM_HD uint64_t bsm_hash(uint64_t seed, uint64_t a, uint64_t b, uint64_t salt) {
    uint64_t h = bsm_mix64(seed ^ (salt * 0xd1b54a32d192ed03ULL));
    h = bsm_mix64(h ^ a);
    return bsm_mix64(h ^ (b * 0x9e3779b97f4a7c15ULL));
}

enum {
    BSM_SALT_ROWLEN = 1,
    BSM_SALT_COL = 2,
    BSM_SALT_VAL = 3,
    BSM_SALT_X = 4,
    BSM_SALT_STREAM = 5
};

/* Value families (bsm_gen_spec.value_kind). */
enum {
    BSM_VAL_UNIFORM = 0, /* uniform [0.5, 1.5): positive, zero pattern order-independent */
    BSM_VAL_SMALLINT = 1 /* integers in {-3..-1, 1..3}: exact f64 arithmetic, exact cancellations */
};

/* Row-length families (bsm_gen_spec.rowlen_kind). */
enum {
    BSM_ROWLEN_CONST = 0,   /* every row has exactly `rowlen_a` entries */
    BSM_ROWLEN_UNIFORM = 1, /* uniform in [rowlen_a, rowlen_b] */
    BSM_ROWLEN_BINOMIAL = 2 /* Binomial(n_cols, p) with p = rowlen_a / 2^32 (host-only, O(n_cols)/row) */
};

/* Uniform double in [0.5, 1.5) from 53 hash bits. Exact on host and device. */
BSM_HD double bsm_unit_uniform(uint64_t h) {
    return 0.5 + (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

BSM_HD double bsm_val_from_hash(uint64_t h, int kind) {
    if (kind == BSM_VAL_SMALLINT) {
        int m = (int)(h % 6u); /* 0..5 -> -3,-2,-1,1,2,3 */
        return (double)(m < 3 ? m - 3 : m - 2);
    }
    return bsm_unit_uniform(h);
}

/* Dense RHS element X[col][j] (seed 1001 in the bench). For SMALLINT the
 * family also produces exact zeros (the bench's mostly-zero X,
 * sparse_dense_mul.rs:24-29). */
BSM_HD double bsm_x_value(uint64_t seed, uint64_t col, uint64_t j, int kind) {
    uint64_t h = bsm_hash(seed, col, j, BSM_SALT_X);
    if (kind == BSM_VAL_SMALLINT) {
        return (double)((int)(h % 7u) - 3); /* -3..3, includes 0 */
    }
    return bsm_unit_uniform(h);
}

/* Column draw j of row r: uniform in [0, n_cols). */
BSM_HD uint32_t bsm_col_draw(uint64_t seed, uint64_t row, uint64_t j, uint32_t n_cols) {
    uint64_t h = bsm_hash(seed, row, j, BSM_SALT_COL);
    return (uint32_t)(((h >> 32) * (uint64_t)n_cols) >> 32);
}

BSM_HD double bsm_a_value(uint64_t seed, uint64_t row, uint64_t j, int kind) {
    return bsm_val_from_hash(bsm_hash(seed, row, j, BSM_SALT_VAL), kind);
}

/* Row length of the BINOMIAL family: the number of columns j < n_cols whose
 * hash falls below p * 2^32 (p = a / 2^32), i.e. Binomial(n_cols, p); O(n_cols)
 * per row, meant for small matrices (C1: 1024 x 1024, p = 0.01). */
BSM_HD uint32_t bsm_rowlen_binomial(uint64_t seed, uint64_t row, uint32_t n_cols, uint32_t a) {
    uint32_t len = 0;
    for (uint32_t j = 0; j < n_cols; ++j)
        if ((bsm_hash(seed, row, j, BSM_SALT_ROWLEN) >> 32) < (uint64_t)a) ++len;
    return len;
}

/* Row length for the CONST / UNIFORM families (BINOMIAL: bsm_rowlen_binomial). */
BSM_HD uint32_t bsm_rowlen(uint64_t seed, uint64_t row, int kind, uint32_t a, uint32_t b) {
    if (kind == BSM_ROWLEN_UNIFORM) {
        uint64_t h = bsm_hash(seed, row, 0, BSM_SALT_ROWLEN);
        uint64_t span = (uint64_t)b - (uint64_t)a + 1u;
        return a + (uint32_t)(((h >> 32) * span) >> 32);
    }
    return a;
}

/* Insert stream shaped like the reference bench (sparse_dense_mul.rs:16-22):
 * entry i is insert(v, row, col) with row = draw0 % rows, col = draw1 % cols,
 * v = draw2 % vmod (the bench: 1000, 1000, 255 -- v == 0 is skipped by
 * insert, and the running-max row rule of insert_unchecked piles almost
 * every entry into the last rows). Draw f of entry i is
 * bsm_hash(seed, i, f, BSM_SALT_STREAM); StdRng itself is not vendored. */
BSM_HD uint64_t bsm_stream_draw(uint64_t seed, uint64_t i, uint64_t field) {
    return bsm_hash(seed, i, field, BSM_SALT_STREAM);
}

#endif /* BSM_SYNTH_H */
