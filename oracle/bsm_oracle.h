/*
 * bsm_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference crate's hot path
 * (jamieapps101/Basic_Sparse_Matrix, pure Rust, src/sparse.rs + src/lib.rs),
 * used ONLY by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg as the checker. Nothing in basic_sparse_matrix_amd/ links or calls it.
 *
 * Parity pinning: the reference cannot be built here (no Rust toolchain,
 * SURVEY.md §8c), so this restatement is pinned by the reference's own unit
 * test golden vectors (tests/golden/reference_unit_tests.json, every value
 * transcribed from src/sparse.rs / src/lib.rs #[test] functions).
 *
 * Conventions mirrored from the reference:
 *  - indices are usize -> uint64_t;
 *  - a CSR is (row_index, col_index, v); row_index has length rows+1 once
 *    finalised (sparse.rs:206-219);
 *  - integer arithmetic WRAPS (bench profile overflow-checks=false,
 *    Cargo.toml:18);
 *  - float arithmetic is plain IEEE, no FMA contraction (Rust never fuses);
 *    this file must be compiled with -ffp-contract=off.
 *
 * Return codes: 0 = ok, ORC_ERR_* otherwise (a reference `panic!` maps to
 * ORC_ERR_PANIC, a reference `Err(MatErr::X)` to the matching code).
 */
#ifndef BSM_ORACLE_H
#define BSM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_OK = 0,
    ORC_ERR_INCORRECT_DIMENSIONS = 1, /* MatErr::IncorrectDimensions */
    ORC_ERR_NON_SQUARE = 2,           /* MatErr::NonSquareMatrix */
    ORC_ERR_PANIC = 3,                /* reference would panic (OOB, unwrap on None) */
    ORC_ERR_ALLOC = 4,                /* output capacity too small */
    ORC_ERR_UNSUPPORTED = 5           /* band restatement not exact for this input */
};

/* ---- SpMM: Csr::mul_dense (sparse.rs:426-446) --------------------------
 * A: rows x cols with row_index (length ri_len, rows+1 when finalised),
 * col_index/v of length nnz. X: k columns of length cols, column c at
 * x + c*ldx (Dense<T> is Vec<Vec<T>>, one Vec per column, dense.rs:8).
 * Output: CSR rows x k; out_row (rows+1), out_col/out_v with capacity
 * rows*k; *out_nnz receives the output nnz. */
#define ORC_DECL_MUL_DENSE(SUF, T)                                                        \
    int orc_mul_dense_##SUF(uint64_t rows, uint64_t cols, const uint64_t* row_index,       \
                            uint64_t ri_len, const uint64_t* col_index, const T* v,        \
                            uint64_t nnz, uint64_t k, uint64_t x_rows, const T* x,         \
                            uint64_t ldx, uint64_t* out_row, uint64_t* out_col, T* out_v,  \
                            uint64_t* out_nnz);                                            \
    int orc_mul_vector_##SUF(uint64_t rows, uint64_t cols, const uint64_t* row_index,      \
                             uint64_t ri_len, const uint64_t* col_index, const T* v,       \
                             uint64_t nnz, const T* rhs, uint64_t rhs_len, T* out,         \
                             uint64_t out_len);                                            \
    int orc_transpose_##SUF(uint64_t rows, uint64_t cols, const uint64_t* row_index,       \
                            uint64_t ri_len, const uint64_t* col_index, const T* v,        \
                            uint64_t nnz, uint64_t* t_row, uint64_t* t_col, T* t_v);

/* ---- Construction: a sequence of Csr::insert calls then finalise ---------
 * insert (sparse.rs:222-233) skips value == default; insert_unchecked
 * (sparse.rs:237-250) appends and extends row_index only when `row` exceeds
 * the rows recorded so far (running max); finalise (sparse.rs:206-220)
 * panics ("big eek") when rows < row_index.len(), else pads to rows + 1.
 * Output: out_row (rows+1), out_col/out_v (capacity n); ORC_ERR_PANIC on
 * the finalise panic.
 * orc_csr_from_coo: From<COO<T>> for Csr<T> (sparse.rs:56-66), a stable sort
 * by (row, col) then the same insert sequence; an entry outside dims is
 * COO::insert's Err(OutOfBounds) (sparse.rs:45-53) -> ORC_ERR_PANIC. */
#define ORC_DECL_FROM_INSERTS(SUF, T)                                                      \
    int orc_csr_from_inserts_##SUF(uint64_t rows, uint64_t n, const uint64_t* row,         \
                                   const uint64_t* col, const T* v, uint64_t* out_row,     \
                                   uint64_t* out_col, T* out_v, uint64_t* out_nnz);        \
    int orc_csr_from_coo_##SUF(uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row, \
                               const uint64_t* col, const T* v, uint64_t* out_row,          \
                               uint64_t* out_col, T* out_v, uint64_t* out_nnz);

/* ---- add_sparse / sub_sparse (sparse.rs:484-599), mul_sparse (:601-635) --
 * Inputs are finalised CSRs (row arrays of rows+1). add/sub: out capacity
 * a_nnz + b_nnz; ORC_ERR_INCORRECT_DIMENSIONS on a dims mismatch,
 * ORC_ERR_PANIC for rows == 0 (the reference's row loop never ends). mul:
 * out capacity rows * b_cols. */
#define ORC_DECL_SPARSE_OPS(SUF, T)                                                                 \
    int orc_addsub_sparse_##SUF(int sub, uint64_t rows, uint64_t cols, const uint64_t* a_row,        \
                                const uint64_t* a_col, const T* a_v, uint64_t b_rows, uint64_t b_cols, \
                                const uint64_t* b_row, const uint64_t* b_col, const T* b_v,          \
                                uint64_t* out_row, uint64_t* out_col, T* out_v, uint64_t* out_nnz);  \
    int orc_mul_sparse_##SUF(uint64_t rows, uint64_t cols, const uint64_t* a_row, const uint64_t* a_col, \
                             const T* a_v, uint64_t b_rows, uint64_t b_cols, const uint64_t* b_row,    \
                             const uint64_t* b_col, const T* b_v, uint64_t* out_row,                  \
                             uint64_t* out_col, T* out_v, uint64_t* out_nnz);

ORC_DECL_SPARSE_OPS(f64, double)
ORC_DECL_SPARSE_OPS(f32, float)
ORC_DECL_SPARSE_OPS(i32, int32_t)
ORC_DECL_SPARSE_OPS(u32, uint32_t)
ORC_DECL_SPARSE_OPS(i64, int64_t)
ORC_DECL_SPARSE_OPS(u64, uint64_t)

ORC_DECL_FROM_INSERTS(f64, double)
ORC_DECL_FROM_INSERTS(f32, float)
ORC_DECL_FROM_INSERTS(i32, int32_t)
ORC_DECL_FROM_INSERTS(u32, uint32_t)
ORC_DECL_FROM_INSERTS(i64, int64_t)
ORC_DECL_FROM_INSERTS(u64, uint64_t)

ORC_DECL_MUL_DENSE(f64, double)
ORC_DECL_MUL_DENSE(f32, float)
ORC_DECL_MUL_DENSE(i32, int32_t)
ORC_DECL_MUL_DENSE(u32, uint32_t)
ORC_DECL_MUL_DENSE(i64, int64_t)
ORC_DECL_MUL_DENSE(u64, uint64_t)

/* ---- Cholesky (sparse.rs:682-714), tri-solves and solve (lib.rs:11-65) ---
 * Literal restatement: dense O(N^3) working arrays, identical operation
 * order to the reference loops (ascending k sums, sqrt for powf(0.5),
 * reciprocal-then-multiply off-diagonal, zero-skipping insert).
 * Band restatement: identical per-entry operation order restricted to the
 * envelope of A (skipped terms are +-0 products,
 * which never change a sum that starts at +0), O(N b^2).
 * Output L as CSR: l_row (n+1), l_col/l_v with capacity given by *l_cap;
 * on ORC_ERR_ALLOC *l_cap receives the needed capacity. */
#define ORC_DECL_CHOL(SUF, T)                                                              \
    int orc_cholesky_literal_##SUF(uint64_t n_rows, uint64_t n_cols,                       \
                                   const uint64_t* row_index, const uint64_t* col_index,   \
                                   const T* v, uint64_t* l_row, uint64_t* l_col, T* l_v,   \
                                   uint64_t* l_cap);                                       \
    int orc_cholesky_band_##SUF(uint64_t n_rows, uint64_t n_cols,                          \
                                const uint64_t* row_index, const uint64_t* col_index,      \
                                const T* v, uint64_t* l_row, uint64_t* l_col, T* l_v,      \
                                uint64_t* l_cap);                                          \
    int orc_forward_substitution_##SUF(uint64_t n, const uint64_t* l_row,                 \
                                       const uint64_t* l_col, const T* l_v, uint64_t k,    \
                                       const T* b, uint64_t ldb, T* y, uint64_t ldy);      \
    int orc_backward_substitution_##SUF(uint64_t n, const uint64_t* u_row,                \
                                        const uint64_t* u_col, const T* u_v, uint64_t k,   \
                                        const T* y, uint64_t ldy, T* x, uint64_t ldx);     \
    int orc_solve_##SUF(uint64_t n, const uint64_t* row_index, const uint64_t* col_index,  \
                        const T* v, uint64_t k, const T* b, uint64_t ldb, T* x,            \
                        uint64_t ldx, int use_band);

ORC_DECL_CHOL(f64, double)
ORC_DECL_CHOL(f32, float)

/* ---- Synthetic inputs (bsm_synth.h recipe, host side) -------------------- */
/* Timing fidelity switch for the CPU baseline: emulate get_row_compact's
 * per-row Vec allocation (capacity dims.cols x 24 B, sparse.rs:254). */
void orc_set_emulate_row_alloc(int on);

/* Row lengths for CONST/UNIFORM/BINOMIAL families -> row_ptr (rows+1). */
int orc_gen_row_ptr(uint64_t seed, uint64_t rows, uint32_t n_cols, int rowlen_kind,
                    uint32_t a, uint32_t b, uint64_t* row_ptr);
/* Fill col_idx (sorted, distinct) and values (as double) for rows [r0, r1). */
int orc_gen_entries(uint64_t seed, uint64_t r0, uint64_t r1, uint32_t n_cols,
                    const uint64_t* row_ptr, int value_kind, uint64_t* col_idx,
                    double* vals);
/* X column-major (k columns of n_cols) from seed. */
void orc_gen_x_colmajor(uint64_t seed, uint64_t n_cols, uint64_t k, int value_kind,
                        double* x);
/* Bench-shaped insert stream (bsm_synth.h bsm_stream_draw): row/col/v of
 * entries [0, n) with the given moduli. */
void orc_gen_insert_stream(uint64_t seed, uint64_t n, uint64_t rows, uint64_t cols, uint64_t vmod,
                           uint64_t* row, uint64_t* col, uint64_t* v);
/* 5-point 2D Poisson on a g x g grid, natural row-major ordering: diag 4,
 * neighbours -1 (Dirichlet). Sorted columns per row. Returns nnz. */
uint64_t orc_gen_poisson2d(uint64_t g, uint64_t* row_ptr, uint64_t* col_idx, double* v);

#ifdef __cplusplus
}
#endif

#endif /* BSM_ORACLE_H */
