/*
 * bsm.h -- C-ABI of the MI355X-native sparse-matrix hot path
 * (libbsm_hip.so, built from basic_sparse_matrix_amd/csrc/).
 *
 * This is the drop-in boundary for the reference crate
 * jamieapps101/Basic_Sparse_Matrix (pure Rust). The reference has no FFI of
 * its own; these are the entry points its hot-path methods would bind
 * through `extern "C"` (see INTEGRATION.md for the Rust-side binding). Every
 * function below names the reference item it replaces.
 *
 * Conventions
 *  - Plain pointers and sizes only; indices are uint64_t like Rust's usize.
 *  - Host-buffer entry points (bsm_csr_*, bsm_solve, ...) are synchronous:
 *    when they return, device work is complete and output host buffers are
 *    filled. The library NEVER takes ownership of caller memory; device
 *    memory is owned by opaque handles released with bsm_csr_free.
 *  - Device entry points (bsm_dev_*) take device (HBM) pointers and a
 *    hipStream_t passed as void*; they enqueue work and return immediately.
 *  - Return value: BSM_OK (0) or a bsm_status; bsm_last_error() gives a
 *    thread-local message. Dimension checks that the reference answers with
 *    Err(MatErr::...) are repeated here (BSM_ERR_DIMENSIONS /
 *    BSM_ERR_NON_SQUARE) but callers are expected to check first, as the
 *    reference does, so that Err values stay identical.
 *  - Arithmetic: floating point is IEEE with no FMA contraction and the
 *    reference's summation order (bit-exact); integers wrap
 *    (reference bench profile overflow-checks=false, Cargo.toml:18).
 *  - Device CSR layout: row_ptr int64[rows+1], col int32[nnz] (so cols must
 *    be < 2^31), values T[nnz]. Dense operands on device are ROW-major
 *    (n x k, element (r,j) at r*k + j) so one CSR entry gathers k contiguous
 *    values; host Dense operands are the reference's column list
 *    (Vec<Vec<T>>, dense.rs:8) passed as an array of k column pointers.
 */
#ifndef BSM_H
#define BSM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSM_API_VERSION 1

/* Scalar types of the reference's generic T that run on the GPU. */
typedef enum bsm_dtype {
    BSM_F64 = 0,
    BSM_F32 = 1,
    BSM_I32 = 2,
    BSM_U32 = 3,
    BSM_I64 = 4,
    BSM_U64 = 5
} bsm_dtype;

typedef enum bsm_status {
    BSM_OK = 0,
    BSM_ERR_INVALID = 1,     /* bad argument (null pointer, unknown dtype, ...) */
    BSM_ERR_DIMENSIONS = 2,  /* MatErr::IncorrectDimensions (util.rs:51) */
    BSM_ERR_NON_SQUARE = 3,  /* MatErr::NonSquareMatrix (util.rs:50) */
    BSM_ERR_PANIC = 4,       /* input on which the reference panics (OOB index, empty row) */
    BSM_ERR_HIP = 5,         /* HIP runtime error */
    BSM_ERR_OOM = 6,         /* device allocation failed */
    BSM_ERR_UNSUPPORTED = 7, /* valid input outside what this build implements */
    BSM_ERR_NO_DEVICE = 8,   /* no usable gfx950 device */
    BSM_ERR_OUT_OF_BOUNDS = 9, /* MatErr::OutOfBounds (util.rs:54; COO::insert, sparse.rs:45-53) */
    BSM_ERR_COMM = 10          /* RCCL error (multi-GPU entry points) */
} bsm_status;

/* Opaque device-resident CSR matrix (a finalised Csr<T>, sparse.rs:68-78). */
typedef struct bsm_csr bsm_csr;

/* ---- library ------------------------------------------------------------ */
int bsm_api_version(void);
/* Thread-local description of the last failure on this thread. */
const char* bsm_last_error(void);
/* Device time of the stages of the last bsm_solve / bsm_solve_blocked /
 * bsm_csr_cholesky on this thread (HIP events on its stream): *n stages; the
 * first min(max, *n) names (32 chars each, NUL-terminated) and durations in
 * ms. Diagnostic, recorded only while armed by bsm_stage_timing(1) (or env
 * BSM_STAGE_TIMES=1). */
int bsm_stage_timing(int on);
int bsm_stage_times(int max, int* n, char* names, double* ms);
int bsm_device_count(int* n);
/* Select the device used by subsequent calls on this thread. */
int bsm_set_device(int ordinal);

/* ---- device-resident CSR handles ---------------------------------------- */
/* Upload a finalised Csr<T> (sparse.rs:68-78: row_index = row_ptr of length
 * rows+1, col_index, v). Replaces nothing in the reference: it is the
 * marshalling step a Rust `mul_dense` performs before the kernel call (the
 * handle can be cached by the caller because a finalised Csr is immutable:
 * insert returns Err(MatrixFinalised), sparse.rs:223-225). */
int bsm_csr_upload(int dtype, uint64_t rows, uint64_t cols, uint64_t nnz,
                   const uint64_t* row_ptr, const uint64_t* col_idx, const void* vals,
                   bsm_csr** out);
/* Build a finalised Csr on the device from a SEQUENCE of Csr::insert(v[i],
 * row[i], col[i]) calls followed by finalise (sparse.rs:206-250): zero
 * values are skipped, an entry belongs to the running maximum of the rows
 * inserted so far (insert_unchecked, sparse.rs:237-250), skipped rows get
 * empty ranges, and finalise pads row_index. A kept row >= rows is the
 * reference's finalise panic ("big eek", sparse.rs:210) -> BSM_ERR_PANIC;
 * a kept col >= cols -> BSM_ERR_PANIC (the device Csr holds in-bounds
 * columns). Host arrays of n entries. */
int bsm_csr_from_inserts(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                         const uint64_t* col, const void* vals, bsm_csr** out);
/* From<COO<T>> for Csr<T> (sparse.rs:56-66): the n COO entries (row[i],
 * col[i], vals[i]) in insert order, stably sorted by (row, col) (Rust's
 * sort_by is stable), then inserted (zero skip) and finalised. The
 * reference's per-entry println! is not reproduced. An entry outside dims
 * (COO::insert would have returned Err(OutOfBounds)) -> BSM_ERR_OUT_OF_BOUNDS.
 * Host arrays. */
int bsm_csr_from_coo(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                     const uint64_t* col, const void* vals, bsm_csr** out);
int bsm_csr_shape(const bsm_csr* m, uint64_t* rows, uint64_t* cols, uint64_t* nnz,
                  int* dtype);
/* Copy a handle back into caller-allocated host arrays (rows+1, nnz, nnz).
 * A small bsm_csr_mul_dense result (at most 8,192 rows and 131,072 row x
 * column slots) carries a host copy written by the same kernel as its device
 * arrays: its download is a host copy with no device work. */
int bsm_csr_download(const bsm_csr* m, uint64_t* row_ptr, uint64_t* col_idx, void* vals);
/* Page-lock (hipHostRegister) / release a caller-owned host range that result
 * arrays are downloaded into again and again (this build's addition; no
 * reference counterpart). bsm_csr_download into registered arrays is one
 * direct DMA per array, the columns widened to usize on the device; into
 * pageable arrays it stages through pinned buffers. The Python mirror's host
 * result pool (hostpool.py) registers its mappings once. */
int bsm_host_register(void* p, uint64_t bytes);
int bsm_host_unregister(void* p);
void bsm_csr_free(bsm_csr* m);

/* ---- hot path (host buffers in/out, synchronous) ------------------------- */
/* Csr::mul_dense (sparse.rs:426-446) and Csr::mul_dense_s (sparse.rs:448-466):
 * out = a * X as a new finalised Csr with dims (rows, k), zero results
 * dropped (sparse.rs:229). X is k columns of x_rows values each
 * (Dense::get_col, dense.rs:31-33). x_rows != cols -> BSM_ERR_DIMENSIONS. */
int bsm_csr_mul_dense(const bsm_csr* a, uint64_t k, uint64_t x_rows, const void* const* x_cols,
                      bsm_csr** out);
/* Csr::mul_vector (sparse.rs:468-482): out[i] = sum over row i of
 * v * rhs[col] in ascending column order, dense output, no zero skip. */
int bsm_csr_mul_vector(const bsm_csr* a, const void* rhs, uint64_t rhs_len, void* out,
                       uint64_t out_len);
/* Csr::transpose (sparse.rs:296-318): stable CSR -> CSC. */
int bsm_csr_transpose(const bsm_csr* a, bsm_csr** out);
/* Csr::add_sparse (sparse.rs:484-540) / Csr::sub_sparse (sparse.rs:542-599):
 * the reference's per-row two-pointer merge over the operands' entries in
 * storage order (rhs-only entries of sub become T::default() - v), zero
 * results dropped. Dims differ -> BSM_ERR_DIMENSIONS; 0 rows -> BSM_ERR_PANIC
 * (the reference's row loop never ends). Same dtype required. */
int bsm_csr_add_sparse(const bsm_csr* a, const bsm_csr* b, bsm_csr** out);
int bsm_csr_sub_sparse(const bsm_csr* a, const bsm_csr* b, bsm_csr** out);
/* Csr::mul_sparse (sparse.rs:601-635): dims (a.rows, b.cols), no dimension
 * check; every result entry is the reference's merge of a's row (storage
 * order) with row j of b.transpose(), kept when nonzero. */
int bsm_csr_mul_sparse(const bsm_csr* a, const bsm_csr* b, bsm_csr** out);
/* impl Csr<f32>::cholesky_decomp (sparse.rs:682-714); F64 is this build's
 * addition. Square check -> BSM_ERR_NON_SQUARE.
 * Non-SPD inputs store the reference's NaN/inf, unsorted rows are read as
 * get_row_complete does, the :707 unwrap on an unregistered L row ->
 * BSM_ERR_PANIC; those (and bands > 1073) need n <= 16384, else
 * BSM_ERR_UNSUPPORTED. bsm_solve follows the same rules. */
int bsm_csr_cholesky(const bsm_csr* a, bsm_csr** out);
/* forward_substitution (lib.rs:28-46): solve L y = b for k RHS columns of n. */
int bsm_forward_substitution(const bsm_csr* l, uint64_t k, uint64_t n,
                             const void* const* b_cols, void* const* y_cols);
/* backward_substitution (lib.rs:49-65): solve U x = y, U = L^T as a Csr. */
int bsm_backward_substitution(const bsm_csr* u, uint64_t k, uint64_t n,
                              const void* const* y_cols, void* const* x_cols);
/* solve (lib.rs:11-24): x = A^-1 b via cholesky_decomp + transpose +
 * forward/backward substitution, all on the device. */
int bsm_solve(const bsm_csr* a, uint64_t k, uint64_t n, const void* const* b_cols,
              void* const* x_cols);
/* solve (lib.rs:11-24) with the triangular solves REASSOCIATED: 64-row
 * blocks, precomputed inverse diagonal blocks, far sums in any order. The
 * factor is the reference-order one; x is NOT bit-exact with the reference but
 * within its f64 tolerance (1e-6 relative, BASELINE.json north_star). Same
 * arguments, errors and panics as bsm_solve. This build's addition. */
int bsm_solve_blocked(const bsm_csr* a, uint64_t k, uint64_t n, const void* const* b_cols,
                      void* const* x_cols);
/* solve (lib.rs:11-24) by a nested-dissection multifrontal Cholesky of
 * P A P^T: P from recursive BFS level-set bisection of A's graph (host), the
 * separator tree's dense fronts factored level by level on the device. x is
 * NOT bit-exact with the reference (another elimination order) but within its
 * f64 tolerance (1e-6 relative, BASELINE.json north_star). A is its lower
 * triangle (j <= i) mirrored, as cholesky_decomp reads it; rows must have
 * strictly increasing columns, and a pivot <= 0 (not SPD) -> BSM_ERR_UNSUPPORTED.
 * Same arguments and panics as bsm_solve. This build's addition.
 * Plans: the analysis of a pattern (ordering, tree, device index arrays) is
 * kept on the handle AND in a library-wide cache keyed by the pattern (a
 * 128-bit device hash of row_ptr and col, each hit confirmed by comparing
 * the pattern itself), because solve takes `a` by value (lib.rs:11) and a
 * drop-in caller uploads a new handle for every call: a new handle with a
 * pattern seen before skips the analysis. Retention: after a solve the plan
 * keeps its numeric storage (the fronts, inverse diagonal tiles and flags:
 * ~5.6 GB at C5 in f64) for the next solve of that pattern. The cache holds
 * at most BSM_ND_CACHE_ENTRIES patterns (default 4, least recently used
 * out) and at most BSM_ND_CACHE_MB of kept storage (default 32768) across
 * them; an allocation that fails for lack of memory first drops the other
 * plans' kept storage and retries. bsm_nd_cache_clear releases every cached
 * plan not also held by a live handle (bsm_csr_free releases the handle's).
 * Env BSM_ND_CACHE=0: no plan kept anywhere; BSM_ND_SHARED=0: per handle only;
 * BSM_ND_KEEP=0: numeric storage freed after every solve. A plan also holds
 * A's lower entries sorted by front tile (8 bytes each) and two small
 * per-task arrays. With one right-hand side (k == 1) the forward solve is
 * formed inside the factor (another summation order than k > 1, within
 * rounding; BSM_ND_FOLD=0 turns it off). The factor's other switches
 * (README.md's table) change no bits. */
int bsm_solve_nd(const bsm_csr* a, uint64_t k, uint64_t n, const void* const* b_cols,
                 void* const* x_cols);
/* The cross-handle plan cache of bsm_solve_nd: drop every entry, or read its
 * state (entries, kept numeric bytes, lookups that hit / missed since load).
 * Any pointer may be NULL. This build's addition. */
int bsm_nd_cache_clear(void);
int bsm_nd_cache_info(uint64_t* entries, uint64_t* kept_bytes, uint64_t* hits, uint64_t* misses);
/* The analysis of bsm_solve_nd alone, on a host pattern (row_ptr n+1, col_idx
 * row_ptr[n]); no device use (tests, diagnostics). Writes perm (n entries,
 * perm[new] = old) when non-null; *n_nodes and *st_len always; when cap >=
 * *n_nodes and st_cap >= *st_len, the tree in post-order as 8 int64 per node
 * (start, end, parent, level, slot, m, offset into st, 0) and every node's m
 * front rows (new indices, ascending) into st. This build's addition. */
int bsm_nd_analyse(uint64_t n, const uint64_t* row_ptr, const uint64_t* col_idx, uint64_t leaf,
                   int64_t* perm, int64_t* nodes, uint64_t cap, uint64_t* n_nodes, int64_t* st,
                   uint64_t st_cap, uint64_t* st_len);

/* ---- device-level entry points (HBM pointers, async on `stream`) --------- */
/* Synthetic CSR generator (bsm_synth.h recipe): rows [row0, row0+rows) of a
 * matrix with n_cols columns, rowlen_kind CONST/UNIFORM (a, b), value_kind
 * UNIFORM/SMALLINT. Writes row_ptr (rows+1, local, starting at 0), col, vals.
 * bsm_dev_gen_row_ptr must run first; its nnz is row_ptr[rows]. Rows longer
 * than 4096 are not supported by the device generator. */
int bsm_dev_gen_row_ptr(uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols,
                        int rowlen_kind, uint32_t a, uint32_t b, int64_t* row_ptr,
                        void* workspace, uint64_t workspace_bytes, void* stream);
int bsm_dev_gen_entries(int dtype, uint64_t seed, uint64_t row0, uint64_t rows,
                        uint32_t n_cols, int value_kind, const int64_t* row_ptr,
                        int32_t* col, void* vals, void* stream);
/* Insert stream shaped like the reference bench (sparse_dense_mul.rs:16-22;
 * bsm_synth.h bsm_stream_draw): entries i0 .. i0+n-1 with row = draw % rows,
 * col = draw % cols, v = draw % vmod (as dtype). Device arrays. */
int bsm_dev_gen_insert_stream(int dtype, uint64_t seed, uint64_t i0, uint64_t n, uint64_t rows,
                              uint64_t cols, uint64_t vmod, uint64_t* row, uint64_t* col, void* vals,
                              void* stream);
/* bsm_csr_from_inserts on device arrays (synchronous on `stream`). */
int bsm_dev_csr_from_inserts(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                             const uint64_t* col, const void* vals, bsm_csr** out, void* stream);
/* Dense ROW-major n x k operand: X[r][j] = bsm_x_value(seed, row0 + r, j). */
int bsm_dev_gen_dense(int dtype, uint64_t seed, uint64_t row0, uint64_t n, uint64_t k,
                      int value_kind, void* x, void* stream);
/* Workspace bytes needed by the scans of bsm_dev_gen_row_ptr / bsm_dev_spmm_csr. */
uint64_t bsm_dev_scan_workspace_bytes(uint64_t n);
/* Y = A X (dense ROW-major Y, rows x k), the kernel of mul_dense. row_nnz
 * (int32[rows], may be NULL) receives the count of nonzero results per row
 * for compaction. */
int bsm_dev_spmm(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz,
                 const int64_t* row_ptr, const int32_t* col, const void* vals, uint64_t k,
                 const void* x, void* y, int32_t* row_nnz, void* stream);
/* Width of the column-panel plan bsm_csr_mul_dense has cached for this
 * handle and uses (0 = one pass); diagnostic (see bsm_dev_spmm_plan). */
int bsm_csr_panel_cols(const bsm_csr* m, uint64_t* panel_cols);
/* Column-panel schedule of bsm_dev_spmm for an X larger than the 256 MiB
 * Infinity Cache (DESIGN.md "SpMM: column panels"); same results, bit for
 * bit. bsm_dev_spmm_panel_cols gives the panel width for (dtype, n_cols, k)
 * (0 = one pass is best: the schedule is used for f64, k = 32, X > 1 GiB;
 * env BSM_SPMM_PANEL_COLS overrides). bsm_dev_spmm_plan fills seg
 * (bsm_dev_spmm_plan_bytes bytes) once per matrix, synchronously, and sets
 * *usable = 0 when some row's columns do not visit the panels in order (then
 * call bsm_dev_spmm). bsm_dev_spmm_panelled = bsm_dev_spmm with the plan. */
uint64_t bsm_dev_spmm_panel_cols(int dtype, uint64_t n_cols, uint64_t k);
uint64_t bsm_dev_spmm_plan_bytes(uint64_t rows, uint64_t n_cols, uint64_t panel_cols);
int bsm_dev_spmm_plan(uint64_t rows, uint64_t n_cols, const int64_t* row_ptr, const int32_t* col,
                      uint64_t panel_cols, int32_t* seg, int* usable, void* stream);
int bsm_dev_spmm_panelled(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz,
                          const int64_t* row_ptr, const int32_t* col, const void* vals, uint64_t k,
                          const void* x, void* y, int32_t* row_nnz, uint64_t panel_cols,
                          const int32_t* seg, void* stream);
/* Row-block x column-panel schedule of bsm_dev_spmm (Csr::mul_dense,
 * sparse.rs:426-446) with k = 32 and X beyond the Infinity Cache (the C4
 * shape), or k = 1 and X beyond an XCD's L2 (C2); the copy is built for one k
 * (DESIGN.md "SpMM: row blocks x column panels"). bsm_csr_mul_dense builds
 * it for f64 and f32; these device-level entry points are the f64 form.
 * bsm_dev_tiled_create re-lays the matrix once (12 B per entry, 16 B from
 * 2^24 columns on at k = 32, plus chunk padding: a copy beside the CSR;
 * synchronous on `stream`) and returns BSM_ERR_UNSUPPORTED for a shape it
 * does not serve (cols >= 2^31 at k = 32, >= 2^21 at k = 1; rows so uneven
 * that chunk padding passes 25 % of the entries, unless flags has
 * BSM_TILED_ANY_PADDING) or BSM_ERR_OOM.
 * bsm_dev_spmm_tiled = bsm_dev_spmm on that copy: the same Y and row_nnz,
 * bit for bit (each row still sums in storage order). bsm_dev_tiled_wanted
 * says whether the library would use it for this shape (env BSM_SPMM_TILED:
 * 0 = never, 2 = whenever possible). bsm_tiled_info: bytes of the copy,
 * entry slots (entries + dummies) and the panel width in columns. */
typedef struct bsm_tiled bsm_tiled;
#define BSM_TILED_ANY_PADDING 1
int bsm_dev_tiled_wanted(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, uint64_t k,
                         uint64_t max_row_len);
int bsm_dev_tiled_create(uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* row_ptr,
                         const int32_t* col, const double* vals, uint64_t k, int flags,
                         bsm_tiled** out, void* stream);
int bsm_dev_spmm_tiled(const bsm_tiled* t, const double* x, double* y, int32_t* row_nnz,
                       void* stream);
int bsm_tiled_info(const bsm_tiled* t, uint64_t* bytes, uint64_t* slots, uint64_t* panel_cols);
/* Whether bsm_csr_mul_dense has built (and uses) the tiled copy for this
 * handle; diagnostic. */
int bsm_csr_tiled(const bsm_csr* m, int* in_use);
void bsm_tiled_destroy(bsm_tiled* t);
/* Compaction of a dense result into the reference's output Csr (insert's
 * zero skip, sparse.rs:229): out_row_ptr (rows+1), out_col/out_vals with
 * capacity rows*k. */
int bsm_dev_compact(int dtype, uint64_t rows, uint64_t k, const void* y,
                    const int32_t* row_nnz, int64_t* out_row_ptr, int32_t* out_col,
                    void* out_vals, void* workspace, uint64_t workspace_bytes, void* stream);

/* ---- multi-GPU: row blocks + RCCL all-gather (north_star) ----
 * Csr::mul_dense (sparse.rs:426-446) has independent rows (:431-444), so the
 * CSR is cut into P = chunks x world contiguous row blocks ("pieces") of
 * near-equal cost, a row costing its entries plus max(1, nnz/rows) (its output
 * row): bsm_partition_rows. For equal row lengths that is the nnz split; on
 * skewed matrices it keeps every piece under 2*rows/P + 1 rows. Piece
 * c*world + g belongs to global rank g and is computed in round c. Every
 * device keeps a replica of X. The dense Y blocks are assembled on every
 * device by RCCL all-gathers, one per round, in place and issued on a
 * communication stream as soon as the round's SpMM is done, so they overlap
 * the next round's SpMM. The output Csr is compacted on the first local
 * device of each process. Per-row sums do not depend on the partition, so
 * the result is bit-identical to bsm_csr_mul_dense.
 *
 * Two ways to build the context:
 *  - one process drives n_gpus devices (the reference's single-threaded Rust
 *    caller on an 8-GPU node): bsm_multi_create, i.e. SURVEY.md §8b's
 *    bsm_init(int n_gpus) with ncclCommInitAll;
 *  - one process per GPU (bench.py under torch.distributed.run): rank 0 calls
 *    bsm_multi_unique_id, the caller ships the BSM_UNIQUE_ID_BYTES bytes to
 *    every rank, and each rank calls bsm_multi_create_rank (ncclCommInitRank).
 *  - one process per rank with the caller's own transport (no RCCL
 *    communicator): bsm_multi_create_external. bsm_mcsr_step then only runs
 *    this rank's SpMM rounds into its slots of the gathered Y; the caller moves
 *    the slots between ranks (bsm_mcsr_slot_read / _write: slot c*world + r is
 *    round c of rank r, as the all-gather would place it) and calls
 *    bsm_mcsr_compact. bsm_mcsr_mul_dense and bsm_multi_broadcast return
 *    BSM_ERR_UNSUPPORTED on such a context.
 * Every rank of a communicator must make the same collective calls
 * (bsm_mcsr_mul_dense, bsm_mcsr_step, bsm_multi_broadcast) in the same order.
 * Threading: the calls on one bsm_mcsr are serialised by a lock held for the
 * whole call (a mul_dense from several threads on one matrix runs one after
 * the other); different matrices on one context may be driven from different
 * threads only if the context's communicator is not in use by two of them at
 * once (RCCL's rule for a communicator). */
typedef struct bsm_multi bsm_multi;
typedef struct bsm_mcsr bsm_mcsr;
#define BSM_UNIQUE_ID_BYTES 128
int bsm_multi_create(int n_gpus, const int* devices, bsm_multi** out);
int bsm_multi_unique_id(void* id);
int bsm_multi_create_rank(const void* id, int world, int rank, int device, bsm_multi** out);
int bsm_multi_create_external(int world, int rank, int device, bsm_multi** out);
int bsm_multi_is_external(const bsm_multi* ctx, int* external);
/* The piece bounds the multi-GPU path uses (host only, no device needed):
 * bounds[0..pieces] for row_ptr[0..rows]. row_ptr must hold rows + 1 entries
 * (it is not validated against anything: rows is trusted). */
int bsm_partition_rows(const uint64_t* row_ptr, uint64_t rows, uint32_t pieces, uint64_t* bounds);
/* world size, devices driven by this process, global rank of the first one */
int bsm_multi_info(const bsm_multi* ctx, int* world, int* n_local, int* first_rank);
/* Broadcast `bytes` from global rank `root` (its first local device's buffer)
 * into bufs[i] on every local device i (ncclBroadcast; synchronous). */
int bsm_multi_broadcast(bsm_multi* ctx, void* const* bufs, uint64_t bytes, int root);
/* SURVEY.md §8b bsm_finalize: releases streams and communicators. Matrices
 * made on the context must be freed first. */
void bsm_multi_destroy(bsm_multi* ctx);

/* Partitioned upload of a finalised Csr<T> (host arrays, as bsm_csr_upload):
 * each process uploads only its own devices' pieces. chunks >= 1. */
int bsm_mcsr_upload(bsm_multi* ctx, int dtype, uint64_t rows, uint64_t cols, uint64_t nnz,
                    const uint64_t* row_ptr, const uint64_t* col_idx, const void* vals, uint32_t chunks,
                    bsm_mcsr** out);
/* The synthetic matrix of bsm_dev_gen_row_ptr/bsm_dev_gen_entries (seed,
 * row-length family, value family), every device generating only its own
 * pieces (C4's 1e10 entries do not fit a host). */
int bsm_mcsr_generate(bsm_multi* ctx, int dtype, uint64_t seed, uint64_t rows, uint32_t n_cols, int rowlen_kind,
                      uint32_t a, uint32_t b, int value_kind, uint32_t chunks, bsm_mcsr** out);
/* rows, cols, nnz, pieces P, padded piece rows; bounds (P+1 entries, may be NULL) */
int bsm_mcsr_info(const bsm_mcsr* m, uint64_t* rows, uint64_t* cols, uint64_t* nnz, uint32_t* pieces,
                  uint64_t* piece_rows, uint64_t* bounds);
/* Build the per-piece SpMM schedules (schedule: 0 = the library's choice as
 * in bsm_csr_mul_dense, 1 = the row-block x column-panel copy whenever
 * possible, 2 = never the copy) and the gathered-Y and output buffers for k
 * right-hand columns. Synchronous; bsm_mcsr_mul_dense calls it when needed.
 * *plan_ms (may be NULL) receives per-phase host times of the slowest local
 * device: {total, tiled count pass, tiled scan, tiled allocation, tiled
 * write pass, panel plans, buffers}. */
int bsm_mcsr_prepare(bsm_mcsr* m, uint64_t k, int schedule, double* plan_ms);
/* The schedule prepare built, over this process's pieces: how many use the
 * row-block x column-panel copy, its bytes in total, and the panel width in
 * columns (the copy's, else the column-panel plan's; 0 = one pass). */
int bsm_mcsr_plan_info(const bsm_mcsr* m, int* tiled_pieces, int* local_pieces, uint64_t* copy_bytes,
                       uint64_t* panel_cols);
/* Csr::mul_dense on all GPUs: X (k host columns of x_rows, Dense::get_col)
 * uploaded to every local device, the step below, then the output Csr (dims
 * rows x k, zero results dropped, sparse.rs:229) as a new handle on the
 * first local device. x_rows != cols -> BSM_ERR_DIMENSIONS. */
int bsm_mcsr_mul_dense(bsm_mcsr* m, uint64_t k, uint64_t x_rows, const void* const* x_cols, bsm_csr** out);
/* Device level, asynchronous: x_dev[i] = X on local device i (ROW-major
 * cols x k). Enqueues the rounds' SpMMs, the all-gathers of Y and of the
 * per-row nonzero counts, and the compaction; bsm_mcsr_sync waits. */
int bsm_mcsr_step(bsm_mcsr* m, const void* const* x_dev);
int bsm_mcsr_sync(bsm_mcsr* m);
/* HIP-event times of the steps since the last reset on local device i, per
 * step {SpMM rounds (first SpMM start .. last SpMM end on the compute
 * stream), all-gather tail (last SpMM end .. last all-gather end), compaction,
 * whole step}: *n steps, the first min(max, *n) written to ms[4*s ..]. */
int bsm_mcsr_step_times(bsm_mcsr* m, int local, int max, int* n, double* ms);
void bsm_mcsr_reset_times(bsm_mcsr* m);
/* The assembled dense Y (rows x k ROW-major, global row order) and per-row
 * nonzero counts on local device i, copied into caller device buffers
 * (either may be NULL); synchronous. */
int bsm_mcsr_copy_y(const bsm_mcsr* m, int local, void* y, int32_t* row_nnz);
/* The last step's output Csr as a new handle on the local device that
 * compacts it (the first local device, or the output rank's: below). */
int bsm_mcsr_output(const bsm_mcsr* m, bsm_csr** out);
/* Which global rank compacts the gathered Y into the output Csr: -1 (the
 * default) every process (its first local device), r >= 0 only rank r. The
 * other ranks then allocate no output buffers (rows x k x (4 + sizeof(T)) B,
 * 3.84 GB per rank at C4) and skip the compaction; bsm_mcsr_output there
 * returns BSM_ERR_INVALID. Drops a prepared schedule's buffers (call before
 * bsm_mcsr_prepare). Reference: Csr::mul_dense returns one Csr to its one
 * caller (src/sparse.rs:426-446); the row split is this build's. */
int bsm_mcsr_set_output_rank(bsm_mcsr* m, int rank);
/* The compaction of the gathered Y into the output Csr (asynchronous, on the
 * compute stream; bsm_mcsr_step does it itself on a context with a
 * communicator). For an external context, after the slot exchange. */
int bsm_mcsr_compact(bsm_mcsr* m);
/* Slots [first, first + n) of the gathered Y (each piece_rows x k values,
 * ROW-major) and of its per-row nonzero counts (piece_rows int32 each) on local
 * device `local`, to / from caller buffers, host or device (either may be
 * NULL); synchronous. Slot c*world + r holds round c of rank r. */
int bsm_mcsr_slot_read(const bsm_mcsr* m, int local, uint32_t first, uint32_t n, void* y, int32_t* row_nnz);
int bsm_mcsr_slot_write(bsm_mcsr* m, int local, uint32_t first, uint32_t n, const void* y, const int32_t* row_nnz);
void bsm_mcsr_free(bsm_mcsr* m);

#ifdef __cplusplus
}
#endif

#endif /* BSM_H */
