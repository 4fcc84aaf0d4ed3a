// bsm_internal.hpp -- shared internals of libbsm_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/bsm.h"

namespace bsm {

// ---------------------------------------------------------------------------
// errors: thread-local message + status codes
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);
const char* last_error();
// stage timer of the solver (bsm_stage_times): reset, then mark the end of each stage
void stage_reset(hipStream_t s);
void stage_mark(const char* name, hipStream_t s);

#define BSM_HIP_TRY(expr)                                                                   \
    do {                                                                                    \
        hipError_t bsm_e_ = (expr);                                                         \
        if (bsm_e_ != hipSuccess) {                                                         \
            ::bsm::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(bsm_e_),     \
                             __FILE__, __LINE__);                                           \
            return bsm_e_ == hipErrorOutOfMemory ? BSM_ERR_OOM : BSM_ERR_HIP;               \
        }                                                                                   \
    } while (0)

#define BSM_TRY(expr)                 \
    do {                              \
        int bsm_rc_ = (expr);         \
        if (bsm_rc_ != BSM_OK) return bsm_rc_; \
    } while (0)

#define BSM_REQUIRE(cond, code, ...)           \
    do {                                       \
        if (!(cond)) {                         \
            ::bsm::set_error(__VA_ARGS__);     \
            return (code);                     \
        }                                      \
    } while (0)

// ---------------------------------------------------------------------------
// arithmetic with the reference's semantics: IEEE, no contraction, integers
// wrap (Cargo.toml:18). Signed integers are computed in the same-width
// unsigned type so device code never hits C++ signed-overflow UB.
// ---------------------------------------------------------------------------
template <typename T> struct Arith;
template <> struct Arith<double> {
    __device__ __forceinline__ static double add(double a, double b) { return __dadd_rn(a, b); }
    __device__ __forceinline__ static double sub(double a, double b) { return __dsub_rn(a, b); }
    __device__ __forceinline__ static double mul(double a, double b) { return __dmul_rn(a, b); }
    __device__ __forceinline__ static bool nz(double v) { return !(v == 0.0); }
    __device__ __forceinline__ static double zero() { return 0.0; }
    __device__ __forceinline__ static double neg_zero() { return -0.0; }
};
template <> struct Arith<float> {
    __device__ __forceinline__ static float add(float a, float b) { return __fadd_rn(a, b); }
    __device__ __forceinline__ static float sub(float a, float b) { return __fsub_rn(a, b); }
    __device__ __forceinline__ static float mul(float a, float b) { return __fmul_rn(a, b); }
    __device__ __forceinline__ static bool nz(float v) { return !(v == 0.0f); }
    __device__ __forceinline__ static float zero() { return 0.0f; }
    __device__ __forceinline__ static float neg_zero() { return -0.0f; }
};
template <typename T, typename U> struct ArithInt {
    __device__ __forceinline__ static T add(T a, T b) { return (T)((U)a + (U)b); }
    __device__ __forceinline__ static T sub(T a, T b) { return (T)((U)a - (U)b); }
    __device__ __forceinline__ static T mul(T a, T b) { return (T)((U)a * (U)b); }
    __device__ __forceinline__ static bool nz(T v) { return v != 0; }
    __device__ __forceinline__ static T zero() { return 0; }
    __device__ __forceinline__ static T neg_zero() { return 0; }
};
template <> struct Arith<int32_t> : ArithInt<int32_t, uint32_t> {};
template <> struct Arith<uint32_t> : ArithInt<uint32_t, uint32_t> {};
template <> struct Arith<int64_t> : ArithInt<int64_t, uint64_t> {};
template <> struct Arith<uint64_t> : ArithInt<uint64_t, uint64_t> {};

template <typename T> struct IsFloat { static constexpr bool value = false; };
template <> struct IsFloat<double> { static constexpr bool value = true; };
template <> struct IsFloat<float> { static constexpr bool value = true; };

inline size_t dtype_size(int dt) {
    switch (dt) {
        case BSM_F64: case BSM_I64: case BSM_U64: return 8;
        case BSM_F32: case BSM_I32: case BSM_U32: return 4;
        default: return 0;
    }
}

// Invoke F.template operator()<T>() for the runtime dtype.
template <typename F> int dispatch_dtype(int dt, F&& f) {
    switch (dt) {
        case BSM_F64: return f.template operator()<double>();
        case BSM_F32: return f.template operator()<float>();
        case BSM_I32: return f.template operator()<int32_t>();
        case BSM_U32: return f.template operator()<uint32_t>();
        case BSM_I64: return f.template operator()<int64_t>();
        case BSM_U64: return f.template operator()<uint64_t>();
        default: set_error("unknown dtype %d", dt); return BSM_ERR_INVALID;
    }
}

// ---------------------------------------------------------------------------
// device context: one non-blocking stream per device, created lazily.
// ---------------------------------------------------------------------------
int current_device(int* dev);
int ctx_stream(hipStream_t* s);  // stream of the calling thread's device
// Small device -> host read through a pinned bounce buffer, synchronous on s
// (a pageable hipMemcpyAsync costs ~19 us; this is a few).
hipError_t read_dev(void* host, const void* dev, size_t bytes, hipStream_t s);

// Per-thread cache of device temporaries (tmp_get / tmp_put): a hipFree
// waits for the whole device, and a call such as add_sparse makes ~25 of
// them (1.3-2 ms per call at the reference bench's e = 300k,
// profiles/r03_u_*). A cached block is only handed out again to the same
// thread for the same device and stream, so stream order separates its uses
// (the device is part of the key: the null stream names a different queue on
// every device). Every block is a plain hipMalloc allocation.
void* tmp_get(size_t n, int device, hipStream_t s, size_t* cap);
void tmp_put(void* p, size_t cap, int device, hipStream_t s);

// RAII device buffer for host-path temporaries. alloc(n) is hipMalloc /
// hipFree; alloc(n, s) takes the block from the calling thread's cache for
// stream s and gives it back there, for the many small temporaries of a call.
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t st = nullptr;
    int dev = -1;
    size_t cap = 0;  // > 0: a cached temporary of this capacity
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { reset(); }
    void reset() {
        if (p) {
            if (cap) tmp_put(p, cap, dev, st);
            else (void)hipFree(p);
        }
        p = nullptr;
        bytes = 0;
        cap = 0;
    }
    int alloc(size_t n, hipStream_t s) {
        reset();
        if (n == 0) n = 16;
        if (hipGetDevice(&dev) != hipSuccess) {
            set_error("device temporary: no current device");
            return BSM_ERR_HIP;
        }
        p = tmp_get(n, dev, s, &cap);
        if (!p) {
            cap = 0;
            set_error("device temporary of %zu bytes: out of memory", n);
            return BSM_ERR_OOM;
        }
        bytes = n;
        st = s;
        return BSM_OK;
    }
    int alloc(size_t n) {
        reset();
        if (n == 0) n = 16;
        hipError_t e = hipMalloc(&p, n);
        if (e != hipSuccess) {
            p = nullptr;
            set_error("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? BSM_ERR_OOM : BSM_ERR_HIP;
        }
        bytes = n;
        return BSM_OK;
    }
    // The caller takes the block and frees it with hipFree. A cached
    // temporary is a hipMalloc block too: it simply leaves the cache's care.
    void* release() {
        void* q = p;
        p = nullptr;
        bytes = 0;
        cap = 0;
        return q;
    }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

}  // namespace bsm

// Row-block x column-panel copy of a matrix (kernels_tiled.hip).
struct bsm_tiled {
    int device = 0;
    int dtype = BSM_F64;         // BSM_F64 or BSM_F32 (the value stream's type)
    uint64_t k = 32;             // right-hand columns the copy serves (32 or 1)
    uint32_t overread = 4;       // chunks of dummy padding past the last task
    uint32_t stage = 4;          // k = 1: chunks per pipeline stage
    uint64_t rows = 0, n_cols = 0, nnz = 0;
    uint32_t nw = 0, rpw = 0, nb = 0, rw = 0, pshift = 0;
    uint64_t chunks = 0;         // total, without the over-read padding
    int64_t* offs = nullptr;     // nw*nb + 1 chunk offsets
    void* meta = nullptr;        // (chunks + overread) * 64 meta words (col << 8 | row, or col << 11 | row at k = 1)
    uint32_t meta_bytes = 4;     // 8: k = 32 on 2^24 columns or more
    void* val = nullptr;         // (chunks + overread) * 64 values of dtype
    unsigned* bar = nullptr;     // batch arrival counters of the SpMM (one launch at a time per copy)
};

// Device-resident finalised Csr<T>.
struct bsm_csr {
    int dtype = BSM_F64;
    int device = 0;
    uint64_t rows = 0, cols = 0, nnz = 0;
    int64_t* row_ptr = nullptr;  // rows+1
    int32_t* col = nullptr;      // nnz
    void* vals = nullptr;        // nnz * sizeof(T)
    // lazily computed analysis (see bsm_analyse)
    // analysis (csr_analyse) is cached on the handle: computed when the handle
    // is made from host data, lazily for device-built results (add / sub /
    // mul_sparse) the first time a kernel choice needs it
    mutable bool analysed = false;
    mutable bool rows_sorted = true;  // col non-decreasing inside every row
    mutable uint64_t max_row_len = 0;
    // cached column-panel plan of mul_dense (spmm_plan), keyed by panel width;
    // plan_mu serialises its (re)build and use across threads sharing the handle
    mutable std::mutex plan_mu;
    mutable int32_t* plan_seg = nullptr;
    mutable uint64_t plan_cols = 0;
    mutable bool plan_usable = false;
    // cached row-block x column-panel copy (kernels_tiled.hip), same mutex
    mutable bsm_tiled* tiled = nullptr;
    mutable bool tiled_tried = false;
    // solve(order="nd")'s plan (kernels_nd.hip): the pattern's ordering, tree
    // and device index arrays, built on first use (the pattern is immutable),
    // same mutex; released with the handle
    mutable std::shared_ptr<void> nd_plan;
    // row_ptr / col / vals from the result cache (csr_alloc): their block
    // capacities, 0 = plain hipMalloc (bsm_csr_free hipFrees those)
    size_t cache_cap[3] = {0, 0, 0};
    // small mul_dense results: a host copy written by the same kernel as the
    // device arrays (row_ptr int64 [rows + 1], cols int32 [nnz], values
    // [nnz]); bsm_csr_download serves it without touching the device. The
    // device arrays never change after creation, so it cannot go stale.
    std::unique_ptr<char[]> host_copy;
};


namespace bsm {
// Host-side phase times of a schedule build (bsm_mcsr_prepare's plan_ms).
struct PlanTimes {
    double total_ms = 0, count_ms = 0, scan_ms = 0, alloc_ms = 0, write_ms = 0, panel_ms = 0, buffers_ms = 0;
};
inline std::chrono::steady_clock::time_point host_now() { return std::chrono::steady_clock::now(); }
inline double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int csr_alloc(bsm_csr** out, int dtype, uint64_t rows, uint64_t cols, uint64_t nnz);
int csr_analyse(const bsm_csr* m, hipStream_t s);
// mul_dense's schedule (capi.hip): build once per handle and k (synchronous;
// schedule 0 auto, 1 the tiled copy whenever possible, 2 never), then launch.
// The caller holds a->plan_mu for both.
int spmm_prepare_locked(const bsm_csr* a, uint64_t k, int schedule, uint64_t reserve, hipStream_t s,
                        PlanTimes* pt);
int spmm_launch_locked(const bsm_csr* a, uint64_t k, bool allow_tiled, const void* x, void* y, int32_t* nz,
                       hipStream_t s);
// pinned host staging / per-thread device arena (capi.hip)
void* pinned(size_t bytes);
// host columns (Dense::get_col) -> a device ROW-major n x k array in `out`
// (synchronous) (capi.hip)
int upload_dense_cols(int dtype, uint64_t n, uint64_t k, const void* const* cols, DBuf& out, hipStream_t s);
// staged pinned pipelines (transfer.hip); all synchronous
int h2d_staged(void* dst, const void* src, size_t bytes, hipStream_t s);
int d2h_staged(void* dst, const void* src, size_t bytes, hipStream_t s);
int h2d_cols_narrow(int32_t* dst, const uint64_t* src, uint64_t n, uint64_t cols, uint64_t* bad, hipStream_t s);
int h2d_row_ptr(int64_t* dst, const uint64_t* src, uint64_t n, uint64_t base, hipStream_t s);
bool host_registered(const void* p);
int d2h_csr_direct(const int64_t* rp, const int32_t* col, const void* vals, uint64_t rows, uint64_t nnz, size_t es,
                   uint64_t* row_ptr, uint64_t* col_idx, void* vals_out, hipStream_t s);
int d2h_cols_widen(uint64_t* dst, const int32_t* src, uint64_t n, hipStream_t s);

// kernels (kernels_*.hip), all async on stream s
uint64_t scan_workspace_bytes(uint64_t n);
int exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, uint64_t n, void* ws,
                              uint64_t ws_bytes, hipStream_t s);  // out has n+1 entries
int spmm_dispatch(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* rp,
                  const int32_t* col, const void* vals, uint64_t k, const void* x, void* y,
                  int32_t* row_nnz, bool neg_zero_init, hipStream_t s,
                  uint64_t max_row_len = UINT64_MAX);  // the longest row, when known (kernel choice)
// nnz-balanced integer SpMM for skewed rows (zeroes y; row_nnz may be null)
bool spmm_wants_split(int dtype, uint64_t k, uint64_t max_row_len);
int spmm_split_dispatch(int dtype, uint64_t rows, uint64_t nnz, const int64_t* rp, const int32_t* col,
                        const void* vals, uint64_t k, const void* x, void* y, int32_t* row_nnz, hipStream_t s);
// device construction from an insert sequence (kernels_build.hip)
int csr_from_inserts_device(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                            const uint64_t* col, const void* vals, bsm_csr** out, hipStream_t s);
// sparse x sparse (kernels_sparse.hip); synchronous
int sparse_addsub_dispatch(const bsm_csr* a, const bsm_csr* b, bool sub, bsm_csr** out, hipStream_t s);
int sparse_mul_dispatch(const bsm_csr* a, const bsm_csr* b, bsm_csr** out, hipStream_t s);
int csr_from_coo_device(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                        const uint64_t* col, const void* vals, bsm_csr** out, hipStream_t s);
int gen_insert_stream(int dtype, uint64_t seed, uint64_t i0, uint64_t n, uint64_t rows, uint64_t cols,
                      uint64_t vmod, uint64_t* row, uint64_t* col, void* vals, hipStream_t s);
uint64_t spmm_panel_cols(int dtype, uint64_t n_cols, uint64_t k);  // 0 = single pass
uint64_t spmm_plan_bytes(uint64_t rows, uint64_t n_cols, uint64_t panel_cols);
int spmm_plan(uint64_t rows, uint64_t n_cols, const int64_t* rp, const int32_t* col,
              uint64_t panel_cols, int32_t* seg, int* usable, hipStream_t s);  // synchronous
int spmm_panelled(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* rp,
                  const int32_t* col, const void* vals, uint64_t k, const void* x, void* y,
                  int32_t* row_nnz, uint64_t panel_cols, const int32_t* seg, hipStream_t s);
// row-block x column-panel schedule (kernels_tiled.hip)
bool tiled_wanted(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, uint64_t k, uint64_t max_row_len);
// synchronous; the copy must leave `reserve` device bytes free; pt (may be
// null) receives host times of its phases
int tiled_create(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* rp, const int32_t* col,
                 const void* vals, uint64_t k, int flags, bsm_tiled** out, hipStream_t s, uint64_t reserve = 0,
                 PlanTimes* pt = nullptr);
int tiled_spmm(const bsm_tiled* t, const void* x, void* y, int32_t* row_nnz, bool neg_init, hipStream_t s);
void tiled_destroy(bsm_tiled* t);
int compact_dispatch(int dtype, uint64_t rows, uint64_t k, const void* y, const int64_t* out_rp,
                     int32_t* out_col, void* out_vals, hipStream_t s);
// Small results (rows <= SMALL_OUT_ROWS, rows x k <= SMALL_OUT_CAP): the
// row-count scan and the compaction in one workgroup, which also writes the
// result into `host` (page-locked: row_ptr int64 [rows + 1], then cols int32
// [cap] at small_col_bytes alignment, then values [cap]); kernels_spmm.hip.
constexpr uint64_t SMALL_OUT_ROWS = 8192;
constexpr uint64_t SMALL_OUT_CAP = 131072;
inline size_t small_col_bytes(uint64_t cap) { return (cap * sizeof(int32_t) + 15) / 16 * 16; }
int compact_small_dispatch(int dtype, uint64_t rows, uint64_t k, const int32_t* nz, const void* y, int64_t* out_rp,
                           int32_t* out_col, void* out_vals, void* host, uint64_t cap, hipStream_t s);
int pack_cols_to_rowmajor(int dtype, uint64_t n, uint64_t k, const void* colmajor, void* rowmajor,
                          hipStream_t s);
int unpack_rowmajor_to_cols(int dtype, uint64_t n, uint64_t k, const void* rowmajor,
                            void* colmajor, hipStream_t s);
int transpose_dispatch(const bsm_csr* a, bsm_csr** out, hipStream_t s);
int analyse_dispatch(const int64_t* rp, const int32_t* col, uint64_t rows, uint64_t cols,
                     uint64_t* d_out3, hipStream_t s);
int gen_row_ptr(uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols, int kind,
                uint32_t a, uint32_t b, int64_t* rp, void* ws, uint64_t ws_bytes, hipStream_t s);
int gen_entries(int dtype, uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols,
                int value_kind, const int64_t* rp, int32_t* col, void* vals, hipStream_t s);
int gen_dense(int dtype, uint64_t seed, uint64_t row0, uint64_t n, uint64_t k, int value_kind,
              void* x, hipStream_t s);
int solve_dispatch_cholesky(const bsm_csr* a, bsm_csr** out, hipStream_t s);
int solve_dispatch_trsv(const bsm_csr* m, bool lower, uint64_t k, uint64_t n, const void* b_dev,
                        void* x_dev, hipStream_t s);
int solve_dispatch_full(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev,
                        hipStream_t s);
int solve_dispatch_blocked(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev,
                           hipStream_t s);
int solve_dispatch_nd(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev, hipStream_t s);
}  // namespace bsm
