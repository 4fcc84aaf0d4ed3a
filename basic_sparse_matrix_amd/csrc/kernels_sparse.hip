// kernels_sparse.hip -- sparse x sparse operations of the reference
// (SURVEY.md §8f-4): Csr::add_sparse / sub_sparse (sparse.rs:484-599) and
// Csr::mul_sparse (sparse.rs:601-635), bit-exact for every input, including
// rows with unsorted or repeated columns (the reference's bench builds such
// rows: random insert order).
//
// add / sub: the reference merges row r of both operands with two pointers
// over their entries in STORAGE order (the smaller column goes out first, an
// equal column goes out once as the sum / difference, for sub an rhs-only
// entry is T::default() - v), each output through the zero-skipping insert.
// One thread per row runs that merge twice: once to count the kept outputs
// (then an exclusive scan gives row_ptr), once to write them.
//
// mul: the reference visits every (row, col) pair of the result and merges
// the self row (storage order) with row `col` of rhs.transpose(); val starts
// at T::default(), gains the product of each equal-column step in merge
// order, and is inserted when nonzero. On the device:
//   1. rhs_t = transpose(rhs) (the stable device transpose);
//   2. candidates: every (i, j) that can have an equal-column step pairs an
//      entry (i, k) of self with an entry (k, j) of rhs. Expand those
//      (balanced: one thread per expanded slot, binary search on the scan of
//      the per-entry counts), radix-sort the keys (i, j) and keep the unique
//      ones -- ascending i then j, the reference's output order;
//   3. per candidate, the literal merge (so duplicate or unsorted columns
//      skip exactly the steps the reference skips);
//   4. keep val != default: a flag scan, a scatter, row_ptr by binary search.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>

#include "bsm_internal.hpp"

namespace bsm {
namespace {

unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

unsigned bits_for(uint64_t x) {  // bits to hold values < x
    unsigned b = 0;
    while (b < 64 && (x - 1) >> b) ++b;
    return b;
}

// ---- add / sub -------------------------------------------------------------
// The merge of row r; emit(col, value) for every output the reference
// inserts (zero results are dropped by the caller, like insert).
template <typename T, bool SUB, typename F>
__device__ __forceinline__ void merge_row(int64_t r, const int64_t* __restrict__ arp, const int32_t* __restrict__ acol,
                                          const T* __restrict__ av, const int64_t* __restrict__ brp,
                                          const int32_t* __restrict__ bcol, const T* __restrict__ bv, F&& emit) {
    using A = Arith<T>;
    int64_t ia = arp[r], ib = brp[r];
    const int64_t ea = arp[r + 1], eb = brp[r + 1];
    while (ia < ea || ib < eb) {
        if (ia < ea && ib < eb) {
            const int32_t ca = acol[ia], cb = bcol[ib];
            if (ca > cb) {
                emit(cb, SUB ? A::sub(A::zero(), bv[ib]) : bv[ib]);
                ++ib;
            } else if (ca < cb) {
                emit(ca, av[ia]);
                ++ia;
            } else {
                emit(ca, SUB ? A::sub(av[ia], bv[ib]) : A::add(av[ia], bv[ib]));
                ++ia;
                ++ib;
            }
        } else if (ia < ea) {
            emit(acol[ia], av[ia]);
            ++ia;
        } else {
            emit(bcol[ib], SUB ? A::sub(A::zero(), bv[ib]) : bv[ib]);
            ++ib;
        }
    }
}

template <typename T, bool SUB>
__global__ __launch_bounds__(256) void addsub_count(int64_t rows, const int64_t* __restrict__ arp,
                                                    const int32_t* __restrict__ acol, const T* __restrict__ av,
                                                    const int64_t* __restrict__ brp, const int32_t* __restrict__ bcol,
                                                    const T* __restrict__ bv, int32_t* __restrict__ cnt) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    int32_t n = 0;
    merge_row<T, SUB>(r, arp, acol, av, brp, bcol, bv, [&](int32_t, T v) { n += Arith<T>::nz(v) ? 1 : 0; });
    cnt[r] = n;
}

template <typename T, bool SUB>
__global__ __launch_bounds__(256) void addsub_fill(int64_t rows, const int64_t* __restrict__ arp,
                                                   const int32_t* __restrict__ acol, const T* __restrict__ av,
                                                   const int64_t* __restrict__ brp, const int32_t* __restrict__ bcol,
                                                   const T* __restrict__ bv, const int64_t* __restrict__ orp,
                                                   int32_t* __restrict__ ocol, T* __restrict__ ov) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    int64_t p = orp[r];
    merge_row<T, SUB>(r, arp, acol, av, brp, bcol, bv, [&](int32_t c, T v) {
        if (Arith<T>::nz(v)) {
            ocol[p] = c;
            ov[p] = v;
            ++p;
        }
    });
}

// ---- mul -------------------------------------------------------------------
// expansion count of self entry e = (i, k): the length of rhs row k
__global__ __launch_bounds__(256) void spgemm_count(uint64_t nnz_a, const int32_t* __restrict__ acol,
                                                    uint64_t b_rows, const int64_t* __restrict__ brp,
                                                    int32_t* __restrict__ cnt) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nnz_a) return;
    const uint64_t k = (uint64_t)acol[e];
    cnt[e] = k < b_rows ? (int32_t)(brp[k + 1] - brp[k]) : 0;
}

// last e with off[e] <= p (off: exclusive scan of the counts, n + 1 entries)
__device__ __forceinline__ uint64_t owner_of(const int64_t* __restrict__ off, uint64_t n, int64_t p) {
    uint64_t lo = 0, hi = n;  // off[lo] <= p < off[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] <= p) lo = mid; else hi = mid;
    }
    return lo;
}

// expanded slot p -> key (i << cb) | j
__global__ __launch_bounds__(256) void spgemm_expand(uint64_t total, uint64_t nnz_a, const int64_t* __restrict__ off,
                                                     const int64_t* __restrict__ arp, uint64_t a_rows,
                                                     const int32_t* __restrict__ acol, const int64_t* __restrict__ brp,
                                                     const int32_t* __restrict__ bcol, unsigned cb,
                                                     uint64_t* __restrict__ key) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= total) return;
    const uint64_t e = owner_of(off, nnz_a, (int64_t)p);
    const uint64_t i = owner_of(arp, a_rows, (int64_t)e);  // the self row holding entry e
    const int64_t k = acol[e];
    const int32_t j = bcol[brp[k] + ((int64_t)p - off[e])];
    key[p] = ((uint64_t)i << cb) | (uint64_t)j;
}

// the reference's merge for candidate (i, j); flag = val != default
template <typename T>
__global__ __launch_bounds__(256) void spgemm_merge(uint64_t n_cand, const uint64_t* __restrict__ key, unsigned cb,
                                                    const int64_t* __restrict__ arp, const int32_t* __restrict__ acol,
                                                    const T* __restrict__ av, const int64_t* __restrict__ trp,
                                                    const int32_t* __restrict__ tcol, const T* __restrict__ tv,
                                                    T* __restrict__ val, int32_t* __restrict__ keep) {
    using A = Arith<T>;
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cand) return;
    const uint64_t kk = key[c];
    const uint64_t i = kk >> cb, j = kk & ((1ull << cb) - 1);
    int64_t p = arp[i], q = trp[j];
    const int64_t ep = arp[i + 1], eq = trp[j + 1];
    T v = A::zero();
    while (q != eq && p != ep) {
        const int32_t ca = acol[p], ct = tcol[q];
        if (ca == ct) {
            v = A::add(v, A::mul(av[p], tv[q]));
            ++p;
            ++q;
        } else if (ca > ct) {
            ++q;
        } else {
            ++p;
        }
    }
    val[c] = v;
    keep[c] = A::nz(v) ? 1 : 0;
}

template <typename T>
__global__ __launch_bounds__(256) void spgemm_scatter(uint64_t n_cand, const uint64_t* __restrict__ key, unsigned cb,
                                                      const T* __restrict__ val, const int64_t* __restrict__ pos,
                                                      int64_t* __restrict__ orow, int32_t* __restrict__ ocol,
                                                      T* __restrict__ ov) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cand) return;
    const int64_t p = pos[c];
    if (pos[c + 1] == p) return;
    const uint64_t kk = key[c];
    orow[p] = (int64_t)(kk >> cb);
    ocol[p] = (int32_t)(kk & ((1ull << cb) - 1));
    ov[p] = val[c];
}

// row_ptr[r] = first p with orow[p] >= r, r in [0, rows]
__global__ __launch_bounds__(256) void rows_to_ptr(uint64_t rows, int64_t nnz, const int64_t* __restrict__ orow,
                                                   int64_t* __restrict__ rp) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > rows) return;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (orow[mid] < (int64_t)r) lo = mid + 1; else hi = mid;
    }
    rp[r] = lo;
}

struct CsrGuard {  // frees a half-built output on error paths
    bsm_csr* m = nullptr;
    ~CsrGuard() { if (m) bsm_csr_free(m); }
    bsm_csr* release() { bsm_csr* r = m; m = nullptr; return r; }
};

}  // namespace

int sparse_addsub_dispatch(const bsm_csr* a, const bsm_csr* b, bool sub, bsm_csr** out, hipStream_t s) {
    BSM_REQUIRE(a && b && out, BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->dtype == b->dtype, BSM_ERR_INVALID, "operands have different scalar types");
    BSM_REQUIRE(a->rows == b->rows && a->cols == b->cols, BSM_ERR_DIMENSIONS, "IncorrectDimensions");
    BSM_REQUIRE(a->rows > 0, BSM_ERR_PANIC,
                "%s on a matrix with 0 rows: the reference's row loop never terminates (sparse.rs:%s)",
                sub ? "sub_sparse" : "add_sparse", sub ? "593-596" : "533-537");
    const uint64_t rows = a->rows;
    DBuf cnt, ws;
    CsrGuard g;
    BSM_TRY(cnt.alloc(rows * sizeof(int32_t)));
    BSM_TRY(ws.alloc(scan_workspace_bytes(rows)));
    DBuf orp;
    BSM_TRY(orp.alloc((rows + 1) * sizeof(int64_t)));
    auto run = [&]<typename T>() -> int {
        const T* av = static_cast<const T*>(a->vals);
        const T* bv = static_cast<const T*>(b->vals);
        if (sub)
            addsub_count<T, true><<<grid_of(rows), 256, 0, s>>>((int64_t)rows, a->row_ptr, a->col, av, b->row_ptr,
                                                                 b->col, bv, cnt.as<int32_t>());
        else
            addsub_count<T, false><<<grid_of(rows), 256, 0, s>>>((int64_t)rows, a->row_ptr, a->col, av, b->row_ptr,
                                                                  b->col, bv, cnt.as<int32_t>());
        BSM_HIP_TRY(hipGetLastError());
        BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), orp.as<int64_t>(), rows, ws.p, ws.bytes, s));
        int64_t nnz = 0;
        BSM_HIP_TRY(hipMemcpyAsync(&nnz, orp.as<int64_t>() + rows, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        BSM_TRY(csr_alloc(&g.m, a->dtype, rows, a->cols, (uint64_t)nnz));
        BSM_HIP_TRY(hipMemcpyAsync(g.m->row_ptr, orp.p, (rows + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
        if (sub)
            addsub_fill<T, true><<<grid_of(rows), 256, 0, s>>>((int64_t)rows, a->row_ptr, a->col, av, b->row_ptr,
                                                                b->col, bv, orp.as<int64_t>(), g.m->col,
                                                                static_cast<T*>(g.m->vals));
        else
            addsub_fill<T, false><<<grid_of(rows), 256, 0, s>>>((int64_t)rows, a->row_ptr, a->col, av, b->row_ptr,
                                                                 b->col, bv, orp.as<int64_t>(), g.m->col,
                                                                 static_cast<T*>(g.m->vals));
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    };
    BSM_TRY(dispatch_dtype(a->dtype, run));
    BSM_TRY(csr_analyse(g.m, s));  // synchronises
    *out = g.release();
    return BSM_OK;
}

int sparse_mul_dispatch(const bsm_csr* a, const bsm_csr* b, bsm_csr** out, hipStream_t s) {
    BSM_REQUIRE(a && b && out, BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->dtype == b->dtype, BSM_ERR_INVALID, "operands have different scalar types");
    const uint64_t rows = a->rows, cols = b->cols;
    const unsigned cb = bits_for(cols), rb = bits_for(rows);
    BSM_REQUIRE(cb + rb <= 64 && cb < 64, BSM_ERR_UNSUPPORTED, "mul_sparse: rows x cols too large for 64-bit keys");
    CsrGuard g;
    // 1. rhs^T (stable, like the reference's transpose)
    bsm_csr* bt_raw = nullptr;
    BSM_TRY(transpose_dispatch(b, &bt_raw, s));
    CsrGuard bt;
    bt.m = bt_raw;
    // 2. candidates
    const uint64_t nnz_a = a->nnz;
    DBuf cnt, off, ws;
    BSM_TRY(cnt.alloc((nnz_a ? nnz_a : 1) * sizeof(int32_t)));
    BSM_TRY(off.alloc((nnz_a + 1) * sizeof(int64_t)));
    BSM_TRY(ws.alloc(scan_workspace_bytes(nnz_a ? nnz_a : 1)));
    if (nnz_a) {
        spgemm_count<<<grid_of(nnz_a), 256, 0, s>>>(nnz_a, a->col, b->rows, b->row_ptr, cnt.as<int32_t>());
        BSM_HIP_TRY(hipGetLastError());
    }
    BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), off.as<int64_t>(), nnz_a, ws.p, ws.bytes, s));
    int64_t total = 0;
    BSM_HIP_TRY(hipMemcpyAsync(&total, off.as<int64_t>() + nnz_a, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_REQUIRE(total < (int64_t)UINT32_MAX, BSM_ERR_UNSUPPORTED,
                "mul_sparse: %lld expanded products (limit 2^32)", (long long)total);
    uint64_t n_cand = 0;
    DBuf keys, keys_s, tmp, cand, n_dev;
    if (total > 0) {
        BSM_TRY(keys.alloc(total * sizeof(uint64_t)));
        BSM_TRY(keys_s.alloc(total * sizeof(uint64_t)));
        spgemm_expand<<<grid_of(total), 256, 0, s>>>((uint64_t)total, nnz_a, off.as<int64_t>(), a->row_ptr, rows,
                                                     a->col, b->row_ptr, b->col, cb, keys.as<uint64_t>());
        BSM_HIP_TRY(hipGetLastError());
        const unsigned end_bit = cb + rb > 0 ? cb + rb : 1;
        size_t tb = 0;
        BSM_HIP_TRY(rocprim::radix_sort_keys(nullptr, tb, keys.as<uint64_t>(), keys_s.as<uint64_t>(), (size_t)total,
                                             0u, end_bit, s));
        BSM_TRY(tmp.alloc(tb ? tb : 1));
        BSM_HIP_TRY(rocprim::radix_sort_keys(tmp.p, tb, keys.as<uint64_t>(), keys_s.as<uint64_t>(), (size_t)total,
                                             0u, end_bit, s));
        BSM_TRY(n_dev.alloc(sizeof(uint64_t)));
        // unique into `keys` (free after the sort)
        size_t ub = 0;
        BSM_HIP_TRY(rocprim::unique(nullptr, ub, keys_s.as<uint64_t>(), keys.as<uint64_t>(), n_dev.as<uint64_t>(),
                                    (size_t)total, rocprim::equal_to<uint64_t>(), s));
        DBuf tmp2;
        BSM_TRY(tmp2.alloc(ub ? ub : 1));
        BSM_HIP_TRY(rocprim::unique(tmp2.p, ub, keys_s.as<uint64_t>(), keys.as<uint64_t>(), n_dev.as<uint64_t>(),
                                    (size_t)total, rocprim::equal_to<uint64_t>(), s));
        BSM_HIP_TRY(hipMemcpyAsync(&n_cand, n_dev.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
    }
    // 3. the merge per candidate, 4. keep the nonzero ones
    const size_t es = dtype_size(a->dtype);
    DBuf val, keep, pos, orow;
    BSM_TRY(val.alloc((n_cand ? n_cand : 1) * es));
    BSM_TRY(keep.alloc((n_cand ? n_cand : 1) * sizeof(int32_t)));
    BSM_TRY(pos.alloc((n_cand + 1) * sizeof(int64_t)));
    DBuf ws2;
    BSM_TRY(ws2.alloc(scan_workspace_bytes(n_cand ? n_cand : 1)));
    int64_t nnz = 0;
    auto run = [&]<typename T>() -> int {
        if (n_cand) {
            spgemm_merge<T><<<grid_of(n_cand), 256, 0, s>>>(n_cand, keys.as<uint64_t>(), cb, a->row_ptr, a->col,
                                                            static_cast<const T*>(a->vals), bt.m->row_ptr, bt.m->col,
                                                            static_cast<const T*>(bt.m->vals), val.as<T>(),
                                                            keep.as<int32_t>());
            BSM_HIP_TRY(hipGetLastError());
        }
        BSM_TRY(exclusive_scan_i32_to_i64(keep.as<int32_t>(), pos.as<int64_t>(), n_cand, ws2.p, ws2.bytes, s));
        BSM_HIP_TRY(hipMemcpyAsync(&nnz, pos.as<int64_t>() + n_cand, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        BSM_TRY(csr_alloc(&g.m, a->dtype, rows, cols, (uint64_t)nnz));
        BSM_TRY(orow.alloc((nnz ? nnz : 1) * sizeof(int64_t)));
        if (n_cand) {
            spgemm_scatter<T><<<grid_of(n_cand), 256, 0, s>>>(n_cand, keys.as<uint64_t>(), cb, val.as<T>(),
                                                              pos.as<int64_t>(), orow.as<int64_t>(), g.m->col,
                                                              static_cast<T*>(g.m->vals));
            BSM_HIP_TRY(hipGetLastError());
        }
        rows_to_ptr<<<grid_of(rows + 1), 256, 0, s>>>(rows, nnz, orow.as<int64_t>(), g.m->row_ptr);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    };
    BSM_TRY(dispatch_dtype(a->dtype, run));
    BSM_TRY(csr_analyse(g.m, s));  // synchronises: every temporary above is idle
    *out = g.release();
    return BSM_OK;
}

}  // namespace bsm
