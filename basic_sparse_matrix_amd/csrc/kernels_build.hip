// kernels_build.hip -- device construction of a finalised Csr from a
// sequence of Csr::insert(value, row, col) calls.
//
// The reference builds matrices one insert at a time (sparse.rs:222-250)
// and then calls finalise (sparse.rs:206-220):
//   * insert skips value == T::default() (for floats both zeros; NaN is kept);
//   * insert_unchecked appends value and col in call order, and extends
//     row_index only when `row` exceeds the rows recorded so far: an entry
//     belongs to the running maximum of the rows inserted before it
//     (inclusive), never to an earlier row;
//   * finalise panics ("big eek") when rows < row_index.len(), i.e. when some
//     kept entry named a row >= rows, and pads row_index with nnz.
// On the device that is: keep-flags, an exclusive scan (positions), a
// scatter of the kept entries, an inclusive max-scan of their rows (the
// running maximum), and row_ptr[r] = the first kept entry whose running row
// is >= r (a binary search per row), which equals what the incremental
// row_index pushes produce, including the repeated entries of skipped rows.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "bsm_internal.hpp"
#include "bsm_synth.h"

namespace bsm {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void insert_keep_flags(uint64_t n, const T* __restrict__ v,
                                                         int32_t* __restrict__ flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = Arith<T>::nz(v[i]) ? 1 : 0;
}

// kept entry i -> position pos[i]; err[0] |= 1 when a kept column is >= cols
template <typename T>
__global__ __launch_bounds__(256) void insert_scatter(uint64_t n, uint64_t cols, const uint64_t* __restrict__ row,
                                                      const uint64_t* __restrict__ col, const T* __restrict__ v,
                                                      const int64_t* __restrict__ pos, int64_t* __restrict__ erow,
                                                      int32_t* __restrict__ ocol, T* __restrict__ ov,
                                                      unsigned* __restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t p = pos[i];
    if (pos[i + 1] == p) return;  // skipped by insert
    const uint64_t c = col[i];
    if (c >= cols) atomicOr(err, 1u);
    const uint64_t r = row[i];
    erow[p] = r > (uint64_t)INT64_MAX ? INT64_MAX : (int64_t)r;
    ocol[p] = (int32_t)(c < cols ? c : 0);
    ov[p] = v[i];
}

// row_ptr[r] = first p with erow[p] >= r (erow non-decreasing), r in [0, rows]
__global__ __launch_bounds__(256) void insert_row_ptr(uint64_t rows, int64_t nnz, const int64_t* __restrict__ erow,
                                                      int64_t* __restrict__ rp) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > rows) return;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (erow[mid] < (int64_t)r) lo = mid + 1; else hi = mid;
    }
    rp[r] = lo;
}

template <typename T>
__global__ __launch_bounds__(256) void insert_stream_gen(uint64_t seed, uint64_t i0, uint64_t n, uint64_t rows,
                                                         uint64_t cols, uint64_t vmod, uint64_t* __restrict__ row,
                                                         uint64_t* __restrict__ col, T* __restrict__ v) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    row[i] = bsm_stream_draw(seed, i0 + i, 0) % rows;
    col[i] = bsm_stream_draw(seed, i0 + i, 1) % cols;
    v[i] = (T)(bsm_stream_draw(seed, i0 + i, 2) % vmod);
}

unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

// From<COO>: sort key (row << cb) | col and entry index; err |= 1 outside dims
__global__ __launch_bounds__(256) void coo_keys(uint64_t n, uint64_t rows, uint64_t cols, unsigned cb,
                                                const uint64_t* __restrict__ row, const uint64_t* __restrict__ col,
                                                uint64_t* __restrict__ key, uint64_t* __restrict__ idx,
                                                unsigned* __restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = row[i], c = col[i];
    if (r >= rows || c >= cols) atomicOr(err, 1u);
    key[i] = ((r < rows ? r : 0) << cb) | (c < cols ? c : 0);
    idx[i] = i;
}

template <typename T>
__global__ __launch_bounds__(256) void coo_gather(uint64_t n, const uint64_t* __restrict__ perm,
                                                  const uint64_t* __restrict__ row, const uint64_t* __restrict__ col,
                                                  const T* __restrict__ v, uint64_t* __restrict__ srow,
                                                  uint64_t* __restrict__ scol, T* __restrict__ sv) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t j = perm[i];
    srow[i] = row[j];
    scol[i] = col[j];
    sv[i] = v[j];
}

unsigned bits_for(uint64_t x) {  // bits to hold values < x
    unsigned b = 0;
    while (b < 64 && (x - 1) >> b) ++b;
    return b;
}

}  // namespace

int gen_insert_stream(int dtype, uint64_t seed, uint64_t i0, uint64_t n, uint64_t rows, uint64_t cols,
                      uint64_t vmod, uint64_t* row, uint64_t* col, void* vals, hipStream_t s) {
    BSM_REQUIRE(rows && cols && vmod, BSM_ERR_INVALID, "insert stream: rows, cols and vmod must be > 0");
    BSM_REQUIRE(n < (1ull << 40), BSM_ERR_UNSUPPORTED, "insert stream too long");
    if (n == 0) return BSM_OK;
    return dispatch_dtype(dtype, [&]<typename T>() -> int {
        insert_stream_gen<T><<<grid_of(n), 256, 0, s>>>(seed, i0, n, rows, cols, vmod, row, col,
                                                        static_cast<T*>(vals));
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
}

int csr_from_inserts_device(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                            const uint64_t* col, const void* vals, bsm_csr** out, hipStream_t s) {
    BSM_REQUIRE(out && (n == 0 || (row && col && vals)), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(cols <= (uint64_t)INT32_MAX, BSM_ERR_UNSUPPORTED, "cols must be < 2^31 on the device");
    BSM_REQUIRE(n < (1ull << 40), BSM_ERR_UNSUPPORTED, "too many inserts");
    const size_t es = dtype_size(dtype);
    BSM_REQUIRE(es, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    // 1. keep flags and their exclusive scan: positions of the kept entries
    DBuf flag, pos, ws;
    BSM_TRY(flag.alloc((n ? n : 1) * sizeof(int32_t)));
    BSM_TRY(pos.alloc((n + 1) * sizeof(int64_t)));
    BSM_TRY(ws.alloc(scan_workspace_bytes(n ? n : 1)));
    int rc = dispatch_dtype(dtype, [&]<typename T>() -> int {
        if (n) insert_keep_flags<T><<<grid_of(n), 256, 0, s>>>(n, static_cast<const T*>(vals), flag.as<int32_t>());
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
    BSM_TRY(rc);
    BSM_TRY(exclusive_scan_i32_to_i64(flag.as<int32_t>(), pos.as<int64_t>(), n, ws.p, ws.bytes, s));
    int64_t nnz = 0;
    BSM_HIP_TRY(read_dev(&nnz, pos.as<int64_t>() + n, sizeof(int64_t), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    // 2. scatter the kept entries, then the running maximum of their rows
    bsm_csr* m = nullptr;
    BSM_TRY(csr_alloc(&m, dtype, rows, cols, (uint64_t)nnz));
    auto fail = [&](int code) {
        bsm_csr_free(m);
        return code;
    };
    DBuf erow, err;
    if ((rc = erow.alloc((nnz ? nnz : 1) * sizeof(int64_t))) != BSM_OK) return fail(rc);
    if ((rc = err.alloc(sizeof(unsigned))) != BSM_OK) return fail(rc);
    if (hipMemsetAsync(err.p, 0, sizeof(unsigned), s) != hipSuccess) return fail(BSM_ERR_HIP);
    rc = dispatch_dtype(dtype, [&]<typename T>() -> int {
        if (n)
            insert_scatter<T><<<grid_of(n), 256, 0, s>>>(n, cols, row, col, static_cast<const T*>(vals),
                                                         pos.as<int64_t>(), erow.as<int64_t>(), m->col,
                                                         static_cast<T*>(m->vals), err.as<unsigned>());
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
    if (rc != BSM_OK) return fail(rc);
    if (nnz) {
        size_t tmp_bytes = 0;
        int64_t* er = erow.as<int64_t>();
        if (rocprim::inclusive_scan(nullptr, tmp_bytes, er, er, (size_t)nnz, rocprim::maximum<int64_t>(), s) !=
            hipSuccess)
            return fail(BSM_ERR_HIP);
        DBuf tmp;
        if ((rc = tmp.alloc(tmp_bytes ? tmp_bytes : 1)) != BSM_OK) return fail(rc);
        if (rocprim::inclusive_scan(tmp.p, tmp_bytes, er, er, (size_t)nnz, rocprim::maximum<int64_t>(), s) !=
            hipSuccess) {
            set_error("rocprim::inclusive_scan failed");
            return fail(BSM_ERR_HIP);
        }
        // the scan reads tmp asynchronously: keep it alive until it is done
        if (hipStreamSynchronize(s) != hipSuccess) return fail(BSM_ERR_HIP);
    }
    // 3. checks: finalise's "big eek" (a kept row >= rows) and column bounds
    int64_t last_row = -1;
    unsigned bad_col = 0;
    if (nnz && read_dev(&last_row, erow.as<int64_t>() + nnz - 1, sizeof(int64_t), s) != hipSuccess)
        return fail(BSM_ERR_HIP);
    if (read_dev(&bad_col, err.p, sizeof(unsigned), s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return fail(BSM_ERR_HIP);
    if (nnz && (uint64_t)last_row >= rows) {
        set_error("big eek: finalise with row_index longer than rows (row %lld >= rows %llu), sparse.rs:210",
                  (long long)last_row, (unsigned long long)rows);
        return fail(BSM_ERR_PANIC);
    }
    if (bad_col) {
        set_error("column index >= cols %llu (the device Csr needs in-bounds columns)", (unsigned long long)cols);
        return fail(BSM_ERR_PANIC);
    }
    // 4. row_ptr by binary search over the running rows
    insert_row_ptr<<<grid_of(rows + 1), 256, 0, s>>>(rows, nnz, erow.as<int64_t>(), m->row_ptr);
    if (hipGetLastError() != hipSuccess) return fail(BSM_ERR_HIP);
    if ((rc = csr_analyse(m, s)) != BSM_OK) return fail(rc);  // synchronises
    *out = m;
    return BSM_OK;
}

// From<COO<T>> for Csr<T> (sparse.rs:56-66): a STABLE sort by (row, col)
// (Rust's sort_by is stable; rocPRIM's LSD radix sort is too), then the
// insert sequence of csr_from_inserts_device (zero skip; sorted rows make
// the running maximum the row itself). Entries outside dims are COO::insert's
// Err(OutOfBounds) (sparse.rs:45-53), which the caller normally reports
// before ever building the COO.
int csr_from_coo_device(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                        const uint64_t* col, const void* vals, bsm_csr** out, hipStream_t s) {
    BSM_REQUIRE(out && (n == 0 || (row && col && vals)), BSM_ERR_INVALID, "null argument");
    const size_t es = dtype_size(dtype);
    BSM_REQUIRE(es, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    if (n == 0) return csr_from_inserts_device(dtype, rows, cols, 0, row, col, vals, out, s);
    const unsigned cb = bits_for(cols), rb = bits_for(rows);
    BSM_REQUIRE(cb + rb <= 64, BSM_ERR_UNSUPPORTED, "COO: rows x cols too large for a 64-bit sort key");
    DBuf key, key_s, idx, idx_s, err, srow, scol, sv, tmp;
    BSM_TRY(key.alloc(n * sizeof(uint64_t)));
    BSM_TRY(key_s.alloc(n * sizeof(uint64_t)));
    BSM_TRY(idx.alloc(n * sizeof(uint64_t)));
    BSM_TRY(idx_s.alloc(n * sizeof(uint64_t)));
    BSM_TRY(err.alloc(sizeof(unsigned)));
    BSM_HIP_TRY(hipMemsetAsync(err.p, 0, sizeof(unsigned), s));
    coo_keys<<<grid_of(n), 256, 0, s>>>(n, rows, cols, cb, row, col, key.as<uint64_t>(), idx.as<uint64_t>(),
                                        err.as<unsigned>());
    BSM_HIP_TRY(hipGetLastError());
    unsigned bad = 0;
    BSM_HIP_TRY(read_dev(&bad, err.p, sizeof(unsigned), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    if (bad) {
        set_error("COO entry outside dims %llu x %llu (MatErr::OutOfBounds, sparse.rs:47-49)",
                  (unsigned long long)rows, (unsigned long long)cols);
        return BSM_ERR_OUT_OF_BOUNDS;
    }
    const unsigned end_bit = cb + rb > 0 ? cb + rb : 1;
    size_t tmp_bytes = 0;
    BSM_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key.as<uint64_t>(), key_s.as<uint64_t>(),
                                          idx.as<uint64_t>(), idx_s.as<uint64_t>(), (size_t)n, 0u, end_bit, s));
    BSM_TRY(tmp.alloc(tmp_bytes ? tmp_bytes : 1));
    BSM_HIP_TRY(rocprim::radix_sort_pairs(tmp.p, tmp_bytes, key.as<uint64_t>(), key_s.as<uint64_t>(),
                                          idx.as<uint64_t>(), idx_s.as<uint64_t>(), (size_t)n, 0u, end_bit, s));
    BSM_TRY(srow.alloc(n * sizeof(uint64_t)));
    BSM_TRY(scol.alloc(n * sizeof(uint64_t)));
    BSM_TRY(sv.alloc(n * es));
    BSM_TRY(dispatch_dtype(dtype, [&]<typename T>() -> int {
        coo_gather<T><<<grid_of(n), 256, 0, s>>>(n, idx_s.as<uint64_t>(), row, col, static_cast<const T*>(vals),
                                                 srow.as<uint64_t>(), scol.as<uint64_t>(), sv.as<T>());
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    }));
    // csr_from_inserts_device synchronises before returning, so the sorted
    // temporaries stay alive for as long as its kernels read them
    return csr_from_inserts_device(dtype, rows, cols, n, srow.as<uint64_t>(), scol.as<uint64_t>(), sv.p, out, s);
}

}  // namespace bsm
