// kernels_transpose.hip -- Csr::transpose (reference: src/sparse.rs:296-318)
// as a stable CSR -> CSC on gfx950.
//
// The reference visits source columns in ascending order and, for each,
// every entry in storage order, appending (val, col, row) to the output with
// insert_unchecked (no zero skip). That is exactly a STABLE sort of the
// entries by column: output row c holds the entries of source column c in
// ascending source-entry order. Here: expand each entry's source row, stable
// LSD radix sort of (column, entry index) pairs (rocPRIM), then gather.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include "bsm_internal.hpp"

namespace bsm {
namespace {

__global__ __launch_bounds__(256) void expand_rows(const int64_t* __restrict__ rp, int64_t rows,
                                                   int32_t* __restrict__ row_of) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    for (int64_t e = rp[row] + lane; e < rp[row + 1]; e += 64) row_of[e] = (int32_t)row;
}

__global__ __launch_bounds__(256) void iota_u32(uint32_t* __restrict__ p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

// t_rp[c] = first position in sorted keys with key >= c (c in [0, cols]).
__global__ __launch_bounds__(256) void bounds_from_sorted(const uint32_t* __restrict__ keys,
                                                          uint64_t nnz, uint64_t cols,
                                                          int64_t* __restrict__ t_rp) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > cols) return;
    uint64_t lo = 0, hi = nnz;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (keys[mid] < c) lo = mid + 1; else hi = mid;
    }
    t_rp[c] = (int64_t)lo;
}

template <typename T>
__global__ __launch_bounds__(256) void gather_transposed(const uint32_t* __restrict__ perm,
                                                         uint64_t nnz,
                                                         const int32_t* __restrict__ row_of,
                                                         const T* __restrict__ val,
                                                         int32_t* __restrict__ t_col,
                                                         T* __restrict__ t_val) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nnz) return;
    const uint32_t e = perm[p];
    t_col[p] = row_of[e];
    t_val[p] = val[e];
}

inline unsigned blocks_for(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

int transpose_dispatch(const bsm_csr* a, bsm_csr** out, hipStream_t s) {
    const uint64_t nnz = a->nnz, rows = a->rows, cols = a->cols;
    BSM_REQUIRE(nnz < (1ull << 32), BSM_ERR_UNSUPPORTED, "transpose supports nnz < 2^32");
    BSM_REQUIRE(rows < (1ull << 31), BSM_ERR_UNSUPPORTED, "transpose supports rows < 2^31");
    bsm_csr* t = nullptr;
    BSM_TRY(csr_alloc(&t, a->dtype, cols, rows, nnz));
    struct Guard {
        bsm_csr*& t;
        bool ok = false;
        ~Guard() { if (!ok) bsm_csr_free(t); }
    } guard{t};

    DBuf row_of, keys_in, keys_out, vals_in, vals_out, tmp;
    BSM_TRY(row_of.alloc(nnz * sizeof(int32_t)));
    BSM_TRY(keys_out.alloc(nnz * sizeof(uint32_t)));
    BSM_TRY(vals_in.alloc(nnz * sizeof(uint32_t)));
    BSM_TRY(vals_out.alloc(nnz * sizeof(uint32_t)));
    if (nnz) {
        expand_rows<<<blocks_for(rows, 4), 256, 0, s>>>(a->row_ptr, (int64_t)rows, row_of.as<int32_t>());
        iota_u32<<<blocks_for(nnz, 256), 256, 0, s>>>(vals_in.as<uint32_t>(), nnz);
        BSM_HIP_TRY(hipGetLastError());
        unsigned end_bit = 1;
        while (end_bit < 32 && (1ull << end_bit) < cols) ++end_bit;
        // columns are int32 >= 0 (checked at upload): sort them as uint32 keys
        const uint32_t* keys = reinterpret_cast<const uint32_t*>(a->col);
        size_t tmp_bytes = 0;
        BSM_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys, keys_out.as<uint32_t>(),
                                              vals_in.as<uint32_t>(), vals_out.as<uint32_t>(),
                                              (size_t)nnz, 0u, end_bit, s));
        BSM_TRY(tmp.alloc(tmp_bytes));
        BSM_HIP_TRY(rocprim::radix_sort_pairs(tmp.p, tmp_bytes, keys, keys_out.as<uint32_t>(),
                                              vals_in.as<uint32_t>(), vals_out.as<uint32_t>(),
                                              (size_t)nnz, 0u, end_bit, s));
        bsm::dispatch_dtype(a->dtype, [&]<typename T>() {
            gather_transposed<T><<<blocks_for(nnz, 256), 256, 0, s>>>(
                vals_out.as<uint32_t>(), nnz, row_of.as<int32_t>(), static_cast<const T*>(a->vals),
                t->col, static_cast<T*>(t->vals));
            return BSM_OK;
        });
    }
    bounds_from_sorted<<<blocks_for(cols + 1, 256), 256, 0, s>>>(keys_out.as<uint32_t>(), nnz, cols,
                                                                t->row_ptr);
    BSM_HIP_TRY(hipGetLastError());
    // temporaries are freed when this returns: finish before releasing them
    BSM_HIP_TRY(hipStreamSynchronize(s));
    guard.ok = true;
    *out = t;
    return BSM_OK;
}

}  // namespace bsm
