// kernels_solve.hip -- Cholesky and triangular solves (reference:
// src/sparse.rs:682-714, src/lib.rs:11-65). Filled in below.
#include "bsm_internal.hpp"

namespace bsm {
int solve_dispatch_cholesky(const bsm_csr*, bsm_csr**, hipStream_t) {
    set_error("cholesky not built yet");
    return BSM_ERR_UNSUPPORTED;
}
int solve_dispatch_trsv(const bsm_csr*, bool, uint64_t, uint64_t, const void*, void*, hipStream_t) {
    set_error("trsv not built yet");
    return BSM_ERR_UNSUPPORTED;
}
int solve_dispatch_full(const bsm_csr*, uint64_t, uint64_t, const void*, void*, hipStream_t) {
    set_error("solve not built yet");
    return BSM_ERR_UNSUPPORTED;
}
}  // namespace bsm
