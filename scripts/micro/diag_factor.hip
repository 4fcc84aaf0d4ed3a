// Cycles per call of diag_factor16 (the 16 x 16 diagonal-block Cholesky of
// band_chol4) on one wave, gfx950: with stores (n = 16) and without (n = 0).
#include "../../basic_sparse_matrix_amd/csrc/kernels_solve.hip"
#include <cstdio>

namespace bsm {
namespace {
__global__ __launch_bounds__(64) void diag_bench(const double* in, double* CB, double* R, int* status, int64_t n,
                                                 int iters, long long* cyc) {
    __shared__ double dacc[16][17], dA[16][17], xl[16];
    const int c = threadIdx.x;
    if (c < 16)
        for (int j = 0; j < 16; ++j) {
            dacc[c][j] = 0.0;
            dA[c][j] = in[c * 16 + j];
        }
    __syncthreads();
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) diag_factor16<double>(dacc, dA, xl, 0, n, 15, 16, CB, R, status, c);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    long long t1 = clock64();
    if (c == 0) *cyc = (t1 - t0) / iters;
}
}  // namespace
}  // namespace bsm

int main() {
    double h[256];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) h[i * 16 + j] = i == j ? 20.0 : (i > j ? -1.0 / (1 + i + j) : 0.0);
    double *in, *CB, *R;
    int* st;
    long long* cyc;
    hipMalloc(&in, 256 * 8);
    hipMalloc(&CB, 64 * 1024 * 8);
    hipMalloc(&R, 1024 * 8);
    hipMalloc(&st, 64);
    hipMalloc(&cyc, 8);
    hipMemcpy(in, h, 256 * 8, hipMemcpyHostToDevice);
    for (int64_t n : {16, 0}) {
        for (int rep = 0; rep < 2; ++rep) {
            bsm::diag_bench<<<1, 64>>>(in, CB, R, st, n, 200, cyc);
            long long hc = 0;
            hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
            if (rep) printf("diag_factor16<double>: %lld cycles per call (%s)\n", hc, n ? "with stores" : "no stores");
        }
    }
    return 0;
}
