// Cycles per call of the 16 x 16 diagonal-block Cholesky of the band kernels
// on gfx950, one wave factoring:
//   orig      diag_factor16 (stores and the pivot check inside every step)
//   x1        diag_factor16x<SM = 1, IL = false> (check folded into a flag, stores after the steps)
//   x1il      diag_factor16x<SM = 1, IL = true> (+ updates interleaved with the next pivot chain)
//   x2+store  diag_factor16x<SM = 2, IL = true> (block to LDS) + diag_store16 by the same wave
//   x2/4w     the same with the stores by 4 waves behind a barrier (as in the kernels)
// with stores (n = 16) and, for orig, without (n = 0). Checks that every
// variant stores the same bits as orig.
#include "../../basic_sparse_matrix_amd/csrc/kernels_solve.hip"
#include <cstdio>
#include <cstring>

namespace bsm {
namespace {
template <int V>
__global__ __launch_bounds__(256) void diag_bench(const double* in, double* CB, double* R, int* status, int64_t n,
                                                  int iters, long long* cyc) {
    __shared__ double dacc[16][17], dA[16][17], xl[16], Ls[16][17], Rs[16];
    const int tid = threadIdx.x, c = tid & 63;
    if (tid < 16)
        for (int j = 0; j < 16; ++j) {
            dacc[tid][j] = 0.0;
            dA[tid][j] = in[tid * 16 + j];
        }
    __syncthreads();
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        if (tid < 64) {
            if constexpr (V == 0) diag_factor16<double>(dacc, dA, xl, 0, n, 15, 16, CB, R, status, c);
            if constexpr (V == 1) diag_factor16x<double, 1, false>(dacc, dA, Ls, Rs, 0, n, 15, 16, CB, R, status, c);
            if constexpr (V == 4) diag_factor16x<double, 1, true>(dacc, dA, Ls, Rs, 0, n, 15, 16, CB, R, status, c);
            if constexpr (V == 2) {
                diag_factor16x<double, 2>(dacc, dA, Ls, Rs, 0, n, 15, 16, CB, R, status, c);
                diag_store16<double, 64>(Ls, Rs, 0, n, 15, 16, CB, R, c);
            }
            if constexpr (V == 3) diag_factor16x<double, 2>(dacc, dA, Ls, Rs, 0, n, 15, 16, CB, R, status, c);
        }
        if constexpr (V == 3) {
            __syncthreads();
            diag_store16<double, 256>(Ls, Rs, 0, n, 15, 16, CB, R, tid);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    long long t1 = clock64();
    if (tid == 0) *cyc = (t1 - t0) / iters;
}
}  // namespace
}  // namespace bsm

template <int V>
static long long run(const double* in, double* CB, double* R, int* st, long long* cyc, int64_t n, int threads) {
    long long hc = 0;
    for (int rep = 0; rep < 2; ++rep) {
        bsm::diag_bench<V><<<1, threads>>>(in, CB, R, st, n, 200, cyc);
        (void)hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
    }
    return hc;
}

int main() {
    double h[256];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) h[i * 16 + j] = i == j ? 20.0 : (i > j ? -1.0 / (1 + i + j) : 0.0);
    double *in, *CB, *R;
    int* st;
    long long* cyc;
    (void)hipMalloc(&in, 256 * 8);
    (void)hipMalloc(&CB, 64 * 1024 * 8);
    (void)hipMalloc(&R, 1024 * 8);
    (void)hipMalloc(&st, 64);
    (void)hipMalloc(&cyc, 8);
    (void)hipMemcpy(in, h, 256 * 8, hipMemcpyHostToDevice);
    static double ref[16 * 16 + 16], got[16 * 16 + 16];
    auto grab = [&](double* dst) {
        (void)hipMemcpy(dst, CB, 256 * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(dst + 256, R, 16 * 8, hipMemcpyDeviceToHost);
    };
    const char* names[] = {"orig", "x1", "x2+store", "x2/4w", "x1il"};
    long long cy[5];
    (void)hipMemset(CB, 0, 64 * 1024 * 8);
    cy[0] = run<0>(in, CB, R, st, cyc, 16, 64);
    grab(ref);
    for (int v = 1; v < 5; ++v) {
        (void)hipMemset(CB, 0, 64 * 1024 * 8);
        (void)hipMemset(R, 0, 1024 * 8);
        cy[v] = v == 1   ? run<1>(in, CB, R, st, cyc, 16, 64)
                : v == 2 ? run<2>(in, CB, R, st, cyc, 16, 64)
                : v == 3 ? run<3>(in, CB, R, st, cyc, 16, 256)
                         : run<4>(in, CB, R, st, cyc, 16, 64);
        grab(got);
        printf("%-9s %lld cycles per call, same bits as orig: %s\n", names[v], cy[v],
               memcmp(ref, got, sizeof ref) == 0 ? "yes" : "NO");
    }
    printf("%-9s %lld cycles per call (with stores); ", names[0], cy[0]);
    printf("no stores %lld\n", run<0>(in, CB, R, st, cyc, 0, 64));
    return 0;
}
