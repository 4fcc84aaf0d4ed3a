// Latency (cycles per dependent iteration, one wave) of the f64 operations on
// the solver chains, gfx950: correctly rounded division (__ddiv_rn), the
// Markstein quotient q' = q + (a - b q) y with y = RN(1/b) precomputed,
// sqrt (__dsqrt_rn), a mul + add pair, and v_readlane round trips.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double markstein(double a, double b, double y) {
    const double q = __dmul_rn(a, y);
    const double r = __fma_rn(-q, b, a);
    return __fma_rn(r, y, q);
}

template <int KIND>
__global__ void chain(const double* in, double* out, long long* cyc, int iters) {
    double x = in[threadIdx.x], c = in[64], d = in[65];
    const double y = __ddiv_rn(1.0, d);
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if constexpr (KIND == 0) x = __ddiv_rn(__dadd_rn(x, c), d);
        if constexpr (KIND == 1) x = markstein(__dadd_rn(x, c), d, y);
        if constexpr (KIND == 2) x = __dsqrt_rn(__dadd_rn(x, c));
        if constexpr (KIND == 3) x = __dadd_rn(__dmul_rn(x, c), d);
        if constexpr (KIND == 4) {
            const int lo = __builtin_amdgcn_readlane(__double2loint(x), 5);
            const int hi = __builtin_amdgcn_readlane(__double2hiint(x), 5);
            x = __dadd_rn(__hiloint2double(hi, lo), c);
        }
        if constexpr (KIND == 5) x = __dadd_rn(x, c);
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) *cyc = (t1 - t0) / iters;
}

int main() {
    double h[66];
    for (int i = 0; i < 64; ++i) h[i] = 1.0 + i * 1e-3;
    h[64] = 0.75;
    h[65] = 1.7;
    double *in, *out;
    long long* cyc;
    hipMalloc(&in, sizeof(h));
    hipMalloc(&out, 64 * 8);
    hipMalloc(&cyc, 8);
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[] = {"div_rn (add + __ddiv_rn)", "markstein (add + mul + 2 fma)", "sqrt_rn (add + __dsqrt_rn)",
                           "mul + add", "readlane pair + add", "add"};
    auto run = [&](auto kernel, int kind) {
        long long hc = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kernel, dim3(1), dim3(64), 0, 0, in, out, cyc, 4096);
            hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
        }
        printf("%-34s %lld cycles per dependent iteration\n", names[kind], hc);
    };
    run(chain<0>, 0);
    run(chain<1>, 1);
    run(chain<2>, 2);
    run(chain<3>, 3);
    run(chain<4>, 4);
    run(chain<5>, 5);
    return 0;
}
