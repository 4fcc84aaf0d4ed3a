// Dependent v_add_f64 latency on gfx950 measured on straight-line code
// (no loop branch inside the timed chain): 1024 adds per launch, the
// dependent operand as src0 or src1, and with 1 or 2 other waves competing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>

template <int... I>
__device__ __forceinline__ double chain(double s, const double* a, std::integer_sequence<int, I...>) {
    ((s = __dadd_rn(s, a[I & 7])), ...);
    return s;
}
template <int... I>
__device__ __forceinline__ double chain_mul(double s, const double* a, std::integer_sequence<int, I...>) {
    ((s = __dadd_rn(s, __dmul_rn(a[I & 7], a[(I + 3) & 7]))), ...);
    return s;
}

__global__ void k_straight(const double* in, double* out, long long* cyc) {
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = in[u + threadIdx.x];
    double s = in[9];
    __builtin_amdgcn_s_waitcnt(0);
    const long long c0 = clock64();
    __builtin_amdgcn_sched_barrier(0);
    s = chain(s, a, std::make_integer_sequence<int, 1024>{});
    asm volatile("" : "+v"(s));
    __builtin_amdgcn_sched_barrier(0);
    const long long c1 = clock64();
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = c1 - c0;
    out[threadIdx.x] = s;
}
// products of loop-invariant values: the muls are independent of s and may be
// scheduled between the adds
__global__ void k_mixed(const double* in, double* out, long long* cyc) {
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = in[u + threadIdx.x];
    double s = in[9];
    __builtin_amdgcn_s_waitcnt(0);
    const long long c0 = clock64();
    __builtin_amdgcn_sched_barrier(0);
    s = chain_mul(s, a, std::make_integer_sequence<int, 1024>{});
    asm volatile("" : "+v"(s));
    __builtin_amdgcn_sched_barrier(0);
    const long long c1 = clock64();
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = c1 - c0;
    out[threadIdx.x] = s;
}

int main() {
    double *in, *out;
    long long* c;
    (void)hipMalloc(&in, 4096 * sizeof(double));
    (void)hipMalloc(&out, 4096 * sizeof(double));
    (void)hipMalloc(&c, 64 * sizeof(long long));
    static double h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0 / (i + 3);
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    long long hc[64];
    for (int rep = 0; rep < 2; ++rep) {
        for (int waves : {1, 4, 8}) {
            k_straight<<<1, 64 * waves>>>(in, out, c);
            (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
            printf("straight add chain, %d wave(s)/CU: %.2f cyc/add\n", waves, hc[0] / 1024.0);
            k_mixed<<<1, 64 * waves>>>(in, out, c);
            (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
            printf("add chain + independent muls, %d wave(s)/CU: %.2f cyc/add\n", waves, hc[0] / 1024.0);
        }
    }
    return 0;
}
