// Feeding a dependent f64 add chain (one lane) from LDS: which read shape
// and prefetch depth reaches the 8-cycle add latency?
#include <hip/hip_runtime.h>
#include <cstdio>

template <int B, int D>  // B doubles per batch via ds_read_b64, D batches in flight
__global__ void k_b64(double* out, long long n, long long* cyc) {
    __shared__ double buf[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = out[3 + (i & 7)];
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s = out[0];
    double v[D][B];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int u = 0; u < B; ++u) v[d][u] = buf[d * B + u];
    const long long c0 = clock64();
    int pos = D * B;
    for (long long i = 0; i < n; i += B * D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int u = 0; u < B; ++u) s = __dadd_rn(s, v[d][u]);
#pragma unroll
            for (int u = 0; u < B; ++u) v[d][u] = buf[(pos + u) & 4095];
            pos += B;
        }
    }
    cyc[0] = clock64() - c0;
    out[2] = s;
}

template <int B, int D>  // ds_read_b128: B doubles per batch (B even)
__global__ void k_b128(double* out, long long n, long long* cyc) {
    __shared__ double2 buf[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) buf[i] = make_double2(out[3 + (i & 7)], out[4]);
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s = out[0];
    double2 v[D][B / 2];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int u = 0; u < B / 2; ++u) v[d][u] = buf[d * B / 2 + u];
    const long long c0 = clock64();
    int pos = D * B / 2;
    for (long long i = 0; i < n; i += B * D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int u = 0; u < B / 2; ++u) { s = __dadd_rn(s, v[d][u].x); s = __dadd_rn(s, v[d][u].y); }
#pragma unroll
            for (int u = 0; u < B / 2; ++u) v[d][u] = buf[(pos + u) & 2047];
            pos += B / 2;
        }
    }
    cyc[0] = clock64() - c0;
    out[2] = s;
}


template <int B, int D>  // ds_read_b128, reads interleaved into the add chain's latency shadow
__global__ void k_b128_il(double* out, long long n, long long* cyc) {
    __shared__ double2 buf[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) buf[i] = make_double2(out[3 + (i & 7)], out[4]);
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s = out[0];
    double2 v[D][B / 2];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int u = 0; u < B / 2; ++u) v[d][u] = buf[d * B / 2 + u];
    const long long c0 = clock64();
    int pos = D * B / 2;
    for (long long i = 0; i < n; i += B * D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int u = 0; u < B / 2; ++u) {
                s = __dadd_rn(s, v[d][u].x);
                s = __dadd_rn(s, v[d][u].y);
                v[d][u] = buf[(pos + u) & 2047];
            }
#pragma unroll
            for (int u = 0; u < B / 2; ++u) {
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // one VALU
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // one VALU
            }
            pos += B / 2;
        }
    }
    cyc[0] = clock64() - c0;
    out[2] = s;
}

template <typename K>
void run(const char* name, K kern, double* d, long long* c, long long n) {
    long long hc[4];
    kern<<<1, 64>>>(d, n, c);
    kern<<<1, 64>>>(d, n, c);
    (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    printf("%-28s %.2f cyc/add\n", name, (double)hc[0] / n);
}

int main() {
    double* d;
    long long* c;
    (void)hipMalloc(&d, 64 * sizeof(double));
    (void)hipMalloc(&c, 4 * sizeof(long long));
    double h[16] = {1.0, 1e-17, 0, 1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0};
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const long long n = 1 << 22;
    run("b64  B=8  D=2", k_b64<8, 2>, d, c, n);
    run("b64  B=8  D=4", k_b64<8, 4>, d, c, n);
    run("b64  B=16 D=2", k_b64<16, 2>, d, c, n);
    run("b64  B=4  D=8", k_b64<4, 8>, d, c, n);
    run("b128 B=8  D=2", k_b128<8, 2>, d, c, n);
    run("b128 B=8  D=4", k_b128<8, 4>, d, c, n);
    run("b128 B=16 D=2", k_b128<16, 2>, d, c, n);
    run("b128 B=4  D=8", k_b128<4, 8>, d, c, n);
    run("b128il B=8 D=4", k_b128_il<8, 4>, d, c, n);
    run("b128il B=8 D=2", k_b128_il<8, 2>, d, c, n);
    run("b128il B=16 D=2", k_b128_il<16, 2>, d, c, n);
    run("b128il B=4 D=4", k_b128_il<4, 4>, d, c, n);
    return 0;
}
