// Dependent-chain latencies on gfx950 (one lane of one wave active):
// f64 add, f64 mul+add, f64 div (__ddiv_rn), and an add chain fed from LDS
// by ds_read_b128 (two doubles per read, software-pipelined).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_add(double* out, long long n, long long* cyc) {
    double s = out[0], a = out[1];
    const long long t0 = wall_clock64();
    const long long c0 = clock64();
    for (long long i = 0; i < n; i += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) s = __dadd_rn(s, a);
    }
    cyc[0] = clock64() - c0;
    cyc[1] = wall_clock64() - t0;
    out[2] = s;
}
__global__ void k_muladd(double* out, long long n, long long* cyc) {
    double s = out[0], a = out[1];
    const long long c0 = clock64();
    for (long long i = 0; i < n; i += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) s = __dadd_rn(__dmul_rn(s, a), a);
    }
    cyc[0] = clock64() - c0;
    out[2] = s;
}
__global__ void k_div(double* out, long long n, long long* cyc) {
    double s = out[0], a = out[1];
    const long long c0 = clock64();
    for (long long i = 0; i < n; ++i) s = __ddiv_rn(s, a);
    cyc[0] = clock64() - c0;
    out[2] = s;
}
__global__ void k_lds_chain(double* out, long long n, long long* cyc) {
    __shared__ double buf[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) buf[i] = out[3 + (i & 7)];
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s = out[0];
    const double2* p = reinterpret_cast<const double2*>(buf);
    const long long c0 = clock64();
    for (long long i = 0; i < n; i += 1024) {
        double2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[u];
        for (int j = 8; j < 1024; j += 8) {
            double2 w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) w[u] = p[(j + u) & 1023];
#pragma unroll
            for (int u = 0; u < 8; ++u) { s = __dadd_rn(s, v[u].x); s = __dadd_rn(s, v[u].y); }
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = w[u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) { s = __dadd_rn(s, v[u].x); s = __dadd_rn(s, v[u].y); }
    }
    cyc[0] = clock64() - c0;
    out[2] = s;
}

int main() {
    double* d;
    long long* c;
    hipMalloc(&d, 64 * sizeof(double));
    hipMalloc(&c, 4 * sizeof(long long));
    double h[16] = {1.0, 1e-17, 0, 1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0};
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    long long hc[4];
    const long long n = 1 << 22;
    for (int rep = 0; rep < 2; ++rep) {
        k_add<<<1, 64>>>(d, n, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("f64 add chain: %.2f cyc/op (clock64), %.3f ns/op (wall 100 MHz)\n", (double)hc[0] / n, hc[1] * 10.0 / n);
        k_muladd<<<1, 64>>>(d, n, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("f64 mul->add chain: %.2f cyc per mul+add\n", (double)hc[0] / n);
        k_div<<<1, 64>>>(d, n / 16, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("f64 div chain: %.2f cyc/op\n", (double)hc[0] / (n / 16));
        k_lds_chain<<<1, 64>>>(d, n, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("f64 add chain fed by ds_read_b128: %.2f cyc/add\n", (double)hc[0] / n);
    }
    return 0;
}
