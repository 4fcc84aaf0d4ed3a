// LDS-fed f64 add chain with ds_read_b128 issued by inline asm (2 values per
// read), explicit lgkmcnt waits tied to the consumed registers, adds in C++.
#include <hip/hip_runtime.h>
#include <cstdio>

#define RD(r, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(r) : "v"(addr))
#define WT(r, n) asm volatile("s_waitcnt lgkmcnt(" #n ")" : "+v"(r.x), "+v"(r.y))
#define ADD2(r) { s = __dadd_rn(s, r.x); s = __dadd_rn(s, r.y); }

template <int LA>
__global__ void k_b128(double* out, long long n, long long* cyc) {
    __shared__ double buf[4096 + 64];
    for (int i = threadIdx.x; i < 4096 + 64; i += blockDim.x) buf[i] = out[3 + (i & 7)];
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s = out[0];
    const unsigned base = (unsigned)(uintptr_t)buf;
    const long long c0 = clock64();
    for (long long i = 0; i < n; i += 4096) {
        unsigned addr = base;
        double2 a0, a1, a2, a3, a4, a5, a6, a7;
        RD(a0, 0); RD(a1, 16); RD(a2, 32); RD(a3, 48);
        if (LA == 8) { RD(a4, 64); RD(a5, 80); RD(a6, 96); RD(a7, 112); }
        for (int j = 0; j < 4096; j += 16) {
            if (LA == 4) {
                WT(a0, 3); ADD2(a0); RD(a4, 64);
                WT(a1, 3); ADD2(a1); RD(a5, 80);
                WT(a2, 3); ADD2(a2); RD(a6, 96);
                WT(a3, 3); ADD2(a3); RD(a7, 112);
                WT(a4, 3); ADD2(a4); RD(a0, 128);
                WT(a5, 3); ADD2(a5); RD(a1, 144);
                WT(a6, 3); ADD2(a6); RD(a2, 160);
                WT(a7, 3); ADD2(a7); RD(a3, 176);
            } else {
                WT(a0, 7); ADD2(a0); RD(a0, 128);
                WT(a1, 7); ADD2(a1); RD(a1, 144);
                WT(a2, 7); ADD2(a2); RD(a2, 160);
                WT(a3, 7); ADD2(a3); RD(a3, 176);
                WT(a4, 7); ADD2(a4); RD(a4, 192);
                WT(a5, 7); ADD2(a5); RD(a5, 208);
                WT(a6, 7); ADD2(a6); RD(a6, 224);
                WT(a7, 7); ADD2(a7); RD(a7, 240);
            }
            addr += 128;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    cyc[0] = clock64() - c0;
    out[2] = s;
    double t = out[0];
    for (long long i = 0; i < n; i += 4096)
        for (int j = 0; j < 4096; ++j) t = __dadd_rn(t, buf[j]);
    out[5] = t;
}

int main() {
    double* d;
    long long* c;
    (void)hipMalloc(&d, 64 * sizeof(double));
    (void)hipMalloc(&c, 4 * sizeof(long long));
    double h[16] = {1.0, 1e-17, 0, 1.1, 2.3, 3.7, 4.1, 5.9, 6.2, 7.4, 8.8};
    const long long n = 1 << 22;
    long long hc[4];
    double o[8];
    for (int la : {4, 8}) {
        (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
        if (la == 4) { k_b128<4><<<1, 64>>>(d, n, c); k_b128<4><<<1, 64>>>(d, n, c); }
        else { k_b128<8><<<1, 64>>>(d, n, c); k_b128<8><<<1, 64>>>(d, n, c); }
        (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        (void)hipMemcpy(o, d, sizeof(o), hipMemcpyDeviceToHost);
        printf("asm b128 lookahead %d reads: %.2f cyc/add; sums %s\n", la, (double)hc[0] / n,
               o[2] == o[5] ? "identical" : "DIFFER");
    }
    return 0;
}
