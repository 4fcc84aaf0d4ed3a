// What clock does clock64() (s_memtime) count on gfx950, and how fast does it
// run with the chip idle vs busy with f64 VALU work (the band Cholesky's
// traces are in these cycles)? Wave 0 of each block spins until clock64()
// has advanced by N; the other waves of the block (busy = 1) run dependent
// f64 multiply-adds meanwhile. Rate = N / the hipEvent time of the launch.
// hipcc --offload-arch=gfx950 -O3 clock_rate.hip -o clock_rate
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(512) void spin(long long n, int busy, double* sink) {
    __shared__ int done;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (threadIdx.x < 64) {
        const long long t0 = clock64();
        while (clock64() - t0 < n) __builtin_amdgcn_s_sleep(1);
        if (threadIdx.x == 0) __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (busy) {
        double a = threadIdx.x * 1e-3, b = 1.0000001;
        while (!__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
#pragma unroll
            for (int i = 0; i < 64; ++i) a = a * b + 1e-9;
        }
        if (a == 12345.0) sink[0] = a;
    }
}

int main() {
    double* sink;
    (void)hipMalloc(&sink, 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const long long N = 400000000;  // clock64 ticks
    struct Case {
        const char* name;
        int blocks, busy;
    } cases[] = {{"1 block, idle chip", 1, 0}, {"256 blocks, wave 0 spins only", 256, 0},
                 {"256 blocks, 7 waves of f64 FMA each", 256, 1}};
    for (auto& c : cases) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            spin<<<c.blocks, 512>>>(N, c.busy, sink);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%-40s %lld ticks in %.2f ms: %.3f GHz\n", c.name, N, ms, N / (ms * 1e6));
        }
    }
    return 0;
}
