// Issue cost of independent instructions placed between the dependent
// v_add_f64 of a serial chain (one wave per SIMD), gfx950. Each step is one
// chain add plus the listed filler; the result is cycles per step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>

#define STEP_ADD "v_add_f64 %0, %1, %0\n\t"
#define STEPS 64  // asm blocks of 8 steps each (one compiler-inserted s_nop per block)
#define R8(x) x x x x x x x x

template <int KIND>
__device__ __forceinline__ void step(double& s, double a, double& t0, double& t1, int& i0, float& f0, const double* in_ptr) {
    if constexpr (KIND == 0) asm volatile(R8(STEP_ADD "\n\t") : "+v"(s) : "v"(a));
    if constexpr (KIND == 1) asm volatile(R8(STEP_ADD "v_mul_f64 %2, %1, %1" "\n\t") : "+v"(s) : "v"(a), "v"(t0));
    if constexpr (KIND == 2) asm volatile(R8(STEP_ADD "v_mul_f64 %2, %1, %1\n\tv_mul_f64 %3, %1, %1" "\n\t") : "+v"(s) : "v"(a), "v"(t0), "v"(t1));
    if constexpr (KIND == 3) asm volatile(R8(STEP_ADD "v_cndmask_b32 %2, 0, %2, vcc" "\n\t") : "+v"(s) : "v"(a), "v"(i0));
    if constexpr (KIND == 4) asm volatile(R8(STEP_ADD "v_mov_b64 %2, %1" "\n\t") : "+v"(s) : "v"(a), "v"(t0));
    if constexpr (KIND == 5) asm volatile(R8(STEP_ADD "s_add_u32 s20, s20, 1" "\n\t") : "+v"(s) : "v"(a) : "s20");
    if constexpr (KIND == 6) asm volatile(R8(STEP_ADD "v_mul_f32 %2, %2, %2" "\n\t") : "+v"(s) : "v"(a), "v"(f0));
    if constexpr (KIND == 7) asm volatile(R8(STEP_ADD "v_mul_f64 %2, %1, %1\n\tv_mul_f64 %3, %1, %1\n\tv_mov_b64 %2, %1\n\tv_mov_b64 %3, %1" "\n\t") : "+v"(s) : "v"(a), "v"(t0), "v"(t1));
    if constexpr (KIND == 8) asm volatile(R8(STEP_ADD "ds_read_b64 %2, %3" "\n\t") : "+v"(s) : "v"(a), "v"(t0), "v"(i0));
    if constexpr (KIND == 9) asm volatile(R8(STEP_ADD "v_fma_f64 %2, %1, %1, %2" "\n\t") : "+v"(s) : "v"(a), "v"(t0));
    if constexpr (KIND == 10) asm volatile(R8(STEP_ADD "s_nop 0" "\n\t") : "+v"(s) : "v"(a));
    if constexpr (KIND == 11) asm volatile(R8(STEP_ADD "v_readlane_b32 s20, %2, 3\n\tv_readlane_b32 s21, %2, 3" "\n\t") : "+v"(s) : "v"(a), "v"(i0) : "s20", "s21");
    if constexpr (KIND == 12) asm volatile(R8("v_add_f64 %0, %0, %1" "\n\t") : "+v"(s) : "v"(a));
    if constexpr (KIND == 13) asm volatile(R8(STEP_ADD "v_mov_b32_dpp %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" "\n\t") : "+v"(s) : "v"(a), "v"(i0));
    if constexpr (KIND == 14) asm volatile(R8(STEP_ADD "global_load_dwordx2 %2, %3, off" "\n\t") : "+v"(s) : "v"(a), "v"(t0), "v"(in_ptr));
}

template <int KIND, int... I>
__device__ __forceinline__ void run(double& s, double a, double& t0, double& t1, int& i0, float& f0,
                                    std::integer_sequence<int, I...>, const double* in_ptr) {
    ((step<KIND>(s, a, t0, t1, i0, f0, in_ptr), (void)I), ...);
}

template <int KIND>
__global__ void k(const double* in, double* out, long long* cyc) {
    __shared__ double lds[512];
    lds[threadIdx.x] = in[threadIdx.x];
    __syncthreads();
    double s = in[1], a = in[2], t0 = in[3], t1 = in[4];
    int i0 = (threadIdx.x & 63) * 8;
    float f0 = (float)in[5];
    __builtin_amdgcn_s_waitcnt(0);
    const long long c0 = clock64();
    __builtin_amdgcn_sched_barrier(0);
    run<KIND>(s, a, t0, t1, i0, f0, std::make_integer_sequence<int, STEPS>{}, in + (threadIdx.x & 63));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const long long c1 = clock64();
    if (threadIdx.x == 0) cyc[KIND] = c1 - c0;
    out[threadIdx.x] = s + t0 + t1 + i0 + f0;
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
    const char* names[] = {"add only", "+1 v_mul_f64", "+2 v_mul_f64", "+1 v_cndmask_b32", "+1 v_mov_b64",
                           "+1 s_add_u32", "+1 v_mul_f32", "+2 mul_f64 +2 mov_b64", "+1 ds_read_b64",
                           "+1 v_fma_f64", "+1 s_nop 0", "+2 v_readlane_b32", "add, dependent src0",
                           "+1 v_mov_b32_dpp wave_shr", "+1 global_load_dwordx2"};
    long long hc[64];
    for (int rep = 0; rep < 2; ++rep) {
        k<0><<<1, 64>>>(in, out, c); k<1><<<1, 64>>>(in, out, c); k<2><<<1, 64>>>(in, out, c);
        k<3><<<1, 64>>>(in, out, c); k<4><<<1, 64>>>(in, out, c); k<5><<<1, 64>>>(in, out, c);
        k<6><<<1, 64>>>(in, out, c); k<7><<<1, 64>>>(in, out, c); k<8><<<1, 64>>>(in, out, c);
        k<9><<<1, 64>>>(in, out, c); k<10><<<1, 64>>>(in, out, c); k<11><<<1, 64>>>(in, out, c);
        k<12><<<1, 64>>>(in, out, c); k<13><<<1, 64>>>(in, out, c); k<14><<<1, 64>>>(in, out, c);
        (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        for (int i = 0; i < 15; ++i) printf("%-24s %.2f cyc/step\n", names[i], hc[i] / (8.0 * STEPS));
    }
    return 0;
}
