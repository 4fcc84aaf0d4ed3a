// Cost of moving a running f64 sum from lane l to lane l+1 on gfx950, per hop,
// on top of SEG dependent v_add_f64 (8 cycles each). One wave; every variant
// walks 64 lanes x SEG adds per "row", rows repeated.
//  loop  : runtime loop over lanes, v_readlane x2 with an SGPR lane index
//  unroll: lanes unrolled, constant lane index (v_readlane with literal)
//  dpp   : the sum stays in a VGPR, moved one lane up with v_mov_b32_dpp
//          wave_shr:1 (two halves); every lane adds, lane l's result is used
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>

constexpr int SEG = 16;

__device__ __forceinline__ double rl(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

__global__ void k_loop(const double* in, double* out, int rows, int nseg, long long* cyc) {
    double p[SEG];
#pragma unroll
    for (int u = 0; u < SEG; ++u) p[u] = in[threadIdx.x * SEG + u];
    double sv = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < rows; ++r) {
        for (int l = 0; l < nseg; ++l) {
            double sl = sv;
#pragma unroll
            for (int u = 0; u < SEG; ++u) sl = __dadd_rn(sl, p[u]);
            sv = rl(sl, l);
        }
    }
    cyc[0] = clock64() - c0;
    out[threadIdx.x] = sv;
}

template <int... L>
__device__ __forceinline__ double walk(double sv, const double (&p)[SEG], std::integer_sequence<int, L...>) {
    auto hop = [&](auto lc) __attribute__((always_inline)) {
        constexpr int l = decltype(lc)::value;
        double sl = sv;
#pragma unroll
        for (int u = 0; u < SEG; ++u) sl = __dadd_rn(sl, p[u]);
        sv = rl(sl, l);
    };
    (hop(std::integral_constant<int, L>{}), ...);
    return sv;
}

__global__ void k_unroll(const double* in, double* out, int rows, int nseg, long long* cyc) {
    double p[SEG];
#pragma unroll
    for (int u = 0; u < SEG; ++u) p[u] = in[threadIdx.x * SEG + u];
    double sv = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < rows; ++r) sv = walk(sv, p, std::make_integer_sequence<int, 63>{});
    cyc[0] = clock64() - c0;
    out[threadIdx.x] = sv;
}

__device__ __forceinline__ double shr1(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    int rlo, rhi;
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b32_dpp %1, %3 wave_shr:1 row_mask:0xf bank_mask:0xf"
                 : "=&v"(rlo), "=&v"(rhi) : "v"(lo), "v"(hi));
    return __hiloint2double(rhi, rlo);
}

__global__ void k_dpp(const double* in, double* out, int rows, int nseg, long long* cyc) {
    double p[SEG];
#pragma unroll
    for (int u = 0; u < SEG; ++u) p[u] = in[threadIdx.x * SEG + u];
    double s = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < rows; ++r) {
        for (int l = 0; l < nseg; ++l) {
#pragma unroll
            for (int u = 0; u < SEG; ++u) s = __dadd_rn(s, p[u]);
            s = shr1(s);
        }
    }
    cyc[0] = clock64() - c0;
    out[threadIdx.x] = s;
}

int main() {
    double *in, *out;
    long long* c;
    hipMalloc(&in, 64 * SEG * sizeof(double));
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&c, 4 * sizeof(long long));
    double h[64 * SEG];
    for (int i = 0; i < 64 * SEG; ++i) h[i] = 1.0 / (i + 3);
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    const int rows = 2000, nseg = 63;
    long long hc[4];
    for (int rep = 0; rep < 2; ++rep) {
        const double hops = (double)rows * nseg;
        k_loop<<<1, 64>>>(in, out, rows, nseg, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("loop  : %.2f cyc/hop (%.2f beyond %d adds)\n", hc[0] / hops, hc[0] / hops - 8.0 * SEG, SEG);
        k_unroll<<<1, 64>>>(in, out, rows, nseg, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("unroll: %.2f cyc/hop (%.2f beyond %d adds)\n", hc[0] / hops, hc[0] / hops - 8.0 * SEG, SEG);
        k_dpp<<<1, 64>>>(in, out, rows, nseg, c);
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("dpp   : %.2f cyc/hop (%.2f beyond %d adds)\n", hc[0] / hops, hc[0] / hops - 8.0 * SEG, SEG);
    }
    return 0;
}
