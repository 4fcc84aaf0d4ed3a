// Row-block x column-panel SpMM schedule, k = 32, f64: how fast can a CU
// gather X rows when the X panel is small enough to stay in its XCD's L2 and
// the Y rows of its row block stay in LDS across the whole panel sweep?
//
// Synthetic tiled stream (no CSR): every wave owns RW rows (Y in LDS, 256 B
// each) and walks one flat stream of quads (4 entries, distinct rows, one per
// 16-lane group) ordered panel by panel. An entry is meta = (col << 8) | row
// and a value; lane q of group g gathers X[col][2q..2q+1] (16 B, 256 B per
// entry) and adds v*x into its row's LDS slot (read, add, write).
//
//   ./tile_gather RW PANEL_COLS N_PANELS BATCHES [MODE [COLMASK [SLACK [JITTER]]]]
//   MODE 0 = LDS RMW quad by quad, 1 = register sum only (gather bound),
//   2 = LDS RMW batched per chunk (64 distinct rows), 3 = 2 + XCD pacing
//   (a wave enters panel p once its XCD's waves have on average finished
//   panel p - SLACK; bounded spin, a hint only)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <utility>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int WAVES = 4;
constexpr double DENS = 1e-4;
constexpr int64_t NCOLS = 10000000;

__device__ __host__ inline uint64_t mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// stream of wave (gw): quads [qoff*gw, qoff*(gw+1)); panel p owns qpp quads
__global__ void fillx(double* x, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = 0.5 + (double)(mix(i) >> 40) * (1.0 / 16777216.0);
}

// per-wave panel of every quad with jittered panel lengths (qpp +- jit quads,
// uniform): the waves of an XCD drift apart like the real layout's
__global__ void gen_pmap(int32_t* pmap, int64_t n_waves, int64_t per, int qpp, int n_panels, int jit) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_waves) return;
    int p = 0;
    uint64_t h = mix(w * 31 + 7);
    int left = qpp;
    for (int64_t j = 0; j < per; ++j) {
        pmap[w * per + j] = p % n_panels;
        if (--left <= 0) {
            ++p;
            h = mix(h);
            left = qpp - jit + (int)(h % (uint64_t)(2 * jit + 1));
            if (left < 1) left = 1;
        }
    }
}

__global__ void gen(uint32_t* meta, double* val, int64_t n_waves, int64_t per, int qpp, int n_panels, int rw, uint32_t pc,
                    const int32_t* pmap) {
    const int64_t tot = n_waves * per;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = i / per, j = i % per;
        const int p = pmap ? pmap[i] : (int)(j / qpp) % n_panels;
        const uint64_t h = mix(i * 7919 + 17);
        const int base = (int)(mix(i / 16 + 5) % (uint64_t)rw);  // per chunk of 16 quads
        for (int g = 0; g < 4; ++g) {
            const uint64_t h2 = mix(h + g + 1);
            const int row = (base + (int)(i % 16) * 4 + g) % rw;  // 64 distinct rows per chunk
            const uint32_t col = (uint32_t)(((int64_t)p * pc + (int64_t)(h2 % pc)) % NCOLS);
            meta[i * 4 + g] = (col << 8) | (uint32_t)row;
            val[i * 4 + g] = 0.5 + (double)(h2 >> 40) * (1.0 / 16777216.0);
        }
        (void)w;
    }
}

// Unrolled three-phase pipeline (static buffer names, no copies, loads
// unconditional; the stream is padded so that chunk i+2's loads stay in
// bounds): phase k loads the indices of chunk i+k+2, gathers chunk i+k+1 and
// sums chunk i+k.
// chunk = 16 quads = 64 entries stored group-major ([g][u]): one coalesced
// load per field (lane 16g+q holds entry (quad q, group g)), then a DPP row
// broadcast hands entry (u, g) to every lane of group g.
struct Meta {
    uint32_t mi;
    double vi;
};
template <int U>
__device__ __forceinline__ void load_idx(Meta& c, const uint32_t* m, const double* v, int64_t q0, int lane) {
    c.mi = m[4 * q0 + lane];
    c.vi = v[4 * q0 + lane];
}
template <int I>
__device__ __forceinline__ uint32_t bm(const Meta& c) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c.mi, 0x150 + I, 0xf, 0xf, false);
}
template <int I>
__device__ __forceinline__ double bv(const Meta& c) {
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(c.vi), 0x150 + I, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(0, __double2loint(c.vi), 0x150 + I, 0xf, 0xf, false));
}
template <int... I>
__device__ __forceinline__ void gather(double2 (&x)[16], const Meta& c, const double2* X, int q, uint32_t cmask,
                                       std::integer_sequence<int, I...>) {
    ((x[I] = X[(int64_t)((bm<I>(c) >> 8) & cmask) * 16 + q]), ...);
}
template <int MODE, int I>
__device__ __forceinline__ void sum1(const double2& x, const Meta& c, double2* yw, int q, double& a0, double& a1) {
    const double vv = bv<I>(c);
    const double p0 = __dmul_rn(vv, x.x), p1 = __dmul_rn(vv, x.y);
    if (MODE == 0) {
        double2* yp = yw + (bm<I>(c) & 255) * 16 + q;
        double2 y = *yp;
        y.x = __dadd_rn(y.x, p0);
        y.y = __dadd_rn(y.y, p1);
        *yp = y;
    } else {
        a0 = __dadd_rn(a0, p0);
        a1 = __dadd_rn(a1, p1);
    }
}
template <int I>
__device__ __forceinline__ double2* yaddr(const Meta& c, double2* yw, int q) { return yw + (bm<I>(c) & 255) * 16 + q; }
template <int I>
__device__ __forceinline__ void madd(double2& y, const double2& x, const Meta& c) {
    const double vv = bv<I>(c);
    y.x = __dadd_rn(y.x, __dmul_rn(vv, x.x));
    y.y = __dadd_rn(y.y, __dmul_rn(vv, x.y));
}
// rows of a chunk are distinct: all 16 LDS reads, the sums, all 16 writes
template <int... I>
__device__ __forceinline__ void sum_batched(const double2 (&x)[16], const Meta& c, double2* yw, int q,
                                            std::integer_sequence<int, I...>) {
    double2 y[16];
    ((y[I] = *yaddr<I>(c, yw, q)), ...);
    (madd<I>(y[I], x[I], c), ...);
    ((*yaddr<I>(c, yw, q) = y[I]), ...);
}
template <int MODE, int... I>
__device__ __forceinline__ void sum(const double2 (&x)[16], const Meta& c, double2* yw, int q, double& a0, double& a1,
                                    std::integer_sequence<int, I...>) {
    (sum1<MODE, I>(x[I], c, yw, q, a0, a1), ...);
}

// Six-phase pipeline: phase k loads the indices of chunk i+k+4, gathers
// chunk i+k+2 and sums chunk i+k (meta 4 chunks ahead, gathers 2 ahead).
template <int U, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void tile(const uint32_t* __restrict__ meta, const double* __restrict__ val,
                                            int64_t quads_per_wave, int rw, const double2* __restrict__ X,
                                            double* __restrict__ out, uint32_t cmask, unsigned* pace, uint32_t pc,
                                            uint32_t slack) {
    static_assert(U == 16, "chunk = 16 quads");
    extern __shared__ double2 ylds[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4, q = lane & 15;
    double2* yw = ylds + (size_t)wave * (rw + 1) * 16;
    for (int r = g; r < rw + 1; r += 4) yw[r * 16 + q] = make_double2(0.0, 0.0);
    const int64_t stride = quads_per_wave + 160;  // padded stream (host: qst)
    const int64_t gw = (int64_t)blockIdx.x * WAVES + wave;
    const uint32_t* m = meta + gw * stride * 4;
    const double* v = val + gw * stride * 4;
    double a0 = 0.0, a1 = 0.0;
    constexpr auto SEQ = std::make_integer_sequence<int, 16>{};
    Meta M[6];
    double2 XS[3][16];
    uint32_t cur = 0;
    // pacing group = the blocks that share an XCD under round-robin dealing
    // (b % 8); lane l watches the progress words of block x + 8(l/2), waves
    // 2(l%2) and 2(l%2)+1 (gridDim.x == 256 here)
    bool gave_up = false;
    uint2* pslot = (uint2*)(pace + ((blockIdx.x & 7) + 8 * (lane >> 1)) * 4 + 2 * (lane & 1));
    uint2 pv[2] = {make_uint2(0u, 0u), make_uint2(0u, 0u)};
#pragma unroll
    for (int k = 0; k < 4; ++k) load_idx<U>(M[k], m, v, k * U, lane);
    gather(XS[0], M[0], X, q, cmask, SEQ);
    gather(XS[1], M[1], X, q, cmask, SEQ);
    for (int64_t i = 0; i < quads_per_wave; i += 6 * U) {  // quads_per_wave % (6U) == 0
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            load_idx<U>(M[(k + 4) % 6], m, v, i + (k + 4) * U, lane);
            if (MODE == 4) __hip_atomic_store(pace + gw, (uint32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (MODE == 5) { pv[k % 2] = __hip_atomic_load(pslot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); cur += pv[(k + 1) % 2].x; }
            if (MODE == 6) pace[gw] = (uint32_t)k;
            if (MODE == 7) { pv[k % 2] = pslot[0]; cur += pv[(k + 1) % 2].x; }
            if (MODE == 3) {  // XCD pacing: no wave gathers more than `slack` panels ahead of its group's slowest
                const uint32_t p = ((uint32_t)__builtin_amdgcn_readfirstlane((int)M[(k + 2) % 6].mi) >> 8) / pc;
                cur = p > cur ? p : cur;
                __hip_atomic_store(pace + gw, cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // all lanes, one word
                uint32_t mn = pv[k % 2].x < pv[k % 2].y ? pv[k % 2].x : pv[k % 2].y;  // polled two phases ago
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) { const uint32_t o = (uint32_t)__shfl_xor((int)mn, off); mn = o < mn ? o : mn; }
                if (!gave_up && cur > mn + slack) {
                    int spin = 0;
                    for (; spin < 2000 && cur > mn + slack; ++spin) {
                        __builtin_amdgcn_s_sleep(4);
                        const uint2 w = __hip_atomic_load(pslot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        mn = w.x < w.y ? w.x : w.y;
#pragma unroll
                        for (int off = 1; off < 64; off <<= 1) { const uint32_t o = (uint32_t)__shfl_xor((int)mn, off); mn = o < mn ? o : mn; }
                    }
                    gave_up = spin == 2000;
                }
                pv[k % 2] = __hip_atomic_load(pslot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // read two phases on
            }
            gather(XS[(k + 2) % 3], M[(k + 2) % 6], X, q, cmask, SEQ);
            __builtin_amdgcn_sched_barrier(0);  // keep this phase's loads ahead of its sums
            if (MODE >= 2) sum_batched(XS[k % 3], M[k], yw, q, SEQ);
            else sum<MODE>(XS[k % 3], M[k], yw, q, a0, a1, SEQ);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (MODE != 1) {
        for (int r = g; r < rw; r += 4) { const double2 y = yw[r * 16 + q]; a0 += y.x; a1 += y.y; }
    }
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = a0 + a1 + cur;
}

template <int U, int MODE>
float run(const uint32_t* meta, const double* val, int64_t qpw, int rw, const double2* X, double* out, int grid, uint32_t cm, unsigned* pace, uint32_t pc, uint32_t slack) {
    const size_t lds = (size_t)WAVES * (rw + 1) * 256;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMemset(pace, 0, 1 << 16));
    tile<U, MODE><<<grid, 256, lds>>>(meta, val, qpw, rw, X, out, cm, pace, pc, slack);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int it = 0; it < 3; ++it) {
        CHECK(hipMemset(pace, 0, 1 << 16));
        CHECK(hipEventRecord(e0));
        tile<U, MODE><<<grid, 256, lds>>>(meta, val, qpw, rw, X, out, cm, pace, pc, slack);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    return best;
}

int main(int argc, char** argv) {
    const int rw = argc > 1 ? atoi(argv[1]) : 144;
    const uint32_t pc = argc > 2 ? (uint32_t)atoi(argv[2]) : 8192;
    const int n_panels = argc > 3 ? atoi(argv[3]) : 200;
    const int batches = argc > 4 ? atoi(argv[4]) : 1;
    const int mode = argc > 5 ? atoi(argv[5]) : 0;
    const uint32_t cm = argc > 6 ? (uint32_t)strtoul(argv[6], nullptr, 0) : 0xffffffffu;
    if (rw > 255 || (size_t)WAVES * (rw + 1) * 256 > 160 * 1024) { printf("rw too large\n"); return 1; }
    const int grid = 256 * batches;
    const int64_t n_waves = (int64_t)grid * WAVES;
    const int qpp = (int)((rw * (double)pc * DENS + 3) / 4);
    const int64_t qpw = ((int64_t)qpp * n_panels + 95) / 96 * 96;  // multiple of 6U
    uint32_t* meta;
    double* val;
    double2* X;
    double* out;
    const int64_t qst = qpw + 160;
    CHECK(hipMalloc(&meta, n_waves * qst * 4 * 4));
    CHECK(hipMalloc(&val, n_waves * qst * 4 * 8));
    CHECK(hipMalloc(&X, NCOLS * 256));
    CHECK(hipMalloc(&out, (size_t)grid * 256 * 8));
    CHECK(hipMemset(X, 0, NCOLS * 256));
    if (getenv("XFILL")) fillx<<<4096, 256>>>((double*)X, NCOLS * 32);
    CHECK(hipMemset(meta, 0, n_waves * qst * 16));
    CHECK(hipMemset(val, 0, n_waves * qst * 32));
    const int jit = argc > 8 ? atoi(argv[8]) : 0;
    int32_t* pmap = nullptr;
    if (jit > 0) {
        CHECK(hipMalloc(&pmap, n_waves * qst * 4));
        gen_pmap<<<(unsigned)((n_waves + 63) / 64), 64>>>(pmap, n_waves, qst, qpp, n_panels, jit);
    }
    gen<<<4096, 256>>>(meta, val, n_waves, qst, qpp, n_panels, rw, pc, pmap);
    CHECK(hipDeviceSynchronize());
    const double entries = (double)n_waves * qpw * 4;
    float ms;
    unsigned* pace;
    CHECK(hipMalloc(&pace, 1 << 16));
    const uint32_t slack = argc > 7 ? (uint32_t)atoi(argv[7]) : 1;
    if (mode == 1) ms = run<16, 1>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else if (mode == 2) ms = run<16, 2>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else if (mode == 3) ms = run<16, 3>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else if (mode == 4) ms = run<16, 4>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else if (mode == 5) ms = run<16, 5>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else if (mode == 6) ms = run<16, 6>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else if (mode == 7) ms = run<16, 7>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    else ms = run<16, 0>(meta, val, qpw, rw, X, out, grid, cm, pace, pc, slack);
    const double gather_tbs = entries * 256 / (ms * 1e-3) / 1e12;
    const double c4_ms = 1e10 / entries * ms;
    printf("rw %d panel_cols %u (%.1f MB) panels %d batches %d mode %d: entries %.3g, %.3f ms, "
           "gather %.2f TB/s, quads/wave/panel %d, C4 extrapolated %.1f ms\n",
           rw, pc, pc * 256.0 / 1e6, n_panels, batches, mode, entries, ms, gather_tbs, qpp, c4_ms);
    return 0;
}
