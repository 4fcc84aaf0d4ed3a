// kernels_tiled.hip -- row-block x column-panel schedule of Csr::mul_dense
// for k = 32, f64 (reference: src/sparse.rs:426-446; the C4 shape).
//
// Why. At C4 every entry gathers a whole 256-B row of X (2.56 TB per SpMM)
// from a 2.56 GB table: the one-row-per-wave kernels read it at the
// Infinity-Cache/HBM rate (7.2 TB/s). Here each wave keeps the Y rows of a
// block of RW rows in LDS for a whole sweep of X in panels of PC columns
// (1 MiB of X at PC = 4096, well inside one XCD's 4 MiB L2). All waves sweep
// the panels in step, so an XCD's 32 CUs (18k rows) gather each panel from
// their shared L2; an X row is re-used about 1.8 times per L2 fill and the
// misses go to the Infinity Cache, which holds the panels the 8 XCDs are on.
// Measured at C4: 14.2 TB/s of gathers (180 ms) against 7.2 (353 ms).
//
// Layout (tiled_layout, once per matrix). Wave gw of NW owns the rows
// [gw*RPW, (gw+1)*RPW), taken in NB batches of RW rows. A (wave, batch) task
// is a stream of chunks of 64 entries; a chunk holds at most one entry of a
// row, so the kernel reads, adds and writes back the 64 LDS rows of a chunk
// as one batch. Chunks are filled greedily: the 64 rows whose next entry
// (in storage order) has the lowest column panel, ties by row. Every row's
// entries therefore stay in storage order and the per-element sum is the
// reference's sequential sum: bit-exact. Chunk n may only take entries of
// panels <= n / R, R = the task's mean chunks per panel + 3 %: waves with
// equal work then sweep the panels in step without talking to each other.
// Free slots hold dummy entries (row RW, a scratch LDS row; X row 0; value
// 0). Entry = meta (col << 8 | row-in-batch, so cols < 2^24) + the f64
// value: 12 B, like CSR's col + val.
//
// Kernel (spmm_tiled_k32). One 256-thread workgroup per CU (LDS-bound), four
// waves. Per task: zero the LDS rows, stream the chunks through a six-phase
// pipeline (indices four chunks ahead, gathers two ahead, so 32 gathers of
// 1 KiB are in flight per wave), write the Y rows and their nonzero counts,
// then meet the other waves at a bounded batch barrier (time noise would
// otherwise spread the waves over the batch cycle: 369 ms without it).
// Lane 16g+q of a chunk handles entry (quad q, group g) at load time; a DPP
// row broadcast hands entry (u, g) to the 16 lanes of group g, which gather
// X[col][2q..2q+1] (16 B each, one 256-B row per group).
#include "bsm_internal.hpp"

#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>


namespace bsm {
namespace {

constexpr int WAVE = 64;
constexpr int CHUNK = 64;        // entries per chunk = 16 quads x 4 lane groups
constexpr int PHASES = 6;        // pipeline unroll; task chunk counts are multiples of it
constexpr int OVERREAD = 4;      // chunks the pipeline reads past a task's end
constexpr uint32_t DONE = 0xffffffffu;
constexpr uint32_t RW_MAX = 155;  // 4 waves x (RW+1) rows x 256 B <= 160 KiB of LDS
constexpr uint32_t RW_MAX_F32 = 255;  // f32: 128-B rows; the 8-bit row field (dummy row = RW) caps it
constexpr uint32_t PSHIFT = 12;   // panel = 4096 columns = 1 MiB of X (C4 sweep: 2^10..2^12 flat, 2^13 +12 %, 2^14 +42 %)
constexpr uint32_t PACE_PCT = 3;  // chunk budget per panel over the task's mean (padding ~ this; C4: 2 % +19 %, 6 % +2 %)

__device__ __forceinline__ uint64_t lanemask_lt(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, WAVE));
    return v;
}

// ---------------------------------------------------------------------------
// layout builder: one wave per task (gw, b). COUNT pass writes the task's
// chunk count (a multiple of PHASES); WRITE pass fills its chunks from offs.
// ---------------------------------------------------------------------------
template <bool WRITE, int SLOTS, typename V, typename M = uint32_t>
__global__ __launch_bounds__(256) void tiled_layout(uint64_t rows, uint64_t n_cols, double pace, uint32_t rbits,
                                                    uint32_t pad, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const V* __restrict__ vals, uint32_t nw,
                                                    uint32_t rpw, uint32_t nb, uint32_t rw, uint32_t pshift,
                                                    int32_t* __restrict__ counts,
                                                    const int64_t* __restrict__ offs,
                                                    M* __restrict__ meta, V* __restrict__ val) {
    const int lane = threadIdx.x & (WAVE - 1);
    const uint64_t task = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    if (task >= (uint64_t)nw * nb) return;
    const uint64_t gw = task / nb, b = task % nb;
    const uint64_t w0 = gw * rpw;
    const uint64_t wend = min<uint64_t>(rows, w0 + rpw);
    const uint64_t r0 = w0 + b * rw;
    int64_t cur[SLOTS], end[SLOTS];
    uint32_t h[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
        const uint32_t s = lane + WAVE * j;
        const bool live = s < rw && r0 + s < wend;
        cur[j] = live ? rp[r0 + s] : 0;
        end[j] = live ? rp[r0 + s + 1] : 0;
        h[j] = cur[j] < end[j] ? (uint32_t)col[cur[j]] >> pshift : DONE;
    }
    // pace: chunk n may take entries from panels <= n * inv_r, inv_r = panels
    // per chunk at the task's own density plus a margin, so that the waves of a
    // batch (equal work at C4) stay on the same panels in step without talking
    // to each other; a wave that falls behind catches up by the margin
    // a task past the last row (rows < nw, or a wave's trailing batches) is
    // empty: it must not read row_ptr beyond rows + 1 entries
    const bool any = r0 < wend;
    const int64_t t0 = any ? rp[r0] : 0, t1 = any ? rp[min<uint64_t>(r0 + rw, wend)] : 0;
    const double np = (double)(((n_cols - 1) >> pshift) + 1);
    const double inv_r = t1 > t0 ? (double)CHUNK * np / ((double)(t1 - t0) * pace) : 1e30;
    int64_t c = WRITE ? offs[task] : 0;
    int64_t n = 0;
    for (;;) {
        bool sel[SLOTS];
        int pos[SLOTS];
#pragma unroll
        for (int j = 0; j < SLOTS; ++j) {
            sel[j] = false;
            pos[j] = 0;
        }
        int taken = 0;
        const double pm = (double)n * inv_r;
        const uint32_t pmax = pm >= 4.0e9 ? DONE - 1 : (uint32_t)pm;
        bool done = false;
        while (taken < CHUNK) {  // the lowest panels first, ties by row
            uint32_t m = DONE;
#pragma unroll
            for (int j = 0; j < SLOTS; ++j) m = min(m, sel[j] ? DONE : h[j]);
            m = wave_min_u32(m);
            if (m == DONE) {
                done = taken == 0;
                break;
            }
            if (m > pmax) break;  // ahead of the pace: the rest of the chunk is padding
            int before = 0;  // candidates in the slots before j (slot order = row order)
#pragma unroll
            for (int j = 0; j < SLOTS; ++j) {
                const bool cand = !sel[j] && h[j] == m;
                const uint64_t bal = __ballot(cand);
                const int rank = before + __popcll(bal & lanemask_lt(lane));
                if (cand && taken + rank < CHUNK) {
                    sel[j] = true;
                    pos[j] = taken + rank;
                }
                before += __popcll(bal);
            }
            taken = min(taken + before, CHUNK);
        }
        if (done) break;
#pragma unroll
        for (int j = 0; j < SLOTS; ++j) {
            if (sel[j]) {
                const int64_t e = cur[j];
                if (WRITE) {
                    meta[c * CHUNK + pos[j]] = ((M)(uint32_t)col[e] << rbits) | (M)(lane + WAVE * j);
                    val[c * CHUNK + pos[j]] = vals[e];
                }
                cur[j] = e + 1;
                h[j] = cur[j] < end[j] ? (uint32_t)col[cur[j]] >> pshift : DONE;
            }
        }
        if (WRITE && lane >= taken) {  // dummy entries: scratch row rw, X row 0, value 0
            meta[c * CHUNK + lane] = (M)rw;
            val[c * CHUNK + lane] = (V)0;
        }
        ++c;
        ++n;
    }
    const int64_t padded = (n + pad - 1) / pad * pad;
    if (WRITE) {
        for (int64_t p = n; p < padded; ++p, ++c) {
            meta[c * CHUNK + lane] = (M)rw;
            val[c * CHUNK + lane] = (V)0;
        }
    } else if (lane == 0) {
        counts[task] = (int32_t)padded;
    }
}

// ---------------------------------------------------------------------------
// the SpMM
// ---------------------------------------------------------------------------
// T = f64 (the C4 kernel) or f32: an X / Y row of k = 32 is 16 vec2<T>
// (256 or 128 B), lane q of a 16-lane group holding columns 2q, 2q + 1.
template <typename T> struct Vec2;
template <> struct Vec2<double> { using type = double2; };
// f32: two floats in one 64-bit word (an 8-B lane load, unpacked for the
// math). With HIP's float2 the compiler parked the gathered rows in AGPRs and
// waited for every outstanding load before the copies (vmcnt(0) in the loop,
// the pipeline collapsed: 338 ms at C4).
struct F2 {
    uint64_t u;
};
template <> struct Vec2<float> { using type = F2; };
__device__ __forceinline__ double lo_of(const double2& v) { return v.x; }
__device__ __forceinline__ double hi_of(const double2& v) { return v.y; }
__device__ __forceinline__ float lo_of(const F2& v) { return __uint_as_float((uint32_t)v.u); }
__device__ __forceinline__ float hi_of(const F2& v) { return __uint_as_float((uint32_t)(v.u >> 32)); }
__device__ __forceinline__ double2 make_v2(double a, double b) { return make_double2(a, b); }
__device__ __forceinline__ F2 make_v2(float a, float b) {
    return F2{((uint64_t)__float_as_uint(b) << 32) | (uint64_t)__float_as_uint(a)};
}
template <typename T> using vec2_t = typename Vec2<T>::type;

// M: the meta word, col << 8 | row-in-batch: uint32_t for columns < 2^24,
// uint64_t for wider matrices (k = 32; 8 B more per entry)
template <typename T = double, typename M = uint32_t>
struct Idx {
    M mi;  // lane 16g+q: entry (quad q, group g) of the chunk
    T vi;
};
template <typename T, typename M>
__device__ __forceinline__ void load_idx(Idx<T, M>& c, const M* __restrict__ meta, const T* __restrict__ val,
                                         int64_t chunk, int lane) {
    c.mi = meta[chunk * CHUNK + lane];
    c.vi = val[chunk * CHUNK + lane];
}
template <int I, typename T>
__device__ __forceinline__ uint32_t bm(const Idx<T, uint32_t>& c) {  // entry (I, g) to every lane of group g
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c.mi, 0x150 + I, 0xf, 0xf, false);
}
template <int I, typename T>
__device__ __forceinline__ uint64_t bm(const Idx<T, uint64_t>& c) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)c.mi, 0x150 + I, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(c.mi >> 32), 0x150 + I, 0xf, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}
template <int I, typename M>
__device__ __forceinline__ double bv(const Idx<double, M>& c) {
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(c.vi), 0x150 + I, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(0, __double2loint(c.vi), 0x150 + I, 0xf, 0xf, false));
}
template <int I, typename M>
__device__ __forceinline__ float bv(const Idx<float, M>& c) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c.vi), 0x150 + I, 0xf, 0xf, false));
}
__device__ __forceinline__ double mul_rn(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double add_rn(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
// PROBE (measurement only, wrong results): every gather reads X row
// (col & xmask), e.g. xmask = 0 leaves the index/value stream alone on the
// memory side (the PMC calibration of its 4-B / 8-B per-lane reads)
template <bool PROBE, typename T, typename M, int... I>
__device__ __forceinline__ void gather(vec2_t<T> (&x)[16], const Idx<T, M>& c, const vec2_t<T>* __restrict__ X, int q,
                                       uint32_t xmask, std::integer_sequence<int, I...>) {
    if (PROBE) ((x[I] = X[(int64_t)((bm<I>(c) >> 8) & xmask) * 16 + q]), ...);
    else ((x[I] = X[(int64_t)(bm<I>(c) >> 8) * 16 + q]), ...);
}
template <int I, typename T, typename M>
__device__ __forceinline__ vec2_t<T>* yaddr(const Idx<T, M>& c, vec2_t<T>* yw, int q) {
    return yw + (uint32_t)(bm<I>(c) & 255u) * 16 + q;
}
template <int I, typename T, typename M>
__device__ __forceinline__ void madd(vec2_t<T>& y, const vec2_t<T>& x, const Idx<T, M>& c) {
    const T v = bv<I>(c);
    y = make_v2(add_rn(lo_of(y), mul_rn(v, lo_of(x))), add_rn(hi_of(y), mul_rn(v, hi_of(x))));
}
// the chunk's rows are distinct (dummies all hit the scratch row), so its
// 16 read-add-write updates are independent: all 16 LDS reads, then the
// multiply-adds, then the writes (split into parts of 8 or 4 they measured
// 33 % slower at C4: round 4)
template <typename T, typename M, int... I>
__device__ __forceinline__ void sum_chunk(const vec2_t<T> (&x)[16], const Idx<T, M>& c, vec2_t<T>* yw, int q,
                                          std::integer_sequence<int, I...>) {
    vec2_t<T> y[sizeof...(I)];
    ((y[I] = *yaddr<I>(c, yw, q)), ...);
    (madd<I>(y[I], x[I], c), ...);
    ((*yaddr<I>(c, yw, q) = y[I]), ...);
}

// Batch pacing. Within a batch the layout keeps the waves on the same
// panels (equal chunks per panel), but time noise accumulates from batch to
// batch; once the waves are spread over the batch cycle, every XCD gathers
// from all of X again. So the waves meet at every batch start: arrivals are
// counted in 8 words (one per blockIdx % 8, 128-B apart) by relaxed agent
// atomics and a wave polls their sum. A pacing aid only: nothing is handed
// off (X, the stream and the wave's own LDS rows are all it reads), and the
// wait is bounded, so a grid that is not all resident (other kernels on the
// CUs) costs one timeout per wave and then runs unpaced.
constexpr int BAR_STRIDE = 32;  // words between the arrival counters
__device__ __forceinline__ void batch_arrive(unsigned* bar, uint32_t n, int lane) {
    if (lane == 0) __hip_atomic_fetch_add(bar + (blockIdx.x & 7) * BAR_STRIDE, n, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool batch_wait(unsigned* bar, uint32_t target, int lane, uint32_t spins = 4000) {
    for (uint32_t spin = 0; spin < spins; ++spin) {
        uint32_t v = lane < 8 ? __hip_atomic_load(bar + lane * BAR_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : 0u;
        v += (uint32_t)__shfl_xor((int)v, 1);
        v += (uint32_t)__shfl_xor((int)v, 2);
        v += (uint32_t)__shfl_xor((int)v, 4);
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)v) >= target) return true;
        __builtin_amdgcn_s_sleep(8);
    }
    return false;  // not all resident: stop pacing
}

template <bool PROBE, typename T, typename M>
__device__ __forceinline__ void spmm_tiled_k32_body(
    uint64_t rows, uint32_t rpw, uint32_t nb, uint32_t rw, const int64_t* __restrict__ offs,
    const M* __restrict__ meta, const T* __restrict__ val, const vec2_t<T>* __restrict__ X,
    vec2_t<T>* __restrict__ Y, int32_t* __restrict__ row_nnz, unsigned* bar, uint32_t xmask, uint32_t spins) {
    using V2 = vec2_t<T>;
    extern __shared__ __align__(16) unsigned char ylds_raw[];
    V2* const ylds = reinterpret_cast<V2*>(ylds_raw);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wave = threadIdx.x / WAVE;
    const int g = lane >> 4, q = lane & 15;
    V2* yw = ylds + (size_t)wave * (rw + 1) * 16;
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + wave;
    const uint64_t w0 = gw * rpw;
    const uint64_t wend = min<uint64_t>(rows, w0 + rpw);
    constexpr auto SEQ = std::make_integer_sequence<int, 16>{};
    bool sync = bar != nullptr;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint64_t r0 = w0 + (uint64_t)b * rw;
        if (r0 >= wend) {  // out of rows: arrive for the batches left and stop
            if (sync) batch_arrive(bar, nb - b, lane);
            break;
        }
        if (sync && b > 0) sync = batch_wait(bar, (uint32_t)gridDim.x * (blockDim.x / WAVE) * b, lane, spins);
        const int nr = (int)min<uint64_t>(rw, wend - r0);
        for (int r = g; r < nr; r += 4) yw[r * 16 + q] = make_v2((T)0, (T)0);
        const int64_t c0 = offs[gw * nb + b], c1 = offs[gw * nb + b + 1];
        if (c1 > c0) {  // (c1 - c0) % PHASES == 0
            Idx<T, M> MI[6];
            V2 XS[3][16];
#pragma unroll
            for (int k = 0; k < 4; ++k) load_idx(MI[k], meta, val, c0 + k, lane);
            gather<PROBE>(XS[0], MI[0], X, q, xmask, SEQ);
            gather<PROBE>(XS[1], MI[1], X, q, xmask, SEQ);
            for (int64_t i = c0; i < c1; i += PHASES) {
#pragma unroll
                for (int k = 0; k < PHASES; ++k) {
                    load_idx(MI[(k + 4) % 6], meta, val, i + k + 4, lane);
                    gather<PROBE>(XS[(k + 2) % 3], MI[(k + 2) % 6], X, q, xmask, SEQ);
                    __builtin_amdgcn_sched_barrier(0);  // this phase's loads stay ahead of its sums
                    sum_chunk<T>(XS[k % 3], MI[k], yw, q, SEQ);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        for (int rb = 0; rb < nr; rb += 4) {  // Y rows and their nonzero counts
            const int r = rb + g;
            const bool live = r < nr;
            const V2 y = live ? yw[r * 16 + q] : make_v2((T)0, (T)0);
            if (live) Y[(r0 + r) * 16 + q] = y;
            const uint64_t m0 = __ballot(lo_of(y) != (T)0), m1 = __ballot(hi_of(y) != (T)0);
            if (live && q == 0 && row_nnz)
                row_nnz[r0 + r] = __popcll((m0 >> (16 * g)) & 0xffffull) + __popcll((m1 >> (16 * g)) & 0xffffull);
        }
        if (sync) batch_arrive(bar, 1, lane);
    }
}

// f64: the whole 512-register budget of one wave per SIMD (LDS allows one
// workgroup per CU anyway); the gathers two chunks ahead take 192 of it.
template <bool PROBE, typename T = double, typename M = uint32_t>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void spmm_tiled_k32(
    uint64_t rows, uint32_t rpw, uint32_t nb, uint32_t rw, const int64_t* __restrict__ offs,
    const M* __restrict__ meta, const T* __restrict__ val, const vec2_t<T>* __restrict__ X,
    vec2_t<T>* __restrict__ Y, int32_t* __restrict__ row_nnz, unsigned* bar, uint32_t xmask, uint32_t spins) {
    spmm_tiled_k32_body<PROBE, T, M>(rows, rpw, nb, rw, offs, meta, val, X, Y, row_nnz, bar, xmask, spins);
}
// f32 (F2 words, see Vec2<float>)
template <typename M = uint32_t>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void spmm_tiled_k32_f32(
    uint64_t rows, uint32_t rpw, uint32_t nb, uint32_t rw, const int64_t* __restrict__ offs,
    const M* __restrict__ meta, const float* __restrict__ val, const F2* __restrict__ X, F2* __restrict__ Y,
    int32_t* __restrict__ row_nnz, unsigned* bar, uint32_t xmask, uint32_t spins) {
    spmm_tiled_k32_body<false, float, M>(rows, rpw, nb, rw, offs, meta, val, X, Y, row_nnz, bar, xmask, spins);
}

// ---------------------------------------------------------------------------
// k = 1 (SpMV, C2's shape): the same copy with RW up to 2047 rows per wave (Y
// is one double per row: 4 waves x 2048 x 8 B of LDS) and meta = col << 11 |
// row, so an XCD holds ~125k rows and an X panel of 2 MiB (2^18 columns) is
// re-read from L2 about 20 times per 128-B line. Lane l takes entry l of a
// chunk; eight chunks make a stage; three stages are in flight (indices two
// stages ahead, gathers one ahead). The 64 rows of a chunk are distinct, so
// a chunk's LDS read-add-writes are one instruction each; the chunks of a
// stage go in order.
// ---------------------------------------------------------------------------
constexpr int K1_STAGE_DEFAULT = 4;          // chunks per stage (4 or 8)
constexpr uint32_t K1_RBITS = 11;
constexpr uint32_t K1_RW_MAX = (1u << K1_RBITS) - 1;
constexpr uint32_t K1_PSHIFT = 18;           // panel = 2^18 columns = 2 MiB of X
constexpr uint32_t K1_WAVES_PER_CU = 4;      // one workgroup per CU (C2: 59 us against 69 at 12)

template <int ST, typename T>
struct Stage1 {
    uint32_t m[ST];
    T v[ST];
    T x[ST];
};
template <int ST, typename T>
__device__ __forceinline__ void k1_load(Stage1<ST, T>& st, const uint32_t* __restrict__ meta,
                                        const T* __restrict__ val, int64_t c, int lane) {
#pragma unroll
    for (int j = 0; j < ST; ++j) {
        st.m[j] = meta[(c + j) * CHUNK + lane];
        st.v[j] = val[(c + j) * CHUNK + lane];
    }
}
template <int ST, typename T>
__device__ __forceinline__ void k1_gather(Stage1<ST, T>& st, const T* __restrict__ X, uint32_t xmask) {
#pragma unroll
    for (int j = 0; j < ST; ++j) st.x[j] = X[(st.m[j] >> K1_RBITS) & xmask];
}
template <int ST, typename T>
__device__ __forceinline__ void k1_sum(const Stage1<ST, T>& st, T* yl) {
#pragma unroll
    for (int j = 0; j < ST; ++j) {
        T* yp = yl + (st.m[j] & K1_RW_MAX);
        *yp = add_rn(*yp, mul_rn(st.v[j], st.x[j]));
    }
}

template <int K1_STAGE, typename T = double>
__global__ __launch_bounds__(256) void spmm_tiled_k1(uint64_t rows, uint32_t rpw, uint32_t nb, uint32_t rw,
                                                     const int64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ meta,
                                                     const T* __restrict__ val, const T* __restrict__ X,
                                                     T* __restrict__ Y, int32_t* __restrict__ row_nnz,
                                                     unsigned* bar, bool neg_init, uint32_t xmask) {
    extern __shared__ __align__(16) unsigned char y1lds_raw[];
    T* const y1lds = reinterpret_cast<T*>(y1lds_raw);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wave = threadIdx.x / WAVE;
    T* yl = y1lds + (size_t)wave * (rw + 1);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + wave;
    const uint64_t w0 = gw * rpw;
    const uint64_t wend = min<uint64_t>(rows, w0 + rpw);
    const T init = neg_init ? (T)-0.0 : (T)0.0;
    bool sync = bar != nullptr;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint64_t r0 = w0 + (uint64_t)b * rw;
        if (r0 >= wend) {
            if (sync) batch_arrive(bar, nb - b, lane);
            break;
        }
        if (sync && b > 0) sync = batch_wait(bar, (uint32_t)gridDim.x * (blockDim.x / WAVE) * b, lane);
        const int nr = (int)min<uint64_t>(rw, wend - r0);
        for (int r = lane; r < nr; r += WAVE) yl[r] = init;
        const int64_t c0 = offs[gw * nb + b], c1 = offs[gw * nb + b + 1];
        int64_t i = c0;
        if (c1 - c0 >= 3 * K1_STAGE) {  // whole groups of three stages, pipelined
            constexpr int K1_GROUP = 3 * K1_STAGE;
            Stage1<K1_STAGE, T> S0, S1, S2;
            k1_load(S0, meta, val, c0, lane);
            k1_load(S1, meta, val, c0 + K1_STAGE, lane);
            k1_gather(S0, X, xmask);
            for (; i + K1_GROUP <= c1; i += K1_GROUP) {
                k1_load(S2, meta, val, i + 2 * K1_STAGE, lane);
                k1_gather(S1, X, xmask);
                __builtin_amdgcn_sched_barrier(0);
                k1_sum(S0, yl);
                __builtin_amdgcn_sched_barrier(0);
                k1_load(S0, meta, val, i + 3 * K1_STAGE, lane);
                k1_gather(S2, X, xmask);
                __builtin_amdgcn_sched_barrier(0);
                k1_sum(S1, yl);
                __builtin_amdgcn_sched_barrier(0);
                k1_load(S1, meta, val, i + 4 * K1_STAGE, lane);
                k1_gather(S0, X, xmask);
                __builtin_amdgcn_sched_barrier(0);
                k1_sum(S2, yl);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        for (; i < c1; ++i) {  // the task's last chunks, one at a time
            const uint32_t m = meta[i * CHUNK + lane];
            const T v = val[i * CHUNK + lane];
            const T xv = X[(m >> K1_RBITS) & xmask];
            T* yp = yl + (m & K1_RW_MAX);
            *yp = add_rn(*yp, mul_rn(v, xv));
        }
        for (int r = lane; r < nr; r += WAVE) {
            const T y = yl[r];
            Y[r0 + r] = y;
            if (row_nnz) row_nnz[r0 + r] = y != (T)0 ? 1 : 0;
        }
        if (sync) batch_arrive(bar, 1, lane);
    }
}

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = getenv(name);
    return e ? (uint32_t)strtoul(e, nullptr, 10) : dflt;
}

}  // namespace

// Shape test. k = 32: f64, X beyond 1 GiB (the Infinity Cache holds less),
// columns < 2^24. k = 1: f64, X beyond one XCD's 4 MiB L2, columns < 2^21.
// Both: rows at most a few times their mean length (a long row serialises
// its chunks, one entry per chunk).
bool tiled_wanted(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, uint64_t k, uint64_t max_row_len) {
    const bool shape = (dtype == BSM_F64 || dtype == BSM_F32) && rows > 0 && nnz > 0 &&
                       ((k == 32 && n_cols <= 0x7fffffffull) || (k == 1 && n_cols < (1u << (32 - K1_RBITS))));
    if (const char* e = getenv("BSM_SPMM_TILED")) {
        if (atoi(e) == 0) return false;
        if (atoi(e) == 2) return shape;
    }
    if (!shape) return false;
    const uint64_t x_bytes = n_cols * k * (dtype == BSM_F32 ? 4 : 8);
    if (x_bytes <= (k == 32 ? (1ull << 30) : (4ull << 20))) return false;
    const uint64_t mean = (nnz + rows - 1) / rows;
    return max_row_len <= 2 * mean + 256;
}

int tiled_create(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* rp, const int32_t* col,
                 const void* vals, uint64_t k, int flags, bsm_tiled** out, hipStream_t s, uint64_t reserve,
                 PlanTimes* pt) {
    BSM_REQUIRE(out && rp && (nnz == 0 || (col && vals)), BSM_ERR_INVALID, "tiled: null argument");
    BSM_REQUIRE(k == 32 || k == 1, BSM_ERR_UNSUPPORTED, "tiled: k must be 32 or 1");
    BSM_REQUIRE(dtype == BSM_F64 || dtype == BSM_F32, BSM_ERR_UNSUPPORTED, "tiled: f64 or f32 only");
    const bool f32 = dtype == BSM_F32;
    const size_t es = f32 ? 4 : 8;
    // k = 32 on 2^24 columns or more: 64-bit meta words (col << 8 | row)
    const bool wide = k == 32 && n_cols >= (1ull << 24);
    const size_t mb = wide ? 8 : 4;
    const uint32_t rbits = k == 1 ? K1_RBITS : 8;
    BSM_REQUIRE(k == 32 ? n_cols <= 0x7fffffffull : n_cols < (1ull << (32 - rbits)), BSM_ERR_UNSUPPORTED,
                "tiled: columns must be < 2^%u", k == 32 ? 31u : 32 - rbits);
    *out = nullptr;
    int dev = 0;
    BSM_TRY(current_device(&dev));
    int cus = 0;
    BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // a CU-masked stream (multi.hip leaves CUs to the all-gathers): one
    // workgroup per CU the stream may use, so the persistent grid stays resident
    if (s && cus > 0) {
        std::vector<uint32_t> mk((size_t)(cus + 31) / 32, 0u);
        if (hipExtStreamGetCUMask(s, (uint32_t)mk.size(), mk.data()) == hipSuccess) {
            int n = 0;
            for (int i = 0; i < cus; ++i) n += (mk[i / 32] >> (i % 32)) & 1u;
            if (n > 0 && n < cus) cus = n;
        } else {
            (void)hipGetLastError();
        }
    }
    const uint32_t wpc = k == 1 ? K1_WAVES_PER_CU : 4u;
    const uint32_t nw_env = env_u32("BSM_TILED_WAVES", wpc * (uint32_t)cus);
    const uint32_t nw = nw_env;
    const uint32_t k1_stage = env_u32("BSM_TILED_K1_STAGE", K1_STAGE_DEFAULT) == 8 ? 8u : 4u;
    const uint32_t rw_cap =
        k == 1 ? K1_RW_MAX : (f32 ? RW_MAX_F32 : RW_MAX);
    uint32_t rw_max = env_u32("BSM_TILED_RW", rw_cap);
    rw_max = rw_max < 8u ? 8u : (rw_max > rw_cap ? rw_cap : rw_max);
    const uint32_t pshift = env_u32("BSM_TILED_PSHIFT", k == 1 ? K1_PSHIFT : PSHIFT);
    const double pace = 1.0 + env_u32("BSM_TILED_PACE_PCT", PACE_PCT) / 100.0;
    const uint32_t pad = k == 1 ? 1u : PHASES;  // k = 1 runs a task's tail chunks unpipelined
    const uint32_t overread = k == 1 ? 2 * k1_stage : OVERREAD;
    BSM_REQUIRE(nw >= wpc && nw % wpc == 0 && pshift < 32, BSM_ERR_INVALID, "tiled: bad geometry");
    const uint64_t rpw64 = (rows + nw - 1) / nw;
    BSM_REQUIRE(rpw64 < (1ull << 31), BSM_ERR_UNSUPPORTED, "tiled: too many rows per wave");
    const uint32_t rpw = rpw64 ? (uint32_t)rpw64 : 1u;
    const uint32_t nb = (rpw + rw_max - 1) / rw_max;
    const uint32_t rw = (rpw + nb - 1) / nb;  // equal batches
    const uint64_t tasks = (uint64_t)nw * nb;

    DBuf counts, offs, ws;
    BSM_TRY(counts.alloc(tasks * sizeof(int32_t)));
    BSM_TRY(offs.alloc((tasks + 1) * sizeof(int64_t)));
    const uint64_t grid = (tasks + 3) / 4;
    auto layout = [&](auto write_tag, int32_t* cnt, const int64_t* of, void* me, void* va) -> int {
        constexpr bool W = decltype(write_tag)::value;
        auto go = [&]<typename V, typename MT>(V*, MT*) {
            if (k == 1)
                tiled_layout<W, (K1_RW_MAX + 1) / WAVE, V, MT><<<dim3((unsigned)grid), 256, 0, s>>>(
                    rows, n_cols, pace, rbits, pad, rp, col, static_cast<const V*>(vals), nw, rpw, nb, rw, pshift,
                    cnt, of, static_cast<MT*>(me), static_cast<V*>(va));
            else if (rw_cap > 192)  // f32 batches up to 255 rows: four row slots per lane
                tiled_layout<W, 4, V, MT><<<dim3((unsigned)grid), 256, 0, s>>>(
                    rows, n_cols, pace, rbits, pad, rp, col, static_cast<const V*>(vals), nw, rpw, nb, rw, pshift,
                    cnt, of, static_cast<MT*>(me), static_cast<V*>(va));
            else
                tiled_layout<W, 3, V, MT><<<dim3((unsigned)grid), 256, 0, s>>>(
                    rows, n_cols, pace, rbits, pad, rp, col, static_cast<const V*>(vals), nw, rpw, nb, rw, pshift,
                    cnt, of, static_cast<MT*>(me), static_cast<V*>(va));
        };
        if (f32 && wide) go((float*)nullptr, (uint64_t*)nullptr);
        else if (f32) go((float*)nullptr, (uint32_t*)nullptr);
        else if (wide) go((double*)nullptr, (uint64_t*)nullptr);
        else go((double*)nullptr, (uint32_t*)nullptr);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    };
    // phase timers (bsm_mcsr_prepare's plan_ms): host clock around each
    // phase, the stream synchronised at its end (the phases are long)
    auto t_phase = host_now();
    auto phase_end = [&](double* acc) -> int {
        if (!pt) return BSM_OK;
        BSM_HIP_TRY(hipStreamSynchronize(s));
        *acc += ms_since(t_phase);
        t_phase = host_now();
        return BSM_OK;
    };
    BSM_TRY(layout(std::false_type{}, counts.as<int32_t>(), nullptr, nullptr, nullptr));
    BSM_TRY(phase_end(pt ? &pt->count_ms : nullptr));
    const uint64_t wsb = scan_workspace_bytes(tasks);
    BSM_TRY(ws.alloc(wsb));
    BSM_TRY(exclusive_scan_i32_to_i64(counts.as<int32_t>(), offs.as<int64_t>(), tasks, ws.p, wsb, s));
    int64_t total = 0;
    BSM_HIP_TRY(read_dev(&total, offs.as<int64_t>() + tasks, sizeof(total), s));
    BSM_TRY(phase_end(pt ? &pt->scan_ms : nullptr));
    // a stream much longer than the matrix means rows too uneven for 64-row chunks
    BSM_REQUIRE((flags & BSM_TILED_ANY_PADDING) ||
                    (uint64_t)total * CHUNK <= nnz + nnz / 4 + tasks * pad * CHUNK + (uint64_t)CHUNK * 64,
                BSM_ERR_UNSUPPORTED, "tiled: %lld chunks for %llu entries (rows too uneven)", (long long)total,
                (unsigned long long)nnz);
    const uint64_t slots = ((uint64_t)total + overread) * CHUNK;
    size_t free_b = 0, total_b = 0;
    BSM_HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    BSM_REQUIRE(slots * (mb + es) + (256ull << 20) + reserve < free_b, BSM_ERR_OOM,
                "tiled: %llu MB stream (+%llu MB reserved) does not fit", (unsigned long long)(slots * (mb + es) >> 20),
                (unsigned long long)(reserve >> 20));
    DBuf meta, val, bar;
    BSM_TRY(bar.alloc(8 * BAR_STRIDE * sizeof(unsigned)));
    BSM_TRY(meta.alloc(slots * mb));
    BSM_TRY(val.alloc(slots * es));
    BSM_TRY(phase_end(pt ? &pt->alloc_ms : nullptr));
    BSM_TRY(layout(std::true_type{}, nullptr, offs.as<int64_t>(), meta.p, val.p));
    // over-read padding: valid dummy entries (X row 0)
    BSM_HIP_TRY(hipMemsetAsync(static_cast<char*>(meta.p) + (uint64_t)total * CHUNK * mb, 0, overread * CHUNK * mb, s));
    BSM_HIP_TRY(hipMemsetAsync(static_cast<char*>(val.p) + (uint64_t)total * CHUNK * es, 0, overread * CHUNK * es, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_TRY(phase_end(pt ? &pt->write_ms : nullptr));
    auto* t = new bsm_tiled;
    t->device = dev;
    t->dtype = dtype;
    t->k = k;
    t->rows = rows;
    t->n_cols = n_cols;
    t->nnz = nnz;
    t->nw = nw;
    t->rpw = rpw;
    t->nb = nb;
    t->rw = rw;
    t->pshift = pshift;
    t->chunks = (uint64_t)total;
    t->overread = overread;
    t->stage = k1_stage;
    t->offs = static_cast<int64_t*>(offs.release());
    t->meta_bytes = (uint32_t)mb;
    t->meta = meta.release();
    t->val = val.release();
    t->bar = static_cast<unsigned*>(bar.release());
    *out = t;
    return BSM_OK;
}

int tiled_spmm(const bsm_tiled* t, const void* x, void* y, int32_t* row_nnz, bool neg_init, hipStream_t s) {
    BSM_REQUIRE(t && (t->rows == 0 || (x && y)), BSM_ERR_INVALID, "tiled: null argument");
    BSM_REQUIRE(!neg_init || t->k == 1, BSM_ERR_INVALID, "tiled: -0 init only for k = 1");
    if (t->rows == 0) return BSM_OK;
    unsigned* bar = nullptr;
    if (t->bar && t->nb > 1 && env_u32("BSM_TILED_SYNC", 1)) {
        BSM_HIP_TRY(hipMemsetAsync(t->bar, 0, 8 * BAR_STRIDE * sizeof(unsigned), s));
        bar = t->bar;
    }
    // BSM_TILED_K1_PROBE=<mask> (measurement only, wrong results): gather
    // X[col & mask], e.g. 0 (one line: the stream alone) or 4095 (a 32 KB window)
    static const uint32_t k1mask = env_u32("BSM_TILED_K1_PROBE", 0xffffffffu);
    if (t->k == 1 && t->dtype == BSM_F32) {
        const size_t lds = (size_t)4 * (t->rw + 1) * sizeof(float);
        auto kern = t->stage == 8 ? spmm_tiled_k1<8, float> : spmm_tiled_k1<4, float>;
        kern<<<dim3(t->nw / 4), 256, lds, s>>>(t->rows, t->rpw, t->nb, t->rw, t->offs,
                                              static_cast<const uint32_t*>(t->meta),
                                              static_cast<const float*>(t->val), static_cast<const float*>(x),
                                              static_cast<float*>(y), row_nnz, bar, neg_init, k1mask);
    } else if (t->k == 1) {
        const size_t lds = (size_t)4 * (t->rw + 1) * sizeof(double);
        auto kern = t->stage == 8 ? spmm_tiled_k1<8> : spmm_tiled_k1<4>;
        kern<<<dim3(t->nw / 4), 256, lds, s>>>(t->rows, t->rpw, t->nb, t->rw, t->offs,
                                              static_cast<const uint32_t*>(t->meta),
                                              static_cast<const double*>(t->val), static_cast<const double*>(x),
                                              static_cast<double*>(y), row_nnz, bar, neg_init, k1mask);
    } else if (t->dtype == BSM_F32) {  // k = 32, f32: 128-B rows, up to 255 per batch
        const size_t lds = (size_t)4 * (t->rw + 1) * 128;
        // BSM_TILED_SPINS: the batch barrier's poll bound (default 4000 polls
        // of s_sleep 8, ~0.9 ms; A/B for the f32 batches, ~3x longer)
        static const uint32_t spins = env_u32("BSM_TILED_SPINS", 4000);
        if (t->meta_bytes == 8)
            spmm_tiled_k32_f32<uint64_t><<<dim3(t->nw / 4), 256, lds, s>>>(
                t->rows, t->rpw, t->nb, t->rw, t->offs, static_cast<const uint64_t*>(t->meta),
                static_cast<const float*>(t->val), static_cast<const F2*>(x), static_cast<F2*>(y), row_nnz,
                bar, 0xffffffffu, spins);
        else
            spmm_tiled_k32_f32<uint32_t><<<dim3(t->nw / 4), 256, lds, s>>>(
                t->rows, t->rpw, t->nb, t->rw, t->offs, static_cast<const uint32_t*>(t->meta),
                static_cast<const float*>(t->val), static_cast<const F2*>(x), static_cast<F2*>(y), row_nnz,
                bar, 0xffffffffu, spins);
    } else {
        const size_t lds = (size_t)4 * (t->rw + 1) * 256;
        // BSM_TILED_PROBE_MASK=<mask> (measurement only, wrong results): see gather()
        static const uint32_t xmask = env_u32("BSM_TILED_PROBE_MASK", 0xffffffffu);
        auto kern = xmask != 0xffffffffu ? spmm_tiled_k32<true>
                                         : spmm_tiled_k32<false>;
        static const uint32_t spins = env_u32("BSM_TILED_SPINS", 4000);
        if (t->meta_bytes == 8)  // 2^24 columns or more
            spmm_tiled_k32<false, double, uint64_t><<<dim3(t->nw / 4), 256, lds, s>>>(
                t->rows, t->rpw, t->nb, t->rw, t->offs, static_cast<const uint64_t*>(t->meta),
                static_cast<const double*>(t->val), static_cast<const double2*>(x), static_cast<double2*>(y), row_nnz,
                bar, 0xffffffffu, spins);
        else
            kern<<<dim3(t->nw / 4), 256, lds, s>>>(t->rows, t->rpw, t->nb, t->rw, t->offs,
                                                  static_cast<const uint32_t*>(t->meta),
                                                  static_cast<const double*>(t->val), static_cast<const double2*>(x),
                                                  static_cast<double2*>(y), row_nnz, bar, xmask, spins);
    }
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

void tiled_destroy(bsm_tiled* t) {
    if (!t) return;
    if (t->offs) (void)hipFree(t->offs);
    if (t->meta) (void)hipFree(t->meta);
    if (t->val) (void)hipFree(t->val);
    if (t->bar) (void)hipFree(t->bar);
    delete t;
}

}  // namespace bsm
