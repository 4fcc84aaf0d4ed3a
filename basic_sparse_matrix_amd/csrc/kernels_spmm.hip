// kernels_spmm.hip -- gfx950 kernels of Csr::mul_dense / mul_vector
// (reference: src/sparse.rs:426-482) and their compaction into the
// reference's output Csr, plus the device-wide scan they share.
//
// Summation order. The reference sums each output element sequentially in
// the row's storage order starting from T::default() (sparse.rs:434-440) and
// never fuses multiply-add. Every kernel here keeps exactly that order per
// output element (lanes own output columns; products of one column are
// combined in entry order), so f32/f64 results are bit-identical to the
// reference, not merely within tolerance. See DESIGN.md "SpMM kernels".
#include "bsm_internal.hpp"
#include "bsm_synth.h"

#include <cstdlib>
#include <type_traits>

namespace bsm {
namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ uint64_t lanemask_lt(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// first r in [0, n) with rp[r] >= v, else n
__device__ __forceinline__ int64_t lower_bound_rp(const int64_t* rp, int64_t n, int64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (rp[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// The same, searched by a whole wavefront: 64 probes per step, so
// ceil(log64 n) dependent loads instead of log2 n. Call from all 64 lanes;
// the result is the same in every lane.
__device__ __forceinline__ int64_t wave_lower_bound_rp(const int64_t* rp, int64_t n, int64_t v) {
    const int lane = threadIdx.x & (WAVE - 1);
    int64_t lo = 0, hi = n;  // answer in [lo, hi]
    while (lo < hi) {
        const int64_t step = (hi - lo + WAVE - 1) / WAVE;
        const int64_t pos = lo + (int64_t)lane * step;
        const bool ge = pos >= hi || rp[pos] >= v;
        const uint64_t m = __ballot(ge);
        const int f = m ? __builtin_ctzll(m) : WAVE;  // first probe at or past the answer
        if (f == 0) break;                             // rp[lo] >= v
        const int64_t nlo = lo + (int64_t)(f - 1) * step + 1;
        hi = min<int64_t>(hi, lo + (int64_t)f * step);
        lo = nlo;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// Exclusive scan int32 -> int64 (n+1 outputs; out[n] = total).
// Three launches: per-tile sums, scan of tile sums (one workgroup), apply.
// ---------------------------------------------------------------------------
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t* smem, int64_t* total) {
    // smem: SCAN_BLOCK entries. Hillis-Steele over 256 threads.
    const int t = threadIdx.x;
    smem[t] = v;
    __syncthreads();
    for (int off = 1; off < SCAN_BLOCK; off <<= 1) {
        int64_t add = (t >= off) ? smem[t - off] : 0;
        __syncthreads();
        smem[t] += add;
        __syncthreads();
    }
    int64_t incl = smem[t];
    *total = smem[SCAN_BLOCK - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(SCAN_BLOCK) void scan_tile_sums(const int32_t* in, uint64_t n,
                                                             int64_t* tile_sums) {
    __shared__ int64_t red[SCAN_BLOCK];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    int64_t acc = 0;
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint64_t idx = base + (uint64_t)i * SCAN_BLOCK + threadIdx.x;
        if (idx < n) acc += in[idx];
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = SCAN_BLOCK / 2; off > 0; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(SCAN_BLOCK) void scan_tile_prefix(int64_t* tile_sums, uint64_t n_tiles) {
    __shared__ int64_t smem[SCAN_BLOCK];
    int64_t carry = 0;
    for (uint64_t base = 0; base < n_tiles; base += SCAN_BLOCK) {
        uint64_t idx = base + threadIdx.x;
        int64_t v = idx < n_tiles ? tile_sums[idx] : 0;
        int64_t total;
        int64_t ex = block_exclusive_scan(v, smem, &total);
        if (idx < n_tiles) tile_sums[idx] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) tile_sums[n_tiles] = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void scan_apply(const int32_t* in, uint64_t n,
                                                         const int64_t* tile_prefix, int64_t* out) {
    __shared__ int64_t smem[SCAN_BLOCK];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    // each thread owns SCAN_ITEMS consecutive elements
    int32_t v[SCAN_ITEMS];
    int64_t local = 0;
    const uint64_t my0 = base + (uint64_t)threadIdx.x * SCAN_ITEMS;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint64_t idx = my0 + i;
        v[i] = idx < n ? in[idx] : 0;
        local += v[i];
    }
    int64_t total;
    int64_t ex = block_exclusive_scan(local, smem, &total) + tile_prefix[blockIdx.x];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint64_t idx = my0 + i;
        if (idx < n) out[idx] = ex;
        ex += v[i];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = tile_prefix[gridDim.x];
}

// n <= SCAN_TILE (the small calls: C1's 1,024 rows): the whole scan in one
// launch instead of three
__global__ __launch_bounds__(SCAN_BLOCK) void scan_one_tile(const int32_t* in, uint64_t n, int64_t* out) {
    __shared__ int64_t smem[SCAN_BLOCK];
    int32_t v[SCAN_ITEMS];
    int64_t local = 0;
    const uint64_t my0 = (uint64_t)threadIdx.x * SCAN_ITEMS;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t idx = my0 + i;
        v[i] = idx < n ? in[idx] : 0;
        local += v[i];
    }
    int64_t total;
    int64_t ex = block_exclusive_scan(local, smem, &total);
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t idx = my0 + i;
        if (idx < n) out[idx] = ex;
        ex += v[i];
    }
    if (threadIdx.x == 0) out[n] = total;
}

__global__ void write_zero_i64(int64_t* p) { *p = 0; }

// ---------------------------------------------------------------------------
// SpMM, lanes own output columns ("row-wave"): one wavefront per CSR row.
// KL = lanes per entry group (power of two >= min(k,64)); S = 64/KL entries
// are gathered per wave instruction, U groups are kept in flight. Lane
// (s, c) multiplies entry e0+u*S+s by X[col][cb+c]; the S products of a
// column are then added to that column's accumulator in entry order via
// cross-lane reads, so every lane of column c holds the same, in-order sum.
// For k = 32 f64 one wave instruction gathers two 256-B X rows.
// ---------------------------------------------------------------------------
template <typename T, int KL, int U>
__global__ __launch_bounds__(256) void spmm_rowwave(int64_t rows, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const T* __restrict__ val, int k,
                                                    const T* __restrict__ X, T* __restrict__ Y,
                                                    int32_t* __restrict__ row_nnz) {
    using A = Arith<T>;
    constexpr int S = WAVE / KL;
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x / WAVE);
    if (row >= rows) return;  // wave-uniform
    const int s = lane / KL;
    const int c = lane % KL;
    const int64_t start = rp[row], end = rp[row + 1];
    int nz_count = 0;
    for (int cb = 0; cb < k; cb += KL) {
        const int jc = cb + c;
        const bool cval = jc < k;
        T acc = A::zero();
        for (int64_t e0 = start; e0 < end; e0 += (int64_t)S * U) {
            T p[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t e = e0 + (int64_t)u * S + s;
                T pr = A::zero();
                if (e < end && cval) {
                    const int64_t cc = col[e];
                    pr = A::mul(val[e], X[cc * k + jc]);
                }
                p[u] = pr;
            }
            // number of real entries in this step (wave-uniform); padding
            // products are +0 and only ever trail the real ones, and the
            // accumulator is never -0, so they cannot change the sum.
            const int64_t left = end - e0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (S == 1) {
                    acc = A::add(acc, p[u]);
                } else {
                    int nv = (int)min<int64_t>(S, left - (int64_t)u * S);
                    for (int t = 0; t < nv; ++t) acc = A::add(acc, __shfl(p[u], t * KL + c, WAVE));
                }
            }
        }
        if (s == 0 && cval) Y[row * (int64_t)k + jc] = acc;
        const uint64_t m = __ballot(s == 0 && cval && A::nz(acc));
        nz_count += __popcll(m);
    }
    if (lane == 0 && row_nnz) row_nnz[row] = nz_count;
}

// ---------------------------------------------------------------------------
// SpMM specialised for f64 with k = 32 (the C3/C4 shape): one wavefront per
// CSR row; lane l = 16*g + q gathers the 16-byte pair X[col_e][2q..2q+1] of
// entry e = e0 + 4u + g, so ONE global_load_dwordx4 wave instruction fetches
// four whole 256-B X rows. The four products of a column pair are
// brought to the group-0 lanes with v_permlane16/32_swap (no LDS) and added
// in entry order: own (g0), lane^16 (g1), lane^32 (g2), lane^48 (g3).
// Per 4 entries: 1 gather + 2 index/value loads (VMEM), 12 permlanes, 8 adds.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double from_u2(unsigned lo, unsigned hi) {
    return __hiloint2double((int)hi, (int)lo);
}
// value of lane^16 (valid in even 16-lane rows, i.e. lanes 0-15 and 32-47)
__device__ __forceinline__ double xchg16_even(double v) {
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return from_u2(rl[1], rh[1]);
}
// value of lane^32 (valid in lanes 0-31)
__device__ __forceinline__ double xchg32_low(double v) {
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return from_u2(rl[1], rh[1]);
}

//
// PANEL = one pass of the column-panel schedule (spmm_panelled below): the
// row's entries are cut at panel boundaries, seg_lo/seg_hi give the pass's
// entry range relative to the row start (nullptr = row start / row end) and a
// pass other than the first resumes the running sums from Y. Carrying the
// f64 sum through Y is exact, so the per-element order is unchanged.
template <int STEPS, bool PIPE, bool PANEL = false>
__global__ __launch_bounds__(256) void spmm_k32_f64(int64_t rows, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const double* __restrict__ val,
                                                    const double2* __restrict__ X,
                                                    double2* __restrict__ Y,
                                                    int32_t* __restrict__ row_nnz,
                                                    const int32_t* __restrict__ seg_lo = nullptr,
                                                    const int32_t* __restrict__ seg_hi = nullptr) {
    constexpr int CH = 4 * STEPS;  // entries per iteration
    const int lane = threadIdx.x & (WAVE - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / WAVE) + wave;
    if (row >= rows) return;
    const int g = lane >> 4, q = lane & 15;
    int64_t start = rp[row], end = rp[row + 1];
    double a0 = 0.0, a1 = 0.0;
    if constexpr (PANEL) {
        if (seg_hi) end = start + seg_hi[row];
        if (seg_lo) {
            start += seg_lo[row];
            const double2 y0 = Y[row * 16 + q];
            a0 = y0.x;
            a1 = y0.y;
        }
    }
    int64_t e0 = start;
    // each lane loads the index/value of ITS entry (4 distinct addresses per
    // wave instruction, one cache line)
    int32_t c[STEPS];
    double v[STEPS];
    if (PIPE && e0 + CH <= end) {
#pragma unroll
        for (int u = 0; u < STEPS; ++u) { c[u] = col[e0 + 4 * u + g]; v[u] = val[e0 + 4 * u + g]; }
    }
    for (; e0 + CH <= end; e0 += CH) {  // full chunks
        if (!PIPE) {
#pragma unroll
            for (int u = 0; u < STEPS; ++u) { c[u] = col[e0 + 4 * u + g]; v[u] = val[e0 + 4 * u + g]; }
        }
        double2 x[STEPS];
#pragma unroll
        for (int u = 0; u < STEPS; ++u) x[u] = X[(int64_t)c[u] * 16 + q];
        double vc[STEPS];
#pragma unroll
        for (int u = 0; u < STEPS; ++u) vc[u] = v[u];
        if (PIPE && e0 + 2 * CH <= end) {  // software pipeline: next chunk's indices
#pragma unroll
            for (int u = 0; u < STEPS; ++u) {
                c[u] = col[e0 + CH + 4 * u + g];
                v[u] = val[e0 + CH + 4 * u + g];
            }
        }
#pragma unroll
        for (int u = 0; u < STEPS; ++u) {
            const double vv = vc[u];
            const double p0 = __dmul_rn(vv, x[u].x), p1 = __dmul_rn(vv, x[u].y);
            const double p0_16 = xchg16_even(p0), p1_16 = xchg16_even(p1);
            const double p0_32 = xchg32_low(p0), p1_32 = xchg32_low(p1);
            const double p0_48 = xchg32_low(p0_16), p1_48 = xchg32_low(p1_16);
            a0 = __dadd_rn(a0, p0); a1 = __dadd_rn(a1, p1);
            a0 = __dadd_rn(a0, p0_16); a1 = __dadd_rn(a1, p1_16);
            a0 = __dadd_rn(a0, p0_32); a1 = __dadd_rn(a1, p1_32);
            a0 = __dadd_rn(a0, p0_48); a1 = __dadd_rn(a1, p1_48);
        }
    }
    for (; e0 < end; e0 += 4) {  // tail: < CH entries, 4 at a time, clamped
        const int64_t e = min<int64_t>(e0 + g, end - 1);
        const int nv = (int)min<int64_t>(4, end - e0);
        const double2 x = X[(int64_t)col[e] * 16 + q];
        const double vv = val[e];
        const double p0 = __dmul_rn(vv, x.x), p1 = __dmul_rn(vv, x.y);
        const double p0_16 = xchg16_even(p0), p1_16 = xchg16_even(p1);
        const double p0_32 = xchg32_low(p0), p1_32 = xchg32_low(p1);
        const double p0_48 = xchg32_low(p0_16), p1_48 = xchg32_low(p1_16);
        a0 = __dadd_rn(a0, p0); a1 = __dadd_rn(a1, p1);
        if (nv > 1) { a0 = __dadd_rn(a0, p0_16); a1 = __dadd_rn(a1, p1_16); }
        if (nv > 2) { a0 = __dadd_rn(a0, p0_32); a1 = __dadd_rn(a1, p1_32); }
        if (nv > 3) { a0 = __dadd_rn(a0, p0_48); a1 = __dadd_rn(a1, p1_48); }
    }
    if (g == 0) Y[row * 16 + q] = make_double2(a0, a1);
    const uint64_t m0 = __ballot(g == 0 && a0 != 0.0), m1 = __ballot(g == 0 && a1 != 0.0);
    if (lane == 0 && row_nnz) row_nnz[row] = __popcll(m0) + __popcll(m1);
}

// k = 32, f64, SHORT rows (C3: 10 entries): four CSR rows per wavefront, one
// per 16-lane group. Lane q of group g owns Y[row][2q..2q+1] and walks its
// row's entries in storage order (sequential sums, no cross-lane combine);
// a wave instruction still gathers four whole 256-B X rows, one per group.
// U entries per group are in flight per iteration (clamped, unconditional
// loads); the wave runs to the longest of its four rows.
// PROBE (measurement only, wrong results; BSM_SPMM_PROBE_MASK): every gather
// reads X row (col & xmask), e.g. 0: the PMC calibration of the col / val
// stream alone (the gathers all hit one line).
template <int U, bool PROBE = false>
__global__ __launch_bounds__(256) void spmm_k32_f64_rows4(int64_t rows, const int64_t* __restrict__ rp,
                                                          const int32_t* __restrict__ col,
                                                          const double* __restrict__ val,
                                                          const double2* __restrict__ X,
                                                          double2* __restrict__ Y,
                                                          int32_t* __restrict__ row_nnz, uint32_t xmask = ~0u) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int g = lane >> 4, q = lane & 15;
    const int64_t row = ((int64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE) * 4 + g;
    const bool live = row < rows;
    int64_t start = 0, len = 0;
    if (live) {
        start = rp[row];
        len = rp[row + 1] - start;
    }
    long long m = len;  // longest row of the wave
    m = max(m, (long long)__shfl_xor(m, 16));
    m = max(m, (long long)__shfl_xor(m, 32));
    double a0 = 0.0, a1 = 0.0;
    for (int64_t b = 0; b < m; b += U) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = len ? start + min<int64_t>(b + u, len - 1) : 0;  // nnz > 0 here
            c[u] = col[e];
            v[u] = val[e];
        }
        double2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = X[(int64_t)(PROBE ? (uint32_t)c[u] & xmask : (uint32_t)c[u]) * 16 + q];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double s0 = __dadd_rn(a0, __dmul_rn(v[u], x[u].x));
            const double s1 = __dadd_rn(a1, __dmul_rn(v[u], x[u].y));
            const bool in = b + u < len;
            a0 = in ? s0 : a0;
            a1 = in ? s1 : a1;
        }
    }
    if (live) Y[row * 16 + q] = make_double2(a0, a1);
    const uint64_t m0 = __ballot(live && a0 != 0.0), m1 = __ballot(live && a1 != 0.0);
    if (q == 0 && live && row_nnz)
        row_nnz[row] = __popcll((m0 >> (16 * g)) & 0xffffull) + __popcll((m1 >> (16 * g)) & 0xffffull);
}

// Column-panel plan: seg[(p-1)*rows + r] = offset (from the row start) of
// the first entry of row r whose column lies in panel p = col / panel_cols,
// for p = 1 .. n_panels-1. One wavefront per row; lane e finds the panels
// that start at its entry. *bad |= 1 if a row's panels are not
// non-decreasing in storage order (the schedule would reorder its sum),
// |= 2 if a row is longer than int32.
__global__ __launch_bounds__(256) void spmm_plan_panels(int64_t rows, const int64_t* __restrict__ rp,
                                                        const int32_t* __restrict__ col,
                                                        uint32_t panel_cols, int n_panels,
                                                        int32_t* __restrict__ seg,
                                                        unsigned* __restrict__ bad) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    if (row >= rows) return;
    const int64_t start = rp[row], end = rp[row + 1];
    if (end - start > INT32_MAX) {
        if (lane == 0) atomicOr(bad, 2u);
        return;
    }
    const int last = n_panels - 1;
    for (int64_t e = start + lane; e < end; e += WAVE) {
        const int pe = (int)min<uint32_t>((uint32_t)col[e] / panel_cols, (uint32_t)last);
        const int pp = e > start ? (int)min<uint32_t>((uint32_t)col[e - 1] / panel_cols, (uint32_t)last) : 0;
        if (pe < pp) atomicOr(bad, 1u);
        for (int p = pp + 1; p <= pe; ++p) seg[(int64_t)(p - 1) * rows + row] = (int32_t)(e - start);
    }
    if (lane == 0) {  // panels after the row's last entry (all of them for an empty row)
        const int pl = end > start ? (int)min<uint32_t>((uint32_t)col[end - 1] / panel_cols, (uint32_t)last) : 0;
        for (int p = pl + 1; p <= last; ++p) seg[(int64_t)(p - 1) * rows + row] = (int32_t)(end - start);
    }
}

// ---------------------------------------------------------------------------
// SpMV (k = 1), CSR-stream with in-order row sums. Workgroup b owns the rows
// whose first entry lies in [b*CHUNK, (b+1)*CHUNK); their products are
// computed with coalesced col/val loads into LDS, then one thread per row
// adds its row's products in storage order (bit-exact). A workgroup whose
// entry range exceeds LDS (it holds a row longer than CHUNK) falls back to
// thread-per-row sums for short rows and a workgroup-wide pass per long row.
// init = +0 for mul_dense (T::default()), -0 for mul_vector (float Sum).
// ---------------------------------------------------------------------------
template <typename T, int ITEMS>
__global__ __launch_bounds__(256) void spmv_stream(int64_t rows, int64_t nnz,
                                                   const int64_t* __restrict__ rp,
                                                   const int32_t* __restrict__ col,
                                                   const T* __restrict__ val,
                                                   const T* __restrict__ x, T* __restrict__ y,
                                                   int32_t* __restrict__ row_nnz, bool neg_init) {
    using A = Arith<T>;
    constexpr int CHUNK = 256 * ITEMS, CAP = 2 * CHUNK;
    __shared__ T prod[CAP];
    __shared__ int64_t s_r[2];
    const int64_t lo = (int64_t)blockIdx.x * CHUNK;
    const int64_t hi = lo + CHUNK;
    const int wave = threadIdx.x / WAVE;  // waves 0 and 1 find the two row bounds
    if (wave == 0) {
        const int64_t r = wave_lower_bound_rp(rp, rows, lo);
        if (threadIdx.x == 0) s_r[0] = r;
    } else if (wave == 1) {
        const int64_t r = hi > nnz ? rows : wave_lower_bound_rp(rp, rows, hi);
        if (threadIdx.x == WAVE) s_r[1] = r;
    }
    __syncthreads();
    const int64_t r0 = s_r[0], r1 = s_r[1];
    if (r0 >= r1) return;
    const T init = neg_init ? A::neg_zero() : A::zero();
    const int64_t e0 = rp[r0], e1 = rp[r1];
    const int64_t n = e1 - e0;
    if (n <= CAP) {
        // this thread's first row bounds, in flight with the products
        const int64_t rr = r0 + threadIdx.x;
        int64_t ra = 0, rb = 0;
        if (rr < r1) {
            ra = rp[rr];
            rb = rp[rr + 1];
        }
        // products: ITEMS coalesced col/val loads per thread issued together,
        // then ITEMS gathers (clamped indices, unconditional loads)
        for (int64_t base = 0; base < n; base += CHUNK) {
            int32_t c[ITEMS];
            T v[ITEMS];
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                const int64_t e = e0 + min<int64_t>(base + it * 256 + threadIdx.x, n - 1);
                c[it] = col[e];
                v[it] = val[e];
            }
            T xv[ITEMS];
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) xv[it] = x[c[it]];
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                const int64_t i = base + it * 256 + threadIdx.x;
                if (i < n) prod[i] = A::mul(v[it], xv[it]);
            }
        }
        __syncthreads();
        for (int64_t r = rr; r < r1; r += blockDim.x) {
            const int64_t a = (r == rr ? ra : rp[r]) - e0, b = (r == rr ? rb : rp[r + 1]) - e0;
            T acc = init;
            for (int64_t i = a; i < b; ++i) acc = A::add(acc, prod[i]);
            y[r] = acc;
            if (row_nnz) row_nnz[r] = A::nz(acc) ? 1 : 0;
        }
        return;
    }
    // fallback: block contains a row longer than CHUNK
    for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
        const int64_t a = rp[r], b = rp[r + 1];
        if (b - a > CHUNK) continue;
        T acc = init;
        for (int64_t e = a; e < b; ++e) acc = A::add(acc, A::mul(val[e], x[col[e]]));
        y[r] = acc;
        if (row_nnz) row_nnz[r] = A::nz(acc) ? 1 : 0;
    }
    for (int64_t r = r0; r < r1; ++r) {  // uniform loop over long rows
        const int64_t a = rp[r], b = rp[r + 1];
        if (b - a <= CHUNK) continue;
        T acc = init;
        for (int64_t cs = a; cs < b; cs += CAP) {
            const int64_t n = min<int64_t>(CAP, b - cs);
            __syncthreads();
            for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
                const int64_t e = cs + i;
                prod[i] = A::mul(val[e], x[col[e]]);
            }
            __syncthreads();
            if (threadIdx.x == 0)
                for (int64_t i = 0; i < n; ++i) acc = A::add(acc, prod[i]);
        }
        if (threadIdx.x == 0) {
            y[r] = acc;
            if (row_nnz) row_nnz[r] = A::nz(acc) ? 1 : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// SpMV (k = 1), rows-blocked: workgroup b owns rows [256b, 256b + 256), one
// per thread. Its entry range [rp[r0], rp[r1]) is swept in chunks of
// 256 * ITEMS entries: coalesced col/val loads and the x gathers of a chunk
// are all in flight together, the products land in LDS, and each thread then
// adds the part of its row that lies in the chunk, in storage order, onto its
// running sum (chunks ascend, so the per-row order is the reference's,
// sparse.rs:434-440). No search: the row bounds are direct loads, so a
// workgroup is three dependent memory round trips (row bounds -> entries ->
// x) instead of spmv_stream's binary search in front of them. A long row is
// summed by its one thread across chunks (order kept, slower); rows this
// long on average go to spmv_stream instead.
// ---------------------------------------------------------------------------
template <typename T, int ITEMS>
__global__ __launch_bounds__(256) void spmv_rows(int64_t rows, const int64_t* __restrict__ rp,
                                                 const int32_t* __restrict__ col, const T* __restrict__ val,
                                                 const T* __restrict__ x, T* __restrict__ y,
                                                 int32_t* __restrict__ row_nnz, bool neg_init) {
    using A = Arith<T>;
    constexpr int CAP = 256 * ITEMS;
    __shared__ T prod[CAP];
    const int tid = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    const int64_t r1 = r0 + 256 < rows ? r0 + 256 : rows;
    const int64_t rr = r0 + tid;
    const bool live = rr < r1;
    // the workgroup's entry range and this thread's row, loaded together
    const int64_t e0 = rp[r0], e1 = rp[r1];
    const int64_t ra = live ? rp[rr] : e1, rb = live ? rp[rr + 1] : e1;
    T acc = neg_init ? A::neg_zero() : A::zero();
    for (int64_t base = e0; base < e1; base += CAP) {
        const int64_t n = e1 - base < CAP ? e1 - base : CAP;
        const int nit = (int)((n + 255) / 256);  // uniform over the workgroup
        int32_t c[ITEMS];
        T v[ITEMS];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (it < nit) {
                const int64_t e = base + min<int64_t>(it * 256 + tid, n - 1);
                c[it] = col[e];
                v[it] = val[e];
            }
        T xv[ITEMS];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (it < nit) xv[it] = x[c[it]];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (it < nit && it * 256 + tid < n) prod[it * 256 + tid] = A::mul(v[it], xv[it]);
        __syncthreads();
        const int64_t a = ra > base ? ra : base, b = rb < base + n ? rb : base + n;
        for (int64_t i = a; i < b; ++i) acc = A::add(acc, prod[i - base]);
        __syncthreads();
    }
    if (live) {
        y[rr] = acc;
        if (row_nnz) row_nnz[rr] = A::nz(acc) ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// SpMV (k = 1), short rows, one WAVE per 64 rows: the rows' entries loaded
// coalesced (lane l takes entry e0 + l + 64 i), their products written to the
// wave's own LDS slice, then lane r adds row r's products in storage order.
// LDS operations of one wave complete in order, so no barrier is needed and
// the waves of a workgroup never wait for each other.
// ---------------------------------------------------------------------------
template <typename T, int ITEMS>
__global__ __launch_bounds__(256) void spmv_wave(int64_t rows, const int64_t* __restrict__ rp,
                                                 const int32_t* __restrict__ col, const T* __restrict__ val,
                                                 const T* __restrict__ x, T* __restrict__ y,
                                                 int32_t* __restrict__ row_nnz, bool neg_init) {
    using A = Arith<T>;
    constexpr int CAP = WAVE * ITEMS;
    __shared__ T prod_all[4][CAP];
    T* prod = prod_all[threadIdx.x / WAVE];
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + threadIdx.x / WAVE) * WAVE;
    if (r0 >= rows) return;
    const int64_t r1 = r0 + WAVE < rows ? r0 + WAVE : rows;
    const int64_t rr = r0 + lane;
    const bool live = rr < r1;
    const int64_t e0 = rp[r0], e1 = rp[r1];
    const int64_t ra = live ? rp[rr] : e1, rb = live ? rp[rr + 1] : e1;
    T acc = neg_init ? A::neg_zero() : A::zero();
    for (int64_t base = e0; base < e1; base += CAP) {
        const int64_t n = e1 - base < CAP ? e1 - base : CAP;
        const int nit = (int)((n + WAVE - 1) / WAVE);
        int32_t c[ITEMS];
        T v[ITEMS];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (it < nit) {
                const int64_t e = base + min<int64_t>(it * WAVE + lane, n - 1);
                c[it] = col[e];
                v[it] = val[e];
            }
        T xv[ITEMS];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (it < nit) xv[it] = x[c[it]];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (it < nit && it * WAVE + lane < n) prod[it * WAVE + lane] = A::mul(v[it], xv[it]);
        const int64_t a = ra > base ? ra : base, b = rb < base + n ? rb : base + n;
        for (int64_t i = a; i < b; ++i) acc = A::add(acc, prod[i - base]);
    }
    if (live) {
        y[rr] = acc;
        if (row_nnz) row_nnz[rr] = A::nz(acc) ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// SpMV (k = 1) for short rows (C2: 10 entries): one thread per row, the
// row's entries and their x gathers all in flight at once (U per pass,
// indices clamped into the row so every load is unconditional), then the
// products added in storage order in a register: no LDS, no barrier, two
// dependent memory round trips after the row bounds. Rows longer than U take
// more passes (the wave runs to its longest row).
// ---------------------------------------------------------------------------
template <typename T, int U>
__global__ __launch_bounds__(256) void spmv_thread(int64_t rows, const int64_t* __restrict__ rp,
                                                   const int32_t* __restrict__ col, const T* __restrict__ val,
                                                   const T* __restrict__ x, T* __restrict__ y,
                                                   int32_t* __restrict__ row_nnz, bool neg_init) {
    using A = Arith<T>;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int64_t a = rp[r], b = rp[r + 1];
    T acc = neg_init ? A::neg_zero() : A::zero();
    for (int64_t base = a; base < b; base += U) {
        const int n = (int)(b - base < U ? b - base : U);
        int32_t c[U];
        T v[U];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const int64_t e = base + (i < n ? i : n - 1);
            c[i] = col[e];
            v[i] = val[e];
        }
        T xv[U];
#pragma unroll
        for (int i = 0; i < U; ++i) xv[i] = x[c[i]];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const T t = A::add(acc, A::mul(v[i], xv[i]));
            acc = i < n ? t : acc;
        }
    }
    y[r] = acc;
    if (row_nnz) row_nnz[r] = A::nz(acc) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Compaction of dense Y (rows x k, row-major) into the output Csr: entry
// (r, j) is kept iff Y[r][j] != 0 (insert's zero skip, sparse.rs:229), in
// ascending j, at out_rp[r] + (kept entries of row r before j).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void compact_wave(int64_t rows, int k, const T* __restrict__ Y,
                                                    const int64_t* __restrict__ out_rp,
                                                    int32_t* __restrict__ out_col,
                                                    T* __restrict__ out_val) {
    using A = Arith<T>;
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x / WAVE);
    if (row >= rows) return;
    int64_t pos = out_rp[row];
    for (int cb = 0; cb < k; cb += WAVE) {
        const int j = cb + lane;
        T v = j < k ? Y[row * (int64_t)k + j] : A::zero();
        const bool keep = j < k && A::nz(v);
        const uint64_t m = __ballot(keep);
        if (keep) {
            const int64_t p = pos + __popcll(m & lanemask_lt(lane));
            out_col[p] = j;
            out_val[p] = v;
        }
        pos += __popcll(m);
    }
}

// k <= 32: KL = pow2 >= k lanes per row, 64 / KL rows per wave (C3's k = 32:
// two rows per wave instead of one with half the lanes idle)
template <typename T, int KL>
__global__ __launch_bounds__(256) void compact_seg(int64_t rows, int k, const T* __restrict__ Y,
                                                   const int64_t* __restrict__ out_rp, int32_t* __restrict__ out_col,
                                                   T* __restrict__ out_val) {
    using A = Arith<T>;
    const int lane = threadIdx.x & (WAVE - 1);
    const int j = lane & (KL - 1);
    const int64_t row = ((int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x / WAVE)) * (WAVE / KL) + lane / KL;
    const bool in = row < rows && j < k;
    const T v = in ? Y[row * (int64_t)k + j] : A::zero();
    const bool keep = in && A::nz(v);
    const uint64_t m = __ballot(keep);
    if (keep) {
        const uint64_t seg = (KL == 64 ? ~0ull : ((1ull << KL) - 1)) << (lane & ~(KL - 1));
        const int64_t p = out_rp[row] + __popcll(m & seg & lanemask_lt(lane));
        out_col[p] = j;
        out_val[p] = v;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void compact_k1(int64_t rows, const T* __restrict__ y,
                                                  const int64_t* __restrict__ out_rp,
                                                  int32_t* __restrict__ out_col,
                                                  T* __restrict__ out_val) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int64_t p = out_rp[r];
    if (out_rp[r + 1] != p) {
        out_col[p] = 0;
        out_val[p] = y[r];
    }
}

// ---------------------------------------------------------------------------
// Dense operand layout conversion: host Dense is column-major (one Vec per
// column); the kernels want row-major so that an entry gathers k
// contiguous values. 64x64 LDS tiles.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void transpose_tiles(const T* __restrict__ in, T* __restrict__ out,
                                                       int64_t in_rows, int64_t in_cols,
                                                       int64_t tiles_c) {
    // in: in_rows x in_cols row-major; out: in_cols x in_rows row-major.
    // 1-D grid over 64x64 tiles (one of the two extents is large).
    __shared__ T tile[64][65];
    const int64_t t = blockIdx.x;
    const int64_t br = (t / tiles_c) * 64, bc = (t % tiles_c) * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    for (int i = ty; i < 64; i += 4) {
        const int64_t r = br + i, c = bc + tx;
        if (r < in_rows && c < in_cols) tile[i][tx] = in[r * in_cols + c];
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        const int64_t r = bc + i, c = br + tx;  // out row = in col
        if (r < in_cols && c < in_rows) out[r * in_rows + c] = tile[tx][i];
    }
}

template <typename T>
int launch_transpose_tiles(const T* in, T* out, uint64_t in_rows, uint64_t in_cols, hipStream_t s) {
    const uint64_t tr = (in_rows + 63) / 64, tc = (in_cols + 63) / 64;
    BSM_REQUIRE(tr * tc < (1ull << 31), BSM_ERR_UNSUPPORTED, "dense operand too large");
    transpose_tiles<T><<<(unsigned)(tr * tc), 256, 0, s>>>(in, out, (int64_t)in_rows,
                                                           (int64_t)in_cols, (int64_t)tc);
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

// ---------------------------------------------------------------------------
// Analysis: max row length and whether every row's columns are
// non-decreasing (then storage order == ascending-column order, which is
// what mul_vector's transpose-based sum uses, sparse.rs:474-479).
// out3 = {max_row_len, unsorted_rows, bad_col (col >= cols or < 0)}.
// ---------------------------------------------------------------------------
// Matrix analysis, nnz-parallel (a wave per row serialised on the benches'
// one-huge-row matrices): per row the length (max) and a row-start bit;
// per entry the column bound and a descent against the previous entry of
// the same row (not a row start). out3 = {max row length, descents (> 0:
// some row is unsorted), out-of-bounds columns}.
__global__ __launch_bounds__(256) void analyse_row_starts(const int64_t* __restrict__ rp, int64_t rows,
                                                          unsigned* __restrict__ start_bits,
                                                          unsigned long long* __restrict__ out3) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int64_t a = rp[r], b = rp[r + 1];
    if (b > a) {
        atomicMax(&out3[0], (unsigned long long)(b - a));
        atomicOr(&start_bits[a >> 5], 1u << (a & 31));
    }
}

__global__ __launch_bounds__(256) void analyse_entries(const int32_t* __restrict__ col, int64_t nnz, int64_t cols,
                                                       const unsigned* __restrict__ start_bits,
                                                       unsigned long long* __restrict__ out3) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false, desc = false;
    if (e < nnz) {
        const int32_t c = col[e];
        bad = c < 0 || c >= cols;
        desc = e > 0 && !((start_bits[e >> 5] >> (e & 31)) & 1u) && col[e - 1] > c;
    }
    const uint64_t mb = __ballot(bad), md = __ballot(desc);
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        // out3[1] is a flag (any row out of order), set once: a count by
        // atomics (98 us for 600k unsorted entries) or a store from every
        // wave (260 us) serialised ~10k waves on one address
        if (md && __hip_atomic_load(&out3[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
            __hip_atomic_store(&out3[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mb) atomicAdd(&out3[2], (unsigned long long)__popcll(mb));
    }
}

// ---------------------------------------------------------------------------
// Synthetic generator (bsm_synth.h). Row lengths, then one workgroup per row
// draws its columns, bitonic-sorts them in LDS and applies the bump passes
// (forward prefix-max, backward suffix-min) sequentially in one lane, which
// matches the host restatement integer for integer.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gen_rowlen(uint64_t seed, uint64_t row0, int64_t rows,
                                                  uint32_t n_cols, int kind, uint32_t a, uint32_t b,
                                                  int32_t* len) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    uint32_t l = kind == BSM_ROWLEN_BINOMIAL ? bsm_rowlen_binomial(seed, row0 + r, n_cols, a)
                                             : bsm_rowlen(seed, row0 + r, kind, a, b);
    if (l > n_cols) l = n_cols;
    len[r] = (int32_t)l;
}

constexpr int GEN_MAX = 4096;

template <typename T>
__global__ __launch_bounds__(256) void gen_row_entries(uint64_t seed, uint64_t row0, int64_t rows,
                                                       uint32_t n_cols, int value_kind,
                                                       const int64_t* __restrict__ rp,
                                                       int32_t* __restrict__ col,
                                                       T* __restrict__ vals) {
    __shared__ uint32_t key[GEN_MAX];
    const int64_t r = blockIdx.x;
    if (r >= rows) return;
    const int64_t s = rp[r];
    const int len = (int)(rp[r + 1] - s);
    int P = 1;
    while (P < len) P <<= 1;
    const uint64_t grow = row0 + r;
    for (int j = threadIdx.x; j < P; j += blockDim.x)
        key[j] = j < len ? bsm_col_draw(seed, grow, j, n_cols) : 0xffffffffu;
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < P / 2; i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const uint32_t x = key[lo], y = key[hi];
                if ((x > y) == asc) { key[lo] = y; key[hi] = x; }
            }
            __syncthreads();
        }
    }
    if (threadIdx.x == 0 && len > 0) {
        for (int j = 1; j < len; ++j)
            if (key[j] <= key[j - 1]) key[j] = key[j - 1] + 1;
        if (key[len - 1] > n_cols - 1) key[len - 1] = n_cols - 1;
        for (int j = len - 2; j >= 0; --j)
            if (key[j] >= key[j + 1]) key[j] = key[j + 1] - 1;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < len; j += blockDim.x) {
        col[s + j] = (int32_t)key[j];
        vals[s + j] = (T)bsm_a_value(seed, grow, j, value_kind);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void gen_dense_rowmajor(uint64_t seed, uint64_t row0, int64_t n,
                                                          int64_t k, int value_kind, T* __restrict__ x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * k) return;
    const int64_t r = i / k, j = i % k;
    x[i] = (T)bsm_x_value(seed, row0 + r, j, value_kind);
}

inline unsigned grid1d(uint64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

}  // namespace

// ===========================================================================
// host-side launchers
// ===========================================================================
uint64_t scan_workspace_bytes(uint64_t n) {
    const uint64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    return (tiles + 1) * sizeof(int64_t) + 256;
}

int exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, uint64_t n, void* ws,
                              uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) {
        write_zero_i64<<<1, 1, 0, s>>>(out);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    }
    const uint64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    BSM_REQUIRE(ws && ws_bytes >= scan_workspace_bytes(n), BSM_ERR_INVALID,
                "scan workspace too small (%llu < %llu)", (unsigned long long)ws_bytes,
                (unsigned long long)scan_workspace_bytes(n));
    BSM_REQUIRE(tiles < (1ull << 31), BSM_ERR_UNSUPPORTED, "scan too large");
    if (tiles == 1) {
        scan_one_tile<<<1, SCAN_BLOCK, 0, s>>>(in, n, out);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    }
    int64_t* tile_sums = static_cast<int64_t*>(ws);
    scan_tile_sums<<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(in, n, tile_sums);
    scan_tile_prefix<<<1, SCAN_BLOCK, 0, s>>>(tile_sums, tiles);
    scan_apply<<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(in, n, tile_sums, out);
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

namespace {
// Kernel-variant override for A/B timing (BSM_SPMM_VARIANT): 0 default,
// 1 generic row-wave, 2 k32 unpipelined, 3 k32 pipelined x4, 4 k32 pipelined x8,
// 5 k32 four rows per wave (U = 4), 6 the same with U = 2.
// entries per thread of spmv_stream (BSM_SPMV_ITEMS = 2, 4 or 8 for A/B)
int spmv_items() {
    const char* e = getenv("BSM_SPMV_ITEMS");
    const int v = e ? atoi(e) : 4;
    return (v == 2 || v == 8) ? v : 4;
}
constexpr uint64_t SHORT_ROW_AVG = 24;  // nnz/rows at or below: four rows per wave
constexpr uint64_t SPMV_THREAD_ROWS = 16384, SPMV_THREAD_MAX_LEN = 48;  // spmv_thread's shapes
constexpr uint64_t SPMV_ROWS_AVG = 12;  // k = 1, nnz/rows at or below: spmv_rows (one chunk per workgroup)
int spmm_variant() {
    const char* e = getenv("BSM_SPMM_VARIANT");
    return e ? atoi(e) : 0;
}

template <typename T>
int launch_spmm(uint64_t rows, uint64_t nnz, const int64_t* rp, const int32_t* col,
                const T* vals, uint64_t k, const T* x, T* y, int32_t* row_nnz, bool neg_init,
                hipStream_t s, uint64_t max_row_len) {
    if (rows == 0) return BSM_OK;
    // short rows on average (C2: 10): the rows-blocked SpMV; BSM_SPMV_VARIANT=1
    // forces the nnz-balanced spmv_stream (A/B)
    const char* sv = getenv("BSM_SPMV_VARIANT");
    if (k == 1 && nnz <= SPMV_ROWS_AVG * rows && !(sv && atoi(sv) == 1)) {
        const uint64_t blocks = (rows + 255) / 256;
        BSM_REQUIRE(blocks < (1ull << 31), BSM_ERR_UNSUPPORTED, "too many rows for one launch");
        const int64_t r = (int64_t)rows;
        const int svv = sv ? atoi(sv) : 0;
        if (svv == 2)  // the workgroup-chunk version (A/B)
            spmv_rows<T, 16><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        else if (svv == 3)
            spmv_wave<T, 16><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        else if (svv == 4)
            spmv_wave<T, 12><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        else if (svv == 5)
            spmv_wave<T, 8><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        else if (svv == 6)
            spmv_thread<T, 12><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        else if (svv == 0 && rows <= SPMV_THREAD_ROWS && max_row_len <= SPMV_THREAD_MAX_LEN)
            // few short rows (C1: 1,024 x ~10): latency-bound, one thread per
            // row has the fewest dependent round trips (4.5 against 6.4 us at
            // C1, profiles/r05_z_*)
            spmv_thread<T, 12><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        else  // default (C2: 111 us against 117-167 for the others, scripts/perf/spmv_variants.py)
            spmv_wave<T, 8><<<(unsigned)blocks, 256, 0, s>>>(r, rp, col, vals, x, y, row_nnz, neg_init);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    }
    if (k == 1) {
        const int items = spmv_items();
        const uint64_t blocks = nnz / (256ull * items) + 1;
        BSM_REQUIRE(blocks < (1ull << 31), BSM_ERR_UNSUPPORTED, "nnz too large for one launch");
        const int64_t r = (int64_t)rows, z = (int64_t)nnz;
        if (items == 2)
            spmv_stream<T, 2><<<(unsigned)blocks, 256, 0, s>>>(r, z, rp, col, vals, x, y, row_nnz, neg_init);
        else if (items == 8)
            spmv_stream<T, 8><<<(unsigned)blocks, 256, 0, s>>>(r, z, rp, col, vals, x, y, row_nnz, neg_init);
        else
            spmv_stream<T, 4><<<(unsigned)blocks, 256, 0, s>>>(r, z, rp, col, vals, x, y, row_nnz, neg_init);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    }
    BSM_REQUIRE(!neg_init, BSM_ERR_INVALID, "-0 init only for k = 1");
    const int variant = spmm_variant();
    if constexpr (std::is_same_v<T, double>) {
        if (k == 32 && variant != 1 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0) {
            const uint64_t nb = (rows + 3) / 4;
            BSM_REQUIRE(nb < (1ull << 32), BSM_ERR_UNSUPPORTED, "too many rows for one launch");
            auto X2 = reinterpret_cast<const double2*>(x);
            auto Y2 = reinterpret_cast<double2*>(y);
            const int64_t r = (int64_t)rows;
            // short rows on average: four rows per wave (variants 5/6 force it)
            const bool short_rows = nnz <= SHORT_ROW_AVG * rows;
            if (variant == 5 || variant == 6 || (variant == 0 && short_rows)) {
                const uint64_t nb4 = (rows + 15) / 16;
                static const char* pm = getenv("BSM_SPMM_PROBE_MASK");
                if (pm)
                    spmm_k32_f64_rows4<4, true><<<(unsigned)nb4, 256, 0, s>>>(r, rp, col, vals, X2, Y2, row_nnz,
                                                                              (uint32_t)strtoul(pm, nullptr, 10));
                else if (variant == 6)
                    spmm_k32_f64_rows4<2><<<(unsigned)nb4, 256, 0, s>>>(r, rp, col, vals, X2, Y2, row_nnz);
                else
                    spmm_k32_f64_rows4<4><<<(unsigned)nb4, 256, 0, s>>>(r, rp, col, vals, X2, Y2, row_nnz);
                BSM_HIP_TRY(hipGetLastError());
                return BSM_OK;
            }
            if (variant == 2)
                spmm_k32_f64<4, false><<<(unsigned)nb, 256, 0, s>>>(r, rp, col, vals, X2, Y2, row_nnz);
            else if (variant == 4)
                spmm_k32_f64<8, true><<<(unsigned)nb, 256, 0, s>>>(r, rp, col, vals, X2, Y2, row_nnz);
            else
                spmm_k32_f64<4, true><<<(unsigned)nb, 256, 0, s>>>(r, rp, col, vals, X2, Y2, row_nnz);
            BSM_HIP_TRY(hipGetLastError());
            return BSM_OK;
        }
    }
    const uint64_t blocks = (rows + 3) / 4;
    BSM_REQUIRE(blocks < (1ull << 32), BSM_ERR_UNSUPPORTED, "too many rows for one launch");
    const int ki = (int)k;
    const dim3 g((unsigned)blocks), b(256);
    if (k <= 2) spmm_rowwave<T, 2, 4><<<g, b, 0, s>>>(rows, rp, col, vals, ki, x, y, row_nnz);
    else if (k <= 4) spmm_rowwave<T, 4, 4><<<g, b, 0, s>>>(rows, rp, col, vals, ki, x, y, row_nnz);
    else if (k <= 8) spmm_rowwave<T, 8, 4><<<g, b, 0, s>>>(rows, rp, col, vals, ki, x, y, row_nnz);
    else if (k <= 16) spmm_rowwave<T, 16, 8><<<g, b, 0, s>>>(rows, rp, col, vals, ki, x, y, row_nnz);
    else if (k <= 32) spmm_rowwave<T, 32, 8><<<g, b, 0, s>>>(rows, rp, col, vals, ki, x, y, row_nnz);
    else spmm_rowwave<T, 64, 8><<<g, b, 0, s>>>(rows, rp, col, vals, ki, x, y, row_nnz);
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}
}  // namespace

// ---------------------------------------------------------------------------
// nnz-balanced SpMM for INTEGER scalars (split rows). The reference bench's
// insert order piles almost every entry into the last row (running-max row
// rule, sparse.rs:237-250), so one wave per row
// serialises the whole product. Integer sums wrap (Cargo.toml:18) and are
// therefore order-free: each wave takes a fixed slice of SPLIT_CHUNK entries,
// sums its part of every row it touches (lanes (s, c): entry slot s, output
// column c, then an xor-butterfly over s) and stores rows it covers entirely.
// A row cut by the slices leaves one partial per slice (slot 1 in the slice
// where it starts, slot 0 in the later ones) and split_reduce adds them: no
// atomics (the bench's one long row made ~4,400 atomics on one cache line,
// 131 us a call). Floating point keeps the in-order row-wave kernels: its sums
// are not associative.
// ---------------------------------------------------------------------------
constexpr int64_t SPLIT_CHUNK = 512;    // entries per wave
constexpr uint64_t SPLIT_MIN_ROW = 8192;  // use the split kernel when some row is longer

template <typename T> struct UnsignedOf;
template <> struct UnsignedOf<int32_t> { using type = uint32_t; };
template <> struct UnsignedOf<uint32_t> { using type = uint32_t; };
template <> struct UnsignedOf<int64_t> { using type = unsigned long long; };
template <> struct UnsignedOf<uint64_t> { using type = unsigned long long; };

template <typename T, int KL>
__global__ __launch_bounds__(256) void spmm_split_int(int64_t rows, int64_t nnz, const int64_t* __restrict__ rp,
                                                      const int32_t* __restrict__ col, const T* __restrict__ val,
                                                      int k, const T* __restrict__ X, T* __restrict__ Y,
                                                      T* __restrict__ part) {
    using U = typename UnsignedOf<T>::type;
    constexpr int S = WAVE / KL;
    const int lane = threadIdx.x & (WAVE - 1);
    const int s = lane / KL, c = lane % KL;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x / WAVE);
    const int64_t e0 = w * SPLIT_CHUNK;
    if (e0 >= nnz) return;  // wave-uniform
    const int64_t e1 = min<int64_t>(nnz, e0 + SPLIT_CHUNK);
    // the row holding e0: the last r with rp[r] <= e0 (rows before it are empty)
    int64_t r = wave_lower_bound_rp(rp, rows + 1, e0 + 1) - 1;
    for (; r < rows; ++r) {
        const int64_t rs = rp[r], re = rp[r + 1];
        if (rs >= e1) break;
        const int64_t a = max<int64_t>(e0, rs), b = min<int64_t>(e1, re);
        if (a >= b) continue;
        const bool whole = a == rs && b == re;
        for (int cb = 0; cb < k; cb += KL) {
            const int jc = cb + c;
            const bool cval = jc < k;
            U acc = 0;
#pragma unroll 4
            for (int64_t e = a + s; e < b; e += S) {
                if (cval) acc += (U)val[e] * (U)X[(int64_t)col[e] * k + jc];
            }
#pragma unroll
            for (int off = KL; off < WAVE; off <<= 1) acc += (U)__shfl_xor(acc, off, WAVE);
            if (s == 0 && cval) {
                if (whole)
                    Y[r * (int64_t)k + jc] = (T)acc;
                else  // slot 0: the row started before this slice; 1: it starts in it
                    part[(w * 2 + (a == e0 && rs < e0 ? 0 : 1)) * (int64_t)k + jc] = (T)acc;
            }
        }
    }
}

// rows cut by the slices: Y[r] = the sum of their partials (one wave per row)
template <typename T>
__global__ __launch_bounds__(256) void split_reduce(int64_t rows, const int64_t* __restrict__ rp, int k,
                                                    const T* __restrict__ part, T* __restrict__ Y) {
    using U = typename UnsignedOf<T>::type;
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x / WAVE);
    if (r >= rows) return;
    const int64_t rs = rp[r], re = rp[r + 1];
    if (re == rs) return;
    const int64_t wf = rs / SPLIT_CHUNK, wl = (re - 1) / SPLIT_CHUNK;
    if (wf == wl) return;  // stored whole by its slice
    for (int j = 0; j < k; ++j) {
        U acc = 0;
        for (int64_t w = wf + lane; w <= wl; w += WAVE)
            acc += (U)part[(w * 2 + (w == wf ? 1 : 0)) * (int64_t)k + j];
#pragma unroll
        for (int off = 1; off < WAVE; off <<= 1) acc += (U)__shfl_xor(acc, off, WAVE);
        if (lane == 0) Y[r * (int64_t)k + j] = (T)acc;
    }
}

// nonzero results per row of a dense Y (rows x k), for the compaction
template <typename T>
__global__ __launch_bounds__(256) void count_row_nnz(int64_t rows, int k, const T* __restrict__ Y,
                                                     int32_t* __restrict__ row_nnz) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    int32_t n = 0;
    for (int j = 0; j < k; ++j) n += Arith<T>::nz(Y[r * (int64_t)k + j]) ? 1 : 0;
    row_nnz[r] = n;
}

bool spmm_wants_split(int dtype, uint64_t k, uint64_t max_row_len) {
    if (const char* e = getenv("BSM_SPMM_SPLIT")) return atoi(e) != 0 && k >= 2 &&
                                                          !(dtype == BSM_F64 || dtype == BSM_F32);
    return k >= 2 && max_row_len >= SPLIT_MIN_ROW && !(dtype == BSM_F64 || dtype == BSM_F32);
}

int spmm_split_dispatch(int dtype, uint64_t rows, uint64_t nnz, const int64_t* rp, const int32_t* col,
                        const void* vals, uint64_t k, const void* x, void* y, int32_t* row_nnz, hipStream_t s) {
    BSM_REQUIRE(!(dtype == BSM_F64 || dtype == BSM_F32), BSM_ERR_INVALID, "split SpMM: integer scalars only");
    if (rows == 0) return BSM_OK;
    const size_t es = dtype_size(dtype);
    BSM_HIP_TRY(hipMemsetAsync(y, 0, rows * k * es, s));
    const uint64_t waves = (nnz + SPLIT_CHUNK - 1) / SPLIT_CHUNK;
    const uint64_t blocks = (waves + 3) / 4;
    BSM_REQUIRE(blocks < (1ull << 31) && k < (1ull << 31), BSM_ERR_UNSUPPORTED, "split SpMM: too large");
    const int ki = (int)k;
    DBuf part;  // two partial rows per slice
    BSM_TRY(part.alloc(waves * 2 * k * es));
    return dispatch_dtype(dtype, [&]<typename T>() -> int {
        if constexpr (std::is_integral_v<T>) {
            auto go = [&]<int KL>() {
                if (blocks) {
                    spmm_split_int<T, KL><<<(unsigned)blocks, 256, 0, s>>>(
                        (int64_t)rows, (int64_t)nnz, rp, col, static_cast<const T*>(vals), ki,
                        static_cast<const T*>(x), static_cast<T*>(y), part.as<T>());
                    split_reduce<T><<<(unsigned)((rows + 3) / 4), 256, 0, s>>>((int64_t)rows, rp, ki,
                                                                              part.as<T>(), static_cast<T*>(y));
                }
            };
            if (k <= 2) go.template operator()<2>();
            else if (k <= 4) go.template operator()<4>();
            else if (k <= 8) go.template operator()<8>();
            else if (k <= 16) go.template operator()<16>();
            else if (k <= 32) go.template operator()<32>();
            else go.template operator()<64>();
            BSM_HIP_TRY(hipGetLastError());
            if (row_nnz) {
                count_row_nnz<T><<<(unsigned)((rows + 255) / 256), 256, 0, s>>>((int64_t)rows, ki,
                                                                                static_cast<const T*>(y), row_nnz);
                BSM_HIP_TRY(hipGetLastError());
            }
            return BSM_OK;
        } else {
            return BSM_ERR_INVALID;
        }
    });
}

int spmm_dispatch(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* rp,
                  const int32_t* col, const void* vals, uint64_t k, const void* x, void* y,
                  int32_t* row_nnz, bool neg_zero_init, hipStream_t s, uint64_t max_row_len) {
    (void)n_cols;
    return dispatch_dtype(dtype, [&]<typename T>() {
        return launch_spmm<T>(rows, nnz, rp, col, static_cast<const T*>(vals), k,
                              static_cast<const T*>(x), static_cast<T*>(y), row_nnz,
                              neg_zero_init, s, max_row_len);
    });
}

// ---------------------------------------------------------------------------
// Column-panel schedule for large X (DESIGN.md "SpMM: column panels"). With
// uniformly random columns every CSR entry gathers a whole X row and X
// (C4: 2.56 GB) is far larger than the 256 MiB Infinity Cache, so gathers
// are served by HBM. Cutting the columns into panels whose slice of X fits
// the Infinity Cache and sweeping the rows once per panel serves the gathers
// on-die; the running sums travel through Y between passes (exact).
// ---------------------------------------------------------------------------
namespace {
constexpr uint64_t PANEL_X_BYTES = 512ull << 20;      // X slice per pass (C4: 5 passes)
constexpr uint64_t PANEL_MIN_X_BYTES = 1ull << 30;    // below: one pass
}  // namespace

uint64_t spmm_panel_cols(int dtype, uint64_t n_cols, uint64_t k) {
    if (dtype != BSM_F64 || k != 32 || n_cols == 0) return 0;  // panelled kernel: k32 f64 only
    uint64_t w;
    if (const char* e = getenv("BSM_SPMM_PANEL_COLS")) {  // A/B and tests; 0 = off
        w = strtoull(e, nullptr, 10);
    } else {
        const uint64_t x_bytes = n_cols * k * sizeof(double);
        if (x_bytes <= PANEL_MIN_X_BYTES) return 0;
        const uint64_t passes = (x_bytes + PANEL_X_BYTES - 1) / PANEL_X_BYTES;
        w = (n_cols + passes - 1) / passes;
    }
    return (w == 0 || w >= n_cols || w > UINT32_MAX) ? 0 : w;
}

uint64_t spmm_plan_bytes(uint64_t rows, uint64_t n_cols, uint64_t panel_cols) {
    if (panel_cols == 0 || panel_cols >= n_cols) return 0;
    const uint64_t passes = (n_cols + panel_cols - 1) / panel_cols;
    return (passes - 1) * rows * sizeof(int32_t);
}

int spmm_plan(uint64_t rows, uint64_t n_cols, const int64_t* rp, const int32_t* col,
              uint64_t panel_cols, int32_t* seg, int* usable, hipStream_t s) {
    *usable = 0;
    if (panel_cols == 0 || panel_cols >= n_cols) return BSM_OK;
    const uint64_t passes = (n_cols + panel_cols - 1) / panel_cols;
    BSM_REQUIRE(passes < (1u << 20) && panel_cols <= UINT32_MAX, BSM_ERR_UNSUPPORTED, "too many panels");
    DBuf flag;
    BSM_TRY(flag.alloc(sizeof(unsigned)));
    BSM_HIP_TRY(hipMemsetAsync(flag.p, 0, sizeof(unsigned), s));
    if (rows) {
        spmm_plan_panels<<<grid1d(rows, 4), 256, 0, s>>>((int64_t)rows, rp, col, (uint32_t)panel_cols,
                                                          (int)passes, seg, flag.as<unsigned>());
        BSM_HIP_TRY(hipGetLastError());
    }
    unsigned bad = 0;
    BSM_HIP_TRY(read_dev(&bad, flag.p, sizeof(unsigned), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    *usable = bad == 0;
    return BSM_OK;
}

int spmm_panelled(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* rp,
                  const int32_t* col, const void* vals, uint64_t k, const void* x, void* y,
                  int32_t* row_nnz, uint64_t panel_cols, const int32_t* seg, hipStream_t s) {
    const bool aligned = ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0;
    if (!seg || panel_cols == 0 || panel_cols >= n_cols || dtype != BSM_F64 || k != 32 || !aligned ||
        rows == 0)
        return spmm_dispatch(dtype, rows, n_cols, nnz, rp, col, vals, k, x, y, row_nnz, false, s);
    const uint64_t passes = (n_cols + panel_cols - 1) / panel_cols;
    const uint64_t nb = (rows + 3) / 4;
    BSM_REQUIRE(nb < (1ull << 32), BSM_ERR_UNSUPPORTED, "too many rows for one launch");
    auto X2 = static_cast<const double2*>(x);
    auto Y2 = static_cast<double2*>(y);
    auto V = static_cast<const double*>(vals);
    for (uint64_t p = 0; p < passes; ++p) {
        const int32_t* lo = p ? seg + (p - 1) * rows : nullptr;
        const int32_t* hi = p + 1 < passes ? seg + p * rows : nullptr;
        spmm_k32_f64<4, true, true><<<(unsigned)nb, 256, 0, s>>>((int64_t)rows, rp, col, V, X2, Y2,
                                                                 p + 1 < passes ? nullptr : row_nnz, lo, hi);
        BSM_HIP_TRY(hipGetLastError());
    }
    return BSM_OK;
}

int compact_dispatch(int dtype, uint64_t rows, uint64_t k, const void* y, const int64_t* out_rp,
                     int32_t* out_col, void* out_vals, hipStream_t s) {
    if (rows == 0 || k == 0) return BSM_OK;
    return dispatch_dtype(dtype, [&]<typename T>() {
        if (k == 1) {
            compact_k1<T><<<grid1d(rows, 256), 256, 0, s>>>((int64_t)rows, static_cast<const T*>(y),
                                                           out_rp, out_col, static_cast<T*>(out_vals));
        } else if (k <= 32) {
            auto seg = [&]<int KL>() {
                compact_seg<T, KL><<<grid1d(rows, 4 * (WAVE / KL)), 256, 0, s>>>(
                    (int64_t)rows, (int)k, static_cast<const T*>(y), out_rp, out_col, static_cast<T*>(out_vals));
            };
            if (k <= 2) seg.template operator()<2>();
            else if (k <= 4) seg.template operator()<4>();
            else if (k <= 8) seg.template operator()<8>();
            else if (k <= 16) seg.template operator()<16>();
            else seg.template operator()<32>();
        } else {
            compact_wave<T><<<grid1d(rows, 4), 256, 0, s>>>((int64_t)rows, (int)k,
                                                           static_cast<const T*>(y), out_rp, out_col,
                                                           static_cast<T*>(out_vals));
        }
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
}

// ---------------------------------------------------------------------------
// Small results (C1: 1,024 rows x 1 column): the row-count scan and the
// compaction in ONE workgroup, writing the result twice -- into its device
// arrays and into a page-locked host copy -- so that the call's one
// synchronisation also delivers what bsm_csr_download returns (no scan
// launch, no compaction launch, no read-back of nnz, no download copies).
// Offsets live in LDS (rows <= SMALL_OUT_ROWS). Same entries, same order as
// scan + compact_k1 / compact_seg: the row's nonzero columns ascending.
// ---------------------------------------------------------------------------
constexpr int SMALL_OUT_THREADS = 1024;

template <typename T>
__global__ __launch_bounds__(SMALL_OUT_THREADS) void compact_small(int64_t rows, int k, const int32_t* __restrict__ nz,
                                                                   const T* __restrict__ Y, int64_t* __restrict__ out_rp,
                                                                   int32_t* __restrict__ out_col, T* __restrict__ out_val,
                                                                   int64_t* __restrict__ h_rp, int32_t* __restrict__ h_col,
                                                                   T* __restrict__ h_val) {
    using A = Arith<T>;
    __shared__ int32_t off[SMALL_OUT_ROWS];
    __shared__ int32_t wsum[SMALL_OUT_THREADS / WAVE];
    const int t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
    const int R = (int)((rows + SMALL_OUT_THREADS - 1) / SMALL_OUT_THREADS);
    const int r0 = t * R, r1 = (int)min<int64_t>(rows, (int64_t)r0 + R);
    int local = 0;
    for (int r = r0; r < r1; ++r) local += nz[r];
    int incl = local;  // wave inclusive scan, then the waves' totals
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == WAVE - 1) wsum[w] = incl;
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < SMALL_OUT_THREADS / WAVE; ++q) {
        before += q < w ? wsum[q] : 0;
        total += wsum[q];
    }
    int ex = before + incl - local;
    for (int r = r0; r < r1; ++r) {
        off[r] = ex;
        out_rp[r] = ex;
        h_rp[r] = ex;
        ex += nz[r];
    }
    if (t == 0) {
        out_rp[rows] = total;
        h_rp[rows] = total;
    }
    __syncthreads();
    if (k == 1) {
        for (int r = t; r < rows; r += SMALL_OUT_THREADS) {
            const T v = Y[r];
            if (A::nz(v)) {
                const int p = off[r];
                out_col[p] = 0;
                out_val[p] = v;
                h_col[p] = 0;
                h_val[p] = v;
            }
        }
        return;
    }
    for (int r = w; r < rows; r += SMALL_OUT_THREADS / WAVE) {  // one wave per row, lanes over columns
        int base = off[r];
        for (int j0 = 0; j0 < k; j0 += WAVE) {
            const int j = j0 + lane;
            const T v = j < k ? Y[(int64_t)r * k + j] : A::zero();
            const bool keep = j < k && A::nz(v);
            const uint64_t m = __ballot(keep);
            if (keep) {
                const int p = base + __popcll(m & lanemask_lt(lane));
                out_col[p] = j;
                out_val[p] = v;
                h_col[p] = j;
                h_val[p] = v;
            }
            base += __popcll(m);
        }
    }
}

int compact_small_dispatch(int dtype, uint64_t rows, uint64_t k, const int32_t* nz, const void* y, int64_t* out_rp,
                           int32_t* out_col, void* out_vals, void* host, uint64_t cap, hipStream_t s) {
    BSM_REQUIRE(rows <= (uint64_t)SMALL_OUT_ROWS && k > 0 && rows * k <= SMALL_OUT_CAP && cap >= rows * k,
                BSM_ERR_INVALID, "compact_small: %llu x %llu is not a small result", (unsigned long long)rows,
                (unsigned long long)k);
    const size_t es = dtype_size(dtype);
    char* h = static_cast<char*>(host);
    int64_t* h_rp = reinterpret_cast<int64_t*>(h);
    int32_t* h_col = reinterpret_cast<int32_t*>(h + (rows + 1) * sizeof(int64_t));
    void* h_val = h + (rows + 1) * sizeof(int64_t) + small_col_bytes(cap);
    (void)es;
    return dispatch_dtype(dtype, [&]<typename T>() {
        compact_small<T><<<1, SMALL_OUT_THREADS, 0, s>>>((int64_t)rows, (int)k, nz, static_cast<const T*>(y), out_rp,
                                                         out_col, static_cast<T*>(out_vals), h_rp, h_col,
                                                         static_cast<T*>(h_val));
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
}

int pack_cols_to_rowmajor(int dtype, uint64_t n, uint64_t k, const void* colmajor, void* rowmajor,
                          hipStream_t s) {
    if (n == 0 || k == 0) return BSM_OK;
    return dispatch_dtype(dtype, [&]<typename T>() {
        // colmajor = k x n row-major; rowmajor = n x k
        return launch_transpose_tiles<T>(static_cast<const T*>(colmajor), static_cast<T*>(rowmajor),
                                         k, n, s);
    });
}

int unpack_rowmajor_to_cols(int dtype, uint64_t n, uint64_t k, const void* rowmajor, void* colmajor,
                            hipStream_t s) {
    if (n == 0 || k == 0) return BSM_OK;
    return dispatch_dtype(dtype, [&]<typename T>() {
        return launch_transpose_tiles<T>(static_cast<const T*>(rowmajor), static_cast<T*>(colmajor),
                                         n, k, s);
    });
}

int analyse_dispatch(const int64_t* rp, const int32_t* col, uint64_t rows, uint64_t cols,
                     uint64_t* d_out3, hipStream_t s) {
    BSM_HIP_TRY(hipMemsetAsync(d_out3, 0, 3 * sizeof(uint64_t), s));
    if (rows == 0) return BSM_OK;
    int64_t nnz = 0;
    BSM_HIP_TRY(read_dev(&nnz, rp + rows, sizeof(int64_t), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    DBuf bits;
    const uint64_t words = (uint64_t)nnz / 32 + 1;
    BSM_TRY(bits.alloc(words * sizeof(unsigned)));
    BSM_HIP_TRY(hipMemsetAsync(bits.p, 0, words * sizeof(unsigned), s));
    auto out3 = reinterpret_cast<unsigned long long*>(d_out3);
    analyse_row_starts<<<grid1d(rows, 256), 256, 0, s>>>(rp, (int64_t)rows, bits.as<unsigned>(), out3);
    if (nnz > 0)
        analyse_entries<<<grid1d((uint64_t)nnz, 256), 256, 0, s>>>(col, nnz, (int64_t)cols, bits.as<unsigned>(), out3);
    BSM_HIP_TRY(hipGetLastError());
    BSM_HIP_TRY(hipStreamSynchronize(s));  // bits dies here
    return BSM_OK;
}

int gen_row_ptr(uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols, int kind, uint32_t a,
                uint32_t b, int64_t* rp, void* ws, uint64_t ws_bytes, hipStream_t s) {
    BSM_REQUIRE(kind == BSM_ROWLEN_CONST || kind == BSM_ROWLEN_UNIFORM ||
                    (kind == BSM_ROWLEN_BINOMIAL && n_cols <= GEN_MAX),
                BSM_ERR_UNSUPPORTED, "device generator: CONST/UNIFORM row lengths, or BINOMIAL up to %d columns",
                GEN_MAX);
    BSM_REQUIRE(kind == BSM_ROWLEN_BINOMIAL || (b <= GEN_MAX && a <= GEN_MAX), BSM_ERR_UNSUPPORTED,
                "row length > %d", GEN_MAX);
    // workspace: [len int32 rows][scan ws]
    const uint64_t len_bytes = ((rows * sizeof(int32_t)) + 255) / 256 * 256;
    BSM_REQUIRE(ws && ws_bytes >= len_bytes + scan_workspace_bytes(rows), BSM_ERR_INVALID,
                "generator workspace too small");
    int32_t* len = static_cast<int32_t*>(ws);
    if (rows) {
        gen_rowlen<<<grid1d(rows, 256), 256, 0, s>>>(seed, row0, (int64_t)rows, n_cols, kind, a, b, len);
        BSM_HIP_TRY(hipGetLastError());
    }
    return exclusive_scan_i32_to_i64(len, rp, rows, static_cast<char*>(ws) + len_bytes,
                                     ws_bytes - len_bytes, s);
}

int gen_entries(int dtype, uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols,
                int value_kind, const int64_t* rp, int32_t* col, void* vals, hipStream_t s) {
    if (rows == 0) return BSM_OK;
    BSM_REQUIRE(rows < (1ull << 31), BSM_ERR_UNSUPPORTED, "too many rows for one launch");
    BSM_REQUIRE(value_kind == BSM_VAL_SMALLINT || dtype == BSM_F64 || dtype == BSM_F32,
                BSM_ERR_INVALID, "integer dtypes need value_kind SMALLINT (UNIFORM would give zeros)");
    return dispatch_dtype(dtype, [&]<typename T>() {
        gen_row_entries<T><<<(unsigned)rows, 256, 0, s>>>(seed, row0, (int64_t)rows, n_cols,
                                                          value_kind, rp, col, static_cast<T*>(vals));
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
}

int gen_dense(int dtype, uint64_t seed, uint64_t row0, uint64_t n, uint64_t k, int value_kind,
              void* x, hipStream_t s) {
    if (n == 0 || k == 0) return BSM_OK;
    return dispatch_dtype(dtype, [&]<typename T>() {
        const uint64_t total = n * k;
        BSM_REQUIRE(total / 256 < (1ull << 31), BSM_ERR_UNSUPPORTED, "dense too large");
        gen_dense_rowmajor<T><<<grid1d(total, 256), 256, 0, s>>>(seed, row0, (int64_t)n, (int64_t)k,
                                                                value_kind, static_cast<T*>(x));
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
}

}  // namespace bsm
