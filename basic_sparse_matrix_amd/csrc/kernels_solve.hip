// kernels_solve.hip -- Csr::cholesky_decomp (reference src/sparse.rs:682-714),
// forward_substitution / backward_substitution / solve (src/lib.rs:11-65)
// on gfx950, with the reference's exact floating-point operation order.
//
// Exactness. The reference computes, for every L[i][j],
//     sum = 0; for k in 0..j { sum += L[i][k] * L[j][k] }          (f32 or f64)
//     L[i][i] = (A[i][i] - sum).powf(0.5);  L[i][j] = (1/L[j][j]) * (A[i][j] - sum)
// Products of a structural zero are +-0 and never change a sum that starts
// at +0, so only k inside the band matter. Every
// kernel below adds each element's terms one at a time, in ascending k, with
// no FMA: results are bit-identical to the oracle (and to the reference).
//
// Layout. Factorisation works on a dense BAND stored by columns:
//     CB[k * ld + d] = L[k + d][k],  d in [0, b],  ld = b + 1
// (b = max over rows of i - first_col(i)). Column k of L is contiguous, which
// is what the right-looking update and the backward solve (rows of L^T) read.
//
// band_chol: persistent kernel, one 1024-thread workgroup per CU. Tile-row I
// (32 rows) is swept column by column (right-looking): at column k the owner
// threads finalise L[i][k] for the 32 rows, then every (i, j > k) accumulator
// of the tile-row adds L[i][k] * L[j][k]. The accumulators (32 rows x b+32
// columns) live in registers. Tile-row I needs column k of the rows above it,
// i.e. of tile-rows < I: it waits on tile-row I-1's progress counter, which
// is published every few columns (write-through sc1 stores + counter, the
// hand-off of MI355X_MICROARCH.md "Valid forms", table row 1).
#include <cmath>

#include "bsm_internal.hpp"

namespace bsm {
namespace {

constexpr int TR = 32;              // rows per tile-row
constexpr int CH_THREADS = 1024;    // 16 row pairs x 64 column lanes
constexpr int PUBLISH_EVERY = 8;    // columns between progress publications
constexpr long long SPIN_LIMIT = 1ll << 25;

enum { ST_NOT_PD = 1, ST_TIMEOUT = 2, ST_EMPTY_ROW = 4 };

// ---- write-through (sc1) loads/stores of T via same-width integers --------
template <typename T> struct Bits;
template <> struct Bits<double> { using U = unsigned long long; };
template <> struct Bits<float> { using U = unsigned int; };

template <typename T> __device__ __forceinline__ T ld_sc1(const T* p) {
    using U = typename Bits<T>::U;
    U u = __hip_atomic_load(reinterpret_cast<const U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_bit_cast(T, u);
}
template <typename T> __device__ __forceinline__ void st_sc1(T* p, T v) {
    using U = typename Bits<T>::U;
    __hip_atomic_store(reinterpret_cast<U*>(p), __builtin_bit_cast(U, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// powf(x, 0.5) as LLVM lowers it: x == -inf ? +inf : |sqrt(x)| (correctly
// rounded sqrt; -0 -> +0). Matches the oracle and the reference's goldens.
__device__ __forceinline__ double pow_half(double x) {
    if (isinf(x) && x < 0) return INFINITY;
    return fabs(__dsqrt_rn(x));
}
// f32 sqrt and division are formed in f64 and rounded once to f32: for
// sqrt and '/', a result correctly rounded to 53 bits and then rounded to 24
// is the correctly rounded f32 result (53 >= 2*24 + 2), i.e. IEEE f32 exactly
// as the reference's host computes it, independent of device math flags.
__device__ __forceinline__ float pow_half(float x) {
    if (isinf(x) && x < 0) return INFINITY;
    return fabsf(__double2float_rn(__dsqrt_rn((double)x)));
}
template <typename T> __device__ __forceinline__ T div_rn(T a, T b);
template <> __device__ __forceinline__ double div_rn(double a, double b) { return __ddiv_rn(a, b); }
template <> __device__ __forceinline__ float div_rn(float a, float b) {
    return __double2float_rn(__ddiv_rn((double)a, (double)b));
}

// ---------------------------------------------------------------------------
// band construction
// ---------------------------------------------------------------------------
// bw[0] = max(i - first stored col of row i over cols <= i); bw[1] = rows whose
// columns are not strictly increasing; bw[2] = empty rows.
__global__ __launch_bounds__(256) void band_width(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                  int64_t n, unsigned long long* bw) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t a = rp[i], b = rp[i + 1];
    int64_t f = i;
    bool bad = false;
    for (int64_t e = a; e < b; ++e) {
        const int64_t c = col[e];
        if (e > a && col[e - 1] >= c) bad = true;
        if (c < f) f = c;
    }
    atomicMax(&bw[0], (unsigned long long)(i - f));
    if (bad) atomicAdd(&bw[1], 1ull);
    if (a == b) atomicAdd(&bw[2], 1ull);
}

template <typename T>
__global__ __launch_bounds__(256) void band_fill(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                 const T* __restrict__ val, int64_t n, int64_t ld,
                                                 T* __restrict__ CB) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
        const int64_t j = col[e];
        if (j <= i) CB[j * ld + (i - j)] = val[e];  // reference reads A[i][j] for j <= i only
    }
}

// ---------------------------------------------------------------------------
// band_chol: see file header. Thread t: row pair rp2 = t >> 6 (rows 2*rp2,
// 2*rp2+1 of the tile-row), column lane c = t & 63, accumulators for
// j = jb + c + 64 m, m < M.
// ---------------------------------------------------------------------------
template <typename T, int M>
__global__ __launch_bounds__(CH_THREADS) void band_chol(int64_t n, int64_t b, int64_t ld, T* __restrict__ CB,
                                                         int* __restrict__ progress, int* __restrict__ status,
                                                         int64_t n_tiles) {
    using A = Arith<T>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* colL = reinterpret_cast<T*>(smem_raw);  // [b + 1]: L[k + d][k]
    __shared__ T rowval[TR];                   // L[i][k] of the 32 rows at this step
    __shared__ T s_pivot;
    const int tid = threadIdx.x;
    const int rp2 = tid >> 6, c = tid & 63;
    for (int64_t I = blockIdx.x; I < n_tiles; I += gridDim.x) {
        const int64_t i0 = I * TR;
        const int64_t iA = i0 + 2 * rp2;  // this thread: rows iA, iA + 1
        const int64_t jb = i0 - b > 0 ? i0 - b : 0;
        const int64_t kend = i0 + TR < n ? i0 + TR : n;
        T acc[2][M];
#pragma unroll
        for (int m = 0; m < M; ++m) { acc[0][m] = A::zero(); acc[1][m] = A::zero(); }
        int64_t seen = -1;  // thread 0: last observed progress of tile-row I-1
        T pre = A::zero();  // prefetched L[k + 1 + tid][k]
        bool have_pre = false;
        for (int64_t k = jb; k < kend; ++k) {
            // (a) column k (and k+1, for the prefetch) of the rows above must be final
            if (tid == 0 && I > 0) {
                const int64_t need = (k + 2 < i0 ? k + 2 : i0);  // progress counts columns done
                long long spins = 0;
                while (seen < need) {
                    seen = __hip_atomic_load(&progress[I - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (seen >= need) break;
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > SPIN_LIMIT ||
                        ((spins & 1023) == 0 &&
                         (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ST_TIMEOUT))) {
                        atomicOr(status, ST_TIMEOUT);
                        seen = INT32_MAX;
                        break;
                    }
                }
            }
            __syncthreads();  // B1: colL / rowval of step k-1 are no longer read
            const int64_t kk = k - jb;
            const int mk = (int)(kk >> 6), ck = (int)(kk & 63);
            // (b) finalise column k. Diagonal first when row k is ours.
            T piv;
            if (k >= i0) {
                if ((k - i0) >> 1 == rp2 && c == ck) {
                    const int w = (int)((k - i0) & 1);
                    T s = A::zero();
#pragma unroll
                    for (int m = 0; m < M; ++m) if (m == mk) s = acc[w][m];
                    const T a = CB[k * ld];
                    const T l = pow_half(A::sub(a, s));
                    if (!(l > A::zero()) || isinf(l)) atomicOr(status, ST_NOT_PD);
                    st_sc1(&CB[k * ld], l);
                    s_pivot = l;
                }
                __syncthreads();
                piv = s_pivot;
            } else {
                piv = (c == ck) ? ld_sc1(&CB[k * ld]) : A::zero();
            }
            if (c == ck) {
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    const int64_t i = iA + w;
                    T lik = A::zero();
                    if (i < n && i >= k && i - k <= b) {
                        if (i == k) {
                            lik = piv;
                        } else {
                            T s = A::zero();
#pragma unroll
                            for (int m = 0; m < M; ++m) if (m == mk) s = acc[w][m];
                            const T a = CB[k * ld + (i - k)];
                            const T one = (T)1;
                            lik = A::mul(div_rn(one, piv), A::sub(a, s));
                            st_sc1(&CB[k * ld + (i - k)], lik);
                        }
                        if (i > k) colL[i - k] = lik;
                    }
                    rowval[2 * rp2 + w] = lik;
                }
            }
            // (c) column k of the rows above this tile-row (prefetched last step)
            if (have_pre) colL[1 + tid] = pre;
            {
                const int64_t dmax = (i0 - 1 - k < b) ? i0 - 1 - k : b;  // rows k+1 .. i0-1
                for (int64_t d = 1 + tid + CH_THREADS; d <= dmax; d += CH_THREADS) colL[d] = ld_sc1(&CB[k * ld + d]);
                if (!have_pre && 1 + tid <= dmax) colL[1 + tid] = ld_sc1(&CB[k * ld + 1 + tid]);
            }
            __syncthreads();  // B2
            // prefetch column k+1 for the next step (rows above the tile-row)
            {
                const int64_t k1 = k + 1;
                const int64_t dmax1 = (i0 - 1 - k1 < b) ? i0 - 1 - k1 : b;
                have_pre = (k1 < kend) && (1 + tid <= dmax1);
                if (have_pre) pre = ld_sc1(&CB[k1 * ld + 1 + tid]);
            }
            // (d) right-looking update of this thread's accumulators
            const T l0 = rowval[2 * rp2], l1 = rowval[2 * rp2 + 1];
            {
                // 32-bit relative indices: d = j - k, j = jb + c + 64 m
                const int dbase = (int)(jb - k) + c;
                const int dA = (int)(iA - k), dB = dA + 1, bb = (int)b;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const int d = dbase + 64 * m;
                    if (d >= 1 && d <= bb) {
                        const T ljk = colL[d];
                        if (d <= dA) acc[0][m] = A::add(acc[0][m], A::mul(l0, ljk));
                        if (d <= dB) acc[1][m] = A::add(acc[1][m], A::mul(l1, ljk));
                    }
                }
            }
            // (e) publish progress: all stores of columns <= k drained first
            if ((kk + 1) % PUBLISH_EVERY == 0 || k + 1 == kend) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0)
                    __hip_atomic_store(&progress[I], (int)(k + 1 == kend ? kend : k + 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// forward substitution on the band (lib.rs:28-46): y_i = (b_i - sum_{j<i}
// L_ij y_j) / L_ii, sum in ascending j. One workgroup per RHS column; blocks
// of 256 rows: the "far" terms (j < block start) are summed first, one thread
// per row, then the in-block terms column by column. y lives in an LDS ring.
// ---------------------------------------------------------------------------
constexpr int FW_BLOCK = 256;
constexpr int FW_RING = 2048;  // >= b + FW_BLOCK

template <typename T>
__global__ __launch_bounds__(FW_BLOCK) void band_forward(int64_t n, int64_t b, int64_t ld,
                                                         const T* __restrict__ CB, const T* __restrict__ B,
                                                         T* __restrict__ Y) {
    using A = Arith<T>;
    __shared__ T ring[FW_RING];
    __shared__ T s_y;
    const int t = threadIdx.x;
    const T* bc = B + (int64_t)blockIdx.x * n;
    T* yc = Y + (int64_t)blockIdx.x * n;
    for (int64_t i0 = 0; i0 < n; i0 += FW_BLOCK) {
        const int64_t i = i0 + t;
        T s = A::zero();
        const int64_t j0 = (i - b > 0) ? i - b : 0;
        if (i < n)
            for (int64_t j = j0; j < i0; ++j) s = A::add(s, A::mul(CB[j * ld + (i - j)], ring[j & (FW_RING - 1)]));
        const int64_t nb = (n - i0 < FW_BLOCK) ? n - i0 : FW_BLOCK;
        for (int64_t tt = 0; tt < nb; ++tt) {
            const int64_t j = i0 + tt;
            if (t == tt) {
                const T y = div_rn(A::sub(bc[i], s), CB[i * ld]);
                ring[i & (FW_RING - 1)] = y;
                s_y = y;
                yc[i] = y;
            }
            __syncthreads();
            if (i < n && i > j && i - j <= b) s = A::add(s, A::mul(CB[j * ld + (i - j)], s_y));
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// backward substitution on the band (lib.rs:49-65) with L* = L^T: x_i =
// (y_i - sum_{j>i} L_ji x_j) / L_ii, sum in ascending j. The ascending order
// makes each row's sum start with the most recent x, so the solve is one
// serial chain; one wavefront per RHS column: lanes form the products, lane
// 0 adds them in order.
// ---------------------------------------------------------------------------
constexpr int BW_RING = 2048;

template <typename T>
__global__ __launch_bounds__(64) void band_backward(int64_t n, int64_t b, int64_t ld, const T* __restrict__ CB,
                                                    const T* __restrict__ Yin, T* __restrict__ X) {
    using A = Arith<T>;
    __shared__ T ring[BW_RING];
    __shared__ T prod[BW_RING];
    const int lane = threadIdx.x;
    const T* yc = Yin + (int64_t)blockIdx.x * n;
    T* xc = X + (int64_t)blockIdx.x * n;
    for (int64_t i = n - 1; i >= 0; --i) {
        const int64_t dmax = (n - 1 - i < b) ? n - 1 - i : b;
        const T* colI = CB + i * ld;
        for (int64_t d = 1 + lane; d <= dmax; d += 64) prod[d] = A::mul(colI[d], ring[(i + d) & (BW_RING - 1)]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            T s = A::zero();
            for (int64_t d = 1; d <= dmax; ++d) s = A::add(s, prod[d]);
            const T x = div_rn(A::sub(yc[i], s), colI[0]);
            ring[i & (BW_RING - 1)] = x;
            xc[i] = x;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// band -> CSR (the Csr returned by cholesky_decomp: zero results are not
// stored, sparse.rs:229,710; row i lists columns ascending, diagonal last).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void band_row_count(int64_t n, int64_t b, int64_t ld, const T* __restrict__ CB,
                                                      int32_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t c = 0;
    for (int64_t j = (i - b > 0 ? i - b : 0); j <= i; ++j) c += Arith<T>::nz(CB[j * ld + (i - j)]) ? 1 : 0;
    cnt[i] = c;
}

template <typename T>
__global__ __launch_bounds__(256) void band_to_csr(int64_t n, int64_t b, int64_t ld, const T* __restrict__ CB,
                                                   const int64_t* __restrict__ rp, int32_t* __restrict__ col,
                                                   T* __restrict__ val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t p = rp[i];
    for (int64_t j = (i - b > 0 ? i - b : 0); j <= i; ++j) {
        const T v = CB[j * ld + (i - j)];
        if (Arith<T>::nz(v)) { col[p] = (int32_t)j; val[p] = v; ++p; }
    }
}

// ---------------------------------------------------------------------------
// General-CSR triangular solves for the public forward_substitution /
// backward_substitution (lib.rs:28-65), rows sorted by column.
// forward: one workgroup per RHS column, 256-row blocks; far entries (col <
// block start) summed first per row, then in-block entries column by column;
// entries with col >= row read y == 0 in the reference (not yet computed) and
// contribute +-0: skipped. Divisor = LAST stored entry of the row.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(FW_BLOCK) void csr_forward(int64_t n, const int64_t* __restrict__ rp,
                                                        const int32_t* __restrict__ col, const T* __restrict__ val,
                                                        const T* __restrict__ B, T* __restrict__ Y,
                                                        int* __restrict__ status) {
    using A = Arith<T>;
    __shared__ T s_y[FW_BLOCK];
    const int t = threadIdx.x;
    const T* bc = B + (int64_t)blockIdx.x * n;
    T* yc = Y + (int64_t)blockIdx.x * n;
    for (int64_t i0 = 0; i0 < n; i0 += FW_BLOCK) {
        const int64_t i = i0 + t;
        T s = A::zero();
        int64_t e = 0, e1 = 0;
        if (i < n) {
            e = rp[i];
            e1 = rp[i + 1];
            if (e == e1) atomicOr(status, ST_EMPTY_ROW);
            for (; e < e1 && col[e] < i0; ++e) s = A::add(s, A::mul(val[e], ld_sc1(&yc[col[e]])));
        }
        const int64_t nb = (n - i0 < FW_BLOCK) ? n - i0 : FW_BLOCK;
        for (int64_t tt = 0; tt < nb; ++tt) {
            const int64_t j = i0 + tt;
            if (t == tt && e1 > rp[i]) {
                const T y = div_rn(A::sub(bc[i], s), val[e1 - 1]);
                s_y[tt] = y;
                st_sc1(&yc[i], y);
            } else if (t == tt) {
                s_y[tt] = A::zero();
            }
            __syncthreads();
            if (i < n && i > j)
                for (; e < e1 && col[e] == j; ++e) s = A::add(s, A::mul(val[e], s_y[tt]));
            __syncthreads();
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// backward: rows descending; sum over the row's entries after the FIRST, in
// storage order; x of not-yet-solved rows reads 0 (as the reference's zero-
// initialised Dense does). One wavefront per RHS column.
template <typename T>
__global__ __launch_bounds__(64) void csr_backward(int64_t n, const int64_t* __restrict__ rp,
                                                   const int32_t* __restrict__ col, const T* __restrict__ val,
                                                   const T* __restrict__ Yin, T* __restrict__ X,
                                                   int* __restrict__ status) {
    using A = Arith<T>;
    __shared__ T prod[2048];
    const int lane = threadIdx.x;
    const T* yc = Yin + (int64_t)blockIdx.x * n;
    T* xc = X + (int64_t)blockIdx.x * n;
    for (int64_t i = n - 1; i >= 0; --i) {
        const int64_t a = rp[i], e1 = rp[i + 1];
        if (a == e1) {
            if (lane == 0) atomicOr(status, ST_EMPTY_ROW);
            continue;
        }
        T s = A::zero();
        for (int64_t cs = a + 1; cs < e1; cs += 2048) {
            const int64_t cn = (e1 - cs < 2048) ? e1 - cs : 2048;
            for (int64_t d = lane; d < cn; d += 64) prod[d] = A::mul(val[cs + d], ld_sc1(&xc[col[cs + d]]));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0)
                for (int64_t d = 0; d < cn; ++d) s = A::add(s, prod[d]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0) {
            st_sc1(&xc[i], div_rn(A::sub(yc[i], s), val[a]));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_wave_barrier();
    }
}

inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------
struct Band {
    DBuf cb;
    int64_t n = 0, b = 0, ld = 1;
};

int band_analyse(const bsm_csr* a, hipStream_t s, int64_t* bw_out, bool* sorted, bool* empty_rows) {
    DBuf bw;
    BSM_TRY(bw.alloc(3 * sizeof(uint64_t)));
    BSM_HIP_TRY(hipMemsetAsync(bw.p, 0, 3 * sizeof(uint64_t), s));
    if (a->rows) {
        band_width<<<nblk(a->rows, 256), 256, 0, s>>>(a->row_ptr, a->col, (int64_t)a->rows,
                                                      bw.as<unsigned long long>());
        BSM_HIP_TRY(hipGetLastError());
    }
    uint64_t h[3];
    BSM_HIP_TRY(hipMemcpyAsync(h, bw.p, sizeof(h), hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    *bw_out = (int64_t)h[0];
    *sorted = h[1] == 0;
    *empty_rows = h[2] != 0;
    return BSM_OK;
}

template <typename T, int M>
int launch_chol(Band& bd, int* progress, int* status, hipStream_t s) {
    const int64_t n_tiles = (bd.n + TR - 1) / TR;
    const size_t shm = (size_t)(bd.b + 1) * sizeof(T);
    int dev = 0, cus = 0;
    BSM_HIP_TRY(hipGetDevice(&dev));
    BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int per_cu = 0;
    BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, band_chol<T, M>, CH_THREADS, shm));
    BSM_REQUIRE(per_cu >= 1, BSM_ERR_UNSUPPORTED, "band_chol does not fit a CU");
    // every workgroup must be resident (tile-row I waits on tile-row I-1)
    int64_t grid = cus;
    if (grid > n_tiles) grid = n_tiles;
    if (grid < 1) grid = 1;
    band_chol<T, M><<<(unsigned)grid, CH_THREADS, shm, s>>>(bd.n, bd.b, bd.ld, bd.cb.as<T>(), progress, status,
                                                             n_tiles);
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

template <typename T>
int band_factor(const bsm_csr* a, Band& bd, hipStream_t s) {
    int64_t bw = 0;
    bool sorted = true, empty = false;
    BSM_TRY(band_analyse(a, s, &bw, &sorted, &empty));
    BSM_REQUIRE(sorted, BSM_ERR_UNSUPPORTED,
                "cholesky: rows must have strictly increasing columns (get_row_complete semantics)");
    const int64_t need = bw + TR;  // accumulators per row pair lane set
    BSM_REQUIRE(need <= 64 * 17, BSM_ERR_UNSUPPORTED, "cholesky: bandwidth %lld > %d not supported",
                (long long)bw, 64 * 17 - TR);
    bd.n = (int64_t)a->rows;
    bd.b = bw;
    bd.ld = bw + 1;
    BSM_TRY(bd.cb.alloc((size_t)bd.n * bd.ld * sizeof(T)));
    BSM_HIP_TRY(hipMemsetAsync(bd.cb.p, 0, (size_t)bd.n * bd.ld * sizeof(T), s));
    if (bd.n == 0) return BSM_OK;
    band_fill<T><<<nblk(bd.n, 256), 256, 0, s>>>(a->row_ptr, a->col, static_cast<const T*>(a->vals), bd.n, bd.ld,
                                                 bd.cb.as<T>());
    BSM_HIP_TRY(hipGetLastError());
    const int64_t n_tiles = (bd.n + TR - 1) / TR;
    DBuf prog;
    BSM_TRY(prog.alloc((n_tiles + 1) * sizeof(int) + 16));
    BSM_HIP_TRY(hipMemsetAsync(prog.p, 0, (n_tiles + 1) * sizeof(int) + 16, s));
    int* status = prog.as<int>() + n_tiles;
    int rc;
    if (need <= 64) rc = launch_chol<T, 1>(bd, prog.as<int>(), status, s);
    else if (need <= 128) rc = launch_chol<T, 2>(bd, prog.as<int>(), status, s);
    else if (need <= 256) rc = launch_chol<T, 4>(bd, prog.as<int>(), status, s);
    else if (need <= 512) rc = launch_chol<T, 8>(bd, prog.as<int>(), status, s);
    else rc = launch_chol<T, 17>(bd, prog.as<int>(), status, s);
    BSM_TRY(rc);
    int st = 0;
    BSM_HIP_TRY(hipMemcpyAsync(&st, status, sizeof(int), hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_REQUIRE(!(st & ST_TIMEOUT), BSM_ERR_HIP, "cholesky: tile-row hand-off timed out");
    BSM_REQUIRE(!(st & ST_NOT_PD), BSM_ERR_UNSUPPORTED,
                "cholesky: matrix is not positive definite (a pivot is <= 0 or not finite); the reference "
                "would store NaN/inf there, which this build does not reproduce");
    return BSM_OK;
}

template <typename T>
int band_to_csr_host(const Band& bd, int dtype, bsm_csr** out, hipStream_t s) {
    const uint64_t n = (uint64_t)bd.n;
    DBuf cnt, ws;
    BSM_TRY(cnt.alloc(n * sizeof(int32_t)));
    BSM_TRY(ws.alloc(scan_workspace_bytes(n)));
    DBuf rp;
    BSM_TRY(rp.alloc((n + 1) * sizeof(int64_t)));
    if (n)
        band_row_count<T><<<nblk(n, 256), 256, 0, s>>>(bd.n, bd.b, bd.ld, bd.cb.as<T>(), cnt.as<int32_t>());
    BSM_HIP_TRY(hipGetLastError());
    BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), rp.as<int64_t>(), n, ws.p, ws.bytes, s));
    int64_t nnz = 0;
    BSM_HIP_TRY(hipMemcpyAsync(&nnz, rp.as<int64_t>() + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    auto* m = new bsm_csr();
    m->dtype = dtype;
    m->rows = n;
    m->cols = n;
    m->nnz = (uint64_t)nnz;
    BSM_HIP_TRY(hipGetDevice(&m->device));
    DBuf c, v;
    int rc = c.alloc((uint64_t)nnz * sizeof(int32_t));
    if (rc == BSM_OK) rc = v.alloc((uint64_t)nnz * sizeof(T));
    if (rc != BSM_OK) { delete m; return rc; }
    m->row_ptr = static_cast<int64_t*>(rp.release());
    m->col = static_cast<int32_t*>(c.release());
    m->vals = v.release();
    m->analysed = true;
    m->rows_sorted = true;
    if (n)
        band_to_csr<T><<<nblk(n, 256), 256, 0, s>>>(bd.n, bd.b, bd.ld, bd.cb.as<T>(), m->row_ptr, m->col,
                                                    static_cast<T*>(m->vals));
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        bsm_csr_free(m);
        set_error("band_to_csr: %s", hipGetErrorString(e));
        return BSM_ERR_HIP;
    }
    *out = m;
    return BSM_OK;
}

}  // namespace

// b_dev / x_dev: k columns of n values each, column-major (column j at j*n).
// NOTE: the host entry points pass ROW-major n x k device buffers; for k > 1
// they are transposed into column-major scratch first (see solve_io).
static int to_colmajor(int dtype, uint64_t n, uint64_t k, const void* rowmajor, DBuf& out, hipStream_t s) {
    BSM_TRY(out.alloc(n * k * dtype_size(dtype)));
    if (k == 1) {
        if (n) BSM_HIP_TRY(hipMemcpyAsync(out.p, rowmajor, n * dtype_size(dtype), hipMemcpyDeviceToDevice, s));
        return BSM_OK;
    }
    return unpack_rowmajor_to_cols(dtype, n, k, rowmajor, out.p, s);
}
static int from_colmajor(int dtype, uint64_t n, uint64_t k, const void* colmajor, void* rowmajor, hipStream_t s) {
    if (k == 1) {
        if (n) BSM_HIP_TRY(hipMemcpyAsync(rowmajor, colmajor, n * dtype_size(dtype), hipMemcpyDeviceToDevice, s));
        return BSM_OK;
    }
    return pack_cols_to_rowmajor(dtype, n, k, colmajor, rowmajor, s);
}

int solve_dispatch_cholesky(const bsm_csr* a, bsm_csr** out, hipStream_t s) {
    auto run = [&]<typename T>() -> int {
        Band bd;
        BSM_TRY(band_factor<T>(a, bd, s));
        return band_to_csr_host<T>(bd, a->dtype, out, s);
    };
    if (a->dtype == BSM_F64) return run.template operator()<double>();
    if (a->dtype == BSM_F32) return run.template operator()<float>();
    set_error("cholesky: f32/f64 only");
    return BSM_ERR_INVALID;
}

int solve_dispatch_trsv(const bsm_csr* m, bool lower, uint64_t k, uint64_t n, const void* b_dev, void* x_dev,
                        hipStream_t s) {
    auto run = [&]<typename T>() -> int {
        bsm_csr* mm = const_cast<bsm_csr*>(m);
        BSM_TRY(csr_analyse(mm, s));
        BSM_REQUIRE(m->rows_sorted, BSM_ERR_UNSUPPORTED,
                    "triangular solve: rows must be sorted by column (storage order = column order)");
        DBuf bc, xc, st;
        BSM_TRY(to_colmajor(m->dtype, n, k, b_dev, bc, s));
        BSM_TRY(xc.alloc(n * k * sizeof(T)));
        BSM_HIP_TRY(hipMemsetAsync(xc.p, 0, n * k * sizeof(T), s));  // Dense::new_default_with_dims
        BSM_TRY(st.alloc(16));
        BSM_HIP_TRY(hipMemsetAsync(st.p, 0, 16, s));
        if (n && k) {
            if (lower)
                csr_forward<T><<<(unsigned)k, FW_BLOCK, 0, s>>>((int64_t)n, m->row_ptr, m->col,
                                                               static_cast<const T*>(m->vals), bc.as<T>(),
                                                               xc.as<T>(), st.as<int>());
            else
                csr_backward<T><<<(unsigned)k, 64, 0, s>>>((int64_t)n, m->row_ptr, m->col,
                                                          static_cast<const T*>(m->vals), bc.as<T>(), xc.as<T>(),
                                                          st.as<int>());
            BSM_HIP_TRY(hipGetLastError());
        }
        int h = 0;
        BSM_HIP_TRY(hipMemcpyAsync(&h, st.p, sizeof(int), hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        BSM_REQUIRE(!(h & ST_EMPTY_ROW), BSM_ERR_PANIC,
                    "called `Option::unwrap()` on a `None` value: empty row (lib.rs:41 / :60)");
        BSM_TRY(from_colmajor(m->dtype, n, k, xc.p, x_dev, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        return BSM_OK;
    };
    if (m->dtype == BSM_F64) return run.template operator()<double>();
    if (m->dtype == BSM_F32) return run.template operator()<float>();
    set_error("triangular solve: f32/f64 only");
    return BSM_ERR_INVALID;
}

int solve_dispatch_full(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev, hipStream_t s) {
    auto run = [&]<typename T>() -> int {
        BSM_REQUIRE(a->rows == n, BSM_ERR_PANIC,
                    "solve: b has %llu rows but A has %llu (index out of bounds in the reference)",
                    (unsigned long long)n, (unsigned long long)a->rows);
        Band bd;
        BSM_TRY(band_factor<T>(a, bd, s));
        // the reference's forward pass divides by the LAST stored entry of
        // each L row and its backward pass by the FIRST of each L^T row: with
        // every pivot > 0 (checked) both are L_ii, as used below.
        BSM_REQUIRE(bd.b < FW_RING - FW_BLOCK && bd.b < BW_RING, BSM_ERR_UNSUPPORTED, "band too wide");
        DBuf bc, yc, xc;
        BSM_TRY(to_colmajor(a->dtype, n, k, b_dev, bc, s));
        BSM_TRY(yc.alloc(n * k * sizeof(T)));
        BSM_TRY(xc.alloc(n * k * sizeof(T)));
        if (n && k) {
            // forward_substitution(l, b) over rows 0..n of L (lib.rs:31-44)
            band_forward<T><<<(unsigned)k, FW_BLOCK, 0, s>>>((int64_t)n, bd.b, bd.ld, bd.cb.as<T>(), bc.as<T>(),
                                                             yc.as<T>());
            BSM_HIP_TRY(hipGetLastError());
            band_backward<T><<<(unsigned)k, 64, 0, s>>>((int64_t)n, bd.b, bd.ld, bd.cb.as<T>(), yc.as<T>(),
                                                        xc.as<T>());
            BSM_HIP_TRY(hipGetLastError());
        }
        BSM_TRY(from_colmajor(a->dtype, n, k, xc.p, x_dev, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        return BSM_OK;
    };
    if (a->dtype == BSM_F64) return run.template operator()<double>();
    if (a->dtype == BSM_F32) return run.template operator()<float>();
    set_error("solve: f32/f64 only");
    return BSM_ERR_INVALID;
}

}  // namespace bsm
