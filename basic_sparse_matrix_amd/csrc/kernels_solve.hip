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
// Kernels, one per stage and order (the measured variants they replaced
// are in DESIGN.md §4.5-§4.6 and in git history):
//   reference order (bit-exact): band_chol5 -> band_forward2 -> band_backward_reg;
//   general exact path (non-SPD, unsorted, b > 1073; n <= 16384): chol_general;
//   blocked (reassociated, within BASELINE's 1e-6 on f64): blk_chol ->
//   blk_prep -> blk_trsv (forward, backward).
// Hand-offs between workgroups use write-through (sc1) stores, a drain and a
// relaxed agent flag (MI355X_MICROARCH.md "Valid forms", table row 1).
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

#include <unistd.h>

#include <atomic>
#include <thread>

#include "bsm_internal.hpp"

namespace bsm {
namespace {

#include "solve_tiles.hpp"

constexpr int TR = 16;              // rows per tile-row


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

// a / b correctly rounded with b's reciprocal y = RN(1/b) computed off the
// chain (Markstein: q = RN(a y), r = a - b q exactly by FMA, RN(q + r y) =
// RN(a / b) when y = RN(1/b) and nothing underflows or overflows). 28 instead
// of 76 cycles of dependent latency (scripts/micro/div_latency.hip); checked
// against IEEE division on 4e8 random pairs, significands near all-ones
// included. Outside |a| in [2^-900, 2^900] (zeros, subnormals, inf, NaN) the
// IEEE division is used (wave-uniform branch, out of line).
__device__ __forceinline__ double div_by(double a, double b, double y) {
    const double aa = fabs(a);
    if (__builtin_expect(__all(aa >= 0x1p-900 && aa <= 0x1p900), 1)) {
        const double q = __dmul_rn(a, y);
        const double r = __fma_rn(-q, b, a);
        return __fma_rn(r, y, q);
    }
    return __ddiv_rn(a, b);
}
__device__ __forceinline__ float div_by(float a, float b, float) { return div_rn(a, b); }

// zero elements after the band: the backward solve's fixed-length walks of
// the last rows read them
__host__ __device__ inline int64_t band_pad(int64_t ld) { return 32 * ld + 4096; }

__device__ __forceinline__ double readlane_t(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float readlane_t(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}


// √ of a pivot the caller has checked positive and finite: IEEE sqrt
// correctly rounded (f32: formed in f64, rounded once, as pow_half). A pivot
// that fails the check flags ST_NOT_PD and its factor is discarded, so the
// -inf / -0 cases of pow_half need no handling here.
__device__ __forceinline__ double sqrt_pos(double x) { return __dsqrt_rn(x); }
__device__ __forceinline__ float sqrt_pos(float x) { return __double2float_rn(__dsqrt_rn((double)x)); }

// diag_factor16 with the per-step side work taken off the pivot chain: the
// pivot check is one class test per step folded into a flag (one atomic at
// the end), 1/L[t][t] is kept by lane t (one select), and L's column t goes
// to registers. Then, by SM:
//   SM = 1: wave 0 stores the block and R after the 16 steps;
//   SM = 2: the block and R go to LDS (Ls[r][t], Rs[t]) for the whole
//           workgroup to store (diag_store16) behind a barrier.
// IL: each step's updates of the columns past the next pivot's are issued in
// the following step, beside its sqrt -> reciprocal chain (measured slower:
// 8.7k against 8.1k cycles per block without, against 9.1k for diag_factor16;
// scripts/micro/diag_factor.hip).
// Same operations per element in the same order: the same bits as diag_factor16.
template <typename T, int SM, bool IL = false>
__device__ __forceinline__ void diag_factor16x(const T (*dacc)[17], const T (*dA)[17], T (*Ls)[17], T* Rs, int i0,
                                               int64_t n, int64_t b, int64_t ld, T* CB, T* R, int* status, int c) {
    using A = Arith<T>;
    constexpr int NB = 16;
    asm volatile("" : "+v"(c));
    const int r = c & (NB - 1);
    const bool live = i0 + r < n;
    T q[NB], a[NB], xs[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        q[j] = live ? dacc[r][j] : A::zero();
        a[j] = live ? dA[r][j] : (r == j ? (T)1 : A::zero());
    }
    T myrt = A::zero();
    bool pd = true;
    auto step = [&]<int t>(std::integral_constant<int, t>) __attribute__((always_inline)) {
        const T v = A::sub(a[t], q[t]);
        const T vv = rowbcast<t>(v);
        pd = pd && __builtin_isfinite(vv) && vv > A::zero();
        const T piv = sqrt_pos(vv);
        const T rt = div_rn((T)1, piv);
        const T x = r == t ? piv : A::mul(rt, v);  // L[i0 + r][i0 + t] for r >= t
        xs[t] = x;
        myrt = c == t ? rt : myrt;
        if constexpr (IL) {
            // step t - 1's updates of the columns after t + 1, placed beside this
            // step's pivot chain (one scheduling region: they fill its latency),
            // then this step's update of column t + 1 (the next pivot's)
            if constexpr (t >= 1) {
                const T xp = xs[t - 1];
                [&]<int... js>(std::integer_sequence<int, js...>) __attribute__((always_inline)) {
                    ((q[t + 1 + js] = A::add(q[t + 1 + js], A::mul(xp, rowbcast<t + 1 + js>(xp)))), ...);
                }(std::make_integer_sequence<int, NB - 1 - t>{});
            }
            if constexpr (t + 1 < NB) q[t + 1] = A::add(q[t + 1], A::mul(x, rowbcast<t + 1>(x)));
        } else {
            [&]<int... js>(std::integer_sequence<int, js...>) __attribute__((always_inline)) {
                ((q[t + 1 + js] = A::add(q[t + 1 + js], A::mul(x, rowbcast<t + 1 + js>(x)))), ...);
            }(std::make_integer_sequence<int, NB - 1 - t>{});
        }
#pragma unroll
        for (int j = t + 1; j < NB; ++j) asm volatile("" : "+v"(q[j]));
    };
    [&]<int... ts>(std::integer_sequence<int, ts...>) __attribute__((always_inline)) {
        (step(std::integral_constant<int, ts>{}), ...);
    }(std::make_integer_sequence<int, NB>{});
    if (c == 0 && !pd) atomicOr(status, ST_NOT_PD);
    if constexpr (SM == 1) {
        if (c < NB && live) {
            T* p = CB + (int64_t)i0 * ld + r;  // L[i0 + r][i0 + t] = CB[(i0 + t) ld + r - t]
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                if (r >= t && r - t <= b) st_sc1(p, xs[t]);
                p += ld - 1;
            }
            st_sc1(&R[i0 + r], myrt);
        }
    } else {
        if (c < NB) {
#pragma unroll
            for (int t = 0; t < NB; ++t) Ls[r][t] = xs[t];
            Rs[r] = myrt;
        }
    }
}

// The stores of diag_factor16x<T, 2>'s block, by NT threads (after a barrier
// behind the factor): L[i0 + r][i0 + t] for r >= t, r - t <= b, and R.
template <typename T, int NT>
__device__ __forceinline__ void diag_store16(const T (*Ls)[17], const T* Rs, int i0, int64_t n, int64_t b,
                                             int64_t ld, T* CB, T* R, int tid) {
    for (int e = tid; e < 16 * 16 + 16; e += NT) {
        if (e < 256) {
            const int t = e >> 4, d = e & 15, r = t + d;  // column t, offset d: coalesced along the band
            if (r < 16 && d <= b && i0 + r < n) st_sc1(&CB[(int64_t)(i0 + t) * ld + d], Ls[r][t]);
        } else {
            const int r = e - 256;
            if (i0 + r < n) st_sc1(&R[i0 + r], Rs[r]);
        }
    }
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

constexpr int C4_TB = 16;  // rows per row-block / columns per tile

// fprog[J]: row-block J's progress (tiles final); tiles before the band are
// structurally zero
__global__ __launch_bounds__(256) void chol_prog_init(int64_t n_tiles, int64_t b, int* __restrict__ fprog) {
    const int64_t J = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (J >= n_tiles) return;
    const int64_t lo = C4_TB * J - b;
    fprog[J] = (int)((lo > 0 ? lo : 0) / C4_TB);  // tiles before the band: structurally zero
}

// ---------------------------------------------------------------------------
// band_chol5: the exact (reference-order) band Cholesky, b <= 1073.
// Tile events. Row-block I = rows [16 I, 16 I + 16) is one workgroup of
// 16 / RP waves (RP rows per wave; RP = 2 is instantiated), taken by ticket
// in ascending order. Column tile K = columns [16 K, 16 K + 16). Row i's
// accumulators for the columns left of its row-block sit in M register
// slots (lane c of slot m: column jb + c + 64 m, jb = 16 K0 the band start
// aligned down), so tile K is lanes 16 e .. 16 e + 15 of slot m, 16 (K - K0)
// = 64 m + 16 e. Per off-diagonal tile K, in ascending order:
//   T (needs row-block K complete, fprog[K] > K): the rows' x across the
//     tile's 16 columns, x_t = (1/L[t][t]) (A - acc_t), acc_t' += x_t L[t'][t]:
//     row-block K's diagonal tile, 1/L and the rows' own A values go straight
//     into registers and the 16 chain steps take lane t's values by DPP
//     row_newbcast (VALU only); write-through stores, drain, barrier,
//     fprog[I] = K + 1;
//   U (needs fprog[J] > K for the row-blocks J in (K, I), one vector poll):
//     stage column tile K of those rows in LDS and add its 16 terms to every
//     later accumulator (software-pipelined: step t + 1's LDS reads before
//     step t's multiply-adds), and to the diagonal-block sums. Look-ahead: the
//     slot holding tile K + 1 right after the staging, then T(K + 1), then the
//     other slots (per accumulator the tiles still come in ascending order).
// Then the 16 x 16 diagonal block (wave 0, diag_factor16x) while the other
// waves store the last tile's L from LDS; completion (fprog[I] = I + 1) is
// raised by the last wave to arrive after its own drain.
// Per element the reference's operations in its order (ascending k, no FMA,
// (1/L[k][k]) * (A - sum), sparse.rs:689-708): bit-identical to the oracle.
// Measured variants (each dropped, DESIGN.md §4.5b'): four rows per wave,
// the last tile stored before the factor, late T publication, per-wave polls,
// split staging of U, two staging rows per thread.
// ---------------------------------------------------------------------------
template <typename T, int M, int RP>  // RP rows per wave: 16 / RP waves
__global__ __launch_bounds__(64 * (16 / RP)) void band_chol5(int64_t n, int64_t b, int64_t ld, T* __restrict__ CB,
                                                    T* __restrict__ R, int* __restrict__ fprog,
                                                    int* __restrict__ status, int* __restrict__ ticket,
                                                    int64_t n_tiles, unsigned long long* __restrict__ trace,
                                                    int delay) {
    using A = Arith<T>;
    constexpr int CS = 64 + 64 * M;
    constexpr int C5_NT = 64 * (16 / RP);
    __shared__ T colK[C4_TB][CS];
    __shared__ T hist2[2][C4_TB][C4_TB + 1];  // by tile parity: T(K + 1) may write while U(K) reads
    __shared__ T dacc[TR][TR + 1], dA[TR][TR + 1];
    __shared__ T xl[16];
    __shared__ long long tph[16];
    __shared__ int s_arr;  // waves past the last tile's stores (after the windows)
    if (threadIdx.x == 0) s_arr = 0;
    const int tid = threadIdx.x, w = tid >> 6, c = tid & 63;
    for (int q = tid; q < C4_TB * 64; q += C5_NT) colK[q >> 6][q & 63] = A::zero();
    const int ib = (int)b;
    auto poll_all = [&](int jlo, int jhi, int need) {  // wave 0: fprog[J] >= need for J in [jlo, jhi)
        bool ok = true;
        for (int base = jlo; base < jhi; base += 64) {  // more than 64 row-blocks: several lanes' worth
            const int J = base + c;
            bool okj = J >= jhi;
            long long spins = 0;
            while (true) {
                if (!okj) okj = __hip_atomic_load(&fprog[J], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need;
                if (__all(okj)) break;
                __builtin_amdgcn_s_sleep(1);
                if (++spins > SPIN_LIMIT ||
                    ((spins & 1023) == 0 &&
                     (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ST_TIMEOUT))) {
                    if (c == 0) atomicOr(status, ST_TIMEOUT);
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
        }
    };
    __shared__ int s_tk;
    for (int64_t I = next_ticket(ticket, &s_tk); I < n_tiles; I = next_ticket(ticket, &s_tk)) {
        const int i0 = (int)(I * C4_TB);
        const int K0 = (i0 - ib > 0 ? i0 - ib : 0) / C4_TB, jb = C4_TB * K0;
        const int r0 = RP * w;  // this wave's rows: i0 + r0 .. i0 + r0 + RP - 1
        long long tlast = 0;
        const bool tr0 = trace && tid == 0;
        if (tr0) {
#pragma unroll
            for (int q = 0; q < 16; ++q) tph[q] = 0;
            tlast = clock64();
        }
        auto mark = [&](bool last, int ph) {
            if (tr0) {
                const long long t = clock64();
                if (last) tph[6 + ph] += t - tlast;
                else tph[ph] += t - tlast;
                tlast = t;
            }
        };
        T acc[RP][M];
#pragma unroll
        for (int q = 0; q < RP; ++q)
#pragma unroll
            for (int m = 0; m < M; ++m) acc[q][m] = A::zero();
        // the diagonal block's A values go to LDS now (dA is free since the
        // last row-block's factor): their load is waited for here, not behind
        // the last tile's stores
        T accT[RP];
#pragma unroll
        for (int q = 0; q < RP; ++q) {
            const int rw = r0 + q;
            accT[q] = A::zero();
            const T aT = (c < C4_TB && c <= rw && rw - c <= ib && i0 + rw < n)
                             ? ld_sc1(CB + (int64_t)(i0 + c) * ld + (rw - c))
                             : A::zero();
            if (c < TR) dA[rw][c] = aT;
        }
        // U over accumulator slots [LO, HI) for the column tile staged in colK
        // (tile slot mK, lanes lbK..lbK+15) with the tile's x in hs; WT: also the
        // diagonal-block sums. Software-pipelined: step t + 1's LDS reads (x,
        // column values, diagonal-block value) go out before step t's
        // multiply-adds. Each tile's U is split (look-ahead): the slot holding
        // the next tile's columns right after the tile's T, so the next T can
        // start, the other slots after that T. Per accumulator the tiles still
        // come in ascending order (T touches only its own tile's slot), so the
        // bits are unchanged; the split takes U's bulk off the dependency from
        // one row-block's T(K) to the next one's T(K + 1) (~40k cycles per
        // row-block before, with the whole U(K) on that path).
        // column tile K's rows k0 + 16 + rr, rr in [lo, hi), into colK
        auto stage_rows = [&](int k0s, int lo, int hi) __attribute__((always_inline)) {
            for (int rr = lo + tid; rr < hi; rr += C5_NT) {
                const T* base = CB + (int64_t)k0s * ld + C4_TB + rr;
                T v[C4_TB];
#pragma unroll
                for (int t = 0; t < C4_TB; ++t) v[t] = ld_sc1(base + (int64_t)t * (ld - 1));
#pragma unroll
                for (int t = 0; t < C4_TB; ++t) colK[t][64 + rr] = C4_TB + rr - t <= ib ? v[t] : A::zero();
            }
        };
        auto u_run = [&]<int LO, int HI, bool WT>(std::integral_constant<int, LO>, std::integral_constant<int, HI>,
                                                  std::bool_constant<WT>, int mK, int lbK,
                                                  T (*hs)[C4_TB + 1]) __attribute__((always_inline)) {
            if constexpr (LO < HI) {
                struct UB {
                    T cv[HI - LO], x[RP], hv;
                };
                auto u_load = [&](int t, UB& ub) __attribute__((always_inline)) {
#pragma unroll
                    for (int q = 0; q < RP; ++q) ub.x[q] = hs[t][r0 + q];
                    const T* col = &colK[t][64 + c - lbK - C4_TB];  // col[64 (mm - mK)]: column jb + c + 64 mm
#pragma unroll
                    for (int mm = LO; mm < HI; ++mm) ub.cv[mm - LO] = col[64 * (mm - mK)];
                    if constexpr (WT) ub.hv = hs[t][c & 15];
                };
                auto u_add = [&](const UB& ub) __attribute__((always_inline)) {
#pragma unroll
                    for (int mm = LO; mm < HI; ++mm)
                        if (jb + 64 * mm < i0) {
#pragma unroll
                            for (int q = 0; q < RP; ++q)
                                acc[q][mm] = A::add(acc[q][mm], A::mul(ub.x[q], ub.cv[mm - LO]));
                        }
                    if constexpr (WT) {
                        if (c < C4_TB) {
#pragma unroll
                            for (int q = 0; q < RP; ++q) accT[q] = A::add(accT[q], A::mul(ub.x[q], ub.hv));
                        }
                    }
                };
                UB ua, ubb;
                u_load(0, ua);
#pragma unroll 1
                for (int t = 0; t < C4_TB; t += 2) {
                    u_load(t + 1, ubb);
                    __builtin_amdgcn_sched_barrier(0);
                    u_add(ua);
                    if (t + 2 < C4_TB) u_load(t + 2, ua);
                    __builtin_amdgcn_sched_barrier(0);
                    u_add(ubb);
                }
            }
        };
        auto window = [&]<int m>(std::integral_constant<int, m>) __attribute__((always_inline)) {
#pragma unroll 1
            for (int e = 0; e < 4; ++e) {
                const int K = K0 + 4 * m + e;
                if (K >= (int)I) return;
                const int k0 = C4_TB * K, lb = 16 * e;
                const bool lastK = K == (int)I - 1;
                // ---------------- T: this row-block's tile K
                // the rows' own A values for the tile's columns (nobody else writes
                // them): loaded before the wait, straight into the lanes (lane c:
                // column k0 + (c & 15))
                T myA[RP];
#pragma unroll
                for (int q = 0; q < RP; ++q) {
                    const int rw = r0 + q, cl = c & 15, d = i0 + rw - k0 - cl;
                    const bool ok = d <= ib && i0 + rw < n;
                    const T v = ld_sc1(CB + (((int64_t)(k0 + cl) * ld + d) & -(int64_t)ok));
                    myA[q] = ok ? v : A::zero();
                }
                // row-block K's diagonal tile and 1/L, per lane, straight into
                // registers (no LDS staging, no second barrier): lane c takes
                // L[k0 + t + u][k0 + t], u = c - lb - t, for every t
                T dvr[C4_TB], myR;
                if (w == 0) poll_all(K, K + 1, K + 1);
                mark(lastK, 0);
                __syncthreads();
                auto& hist = hist2[K & 1];
#pragma unroll
                for (int t = 0; t < C4_TB; ++t) {
                    const int u = c - lb - t;
                    const bool ok = u >= 1 && t + u <= 15 && u <= ib;
                    const T v = ld_sc1(CB + (((int64_t)(k0 + t) * ld + u) & -(int64_t)ok));
                    dvr[t] = ok ? v : A::zero();
                }
                myR = ld_sc1(&R[k0 + (c & 15)]);
                mark(lastK, 1);
                // The tile's 16 columns are lanes lb .. lb + 15 of slot m: one DPP row
                // (row e). Step t takes lane lb + t's accumulator, 1/L and A by
                // row_newbcast (VALU, no SGPR round trip on the chain); every row of
                // lanes gets its own lane t, so x is right in row e only and is
                // zeroed elsewhere (dv is 0 there too: no term reaches other columns)
                const bool inrow = (c >> 4) == e;
                T xv[RP];
#pragma unroll
                for (int q = 0; q < RP; ++q) xv[q] = A::zero();
                [&]<int... ts>(std::integer_sequence<int, ts...>) __attribute__((always_inline)) {
                    (([&] {
                         constexpr int t = ts;
                         const T dv = dvr[t];
                         const T rt = rowbcast<t>(myR);
#pragma unroll
                         for (int q = 0; q < RP; ++q) {
                             const T sq = rowbcast<t>(acc[q][m]);
                             const T x0 = A::mul(rt, A::sub(rowbcast<t>(myA[q]), sq));
                             const T x = inrow ? x0 : A::zero();
                             acc[q][m] = A::add(acc[q][m], A::mul(x, dv));
                             if (c == lb + t) xv[q] = x;
                         }
                     }()),
                     ...);
                }(std::make_integer_sequence<int, C4_TB>{});
                if (inrow) {  // (the last tile's band stores wait until the factor runs: below)
                    const int cl = c & 15;
#pragma unroll
                    for (int q = 0; q < RP; ++q) {
                        const int rw = r0 + q;
                        hist[cl][rw] = xv[q];
                        const int d = i0 + rw - k0 - cl;
                        if (!lastK && d <= ib && i0 + rw < n)
                            st_sc1(&CB[(int64_t)(k0 + cl) * ld + d], xv[q]);
                    }
                }
                if (lastK) {  // no rows in between: the diagonal-block sums of this tile
                    mark(true, 2);
                    __syncthreads();
                    mark(true, 4);
                    // the rows' own x come from hist (an LDS broadcast), NOT by
                    // v_readlane of xv from lane lb + t: inside this lane-divergent
                    // branch (exec = lanes 0-15) lanes 16-63 of xv are dead to the
                    // compiler, and an exec-masked copy of xv (the RP = 4 build,
                    // 442 registers) left lane lb + t stale: the diagonal sums of
                    // row-blocks whose last tile sits at e >= 1 missed that tile
                    // (round 5, scripts/chol_rp4_debug.py; DESIGN.md §4.5b')
                    if (c < C4_TB) {
                        T hc[C4_TB];
#pragma unroll
                        for (int t = 0; t < C4_TB; ++t) hc[t] = hist[t][c];
#pragma unroll
                        for (int t = 0; t < C4_TB; ++t)
#pragma unroll
                            for (int q = 0; q < RP; ++q)
                                accT[q] = A::add(accT[q], A::mul(hist[t][r0 + q], hc[t]));
                    }
                    mark(true, 5);
                    return;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                mark(false, 2);
                __syncthreads();
                if (tid == 0) __hip_atomic_store(&fprog[I], K + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // ---------------- the rest of U(K - 1): the slots after tile K's,
                // which T(K) did not need (look-ahead: see u_run below)
                mark(false, 3);
                if (K > K0) {
                    if (e) u_run(std::integral_constant<int, m + 1>{}, std::integral_constant<int, M>{},
                                 std::false_type{}, m, lb - C4_TB, hist2[(K - 1) & 1]);
                    else if constexpr (m >= 1)
                        u_run(std::integral_constant<int, m + 1>{}, std::integral_constant<int, M>{},
                              std::false_type{}, m - 1, 48, hist2[(K - 1) & 1]);
                }
                mark(false, 5);
                // ---------------- U(K): column tile K of the rows between, once they have it
                const int cnt = i0 - k0 - C4_TB;  // rows k0 + 16 .. i0 - 1
                if (w == 0) poll_all(K + 1, (int)I, K + 1);  // (K + 1 <= I - 1)
                __syncthreads();
                stage_rows(k0, 0, cnt);
                __syncthreads();
                mark(false, 4);
                // now only the slot holding tile K + 1 (and the diagonal-block
                // sums); the other slots after the next T
                if (e < 3) {
                    u_run(std::integral_constant<int, m>{}, std::integral_constant<int, m + 1>{}, std::true_type{}, m,
                          lb, hist);
                } else if constexpr (m + 1 < M) {
                    u_run(std::integral_constant<int, m + 1>{}, std::integral_constant<int, m + 2>{},
                          std::true_type{}, m, lb, hist);
                }
                mark(lastK, 5);
            }
        };
        [&]<int... ms>(std::integer_sequence<int, ms...>) __attribute__((always_inline)) {
            (window(std::integral_constant<int, ms>{}), ...);
        }(std::make_integer_sequence<int, M>{});
        // ---------------- the 16 x 16 diagonal block (wave 0)
        // (the LDS addresses from an opaque copy of the thread index: hoisted,
        // they were spilled, and the reload's vmcnt(0) waited for the last
        // tile's write-through stores: 3.6k cycles on the chain)
        int tix = tid;
        asm volatile("" : "+v"(tix));
        if ((tix & 63) < TR) {
#pragma unroll
            for (int q = 0; q < RP; ++q) dacc[RP * (tix >> 6) + q][tix & 63] = accT[q];
        }
        __syncthreads();  // dacc visible
        mark(false, 12);
        // Completion (fprog[I] = I + 1) is raised by whichever of the 16 / RP
        // waves arrives LAST at s_arr after its own drain: wave 0 (the factor)
        // adds C5_W0, a store wave adds 1. Wave 0 publishing on its own drain
        // could let a consumer's U(I - 1) (it waits for fprog[I] >= I) read
        // the last tile's rows before the store waves' stores have landed
        // (ADVICE r4). The last store wave raises fprog[I] = I if wave 0 is
        // still factoring. Atomic max: the two values may land in either order.
        constexpr int C5_NSW = C5_NT / 64 - 1;  // store waves
        constexpr int C5_W0 = 0x100;
        const bool store_waves = K0 < (int)I;
        if (tid < 64) {
            diag_factor16x<T, 1>(dacc, dA, dacc, xl, i0, n, b, ld, CB, R, status, c);
            mark(false, 13);
            for (int q = delay; q < 0; ++q) __builtin_amdgcn_s_sleep(127);  // stress: wave 0 arrives last
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (c == 0) {
                if (!store_waves || (atomicAdd(&s_arr, C5_W0) & 0xff) == C5_NSW) {
                    if (store_waves) s_arr = 0;
                    __hip_atomic_fetch_max(&fprog[I], (int)I + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            mark(false, 14);
            if (tr0) {
#pragma unroll
                for (int q = 0; q < 15; ++q) atomicAdd(&trace[q], (unsigned long long)tph[q]);
                atomicAdd(&trace[15], 1ull);
                atomicAdd(&trace[16], (unsigned long long)((int)I - K0 - 1));
            }
        } else if (store_waves) {
            // While wave 0 factors, the other waves store the last tile's L
            // (from hist) and raise its progress flag (fprog[I] = I, which the
            // next row-blocks' U of tile I - 1 waits for): no store was in
            // flight before the barrier, so no wait there drained one. Each
            // wave waits for its own stores and arrives at s_arr; the last
            // store wave raises the flag, or completion if wave 0 has already
            // arrived (MI355X_MICROARCH.md "Valid forms": per-wave arrival).
            const int k0 = i0 - C4_TB;
            for (int q = 0; q < delay; ++q) __builtin_amdgcn_s_sleep(127);  // stress: the stores land late
            for (int e = tid - 64; e < C4_TB * C4_TB; e += C5_NT - 64) {
                const int t = e >> 4, rw = e & 15, d = i0 + rw - k0 - t;
                if (d <= ib && i0 + rw < n) st_sc1(&CB[(int64_t)(k0 + t) * ld + d], hist2[(I - 1) & 1][t][rw]);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (c == 0) {
                const int old = atomicAdd(&s_arr, 1);
                if ((old & 0xff) == C5_NSW - 1) {  // the last store wave
                    if (old >= C5_W0) s_arr = 0;   // wave 0 is done too: complete
                    __hip_atomic_fetch_max(&fprog[I], old >= C5_W0 ? (int)I + 1 : (int)I, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        __syncthreads();
    }
}

constexpr int FW_BLOCK = 256;  // csr_forward's rows per block

// ---------------------------------------------------------------------------
// band_forward2: the forward solve with one 64-row block per wave and no
// workgroup barrier. 16 waves per workgroup (one workgroup per RHS column);
// block B belongs to wave B % 16. A wave first adds, in ascending j, the
// terms of its rows left of the block -- following the "frontier" (rows
// whose y is final, an LDS counter) as the earlier blocks are solved -- and
// stages its block's 64 x 64 triangle of L into LDS. When the frontier
// reaches the block, it solves the block row by row: lane t forms
// y = (b - sum) / L[i][i] (true division, lib.rs:41), v_readlane broadcasts
// y, every later lane adds L[i][i0+t] * y. The serial chain per row is one
// subtraction, one division, one multiply and one add; the reads of the band
// (8 B per nonzero) are spread over the waiting waves.
// Terms outside the band are +0 products, which never change a sum that
// starts at +0 (bit-exact, as band_forward).
// ---------------------------------------------------------------------------
constexpr int FW2_RING = 4096;  // y ring (power of two >= b + NW * 64 + 64)

// NW waves, FW2_PF far-term loads in flight per lane: the waiting waves'
// bytes in flight are what hides the HBM latency of the row-wise band reads
//
// NH > 0: the far terms are split off. Per RHS column the grid holds one
// solving workgroup (role 0) and NH helper workgroups. For block blk a helper
// wave forms the PREFIX P[i] = sum_{j < i0 - FW3_NEAR} L[i][j] y[j] of each
// row's ascending sum, reading y as the solver publishes it (gfront, per
// block). The solver's wave starts the row's sum from P and adds the last
// FW3_NEAR columns and the triangle itself. Same terms, same order: the
// result is bit-identical. The L band (8 B per nonzero) is then read by
// NH + 1 CUs instead of one. Hand-offs: write-through (sc1) stores, drained,
// then a relaxed agent-scope flag; sc1 loads on the reading side
// (MI355X_MICROARCH.md "Valid forms", row 1).
constexpr int FW3_NEAR = 192;  // columns left of the block that the solving wave adds itself
constexpr int FW3_HELPERS = 16;  // helper workgroups per RHS column

template <typename T, int NW, int FW2_PF, int NH = 0>
__global__ __launch_bounds__(64 * NW) void band_forward2(int64_t n, int64_t b, int64_t ld, const T* __restrict__ CB,
                                                         const T* __restrict__ B, T* __restrict__ Y,
                                                         unsigned long long* __restrict__ trace,
                                                         T* __restrict__ P = nullptr, int* __restrict__ pflag = nullptr,
                                                         int* __restrict__ gfront = nullptr,
                                                         int* __restrict__ status = nullptr) {
    using A = Arith<T>;
    __shared__ T yr[FW2_RING];
    __shared__ T tri[2][64][64];  // tri[buf][t][l] = L[i0 + l][i0 + t]
    __shared__ int frontier;      // y[0 .. frontier) are final in yr
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t colx = blockIdx.x / (1 + NH);
    const int role = (int)(blockIdx.x % (1 + NH));
    const T* bc = B + colx * n;
    T* yc = Y + colx * n;
    const int64_t nblk = (n + 63) / 64;
    const int64_t pad_off = n * ld;  // band_pad zeros follow the band
    if constexpr (NH > 0) {
        P += colx * nblk * 64;
        pflag += colx * nblk;
        gfront += colx;
        if (role > 0) {  // ---- helper: prefixes of the rows' sums, block by block
            const uint32_t stride = (uint32_t)(ld - 1);  // L[i][jj] = CB[i + jj * (ld - 1)]
            int64_t gf = 0;
            for (int64_t blk = (int64_t)(role - 1) * NW + w; blk < nblk; blk += (int64_t)NH * NW) {
                const int64_t i0 = blk * 64, i = i0 + lane;
                const bool live = i < n;
                const int64_t j0 = i0 - b > 0 ? i0 - b : 0, jn = i0 - FW3_NEAR;
                if (jn <= j0) continue;  // the solving wave forms the whole sum
                constexpr int HB = 32;  // terms per batch: one round trip for its L and y loads
                const long long h0 = trace ? clock64() : 0;
                long long hw = 0;
                T s = A::zero();
                for (int64_t j = j0; j < jn; j += HB) {
                    const int64_t je = j + HB < jn ? j + HB : jn;
                    long long spins = 0;
                    const long long hw0 = trace && gf < je ? clock64() : 0;
                    if (trace && gf < je) hw -= hw0;
                    while (gf < je) {  // y[0 .. je) published (polled only when the cached value is short)
                        gf = __hip_atomic_load(gfront, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (gf >= je) break;
                        __builtin_amdgcn_s_sleep(2);
                        if (++spins > SPIN_LIMIT) {
                            if (lane == 0) atomicOr(status, ST_TIMEOUT);
                            gf = INT64_MAX;
                        }
                    }
                    if (trace && hw0) hw += clock64();
                    T lv[HB], yv[HB];
#pragma unroll
                    for (int q = 0; q < HB; ++q) {  // out of band / past je: a zero of the padding
                        const int64_t jj = j + q;
                        const bool ok = live & (jj < je) & (i - jj <= b);
                        lv[q] = CB[(ok ? i : pad_off) + (int64_t)((uint64_t)(ok ? (uint32_t)jj : 0u) * stride)];
                        yv[q] = ld_sc1(&yc[jj < je ? jj : je - 1]);
                    }
#pragma unroll
                    for (int q = 0; q < HB; ++q) s = A::add(s, j + q < je ? A::mul(lv[q], yv[q]) : A::zero());
                }
                if (live) st_sc1(&P[i], s);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(&pflag[blk], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (trace && lane == 0) {
                    atomicAdd(&trace[5], (unsigned long long)(clock64() - h0));
                    atomicAdd(&trace[6], (unsigned long long)hw);
                    atomicAdd(&trace[7], 1ull);
                }
            }
            return;
        }
    }
    if (threadIdx.x == 0) frontier = 0;
    __syncthreads();
    // LDS atomics on the __shared__ counter itself (a volatile generic
    // pointer compiles to flat_* accesses, and a flat store is waited on
    // with vmcnt(0) together with the global y store)
    auto fr_load = [&]() -> int64_t { return __hip_atomic_load(&frontier, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    // diagnostic (BSM_FW_TRACE): cycles per block in the far phase, waiting
    // for the previous block, and solving the block -- summed over blocks
    long long t_far = 0, t_wait = 0, t_step = 0, t_spin = 0, t_pwait = 0;
    for (int64_t blk = w; blk < nblk; blk += NW) {
        const long long c0 = trace ? clock64() : 0;
        const int64_t i0 = blk * 64, i = i0 + lane;
        const bool live = i < n;
        const int buf = (int)(blk & 1);
        const T bi = live ? bc[i] : A::zero();
        const T lii = live ? CB[i * ld] : (T)1;
        // the block's triangle: column t of rows i0 + l, l > t (coalesced per
        // t). Staged once block blk - 2 is solved: tri[buf] was block blk - 2's
        // and block blk - 1 (being solved meanwhile) uses the other buffer.
        bool staged = false;
        auto stage_tri = [&]() {  // 16 loads in flight at a time (a load-store loop waits per row)
#pragma unroll 1
            for (int h = 0; h < 64; h += 16) {
                T v[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int t = h + q;
                    const bool ok = live && lane > t && lane - t <= b;
                    v[q] = CB[ok ? (i0 + t) * ld + (lane - t) : 0];
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int t = h + q;
                    tri[buf][t][lane] = (live && lane > t && lane - t <= b) ? v[q] : A::zero();
                }
            }
            staged = true;
        };
        // wait until y[0 .. need) are final, staging the triangle on the way
        // (once block blk - 2 is solved); the only call site of stage_tri
        auto wait_frontier = [&](int64_t need) {
            for (;;) {
                const int64_t f = fr_load();
                if (!staged && f >= i0 - 64) stage_tri();
                if (f >= need && staged) break;
                if (f >= need && i0 - 64 > f) break;
                __builtin_amdgcn_s_sleep(1);
            }
        };
        // far terms j in [i0 - b, i0), ascending, as the frontier allows;
        // out-of-band terms (j < i - b) are +0 products
        T s = A::zero();
        int64_t j = i0 - b > 0 ? i0 - b : 0;
        bool from_helper = false;  // the prefix [j, i0 - FW3_NEAR) comes from a helper
        if constexpr (NH > 0) {
            if (i0 - FW3_NEAR > j) {
                from_helper = true;
                j = i0 - FW3_NEAR;
            }
        }
        // L[i][jj], or a zero of the band's padding outside the band / past
        // the matrix: the ADDRESS is selected, the load is unconditional (a
        // load under a branch costs a vmcnt(0) per term)
        const uint32_t stride = (uint32_t)(ld - 1);  // L[i][jj] = CB[i + jj * (ld - 1)]
        auto lfar = [&](int64_t jj) -> T {
            const bool ok = live & (jj < i0) & (i - jj <= b);  // bitwise: no short-circuit branches
            // select the operands, not the address: a selected address is
            // lowered to an exec-masked branch around the address math
            const uint32_t je = ok ? (uint32_t)jj : 0u;
            const int64_t ie = ok ? i : pad_off;
            return CB[ie + (int64_t)((uint64_t)je * stride)];
        };
        // batches of FW2_PF terms once the frontier covers them (terms at or
        // past i0 predicated off); two register banks, so the loads of the
        // batch after next are in flight while a batch is added
        T pa[FW2_PF], pb[FW2_PF];
#pragma unroll
        for (int q = 0; q < FW2_PF; ++q) {
            pa[q] = lfar(j + q);
            pb[q] = lfar(j + FW2_PF + q);
        }
        if constexpr (NH > 0) {
            if (from_helper) {  // after the first loads of the near terms are in flight
                const long long cp = trace ? clock64() : 0;
                long long spins = 0;
                while (__hip_atomic_load(&pflag[blk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > SPIN_LIMIT) {
                        if (lane == 0) atomicOr(status, ST_TIMEOUT);
                        break;
                    }
                }
                s = live ? ld_sc1(&P[i]) : A::zero();
                if (trace) t_pwait += clock64() - cp;
            }
        }
        auto batch = [&](T (&pf)[FW2_PF]) {
            const int64_t need = j + FW2_PF < i0 ? j + FW2_PF : i0;
            const long long cs = trace ? clock64() : 0;
            wait_frontier(need);
            if (trace) t_spin += clock64() - cs;
            T pr[FW2_PF];  // the batch's products (y read from LDS all at once)
#pragma unroll
            for (int q = 0; q < FW2_PF; ++q) pr[q] = A::mul(pf[q], yr[(j + q) & (FW2_RING - 1)]);
#pragma unroll
            for (int q = 0; q < FW2_PF; ++q) pf[q] = lfar(j + 2 * FW2_PF + q);
            // terms at or past i0: a +0 product (select, no branch), which
            // leaves the sum unchanged (it starts at +0, never becomes -0)
#pragma unroll
            for (int q = 0; q < FW2_PF; ++q) s = A::add(s, j + q < i0 ? pr[q] : A::zero());
            j += FW2_PF;
        };
        while (j < i0) {
            batch(pa);
            if (j >= i0) break;
            batch(pb);
        }
        const long long c1 = trace ? clock64() : 0;
        wait_frontier(i0);  // block blk - 1 solved (and the triangle staged)
        const long long c2 = trace ? clock64() : 0;
        // the block: one row per step. The solving wave runs at raised priority
        // (the other waves stream far terms on the same SIMDs)
        const int nb = (int)(n - i0 < 64 ? n - i0 : 64);
        const T rl = div_rn((T)1, lii);  // for div_by: off the chain
        __builtin_amdgcn_s_setprio(3);
        auto row = [&](int t) __attribute__((always_inline)) {
            const T lt = tri[buf][t][lane];  // read before the division: off the chain
            const T yv = div_by(A::sub(bi, s), lii, rl);
            const T y = readlane_t(yv, t);
            if (lane == t) {
                yr[(i0 + t) & (FW2_RING - 1)] = y;
                if constexpr (NH > 0) st_sc1(&yc[i0 + t], y);  // read by the helpers on other CUs
                else yc[i0 + t] = y;
                // y is in LDS before the frontier moves: LDS ops of one wave are performed
                // in order, so a relaxed store suffices (a release would wait for the y stores)
                __hip_atomic_store(&frontier, (int)(i0 + t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (lane > t) s = A::add(s, A::mul(lt, y));
        };
        if (nb == 64) {
#pragma unroll 8
            for (int t = 0; t < 64; ++t) row(t);
        } else {
            for (int t = 0; t < nb; ++t) row(t);
        }
        __builtin_amdgcn_s_setprio(0);
        if constexpr (NH > 0) {
            // publish the block's y to the helpers: this wave's stores drained, and only
            // after the previous block's wave has published (its stores are not ours to drain)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            long long spins = 0;
            while (__hip_atomic_load(gfront, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < i0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > SPIN_LIMIT) {
                    if (lane == 0) atomicOr(status, ST_TIMEOUT);
                    break;
                }
            }
            if (lane == 0) __hip_atomic_store(gfront, (int)(i0 + nb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (trace) {
            const long long c3 = clock64();
            t_far += c1 - c0;
            t_wait += c2 - c1;
            t_step += c3 - c2;
        }
    }
    if (trace && lane == 0) {
        atomicAdd(&trace[0], (unsigned long long)t_far);
        atomicAdd(&trace[1], (unsigned long long)t_wait);
        atomicAdd(&trace[2], (unsigned long long)t_step);
        atomicAdd(&trace[3], (unsigned long long)t_spin);
        atomicAdd(&trace[4], (unsigned long long)t_pwait);
    }
}

// ---------------------------------------------------------------------------
// backward substitution on the band (lib.rs:49-65) with L* = L^T: x_i =
// (y_i - sum_{j>i} L_ji x_j) / L_ii, sum in ascending j. Ascending order makes
// each row's sum START with the newest x, so the solve is one serial chain of
// N*b dependent adds: band_backward_reg, one wave per RHS column, lane l
// holding the products of terms SEG*l+1 .. SEG*l+SEG of the row. On gfx950
// one wave issues about one instruction per 4 cycles and a dependent
// v_add_f64 every ~4.5 (scripts/micro/issue_cost.hip), so a row costs ~4.5
// cycles per chain add plus ~4 per other instruction; a runtime loop over
// lanes also paid a taken branch per hop (153 cycles per 16-add hop against
// 85 unrolled, hop_latency.hip). So:
//  * the NL hops are unrolled (straight-line code per row pair). The running
//    sum moves from lane l to lane l+1 by DPP wave_shr:1 (every lane adds its
//    own products; lane l+1 then takes lane l's sum);
//  * lane l keeps x[i+m] for its segment m = SEG*l+1 .. SEG*l+SEG in a
//    register window; moving to row i-1 shifts every window by one: lane l
//    takes lane l-1's last value through DPP and lane 0 takes the new x_i
//    (no LDS ring, no barrier);
//  * terms b < m <= W = SEG*NL read the zero padding of a band stored with
//    ld >= W + 1 (band_walk_terms), so rows with all b terms need no masking;
//    the first b rows (dmax < b) take the masked path. Every padding term is
//    +-0 and the sum starts at +0, so it never changes the sum (bit-exact);
//  * y_i and L_ii are uniform loads issued two rows ahead, like the band
//    column, and x_i is stored by every lane to the same address (no
//    exec-masked branch).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double shr1_t(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, false);  // wave_shr:1
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float shr1_t(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, false));
}

template <typename T, int SEG, int NL, int... L>
__device__ __forceinline__ T lane_walk(const T (&p)[SEG], std::integer_sequence<int, L...>) {
    using A = Arith<T>;
    T sv = A::zero();
    auto hop = [&](auto lc) __attribute__((always_inline)) {
        constexpr int l = decltype(lc)::value;
#pragma unroll
        for (int u = 0; u < SEG; ++u) sv = A::add(sv, p[u]);
        if constexpr (l + 1 < NL) sv = shr1_t(sv);
    };
    (hop(std::integral_constant<int, L>{}), ...);
    return readlane_t(sv, NL - 1);
}

// (SEG, NL) of band_backward_reg for bandwidth b: NL lanes of SEG terms,
// W = SEG * NL >= b terms walked per row. Fewer, longer segments save lane
// hops (3 instructions each) but cost registers; (40, 25) walks exactly the
// C5 band (b = 1000): 2,428 ms at C5 against 2,488 for (20, 50) and 2,669
// for (25, 40), same box (profiles/r04_b_*). The band is stored with
// ld = max(b, W) + 1.
struct BwCfg {
    int seg, nl;
};
inline BwCfg band_walk_cfg(int64_t b) {
    if (b <= 64) return {1, 64};
    if (b <= 128) return {2, 64};
    if (b <= 256) return {4, 64};
    if (b <= 512) return {8, 64};
    if (b <= 768) return {12, 64};
    if (b <= 896) return {16, 56};
    if (b <= 1000) return {40, 25};
    if (b <= 1024) return {16, 64};
    if (b <= 2048) return {32, 64};
    return {0, 0};
}
inline int64_t band_walk_terms(int64_t b) {
    const BwCfg c = band_walk_cfg(b);
    return (int64_t)c.seg * c.nl;
}

template <typename T, int SEG, int NL>
__global__ __launch_bounds__(64) void band_backward_reg(int64_t n, int64_t b, int64_t ld, const T* __restrict__ CB,
                                                        const T* __restrict__ Yin, T* __restrict__ X) {
    using A = Arith<T>;
    const int lane = threadIdx.x;
    const T* yc = Yin + (int64_t)blockIdx.x * n;
    T* xc = X + (int64_t)blockIdx.x * n;
    const int m0 = SEG * lane + 1;  // first term of this lane's segment
    T lvA[SEG], lvB[SEG], xw[SEG];
    T yA, dA, yB, dB;
#pragma unroll
    for (int u = 0; u < SEG; ++u) xw[u] = A::zero();  // x[i+m] = 0 past row n-1
    // L[i+m][i] = CB[i*ld + m]; CB is padded by band_pad zeros, so row
    // n-1's reads stay in bounds; rows < 0 (prefetch past the end) read row 0
    auto load_row = [&](T (&lv)[SEG], T& y, T& d, int64_t r) __attribute__((always_inline)) {
        const int64_t rr = r < 0 ? 0 : r;
        const T* src = CB + rr * ld;
#pragma unroll
        for (int u = 0; u < SEG; ++u) lv[u] = src[m0 + u];
        d = src[0];
        y = yc[rr];
    };
    // row i; lv becomes the products. MASK: rows with dmax < b.
    auto do_row = [&](auto mask, T (&lv)[SEG], T y, T d, int64_t i) __attribute__((always_inline)) {
        if constexpr (decltype(mask)::value) {
            const int64_t dmax = (n - 1 - i < b) ? n - 1 - i : b;
#pragma unroll
            for (int u = 0; u < SEG; ++u) {
                const T pr = A::mul(lv[u], xw[u]);
                lv[u] = m0 + u <= dmax ? pr : A::zero();
            }
        } else {
#pragma unroll
            for (int u = 0; u < SEG; ++u) lv[u] = A::mul(lv[u], xw[u]);
        }
        const T sv = lane_walk<T, SEG, NL>(lv, std::make_integer_sequence<int, NL>{});
        const T x = div_rn(A::sub(y, sv), d);
        xc[i] = x;  // every lane, same address and value
        const T t = shr1_t(xw[SEG - 1]);
#pragma unroll
        for (int u = SEG - 1; u > 0; --u) xw[u] = xw[u - 1];
        xw[0] = lane == 0 ? x : t;
    };
    constexpr std::true_type masked{};
    constexpr std::false_type full{};
    int64_t i = n - 1;
    const int64_t i_full = n - 1 - b;  // rows <= i_full have all b terms
    load_row(lvA, yA, dA, i);
    load_row(lvB, yB, dB, i - 1);
    for (; i >= 1 && i > i_full; i -= 2) {
        do_row(masked, lvA, yA, dA, i);
        load_row(lvA, yA, dA, i - 2);
        do_row(masked, lvB, yB, dB, i - 1);
        load_row(lvB, yB, dB, i - 3);
    }
    for (; i >= 1; i -= 2) {
        do_row(full, lvA, yA, dA, i);
        load_row(lvA, yA, dA, i - 2);
        do_row(full, lvB, yB, dB, i - 1);
        load_row(lvB, yB, dB, i - 3);
    }
    if (i == 0) do_row(masked, lvA, yA, dA, 0);
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
// contribute +-0: skipped, unless one is inf/NaN (v * 0 = NaN: y[i] = NaN).
// Divisor = LAST stored entry of the row.
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
        bool tail_nan = false;  // an inf/NaN entry past the diagonal: its v * 0 is NaN
        if (i < n) {
            e = rp[i];
            e1 = rp[i + 1];
            if (e == e1) atomicOr(status, ST_EMPTY_ROW);
            for (int64_t q = e1 - 1; q >= e && col[q] > i; --q) tail_nan |= !isfinite(val[q]);
            for (; e < e1 && col[e] < i0; ++e) s = A::add(s, A::mul(val[e], ld_sc1(&yc[col[e]])));
        }
        const int64_t nb = (n - i0 < FW_BLOCK) ? n - i0 : FW_BLOCK;
        for (int64_t tt = 0; tt < nb; ++tt) {
            const int64_t j = i0 + tt;
            if (t == tt && e1 > rp[i]) {
                const T y = div_rn(A::sub(bc[i], tail_nan ? T(NAN) : s), val[e1 - 1]);
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

// The tri-solves index the n-row y / x with the column of every entry of
// rows [0, n) they read: forward all of them (col != row, lib.rs:37-38),
// backward all but the first (row.iter().skip(1), lib.rs:57-58). A column
// >= n there is an index-out-of-bounds panic in the reference. One thread
// per row (only launched when the matrix is wider than the RHS).
__global__ __launch_bounds__(256) void csr_cols_past_rhs(int64_t n, const int64_t* __restrict__ rp,
                                                         const int32_t* __restrict__ col, bool skip_first,
                                                         int* __restrict__ status) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t a = rp[i] + (skip_first ? 1 : 0), e1 = rp[i + 1];
    for (int64_t e = a; e < e1; ++e)
        if (col[e] >= n) {
            atomicOr(status, ST_COL_OOB);
            return;
        }
}

// ---------------------------------------------------------------------------
// Blocked band solves (bsm_solve_blocked): the same L L^T x = b as solve
// (lib.rs:11-24), with the sums REASSOCIATED. Not bit-exact with the
// reference; within its f64 tolerance (relative error of a backward-stable
// solve, tests/test_gpu_solver_blocked.py). The rows are cut into 64-row
// blocks I. Forward (L y = b):
//     y_I = Linv_I (b_I - sum_{J <= I-2} L_{I,J} y_J) - MF_I y_{I-1},
//     Linv_I = L_{I,I}^-1,  MF_I = Linv_I L_{I,I-1};
// backward (L^T x = y):
//     x_I = Linv_I^T (y_I - sum_{J >= I+2} L_{J,I}^T x_J) - MB_I^T x_{I+1},
//     MB_I = L_{I+1,I} Linv_I.
// Linv, MF, MB depend on L only (blk_prep, fully parallel). In the solve the
// far sums run ahead on many workgroups; the serial chain per block is one
// 64 x 64 matrix-vector product (MF_I or MB_I) in one wave, against the N*b
// dependent adds of the reference order (band_backward_reg).
// ---------------------------------------------------------------------------

// M[q * 64 + l] layouts (one 64 x 64 matrix per block, 4096 elements):
//   G[I]  = Linv_I[l][q]   (forward:  u[l] = sum_q Linv[l][q] r[q])
//   H[I]  = Linv_I[q][l]   (backward: u[l] = sum_q Linv[q][l] r[q])
//   MF[I] = MF_I[l][q],  MB[I] = MB_I[q][l]
template <typename T>
__global__ __launch_bounds__(256) void blk_prep(int64_t n, int64_t b, int64_t ld, const T* __restrict__ CB,
                                                T* __restrict__ G, T* __restrict__ H, T* __restrict__ MF,
                                                T* __restrict__ MB) {
    __shared__ T Ls[64][65];  // Ls[r][c] = L[i0 + r][i0 + c] (r >= c); identity rows past n
    __shared__ T Xs[64][65];  // Linv
    __shared__ T As[64][65];  // the neighbouring block, then the product
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t I = blockIdx.x, i0 = I * 64, nb64 = (n + 63) / 64;
    const int64_t o = I * 4096;
    for (int e = tid; e < 4096; e += 256) {  // r fastest: a column's rows are contiguous in CB
        const int r = e & 63, c = e >> 6;
        const int64_t i = i0 + r;
        T v = (T)0;
        if (r == c) v = i < n ? CB[i * ld] : (T)1;
        else if (r > c && i < n && r - c <= b) v = CB[(i0 + c) * ld + (r - c)];
        Ls[r][c] = v;
    }
    __syncthreads();
    if (w == 0) {  // lane l forms column l of the inverse: L x = e_l, rows ascending
        T x[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            T acc = (T)0;
#pragma unroll
            for (int t = 0; t < r; ++t) acc = fma_t(Ls[r][t], x[t], acc);
            x[r] = ((r == lane ? (T)1 : (T)0) - acc) / Ls[r][r];
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int r = 0; r < 64; ++r) Xs[r][lane] = x[r];
    }
    __syncthreads();
    for (int e = tid; e < 4096; e += 256) {
        const int q = e >> 6, l = e & 63;
        G[o + e] = Xs[l][q];
        H[o + e] = Xs[q][l];
    }
    if (I > 0) {  // MF = Linv L_{I,I-1}: As[t][c] = L[i0 + t][i0 - 64 + c]
        for (int e = tid; e < 4096; e += 256) {
            const int t = e & 63, c = e >> 6;
            const int64_t i = i0 + t;
            As[t][c] = (i < n && t + 64 - c <= b) ? CB[(i0 - 64 + c) * ld + (t + 64 - c)] : (T)0;
        }
        __syncthreads();
        T acc[16];
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) acc[rr] = (T)0;
        for (int t = 0; t < 64; ++t) {
            const T a = As[t][lane];
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) acc[rr] = fma_t(Xs[16 * w + rr][t], a, acc[rr]);
        }
        __syncthreads();
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) As[16 * w + rr][lane] = acc[rr];  // MF[r][c]
        __syncthreads();
        for (int e = tid; e < 4096; e += 256) MF[o + e] = As[e & 63][e >> 6];
        __syncthreads();
    }
    if (I + 1 < nb64) {  // MB = L_{I+1,I} Linv: As[a][t] = L[i0 + 64 + a][i0 + t]
        for (int e = tid; e < 4096; e += 256) {
            const int a = e & 63, t = e >> 6;
            const int64_t i = i0 + 64 + a;
            As[a][t] = (i < n && a + 64 - t <= b) ? CB[(i0 + t) * ld + (a + 64 - t)] : (T)0;
        }
        __syncthreads();
        T acc[16];
#pragma unroll
        for (int aa = 0; aa < 16; ++aa) acc[aa] = (T)0;
        for (int t = 0; t < 64; ++t) {
            const T xv = Xs[t][lane];
#pragma unroll
            for (int aa = 0; aa < 16; ++aa) acc[aa] = fma_t(As[16 * w + aa][t], xv, acc[aa]);
        }
#pragma unroll
        for (int aa = 0; aa < 16; ++aa) MB[o + (16 * w + aa) * 64 + lane] = acc[aa];
    }
}

// One 64-row block per ticket; tickets are taken in dependency order (per RHS
// column, FWD: blocks ascending, else descending), so a workgroup only waits
// on blocks already held by running workgroups. Y: padded solution columns
// (nb64 * 64 each), flags[col * nb64 + I] = 1 once block I of Y is final
// (write-through stores, drained, then a relaxed agent-scope flag; sc1 loads
// on the reading side: MI355X_MICROARCH.md "Valid forms", row 1).
// One band (segment) of a blk_trsv launch: its factor (rows [0, n) of the
// band at CB), blk_prep's Linv and coupling blocks, the right-hand sides
// (column j at rhs + j * rhs_stride) and the padded solution (column j at
// Y + j * nb64 * 64) with its per-block flags (column j at flags + j * nb64).
template <typename T>
struct TrsvSeg {
    const T* CB;
    int64_t n;
    const T* Minv;
    const T* Madj;
    const T* rhs;
    int64_t rhs_stride;
    T* Y;
    int* flags;
};

template <typename T, bool FWD>
__global__ __launch_bounds__(256) void blk_trsv(int64_t b, int64_t ld, const TrsvSeg<T>* __restrict__ segs, int nseg,
                                                int64_t nb64max, int* __restrict__ ticket, int* __restrict__ status,
                                                int64_t k) {
    __shared__ T red[4][64];
    __shared__ T rv[64];
    __shared__ int64_t tk;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto wait_flag = [&](const int* f) {
        long long spins = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > SPIN_LIMIT) {
                if (lane == 0) atomicOr(status, ST_TIMEOUT);
                return;
            }
        }
    };
    for (;;) {
        if (threadIdx.x == 0) tk = atomicAdd(ticket, 1);
        __syncthreads();
        const int64_t t = tk;
        if (t >= nb64max * k * nseg) break;
        // tickets: step s of every (segment, column) in turn
        const int64_t step = t / (k * nseg), col = t % k;
        const TrsvSeg<T> sg = segs[(t / k) % nseg];
        const int64_t n = sg.n, nb64 = (n + 63) / 64, NP = nb64 * 64;
        if (step >= nb64) {
            __syncthreads();
            continue;
        }
        const T* const CB = sg.CB;
        const T* const Minv = sg.Minv;
        const T* const Madj = sg.Madj;
        const T* const rhs = sg.rhs;
        const int64_t rhs_stride = sg.rhs_stride;
        const int64_t I = FWD ? step : nb64 - 1 - step, i0 = I * 64, i = i0 + lane;
        T* Yc = sg.Y + col * NP;
        int* fl = sg.flags + col * nb64;
        const bool has_adj = FWD ? I > 0 : I + 1 < nb64;
        // x-independent operands first: this wave's slice of Linv, wave 0's coupling matrix
        T minv[16], madj[64];
#pragma unroll
        for (int q = 0; q < 16; ++q) minv[q] = Minv[I * 4096 + (16 * w + q) * 64 + lane];
        if (w == 0 && has_adj) {
#pragma unroll
            for (int q = 0; q < 64; ++q) madj[q] = Madj[I * 4096 + q * 64 + lane];
        }
        // far blocks: FWD columns [max(0, i0 - b), i0 - 64), else [i0 + 128, i0 + 63 + b];
        // wave w takes columns 16w .. 16w + 15 of each, lane = row
        T acc = (T)0;
        int64_t J0, J1;  // in the order their solutions complete
        if (FWD) {
            J0 = (i0 - b > 0 ? i0 - b : 0) / 64;
            J1 = I - 2;
        } else {
            const int64_t jl = i0 + 63 + b < n - 1 ? i0 + 63 + b : n - 1;
            J0 = jl / 64;
            J1 = I + 2;
        }
        for (int64_t J = J0; FWD ? J <= J1 : J >= J1; J += FWD ? 1 : -1) {
            T lv[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t j = J * 64 + 16 * w + q;
                // L[i][j] (FWD) or L[j][i] in the band and the segment, else zero (the
                // load reads element 0, the select drops it: past a segment's end
                // the band holds the next rows' values, not padding)
                const bool ok = FWD ? (i < n) & (i - j <= b) : (j < n) & (j - i <= b);
                const int64_t idx = FWD ? j * ld + (i - j) : i * ld + (j - i);
                const T lw = CB[idx & -(int64_t)ok];
                lv[q] = ok ? lw : (T)0;
            }
            wait_flag(&fl[J]);
            const T v = ld_sc1(&Yc[J * 64 + lane]);
#pragma unroll
            for (int q = 0; q < 16; ++q) acc = fma_t(lv[q], readlane_t(v, 16 * w + q), acc);
        }
        red[w][lane] = acc;
        __syncthreads();
        if (w == 0) {
            const T bi = i < n ? rhs[col * rhs_stride + i] : (T)0;
            rv[lane] = bi - ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]));
        }
        __syncthreads();
        T uu = (T)0;
#pragma unroll
        for (int q = 0; q < 16; ++q) uu = fma_t(minv[q], rv[16 * w + q], uu);
        red[w][lane] = uu;
        __syncthreads();
        if (w == 0) {
            T u = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
            if (has_adj) {  // the serial step: the neighbour's solution through the coupling matrix
                const int64_t Ja = FWD ? I - 1 : I + 1;
                wait_flag(&fl[Ja]);
                const T v = ld_sc1(&Yc[Ja * 64 + lane]);
                T s0 = (T)0, s1 = (T)0, s2 = (T)0, s3 = (T)0;
                // the neighbour's 64 values to every lane through LDS (one
                // write, broadcast reads) rather than 64 v_readlane pairs
                rv[lane] = v;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int q = 0; q < 64; q += 4) {
                    s0 = fma_t(madj[q], rv[q], s0);
                    s1 = fma_t(madj[q + 1], rv[q + 1], s1);
                    s2 = fma_t(madj[q + 2], rv[q + 2], s2);
                    s3 = fma_t(madj[q + 3], rv[q + 3], s3);
                }
                u = u - ((s0 + s1) + (s2 + s3));
            }
            st_sc1(&Yc[i], u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(&fl[I], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Blocked band Cholesky (solve order="blocked"): left-looking over 64 x 64
// tiles of the band, sums reassociated (FMA, any order). Tile (I, K), I >= K:
//     S = A_{I,K} - sum_{J < K} L_{I,J} L_{K,J}^T
//     I == K: L_{K,K} = chol(S), Dinv[K] = L_{K,K}^-1 (G layout of blk_prep)
//     I >  K: L_{I,K} = S L_{K,K}^-T
// One 256-thread workgroup per tile, tickets in (K, I - K) order, one flag per
// tile (write-through stores, drained, then the flag). Out-of-band entries of
// L are exact zeros (every product there has an out-of-band factor), so tiles
// read zeros outside the band and write only inside it.
// ---------------------------------------------------------------------------

// One band (segment) of a blk_chol launch: rows [0, n) of the band at CB
// (CB[k * ld + d] = A[k + d][k]), its Dinv blocks and flags. Several segments
// (the interiors of solve(order="partitioned"), §4.9) are factored by one
// launch, their tickets interleaved block column by block column.
template <typename T>
struct CholSeg {
    T* CB;
    int64_t n;
    T* Dinv;     // nb64 * 4096
    int* flags;  // nb64 * DM
    int* rbf;    // 4 * nb64
};

template <typename T>
__global__ __launch_bounds__(256) void blk_chol(int64_t b, int64_t ld, const CholSeg<T>* __restrict__ segs, int nseg,
                                                int64_t nb64max, int* __restrict__ ticket, int* __restrict__ status,
                                                unsigned long long* __restrict__ dbg, unsigned long long* __restrict__ tdbg) {
    __shared__ T PT[64][TLD];  // PT[t][r] = L_{I,J}[r][t], later S^T / the tile
    __shared__ T QT[64][TLD];  // QT[t][c] = L_{K,J}[c][t], later Linv^T
    __shared__ T AT[64][TLD];  // L_{K,K-1}^T as its column blocks form
    __shared__ T rd[64];
    __shared__ T Di[4 * 256];  // blk_diag_panels: the 16 x 16 diagonal blocks' inverses
    __shared__ T Tb[3 * 256];  //                  and its block products
    __shared__ int64_t tk;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t DM = (63 + b) / 64 + 1;  // tiles per block column (incl. diagonal)
    // the current ticket's segment
    int64_t n = 0, nb64 = 0;
    T* CB = nullptr;
    T* Dinv = nullptr;
    int* flags = nullptr;
    int* rbf = nullptr;
    auto wait_flag = [&](const int* f) {
        long long spins = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            __builtin_amdgcn_s_sleep(1);
            if (dbg && spins == 100000 && tid == 0) {  // BSM_BLK_DEBUG: which flag a stuck tile waits on
                __hip_atomic_store(&dbg[1], (unsigned long long)(f - flags), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_fetch_add(&dbg[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (++spins > SPIN_LIMIT) {
                if (lane == 0) atomicOr(status, ST_TIMEOUT);
                return;
            }
        }
    };
    // element (r, c) of tile (I, K) in the band: offset (c-th column, band row 64(I-K) + r - c)
    auto in_band = [&](int64_t I, int64_t K, int r, int c) -> bool {
        const int64_t off = 64 * (I - K) + r - c;
        return (off >= 0) & (off <= b) & (64 * I + r < n);
    };
    auto band_idx = [&](int64_t I, int64_t K, int r, int c) -> int64_t {
        return (64 * K + c) * ld + 64 * (I - K) + r - c;
    };
    // stage the transpose of tile (I, J) of L: X[t][r] = L[64I + r][64J + t] (sc1: other workgroups wrote it).
    // All 16 loads of a thread are in flight before the first LDS write (a loop
    // of load, wait, write is 16 memory round trips); out-of-band elements load
    // element 0 and are replaced by zero (a selected address is not a branch).
    auto stage = [&](T (*X)[TLD], int64_t I, int64_t J) {
        T v[16];
        unsigned okm = 0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = tid + 256 * u, r = e & 63, t = e >> 6;
            const bool ok = in_band(I, J, r, t);
            okm |= (unsigned)ok << u;
            v[u] = ld_sc1(&CB[band_idx(I, J, r, t) & -(int64_t)ok]);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = tid + 256 * u;
            X[e >> 6][e & 63] = (okm >> u) & 1 ? v[u] : (T)0;
        }
    };
    // X[q][l] = Dinv[Kd][q * 64 + l], the same way
    auto stage_dinv = [&](T (*X)[TLD], int64_t Kd) {
        T v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = ld_sc1(&Dinv[Kd * 4096 + tid + 256 * u]);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = tid + 256 * u;
            X[e >> 6][e & 63] = v[u];
        }
    };
    // this thread's 16 elements of a 64 x 64 tile, in the f64 MFMA accumulator
    // layout: X[cb][q] = element (row rb + 4q, column 16cb + cm)
    const int rb = 16 * w + (lane >> 4), cm = lane & 15;
    lds_t<T>* const PTl = (lds_t<T>*)&PT[0][0];
    lds_t<T>* const QTl = (lds_t<T>*)&QT[0][0];
    for (;;) {
        if (tid == 0) tk = atomicAdd(ticket, 1);
        __syncthreads();
        const int64_t t0 = tk;
        if (dbg && tid == 0) __hip_atomic_fetch_max(&dbg[0], (unsigned long long)t0, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_SYSTEM);
        const int64_t t = t0;
        if (t >= nb64max * DM * nseg) break;
        // tickets: block column K of every segment in turn, tiles d within it
        const int64_t K = t / (DM * nseg), d = t % DM, I = K + d;
        {
            const int sg = (int)((t / DM) % nseg);
            n = segs[sg].n;
            CB = segs[sg].CB;
            Dinv = segs[sg].Dinv;
            flags = segs[sg].flags;
            rbf = segs[sg].rbf;
            nb64 = (n + 63) / 64;
        }
        if (K >= nb64) {
            __syncthreads();
            continue;
        }
        int* fl = flags + K * DM;
        // no such tile (past the matrix or the band), or the sub-diagonal tile
        // (K + 1, K), which diagonal tile K + 1's workgroup forms
        // (one hand-off on the chain per block column instead of two)
        if (I >= nb64 || 64 * d - 63 > b || d == 1) {
            __syncthreads();
            continue;
        }
        const bool sub = d == 0 && K > 0 && DM > 1;  // this workgroup also forms tile (K, K - 1)
        T acc[4][4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = rb + 4 * q, c = 16 * cb + cm;
                // A itself (band_fill; rows past n: identity on the diagonal)
                T a = in_band(I, K, r, c) ? CB[band_idx(I, K, r, c)] : (T)0;
                if (d == 0 && r == c && 64 * I + r >= n) a = (T)1;
                acc[cb][q] = a;
            }
        T acc2[4][4];  // sub: tile (K, K - 1) = A_{K,K-1} - sum_{J < K-1} L_{K,J} L_{K-1,J}^T
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = rb + 4 * q, c = 16 * cb + cm;
                acc2[cb][q] = sub && in_band(K, K - 1, r, c) ? CB[band_idx(K, K - 1, r, c)] : (T)0;
            }
        // left-looking updates from block columns J in the band of both I and K
        // (with sub, J = K - 1 comes after tile (K, K - 1) is formed, below)
        const int64_t Jlo = I - (DM - 1) > 0 ? I - (DM - 1) : 0;
        for (int64_t J = Jlo; J < (sub ? K - 1 : K); ++J) {
            wait_flag(&flags[J * DM + (I - J)]);
            if (d > 0) wait_flag(&flags[J * DM + (K - J)]);
            if (sub) wait_flag(&flags[J * DM + (K - 1 - J)]);
            stage(PT, I, J);
            if (d > 0) stage(QT, K, J);
            if (sub) stage(QT, K - 1, J);
            __syncthreads();
            mfma_tile<T, true>(PTl, d > 0 ? QTl : PTl, acc, w, lane);
            if (sub) mfma_tile<T, true>(PTl, QTl, acc2, w, lane);
            __syncthreads();
        }
        long long cw0 = 0, cw1 = 0, cs1 = 0, cs2 = 0, cs3 = 0;  // BSM_BLK_DEBUG: the chain's steps
        if (sub) {
            // Progressive: column block c of L_{K,K-1} = S_{K,K-1} (row block c
            // of Linv_{K-1})^T as soon as tile K - 1 has published that row
            // block, then its share of the update S_{K,K} -= L_{K,K-1}[:, c]
            // L_{K,K-1}[:, c]^T. Blocks 0-2 overlap tile K - 1's factor. Per
            // output element the MFMA sequence is mfma_tile's (k ascending from
            // the same start), so the bits are those of the whole-tile form.
            lds_t<T>* const ATl = (lds_t<T>*)&AT[0][0];
            const int kq = lane >> 4, m = lane & 15;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) PT[16 * cb + cm][rb + 4 * q] = acc2[cb][q];
            bsm_d4 ca[4];
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) ca[cb][q] = (double)acc[cb][q];
            const T* dk = Dinv + (K - 1) * 4096;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (tdbg && c == 3) cw0 = clock64();
                wait_flag(c < 3 ? &rbf[(K - 1) * 4 + c] : &flags[(K - 1) * DM]);
                if (tdbg && c == 3) cw1 = clock64();
                T v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {  // QT[s][16c + j] = Linv[16c + j][s], s < 16c + 16
                    const int i = tid + 256 * u, s = i >> 4, j = i & 15;
                    v[u] = s < 16 * c + 16 ? ld_sc1(&dk[s * 64 + 16 * c + j]) : (T)0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = tid + 256 * u, s = i >> 4, j = i & 15;
                    if (s < 16 * c + 16) QT[s][16 * c + j] = v[u];
                }
                __syncthreads();
                if (tdbg && c == 3) cs1 = clock64();
                bsm_d4 oc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int k4 = 0; k4 < 4 * c + 4; ++k4) {
                    const int k = 4 * k4 + kq;
                    oc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)PT[k][16 * w + m], (double)QT[k][16 * c + m],
                                                              oc, 0, 0, 0);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = rb + 4 * q, cc = 16 * c + cm;
                    const T o = (T)oc[q];
                    if (in_band(K, K - 1, r, cc)) st_sc1(&CB[band_idx(K, K - 1, r, cc)], o);
                    AT[cc][r] = o;  // AT[t][r] = L_{K,K-1}[r][t]
                }
                __syncthreads();
                if (tdbg && c == 3) cs2 = clock64();
#pragma unroll
                for (int k4 = 0; k4 < 4; ++k4) {
                    const int k = 16 * c + 4 * k4 + kq;
                    const double a = -(double)ATl[k * TLD + 16 * w + m];
#pragma unroll
                    for (int cb = 0; cb < 4; ++cb)
                        ca[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, (double)ATl[k * TLD + 16 * cb + m], ca[cb],
                                                                      0, 0, 0);
                }
            }
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[cb][q] = (T)ca[cb][q];
            // the tile's flag (read by tiles below, not by this chain) is raised
            // inside the factor, once every wave's stores have drained there
            if (tdbg) cs3 = clock64();
        }
        if (d == 0) {
            const long long c0 = tdbg ? clock64() : 0;
            // S to LDS (PT[r][c]), then wave 0 factors it: lane r holds row r
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) PT[rb + 4 * q][16 * cb + cm] = acc[cb][q];
            __syncthreads();
            // factor and inverse by 16-column panels on all four waves, the
            // products on f64 MFMA; one Newton step per pivot (C5 factor 317 ->
            // 311 ms, x error 8.8e-11 -> 9.7e-11 against two); Linv's row blocks
            // 0-2 published as they form (rbf), its flag and L_{K,K-1}'s after
            // the first barrier
            blk_diag_panels<T>((lds_t<T>*)&PT[0][0], (lds_t<T>*)&QT[0][0], (lds_t<T>*)Di, (lds_t<T>*)Tb,
                               (lds_t<T>*)rd, status, tid, tdbg, Dinv + K * 4096, rbf + K * 4,
                               sub ? &flags[(K - 1) * DM + 1] : nullptr);
            const long long c1 = tdbg ? clock64() : 0;
            __syncthreads();
            if (tdbg && tid == 0) {  // cycles: factor, inverse (BSM_BLK_DEBUG)
                const long long c2 = clock64();
                __hip_atomic_fetch_add(&tdbg[4], (unsigned long long)(c1 - c0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(&tdbg[5], (unsigned long long)(c2 - c1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(&tdbg[7], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (sub) {  // the chain: waiting for tile K - 1, then the sub-diagonal tile and its update
                    __hip_atomic_fetch_add(&tdbg[8], (unsigned long long)(cw1 - cw0), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(&tdbg[9], (unsigned long long)(c0 - cw1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(&tdbg[10], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(&tdbg[14], (unsigned long long)(cs1 - cw1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(&tdbg[15], (unsigned long long)(cs2 - cs1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(&tdbg[16], (unsigned long long)(cs3 - cs2), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            // Dinv[K][q * 64 + l] = Linv[l][q] = QT[q][l] (row blocks 0-2 are
            // out already, row block 3 is left)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = tid + 256 * u, q = i >> 4, j = i & 15;
                st_sc1(&Dinv[K * 4096 + q * 64 + 48 + j], QT[q][48 + j]);
            }
            if (tdbg) {  // the publication: stores drained, then the flag (below)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (tid == 0) {
                    const long long c3 = clock64();
                    __hip_atomic_fetch_add(&tdbg[11], (unsigned long long)(c3 - c0), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    // clock calibration: the constant 100 MHz counter at each diagonal tile's end
                    const unsigned long long wc = wall_clock64();
                    if (K == 0) __hip_atomic_store(&tdbg[12], wc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (K == nb64 - 1) __hip_atomic_store(&tdbg[13], wc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        } else {
            const long long c0 = tdbg ? clock64() : 0;
            wait_flag(&fl[0]);  // L_{K,K} and its inverse
            if (tdbg && tid == 0 && d == 1)
                __hip_atomic_fetch_add(&tdbg[6], (unsigned long long)(clock64() - c0), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            // PT[s][r] = S[r][s]; QT[s][c] = Linv[c][s] = Dinv[K][s * TLD + c]
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) PT[16 * cb + cm][rb + 4 * q] = acc[cb][q];
            stage_dinv(QT, K);
            __syncthreads();
            T o[4][4] = {};
            mfma_tile<T, false, true>(PTl, QTl, o, w, lane);
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = rb + 4 * q, c = 16 * cb + cm;
                    if (in_band(I, K, r, c)) st_sc1(&CB[band_idx(I, K, r, c)], o[cb][q]);
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(&fl[d], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
            // L_{K,K} to the band after the flag: no tile of this kernel reads it
            // (they take Dinv), so its stores drain with the next tile's
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = tid + 256 * u, r = e & 63, c = e >> 6;
                if (r >= c && in_band(I, K, r, c)) st_sc1(&CB[band_idx(I, K, r, c)], PT[r][c]);
            }
        }
        if (dbg && tid == 0) __hip_atomic_fetch_add(&dbg[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------
struct Band {
    DBuf cb;
    DBuf r;  // 1 / L[k][k] per column (+64 scratch entries)
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

template <typename T, int M, int RP>
int launch_chol5(Band& bd, int* fprog, int* status, hipStream_t s, unsigned long long* trace) {
    constexpr int C5_NT = 64 * (16 / RP);
    const int64_t n_tiles = (bd.n + C4_TB - 1) / C4_TB;
    int dev = 0, cus = 0;
    BSM_HIP_TRY(hipGetDevice(&dev));
    BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int per_cu = 0;
    BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, band_chol5<T, M, RP>, C5_NT, 0));
    BSM_REQUIRE(per_cu >= 1, BSM_ERR_UNSUPPORTED, "band_chol5 does not fit a CU");
    chol_prog_init<<<nblk(n_tiles, 256), 256, 0, s>>>(n_tiles, bd.b, fprog);
    BSM_HIP_TRY(hipGetLastError());
    int64_t grid = (int64_t)cus * per_cu;
    if (grid > n_tiles) grid = n_tiles;
    if (grid < 1) grid = 1;
    // BSM_CHOL5_DELAY=d (stress tests only): every row-block's store waves
    // sleep d x 127 x 64 cycles before storing the last tile (d < 0: wave 0
    // sleeps -d times that before its drain), so completion must wait for the
    // late side whichever it is (tests/test_gpu_solver.py)
    const char* de = getenv("BSM_CHOL5_DELAY");
    const int delay = de ? std::max(-64, std::min(64, atoi(de))) : 0;
    band_chol5<T, M, RP><<<(unsigned)grid, C5_NT, 0, s>>>(bd.n, bd.b, bd.ld, bd.cb.as<T>(), bd.r.as<T>(), fprog, status,
                                                         status + 1, n_tiles, trace, delay);
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

// A into the band layout CB (zeros elsewhere); bw_max: the widest band accepted
template <typename T>
int band_setup(const bsm_csr* a, Band& bd, hipStream_t s, int64_t bw_max) {
    int64_t bw = 0;
    bool sorted = true, empty = false;
    BSM_TRY(band_analyse(a, s, &bw, &sorted, &empty));
    BSM_REQUIRE(sorted, BSM_ERR_UNSUPPORTED,
                "cholesky: rows must have strictly increasing columns (get_row_complete semantics)");
    BSM_REQUIRE(bw <= bw_max, BSM_ERR_UNSUPPORTED, "cholesky: bandwidth %lld > %lld not supported",
                (long long)bw, (long long)bw_max);
    bd.n = (int64_t)a->rows;
    bd.b = bw;
    // the backward solve walks band_walk_terms(b) terms per row and reads the
    // ones past b from this padding (zeros)
    bd.ld = (band_walk_terms(bw) > bw ? band_walk_terms(bw) : bw) + 1;
    const size_t cb_elems = (size_t)bd.n * bd.ld + (size_t)band_pad(bd.ld);
    BSM_TRY(bd.cb.alloc(cb_elems * sizeof(T)));
    BSM_HIP_TRY(hipMemsetAsync(bd.cb.p, 0, cb_elems * sizeof(T), s));
    if (bd.n == 0) return BSM_OK;
    band_fill<T><<<nblk(bd.n, 256), 256, 0, s>>>(a->row_ptr, a->col, static_cast<const T*>(a->vals), bd.n, bd.ld,
                                                 bd.cb.as<T>());
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

template <typename T>
int band_factor(const bsm_csr* a, Band& bd, hipStream_t s) {
    BSM_TRY(band_setup<T>(a, bd, s, 64 * 17 - TR));  // accumulators per row pair lane set
    stage_mark("band_setup", s);
    if (bd.n == 0) return BSM_OK;
    const int64_t bw = bd.b;
    const int64_t n_tiles = (bd.n + TR - 1) / TR;
    DBuf prog;
    BSM_TRY(prog.alloc((n_tiles + 1) * sizeof(int) + 16));
    BSM_HIP_TRY(hipMemsetAsync(prog.p, 0, (n_tiles + 1) * sizeof(int) + 16, s));
    int* status = prog.as<int>() + n_tiles;
    // optional diagnostic trace (BSM_CHOL_TRACE=1): cycles per phase of the row-blocks
    DBuf trace_buf;
    const bool tracing = getenv("BSM_CHOL_TRACE") != nullptr;
    if (tracing) {
        BSM_TRY(trace_buf.alloc(24 * sizeof(unsigned long long)));
        BSM_HIP_TRY(hipMemsetAsync(trace_buf.p, 0, 24 * sizeof(unsigned long long), s));
    }
    unsigned long long* tr = tracing ? trace_buf.as<unsigned long long>() : nullptr;
    int rc;
    BSM_TRY(bd.r.alloc((bd.n + 64) * sizeof(T)));
    const int64_t w4 = bw + C4_TB - 1;  // accumulator columns: i0 - jb <= b + 15
    if (w4 <= 64) rc = launch_chol5<T, 1, 2>(bd, prog.as<int>(), status, s, tr);
    else if (w4 <= 128) rc = launch_chol5<T, 2, 2>(bd, prog.as<int>(), status, s, tr);
    else if (w4 <= 256) rc = launch_chol5<T, 4, 2>(bd, prog.as<int>(), status, s, tr);
    else if (w4 <= 512) rc = launch_chol5<T, 8, 2>(bd, prog.as<int>(), status, s, tr);
    else if (w4 <= 1024) rc = launch_chol5<T, 16, 2>(bd, prog.as<int>(), status, s, tr);
    else rc = launch_chol5<T, 17, 2>(bd, prog.as<int>(), status, s, tr);  // b <= 1073
    BSM_TRY(rc);
    stage_mark("cholesky", s);
    if (tracing) {
        std::vector<unsigned long long> h(17);
        BSM_HIP_TRY(hipMemcpyAsync(h.data(), trace_buf.p, h.size() * 8, hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        const double nb = h[15] ? (double)h[15] : 1.0, nt = h[16] ? (double)h[16] : 1.0;
        fprintf(stderr,
                "[bsm chol trace] row-blocks %llu; cycles per tile (non-last): pollT %.0f stageT %.0f trsm %.0f "
                "publish %.0f pollU+stageU %.0f update %.0f; last tile: pollT %.0f stageT %.0f trsm %.0f (-%.0f) "
                "publish %.0f diag-sums %.0f; diagonal block: barrier %.0f factor %.0f publish %.0f; per "
                "row-block: non-last tiles %.0f\n",
                h[15], h[0] / nt, h[1] / nt, h[2] / nt, h[3] / nt, h[4] / nt, h[5] / nt, h[6] / nb, h[7] / nb,
                h[8] / nb, h[9] / nb, h[10] / nb, h[11] / nb, h[12] / nb, h[13] / nb, h[14] / nb,
                (double)(h[0] + h[1] + h[2] + h[3] + h[4] + h[5]) / nb);
    }
    int st = 0;
    BSM_HIP_TRY(read_dev(&st, status, sizeof(int), s));
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
    BSM_HIP_TRY(read_dev(&nnz, rp.as<int64_t>() + n, sizeof(int64_t), s));
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

// ---------------------------------------------------------------------------
// General exact Cholesky (dense, n <= CHOL_GENERAL_MAX): the inputs the band
// kernels refuse -- a pivot <= 0 or not finite (the reference stores the NaN /
// inf that powf(0.5) and 1/0 give and carries on, sparse.rs:703-710), rows
// with unsorted or duplicate columns (get_row_complete's shifted vector,
// sparse.rs:267-294), or a band too wide for the band kernels. A non-finite
// pivot makes every later L[i][j] non-zero, so L is dense there: this path
// keeps L dense, column-major (Lc[k*n + i] = L[i][k]), and runs the literal
// loop nest of sparse.rs:687-711 one column per launch, every element's sum
// in ascending k with every product kept (no band shortcut).
// ---------------------------------------------------------------------------
constexpr int64_t CHOL_GENERAL_MAX = 16384;

// A as get_row_complete(i) presents it (sparse.rs:279-292): entry p lands at
// position pos, which gains (col - prev_col) padding zeros when col > prev_col
// and then 1; prev_col = col + 1. Positions increase strictly within a row.
// Positions >= n are never read (j <= i < n). Ad is column-major.
template <typename T>
__global__ __launch_bounds__(256) void complete_rows(int64_t n, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ col, const T* __restrict__ v,
                                                     T* __restrict__ Ad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t pos = 0, prev = 0;
    for (int64_t p = rp[i]; p < rp[i + 1]; ++p) {
        const int64_t c = col[p];
        if (c > prev) pos += c - prev;
        prev = c + 1;
        if (pos >= n) break;
        Ad[pos * n + i] = v[p];
        ++pos;
    }
}

// the zero-skipping insert (sparse.rs:229): a zero is not stored and reads
// back as T::default() = +0
template <typename T> __device__ __forceinline__ T stored(T v) { return v == T(0) ? T(0) : v; }

// L[0][0] = powf(A[0][0], 0.5)
template <typename T> __global__ void gchol_pivot0(const T* __restrict__ Ad, T* __restrict__ Lc) {
    if (threadIdx.x == 0) Lc[0] = stored(pow_half(Ad[0]));
}

// column j: L[i][j] = (1 / L[j][j]) * (A[i][j] - sum_k<j L[i][k] L[j][k]) for
// i > j (one thread per row); the thread of row j+1 then forms pivot
// L[j+1][j+1] = powf(A[j+1][j+1] - sum_k<=j L[j+1][k]^2, 0.5), which the next
// launch reads.
template <typename T>
__global__ __launch_bounds__(256) void gchol_column(int64_t n, int64_t j, const T* __restrict__ Ad,
                                                    T* __restrict__ Lc) {
    using A = Arith<T>;
    const int64_t i = j + 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    T sum = A::zero();
#pragma unroll 8
    for (int64_t k = 0; k < j; ++k) sum = A::add(sum, A::mul(Lc[k * n + i], Lc[k * n + j]));
    const T lij = stored(A::mul(div_rn(T(1), Lc[j * n + j]), A::sub(Ad[j * n + i], sum)));
    Lc[j * n + i] = lij;
    if (i == j + 1) {
        T s2 = A::zero();
#pragma unroll 8
        for (int64_t k = 0; k < j; ++k) s2 = A::add(s2, A::mul(Lc[k * n + i], Lc[k * n + i]));
        s2 = A::add(s2, A::mul(lij, lij));
        Lc[i * n + i] = stored(pow_half(A::sub(Ad[i * n + i], s2)));
    }
}

// per row of L: stored entries (j <= i, value != 0; NaN counts) and the first
// stored column
template <typename T>
__global__ __launch_bounds__(256) void gchol_row_count(int64_t n, const T* __restrict__ Lc, int32_t* __restrict__ cnt,
                                                       int32_t* __restrict__ first) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t c = 0, f = INT32_MAX;
    for (int64_t j = 0; j <= i; ++j)
        if (Lc[j * n + i] != T(0)) {
            if (!c) f = (int32_t)j;
            ++c;
        }
    cnt[i] = c;
    first[i] = f;
}

// sparse.rs:707 `l.get_row_complete(j).unwrap()` is None when no row >= j of
// the partial L is registered yet: row j empty and row j+1 has nothing stored
// before column j (longer runs of empty rows contain this case).
__global__ __launch_bounds__(256) void gchol_unregistered(int64_t n, const int32_t* __restrict__ cnt,
                                                          const int32_t* __restrict__ first, int* status) {
    const int64_t j = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= n) return;
    if (cnt[j] == 0 && first[j + 1] >= j) atomicOr(status, ST_EMPTY_ROW);
}

template <typename T>
__global__ __launch_bounds__(256) void gchol_to_csr(int64_t n, const T* __restrict__ Lc, const int64_t* __restrict__ rp,
                                                    int32_t* __restrict__ col, T* __restrict__ val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t e = rp[i];
    for (int64_t j = 0; j <= i; ++j) {
        const T v = Lc[j * n + i];
        if (v != T(0)) {
            col[e] = (int32_t)j;
            val[e] = v;
            ++e;
        }
    }
}

template <typename T>
int chol_general(const bsm_csr* a, int dtype, bsm_csr** out, hipStream_t s) {
    const int64_t n = (int64_t)a->rows;
    const size_t nn = (size_t)n * (size_t)n;
    DBuf ad, lc, cnt, first, ws, rp, st;
    BSM_TRY(ad.alloc(nn * sizeof(T)));
    BSM_TRY(lc.alloc(nn * sizeof(T)));
    BSM_TRY(cnt.alloc(n * sizeof(int32_t)));
    BSM_TRY(first.alloc(n * sizeof(int32_t)));
    BSM_TRY(ws.alloc(scan_workspace_bytes(n)));
    BSM_TRY(rp.alloc((n + 1) * sizeof(int64_t)));
    BSM_TRY(st.alloc(16));
    BSM_HIP_TRY(hipMemsetAsync(ad.p, 0, nn * sizeof(T), s));
    BSM_HIP_TRY(hipMemsetAsync(lc.p, 0, nn * sizeof(T), s));
    BSM_HIP_TRY(hipMemsetAsync(st.p, 0, 16, s));
    complete_rows<T><<<nblk(n, 256), 256, 0, s>>>(n, a->row_ptr, a->col, static_cast<const T*>(a->vals), ad.as<T>());
    gchol_pivot0<T><<<1, 64, 0, s>>>(ad.as<T>(), lc.as<T>());
    for (int64_t j = 0; j + 1 < n; ++j)
        gchol_column<T><<<nblk(n - j - 1, 256), 256, 0, s>>>(n, j, ad.as<T>(), lc.as<T>());
    gchol_row_count<T><<<nblk(n, 256), 256, 0, s>>>(n, lc.as<T>(), cnt.as<int32_t>(), first.as<int32_t>());
    if (n > 2)
        gchol_unregistered<<<nblk(n - 2, 256), 256, 0, s>>>(n, cnt.as<int32_t>(), first.as<int32_t>(), st.as<int>());
    BSM_HIP_TRY(hipGetLastError());
    int h = 0;
    BSM_HIP_TRY(read_dev(&h, st.p, sizeof(int), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_REQUIRE(!(h & ST_EMPTY_ROW), BSM_ERR_PANIC,
                "cholesky: called `Option::unwrap()` on a `None` value (sparse.rs:707: no row >= j of L stored)");
    BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), rp.as<int64_t>(), n, ws.p, ws.bytes, s));
    int64_t nnz = 0;
    BSM_HIP_TRY(read_dev(&nnz, rp.as<int64_t>() + n, sizeof(int64_t), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    auto* m = new bsm_csr();
    m->dtype = dtype;
    m->rows = m->cols = (uint64_t)n;
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
    gchol_to_csr<T><<<nblk(n, 256), 256, 0, s>>>(n, lc.as<T>(), m->row_ptr, m->col, static_cast<T*>(m->vals));
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        bsm_csr_free(m);
        set_error("cholesky (general): %s", hipGetErrorString(e));
        return BSM_ERR_HIP;
    }
    *out = m;
    return BSM_OK;
}

// BSM_BLK_WATCH: a passive host thread that names the step a blocked solve
// is in if it takes longer than 15 s, then ends the process (no GPU calls)
static std::atomic<const char*> g_blk_phase{"idle"};
static std::atomic<int> g_blk_gen{0};
static void blk_watch_start() {
    if (!getenv("BSM_BLK_WATCH")) return;
    const int gen = ++g_blk_gen;
    std::thread([gen] {
        for (int i = 0; i < 150; ++i) {
            usleep(100000);
            if (g_blk_gen.load() != gen) return;
        }
        fprintf(stderr, "[blk watch] stuck in: %s\n", g_blk_phase.load());
        fflush(stderr);
        _exit(3);
    }).detach();
}
static void blk_watch_stop() { ++g_blk_gen; }

// BSM_BLK_DEBUG: wait up to 10 s for the stream, else print the kernel's
// progress (mapped host counters) and end the process (a hung kernel would
// otherwise hold the test until its timeout)
static void blk_watchdog(hipStream_t s, const char* what, unsigned long long* hdbg, long long tickets,
                         long long grid, const unsigned long long* tdev = nullptr) {
    if (!getenv("BSM_BLK_DEBUG")) return;
    for (int i = 0; i < 200; ++i) {
        if (hipStreamQuery(s) == hipSuccess) {
            fprintf(stderr, "[blk debug] %s done: tickets %lld grid %lld", what, tickets, grid);
            unsigned long long t[48] = {};
            if (tdev && hipMemcpy(t, tdev, sizeof(t), hipMemcpyDeviceToHost) != hipSuccess) t[7] = t[10] = 0;
            if (t[7])
                fprintf(stderr, "; per diagonal tile: factor %.0f cycles, inverse %.0f, factor..drained %.0f; "
                        "diagonal tiles 0..last %.3f ms (100 MHz clock, %.2f us per tile)",
                        (double)t[4] / t[7], (double)t[5] / t[7], (double)t[11] / t[7], (t[13] - t[12]) * 1e-5,
                        (t[13] - t[12]) * 1e-2 / (double)t[7]);
            if (t[10])
                fprintf(stderr, "; chain: waits for K-1 %.0f, from K-1 visible to the factor %.0f (stage Linv %.0f, "
                        "product + stores %.0f, update + drain + flag %.0f, the rest)",
                        (double)t[8] / t[10], (double)t[9] / t[10], (double)t[14] / t[10], (double)t[15] / t[10],
                        (double)t[16] / t[10]);
            if (t[23])
                fprintf(stderr, "; chain workgroup per block column: L_{K,K-1} + update + flags %.0f cycles, factor "
                        "%.0f, publish + next pending %.0f; %.3f ms over %llu block columns (%.2f us each, 100 MHz "
                        "clock)",
                        (double)t[20] / t[23], (double)t[21] / t[23], (double)t[22] / t[23], (t[13] - t[12]) * 1e-5,
                        t[23], (t[13] - t[12]) * 1e-2 / (double)t[23]);
            if (t[23] && t[3])
                fprintf(stderr, "; chain waits for the next pending tile %.0f cycles; pending tiles: last block "
                        "column's flags waited %.0f, its update to the publication %.0f",
                        (double)t[0] / t[23], (double)t[1] / t[3], (double)t[2] / t[3]);
            if (t[23] && t[17])
                fprintf(stderr, "; panel factor: wave 0's blocks %.0f, rows below %.0f, trailing %.0f",
                        (double)t[17] / t[23], (double)t[18] / t[23], (double)t[19] / t[23]);
            else if (t[7] && t[17])
                fprintf(stderr, "; panel factor: wave 0's blocks %.0f, rows below %.0f, trailing %.0f",
                        (double)t[17] / t[7], (double)t[18] / t[7], (double)t[19] / t[7]);
            if (t[23] && t[36]) {
                fprintf(stderr, "; wave 0's tasks (wait/run cycles):");
                for (int i = 0; i < 11; ++i)
                    fprintf(stderr, " %.0f/%.0f", (double)t[24 + i] / t[23], (double)t[36 + i] / t[23]);
            }
            fprintf(stderr, "\n");
            return;
        }
        usleep(50000);
    }
    fprintf(stderr, "[blk debug] %s HUNG: tickets %lld grid %lld max ticket %llu, waiting on flag %llu "
            "(stuck waits %llu), tiles done %llu\n", what, tickets, grid, hdbg ? hdbg[0] : 0ull,
            hdbg ? hdbg[1] : 0ull, hdbg ? hdbg[2] : 0ull, hdbg ? hdbg[3] : 0ull);
    fflush(stderr);
    _exit(3);
}

// blocked (reassociated) band Cholesky into bd; Dinv (nb64 x 4096) receives
// the inverse diagonal tiles
template <typename T>
int band_factor_blocked(const bsm_csr* a, Band& bd, DBuf& dinv, hipStream_t s) {
    BSM_TRY(band_setup<T>(a, bd, s, (int64_t)1 << 16));
    stage_mark("band_setup", s);
    const int64_t n = bd.n, nb64 = (n + 63) / 64, DM = (63 + bd.b) / 64 + 1;
    BSM_TRY(dinv.alloc((size_t)(nb64 > 0 ? nb64 : 1) * 4096 * sizeof(T)));
    if (n == 0) return BSM_OK;
    // flags: one per tile, the ticket, the status word, then 4 per block
    // column for Linv's progressive row blocks (rbf)
    DBuf fl;
    const size_t nfl = (size_t)(nb64 * DM + 2 + 4 * nb64);
    BSM_TRY(fl.alloc(nfl * sizeof(int)));
    BSM_HIP_TRY(hipMemsetAsync(fl.p, 0, nfl * sizeof(int), s));
    int* flags = fl.as<int>();
    int* tix = flags + nb64 * DM;
    int* st = tix + 1;
    int* rbf = st + 1;
    int dev = 0, cus = 0, per_cu = 0;
    BSM_HIP_TRY(hipGetDevice(&dev));
    BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, blk_chol<T>, 256, 0));
    BSM_REQUIRE(per_cu >= 1, BSM_ERR_UNSUPPORTED, "blk_chol does not fit a CU");
    int64_t grid = (int64_t)cus * per_cu;
    if (grid > nb64 * DM) grid = nb64 * DM;
    // BSM_BLK_DEBUG=1: watchdog counters in host memory and chain timers;
    // =2: the chain timers alone (device memory: no PCIe atomics on the chain)
    unsigned long long* hdbg = nullptr;
    DBuf tdb;
    const char* dbe = getenv("BSM_BLK_DEBUG");
    if (dbe && atoi(dbe) != 2) {
        BSM_HIP_TRY(hipHostMalloc((void**)&hdbg, 24 * sizeof(unsigned long long), hipHostMallocCoherent));
        memset(hdbg, 0, 24 * sizeof(unsigned long long));
    }
    if (dbe) {
        BSM_TRY(tdb.alloc(48 * sizeof(unsigned long long)));
        BSM_HIP_TRY(hipMemsetAsync(tdb.p, 0, 48 * sizeof(unsigned long long), s));
    }
    g_blk_phase = "blk_chol launch";
    const CholSeg<T> seg{bd.cb.as<T>(), n, dinv.as<T>(), flags, rbf};
    DBuf segd;
    BSM_TRY(segd.alloc(sizeof(seg)));
    BSM_HIP_TRY(hipMemcpyAsync(segd.p, &seg, sizeof(seg), hipMemcpyHostToDevice, s));
    blk_chol<T><<<(unsigned)grid, 256, 0, s>>>(bd.b, bd.ld, segd.as<CholSeg<T>>(), 1, nb64, tix, st, hdbg,
                                                tdb.as<unsigned long long>());
    BSM_HIP_TRY(hipGetLastError());
    stage_mark("cholesky", s);
    blk_watchdog(s, "blk_chol", hdbg, (long long)(nb64 * DM), grid, tdb.as<unsigned long long>());
    g_blk_phase = "blk_chol sync";
    int h = 0;
    BSM_HIP_TRY(read_dev(&h, st, sizeof(int), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_REQUIRE(!(h & ST_TIMEOUT), BSM_ERR_HIP, "blocked cholesky: tile hand-off timed out");
    BSM_REQUIRE(!(h & ST_NOT_PD), BSM_ERR_UNSUPPORTED,
                "cholesky: matrix is not positive definite (a pivot is <= 0 or not finite)");
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

// the general exact path takes what the band kernels refuse (non-finite or
// non-positive pivots, unsorted rows, too wide a band) when L fits densely;
// BSM_CHOL_GENERAL=1 forces it (A/B against the band kernels)
static bool chol_general_forced(const bsm_csr* a) {
    const char* e = getenv("BSM_CHOL_GENERAL");
    return e && atoi(e) == 1 && a->rows >= 1 && (int64_t)a->rows <= CHOL_GENERAL_MAX;
}
static bool chol_general_fits(const bsm_csr* a) { return a->rows >= 1 && (int64_t)a->rows <= CHOL_GENERAL_MAX; }

int solve_dispatch_cholesky(const bsm_csr* a, bsm_csr** out, hipStream_t s) {
    auto run = [&]<typename T>() -> int {
        if (!chol_general_forced(a)) {
            Band bd;
            const int rc = band_factor<T>(a, bd, s);
            if (rc == BSM_OK) return band_to_csr_host<T>(bd, a->dtype, out, s);
            if (rc != BSM_ERR_UNSUPPORTED || !chol_general_fits(a)) return rc;
        }
        return chol_general<T>(a, a->dtype, out, s);
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
        if (n && k && m->cols > n) {  // columns past the RHS rows: the reference panics on them
            csr_cols_past_rhs<<<nblk(n, 256), 256, 0, s>>>((int64_t)n, m->row_ptr, m->col, !lower, st.as<int>());
            BSM_HIP_TRY(hipGetLastError());
            int h = 0;
            BSM_HIP_TRY(read_dev(&h, st.p, sizeof(int), s));
            BSM_REQUIRE(!(h & ST_COL_OOB), BSM_ERR_PANIC,
                        "index out of bounds: a column index >= the %llu rows of the right-hand side "
                        "(lib.rs:38 / :58)", (unsigned long long)n);
        }
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
        BSM_HIP_TRY(read_dev(&h, st.p, sizeof(int), s));
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

// solve (lib.rs:11-24) on the general factor: L dense-exact, L* =
// transpose, then the general-CSR forward and backward solves, which divide
// by the last / first stored entry of each row as the reference does
template <typename T>
static int solve_general(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev, hipStream_t s) {
    bsm_csr* l = nullptr;
    bsm_csr* lt = nullptr;
    BSM_TRY(chol_general<T>(a, a->dtype, &l, s));
    stage_mark("cholesky", s);
    int rc = transpose_dispatch(l, &lt, s);
    DBuf y;
    if (rc == BSM_OK) rc = y.alloc(n * k * sizeof(T));
    if (rc == BSM_OK) rc = solve_dispatch_trsv(l, true, k, n, b_dev, y.p, s);
    if (rc == BSM_OK) stage_mark("forward", s);
    if (rc == BSM_OK) rc = solve_dispatch_trsv(lt, false, k, n, y.p, x_dev, s);
    if (rc == BSM_OK) stage_mark("backward", s);
    bsm_csr_free(l);
    if (lt) bsm_csr_free(lt);
    return rc;
}

// band backward solve: band_backward_reg over W = band_walk_terms(b) terms
// per row (ld >= W + 1 is set by band_setup)
template <typename T>
static int launch_backward(uint64_t n, uint64_t k, int64_t b, int64_t ld, const T* cb, const T* y, T* x,
                           hipStream_t s) {
    const int64_t N = (int64_t)n;
    BSM_REQUIRE(ld >= band_walk_terms(b) + 1, BSM_ERR_INVALID, "backward: band ld %lld too small", (long long)ld);
    auto go = [&]<int SEG, int NL>() { band_backward_reg<T, SEG, NL><<<(unsigned)k, 64, 0, s>>>(N, b, ld, cb, y, x); };
    const BwCfg c = band_walk_cfg(b);
    if (c.seg == 40) go.template operator()<40, 25>();
    else if (c.seg == 1) go.template operator()<1, 64>();
    else if (c.seg == 2) go.template operator()<2, 64>();
    else if (c.seg == 4) go.template operator()<4, 64>();
    else if (c.seg == 8) go.template operator()<8, 64>();
    else if (c.seg == 12) go.template operator()<12, 64>();
    else if (c.seg == 16 && c.nl == 56) go.template operator()<16, 56>();
    else if (c.seg == 16) go.template operator()<16, 64>();
    else if (c.seg == 32) go.template operator()<32, 64>();
    else BSM_REQUIRE(false, BSM_ERR_UNSUPPORTED, "backward: band %lld too wide", (long long)b);
    BSM_HIP_TRY(hipGetLastError());
    return BSM_OK;
}

int solve_dispatch_full(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev, hipStream_t s) {
    auto run = [&]<typename T>() -> int {
        BSM_REQUIRE(a->rows == n, BSM_ERR_PANIC,
                    "solve: b has %llu rows but A has %llu (index out of bounds in the reference)",
                    (unsigned long long)n, (unsigned long long)a->rows);
        stage_reset(s);
        Band bd;
        const int frc = chol_general_forced(a) ? BSM_ERR_UNSUPPORTED : band_factor<T>(a, bd, s);
        if (frc == BSM_ERR_UNSUPPORTED && chol_general_fits(a)) {
            bd.cb.reset();
            bd.r.reset();
            return solve_general<T>(a, k, n, b_dev, x_dev, s);
        }
        BSM_TRY(frc);
        // the reference's forward pass divides by the LAST stored entry of
        // each L row and its backward pass by the FIRST of each L^T row: with
        // every pivot > 0 (checked) both are L_ii, as used below.
        DBuf bc, yc, xc;
        BSM_TRY(to_colmajor(a->dtype, n, k, b_dev, bc, s));
        BSM_TRY(yc.alloc(n * k * sizeof(T)));
        BSM_TRY(xc.alloc(n * k * sizeof(T)));
        if (n && k) {
            // forward_substitution(l, b) over rows 0..n of L (lib.rs:31-44);
            // BSM_FW_TRACE=1: cycles per phase
            DBuf ftr;
            unsigned long long* ftp = nullptr;
            if (getenv("BSM_FW_TRACE")) {
                BSM_TRY(ftr.alloc(8 * sizeof(unsigned long long)));
                BSM_HIP_TRY(hipMemsetAsync(ftr.p, 0, 8 * sizeof(unsigned long long), s));
                ftp = ftr.as<unsigned long long>();
            }
            // one solving workgroup per column for narrow bands (or many columns)
            if (bd.b <= FW3_NEAR || k * (1 + FW3_HELPERS) > 256)
                band_forward2<T, 8, 24><<<(unsigned)k, 512, 0, s>>>((int64_t)n, bd.b, bd.ld, bd.cb.as<T>(),
                                                                    bc.as<T>(), yc.as<T>(), ftp);
            else {  // default: the far prefixes on FW3_HELPERS helper workgroups per column
                const uint64_t nblk = (n + 63) / 64;
                DBuf pbuf, flags;
                BSM_TRY(pbuf.alloc(k * nblk * 64 * sizeof(T)));
                BSM_TRY(flags.alloc((k * nblk + k + 1) * sizeof(int)));
                BSM_HIP_TRY(hipMemsetAsync(flags.p, 0, (k * nblk + k + 1) * sizeof(int), s));
                int* pflag = flags.as<int>();
                int* gfront = pflag + k * nblk;
                int* fst = gfront + k;
                band_forward2<T, 8, 8, FW3_HELPERS><<<(unsigned)(k * (1 + FW3_HELPERS)), 512, 0, s>>>(
                    (int64_t)n, bd.b, bd.ld, bd.cb.as<T>(), bc.as<T>(), yc.as<T>(), ftp, pbuf.as<T>(), pflag, gfront,
                    fst);
                BSM_HIP_TRY(hipGetLastError());
                int st = 0;
                BSM_HIP_TRY(read_dev(&st, fst, sizeof(int), s));
                BSM_HIP_TRY(hipStreamSynchronize(s));
                BSM_REQUIRE(!(st & ST_TIMEOUT), BSM_ERR_HIP, "forward: helper hand-off timed out");
            }
            BSM_HIP_TRY(hipGetLastError());
            if (ftp) {
                unsigned long long h[8];
                BSM_HIP_TRY(hipMemcpyAsync(h, ftp, sizeof(h), hipMemcpyDeviceToHost, s));
                BSM_HIP_TRY(hipStreamSynchronize(s));
                const double nb = (double)((n + 63) / 64) * (double)k, hb = h[7] ? (double)h[7] : 1.0;
                fprintf(stderr,
                        "[bsm fw trace] cycles per 64-row block: far phase %.0f (of which waiting for the "
                        "frontier %.0f, for the helper prefix %.0f), wait %.0f, solve %.0f; helper blocks %llu: "
                        "%.0f cycles each, %.0f of them waiting for y\n",
                        h[0] / nb, h[3] / nb, h[4] / nb, h[1] / nb, h[2] / nb, h[7], h[5] / hb, h[6] / hb);
            }
            stage_mark("forward", s);
            BSM_TRY(launch_backward<T>(n, k, bd.b, bd.ld, bd.cb.as<T>(), yc.as<T>(), xc.as<T>(), s));
            stage_mark("backward", s);
        }
        BSM_TRY(from_colmajor(a->dtype, n, k, xc.p, x_dev, s));
        stage_mark("copy_out", s);
        BSM_HIP_TRY(hipStreamSynchronize(s));
        return BSM_OK;
    };
    if (a->dtype == BSM_F64) return run.template operator()<double>();
    if (a->dtype == BSM_F32) return run.template operator()<float>();
    set_error("solve: f32/f64 only");
    return BSM_ERR_INVALID;
}

// solve with reassociated (blocked) triangular solves: the factor is the
// reference-order band Cholesky; the two solves are blk_trsv (see there).
int solve_dispatch_blocked(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev,
                           hipStream_t s) {
    auto run = [&]<typename T>() -> int {
        BSM_REQUIRE(a->rows == n, BSM_ERR_PANIC,
                    "solve: b has %llu rows but A has %llu (index out of bounds in the reference)",
                    (unsigned long long)n, (unsigned long long)a->rows);
        blk_watch_start();
        stage_reset(s);
        g_blk_phase = "band setup";
        Band bd;
        DBuf dinv;
        // BSM_BLK_CHOL=0: the reference-order factor (band_factor: band_chol5 by default) under the blocked solves (A/B)
        const char* bc_env = getenv("BSM_BLK_CHOL");
        if (bc_env && atoi(bc_env) == 0) BSM_TRY(band_factor<T>(a, bd, s));
        else BSM_TRY(band_factor_blocked<T>(a, bd, dinv, s));
        DBuf bc, xc;
        BSM_TRY(to_colmajor(a->dtype, n, k, b_dev, bc, s));
        BSM_TRY(xc.alloc(n * k * sizeof(T)));
        if (n && k) {
            const uint64_t nb64 = (n + 63) / 64, NP = nb64 * 64;
            DBuf g, h, mf, mb, yp, xp, fl;
            BSM_TRY(g.alloc(nb64 * 4096 * sizeof(T)));
            BSM_TRY(h.alloc(nb64 * 4096 * sizeof(T)));
            BSM_TRY(mf.alloc(nb64 * 4096 * sizeof(T)));
            BSM_TRY(mb.alloc(nb64 * 4096 * sizeof(T)));
            BSM_TRY(yp.alloc(k * NP * sizeof(T)));
            BSM_TRY(xp.alloc(k * NP * sizeof(T)));
            const uint64_t nfl = 2 * k * nb64 + 4;  // forward flags, backward flags, 2 tickets, status
            BSM_TRY(fl.alloc(nfl * sizeof(int)));
            BSM_HIP_TRY(hipMemsetAsync(fl.p, 0, nfl * sizeof(int), s));
            int* ff = fl.as<int>();
            int* fb = ff + k * nb64;
            int* tix = fb + k * nb64;
            int* st = tix + 2;
            g_blk_phase = "blk_prep + trsv launches";
            blk_prep<T><<<(unsigned)nb64, 256, 0, s>>>((int64_t)n, bd.b, bd.ld, bd.cb.as<T>(), g.as<T>(), h.as<T>(),
                                                      mf.as<T>(), mb.as<T>());
            BSM_HIP_TRY(hipGetLastError());
            stage_mark("blk_prep", s);
            int dev = 0, cus = 0, per_cu = 0;
            BSM_HIP_TRY(hipGetDevice(&dev));
            BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, blk_trsv<T, false>, 256, 0));
            BSM_REQUIRE(per_cu >= 1, BSM_ERR_UNSUPPORTED, "blk_trsv does not fit a CU");
            uint64_t grid = (uint64_t)cus * (uint64_t)per_cu;
            if (grid > nb64 * k) grid = nb64 * k;
            const TrsvSeg<T> sg[2] = {
                {bd.cb.as<T>(), (int64_t)n, g.as<T>(), mf.as<T>(), bc.as<T>(), (int64_t)n, yp.as<T>(), ff},
                {bd.cb.as<T>(), (int64_t)n, h.as<T>(), mb.as<T>(), yp.as<T>(), (int64_t)NP, xp.as<T>(), fb}};
            DBuf sgd;
            BSM_TRY(sgd.alloc(sizeof(sg)));
            BSM_HIP_TRY(hipMemcpyAsync(sgd.p, sg, sizeof(sg), hipMemcpyHostToDevice, s));
            blk_trsv<T, true><<<(unsigned)grid, 256, 0, s>>>(bd.b, bd.ld, sgd.as<TrsvSeg<T>>(), 1, (int64_t)nb64,
                                                            tix, st, (int64_t)k);
            BSM_HIP_TRY(hipGetLastError());
            stage_mark("forward", s);
            blk_watchdog(s, "blk_trsv forward", nullptr, (long long)(nb64 * k), (long long)grid);
            blk_trsv<T, false><<<(unsigned)grid, 256, 0, s>>>(bd.b, bd.ld, sgd.as<TrsvSeg<T>>() + 1, 1,
                                                             (int64_t)nb64, tix + 1, st, (int64_t)k);
            BSM_HIP_TRY(hipGetLastError());
            stage_mark("backward", s);
            blk_watchdog(s, "blk_trsv backward", nullptr, (long long)(nb64 * k), (long long)grid);
            int hst = 0;
            g_blk_phase = "trsv sync";
            BSM_HIP_TRY(read_dev(&hst, st, sizeof(int), s));
            BSM_HIP_TRY(hipStreamSynchronize(s));
            BSM_REQUIRE(!(hst & ST_TIMEOUT), BSM_ERR_HIP, "blocked solve: block hand-off timed out");
            BSM_HIP_TRY(hipMemcpy2DAsync(xc.p, n * sizeof(T), xp.p, NP * sizeof(T), n * sizeof(T), k,
                                         hipMemcpyDeviceToDevice, s));
        }
        g_blk_phase = "unpack + final sync";
        BSM_TRY(from_colmajor(a->dtype, n, k, xc.p, x_dev, s));
        stage_mark("copy_out", s);
        BSM_HIP_TRY(hipStreamSynchronize(s));
        g_blk_phase = "idle";
        blk_watch_stop();
        return BSM_OK;
    };
    if (a->dtype == BSM_F64) return run.template operator()<double>();
    if (a->dtype == BSM_F32) return run.template operator()<float>();
    set_error("solve: f32/f64 only");
    return BSM_ERR_INVALID;
}

}  // namespace bsm
