// solve_tiles.hpp -- device helpers shared by the blocked band solver
// (kernels_solve.hip) and the nested-dissection multifrontal solver
// (kernels_nd.hip): write-through hand-offs, DPP row broadcasts, and the
// 64 x 64 tile operations on f64 MFMA (factor + inverse of a diagonal tile,
// tile products). Included inside namespace bsm { namespace { ... } }.
#pragma once

constexpr long long SPIN_LIMIT = 1ll << 25;

enum { ST_NOT_PD = 1, ST_TIMEOUT = 2, ST_EMPTY_ROW = 4, ST_COL_OOB = 8 };

// Row-block tickets for the persistent Cholesky grids, handed out in
// ascending order: a workgroup only ever waits on LOWER row-blocks, which
// workgroups already running hold, so progress needs no co-residency of the
// grid (a CU held by another kernel or stream only slows the factor down).
__device__ __forceinline__ int64_t next_ticket(int* ticket, int* s_tk) {
    __syncthreads();  // every thread has read the previous ticket
    if (threadIdx.x == 0) *s_tk = atomicAdd(ticket, 1);
    __syncthreads();
    return *s_tk;
}

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

// Lane j of each 16-lane row to the whole row (DPP row_newbcast:j, gfx90a+; the
// one DPP form 64-bit data may use): a VALU move, no LDS, no SGPR. Full masks
// and bound_ctrl make the old value dead, so a double is ONE v_mov_b64_dpp
// (with old = 0 and no bound_ctrl it was two v_mov_b32_dpp after two moves
// initialising the destination).
template <int J> __device__ __forceinline__ int rowbcast_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + J, 0xf, 0xf, true);
}
template <int J> __device__ __forceinline__ double rowbcast(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xf, 0xf, true);
}
template <int J> __device__ __forceinline__ float rowbcast(float v) {
    return __int_as_float(rowbcast_i<J>(__float_as_int(v)));
}

__device__ __forceinline__ double fma_t(double a, double b, double c) { return __fma_rn(a, b, c); }
__device__ __forceinline__ float fma_t(float a, float b, float c) { return __fmaf_rn(a, b, c); }

// tiles in LDS: rows padded to 65 elements (row-strided accesses hit distinct banks)
constexpr int TLD = 65;

// LDS pointers that keep their address space across a call
template <typename T> using lds_t = __attribute__((address_space(3))) T;
// the f64 MFMA 16x16x4 accumulator
typedef double bsm_d4 __attribute__((ext_vector_type(4)));

// 1/sqrt(x): the hardware estimate and one Newton step (its error squared
// once): a short dependent chain for the blocked factor's pivots (two steps:
// 317 against 311 ms at C5, x error 8.8e-11 against 9.7e-11)
__device__ __forceinline__ double rsqrt_nr1(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double h = __fma_rn(-x * y, y, 1.0);
    return __fma_rn(0.5 * y, h, y);
}
__device__ __forceinline__ float rsqrt_nr(float x) {
    float y = __builtin_amdgcn_rsqf(x);
    const float h = __fmaf_rn(-x * y, y, 1.0f);
    return __fmaf_rn(0.5f * y, h, y);
}
__device__ __forceinline__ float rsqrt_nr1(float x) { return rsqrt_nr(x); }

// Block (p2, p1), p1 < p2, of Linv on one wave (f64 MFMA 16x16x4):
// Linv[p2][p1] = -Di[p2] sum_{q = p1}^{p2 - 1} L[p2][q] Linv[q][p1],
// from row blocks < p2 of Linv already in Q (Q[c * TLD + r] = Linv[r][c]).
template <typename T>
__device__ __forceinline__ void blk_linv_block(const lds_t<T>* P, lds_t<T>* Q, const lds_t<T>* Di, int p2, int p1,
                                               int l) {
    const int m = l & 15, kq = l >> 4;
    bsm_d4 t = {0.0, 0.0, 0.0, 0.0};
    for (int qb = p1; qb < p2; ++qb) {
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            const int k = 16 * qb + 4 * k4 + kq;
            t = __builtin_amdgcn_mfma_f64_16x16x4f64((double)P[(16 * p2 + m) * TLD + k],
                                                     (double)Q[(16 * p1 + m) * TLD + k], t, 0, 0, 0);
        }
    }
    bsm_d4 o = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4)
        o = __builtin_amdgcn_mfma_f64_16x16x4f64(-(double)Di[p2 * 256 + m * 16 + 4 * k4 + kq], t[k4], o, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) Q[(16 * p1 + m) * TLD + 16 * p2 + kq + 4 * q] = (T)o[q];
}

// Q's diagonal block p = Di[p] (Di[p][row][col] -> Q[col * TLD + row]), one wave
template <typename T>
__device__ __forceinline__ void blk_linv_diag(lds_t<T>* Q, const lds_t<T>* Di, int p, int l) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = l + 64 * u, row = e >> 4, col = e & 15;
        Q[(16 * p + col) * TLD + 16 * p + row] = Di[p * 256 + e];
    }
}

// Factor AND invert the 64 x 64 tile S (P[r * TLD + c], lower part) on all
// four waves, by 16-column panels p (columns c0 = 16p ...):
//   1. wave 0 factors the 16 x 16 diagonal block (lane r & 15 = row, pivots
//      and L[j][t] by DPP row broadcast: no LDS, no barrier) and inverts it
//      into Di[p];
//   2. the rows below: L[i][c0 + j] = sum_t S[i][c0 + t] Di[p][j][t];
//   3. the trailing lower part: S[i][j] -= sum_t L[i][c0 + t] L[j][c0 + t].
// Steps 2 and 3 are 16 x 16 blocks on f64 MFMA, one block per wave at a time.
// Linv by row blocks: row block p - 1 on waves 1-3 while wave 0 factors
// block p, the last one at the end. rd[r] = 1 / L[r][r].
// Every thread of the workgroup must call it (barriers inside).
// Progressive publication (dpub): Linv's row block
// p - 1 is complete once wave 0 has factored block p; wave 3, idle in the rows
// below and the trailing update from panel 1 on, stores it to dpub (this
// tile's Dinv, dpub[s * 64 + l] = Linv[l][s]) and raises rbf[p - 1] when the
// stores have drained, one panel later. The next diagonal tile forms the
// matching column block of its sub-diagonal tile and that block's update
// while this factor runs (blk_chol): only row block 3 is left on the
// chain. Row block 3 goes out with the tile's flag, as before.
template <typename T>
__device__ __forceinline__ void blk_publish_rowblock(const lds_t<T>* Q, T* __restrict__ dpub, int c, int lane) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int i = lane + 64 * u, s = i >> 4, j = i & 15;
        st_sc1(&dpub[s * 64 + 16 * c + j], (T)Q[s * TLD + 16 * c + j]);
    }
}
__device__ __forceinline__ void blk_publish_flag(int* rbf, int c, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&rbf[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

//
// npan < 4 (the nested-dissection fronts' last pivot tile, whose pivots past
// np are padding: identity rows and columns, zero elsewhere): only panels
// p < npan hold real pivots. A padding panel's factor, rows below, trailing
// update and Linv blocks would produce exactly the identity and zeros it
// already holds (pivot 1: rsqrt 1, L 1, x 1; products with zero rows leave
// S's bits), so they are skipped and Q's padding diagonal set to 1: the same
// bits in ~npan / 4 of the time. Uniform across the workgroup (the barriers).
template <typename T>
__device__ __forceinline__ void blk_diag_panels(lds_t<T>* P, lds_t<T>* Q, lds_t<T>* Di, lds_t<T>* Tb, lds_t<T>* rd,
                                                int* status, int tid, unsigned long long* tdbg,
                                                T* __restrict__ dpub, int* rbf, int* pflag, int npan = 4) {
    long long ta = 0, tb = 0, tc = 0;  // BSM_BLK_DEBUG: wave 0's block, the rows below, the trailing update
    asm volatile("" : "+v"(tid));  // opaque: keep the per-step masks out of the ticket loop
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    bool pd = true;
#pragma unroll
    for (int u = 0; u < 16; ++u) Q[(tid >> 2) * TLD + 16 * (tid & 3) + u] = (T)0;  // rows of Linv^T
    npan = __builtin_amdgcn_readfirstlane(npan);
    for (int p = 0; p < npan; ++p) {
        const int c0 = 16 * p;
        const long long t0 = tdbg ? clock64() : 0;
        if (dpub && w == 3 && p >= 2) blk_publish_flag(rbf, p - 2, tid & 63);  // row block p - 2, stored a panel ago
        if (w > 0) {
            // while wave 0 factors block p: Linv's row block p - 1 (its blocks
            // need row blocks < p - 1, Di[p - 1] and L's columns < p - 1, all
            // complete) and diagonal block p - 1
            if (p >= 2 && w - 1 < p - 1) blk_linv_block<T>(P, Q, Di, p - 1, w - 1, tid & 63);
            if (p >= 1 && w == 3) blk_linv_diag<T>(Q, Di, p - 1, tid & 63);
        } else {
            const int r = tid & 15;
            T dv[16], rps[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) dv[j] = P[(c0 + r) * TLD + c0 + j];
            // The factor and the block's inverse in one pass. Step t: the pivot,
            // column t of L (l, lane j: L[j][t]), the trailing update of the
            // rows below by L[j][t] broadcast from lane j; and, with the same
            // broadcasts, x[t] = Linv[t][r] of lane r's inverse column and its
            // terms in the later rows' sums (acc[j] += L[j][t] x[t]): the FMAs
            // of the row-by-row inverse, in the same order per row, so the
            // same bits, with no second pass and no second set of broadcasts.
            // The next pivot is lane t+1's own update fma(-l, l, dv[t+1]) (its
            // broadcast of l is its own l): the pivot chain skips that broadcast.
            T x[16], acc[16];
#pragma unroll
            for (int q2 = 0; q2 < 16; ++q2) acc[q2] = (T)0;
            T nxt = dv[0];
            auto step = [&]<int t>(std::integral_constant<int, t>) __attribute__((always_inline)) {
                const T piv = rowbcast<t>(nxt);
                pd = pd & (piv > (T)0) & (piv < (T)INFINITY);
                const T rp = rsqrt_nr1(piv);
                rps[t] = rp;
                const T l = dv[t] * rp;  // lane t: the pivot's square root
                dv[t] = l;
                x[t] = ((t == r ? (T)1 : (T)0) - acc[t]) * rp;
                if constexpr (t < 15) nxt = fma_t(-l, l, dv[t + 1]);
                [&]<int... js>(std::integer_sequence<int, js...>) __attribute__((always_inline)) {
                    (([&] {
                         const T bl = rowbcast<t + 1 + js>(l);
                         dv[t + 1 + js] = fma_t(-l, bl, dv[t + 1 + js]);
                         acc[t + 1 + js] = fma_t(bl, x[t], acc[t + 1 + js]);
                     }()),
                     ...);
                }(std::make_integer_sequence<int, 15 - t>{});
            };
            [&]<int... ts>(std::integer_sequence<int, ts...>) __attribute__((always_inline)) {
                (step(std::integral_constant<int, ts>{}), ...);
            }(std::make_integer_sequence<int, 16>{});
#pragma unroll
            for (int j = 0; j < 16; ++j) P[(c0 + r) * TLD + c0 + j] = j <= r ? dv[j] : (T)0;
#pragma unroll
            for (int q2 = 0; q2 < 16; ++q2) Di[p * 256 + q2 * 16 + r] = x[q2];  // Di[p][row][col]
#pragma unroll
            for (int t = 0; t < 16; ++t) rd[c0 + t] = rps[t];
        }
        // pflag: the caller's global stores (the sub-diagonal tile) drain on
        // every wave during block 0's factor; the flag follows the barrier
        if (pflag && p == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const long long t1 = tdbg ? clock64() : 0;
        if (pflag && p == 0 && tid == 192) __hip_atomic_store(pflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dpub && w == 3 && p >= 1) blk_publish_rowblock<T>(Q, dpub, p - 1, tid & 63);
        // 2. rows below the block, one 16-row block per wave on f64 MFMA
        //    16x16x4: L[pb][p] = S[pb][p] Di[p]^T (read and written by the same wave)
        const int l = tid & 63, m = l & 15, kq = l >> 4;
        if (w < 3 - p) {
            const int r0 = 16 * (p + 1 + w);
            bsm_d4 o = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const int k = 4 * k4 + kq;
                o = __builtin_amdgcn_mfma_f64_16x16x4f64((double)P[(r0 + m) * TLD + c0 + k],
                                                         (double)Di[p * 256 + m * 16 + k], o, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) P[(r0 + kq + 4 * q) * TLD + c0 + m] = (T)o[q];
        }
        __syncthreads();
        const long long t2 = tdbg ? clock64() : 0;
        // 3. the trailing lower part by 16 x 16 blocks (pi, pj), p < pj <= pi:
        //    S[pi][pj] -= L[pi][p] L[pj][p]^T, blocks dealt to the waves in turn
        const int nbk = 3 - p;
        for (int bk = w; bk < nbk * (nbk + 1) / 2; bk += 4) {
            int pi = 0, pj = bk;  // bk -> (pi, pj), pj <= pi, both relative to p + 1
            while (pj > pi) pj -= ++pi;
            const int i0 = 16 * (p + 1 + pi), j0 = 16 * (p + 1 + pj);
            bsm_d4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = (double)P[(i0 + kq + 4 * q) * TLD + j0 + m];
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const int k = 4 * k4 + kq;
                o = __builtin_amdgcn_mfma_f64_16x16x4f64(-(double)P[(i0 + m) * TLD + c0 + k],
                                                         (double)P[(j0 + m) * TLD + c0 + k], o, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) P[(i0 + kq + 4 * q) * TLD + j0 + m] = (T)o[q];
        }
        __syncthreads();
        if (tdbg) {
            const long long t3 = clock64();
            ta += t1 - t0;
            tb += t2 - t1;
            tc += t3 - t2;
        }
    }
    // Linv's last row block and diagonal block (of the real panels)
    const int pl = npan - 1;
    if (w < pl) {
        blk_linv_block<T>(P, Q, Di, pl, w, tid & 63);
    } else if (w == 3) {
        if (dpub) blk_publish_flag(rbf, 2, tid & 63);
        blk_linv_diag<T>(Q, Di, pl, tid & 63);
    }
    if (tid < 64 - 16 * npan) {  // the padding pivots: Linv's diagonal 1 (the rest of Q is zero), rd 1
        const int c = 16 * npan + tid;
        Q[c * TLD + c] = (T)1;
        rd[c] = (T)1;
    }
    __syncthreads();
    if (w == 0 && (tid & 63) == 0 && !pd) atomicOr(status, ST_NOT_PD);
    if (tdbg && tid == 0) {
        __hip_atomic_fetch_add(&tdbg[17], (unsigned long long)ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&tdbg[18], (unsigned long long)tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&tdbg[19], (unsigned long long)tc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// X[cb][q] (element (row 16w + (lane >> 4) + 4q, column 16cb + (lane & 15)) of
// a 64 x 64 tile) += (NEG ? -1 : 1) * sum_k AT[k][row] * B[k][col], one
// v_mfma_f64_16x16x4 per 16 x 16 block and 4 k: wave w forms rows 16w..16w+15
// (A operand: lane l holds A[l & 15][l >> 4]; B: B[l >> 4][l & 15]). Two LDS
// reads per 4 x 16 x 16 FMAs instead of eight per 16 on the VALU. f32 tiles
// are carried in f64.
// TRI_B: B[k][c] = 0 for k > c (B = Linv^T), so column block cb stops at k = 16cb + 15.
template <typename T, bool NEG, bool TRI_B = false>
__device__ __forceinline__ void mfma_tile(const lds_t<T>* AT, const lds_t<T>* B, T (&X)[4][4], int w, int lane) {
    bsm_d4 c[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int q = 0; q < 4; ++q) c[cb][q] = (double)X[cb][q];
    const int kq = lane >> 4, m = lane & 15;
#pragma unroll
    for (int k4 = 0; k4 < 16; ++k4) {
        const int k = 4 * k4 + kq;
        double a = (double)AT[k * TLD + 16 * w + m];
        if (NEG) a = -a;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
            if (!TRI_B || k4 < 4 * (cb + 1))
                c[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, (double)B[k * TLD + 16 * cb + m], c[cb], 0, 0, 0);
        if ((k4 & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // operand loads of 4 k-steps in flight, not all 16
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int q = 0; q < 4; ++q) X[cb][q] = (T)c[cb][q];
}
