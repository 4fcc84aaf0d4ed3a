// kernels_nd.hip -- solve(order="nd"): x = A^-1 b (src/lib.rs:11-24) by a
// multifrontal Cholesky of P A P^T on the nested-dissection separator tree
// (nd_order.cpp), on gfx950. DESIGN.md §4.9.
//
// Each tree node is a dense front F (f_pad x f_pad, column-major): its own
// np columns (padded to np_pad = 64 * npt with identity pivots), then its m
// front rows st (ancestors' columns), f = np_pad + m, f_pad = 64 * nt. Per
// level of the tree (height), bottom-up:
//   nd_factor  -- partial Cholesky of every front of the level: left-looking
//                 64 x 64 tiles on f64 MFMA, tickets in column order across
//                 the level's fronts, one flag per tile (write-through
//                 hand-offs as in blk_chol). Pivot tiles: L and the inverse
//                 diagonal tiles Dinv; trailing tiles: the update block
//                 U = F22 - L21 L21^T left in place.
//   the extend-add -- U of each child added into its parent's front (the
//                 lower-level child first, then slot 0: a fixed order, so
//                 the bits repeat): by default inside the parent's nd_factor
//                 tiles as they load (the "pull"); BSM_ND_PULL=0 runs
//                 nd_extend2 (or nd_extend per slot) after each level.
// The solves walk the same levels: forward bottom-up (a child's update
// vector into its parent), backward top-down (the ancestors' x gathered).
// Not bit-exact with the reference (another elimination order, FMA); within
// the north star's f64 tolerance (tests/test_gpu_solver_nd.py).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "bsm_internal.hpp"
#include "nd.hpp"

namespace bsm {
namespace {

#include "solve_tiles.hpp"

struct NdDev {
    int64_t foff;      // the front at F + foff
    int64_t dinv_off;  // npt inverse diagonal tiles (Dinv[q * 64 + l] = Linv[l][q])
    int64_t flag_off;  // nt x npt tile flags
    int64_t st_off;    // m front rows (st) and their places in the parent's front (ri)
    int64_t voff;      // f_pad solve-vector entries per right-hand column
    int64_t start;     // own columns [start, start + np)
    int32_t ld, np, np_pad, m, npt, nt, parent, kid0, kid1;
    int32_t tb_off;     // (child) nt + 1 bounds of the parent's tile rows in ri: tb[t] = first a, ri[a] >= 64 t
    int32_t pull_swap;  // (parent) kid1's update block is added before kid0's (kid1 on a lower level)
    int32_t tile_off;   // the front's lower tiles' index base (nd_lower_idx) in the plan's per-tile flags
};

// (I, K), I >= K, among a front's nt (nt + 1) / 2 lower tiles, column by column
__host__ __device__ inline int64_t nd_lower_idx(int32_t nt, int32_t I, int32_t K) {
    return (int64_t)K * nt - (int64_t)K * (K - 1) / 2 + (I - K);
}

__device__ __forceinline__ int32_t lower_bound_i32(const int32_t* a, int32_t len, int64_t x) {
    int32_t lo = 0, hi = len;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// A's lower triangle (j <= i, as band_fill reads it) into the fronts: entry
// (i, j) goes to the front owning column min(pinv i, pinv j)
template <typename T>
__global__ __launch_bounds__(256) void nd_assemble(int64_t n, const int64_t* __restrict__ rp,
                                                   const int32_t* __restrict__ col, const T* __restrict__ val,
                                                   const int32_t* __restrict__ pinv, const int32_t* __restrict__ owner,
                                                   const NdDev* __restrict__ nodes, const int32_t* __restrict__ st,
                                                   T* __restrict__ F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t pi = pinv[i];
    for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
        const int64_t j = col[e];
        if (j > i) continue;
        const int64_t pj = pinv[j];
        const int64_t r = pi > pj ? pi : pj, c = pi > pj ? pj : pi;
        const NdDev& nd = nodes[owner[c]];
        const int64_t lc = c - nd.start;
        const int64_t lr = r < nd.start + nd.np ? r - nd.start : nd.np_pad + lower_bound_i32(st + nd.st_off, nd.m, r);
        F[nd.foff + lc * nd.ld + lr] = val[e];
    }
}

// The tiles A's entries land in (once per plan, from the pattern, with
// nd_assemble's addressing): zf[tile_off + nd_lower_idx] = 1. The others
// start from zero without being zeroed or read (the pulled extend-add: no
// kernel writes them before their factor tile).
__global__ __launch_bounds__(256) void nd_mark_tiles(int64_t n, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ col, const int32_t* __restrict__ pinv,
                                                     const int32_t* __restrict__ owner,
                                                     const NdDev* __restrict__ nodes, const int32_t* __restrict__ st,
                                                     uint8_t* __restrict__ zf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t pi = pinv[i];
    for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
        const int64_t j = col[e];
        if (j > i) continue;
        const int64_t pj = pinv[j];
        const int64_t r = pi > pj ? pi : pj, c = pi > pj ? pj : pi;
        const NdDev& nd = nodes[owner[c]];
        const int64_t lc = c - nd.start;
        const int64_t lr = r < nd.start + nd.np ? r - nd.start : nd.np_pad + lower_bound_i32(st + nd.st_off, nd.m, r);
        zf[nd.tile_off + nd_lower_idx(nd.nt, (int32_t)(lr >> 6), (int32_t)(lc >> 6))] = 1;
    }
}
// the factor's tasks of unmarked tiles: .w |= 2 (a whole-front task keeps its tiles' loads)
__global__ __launch_bounds__(256) void nd_mark_tasks(int64_t ntasks, const NdDev* __restrict__ nodes,
                                                     const uint8_t* __restrict__ zf, int4* __restrict__ tiles) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntasks) return;
    const int4 tl = tiles[t];
    if (tl.w != 0) return;
    const NdDev& nd = nodes[tl.x];
    if (!zf[nd.tile_off + nd_lower_idx(nd.nt, tl.y, tl.z)]) tiles[t].w = 2;
}

// A's entries by tile (once per plan, from the pattern, with nd_assemble's
// addressing): aoff[g] .. aoff[g + 1] are tile g's entries in aent, each
// (CSR index << 12) | (column << 6 | row) within the tile. A counting sort:
// nd_aent_count, nd_scan_tiles, nd_aent_fill (the order within a tile is
// the atomics', but the places are distinct, so the tile they form is not).
__device__ __forceinline__ int64_t nd_aent_key(int64_t i, int64_t j, const int32_t* __restrict__ pinv,
                                               const int32_t* __restrict__ owner, const NdDev* __restrict__ nodes,
                                               const int32_t* __restrict__ st, int32_t* pos) {
    const int64_t pi = pinv[i], pj = pinv[j];
    const int64_t r = pi > pj ? pi : pj, c = pi > pj ? pj : pi;
    const NdDev& nd = nodes[owner[c]];
    const int64_t lc = c - nd.start;
    const int64_t lr = r < nd.start + nd.np ? r - nd.start : nd.np_pad + lower_bound_i32(st + nd.st_off, nd.m, r);
    *pos = (int32_t)((lr & 63) | ((lc & 63) << 6));
    return nd.tile_off + nd_lower_idx(nd.nt, (int32_t)(lr >> 6), (int32_t)(lc >> 6));
}
__global__ __launch_bounds__(256) void nd_aent_count(int64_t n, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ col, const int32_t* __restrict__ pinv,
                                                     const int32_t* __restrict__ owner,
                                                     const NdDev* __restrict__ nodes, const int32_t* __restrict__ st,
                                                     int32_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
        if (col[e] > i) continue;
        int32_t pos;
        atomicAdd(&cnt[nd_aent_key(i, col[e], pinv, owner, nodes, st, &pos)], 1);
    }
}
// cnt[0 .. m) -> its exclusive prefix sums in aoff[0 .. m], one workgroup
__global__ __launch_bounds__(1024) void nd_scan_tiles(int64_t m, const int32_t* __restrict__ cnt,
                                                      int32_t* __restrict__ aoff) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t lo = m * t / 1024, hi = m * (t + 1) / 1024;
    int64_t sum = 0;
    for (int64_t g = lo; g < hi; ++g) sum += cnt[g];
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the chunk sums
        const int64_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int64_t run = part[t] - sum;
    for (int64_t g = lo; g < hi; ++g) {
        aoff[g] = (int32_t)run;
        run += cnt[g];
    }
    if (t == 1023) aoff[m] = (int32_t)part[1023];
}
__global__ __launch_bounds__(256) void nd_aent_fill(int64_t n, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col, const int32_t* __restrict__ pinv,
                                                    const int32_t* __restrict__ owner, const NdDev* __restrict__ nodes,
                                                    const int32_t* __restrict__ st, const int32_t* __restrict__ aoff,
                                                    int32_t* __restrict__ cur, int64_t* __restrict__ aent) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
        if (col[e] > i) continue;
        int32_t pos;
        const int64_t g = nd_aent_key(i, col[e], pinv, owner, nodes, st, &pos);
        const int32_t slot = atomicAdd(&cur[g], 1);
        aent[aoff[g] + slot] = (e << 12) | pos;
    }
}
// per factor task (not a whole front): its tile's entry range (offset, count)
__global__ __launch_bounds__(256) void nd_task_ranges(int64_t ntasks, const int4* __restrict__ tiles,
                                                      const NdDev* __restrict__ nodes, const int32_t* __restrict__ aoff,
                                                      int2* __restrict__ tq) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntasks) return;
    const int4 tl = tiles[t];
    if (tl.w == 1) {
        tq[t] = make_int2(0, 0);
        return;
    }
    const NdDev& nd = nodes[tl.x];
    const int64_t g = nd.tile_off + nd_lower_idx(nd.nt, tl.y, tl.z);
    tq[t] = make_int2(aoff[g], aoff[g + 1] - aoff[g]);
}
// per factor task (not a whole front): its children's blocks, first and
// second in nd_extend2's order (NdPull::ra = 0: none), so the tile reads
// them with its task instead of through node -> child -> bounds
struct NdPull {
    int64_t uoff;   // the child's update block U at F + uoff (U[a][b] at uoff + b ld + a)
    int64_t uvoff;  // its update vector at V + uvoff (the folded forward solve)
    int32_t rcoff, ld, a0, ra, b0, rbn;
};
__global__ __launch_bounds__(256) void nd_task_pull(int64_t ntasks, const int4* __restrict__ tiles,
                                                    const NdDev* __restrict__ nodes, const int32_t* __restrict__ tb,
                                                    NdPull* __restrict__ pd) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntasks) return;
    const int4 tl = tiles[t];
    const NdDev& nd = nodes[tl.x];
    for (int h = 0; h < 2; ++h) {
        NdPull o{0, 0, 0, 0, 0, 0, 0, 0};
        const int c = h == nd.pull_swap ? nd.kid0 : nd.kid1;
        if (c >= 0 && tl.w != 1) {
            const NdDev& cd = nodes[c];
            const int32_t* const tbc = tb + cd.tb_off;
            o.uoff = cd.foff + (int64_t)cd.np_pad * cd.ld + cd.np_pad;
            o.uvoff = cd.voff + cd.np_pad;
            o.rcoff = (int32_t)cd.st_off;
            o.ld = cd.ld;
            o.a0 = tbc[tl.y];
            o.ra = tbc[tl.y + 1] - o.a0;
            o.b0 = tbc[tl.z];
            o.rbn = tbc[tl.z + 1] - o.b0;
            if (o.rbn <= 0) o.ra = 0;
        }
        pd[2 * t + h] = o;
    }
}

// per solve: the entries' values in tile order (a contiguous read per tile)
template <typename T>
__global__ __launch_bounds__(256) void nd_aent_vals(int64_t na, const int64_t* __restrict__ aent,
                                                    const T* __restrict__ val, T* __restrict__ av) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < na) av[q] = val[aent[q] >> 12];
}

// zero the fronts' lower tiles (the only ones any kernel reads: every tile
// of the factor's lists): 55 % of the bytes a memset of the whole squares
// writes; with zf, only the tiles A's entries land in (nd_mark_tiles)
template <typename T>
__global__ __launch_bounds__(256) void nd_zero_tiles(const NdDev* __restrict__ nodes, const int4* __restrict__ tiles,
                                                     T* __restrict__ F, const uint8_t* __restrict__ zf) {
    const int4 tl = tiles[blockIdx.x];
    const NdDev& nd = nodes[tl.x];
    if (zf && !zf[nd.tile_off + nd_lower_idx(nd.nt, tl.y, tl.z)]) return;
    T* const t0 = F + nd.foff + (int64_t)64 * tl.z * nd.ld + 64 * tl.y;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int e = threadIdx.x + 256 * u;
        t0[(int64_t)(e >> 6) * nd.ld + (e & 63)] = (T)0;
    }
}

// identity on the padding pivots [np, np_pad) of every front
template <typename T>
__global__ __launch_bounds__(64) void nd_pad_pivots(const NdDev* __restrict__ nodes, T* __restrict__ F) {
    const NdDev& nd = nodes[blockIdx.x];
    for (int d = nd.np + (int)threadIdx.x; d < nd.np_pad; d += 64) F[nd.foff + (int64_t)d * nd.ld + d] = (T)1;
}

// Partial Cholesky of the fronts of one level. tiles[t] = (node, I, K, 0):
// column-major order across the level's fronts (K; the diagonal tiles of all
// fronts, then the tiles below them), so a tile only waits on tiles of
// earlier tickets. Tile (I, K), I >= K:
//     S = F_IK - sum_{J < min(K, npt)} L_IJ L_KJ^T
//     K < npt, I == K: L_KK = chol(S), Dinv_K = L_KK^-1   (flag)
//     K < npt, I >  K: L_IK = S L_KK^-T                    (flag)
//     K >= npt       : U_IK = S (the update block, for nd_extend)
// tiles[t] = (node, 0, 0, 1): the whole front of a small node (a few tiles:
// most of the leaf level) on this workgroup, its tiles in column order one
// after the other. Its flags are its own (a tile's waits find them set), so
// it waits on nobody: these tasks follow the tiled fronts' tickets and fill
// the CUs while those fronts' chains run, without a ticket and a flag
// hand-off through L2 per tile.
// fV (the forward solve folded in, one right-hand side; BSM_ND_FOLD): the
// diagonal tile (I, I) also forms w_I = b_I + the children's update-vector
// entries landing in its rows - sum_{J < min(I, npt)} L_IJ y_J (the L_IJ are
// the tiles its products stage anyway; y_J is published before the flags
// its waits follow), then y_I = Linv_I w_I for a pivot tile or the update
// vector u_I = w_I for a front-row tile, into fV (V's layout: the separate
// forward's output), so no forward pass reads L again.
// STAMPS (BSM_ND_STAMPS=1, a diagnostic instantiation: the counters cost
// SGPRs the product build cannot spare): per workgroup,
// thread 0's shader-clock cycles in the flag waits, the products (loads,
// LDS staging, MFMA), the diagonal factors, the sub-diagonal solves, the
// update tiles' stores and the drains, and the tile counts of each kind,
// added into stamps[0..11] at the end
constexpr int ND_NSTAMP = 18;  // per level: BSM_ND_STAMPS's counters
template <typename T, bool STAMPS = false>
__global__ __launch_bounds__(256, 2) void nd_factor(const NdDev* __restrict__ nodes, const int4* __restrict__ tiles,
                                                 int64_t ntiles, T* __restrict__ F, T* __restrict__ Dinv,
                                                 int* __restrict__ flags, int* __restrict__ ticket,
                                                 int* __restrict__ status, int pad_skip,
                                                 const int32_t* __restrict__ tb, const int32_t* __restrict__ ri,
                                                 int zskip, T* __restrict__ fV, const T* __restrict__ fbp,
                                                 const int64_t* __restrict__ aent, const T* __restrict__ av,
                                                 const int32_t* __restrict__ aoff, const int2* __restrict__ tq,
                                                 const NdPull* __restrict__ pdesc,
                                                 unsigned long long* __restrict__ stamps = nullptr) {
    long long c_wait = 0, c_prod = 0, c_diag = 0, c_trsm = 0, c_upd = 0, c_drain = 0;
    long long n_prod = 0, n_diag = 0, n_trsm = 0, n_upd = 0, c_total = 0, n_tiles = 0;
    long long c_pl[4] = {0, 0, 0, 0}, n_pull = 0;  // the pull's phases: tile + first child's loads, its adds, second, read-back
    const long long c_start = STAMPS ? (long long)clock64() : 0;
    __shared__ T PT[64][TLD];
    __shared__ T QT[64][TLD];
    __shared__ T rd[64];
    __shared__ T Di[4 * 256];
    __shared__ T Tb[3 * 256];
    __shared__ int pcs[2][64];  // the pull: a child block's columns' places in the tile
    __shared__ T fw[64], fyk[64], fpart[4][64];  // the folded forward solve (fV): w, y_J, partial sums
    __shared__ int tk;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rb = 16 * w + (lane >> 4), cm = lane & 15;
    lds_t<T>* const PTl = (lds_t<T>*)&PT[0][0];
    lds_t<T>* const QTl = (lds_t<T>*)&QT[0][0];
    // the poll has no break (the structurizer's hazard in nd_backward_tiles)
    auto wait_flag = [&](const int* f) {
        long long spins = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && spins <= SPIN_LIMIT) {
            __builtin_amdgcn_s_sleep(1);
            ++spins;
        }
        if (spins > SPIN_LIMIT && lane == 0) atomicOr(status, ST_TIMEOUT);
    };
    // the ticket at the END of each task and counted inner loops (the
    // control-flow shape of nd_backward_tiles)
    if (tid == 0) tk = atomicAdd(ticket, 1);
    __syncthreads();
    int64_t t = __builtin_amdgcn_readfirstlane(tk);
    while (t < ntiles) {
      const int4 tl = tiles[t];
      const NdDev& nd = nodes[tl.x];
      const bool whole = tl.w == 1;
      // zskip: a tile no A entry lands in starts from zero (tl.w == 2,
      // nd_mark_tasks): it was neither zeroed nor written, and is not read
      const bool fz = zskip && tl.w == 2;
      const int npt = nd.npt, ntf = nd.nt;
      const int cnt = whole ? ntf * (ntf + 1) / 2 : 1;
      int I = whole ? 0 : tl.y, K = whole ? 0 : tl.z;
      for (int jt = 0; jt < cnt; ++jt) {
        const int64_t ld = nd.ld;
        T* const Fn = F + nd.foff;
        int* const fl = flags + nd.flag_off;
        // tile (I2, J) of L into registers (sc1: other workgroups wrote it),
        // then X[t][r] = L[64 I2 + r][64 J + t] in LDS
        auto load = [&](T (&v)[16], int I2, int J) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = tid + 256 * u, r = e & 63, c = e >> 6;
                v[u] = ld_sc1(&Fn[(int64_t)(64 * J + c) * ld + 64 * I2 + r]);
            }
        };
        auto store = [&](T (*X)[TLD], const T (&v)[16]) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = tid + 256 * u;
                X[e >> 6][e & 63] = v[u];
            }
        };
        long long c0 = STAMPS ? (long long)clock64() : 0;
        T acc[4][4];
        // the folded forward solve on this diagonal tile: w = b (pivot rows)
        const bool fold = fV && I == K;
        if (fold && tid < 64) fw[tid] = 64 * K + tid < nd.np ? fbp[nd.start + 64 * K + tid] : (T)0;
        const bool kids = tb && (nd.kid0 >= 0 || nd.kid1 >= 0);
        if (kids || aent) {
            // aent: the tile starts from A's entries in it (and the padding
            // pivots' identity), staged in LDS from the plan's per-tile lists,
            // instead of from F (no zeroing, no assembly, no read of F): the
            // same values, written the same way.
            // The children's update blocks, pulled into this tile (tb: no
            // nd_extend launches): the entries (a, b), a >= b, of child c
            // with ri[a] in tile row I and ri[b] in tile column K, i.e. a in
            // [tb[I], tb[I + 1]), b in [tb[K], tb[K + 1]) (ri ascending).
            // The tile goes to LDS by coalesced columns; thread (lane, wave)
            // takes the child's a = a0 + lane and b = b0 + 4 u + w, its
            // row's place one load per lane and the columns' places through
            // LDS (pcs). Every load is unconditional (indices clamped to
            // the block, so they all go out together), and each child's 16
            // additions read their LDS elements first and then write them
            // (the block's places are distinct). The children's entries are
            // added in the order nd_extend2 adds them (the lower level first,
            // then slot 0): F + U_first + U_second, the same roundings, the
            // same bits.
            struct Blk {
                const T* U;
                const int32_t* rc;
                const T* u;  // the child's update vector (fold)
                int ld, a0, ra, b0, rbn;
            } bk[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                bk[h].ra = 0;
                if (!kids) continue;
                if (pdesc && !whole) {  // the task's own descriptors (nd_task_pull)
                    const NdPull& o = pdesc[2 * t + h];
                    bk[h].U = F + o.uoff;
                    bk[h].rc = ri + o.rcoff;
                    bk[h].u = fV ? fV + o.uvoff : nullptr;
                    bk[h].ld = o.ld;
                    bk[h].a0 = o.a0;
                    bk[h].ra = o.ra;
                    bk[h].b0 = o.b0;
                    bk[h].rbn = o.rbn;
                    continue;
                }
                const int c = h == nd.pull_swap ? nd.kid0 : nd.kid1;
                if (c < 0) continue;
                const NdDev& cd = nodes[c];
                const int32_t* const tbc = tb + cd.tb_off;
                bk[h].U = F + cd.foff + (int64_t)cd.np_pad * cd.ld + cd.np_pad;  // U[a][b] at U[b ld + a]
                bk[h].rc = ri + cd.st_off;
                bk[h].u = fV ? fV + cd.voff + cd.np_pad : nullptr;
                bk[h].ld = cd.ld;
                bk[h].a0 = tbc[I];
                bk[h].ra = tbc[I + 1] - bk[h].a0;
                bk[h].b0 = tbc[K];
                bk[h].rbn = tbc[K + 1] - bk[h].b0;
                if (bk[h].rbn <= 0) bk[h].ra = 0;
            }
            T v[16];
            int pr[2] = {0, 0};
            // the rows' places (per lane) and the columns' (into pcs, read
            // back wave-uniform) of both children
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (bk[h].ra > 0) {
                    pr[h] = bk[h].rc[bk[h].a0 + min(lane, bk[h].ra - 1)] - 64 * I;
                    if (tid < 64) pcs[h][tid] = bk[h].rc[bk[h].b0 + min(tid, bk[h].rbn - 1)] - 64 * K;
                }
            T uv = (T)0;
            auto issue = [&](const Blk& k) {
                const int a = k.a0 + min(lane, k.ra - 1);
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = k.U[(int64_t)(k.b0 + min(4 * u + w, k.rbn - 1)) * k.ld + a];
                if (fold && w == 0) uv = k.u[a];
            };
            auto add = [&](const Blk& k, int h) {
                T cur[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) cur[u] = PT[pr[h]][pcs[h][4 * u + w]];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int bl = 4 * u + w;
                    if (lane < k.ra && bl < k.rbn && k.a0 + lane >= k.b0 + bl) PT[pr[h]][pcs[h][bl]] = cur[u] + v[u];
                }
                if (fold && w == 0 && lane < k.ra) fw[pr[h]] += uv;
            };
            if (aent) {
                int2 rq;
                if (whole) {
                    const int64_t g = nd.tile_off + nd_lower_idx(ntf, I, K);
                    rq = make_int2(aoff[g], aoff[g + 1] - aoff[g]);
                } else {
                    rq = tq[t];
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) PT[lane][4 * u + w] = (T)0;
                __syncthreads();
                for (int q = tid; q < rq.y; q += 256) {
                    const int64_t x = aent[rq.x + q];
                    PT[x & 63][(x >> 6) & 63] = av[rq.x + q];
                }
                if (I == K && K < npt && tid < 64 && 64 * K + tid >= nd.np) PT[tid][tid] = (T)1;
            } else {
                T fv[16];  // the tile by columns: element (lane, 4 u + w)
#pragma unroll
                for (int u = 0; u < 16; ++u) fv[u] = (T)0;
                if (!fz)
#pragma unroll
                    for (int u = 0; u < 16; ++u) fv[u] = Fn[(int64_t)(64 * K + 4 * u + w) * ld + 64 * I + lane];
#pragma unroll
                for (int u = 0; u < 16; ++u) PT[lane][4 * u + w] = fv[u];
            }
            if (bk[0].ra > 0) issue(bk[0]);
            long long ps = 0;
            auto pstamp = [&](int i) {
                if (STAMPS) {
                    const long long c = (long long)clock64();
                    c_pl[i] += c - ps;
                    ps = c;
                }
            };
            if (STAMPS) ps = c0, ++n_pull;
            __syncthreads();  // the staged tile
            pstamp(0);
            if (bk[0].ra > 0) add(bk[0], 0);
            pstamp(1);
            if (bk[1].ra > 0) {
                issue(bk[1]);
                __syncthreads();  // the first child's additions
                add(bk[1], 1);
            }
            pstamp(2);
            __syncthreads();
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[cb][q] = PT[rb + 4 * q][16 * cb + cm];
            __syncthreads();  // PT is the products' staging next
            pstamp(3);
        } else if (fz) {
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[cb][q] = (T)0;
        } else {
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[cb][q] = Fn[(int64_t)(64 * K + 16 * cb + cm) * ld + 64 * I + rb + 4 * q];
        }
        // left-looking products (two workgroups per CU: __launch_bounds__
        // (256, 2) keeps the VGPRs at 128; at 136 the occupancy query gave one
        // and the C5 factor took 8.5 instead of 5.7 ms)
        const int Jn = K < npt ? K : npt;
        T fp = (T)0;  // fold: this thread's share of (L_IJ y_J)[lane], terms 16 w .. 16 w + 15
        for (int J = 0; J < Jn; ++J) {
            const long long cw = STAMPS ? (long long)clock64() : 0;
            wait_flag(&fl[I * npt + J]);
            if (I != K) wait_flag(&fl[K * npt + J]);
            if (STAMPS) c_wait += (long long)clock64() - cw;
            T va[16];
            load(va, I, J);
            if (fold && tid < 64) fyk[tid] = ld_sc1(&fV[nd.voff + 64 * J + tid]);  // y_J (before (J, J)'s flag)
            store(PT, va);
            if (I != K) {
                load(va, K, J);
                store(QT, va);
            }
            __syncthreads();
            mfma_tile<T, true>(PTl, I != K ? QTl : PTl, acc, w, lane);
            if (fold) {
#pragma unroll
                for (int t = 0; t < 16; ++t) fp = fma_t((T)PT[16 * w + t][lane], fyk[16 * w + t], fp);  // PT[t][r] = L[r][t]
            }
            __syncthreads();
        }
        if (fold) {  // w_I = b + children's entries - sum_J L_IJ y_J
            fpart[w][lane] = fp;
            __syncthreads();
            if (tid < 64) fw[tid] = fw[tid] - ((fpart[0][tid] + fpart[1][tid]) + (fpart[2][tid] + fpart[3][tid]));
            __syncthreads();
        }
        if (STAMPS) {
            const long long c1 = (long long)clock64();
            c_prod += c1 - c0;
            n_prod += Jn;
            c0 = c1;
        }
        if (K < npt && I == K) {
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) PT[rb + 4 * q][16 * cb + cm] = acc[cb][q];
            __syncthreads();
            // the panels holding real pivots (the front's last pivot tile may
            // end in identity padding: blk_diag_panels skips those panels)
            const int rem = nd.np - 64 * K;
            blk_diag_panels<T>(PTl, QTl, (lds_t<T>*)Di, (lds_t<T>*)Tb, (lds_t<T>*)rd, status, tid, nullptr, nullptr,
                               nullptr, nullptr, rem >= 64 || !pad_skip ? 4 : (rem + 15) / 16);
            __syncthreads();
            T* const dk = Dinv + nd.dinv_off + (int64_t)K * 4096;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = tid + 256 * u, q = e >> 6, l = e & 63;
                st_sc1(&dk[e], (T)QT[q][l]);  // Dinv[q * 64 + l] = Linv[l][q]
                const int r = e & 63, c = e >> 6;
                Fn[(int64_t)(64 * K + c) * ld + 64 * K + r] = r >= c ? (T)PT[r][c] : (T)0;
            }
            if (fold) {  // y_K = Linv_K w_K (QT[q][l] = Linv[l][q]), published with the tile's flag
                T y = (T)0;
#pragma unroll
                for (int j = 0; j < 16; ++j) y = fma_t((T)QT[16 * w + j][lane], fw[16 * w + j], y);
                fpart[w][lane] = y;
                __syncthreads();
                if (tid < 64)
                    st_sc1(&fV[nd.voff + 64 * K + tid], (fpart[0][tid] + fpart[1][tid]) + (fpart[2][tid] + fpart[3][tid]));
            }
        } else if (K < npt) {
            wait_flag(&fl[K * npt + K]);
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) PT[16 * cb + cm][rb + 4 * q] = acc[cb][q];  // S^T
            const T* const dk = Dinv + nd.dinv_off + (int64_t)K * 4096;
            T v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = ld_sc1(&dk[tid + 256 * u]);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = tid + 256 * u;
                QT[e >> 6][e & 63] = v[u];  // QT[s][c] = Linv[c][s]
            }
            __syncthreads();
            T o[4][4] = {};
            mfma_tile<T, false, true>(PTl, QTl, o, w, lane);
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_sc1(&Fn[(int64_t)(64 * K + 16 * cb + cm) * ld + 64 * I + rb + 4 * q], o[cb][q]);
        } else {
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) Fn[(int64_t)(64 * K + 16 * cb + cm) * ld + 64 * I + rb + 4 * q] = acc[cb][q];
            if (fold && tid < 64) st_sc1(&fV[nd.voff + 64 * K + tid], (T)fw[tid]);  // the update vector u_K
        }
        long long c2 = 0;
        if (STAMPS) {
            c2 = (long long)clock64();
            if (K < npt && I == K) c_diag += c2 - c0, ++n_diag;
            else if (K < npt) c_trsm += c2 - c0, ++n_trsm;
            else c_upd += c2 - c0, ++n_upd;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (K < npt && tid == 0) __hip_atomic_store(&fl[I * npt + K], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (STAMPS) c_drain += (long long)clock64() - c2, ++n_tiles;
        if (++I == ntf) {  // a whole front: the next tile in column order
            ++K;
            I = K;
        }
      }
      __syncthreads();
      if (tid == 0) tk = atomicAdd(ticket, 1);
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane(tk);
    }
    if (STAMPS && tid == 0) {
        c_total = (long long)clock64() - c_start;
        const long long v[ND_NSTAMP] = {c_total, c_wait, c_prod,  c_diag,  c_trsm,  c_upd,  c_drain, n_tiles,
                                        n_prod,  n_diag, n_trsm,  n_upd,   c_pl[0], c_pl[1], c_pl[2], c_pl[3],
                                        n_pull,  0};
        for (int i = 0; i < ND_NSTAMP; ++i) atomicAdd(&stamps[i], (unsigned long long)v[i]);
    }
}

// U of a child into its parent's front: task (child, b) adds column b of the
// child's update block, rows a >= b, at (ri[a], ri[b]). One wave per task.
template <typename T>
__global__ __launch_bounds__(256) void nd_extend(const NdDev* __restrict__ nodes, const int2* __restrict__ tasks,
                                                 int64_t ntasks, const int32_t* __restrict__ ri, T* __restrict__ F) {
    const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (task >= ntasks) return;
    const int lane = threadIdx.x & 63;
    const int2 tk = tasks[task];
    const NdDev& c = nodes[tk.x];
    const NdDev& p = nodes[c.parent];
    const int32_t* rc = ri + c.st_off;
    const int b = tk.y;
    const T* src = F + c.foff + (int64_t)(c.np_pad + b) * c.ld + c.np_pad;
    T* dst = F + p.foff + (int64_t)rc[b] * p.ld;
    for (int a = b + lane; a < c.m; a += 64) dst[rc[a]] += src[a];
}

// Both children of a parent in one launch: task (c0, b0, c1, b1) adds column
// b0 of child c0's update block, then column b1 of child c1's, into the SAME
// parent column (ri[b0] of c0 == ri[b1] of c1; -1: that child has none), in
// that order, on one wave: the same sums in the same order as a slot-0 launch
// followed by a slot-1 launch, and the tasks of a launch own distinct parent
// columns. The second child's loads are write-through (the first child's
// stores came from other lanes of this wave) after the wave's stores drain.
template <typename T>
__global__ __launch_bounds__(256) void nd_extend2(const NdDev* __restrict__ nodes, const int4* __restrict__ tasks,
                                                  int64_t ntasks, const int32_t* __restrict__ ri, T* __restrict__ F) {
    const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (task >= ntasks) return;
    const int lane = threadIdx.x & 63;
    const int4 tk = tasks[task];
    auto add = [&](int ci, int b, bool coherent) {
        const NdDev& c = nodes[ci];
        const NdDev& p = nodes[c.parent];
        const int32_t* rc = ri + c.st_off;
        const T* src = F + c.foff + (int64_t)(c.np_pad + b) * c.ld + c.np_pad;
        T* dst = F + p.foff + (int64_t)rc[b] * p.ld;
        for (int a = b + lane; a < c.m; a += 64) {
            T* d = dst + rc[a];
            *d = (coherent ? ld_sc1(d) : *d) + src[a];
        }
    };
    if (tk.x >= 0) add(tk.x, tk.y, false);
    if (tk.z >= 0) {
        if (tk.x >= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        add(tk.z, tk.w, tk.x >= 0);
    }
}

// right-hand sides into the new order: bp[col * n + q] = b[perm[q] * k + col] (b row-major n x k)
template <typename T>
__global__ __launch_bounds__(256) void nd_gather(int64_t n, int64_t k, const int64_t* __restrict__ perm,
                                                 const T* __restrict__ b, T* __restrict__ bp) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const int64_t o = perm[q];
    for (int64_t c = 0; c < k; ++c) bp[c * n + q] = b[o * k + c];
}
template <typename T>
__global__ __launch_bounds__(256) void nd_scatter(int64_t n, int64_t k, const int64_t* __restrict__ perm,
                                                  const T* __restrict__ xp, T* __restrict__ x) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const int64_t o = perm[q];
    for (int64_t c = 0; c < k; ++c) x[o * k + c] = xp[c * n + q];
}

// Forward solve of one level, one workgroup per (node, column): v = the
// node's pivots of bp plus its children's update vectors; per pivot tile K
// y_K = Dinv_K v_K, then v_I -= L_IK y_K below. v (at V + voff) ends as y
// over the pivots and the update vector u over the front rows. V is read and
// written write-through (rows change hands between threads). Every product's
// loads are issued together (unrolled): a loop of load, wait, FMA is one
// L2 round trip per term, 64 per tile step.
template <typename T>
__global__ __launch_bounds__(256, 4) void nd_forward(const NdDev* __restrict__ nodes, const int32_t* __restrict__ lvl,
                                                  int64_t n, const T* __restrict__ bp, T* __restrict__ V, int64_t vtot,
                                                  const T* __restrict__ F, const T* __restrict__ Dinv,
                                                  const int32_t* __restrict__ ri) {
    __shared__ T vk[64], yk[64];
    __shared__ T part[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const NdDev& nd = nodes[lvl[blockIdx.x]];
    const int64_t col = blockIdx.y;
    T* const v = V + col * vtot + nd.voff;
    const int fp = 64 * nd.nt;
    for (int r = tid; r < fp; r += 256) st_sc1(&v[r], r < nd.np ? bp[col * n + nd.start + r] : (T)0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int kid = s == 0 ? nd.kid0 : nd.kid1;
        if (kid < 0) continue;
        const NdDev& c = nodes[kid];
        const T* u = V + col * vtot + c.voff + c.np_pad;
        const int32_t* rc = ri + c.st_off;
        for (int a = tid; a < c.m; a += 256) {
            T* d = &v[rc[a]];
            st_sc1(d, ld_sc1(d) + u[a]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const T* const Fn = F + nd.foff;
    const int64_t ld = nd.ld;
    for (int K = 0; K < nd.npt; ++K) {
        if (tid < 64) vk[tid] = ld_sc1(&v[64 * K + tid]);
        __syncthreads();
        {  // y_K = Dinv_K v_K: wave wv sums terms q in [16 wv, 16 wv + 16)
            const T* g = Dinv + nd.dinv_off + (int64_t)K * 4096 + 16 * wv * 64 + lane;
            T gv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) gv[j] = g[j * 64];
            T y0 = (T)0, y1 = (T)0;
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                y0 = fma_t(gv[j], vk[16 * wv + j], y0);
                y1 = fma_t(gv[j + 1], vk[16 * wv + j + 1], y1);
            }
            part[wv][lane] = y0 + y1;
        }
        __syncthreads();
        if (tid < 64) {
            const T y = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
            yk[tid] = y;
            st_sc1(&v[64 * K + tid], y);
        }
        __syncthreads();
        // rows past f and the pivot padding rows are zero in L (and stay
        // zero in v): skipped whole (the loads inside stay unconditional, so
        // they go out together)
        const int f = nd.np_pad + nd.m;
        for (int r = 64 * (K + 1) + tid; r < f; r += 256) {
            if (r >= nd.np && r < nd.np_pad) continue;
            // the row's 64 terms in two halves of 32 loads in flight: at 226
            // VGPRs (all 64 at once) two workgroups fit a CU, at <= 128 four
            // (the leaf level is latency bound: 7,699 fronts at C5); same
            // accumulators, same order, same bits
            const T* lc = Fn + (int64_t)64 * K * ld + r;
            const T vr = ld_sc1(&v[r]);
            T s0 = (T)0, s1 = (T)0, s2 = (T)0, s3 = (T)0;
#pragma unroll
            for (int h = 0; h < 64; h += 32) {
                T lv[32];
#pragma unroll
                for (int t = 0; t < 32; ++t) lv[t] = lc[(int64_t)(h + t) * ld];
#pragma unroll
                for (int t = 0; t < 32; t += 4) {
                    s0 = fma_t(lv[t], yk[h + t], s0);
                    s1 = fma_t(lv[t + 1], yk[h + t + 1], s1);
                    s2 = fma_t(lv[t + 2], yk[h + t + 2], s2);
                    s3 = fma_t(lv[t + 3], yk[h + t + 3], s3);
                }
            }
            st_sc1(&v[r], vr - ((s0 + s1) + (s2 + s3)));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// A solve wave waits on a pivot tile of its own front that a running wave
// publishes within microseconds: ~1 s of polls is a hang (reported as
// ST_TIMEOUT, not spun on for the factor's ~30 s)
constexpr long long ND_SOLVE_SPIN_LIMIT = 1ll << 20;

// Forward solve of one level by tile rows: one wave per (node, tile row I,
// column), taken by ticket in I-major order across the level's fronts (a
// wave only waits on lower tickets, which are running or done). The wave
// forms its 64 rows' v (the pivots of bp, then child 0's and child 1's
// update entries landing in these rows), subtracts L_IK y_K for K < min(I,
// npt) as each y_K is published (flag per node, column and pivot tile), and,
// for a pivot tile, forms y_I = Dinv_I v_I and publishes it. Per row the
// same operations in the same order as nd_forward (one thread per row, the
// 64-term products in four accumulators; y from four 16-term partials):
// the same bits, with the fronts' chains of pivot tiles running on as many
// waves as the front has tile rows instead of one workgroup
// (BSM_ND_FWD_TILES=0: nd_forward, for the A/B).
template <typename T>
__global__ __launch_bounds__(64) void nd_forward_tiles(const NdDev* __restrict__ nodes, const int2* __restrict__ tasks,
                                                       int64_t ntasks, int k, int64_t n, const T* __restrict__ bp,
                                                       T* __restrict__ V, int64_t vtot, const T* __restrict__ F,
                                                       const T* __restrict__ Dinv, const int32_t* __restrict__ ri,
                                                       int* __restrict__ yflags, int* __restrict__ ticket,
                                                       int* __restrict__ status) {
    __shared__ T yk[64];
    __shared__ T add[2][64];
    __shared__ int hit[2][64];
    __shared__ int tk;
    const int lane = threadIdx.x;
    const int64_t total = ntasks * k;
    // The control-flow shape of nd_backward_tiles (whose first form, with the
    // ticket at the loop head, compiled to a loop that never took a new
    // ticket): the ticket is taken at the END of each task, the flag poll has
    // no break, and no barrier sits inside a branch.
    if (lane == 0) tk = atomicAdd(ticket, 1);
    __syncthreads();
    int64_t t = __builtin_amdgcn_readfirstlane(tk);
    while (t < total) {
        const int2 task = tasks[t / k];
        const int col = (int)(t % k);
        const NdDev& nd = nodes[task.x];
        const int I = task.y;
        T* const v = V + (int64_t)col * vtot + nd.voff;
        int* const yf = yflags + (nd.dinv_off / 4096) * k + (int64_t)col * nd.npt;
        const int r = 64 * I + lane;
        T val = r < nd.np ? bp[(int64_t)col * n + nd.start + r] : (T)0;
        // the children's update entries in rows [64 I, 64 I + 64): ri is
        // ascending, so they are one range of each child's entries
        hit[0][lane] = 0;
        hit[1][lane] = 0;
        __syncthreads();
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
            const int kid = sl == 0 ? nd.kid0 : nd.kid1;
            if (kid >= 0) {
                const NdDev& c = nodes[kid];
                const int32_t* rc = ri + c.st_off;
                const int32_t lo = lower_bound_i32(rc, c.m, 64 * I), hi = lower_bound_i32(rc, c.m, 64 * I + 64);
                const T* u = V + (int64_t)col * vtot + c.voff + c.np_pad;
                for (int32_t a = lo + lane; a < hi; a += 64) {
                    add[sl][rc[a] - 64 * I] = u[a];
                    hit[sl][rc[a] - 64 * I] = 1;
                }
            }
        }
        __syncthreads();
        if (nd.kid0 >= 0 && hit[0][lane]) val = val + add[0][lane];
        if (nd.kid1 >= 0 && hit[1][lane]) val = val + add[1][lane];
        const T* const lrow = F + nd.foff + r;
        const int64_t ld = nd.ld;
        const int Kn = I < nd.npt ? I : nd.npt;
        for (int K = 0; K < Kn; ++K) {
            if (lane == 0) {
                long long spins = 0;
                while (__hip_atomic_load(&yf[K], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                       spins < ND_SOLVE_SPIN_LIMIT) {
                    __builtin_amdgcn_s_sleep(1);
                    ++spins;
                }
                if (spins >= ND_SOLVE_SPIN_LIMIT) atomicOr(status, ST_TIMEOUT);
            }
            __syncthreads();
            T lv[64];
#pragma unroll
            for (int q = 0; q < 64; ++q) lv[q] = lrow[(int64_t)(64 * K + q) * ld];
            yk[lane] = ld_sc1(&v[64 * K + lane]);
            __syncthreads();
            T s0 = (T)0, s1 = (T)0, s2 = (T)0, s3 = (T)0;
#pragma unroll
            for (int q = 0; q < 64; q += 4) {
                s0 = fma_t(lv[q], yk[q], s0);
                s1 = fma_t(lv[q + 1], yk[q + 1], s1);
                s2 = fma_t(lv[q + 2], yk[q + 2], s2);
                s3 = fma_t(lv[q + 3], yk[q + 3], s3);
            }
            val = val - ((s0 + s1) + (s2 + s3));
            __syncthreads();
        }
        // a pivot tile: y_I = Dinv_I v_I, as nd_forward's four 16-term partials
        const bool pivot = I < nd.npt;
        yk[lane] = val;
        __syncthreads();
        T out = val;
        if (pivot) {
            const T* g = Dinv + nd.dinv_off + (int64_t)I * 4096 + lane;
            T part[4];
#pragma unroll
            for (int wv = 0; wv < 4; ++wv) {
                T gv[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) gv[j] = g[(16 * wv + j) * 64];
                T y0 = (T)0, y1 = (T)0;
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    y0 = fma_t(gv[j], yk[16 * wv + j], y0);
                    y1 = fma_t(gv[j + 1], yk[16 * wv + j + 1], y1);
                }
                part[wv] = y0 + y1;
            }
            out = (part[0] + part[1]) + (part[2] + part[3]);
        }
        st_sc1(&v[r], out);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (lane == 0) {
            if (pivot) __hip_atomic_store(&yf[I], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tk = atomicAdd(ticket, 1);
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(tk);
    }
}

// Backward solve of one level, one workgroup per (node, column): w = y over
// the pivots, the ancestors' x over the front rows; per pivot tile K from the
// last, x_K = Dinv_K^T (y_K - L_{>K,K}^T w_{>K}); the pivots' x to xp.
template <typename T>
__global__ __launch_bounds__(256) void nd_backward(const NdDev* __restrict__ nodes, const int32_t* __restrict__ lvl,
                                                   int64_t n, T* __restrict__ xp, T* __restrict__ V, int64_t vtot,
                                                   const T* __restrict__ F, const T* __restrict__ Dinv,
                                                   const int32_t* __restrict__ st) {
    __shared__ T red[64][65];
    __shared__ T zk[64];
    __shared__ T part[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const NdDev& nd = nodes[lvl[blockIdx.x]];
    const int64_t col = blockIdx.y;
    T* const w = V + col * vtot + nd.voff;
    const int fp = 64 * nd.nt;
    for (int a = tid; a < nd.m; a += 256) st_sc1(&w[nd.np_pad + a], xp[col * n + st[nd.st_off + a]]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const T* const Fn = F + nd.foff;
    const int64_t ld = nd.ld;
    for (int K = nd.npt - 1; K >= 0; --K) {
        // column sums below the tile: wave wv takes columns 16 wv .. 16 wv + 15,
        // lanes the rows, two rows per lane in flight
        T acc[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) acc[c] = (T)0;
        // rows by tile from the LAST tile down to K + 1 (the front rows, known
        // from the start, first: nd_backward_tiles sums in this order while
        // the pivot tiles' x arrive)
        const T* lc = Fn + (int64_t)(64 * K + 16 * wv) * ld;
        const int rlo = 64 * (K + 1);
        // a zero row of L (past f, or a pivot padding row) has w = 0 exactly:
        // its loads go to a real row's address instead (the same cache lines
        // for every such lane, so no HBM bytes), unconditionally (they still
        // go out together), and the term stays 0 (an accumulator that starts
        // at +0 never becomes -0): the same sums, the same bits
        const int f = nd.np_pad + nd.m;
        auto row = [&](int rr) { return rr >= f ? f - 1 : (rr >= nd.np && rr < nd.np_pad ? nd.np - 1 : rr); };
        int r = fp - 64 + lane;
        for (; r - 64 >= rlo; r -= 128) {
            const T w0 = ld_sc1(&w[r]), w1 = ld_sc1(&w[r - 64]);
            const int q0 = row(r), q1 = row(r - 64);
            T l0[16], l1[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                l0[c] = lc[(int64_t)c * ld + q0];
                l1[c] = lc[(int64_t)c * ld + q1];
            }
#pragma unroll
            for (int c = 0; c < 16; ++c) acc[c] = fma_t(l1[c], w1, fma_t(l0[c], w0, acc[c]));
        }
        if (r >= rlo) {
            const T w0 = ld_sc1(&w[r]);
#pragma unroll
            for (int c = 0; c < 16; ++c) acc[c] = fma_t(lc[(int64_t)c * ld + r], w0, acc[c]);
        }
#pragma unroll
        for (int c = 0; c < 16; ++c) red[16 * wv + c][lane] = acc[c];
        __syncthreads();
        if (tid < 64) {
            T s0 = (T)0, s1 = (T)0, s2 = (T)0, s3 = (T)0;
#pragma unroll
            for (int l = 0; l < 64; l += 4) {
                s0 += red[tid][l];
                s1 += red[tid][l + 1];
                s2 += red[tid][l + 2];
                s3 += red[tid][l + 3];
            }
            zk[tid] = ld_sc1(&w[64 * K + tid]) - ((s0 + s1) + (s2 + s3));
        }
        __syncthreads();
        {  // x_K = Dinv_K^T z: Linv[q][l] = Dinv[l * 64 + q]; wave wv sums q in [16 wv, 16 wv + 16)
            const T* g = Dinv + nd.dinv_off + (int64_t)K * 4096 + (int64_t)lane * 64 + 16 * wv;
            T gv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) gv[j] = g[j];
            T x0 = (T)0, x1 = (T)0;
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                x0 = fma_t(gv[j], zk[16 * wv + j], x0);
                x1 = fma_t(gv[j + 1], zk[16 * wv + j + 1], x1);
            }
            part[wv][lane] = x0 + x1;
        }
        __syncthreads();
        if (tid < 64) st_sc1(&w[64 * K + tid], (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    for (int p = tid; p < nd.np; p += 256) xp[col * n + nd.start + p] = ld_sc1(&w[p]);
}

// Backward solve of one level by pivot tiles: one workgroup per (node, pivot
// tile K, column), taken by ticket from the fronts' last pivot tiles down (a
// workgroup only waits on lower tickets). It sums the column products of
// the rows below tile K as nd_backward does, tile by tile from the last: the
// front rows (the ancestors' x, read through st) at once, then each pivot
// tile J > K as its x_J is published (flag per node, column and pivot tile);
// then x_K = Dinv_K^T (y_K - sums) and its pivots to xp. The same operations
// in the same order per lane as nd_backward: the same bits
// (BSM_ND_BWD_TILES=0 for the A/B).
template <typename T>
__global__ __launch_bounds__(256) void nd_backward_tiles(const NdDev* __restrict__ nodes,
                                                         const int2* __restrict__ tasks, int64_t ntasks, int k,
                                                         int64_t n, T* __restrict__ xp, T* __restrict__ V,
                                                         int64_t vtot, const T* __restrict__ F,
                                                         const T* __restrict__ Dinv, const int32_t* __restrict__ st,
                                                         int* __restrict__ xflags, int* __restrict__ ticket,
                                                         int* __restrict__ status) {
    __shared__ T red[64][65];
    __shared__ T zk[64];
    __shared__ T part[4][64];
    __shared__ int tk;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t total = ntasks * k;
    // Control flow kept simple for the structurizer (a first form, with the
    // ticket taken at the loop head and a barrier inside an if / else of the
    // row loop, compiled to a loop whose back edge skipped the ticket: the
    // workgroup redid its first task forever): the ticket is taken at the
    // END of each task, both row loops are plain counted loops, and the
    // flag poll has no break.
    if (tid == 0) tk = atomicAdd(ticket, 1);
    __syncthreads();
    int64_t t = __builtin_amdgcn_readfirstlane(tk);
    while (t < total) {
        const int2 task = tasks[t / k];
        const int col = (int)(t % k);
        const NdDev& nd = nodes[task.x];
        const int K = task.y;
        T* const w = V + (int64_t)col * vtot + nd.voff;
        int* const xf = xflags + (nd.dinv_off / 4096) * k + (int64_t)col * nd.npt;
        const int32_t* const sr = st + nd.st_off;
        const T* const lc = F + nd.foff + (int64_t)(64 * K + 16 * wv) * nd.ld;
        const int64_t ld = nd.ld;
        T acc[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) acc[c] = (T)0;
        // the front rows' tiles, last first: the ancestors' x (0 past the m rows)
        const int jf = nd.npt > K + 1 ? nd.npt : K + 1;
        for (int J = nd.nt - 1; J >= jf; --J) {
            const int r = 64 * J + lane, a = r - nd.np_pad;
            const T wr = a < nd.m ? xp[(int64_t)col * n + sr[a]] : (T)0;
            T l[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) l[c] = lc[(int64_t)c * ld + r];
#pragma unroll
            for (int c = 0; c < 16; ++c) acc[c] = fma_t(l[c], wr, acc[c]);
        }
        // then the pivot tiles below K, each as its x is published
        for (int J = nd.npt - 1; J > K; --J) {
            if (tid == 0) {
                long long spins = 0;
                while (__hip_atomic_load(&xf[J], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                       spins < ND_SOLVE_SPIN_LIMIT) {
                    __builtin_amdgcn_s_sleep(1);
                    ++spins;
                }
                if (spins >= ND_SOLVE_SPIN_LIMIT) atomicOr(status, ST_TIMEOUT);
            }
            __syncthreads();
            const int r = 64 * J + lane;
            const T wr = ld_sc1(&w[r]);
            T l[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) l[c] = lc[(int64_t)c * ld + r];
#pragma unroll
            for (int c = 0; c < 16; ++c) acc[c] = fma_t(l[c], wr, acc[c]);
        }
#pragma unroll
        for (int c = 0; c < 16; ++c) red[16 * wv + c][lane] = acc[c];
        __syncthreads();
        if (tid < 64) {
            T s0 = (T)0, s1 = (T)0, s2 = (T)0, s3 = (T)0;
#pragma unroll
            for (int l = 0; l < 64; l += 4) {
                s0 += red[tid][l];
                s1 += red[tid][l + 1];
                s2 += red[tid][l + 2];
                s3 += red[tid][l + 3];
            }
            zk[tid] = ld_sc1(&w[64 * K + tid]) - ((s0 + s1) + (s2 + s3));
        }
        __syncthreads();
        {  // x_K = Dinv_K^T z, as nd_backward
            const T* g = Dinv + nd.dinv_off + (int64_t)K * 4096 + (int64_t)lane * 64 + 16 * wv;
            T gv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) gv[j] = g[j];
            T x0 = (T)0, x1 = (T)0;
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                x0 = fma_t(gv[j], zk[16 * wv + j], x0);
                x1 = fma_t(gv[j + 1], zk[16 * wv + j + 1], x1);
            }
            part[wv][lane] = x0 + x1;
        }
        __syncthreads();
        if (tid < 64) {
            const T x = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
            st_sc1(&w[64 * K + tid], x);
            if (64 * K + tid < nd.np) xp[(int64_t)col * n + nd.start + 64 * K + tid] = x;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_store(&xf[K], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tk = atomicAdd(ticket, 1);
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(tk);
    }
}

inline unsigned nd_blocks(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

// the device form of a plan: node descriptors, front rows, tile and task lists
struct NdLayout {
    std::vector<NdDev> dev;
    std::vector<int32_t> st, ri, pinv, owner, lvl_nodes;
    std::vector<int32_t> tb;   // per child: its rows' bounds per tile row of the parent (NdDev::tb_off)
    std::vector<int4> tiles;   // nd_factor's tasks: tiles of the tiled fronts, then the small fronts whole
    std::vector<int4> ztiles;  // every front's lower tiles (nd_zero_tiles)
    std::vector<int2> ext;
    std::vector<int64_t> tiles_off, lvl_off, ext_off;  // per level (ext: per level and slot)
    std::vector<int4> ext2;                             // nd_extend2's tasks (both slots)
    std::vector<int64_t> ext2_off;                      // per level
    std::vector<int2> ftasks;                           // nd_forward_tiles' (node, tile row), I-major
    std::vector<int64_t> ftask_off;                     // per level
    std::vector<int2> btasks;                           // nd_backward_tiles' (node, pivot tile), last tiles first
    std::vector<int64_t> btask_off;                     // per level
    int64_t f_elems = 0, dinv_elems = 0, n_flags = 0, vtot = 0, n_lower = 0;
};

// lay: the layout's options. Bits 0-15: fronts of at most this many tile
// rows are one whole-front task of nd_factor (0: every front by tiles); bit
// 16: the per-slot extend lists too (BSM_ND_EXT_MERGE=0's A/B path; ~1M
// entries at C5 that the default merged launches never read); bits 17-27:
// the lag of the tiles below a diagonal, in fronts (0: none); bit 28: the
// extend-add by nd_extend2 / nd_extend launches (BSM_ND_PULL=0) instead of
// inside nd_factor's tile loads (the extend task lists are only built then)
void nd_layout(const NdPlan& P, int32_t lay, NdLayout& L) {
    const int32_t small_nt = lay & 0xffff;
    const bool per_slot = (lay >> 16) & 1;
    const bool push = (lay >> 28) & 1;
    const int32_t nn = (int32_t)P.nodes.size();
    L.dev.resize((size_t)nn);
    int64_t st_total = 0;
    for (int32_t i = 0; i < nn; ++i) {
        const NdNode& x = P.nodes[(size_t)i];
        NdDev& d = L.dev[(size_t)i];
        d.np = (int32_t)(x.end - x.start);
        d.npt = (d.np + 63) / 64;
        d.np_pad = 64 * d.npt;
        d.m = (int32_t)x.st.size();
        d.nt = (d.np_pad + d.m + 63) / 64;
        d.ld = 64 * d.nt;
        d.start = x.start;
        d.parent = x.parent;
        d.kid0 = x.kids[0];
        d.kid1 = x.kids[1];
        d.tb_off = -1;
        d.tile_off = (int32_t)L.n_lower;
        L.n_lower += (int64_t)d.nt * (d.nt + 1) / 2;
        d.pull_swap = x.kids[0] >= 0 && x.kids[1] >= 0 &&
                      P.nodes[(size_t)x.kids[1]].level < P.nodes[(size_t)x.kids[0]].level;
        d.foff = L.f_elems;
        L.f_elems += (int64_t)d.ld * d.ld;
        d.dinv_off = L.dinv_elems;
        L.dinv_elems += (int64_t)d.npt * 4096;
        d.flag_off = L.n_flags;
        L.n_flags += (int64_t)d.nt * d.npt;
        d.voff = L.vtot;
        L.vtot += d.ld;
        d.st_off = st_total;
        st_total += d.m;
    }
    int64_t tb_total = 0;  // a child's bounds: its parent's nt + 1 (parents follow their children)
    for (int32_t i = 0; i < nn; ++i)
        if (L.dev[(size_t)i].parent >= 0) {
            L.dev[(size_t)i].tb_off = (int32_t)tb_total;
            tb_total += L.dev[(size_t)L.dev[(size_t)i].parent].nt + 1;
        }
    L.tb.resize((size_t)tb_total);
    L.st.resize((size_t)st_total);
    L.ri.resize((size_t)st_total);
    L.pinv.resize((size_t)P.n);
    L.owner.resize((size_t)P.n);
    // per node, disjoint ranges: on a few threads (the C5 plan's ~1M front
    // rows and 1M columns)
    auto per_node = [&](int32_t lo, int32_t hi) {
        for (int32_t i = lo; i < hi; ++i) {
            const NdNode& x = P.nodes[(size_t)i];
            const NdDev& d = L.dev[(size_t)i];
            for (int64_t q = x.start; q < x.end; ++q) {
                L.owner[(size_t)q] = i;
                L.pinv[(size_t)P.perm[(size_t)q]] = (int32_t)q;
            }
            for (int32_t a = 0; a < d.m; ++a) L.st[(size_t)(d.st_off + a)] = (int32_t)x.st[(size_t)a];
            if (x.parent < 0) continue;
            // a front row of the child is a pivot of the parent or one of its front rows
            const NdNode& px = P.nodes[(size_t)x.parent];
            const NdDev& pd = L.dev[(size_t)x.parent];
            size_t j = 0;
            for (int32_t a = 0; a < d.m; ++a) {
                const int64_t q = x.st[(size_t)a];
                if (q < px.end) {
                    L.ri[(size_t)(d.st_off + a)] = (int32_t)(q - px.start);
                } else {
                    while (px.st[j] < q) ++j;
                    L.ri[(size_t)(d.st_off + a)] = pd.np_pad + (int32_t)j;
                }
            }
            const int32_t* r = L.ri.data() + d.st_off;
            int32_t* t = L.tb.data() + d.tb_off;
            for (int32_t u = 0, a = 0; u <= pd.nt; ++u) {
                while (a < d.m && r[a] < 64 * u) ++a;
                t[u] = a;
            }
        }
    };
    {
        const int nt = (int)std::min<int32_t>(8, std::max<int32_t>(1, nn / 1024));
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; ++t) pool.emplace_back(per_node, (int32_t)((int64_t)nn * t / nt), (int32_t)((int64_t)nn * (t + 1) / nt));
        per_node(0, (int32_t)((int64_t)nn / nt));
        for (auto& th : pool) th.join();
    }
    // per level: the nodes, the factor's tiles (K, node, I) and the extend tasks (slot, node, b)
    std::vector<std::vector<int32_t>> by_level((size_t)P.n_levels);
    for (int32_t i = 0; i < nn; ++i) by_level[(size_t)P.nodes[(size_t)i].level].push_back(i);
    {  // the lists' sizes up front (no regrowth of ~1M-entry vectors)
        size_t zt = 0, ft = 0, bt = 0, ex = 0;
        for (const NdDev& d : L.dev) {
            zt += (size_t)d.nt * (d.nt + 1) / 2;
            ft += (size_t)d.nt;
            bt += (size_t)d.npt;
            ex += d.parent >= 0 && push ? (size_t)d.m : 0;
        }
        L.ztiles.reserve(zt);
        L.tiles.reserve(zt);
        L.ftasks.reserve(ft);
        L.btasks.reserve(bt);
        if (per_slot) L.ext.reserve(ex);
        L.ext2.reserve(ex);
        L.lvl_nodes.reserve((size_t)nn);
    }
    // The levels' lists are independent: built on threads (the leaf level,
    // the largest, sets the time), then concatenated in level order
    struct LevelLists {
        std::vector<int4> zt, tiles, ext2;
        std::vector<int2> ext[2], ft, bt;
    };
    std::vector<LevelLists> per((size_t)P.n_levels);
    auto build_level = [&](size_t li) {
        const auto& lv = by_level[li];
        LevelLists& o = per[li];
        std::vector<char> used;  // the merge walk's marks, reused
        int32_t kmax = 0;
        for (int32_t i : lv) kmax = std::max(kmax, L.dev[(size_t)i].nt);
        // every front's lower tiles (nd_zero_tiles)
        for (int32_t i : lv)
            for (int32_t K = 0; K < L.dev[(size_t)i].nt; ++K)
                for (int32_t I = K; I < L.dev[(size_t)i].nt; ++I) o.zt.push_back(make_int4(i, I, K, 0));
        // tiled fronts, column K of every front: the diagonal tiles first,
        // then the tiles below (which wait for their diagonal tile's
        // inverse), so the waiting tiles' diagonals are well under way when
        // they are taken; then the small fronts, one task each
        // With a lag (bits 17-27 of lay, in fronts), a front's tiles below the
        // diagonal follow its diagonal tile by `lag` fronts' diagonals
        // instead of all of them: at about the grid's size (512 workgroups)
        // the diagonal is done when they are taken, and the level's other
        // fronts are not held up behind the whole column of diagonals. 0: all
        // of a column's diagonal tiles first (round 5). Either way a tile only
        // waits on earlier tickets.
        auto small = [&](int32_t i) { return L.dev[(size_t)i].nt <= small_nt; };
        const size_t lag_units = (size_t)((lay >> 17) & 0x7ff);
        std::vector<int32_t> fr;
        for (int32_t K = 0; K < kmax; ++K) {
            fr.clear();
            for (int32_t i : lv)
                if (!small(i) && K < L.dev[(size_t)i].nt) fr.push_back(i);
            const size_t nf = fr.size(), lag = lag_units ? lag_units : nf;
            for (size_t idx = 0; idx < nf + lag; ++idx) {
                if (idx < nf) o.tiles.push_back(make_int4(fr[idx], K, K, 0));
                if (idx >= lag && idx - lag < nf) {
                    const int32_t i = fr[idx - lag];
                    for (int32_t I = K + 1; I < L.dev[(size_t)i].nt; ++I) o.tiles.push_back(make_int4(i, I, K, 0));
                }
            }
        }
        for (int32_t i : lv)
            if (small(i)) o.tiles.push_back(make_int4(i, 0, 0, 1));
        for (int s = 0; s < 2 && per_slot && push; ++s)
            for (int32_t i : lv) {
                const NdNode& x = P.nodes[(size_t)i];
                if (x.parent < 0 || x.slot != s) continue;
                for (int32_t b = 0; b < L.dev[(size_t)i].m; ++b) o.ext[s].push_back(make_int2(i, b));
            }
        for (int32_t I = 0; I < kmax; ++I)
            for (int32_t i : lv)
                if (I < L.dev[(size_t)i].nt) o.ft.push_back(make_int2(i, I));
        int32_t pmax = 0;
        for (int32_t i : lv) pmax = std::max(pmax, L.dev[(size_t)i].npt);
        for (int32_t d = 0; d < pmax; ++d)
            for (int32_t i : lv)
                if (d < L.dev[(size_t)i].npt) o.bt.push_back(make_int2(i, L.dev[(size_t)i].npt - 1 - d));
        if (lv.empty() || !push) return;
        // both slots in one launch: a slot-0 child's columns, each paired with
        // the slot-1 sibling's column landing on the same parent column when
        // that sibling is on this level too, then the sibling's unpaired ones
        const int32_t level = P.nodes[(size_t)lv.front()].level;
        for (int32_t i : lv) {
            const NdNode& x = P.nodes[(size_t)i];
            if (x.parent < 0) continue;
            const NdNode& px = P.nodes[(size_t)x.parent];
            const int32_t sib = px.kids[1 - x.slot];
            const bool pair = sib >= 0 && P.nodes[(size_t)sib].level == level;
            if (pair && x.slot == 1) continue;  // taken with its slot-0 sibling
            const int32_t m0 = L.dev[(size_t)i].m;
            const int32_t* r0 = L.ri.data() + L.dev[(size_t)i].st_off;
            if (!pair) {
                for (int32_t b = 0; b < m0; ++b) o.ext2.push_back(make_int4(i, b, -1, -1));
                continue;
            }
            const int32_t m1 = L.dev[(size_t)sib].m;
            const int32_t* r1 = L.ri.data() + L.dev[(size_t)sib].st_off;
            used.assign((size_t)m1, 0);
            int32_t b1 = 0;
            for (int32_t b = 0; b < m0; ++b) {  // ri ascending on both sides: one merge walk
                while (b1 < m1 && r1[b1] < r0[b]) ++b1;
                const bool hit = b1 < m1 && r1[b1] == r0[b];
                if (hit) used[(size_t)b1] = 1;
                o.ext2.push_back(make_int4(i, b, hit ? sib : -1, hit ? b1 : -1));
            }
            for (int32_t b = 0; b < m1; ++b)
                if (!used[(size_t)b]) o.ext2.push_back(make_int4(sib, b, -1, -1));
        }
    };
    {
        std::atomic<size_t> next{0};
        auto work = [&] {
            for (size_t li; (li = next.fetch_add(1)) < per.size();) build_level(li);
        };
        std::vector<std::thread> pool;
        const int nt = (int)std::min<size_t>(8, per.size());
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();
    }
    for (size_t li = 0; li < per.size(); ++li) {
        const auto& lv = by_level[li];
        const LevelLists& o = per[li];
        L.lvl_off.push_back((int64_t)L.lvl_nodes.size());
        L.lvl_nodes.insert(L.lvl_nodes.end(), lv.begin(), lv.end());
        L.tiles_off.push_back((int64_t)L.tiles.size());
        L.ztiles.insert(L.ztiles.end(), o.zt.begin(), o.zt.end());
        L.tiles.insert(L.tiles.end(), o.tiles.begin(), o.tiles.end());
        for (int sl = 0; sl < 2; ++sl) {
            L.ext_off.push_back((int64_t)L.ext.size());
            L.ext.insert(L.ext.end(), o.ext[sl].begin(), o.ext[sl].end());
        }
        L.ftask_off.push_back((int64_t)L.ftasks.size());
        L.ftasks.insert(L.ftasks.end(), o.ft.begin(), o.ft.end());
        L.btask_off.push_back((int64_t)L.btasks.size());
        L.btasks.insert(L.btasks.end(), o.bt.begin(), o.bt.end());
        L.ext2_off.push_back((int64_t)L.ext2.size());
        L.ext2.insert(L.ext2.end(), o.ext2.begin(), o.ext2.end());
    }
    L.lvl_off.push_back((int64_t)L.lvl_nodes.size());
    L.tiles_off.push_back((int64_t)L.tiles.size());
    L.ext_off.push_back((int64_t)L.ext.size());
    L.ext2_off.push_back((int64_t)L.ext2.size());
    L.ftask_off.push_back((int64_t)L.ftasks.size());
    L.btask_off.push_back((int64_t)L.btasks.size());
}

// A pattern's plan, device side: one allocation holding the node
// descriptors, front rows, their places in the parents, pinv / owner, the
// level lists, tiles and extend tasks, and perm; plus the per-level offsets
// the launches need. Cached on the handle (bsm_csr::nd_plan) unless
// BSM_ND_CACHE=0: the pattern of a finalised Csr never changes.
struct NdCached {
    int64_t leaf = 0;
    int32_t nn = 0, n_levels = 0;
    std::vector<int64_t> tiles_off, lvl_off, ext_off, ext2_off, ftask_off, btask_off;
    int64_t f_elems = 0, dinv_elems = 0, n_flags = 0, vtot = 0, max_front = 0;
    size_t o_dev = 0, o_st = 0, o_ri = 0, o_pinv = 0, o_owner = 0, o_lvl = 0, o_tiles = 0, o_ext = 0, o_ext2 = 0,
           o_ftask = 0, o_btask = 0, o_perm = 0, o_ztiles = 0, o_tb = 0, o_zf = 0;
    size_t n_tiles = 0, n_ztiles = 0, n_ext = 0;
    int64_t n_lower = 0, n_aent = 0;  // the fronts' lower tiles; A's lower entries
    DBuf aoff, aent, tq;              // A's entries by tile (nd_aent_*), per task ranges
    DBuf pdesc;                       // per task: its children's blocks (nd_task_pull)
    int32_t small_nt = 0;
    double ms_graph = 0, ms_order = 0, ms_symbolic = 0, ms_layout = 0, ms_pack = 0;
    DBuf plan;
    // The numeric storage (fronts, inverse diagonal tiles, flags) stays with
    // the cached plan for the handle's next solve: hipFree of the 5.6 GB of
    // fronts and hipMalloc again cost ~0.9 ms of a C5 solve's 11.4
    // (profiles/r05_q_*). One solve at a time uses them (num_mu; a concurrent
    // solve on the same handle allocates its own). BSM_ND_KEEP=0: freed after
    // every solve.
    std::mutex num_mu;
    DBuf fr, dv, fl;
    std::atomic<size_t> kept_bytes{0};  // fr + dv + fl, written under num_mu
    hipEvent_t fr_zeroed = nullptr;     // fr was just allocated and is being zeroed (nd_build_plan)
    // drop the kept numeric storage unless a solve holds it
    void drop_zeroed() {  // fr no longer the freshly zeroed allocation (under num_mu)
        if (fr_zeroed) (void)hipEventDestroy(fr_zeroed);
        fr_zeroed = nullptr;
    }
    ~NdCached() { drop_zeroed(); }
    bool release_numeric() {
        std::unique_lock<std::mutex> l(num_mu, std::try_to_lock);
        if (!l.owns_lock()) return false;
        drop_zeroed();
        fr.reset();
        dv.reset();
        fl.reset();
        kept_bytes = 0;
        return true;
    }
};

// ---- the plan cache across handles ------------------------------------------
// solve(a: Csr<f32>, b) takes `a` by value (src/lib.rs:11): a drop-in caller
// builds a new Csr, hence a new handle, for every solve, and a plan kept only
// on the handle is rebuilt every time (the host analysis is ~90 % of a cold
// C5 solve). So plans are also kept in a library-wide cache keyed by the
// pattern: (device, n, nnz, leaf) and a 128-bit hash of row_ptr and col
// computed on the device; a hash hit is confirmed by comparing the pattern
// with the entry's own copy of it (no false hit on a collision). Bounded:
// at most BSM_ND_CACHE_ENTRIES entries (default 4, least recently used out)
// and at most BSM_ND_CACHE_MB of kept numeric storage (default 32768) over
// the entries no solve is using; bsm_nd_cache_clear drops them all.

__device__ __forceinline__ uint64_t nd_mix64(uint64_t z) {  // SplitMix64's finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// two sums (mod 2^64) of per-element hashes of (position, value): order-free
// integer sums, so the key does not depend on the grid; one pair of atomics
// per workgroup (one per wave on 4096 workgroups contended for 0.4 ms)
__global__ __launch_bounds__(256) void nd_pattern_hash(const int64_t* __restrict__ rp, int64_t n1,
                                                       const int32_t* __restrict__ col, int64_t nnz,
                                                       unsigned long long* __restrict__ h) {
    __shared__ unsigned long long part[2][4];
    uint64_t s0 = 0, s1 = 0;
    const int64_t total = n1 + nnz;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const uint64_t x = e < n1 ? (uint64_t)rp[e] : (uint64_t)(uint32_t)col[e - n1];
        const uint64_t k = (uint64_t)e * 0x9e3779b97f4a7c15ull;
        s0 += nd_mix64(x ^ k);
        s1 += nd_mix64(x + k + 0x632be59bd9b4e019ull);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s0 += (uint64_t)__shfl_xor((unsigned long long)s0, o);
        s1 += (uint64_t)__shfl_xor((unsigned long long)s1, o);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = s0;
        part[1][threadIdx.x >> 6] = s1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned long long* p = part[threadIdx.x];
        atomicAdd(&h[threadIdx.x], p[0] + p[1] + p[2] + p[3]);
    }
}

// *diff != 0 when the patterns differ anywhere
__global__ __launch_bounds__(256) void nd_pattern_diff(const int64_t* __restrict__ rpa, const int64_t* __restrict__ rpb,
                                                       int64_t n1, const int32_t* __restrict__ ca,
                                                       const int32_t* __restrict__ cb, int64_t nnz,
                                                       int* __restrict__ diff) {
    bool d = false;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n1 + nnz; e += (int64_t)gridDim.x * 256)
        d |= e < n1 ? rpa[e] != rpb[e] : ca[e - n1] != cb[e - n1];
    if (__any(d) && (threadIdx.x & 63) == 0) atomicOr(diff, 1);
}

struct NdKey {
    int device = 0;
    int32_t small_nt = 0;
    int64_t n = 0, leaf = 0;
    uint64_t nnz = 0, h0 = 0, h1 = 0;
    bool operator==(const NdKey& o) const {
        return device == o.device && small_nt == o.small_nt && n == o.n && leaf == o.leaf && nnz == o.nnz &&
               h0 == o.h0 && h1 == o.h1;
    }
};

struct NdCacheEntry {
    NdKey key;
    uint64_t tick = 0;
    std::shared_ptr<DBuf> pattern;  // row_ptr (n + 1 int64), then col (nnz int32)
    std::shared_ptr<NdCached> plan;
};

struct NdCache {
    std::mutex mu;
    std::vector<NdCacheEntry> entries;
    uint64_t tick = 0, hits = 0, misses = 0;
};

NdCache& nd_cache() {  // never destroyed: no hipFree after the runtime's teardown at exit
    static NdCache* c = new NdCache;
    return *c;
}

size_t nd_cache_limit(const char* env, size_t dflt) {
    const char* e = getenv(env);
    return e ? (size_t)atoll(e) : dflt;
}

// The calling thread's page-locked staging buffer (grown on demand, kept for
// the thread's later plans): the pattern's download and the plan's upload
// are direct DMA (~30 MB each at C5) instead of pageable copies.
struct PinnedStage {
    char* buf = nullptr;
    size_t cap = 0;
};
PinnedStage& pinned_stage() {
    thread_local PinnedStage st;
    return st;
}
int pinned_grow(PinnedStage& st, size_t bytes) {
    if (st.cap >= bytes) return BSM_OK;
    if (st.buf) (void)hipHostFree(st.buf);
    st.buf = nullptr;
    st.cap = 0;
    BSM_HIP_TRY(hipHostMalloc((void**)&st.buf, bytes, hipHostMallocDefault));
    st.cap = bytes;
    return BSM_OK;
}
int pinned_staging(size_t bytes, char** out) {
    PinnedStage& st = pinned_stage();
    BSM_TRY(pinned_grow(st, bytes));
    *out = st.buf;
    return BSM_OK;
}

// An upper bound of nd_build_plan's packed plan bytes, from the analysis
// alone (the same arrays as the layout; the merged extend tasks and the
// factor's tasks are at most the child columns and the lower tiles)
size_t nd_plan_bytes_bound(const NdPlan& P, int32_t lay) {
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    size_t sm = 0, zt = 0, ft = 0, bt = 0;
    for (const auto& x : P.nodes) {
        const int64_t npt = (x.end - x.start + 63) / 64, nt = (64 * npt + (int64_t)x.st.size() + 63) / 64;
        sm += x.st.size();
        zt += (size_t)(nt * (nt + 1) / 2);
        ft += (size_t)nt;
        bt += (size_t)npt;
    }
    const size_t nn = P.nodes.size(), n = (size_t)P.n;
    const bool push = (lay >> 28) & 1;
    // the children's tile bounds: at most two children of nt + 1 per node
    return al(nn * sizeof(NdDev)) + 2 * al(sm * 4) + 2 * al(n * 4) + al(nn * 4) + al(zt * sizeof(int4)) +
           al(push && ((lay >> 16) & 1) ? sm * sizeof(int2) : 0) + al(push ? sm * sizeof(int4) : 0) +
           al(ft * sizeof(int2)) + al(bt * sizeof(int2)) + al(n * 8) + al(zt * sizeof(int4)) +
           al(2 * (ft + nn) * 4) + al(zt);
}

// es > 0: the fronts (es-byte values) are allocated into C.fr on a helper
// thread while the layout, the packing and the plan's upload run: a first
// solve's 5 GB hipMalloc (C5) then costs no time of its own
int nd_build_plan(const bsm_csr* a, int64_t leaf, int32_t small_nt, size_t es, hipStream_t s, NdCached& C) {
    const int64_t N = (int64_t)a->rows;
    // A's pattern to the host for the analysis
    char* stg = nullptr;
    const size_t rp_bytes = ((size_t)(N + 1) * sizeof(int64_t) + 255) / 256 * 256;
    BSM_TRY(pinned_staging(rp_bytes + (size_t)a->nnz * sizeof(int32_t), &stg));
    const int64_t* rp = (const int64_t*)stg;
    const int32_t* cl = (const int32_t*)(stg + rp_bytes);
    BSM_HIP_TRY(hipMemcpyAsync(stg, a->row_ptr, (size_t)(N + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    if (a->nnz)
        BSM_HIP_TRY(hipMemcpyAsync(stg + rp_bytes, a->col, (size_t)a->nnz * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    stage_mark("nd_pattern_d2h", s);
    const char* te = getenv("BSM_ND_THREADS");
    const int threads = te ? atoi(te) : (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
    NdPlan P;
    const int arc = nd_analyse(N, rp, cl, leaf, threads, P);
    BSM_REQUIRE(arc == 0, BSM_ERR_UNSUPPORTED,
                "cholesky: rows must have strictly increasing columns (get_row_complete semantics)");
    std::thread pre;
    struct Join {
        std::thread& t;
        ~Join() {
            if (t.joinable()) t.join();
        }
    } join_pre{pre};
    // on the helper as well (the pattern in the staging buffer is no longer
    // read): the plan's device buffer and the calling thread's page-locked
    // staging buffer, both at an upper bound of the packed plan (~42 MB at
    // C5), so the packing and the upload below allocate nothing
    const size_t plan_bound = nd_plan_bytes_bound(P, small_nt);
    PinnedStage* const stage = &pinned_stage();
    {
        const int dev0 = a->device;
        pre = std::thread([&C, plan_bound, stage, dev0] {
            if (hipSetDevice(dev0) != hipSuccess) return;
            (void)C.plan.alloc(plan_bound);      // the main thread allocates again if this failed
            (void)pinned_grow(*stage, plan_bound);  // likewise (pinned_staging)
        });
    }
    std::thread pre_fronts;
    struct JoinF {
        std::thread& t;
        ~JoinF() {
            if (t.joinable()) t.join();
        }
    } join_fronts{pre_fronts};
    if (es) {
        int64_t f_elems = 0, dinv_elems = 0, n_flags = 0;  // nd_layout's sums (fronts, inverse tiles, flags)
        for (const auto& x : P.nodes) {
            const int64_t npt = (x.end - x.start + 63) / 64, np_pad = 64 * npt;
            const int64_t nt = (np_pad + (int64_t)x.st.size() + 63) / 64, ld = 64 * nt;
            f_elems += ld * ld;
            dinv_elems += npt * 4096;
            n_flags += nt * npt;
        }
        // the inverse diagonal tiles and the flags too, at the sizes nd_solve
        // asks for (a fresh hipMalloc of ~0.8 GB took ms inside the first
        // solve when the box had just freed memory)
        const size_t dv_bytes = (size_t)std::max<int64_t>(dinv_elems, 1) * es;
        const size_t fl_bytes = ((size_t)n_flags + (size_t)P.n_levels + 2) * sizeof(int);
        const int dev = a->device;
        // BSM_ND_PREZERO=1: also zeroed whole there, on a stream of its own
        // (round 6 before the marked tiles: a fresh allocation's first touch
        // cost ~10 ms at C5 inside the solve's first kernel). Off by default:
        // with the layout at ~6 ms the solve waited ~7 ms for that memset,
        // while zeroing only the marked tiles in the solve takes ~3 ms
        // (profiles/r06_m_*)
        const char* pze = getenv("BSM_ND_PREZERO");
        const bool prezero = pze && atoi(pze) == 1;
        pre_fronts = std::thread([&C, f_elems, es, dev, prezero, dv_bytes, fl_bytes] {
            if (hipSetDevice(dev) != hipSuccess || C.fr.alloc((size_t)f_elems * es) != BSM_OK) return;
            (void)C.dv.alloc(dv_bytes);  // nd_solve allocates again if this failed
            (void)C.fl.alloc(fl_bytes);
            if (!prezero) return;
            hipStream_t z = nullptr;
            hipEvent_t ev = nullptr;
            if (hipStreamCreateWithFlags(&z, hipStreamNonBlocking) != hipSuccess) return;
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
                hipMemsetAsync(C.fr.p, 0, C.fr.bytes, z) == hipSuccess && hipEventRecord(ev, z) == hipSuccess) {
                C.fr_zeroed = ev;  // nd_solve waits for it and skips nd_zero_tiles once
            } else if (ev) {
                (void)hipEventDestroy(ev);
            }
            (void)hipStreamDestroy(z);  // released once its work is done
        });
    }
    const auto tl0 = host_now();
    NdLayout L;
    C.small_nt = small_nt;
    nd_layout(P, small_nt, L);
    C.ms_layout = ms_since(tl0);
    C.leaf = leaf;
    C.nn = (int32_t)L.dev.size();
    C.n_levels = P.n_levels;
    C.tiles_off = L.tiles_off;
    C.lvl_off = L.lvl_off;
    C.ext_off = L.ext_off;
    C.ext2_off = L.ext2_off;
    C.ftask_off = L.ftask_off;
    C.btask_off = L.btask_off;
    C.f_elems = L.f_elems;
    C.dinv_elems = L.dinv_elems;
    C.n_flags = L.n_flags;
    C.vtot = L.vtot;
    C.n_tiles = L.tiles.size();
    C.n_lower = L.n_lower;
    C.n_ztiles = L.ztiles.size();
    C.n_ext = L.ext.size();
    C.ms_graph = P.ms_graph;
    C.ms_order = P.ms_order;
    C.ms_symbolic = P.ms_symbolic;
    for (const auto& d : L.dev) C.max_front = std::max<int64_t>(C.max_front, d.ld);
    stage_mark("nd_analyse", s);
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    C.o_dev = 0;
    C.o_st = C.o_dev + al(L.dev.size() * sizeof(NdDev));
    C.o_ri = C.o_st + al(L.st.size() * 4);
    C.o_pinv = C.o_ri + al(L.ri.size() * 4);
    C.o_owner = C.o_pinv + al(L.pinv.size() * 4);
    C.o_lvl = C.o_owner + al(L.owner.size() * 4);
    C.o_tiles = C.o_lvl + al(L.lvl_nodes.size() * 4);
    C.o_ext = C.o_tiles + al(L.tiles.size() * sizeof(int4));
    C.o_ext2 = C.o_ext + al(L.ext.size() * sizeof(int2));
    C.o_ftask = C.o_ext2 + al(L.ext2.size() * sizeof(int4));
    C.o_btask = C.o_ftask + al(L.ftasks.size() * sizeof(int2));
    C.o_perm = C.o_btask + al(L.btasks.size() * sizeof(int2));
    C.o_ztiles = C.o_perm + al((size_t)N * 8);
    C.o_tb = C.o_ztiles + al(L.ztiles.size() * sizeof(int4));
    C.o_zf = C.o_tb + al(L.tb.size() * 4);
    const size_t total = C.o_zf + al((size_t)L.n_lower);
    if (pre.joinable()) pre.join();  // the plan's buffers (device, page-locked staging)
    const auto tp0 = host_now();
    char* hp = nullptr;
    BSM_TRY(pinned_staging(total, &hp));  // the pattern is no longer needed
    // the arrays into the staging buffer in 1-MiB pieces on four threads
    // (~40 MB at C5: one thread's memcpy into fresh pinned pages is ms)
    struct Piece {
        size_t o;
        const char* p;
        size_t b;
    };
    std::vector<Piece> pieces;
    auto put = [&](size_t o, const void* p, size_t b) {
        for (size_t c = 0; c < b; c += (1 << 20))
            pieces.push_back({o + c, static_cast<const char*>(p) + c, std::min<size_t>(b - c, 1 << 20)});
    };
    put(C.o_dev, L.dev.data(), L.dev.size() * sizeof(NdDev));
    put(C.o_st, L.st.data(), L.st.size() * 4);
    put(C.o_ri, L.ri.data(), L.ri.size() * 4);
    put(C.o_pinv, L.pinv.data(), L.pinv.size() * 4);
    put(C.o_owner, L.owner.data(), L.owner.size() * 4);
    put(C.o_lvl, L.lvl_nodes.data(), L.lvl_nodes.size() * 4);
    put(C.o_tiles, L.tiles.data(), L.tiles.size() * sizeof(int4));
    put(C.o_ext, L.ext.data(), L.ext.size() * sizeof(int2));
    put(C.o_ext2, L.ext2.data(), L.ext2.size() * sizeof(int4));
    put(C.o_ftask, L.ftasks.data(), L.ftasks.size() * sizeof(int2));
    put(C.o_btask, L.btasks.data(), L.btasks.size() * sizeof(int2));
    put(C.o_perm, P.perm.data(), (size_t)N * 8);
    put(C.o_ztiles, L.ztiles.data(), L.ztiles.size() * sizeof(int4));
    put(C.o_tb, L.tb.data(), L.tb.size() * 4);
    {
        std::atomic<size_t> next{0};
        auto copy = [&] {
            for (size_t i; (i = next.fetch_add(1)) < pieces.size();) memcpy(hp + pieces[i].o, pieces[i].p, pieces[i].b);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < 4 && (size_t)t < pieces.size(); ++t) pool.emplace_back(copy);
        copy();
        for (auto& th : pool) th.join();
    }
    // the per-tile marks: the pivot columns' diagonal tiles (their padding
    // pivots' identity, nd_pad_pivots), then nd_mark_tiles on the device
    memset(hp + C.o_zf, 0, (size_t)L.n_lower);
    // (and every tile of a whole-front task: nd_factor reads those tiles as
    // they are)
    for (const NdDev& d : L.dev) {
        if (d.nt <= (small_nt & 0xffff)) {
            memset(hp + C.o_zf + d.tile_off, 1, (size_t)d.nt * (d.nt + 1) / 2);
            continue;
        }
        for (int32_t K = 0; K < d.npt; ++K) hp[C.o_zf + d.tile_off + nd_lower_idx(d.nt, K, K)] = 1;
    }
    C.ms_pack = ms_since(tp0);
    if (C.plan.bytes < total) BSM_TRY(C.plan.alloc(total));
    BSM_HIP_TRY(hipMemcpyAsync(C.plan.p, hp, total, hipMemcpyHostToDevice, s));
    {
        char* pb = C.plan.as<char>();
        uint8_t* zf = (uint8_t*)(pb + C.o_zf);
        nd_mark_tiles<<<nd_blocks(N, 256), 256, 0, s>>>(N, a->row_ptr, a->col, (const int32_t*)(pb + C.o_pinv),
                                                        (const int32_t*)(pb + C.o_owner), (const NdDev*)(pb + C.o_dev),
                                                        (const int32_t*)(pb + C.o_st), zf);
        BSM_HIP_TRY(hipGetLastError());
        if (C.n_tiles) {
            nd_mark_tasks<<<nd_blocks((int64_t)C.n_tiles, 256), 256, 0, s>>>((int64_t)C.n_tiles,
                                                                             (const NdDev*)(pb + C.o_dev), zf,
                                                                             (int4*)(pb + C.o_tiles));
            BSM_HIP_TRY(hipGetLastError());
        }
    }
    // A's entries by tile: count, scan, fill; the factor tasks' ranges (the
    // offsets are 32-bit: a pattern with 2^31 or more lower entries keeps
    // the zeroing and the assembly instead, BSM_ND_APULL=0's path)
    if (a->nnz < ((uint64_t)1 << 31)) {
        char* pb = C.plan.as<char>();
        const int32_t* d_pinv = (const int32_t*)(pb + C.o_pinv);
        const int32_t* d_owner = (const int32_t*)(pb + C.o_owner);
        const NdDev* d_dev = (const NdDev*)(pb + C.o_dev);
        const int32_t* d_st = (const int32_t*)(pb + C.o_st);
        // every buffer first: an error return after a launch would free
        // buffers queued kernels still write (and the guard drains the stream)
        DBuf cnt;
        BSM_TRY(cnt.alloc((size_t)std::max<int64_t>(2 * C.n_lower, 1) * sizeof(int32_t), s));
        BSM_TRY(C.aoff.alloc((size_t)(C.n_lower + 1) * sizeof(int32_t)));
        BSM_TRY(C.aent.alloc((size_t)std::max<uint64_t>(a->nnz, 1) * sizeof(int64_t)));
        BSM_TRY(C.tq.alloc((size_t)std::max<size_t>(C.n_tiles, 1) * sizeof(int2)));
        BSM_TRY(C.pdesc.alloc((size_t)std::max<size_t>(C.n_tiles, 1) * 2 * sizeof(NdPull)));
        struct Drain {
            hipStream_t s;
            ~Drain() { (void)hipStreamSynchronize(s); }
        } drain{s};
        BSM_HIP_TRY(hipMemsetAsync(cnt.p, 0, (size_t)std::max<int64_t>(2 * C.n_lower, 1) * sizeof(int32_t), s));
        int32_t* d_cnt = cnt.as<int32_t>();
        nd_aent_count<<<nd_blocks(N, 256), 256, 0, s>>>(N, a->row_ptr, a->col, d_pinv, d_owner, d_dev, d_st, d_cnt);
        BSM_HIP_TRY(hipGetLastError());
        nd_scan_tiles<<<1, 1024, 0, s>>>(C.n_lower, d_cnt, C.aoff.as<int32_t>());
        BSM_HIP_TRY(hipGetLastError());
        nd_aent_fill<<<nd_blocks(N, 256), 256, 0, s>>>(N, a->row_ptr, a->col, d_pinv, d_owner, d_dev, d_st,
                                                       C.aoff.as<int32_t>(), d_cnt + C.n_lower, C.aent.as<int64_t>());
        BSM_HIP_TRY(hipGetLastError());
        if (C.n_tiles) {
            nd_task_ranges<<<nd_blocks((int64_t)C.n_tiles, 256), 256, 0, s>>>(
                (int64_t)C.n_tiles, (const int4*)(pb + C.o_tiles), d_dev, C.aoff.as<int32_t>(), C.tq.as<int2>());
            BSM_HIP_TRY(hipGetLastError());
            nd_task_pull<<<nd_blocks((int64_t)C.n_tiles, 256), 256, 0, s>>>(
                (int64_t)C.n_tiles, (const int4*)(pb + C.o_tiles), d_dev, (const int32_t*)(pb + C.o_tb),
                C.pdesc.as<NdPull>());
            BSM_HIP_TRY(hipGetLastError());
        }
        int32_t na = 0;
        BSM_HIP_TRY(hipMemcpyAsync(&na, C.aoff.as<int32_t>() + C.n_lower, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipStreamSynchronize(s));  // also: the staging buffer is reused by the next plan
        C.n_aent = na;
    }
    stage_mark("nd_upload", s);
    if (pre_fronts.joinable()) {  // the fronts' allocation: the wait for it as a stage of its own
        pre_fronts.join();
        stage_mark("nd_fronts_alloc", s);
    }
    return BSM_OK;
}

size_t nd_pattern_rp_bytes(int64_t n) { return ((size_t)(n + 1) * sizeof(int64_t) + 255) / 256 * 256; }

// the pattern's key (synchronous on s: a ~6M-element pass at C5, ~10 us)
int nd_pattern_key(const bsm_csr* a, int64_t leaf, int32_t small_nt, hipStream_t s, NdKey& key) {
    const int64_t n = (int64_t)a->rows, total = n + 1 + (int64_t)a->nnz;
    key.device = a->device;
    key.small_nt = small_nt;
    key.n = n;
    key.leaf = leaf;
    key.nnz = a->nnz;
    DBuf hb;
    BSM_TRY(hb.alloc(16, s));
    BSM_HIP_TRY(hipMemsetAsync(hb.p, 0, 16, s));
    nd_pattern_hash<<<(unsigned)std::min<int64_t>((total + 255) / 256, 1024), 256, 0, s>>>(
        a->row_ptr, n + 1, a->col, (int64_t)a->nnz, hb.as<unsigned long long>());
    BSM_HIP_TRY(hipGetLastError());
    uint64_t h[2] = {0, 0};
    BSM_HIP_TRY(read_dev(h, hb.p, 16, s));
    key.h0 = h[0];
    key.h1 = h[1];
    const char* hz = getenv("BSM_ND_HASH_ZERO");  // tests: every pattern of one (n, nnz) collides
    if (hz && atoi(hz) == 1) key.h0 = key.h1 = 0;
    return BSM_OK;
}

// Drop kept numeric storage, least recently used first, until the entries'
// total is at most `budget` bytes; `keep` and storage a running solve holds
// stay. The caller holds the cache's mutex.
void nd_cache_trim_locked(NdCache& c, size_t budget, const NdCached* keep) {
    std::vector<NdCacheEntry*> by_age;
    size_t total = 0;
    for (auto& e : c.entries) {
        total += e.plan->kept_bytes;
        by_age.push_back(&e);
    }
    std::sort(by_age.begin(), by_age.end(), [](auto* x, auto* y) { return x->tick < y->tick; });
    for (NdCacheEntry* e : by_age) {
        if (total <= budget) break;
        if (e->plan.get() == keep) continue;
        const size_t b = e->plan->kept_bytes;
        if (b && e->plan->release_numeric()) total -= b;
    }
}

void nd_cache_trim(size_t budget, const NdCached* keep) {
    NdCache& c = nd_cache();
    std::lock_guard<std::mutex> l(c.mu);
    nd_cache_trim_locked(c, budget, keep);
}

// A cached plan for this pattern (confirmed against the entry's copy of the
// pattern), or null
int nd_cache_find(const bsm_csr* a, const NdKey& key, hipStream_t s, std::shared_ptr<NdCached>& out) {
    out.reset();
    NdCache& c = nd_cache();
    std::shared_ptr<DBuf> pat;
    std::shared_ptr<NdCached> plan;
    {
        std::lock_guard<std::mutex> l(c.mu);
        for (auto& e : c.entries)
            if (e.key == key) {
                e.tick = ++c.tick;
                pat = e.pattern;
                plan = e.plan;
                break;
            }
    }
    if (plan) {
        const int64_t n1 = key.n + 1, total = n1 + (int64_t)key.nnz;
        const char* pb = pat->as<char>();
        DBuf db;
        BSM_TRY(db.alloc(4, s));
        BSM_HIP_TRY(hipMemsetAsync(db.p, 0, 4, s));
        nd_pattern_diff<<<(unsigned)std::min<int64_t>((total + 255) / 256, 4096), 256, 0, s>>>(
            a->row_ptr, (const int64_t*)pb, n1, a->col, (const int32_t*)(pb + nd_pattern_rp_bytes(key.n)),
            (int64_t)key.nnz, db.as<int>());
        BSM_HIP_TRY(hipGetLastError());
        int diff = 1;
        BSM_HIP_TRY(read_dev(&diff, db.p, 4, s));
        if (!diff) out = plan;
    }
    std::lock_guard<std::mutex> l(c.mu);
    ++(out ? c.hits : c.misses);
    return BSM_OK;
}

int nd_cache_insert(const bsm_csr* a, const NdKey& key, const std::shared_ptr<NdCached>& plan, hipStream_t s) {
    auto pat = std::make_shared<DBuf>();
    const size_t rpb = nd_pattern_rp_bytes(key.n);
    BSM_TRY(pat->alloc(rpb + (size_t)key.nnz * sizeof(int32_t)));
    BSM_HIP_TRY(hipMemcpyAsync(pat->p, a->row_ptr, (size_t)(key.n + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    if (key.nnz)
        BSM_HIP_TRY(hipMemcpyAsync(pat->as<char>() + rpb, a->col, (size_t)key.nnz * sizeof(int32_t),
                                   hipMemcpyDeviceToDevice, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));  // a lookup on another stream may compare against it next
    NdCache& c = nd_cache();
    std::lock_guard<std::mutex> l(c.mu);
    c.entries.erase(std::remove_if(c.entries.begin(), c.entries.end(),
                                   [&](const NdCacheEntry& e) { return e.key == key; }),
                    c.entries.end());
    NdCacheEntry e;
    e.key = key;
    e.tick = ++c.tick;
    e.pattern = std::move(pat);
    e.plan = plan;
    c.entries.push_back(std::move(e));
    const size_t cap = std::max<size_t>(1, nd_cache_limit("BSM_ND_CACHE_ENTRIES", 4));
    while (c.entries.size() > cap) {
        auto old = std::min_element(c.entries.begin(), c.entries.end(),
                                    [](const NdCacheEntry& x, const NdCacheEntry& y) { return x.tick < y.tick; });
        c.entries.erase(old);  // a handle still holding the plan keeps it alive
    }
    return BSM_OK;
}

// Numeric storage for a solve: on BSM_ERR_OOM, drop every other cached
// plan's kept storage and try once more
int nd_alloc_numeric(DBuf& b, size_t bytes, const NdCached* keep) {
    if (b.bytes == bytes) return BSM_OK;
    int rc = b.alloc(bytes);
    if (rc == BSM_ERR_OOM) {
        nd_cache_trim(0, keep);
        rc = b.alloc(bytes);
    }
    return rc;
}

// Waits for the stream when an error return leaves kernels queued that
// write the kept numeric storage, so no other solve takes that storage
// (num_mu is released after this guard runs) while they still run.
struct NdDrainOnError {
    hipStream_t s;
    bool armed = false;
    ~NdDrainOnError() {
        if (armed) (void)hipStreamSynchronize(s);
    }
};

template <typename T>
int nd_solve(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev, hipStream_t s) {
    stage_reset(s);
    const int64_t N = (int64_t)n;
    const char* le = getenv("BSM_ND_LEAF");
    const char* ce = getenv("BSM_ND_CACHE");
    const char* she = getenv("BSM_ND_SHARED");
    const int64_t leaf = le ? atoll(le) : 192;  // C5 leaf sweep: 128 / 192 / 256 / 320 -> 11.9 / 11.4 / 12.3 / 12.5 ms
    const bool cache = !(ce && atoi(ce) == 0);
    const bool shared = cache && !(she && atoi(she) == 0);  // the cache across handles (BSM_ND_SHARED=0: off)
    // BSM_ND_FRONT_NT=n: fronts of at most n tile rows factor as one task
    // each (C5: most fronts of levels 0-4 have 2-4). Default 0, every front by
    // tiles: measured at C5, n = 3 matches it and n = 4 / 5 are 0.25 / 0.5 ms
    // slower (a middle level's 10-15 tiles in a row on one workgroup cost more
    // than the tickets and flags they save; profiles/r06_b_*)
    const char* fne = getenv("BSM_ND_FRONT_NT");
    // BSM_ND_EXT_MERGE=0: one extend launch per child slot (A/B; same bits)
    const char* eme = getenv("BSM_ND_EXT_MERGE");
    const bool ext_merge = !(eme && atoi(eme) == 0);
    // the layout's options (nd_layout's `lay`): part of the plan's keys
    // BSM_ND_LAG=u: a front's tiles below the diagonal trail its diagonal
    // tile by u fronts' diagonals (nd_layout; 0: all diagonals of a column
    // first, the round-5 order)
    const char* lge = getenv("BSM_ND_LAG");
    const int32_t lag_units = std::min(0x7ff, std::max(0, lge ? atoi(lge) : 512));
    // BSM_ND_PULL=0: the children's update blocks added by nd_extend2 /
    // nd_extend launches after each level (round 5) instead of inside the
    // parent's nd_factor tiles (same bits)
    const char* pue = getenv("BSM_ND_PULL");
    const bool pull = !(pue && atoi(pue) == 0);
    const int32_t small_nt =
        (fne ? atoi(fne) : 0) | (ext_merge ? 0 : 1 << 16) | (lag_units << 17) | (pull ? 0 : 1 << 28);
    std::shared_ptr<NdCached> pc;
    if (cache) {
        std::lock_guard<std::mutex> lk(a->plan_mu);
        auto c = std::static_pointer_cast<NdCached>(a->nd_plan);
        if (c && c->leaf == leaf && c->small_nt == small_nt) pc = c;
    }
    NdKey key;
    if (pc) {
        stage_mark("nd_plan_cached", s);
    } else {
        if (shared) {
            BSM_TRY(nd_pattern_key(a, leaf, small_nt, s, key));
            BSM_TRY(nd_cache_find(a, key, s, pc));
            stage_mark(pc ? "nd_plan_shared" : "nd_pattern_key", s);
        }
        if (!pc) {
            pc = std::make_shared<NdCached>();
            const char* ke0 = getenv("BSM_ND_KEEP");
            const bool prealloc = cache && !(ke0 && atoi(ke0) == 0);  // the fronts will be this plan's own
            BSM_TRY(nd_build_plan(a, leaf, small_nt, prealloc ? sizeof(T) : 0, s, *pc));
            if (shared) BSM_TRY(nd_cache_insert(a, key, pc, s));
        }
        if (cache) {
            std::lock_guard<std::mutex> lk(a->plan_mu);
            a->nd_plan = pc;
        }
    }
    NdCached& C = *pc;
    if (getenv("BSM_ND_TRACE"))
        fprintf(stderr,
                "[bsm nd] n %lld nodes %d levels %d: graph %.1f ms, bisection %.1f ms, symbolic %.1f ms, layout "
                "%.1f ms, packing %.1f ms; fronts %.3f GB (largest %lld), tiles %zu, extend columns %zu\n",
                (long long)N, C.nn, C.n_levels, C.ms_graph, C.ms_order, C.ms_symbolic, C.ms_layout, C.ms_pack,
                (double)C.f_elems * sizeof(T) * 1e-9, (long long)C.max_front, C.n_tiles, C.n_ext);
    char* pb = C.plan.as<char>();
    const NdDev* d_nodes = (const NdDev*)(pb + C.o_dev);
    const int32_t* d_st = (const int32_t*)(pb + C.o_st);
    const int32_t* d_ri = (const int32_t*)(pb + C.o_ri);
    const int32_t* d_pinv = (const int32_t*)(pb + C.o_pinv);
    const int32_t* d_owner = (const int32_t*)(pb + C.o_owner);
    const int32_t* d_lvl = (const int32_t*)(pb + C.o_lvl);
    const int4* d_tiles = (const int4*)(pb + C.o_tiles);
    const int4* d_ztiles = (const int4*)(pb + C.o_ztiles);
    const int2* d_ext = (const int2*)(pb + C.o_ext);
    const int4* d_ext2 = (const int4*)(pb + C.o_ext2);
    const int2* d_ftask = (const int2*)(pb + C.o_ftask);
    const int2* d_btask = (const int2*)(pb + C.o_btask);
    const int64_t* d_perm = (const int64_t*)(pb + C.o_perm);
    const int32_t* d_tb = pull ? (const int32_t*)(pb + C.o_tb) : nullptr;
    // BSM_ND_ZSKIP=0: every lower tile zeroed and read (A/B; same bits). By
    // default, with the pulled extend-add, only the tiles A's entries land in
    const char* zse = getenv("BSM_ND_ZSKIP");
    const int zskip = pull && !(zse && atoi(zse) == 0);
    const uint8_t* d_zf = zskip ? (const uint8_t*)(pb + C.o_zf) : nullptr;
    // BSM_ND_FOLD=0: the forward solve as its own pass over L after the
    // factor. By default, with one right-hand side and the pull, the
    // factor's diagonal tiles form y and the update vectors themselves
    // BSM_ND_APULL=0: the fronts zeroed (the marked tiles) and A assembled
    // into them before the factor. By default, with the pull, each factor
    // tile stages its own A entries from the plan's per-tile lists
    const char* ape = getenv("BSM_ND_APULL");
    const bool apull = pull && C.aent.p && !(ape && atoi(ape) == 0);
    const char* foe = getenv("BSM_ND_FOLD");
    const bool fold = k == 1 && pull && !(foe && atoi(foe) == 0);
    // numeric storage: the plan's own buffers when this solve may hold them
    const char* ke = getenv("BSM_ND_KEEP");
    std::unique_lock<std::mutex> num_lock(C.num_mu, std::defer_lock);
    const bool keep = cache && !(ke && atoi(ke) == 0) && num_lock.try_lock();
    DBuf own_fr, own_dv, own_fl;
    DBuf& fr = keep ? C.fr : own_fr;
    DBuf& dv = keep ? C.dv : own_dv;
    DBuf& fl = keep ? C.fl : own_fl;
    const size_t fr_b = (size_t)C.f_elems * sizeof(T), dv_b = (size_t)std::max<int64_t>(C.dinv_elems, 1) * sizeof(T);
    const size_t nfl = (size_t)C.n_flags + (size_t)C.n_levels + 2;
    // a plan serves one dtype per handle; sizes match after the first solve
    const void* fr_was = fr.p;
    BSM_TRY(nd_alloc_numeric(fr, fr_b, &C));
    if (keep && fr.p != fr_was) C.drop_zeroed();  // reallocated: zeroed by nd_zero_tiles as usual
    const char* poe = getenv("BSM_ND_POISON");  // tests: the fronts start as NaN (nothing may read unzeroed tiles)
    if (poe && atoi(poe) == 1) {
        if (C.fr_zeroed) hipStreamWaitEvent(s, C.fr_zeroed, 0);
        C.drop_zeroed();
        BSM_HIP_TRY(hipMemsetAsync(fr.p, 0xff, fr_b, s));
    }
    BSM_TRY(nd_alloc_numeric(dv, dv_b, &C));
    BSM_TRY(nd_alloc_numeric(fl, nfl * sizeof(int), &C));
    if (keep) C.kept_bytes = fr.bytes + dv.bytes + fl.bytes;
    // everything that can fail before the first launch: the occupancy
    // queries and the solves' temporaries (an error return after
    // the launches would release num_mu under running kernels)
    int dev = 0, cus = 0, per_cu = 0, fper = 0, bper = 0;
    BSM_HIP_TRY(hipGetDevice(&dev));
    BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nd_factor<T>, 256, 0));
    BSM_REQUIRE(per_cu >= 1, BSM_ERR_UNSUPPORTED, "nd_factor does not fit a CU");
    BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&fper, nd_forward_tiles<T>, 64, 0));
    BSM_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bper, nd_backward_tiles<T>, 256, 0));
    BSM_REQUIRE(fper >= 1 && bper >= 1, BSM_ERR_UNSUPPORTED, "nd solve kernels do not fit a CU");
    const int64_t n_pf = (C.dinv_elems / 4096) * (int64_t)k;  // flags per pass: one per node, column, pivot tile
    const size_t n_tf = 2 * (size_t)n_pf + 2 * (size_t)C.n_levels;  // forward flags, backward flags, tickets
    DBuf bpb, vb, tfl, avb;  // from the thread's cache of temporaries (no hipFree per solve)
    if (apull) BSM_TRY(avb.alloc((size_t)std::max<int64_t>(C.n_aent, 1) * sizeof(T), s));
    if (k > 0) {
        BSM_TRY(bpb.alloc((size_t)N * k * sizeof(T), s));
        BSM_TRY(vb.alloc((size_t)std::max<int64_t>(C.vtot, 1) * k * sizeof(T), s));
        BSM_TRY(tfl.alloc(n_tf * sizeof(int), s));
    }
    NdDrainOnError drain{s};  // destroyed before num_lock is released
    drain.armed = true;
    BSM_HIP_TRY(hipMemsetAsync(fl.p, 0, nfl * sizeof(int), s));
    int* d_flags = fl.as<int>();
    int* d_tickets = d_flags + C.n_flags;
    int* d_status = d_tickets + C.n_levels;
    T* F = fr.as<T>();
    if (keep && C.fr_zeroed) {  // the plan's first solve: fr is zeroed whole on another stream
        const hipEvent_t ev = C.fr_zeroed;
        C.fr_zeroed = nullptr;
        const hipError_t we = hipStreamWaitEvent(s, ev, 0);
        (void)hipEventDestroy(ev);
        BSM_HIP_TRY(we);
    } else if (C.n_ztiles && !apull) {
        nd_zero_tiles<T><<<(unsigned)C.n_ztiles, 256, 0, s>>>(d_nodes, d_ztiles, F, d_zf);
        BSM_HIP_TRY(hipGetLastError());
    }
    if (apull) {  // A's values in the per-tile lists' order
        if (C.n_aent > 0) {
            nd_aent_vals<T><<<nd_blocks(C.n_aent, 256), 256, 0, s>>>(C.n_aent, C.aent.as<int64_t>(),
                                                                    static_cast<const T*>(a->vals), avb.as<T>());
            BSM_HIP_TRY(hipGetLastError());
        }
    } else {
        nd_assemble<T><<<nd_blocks(N, 256), 256, 0, s>>>(N, a->row_ptr, a->col, static_cast<const T*>(a->vals),
                                                         d_pinv, d_owner, d_nodes, d_st, F);
        BSM_HIP_TRY(hipGetLastError());
        nd_pad_pivots<T><<<(unsigned)C.nn, 64, 0, s>>>(d_nodes, F);
        BSM_HIP_TRY(hipGetLastError());
    }
    stage_mark("nd_assemble", s);
    const int64_t* const d_aent = apull ? C.aent.as<int64_t>() : nullptr;
    const T* const d_av = apull ? avb.as<T>() : nullptr;
    const int32_t* const d_aoff = apull ? C.aoff.as<int32_t>() : nullptr;
    const int2* const d_tq = apull ? C.tq.as<int2>() : nullptr;
    // BSM_ND_PDESC=0: the pull finds its children's blocks through the
    // node, the child and the bounds (A/B; same bits)
    const char* pde = getenv("BSM_ND_PDESC");
    const NdPull* const d_pd = pull && C.pdesc.p && !(pde && atoi(pde) == 0) ? C.pdesc.as<NdPull>() : nullptr;
    // BSM_ND_STAMPS=1: nd_factor's per-level cycle stamps, printed after the solve
    const char* sde = getenv("BSM_ND_STAMPS");
    DBuf stamps;
    if (sde && atoi(sde) == 1) {
        BSM_TRY(stamps.alloc((size_t)C.n_levels * ND_NSTAMP * sizeof(unsigned long long)));
        BSM_HIP_TRY(hipMemsetAsync(stamps.p, 0, (size_t)C.n_levels * ND_NSTAMP * sizeof(unsigned long long), s));
    }
    if (fold) {  // b into the new order before the factor; V's padding rows stay 0
        nd_gather<T><<<nd_blocks(N, 256), 256, 0, s>>>(N, (int64_t)k, d_perm, static_cast<const T*>(b_dev),
                                                       bpb.as<T>());
        BSM_HIP_TRY(hipGetLastError());
        BSM_HIP_TRY(hipMemsetAsync(vb.p, 0, (size_t)std::max<int64_t>(C.vtot, 1) * sizeof(T), s));
    }
    T* const fV = fold ? vb.as<T>() : nullptr;
    const T* const fbp = fold ? bpb.as<T>() : nullptr;
    // BSM_ND_PAD_SKIP=0: diagonal tiles factor their padding panels too (A/B; same bits)
    const char* pse = getenv("BSM_ND_PAD_SKIP");
    const int pad_skip = !(pse && atoi(pse) == 0);
    for (int32_t lv = 0; lv < C.n_levels; ++lv) {
        const int64_t t0 = C.tiles_off[(size_t)lv], nt = C.tiles_off[(size_t)lv + 1] - t0;
        if (nt > 0) {
            const int64_t grid = std::min<int64_t>(nt, (int64_t)cus * per_cu);
            if (stamps.p)
                nd_factor<T, true><<<(unsigned)grid, 256, 0, s>>>(d_nodes, d_tiles + t0, nt, F, dv.as<T>(), d_flags,
                                                                  d_tickets + lv, d_status, pad_skip, d_tb, d_ri,
                                                                  zskip, fV, fbp, d_aent, d_av, d_aoff, d_tq ? d_tq + t0 : nullptr,
                                                                  d_pd ? d_pd + 2 * t0 : nullptr,
                                                                  stamps.as<unsigned long long>() + ND_NSTAMP * lv);
            else
                nd_factor<T><<<(unsigned)grid, 256, 0, s>>>(d_nodes, d_tiles + t0, nt, F, dv.as<T>(), d_flags,
                                                            d_tickets + lv, d_status, pad_skip, d_tb, d_ri, zskip,
                                                            fV, fbp, d_aent, d_av, d_aoff, d_tq ? d_tq + t0 : nullptr,
                                                            d_pd ? d_pd + 2 * t0 : nullptr);
            BSM_HIP_TRY(hipGetLastError());
        }
        if (ext_merge && !pull) {
            const int64_t e0 = C.ext2_off[(size_t)lv], ne = C.ext2_off[(size_t)lv + 1] - e0;
            if (ne > 0) {
                nd_extend2<T><<<nd_blocks(ne, 4), 256, 0, s>>>(d_nodes, d_ext2 + e0, ne, d_ri, F);
                BSM_HIP_TRY(hipGetLastError());
            }
        }
        for (int sl = 0; sl < 2 && !ext_merge && !pull; ++sl) {
            const int64_t e0 = C.ext_off[(size_t)(2 * lv + sl)], ne = C.ext_off[(size_t)(2 * lv + sl) + 1] - e0;
            if (ne <= 0) continue;
            nd_extend<T><<<nd_blocks(ne, 4), 256, 0, s>>>(d_nodes, d_ext + e0, ne, d_ri, F);
            BSM_HIP_TRY(hipGetLastError());
        }
    }
    stage_mark("nd_factor", s);
    if (k > 0) {
        if (!fold) {
            nd_gather<T><<<nd_blocks(N, 256), 256, 0, s>>>(N, (int64_t)k, d_perm, static_cast<const T*>(b_dev),
                                                           bpb.as<T>());
            BSM_HIP_TRY(hipGetLastError());
        }
        // Levels with fewer (node, column) pairs than CUs run their solves by
        // tiles (nd_forward_tiles / nd_backward_tiles: a front's chain of pivot
        // tiles on many waves), the others one workgroup per pair (nd_forward /
        // nd_backward: less bookkeeping per front). Same bits either way.
        // BSM_ND_FWD_TILES / BSM_ND_BWD_TILES = 0: never, 1: every level.
        const char* fte = getenv("BSM_ND_FWD_TILES");
        const char* bte = getenv("BSM_ND_BWD_TILES");
        const int fwd_mode = fte ? atoi(fte) : 2, bwd_mode = bte ? atoi(bte) : 2;
        auto by_tiles = [&](int mode, int64_t pairs) { return mode == 1 || (mode == 2 && pairs < cus); };
        BSM_HIP_TRY(hipMemsetAsync(tfl.p, 0, n_tf * sizeof(int), s));
        int* const d_yf = tfl.as<int>();
        int* const d_xf = d_yf + n_pf;
        int* const d_ftk = d_xf + n_pf;
        int* const d_btk = d_ftk + C.n_levels;
        const int64_t fwd_grid = (int64_t)cus * fper, bwd_grid = (int64_t)cus * bper;
        for (int32_t lv = 0; lv < C.n_levels && !fold; ++lv) {
            const int64_t o = C.lvl_off[(size_t)lv], c = C.lvl_off[(size_t)lv + 1] - o;
            if (c <= 0) continue;
            if (by_tiles(fwd_mode, c * (int64_t)k)) {
                const int64_t f0 = C.ftask_off[(size_t)lv], nf = C.ftask_off[(size_t)lv + 1] - f0;
                const int64_t grid = std::min<int64_t>(nf * (int64_t)k, fwd_grid);
                if (grid <= 0) continue;  // fronts without rows (no pivots, no front rows)
                nd_forward_tiles<T><<<(unsigned)grid, 64, 0, s>>>(d_nodes, d_ftask + f0, nf, (int)k, N, bpb.as<T>(),
                                                                  vb.as<T>(), C.vtot, F, dv.as<T>(), d_ri, d_yf,
                                                                  d_ftk + lv, d_status);
            } else {
                nd_forward<T><<<dim3((unsigned)c, (unsigned)k), 256, 0, s>>>(d_nodes, d_lvl + o, N, bpb.as<T>(),
                                                                            vb.as<T>(), C.vtot, F, dv.as<T>(), d_ri);
            }
            BSM_HIP_TRY(hipGetLastError());
        }
        stage_mark("nd_forward", s);
        for (int32_t lv = C.n_levels - 1; lv >= 0; --lv) {
            const int64_t o = C.lvl_off[(size_t)lv], c = C.lvl_off[(size_t)lv + 1] - o;
            if (c <= 0) continue;
            if (by_tiles(bwd_mode, c * (int64_t)k)) {
                const int64_t b0 = C.btask_off[(size_t)lv], nb = C.btask_off[(size_t)lv + 1] - b0;
                const int64_t grid = std::min<int64_t>(nb * (int64_t)k, bwd_grid);
                if (grid <= 0) continue;  // no pivots on this level
                nd_backward_tiles<T><<<(unsigned)grid, 256, 0, s>>>(d_nodes, d_btask + b0, nb, (int)k, N,
                                                                    bpb.as<T>(), vb.as<T>(), C.vtot, F, dv.as<T>(),
                                                                    d_st, d_xf, d_btk + lv, d_status);
            } else {
                nd_backward<T><<<dim3((unsigned)c, (unsigned)k), 256, 0, s>>>(d_nodes, d_lvl + o, N, bpb.as<T>(),
                                                                             vb.as<T>(), C.vtot, F, dv.as<T>(), d_st);
            }
            BSM_HIP_TRY(hipGetLastError());
        }
        stage_mark("nd_backward", s);
        nd_scatter<T><<<nd_blocks(N, 256), 256, 0, s>>>(N, (int64_t)k, d_perm, bpb.as<T>(), static_cast<T*>(x_dev));
        BSM_HIP_TRY(hipGetLastError());
    }
    int h = 0;
    BSM_HIP_TRY(read_dev(&h, d_status, sizeof(int), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    stage_mark("nd_copy_out", s);
    if (stamps.p) {
        std::vector<unsigned long long> h((size_t)C.n_levels * ND_NSTAMP);
        BSM_HIP_TRY(hipMemcpy(h.data(), stamps.p, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (int32_t lv = 0; lv < C.n_levels; ++lv) {
            const unsigned long long* v = &h[(size_t)lv * ND_NSTAMP];
            const double nt = v[7] ? (double)v[7] : 1.0;
            fprintf(stderr,
                    "[bsm nd stamps] level %2d: %6llu tiles (prod %llu, diag %llu, trsm %llu, upd %llu); cycles per "
                    "tile: wait %.0f, products %.0f, diag %.0f, trsm %.0f, update %.0f, drain %.0f; workgroup total "
                    "%.0f per tile\n",
                    lv, v[7], v[8], v[9], v[10], v[11], v[1] / nt, (v[2] - v[1]) / nt, v[3] / nt, v[4] / nt,
                    v[5] / nt, v[6] / nt, v[0] / nt);
            if (v[16])
                fprintf(stderr,
                        "[bsm nd stamps] level %2d: pull into %llu tiles, cycles per pulling tile: tile and first "
                        "child's loads %.0f, its additions %.0f, second child %.0f, read-back %.0f\n",
                        lv, v[16], (double)v[12] / v[16], (double)v[13] / v[16], (double)v[14] / v[16],
                        (double)v[15] / v[16]);
        }
    }
    BSM_REQUIRE(!(h & ST_TIMEOUT), BSM_ERR_HIP, "nd factor: tile hand-off timed out");
    BSM_REQUIRE(!(h & ST_NOT_PD), BSM_ERR_UNSUPPORTED,
                "cholesky: matrix is not positive definite (a pivot is <= 0 or not finite)");
    if (keep && shared) {  // the cached plans' kept storage within its budget (this plan's stays)
        num_lock.unlock();
        nd_cache_trim(nd_cache_limit("BSM_ND_CACHE_MB", 32768) << 20, &C);
    }
    return BSM_OK;
}

}  // namespace

// solve (lib.rs:11-24) by the nested-dissection multifrontal factorisation
int solve_dispatch_nd(const bsm_csr* a, uint64_t k, uint64_t n, const void* b_dev, void* x_dev, hipStream_t s) {
    BSM_REQUIRE(a->rows == n, BSM_ERR_PANIC,
                "solve: b has %llu rows but A has %llu (index out of bounds in the reference)", (unsigned long long)n,
                (unsigned long long)a->rows);
    BSM_REQUIRE(n < ((uint64_t)1 << 31), BSM_ERR_UNSUPPORTED, "solve nd: n >= 2^31");
    if (n == 0) return BSM_OK;
    if (a->dtype == BSM_F64) return nd_solve<double>(a, k, n, b_dev, x_dev, s);
    if (a->dtype == BSM_F32) return nd_solve<float>(a, k, n, b_dev, x_dev, s);
    set_error("solve: f32/f64 only");
    return BSM_ERR_INVALID;
}

}  // namespace bsm

// ---- C-ABI: the nd plan cache across handles ----
extern "C" int bsm_nd_cache_clear(void) {
    bsm::NdCache& c = bsm::nd_cache();
    std::vector<bsm::NdCacheEntry> gone;
    {
        std::lock_guard<std::mutex> l(c.mu);
        gone.swap(c.entries);
    }
    return BSM_OK;  // `gone` frees outside the lock (a handle still holding a plan keeps it)
}

extern "C" int bsm_nd_cache_info(uint64_t* entries, uint64_t* kept_bytes, uint64_t* hits, uint64_t* misses) {
    bsm::NdCache& c = bsm::nd_cache();
    std::lock_guard<std::mutex> l(c.mu);
    uint64_t kb = 0;
    for (const auto& e : c.entries) kb += e.plan->kept_bytes;
    if (entries) *entries = c.entries.size();
    if (kept_bytes) *kept_bytes = kb;
    if (hits) *hits = c.hits;
    if (misses) *misses = c.misses;
    return BSM_OK;
}
