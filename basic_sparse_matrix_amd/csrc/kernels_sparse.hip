// kernels_sparse.hip -- sparse x sparse operations of the reference
// (SURVEY.md §8f-4): Csr::add_sparse / sub_sparse (sparse.rs:484-599) and
// Csr::mul_sparse (sparse.rs:601-635), bit-exact for every input, including
// rows with unsorted or repeated columns (the reference's bench builds such
// rows: random insert order).
//
// add / sub: the reference merges row r of both operands with two pointers
// over their entries in STORAGE order (the smaller column goes out first, an
// equal column goes out once as the sum / difference, for sub an rhs-only
// entry is T::default() - v), each output through the zero-skipping insert.
// One thread per row runs that merge twice: once to count the kept outputs
// (then an exclusive scan gives row_ptr), once to write them.
// Long rows (the benches' running-max rule piles ~all entries into one row,
// with columns in random order) are cut into independent pieces first. Let
// M be the largest column of the two rows: the merge never passes an M on
// one side before pairing it with the next M of the other side (every other
// value is smaller), so the k-th M of the self row pairs with the k-th M of
// the rhs row, and the stretches between consecutive pairs merge on their
// own, in order. Piece k = (self stretch k, rhs stretch k, the k-th M pair);
// the last piece is the two tails (standard merge, M left over on at most one
// side). Each piece is one thread's sequential merge; results are identical
// to the whole-row merge (checked against the literal oracle).
//
// mul: the reference visits every (row, col) pair of the result and merges
// the self row (storage order) with row `col` of rhs.transpose(); val starts
// at T::default(), gains the product of each equal-column step in merge
// order, and is inserted when nonzero. On the device:
//   1. rhs_t = transpose(rhs) (the stable device transpose);
//   2. candidates: every (i, j) that can have an equal-column step pairs an
//      entry (i, k) of self with an entry (k, j) of rhs. Expand those
//      (balanced: one thread per expanded slot, binary search on the scan of
//      the per-entry counts), radix-sort the keys (i, j) and keep the unique
//      ones -- ascending i then j, the reference's output order;
//   3. per candidate, the literal merge (so duplicate or unsorted columns
//      skip exactly the steps the reference skips);
//   4. keep val != default: a flag scan, a scatter, row_ptr by binary search.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>

#include <cstring>
#include <vector>

#include "bsm_internal.hpp"

namespace bsm {
namespace {

unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

unsigned bits_for(uint64_t x) {  // bits to hold values < x
    unsigned b = 0;
    while (b < 64 && (x - 1) >> b) ++b;
    return b;
}

// ---- add / sub -------------------------------------------------------------
// The reference's merge of self entries [ia, ea) with rhs entries [ib, eb);
// emit(col, value) for every output it inserts (zero results are dropped by
// the caller, like insert).
template <typename T, bool SUB, typename F>
__device__ __forceinline__ void merge_range(int64_t ia, int64_t ea, int64_t ib, int64_t eb,
                                            const int32_t* __restrict__ acol, const T* __restrict__ av,
                                            const int32_t* __restrict__ bcol, const T* __restrict__ bv, F&& emit) {
    using A = Arith<T>;
    while (ia < ea || ib < eb) {
        if (ia < ea && ib < eb) {
            const int32_t ca = acol[ia], cb = bcol[ib];
            if (ca > cb) {
                emit(cb, SUB ? A::sub(A::zero(), bv[ib]) : bv[ib]);
                ++ib;
            } else if (ca < cb) {
                emit(ca, av[ia]);
                ++ia;
            } else {
                emit(ca, SUB ? A::sub(av[ia], bv[ib]) : A::add(av[ia], bv[ib]));
                ++ia;
                ++ib;
            }
        } else if (ia < ea) {
            emit(acol[ia], av[ia]);
            ++ia;
        } else {
            emit(bcol[ib], SUB ? A::sub(A::zero(), bv[ib]) : bv[ib]);
            ++ib;
        }
    }
}

constexpr int64_t PIECE_CAP = 2048;  // entries per side staged in LDS by piece_merge
constexpr int64_t LONG_ROW = 64;  // la + lb above this: cut the row into pieces (one thread's merge costs
                                  // ~350 ns per step, dependent global loads: a 2,000-entry row took 55 + 108
                                  // us of count + fill at e = 100k)

__device__ __forceinline__ bool is_long(const int64_t* arp, const int64_t* brp, int64_t r) {
    return (arp[r + 1] - arp[r]) + (brp[r + 1] - brp[r]) > LONG_ROW;
}

template <typename T, bool SUB>
__global__ __launch_bounds__(256) void addsub_count(int64_t rows, const int64_t* __restrict__ arp,
                                                    const int32_t* __restrict__ acol, const T* __restrict__ av,
                                                    const int64_t* __restrict__ brp, const int32_t* __restrict__ bcol,
                                                    const T* __restrict__ bv, int32_t* __restrict__ cnt,
                                                    int32_t* __restrict__ long_flag) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const bool lg = is_long(arp, brp, r);
    long_flag[r] = lg ? 1 : 0;
    int32_t n = 0;
    if (!lg)
        merge_range<T, SUB>(arp[r], arp[r + 1], brp[r], brp[r + 1], acol, av, bcol, bv,
                            [&](int32_t, T v) { n += Arith<T>::nz(v) ? 1 : 0; });
    cnt[r] = n;  // long rows: filled from their pieces
}

template <typename T, bool SUB>
__global__ __launch_bounds__(256) void addsub_fill(int64_t rows, const int64_t* __restrict__ arp,
                                                   const int32_t* __restrict__ acol, const T* __restrict__ av,
                                                   const int64_t* __restrict__ brp, const int32_t* __restrict__ bcol,
                                                   const T* __restrict__ bv, const int64_t* __restrict__ orp,
                                                   int32_t* __restrict__ ocol, T* __restrict__ ov) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows || is_long(arp, brp, r)) return;
    int64_t p = orp[r];
    merge_range<T, SUB>(arp[r], arp[r + 1], brp[r], brp[r + 1], acol, av, bcol, bv, [&](int32_t c, T v) {
        if (Arith<T>::nz(v)) {
            ocol[p] = c;
            ov[p] = v;
            ++p;
        }
    });
}

// long rows ------------------------------------------------------------------
struct Piece {
    int64_t a0, a1, b0, b1;  // the two stretches
    int64_t pa, pb;          // the M pair that closes the piece (-1: none, the tails)
    int64_t row;
};

// Long-row setup, chunk-parallel: a long row's two sides are cut into
// chunks of LR_CHUNK entries (listed on the host from the rows' extents).
constexpr int64_t LR_CHUNK = 2048;

struct LrChunk {
    int64_t l;     // long-row index
    int64_t side;  // 0: self row, 1: rhs row
    int64_t b, e;  // entry range
    int64_t off;   // occurrences of M in the earlier chunks of the same row side
};

// rank of `flag` within a 256-thread block, and the block total
__device__ __forceinline__ int block_rank256(bool flag, int* wsum, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t m = __ballot(flag);
    const int before = __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
    __syncthreads();
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int off = 0;
    for (int i = 0; i < w; ++i) off += wsum[i];
    *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    return off + before;
}

__global__ __launch_bounds__(256) void long_extents(int64_t n_long, const int64_t* __restrict__ long_rows,
                                                    const int64_t* __restrict__ arp, const int64_t* __restrict__ brp,
                                                    int64_t* __restrict__ ext) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n_long) return;
    const int64_t r = long_rows[l];
    ext[4 * l + 0] = arp[r];
    ext[4 * l + 1] = arp[r + 1];
    ext[4 * l + 2] = brp[r];
    ext[4 * l + 3] = brp[r + 1];
}

// MAX: mval[l] = max column over the chunks of row l; else the count of
// mval[l] in each chunk
template <bool MAX>
__global__ __launch_bounds__(256) void chunk_reduce(const LrChunk* __restrict__ chunks, const int32_t* __restrict__ acol,
                                                    const int32_t* __restrict__ bcol, int32_t* __restrict__ mval,
                                                    int64_t* __restrict__ ccnt) {
    __shared__ int red[256];
    const LrChunk ch = chunks[blockIdx.x];
    const int32_t* col = ch.side ? bcol : acol;
    const int t = threadIdx.x;
    const int M = MAX ? 0 : mval[ch.l];
    int v = MAX ? -1 : 0;
    for (int64_t e = ch.b + t; e < ch.e; e += 256) v = MAX ? max(v, col[e]) : v + (col[e] == M);
    red[t] = v;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (t < s) red[t] = MAX ? max(red[t], red[t + s]) : red[t] + red[t + s];
        __syncthreads();
    }
    if (t == 0) {
        if (MAX) atomicMax(&mval[ch.l], red[0]);
        else ccnt[blockIdx.x] = red[0];
    }
}

// the first and last piece of each long row, and every piece's row
__global__ __launch_bounds__(256) void long_piece_init(int64_t n_long, const int64_t* __restrict__ long_rows,
                                                       const int64_t* __restrict__ ext,
                                                       const int64_t* __restrict__ pstart, Piece* __restrict__ pieces,
                                                       int64_t* __restrict__ first_piece) {
    const int64_t l = blockIdx.x;
    const int64_t p0 = pstart[l], c = pstart[l + 1] - p0 - 1;
    Piece* pc = pieces + p0;
    if (threadIdx.x == 0) {
        pc[0].a0 = ext[4 * l + 0];
        pc[0].b0 = ext[4 * l + 2];
        pc[c].a1 = ext[4 * l + 1];
        pc[c].b1 = ext[4 * l + 3];
        pc[c].pa = pc[c].pb = -1;
    }
    for (int64_t k = threadIdx.x; k <= c; k += blockDim.x) {
        pc[k].row = long_rows[l];
        first_piece[p0 + k] = p0;
    }
}

// the k-th M of a side (k < c) closes piece k and opens piece k + 1
__global__ __launch_bounds__(256) void chunk_pieces(const LrChunk* __restrict__ chunks, const int32_t* __restrict__ acol,
                                                    const int32_t* __restrict__ bcol, const int32_t* __restrict__ mval,
                                                    const int64_t* __restrict__ pstart, Piece* __restrict__ pieces) {
    __shared__ int wsum[4];
    const LrChunk ch = chunks[blockIdx.x];
    const int32_t* col = ch.side ? bcol : acol;
    const int M = mval[ch.l];
    const int64_t p0 = pstart[ch.l], c = pstart[ch.l + 1] - p0 - 1;
    Piece* pc = pieces + p0;
    int64_t base = ch.off;
    for (int64_t e0 = ch.b; e0 < ch.e && base < c; e0 += 256) {
        const int64_t e = e0 + threadIdx.x;
        const bool f = e < ch.e && col[e] == M;
        int tot;
        const int64_t k = base + block_rank256(f, wsum, &tot);
        if (f && k < c) {
            if (ch.side) {
                pc[k].b1 = e;
                pc[k].pb = e;
                pc[k + 1].b0 = e + 1;
            } else {
                pc[k].a1 = e;
                pc[k].pa = e;
                pc[k + 1].a0 = e + 1;
            }
        }
        base += tot;
    }
}

__device__ __forceinline__ int32_t rl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t rl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ float rl(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint64_t rl(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int64_t rl(int64_t v, int l) { return (int64_t)rl((uint64_t)v, l); }
__device__ __forceinline__ double rl(double v, int l) {
    return __longlong_as_double((long long)rl((uint64_t)__double_as_longlong(v), l));
}

// One WAVE per piece. The merge itself is uniform scalar control flow: both
// stretches are read 64 entries at a time into a lane window, the current
// entries come out with v_readlane, and the kept
// outputs collect one per lane until 64 are stored at once. Outputs go to a
// scratch slot at a0 + b0 (pieces' slots never overlap: a piece emits at
// most its two lengths plus one pair); piece_copy moves them into place.
template <typename T, bool SUB>
__global__ __launch_bounds__(64) void piece_merge(const Piece* __restrict__ pieces, const int32_t* __restrict__ acol,
                                                  const T* __restrict__ av, const int32_t* __restrict__ bcol,
                                                  const T* __restrict__ bv, int32_t* __restrict__ tcol,
                                                  T* __restrict__ tval, int32_t* __restrict__ pcnt,
                                                  unsigned long long* __restrict__ pdbg) {
    using A = Arith<T>;
    const long long c_start = pdbg ? clock64() : 0;  // BSM_SS_DEBUG=2: s_memtime stamps per piece
    extern __shared__ __attribute__((aligned(16))) unsigned char piece_sm[];
    int32_t* sac = reinterpret_cast<int32_t*>(piece_sm);
    int32_t* sbc = sac + PIECE_CAP;
    T* sav = reinterpret_cast<T*>(sbc + PIECE_CAP);
    T* sbv = sav + PIECE_CAP;
    const int lane = threadIdx.x;
    const Piece pc = pieces[blockIdx.x];
    const int64_t ea = pc.a1, eb = pc.b1;
    int64_t ia = pc.a0, ib = pc.b0, wa = pc.a0, wb = pc.b0;
    // stage both stretches in LDS when they fit: the windows then refill from
    // LDS instead of waiting on global memory every 64 steps
    const bool staged = ea - pc.a0 <= PIECE_CAP && eb - pc.b0 <= PIECE_CAP;
    if (staged) {
        for (int64_t i = lane; i < ea - pc.a0; i += 64) {
            sac[i] = acol[pc.a0 + i];
            sav[i] = av[pc.a0 + i];
        }
        for (int64_t i = lane; i < eb - pc.b0; i += 64) {
            sbc[i] = bcol[pc.b0 + i];
            sbv[i] = bv[pc.b0 + i];
        }
        __syncthreads();
    }
    auto load = [&](bool side_b, int64_t base, int32_t& c, T& x) {
        const int64_t s0 = side_b ? pc.b0 : pc.a0, end = side_b ? eb : ea;
        const int64_t e = base + lane < end ? base + lane : (end > s0 ? end - 1 : s0);
        if (staged) {
            c = side_b ? sbc[e - s0] : sac[e - s0];
            x = side_b ? sbv[e - s0] : sav[e - s0];
        } else {
            c = side_b ? bcol[e] : acol[e];
            x = side_b ? bv[e] : av[e];
        }
    };
    // windows are loaded when the merge reaches them, not prefetched: a
    // prefetch into a second register set made the compiler rotate the sets
    // every step, with a wait for the outstanding loads in each (~550 ns a
    // step); now one wait per 64 steps
    int32_t caw = 0, cbw = 0;
    T vaw = A::zero(), vbw = A::zero();
    if (ea > pc.a0) load(false, wa, caw, vaw);
    if (eb > pc.b0) load(true, wb, cbw, vbw);
    const long long c_staged = pdbg ? clock64() : 0;
    long long c_win = 0;  // cycles spent refilling the windows
    int64_t o = pc.a0 + pc.b0;
    int nbuf = 0;
    int32_t cnt = 0, oc = 0;
    T ov = A::zero();
    auto emit = [&](int32_t c, T v) {
        if (A::nz(v)) {
            if (lane == nbuf) {
                oc = c;
                ov = v;
            }
            ++cnt;
            if (++nbuf == 64) {
                tcol[o + lane] = oc;
                tval[o + lane] = ov;
                o += 64;
                nbuf = 0;
            }
        }
    };
    while (ia < ea && ib < eb) {
        if (ia - wa == 64) {
            const long long c0 = pdbg ? clock64() : 0;
            wa += 64;
            load(false, wa, caw, vaw);
            if (pdbg) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                c_win += clock64() - c0;
            }
        }
        if (ib - wb == 64) {
            const long long c0 = pdbg ? clock64() : 0;
            wb += 64;
            load(true, wb, cbw, vbw);
            if (pdbg) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                c_win += clock64() - c0;
            }
        }
        const int32_t ca = rl(caw, (int)(ia - wa)), cb = rl(cbw, (int)(ib - wb));
        if (ca > cb) {
            const T x = rl(vbw, (int)(ib - wb));
            emit(cb, SUB ? A::sub(A::zero(), x) : x);
            ++ib;
        } else if (ca < cb) {
            emit(ca, rl(vaw, (int)(ia - wa)));
            ++ia;
        } else {
            const T x = rl(vaw, (int)(ia - wa)), y = rl(vbw, (int)(ib - wb));
            emit(ca, SUB ? A::sub(x, y) : A::add(x, y));
            ++ia;
            ++ib;
        }
    }
    const long long c_merged = pdbg ? clock64() : 0;
    const int64_t steps = (ia - pc.a0) + (ib - pc.b0);
    // one side is exhausted: the rest of the other side goes out in order,
    // 64 entries per step (ballot compaction of the kept ones)
    if (ia < ea || ib < eb) {
        if (lane < nbuf) {
            tcol[o + lane] = oc;
            tval[o + lane] = ov;
        }
        o += nbuf;
        nbuf = 0;
        const bool side_b = ib < eb;
        const int64_t s0 = side_b ? ib : ia, s1 = side_b ? eb : ea;
        const int32_t* col = side_b ? bcol : acol;
        const T* val = side_b ? bv : av;
        for (int64_t base = s0; base < s1; base += 64) {
            const int64_t e = base + lane;
            const bool valid = e < s1;
            T x = valid ? val[e] : A::zero();
            if (SUB && side_b) x = A::sub(A::zero(), x);
            const bool keep = valid && A::nz(x);
            const uint64_t m = __ballot(keep);
            if (keep) {
                const int r = __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
                tcol[o + r] = col[e];
                tval[o + r] = x;
            }
            o += __popcll(m);
            cnt += __popcll(m);
        }
    }
    if (pc.pa >= 0) {
        const T x = av[pc.pa], y = bv[pc.pb];
        emit(acol[pc.pa], SUB ? A::sub(x, y) : A::add(x, y));
    }
    if (lane < nbuf) {
        tcol[o + lane] = oc;
        tval[o + lane] = ov;
    }
    if (lane == 0) pcnt[blockIdx.x] = cnt;
    if (pdbg && lane == 0) {
        unsigned long long* d = pdbg + 6 * (int64_t)blockIdx.x;
        d[0] = (unsigned long long)(c_staged - c_start);   // piece descriptor + LDS staging + first windows
        d[1] = (unsigned long long)(c_merged - c_staged);  // the two-sided merge loop
        d[2] = (unsigned long long)c_win;                  //   of which window refills (waited)
        d[3] = (unsigned long long)steps;                  //   its steps
        d[4] = (unsigned long long)(clock64() - c_merged); // the one-sided tail
        d[5] = (unsigned long long)((ea - pc.a0) + (eb - pc.b0));
    }
}

// ---- long rows, round 3: recursive cut + one lane per leaf ------------------
// piece_merge above walks a piece with one wave, ~450 cycles per merge step
// (BSM_SS_DEBUG=2 stamps, profiles/r03_j_ss_add_piece_stamps.log), and the
// longest piece (up to ~20k steps at e = 100k) sets the kernel's time. The cut
// that made the pieces applies again inside each one, with m = the largest
// column of the PIECE:
//   * both sides hold an m: the first m of each pair up (every smaller value
//     goes out first), so (a0..qa, b0..qb) + that pair, then the rest;
//   * only one side holds an m, say self at qa: the rhs side is all smaller,
//     so once the self pointer reaches qa the rhs drains and self continues
//     alone: merge(a0..qa, all of rhs) then a plain copy of self from qa on
//     (the piece's closing pair, if any, after it).
// Sub-pieces of at most LEAF entries become leaves; leaf l is merged by lane l
// of the wave (the reference's two-pointer loop, merge_range), one-sided
// pieces are copied by the whole wave. Every sub-piece writes its kept outputs
// from scratch position a0 + b0 on: the ranges of a piece's parts are disjoint
// and in output order (a part emits at most its two lengths plus its pair),
// so a scan of the used-position flags places every output (pos_copy). The
// work stack and the leaf list live in registers, entry i in lane i.
struct SubPiece {
    int64_t a0, a1, b0, b1, pa, pb;  // pa < 0: no closing pair
};
// A leaf costs its length in serial steps on one lane (~650 cycles per step
// from LDS, branch-free); a cut costs ~700 cycles of wave-wide work plus its
// scan. Measured per 1,900-entry piece at e = 300k (BSM_SS_DEBUG=4,
// profiles/r03_x_ss_split_stamps.log, r03_za_*): LEAF 64: 182k cycles, the
// longest piece 632k; LEAF 128: 186k / 786k; LEAF 192: 255k / 909k.
constexpr int64_t LEAF = 64;
// entries per side staged in LDS by piece_split: 4096 for 4-B values (64 KiB
// per wave; the benches' pieces average ~950 entries per side and the longest
// reach ~3,400 at every e, so one staging covers the whole subtree), 2048 for
// 8-B values (48 KiB)
template <typename T> constexpr int64_t split_cap() { return sizeof(T) <= 4 ? 4096 : 2048; }

__device__ __forceinline__ int64_t rl64(int64_t v, int l) { return rl(v, l); }
__device__ __forceinline__ SubPiece sp_read(const SubPiece& x, int l) {
    return {rl64(x.a0, l), rl64(x.a1, l), rl64(x.b0, l), rl64(x.b1, l), rl64(x.pa, l), rl64(x.pb, l)};
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v = max(v, __shfl_xor(v, off, 64));
    return __builtin_amdgcn_readfirstlane(v);
}
// One side of a piece: its entries in global memory, or staged in LDS
// (entry e at offset e - base). LDS is indexed by offset, never through a
// generic pointer moved below the LDS aperture.
template <typename T>
struct SideView {
    const int32_t* __restrict__ gc;
    const T* __restrict__ gv;
    const __attribute__((address_space(3))) int32_t* lc;
    const __attribute__((address_space(3))) T* lv;
    int64_t base;
    bool staged;
    __device__ __forceinline__ int32_t col(int64_t e) const { return staged ? lc[e - base] : gc[e]; }
    __device__ __forceinline__ T val(int64_t e) const { return staged ? lv[e - base] : gv[e]; }
};

// first e in [e0, e1) with col(e) == m, else e1 (uniform)
template <typename S>
__device__ __forceinline__ int64_t first_eq(const S& sd, int64_t e0, int64_t e1, int32_t m, int lane) {
    for (int64_t base = e0; base < e1; base += 4 * 64) {  // four windows' loads in flight
        bool h[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t e = base + 64 * u + lane;
            h[u] = e < e1 && sd.col(e) == m;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t bal = __ballot(h[u]);
            if (bal) return base + 64 * u + __builtin_ctzll(bal);
        }
    }
    return e1;
}

// first e in [e0, e1) with col(e) >= v, else e1; col non-decreasing on
// [e0, e1) (uniform): 64 samples per round narrow the range 64-fold
template <typename S>
__device__ __forceinline__ int64_t lower_bound_wave(const S& sd, int64_t e0, int64_t e1, int32_t v, int lane) {
    int64_t lo = e0, hi = e1;  // the answer is in [lo, hi]
    while (hi - lo > 64) {
        const int64_t step = (hi - lo + 63) / 64, p = lo + lane * step;
        const uint64_t bal = __ballot(p >= hi || sd.col(p) >= v);  // monotone in the lane
        const int k = bal ? __builtin_ctzll(bal) : 64;
        if (k == 0) return lo;
        const int64_t nlo = lo + (int64_t)(k - 1) * step + 1, nhi = lo + (int64_t)k * step;
        lo = nlo;
        hi = nhi < hi ? nhi : hi;
    }
    const int64_t e = lo + lane;
    const uint64_t bal = __ballot(e < hi && sd.col(e) >= v);
    return bal ? lo + __builtin_ctzll(bal) : hi;
}

// PRESPLIT (a first pass over the long rows' pieces): only cuts, the largest
// sub-piece first, at most PRE_CUTS per piece and none below PRE_MIN
// entries; the sub-pieces left go out as pieces of their own (out, *n_out),
// which the second pass (the full piece_split, its grid bounded by *n_in)
// takes one workgroup each. A piece's sub-pieces are independent (each
// writes from its own scratch position a0 + b0), so the longest piece's
// serial cut chain, which sets the kernel's time, is spread over up to
// PRE_CUTS + 1 workgroups. Same leaves, same outputs, same positions.
constexpr int PRE_CUTS = 7;
constexpr int64_t PRE_MIN = 512;

template <typename T, bool SUB, bool PRESPLIT = false>
__global__ __launch_bounds__(64) void piece_split(const Piece* __restrict__ pieces, const int32_t* __restrict__ acol,
                                                  const T* __restrict__ av, const int32_t* __restrict__ bcol,
                                                  const T* __restrict__ bv, int32_t* __restrict__ tcol,
                                                  T* __restrict__ tval, unsigned long long* __restrict__ sdbg,
                                                  const unsigned* __restrict__ n_in = nullptr,
                                                  Piece* __restrict__ out = nullptr,
                                                  unsigned* __restrict__ n_out = nullptr) {
    using A = Arith<T>;
    if (n_in && blockIdx.x >= *n_in) return;  // the second pass's grid is an upper bound
    // BSM_SS_DEBUG=4: cycles per piece (total, cut scans, leaf merges, one-sided
    // copies, staging), entries scanned, flushes, leaves, the piece's size
    long long k_cut = 0, k_flush = 0, k_bulk = 0, k_stage = 0, n_scan = 0, n_flush = 0, n_leaf = 0;
    const long long k_start = sdbg ? clock64() : 0;
    using lds_i = __attribute__((address_space(3))) int32_t;
    using lds_v = __attribute__((address_space(3))) T;
    const int lane = threadIdx.x;
    const Piece pc = pieces[blockIdx.x];
    // A sub-piece that still needs cutting and fits in LDS (both sides, and
    // its closing pair, which always sits at a1 / b1) is staged there with
    // its whole subtree: every cut scan and leaf step of it then reads LDS
    // (~100 cycles) instead of global memory (~1 us per dependent step). The
    // top piece is staged at once when it fits; a piece too long for LDS (a
    // row's tail) is cut from global memory until its parts fit.
    extern __shared__ __attribute__((aligned(16))) unsigned char split_sm[];
    lds_i* sac = (lds_i*)split_sm;
    constexpr int64_t SPLIT_CAP = split_cap<T>();
    lds_i* sbc = sac + SPLIT_CAP;
    lds_v* sav = (lds_v*)(sbc + SPLIT_CAP);
    lds_v* sbv = sav + SPLIT_CAP;
    SideView<T> SA{acol, av, sac, sav, 0, false}, SB{bcol, bv, sbc, sbv, 0, false};
    bool staged = false;
    int sp_base = 0;  // staged: the stack level below the staged subtree
    auto stage_piece = [&](const SubPiece& x) {
        const int64_t la = (x.a1 - x.a0) + (x.pa >= 0 ? 1 : 0), lb = (x.b1 - x.b0) + (x.pb >= 0 ? 1 : 0);
        for (int64_t i = lane; i < la; i += 64) {
            sac[i] = acol[x.a0 + i];
            sav[i] = av[x.a0 + i];
        }
        for (int64_t i = lane; i < lb; i += 64) {
            sbc[i] = bcol[x.b0 + i];
            sbv[i] = bv[x.b0 + i];
        }
        __syncthreads();
        SA.base = x.a0;
        SB.base = x.b0;
        SA.staged = SB.staged = staged = true;
    };
    auto unstage = [&] {
        SA.staged = SB.staged = staged = false;
        __syncthreads();  // every lane's LDS reads are done before the next staging
    };
    SubPiece stk{}, lf{};  // lane i: stack entry i / leaf i
    int sp = 0, nl = 0;    // uniform
    auto pair_val = [&](int64_t pa, int64_t pb) -> T {
        return SUB ? A::sub(SA.val(pa), SB.val(pb)) : A::add(SA.val(pa), SB.val(pb));
    };
    auto emit = [&](int64_t o, int32_t c, T v) {
        tcol[o] = c;
        tval[o] = v;
    };
    auto flush = [&] {  // lane l < nl merges leaf l from position a0 + b0 on (sparse.rs:493-531)
        const long long k0 = sdbg ? clock64() : 0;
        n_leaf += nl;
        n_flush += nl > 0;
        if (lane < nl) {
            // one reference merge step per iteration, without branches (the
            // 64 leaves of a wave differ in every comparison): an exhausted
            // side reads as column INT32_MAX (device columns are < 2^31 - 1),
            // so the other side goes out; an equal pair goes out as one entry
            int64_t o = lf.a0 + lf.b0, ia = lf.a0, ib = lf.b0;
            while (ia < lf.a1 || ib < lf.b1) {
                const bool ha = ia < lf.a1, hb = ib < lf.b1;
                const int32_t ca = ha ? SA.col(ia) : 0x7fffffff, cb = hb ? SB.col(ib) : 0x7fffffff;
                const T va = ha ? SA.val(ia) : A::zero(), vb = hb ? SB.val(ib) : A::zero();
                const bool ta = ca <= cb, tb = cb <= ca;  // both: the pair
                const T v = ta && tb ? (SUB ? A::sub(va, vb) : A::add(va, vb))
                                     : (ta ? va : (SUB ? A::sub(A::zero(), vb) : vb));
                if (A::nz(v)) {
                    tcol[o] = ta ? ca : cb;
                    tval[o] = v;
                    ++o;
                }
                ia += ta ? 1 : 0;
                ib += tb ? 1 : 0;
            }
            if (lf.pa >= 0) {
                const T v = pair_val(lf.pa, lf.pb);
                if (A::nz(v)) {
                    tcol[o] = SA.col(lf.pa);
                    tval[o] = v;
                }
            }
        }
        nl = 0;
        if (sdbg) k_flush += clock64() - k0;
    };
    auto push = [&](const SubPiece& x) {
        if (sp == 64) {  // stack full (deeply nested columns): merge it on one lane, serially
            if (nl == 64) flush();
            if (lane == nl) lf = x;
            ++nl;
            return;
        }
        if (lane == sp) stk = x;
        ++sp;
    };
    push({pc.a0, pc.a1, pc.b0, pc.b1, pc.pa, pc.pb});
    // scan budget: inputs that make every cut peel off O(1) entries (e.g. equal
    // descending rows) stop being cut after ~32 passes over the piece and
    // merge as they stand, one lane per piece
    int64_t budget = 32 * ((pc.a1 - pc.a0) + (pc.b1 - pc.b0)) + 4096;
    auto cut_piece = [&](const SubPiece& x, int64_t na, int64_t nb) {
        budget -= na + nb;
        const long long kc0 = sdbg ? clock64() : 0;
        n_scan += na + nb;
        // the piece's largest column, and whether both sides are sorted
        int mx = -1;
        bool srt = true;
        auto scan_side = [&](const SideView<T>& sd, int64_t e0, int64_t e1) {
            for (int64_t base = e0; base < e1; base += 8 * 64) {  // eight windows' loads in flight
                int32_t c[8], n[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int64_t e = base + 64 * u + lane;
                    c[u] = e < e1 ? sd.col(e) : -1;
                    n[u] = e + 1 < e1 ? sd.col(e + 1) : 0x7fffffff;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    mx = max(mx, c[u]);
                    srt = srt && c[u] <= n[u];
                }
            }
        };
        scan_side(SA, x.a0, x.a1);
        scan_side(SB, x.b0, x.b1);
        mx = wave_max_i32(mx);
        if (__ballot(!srt) == 0) {
            // sorted sides (the cut at the maximum would peel one pair off the
            // end): cut by value at the longer side's median v. Everything
            // below v merges first, on both sides, then the rest.
            const int32_t v = na >= nb ? SA.col(x.a0 + na / 2) : SB.col(x.b0 + nb / 2);
            int64_t qa = lower_bound_wave(SA, x.a0, x.a1, v, lane), qb = lower_bound_wave(SB, x.b0, x.b1, v, lane);
            if (qa == x.a0 && qb == x.b0 && v < 0x7fffffff) {  // nothing below v: cut above it
                qa = lower_bound_wave(SA, x.a0, x.a1, v + 1, lane);
                qb = lower_bound_wave(SB, x.b0, x.b1, v + 1, lane);
            }
            if (!(qa == x.a0 && qb == x.b0) && !(qa == x.a1 && qb == x.b1)) {
                if (sdbg) k_cut += clock64() - kc0;
                push({qa, x.a1, qb, x.b1, x.pa, x.pb});
                push({x.a0, qa, x.b0, qb, -1, -1});
                return;
            }
        }
        // the first occurrence of the maximum on each side
        const int64_t qa = first_eq(SA, x.a0, x.a1, mx, lane), qb = first_eq(SB, x.b0, x.b1, mx, lane);
        if (sdbg) k_cut += clock64() - kc0;
        if (qa < x.a1 && qb < x.b1) {  // the first pair of m splits the piece
            push({qa + 1, x.a1, qb + 1, x.b1, x.pa, x.pb});
            push({x.a0, qa, x.b0, qb, qa, qb});
        } else if (qa < x.a1) {  // only self holds m: merge up to it, then self alone
            push({qa, x.a1, x.b1, x.b1, x.pa, x.pb});
            push({x.a0, qa, x.b0, x.b1, -1, -1});
        } else {  // only rhs holds m
            push({x.a1, x.a1, qb, x.b1, x.pa, x.pb});
            push({x.a0, x.a1, x.b0, qb, -1, -1});
        }
    };
    if constexpr (PRESPLIT) {
        for (int cuts = 0; cuts < PRE_CUTS && sp > 0; ++cuts) {
            // the largest sub-piece on the stack to the top
            const int64_t sz = lane < sp ? (stk.a1 - stk.a0) + (stk.b1 - stk.b0) : -1;
            int64_t best = sz;
            int bl = lane;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t ob = __shfl_xor(best, off, 64);
                const int ol = __shfl_xor(bl, off, 64);
                if (ob > best || (ob == best && ol < bl)) {
                    best = ob;
                    bl = ol;
                }
            }
            bl = __builtin_amdgcn_readfirstlane(bl);
            const SubPiece x = sp_read(stk, bl);
            const int64_t na = x.a1 - x.a0, nb = x.b1 - x.b0;
            if (na + nb <= PRE_MIN || na == 0 || nb == 0) break;  // nothing left worth a workgroup
            const SubPiece top = sp_read(stk, sp - 1);
            if (lane == bl) stk = top;
            --sp;
            // the top piece, when it fits, is staged with its whole subtree (every
            // later sub-piece lies inside it); a later one is never staged here,
            // the stack holding entries outside it
            if (!staged && sp == 0 && na + (x.pa >= 0 ? 1 : 0) <= SPLIT_CAP && nb + (x.pb >= 0 ? 1 : 0) <= SPLIT_CAP)
                stage_piece(x);
            cut_piece(x, na, nb);
        }
        // every sub-piece left becomes a piece of the second pass
        unsigned base = 0;
        if (lane == 0 && sp > 0) base = atomicAdd(n_out, (unsigned)sp);
        base = (unsigned)__builtin_amdgcn_readfirstlane((int)base);
        if (lane < sp) out[base + lane] = Piece{stk.a0, stk.a1, stk.b0, stk.b1, stk.pa, stk.pb, pc.row};
        return;
    }
    while (sp > 0) {
        if (staged && sp == sp_base) {  // the staged subtree is done: its leaves first
            flush();
            unstage();
        }
        const SubPiece x = sp_read(stk, --sp);
        const int64_t na = x.a1 - x.a0, nb = x.b1 - x.b0;
        if (!staged && na > 0 && nb > 0 && na + nb > LEAF && budget >= 0 &&
            na + (x.pa >= 0 ? 1 : 0) <= SPLIT_CAP && nb + (x.pb >= 0 ? 1 : 0) <= SPLIT_CAP) {
            flush();  // leaves so far read global memory; the rest reads LDS
            const long long k0 = sdbg ? clock64() : 0;
            stage_piece(x);
            if (sdbg) k_stage += clock64() - k0;
            sp_base = sp;
        }
        if (na + nb <= LEAF || na == 0 || nb == 0 || budget < 0) {
            if (na + nb == 0 && x.pa < 0) continue;
            if (na > 0 && nb > 0) {  // a leaf (a one-sided piece is cheaper as a wave copy)
                if (nl == 64) flush();
                if (lane == nl) lf = x;
                ++nl;
                continue;
            }
            // one side: copied by the wave, entry e to position a0 + b0 + (e -
            // s0) (scratch positions need not be dense: pos_copy ranks the
            // used ones), sixteen windows' loads in flight (a row's tail can
            // leave tens of thousands of entries here, read from global memory)
            const long long kb0 = sdbg ? clock64() : 0;
            const bool side_b = nb > 0;
            const SideView<T> sd = side_b ? SB : SA;
            const int64_t s0 = side_b ? x.b0 : x.a0, s1 = side_b ? x.b1 : x.a1, o0 = x.a0 + x.b0 - s0;
            for (int64_t base = s0; base < s1; base += 16 * 64) {
                T v[16];
                int32_t c[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int64_t e = base + 64 * u + lane;
                    v[u] = e < s1 ? sd.val(e) : A::zero();
                    c[u] = e < s1 ? sd.col(e) : 0;
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int64_t e = base + 64 * u + lane;
                    if (SUB && side_b) v[u] = A::sub(A::zero(), v[u]);
                    if (e < s1 && A::nz(v[u])) emit(o0 + e, c[u], v[u]);
                }
            }
            if (x.pa >= 0) {
                const T v = pair_val(x.pa, x.pb);
                if (A::nz(v) && lane == 0) emit(o0 + s1, SA.col(x.pa), v);
            }
            if (sdbg) k_bulk += clock64() - kb0;
            continue;
        }
        cut_piece(x, na, nb);
    }
    if (nl) flush();
    if (sdbg && lane == 0) {
        unsigned long long* d = sdbg + 9 * (int64_t)blockIdx.x;
        d[0] = (unsigned long long)(clock64() - k_start);
        d[1] = (unsigned long long)k_cut;
        d[2] = (unsigned long long)k_flush;
        d[3] = (unsigned long long)k_bulk;
        d[4] = (unsigned long long)k_stage;
        d[5] = (unsigned long long)n_scan;
        d[6] = (unsigned long long)n_flush;
        d[7] = (unsigned long long)n_leaf;
        d[8] = (unsigned long long)((pc.a1 - pc.a0) + (pc.b1 - pc.b0));
    }
}

// output count of each long row from the position offsets: its positions are
// [arp[r] + brp[r], arp[r+1] + brp[r+1])
__global__ __launch_bounds__(256) void long_row_totals_slots(int64_t n_long, const int64_t* __restrict__ long_rows,
                                                             const int64_t* __restrict__ arp,
                                                             const int64_t* __restrict__ brp,
                                                             const int64_t* __restrict__ soff, int32_t* __restrict__ cnt,
                                                             int64_t* __restrict__ lstart) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n_long) return;
    const int64_t r = long_rows[l];
    lstart[l] = arp[r] + brp[r];
    cnt[r] = (int32_t)(soff[arp[r + 1] + brp[r + 1]] - soff[arp[r] + brp[r]]);
}

// Scratch columns start as -1 (memset): a used position holds its column.
__global__ __launch_bounds__(256) void pos_flags(int64_t n_pos, const int32_t* __restrict__ tcol,
                                                 int32_t* __restrict__ pvalid) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_pos) pvalid[j] = tcol[j] >= 0 ? 1 : 0;
}

// every used scratch position to its place in the output row (the scan of
// the used-position flags gives its rank inside the row); its row is the last
// long row starting at or before it (lstart: the long rows' first positions,
// ascending)
template <typename T>
__global__ __launch_bounds__(256) void pos_copy(int64_t n_pos, const int32_t* __restrict__ tcol,
                                                const int64_t* __restrict__ poff, int64_t n_long,
                                                const int64_t* __restrict__ long_rows,
                                                const int64_t* __restrict__ lstart, const int64_t* __restrict__ orp,
                                                const T* __restrict__ tval, int32_t* __restrict__ ocol,
                                                T* __restrict__ ov) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pos) return;
    const int32_t c = tcol[j];
    if (c < 0) return;
    int64_t lo = 0, hi = n_long - 1;  // last l with lstart[l] <= j
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (lstart[mid] <= j) lo = mid;
        else hi = mid - 1;
    }
    const int64_t r = long_rows[lo];
    const int64_t dst = orp[r] + (poff[j] - poff[lstart[lo]]);
    ocol[dst] = c;
    ov[dst] = tval[j];
}

// one wave per piece: scratch slot -> the output rows
template <typename T>
__global__ __launch_bounds__(64) void piece_copy(const Piece* __restrict__ pieces, const int32_t* __restrict__ pcnt,
                                                 const int64_t* __restrict__ poff,
                                                 const int64_t* __restrict__ first_piece,
                                                 const int64_t* __restrict__ orp, const int32_t* __restrict__ tcol,
                                                 const T* __restrict__ tval, int32_t* __restrict__ ocol,
                                                 T* __restrict__ ov) {
    const int64_t p = blockIdx.x;
    const Piece pc = pieces[p];
    const int64_t src = pc.a0 + pc.b0, dst = orp[pc.row] + (poff[p] - poff[first_piece[p]]);
    const int32_t n = pcnt[p];
    for (int32_t i = threadIdx.x; i < n; i += 64) {
        ocol[dst + i] = tcol[src + i];
        ov[dst + i] = tval[src + i];
    }
}

// output count of each long row = the sum of its pieces' counts
__global__ __launch_bounds__(256) void long_row_totals(int64_t n_long, const int64_t* __restrict__ long_rows,
                                                       const int64_t* __restrict__ pstart,
                                                       const int64_t* __restrict__ poff, int32_t* __restrict__ cnt) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n_long) return;
    cnt[long_rows[l]] = (int32_t)(poff[pstart[l + 1]] - poff[pstart[l]]);
}

template <typename T, bool SUB>
__global__ __launch_bounds__(256) void piece_fill(int64_t n, const Piece* __restrict__ pieces,
                                                  const int32_t* __restrict__ acol, const T* __restrict__ av,
                                                  const int32_t* __restrict__ bcol, const T* __restrict__ bv,
                                                  const int64_t* __restrict__ poff, const int64_t* __restrict__ first_piece,
                                                  const int64_t* __restrict__ orp, int32_t* __restrict__ ocol,
                                                  T* __restrict__ ov) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const Piece pc = pieces[p];
    int64_t q = orp[pc.row] + (poff[p] - poff[first_piece[p]]);
    auto put = [&](int32_t c, T v) {
        if (Arith<T>::nz(v)) {
            ocol[q] = c;
            ov[q] = v;
            ++q;
        }
    };
    merge_range<T, SUB>(pc.a0, pc.a1, pc.b0, pc.b1, acol, av, bcol, bv, put);
    if (pc.pa >= 0) put(acol[pc.pa], SUB ? Arith<T>::sub(av[pc.pa], bv[pc.pb]) : Arith<T>::add(av[pc.pa], bv[pc.pb]));
}

__global__ __launch_bounds__(256) void compact_flags(int64_t rows, const int32_t* __restrict__ flag,
                                                     const int64_t* __restrict__ pos, int64_t* __restrict__ list) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < rows && flag[r]) list[pos[r]] = r;
}

// ---- mul -------------------------------------------------------------------
// expansion count of self entry e = (i, k): the length of rhs row k
__global__ __launch_bounds__(256) void spgemm_count(uint64_t nnz_a, const int32_t* __restrict__ acol,
                                                    uint64_t b_rows, const int64_t* __restrict__ brp,
                                                    int32_t* __restrict__ cnt) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nnz_a) return;
    const uint64_t k = (uint64_t)acol[e];
    cnt[e] = k < b_rows ? (int32_t)(brp[k + 1] - brp[k]) : 0;
}

// last e with off[e] <= p (off: exclusive scan of the counts, n + 1 entries)
__device__ __forceinline__ uint64_t owner_of(const int64_t* __restrict__ off, uint64_t n, int64_t p) {
    uint64_t lo = 0, hi = n;  // off[lo] <= p < off[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] <= p) lo = mid; else hi = mid;
    }
    return lo;
}

// expanded slot p -> key (i << cb) | j
__global__ __launch_bounds__(256) void spgemm_expand(uint64_t total, uint64_t nnz_a, const int64_t* __restrict__ off,
                                                     const int64_t* __restrict__ arp, uint64_t a_rows,
                                                     const int32_t* __restrict__ acol, const int64_t* __restrict__ brp,
                                                     const int32_t* __restrict__ bcol, unsigned cb,
                                                     uint64_t* __restrict__ key) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= total) return;
    const uint64_t e = owner_of(off, nnz_a, (int64_t)p);
    const uint64_t i = owner_of(arp, a_rows, (int64_t)e);  // the self row holding entry e
    const int64_t k = acol[e];
    const int32_t j = bcol[brp[k] + ((int64_t)p - off[e])];
    key[p] = ((uint64_t)i << cb) | (uint64_t)j;
}

// the reference's merge for candidate (i, j); flag = val != default
template <typename T>
__global__ __launch_bounds__(256) void spgemm_merge(uint64_t n_cand, const uint64_t* __restrict__ key, unsigned cb,
                                                    const int64_t* __restrict__ arp, const int32_t* __restrict__ acol,
                                                    const T* __restrict__ av, const int64_t* __restrict__ trp,
                                                    const int32_t* __restrict__ tcol, const T* __restrict__ tv,
                                                    T* __restrict__ val, int32_t* __restrict__ keep) {
    using A = Arith<T>;
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cand) return;
    const uint64_t kk = key[c];
    const uint64_t i = kk >> cb, j = kk & ((1ull << cb) - 1);
    int64_t p = arp[i], q = trp[j];
    const int64_t ep = arp[i + 1], eq = trp[j + 1];
    T v = A::zero();
    while (q != eq && p != ep) {
        const int32_t ca = acol[p], ct = tcol[q];
        if (ca == ct) {
            v = A::add(v, A::mul(av[p], tv[q]));
            ++p;
            ++q;
        } else if (ca > ct) {
            ++q;
        } else {
            ++p;
        }
    }
    val[c] = v;
    keep[c] = A::nz(v) ? 1 : 0;
}

template <typename T>
__global__ __launch_bounds__(256) void spgemm_scatter(uint64_t n_cand, const uint64_t* __restrict__ key, unsigned cb,
                                                      const T* __restrict__ val, const int64_t* __restrict__ pos,
                                                      int64_t* __restrict__ orow, int32_t* __restrict__ ocol,
                                                      T* __restrict__ ov) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cand) return;
    const int64_t p = pos[c];
    if (pos[c + 1] == p) return;
    const uint64_t kk = key[c];
    orow[p] = (int64_t)(kk >> cb);
    ocol[p] = (int32_t)(kk & ((1ull << cb) - 1));
    ov[p] = val[c];
}

// row_ptr[r] = first p with orow[p] >= r, r in [0, rows]
__global__ __launch_bounds__(256) void rows_to_ptr(uint64_t rows, int64_t nnz, const int64_t* __restrict__ orow,
                                                   int64_t* __restrict__ rp) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > rows) return;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (orow[mid] < (int64_t)r) lo = mid + 1; else hi = mid;
    }
    rp[r] = lo;
}

struct CsrGuard {  // frees a half-built output on error paths
    bsm_csr* m = nullptr;
    ~CsrGuard() { if (m) bsm_csr_free(m); }
    bsm_csr* release() { bsm_csr* r = m; m = nullptr; return r; }
};

// ---- add / sub, rows of moderate length: one wave per row -------------------
// When no row has more than WROW_CAP entries on its two sides together (the
// handles' analysed max row lengths say so, no device round trip), each row
// is one 64-lane workgroup: the wave stages the row's two sides in LDS
// (coalesced), lane 0 runs the reference's two-pointer merge (merge_range,
// sparse.rs:493-532) out of LDS and writes the kept outputs at the row's
// upper-bound slot (arp[r] + brp[r]); a scan of the counts and a copy place
// them. One host sync per call (the result's nnz), against the count / long
// row / piece pipeline's five (§6b: the fixed cost of ss_add at e <= 200k).
constexpr int WROW_CAP = 2048;

template <typename T, bool SUB>
__global__ __launch_bounds__(64) void addsub_wave(const int64_t* __restrict__ arp, const int32_t* __restrict__ acol,
                                                  const T* __restrict__ av, const int64_t* __restrict__ brp,
                                                  const int32_t* __restrict__ bcol, const T* __restrict__ bv,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ tcol,
                                                  T* __restrict__ tval) {
    __shared__ int32_t sc[WROW_CAP];
    __shared__ T sv[WROW_CAP];
    const int64_t r = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t a0 = arp[r], la = arp[r + 1] - a0, b0 = brp[r], lb = brp[r + 1] - b0;
    for (int64_t i = lane; i < la; i += 64) {
        sc[i] = acol[a0 + i];
        sv[i] = av[a0 + i];
    }
    for (int64_t i = lane; i < lb; i += 64) {
        sc[la + i] = bcol[b0 + i];
        sv[la + i] = bv[b0 + i];
    }
    __syncthreads();
    if (lane == 0) {
        const int64_t base = a0 + b0;
        int32_t n = 0;
        merge_range<T, SUB>(0, la, la, la + lb, sc, sv, sc, sv, [&](int32_t c, T v) {
            if (Arith<T>::nz(v)) {
                tcol[base + n] = c;
                tval[base + n] = v;
                ++n;
            }
        });
        cnt[r] = n;
    }
}

template <typename T>
__global__ __launch_bounds__(64) void addsub_place(const int64_t* __restrict__ arp, const int64_t* __restrict__ brp,
                                                   const int64_t* __restrict__ orp, const int32_t* __restrict__ tcol,
                                                   const T* __restrict__ tval, int32_t* __restrict__ ocol,
                                                   T* __restrict__ ov) {
    const int64_t r = blockIdx.x, src = arp[r] + brp[r], dst = orp[r], n = orp[r + 1] - dst;
    for (int64_t i = threadIdx.x; i < n; i += 64) {
        ocol[dst + i] = tcol[src + i];
        ov[dst + i] = tval[src + i];
    }
}

int addsub_wave_path(const bsm_csr* a, const bsm_csr* b, bool sub, bsm_csr** out, hipStream_t s) {
    const uint64_t rows = a->rows, ub = a->nnz + b->nnz;
    CsrGuard g;
    DBuf cnt, orp, ws, tcol, tval;
    auto run = [&]<typename T, bool SUB>() -> int {
        BSM_TRY(cnt.alloc(rows * sizeof(int32_t), s));
        BSM_TRY(orp.alloc((rows + 1) * sizeof(int64_t), s));
        BSM_TRY(ws.alloc(scan_workspace_bytes(rows), s));
        BSM_TRY(tcol.alloc((ub + 1) * sizeof(int32_t), s));
        BSM_TRY(tval.alloc((ub + 1) * sizeof(T), s));
        addsub_wave<T, SUB><<<(unsigned)rows, 64, 0, s>>>(a->row_ptr, a->col, static_cast<const T*>(a->vals),
                                                         b->row_ptr, b->col, static_cast<const T*>(b->vals),
                                                         cnt.as<int32_t>(), tcol.as<int32_t>(), tval.as<T>());
        BSM_HIP_TRY(hipGetLastError());
        BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), orp.as<int64_t>(), rows, ws.p, ws.bytes, s));
        // the output at the nnz(a) + nnz(b) bound: its count arrives with the call's one sync
        BSM_TRY(csr_alloc(&g.m, a->dtype, rows, a->cols, ub));
        BSM_HIP_TRY(hipMemcpyAsync(g.m->row_ptr, orp.p, (rows + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
        addsub_place<T><<<(unsigned)rows, 64, 0, s>>>(a->row_ptr, b->row_ptr, orp.as<int64_t>(), tcol.as<int32_t>(),
                                                      tval.as<T>(), g.m->col, static_cast<T*>(g.m->vals));
        BSM_HIP_TRY(hipGetLastError());
        int64_t nnz = 0;
        BSM_HIP_TRY(read_dev(&nnz, orp.as<int64_t>() + rows, sizeof(int64_t), s));  // syncs the stream
        g.m->nnz = (uint64_t)nnz;
        return BSM_OK;
    };
    BSM_TRY(dispatch_dtype(a->dtype, [&]<typename T>() -> int {
        return sub ? run.template operator()<T, true>() : run.template operator()<T, false>();
    }));
    *out = g.release();
    return BSM_OK;
}

}  // namespace

int sparse_addsub_dispatch(const bsm_csr* a, const bsm_csr* b, bool sub, bsm_csr** out, hipStream_t s) {
    BSM_REQUIRE(a && b && out, BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->dtype == b->dtype, BSM_ERR_INVALID, "operands have different scalar types");
    BSM_REQUIRE(a->rows == b->rows && a->cols == b->cols, BSM_ERR_DIMENSIONS, "IncorrectDimensions");
    BSM_REQUIRE(a->rows > 0, BSM_ERR_PANIC,
                "%s on a matrix with 0 rows: the reference's row loop never terminates (sparse.rs:%s)",
                sub ? "sub_sparse" : "add_sparse", sub ? "593-596" : "533-537");
    // every row short enough for one wave (the operands' analysed longest
    // rows; a device-built operand not yet analysed takes the general path);
    // BSM_SS_WAVE=0: the general path always (A/B)
    const bool wave_ok = !getenv("BSM_SS_WAVE") || atoi(getenv("BSM_SS_WAVE")) != 0;
    if (wave_ok && a->analysed && b->analysed && a->max_row_len + b->max_row_len <= (uint64_t)WROW_CAP &&
        (a->nnz + b->nnz) * (sizeof(int32_t) + dtype_size(a->dtype)) <= (1ull << 30))
        return addsub_wave_path(a, b, sub, out, s);
    const uint64_t rows = a->rows;
    DBuf cnt, lflag, lpos, ws;
    CsrGuard g;
    BSM_TRY(cnt.alloc(rows * sizeof(int32_t), s));
    BSM_TRY(lflag.alloc(rows * sizeof(int32_t), s));
    BSM_TRY(lpos.alloc((rows + 1) * sizeof(int64_t), s));
    BSM_TRY(ws.alloc(scan_workspace_bytes(rows), s));
    DBuf orp;
    BSM_TRY(orp.alloc((rows + 1) * sizeof(int64_t), s));
    // BSM_SS_DEBUG=3: host time per phase (each mark synchronises the stream)
    static const bool tdbg = getenv("BSM_SS_DEBUG") && atoi(getenv("BSM_SS_DEBUG")) == 3;
    auto t_last = host_now();
    auto tmark = [&](const char* what) {
        if (!tdbg) return;
        (void)hipStreamSynchronize(s);
        fprintf(stderr, "[bsm ss time] %-28s %8.3f ms\n", what, ms_since(t_last));
        t_last = host_now();
    };
    auto run = [&]<typename T, bool SUB>() -> int {
        const T* av = static_cast<const T*>(a->vals);
        const T* bv = static_cast<const T*>(b->vals);
        addsub_count<T, SUB><<<grid_of(rows), 256, 0, s>>>((int64_t)rows, a->row_ptr, a->col, av, b->row_ptr, b->col,
                                                           bv, cnt.as<int32_t>(), lflag.as<int32_t>());
        BSM_HIP_TRY(hipGetLastError());
        // long rows: list, pieces, piece counts
        BSM_TRY(exclusive_scan_i32_to_i64(lflag.as<int32_t>(), lpos.as<int64_t>(), rows, ws.p, ws.bytes, s));
        int64_t n_long = 0;
        BSM_HIP_TRY(read_dev(&n_long, lpos.as<int64_t>() + rows, sizeof(int64_t), s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        tmark("count + long-row scan");
        DBuf long_rows, mval, pstart, pieces, pcnt, poff, first, ws2, tcol, tval;
        DBuf scnt, srow, soff, ws3;  // the split path's used-position flags, long-row starts, offsets
        // host inputs of queued H2D copies: alive until the call's last sync
        std::vector<LrChunk> hc;
        std::vector<int64_t> ps;
        // BSM_SS_SPLIT=0: the round-2 wave-per-piece merge (piece_merge), for A/B
        static const bool split = !getenv("BSM_SS_SPLIT") || atoi(getenv("BSM_SS_SPLIT")) != 0;
        const int64_t n_slots = (int64_t)(a->nnz + b->nnz + 1);
        int64_t n_pieces = 0;
        if (n_long) {
            BSM_TRY(long_rows.alloc(n_long * sizeof(int64_t), s));
            BSM_TRY(mval.alloc(n_long * sizeof(int32_t), s));
            BSM_TRY(pstart.alloc((n_long + 1) * sizeof(int64_t), s));
            DBuf ext;
            BSM_TRY(ext.alloc(4 * n_long * sizeof(int64_t), s));
            compact_flags<<<grid_of(rows), 256, 0, s>>>((int64_t)rows, lflag.as<int32_t>(), lpos.as<int64_t>(),
                                                        long_rows.as<int64_t>());
            long_extents<<<grid_of(n_long), 256, 0, s>>>(n_long, long_rows.as<int64_t>(), a->row_ptr, b->row_ptr,
                                                         ext.as<int64_t>());
            BSM_HIP_TRY(hipGetLastError());
            std::vector<int64_t> hx(4 * n_long);
            BSM_HIP_TRY(hipMemcpyAsync(hx.data(), ext.p, hx.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s));
            BSM_HIP_TRY(hipStreamSynchronize(s));
        tmark("long rows + extents");
            for (int64_t l = 0; l < n_long; ++l)
                for (int64_t side = 0; side < 2; ++side)
                    for (int64_t b0 = hx[4 * l + 2 * side]; b0 < hx[4 * l + 2 * side + 1]; b0 += LR_CHUNK)
                        hc.push_back({l, side, b0, std::min(b0 + LR_CHUNK, hx[4 * l + 2 * side + 1]), 0});
            const int64_t n_chunks = (int64_t)hc.size();
            // the host-built chunk list and piece starts go up from pinned
            // staging (a pageable copy behind running kernels can stall the
            // host); three regions, all read before the call's last sync
            const size_t hc_b = (size_t)n_chunks * sizeof(LrChunk), ps_b = (size_t)(n_long + 1) * sizeof(int64_t);
            const size_t hc_al = (hc_b + 255) & ~size_t(255);
            char* pin = static_cast<char*>(pinned(2 * hc_al + ps_b));
            auto h2d = [&](void* dst, const void* src, size_t bytes, size_t off) -> int {
                if (!bytes) return BSM_OK;
                if (pin) {
                    std::memcpy(pin + off, src, bytes);
                    BSM_HIP_TRY(hipMemcpyAsync(dst, pin + off, bytes, hipMemcpyHostToDevice, s));
                } else {
                    BSM_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
                }
                return BSM_OK;
            };
            DBuf chunks, ccnt;
            BSM_TRY(chunks.alloc((n_chunks ? n_chunks : 1) * sizeof(LrChunk), s));
            BSM_TRY(ccnt.alloc((n_chunks ? n_chunks : 1) * sizeof(int64_t), s));
            BSM_HIP_TRY(hipMemsetAsync(mval.p, 0xff, n_long * sizeof(int32_t), s));  // -1
            std::vector<int64_t> hcnt(n_chunks);
            if (n_chunks) {
                BSM_TRY(h2d(chunks.p, hc.data(), hc_b, 0));
                chunk_reduce<true><<<(unsigned)n_chunks, 256, 0, s>>>(chunks.as<LrChunk>(), a->col, b->col,
                                                                      mval.as<int32_t>(), nullptr);
                chunk_reduce<false><<<(unsigned)n_chunks, 256, 0, s>>>(chunks.as<LrChunk>(), a->col, b->col,
                                                                       mval.as<int32_t>(), ccnt.as<int64_t>());
                BSM_HIP_TRY(hipGetLastError());
                BSM_HIP_TRY(hipMemcpyAsync(hcnt.data(), ccnt.p, n_chunks * sizeof(int64_t), hipMemcpyDeviceToHost, s));
                BSM_HIP_TRY(hipStreamSynchronize(s));  // hc (host) is read by the copy above
            }
        tmark("row maxima + counts");
            // M pairs per row: min of the two sides' counts; chunk offsets
            std::vector<int64_t> cnt_side(2 * n_long, 0);
            ps.assign(n_long + 1, 0);
            for (int64_t i = 0; i < n_chunks; ++i) {
                hc[i].off = cnt_side[2 * hc[i].l + hc[i].side];
                cnt_side[2 * hc[i].l + hc[i].side] += hcnt[i];
            }
            for (int64_t l = 0; l < n_long; ++l) ps[l + 1] = ps[l] + std::min(cnt_side[2 * l], cnt_side[2 * l + 1]) + 1;
            n_pieces = ps[n_long];
            if (getenv("BSM_SS_DEBUG")) {  // the long rows' cut: M occurrences per side and the pieces
                for (int64_t l = 0; l < n_long && l < 4; ++l)
                    fprintf(stderr, "[bsm ss debug] long row %lld: extents a %lld b %lld, M count a %lld b %lld\n",
                            (long long)l, (long long)(hx[4 * l + 1] - hx[4 * l]), (long long)(hx[4 * l + 3] - hx[4 * l + 2]),
                            (long long)cnt_side[2 * l], (long long)cnt_side[2 * l + 1]);
                fprintf(stderr, "[bsm ss debug] long rows %lld, chunks %lld, pieces %lld\n", (long long)n_long,
                        (long long)n_chunks, (long long)n_pieces);
            }
            BSM_TRY(h2d(pstart.p, ps.data(), ps_b, 2 * hc_al));
            BSM_TRY(pieces.alloc(n_pieces * sizeof(Piece), s));
            BSM_TRY(pcnt.alloc(n_pieces * sizeof(int32_t), s));
            BSM_TRY(poff.alloc((n_pieces + 1) * sizeof(int64_t), s));
            BSM_TRY(first.alloc(n_pieces * sizeof(int64_t), s));
            BSM_TRY(ws2.alloc(scan_workspace_bytes(n_pieces), s));
            long_piece_init<<<(unsigned)n_long, 256, 0, s>>>(n_long, long_rows.as<int64_t>(), ext.as<int64_t>(),
                                                             pstart.as<int64_t>(), pieces.as<Piece>(),
                                                             first.as<int64_t>());
            if (n_chunks) {
                BSM_TRY(h2d(chunks.p, hc.data(), hc_b, hc_al));
                chunk_pieces<<<(unsigned)n_chunks, 256, 0, s>>>(chunks.as<LrChunk>(), a->col, b->col, mval.as<int32_t>(),
                                                                pstart.as<int64_t>(), pieces.as<Piece>());
            }
            BSM_HIP_TRY(hipGetLastError());
        tmark("pieces");
            BSM_TRY(tcol.alloc((a->nnz + b->nnz + 1) * sizeof(int32_t), s));
            BSM_TRY(tval.alloc((a->nnz + b->nnz + 1) * sizeof(T), s));
            BSM_REQUIRE(n_pieces < (1ll << 31), BSM_ERR_UNSUPPORTED, "too many pieces");
            if (split) {  // recursive cut, one lane per leaf; outputs placed by a scan of the slot counts
                BSM_TRY(scnt.alloc(n_slots * sizeof(int32_t), s));
                BSM_TRY(srow.alloc(n_long * sizeof(int64_t), s));  // the long rows' first positions
                BSM_TRY(soff.alloc((n_slots + 1) * sizeof(int64_t), s));
                BSM_TRY(ws3.alloc(scan_workspace_bytes((uint64_t)n_slots), s));
                BSM_HIP_TRY(hipMemsetAsync(tcol.p, 0xff, n_slots * sizeof(int32_t), s));  // -1: unused
                const char* ssd4 = getenv("BSM_SS_DEBUG");
                DBuf sdbg;
                if (ssd4 && atoi(ssd4) == 4) {
                    BSM_TRY(sdbg.alloc(9 * n_pieces * sizeof(unsigned long long), s));
                    BSM_HIP_TRY(hipMemsetAsync(sdbg.p, 0, 9 * n_pieces * sizeof(unsigned long long), s));
                }
                const size_t split_lds = 2 * split_cap<T>() * (sizeof(int32_t) + sizeof(T));
                // BSM_SS_PRESPLIT=1 (A/B; off by default, and under BSM_SS_DEBUG=4,
                // whose stamps are per top piece): a cuts-only pass first spreads
                // every piece over up to PRE_CUTS + 1 workgroups of the full pass.
                // Within +-5 % of the single pass at the benches' sizes
                // (profiles/r03_s2h_*), so the single pass stays the default.
                static const bool presplit = getenv("BSM_SS_PRESPLIT") && atoi(getenv("BSM_SS_PRESPLIT")) != 0;
                if (presplit && !sdbg.p && (uint64_t)n_pieces * (PRE_CUTS + 1) < (1ull << 31)) {
                    const int64_t n2 = n_pieces * (PRE_CUTS + 1);
                    DBuf pieces2, cnt2;
                    BSM_TRY(pieces2.alloc(n2 * sizeof(Piece), s));
                    BSM_TRY(cnt2.alloc(sizeof(unsigned), s));
                    BSM_HIP_TRY(hipMemsetAsync(cnt2.p, 0, sizeof(unsigned), s));
                    piece_split<T, SUB, true><<<(unsigned)n_pieces, 64, split_lds, s>>>(
                        pieces.as<Piece>(), a->col, av, b->col, bv, tcol.as<int32_t>(), tval.as<T>(), nullptr, nullptr,
                        pieces2.as<Piece>(), cnt2.as<unsigned>());
                    piece_split<T, SUB><<<(unsigned)n2, 64, split_lds, s>>>(
                        pieces2.as<Piece>(), a->col, av, b->col, bv, tcol.as<int32_t>(), tval.as<T>(), nullptr,
                        cnt2.as<unsigned>());
                } else {
                    piece_split<T, SUB><<<(unsigned)n_pieces, 64, split_lds, s>>>(
                        pieces.as<Piece>(), a->col, av, b->col, bv, tcol.as<int32_t>(), tval.as<T>(),
                        sdbg.as<unsigned long long>());
                }
                pos_flags<<<grid_of((uint64_t)n_slots), 256, 0, s>>>(n_slots, tcol.as<int32_t>(), scnt.as<int32_t>());
                if (sdbg.p) {
                    std::vector<unsigned long long> h(9 * n_pieces);
                    BSM_HIP_TRY(hipMemcpyAsync(h.data(), sdbg.p, h.size() * 8, hipMemcpyDeviceToHost, s));
                    BSM_HIP_TRY(hipStreamSynchronize(s));
                    int64_t worst = 0;
                    double sum[9] = {};
                    for (int64_t q = 0; q < n_pieces; ++q) {
                        for (int k = 0; k < 9; ++k) sum[k] += (double)h[9 * q + k];
                        if (h[9 * q] > h[9 * worst]) worst = q;
                    }
                    const unsigned long long* w = &h[9 * worst];
                    fprintf(stderr, "[bsm ss split] %lld pieces, mean %.0f cycles (cut %.0f, leaves %.0f, one-sided %.0f, "
                            "staging %.0f; scanned %.0f, flushes %.1f, leaves %.0f, size %.0f); longest: %llu cycles "
                            "(cut %llu, leaves %llu, one-sided %llu, staging %llu; scanned %llu, flushes %llu, leaves "
                            "%llu, size %llu)\n", (long long)n_pieces, sum[0] / n_pieces, sum[1] / n_pieces,
                            sum[2] / n_pieces, sum[3] / n_pieces, sum[4] / n_pieces, sum[5] / n_pieces,
                            sum[6] / n_pieces, sum[7] / n_pieces, sum[8] / n_pieces, w[0], w[1], w[2], w[3], w[4], w[5],
                            w[6], w[7], w[8]);
                }
                // (scnt: 1 at every used scratch position, srow: its row)
                BSM_HIP_TRY(hipGetLastError());
                BSM_TRY(exclusive_scan_i32_to_i64(scnt.as<int32_t>(), soff.as<int64_t>(), (uint64_t)n_slots, ws3.p,
                                                  ws3.bytes, s));
                long_row_totals_slots<<<grid_of(n_long), 256, 0, s>>>(n_long, long_rows.as<int64_t>(), a->row_ptr,
                                                                       b->row_ptr, soff.as<int64_t>(), cnt.as<int32_t>(),
                                                                       srow.as<int64_t>());
                BSM_HIP_TRY(hipGetLastError());
        tmark("piece_split + scan");
            } else {
            const char* ssd = getenv("BSM_SS_DEBUG");
            DBuf pdbg;
            if (ssd && atoi(ssd) >= 2) {
                BSM_TRY(pdbg.alloc(6 * n_pieces * sizeof(unsigned long long), s));
                BSM_HIP_TRY(hipMemsetAsync(pdbg.p, 0, 6 * n_pieces * sizeof(unsigned long long), s));
            }
            piece_merge<T, SUB><<<(unsigned)n_pieces, 64, 2 * PIECE_CAP * (sizeof(int32_t) + sizeof(T)), s>>>(
                pieces.as<Piece>(), a->col, av, b->col, bv, tcol.as<int32_t>(), tval.as<T>(), pcnt.as<int32_t>(),
                pdbg.as<unsigned long long>());
            BSM_HIP_TRY(hipGetLastError());
            if (pdbg.p) {  // per-piece s_memtime stamps: where a merge step's cycles go
                std::vector<unsigned long long> h(6 * n_pieces);
                BSM_HIP_TRY(hipMemcpyAsync(h.data(), pdbg.p, h.size() * sizeof(unsigned long long),
                                           hipMemcpyDeviceToHost, s));
                BSM_HIP_TRY(hipStreamSynchronize(s));
                double sum[6] = {}, mx_len = 0, mx_cyc = 0;
                for (int64_t p = 0; p < n_pieces; ++p) {
                    for (int k = 0; k < 6; ++k) sum[k] += (double)h[6 * p + k];
                    const double cyc = (double)(h[6 * p] + h[6 * p + 1] + h[6 * p + 4]);
                    if (cyc > mx_cyc) {
                        mx_cyc = cyc;
                        mx_len = (double)h[6 * p + 5];
                    }
                }
                fprintf(stderr, "[bsm ss debug] piece_merge over %lld pieces: per piece staging %.0f cycles, merge loop "
                        "%.0f (window refills %.0f) for %.0f steps = %.1f cycles/step, tail %.0f; longest piece %.0f "
                        "cycles over %.0f entries\n", (long long)n_pieces, sum[0] / n_pieces, sum[1] / n_pieces,
                        sum[2] / n_pieces, sum[3] / n_pieces, sum[3] > 0 ? sum[1] / sum[3] : 0.0, sum[4] / n_pieces,
                        mx_cyc, mx_len);
            }
            BSM_TRY(exclusive_scan_i32_to_i64(pcnt.as<int32_t>(), poff.as<int64_t>(), n_pieces, ws2.p, ws2.bytes, s));
            long_row_totals<<<grid_of(n_long), 256, 0, s>>>(n_long, long_rows.as<int64_t>(), pstart.as<int64_t>(),
                                                             poff.as<int64_t>(), cnt.as<int32_t>());
            BSM_HIP_TRY(hipGetLastError());
            }
        }
        BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), orp.as<int64_t>(), rows, ws.p, ws.bytes, s));
        int64_t nnz = 0;
        // the output holds at most nnz(a) + nnz(b) entries: allocated at that
        // bound (when it is small) the fill is queued behind the scan and the
        // count is read with the call's last sync; else the count first
        const uint64_t nnz_ub = a->nnz + b->nnz;
        const bool ub = nnz_ub * (sizeof(int32_t) + sizeof(T)) <= (1ull << 30);
        if (!ub) {
            BSM_HIP_TRY(read_dev(&nnz, orp.as<int64_t>() + rows, sizeof(int64_t), s));
            BSM_HIP_TRY(hipStreamSynchronize(s));
        }
        tmark("row scan + nnz");
        BSM_TRY(csr_alloc(&g.m, a->dtype, rows, a->cols, ub ? nnz_ub : (uint64_t)nnz));
        tmark("output alloc");
        BSM_HIP_TRY(hipMemcpyAsync(g.m->row_ptr, orp.p, (rows + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
        addsub_fill<T, SUB><<<grid_of(rows), 256, 0, s>>>((int64_t)rows, a->row_ptr, a->col, av, b->row_ptr, b->col,
                                                          bv, orp.as<int64_t>(), g.m->col, static_cast<T*>(g.m->vals));
        BSM_HIP_TRY(hipGetLastError());
        if (n_pieces && split) {
            pos_copy<T><<<grid_of((uint64_t)n_slots), 256, 0, s>>>(
                n_slots, tcol.as<int32_t>(), soff.as<int64_t>(), n_long, long_rows.as<int64_t>(), srow.as<int64_t>(),
                orp.as<int64_t>(), tval.as<T>(), g.m->col, static_cast<T*>(g.m->vals));
            BSM_HIP_TRY(hipGetLastError());
        } else if (n_pieces) {
            piece_copy<T><<<(unsigned)n_pieces, 64, 0, s>>>(pieces.as<Piece>(), pcnt.as<int32_t>(), poff.as<int64_t>(),
                                                            first.as<int64_t>(), orp.as<int64_t>(), tcol.as<int32_t>(),
                                                            tval.as<T>(), g.m->col, static_cast<T*>(g.m->vals));
            BSM_HIP_TRY(hipGetLastError());
        }
        if (ub) {
            BSM_HIP_TRY(read_dev(&nnz, orp.as<int64_t>() + rows, sizeof(int64_t), s));  // syncs the stream
            g.m->nnz = (uint64_t)nnz;
        }
        BSM_HIP_TRY(hipStreamSynchronize(s));  // the piece buffers die with this scope
        tmark("fill + copy");
        return BSM_OK;
    };
    BSM_TRY(dispatch_dtype(a->dtype, [&]<typename T>() -> int {
        return sub ? run.template operator()<T, true>() : run.template operator()<T, false>();
    }));
    tmark("scope exit (frees)");
    // no eager csr_analyse: the result's columns come from the operands (in
    // bounds); its row order and longest row are found when first needed
    *out = g.release();
    return BSM_OK;
}

int sparse_mul_dispatch(const bsm_csr* a, const bsm_csr* b, bsm_csr** out, hipStream_t s) {
    BSM_REQUIRE(a && b && out, BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->dtype == b->dtype, BSM_ERR_INVALID, "operands have different scalar types");
    const uint64_t rows = a->rows, cols = b->cols;
    const unsigned cb = bits_for(cols), rb = bits_for(rows);
    BSM_REQUIRE(cb + rb <= 64 && cb < 64, BSM_ERR_UNSUPPORTED, "mul_sparse: rows x cols too large for 64-bit keys");
    CsrGuard g;
    // 1. rhs^T (stable, like the reference's transpose)
    bsm_csr* bt_raw = nullptr;
    BSM_TRY(transpose_dispatch(b, &bt_raw, s));
    CsrGuard bt;
    bt.m = bt_raw;
    // 2. candidates
    const uint64_t nnz_a = a->nnz;
    DBuf cnt, off, ws;
    BSM_TRY(cnt.alloc((nnz_a ? nnz_a : 1) * sizeof(int32_t), s));
    BSM_TRY(off.alloc((nnz_a + 1) * sizeof(int64_t), s));
    BSM_TRY(ws.alloc(scan_workspace_bytes(nnz_a ? nnz_a : 1), s));
    if (nnz_a) {
        spgemm_count<<<grid_of(nnz_a), 256, 0, s>>>(nnz_a, a->col, b->rows, b->row_ptr, cnt.as<int32_t>());
        BSM_HIP_TRY(hipGetLastError());
    }
    BSM_TRY(exclusive_scan_i32_to_i64(cnt.as<int32_t>(), off.as<int64_t>(), nnz_a, ws.p, ws.bytes, s));
    int64_t total = 0;
    BSM_HIP_TRY(read_dev(&total, off.as<int64_t>() + nnz_a, sizeof(int64_t), s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_REQUIRE(total < (int64_t)UINT32_MAX, BSM_ERR_UNSUPPORTED,
                "mul_sparse: %lld expanded products (limit 2^32)", (long long)total);
    uint64_t n_cand = 0;
    DBuf keys, keys_s, tmp, cand, n_dev;
    if (total > 0) {
        BSM_TRY(keys.alloc(total * sizeof(uint64_t), s));
        BSM_TRY(keys_s.alloc(total * sizeof(uint64_t), s));
        spgemm_expand<<<grid_of(total), 256, 0, s>>>((uint64_t)total, nnz_a, off.as<int64_t>(), a->row_ptr, rows,
                                                     a->col, b->row_ptr, b->col, cb, keys.as<uint64_t>());
        BSM_HIP_TRY(hipGetLastError());
        const unsigned end_bit = cb + rb > 0 ? cb + rb : 1;
        size_t tb = 0;
        BSM_HIP_TRY(rocprim::radix_sort_keys(nullptr, tb, keys.as<uint64_t>(), keys_s.as<uint64_t>(), (size_t)total,
                                             0u, end_bit, s));
        BSM_TRY(tmp.alloc(tb ? tb : 1, s));
        BSM_HIP_TRY(rocprim::radix_sort_keys(tmp.p, tb, keys.as<uint64_t>(), keys_s.as<uint64_t>(), (size_t)total,
                                             0u, end_bit, s));
        BSM_TRY(n_dev.alloc(sizeof(uint64_t), s));
        // unique into `keys` (free after the sort)
        size_t ub = 0;
        BSM_HIP_TRY(rocprim::unique(nullptr, ub, keys_s.as<uint64_t>(), keys.as<uint64_t>(), n_dev.as<uint64_t>(),
                                    (size_t)total, rocprim::equal_to<uint64_t>(), s));
        DBuf tmp2;
        BSM_TRY(tmp2.alloc(ub ? ub : 1, s));
        BSM_HIP_TRY(rocprim::unique(tmp2.p, ub, keys_s.as<uint64_t>(), keys.as<uint64_t>(), n_dev.as<uint64_t>(),
                                    (size_t)total, rocprim::equal_to<uint64_t>(), s));
        BSM_HIP_TRY(read_dev(&n_cand, n_dev.p, sizeof(uint64_t), s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
    }
    // 3. the merge per candidate, 4. keep the nonzero ones
    const size_t es = dtype_size(a->dtype);
    DBuf val, keep, pos, orow;
    BSM_TRY(val.alloc((n_cand ? n_cand : 1) * es, s));
    BSM_TRY(keep.alloc((n_cand ? n_cand : 1) * sizeof(int32_t), s));
    BSM_TRY(pos.alloc((n_cand + 1) * sizeof(int64_t), s));
    DBuf ws2;
    BSM_TRY(ws2.alloc(scan_workspace_bytes(n_cand ? n_cand : 1), s));
    int64_t nnz = 0;
    auto run = [&]<typename T>() -> int {
        if (n_cand) {
            spgemm_merge<T><<<grid_of(n_cand), 256, 0, s>>>(n_cand, keys.as<uint64_t>(), cb, a->row_ptr, a->col,
                                                            static_cast<const T*>(a->vals), bt.m->row_ptr, bt.m->col,
                                                            static_cast<const T*>(bt.m->vals), val.as<T>(),
                                                            keep.as<int32_t>());
            BSM_HIP_TRY(hipGetLastError());
        }
        BSM_TRY(exclusive_scan_i32_to_i64(keep.as<int32_t>(), pos.as<int64_t>(), n_cand, ws2.p, ws2.bytes, s));
        BSM_HIP_TRY(read_dev(&nnz, pos.as<int64_t>() + n_cand, sizeof(int64_t), s));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        BSM_TRY(csr_alloc(&g.m, a->dtype, rows, cols, (uint64_t)nnz));
        BSM_TRY(orow.alloc((nnz ? nnz : 1) * sizeof(int64_t), s));
        if (n_cand) {
            spgemm_scatter<T><<<grid_of(n_cand), 256, 0, s>>>(n_cand, keys.as<uint64_t>(), cb, val.as<T>(),
                                                              pos.as<int64_t>(), orow.as<int64_t>(), g.m->col,
                                                              static_cast<T*>(g.m->vals));
            BSM_HIP_TRY(hipGetLastError());
        }
        rows_to_ptr<<<grid_of(rows + 1), 256, 0, s>>>(rows, nnz, orow.as<int64_t>(), g.m->row_ptr);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    };
    BSM_TRY(dispatch_dtype(a->dtype, run));
    BSM_HIP_TRY(hipStreamSynchronize(s));  // the result is complete when the call returns
    // (no eager csr_analyse: see sparse_addsub_dispatch)
    *out = g.release();
    return BSM_OK;
}

}  // namespace bsm
