// multi.hip -- multi-GPU Csr::mul_dense behind the C-ABI (include/bsm.h,
// "multi-GPU"): row blocks of the CSR on every GPU, X replicated, the dense
// Y assembled by RCCL all-gathers over xGMI (BASELINE.json north_star;
// SURVEY.md §8b bsm_init(n_gpus), §8e).
//
// Reference: Csr::mul_dense (src/sparse.rs:426-446) sums every output row on
// its own (:431-444), so rows split across devices with no reduction, and a
// row's sum does not depend on which device computes it: the assembled Y is
// bit-identical to one GPU's.
//
// Partition. P = chunks x world contiguous row blocks ("pieces") of near-equal
// nnz. Piece i = c*world + g is computed by global rank g in round c. The
// gathered Y holds P slots of `pad` rows (pad = the longest piece), slot i at
// rows [i*pad, (i+1)*pad): round c's all-gather is one in-place
// ncclAllGather of `pad` rows per rank that lands slots c*world .. c*world +
// world - 1, already in global row order. Slot rows past a piece's end stay
// zero (never written), so their nonzero counts are 0 and the compaction over
// all P*pad slot rows writes nothing for them; only the output row_ptr needs
// the slot -> row map (squeeze_row_ptr) when a piece other than the last is
// short.
//
// Streams. Per device a compute stream (the SpMMs, the compaction) and a
// communication stream (the all-gathers). The all-gather of round c waits for
// round c's SpMM by an event and runs while round c+1's SpMM computes; the
// compaction waits for the last all-gather.
#include <rccl/rccl.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bsm_internal.hpp"

#define BSM_NCCL_TRY(expr)                                                                              \
    do {                                                                                                \
        ncclResult_t bsm_r_ = (expr);                                                                   \
        if (bsm_r_ != ncclSuccess) {                                                                    \
            ::bsm::set_error("%s failed: %s (%s:%d)", #expr, ncclGetErrorString(bsm_r_), __FILE__,     \
                             __LINE__);                                                                 \
            return BSM_ERR_COMM;                                                                        \
        }                                                                                               \
    } while (0)

struct bsm_multi {
    int world = 1, first_rank = 0, n_local = 0;
    // no communicator (bsm_multi_create_external): step stops before the
    // all-gathers and the caller moves the slots between ranks
    bool external = false;
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> compute, comm;
};

namespace bsm {
namespace {

constexpr int EV_PER_STEP = 5;  // start, last SpMM end (compute), last all-gather end (comm), compaction start, end

struct Local {
    int device = 0, rank = 0;
    std::vector<bsm_csr*> pieces;  // round c: piece c*world + rank
    bool compacts = false;         // this device compacts the output (bsm_mcsr_set_output_rank)
    // prepared for k
    void* y = nullptr;      // P*pad x k, slot order
    int32_t* nz = nullptr;  // P*pad
    int64_t* rp_pad = nullptr;  // P*pad + 1
    int64_t* rp_out = nullptr;  // rows + 1 (rp_pad itself when no slot is short)
    int32_t* ocol = nullptr;
    void* oval = nullptr;
    void* ws = nullptr;
    uint64_t ws_b = 0;
    int64_t* bounds = nullptr;  // P + 1 (squeeze)
    std::vector<hipEvent_t> round_ev;  // per round: its SpMM is done
    std::vector<hipEvent_t> ev;        // EV_PER_STEP per recorded step
    int steps = 0;
};

}  // namespace
}  // namespace bsm

struct bsm_mcsr {
    bsm_multi* ctx = nullptr;
    int dtype = BSM_F64;
    uint64_t rows = 0, cols = 0, nnz = 0;
    uint32_t chunks = 1, P = 1;
    uint64_t pad = 0;
    std::vector<uint64_t> bounds;  // P + 1
    std::vector<bsm::Local> loc;
    uint64_t k = 0;
    bool prepared = false, squeeze = false;
    int schedule = 0;
    int out_rank = -1;  // -1: every process's first local device compacts; r: only rank r
    // one call at a time per matrix: the gathered Y, the output buffers, the
    // events and the collectives of a step are shared state (recursive:
    // mul_dense runs prepare, step and output under the same hold)
    mutable std::recursive_mutex mu;
};

namespace bsm {
namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(d);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Run f(i) for every local device, in parallel threads when there are
// several (schedule builds and uploads are synchronous per device). The first
// failure's message is carried to the calling thread (errors are thread-local).
template <typename F>
int for_each_local(int n, F&& f) {
    if (n == 1) return f(0);
    std::vector<int> rc(n, BSM_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    th.reserve(n);
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            rc[i] = f(i);
            if (rc[i] != BSM_OK) msg[i] = last_error();
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[i] != BSM_OK) {
            set_error("device %d: %s", i, msg[i].c_str());
            return rc[i];
        }
    return BSM_OK;
}

// Piece bounds: contiguous row blocks of near-equal cost, where a row costs
// its entries plus c = max(1, nnz/rows) (its Y row, its count and its share of
// the compaction). bound i = the first row r with cost(rows before r) >=
// i*total/P (binary search on row_ptr), bounds[0] = 0, bounds[P] = rows.
// For equal row lengths (C4) this is the nnz-balanced split; on skewed
// matrices (long runs of empty rows, one huge row) it caps a piece at
// 2*rows/P + 1 rows, so the P*pad slot rows of the gathered Y stay <= ~2x
// rows (a pure nnz split lets one piece take nearly every row, and every
// device would then hold P times the single-GPU Y). Exact integer
// arithmetic: cost is scaled by rows, cost(r) = rp[r]*rows + r*max(nnz, rows).
template <typename RP>
std::vector<uint64_t> partition_by_cost(const RP* rp, uint64_t rows, uint64_t nnz, uint32_t P) {
    std::vector<uint64_t> b(P + 1);
    using u128 = unsigned __int128;
    const u128 per_row = std::max<uint64_t>(nnz, rows);
    const u128 total = (u128)nnz * rows + (u128)rows * per_row;
    for (uint32_t i = 0; i <= P; ++i) {
        const u128 target = total * i / P;
        uint64_t lo = 0, hi = rows;  // first r in [0, rows) with cost(r) >= target, else rows
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if ((u128)(uint64_t)rp[mid] * rows + (u128)mid * per_row >= target) hi = mid;
            else lo = mid + 1;
        }
        b[i] = lo;
    }
    b[0] = 0;
    b[P] = rows;
    for (uint32_t i = 1; i <= P; ++i) b[i] = std::max(b[i], b[i - 1]);
    return b;
}

__global__ __launch_bounds__(256) void squeeze_row_ptr(const int64_t* __restrict__ rp_pad,
                                                       const int64_t* __restrict__ bounds, uint32_t P,
                                                       uint64_t pad, uint64_t rows, int64_t* __restrict__ rp_out) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > rows) return;
    if (r == rows) {
        rp_out[rows] = rp_pad[(uint64_t)P * pad];
        return;
    }
    uint32_t lo = 0, hi = P;  // the piece i with bounds[i] <= r < bounds[i+1]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if ((uint64_t)bounds[mid] <= r) lo = mid;
        else hi = mid;
    }
    rp_out[r] = rp_pad[(uint64_t)lo * pad + (r - (uint64_t)bounds[lo])];
}

void free_local_buffers(Local& L) {
    for (void* p : {(void*)L.y, (void*)L.nz, (void*)L.ocol, L.oval, L.ws, (void*)L.bounds})
        if (p) (void)hipFree(p);
    if (L.rp_out && L.rp_out != L.rp_pad) (void)hipFree(L.rp_out);
    if (L.rp_pad) (void)hipFree(L.rp_pad);
    L.y = L.oval = L.ws = nullptr;
    L.nz = L.ocol = nullptr;
    L.rp_pad = L.rp_out = L.bounds = nullptr;
    for (auto e : L.round_ev) (void)hipEventDestroy(e);
    for (auto e : L.ev) (void)hipEventDestroy(e);
    L.round_ev.clear();
    L.ev.clear();
    L.steps = 0;
}

// CUs per XCD left to the communication stream (the all-gathers), the
// compute stream masked to the rest: the SpMM's persistent grid holds every CU
// it may use (LDS full, one wave per SIMD), so without a mask an all-gather
// issued beside the next round's SpMM waits for it, or holds CUs that grid
// then lacks. BSM_COMM_CUS=n (default 0 = no masks). The mask's bit order
// is BSM_CU_MASK_ORDER: "xcd" (bit i on XCD i % 8; default) or "linear"
// (bits [32x, 32x + 32) on XCD x). scripts/perf/cu_mask_probe.hip shows which.
int comm_cus_per_xcd() {
    const char* e = getenv("BSM_COMM_CUS");
    return e ? std::max(0, atoi(e)) : 0;
}

int create_streams(bsm_multi* c) {
    c->compute.assign(c->n_local, nullptr);
    c->comm.assign(c->n_local, nullptr);
    const int keep = comm_cus_per_xcd();
    const char* ord = getenv("BSM_CU_MASK_ORDER");
    const bool linear = ord && std::string(ord) == "linear";
    for (int i = 0; i < c->n_local; ++i) {
        DeviceGuard g(c->devices[i]);
        int cus = 0;
        BSM_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->devices[i]));
        const int per_xcd = cus / 8;
        if (keep > 0 && keep < per_xcd && cus % 8 == 0) {
            std::vector<uint32_t> mc((size_t)(cus + 31) / 32, 0u), mm(mc.size(), 0u);
            for (int b = 0; b < cus; ++b) {
                const int in_xcd = linear ? b % per_xcd : b / 8;
                (in_xcd < keep ? mm : mc)[b / 32] |= 1u << (b % 32);
            }
            // NOTE: hipExtStreamCreateWithCUMask takes no flags, so these two
            // streams are BLOCKING with respect to the null stream (the
            // unmasked ones below are hipStreamNonBlocking): null-stream work
            // (pageable copies, hipMemset without a stream) serialises against
            // them. The round-4 CU-mask A/B ran this way.
            BSM_HIP_TRY(hipExtStreamCreateWithCUMask(&c->compute[i], (uint32_t)mc.size(), mc.data()));
            BSM_HIP_TRY(hipExtStreamCreateWithCUMask(&c->comm[i], (uint32_t)mm.size(), mm.data()));
        } else {
            BSM_HIP_TRY(hipStreamCreateWithFlags(&c->compute[i], hipStreamNonBlocking));
            BSM_HIP_TRY(hipStreamCreateWithFlags(&c->comm[i], hipStreamNonBlocking));
        }
    }
    return BSM_OK;
}

void destroy_multi(bsm_multi* c) {
    if (!c) return;
    for (int i = 0; i < (int)c->comms.size(); ++i)
        if (c->comms[i]) {
            DeviceGuard g(c->devices[i]);
            (void)ncclCommDestroy(c->comms[i]);
        }
    for (int i = 0; i < (int)c->compute.size(); ++i) {
        DeviceGuard g(c->devices[i]);
        if (c->compute[i]) (void)hipStreamDestroy(c->compute[i]);
        if (c->comm[i]) (void)hipStreamDestroy(c->comm[i]);
    }
    delete c;
}

bsm_mcsr* new_mcsr(bsm_multi* ctx, int dtype, uint64_t rows, uint64_t cols, uint32_t chunks) {
    auto* m = new bsm_mcsr();
    m->ctx = ctx;
    m->dtype = dtype;
    m->rows = rows;
    m->cols = cols;
    m->chunks = chunks;
    m->P = chunks * (uint32_t)ctx->world;
    m->loc.resize(ctx->n_local);
    for (int i = 0; i < ctx->n_local; ++i) {
        m->loc[i].device = ctx->devices[i];
        m->loc[i].rank = ctx->first_rank + i;
        m->loc[i].compacts = i == 0;
        m->loc[i].pieces.assign(chunks, nullptr);
    }
    return m;
}

void set_bounds(bsm_mcsr* m, std::vector<uint64_t> b) {
    m->bounds = std::move(b);
    m->pad = 0;
    bool short_slot = false;
    for (uint32_t i = 0; i < m->P; ++i) m->pad = std::max(m->pad, m->bounds[i + 1] - m->bounds[i]);
    for (uint32_t i = 0; i + 1 < m->P; ++i) short_slot |= m->bounds[i + 1] - m->bounds[i] != m->pad;
    m->squeeze = short_slot;
}

void free_mcsr(bsm_mcsr* m) {
    if (!m) return;
    for (auto& L : m->loc) {
        DeviceGuard g(L.device);
        for (auto* p : L.pieces) bsm_csr_free(p);
        L.pieces.clear();
        free_local_buffers(L);
    }
    delete m;
}

// The gathered Y (P*pad slot rows) -> the output Csr: scan of the row counts,
// compaction (insert's zero skip, sparse.rs:229), and the slot -> row map of
// row_ptr when a piece other than the last is short.
int compact_local(bsm_mcsr* m, Local& L, hipStream_t s) {
    const uint64_t slot_rows = (uint64_t)m->P * m->pad;
    BSM_TRY(exclusive_scan_i32_to_i64(L.nz, L.rp_pad, slot_rows, L.ws, L.ws_b, s));
    BSM_TRY(compact_dispatch(m->dtype, slot_rows, m->k, L.y, L.rp_pad, L.ocol, L.oval, s));
    if (m->squeeze) {
        squeeze_row_ptr<<<(unsigned)((m->rows + 1 + 255) / 256), 256, 0, s>>>(L.rp_pad, L.bounds, m->P, m->pad,
                                                                              m->rows, L.rp_out);
        BSM_HIP_TRY(hipGetLastError());
    }
    return BSM_OK;
}

}  // namespace

// Upload rows [r0, r1) of a host finalised Csr (absolute row_ptr) as a handle
// on the current device (capi.hip's uploader, rebased to the piece).
int csr_upload_rows(int dtype, uint64_t r0, uint64_t r1, uint64_t cols, const uint64_t* row_ptr,
                    const uint64_t* col_idx, const void* vals, bsm_csr** out, hipStream_t s);

}  // namespace bsm

using namespace bsm;

extern "C" {

int bsm_multi_create(int n_gpus, const int* devices, bsm_multi** out) {
    BSM_REQUIRE(out && n_gpus >= 1, BSM_ERR_INVALID, "bsm_multi_create: need n_gpus >= 1 and an output");
    *out = nullptr;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have == 0) {
        (void)hipGetLastError();
        set_error("bsm_multi_create: no HIP device visible");
        return BSM_ERR_NO_DEVICE;
    }
    BSM_REQUIRE(n_gpus <= have, BSM_ERR_INVALID, "bsm_multi_create: %d GPUs asked, %d visible", n_gpus, have);
    auto* c = new bsm_multi();
    c->world = n_gpus;
    c->n_local = n_gpus;
    c->first_rank = 0;
    for (int i = 0; i < n_gpus; ++i) {
        const int d = devices ? devices[i] : i;
        if (d < 0 || d >= have || std::count(c->devices.begin(), c->devices.end(), d)) {
            delete c;
            set_error("bsm_multi_create: bad or repeated device ordinal %d", d);
            return BSM_ERR_INVALID;
        }
        c->devices.push_back(d);
    }
    int rc = create_streams(c);
    if (rc == BSM_OK) {
        c->comms.assign(n_gpus, nullptr);
        const ncclResult_t r = ncclCommInitAll(c->comms.data(), n_gpus, c->devices.data());
        if (r != ncclSuccess) {
            c->comms.assign(n_gpus, nullptr);
            set_error("ncclCommInitAll(%d): %s", n_gpus, ncclGetErrorString(r));
            rc = BSM_ERR_COMM;
        }
    }
    if (rc != BSM_OK) {
        destroy_multi(c);
        return rc;
    }
    *out = c;
    return BSM_OK;
}

int bsm_multi_unique_id(void* id) {
    BSM_REQUIRE(id, BSM_ERR_INVALID, "null argument");
    static_assert(sizeof(ncclUniqueId) == BSM_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    BSM_NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return BSM_OK;
}

int bsm_multi_create_rank(const void* id, int world, int rank, int device, bsm_multi** out) {
    BSM_REQUIRE(id && out && world >= 1 && rank >= 0 && rank < world && device >= 0, BSM_ERR_INVALID,
                "bsm_multi_create_rank: bad argument (world %d, rank %d, device %d)", world, rank, device);
    *out = nullptr;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have == 0) {
        (void)hipGetLastError();
        set_error("bsm_multi_create_rank: no HIP device visible");
        return BSM_ERR_NO_DEVICE;
    }
    BSM_REQUIRE(device < have, BSM_ERR_INVALID, "bsm_multi_create_rank: device %d of %d", device, have);
    auto* c = new bsm_multi();
    c->world = world;
    c->n_local = 1;
    c->first_rank = rank;
    c->devices = {device};
    int rc = create_streams(c);
    if (rc == BSM_OK) {
        DeviceGuard g(device);
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        c->comms.assign(1, nullptr);
        const ncclResult_t r = ncclCommInitRank(&c->comms[0], world, u, rank);
        if (r != ncclSuccess) {
            c->comms[0] = nullptr;
            set_error("ncclCommInitRank(world %d, rank %d): %s", world, rank, ncclGetErrorString(r));
            rc = BSM_ERR_COMM;
        }
    }
    if (rc != BSM_OK) {
        destroy_multi(c);
        return rc;
    }
    *out = c;
    return BSM_OK;
}

int bsm_multi_create_external(int world, int rank, int device, bsm_multi** out) {
    BSM_REQUIRE(out && world >= 1 && rank >= 0 && rank < world && device >= 0, BSM_ERR_INVALID,
                "bsm_multi_create_external: bad argument (world %d, rank %d, device %d)", world, rank, device);
    *out = nullptr;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have == 0) {
        (void)hipGetLastError();
        set_error("bsm_multi_create_external: no HIP device visible");
        return BSM_ERR_NO_DEVICE;
    }
    BSM_REQUIRE(device < have, BSM_ERR_INVALID, "bsm_multi_create_external: device %d of %d", device, have);
    auto* c = new bsm_multi();
    c->world = world;
    c->n_local = 1;
    c->first_rank = rank;
    c->external = true;
    c->devices = {device};
    c->comms.assign(1, nullptr);
    const int rc = create_streams(c);
    if (rc != BSM_OK) {
        destroy_multi(c);
        return rc;
    }
    *out = c;
    return BSM_OK;
}

int bsm_multi_is_external(const bsm_multi* ctx, int* external) {
    BSM_REQUIRE(ctx && external, BSM_ERR_INVALID, "null argument");
    *external = ctx->external ? 1 : 0;
    return BSM_OK;
}

int bsm_partition_rows(const uint64_t* row_ptr, uint64_t rows, uint32_t pieces, uint64_t* bounds) {
    BSM_REQUIRE(row_ptr && bounds && pieces >= 1, BSM_ERR_INVALID, "bsm_partition_rows: bad argument");
    const auto b = partition_by_cost(row_ptr, rows, row_ptr[rows], pieces);
    std::copy(b.begin(), b.end(), bounds);
    return BSM_OK;
}

int bsm_multi_info(const bsm_multi* ctx, int* world, int* n_local, int* first_rank) {
    BSM_REQUIRE(ctx, BSM_ERR_INVALID, "null context");
    if (world) *world = ctx->world;
    if (n_local) *n_local = ctx->n_local;
    if (first_rank) *first_rank = ctx->first_rank;
    return BSM_OK;
}

int bsm_multi_broadcast(bsm_multi* ctx, void* const* bufs, uint64_t bytes, int root) {
    BSM_REQUIRE(ctx && (bytes == 0 || bufs) && root >= 0 && root < ctx->world, BSM_ERR_INVALID,
                "bsm_multi_broadcast: bad argument");
    BSM_REQUIRE(!ctx->external, BSM_ERR_UNSUPPORTED,
                "bsm_multi_broadcast: an external context has no communicator (copy X to every rank yourself)");
    if (bytes == 0) return BSM_OK;
    for (int i = 0; i < ctx->n_local; ++i) BSM_REQUIRE(bufs[i], BSM_ERR_INVALID, "null buffer %d", i);
    BSM_NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < ctx->n_local; ++i) {
        const ncclResult_t r = ncclBroadcast(bufs[i], bufs[i], bytes, ncclChar, root, ctx->comms[i], ctx->comm[i]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            set_error("ncclBroadcast: %s", ncclGetErrorString(r));
            return BSM_ERR_COMM;
        }
    }
    BSM_NCCL_TRY(ncclGroupEnd());
    for (int i = 0; i < ctx->n_local; ++i) {
        DeviceGuard g(ctx->devices[i]);
        BSM_HIP_TRY(hipStreamSynchronize(ctx->comm[i]));
    }
    return BSM_OK;
}

void bsm_multi_destroy(bsm_multi* ctx) { destroy_multi(ctx); }

int bsm_mcsr_upload(bsm_multi* ctx, int dtype, uint64_t rows, uint64_t cols, uint64_t nnz, const uint64_t* row_ptr,
                    const uint64_t* col_idx, const void* vals, uint32_t chunks, bsm_mcsr** out) {
    BSM_REQUIRE(ctx && out && row_ptr && (nnz == 0 || (col_idx && vals)) && chunks >= 1, BSM_ERR_INVALID,
                "bsm_mcsr_upload: null argument or chunks = 0");
    BSM_REQUIRE(dtype_size(dtype) != 0, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    BSM_REQUIRE(row_ptr[0] == 0 && row_ptr[rows] == nnz, BSM_ERR_INVALID, "row_ptr must start at 0 and end at nnz");
    for (uint64_t r = 0; r < rows; ++r)
        BSM_REQUIRE(row_ptr[r] <= row_ptr[r + 1], BSM_ERR_PANIC, "row_ptr not monotone at row %llu",
                    (unsigned long long)r);
    *out = nullptr;
    bsm_mcsr* m = new_mcsr(ctx, dtype, rows, cols, chunks);
    m->nnz = nnz;
    set_bounds(m, partition_by_cost(row_ptr, rows, nnz, m->P));
    const int rc = for_each_local(ctx->n_local, [&](int i) -> int {
        Local& L = m->loc[i];
        DeviceGuard g(L.device);
        for (uint32_t c = 0; c < chunks; ++c) {
            const uint32_t p = c * (uint32_t)ctx->world + (uint32_t)L.rank;
            BSM_TRY(csr_upload_rows(dtype, m->bounds[p], m->bounds[p + 1], cols, row_ptr, col_idx, vals,
                                    &L.pieces[c], ctx->compute[i]));
        }
        return BSM_OK;
    });
    if (rc != BSM_OK) {
        free_mcsr(m);
        return rc;
    }
    *out = m;
    return BSM_OK;
}

int bsm_mcsr_generate(bsm_multi* ctx, int dtype, uint64_t seed, uint64_t rows, uint32_t n_cols, int rowlen_kind,
                      uint32_t a, uint32_t b, int value_kind, uint32_t chunks, bsm_mcsr** out) {
    BSM_REQUIRE(ctx && out && chunks >= 1, BSM_ERR_INVALID, "bsm_mcsr_generate: null argument or chunks = 0");
    BSM_REQUIRE(dtype_size(dtype) != 0, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    *out = nullptr;
    bsm_mcsr* m = new_mcsr(ctx, dtype, rows, n_cols, chunks);
    // the row lengths of the whole matrix (8 B per row) on the first device,
    // for the nnz-balanced bounds
    {
        DeviceGuard g(ctx->devices[0]);
        hipStream_t s = ctx->compute[0];
        DBuf rp, ws;
        std::vector<int64_t> h(rows + 1);
        int rc = rp.alloc((rows + 1) * sizeof(int64_t));
        const uint64_t wsb = bsm_dev_scan_workspace_bytes(rows);
        if (rc == BSM_OK) rc = ws.alloc(wsb);
        if (rc == BSM_OK) rc = gen_row_ptr(seed, 0, rows, n_cols, rowlen_kind, a, b, rp.as<int64_t>(), ws.p, wsb, s);
        if (rc == BSM_OK && hipMemcpyAsync(h.data(), rp.p, (rows + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s) !=
                                hipSuccess)
            rc = BSM_ERR_HIP;
        if (rc == BSM_OK && hipStreamSynchronize(s) != hipSuccess) rc = BSM_ERR_HIP;
        if (rc != BSM_OK) {
            if (rc == BSM_ERR_HIP) set_error("bsm_mcsr_generate: row lengths: %s", hipGetErrorString(hipGetLastError()));
            free_mcsr(m);
            return rc;
        }
        m->nnz = (uint64_t)h[rows];
        set_bounds(m, partition_by_cost(h.data(), rows, m->nnz, m->P));
    }
    const int rc = for_each_local(ctx->n_local, [&](int i) -> int {
        Local& L = m->loc[i];
        DeviceGuard g(L.device);
        hipStream_t s = ctx->compute[i];
        for (uint32_t c = 0; c < chunks; ++c) {
            const uint32_t p = c * (uint32_t)ctx->world + (uint32_t)L.rank;
            const uint64_t r0 = m->bounds[p], nr = m->bounds[p + 1] - r0;
            DBuf ws;
            const uint64_t wsb = bsm_dev_scan_workspace_bytes(nr);
            BSM_TRY(ws.alloc(wsb));
            // rows first (nnz unknown), then the entries
            bsm_csr* piece = nullptr;
            BSM_TRY(csr_alloc(&piece, dtype, nr, n_cols, 0));
            L.pieces[c] = piece;
            BSM_TRY(gen_row_ptr(seed, r0, nr, n_cols, rowlen_kind, a, b, piece->row_ptr, ws.p, wsb, s));
            int64_t pn = 0;
            BSM_HIP_TRY(read_dev(&pn, piece->row_ptr + nr, sizeof(pn), s));
            DBuf col, val;
            BSM_TRY(col.alloc((uint64_t)pn * sizeof(int32_t)));
            BSM_TRY(val.alloc((uint64_t)pn * dtype_size(dtype)));
            (void)hipFree(piece->col);  // csr_alloc's placeholders for nnz = 0
            (void)hipFree(piece->vals);
            piece->cache_cap[1] = piece->cache_cap[2] = 0;  // plain allocations from here on
            piece->col = col.as<int32_t>();
            col.release();
            piece->vals = val.release();
            piece->nnz = (uint64_t)pn;
            BSM_TRY(gen_entries(dtype, seed, r0, nr, n_cols, value_kind, piece->row_ptr, piece->col, piece->vals, s));
            BSM_TRY(csr_analyse(piece, s));
        }
        return BSM_OK;
    });
    if (rc != BSM_OK) {
        free_mcsr(m);
        return rc;
    }
    *out = m;
    return BSM_OK;
}

int bsm_mcsr_info(const bsm_mcsr* m, uint64_t* rows, uint64_t* cols, uint64_t* nnz, uint32_t* pieces,
                  uint64_t* piece_rows, uint64_t* bounds) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    if (rows) *rows = m->rows;
    if (cols) *cols = m->cols;
    if (nnz) *nnz = m->nnz;
    if (pieces) *pieces = m->P;
    if (piece_rows) *piece_rows = m->pad;
    if (bounds) std::copy(m->bounds.begin(), m->bounds.end(), bounds);
    return BSM_OK;
}

int bsm_mcsr_prepare(bsm_mcsr* m, uint64_t k, int schedule, double* plan_ms) {
    BSM_REQUIRE(m && schedule >= 0 && schedule <= 2, BSM_ERR_INVALID, "bsm_mcsr_prepare: bad argument");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    BSM_REQUIRE(k < (1ull << 31), BSM_ERR_UNSUPPORTED, "k too large");
    bsm_multi* ctx = m->ctx;
    const size_t es = dtype_size(m->dtype);
    const uint64_t slot_rows = (uint64_t)m->P * m->pad;
    std::vector<PlanTimes> pt(ctx->n_local);
    const auto t_all = host_now();
    const int rc = for_each_local(ctx->n_local, [&](int i) -> int {
        Local& L = m->loc[i];
        DeviceGuard g(L.device);
        hipStream_t s = ctx->compute[i];
        free_local_buffers(L);
        // buffers first: the schedule's copy then takes what is left
        const auto t_buf = host_now();
        DBuf y, nz;
        BSM_TRY(y.alloc(slot_rows * k * es));
        BSM_TRY(nz.alloc(slot_rows * sizeof(int32_t)));
        // slot rows past a piece's end are never written: zero, so they count
        // 0 nonzeros and compact to nothing
        BSM_HIP_TRY(hipMemsetAsync(y.p, 0, slot_rows * k * es, s));
        BSM_HIP_TRY(hipMemsetAsync(nz.p, 0, slot_rows * sizeof(int32_t), s));
        L.y = y.release();
        L.nz = nz.as<int32_t>();
        nz.release();
        if (L.compacts) {
            DBuf rp, oc, ov, ws, bd;
            BSM_TRY(rp.alloc((slot_rows + 1) * sizeof(int64_t)));
            BSM_TRY(oc.alloc(m->rows * k * sizeof(int32_t)));
            BSM_TRY(ov.alloc(m->rows * k * es));
            L.ws_b = scan_workspace_bytes(slot_rows);
            BSM_TRY(ws.alloc(L.ws_b));
            L.rp_pad = rp.as<int64_t>();
            rp.release();
            L.ocol = oc.as<int32_t>();
            oc.release();
            L.oval = ov.release();
            L.ws = ws.release();
            L.rp_out = L.rp_pad;
            if (m->squeeze) {
                DBuf ro;
                BSM_TRY(ro.alloc((m->rows + 1) * sizeof(int64_t)));
                BSM_TRY(bd.alloc((m->P + 1) * sizeof(int64_t)));
                std::vector<int64_t> hb(m->bounds.begin(), m->bounds.end());
                BSM_HIP_TRY(hipMemcpyAsync(bd.p, hb.data(), hb.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
                BSM_HIP_TRY(hipStreamSynchronize(s));  // hb dies here
                L.rp_out = ro.as<int64_t>();
                ro.release();
                L.bounds = bd.as<int64_t>();
                bd.release();
            }
        }
        L.round_ev.assign(m->chunks, nullptr);
        for (auto& e : L.round_ev) BSM_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        BSM_HIP_TRY(hipStreamSynchronize(s));
        pt[i].buffers_ms = ms_since(t_buf);
        for (uint32_t c = 0; c < m->chunks; ++c) {
            bsm_csr* a = L.pieces[c];
            std::lock_guard<std::mutex> lk(a->plan_mu);
            BSM_TRY(spmm_prepare_locked(a, k, schedule, 0, s, &pt[i]));
        }
        return BSM_OK;
    });
    if (rc != BSM_OK) {
        for (auto& L : m->loc) {
            DeviceGuard g(L.device);
            free_local_buffers(L);
        }
        m->prepared = false;
        return rc;
    }
    m->k = k;
    m->schedule = schedule;
    m->prepared = true;
    if (plan_ms) {
        const PlanTimes* w = &pt[0];
        for (auto& p : pt)
            if (p.total_ms + p.buffers_ms > w->total_ms + w->buffers_ms) w = &p;
        const double v[7] = {ms_since(t_all), w->count_ms, w->scan_ms, w->alloc_ms, w->write_ms, w->panel_ms,
                             w->buffers_ms};
        std::copy(v, v + 7, plan_ms);
    }
    return BSM_OK;
}

int bsm_mcsr_plan_info(const bsm_mcsr* m, int* tiled_pieces, int* local_pieces, uint64_t* copy_bytes,
                       uint64_t* panel_cols) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    int nt = 0, np = 0;
    uint64_t bytes = 0, pc = 0;
    for (const auto& L : m->loc)
        for (const bsm_csr* a : L.pieces) {
            std::lock_guard<std::mutex> lk(a->plan_mu);
            ++np;
            if (m->prepared && m->schedule != 2 && a->tiled && a->tiled->k == m->k) {
                ++nt;
                uint64_t b = 0, w = 0;
                (void)bsm_tiled_info(a->tiled, &b, nullptr, &w);
                bytes += b;
                pc = w;
            } else if (a->plan_usable && !pc) {
                pc = a->plan_cols;
            }
        }
    if (tiled_pieces) *tiled_pieces = nt;
    if (local_pieces) *local_pieces = np;
    if (copy_bytes) *copy_bytes = bytes;
    if (panel_cols) *panel_cols = pc;
    return BSM_OK;
}

int bsm_mcsr_step(bsm_mcsr* m, const void* const* x_dev) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "bsm_mcsr_step: null handle");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    BSM_REQUIRE(m->prepared, BSM_ERR_INVALID, "bsm_mcsr_step: prepare the matrix first");
    bsm_multi* ctx = m->ctx;
    const uint64_t k = m->k;
    BSM_REQUIRE(k == 0 || x_dev, BSM_ERR_INVALID, "null X");
    const size_t es = dtype_size(m->dtype);
    const size_t slot_b = m->pad * k * es;
    const bool allow_tiled = m->schedule != 2;
    // one rank: the all-gathers have nothing to move (every slot is this
    // rank's own), so the step skips them and their stream hops;
    // BSM_MULTI_SOLO_RCCL=1 runs them anyway (tests of the RCCL calls at G = 1)
    const char* sre = getenv("BSM_MULTI_SOLO_RCCL");
    const bool solo = ctx->world == 1 && !ctx->external && !(sre && atoi(sre) == 1);
    // events of this step (timed steps are read after the fact: no host sync)
    for (int i = 0; i < ctx->n_local; ++i) {
        Local& L = m->loc[i];
        DeviceGuard g(L.device);
        if ((size_t)(L.steps + 1) * EV_PER_STEP > L.ev.size()) {
            for (int e = 0; e < EV_PER_STEP; ++e) {
                hipEvent_t ev;
                BSM_HIP_TRY(hipEventCreate(&ev));
                L.ev.push_back(ev);
            }
        }
        BSM_HIP_TRY(hipEventRecord(L.ev[L.steps * EV_PER_STEP + 0], ctx->compute[i]));
    }
    for (uint32_t c = 0; c < m->chunks; ++c) {
        for (int i = 0; i < ctx->n_local; ++i) {
            Local& L = m->loc[i];
            DeviceGuard g(L.device);
            const uint64_t slot = (uint64_t)c * ctx->world + L.rank;
            bsm_csr* a = L.pieces[c];
            {
                std::lock_guard<std::mutex> lk(a->plan_mu);
                BSM_TRY(spmm_launch_locked(a, k, allow_tiled, k ? x_dev[i] : nullptr,
                                           static_cast<char*>(L.y) + slot * slot_b, L.nz + slot * m->pad,
                                           ctx->compute[i]));
            }
            if (!solo) {
                BSM_HIP_TRY(hipEventRecord(L.round_ev[c], ctx->compute[i]));
                BSM_HIP_TRY(hipStreamWaitEvent(ctx->comm[i], L.round_ev[c], 0));
            }
            if (c + 1 == m->chunks)
                BSM_HIP_TRY(hipEventRecord(L.ev[L.steps * EV_PER_STEP + 1], ctx->compute[i]));
        }
        // round c of every rank lands at slots c*world .. c*world + world - 1
        // (an external context leaves that to the caller: bsm_mcsr_slot_read /
        // _write, then bsm_mcsr_compact)
        if (ctx->external || solo) continue;
        BSM_NCCL_TRY(ncclGroupStart());
        for (int i = 0; i < ctx->n_local; ++i) {
            Local& L = m->loc[i];
            char* ybase = static_cast<char*>(L.y) + (uint64_t)c * ctx->world * slot_b;
            int32_t* nbase = L.nz + (uint64_t)c * ctx->world * m->pad;
            ncclResult_t r = ncclSuccess;
            if (slot_b)
                r = ncclAllGather(ybase + (uint64_t)L.rank * slot_b, ybase, slot_b, ncclChar, ctx->comms[i],
                                  ctx->comm[i]);
            if (r == ncclSuccess && m->pad)
                r = ncclAllGather(nbase + (uint64_t)L.rank * m->pad, nbase, m->pad, ncclInt32, ctx->comms[i],
                                  ctx->comm[i]);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                set_error("ncclAllGather (round %u): %s", c, ncclGetErrorString(r));
                return BSM_ERR_COMM;
            }
        }
        BSM_NCCL_TRY(ncclGroupEnd());
    }
    for (int i = 0; i < ctx->n_local; ++i) {
        Local& L = m->loc[i];
        DeviceGuard g(L.device);
        hipStream_t s = ctx->compute[i];
        hipEvent_t* E = &L.ev[L.steps * EV_PER_STEP];
        BSM_HIP_TRY(hipEventRecord(E[2], solo ? s : ctx->comm[i]));
        if (!solo) BSM_HIP_TRY(hipStreamWaitEvent(s, E[2], 0));
        BSM_HIP_TRY(hipEventRecord(E[3], s));
        if (L.compacts && !ctx->external) BSM_TRY(compact_local(m, L, s));
        BSM_HIP_TRY(hipEventRecord(E[4], s));
        ++L.steps;
    }
    return BSM_OK;
}

int bsm_mcsr_sync(bsm_mcsr* m) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    for (int i = 0; i < m->ctx->n_local; ++i) {
        DeviceGuard g(m->loc[i].device);
        BSM_HIP_TRY(hipStreamSynchronize(m->ctx->compute[i]));
        BSM_HIP_TRY(hipStreamSynchronize(m->ctx->comm[i]));
    }
    return BSM_OK;
}

int bsm_mcsr_step_times(bsm_mcsr* m, int local, int max, int* n, double* ms) {
    BSM_REQUIRE(m && n && local >= 0 && local < m->ctx->n_local && (max <= 0 || ms), BSM_ERR_INVALID,
                "bsm_mcsr_step_times: bad argument");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    Local& L = m->loc[local];
    DeviceGuard g(L.device);
    *n = L.steps;
    for (int s = 0; s < L.steps && s < max; ++s) {
        hipEvent_t* E = &L.ev[s * EV_PER_STEP];
        BSM_HIP_TRY(hipEventSynchronize(E[4]));
        float t[4] = {0, 0, 0, 0};
        BSM_HIP_TRY(hipEventElapsedTime(&t[0], E[0], E[1]));
        BSM_HIP_TRY(hipEventElapsedTime(&t[1], E[1], E[2]));
        BSM_HIP_TRY(hipEventElapsedTime(&t[2], E[3], E[4]));
        BSM_HIP_TRY(hipEventElapsedTime(&t[3], E[0], E[4]));
        ms[4 * s + 0] = t[0];
        ms[4 * s + 1] = std::max(0.0f, t[1]);  // the all-gathers may end before the last SpMM does
        ms[4 * s + 2] = t[2];
        ms[4 * s + 3] = t[3];
    }
    return BSM_OK;
}

void bsm_mcsr_reset_times(bsm_mcsr* m) {
    if (!m) return;
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    for (auto& L : m->loc) L.steps = 0;  // events are reused
}

int bsm_mcsr_copy_y(const bsm_mcsr* m, int local, void* y, int32_t* row_nnz) {
    BSM_REQUIRE(m && local >= 0 && local < m->ctx->n_local, BSM_ERR_INVALID, "bsm_mcsr_copy_y: bad argument");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    BSM_REQUIRE(m->prepared, BSM_ERR_INVALID, "bsm_mcsr_copy_y: prepare the matrix first");
    const Local& L = m->loc[local];
    DeviceGuard g(L.device);
    hipStream_t s = m->ctx->compute[local];
    const size_t es = dtype_size(m->dtype);
    const size_t row_b = m->k * es;
    for (uint32_t p = 0; p < m->P; ++p) {
        const uint64_t r0 = m->bounds[p], nr = m->bounds[p + 1] - r0;
        if (!nr) continue;
        if (y && row_b)
            BSM_HIP_TRY(hipMemcpyAsync(static_cast<char*>(y) + r0 * row_b,
                                       static_cast<const char*>(L.y) + (uint64_t)p * m->pad * row_b, nr * row_b,
                                       hipMemcpyDeviceToDevice, s));
        if (row_nnz)
            BSM_HIP_TRY(hipMemcpyAsync(row_nnz + r0, L.nz + (uint64_t)p * m->pad, nr * sizeof(int32_t),
                                       hipMemcpyDeviceToDevice, s));
    }
    BSM_HIP_TRY(hipStreamSynchronize(s));
    return BSM_OK;
}

int bsm_mcsr_output(const bsm_mcsr* m, bsm_csr** out) {
    BSM_REQUIRE(m && out, BSM_ERR_INVALID, "bsm_mcsr_output: bad argument");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    BSM_REQUIRE(m->prepared, BSM_ERR_INVALID, "bsm_mcsr_output: prepare the matrix first");
    int li = 0;
    while (li < m->ctx->n_local && !m->loc[li].compacts) ++li;
    BSM_REQUIRE(li < m->ctx->n_local, BSM_ERR_INVALID,
                "bsm_mcsr_output: no local device compacts the output (output rank %d)", m->out_rank);
    const Local& L = m->loc[li];
    DeviceGuard g(L.device);
    hipStream_t s = m->ctx->compute[li];
    int64_t nnz = 0;
    BSM_HIP_TRY(read_dev(&nnz, L.rp_out + m->rows, sizeof(nnz), s));
    bsm_csr* r = nullptr;
    BSM_TRY(csr_alloc(&r, m->dtype, m->rows, m->k, (uint64_t)nnz));
    int rc = BSM_OK;
    auto cp = [&](void* d, const void* src, size_t b) {
        if (rc == BSM_OK && b && hipMemcpyAsync(d, src, b, hipMemcpyDeviceToDevice, s) != hipSuccess) {
            set_error("bsm_mcsr_output: copy failed");
            rc = BSM_ERR_HIP;
        }
    };
    cp(r->row_ptr, L.rp_out, (m->rows + 1) * sizeof(int64_t));
    cp(r->col, L.ocol, (uint64_t)nnz * sizeof(int32_t));
    cp(r->vals, L.oval, (uint64_t)nnz * dtype_size(m->dtype));
    if (rc == BSM_OK && hipStreamSynchronize(s) != hipSuccess) {
        set_error("bsm_mcsr_output: sync failed");
        rc = BSM_ERR_HIP;
    }
    if (rc != BSM_OK) {
        bsm_csr_free(r);
        return rc;
    }
    r->analysed = true;
    r->rows_sorted = true;
    r->max_row_len = m->k;
    *out = r;
    return BSM_OK;
}

int bsm_mcsr_mul_dense(bsm_mcsr* m, uint64_t k, uint64_t x_rows, const void* const* x_cols, bsm_csr** out) {
    BSM_REQUIRE(m && out && (k == 0 || x_cols), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(m->cols == x_rows, BSM_ERR_DIMENSIONS, "IncorrectDimensions: cols %llu != rhs rows %llu",
                (unsigned long long)m->cols, (unsigned long long)x_rows);
    bsm_multi* ctx = m->ctx;
    BSM_REQUIRE(!ctx->external, BSM_ERR_UNSUPPORTED,
                "bsm_mcsr_mul_dense: an external context has no communicator (bsm_mcsr_step, exchange the slots, "
                "bsm_mcsr_compact)");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    if (!m->prepared || m->k != k) BSM_TRY(bsm_mcsr_prepare(m, k, m->prepared ? m->schedule : 0, nullptr));
    // X to every local device (each over its own link, in parallel)
    std::vector<DBuf> xs(ctx->n_local);
    std::vector<const void*> xp(ctx->n_local, nullptr);
    BSM_TRY(for_each_local(ctx->n_local, [&](int i) -> int {
        DeviceGuard g(m->loc[i].device);
        BSM_TRY(upload_dense_cols(m->dtype, x_rows, k, x_cols, xs[i], ctx->compute[i]));
        xp[i] = xs[i].p;
        return BSM_OK;
    }));
    BSM_TRY(bsm_mcsr_step(m, xp.data()));
    BSM_TRY(bsm_mcsr_sync(m));
    for (auto& L : m->loc) L.steps = std::max(0, L.steps - 1);  // not a timed step
    return bsm_mcsr_output(m, out);
}

int bsm_mcsr_set_output_rank(bsm_mcsr* m, int rank) {
    BSM_REQUIRE(m && rank >= -1 && rank < m->ctx->world, BSM_ERR_INVALID, "bsm_mcsr_set_output_rank: bad argument");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    m->out_rank = rank;
    for (int i = 0; i < m->ctx->n_local; ++i) {
        Local& L = m->loc[i];
        L.compacts = rank < 0 ? i == 0 : L.rank == rank;
        DeviceGuard g(L.device);
        free_local_buffers(L);
    }
    m->prepared = false;
    return BSM_OK;
}

int bsm_mcsr_compact(bsm_mcsr* m) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "bsm_mcsr_compact: null handle");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    BSM_REQUIRE(m->prepared, BSM_ERR_INVALID, "bsm_mcsr_compact: prepare the matrix first");
    for (int i = 0; i < m->ctx->n_local; ++i) {
        Local& L = m->loc[i];
        if (!L.compacts) continue;
        DeviceGuard g(L.device);
        hipStream_t s = m->ctx->compute[i];
        hipEvent_t e;  // after anything still queued on the communication stream
        BSM_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        int rc = hipEventRecord(e, m->ctx->comm[i]) == hipSuccess && hipStreamWaitEvent(s, e, 0) == hipSuccess
                     ? BSM_OK
                     : BSM_ERR_HIP;
        (void)hipEventDestroy(e);
        if (rc != BSM_OK) {
            set_error("bsm_mcsr_compact: stream ordering failed");
            return rc;
        }
        BSM_TRY(compact_local(m, L, s));
    }
    return BSM_OK;
}

namespace {
// slots [first, first + n) of the gathered Y and its row counts on local
// device `local` <-> caller buffers (host or device); synchronous
int slot_copy(const bsm_mcsr* m, int local, uint32_t first, uint32_t n, void* y, int32_t* nz, bool to_slots) {
    BSM_REQUIRE(m && local >= 0 && local < m->ctx->n_local, BSM_ERR_INVALID, "bsm_mcsr_slot_*: bad argument");
    BSM_REQUIRE(m->prepared, BSM_ERR_INVALID, "bsm_mcsr_slot_*: prepare the matrix first");
    BSM_REQUIRE((uint64_t)first + n <= m->P, BSM_ERR_INVALID, "bsm_mcsr_slot_*: slots [%u, %u) of %u", first,
                first + n, m->P);
    const Local& L = m->loc[local];
    DeviceGuard g(L.device);
    hipStream_t s = m->ctx->compute[local];
    const uint64_t slot_b = m->pad * m->k * dtype_size(m->dtype);
    char* ys = static_cast<char*>(L.y) + (uint64_t)first * slot_b;
    int32_t* ns = L.nz + (uint64_t)first * m->pad;
    const uint64_t yb = (uint64_t)n * slot_b, nb = (uint64_t)n * m->pad * sizeof(int32_t);
    BSM_HIP_TRY(hipStreamSynchronize(m->ctx->comm[local]));
    if (y && yb)
        BSM_HIP_TRY(to_slots ? hipMemcpyAsync(ys, y, yb, hipMemcpyDefault, s)
                             : hipMemcpyAsync(y, ys, yb, hipMemcpyDefault, s));
    if (nz && nb)
        BSM_HIP_TRY(to_slots ? hipMemcpyAsync(ns, nz, nb, hipMemcpyDefault, s)
                             : hipMemcpyAsync(nz, ns, nb, hipMemcpyDefault, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    return BSM_OK;
}
}  // namespace

int bsm_mcsr_slot_read(const bsm_mcsr* m, int local, uint32_t first, uint32_t n, void* y, int32_t* row_nnz) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    return slot_copy(m, local, first, n, y, row_nnz, false);
}

int bsm_mcsr_slot_write(bsm_mcsr* m, int local, uint32_t first, uint32_t n, const void* y, const int32_t* row_nnz) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    std::lock_guard<std::recursive_mutex> hold(m->mu);
    return slot_copy(m, local, first, n, const_cast<void*>(y), const_cast<int32_t*>(row_nnz), true);
}

void bsm_mcsr_free(bsm_mcsr* m) { free_mcsr(m); }

}  // extern "C"
