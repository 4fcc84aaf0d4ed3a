// capi.hip -- extern "C" boundary of libbsm_hip.so (declared in include/bsm.h).
//
// Host-buffer entry points mirror the reference crate's hot-path methods
// (src/sparse.rs, src/lib.rs); each is synchronous and owns no caller memory.
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <mutex>
#include <vector>

#include <algorithm>
#include <cstring>

#include "bsm_internal.hpp"

namespace bsm {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
const char* last_error() { return g_err.c_str(); }

// Stage timer of the solver entry points (bsm_stage_times): each mark records
// an event on the stream; stage i spans marks i-1 .. i.
namespace {
struct Stage {
    std::string name;
    hipEvent_t ev = nullptr;
};
thread_local std::vector<Stage> g_stages;
void stage_clear() {
    for (auto& st : g_stages)
        if (st.ev) (void)hipEventDestroy(st.ev);
    g_stages.clear();
}
// Off unless armed (bsm_stage_timing or env BSM_STAGE_TIMES=1): no events are
// created on calls nobody times.
std::atomic<int> g_stage_on{-1};
bool stage_on() {
    int v = g_stage_on.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("BSM_STAGE_TIMES");
        v = (e && atoi(e) != 0) ? 1 : 0;
        g_stage_on.store(v, std::memory_order_relaxed);
    }
    return v != 0;
}
}  // namespace

// Every public entry point that marks stages starts its own list.
void stage_reset(hipStream_t s) {
    stage_clear();
    if (!stage_on()) return;
    Stage st;
    st.name = "start";
    if (hipEventCreate(&st.ev) != hipSuccess) return;
    if (hipEventRecord(st.ev, s) != hipSuccess) {
        (void)hipEventDestroy(st.ev);
        return;
    }
    g_stages.push_back(st);
}
void stage_mark(const char* name, hipStream_t s) {
    if (!stage_on() || g_stages.empty() || g_stages.size() >= 64) return;
    Stage st;
    st.name = name;
    if (hipEventCreate(&st.ev) != hipSuccess) return;
    if (hipEventRecord(st.ev, s) != hipSuccess) {
        (void)hipEventDestroy(st.ev);
        return;
    }
    g_stages.push_back(st);
}

namespace {
std::mutex g_stream_mu;
hipStream_t g_streams[64] = {};
}  // namespace

int current_device(int* dev) {
    BSM_HIP_TRY(hipGetDevice(dev));
    return BSM_OK;
}

int ctx_stream(hipStream_t* s) {
    int dev = 0;
    BSM_TRY(current_device(&dev));
    BSM_REQUIRE(dev >= 0 && dev < 64, BSM_ERR_INVALID, "device ordinal %d out of range", dev);
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if (!g_streams[dev]) BSM_HIP_TRY(hipStreamCreateWithFlags(&g_streams[dev], hipStreamNonBlocking));
    *s = g_streams[dev];
    return BSM_OK;
}

namespace {
// Result buffers. Every small call returns a new bsm_csr whose three arrays
// came from hipMalloc, and the caller's bsm_csr_free gave them back with
// hipFree, which waits for the device and unmaps: ~60 us a malloc / free pair
// on the box (profiles/r03_u_*), three pairs per result. Blocks of up to
// 1 GiB now come from a per-device free list by size class (powers of two to
// 64 MiB, then 16 MiB steps; at most 2 GiB kept per device, the oldest
// released first). bsm_csr_free waits for the device once, as hipFree did,
// so a block is never handed out while work queued on the old result runs.
// BSM_RESULT_CACHE=0: plain hipMalloc / hipFree.
struct ResultCache {
    std::mutex mu;
    std::vector<std::pair<size_t, void*>> free_;  // (class, block), oldest first
    size_t bytes = 0;
};
ResultCache g_rcache[64];
constexpr size_t RC_MAX_BLOCK = 1ull << 30, RC_KEEP = 2ull << 30;
bool rc_enabled() {
    static const bool on = [] {
        const char* e = getenv("BSM_RESULT_CACHE");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
size_t rc_class(size_t n) {
    if (n <= 4096) return 4096;
    if (n <= (64ull << 20)) return size_t(1) << (64 - __builtin_clzll((unsigned long long)(n - 1)));
    return (n + (16ull << 20) - 1) & ~((16ull << 20) - 1);
}
int rc_alloc(int dev, size_t n, void** p, size_t* cap) {
    *p = nullptr;
    *cap = 0;
    if (n == 0) n = 16;
    if (!rc_enabled() || n > RC_MAX_BLOCK || dev < 0 || dev >= 64) {
        hipError_t e = hipMalloc(p, n);
        if (e != hipSuccess) {
            *p = nullptr;
            set_error("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? BSM_ERR_OOM : BSM_ERR_HIP;
        }
        return BSM_OK;
    }
    const size_t c = rc_class(n);
    ResultCache& rc = g_rcache[dev];
    {
        std::lock_guard<std::mutex> lk(rc.mu);
        for (size_t i = rc.free_.size(); i-- > 0;) {  // newest first: likeliest still in L2 / TLB
            if (rc.free_[i].first == c) {
                *p = rc.free_[i].second;
                rc.free_.erase(rc.free_.begin() + (ptrdiff_t)i);
                rc.bytes -= c;
                *cap = c;
                return BSM_OK;
            }
        }
    }
    hipError_t e = hipMalloc(p, c);
    if (e == hipErrorOutOfMemory) {  // give the cached blocks back and retry once
        std::vector<std::pair<size_t, void*>> drop;
        {
            std::lock_guard<std::mutex> lk(rc.mu);
            drop.swap(rc.free_);
            rc.bytes = 0;
        }
        for (auto& b : drop) (void)hipFree(b.second);
        e = hipMalloc(p, c);
    }
    if (e != hipSuccess) {
        *p = nullptr;
        set_error("hipMalloc(%zu) failed: %s", c, hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? BSM_ERR_OOM : BSM_ERR_HIP;
    }
    *cap = c;
    return BSM_OK;
}
// A result block owned by a call until it is handed to the bsm_csr (error
// paths hipFree it: that waits for whatever was queued on it)
struct RcBuf {
    void* p = nullptr;
    size_t cap = 0;
    RcBuf() = default;
    RcBuf(const RcBuf&) = delete;
    RcBuf& operator=(const RcBuf&) = delete;
    ~RcBuf() {
        if (p) (void)hipFree(p);
    }
    int alloc(int dev, size_t n) { return rc_alloc(dev, n, &p, &cap); }
    void* release() {
        void* q = p;
        p = nullptr;
        return q;
    }
    template <typename U> U* as() const { return static_cast<U*>(p); }
};
// the caller has waited for the device
void rc_release(int dev, void* p, size_t cap) {
    if (!p) return;
    if (!cap) {
        (void)hipFree(p);
        return;
    }
    std::vector<void*> drop;
    {
        ResultCache& rc = g_rcache[dev];
        std::lock_guard<std::mutex> lk(rc.mu);
        rc.free_.emplace_back(cap, p);
        rc.bytes += cap;
        while (rc.bytes > RC_KEEP && !rc.free_.empty()) {
            rc.bytes -= rc.free_.front().first;
            drop.push_back(rc.free_.front().second);
            rc.free_.erase(rc.free_.begin());
        }
    }
    for (void* q : drop) (void)hipFree(q);
}
}  // namespace

int csr_alloc(bsm_csr** out, int dtype, uint64_t rows, uint64_t cols, uint64_t nnz) {
    const size_t es = dtype_size(dtype);
    BSM_REQUIRE(es != 0, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    BSM_REQUIRE(cols <= 0x7fffffffull, BSM_ERR_UNSUPPORTED,
                "cols = %llu: device CSR stores int32 column indices", (unsigned long long)cols);
    auto* m = new bsm_csr();
    m->dtype = dtype;
    m->rows = rows;
    m->cols = cols;
    m->nnz = nnz;
    int dev = 0;
    int rc = current_device(&dev);
    m->device = dev;
    void* bufs[3] = {nullptr, nullptr, nullptr};
    const size_t sizes[3] = {(rows + 1) * sizeof(int64_t), nnz * sizeof(int32_t), nnz * es};
    for (int i = 0; i < 3 && rc == BSM_OK; ++i) rc = rc_alloc(dev, sizes[i], &bufs[i], &m->cache_cap[i]);
    if (rc != BSM_OK) {
        for (int i = 0; i < 3; ++i) rc_release(dev, bufs[i], m->cache_cap[i]);  // nothing queued on them yet
        delete m;
        return rc;
    }
    m->row_ptr = static_cast<int64_t*>(bufs[0]);
    m->col = static_cast<int32_t*>(bufs[1]);
    m->vals = bufs[2];
    *out = m;
    return BSM_OK;
}

namespace {
struct TmpCache {
    struct Ent {
        void* p;
        size_t cap;
        int device;
        hipStream_t s;
    };
    std::vector<Ent> free_list;
    size_t held = 0;
    ~TmpCache() {
        for (auto& e : free_list) (void)hipFree(e.p);
    }
};
TmpCache& tmp_cache() {
    static thread_local TmpCache c;
    return c;
}
constexpr size_t TMP_CACHE_MAX = 512ull << 20;   // bytes kept per thread
constexpr size_t TMP_BLOCK_MAX = 256ull << 20;   // larger temporaries are not cached
}  // namespace

void* tmp_get(size_t n, int device, hipStream_t s, size_t* cap) {
    size_t c = 4096;
    while (c < n) c <<= 1;  // power-of-two classes
    TmpCache& tc = tmp_cache();
    for (size_t i = 0; i < tc.free_list.size(); ++i) {
        if (tc.free_list[i].cap == c && tc.free_list[i].s == s && tc.free_list[i].device == device) {
            void* p = tc.free_list[i].p;
            tc.held -= c;
            tc.free_list[i] = tc.free_list.back();
            tc.free_list.pop_back();
            *cap = c;
            return p;
        }
    }
    const size_t want = c <= TMP_BLOCK_MAX ? c : n;
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) return nullptr;
    *cap = want;
    return p;
}

void tmp_put(void* p, size_t cap, int device, hipStream_t s) {
    TmpCache& tc = tmp_cache();
    if (cap > TMP_BLOCK_MAX || (cap & (cap - 1)) || tc.held + cap > TMP_CACHE_MAX) {
        (void)hipFree(p);
        return;
    }
    tc.free_list.push_back({p, cap, device, s});
    tc.held += cap;
}

int csr_analyse(const bsm_csr* m, hipStream_t s) {
    if (m->analysed) return BSM_OK;
    DBuf out;
    BSM_TRY(out.alloc(3 * sizeof(uint64_t), s));
    BSM_TRY(analyse_dispatch(m->row_ptr, m->col, m->rows, m->cols, out.as<uint64_t>(), s));
    uint64_t h[3] = {0, 0, 0};
    BSM_HIP_TRY(hipMemcpyAsync(h, out.p, sizeof(h), hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    BSM_REQUIRE(h[2] == 0, BSM_ERR_PANIC, "column index out of bounds in %llu entries",
                (unsigned long long)h[2]);
    m->max_row_len = h[0];
    m->rows_sorted = (h[1] == 0);
    m->analysed = true;
    return BSM_OK;
}

// Pinned host staging for small transfers: a copy from pageable memory costs
// ~19 us per hipMemcpyAsync on the box, so small operands are packed into one
// pinned buffer and moved with one copy (profiles/r01_z_api_overhead.log).
// One buffer per thread (the library's calls are synchronous per thread).
constexpr size_t PIN_MAX = 32ull << 20;
namespace {
// Per-thread buffers are released when their thread exits (worker
// threads of the multi-GPU path must not leak them).
struct PinnedHolder {
    void* buf = nullptr;
    size_t cap = 0;
    ~PinnedHolder() {
        if (buf) (void)hipHostFree(buf);
    }
};
struct ScratchSlot {
    void* p = nullptr;
    size_t cap = 0;
    int dev = -1;
};
struct ScratchHolder {
    ScratchSlot sl[4];
    ~ScratchHolder() {
        for (auto& x : sl)
            if (x.p) (void)hipFree(x.p);
    }
};
}  // namespace

void* pinned(size_t bytes) {
    static thread_local PinnedHolder h;
    if (bytes > h.cap) {
        if (h.buf) (void)hipHostFree(h.buf);
        h.buf = nullptr;
        h.cap = 0;
        size_t want = std::max<size_t>(bytes, 1 << 20);
        if (hipHostMalloc(&h.buf, want, hipHostMallocDefault) != hipSuccess) {
            h.buf = nullptr;
            (void)hipGetLastError();
            return nullptr;
        }
        h.cap = want;
    }
    return h.buf;
}

// BSM_SMALL_OUT=0: small mul_dense results take the scan + compaction
// launches and the download copies (A/B)
static bool small_out_enabled() {
    const char* e = getenv("BSM_SMALL_OUT");
    return !e || atoi(e) != 0;
}

// Page-locked destination of the small results' host copy (compact_small):
// one per thread, reused by the thread's next small call (the result handle
// keeps its own copy). *dev: the buffer's device address.
static void* pinned_result(size_t bytes, void** dev) {
    static thread_local PinnedHolder h;
    static thread_local void* h_dev = nullptr;
    if (bytes > h.cap) {
        if (h.buf) (void)hipHostFree(h.buf);
        h.buf = h_dev = nullptr;
        h.cap = 0;
        const size_t want = std::max<size_t>(bytes, 1 << 20);
        if (hipHostMalloc(&h.buf, want, hipHostMallocDefault) != hipSuccess ||
            hipHostGetDevicePointer(&h_dev, h.buf, 0) != hipSuccess) {
            if (h.buf) (void)hipHostFree(h.buf);
            h.buf = h_dev = nullptr;
            (void)hipGetLastError();
            return nullptr;
        }
        h.cap = want;
    }
    *dev = h_dev;
    return h.buf;
}

// Per-call temporaries of small calls (the uploaded X, Y, row counts, scan
// workspace) come from a per-thread grow-only device arena: no hipMalloc /
// hipFree per call (hipFree waits for the device). Calls larger than
// SCRATCH_MAX allocate as before.
constexpr size_t SCRATCH_MAX = 64ull << 20;
static void* scratch(int slot, size_t bytes) {
    static thread_local ScratchHolder holder;
    int dev = 0;
    if (slot < 0 || slot >= 4 || bytes > SCRATCH_MAX || hipGetDevice(&dev) != hipSuccess) return nullptr;
    ScratchSlot& x = holder.sl[slot];
    if (bytes > x.cap || dev != x.dev) {
        if (x.p) (void)hipFree(x.p);
        x.p = nullptr;
        x.cap = 0;
        const size_t want = std::max<size_t>(bytes, 1 << 20);
        if (hipMalloc(&x.p, want) != hipSuccess) {
            x.p = nullptr;
            (void)hipGetLastError();
            return nullptr;
        }
        x.cap = want;
        x.dev = dev;
    }
    return x.p;
}

hipError_t read_dev(void* host, const void* dev, size_t bytes, hipStream_t s) {
    static thread_local PinnedHolder holder;
    if (bytes > 4096) {
        hipError_t e = hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s);
        return e != hipSuccess ? e : hipStreamSynchronize(s);
    }
    void*& bounce = holder.buf;
    if (!bounce) {
        hipError_t e = hipHostMalloc(&bounce, 4096, hipHostMallocDefault);
        if (e != hipSuccess) {
            bounce = nullptr;
            return e;
        }
        holder.cap = 4096;
    }
    hipError_t e = hipMemcpyAsync(bounce, dev, bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) std::memcpy(host, bounce, bytes);
    return e;
}

// Upload k host columns (each n values) into a device ROW-major n x k array
// at *data: `out` (allocated here), or, when the caller offers dst_small
// (scratch) and the pinned path serves the call, dst_small with the copy left
// in flight -- the caller then synchronises the stream before it returns
// (the pinned buffer is reused by the next call) and *synced is false.
static int upload_columns(int dtype, uint64_t n, uint64_t k, const void* const* cols, DBuf& out,
                          hipStream_t s, void** data = nullptr, void* dst_small = nullptr,
                          bool* synced = nullptr) {
    const size_t es = dtype_size(dtype);
    if (synced) *synced = true;
    for (uint64_t j = 0; j < k && n; ++j)
        BSM_REQUIRE(cols[j] != nullptr, BSM_ERR_INVALID, "null column pointer %llu", (unsigned long long)j);
    const size_t bytes = n * k * es;
    char* pin = bytes <= PIN_MAX && n && k ? static_cast<char*>(pinned(bytes)) : nullptr;
    void* dst = dst_small && pin && synced ? dst_small : nullptr;
    if (!dst) {
        BSM_TRY(out.alloc(bytes));
        dst = out.p;
    }
    if (data) *data = dst;
    if (n == 0 || k == 0) return BSM_OK;
    // the columns go over as they are (column-major, memcpy per column) and
    // are packed to row-major on the device: a host-side pack is one
    // element-sized copy per value
    if (pin) {  // small: one pinned buffer, one DMA
        void* cm = k == 1 ? dst : scratch(2, bytes);
        DBuf cm_own;
        if (!cm) {
            BSM_TRY(cm_own.alloc(bytes));
            cm = cm_own.p;
        }
        for (uint64_t j = 0; j < k; ++j) std::memcpy(pin + j * n * es, cols[j], n * es);
        BSM_HIP_TRY(hipMemcpyAsync(cm, pin, bytes, hipMemcpyHostToDevice, s));
        if (k > 1) BSM_TRY(pack_cols_to_rowmajor(dtype, n, k, cm, dst, s));
        if (dst == dst_small && !cm_own.p) *synced = false;
        else BSM_HIP_TRY(hipStreamSynchronize(s));  // the pinned buffer is reused by the next call
        return BSM_OK;
    }
    if (k == 1) return h2d_staged(dst, cols[0], n * es, s);
    DBuf staging;
    BSM_TRY(staging.alloc(bytes));
    for (uint64_t j = 0; j < k; ++j) BSM_TRY(h2d_staged(static_cast<char*>(staging.p) + j * n * es, cols[j], n * es, s));
    BSM_TRY(pack_cols_to_rowmajor(dtype, n, k, staging.p, dst, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));  // staging dies here
    return BSM_OK;
}

int upload_dense_cols(int dtype, uint64_t n, uint64_t k, const void* const* cols, DBuf& out, hipStream_t s) {
    return upload_columns(dtype, n, k, cols, out, s);
}

// Download a device ROW-major n x k array into k host columns.
static int download_columns(int dtype, uint64_t n, uint64_t k, const void* dev, void* const* cols,
                            hipStream_t s) {
    const size_t es = dtype_size(dtype);
    if (n == 0 || k == 0) return BSM_OK;
    if (k == 1) return d2h_staged(cols[0], dev, n * es, s);
    DBuf staging;
    BSM_TRY(staging.alloc(n * k * es));
    BSM_TRY(unpack_rowmajor_to_cols(dtype, n, k, dev, staging.p, s));
    for (uint64_t j = 0; j < k; ++j)
        BSM_TRY(d2h_staged(cols[j], static_cast<const char*>(staging.p) + j * n * es, n * es, s));
    return BSM_OK;
}

// Rows [r0, r1) of a host finalised Csr (absolute usize row_ptr) as a new
// handle on the current device: row_ptr rebased to 0, columns narrowed to
// int32 and checked on the device (an out-of-range column is the reference's
// index panic, sparse.rs:437), values copied.
int csr_upload_rows(int dtype, uint64_t r0, uint64_t r1, uint64_t cols, const uint64_t* row_ptr,
                    const uint64_t* col_idx, const void* vals, bsm_csr** out, hipStream_t s) {
    const uint64_t base = row_ptr[r0], nnz = row_ptr[r1] - base, rows = r1 - r0;
    const size_t es = dtype_size(dtype);
    bsm_csr* m = nullptr;
    BSM_TRY(csr_alloc(&m, dtype, rows, cols, nnz));
    uint64_t bad = 0;
    int rc = h2d_row_ptr(m->row_ptr, row_ptr + r0, rows + 1, base, s);
    if (rc == BSM_OK) rc = h2d_cols_narrow(m->col, col_idx + base, nnz, cols, &bad, s);
    if (rc == BSM_OK && bad) {
        set_error("column index out of bounds (>= cols %llu) in %llu entries", (unsigned long long)cols,
                  (unsigned long long)bad);
        rc = BSM_ERR_PANIC;
    }
    if (rc == BSM_OK) rc = h2d_staged(m->vals, static_cast<const char*>(vals) + base * es, nnz * es, s);
    if (rc == BSM_OK) rc = csr_analyse(m, s);
    if (rc != BSM_OK) {
        bsm_csr_free(m);
        return rc;
    }
    *out = m;
    return BSM_OK;
}

// The SpMM schedule of a handle for k right-hand columns, built once per
// matrix (like the matrix itself): the row-block x column-panel copy when
// wanted (schedule 0) or possible (1), else the column-panel plan. Declined
// shapes or no memory for the copy (with `reserve` bytes left free for the
// call's own buffers) fall back to the plans. Caller holds a->plan_mu.
int spmm_prepare_locked(const bsm_csr* a, uint64_t k, int schedule, uint64_t reserve, hipStream_t s,
                        PlanTimes* pt) {
    if (k == 0) return BSM_OK;
    BSM_TRY(csr_analyse(a, s));  // cached; device-built results are analysed here, lazily
    const auto t_start = host_now();
    if (schedule != 2 && !a->tiled_tried && !spmm_wants_split(a->dtype, k, a->max_row_len) &&
        (schedule == 1 ? (a->dtype == BSM_F64 || a->dtype == BSM_F32) && (k == 1 || k == 32) && a->nnz > 0
                       : tiled_wanted(a->dtype, a->rows, a->cols, a->nnz, k, a->max_row_len))) {
        a->tiled_tried = true;
        bsm_tiled* t = nullptr;
        const int rc = tiled_create(a->dtype, a->rows, a->cols, a->nnz, a->row_ptr, a->col, a->vals, k,
                                    schedule == 1 ? BSM_TILED_ANY_PADDING : 0, &t, s, reserve, pt);
        if (rc == BSM_OK) a->tiled = t;
        else if (rc != BSM_ERR_UNSUPPORTED && rc != BSM_ERR_OOM) return rc;
    }
    if (schedule != 2 && a->tiled && a->tiled->k == k) {
        if (pt) pt->total_ms += ms_since(t_start);
        return BSM_OK;
    }
    const uint64_t w = spmm_panel_cols(a->dtype, a->cols, k);
    if (w && a->plan_cols != w) {  // build (once per matrix and width) the column-panel plan
        const auto t0 = host_now();
        if (a->plan_seg) (void)hipFree(a->plan_seg);
        a->plan_seg = nullptr;
        a->plan_cols = 0;
        DBuf seg;
        BSM_TRY(seg.alloc(spmm_plan_bytes(a->rows, a->cols, w)));
        int usable = 0;
        BSM_TRY(spmm_plan(a->rows, a->cols, a->row_ptr, a->col, w, seg.as<int32_t>(), &usable, s));
        a->plan_seg = seg.as<int32_t>();
        seg.release();
        a->plan_cols = w;
        a->plan_usable = usable != 0;
        if (pt) pt->panel_ms += ms_since(t0);
    }
    if (pt) pt->total_ms += ms_since(t_start);
    return BSM_OK;
}

// Launch Y = A X with the schedule spmm_prepare_locked built (async on s).
int spmm_launch_locked(const bsm_csr* a, uint64_t k, bool allow_tiled, const void* x, void* y, int32_t* nz,
                       hipStream_t s) {
    if (k == 0) {
        if (nz && a->rows) BSM_HIP_TRY(hipMemsetAsync(nz, 0, a->rows * sizeof(int32_t), s));
        return BSM_OK;
    }
    BSM_TRY(csr_analyse(a, s));  // cached (a no-op once done)
    const uint64_t w = spmm_panel_cols(a->dtype, a->cols, k);
    if (allow_tiled && a->tiled && a->tiled->k == k) return tiled_spmm(a->tiled, x, y, nz, false, s);
    if (spmm_wants_split(a->dtype, k, a->max_row_len))
        return spmm_split_dispatch(a->dtype, a->rows, a->nnz, a->row_ptr, a->col, a->vals, k, x, y, nz, s);
    if (w && a->plan_usable && a->plan_cols == w)
        return spmm_panelled(a->dtype, a->rows, a->cols, a->nnz, a->row_ptr, a->col, a->vals, k, x, y, nz, w,
                             a->plan_seg, s);
    return spmm_dispatch(a->dtype, a->rows, a->cols, a->nnz, a->row_ptr, a->col, a->vals, k, x, y, nz, false, s,
                         a->max_row_len);
}

// mul_dense core on device operands: Y = A X, then compaction into a Csr.
static int mul_dense_device(const bsm_csr* a, uint64_t k, const void* x_dev, bsm_csr** out,
                            hipStream_t s) {
    const size_t es = dtype_size(a->dtype);
    const uint64_t rows = a->rows;
    DBuf y, row_nnz, ws;
    // small calls: temporaries from the per-thread arena, and the result's
    // col / vals sized for every entry (rows x k), so that the scan, the
    // compaction and the read of nnz share ONE synchronisation
    const size_t y_b = rows * k * es, nz_b = rows * sizeof(int32_t), ws_b = scan_workspace_bytes(rows);
    const bool small = y_b + rows * k * (es + sizeof(int32_t)) <= SCRATCH_MAX && nz_b + ws_b <= SCRATCH_MAX;
    void* yp = small ? scratch(0, y_b) : nullptr;
    const size_t nz_al = (nz_b + 255) / 256 * 256;
    void* nzp = yp ? scratch(1, nz_al + ws_b) : nullptr;
    if (!nzp) {
        BSM_TRY(y.alloc(y_b));
        BSM_TRY(row_nnz.alloc(nz_b));
        BSM_TRY(ws.alloc(ws_b));
        yp = y.p;
        nzp = row_nnz.p;
    }
    int32_t* const nz = static_cast<int32_t*>(nzp);
    void* const wsp = ws.p ? ws.p : static_cast<char*>(nzp) + nz_al;
    bsm_csr* r = nullptr;
    // out row_ptr is allocated first (nnz unknown until the scan completes);
    // the result's blocks come from the result cache
    RcBuf out_rp;
    BSM_TRY(out_rp.alloc(a->device, (rows + 1) * sizeof(int64_t)));
    {
        // one thread at a time builds and launches with the cached plan (a
        // rebuild frees the old plan; hipFree waits for launches using it).
        // The copy must leave room for this call's output: col + vals of up
        // to rows x k entries (no OOM after a copy that fit).
        std::lock_guard<std::mutex> plan_lock(a->plan_mu);
        const uint64_t reserve = small ? 0 : rows * k * (es + sizeof(int32_t)) + (rows + 1) * sizeof(int64_t);
        BSM_TRY(spmm_prepare_locked(a, k, 0, reserve, s, nullptr));
        BSM_TRY(spmm_launch_locked(a, k, true, x_dev, yp, nz, s));
    }
    // the smallest results (C1): scan + compaction in one workgroup that also
    // writes the host copy bsm_csr_download serves (compact_small)
    const bool arena = small && yp != y.p;
    char* host = nullptr;
    void* host_dev = nullptr;
    if (arena && k > 0 && rows > 0 && rows <= SMALL_OUT_ROWS && rows * k <= SMALL_OUT_CAP &&
        small_out_enabled())
        host = static_cast<char*>(pinned_result((rows + 1) * sizeof(int64_t) + small_col_bytes(rows * k) +
                                                    rows * k * es,
                                                &host_dev));
    const size_t wsb = ws.p ? ws.bytes : ws_b;
    if (!host) BSM_TRY(exclusive_scan_i32_to_i64(nz, out_rp.as<int64_t>(), rows, wsp, wsb, s));
    int64_t out_nnz = 0;
    if (!arena) BSM_HIP_TRY(read_dev(&out_nnz, out_rp.as<int64_t>() + rows, sizeof(int64_t), s));
    const uint64_t cap = arena ? rows * k : (uint64_t)out_nnz;
    r = new bsm_csr();
    r->dtype = a->dtype;
    r->device = a->device;
    r->rows = rows;
    r->cols = k;
    RcBuf oc, ov;
    int rc = oc.alloc(a->device, cap * sizeof(int32_t));
    if (rc == BSM_OK) rc = ov.alloc(a->device, cap * es);
    if (rc != BSM_OK) {
        delete r;
        return rc;
    }
    r->cache_cap[0] = out_rp.cap;
    r->cache_cap[1] = oc.cap;
    r->cache_cap[2] = ov.cap;
    r->row_ptr = static_cast<int64_t*>(out_rp.release());
    r->col = static_cast<int32_t*>(oc.release());
    r->vals = ov.release();
    r->analysed = true;
    r->rows_sorted = true;
    r->max_row_len = k;  // a bound: at most k entries per output row
    if (host) {
        rc = compact_small_dispatch(a->dtype, rows, k, nz, yp, r->row_ptr, r->col, r->vals, host_dev, cap, s);
        if (rc == BSM_OK) {
            hipError_t e = hipStreamSynchronize(s);  // the call's one synchronisation
            if (e != hipSuccess) {
                set_error("hipStreamSynchronize: %s", hipGetErrorString(e));
                rc = BSM_ERR_HIP;
            }
        }
        if (rc == BSM_OK) {
            out_nnz = reinterpret_cast<const int64_t*>(host)[rows];
            const size_t rp_b = (rows + 1) * sizeof(int64_t), col_b = (size_t)out_nnz * sizeof(int32_t);
            r->host_copy.reset(new char[rp_b + col_b + (size_t)out_nnz * es]);
            std::memcpy(r->host_copy.get(), host, rp_b + col_b);
            std::memcpy(r->host_copy.get() + rp_b + col_b, host + rp_b + small_col_bytes(cap), (size_t)out_nnz * es);
        }
    } else {
        rc = compact_dispatch(a->dtype, rows, k, yp, r->row_ptr, r->col, r->vals, s);
    }
    if (rc == BSM_OK && arena && !host) {  // nnz with the one synchronisation of the call
        hipError_t e = read_dev(&out_nnz, r->row_ptr + rows, sizeof(int64_t), s);
        if (e != hipSuccess) {
            set_error("read nnz: %s", hipGetErrorString(e));
            rc = BSM_ERR_HIP;
        }
    }
    r->nnz = (uint64_t)out_nnz;
    if (rc == BSM_OK && !host) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            set_error("hipStreamSynchronize: %s", hipGetErrorString(e));
            rc = BSM_ERR_HIP;
        }
    }
    if (rc != BSM_OK) {
        bsm_csr_free(r);
        return rc;
    }
    *out = r;
    return BSM_OK;
}

}  // namespace bsm

using namespace bsm;

extern "C" {

int bsm_stage_timing(int on) {
    g_stage_on.store(on ? 1 : 0, std::memory_order_relaxed);
    if (!on) stage_clear();
    return BSM_OK;
}

int bsm_stage_times(int max, int* n, char* names, double* ms) {
    BSM_REQUIRE(n && (max <= 0 || (names && ms)), BSM_ERR_INVALID, "null argument");
    const int have = g_stages.empty() ? 0 : (int)g_stages.size() - 1;
    *n = have;
    for (int i = 0; i < have && i < max; ++i) {
        BSM_HIP_TRY(hipEventSynchronize(g_stages[i + 1].ev));
        float t = 0.0f;
        BSM_HIP_TRY(hipEventElapsedTime(&t, g_stages[i].ev, g_stages[i + 1].ev));
        ms[i] = t;
        snprintf(names + 32 * i, 32, "%s", g_stages[i + 1].name.c_str());
    }
    return BSM_OK;
}

int bsm_api_version(void) { return BSM_API_VERSION; }

const char* bsm_last_error(void) { return bsm::last_error(); }

int bsm_device_count(int* n) {
    BSM_REQUIRE(n, BSM_ERR_INVALID, "null argument");
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) {
        *n = 0;
        set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
        return BSM_ERR_NO_DEVICE;
    }
    return BSM_OK;
}

int bsm_set_device(int ordinal) {
    BSM_HIP_TRY(hipSetDevice(ordinal));
    return BSM_OK;
}

int bsm_csr_upload(int dtype, uint64_t rows, uint64_t cols, uint64_t nnz, const uint64_t* row_ptr,
                   const uint64_t* col_idx, const void* vals, bsm_csr** out) {
    BSM_REQUIRE(out && row_ptr && (nnz == 0 || (col_idx && vals)), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(row_ptr[0] == 0 && row_ptr[rows] == nnz, BSM_ERR_INVALID,
                "row_ptr must start at 0 and end at nnz");
    for (uint64_t r = 0; r < rows; ++r)
        BSM_REQUIRE(row_ptr[r] <= row_ptr[r + 1], BSM_ERR_PANIC, "row_ptr not monotone at row %llu",
                    (unsigned long long)r);
    BSM_REQUIRE(dtype_size(dtype) != 0, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    return csr_upload_rows(dtype, 0, rows, cols, row_ptr, col_idx, vals, out, s);
}

int bsm_csr_from_inserts(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                         const uint64_t* col, const void* vals, bsm_csr** out) {
    BSM_REQUIRE(out && (n == 0 || (row && col && vals)), BSM_ERR_INVALID, "null argument");
    const size_t es = dtype_size(dtype);
    BSM_REQUIRE(es, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf dr, dc, dv;
    BSM_TRY(dr.alloc((n ? n : 1) * sizeof(uint64_t)));
    BSM_TRY(dc.alloc((n ? n : 1) * sizeof(uint64_t)));
    BSM_TRY(dv.alloc((n ? n : 1) * es));
    if (n) {
        BSM_HIP_TRY(hipMemcpyAsync(dr.p, row, n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        BSM_HIP_TRY(hipMemcpyAsync(dc.p, col, n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        BSM_HIP_TRY(hipMemcpyAsync(dv.p, vals, n * es, hipMemcpyHostToDevice, s));
    }
    return csr_from_inserts_device(dtype, rows, cols, n, dr.as<uint64_t>(), dc.as<uint64_t>(), dv.p, out, s);
}

int bsm_csr_from_coo(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                     const uint64_t* col, const void* vals, bsm_csr** out) {
    BSM_REQUIRE(out && (n == 0 || (row && col && vals)), BSM_ERR_INVALID, "null argument");
    const size_t es = dtype_size(dtype);
    BSM_REQUIRE(es, BSM_ERR_INVALID, "unknown dtype %d", dtype);
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf dr, dc, dv;
    BSM_TRY(dr.alloc((n ? n : 1) * sizeof(uint64_t)));
    BSM_TRY(dc.alloc((n ? n : 1) * sizeof(uint64_t)));
    BSM_TRY(dv.alloc((n ? n : 1) * es));
    if (n) {
        BSM_HIP_TRY(hipMemcpyAsync(dr.p, row, n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        BSM_HIP_TRY(hipMemcpyAsync(dc.p, col, n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        BSM_HIP_TRY(hipMemcpyAsync(dv.p, vals, n * es, hipMemcpyHostToDevice, s));
    }
    return csr_from_coo_device(dtype, rows, cols, n, dr.as<uint64_t>(), dc.as<uint64_t>(), dv.p, out, s);
}

int bsm_dev_csr_from_inserts(int dtype, uint64_t rows, uint64_t cols, uint64_t n, const uint64_t* row,
                             const uint64_t* col, const void* vals, bsm_csr** out, void* stream) {
    return csr_from_inserts_device(dtype, rows, cols, n, row, col, vals, out, static_cast<hipStream_t>(stream));
}

int bsm_dev_gen_insert_stream(int dtype, uint64_t seed, uint64_t i0, uint64_t n, uint64_t rows, uint64_t cols,
                              uint64_t vmod, uint64_t* row, uint64_t* col, void* vals, void* stream) {
    BSM_REQUIRE(n == 0 || (row && col && vals), BSM_ERR_INVALID, "null argument");
    return gen_insert_stream(dtype, seed, i0, n, rows, cols, vmod, row, col, vals, static_cast<hipStream_t>(stream));
}

int bsm_csr_shape(const bsm_csr* m, uint64_t* rows, uint64_t* cols, uint64_t* nnz, int* dtype) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    if (rows) *rows = m->rows;
    if (cols) *cols = m->cols;
    if (nnz) *nnz = m->nnz;
    if (dtype) *dtype = m->dtype;
    return BSM_OK;
}

int bsm_csr_download(const bsm_csr* m, uint64_t* row_ptr, uint64_t* col_idx, void* vals) {
    BSM_REQUIRE(m, BSM_ERR_INVALID, "null handle");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    const size_t es = dtype_size(m->dtype);
    const size_t rp_b = (m->rows + 1) * sizeof(int64_t), col_b = m->nnz * sizeof(int32_t), val_b = m->nnz * es;
    if (m->host_copy) {  // a small mul_dense result: its host copy, no device work
        const int64_t* rp64 = reinterpret_cast<const int64_t*>(m->host_copy.get());
        const int32_t* c32 = reinterpret_cast<const int32_t*>(m->host_copy.get() + rp_b);
        if (row_ptr)
            for (uint64_t r = 0; r <= m->rows; ++r) row_ptr[r] = (uint64_t)rp64[r];
        if (col_idx)
            for (uint64_t e = 0; e < m->nnz; ++e) col_idx[e] = (uint64_t)c32[e];
        if (vals && val_b) std::memcpy(vals, m->host_copy.get() + rp_b + col_b, val_b);
        return BSM_OK;
    }
    // page-locked destinations (bsm_host_register): direct DMA, no host copies
    // (row_ptr may be a small pageable array: its copy is tiny either way)
    // (up to 128M entries: the widened columns need an nnz x 8 B device temporary)
    if (m->nnz >= 4096 && m->nnz <= (128ull << 20) && (col_idx || vals) && (!col_idx || host_registered(col_idx)) &&
        (!vals || host_registered(vals)))
        return d2h_csr_direct(m->row_ptr, m->col, m->vals, m->rows, m->nnz, es, row_ptr, col_idx, vals, s);
    char* pin = rp_b + col_b + val_b <= PIN_MAX ? static_cast<char*>(pinned(rp_b + col_b + val_b)) : nullptr;
    if (!pin) {  // large: staged pipelines, columns widened to usize on the device
        if (row_ptr) BSM_TRY(d2h_staged(row_ptr, m->row_ptr, rp_b, s));  // int64 >= 0: the same bits as u64
        if (col_idx) BSM_TRY(d2h_cols_widen(col_idx, m->col, m->nnz, s));
        if (vals) BSM_TRY(d2h_staged(vals, m->vals, val_b, s));
        return BSM_OK;
    }
    // small: three copies into one pinned buffer, one sync
    int64_t* rp64 = reinterpret_cast<int64_t*>(pin);
    int32_t* c32 = reinterpret_cast<int32_t*>(pin + rp_b);
    char* vdst = pin + rp_b + col_b;
    BSM_HIP_TRY(hipMemcpyAsync(rp64, m->row_ptr, rp_b, hipMemcpyDeviceToHost, s));
    if (m->nnz) {
        BSM_HIP_TRY(hipMemcpyAsync(c32, m->col, col_b, hipMemcpyDeviceToHost, s));
        if (vals) BSM_HIP_TRY(hipMemcpyAsync(vdst, m->vals, val_b, hipMemcpyDeviceToHost, s));
    }
    BSM_HIP_TRY(hipStreamSynchronize(s));
    if (row_ptr)
        for (uint64_t r = 0; r <= m->rows; ++r) row_ptr[r] = (uint64_t)rp64[r];
    if (col_idx)
        for (uint64_t e = 0; e < m->nnz; ++e) col_idx[e] = (uint64_t)c32[e];
    if (vals && val_b) std::memcpy(vals, vdst, val_b);
    return BSM_OK;
}

int bsm_host_register(void* p, uint64_t bytes) {
    BSM_REQUIRE(p && bytes, BSM_ERR_INVALID, "null or empty range");
    BSM_HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterDefault));
    return BSM_OK;
}

int bsm_host_unregister(void* p) {
    BSM_REQUIRE(p, BSM_ERR_INVALID, "null pointer");
    BSM_HIP_TRY(hipHostUnregister(p));
    return BSM_OK;
}

void bsm_csr_free(bsm_csr* m) {
    if (!m) return;
    if (m->cache_cap[0] || m->cache_cap[1] || m->cache_cap[2]) {
        // what hipFree would wait for: work still queued on the result (any
        // stream of its device) must finish before the blocks are reused
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != m->device) (void)hipSetDevice(m->device);
        (void)hipDeviceSynchronize();
        if (cur != m->device && cur >= 0) (void)hipSetDevice(cur);
    }
    rc_release(m->device, m->row_ptr, m->cache_cap[0]);
    rc_release(m->device, m->col, m->cache_cap[1]);
    rc_release(m->device, m->vals, m->cache_cap[2]);
    if (m->plan_seg) (void)hipFree(m->plan_seg);
    if (m->tiled) tiled_destroy(m->tiled);
    delete m;
}

int bsm_csr_mul_dense(const bsm_csr* a, uint64_t k, uint64_t x_rows, const void* const* x_cols,
                      bsm_csr** out) {
    BSM_REQUIRE(a && out && (k == 0 || x_cols), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->cols == x_rows, BSM_ERR_DIMENSIONS, "IncorrectDimensions: cols %llu != rhs rows %llu",
                (unsigned long long)a->cols, (unsigned long long)x_rows);
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf x;
    void* xp = nullptr;
    bool synced = true;
    const size_t x_b = x_rows * k * dtype_size(a->dtype);
    // the arena slot only serves the pinned (small) upload path
    void* small_x = x_b && x_b <= PIN_MAX ? scratch(3, x_b) : nullptr;
    int rc = upload_columns(a->dtype, x_rows, k, x_cols, x, s, &xp, small_x, &synced);
    if (rc == BSM_OK) rc = mul_dense_device(a, k, xp, out, s);
    if (!synced) (void)hipStreamSynchronize(s);  // the pinned upload buffer is free again on every path
    return rc;
}

int bsm_csr_mul_vector(const bsm_csr* a, const void* rhs, uint64_t rhs_len, void* out,
                       uint64_t out_len) {
    BSM_REQUIRE(a, BSM_ERR_INVALID, "null handle");
    BSM_REQUIRE(a->cols == rhs_len && a->rows == out_len, BSM_ERR_DIMENSIONS, "IncorrectDimensions");
    BSM_REQUIRE((rhs || rhs_len == 0) && (out || out_len == 0), BSM_ERR_INVALID, "null argument");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    const size_t es = dtype_size(a->dtype);
    // The reference sums in ascending source-column order (it walks the
    // transpose, sparse.rs:474-479). For row-sorted matrices that is the
    // storage order; otherwise sort each row stably first: (A^T)^T.
    const bsm_csr* src = a;
    bsm_csr* sorted = nullptr;
    BSM_TRY(csr_analyse(a, s));  // rows_sorted (cached)
    if (!a->rows_sorted) {
        bsm_csr* t = nullptr;
        BSM_TRY(transpose_dispatch(a, &t, s));
        int rc = transpose_dispatch(t, &sorted, s);
        bsm_csr_free(t);
        if (rc != BSM_OK) return rc;
        src = sorted;
    }
    DBuf x, y;
    int rc = x.alloc(rhs_len * es);
    if (rc == BSM_OK) rc = y.alloc(out_len * es);
    if (rc == BSM_OK && rhs_len) {
        hipError_t e = hipMemcpyAsync(x.p, rhs, rhs_len * es, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { set_error("H2D: %s", hipGetErrorString(e)); rc = BSM_ERR_HIP; }
    }
    if (rc == BSM_OK)
        rc = spmm_dispatch(src->dtype, src->rows, src->cols, src->nnz, src->row_ptr, src->col,
                           src->vals, 1, x.p, y.p, nullptr, true, s,
                           src->analysed ? src->max_row_len : UINT64_MAX);
    if (rc == BSM_OK && out_len) {
        hipError_t e = hipMemcpyAsync(out, y.p, out_len * es, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) { set_error("D2H: %s", hipGetErrorString(e)); rc = BSM_ERR_HIP; }
    }
    if (rc == BSM_OK) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) { set_error("sync: %s", hipGetErrorString(e)); rc = BSM_ERR_HIP; }
    }
    bsm_csr_free(sorted);
    return rc;
}

int bsm_csr_add_sparse(const bsm_csr* a, const bsm_csr* b, bsm_csr** out) {
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    return sparse_addsub_dispatch(a, b, false, out, s);
}

int bsm_csr_sub_sparse(const bsm_csr* a, const bsm_csr* b, bsm_csr** out) {
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    return sparse_addsub_dispatch(a, b, true, out, s);
}

int bsm_csr_mul_sparse(const bsm_csr* a, const bsm_csr* b, bsm_csr** out) {
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    return sparse_mul_dispatch(a, b, out, s);
}

int bsm_csr_transpose(const bsm_csr* a, bsm_csr** out) {
    BSM_REQUIRE(a && out, BSM_ERR_INVALID, "null argument");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    return transpose_dispatch(a, out, s);
}

int bsm_csr_cholesky(const bsm_csr* a, bsm_csr** out) {
    BSM_REQUIRE(a && out, BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->rows == a->cols, BSM_ERR_NON_SQUARE, "NonSquareMatrix");
    BSM_REQUIRE(a->dtype == BSM_F32 || a->dtype == BSM_F64, BSM_ERR_INVALID,
                "cholesky_decomp is defined for f32 (reference) and f64 only");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    stage_reset(s);
    return solve_dispatch_cholesky(a, out, s);
}

static int trsv_host(const bsm_csr* m, bool lower, uint64_t k, uint64_t n, const void* const* b_cols,
                     void* const* x_cols) {
    BSM_REQUIRE(m && (k == 0 || (b_cols && x_cols)), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(m->dtype == BSM_F32 || m->dtype == BSM_F64, BSM_ERR_INVALID, "f32/f64 only");
    BSM_REQUIRE(m->rows >= n, BSM_ERR_PANIC, "matrix has fewer rows than the RHS (index out of bounds)");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf b, x;
    BSM_TRY(upload_columns(m->dtype, n, k, b_cols, b, s));
    BSM_TRY(x.alloc(n * k * dtype_size(m->dtype)));
    BSM_TRY(solve_dispatch_trsv(m, lower, k, n, b.p, x.p, s));
    return download_columns(m->dtype, n, k, x.p, x_cols, s);
}

int bsm_forward_substitution(const bsm_csr* l, uint64_t k, uint64_t n, const void* const* b_cols,
                             void* const* y_cols) {
    return trsv_host(l, true, k, n, b_cols, y_cols);
}

int bsm_backward_substitution(const bsm_csr* u, uint64_t k, uint64_t n, const void* const* y_cols,
                              void* const* x_cols) {
    return trsv_host(u, false, k, n, y_cols, x_cols);
}

int bsm_solve(const bsm_csr* a, uint64_t k, uint64_t n, const void* const* b_cols, void* const* x_cols) {
    BSM_REQUIRE(a && (k == 0 || (b_cols && x_cols)), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->rows == a->cols, BSM_ERR_PANIC,
                "solve: cholesky_decomp().unwrap() on a non-square matrix panics (lib.rs:20)");
    BSM_REQUIRE(a->dtype == BSM_F32 || a->dtype == BSM_F64, BSM_ERR_INVALID, "f32/f64 only");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf b, x;
    BSM_TRY(upload_columns(a->dtype, n, k, b_cols, b, s));
    BSM_TRY(x.alloc(n * k * dtype_size(a->dtype)));
    BSM_TRY(solve_dispatch_full(a, k, n, b.p, x.p, s));
    return download_columns(a->dtype, n, k, x.p, x_cols, s);
}

int bsm_solve_blocked(const bsm_csr* a, uint64_t k, uint64_t n, const void* const* b_cols, void* const* x_cols) {
    BSM_REQUIRE(a && (k == 0 || (b_cols && x_cols)), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->rows == a->cols, BSM_ERR_PANIC,
                "solve: cholesky_decomp().unwrap() on a non-square matrix panics (lib.rs:20)");
    BSM_REQUIRE(a->dtype == BSM_F32 || a->dtype == BSM_F64, BSM_ERR_INVALID, "f32/f64 only");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf b, x;
    BSM_TRY(upload_columns(a->dtype, n, k, b_cols, b, s));
    BSM_TRY(x.alloc(n * k * dtype_size(a->dtype)));
    BSM_TRY(solve_dispatch_blocked(a, k, n, b.p, x.p, s));
    return download_columns(a->dtype, n, k, x.p, x_cols, s);
}

int bsm_solve_nd(const bsm_csr* a, uint64_t k, uint64_t n, const void* const* b_cols, void* const* x_cols) {
    BSM_REQUIRE(a && (k == 0 || (b_cols && x_cols)), BSM_ERR_INVALID, "null argument");
    BSM_REQUIRE(a->rows == a->cols, BSM_ERR_PANIC,
                "solve: cholesky_decomp().unwrap() on a non-square matrix panics (lib.rs:20)");
    BSM_REQUIRE(a->dtype == BSM_F32 || a->dtype == BSM_F64, BSM_ERR_INVALID, "f32/f64 only");
    hipStream_t s;
    BSM_TRY(ctx_stream(&s));
    DBuf b, x;
    BSM_TRY(upload_columns(a->dtype, n, k, b_cols, b, s));
    BSM_TRY(x.alloc(n * k * dtype_size(a->dtype)));
    BSM_TRY(solve_dispatch_nd(a, k, n, b.p, x.p, s));
    return download_columns(a->dtype, n, k, x.p, x_cols, s);
}

// ---- device-level entry points --------------------------------------------
uint64_t bsm_dev_scan_workspace_bytes(uint64_t n) {
    return ((n * sizeof(int32_t) + 255) / 256) * 256 + scan_workspace_bytes(n);
}

int bsm_dev_gen_row_ptr(uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols, int rowlen_kind,
                        uint32_t a, uint32_t b, int64_t* row_ptr, void* workspace,
                        uint64_t workspace_bytes, void* stream) {
    BSM_REQUIRE(row_ptr, BSM_ERR_INVALID, "null argument");
    return gen_row_ptr(seed, row0, rows, n_cols, rowlen_kind, a, b, row_ptr, workspace, workspace_bytes,
                       static_cast<hipStream_t>(stream));
}

int bsm_dev_gen_entries(int dtype, uint64_t seed, uint64_t row0, uint64_t rows, uint32_t n_cols,
                        int value_kind, const int64_t* row_ptr, int32_t* col, void* vals, void* stream) {
    BSM_REQUIRE(row_ptr && col && vals, BSM_ERR_INVALID, "null argument");
    return gen_entries(dtype, seed, row0, rows, n_cols, value_kind, row_ptr, col, vals,
                       static_cast<hipStream_t>(stream));
}

int bsm_dev_gen_dense(int dtype, uint64_t seed, uint64_t row0, uint64_t n, uint64_t k, int value_kind,
                      void* x, void* stream) {
    BSM_REQUIRE(x || n * k == 0, BSM_ERR_INVALID, "null argument");
    return gen_dense(dtype, seed, row0, n, k, value_kind, x, static_cast<hipStream_t>(stream));
}

int bsm_dev_spmm(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* row_ptr,
                 const int32_t* col, const void* vals, uint64_t k, const void* x, void* y,
                 int32_t* row_nnz, void* stream) {
    BSM_REQUIRE(row_ptr && (nnz == 0 || (col && vals)) && (k == 0 || (x && y)), BSM_ERR_INVALID,
                "null argument");
    if (k == 0) return BSM_OK;
    return spmm_dispatch(dtype, rows, n_cols, nnz, row_ptr, col, vals, k, x, y, row_nnz, false,
                         static_cast<hipStream_t>(stream));
}

int bsm_csr_panel_cols(const bsm_csr* m, uint64_t* panel_cols) {
    BSM_REQUIRE(m && panel_cols, BSM_ERR_INVALID, "null argument");
    *panel_cols = m->plan_usable ? m->plan_cols : 0;
    return BSM_OK;
}

uint64_t bsm_dev_spmm_panel_cols(int dtype, uint64_t n_cols, uint64_t k) {
    return spmm_panel_cols(dtype, n_cols, k);
}

uint64_t bsm_dev_spmm_plan_bytes(uint64_t rows, uint64_t n_cols, uint64_t panel_cols) {
    return spmm_plan_bytes(rows, n_cols, panel_cols);
}

int bsm_dev_spmm_plan(uint64_t rows, uint64_t n_cols, const int64_t* row_ptr, const int32_t* col,
                      uint64_t panel_cols, int32_t* seg, int* usable, void* stream) {
    BSM_REQUIRE(row_ptr && usable && (spmm_plan_bytes(rows, n_cols, panel_cols) == 0 || seg),
                BSM_ERR_INVALID, "null argument");
    return spmm_plan(rows, n_cols, row_ptr, col, panel_cols, seg, usable,
                     static_cast<hipStream_t>(stream));
}

int bsm_dev_spmm_panelled(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz,
                          const int64_t* row_ptr, const int32_t* col, const void* vals, uint64_t k,
                          const void* x, void* y, int32_t* row_nnz, uint64_t panel_cols,
                          const int32_t* seg, void* stream) {
    BSM_REQUIRE(row_ptr && (nnz == 0 || (col && vals)) && (k == 0 || (x && y)), BSM_ERR_INVALID,
                "null argument");
    if (k == 0) return BSM_OK;
    return spmm_panelled(dtype, rows, n_cols, nnz, row_ptr, col, vals, k, x, y, row_nnz, panel_cols,
                         seg, static_cast<hipStream_t>(stream));
}

int bsm_dev_tiled_wanted(int dtype, uint64_t rows, uint64_t n_cols, uint64_t nnz, uint64_t k,
                         uint64_t max_row_len) {
    return tiled_wanted(dtype, rows, n_cols, nnz, k, max_row_len) ? 1 : 0;
}

int bsm_dev_tiled_create(uint64_t rows, uint64_t n_cols, uint64_t nnz, const int64_t* row_ptr,
                         const int32_t* col, const double* vals, uint64_t k, int flags, bsm_tiled** out,
                         void* stream) {
    return tiled_create(BSM_F64, rows, n_cols, nnz, row_ptr, col, vals, k, flags, out, static_cast<hipStream_t>(stream));
}

int bsm_dev_spmm_tiled(const bsm_tiled* t, const double* x, double* y, int32_t* row_nnz, void* stream) {
    return tiled_spmm(t, x, y, row_nnz, false, static_cast<hipStream_t>(stream));
}

int bsm_tiled_info(const bsm_tiled* t, uint64_t* bytes, uint64_t* slots, uint64_t* panel_cols) {
    BSM_REQUIRE(t, BSM_ERR_INVALID, "null argument");
    const uint64_t n = (t->chunks + t->overread) * 64;
    if (bytes) *bytes = n * (t->meta_bytes + (t->dtype == BSM_F32 ? 4 : 8)) + ((uint64_t)t->nw * t->nb + 1) * 8;
    if (slots) *slots = t->chunks * 64;
    if (panel_cols) *panel_cols = 1ull << t->pshift;
    return BSM_OK;
}

void bsm_tiled_destroy(bsm_tiled* t) { tiled_destroy(t); }

int bsm_csr_tiled(const bsm_csr* m, int* in_use) {
    BSM_REQUIRE(m && in_use, BSM_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lock(m->plan_mu);
    *in_use = m->tiled ? 1 : 0;
    return BSM_OK;
}

int bsm_dev_compact(int dtype, uint64_t rows, uint64_t k, const void* y, const int32_t* row_nnz,
                    int64_t* out_row_ptr, int32_t* out_col, void* out_vals, void* workspace,
                    uint64_t workspace_bytes, void* stream) {
    BSM_REQUIRE(row_nnz && out_row_ptr, BSM_ERR_INVALID, "null argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    BSM_TRY(exclusive_scan_i32_to_i64(row_nnz, out_row_ptr, rows, workspace, workspace_bytes, s));
    return compact_dispatch(dtype, rows, k, y, out_row_ptr, out_col, out_vals, s);
}

}  // extern "C"
