// transfer.hip -- host <-> device marshalling of the host-buffer entry points.
//
// A Rust caller of Csr::mul_dense (src/sparse.rs:426-446) hands over pageable
// Vecs: usize column indices (8 B) and k separate Dense columns
// (dense.rs:8), and takes back a fresh Csr with usize indices. Moving those
// through the driver's own pageable path, with the 8 B <-> 4 B index
// conversion as a scalar host loop, cost 7x the device time at C3 (round 2:
// 102 ms against 13.8 ms). Here index conversions run on the device (a
// narrowing / widening kernel per chunk); uploads go by the runtime's pageable
// DMA at the link rate, downloads through two pinned chunk buffers (host
// threads copy chunk i out while the DMA fills chunk i+1), with the caller's
// fresh result pages faulted in ahead by host threads, as huge pages.
#include <algorithm>
#include <atomic>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <sys/mman.h>
#include <vector>

#include "bsm_internal.hpp"

namespace bsm {
namespace {

constexpr size_t STAGE_CHUNK = 16ull << 20;  // bytes per pipeline chunk

size_t env_size(const char* name, size_t dflt) {
    const char* e = getenv(name);
    return e ? (size_t)strtoull(e, nullptr, 10) : dflt;
}

// memcpy split over a few threads (one host thread copies ~10 GB/s, PCIe
// moves ~50 GB/s)
void par_memcpy(void* dst, const void* src, size_t n) {
    static const int threads = (int)std::clamp<size_t>(env_size("BSM_COPY_THREADS", 4), 1, 16);
    const int t = n >= (4ull << 20) ? threads : 1;
    if (t == 1) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t part = (n / t + 4095) & ~size_t(4095);
    std::thread th[16];
    int used = 0;
    for (int i = 1; i < t; ++i) {
        const size_t off = part * i;
        if (off >= n) break;
        th[used++] = std::thread([=] { std::memcpy(static_cast<char*>(dst) + off, static_cast<const char*>(src) + off,
                                                   std::min(part, n - off)); });
    }
    std::memcpy(dst, src, std::min(part, n));
    for (int i = 0; i < used; ++i) th[i].join();
}

// two pinned chunk buffers and their events, per thread
struct Stage {
    void* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    size_t cap = 0;
    ~Stage() {
        for (int i = 0; i < 2; ++i) {
            if (buf[i]) (void)hipHostFree(buf[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
        }
    }
    int get(size_t bytes) {
        if (cap >= bytes && ev[0]) return BSM_OK;
        for (int i = 0; i < 2; ++i) {
            if (buf[i]) (void)hipHostFree(buf[i]);
            buf[i] = nullptr;
        }
        cap = 0;
        for (int i = 0; i < 2; ++i) {
            BSM_HIP_TRY(hipHostMalloc(&buf[i], bytes, hipHostMallocDefault));
            if (!ev[i]) BSM_HIP_TRY(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        }
        cap = bytes;
        return BSM_OK;
    }
};
Stage& stage() {
    static thread_local Stage st;
    return st;
}

// Host -> device: the runtime's own pageable copies (BSM_XFER_H2D=direct,
// the default) reach the link rate (56 GB/s, profiles/r03_b_marshal.log);
// BSM_XFER_H2D=staged selects the pinned two-buffer pipeline. Device ->
// host: staged by default. A direct pageable DMA into the caller's fresh
// result arrays is as fast, but the runtime then holds those pages, and the
// caller's later free of the 520 MB of a C3 result took 25-30 ms
// (profiles/r03_g_xfer_dbg.log) against ~0 after a staged copy.
bool direct_mode(bool h2d) {
    static const bool d_h2d = [] {
        const char* e = getenv("BSM_XFER_H2D");
        return !(e && std::strcmp(e, "staged") == 0);
    }();
    static const bool d_d2h = [] {
        const char* e = getenv("BSM_XFER_D2H");
        return e && std::strcmp(e, "direct") == 0;
    }();
    return h2d ? d_h2d : d_d2h;
}

size_t chunk_bytes() {
    static const size_t c = std::max<size_t>(env_size("BSM_STAGE_CHUNK", STAGE_CHUNK), 1 << 16) & ~size_t(255);
    return c;
}

__global__ __launch_bounds__(256) void narrow_u64_i32(const uint64_t* __restrict__ in, int32_t* __restrict__ out,
                                                      uint64_t n, uint64_t cols, unsigned long long* bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b = false;
    if (i < n) {
        const uint64_t c = in[i];
        b = c >= cols;
        out[i] = (int32_t)c;
    }
    const uint64_t m = __ballot(b);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}

__global__ __launch_bounds__(256) void rebase_u64_i64(int64_t* __restrict__ rp, uint64_t n, uint64_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rp[i] = (int64_t)((uint64_t)rp[i] - base);
}

__global__ __launch_bounds__(256) void widen_i32_u64(const int32_t* __restrict__ in, uint64_t* __restrict__ out,
                                                     uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint64_t)(uint32_t)in[i];
}

inline unsigned blocks(uint64_t n) { return (unsigned)((n + 255) / 256); }

// Fault in [p, p + bytes) chunk by chunk from BSM_TOUCH_THREADS threads
// (default 8): a write per 4 KiB page; wait(i) returns once chunk i is in.
class Prefault {
public:
    Prefault(char* p, size_t bytes, size_t chunk) : p_(p), bytes_(bytes), chunk_(chunk) {
        static const int threads = (int)std::clamp<size_t>(env_size("BSM_TOUCH_THREADS", 8), 0, 32);
        n_ = (bytes + chunk - 1) / chunk;
        if (threads == 0 || bytes < (8ull << 20)) {
            n_ = 0;  // small: the DMA takes its own faults
            return;
        }
        // transparent huge pages for the 2 MiB-aligned interior (advice only;
        // the box runs THP in madvise mode): 520 MB faults in 3.8 ms on 8
        // threads with it, 30-40 ms without (profiles/r03_e_first_touch.log)
        const uintptr_t a0 = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
        const uintptr_t a1 = ((uintptr_t)p + bytes) & ~(uintptr_t)((2u << 20) - 1);
        if (a1 > a0) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
        ready_.reset(new std::atomic<int>[n_]);
        for (size_t i = 0; i < n_; ++i) ready_[i].store(0, std::memory_order_relaxed);
        for (int t = 0; t < threads; ++t)
            th_.emplace_back([this] {
                for (;;) {
                    const size_t i = next_.fetch_add(1, std::memory_order_relaxed);
                    if (i >= n_ || stop_.load(std::memory_order_relaxed)) return;
                    char* q = p_ + i * chunk_;
                    const size_t len = std::min(chunk_, bytes_ - i * chunk_);
                    for (size_t o = 0; o < len; o += 4096) reinterpret_cast<volatile char*>(q)[o] = 0;
                    ready_[i].store(1, std::memory_order_release);
                }
            });
    }
    void wait(size_t i) {
        if (i >= n_) return;
        while (!ready_[i].load(std::memory_order_acquire)) std::this_thread::yield();
    }
    void finish() {
        stop_.store(true, std::memory_order_relaxed);
        for (auto& t : th_) t.join();
        th_.clear();
    }
    ~Prefault() { finish(); }

private:
    char* p_;
    size_t bytes_, chunk_, n_ = 0;
    std::unique_ptr<std::atomic<int>[]> ready_;
    std::atomic<size_t> next_{0};
    std::atomic<bool> stop_{false};
    std::vector<std::thread> th_;
};

}  // namespace

// Host -> device, synchronous (src may be released when it returns). The
// pipeline: chunk i is copied into pinned buffer i % 2 on the host (waiting
// for that buffer's previous DMA), then its DMA is queued; `post(off, len,
// staged_dev)` may enqueue device work on each chunk after its DMA when
// `dev_stage` (two device chunk buffers) is given, else the DMA lands at dst.
template <typename Post>
static int h2d_pipeline(void* dst, const void* src, size_t bytes, hipStream_t s, void* dev_stage, Post&& post) {
    if (bytes == 0) return BSM_OK;
    const size_t C = chunk_bytes();
    if (direct_mode(true)) {  // pageable DMA per chunk, the device work behind it
        const size_t n = (bytes + C - 1) / C;
        for (size_t i = 0; i < n; ++i) {
            const size_t off = i * C, len = std::min(C, bytes - off);
            void* d = dev_stage ? static_cast<char*>(dev_stage) + (i & 1) * C : static_cast<char*>(dst) + off;
            BSM_HIP_TRY(hipMemcpyAsync(d, static_cast<const char*>(src) + off, len, hipMemcpyHostToDevice, s));
            if (dev_stage) BSM_TRY(post(off, len, d));
        }
        BSM_HIP_TRY(hipStreamSynchronize(s));
        return BSM_OK;
    }
    Stage& st = stage();
    BSM_TRY(st.get(std::min(C, bytes)));
    const size_t n = (bytes + C - 1) / C;
    for (size_t i = 0; i < n; ++i) {
        const size_t off = i * C, len = std::min(C, bytes - off);
        const int b = (int)(i & 1);
        if (i >= 2) BSM_HIP_TRY(hipEventSynchronize(st.ev[b]));
        par_memcpy(st.buf[b], static_cast<const char*>(src) + off, len);
        void* d = dev_stage ? static_cast<char*>(dev_stage) + (size_t)b * C : static_cast<char*>(dst) + off;
        BSM_HIP_TRY(hipMemcpyAsync(d, st.buf[b], len, hipMemcpyHostToDevice, s));
        if (dev_stage) BSM_TRY(post(off, len, d));
        BSM_HIP_TRY(hipEventRecord(st.ev[b], s));
    }
    BSM_HIP_TRY(hipStreamSynchronize(s));
    return BSM_OK;
}

int h2d_staged(void* dst, const void* src, size_t bytes, hipStream_t s) {
    return h2d_pipeline(dst, src, bytes, s, nullptr, [](size_t, size_t, void*) { return BSM_OK; });
}

// Device -> host, synchronous. `pre(off, len, staged_dev)` may fill a device
// chunk buffer (two of them in dev_stage) that the DMA then reads, else the
// DMA reads src.
template <typename Pre>
static int d2h_pipeline(void* dst, const void* src, size_t bytes, hipStream_t s, void* dev_stage, Pre&& pre) {
    if (bytes == 0) return BSM_OK;
    const size_t C = chunk_bytes();
    if (direct_mode(false)) {
        // The caller's result arrays are fresh (Rust Vec::with_capacity, numpy
        // empty): their first touch is a zero-fill page fault per 4 KiB, 43 ms
        // for C3's 520 MB against 10 ms for the DMA itself
        // (profiles/r03_c_marshal.log). Host threads fault the chunks in (huge
        // pages where the mapping allows), in order, ahead of the DMA.
        const size_t n = (bytes + C - 1) / C;
        static const bool dbg = getenv("BSM_XFER_DEBUG") != nullptr;
        const auto t0 = host_now();
        Prefault pf(static_cast<char*>(dst), bytes, C);
        double t_wait = 0, t_dma = 0;
        int rc = BSM_OK;
        for (size_t i = 0; i < n && rc == BSM_OK; ++i) {
            const size_t off = i * C, len = std::min(C, bytes - off);
            const void* from = static_cast<const char*>(src) + off;
            if (dev_stage) {
                void* d = static_cast<char*>(dev_stage) + (i & 1) * C;
                rc = pre(off, len, d);
                from = d;
            }
            auto tw = host_now();
            pf.wait(i);
            t_wait += ms_since(tw);
            tw = host_now();
            if (rc == BSM_OK && hipMemcpyAsync(static_cast<char*>(dst) + off, from, len, hipMemcpyDeviceToHost, s) !=
                                    hipSuccess) {
                set_error("d2h: %s", hipGetErrorString(hipGetLastError()));
                rc = BSM_ERR_HIP;
            }
            t_dma += ms_since(tw);
        }
        pf.finish();
        BSM_TRY(rc);
        BSM_HIP_TRY(hipStreamSynchronize(s));
        if (dbg)
            fprintf(stderr, "[bsm xfer] d2h %zu B in %zu chunks: %.2f ms (prefault waits %.2f, DMA calls %.2f)\n",
                    bytes, n, ms_since(t0), t_wait, t_dma);
        return BSM_OK;
    }
    Stage& st = stage();
    BSM_TRY(st.get(std::min(C, bytes)));
    const size_t n = (bytes + C - 1) / C;
    Prefault pf(static_cast<char*>(dst), bytes, C);  // fresh result pages, faulted in ahead of the copies
    auto drain = [&](size_t i) -> int {  // chunk i's DMA done -> copy out of its pinned buffer
        const size_t off = i * C, len = std::min(C, bytes - off);
        BSM_HIP_TRY(hipEventSynchronize(st.ev[i & 1]));
        pf.wait(i);
        par_memcpy(static_cast<char*>(dst) + off, st.buf[i & 1], len);
        return BSM_OK;
    };
    for (size_t i = 0; i < n; ++i) {
        const size_t off = i * C, len = std::min(C, bytes - off);
        const int b = (int)(i & 1);
        const void* from = static_cast<const char*>(src) + off;
        if (dev_stage) {
            void* d = static_cast<char*>(dev_stage) + (size_t)b * C;
            BSM_TRY(pre(off, len, d));
            from = d;
        }
        BSM_HIP_TRY(hipMemcpyAsync(st.buf[b], from, len, hipMemcpyDeviceToHost, s));
        BSM_HIP_TRY(hipEventRecord(st.ev[b], s));
        if (i >= 1) BSM_TRY(drain(i - 1));  // overlaps chunk i's DMA
    }
    BSM_TRY(drain(n - 1));
    return BSM_OK;
}

int d2h_staged(void* dst, const void* src, size_t bytes, hipStream_t s) {
    return d2h_pipeline(dst, src, bytes, s, nullptr, [](size_t, size_t, void*) { return BSM_OK; });
}

// Host usize column indices -> device int32, checked against cols on the
// device; *bad = entries with col >= cols.
int h2d_cols_narrow(int32_t* dst, const uint64_t* src, uint64_t n, uint64_t cols, uint64_t* bad, hipStream_t s) {
    *bad = 0;
    if (n == 0) return BSM_OK;
    DBuf dstage, dbad;
    const size_t C = chunk_bytes();
    BSM_TRY(dstage.alloc(2 * std::min<size_t>(C, n * 8)));
    BSM_TRY(dbad.alloc(sizeof(unsigned long long)));
    BSM_HIP_TRY(hipMemsetAsync(dbad.p, 0, sizeof(unsigned long long), s));
    auto* cnt = dbad.as<unsigned long long>();
    BSM_TRY(h2d_pipeline(nullptr, src, n * 8, s, dstage.p, [&](size_t off, size_t len, void* d) -> int {
        const uint64_t e = off / 8, m = len / 8;
        narrow_u64_i32<<<blocks(m), 256, 0, s>>>(static_cast<const uint64_t*>(d), dst + e, m, cols, cnt);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    }));
    unsigned long long h = 0;
    BSM_HIP_TRY(read_dev(&h, cnt, sizeof(h), s));
    *bad = h;
    return BSM_OK;
}

// Host usize row_ptr (n entries, starting at `base`) -> device int64 rebased to 0.
int h2d_row_ptr(int64_t* dst, const uint64_t* src, uint64_t n, uint64_t base, hipStream_t s) {
    BSM_TRY(h2d_staged(dst, src, n * 8, s));
    if (base && n) {
        rebase_u64_i64<<<blocks(n), 256, 0, s>>>(dst, n, base);
        BSM_HIP_TRY(hipGetLastError());
        BSM_HIP_TRY(hipStreamSynchronize(s));
    }
    return BSM_OK;
}

// Device int32 column indices -> host usize, widened on the device.
// Device -> page-locked host memory (registered or hipHostMalloc'd, e.g. the
// Python mirror's host result pool): the DMA writes the caller's arrays
// directly, the columns widened on the device first; one sync.
bool host_registered(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // plain pageable memory
        return false;
    }
    return at.type == hipMemoryTypeHost;
}
int d2h_csr_direct(const int64_t* rp, const int32_t* col, const void* vals, uint64_t rows, uint64_t nnz, size_t es,
                   uint64_t* row_ptr, uint64_t* col_idx, void* vals_out, hipStream_t s) {
    DBuf wide;
    if (col_idx && nnz) {
        BSM_TRY(wide.alloc(nnz * 8, s));
        widen_i32_u64<<<blocks(nnz), 256, 0, s>>>(col, wide.as<uint64_t>(), nnz);
        BSM_HIP_TRY(hipGetLastError());
    }
    if (row_ptr) BSM_HIP_TRY(hipMemcpyAsync(row_ptr, rp, (rows + 1) * 8, hipMemcpyDeviceToHost, s));
    if (col_idx && nnz) BSM_HIP_TRY(hipMemcpyAsync(col_idx, wide.p, nnz * 8, hipMemcpyDeviceToHost, s));
    if (vals_out && nnz) BSM_HIP_TRY(hipMemcpyAsync(vals_out, vals, nnz * es, hipMemcpyDeviceToHost, s));
    BSM_HIP_TRY(hipStreamSynchronize(s));
    return BSM_OK;
}

int d2h_cols_widen(uint64_t* dst, const int32_t* src, uint64_t n, hipStream_t s) {
    if (n == 0) return BSM_OK;
    DBuf dstage;
    const size_t C = chunk_bytes();
    BSM_TRY(dstage.alloc(2 * std::min<size_t>(C, n * 8)));
    return d2h_pipeline(dst, nullptr, n * 8, s, dstage.p, [&](size_t off, size_t len, void* d) -> int {
        const uint64_t e = off / 8, m = len / 8;
        widen_i32_u64<<<blocks(m), 256, 0, s>>>(src + e, static_cast<uint64_t*>(d), m);
        BSM_HIP_TRY(hipGetLastError());
        return BSM_OK;
    });
}

}  // namespace bsm
