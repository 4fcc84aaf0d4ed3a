// transfer.hip -- host <-> device marshalling of the host-buffer entry points.
//
// A Rust caller of Csr::mul_dense (src/sparse.rs:426-446) hands over pageable
// Vecs: usize column indices (8 B) and k separate Dense columns
// (dense.rs:8), and takes back a fresh Csr with usize indices. Moving those
// through the driver's own pageable path, with the 8 B <-> 4 B index
// conversion as a scalar host loop, cost 7x the device time at C3 (round 2:
// 102 ms against 13.8 ms). Here every large transfer is a pipeline over two
// pinned chunk buffers: a few host threads copy chunk i+1 into one while the
// DMA engine moves chunk i out of the other, and index conversions run on the
// device (a narrowing / widening kernel per chunk), so the host only copies.
#include <algorithm>
#include <cstdlib>
#include <thread>
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
    Stage& st = stage();
    BSM_TRY(st.get(std::min(C, bytes)));
    const size_t n = (bytes + C - 1) / C;
    auto drain = [&](size_t i) -> int {  // chunk i's DMA done -> copy out of its pinned buffer
        const size_t off = i * C, len = std::min(C, bytes - off);
        BSM_HIP_TRY(hipEventSynchronize(st.ev[i & 1]));
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
