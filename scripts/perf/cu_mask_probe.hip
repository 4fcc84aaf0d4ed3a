// Which CUs a CU-masked stream (hipExtStreamCreateWithCUMask) runs on, by
// XCD: bit i of the mask -> ? Launches 512 one-wave blocks on a stream whose
// mask keeps only bits [lo, lo + n), records each block's XCC_ID and HW_ID, and
// prints the distinct (xcc, se, cu) triples seen. Two masks: bits 0..7 and
// bits {0, 32, 64, ..., 224}. hipcc --offload-arch=gfx950 -O2 cu_mask_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void who(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
        // stay a little so the blocks spread over the CUs the mask allows
        for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(2);
    }
}

static void probe(const char* name, const std::vector<unsigned>& mask) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: stream creation failed\n", name);
        return;
    }
    std::vector<unsigned> got(8);
    (void)hipExtStreamGetCUMask(s, 8, got.data());
    const int nb = 512;
    unsigned* d = nullptr;
    (void)hipMalloc(&d, nb * 2 * sizeof(unsigned));
    who<<<nb, 64, 0, s>>>(d);
    std::vector<unsigned> h(nb * 2);
    (void)hipMemcpyAsync(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> seen;
    for (int b = 0; b < nb; ++b) {
        const unsigned xcc = h[2 * b] & 0xf, hw = h[2 * b + 1];
        seen.insert({xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xf});
    }
    printf("%s: mask read back %08x %08x %08x %08x %08x %08x %08x %08x; %zu distinct (xcc, se, sh, cu):", name, got[0],
           got[1], got[2], got[3], got[4], got[5], got[6], got[7], seen.size());
    for (auto& t : seen) printf(" (%u,%u,%u,%u)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
    printf("\n");
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", cus);
    std::vector<unsigned> m(8, 0);
    m[0] = 0xffu;  // bits 0..7
    probe("bits 0-7", m);
    std::fill(m.begin(), m.end(), 1u);  // bit 0 of every word: 0, 32, ..., 224
    probe("bits 0,32,...,224", m);
    std::fill(m.begin(), m.end(), 0xffffffffu);
    m[0] = 0xffffff00u;  // all but bits 0..7
    probe("all but bits 0-7", m);
    return 0;
}
