// Times the host analysis of solve(order="nd") (csrc/nd_order.cpp) on a g x g
// 5-point grid: ./nd_order_time G LEAF THREADS. Built by scripts/perf/build_nd_order_time.sh.
#include "nd.hpp"
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
int main(int argc, char** argv) {
    int64_t g = atoll(argv[1]), leaf = atoll(argv[2]); int th = atoi(argv[3]);
    int64_t n = g * g;
    std::vector<int64_t> rp(n + 1); std::vector<int32_t> col; col.reserve(5 * n);
    for (int64_t i = 0; i < n; ++i) {
        int64_t r = i / g, c = i % g;
        if (r > 0) col.push_back(i - g);
        if (c > 0) col.push_back(i - 1);
        col.push_back(i);
        if (c < g - 1) col.push_back(i + 1);
        if (r < g - 1) col.push_back(i + g);
        rp[i + 1] = col.size();
    }
    for (int rep = 0; rep < 2; ++rep) {
        bsm::NdPlan P;
        auto t0 = std::chrono::steady_clock::now();
        bsm::nd_analyse(n, rp.data(), col.data(), leaf, th, P);
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        double fl = 0, mem = 0; int64_t mx = 0;
        for (auto& x : P.nodes) { int64_t np = x.end - x.start, npp = (np + 63) / 64 * 64, f = npp + x.st.size(), fp = (f + 63) / 64 * 64;
            mem += 8.0 * fp * fp; mx = std::max(mx, fp);
            fl += (double)np * np * np / 3 + (double)np * np * x.st.size() + (double)np * x.st.size() * x.st.size(); }
        uint64_t h = 1469598103934665603ull;  // FNV-1a over perm and every node's (start, end, parent, st)
        auto mix = [&](int64_t x) { h = (h ^ (uint64_t)x) * 1099511628211ull; };
        for (int64_t v : P.perm) mix(v);
        for (auto& x : P.nodes) { mix(x.start); mix(x.end); mix(x.parent); for (int64_t q : x.st) mix(q); }
        printf("plan %016llx | ", (unsigned long long)h);
        printf("total %.1f ms: graph %.1f order %.1f (bisect %.1f) symbolic %.1f nodes %zu levels %d | fronts %.2f GB max %lld, true flops %.2f GF\n", ms, P.ms_graph, P.ms_order, P.ms_bisect, P.ms_symbolic, P.nodes.size(), P.n_levels, mem / 1e9, (long long)mx, fl / 1e9);
    }
}
