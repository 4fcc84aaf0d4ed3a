// The host analysis of solve(order="nd") (csrc/nd_order.cpp) under
// ThreadSanitizer (built by tests/test_nd_tsan.py with -fsanitize=thread):
// 2-D grids (band-window root cut, BFS cuts), a lower-triangle-only pattern
// (the mirrored graph build), a random graph and disconnected blocks, each
// analysed with 8 threads twice and with 1 thread; the three plans must be
// identical (the result may not depend on the workers' timing).
#include <cstdio>
#include <cstdint>
#include <random>
#include <set>
#include <vector>

#include "nd.hpp"

namespace {

struct Pattern {
    int64_t n = 0;
    std::vector<int64_t> rp{0};
    std::vector<int32_t> col;
};

Pattern from_sets(const std::vector<std::set<int32_t>>& rows) {
    Pattern p;
    p.n = (int64_t)rows.size();
    for (const auto& r : rows) {
        for (int32_t c : r) p.col.push_back(c);
        p.rp.push_back((int64_t)p.col.size());
    }
    return p;
}

Pattern grid(int g, bool lower_only) {
    std::vector<std::set<int32_t>> rows((size_t)g * g);
    for (int i = 0; i < g * g; ++i) {
        const int r = i / g, c = i % g;
        rows[(size_t)i].insert(i);
        const int nb[4] = {r > 0 ? i - g : -1, c > 0 ? i - 1 : -1, c < g - 1 ? i + 1 : -1, r < g - 1 ? i + g : -1};
        for (int j : nb)
            if (j >= 0 && (!lower_only || j < i)) rows[(size_t)i].insert(j);
    }
    return from_sets(rows);
}

Pattern random_graph(int n, int deg, unsigned seed, int blocks) {
    std::mt19937 rng(seed);
    std::vector<std::set<int32_t>> rows((size_t)n);
    const int bs = n / blocks;
    for (int i = 0; i < n; ++i) rows[(size_t)i].insert(i);
    for (int b = 0; b < blocks; ++b)
        for (int e = 0; e < bs * deg; ++e) {
            const int i = b * bs + (int)(rng() % (unsigned)bs), j = b * bs + (int)(rng() % (unsigned)bs);
            rows[(size_t)i].insert(j);
            rows[(size_t)j].insert(i);
        }
    return from_sets(rows);
}

bool same(const bsm::NdPlan& a, const bsm::NdPlan& b) {
    if (a.perm != b.perm || a.nodes.size() != b.nodes.size()) return false;
    for (size_t i = 0; i < a.nodes.size(); ++i) {
        const auto &x = a.nodes[i], &y = b.nodes[i];
        if (x.start != y.start || x.end != y.end || x.parent != y.parent || x.level != y.level || x.st != y.st)
            return false;
    }
    return true;
}

}  // namespace

int main() {
    struct Case {
        const char* name;
        Pattern p;
        int64_t leaf;
    };
    std::vector<Case> cases;
    cases.push_back({"grid 300 (band root cut)", grid(300, false), 64});
    cases.push_back({"grid 120 lower only", grid(120, true), 32});
    cases.push_back({"grid 61 leaf 1", grid(61, false), 1});
    cases.push_back({"random 20000", random_graph(20000, 2, 11, 1), 100});
    cases.push_back({"3 disconnected random blocks", random_graph(9000, 2, 5, 3), 50});
    int failed = 0;
    for (auto& c : cases) {
        bsm::NdPlan a, b, s;
        const int ra = bsm::nd_analyse(c.p.n, c.p.rp.data(), c.p.col.data(), c.leaf, 8, a);
        const int rb = bsm::nd_analyse(c.p.n, c.p.rp.data(), c.p.col.data(), c.leaf, 8, b);
        const int rs = bsm::nd_analyse(c.p.n, c.p.rp.data(), c.p.col.data(), c.leaf, 1, s);
        const bool ok = ra == 0 && rb == 0 && rs == 0 && same(a, b) && same(a, s);
        printf("%s: %zu nodes, %s\n", c.name, a.nodes.size(), ok ? "same plan" : "DIFFERENT");
        failed += !ok;
    }
    printf("%d failed\n", failed);
    return failed ? 1 : 0;
}
