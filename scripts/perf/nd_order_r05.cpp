// nd_order.cpp -- the host analysis of solve(order="nd"): nested dissection
// by BFS level-set separators, then the symbolic factorisation of the
// separator tree (each node's front rows). See nd.hpp and DESIGN.md §4.9.
//
// The reference (src/lib.rs:11-24) factors A in its natural order; for f64 the
// north star's bar is x within 1e-6 relative, so solve may factor P A P^T
// instead: a wide elimination tree whose independent
// subtrees are the levels the multifrontal kernels run in parallel.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/bsm.h"
#include "nd.hpp"

namespace bsm {
namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// the undirected graph of A: an edge {i, j} per stored lower entry j < i
struct Graph {
    int64_t n = 0;
    int64_t band = 0;  // max i - j over the stored lower entries
    std::vector<int64_t> xadj;
    std::vector<int32_t> adj;
};

// false: a row's columns are not strictly increasing (the band path's rule)
bool build_graph(int64_t n, const int64_t* rp, const int32_t* col, Graph& g) {
    g.n = n;
    g.xadj.assign((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
            const int64_t j = col[e];
            if (e > rp[i] && col[e - 1] >= j) return false;
            if (j < i) {
                ++g.xadj[i + 1];
                ++g.xadj[j + 1];
                g.band = std::max(g.band, i - j);
            }
        }
    for (int64_t i = 0; i < n; ++i) g.xadj[i + 1] += g.xadj[i];
    g.adj.resize((size_t)g.xadj[n]);
    std::vector<int64_t> pos(g.xadj.begin(), g.xadj.end() - 1);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
            const int64_t j = col[e];
            if (j < i) {
                g.adj[pos[i]++] = (int32_t)j;
                g.adj[pos[j]++] = (int32_t)i;
            }
        }
    return true;
}

struct TNode {
    std::vector<int32_t> own;  // separator (or leaf) vertices, original indices
    int32_t kid[2] = {-1, -1};
};

// Recursive bisection. Every part carries a tag (the id of the tree node
// that receives it) in mark[]; parts are disjoint, so threads working on
// different parts share mark / lvl / seen without conflict.
struct Bisect {
    const Graph& g;
    int64_t leaf;
    std::vector<int32_t> mark, lvl, seen;
    int64_t band = 0;  // max |i - j| over the edges (natural order)
    bool band_hints = true;
    bool trace = false;
    std::deque<TNode> tree;
    std::mutex mu;
    std::atomic<int32_t> stamp{0};

    Bisect(const Graph& g_, int64_t leaf_)
        : g(g_), leaf(leaf_), mark((size_t)g_.n, 0), lvl((size_t)g_.n, 0),
          seen((size_t)g_.n, -1) {}

    int32_t new_node() {
        std::lock_guard<std::mutex> l(mu);
        tree.emplace_back();
        return (int32_t)tree.size() - 1;
    }
    TNode& node(int32_t i) {  // deque: references survive later emplace_back
        std::lock_guard<std::mutex> l(mu);
        return tree[(size_t)i];
    }

    // v itself if tagged `tag`, else a neighbour tagged `tag`, else -1 (search)
    int32_t near_in(int32_t v, int32_t tag) const {
        if (v < 0 || mark[v] == tag) return v;
        for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e)
            if (mark[g.adj[e]] == tag) return g.adj[e];
        return -1;
    }

    // BFS from s over the vertices tagged `tag`, appended to order; levels in lvl
    void bfs(int32_t s, int32_t tag, int32_t id, std::vector<int32_t>& order) {
        size_t h = order.size();
        order.push_back(s);
        seen[s] = id;
        lvl[s] = 0;
        for (; h < order.size(); ++h) {
            const int32_t v = order[h];
            const int32_t lv = lvl[v] + 1;
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e) {
                const int32_t u = g.adj[e];
                if (mark[u] == tag && seen[u] != id) {
                    seen[u] = id;
                    lvl[u] = lv;
                    order.push_back(u);
                }
            }
        }
    }

    // hint >= 0: a vertex of the part to root the level structure at (no
    // search for a far vertex); else the first BFS finds one
    struct Task {
        std::vector<int32_t> verts;
        int32_t id;
        int depth;
        int32_t hint;
    };

    // One part: a leaf, or a separator and two child parts for the pool.
    void split(Task& tk, std::vector<Task>& out) {
        std::vector<int32_t>& verts = tk.verts;
        const int32_t id = tk.id, hint = tk.hint;
        const int depth = tk.depth;
        if ((int64_t)verts.size() <= leaf) {
            node(id).own = std::move(verts);
            return;
        }
        const auto tr0 = Clock::now();
        std::vector<int32_t> order, A, B, S;
        int32_t ha = -1, hb = -1;  // the children's BFS roots (-1: search for a far vertex)
        if (depth == 0 && band > 0 && (int64_t)verts.size() >= 8 * band) {
            // a narrow band in the natural order (a mesh numbered row by row):
            // any band consecutive indices separate those below from those
            // above, so the root's cut needs no BFS (the two of a 1M-vertex
            // part are the largest serial step of the bisection)
            const int64_t n = (int64_t)verts.size(), lo = (n - band) / 2, hi = lo + band;
            for (int64_t v = 0; v < n; ++v) {
                if (v < lo) A.push_back((int32_t)v);
                else if (v >= hi) B.push_back((int32_t)v);
            }
            for (int64_t v = lo; v < hi; ++v) {
                bool beyond = false;  // a separator vertex with no neighbour above joins A
                for (int64_t e = g.xadj[v]; e < g.xadj[v + 1] && !beyond; ++e) beyond = g.adj[e] >= hi;
                (beyond ? S : A).push_back((int32_t)v);
            }
            // the halves' BFS roots: their first and last indices (a mesh's
            // far corners, where the search for a far vertex would also end
            // up), without that search's BFS
            if (band_hints) {
                ha = 0;
                hb = (int32_t)(n - 1);
            }
        } else {
        order.reserve(verts.size());
        bfs(hint >= 0 ? hint : verts[0], id, stamp++, order);
        if (order.size() < verts.size()) {
            // disconnected: whole components to the smaller side, no separator
            const int32_t sid = stamp++;
            order.clear();
            std::vector<std::pair<size_t, size_t>> comps;  // (size, first in order)
            for (int32_t v : verts)
                if (seen[v] != sid) {
                    const size_t f = order.size();
                    bfs(v, id, sid, order);
                    comps.emplace_back(order.size() - f, f);
                }
            std::stable_sort(comps.begin(), comps.end(),
                             [](const auto& x, const auto& y) { return x.first > y.first; });
            for (const auto& c : comps) {
                auto& side = A.size() <= B.size() ? A : B;
                side.insert(side.end(), order.begin() + (long)c.second, order.begin() + (long)(c.second + c.first));
            }
        } else {
            // level structure from a far vertex (the last one reached), its
            // middle level the separator
            if (hint < 0) {
                const int32_t u = order.back();
                order.clear();
                bfs(u, id, stamp++, order);
            }
            const int32_t D = lvl[order.back()];
            if (D < 2) {  // no level to cut at (a clique-like part): one dense front
                node(id).own = std::move(verts);
                return;
            }
            std::vector<int64_t> cnt((size_t)D + 1, 0);
            for (int32_t v : order) ++cnt[(size_t)lvl[v]];
            const int64_t total = (int64_t)verts.size();
            int32_t cut = D - 1;
            int64_t below = cnt[0];
            for (int32_t l = 1; l < D; ++l) {
                if (2 * below + cnt[(size_t)l] >= total) {
                    cut = l;
                    break;
                }
                below += cnt[(size_t)l];
            }
            for (int32_t v : order) {
                const int32_t l = lvl[v];
                if (l < cut) A.push_back(v);
                else if (l > cut) B.push_back(v);
                else {
                    // a separator vertex with no neighbour beyond the cut joins A
                    bool beyond = false;
                    for (int64_t e = g.xadj[v]; e < g.xadj[v + 1] && !beyond; ++e) {
                        const int32_t w = g.adj[e];
                        beyond = mark[w] == id && lvl[w] == cut + 1;
                    }
                    (beyond ? S : A).push_back(v);
                }
            }
        }
        }
        // the children's roots: the separator's first vertex reached (an end
        // of the cut, so the next cut runs across this one); without a
        // separator, a search
        if (!order.empty() && !S.empty()) ha = hb = S.front();
        if (trace && depth < 5) fprintf(stderr, "[nd bisect] depth %d part %zu: split %.2f ms\n", depth, verts.size(), ms_since(tr0));
        const int32_t ka = new_node(), kb = new_node();
        for (int32_t v : A) mark[v] = ka;
        for (int32_t v : B) mark[v] = kb;
        for (int32_t v : S) mark[v] = -1;
        {
            TNode& me = node(id);
            me.own = std::move(S);
            me.kid[0] = ka;
            me.kid[1] = kb;
        }
        if (ha >= 0) {  // a separator vertex is no longer in the parts: its neighbour there
            ha = near_in(ha, ka);
            hb = near_in(hb, kb);
        }
        out.push_back(Task{std::move(A), ka, depth + 1, ha});
        out.push_back(Task{std::move(B), kb, depth + 1, hb});
    }

    // The parts on `threads` workers sharing one LIFO queue (depth first
    // per worker; an idle worker takes the newest waiting part), so the
    // uneven subtrees of the lower levels balance: fixed subtree-per-thread
    // left the last thread 3x behind the first.
    void run_pool(Task root, int threads) {
        std::vector<Task> q;
        std::mutex qm;
        std::condition_variable cv;
        size_t pending = 1;  // queued + being split
        q.push_back(std::move(root));
        auto worker = [&] {
            std::vector<Task> kids;
            for (;;) {
                Task tk;
                {
                    std::unique_lock<std::mutex> lk(qm);
                    cv.wait(lk, [&] { return !q.empty() || pending == 0; });
                    if (q.empty()) return;  // pending == 0: done
                    tk = std::move(q.back());
                    q.pop_back();
                }
                kids.clear();
                split(tk, kids);
                // keep one child here (no queue round trip), publish the rest
                while (!kids.empty()) {
                    std::unique_lock<std::mutex> lk(qm);
                    for (size_t i = 1; i < kids.size(); ++i) q.push_back(std::move(kids[i]));
                    pending += kids.size() - 1;
                    if (kids.size() > 1) cv.notify_all();
                    lk.unlock();
                    Task next = std::move(kids[0]);
                    kids.clear();
                    split(next, kids);
                }
                std::unique_lock<std::mutex> lk(qm);
                if (--pending == 0) cv.notify_all();
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < threads; ++t) pool.emplace_back(worker);
        worker();
        for (auto& t : pool) t.join();
    }
};

}  // namespace

int nd_analyse(int64_t n, const int64_t* row_ptr, const int32_t* col, int64_t leaf, int threads, NdPlan& plan) {
    plan = NdPlan{};
    plan.n = n;
    if (n <= 0) return 0;
    if (leaf < 1) leaf = 1;
    if (threads < 1) threads = 1;
    auto t0 = Clock::now();
    Graph g;
    if (!build_graph(n, row_ptr, col, g)) return 1;
    plan.ms_graph = ms_since(t0);

    // bisection tree
    t0 = Clock::now();
    Bisect bs(g, leaf);
    const int32_t root = bs.new_node();
    {
        std::vector<int32_t> all((size_t)n);
        for (int64_t i = 0; i < n; ++i) all[(size_t)i] = (int32_t)i;
        bs.band = g.band;
        const char* bh = getenv("BSM_ND_BANDHINT");
        bs.band_hints = !(bh && atoi(bh) == 0);
        const char* tt = getenv("BSM_ND_TRACE");
        bs.trace = tt && atoi(tt) == 2;
        bs.run_pool({std::move(all), root, 0, -1}, threads);
    }

    // post-order numbering: kid 0's subtree, kid 1's, then the node's own vertices
    plan.perm.resize((size_t)n);
    plan.pinv.resize((size_t)n);
    plan.nodes.reserve(bs.tree.size());
    std::vector<int32_t> final_id(bs.tree.size(), -1);
    std::vector<std::pair<int32_t, int>> stack{{root, 0}};
    int64_t next = 0;
    while (!stack.empty()) {
        auto& [t, state] = stack.back();
        TNode& tn = bs.tree[(size_t)t];
        if (state < 2) {
            const int32_t k = tn.kid[state++];
            if (k >= 0) stack.emplace_back(k, 0);
            continue;
        }
        NdNode nd;
        std::sort(tn.own.begin(), tn.own.end());
        nd.start = next;
        for (int32_t v : tn.own) {
            plan.perm[(size_t)next] = v;
            plan.pinv[(size_t)v] = next;
            ++next;
        }
        nd.end = next;
        const int32_t me = (int32_t)plan.nodes.size();
        for (int s = 0; s < 2; ++s)
            if (tn.kid[s] >= 0) {
                const int32_t k = final_id[(size_t)tn.kid[s]];
                nd.kids[s] = k;
                plan.nodes[(size_t)k].parent = me;
                plan.nodes[(size_t)k].slot = s;
                nd.level = std::max(nd.level, plan.nodes[(size_t)k].level + 1);
            }
        final_id[(size_t)t] = me;
        plan.nodes.push_back(std::move(nd));
        stack.pop_back();
    }
    plan.ms_order = ms_since(t0);

    // symbolic: a node's front rows past its own columns are its vertices'
    // later neighbours and its children's front rows past its columns
    t0 = Clock::now();
    int32_t top = 0;
    for (const auto& nd : plan.nodes) top = std::max(top, nd.level);
    plan.n_levels = top + 1;
    std::vector<std::vector<int32_t>> by_level((size_t)plan.n_levels);
    for (int32_t i = 0; i < (int32_t)plan.nodes.size(); ++i) by_level[(size_t)plan.nodes[(size_t)i].level].push_back(i);
    auto symbolic = [&](int32_t i) {
        NdNode& nd = plan.nodes[(size_t)i];
        std::vector<int64_t> r;
        for (int64_t p = nd.start; p < nd.end; ++p) {
            const int64_t v = plan.perm[(size_t)p];
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e) {
                const int64_t q = plan.pinv[(size_t)g.adj[e]];
                if (q >= nd.end) r.push_back(q);
            }
        }
        for (int s = 0; s < 2; ++s)
            if (nd.kids[s] >= 0)
                for (int64_t q : plan.nodes[(size_t)nd.kids[s]].st)
                    if (q >= nd.end) r.push_back(q);
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        nd.st = std::move(r);
    };
    for (const auto& lv : by_level) {
        const int nt = (int)std::min<size_t>((size_t)threads, (lv.size() + 63) / 64);
        if (nt <= 1) {
            for (int32_t i : lv) symbolic(i);
            continue;
        }
        std::atomic<size_t> cursor{0};
        std::vector<std::thread> pool;
        for (int w = 0; w < nt; ++w)
            pool.emplace_back([&] {
                for (size_t c; (c = cursor.fetch_add(16)) < lv.size();)
                    for (size_t j = c; j < std::min(c + 16, lv.size()); ++j) symbolic(lv[j]);
            });
        for (auto& t : pool) t.join();
    }
    plan.ms_symbolic = ms_since(t0);
    return 0;
}

}  // namespace bsm

// ---- C-ABI: the analysis alone, on a host pattern (tests and diagnostics) ----
extern "C" int bsm_nd_analyse(uint64_t n, const uint64_t* row_ptr, const uint64_t* col_idx, uint64_t leaf,
                              int64_t* perm, int64_t* nodes, uint64_t cap, uint64_t* n_nodes, int64_t* st,
                              uint64_t st_cap, uint64_t* st_len) {
    if ((n && (!row_ptr || !col_idx)) || !n_nodes || !st_len) return BSM_ERR_INVALID;
    if (n >= ((uint64_t)1 << 31)) return BSM_ERR_UNSUPPORTED;
    const uint64_t nnz = n ? row_ptr[n] : 0;
    std::vector<int64_t> rp((size_t)n + 1);
    std::vector<int32_t> cl((size_t)nnz);
    for (uint64_t i = 0; i <= n; ++i) {
        rp[(size_t)i] = (int64_t)row_ptr[i];
        if (i && row_ptr[i] < row_ptr[i - 1]) return BSM_ERR_INVALID;
    }
    for (uint64_t e = 0; e < nnz; ++e) {
        if (col_idx[e] >= n) return BSM_ERR_INVALID;
        cl[(size_t)e] = (int32_t)col_idx[e];
    }
    bsm::NdPlan P;
    const char* te = getenv("BSM_ND_THREADS");
    if (bsm::nd_analyse((int64_t)n, rp.data(), cl.data(), (int64_t)leaf, te ? atoi(te) : 4, P) != 0)
        return BSM_ERR_UNSUPPORTED;
    *n_nodes = P.nodes.size();
    uint64_t total = 0;
    for (const auto& x : P.nodes) total += x.st.size();
    *st_len = total;
    if (perm)
        for (uint64_t i = 0; i < n; ++i) perm[i] = P.perm[(size_t)i];
    if (nodes && cap >= P.nodes.size() && st && st_cap >= total) {
        uint64_t o = 0;
        for (size_t i = 0; i < P.nodes.size(); ++i) {
            const auto& x = P.nodes[i];
            int64_t* row = nodes + 8 * i;
            row[0] = x.start;
            row[1] = x.end;
            row[2] = x.parent;
            row[3] = x.level;
            row[4] = x.slot;
            row[5] = (int64_t)x.st.size();
            row[6] = (int64_t)o;
            row[7] = 0;
            for (int64_t q : x.st) st[o++] = q;
        }
    }
    return BSM_OK;
}
