// nd_order.cpp -- the host analysis of solve(order="nd"): nested dissection
// by BFS level-set separators, then the symbolic factorisation of the
// separator tree (each node's front rows). See nd.hpp and DESIGN.md §4.9.
//
// The reference (src/lib.rs:11-24) factors A in its natural order; for f64 the
// north star's bar is x within 1e-6 relative, so solve may factor P A P^T
// instead: a wide elimination tree whose independent
// subtrees are the levels the multifrontal kernels run in parallel.
#include <algorithm>
#include <climits>
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

// f(lo, hi, t) over [0, n) in `threads` contiguous ranges
template <class F> void parallel_ranges(int64_t n, int threads, F&& f) {
    threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / 4096 + 1));
    if (threads == 1) {
        f((int64_t)0, n, 0);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back([&, t] { f(n * t / threads, n * (t + 1) / threads, t); });
    f((int64_t)0, n / threads, 0);
    for (auto& th : pool) th.join();
}

// false: a row's columns are not strictly increasing (the band path's rule).
// Every vertex's neighbours come out ascending. A structurally symmetric
// pattern (every lower entry's mirror stored, as many upper entries as
// lower: C5 stores the whole stencil) is the graph itself, off the
// diagonal: checked and copied row-parallel. Otherwise the lower entries are
// mirrored by a serial counting pass. Both give the same adjacency.
bool build_graph(int64_t n, const int64_t* rp, const int32_t* col, int threads, Graph& g) {
    g.n = n;
    g.xadj.assign((size_t)n + 1, 0);
    struct Acc {
        bool sorted = true, mirrored = true;
        int64_t lower = 0, upper = 0, band = 0;
        char pad[64];
    };
    std::vector<Acc> acc((size_t)std::max(threads, 1));
    parallel_ranges(n, threads, [&](int64_t lo, int64_t hi, int t) {
        Acc a;
        for (int64_t i = lo; i < hi; ++i) {
            int64_t deg = 0;
            for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
                const int64_t j = col[e];
                if (e > rp[i] && col[e - 1] >= j) a.sorted = false;
                if (j < i) {
                    ++a.lower;
                    a.band = std::max(a.band, i - j);
                    if (a.mirrored) {  // i in row j (sorted rows: a binary search)
                        const int32_t* r0 = col + rp[j];
                        const int32_t* r1 = col + rp[j + 1];
                        const int32_t* f = std::lower_bound(r0, r1, (int32_t)i);
                        a.mirrored = f != r1 && *f == i;
                    }
                } else if (j > i) {
                    ++a.upper;
                }
                deg += j != i;
            }
            g.xadj[(size_t)i + 1] = deg;
        }
        acc[(size_t)t] = a;
    });
    bool sorted = true, mirrored = true;
    int64_t lower = 0, upper = 0;
    for (const auto& a : acc) {
        sorted &= a.sorted;
        mirrored &= a.mirrored;
        lower += a.lower;
        upper += a.upper;
        g.band = std::max(g.band, a.band);
    }
    if (!sorted) return false;
    if (mirrored && lower == upper) {
        for (int64_t i = 0; i < n; ++i) g.xadj[(size_t)i + 1] += g.xadj[(size_t)i];
        g.adj.resize((size_t)g.xadj[(size_t)n]);
        parallel_ranges(n, threads, [&](int64_t lo, int64_t hi, int) {
            for (int64_t i = lo; i < hi; ++i) {
                int64_t o = g.xadj[(size_t)i];
                for (int64_t e = rp[i]; e < rp[i + 1]; ++e)
                    if (col[e] != i) g.adj[(size_t)o++] = col[e];
            }
        });
        return true;
    }
    std::fill(g.xadj.begin(), g.xadj.end(), 0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
            const int64_t j = col[e];
            if (j < i) {
                ++g.xadj[(size_t)i + 1];
                ++g.xadj[(size_t)j + 1];
            }
        }
    for (int64_t i = 0; i < n; ++i) g.xadj[(size_t)i + 1] += g.xadj[(size_t)i];
    g.adj.resize((size_t)g.xadj[(size_t)n]);
    std::vector<int64_t> pos(g.xadj.begin(), g.xadj.end() - 1);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
            const int64_t j = col[e];
            if (j < i) {
                g.adj[(size_t)pos[(size_t)i]++] = (int32_t)j;
                g.adj[(size_t)pos[(size_t)j]++] = (int32_t)i;
            }
        }
    return true;
}

struct TNode {
    std::vector<int32_t> own;  // separator (or leaf) vertices, original indices
    int32_t kid[2] = {-1, -1};
};

// A part of the graph with its own numbering: local vertex l is global
// vertex gid[l]; its neighbours in the part are J[X[l] .. X[l + 1]), local,
// in the order of the global adjacency (ascending global index). Children
// are numbered in their parent's BFS order, so the BFS of a part walks
// memory that is compact and mostly in order (on the global numbering a BFS
// through a row-major grid touches a new cache line per vertex). A part owns
// all it reads: threads share nothing but the tree.
struct Part {
    std::vector<int32_t> gid;
    std::vector<int64_t> xadj;
    std::vector<int32_t> adj;
    const int64_t* X = nullptr;
    const int32_t* J = nullptr;
    int32_t nv = 0;
};

// Recursive bisection on a pool of workers. The separators and the tree are
// those of a BFS level structure per part; the result does not depend on
// the threads' timing (the tree is numbered by its structure afterwards).
struct Bisect {
    const Graph& g;
    int64_t leaf;
    int64_t band = 0;  // max |i - j| over the edges (natural order)
    bool band_hints = true;
    bool trace = false;
    std::deque<TNode> tree;
    std::mutex mu;

    Bisect(const Graph& g_, int64_t leaf_) : g(g_), leaf(leaf_) {}

    int32_t new_node() {
        std::lock_guard<std::mutex> l(mu);
        tree.emplace_back();
        return (int32_t)tree.size() - 1;
    }
    TNode& node(int32_t i) {  // deque: references survive later emplace_back
        std::lock_guard<std::mutex> l(mu);
        return tree[(size_t)i];
    }

    // hint >= 0: a vertex of the part (local) to root the level structure at
    // (no search for a far vertex); else the first BFS finds one
    struct Task {
        Part p;
        int32_t id;
        int depth;
        int32_t hint;
    };

    // BFS from s over the part (lvl[v] == -1: not reached yet), appended to order
    static void bfs(const Part& p, int32_t s, std::vector<int32_t>& lvl, std::vector<int32_t>& order) {
        size_t h = order.size();
        order.push_back(s);
        lvl[(size_t)s] = 0;
        for (; h < order.size(); ++h) {
            const int32_t v = order[h];
            const int32_t lv = lvl[(size_t)v] + 1;
            for (int64_t e = p.X[v]; e < p.X[v + 1]; ++e) {
                const int32_t u = p.J[e];
                if (lvl[(size_t)u] < 0) {
                    lvl[(size_t)u] = lv;
                    order.push_back(u);
                }
            }
        }
    }

    // the child of `p` made of the vertices `list` (local to p, in this
    // order); to[v]: v's local index in its child, plus 2^30 on side B, -1
    // for the separator (one lookup per neighbour)
    static constexpr int32_t SIDE_B = 1 << 30;
    static void extract(const Part& p, const std::vector<int32_t>& list, const std::vector<int32_t>& to, bool b,
                        Part& c) {
        const int32_t lo = b ? SIDE_B : 0, hi = b ? INT32_MAX : SIDE_B;
        c.nv = (int32_t)list.size();
        c.gid.resize(list.size());
        c.xadj.resize(list.size() + 1);
        int64_t deg = 0;
        for (int32_t v : list) deg += p.X[v + 1] - p.X[v];
        c.adj.resize((size_t)deg);
        int32_t* out = c.adj.data();
        int64_t o = 0;
        c.xadj[0] = 0;
        for (size_t i = 0; i < list.size(); ++i) {
            const int32_t v = list[i];
            c.gid[i] = p.gid[(size_t)v];
            for (int64_t e = p.X[v]; e < p.X[v + 1]; ++e) {
                const int32_t t = to[(size_t)p.J[e]];
                if (t >= lo && t < hi) out[o++] = t - lo;
            }
            c.xadj[i + 1] = o;
        }
        c.adj.resize((size_t)o);
        c.X = c.xadj.data();
        c.J = c.adj.data();
    }

    // One part: a leaf, or a separator and two child parts for the pool.
    void split(Task& tk, std::vector<Task>& out) {
        const Part& p = tk.p;
        const int32_t id = tk.id, hint = tk.hint, nv = p.nv;
        const int depth = tk.depth;
        if ((int64_t)nv <= leaf) {
            node(id).own = std::move(tk.p.gid);
            return;
        }
        const auto tr0 = Clock::now();
        std::vector<int32_t> order, A, B, S, lvl;
        int32_t ha = -1, hb = -1;  // the children's BFS roots (-1: search for a far vertex)
        if (depth == 0 && band > 0 && (int64_t)nv >= 8 * band) {
            // a narrow band in the natural order (a mesh numbered row by row):
            // any band consecutive indices separate those below from those
            // above, so the root's cut needs no BFS (the two of a 1M-vertex
            // part are the largest serial step of the bisection). The root
            // part is the whole graph in its own numbering.
            const int64_t lo = (nv - band) / 2, hi = lo + band;
            for (int64_t v = 0; v < nv; ++v) {
                if (v < lo) A.push_back((int32_t)v);
                else if (v >= hi) B.push_back((int32_t)v);
            }
            for (int64_t v = lo; v < hi; ++v) {
                bool beyond = false;  // a separator vertex with no neighbour above joins A
                for (int64_t e = p.X[v]; e < p.X[v + 1] && !beyond; ++e) beyond = p.J[e] >= hi;
                (beyond ? S : A).push_back((int32_t)v);
            }
            // the halves' BFS roots: their first and last indices (a mesh's
            // far corners, where the search for a far vertex would also end
            // up), without that search's BFS
            if (band_hints) {
                ha = 0;
                hb = nv - 1;
            }
        } else {
            lvl.assign((size_t)nv, -1);
            order.reserve((size_t)nv);
            bfs(p, hint >= 0 ? hint : 0, lvl, order);
            if ((int32_t)order.size() < nv) {
                // disconnected: whole components to the smaller side, no separator
                std::fill(lvl.begin(), lvl.end(), -1);
                order.clear();
                std::vector<std::pair<size_t, size_t>> comps;  // (size, first in order)
                for (int32_t v = 0; v < nv; ++v)
                    if (lvl[(size_t)v] < 0) {
                        const size_t f = order.size();
                        bfs(p, v, lvl, order);
                        comps.emplace_back(order.size() - f, f);
                    }
                std::stable_sort(comps.begin(), comps.end(),
                                 [](const auto& x, const auto& y) { return x.first > y.first; });
                for (const auto& c : comps) {
                    auto& sd = A.size() <= B.size() ? A : B;
                    sd.insert(sd.end(), order.begin() + (long)c.second, order.begin() + (long)(c.second + c.first));
                }
            } else {
                // level structure from a far vertex (the last one reached), its
                // middle level the separator
                if (hint < 0) {
                    const int32_t u = order.back();
                    for (int32_t v : order) lvl[(size_t)v] = -1;
                    order.clear();
                    bfs(p, u, lvl, order);
                }
                const int32_t D = lvl[(size_t)order.back()];
                if (D < 2) {  // no level to cut at (a clique-like part): one dense front
                    node(id).own = std::move(tk.p.gid);
                    return;
                }
                std::vector<int64_t> cnt((size_t)D + 1, 0);
                for (int32_t v : order) ++cnt[(size_t)lvl[(size_t)v]];
                const int64_t total = nv;
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
                    const int32_t l = lvl[(size_t)v];
                    if (l < cut) A.push_back(v);
                    else if (l > cut) B.push_back(v);
                    else {
                        // a separator vertex with no neighbour beyond the cut joins A
                        bool beyond = false;
                        for (int64_t e = p.X[v]; e < p.X[v + 1] && !beyond; ++e)
                            beyond = lvl[(size_t)p.J[e]] == cut + 1;
                        (beyond ? S : A).push_back(v);
                    }
                }
            }
        }
        // the children's roots: the separator's first vertex reached (an end
        // of the cut, so the next cut runs across this one); without a
        // separator, a search
        if (!order.empty() && !S.empty()) ha = hb = S.front();
        if (trace && depth < 5)
            fprintf(stderr, "[nd bisect] depth %d part %d: split %.2f ms\n", depth, nv, ms_since(tr0));
        const auto tx0 = Clock::now();
        std::vector<int32_t> to((size_t)nv, -1);
        for (size_t i = 0; i < A.size(); ++i) to[(size_t)A[i]] = (int32_t)i;
        for (size_t i = 0; i < B.size(); ++i) to[(size_t)B[i]] = SIDE_B + (int32_t)i;
        auto side_of = [&](int32_t v) { return to[(size_t)v] < 0 ? 2 : to[(size_t)v] >= SIDE_B ? 1 : 0; };
        // a separator vertex is in neither part: its first neighbour (in the
        // global adjacency order) in each
        auto near_in = [&](int32_t v, int sd) -> int32_t {
            if (v < 0 || side_of(v) == sd) return v;
            for (int64_t e = p.X[v]; e < p.X[v + 1]; ++e)
                if (side_of(p.J[e]) == sd) return p.J[e];
            return -1;
        };
        if (ha >= 0) {
            ha = near_in(ha, 0);
            hb = near_in(hb, 1);
        }
        const int32_t ka = new_node(), kb = new_node();
        Task ta{Part{}, ka, depth + 1, ha >= 0 ? to[(size_t)ha] : -1};
        Task tb{Part{}, kb, depth + 1, hb >= 0 ? to[(size_t)hb] - SIDE_B : -1};
        if (nv >= (1 << 18)) {  // the largest parts: the two children's graphs side by side
            std::thread th([&] { extract(p, B, to, true, tb.p); });
            extract(p, A, to, false, ta.p);
            th.join();
        } else {
            extract(p, A, to, false, ta.p);
            extract(p, B, to, true, tb.p);
        }
        if (trace && depth < 5)
            fprintf(stderr, "[nd bisect] depth %d part %d: children %.2f ms\n", depth, nv, ms_since(tx0));
        {
            TNode& me = node(id);
            me.own.resize(S.size());
            for (size_t i = 0; i < S.size(); ++i) me.own[i] = p.gid[(size_t)S[i]];
            me.kid[0] = ka;
            me.kid[1] = kb;
        }
        out.push_back(std::move(ta));
        out.push_back(std::move(tb));
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
    if (!build_graph(n, row_ptr, col, threads, g)) return 1;
    plan.ms_graph = ms_since(t0);

    // bisection tree
    t0 = Clock::now();
    Bisect bs(g, leaf);
    const int32_t root = bs.new_node();
    {
        // the root part is the whole graph: its numbering is the global one
        Part all;
        all.nv = (int32_t)n;
        all.gid.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) all.gid[(size_t)i] = (int32_t)i;
        all.X = g.xadj.data();
        all.J = g.adj.data();
        bs.band = g.band;
        const char* bh = getenv("BSM_ND_BANDHINT");
        bs.band_hints = !(bh && atoi(bh) == 0);
        const char* tt = getenv("BSM_ND_TRACE");
        bs.trace = tt && atoi(tt) == 2;
        bs.run_pool({std::move(all), root, 0, -1}, threads);
    }
    plan.ms_bisect = ms_since(t0);

    // post-order numbering: kid 0's subtree, kid 1's, then the node's own
    // vertices. The subtrees' vertex and node counts (one pass up the tree)
    // give every node its column range and its final index, so the nodes'
    // own sorts and their perm / pinv ranges are written in parallel.
    const int32_t ntree = (int32_t)bs.tree.size();
    std::vector<int32_t> up;  // tree nodes, children before parents
    up.reserve((size_t)ntree);
    {
        std::vector<std::pair<int32_t, int>> stack{{root, 0}};
        while (!stack.empty()) {
            auto& [t, state] = stack.back();
            const TNode& tn = bs.tree[(size_t)t];
            if (state < 2) {
                const int32_t k = tn.kid[state++];
                if (k >= 0) stack.emplace_back(k, 0);
                continue;
            }
            up.push_back(t);
            stack.pop_back();
        }
    }
    std::vector<int64_t> vcount((size_t)ntree, 0), vstart((size_t)ntree, 0);
    std::vector<int32_t> ncount((size_t)ntree, 0), nstart((size_t)ntree, 0), height((size_t)ntree, 0);
    for (int32_t t : up) {
        const TNode& tn = bs.tree[(size_t)t];
        vcount[(size_t)t] = (int64_t)tn.own.size();
        ncount[(size_t)t] = 1;
        for (int s = 0; s < 2; ++s)
            if (tn.kid[s] >= 0) {
                vcount[(size_t)t] += vcount[(size_t)tn.kid[s]];
                ncount[(size_t)t] += ncount[(size_t)tn.kid[s]];
                height[(size_t)t] = std::max(height[(size_t)t], height[(size_t)tn.kid[s]] + 1);
            }
    }
    for (auto it = up.rbegin(); it != up.rend(); ++it) {  // parents before children
        const TNode& tn = bs.tree[(size_t)*it];
        int64_t v0 = vstart[(size_t)*it];
        int32_t n0 = nstart[(size_t)*it];
        for (int s = 0; s < 2; ++s)
            if (tn.kid[s] >= 0) {
                vstart[(size_t)tn.kid[s]] = v0;
                nstart[(size_t)tn.kid[s]] = n0;
                v0 += vcount[(size_t)tn.kid[s]];
                n0 += ncount[(size_t)tn.kid[s]];
            }
    }
    std::vector<int32_t> final_id((size_t)ntree);
    for (int32_t t : up) final_id[(size_t)t] = nstart[(size_t)t] + ncount[(size_t)t] - 1;
    plan.perm.resize((size_t)n);
    plan.pinv.resize((size_t)n);
    plan.nodes.resize((size_t)ntree);
    {
        std::atomic<int32_t> cursor{0};
        auto work = [&] {
            for (int32_t c; (c = cursor.fetch_add(64)) < ntree;)
                for (int32_t j = c; j < std::min(c + 64, ntree); ++j) {
                    const int32_t t = up[(size_t)j];
                    TNode& tn = bs.tree[(size_t)t];
                    std::sort(tn.own.begin(), tn.own.end());
                    NdNode& nd = plan.nodes[(size_t)final_id[(size_t)t]];
                    nd.end = vstart[(size_t)t] + vcount[(size_t)t];
                    nd.start = nd.end - (int64_t)tn.own.size();
                    nd.level = height[(size_t)t];
                    int64_t q = nd.start;
                    for (int32_t v : tn.own) {
                        plan.perm[(size_t)q] = v;
                        plan.pinv[(size_t)v] = q;
                        ++q;
                    }
                    for (int s = 0; s < 2; ++s)
                        if (tn.kid[s] >= 0) {
                            const int32_t k = final_id[(size_t)tn.kid[s]];
                            nd.kids[s] = k;
                            plan.nodes[(size_t)k].parent = final_id[(size_t)t];
                            plan.nodes[(size_t)k].slot = s;
                        }
                }
        };
        std::vector<std::thread> pool;
        const int nt = (int)std::min<int64_t>(threads, (ntree + 255) / 256);
        for (int w = 1; w < nt; ++w) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    }
    plan.ms_order = ms_since(t0);

    // symbolic: a node's front rows past its own columns are its vertices'
    // later neighbours and its children's front rows past its columns
    t0 = Clock::now();
    int32_t top = 0;
    for (const auto& nd : plan.nodes) top = std::max(top, nd.level);
    plan.n_levels = top + 1;
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
    // A node needs its children's st, nothing else: the nodes are in
    // post-order, so a subtree is one range [first, root] processed in index
    // order. Whole subtrees go to the workers (taken by a counter), the few
    // nodes above them follow in index order: no barrier per level.
    const int32_t nn = (int32_t)plan.nodes.size();
    std::vector<int32_t> depth((size_t)nn, 0), first((size_t)nn);
    for (int32_t i = nn - 1; i >= 0; --i) {
        const int32_t par = plan.nodes[(size_t)i].parent;
        depth[(size_t)i] = par < 0 ? 0 : depth[(size_t)par] + 1;
    }
    for (int32_t i = 0; i < nn; ++i) {  // the first node of i's subtree in post-order
        const NdNode& nd = plan.nodes[(size_t)i];
        first[(size_t)i] = nd.kids[0] >= 0 ? first[(size_t)nd.kids[0]] : nd.kids[1] >= 0 ? first[(size_t)nd.kids[1]] : i;
    }
    int32_t cut_depth = 0;  // the shallowest depth with enough subtrees for the workers
    for (;; ++cut_depth) {
        int32_t c = 0, deeper = 0;
        for (int32_t i = 0; i < nn; ++i) {
            c += depth[(size_t)i] == cut_depth;
            deeper += depth[(size_t)i] > cut_depth;
        }
        if (c >= 8 * threads || deeper == 0) break;
    }
    std::vector<int32_t> roots;
    for (int32_t i = 0; i < nn; ++i)
        if (depth[(size_t)i] == cut_depth) roots.push_back(i);
    {
        std::atomic<size_t> cursor{0};
        auto work = [&] {
            for (size_t c; (c = cursor.fetch_add(1)) < roots.size();)
                for (int32_t i = first[(size_t)roots[c]]; i <= roots[c]; ++i) symbolic(i);
        };
        std::vector<std::thread> pool;
        const int nt = (int)std::min<size_t>((size_t)threads, roots.size());
        for (int w = 1; w < nt; ++w) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    }
    for (int32_t i = 0; i < nn; ++i)
        if (depth[(size_t)i] < cut_depth) symbolic(i);
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
