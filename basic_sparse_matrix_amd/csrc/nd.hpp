// nd.hpp -- nested-dissection analysis for solve(order="nd") (host C++).
//
// The plan of the multifrontal solve (kernels_nd.hip): a fill-reducing
// permutation from recursive graph bisection (BFS level-set separators) and
// its separator tree, each node a dense front. Pure host code: no HIP here,
// so the CPU tests drive it through bsm_nd_analyse.
#pragma once

#include <cstdint>
#include <vector>

namespace bsm {

struct NdNode {
    int64_t start = 0, end = 0;   // own columns [start, end) in the new order
    int32_t parent = -1;          // -1: a root
    int32_t level = 0;            // height: leaves 0, a parent above its highest child
    int32_t slot = 0;             // index among the parent's children (0 or 1)
    int32_t kids[2] = {-1, -1};
    std::vector<int64_t> st;      // the front's other rows: new indices >= end, ascending
};

struct NdPlan {
    int64_t n = 0;
    std::vector<int64_t> perm;    // perm[new] = old
    std::vector<int64_t> pinv;    // pinv[old] = new
    std::vector<NdNode> nodes;    // children before parents (post-order), roots last
    int32_t n_levels = 0;
    double ms_graph = 0, ms_order = 0, ms_symbolic = 0, ms_bisect = 0;  // ms_order includes ms_bisect
};

// A's pattern (row_ptr: n + 1 entries, col: row_ptr[n]); the matrix is the
// lower triangle (j <= i, as the band path reads it) mirrored, so the graph
// has an edge {i, j} for every stored j < i. leaf: largest part not split
// further; threads: worker threads for the bisection and the symbolic pass.
int nd_analyse(int64_t n, const int64_t* row_ptr, const int32_t* col, int64_t leaf, int threads, NdPlan& plan);

}  // namespace bsm
