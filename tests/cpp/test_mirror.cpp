// C++ parity tests of the host mirror (include/bsm.hpp): the reference's own
// unit tests (src/sparse.rs, src/lib.rs #[test] functions, cited per test)
// restated against bsm::Csr / bsm::Dense / bsm::solve, plus seeded parity
// against the CPU oracle (oracle/). Runs on a GPU box; tests/test_cpp_mirror.py
// builds and drives it.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "bsm.hpp"
#include "../../oracle/bsm_oracle.h"

using bsm::Csr;
using bsm::Dense;
using bsm::MatDim;
using bsm::MatErr;
using bsm::Panic;

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                                          \
    do {                                                                                     \
        ++g_checks;                                                                          \
        if (!(cond)) {                                                                       \
            ++g_fail;                                                                        \
            std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
        }                                                                                    \
    } while (0)
#define CHECK_THROWS(T, expr)                  \
    do {                                       \
        bool thrown = false;                   \
        try {                                  \
            (void)(expr);                      \
        } catch (const T&) {                   \
            thrown = true;                     \
        }                                      \
        CHECK(thrown && #T);                   \
    } while (0)

struct TestCase {
    const char* name;
    std::function<void()> fn;
    bool gpu;
};
static std::vector<TestCase>& registry() {
    static std::vector<TestCase> r;
    return r;
}
struct Reg {
    Reg(const char* n, std::function<void()> f, bool gpu) { registry().push_back({n, std::move(f), gpu}); }
};
// TEST: host logic only; GPU_TEST: runs the hot path on the device
#define TEST(name)                            \
    static void name();                       \
    static Reg reg_##name(#name, name, false); \
    static void name()
#define GPU_TEST(name)                       \
    static void name();                      \
    static Reg reg_##name(#name, name, true); \
    static void name()

template <class T>
using Rows = std::vector<std::vector<T>>;

template <class T>
static bool same_bits(const std::vector<T>& a, const std::vector<T>& b) {
    return a.size() == b.size() && (a.empty() || std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0);
}

// ------------------------------------------------ construction (sparse.rs)
TEST(example_mat_0) {  // sparse.rs:815-827
    auto m = Csr<int32_t>::from_data(Rows<int32_t>{{5, 0, 0, 0}, {0, 8, 0, 0}, {0, 0, 3, 0}, {0, 6, 0, 0}});
    CHECK((m.v() == std::vector<int32_t>{5, 8, 3, 6}));
    CHECK((m.col_index() == std::vector<size_t>{0, 1, 2, 1}));
    CHECK((m.row_index() == std::vector<size_t>{0, 1, 2, 3, 4}));
}

TEST(create_mat_by_insert) {  // sparse.rs:854-868
    auto m = Csr<int32_t>::new_({3, 3});
    m.insert(5, 0, 0).unwrap();
    m.insert(6, 0, 1).unwrap();
    m.insert(7, 0, 2).unwrap();
    auto f = std::move(m).finalise();
    CHECK(f == Csr<int32_t>::from_data(Rows<int32_t>{{5, 6, 7}, {0, 0, 0}, {0, 0, 0}}));
    CHECK(f.insert(1, 2, 2) == MatErr::MatrixFinalised);  // sparse.rs:223-225
}

TEST(finalise_big_eek) {  // sparse.rs:209-211
    auto m = Csr<int32_t>::new_({1, 3});
    m.insert(1, 0, 0).unwrap();
    m.insert(2, 2, 0).unwrap();  // registers rows 1 and 2 of a 1-row matrix
    CHECK_THROWS(Panic, std::move(m).finalise());
}

TEST(get_row_by_index_0) {  // sparse.rs:870-886
    auto m = Csr<int32_t>::from_data(
        Rows<int32_t>{{10, 20, 0, 0, 0, 0}, {0, 30, 0, 40, 0, 0}, {0, 0, 50, 60, 70, 0}, {0, 0, 0, 0, 0, 80}});
    CHECK((*m.get_row_complete(2) == std::vector<int32_t>{0, 0, 50, 60, 70, 0}));
    auto c = m.get_row_compact(2);
    CHECK(c.size() == 3 && *c[0].v == 50 && c[0].col_index == 2 && *c[2].v == 70 && c[2].col_index == 4);
}

TEST(csr_with_empty_rows) {  // sparse.rs:1111-1151
    auto top = Csr<int32_t>::from_data(Rows<int32_t>{{0, 0, 0}, {11, 12, 13}, {0, 0, 0}});
    CHECK((top.row_index() == std::vector<size_t>{0, 0, 3, 3}));
    auto mid = Csr<int32_t>::from_data(Rows<int32_t>{
        {8, 0, 2, 0, 0}, {0, 0, 5, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 7, 1, 2}, {0, 0, 0, 0, 0}, {0, 0, 0, 9, 0}});
    CHECK((mid.v() == std::vector<int32_t>{8, 2, 5, 7, 1, 2, 9}));
    CHECK((mid.col_index() == std::vector<size_t>{0, 2, 2, 2, 3, 4, 3}));
    CHECK((mid.row_index() == std::vector<size_t>{0, 2, 3, 3, 3, 6, 6, 7}));
}

TEST(test_iterator) {  // sparse.rs:1384-1398
    auto m = Csr<int32_t>::from_data(Rows<int32_t>{{5, 0, 0, 0}, {0, 8, 0, 0}, {0, 0, 3, 0}, {0, 6, 0, 0}});
    const int want[4][3] = {{5, 0, 0}, {8, 1, 1}, {3, 2, 2}, {6, 3, 1}};
    for (auto& w : want) {
        auto e = m.next();
        CHECK(e && *e->v == w[0] && e->row_index == (size_t)w[1] && e->col_index == (size_t)w[2]);
    }
    CHECK(!m.next());
}

TEST(create_diagonal) {  // sparse.rs:1473-1499
    CHECK(Csr<int32_t>::create_diagonal({1, 2, 3, 4}) ==
          Csr<int32_t>::from_data(Rows<int32_t>{{1, 0, 0, 0}, {0, 2, 0, 0}, {0, 0, 3, 0}, {0, 0, 0, 4}}));
    auto d = Csr<int32_t>::create_diagonal({0, 1, 0, 2, 0, 3, 0});
    CHECK(d.get_nnz() == 3);
}

// ------------------------------------------------------- hot path (GPU)
GPU_TEST(transpose_nxn) {  // sparse.rs:976-995
    auto m = Csr<int32_t>::from_data(
        Rows<int32_t>{{10, 5, 7, 9, 2}, {10, 8, 5, 9, 3}, {0, 5, 4, 6, 2}, {1, 2, 7, 9, 2}});
    CHECK(m.transpose() == Csr<int32_t>::from_data(Rows<int32_t>{
                               {10, 10, 0, 1}, {5, 8, 5, 2}, {7, 5, 4, 7}, {9, 9, 6, 9}, {2, 3, 2, 2}}));
}

GPU_TEST(transpose_mxn) {  // sparse.rs:997-1017
    auto m = Csr<int32_t>::from_data(
        Rows<int32_t>{{10, 20, 0, 0, 0, 0}, {0, 30, 0, 40, 0, 0}, {0, 0, 50, 60, 70, 0}, {0, 0, 0, 0, 0, 80}});
    CHECK(m.transpose() == Csr<int32_t>::from_data(Rows<int32_t>{
                               {10, 0, 0, 0}, {20, 30, 0, 0}, {0, 0, 50, 0}, {0, 40, 60, 0}, {0, 0, 70, 0}, {0, 0, 0, 80}}));
}

GPU_TEST(test_dense_mul) {  // sparse.rs:1082-1109
    auto d = Dense<int32_t>::from_data({{1, 2, 3, 4}, {5, 6, 7, 8}, {9, 10, 11, 12}});
    auto s = Csr<int32_t>::from_data(Rows<int32_t>{{3, 0, 2, 0}, {7, 0, 0, 0}, {0, 2, 0, 1}, {0, 0, 1, 0}, {1, 0, 0, 0}});
    CHECK(s.mul_dense(d).unwrap() ==
          Csr<int32_t>::from_data(Rows<int32_t>{{9, 29, 49}, {7, 35, 63}, {8, 20, 32}, {3, 7, 11}, {1, 5, 9}}));
    auto ds = bsm::DenseS<int32_t, 4, 3>::from_data({{1, 2, 3, 4}, {5, 6, 7, 8}, {9, 10, 11, 12}});
    CHECK(s.mul_dense_s(ds).unwrap() == s.mul_dense(d).unwrap());
    CHECK(s.mul_dense(Dense<int32_t>::from_data({{1, 2, 3}})) == MatErr::IncorrectDimensions);
}

GPU_TEST(test_nnz) {  // sparse.rs:1153-1178
    auto s = Csr<int32_t>::from_data(Rows<int32_t>{{5, 2, 1, 3}, {7, 0, 1, 3}, {0, 1, 0, 0}, {0, 7, 4, 0}});
    auto out = s.mul_dense(Dense<int32_t>::from_data({{1, 0, 3, 4}, {8, 0, 0, 5}})).unwrap();
    CHECK(out == Csr<int32_t>::from_data(Rows<int32_t>{{20, 55}, {22, 71}, {0, 0}, {12, 0}}));
    CHECK(out.get_nnz() == 5);
}

GPU_TEST(test_mul_vector) {  // sparse.rs:1501-1529
    std::vector<int32_t> v{0, 1, 2, 3, 4}, out(5);
    auto z = Csr<int32_t>::from_data(Rows<int32_t>{{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}});
    CHECK(z.mul_vector(v, out) == MatErr::IncorrectDimensions);
    auto eye = Csr<int32_t>::eye({5, 5}, 1).unwrap();
    eye.mul_vector(v, out).unwrap();
    CHECK(out == v);
    std::vector<int32_t> o2(2);
    Csr<int32_t>::from_data(Rows<int32_t>{{1, 0, 2, 0, 3}, {0, 1, 0, 2, 0}}).mul_vector(v, o2).unwrap();
    CHECK((o2 == std::vector<int32_t>{16, 7}));
}

GPU_TEST(cholesky_decomposition_0) {  // sparse.rs:1030-1060
    auto a = Csr<float>::from_data(Rows<float>{{4.0f, 12.0f, -16.0f}, {12.0f, 37.0f, -43.0f}, {-16.0f, -43.0f, 98.0f}});
    auto l = a.cholesky_decomp().unwrap();
    CHECK(l == Csr<float>::from_data(Rows<float>{{2.0f, 0.0f, 0.0f}, {6.0f, 1.0f, 0.0f}, {-8.0f, 5.0f, 3.0f}}));
    CHECK(l.transpose() ==
          Csr<float>::from_data(Rows<float>{{2.0f, 6.0f, -8.0f}, {0.0f, 1.0f, 5.0f}, {0.0f, 0.0f, 3.0f}}));
}

GPU_TEST(cholesky_decomposition_1) {  // sparse.rs:1062-1080
    auto a = Csr<float>::from_data(
        Rows<float>{{8.0f, 0, 0, 0}, {0, 7.0f, 1.0f, 0}, {0, 1.0f, 3.0f, 0}, {0, 0, 0, 2.0f}});
    CHECK(a.cholesky_decomp().unwrap() ==
          Csr<float>::from_data(Rows<float>{{2.828427f, 0, 0, 0},
                                            {0, 2.6457512f, 0, 0},
                                            {0, 0.37796451f, 1.6903086f, 0},
                                            {0, 0, 0, 1.4142135f}}));
    CHECK(Csr<float>::from_data(Rows<float>{{1, 2, 3}}).cholesky_decomp() == MatErr::NonSquareMatrix);
}

GPU_TEST(forward_substitution_test_0) {  // lib.rs:73-94
    auto l = Csr<float>::from_data(Rows<float>{{5.0f, 0, 0}, {8.0f, 2.0f, 0}, {3.0f, 7.0f, 1.0f}});
    auto y = bsm::forward_substitution(l, Dense<float>::from_data({{7.0f, 3.0f, 1.0f}}));
    CHECK(y == Dense<float>::from_data({{7.0f / 5.0f, -4.1f, 25.5f}}));
}

GPU_TEST(backward_substitution_test_0) {  // lib.rs:96-117
    auto u = Csr<float>::from_data(Rows<float>{{7.0f, 1.0f, 8.0f}, {0, 2.0f, 3.0f}, {0, 0, 5.0f}});
    auto x = bsm::backward_substitution(u, Dense<float>::from_data({{1.0f, 7.0f, 3.0f}}));
    CHECK(x == Dense<float>::from_data({{-32.0f / 35.0f, 2.6f, 0.6f}}));
}

GPU_TEST(solve_test) {  // lib.rs:119-138
    auto a = Csr<float>::from_data(
        Rows<float>{{8.0f, 0, 0, 0}, {0, 7.0f, 1.0f, 0}, {0, 1.0f, 3.0f, 0}, {0, 0, 0, 2.0f}});
    auto x = bsm::solve(a, Dense<float>::from_data({{5.0f, 2.0f, 8.0f, 1.0f}}));
    CHECK(x == Dense<float>::from_data({{0.625f, -0.1f, 2.6999998f, 0.5f}}));
    CHECK_THROWS(Panic, bsm::solve(Csr<float>::from_data(Rows<float>{{1, 2}}), Dense<float>::from_data({{1.0f}})));
}

// ------------------------------------------- seeded parity vs the oracle
GPU_TEST(add_sparse) {  // sparse.rs:1181-1207
    auto a = Csr<int32_t>::from_data(Rows<int32_t>{{5, 6, 7, 8, 9}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 1}, {1, 0, 0, 0, 0}});
    auto b = Csr<int32_t>::from_data(Rows<int32_t>{{9, 8, 7, 6, 5}, {0, 0, 0, 0, 0}, {1, 0, 0, 0, 0}, {1, 0, 0, 0, 0}});
    CHECK(a.add_sparse(b).unwrap() == Csr<int32_t>::from_data(Rows<int32_t>{
                                          {14, 14, 14, 14, 14}, {0, 0, 0, 0, 0}, {1, 0, 0, 0, 1}, {2, 0, 0, 0, 0}}));
    CHECK(a.add_sparse(Csr<int32_t>::from_data(Rows<int32_t>{{1}})) == MatErr::IncorrectDimensions);
}

GPU_TEST(sub_sparse) {  // sparse.rs:1210-1236
    auto a = Csr<int32_t>::from_data(Rows<int32_t>{{5, 6, 7, 8, 9}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 1}, {1, 0, 0, 0, 0}});
    auto b = Csr<int32_t>::from_data(Rows<int32_t>{{9, 8, 7, 6, 5}, {0, 0, 0, 0, 0}, {1, 0, 0, 0, 0}, {1, 0, 0, 0, 0}});
    CHECK(a.sub_sparse(b).unwrap() == Csr<int32_t>::from_data(Rows<int32_t>{
                                          {-4, -2, 0, 2, 4}, {0, 0, 0, 0, 0}, {-1, 0, 0, 0, 1}, {0, 0, 0, 0, 0}}));
}

GPU_TEST(sparse_multiplication) {  // sparse.rs:1284-1301 (round 3)
    auto a = Csr<int32_t>::from_data(Rows<int32_t>{{0}, {1}, {1}});
    auto b = a.transpose();
    CHECK(a.mul_sparse(b).unwrap() == Csr<int32_t>::from_data(Rows<int32_t>{{0, 0, 0}, {0, 1, 1}, {0, 1, 1}}));
}

GPU_TEST(coo_to_csr) {  // sparse.rs:1443-1468
    auto coo = bsm::COO<double>::with_capacity({5, 6}, 8);
    const std::vector<bsm::COOEntry<double>> es = {{0, 0, 1.0}, {1, 1, 2.0}, {1, 2, 3.0}, {2, 2, 4.0}, {2, 3, 5.0},
                                                   {3, 3, 6.0}, {3, 4, 7.0}, {4, 4, 8.0}, {4, 5, 9.0}};
    for (auto e : es) coo.insert(e).unwrap();
    CHECK(Csr<double>::from(coo) == Csr<double>::from_data(Rows<double>{{1.0, 0.0, 0.0, 0.0, 0.0, 0.0},
                                                                        {0.0, 2.0, 3.0, 0.0, 0.0, 0.0},
                                                                        {0.0, 0.0, 4.0, 5.0, 0.0, 0.0},
                                                                        {0.0, 0.0, 0.0, 6.0, 7.0, 0.0},
                                                                        {0.0, 0.0, 0.0, 0.0, 8.0, 9.0}}));
    CHECK(coo.insert({5, 0, 1.0}) == MatErr::OutOfBounds);
}

GPU_TEST(mul_dense_f64_k32_vs_oracle) {
    const uint64_t rows = 1500, cols = 700, k = 32;
    std::vector<uint64_t> rp(rows + 1);
    orc_gen_row_ptr(7, rows, cols, /*UNIFORM*/ 1, 0, 90, rp.data());
    const uint64_t nnz = rp[rows];
    std::vector<uint64_t> ci(nnz);
    std::vector<double> v(nnz);
    orc_gen_entries(7, 0, rows, cols, rp.data(), /*UNIFORM*/ 0, ci.data(), v.data());
    std::vector<double> x(cols * k);
    orc_gen_x_colmajor(8, cols, k, 0, x.data());
    auto a = Csr<double>::from_csr_arrays({rows, cols}, {rp.begin(), rp.end()}, {ci.begin(), ci.end()}, v);
    std::vector<std::vector<double>> xc(k);
    for (uint64_t j = 0; j < k; ++j) xc[j].assign(x.begin() + j * cols, x.begin() + (j + 1) * cols);
    auto y = a.mul_dense(Dense<double>::from_data(xc)).unwrap();
    std::vector<uint64_t> er(rows + 1), ec(rows * k);
    std::vector<double> ev(rows * k);
    uint64_t enz = 0;
    CHECK(orc_mul_dense_f64(rows, cols, rp.data(), rows + 1, ci.data(), v.data(), nnz, k, cols, x.data(), cols,
                            er.data(), ec.data(), ev.data(), &enz) == ORC_OK);
    ev.resize(enz);
    ec.resize(enz);
    CHECK((y.row_index() == std::vector<size_t>(er.begin(), er.end())));
    CHECK((y.col_index() == std::vector<size_t>(ec.begin(), ec.end())));
    CHECK(same_bits(y.v(), ev));
}

GPU_TEST(mul_dense_u32_wrapping_vs_oracle) {  // bench type, overflow-checks=false (Cargo.toml:18)
    const uint64_t rows = 300, cols = 400, k = 3;
    std::vector<uint64_t> rp(rows + 1);
    orc_gen_row_ptr(11, rows, cols, 1, 1, 60, rp.data());
    const uint64_t nnz = rp[rows];
    std::vector<uint64_t> ci(nnz);
    std::vector<double> vd(nnz);
    orc_gen_entries(11, 0, rows, cols, rp.data(), 0, ci.data(), vd.data());
    std::vector<uint32_t> v(nnz);
    for (uint64_t i = 0; i < nnz; ++i) v[i] = 0xF0000000u + (uint32_t)(vd[i] * 1e6);
    std::vector<uint32_t> x(cols * k);
    for (uint64_t i = 0; i < x.size(); ++i) x[i] = (uint32_t)(i * 2654435761u);
    auto a = Csr<uint32_t>::from_csr_arrays({rows, cols}, {rp.begin(), rp.end()}, {ci.begin(), ci.end()}, v);
    std::vector<std::vector<uint32_t>> xc(k);
    for (uint64_t j = 0; j < k; ++j) xc[j].assign(x.begin() + j * cols, x.begin() + (j + 1) * cols);
    auto y = a.mul_dense(Dense<uint32_t>::from_data(xc)).unwrap();
    std::vector<uint64_t> er(rows + 1), ec(rows * k);
    std::vector<uint32_t> ev(rows * k);
    uint64_t enz = 0;
    CHECK(orc_mul_dense_u32(rows, cols, rp.data(), rows + 1, ci.data(), v.data(), nnz, k, cols, x.data(), cols,
                            er.data(), ec.data(), ev.data(), &enz) == ORC_OK);
    ev.resize(enz);
    CHECK(same_bits(y.v(), ev));
    CHECK((y.row_index() == std::vector<size_t>(er.begin(), er.end())));
}

// north_star's multi-GPU path through the C-ABI (bsm_multi_*, bsm_mcsr_*):
// RCCL on the visible GPU(s), bit-identical to the oracle and to one GPU
GPU_TEST(mul_dense_multi_gpu_rccl_vs_oracle) {
    const uint64_t rows = 2500, cols = 900, k = 32;
    std::vector<uint64_t> rp(rows + 1);
    orc_gen_row_ptr(21, rows, cols, /*UNIFORM*/ 1, 0, 60, rp.data());
    const uint64_t nnz = rp[rows];
    std::vector<uint64_t> ci(nnz);
    std::vector<double> v(nnz);
    orc_gen_entries(21, 0, rows, cols, rp.data(), 0, ci.data(), v.data());
    std::vector<double> x(cols * k);
    orc_gen_x_colmajor(22, cols, k, 0, x.data());
    std::vector<uint64_t> er(rows + 1), ec(rows * k);
    std::vector<double> ev(rows * k);
    uint64_t enz = 0;
    CHECK(orc_mul_dense_f64(rows, cols, rp.data(), rows + 1, ci.data(), v.data(), nnz, k, cols, x.data(), cols,
                            er.data(), ec.data(), ev.data(), &enz) == ORC_OK);
    ev.resize(enz);
    ec.resize(enz);
    // the raw C-ABI, as a Rust binding calls it
    bsm_multi* ctx = nullptr;
    CHECK(bsm_multi_create(1, nullptr, &ctx) == BSM_OK);
    bsm_mcsr* m = nullptr;
    CHECK(bsm_mcsr_upload(ctx, BSM_F64, rows, cols, nnz, rp.data(), ci.data(), v.data(), 3, &m) == BSM_OK);
    std::vector<const void*> xc(k);
    for (uint64_t j = 0; j < k; ++j) xc[j] = x.data() + j * cols;
    bsm_csr* out = nullptr;
    CHECK(bsm_mcsr_mul_dense(m, k, cols, xc.data(), &out) == BSM_OK);
    uint64_t orows = 0, ocols = 0, onnz = 0;
    int dt = -1;
    CHECK(bsm_csr_shape(out, &orows, &ocols, &onnz, &dt) == BSM_OK);
    CHECK(orows == rows && ocols == k && onnz == enz && dt == BSM_F64);
    std::vector<uint64_t> gr(rows + 1), gc(onnz);
    std::vector<double> gv(onnz);
    CHECK(bsm_csr_download(out, gr.data(), gc.data(), gv.data()) == BSM_OK);
    CHECK(gr == er && gc == ec && same_bits(gv, ev));
    CHECK(bsm_mcsr_mul_dense(m, k, cols - 1, xc.data(), &out) == BSM_ERR_DIMENSIONS);
    bsm_csr_free(out);
    bsm_mcsr_free(m);
    bsm_multi_destroy(ctx);
    // the mirror's mul_dense routed over the context (bsm::set_gpus)
    auto a = Csr<double>::from_csr_arrays({rows, cols}, {rp.begin(), rp.end()}, {ci.begin(), ci.end()}, v);
    std::vector<std::vector<double>> xcols(k);
    for (uint64_t j = 0; j < k; ++j) xcols[j].assign(x.begin() + j * cols, x.begin() + (j + 1) * cols);
    bsm::set_gpus(1, 4);
    auto y = a.mul_dense(Dense<double>::from_data(xcols)).unwrap();
    auto y2 = a.mul_dense(Dense<double>::from_data(xcols)).unwrap();  // the cached partition
    bsm::set_gpus(0);
    CHECK((y.row_index() == std::vector<size_t>(er.begin(), er.end())));
    CHECK((y.col_index() == std::vector<size_t>(ec.begin(), ec.end())));
    CHECK(same_bits(y.v(), ev) && same_bits(y2.v(), ev));
    CHECK(a.mul_dense(Dense<double>::new_default_with_dims(k, cols - 1)) == MatErr::IncorrectDimensions);
}

GPU_TEST(solve_poisson_f64_vs_band_oracle) {
    const uint64_t g = 24, n = g * g;
    std::vector<uint64_t> rp(n + 1), ci(5 * n);
    std::vector<double> v(5 * n);
    const uint64_t nnz = orc_gen_poisson2d(g, rp.data(), ci.data(), v.data());
    ci.resize(nnz);
    v.resize(nnz);
    std::vector<double> b(n);
    orc_gen_x_colmajor(1002, n, 1, 0, b.data());
    auto a = Csr<double>::from_csr_arrays({n, n}, {rp.begin(), rp.end()}, {ci.begin(), ci.end()}, v);
    auto x = bsm::solve(a, Dense<double>::from_data({b}));
    std::vector<double> ex(n);
    CHECK(orc_solve_f64(n, rp.data(), ci.data(), v.data(), 1, b.data(), n, ex.data(), n, 1) == ORC_OK);
    std::vector<double> got(x.get_col(0).begin(), x.get_col(0).end());
    CHECK(same_bits(got, ex));
    // the reassociated solve: within the f64 tolerance of the reference order
    auto xb = bsm::solve_blocked(a, Dense<double>::from_data({b}));
    double num = 0, den = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const double e = xb.get_col(0)[i] - ex[i];
        num += e * e;
        den += ex[i] * ex[i];
    }
    CHECK(std::sqrt(num / den) < 1e-10);
    // the nested-dissection solve: the same tolerance
    auto xn = bsm::solve_nd(a, Dense<double>::from_data({b}));
    num = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const double e = xn.get_col(0)[i] - ex[i];
        num += e * e;
    }
    CHECK(std::sqrt(num / den) < 1e-10);
}

int main(int argc, char** argv) {
    // --host: only the host-logic tests (no device needed);
    // --expect-no-device: every GPU test must fail with bsm::DeviceError
    const bool host_only = argc > 1 && std::strcmp(argv[1], "--host") == 0;
    const bool no_dev = argc > 1 && std::strcmp(argv[1], "--expect-no-device") == 0;
    int n_fail_tests = 0;
    for (auto& t : registry()) {
        if (host_only && t.gpu) continue;
        if (no_dev) {
            if (!t.gpu) continue;
            bool dev_err = false;
            try {
                t.fn();
            } catch (const bsm::DeviceError&) {
                dev_err = true;
            } catch (...) {
            }
            n_fail_tests += !dev_err;
            std::printf("%s %s (DeviceError without a GPU: no CPU fallback)\n", dev_err ? "PASS" : "FAIL", t.name);
            continue;
        }
        const int before = g_fail;
        try {
            t.fn();
        } catch (const std::exception& e) {
            ++g_fail;
            std::fprintf(stderr, "  EXCEPTION in %s: %s\n", t.name, e.what());
        }
        const bool ok = g_fail == before;
        n_fail_tests += !ok;
        std::printf("%s %s\n", ok ? "PASS" : "FAIL", t.name);
    }
    std::printf("summary: %zu tests, %d failed, %d checks\n", registry().size(), n_fail_tests, g_checks);
    return n_fail_tests ? 1 : 0;
}
