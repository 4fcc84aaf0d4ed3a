// bsm.hpp -- C++20 host mirror of the reference crate's API
// (jamieapps101/Basic_Sparse_Matrix, src/{sparse,dense,dense_static,util,lib}.rs)
// on top of the C-ABI in bsm.h. Header only; link with -lbsm_hip.
//
// The reference is compiled (Rust) code, so its host side is mirrored in a
// compiled language: same type and method names (`new` -> `new_`, a C++
// keyword), the same argument meaning (Dense::new_default_with_dims takes
// COLUMNS first; Csr::from_data takes ROWS, Dense::from_data COLUMNS) and the
// same error behaviour:
//   * Rust `Result<_, MatErr>`  -> bsm::Result<_> holding a value or a MatErr;
//     `unwrap()` on an Err throws bsm::Panic, as Rust's unwrap panics;
//   * Rust `panic!` (index out of bounds, "big eek", unwrap in solve) ->
//     throws bsm::Panic;
//   * device failures (no GPU, HIP error, out of memory) -> throws
//     bsm::DeviceError. There is no CPU fallback on the hot path.
// Construction and accessors are host logic with the reference's exact
// semantics; mul_dense / mul_dense_s / mul_vector / transpose /
// cholesky_decomp / solve run on the GPU (bit-exact with the reference's
// operation order). A finalised Csr is immutable
// (sparse.rs:223-225), so its device copy is uploaded once and cached; the
// cache is not part of operator== (the derived PartialEq of sparse.rs:68-78).
#ifndef BSM_HPP
#define BSM_HPP

#include <algorithm>
#include <array>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <optional>
#include <span>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <variant>
#include <vector>

#include "bsm.h"

namespace bsm {

// ---------------------------------------------------------------- util.rs
/// util.rs:11-34. `MatDim{rows, cols}`; `From<(usize,usize)>` is (rows, cols).
struct MatDim {
    size_t rows = 0, cols = 0;
    MatDim() = default;
    MatDim(size_t r, size_t c) : rows(r), cols(c) {}
    MatDim transpose() const { return {cols, rows}; }
    bool operator==(const MatDim&) const = default;
};

/// util.rs:47-55.
enum class MatErr {
    MatrixFinalised,
    MatrixNotFinalised,
    NonSquareMatrix,
    IncorrectDimensions,
    PaddingSizeSmallerThanOriginal,
    OutOfBounds,
};

inline const char* to_string(MatErr e) {
    switch (e) {
        case MatErr::MatrixFinalised: return "MatrixFinalised";
        case MatErr::MatrixNotFinalised: return "MatrixNotFinalised";
        case MatErr::NonSquareMatrix: return "NonSquareMatrix";
        case MatErr::IncorrectDimensions: return "IncorrectDimensions";
        case MatErr::PaddingSizeSmallerThanOriginal: return "PaddingSizeSmallerThanOriginal";
        case MatErr::OutOfBounds: return "OutOfBounds";
    }
    return "?";
}

/// The reference would `panic!` here.
struct Panic : std::runtime_error {
    using std::runtime_error::runtime_error;
};

/// A device-side failure (no GPU, HIP error, allocation failure): the
/// reference has no such error (MatErr has no device variant).
struct DeviceError : std::runtime_error {
    int code;
    DeviceError(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};

/// `Result<T, MatErr>`.
template <class T>
class Result {
public:
    Result(T v) : v_(std::move(v)) {}
    Result(MatErr e) : v_(e) {}
    bool is_ok() const { return v_.index() == 0; }
    bool is_err() const { return !is_ok(); }
    T& unwrap() & {
        check();
        return std::get<0>(v_);
    }
    T unwrap() && {
        check();
        return std::move(std::get<0>(v_));
    }
    MatErr unwrap_err() const {
        if (is_ok()) throw Panic("called `Result::unwrap_err()` on an `Ok` value");
        return std::get<1>(v_);
    }
    bool operator==(MatErr e) const { return is_err() && std::get<1>(v_) == e; }

private:
    void check() const {
        if (is_err())
            throw Panic(std::string("called `Result::unwrap()` on an `Err` value: ") + to_string(std::get<1>(v_)));
    }
    std::variant<T, MatErr> v_;
};

template <>
class Result<void> {
public:
    Result() = default;
    Result(MatErr e) : e_(e) {}
    bool is_ok() const { return !e_; }
    bool is_err() const { return e_.has_value(); }
    void unwrap() const {
        if (e_) throw Panic(std::string("called `Result::unwrap()` on an `Err` value: ") + to_string(*e_));
    }
    MatErr unwrap_err() const {
        if (!e_) throw Panic("called `Result::unwrap_err()` on an `Ok` value");
        return *e_;
    }
    bool operator==(MatErr e) const { return e_ && *e_ == e; }

private:
    std::optional<MatErr> e_;
};

namespace detail {
template <class T> struct dtype_of;
template <> struct dtype_of<double> { static constexpr int value = BSM_F64; };
template <> struct dtype_of<float> { static constexpr int value = BSM_F32; };
template <> struct dtype_of<int32_t> { static constexpr int value = BSM_I32; };
template <> struct dtype_of<uint32_t> { static constexpr int value = BSM_U32; };
template <> struct dtype_of<int64_t> { static constexpr int value = BSM_I64; };
template <> struct dtype_of<uint64_t> { static constexpr int value = BSM_U64; };

template <class T>
concept GpuScalar = requires { dtype_of<T>::value; };

struct HandleFree {
    void operator()(bsm_csr* p) const { bsm_csr_free(p); }
};
using Handle = std::shared_ptr<bsm_csr>;

/// Map a C-ABI status: OK, or an Err the caller returns, or a throw.
inline std::optional<MatErr> status(int rc) {
    switch (rc) {
        case BSM_OK: return std::nullopt;
        case BSM_ERR_DIMENSIONS: return MatErr::IncorrectDimensions;
        case BSM_ERR_NON_SQUARE: return MatErr::NonSquareMatrix;
        case BSM_ERR_OUT_OF_BOUNDS: return MatErr::OutOfBounds;
        case BSM_ERR_PANIC: throw Panic(bsm_last_error());
        default: throw DeviceError(rc, bsm_last_error());
    }
}
inline void check(int rc) {
    if (auto e = status(rc)) throw Panic(std::string("unexpected ") + to_string(*e) + ": " + bsm_last_error());
}

// The process-wide multi-GPU context of mul_dense (the Rust binding's
// OnceLock): gpus = 0 is the single-GPU path.
struct MultiState {
    std::mutex mu;
    bool init = false;
    int gpus = 0;
    uint32_t chunks = 1;
    std::shared_ptr<bsm_multi> ctx;
};
inline MultiState& multi_state() {
    static MultiState st;
    return st;
}
inline void multi_env(MultiState& st) {  // BSM_N_GPUS / BSM_CHUNKS, read once
    if (st.init) return;
    st.init = true;
    if (const char* e = std::getenv("BSM_N_GPUS")) st.gpus = std::atoi(e);
    if (const char* e = std::getenv("BSM_CHUNKS")) st.chunks = (uint32_t)std::max(1, std::atoi(e));
}
/// The context (created on first use) and its chunks, or nullptr for one GPU.
inline std::shared_ptr<bsm_multi> multi_context(uint32_t* chunks) {
    MultiState& st = multi_state();
    std::lock_guard<std::mutex> lk(st.mu);
    multi_env(st);
    if (st.gpus <= 0) return nullptr;
    if (!st.ctx) {
        bsm_multi* c = nullptr;
        if (auto e = status(bsm_multi_create(st.gpus, nullptr, &c)))
            throw Panic(std::string("bsm_multi_create: ") + to_string(*e));
        st.ctx = std::shared_ptr<bsm_multi>(c, [](bsm_multi* p) { bsm_multi_destroy(p); });
    }
    *chunks = st.chunks;
    return st.ctx;
}
/// A matrix partitioned over a context; keeps the context alive.
struct MultiCopy {
    std::shared_ptr<bsm_multi> ctx;
    uint32_t chunks = 1;
    std::shared_ptr<bsm_mcsr> m;
};
}  // namespace detail

/// Route every Csr::mul_dense of this process over n GPUs (row blocks of the
/// CSR on each, RCCL all-gather of the dense result; bit-identical to one
/// GPU); n = 0 returns to the single-GPU path, n = 1 runs the RCCL path on one
/// GPU. chunks: rounds per GPU (an all-gather per round overlaps the next
/// round's SpMM). Env BSM_N_GPUS / BSM_CHUNKS give the default.
inline void set_gpus(int n, uint32_t chunks = 1) {
    detail::MultiState& st = detail::multi_state();
    std::lock_guard<std::mutex> lk(st.mu);
    st.init = true;
    if (n != st.gpus) st.ctx.reset();
    st.gpus = n > 0 ? n : 0;
    st.chunks = chunks ? chunks : 1;
}

// --------------------------------------------------------------- dense.rs
/// dense.rs:4-62: column-major, one vector per column.
template <class T>
class Dense {
public:
    /// dense.rs:13-15 -- COLUMNS first.
    static Dense new_default_with_dims(size_t col_count, size_t row_count) {
        return new_with_dims(T{}, col_count, row_count);
    }
    /// dense.rs:17-19.
    static Dense new_with_dims(T val, size_t col_count, size_t row_count) {
        Dense d;
        d.col_count_ = col_count;
        d.row_count_ = row_count;
        d.data_.assign(col_count, std::vector<T>(row_count, val));
        return d;
    }
    /// dense.rs:21-29: `data` is a list of COLUMNS; row_count = data[0].len().
    static Dense from_data(const std::vector<std::vector<T>>& data) {
        Dense d;
        d.col_count_ = data.size();
        d.row_count_ = data.at(0).size();
        d.data_ = data;
        return d;
    }
    /// dense.rs:31-37.
    std::span<const T> get_col(size_t col_index) const { return data_.at(col_index); }
    std::span<T> get_col_mut(size_t col_index) { return data_.at(col_index); }
    /// dense.rs:40-47.
    MatDim get_dims() const { return {row_count_, col_count_}; }
    bool operator==(const Dense&) const = default;

private:
    size_t col_count_ = 0, row_count_ = 0;
    std::vector<std::vector<T>> data_;
};

// -------------------------------------------------------- dense_static.rs
/// dense_static.rs:4-62: `[[T; ROWS]; COLS]`, column-major.
template <class T, size_t ROWS, size_t COLS>
class DenseS {
public:
    static DenseS new_default() { return new_(T{}); }
    static DenseS new_(T val) {
        DenseS d;
        for (auto& c : d.data_) c.fill(val);
        return d;
    }
    /// dense_static.rs:21-35: `data` is a list of COLUMNS.
    static DenseS from_data(const std::vector<std::vector<T>>& data) {
        DenseS d = new_default();
        for (size_t c = 0; c < COLS; ++c)
            for (size_t r = 0; r < ROWS; ++r) d.data_[c][r] = data.at(c).at(r);
        return d;
    }
    std::span<const T> get_col(size_t col_index) const { return data_.at(col_index); }
    std::span<T> get_col_mut(size_t col_index) { return data_.at(col_index); }
    MatDim get_dims() const { return {ROWS, COLS}; }
    bool operator==(const DenseS&) const = default;

private:
    std::array<std::array<T, ROWS>, COLS> data_{};
};

// -------------------------------------------------------------- sparse.rs
/// sparse.rs:80-91.
template <class T>
struct CsrEntry {
    const T* v;
    size_t col_index;
    size_t row_index;
    bool operator==(const CsrEntry& o) const {
        return *v == *o.v && col_index == o.col_index && row_index == o.row_index;
    }
};

template <class T>
class Csr;

/// sparse.rs:7-33: a COO entry, ordered by row then col.
template <class T>
struct COOEntry {
    size_t row = 0, col = 0;
    T value{};
};

/// sparse.rs:35-54: an unordered entry list with a bounds-checked insert;
/// Csr<T>::from(coo) is `From<COO<T>> for Csr<T>` (sparse.rs:56-66).
template <class T>
class COO {
public:
    static COO with_capacity(MatDim dims, size_t capacity) {
        COO c;
        c.dims_ = dims;
        c.entries_.reserve(capacity);
        return c;
    }
    /// sparse.rs:45-53: Err(OutOfBounds) unless row < rows and col < cols.
    Result<void> insert(COOEntry<T> e) {
        if (dims_.rows <= e.row || dims_.cols <= e.col) return MatErr::OutOfBounds;
        entries_.push_back(e);
        return {};
    }
    const std::vector<COOEntry<T>>& entries() const { return entries_; }
    MatDim dims() const { return dims_; }

private:
    std::vector<COOEntry<T>> entries_;
    MatDim dims_;
};

template <class T>
class Csr {
public:
    // ---------------------------------------------------------- ctors
    /// sparse.rs:117-119.
    static Csr new_(MatDim dims) { return new_with_capacity(dims, 0); }
    /// sparse.rs:121-132.
    static Csr new_with_capacity(MatDim dims, size_t capacity) {
        Csr m;
        m.dims_ = dims;
        m.v_.reserve(capacity);
        m.col_index_.reserve(capacity);
        m.row_index_ = {0};
        return m;
    }
    /// sparse.rs:134-152 (insert_unchecked: a zero `value` IS stored).
    static Result<Csr> eye(MatDim dims, T value) {
        if (dims.cols != dims.rows) return MatErr::IncorrectDimensions;
        Csr m = new_(dims);
        for (size_t n = 0; n < dims.cols; ++n) m.insert_unchecked(value, n, n);
        return std::move(m).finalise();
    }
    /// sparse.rs:154-160.
    static Csr create_diagonal(const std::vector<T>& contents) {
        Csr m = new_({contents.size(), contents.size()});
        for (size_t i = 0; i < contents.size(); ++i) m.insert(contents[i], i, i).unwrap();
        return std::move(m).finalise();
    }
    /// sparse.rs:193-203: `data` is a list of ROWS; zeros are skipped.
    static Csr from_data(const std::vector<std::vector<T>>& data) {
        Csr m = new_({data.size(), data.at(0).size()});
        for (size_t r = 0; r < data.size(); ++r)
            for (size_t c = 0; c < data[r].size(); ++c) m.insert(data[r][c], r, c).unwrap();
        return std::move(m).finalise();
    }
    /// Bulk constructor (this build's addition): adopt a finalised CSR
    /// (row_index has rows + 1 entries).
    static Csr from_csr_arrays(MatDim dims, std::vector<size_t> row_index, std::vector<size_t> col_index,
                               std::vector<T> v) {
        if (row_index.size() != dims.rows + 1) throw std::invalid_argument("row_index must have rows+1 entries");
        Csr m;
        m.dims_ = dims;
        m.row_index_ = std::move(row_index);
        m.col_index_ = std::move(col_index);
        m.v_ = std::move(v);
        m.is_finalised_ = true;
        return m;
    }

    // ------------------------------------------------------- building
    /// sparse.rs:206-219: pad row_index to rows + 1 with nnz ("big eek" when
    /// more rows were registered than the matrix has).
    Csr finalise() && {
        if (!is_finalised_) {
            is_finalised_ = true;
            if (dims_.rows < row_index_.size()) throw Panic("big eek");
            const size_t nnz = v_.size();
            row_index_.resize(dims_.rows, nnz);
            row_index_.push_back(nnz);
        }
        return std::move(*this);
    }
    Csr finalise() const& { return Csr(*this).finalise_copy(); }

    /// sparse.rs:222-233: Err(MatrixFinalised) after finalise; a value equal
    /// to T::default() is silently skipped.
    Result<void> insert(T value, size_t row, size_t col) {
        if (is_finalised_) return MatErr::MatrixFinalised;
        if (!(value == T{})) insert_unchecked(value, row, col);
        return {};
    }

    // ------------------------------------------------------ accessors
    MatDim get_dims() const { return dims_; }
    /// sparse.rs:162-164: the last row_index entry.
    size_t get_nnz() const { return row_index_.empty() ? 0 : row_index_.back(); }
    /// sparse.rs:166-168.
    float get_density() const { return (float)v_.size() / (float)(dims_.rows * dims_.cols); }
    /// sparse.rs:170-180.
    const T* get_val_at(MatDim at) const {
        const size_t s = row_index_.at(at.rows), e = row_index_.at(at.rows + 1);
        for (size_t i = s; i < e; ++i)
            if (col_index_[i] == at.cols) return &v_[i];
        return nullptr;
    }
    /// sparse.rs:252-265 (the last recorded row extends to v.len()).
    std::vector<CsrEntry<T>> get_row_compact(size_t index) const {
        auto [s, e] = row_bounds(index);
        std::vector<CsrEntry<T>> out;
        out.reserve(e - s);
        for (size_t i = s; i < e; ++i) out.push_back({&v_[i], col_index_[i], index});
        return out;
    }
    /// sparse.rs:267-294 (literal expansion, unsorted/duplicate columns included).
    std::optional<std::vector<T>> get_row_complete(size_t index) const {
        if (row_index_.empty() || index >= row_index_.size()) return std::nullopt;
        const size_t s = row_index_[index];
        const size_t e = row_index_.size() == index + 1 ? v_.size() : row_index_[index + 1];
        std::vector<T> out;
        size_t prev = 0;
        for (size_t i = s; i < e; ++i) {
            const size_t c = col_index_[i];
            if (c != 0 && c > prev) out.insert(out.end(), c - prev, T{});
            prev = c + 1;
            out.push_back(v_[i]);
        }
        if (dims_.cols > prev) out.insert(out.end(), dims_.cols - prev, T{});
        return out;
    }
    /// `Iterator for Csr` (sparse.rs:93-114).
    std::optional<CsrEntry<T>> next() {
        if (iter_v_index_ == v_.size()) return std::nullopt;
        while (row_index_[iter_row_index_] == iter_v_index_) ++iter_row_index_;
        CsrEntry<T> e{&v_[iter_v_index_], col_index_[iter_v_index_], iter_row_index_ - 1};
        ++iter_v_index_;
        return e;
    }
    /// sparse.rs:413-416.
    void reset_iter() { iter_row_index_ = iter_v_index_ = 0; }

    const std::vector<T>& v() const { return v_; }
    const std::vector<size_t>& col_index() const { return col_index_; }
    const std::vector<size_t>& row_index() const { return row_index_; }
    bool is_finalised() const { return is_finalised_; }

    // ------------------------------------------------------- hot path
    /// sparse.rs:426-446: self * rhs as a new finalised Csr (rows, rhs.cols),
    /// zero results dropped. GPU (kernels_spmm.hip).
    Result<Csr> mul_dense(const Dense<T>& rhs) const requires detail::GpuScalar<T> {
        if (dims_.cols != rhs.get_dims().rows) return MatErr::IncorrectDimensions;  // :427-429
        std::vector<const void*> cols(rhs.get_dims().cols);
        for (size_t j = 0; j < cols.size(); ++j) cols[j] = rhs.get_col(j).data();
        return mul_cols(cols, rhs.get_dims().rows);
    }
    /// sparse.rs:448-466 (checked against ROWS, :449).
    template <size_t ROWS, size_t COLS>
    Result<Csr> mul_dense_s(const DenseS<T, ROWS, COLS>& rhs) const requires detail::GpuScalar<T> {
        if (dims_.cols != ROWS) return MatErr::IncorrectDimensions;
        std::vector<const void*> cols(COLS);
        for (size_t j = 0; j < COLS; ++j) cols[j] = rhs.get_col(j).data();
        return mul_cols(cols, ROWS);
    }
    /// sparse.rs:468-482: out[i] = sum of row i (ascending columns), written
    /// into the caller's slice.
    Result<void> mul_vector(std::span<const T> rhs, std::span<T> out) const requires detail::GpuScalar<T> {
        if (dims_.cols != rhs.size() || dims_.rows != out.size()) return MatErr::IncorrectDimensions;
        auto h = device();
        if (auto e = detail::status(bsm_csr_mul_vector(h.get(), rhs.data(), rhs.size(), out.data(), out.size())))
            return *e;
        return {};
    }
    /// sparse.rs:296-318 (stable CSR -> CSC on the GPU).
    Csr transpose() const requires detail::GpuScalar<T> {
        if (!is_finalised_ && !v_.empty())
            throw Panic("index out of bounds (transpose of an unfinalised matrix)");
        auto h = device();
        bsm_csr* out = nullptr;
        detail::check(bsm_csr_transpose(h.get(), &out));
        return from_device(detail::Handle(out, detail::HandleFree{}));
    }
    /// sparse.rs:320-323.
    std::pair<Csr, Csr> pair_with_tranpose() && {
        Csr t = transpose();
        return {std::move(*this), std::move(t)};
    }
    /// `impl Csr<f32>::cholesky_decomp` (sparse.rs:682-714); f64 is this
    /// build's addition.
    Result<Csr> cholesky_decomp() const requires std::is_floating_point_v<T> {
        if (dims_.rows != dims_.cols) return MatErr::NonSquareMatrix;  // :683-685
        auto h = device();
        bsm_csr* out = nullptr;
        if (auto e = detail::status(bsm_csr_cholesky(h.get(), &out))) return *e;
        return from_device(detail::Handle(out, detail::HandleFree{}));
    }

    /// sparse.rs:484-540: the per-row merge in storage order, zero sums dropped.
    Result<Csr> add_sparse(const Csr& rhs) const requires detail::GpuScalar<T> {
        if (dims_ != rhs.dims_) return MatErr::IncorrectDimensions;  // :485-487
        return binary(rhs, bsm_csr_add_sparse);
    }
    /// sparse.rs:542-599 (rhs-only entries become T::default() - v).
    Result<Csr> sub_sparse(const Csr& rhs) const requires detail::GpuScalar<T> {
        if (dims_ != rhs.dims_) return MatErr::IncorrectDimensions;  // :543-546
        return binary(rhs, bsm_csr_sub_sparse);
    }
    /// sparse.rs:601-635: dims (rows, rhs.cols), no dimension check.
    Result<Csr> mul_sparse(const Csr& rhs) const requires detail::GpuScalar<T> {
        return binary(rhs, bsm_csr_mul_sparse);
    }
    /// `From<COO<T>> for Csr<T>` (sparse.rs:56-66): stable sort by (row, col),
    /// then the zero-skipping insert sequence and finalise (on the GPU).
    static Csr from(const class COO<T>& coo) requires detail::GpuScalar<T>;

    /// Derived PartialEq over the seven fields of sparse.rs:68-78.
    bool operator==(const Csr& o) const {
        return dims_ == o.dims_ && v_ == o.v_ && col_index_ == o.col_index_ && row_index_ == o.row_index_ &&
               is_finalised_ == o.is_finalised_ && iter_v_index_ == o.iter_v_index_ &&
               iter_row_index_ == o.iter_row_index_;
    }

    /// The device copy (uploaded once per finalised matrix). Rows as the
    /// reference's row loop sees them; panics where it panics.
    detail::Handle device() const {
        if (dev_) return dev_;
        auto [rp, used] = device_row_ptr();
        bsm_csr* h = nullptr;
        static_assert(sizeof(size_t) == sizeof(uint64_t), "usize is 8 bytes (x86_64)");
        detail::check(bsm_csr_upload(detail::dtype_of<T>::value, dims_.rows, dims_.cols, used, rp.data(),
                                     reinterpret_cast<const uint64_t*>(col_index_.data()), v_.data(), &h));
        detail::Handle hd(h, detail::HandleFree{});
        if (is_finalised_) dev_ = hd;
        return hd;
    }

    /// row_ptr (rows + 1) as the reference's row loop sees the matrix, and
    /// the entries it uses; panics where it panics.
    std::pair<std::vector<uint64_t>, size_t> device_row_ptr() const {
        const size_t rows = dims_.rows, nnz = v_.size();
        std::vector<uint64_t> rp(rows + 1);
        if (row_index_.size() >= rows + 1) {
            for (size_t r = 0; r <= rows; ++r) rp[r] = row_index_[r];
            if (row_index_.size() == rows + 1 && !is_finalised_) rp[rows] = nnz;
        } else if (row_index_.size() == rows) {
            for (size_t r = 0; r < rows; ++r) rp[r] = row_index_[r];
            rp[rows] = nnz;
        } else {
            throw Panic("index out of bounds: the len is " + std::to_string(row_index_.size()) +
                        " but the index is " + std::to_string(row_index_.size()));
        }
        for (size_t r = 0; r < rows; ++r)
            if (rp[r + 1] < rp[r]) throw Panic("slice index starts after end");
        const size_t used = rows ? rp[rows] : 0;
        if (used > nnz) throw Panic("slice index starts after end");
        for (size_t i = 0; i < used; ++i)
            if (col_index_[i] >= dims_.cols)
                throw Panic("index out of bounds: column " + std::to_string(col_index_[i]) + " >= " +
                            std::to_string(dims_.cols));
        return {std::move(rp), used};
    }

private:
    Csr() = default;
    Csr finalise_copy() { return std::move(*this).finalise(); }

    /// sparse.rs:237-250: a row is recorded only when it exceeds the running
    /// maximum; an entry for an earlier row is appended to the current last row.
    void insert_unchecked(T value, size_t row, size_t col) {
        dev_.reset();
        mdev_ = {};
        v_.push_back(value);
        col_index_.push_back(col);
        if (row + 1 > row_index_.size()) {
            const size_t start = v_.size() - 1;
            while (row_index_.size() <= row) row_index_.push_back(start);
        }
    }

    std::pair<size_t, size_t> row_bounds(size_t index) const {
        if (index >= row_index_.size())
            throw Panic("index out of bounds: the len is " + std::to_string(row_index_.size()) +
                        " but the index is " + std::to_string(index));
        const size_t s = row_index_[index];
        const size_t e = index == row_index_.size() - 1 ? v_.size() : row_index_[index + 1];
        if (s > e || e > v_.size()) throw Panic("slice index starts after end");
        return {s, e};
    }

    Result<Csr> mul_cols(const std::vector<const void*>& cols, size_t x_rows) const {
        uint32_t chunks = 1;
        if (auto ctx = detail::multi_context(&chunks)) {  // row blocks on every GPU + RCCL all-gather
            auto m = multi_device(ctx, chunks);
            bsm_csr* out = nullptr;
            if (auto e = detail::status(bsm_mcsr_mul_dense(m.get(), cols.size(), x_rows, cols.data(), &out)))
                return *e;
            return from_device(detail::Handle(out, detail::HandleFree{}));
        }
        auto h = device();
        bsm_csr* out = nullptr;
        if (auto e = detail::status(bsm_csr_mul_dense(h.get(), cols.size(), x_rows, cols.data(), &out))) return *e;
        return from_device(detail::Handle(out, detail::HandleFree{}));
    }

    /// The matrix partitioned over the multi-GPU context, cached like the
    /// single-GPU copy for a finalised matrix.
    std::shared_ptr<bsm_mcsr> multi_device(const std::shared_ptr<bsm_multi>& ctx, uint32_t chunks) const {
        if (mdev_.m && mdev_.ctx == ctx && mdev_.chunks == chunks) return mdev_.m;
        auto [rp, used] = device_row_ptr();
        bsm_mcsr* m = nullptr;
        detail::check(bsm_mcsr_upload(ctx.get(), detail::dtype_of<T>::value, dims_.rows, dims_.cols, used, rp.data(),
                                      reinterpret_cast<const uint64_t*>(col_index_.data()), v_.data(), chunks, &m));
        std::shared_ptr<bsm_mcsr> sp(m, [](bsm_mcsr* p) { bsm_mcsr_free(p); });
        if (is_finalised_) mdev_ = {ctx, chunks, sp};
        return sp;
    }

    Result<Csr> binary(const Csr& rhs, int (*fn)(const bsm_csr*, const bsm_csr*, bsm_csr**)) const {
        auto a = device();
        auto b = rhs.device();
        bsm_csr* out = nullptr;
        if (auto e = detail::status(fn(a.get(), b.get(), &out))) return *e;
        return from_device(detail::Handle(out, detail::HandleFree{}));
    }

public:
    static Csr from_device(detail::Handle h) {
        uint64_t rows = 0, cols = 0, nnz = 0;
        int dt = 0;
        detail::check(bsm_csr_shape(h.get(), &rows, &cols, &nnz, &dt));
        Csr m;
        m.dims_ = {rows, cols};
        m.v_.resize(nnz);
        m.row_index_.resize(rows + 1);
        m.col_index_.resize(nnz);
        // usize Vecs filled in place (the library widens int32 columns on the device)
        detail::check(bsm_csr_download(h.get(), reinterpret_cast<uint64_t*>(m.row_index_.data()),
                                       reinterpret_cast<uint64_t*>(m.col_index_.data()), m.v_.data()));
        m.is_finalised_ = true;  // what finalise() leaves (sparse.rs:206-219)
        m.dev_ = std::move(h);
        return m;
    }

private:
    MatDim dims_;
    std::vector<T> v_;
    std::vector<size_t> col_index_;
    std::vector<size_t> row_index_;
    bool is_finalised_ = false;
    size_t iter_v_index_ = 0, iter_row_index_ = 0;
    mutable detail::Handle dev_;
    mutable detail::MultiCopy mdev_;
};

template <class T>
Csr<T> Csr<T>::from(const COO<T>& coo) requires detail::GpuScalar<T> {
    const auto& es = coo.entries();
    std::vector<uint64_t> r(es.size()), c(es.size());
    std::vector<T> v(es.size());
    for (size_t i = 0; i < es.size(); ++i) {
        r[i] = es[i].row;
        c[i] = es[i].col;
        v[i] = es[i].value;
    }
    bsm_csr* out = nullptr;
    if (auto e = detail::status(bsm_csr_from_coo(detail::dtype_of<T>::value, coo.dims().rows, coo.dims().cols,
                                                 es.size(), r.data(), c.data(), v.data(), &out)))
        throw Panic(std::string("COO entry out of bounds: ") + to_string(*e));
    return from_device(detail::Handle(out, detail::HandleFree{}));
}

// ----------------------------------------------------------------- lib.rs
namespace detail {
template <class T>
Dense<T> run_solver(int (*fn)(const bsm_csr*, uint64_t, uint64_t, const void* const*, void* const*),
                    const Csr<T>& m, const Dense<T>& rhs) {
    const size_t n = rhs.get_dims().rows, k = rhs.get_dims().cols;
    if (m.get_dims().rows < n) throw Panic("index out of bounds: matrix has fewer rows than the right-hand side");
    auto h = m.device();
    Dense<T> out = Dense<T>::new_default_with_dims(k, n);
    std::vector<const void*> in_cols(k);
    std::vector<void*> out_cols(k);
    for (size_t j = 0; j < k; ++j) {
        in_cols[j] = rhs.get_col(j).data();
        out_cols[j] = out.get_col_mut(j).data();
    }
    check(fn(h.get(), k, n, in_cols.data(), out_cols.data()));
    return out;
}
}  // namespace detail

/// lib.rs:28-46: solve L y = b (the diagonal is the LAST entry of each row).
template <class T>
    requires std::is_floating_point_v<T>
Dense<T> forward_substitution(Csr<T> l, Dense<T> b) {
    return detail::run_solver<T>(bsm_forward_substitution, l, b);
}

/// lib.rs:49-65: solve L* x = y (the diagonal is the FIRST entry of each row).
template <class T>
    requires std::is_floating_point_v<T>
Dense<T> backward_substitution(Csr<T> l_star, Dense<T> y) {
    return detail::run_solver<T>(bsm_backward_substitution, l_star, y);
}

/// lib.rs:11-24 (f32 in the reference; f64 is this build's addition). A
/// non-square `a` panics (`cholesky_decomp().unwrap()`, lib.rs:20).
template <class T>
    requires std::is_floating_point_v<T>
Dense<T> solve(Csr<T> a, Dense<T> b) {
    if (a.get_dims().rows != a.get_dims().cols)
        throw Panic("called `Result::unwrap()` on an `Err` value: NonSquareMatrix");
    return detail::run_solver<T>(bsm_solve, a, b);
}

/// solve with the sums reassociated (bsm_solve_blocked; this build's
/// addition): within the f64 tolerance, not bit-exact; same errors/panics.
template <class T>
    requires std::is_floating_point_v<T>
Dense<T> solve_blocked(Csr<T> a, Dense<T> b) {
    if (a.get_dims().rows != a.get_dims().cols)
        throw Panic("called `Result::unwrap()` on an `Err` value: NonSquareMatrix");
    return detail::run_solver<T>(bsm_solve_blocked, a, b);
}

/// solve by a nested-dissection multifrontal factor of P A P^T (bsm_solve_nd;
/// this build's addition): within the f64 tolerance, not bit-exact; the
/// ordering plan is cached on the device handle; same errors/panics.
template <class T>
    requires std::is_floating_point_v<T>
Dense<T> solve_nd(Csr<T> a, Dense<T> b) {
    if (a.get_dims().rows != a.get_dims().cols)
        throw Panic("called `Result::unwrap()` on an `Err` value: NonSquareMatrix");
    return detail::run_solver<T>(bsm_solve_nd, a, b);
}

}  // namespace bsm

#endif  // BSM_HPP
