#pragma once
// Row-major 2D matrix used by the placement solver.
// Parity: reference include/stencil/mat2d.hpp:21-192 (ctor, brace-init, push_back row, resize, ==, /=,
// make_reciprocal 0 -> inf). The reference's dead/uncompilable permute() is not reproduced.
#include <cassert>
#include <initializer_list>
#include <limits>
#include <vector>

#include "stencil/core/dim3.hpp"

template <typename T> class Mat2D {
  std::vector<T> data_;
  size_t rows_ = 0, cols_ = 0;

public:
  struct Shape {
    size_t y, x; // rows, cols
    bool operator==(const Shape &o) const { return y == o.y && x == o.x; }
    bool operator!=(const Shape &o) const { return !(*this == o); }
  };

  Mat2D() = default;
  Mat2D(size_t rows, size_t cols, const T &v = T()) : data_(rows * cols, v), rows_(rows), cols_(cols) {}
  Mat2D(std::initializer_list<std::initializer_list<T>> ll) {
    rows_ = ll.size();
    cols_ = rows_ ? ll.begin()->size() : 0;
    for (const auto &row : ll) {
      assert(row.size() == cols_);
      for (const auto &e : row) data_.push_back(e);
    }
  }

  Shape shape() const { return Shape{rows_, cols_}; }
  size_t rows() const { return rows_; }
  size_t cols() const { return cols_; }

  T &at(size_t i, size_t j) {
    assert(i < rows_ && j < cols_);
    return data_[i * cols_ + j];
  }
  const T &at(size_t i, size_t j) const {
    assert(i < rows_ && j < cols_);
    return data_[i * cols_ + j];
  }

  class Row {
    T *p_;
    size_t n_;

  public:
    Row(T *p, size_t n) : p_(p), n_(n) {}
    T &operator[](size_t j) {
      assert(j < n_);
      return p_[j];
    }
    size_t size() const { return n_; }
  };
  class ConstRow {
    const T *p_;
    size_t n_;

  public:
    ConstRow(const T *p, size_t n) : p_(p), n_(n) {}
    const T &operator[](size_t j) const {
      assert(j < n_);
      return p_[j];
    }
    size_t size() const { return n_; }
  };
  Row operator[](size_t i) { return Row(&data_[i * cols_], cols_); }
  ConstRow operator[](size_t i) const { return ConstRow(&data_[i * cols_], cols_); }

  void push_back(const std::vector<T> &row) {
    if (rows_ == 0 && cols_ == 0) cols_ = row.size();
    assert(row.size() == cols_);
    data_.insert(data_.end(), row.begin(), row.end());
    ++rows_;
  }

  void resize(size_t rows, size_t cols) {
    std::vector<T> nd(rows * cols, T());
    for (size_t i = 0; i < rows && i < rows_; ++i)
      for (size_t j = 0; j < cols && j < cols_; ++j) nd[i * cols + j] = data_[i * cols_ + j];
    data_.swap(nd);
    rows_ = rows;
    cols_ = cols;
  }

  bool operator==(const Mat2D &o) const { return rows_ == o.rows_ && cols_ == o.cols_ && data_ == o.data_; }
  bool operator!=(const Mat2D &o) const { return !(*this == o); }

  Mat2D &operator/=(const T &s) {
    for (auto &e : data_) e /= s;
    return *this;
  }
  const std::vector<T> &data() const { return data_; }
};

// element-wise reciprocal; 0 maps to +inf (reference mat2d.hpp:176-192)
template <typename T> Mat2D<T> make_reciprocal(const Mat2D<T> &m) {
  Mat2D<T> r(m.rows(), m.cols());
  for (size_t i = 0; i < m.rows(); ++i)
    for (size_t j = 0; j < m.cols(); ++j) {
      const T v = m.at(i, j);
      r.at(i, j) = (v == T(0)) ? std::numeric_limits<T>::infinity() : T(1) / v;
    }
  return r;
}
