#pragma once
// Domain decomposition.
// Parity: reference include/stencil/partition.hpp
//   RankPartition  prime-factor splits of the longest axis, uneven remainder to low indices   :23-144
//   NodePartition  two-level (nodes, then GPUs per node) minimum radius-weighted interface       :148-310
#include <algorithm>
#include <cmath>
#include <vector>

#include "stencil/core/geometry.hpp"

namespace stencil {

// prime factors of n, largest first
inline std::vector<int64_t> prime_factors_desc(int64_t n) {
  std::vector<int64_t> r;
  if (n <= 1) return r;
  while (n % 2 == 0) {
    r.push_back(2);
    n /= 2;
  }
  for (int64_t i = 3; i * i <= n; i += 2)
    while (n % i == 0) {
      r.push_back(i);
      n /= i;
    }
  if (n > 2) r.push_back(n);
  std::sort(r.begin(), r.end(), [](int64_t a, int64_t b) { return b < a; });
  return r;
}

inline int64_t div_ceil(int64_t n, int64_t d) { return (n + d - 1) / d; }

// x-fastest linearization
inline int64_t linearize(const Dim3 &idx, const Dim3 &dim) { return idx.x + idx.y * dim.x + idx.z * dim.y * dim.x; }
inline Dim3 dimensionize(int64_t i, const Dim3 &dim) {
  Dim3 r;
  r.x = i % dim.x;
  i /= dim.x;
  r.y = i % dim.y;
  i /= dim.y;
  r.z = i;
  return r;
}

// Common logic: a grid of `dim` sub-domains with approximate size `size_` and remainder `rem_`.
class GridPartition {
protected:
  Dim3 dim_{1, 1, 1};
  Dim3 size_;
  Dim3 rem_;

public:
  Dim3 dim() const { return dim_; }
  Dim3 subdomain_size(const Dim3 &idx) const {
    Dim3 r = size_;
    if (rem_.x != 0 && idx.x >= rem_.x) r.x -= 1;
    if (rem_.y != 0 && idx.y >= rem_.y) r.y -= 1;
    if (rem_.z != 0 && idx.z >= rem_.z) r.z -= 1;
    return r;
  }
  Dim3 subdomain_origin(const Dim3 &idx) const {
    Dim3 r = size_ * idx;
    if (rem_.x != 0 && idx.x >= rem_.x) r.x -= (idx.x - rem_.x);
    if (rem_.y != 0 && idx.y >= rem_.y) r.y -= (idx.y - rem_.y);
    if (rem_.z != 0 && idx.z >= rem_.z) r.z -= (idx.z - rem_.z);
    return r;
  }
  int64_t linearize(const Dim3 &idx) const { return stencil::linearize(idx, dim_); }
  Dim3 dimensionize(int64_t i) const { return stencil::dimensionize(i, dim_); }
};

class RankPartition : public GridPartition {
public:
  RankPartition() = default;
  RankPartition(const Dim3 &size, int64_t n) {
    size_ = size;
    for (int64_t amt : prime_factors_desc(n)) {
      if (size_.x >= size_.y && size_.x >= size_.z) {
        size_.x = div_ceil(size_.x, amt);
        dim_.x *= amt;
      } else if (size_.y >= size_.z) {
        size_.y = div_ceil(size_.y, amt);
        dim_.y *= amt;
      } else {
        size_.z = div_ceil(size_.z, amt);
        dim_.z *= amt;
      }
    }
    rem_ = size % dim_;
  }
};

class NodePartition : public GridPartition {
  Dim3 sysDim_{1, 1, 1};
  Dim3 nodeDim_{1, 1, 1};

  Dim3 cost_{1, 1, 1};

  void split(Dim3 &d, int64_t amt, const Radius &radius) {
    const int64_t xIface = cost_.x * size_.y * size_.z * (radius.dir(1, 0, 0) + radius.dir(-1, 0, 0));
    const int64_t yIface = cost_.y * size_.x * size_.z * (radius.dir(0, 1, 0) + radius.dir(0, -1, 0));
    const int64_t zIface = cost_.z * size_.x * size_.y * (radius.dir(0, 0, 1) + radius.dir(0, 0, -1));
    // minimum radius-weighted interface; ties go to z, then y, then x (the reference prefers x,
    // partition.hpp:224-237). On MI355X a z-face is one contiguous plane (full-rate 16-B copies) while an x-face is a
    // strided column touching one 128-B line per 4-B element, so remote faces are cheapest along z.
    if (zIface <= yIface && zIface <= xIface) {
      size_.z = div_ceil(size_.z, amt);
      d.z *= amt;
    } else if (yIface <= xIface) {
      size_.y = div_ceil(size_.y, amt);
      d.y *= amt;
    } else {
      size_.x = div_ceil(size_.x, amt);
      d.x *= amt;
    }
  }

public:
  NodePartition() = default;
  // axisCost: relative cost per interface cell of a cut normal to x / y / z (default 1,1,1: the reference's plain
  // radius-weighted interface). StencilModel uses (2,1,1): an x face is a strided column (one 128-B line per row
  // for a 2-cell halo, packed and unpacked by gathers) while y/z faces are contiguous rows, and a domain without x
  // cuts can overlap its exchange with row-contiguous exterior slabs only.
  NodePartition(const Dim3 &size, const Radius &radius, int64_t nodes, int64_t gpus, const Dim3 &axisCost = Dim3(1, 1, 1)) {
    size_ = size;
    cost_ = axisCost;
    for (int64_t amt : prime_factors_desc(nodes)) split(sysDim_, amt, radius);
    for (int64_t amt : prime_factors_desc(gpus)) split(nodeDim_, amt, radius);
    dim_ = sysDim_ * nodeDim_;
    rem_ = size % dim_;
  }
  Dim3 sys_dim() const { return sysDim_; }
  Dim3 node_dim() const { return nodeDim_; }
  Dim3 sys_idx(int64_t i) const { return stencil::dimensionize(i, sysDim_); }
  Dim3 node_idx(int64_t i) const { return stencil::dimensionize(i, nodeDim_); }
  Dim3 idx(int64_t i) const { return stencil::dimensionize(i, dim_); }
  // global index of node-local component i on node n
  Dim3 global_idx(int64_t node, int64_t i) const { return sys_idx(node) * nodeDim_ + node_idx(i); }
};

} // namespace stencil
