#pragma once
// Domain decomposition.
// Parity: reference include/stencil/partition.hpp
//   RankPartition  prime-factor splits of the longest axis, uneven remainder to low indices   :23-144
//   NodePartition  two-level (nodes, then GPUs per node) minimum radius-weighted interface       :148-310
#include <algorithm>
#include <cmath>
#include <utility>
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

// How NodePartition chooses the cuts inside a node.
//   Interface  the reference's rule (partition.hpp:210-264): each prime-factor cut goes where the radius-weighted
//              interface (x axis cost) is smallest, greedily.
//   MaxLink    the GPUs of an MI355X node are a fully connected xGMI mesh (7 point-to-point links per GPU, no
//              switch): the neighbours of a sub-domain sit on different links, so an exchange takes as long as its
//              busiest link, not its total surface. Every factorization dx*dy*dz of the node's GPU count is scored by
//              (max over axes of the halo cells one link carries) x axis cost, then by the total halo cells x axis
//              cost; an axis cut into 2 puts both of its faces on the same link (double volume), an axis cut into
//              >= 3 gives each face its own link, an uncut axis wraps on the GPU. For equal cubes per GPU this
//              prefers slabs (1x1xN: two faces per GPU, one per link, x and y wrapped in the stencil kernel) over
//              1x2x4 (four faces, two on one link) or 2x2x2 (six faces, two per link, strided x faces).
//              The node-level cuts (inter-node links) keep the greedy interface rule.
enum class PartitionObjective { Interface, MaxLink };

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
  // (max-link cost, total cost) of cutting a box of `size` into d sub-domains (MaxLink objective)
  static std::pair<int64_t, int64_t> link_cost(const Dim3 &size, const Dim3 &d, const Radius &radius, const Dim3 &cost) {
    const Dim3 s(div_ceil(size.x, d.x), div_ceil(size.y, d.y), div_ceil(size.z, d.z));
    const int64_t face[3] = {s.y * s.z, s.x * s.z, s.x * s.y};
    const int64_t n[3] = {d.x, d.y, d.z};
    const int64_t c[3] = {cost.x, cost.y, cost.z};
    int64_t worst = 0, total = 0;
    for (int a = 0; a < 3; ++a) {
      if (n[a] == 1) continue;
      const Dim3 pd(a == 0, a == 1, a == 2);
      const int64_t rp = radius.dir(pd), rm = radius.dir(Dim3(0, 0, 0) - pd);
      const int64_t link = face[a] * (n[a] == 2 ? rp + rm : std::max(rp, rm)) * c[a];
      worst = std::max(worst, link);
      total += face[a] * (rp + rm) * c[a];
    }
    return {worst, total};
  }

  // the MaxLink choice of dims for `n` parts of a box of `size` (ties: fewer x cuts, then fewer y cuts)
  static Dim3 max_link_dims(const Dim3 &size, int64_t n, const Radius &radius, const Dim3 &cost) {
    Dim3 best(1, 1, n);
    std::pair<int64_t, int64_t> bc{-1, -1};
    for (int64_t dx = 1; dx <= n; ++dx) {
      if (n % dx) continue;
      for (int64_t dy = 1; dy <= n / dx; ++dy) {
        if ((n / dx) % dy) continue;
        const Dim3 d(dx, dy, n / dx / dy);
        if (d.x > size.x || d.y > size.y || d.z > size.z) continue;
        const auto c = link_cost(size, d, radius, cost);
        const bool better = bc.first < 0 || c < bc ||
                            (c == bc && (d.x < best.x || (d.x == best.x && d.y < best.y)));
        if (better) {
          bc = c;
          best = d;
        }
      }
    }
    return best;
  }

  NodePartition() = default;
  // axisCost: relative cost per interface cell of a cut normal to x / y / z (default 1,1,1: the reference's plain
  // radius-weighted interface). StencilModel uses (4,3,2): an x face is a strided column (one 128-B line per row
  // for a 2-cell halo, packed and unpacked by gathers) while y/z faces are contiguous rows, and a domain without x
  // cuts can overlap its exchange with row-contiguous exterior slabs only.
  NodePartition(const Dim3 &size, const Radius &radius, int64_t nodes, int64_t gpus, const Dim3 &axisCost = Dim3(1, 1, 1),
                PartitionObjective objective = PartitionObjective::Interface) {
    size_ = size;
    cost_ = axisCost;
    for (int64_t amt : prime_factors_desc(nodes)) split(sysDim_, amt, radius);
    if (objective == PartitionObjective::MaxLink && gpus > 1) {
      nodeDim_ = max_link_dims(size_, gpus, radius, cost_);
      size_ = Dim3(div_ceil(size_.x, nodeDim_.x), div_ceil(size_.y, nodeDim_.y), div_ceil(size_.z, nodeDim_.z));
    } else {
      for (int64_t amt : prime_factors_desc(gpus)) split(nodeDim_, amt, radius);
    }
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
