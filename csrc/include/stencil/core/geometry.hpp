#pragma once
// Rect3, DirectionMap<T>, Radius, Accessor<T>, next_align_of.
// Parity: reference include/stencil/{rect3,direction_map,radius,accessor,align}.hpp
//   Rect3 half-open [lo,hi)                      rect3.hpp:13-22
//   DirectionMap 3x3x3 indexed by dir            direction_map.hpp:11-57
//   Radius per-direction, face/edge/corner       radius.hpp:16-103
//   Accessor global-coordinate indexing          accessor.hpp:27-35 (here with an explicit x pitch)
//   next_align_of                                align.cuh:7-9
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <ostream>

#include "stencil/core/dim3.hpp"

struct Rect3 {
  Dim3 lo, hi;
  STENCIL_HDI Rect3() {}
  STENCIL_HDI Rect3(const Dim3 &l, const Dim3 &h) : lo(l), hi(h) {}
  STENCIL_HDI Dim3 extent() const { return hi - lo; }
  STENCIL_HDI bool empty() const { return !(hi.x > lo.x && hi.y > lo.y && hi.z > lo.z); }
  STENCIL_HDI bool contains(const Dim3 &p) const { return p.all_ge(lo) && p.all_lt(hi); }
  STENCIL_HDI bool operator==(const Rect3 &o) const { return lo == o.lo && hi == o.hi; }
  STENCIL_HDI bool operator!=(const Rect3 &o) const { return !(*this == o); }
};

inline std::ostream &operator<<(std::ostream &os, const Rect3 &r) { return os << "{" << r.lo << "-" << r.hi << "}"; }

template <typename T> class DirectionMap {
  T data_[27];

public:
  STENCIL_HDI DirectionMap() {
    for (int i = 0; i < 27; ++i) data_[i] = T();
  }
  STENCIL_HDI T &at(int xi, int yi, int zi) { return data_[zi * 9 + yi * 3 + xi]; }
  STENCIL_HDI const T &at(int xi, int yi, int zi) const { return data_[zi * 9 + yi * 3 + xi]; }
  STENCIL_HDI T &at_dir(int x, int y, int z) { return at(x + 1, y + 1, z + 1); }
  STENCIL_HDI const T &at_dir(int x, int y, int z) const { return at(x + 1, y + 1, z + 1); }
  STENCIL_HDI bool operator==(const DirectionMap &o) const {
    for (int i = 0; i < 27; ++i)
      if (!(data_[i] == o.data_[i])) return false;
    return true;
  }
};

class Radius {
  DirectionMap<int64_t> rads_;

public:
  STENCIL_HDI int64_t &dir(int x, int y, int z) { return rads_.at_dir(x, y, z); }
  STENCIL_HDI const int64_t &dir(int x, int y, int z) const { return rads_.at_dir(x, y, z); }
  STENCIL_HDI int64_t &dir(const Dim3 &d) { return dir(int(d.x), int(d.y), int(d.z)); }
  STENCIL_HDI const int64_t &dir(const Dim3 &d) const { return dir(int(d.x), int(d.y), int(d.z)); }

  // face radii
  STENCIL_HDI int64_t x(int d) const { return dir(d, 0, 0); }
  STENCIL_HDI int64_t y(int d) const { return dir(0, d, 0); }
  STENCIL_HDI int64_t z(int d) const { return dir(0, 0, d); }

  STENCIL_HDI bool operator==(const Radius &o) const { return rads_ == o.rads_; }

  void set_face(int64_t r) {
    dir(0, 0, -1) = r;
    dir(0, 0, 1) = r;
    dir(0, -1, 0) = r;
    dir(0, 1, 0) = r;
    dir(-1, 0, 0) = r;
    dir(1, 0, 0) = r;
  }
  void set_edge(int64_t r) {
    for (int z = -1; z <= 1; ++z)
      for (int y = -1; y <= 1; ++y)
        for (int x = -1; x <= 1; ++x)
          if ((x != 0) + (y != 0) + (z != 0) == 2) dir(x, y, z) = r;
  }
  void set_corner(int64_t r) {
    for (int z = -1; z <= 1; z += 2)
      for (int y = -1; y <= 1; y += 2)
        for (int x = -1; x <= 1; x += 2) dir(x, y, z) = r;
  }
  static Radius constant(int64_t r) {
    Radius ret;
    for (int z = -1; z <= 1; ++z)
      for (int y = -1; y <= 1; ++y)
        for (int x = -1; x <= 1; ++x) ret.dir(x, y, z) = r;
    return ret;
  }
  static Radius face_edge_corner(int64_t face, int64_t edge, int64_t corner) {
    Radius ret;
    ret.set_face(face);
    ret.set_edge(edge);
    ret.set_corner(corner);
    ret.dir(0, 0, 0) = 0;
    return ret;
  }
  // largest radius over all 26 directions
  int64_t max() const {
    int64_t m = 0;
    for (int i = 0; i < 27; ++i) {
      Dim3 d = dir_from_index(i);
      if (d == Dim3(0, 0, 0)) continue;
      int64_t v = dir(d);
      m = v > m ? v : m;
    }
    return m;
  }
};

/* Accessor: index a raw allocation by GLOBAL coordinate.
   `origin` is the global coordinate of raw element [0,0,0] (the first halo cell),
   `pitch` is the allocation stride in elements (x is padded for alignment, see LocalDomain). */
template <typename T> class Accessor {
  T *raw_;
  Dim3 origin_;
  Dim3 pitch_;

public:
  STENCIL_HDI Accessor() : raw_(nullptr) {}
  STENCIL_HDI Accessor(T *raw, const Dim3 &origin, const Dim3 &pitch) : raw_(raw), origin_(origin), pitch_(pitch) {}
  STENCIL_HDI int64_t offset(const Dim3 &p) const {
    const Dim3 q = p - origin_;
    return q.x + pitch_.x * (q.y + pitch_.y * q.z);
  }
  STENCIL_HDI T &operator[](const Dim3 &p) const { return raw_[offset(p)]; }
  STENCIL_HDI T *ptr() const { return raw_; }
  STENCIL_HDI const Dim3 &origin() const { return origin_; }
  STENCIL_HDI const Dim3 &pitch() const { return pitch_; }
};

// round x up to a multiple of a (a power of two)
STENCIL_HDI int64_t next_align_of(int64_t x, int64_t a) { return (x + a - 1) & ~(a - 1); }
STENCIL_HDI int64_t round_up(int64_t x, int64_t a) { return ((x + a - 1) / a) * a; }
