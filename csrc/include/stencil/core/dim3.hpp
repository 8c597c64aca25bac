#pragma once
// Dim3: 3-vector of int64 used for sizes, positions and directions.
// Parity: reference include/stencil/dim3.hpp:25-309 (arithmetic, lexicographic <, wrap, flatten).
// Deliberately NOT reproduced: the reference's max() bug (dim3.hpp:65-71) and
// operator!= bug (dim3.hpp:203).
#include <cstdint>
#include <ostream>

#include "stencil/core/hd.hpp"

struct Dim3 {
  int64_t x, y, z;

  STENCIL_HDI constexpr Dim3() : x(0), y(0), z(0) {}
  STENCIL_HDI constexpr Dim3(int64_t x_, int64_t y_, int64_t z_) : x(x_), y(y_), z(z_) {}

  STENCIL_HDI int64_t flatten() const { return x * y * z; }
  STENCIL_HDI bool all_gt(int64_t v) const { return x > v && y > v && z > v; }
  STENCIL_HDI bool all_lt(int64_t v) const { return x < v && y < v && z < v; }
  STENCIL_HDI bool any_gt(int64_t v) const { return x > v || y > v || z > v; }
  STENCIL_HDI bool any_lt(int64_t v) const { return x < v || y < v || z < v; }
  STENCIL_HDI bool all_ge(const Dim3 &o) const { return x >= o.x && y >= o.y && z >= o.z; }
  STENCIL_HDI bool all_lt(const Dim3 &o) const { return x < o.x && y < o.y && z < o.z; }

  STENCIL_HDI int64_t max() const {
    int64_t m = x > y ? x : y;
    return m > z ? m : z;
  }
  STENCIL_HDI int64_t min() const {
    int64_t m = x < y ? x : y;
    return m < z ? m : z;
  }

  // periodic wrap into [0, lims)
  STENCIL_HDI Dim3 wrap(const Dim3 &lims) const {
    Dim3 r = *this;
    r.x = ((r.x % lims.x) + lims.x) % lims.x;
    r.y = ((r.y % lims.y) + lims.y) % lims.y;
    r.z = ((r.z % lims.z) + lims.z) % lims.z;
    return r;
  }

  STENCIL_HDI Dim3 operator+(const Dim3 &o) const { return Dim3(x + o.x, y + o.y, z + o.z); }
  STENCIL_HDI Dim3 operator-(const Dim3 &o) const { return Dim3(x - o.x, y - o.y, z - o.z); }
  STENCIL_HDI Dim3 operator*(const Dim3 &o) const { return Dim3(x * o.x, y * o.y, z * o.z); }
  STENCIL_HDI Dim3 operator/(const Dim3 &o) const { return Dim3(x / o.x, y / o.y, z / o.z); }
  STENCIL_HDI Dim3 operator%(const Dim3 &o) const { return Dim3(x % o.x, y % o.y, z % o.z); }
  STENCIL_HDI Dim3 operator+(int64_t s) const { return Dim3(x + s, y + s, z + s); }
  STENCIL_HDI Dim3 operator-(int64_t s) const { return Dim3(x - s, y - s, z - s); }
  STENCIL_HDI Dim3 operator*(int64_t s) const { return Dim3(x * s, y * s, z * s); }
  STENCIL_HDI Dim3 operator/(int64_t s) const { return Dim3(x / s, y / s, z / s); }
  STENCIL_HDI Dim3 operator-() const { return Dim3(-x, -y, -z); }
  STENCIL_HDI Dim3 &operator+=(const Dim3 &o) {
    x += o.x;
    y += o.y;
    z += o.z;
    return *this;
  }
  STENCIL_HDI Dim3 &operator-=(const Dim3 &o) {
    x -= o.x;
    y -= o.y;
    z -= o.z;
    return *this;
  }

  STENCIL_HDI bool operator==(const Dim3 &o) const { return x == o.x && y == o.y && z == o.z; }
  STENCIL_HDI bool operator!=(const Dim3 &o) const { return !(*this == o); }
  // lexicographic, x most significant (matches reference dim3.hpp:78-92 ordering of messages)
  STENCIL_HDI bool operator<(const Dim3 &o) const {
    if (x != o.x) return x < o.x;
    if (y != o.y) return y < o.y;
    return z < o.z;
  }
  STENCIL_HDI bool operator>(const Dim3 &o) const { return o < *this; }
  STENCIL_HDI bool operator<=(const Dim3 &o) const { return !(o < *this); }
};

inline std::ostream &operator<<(std::ostream &os, const Dim3 &d) {
  return os << "[" << d.x << "," << d.y << "," << d.z << "]";
}

// index of a direction in {-1,0,1}^3 as 0..26 (x fastest)
STENCIL_HDI int dir_index(const Dim3 &d) { return int((d.x + 1) + 3 * (d.y + 1) + 9 * (d.z + 1)); }
STENCIL_HDI Dim3 dir_from_index(int i) { return Dim3(i % 3 - 1, (i / 3) % 3 - 1, i / 9 - 1); }
