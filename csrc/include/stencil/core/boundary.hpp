#pragma once
// Boundary: per-direction global boundary condition of the distributed grid.
// Parity: reference include/stencil/boundary.hpp:7-25 (a per-direction "periodic" flag, default periodic). The
// reference never consults it and only supports periodic grids (src/stencil.cu:155-157). Here it is honoured by
// DistributedDomain::set_boundary: across a non-periodic face of the global grid no halo message is planned, so
// the outermost halo cells keep whatever the application writes there (Dirichlet / Neumann conditions are the
// application's business, exactly like the compute kernels).
#include "stencil/core/geometry.hpp"

class Boundary {
  DirectionMap<bool> periodic_;

public:
  // default: periodic in every direction
  Boundary() {
    for (int z = -1; z <= 1; ++z)
      for (int y = -1; y <= 1; ++y)
        for (int x = -1; x <= 1; ++x) periodic_.at_dir(x, y, z) = true;
  }
  static Boundary periodic() { return Boundary(); }
  // per-axis flags (both faces of an axis share the flag)
  static Boundary axes(bool px, bool py, bool pz) {
    Boundary b;
    b.set_axis(0, px);
    b.set_axis(1, py);
    b.set_axis(2, pz);
    return b;
  }
  static Boundary none() { return axes(false, false, false); }

  void set_face(int x, int y, int z, bool p) { periodic_.at_dir(x, y, z) = p; }
  void set_axis(int axis, bool p) {
    const int d[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    periodic_.at_dir(d[axis][0], d[axis][1], d[axis][2]) = p;
    periodic_.at_dir(-d[axis][0], -d[axis][1], -d[axis][2]) = p;
  }
  // face flag (one of x/y/z non-zero)
  bool face_periodic(int x, int y, int z) const { return periodic_.at_dir(x, y, z); }
  // a direction (face, edge or corner) wraps iff every face it crosses is periodic
  bool wraps(const Dim3 &dir) const {
    if (dir.x != 0 && !periodic_.at_dir(int(dir.x), 0, 0)) return false;
    if (dir.y != 0 && !periodic_.at_dir(0, int(dir.y), 0)) return false;
    if (dir.z != 0 && !periodic_.at_dir(0, 0, int(dir.z))) return false;
    return true;
  }
  bool all_periodic() const {
    for (int a = -1; a <= 1; a += 2)
      if (!face_periodic(a, 0, 0) || !face_periodic(0, a, 0) || !face_periodic(0, 0, a)) return false;
    return true;
  }
  // does stepping from sub-domain `idx` along `dir` stay inside a grid of `dim` sub-domains, or wrap periodically?
  bool reachable(const Dim3 &idx, const Dim3 &dir, const Dim3 &dim) const {
    const int64_t p[3] = {idx.x + dir.x, idx.y + dir.y, idx.z + dir.z};
    const int64_t n[3] = {dim.x, dim.y, dim.z};
    const int64_t dd[3] = {dir.x, dir.y, dir.z};
    for (int a = 0; a < 3; ++a) {
      if (p[a] >= 0 && p[a] < n[a]) continue;
      const int s = int(dd[a]);
      const bool per = a == 0 ? face_periodic(s, 0, 0) : (a == 1 ? face_periodic(0, s, 0) : face_periodic(0, 0, s));
      if (!per) return false;
    }
    return true;
  }
  bool operator==(const Boundary &o) const { return periodic_ == o.periodic_; }
};
