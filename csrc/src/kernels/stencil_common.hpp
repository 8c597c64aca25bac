#pragma once

#include <algorithm>
#include <cmath>
#include <vector>
// Private device helpers shared by the 7-point stencil kernels (stencil7.hip, stencil7x2.hip).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "stencil/domain/local_domain.hpp"
#include "stencil/kernels/stencil_ops.hpp"

namespace stencil {

template <typename T> struct Vec16;
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef double nd2 __attribute__((ext_vector_type(2)));
template <> struct Vec16<float> {
  using type = float4;
  using native = nf4;
  static constexpr int N = 4;
};
template <> struct Vec16<double> {
  using type = double2;
  using native = nd2;
  static constexpr int N = 2;
};

template <typename T> __device__ __forceinline__ T vget(const typename Vec16<T>::type &v, int i);
template <> __device__ __forceinline__ float vget<float>(const float4 &v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
template <> __device__ __forceinline__ double vget<double>(const double2 &v, int i) { return i == 0 ? v.x : v.y; }

template <typename T> __device__ __forceinline__ T shfl_up1(T v);
template <typename T> __device__ __forceinline__ T shfl_down1(T v);
template <> __device__ __forceinline__ float shfl_up1<float>(float v) { return __shfl_up(v, 1, 64); }
template <> __device__ __forceinline__ float shfl_down1<float>(float v) { return __shfl_down(v, 1, 64); }
template <> __device__ __forceinline__ double shfl_up1<double>(double v) { return __shfl_up(v, 1, 64); }
template <> __device__ __forceinline__ double shfl_down1<double>(double v) { return __shfl_down(v, 1, 64); }

template <typename T> struct StencilArgs {
  const T *src; // raw [0,0,0] of curr
  T *dst;       // raw [0,0,0] of next
  int64_t px, pxy;
  int lox, loy, loz, hix, hiy, hiz; // region, raw coordinates
  int x0;                           // raw x of chunk 0 (16-B aligned in memory)
  int nchunks;                      // chunks covering [x0, hix)
  int rawYm1;                       // clamp for row loads
  int rawZm1;                       // clamp for the deep z prefetch
  int zc;                           // planes per block
  int gx, gy, gz;                   // logical grid
  int seg;                          // stencil7x2: 1 = balanced (column, plane) segments over gridDim.x blocks, 2 = lockstep
                                    // z parts, 3 = lockstep rounds of whole columns
  int zparts;                       // stencil7x2 lockstep: z parts per column (4 = quarters)
  int zrounds;                      // stencil7x2 lockstep rounds (seg 3)
  int xfast;                        // stencil7x2: 1 = column index x-major (x-adjacent columns on one XCD)
  int remap;                        // stencil7x2: 1 = XCD-aware block remap
  // spheres, raw coordinates
  int hx, hy, hz, cx, cy, cz;
  int r1sq; // (radius+1)^2, 0 = disabled
  int sphr;  // the sphere radius (stencil7x3: which chunks a sphere can reach)
  int sphchunk; // stencil7x3: test each sphere only on the chunks it can reach
  // halo forwarding (FWD kernels): cells within fwm[a] of the low face send along -a, within fwp[a] of the high
  // face along +a; the receiving halo cell of direction k = (dx+1) + 3(dy+1) + 9(dz+1) is at (own output address +
  // fd[k]) for every k set in fmask (receivers with our pitches; the rest is copied after the kernel)
  int nt;   // non-temporal output stores (block-uniform)
  int flip; // reverse every block's z-march direction (alternated per step, see StencilTune::alternateZ)
  int fwm[3], fwp[3];
  uint32_t fmask;
  int64_t fd[27];
  // in-kernel periodic wrap (fused pairs, StencilTune::wrap): along every axis set in wrapm the sub-domain is its
  // own neighbour, so a cell outside [wlo, wlo + wn) is read at its periodic image inside instead of from a halo
  // the exchange would have to copy first (raw coordinates)
  int wrapm;
  int wlo[3], wn[3];
  // boundary-plane publication (StencilTune::publish): output planes z < pubLo or z >= pubHi (raw) count into *pub
  unsigned long long *pub;
  int pubLo, pubHi;
  // fused triples: rows past the region's y end store here instead of being skipped (same memory ops on every path)
  char *sink;
  int early; // stencil7x2 row / col2: publish the src and u1 rows right after the u1 update, not before the barrier
  unsigned long long *clk; // stencil7x3 measurement: per-block start / end wall clock (null: off)
};

// periodic image of raw coordinate c along axis ax (identity unless the axis wraps)
template <typename T> __device__ __forceinline__ int wrap_coord(const StencilArgs<T> &a, int c, int ax) {
  if (!((a.wrapm >> ax) & 1)) return c;
  int d = (c - a.wlo[ax]) % a.wn[ax];
  if (d < 0) d += a.wn[ax];
  return a.wlo[ax] + d;
}


// bijective XCD-aware remap: consecutive logical ids land on the same XCD (blocks b, b+8, ... share one)
__device__ __forceinline__ uint32_t xcd_remap(uint32_t hw, uint32_t n) {
  const uint32_t q = n / 8, r = n % 8, xcd = hw % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + hw / 8;
}

// x / 6 rounded to nearest-even, bit-identical to IEEE division. fp32: two FMAs around the reciprocal (verified
// exhaustively over all 2^32 inputs for |x| >= 2^-100; the subnormal-result range takes the true division).
template <typename T> __device__ __forceinline__ T div6(T x) { return x / T(6); }
template <> __device__ __forceinline__ float div6<float>(float x) {
  constexpr float c = 1.0f / 6.0f;
  const float q0 = x * c;
  const float r = __builtin_fmaf(-q0, 6.0f, x);
  float q = __builtin_fmaf(r, c, q0);
  if (__builtin_expect(__builtin_fabsf(x) < 0x1p-100f, 0)) q = x / 6.0f;
  return q;
}
// fp64: the same corrected quotient (see div6v in stencil_wave.hpp), true division below 2^-960
template <> __device__ __forceinline__ double div6<double>(double x) {
  constexpr double c = 1.0 / 6.0;
  const double q0 = x * c;
  const double r = __builtin_fma(-q0, 6.0, x);
  double q = __builtin_fma(r, c, q0);
  if (__builtin_expect(__builtin_fabs(x) < 0x1p-960, 0)) q = x / 6.0;
  return q;
}


// kernel arguments for one quantity of one sub-domain over `region` (global coordinates)
template <typename T>
inline StencilArgs<T> make_args(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind,
                                const Spheres &sph) {
  StencilArgs<T> a{};
  const Dim3 org = dom.accessor_origin();
  const Dim3 p = dom.pitch(qi);
  a.src = static_cast<const T *>(dom.curr_data(qi));
  a.dst = static_cast<T *>(dom.next_data(qi));
  a.px = p.x;
  a.pxy = p.x * p.y;
  const Rect3 r(region.lo - org, region.hi - org);
  a.lox = int(r.lo.x);
  a.loy = int(r.lo.y);
  a.loz = int(r.lo.z);
  a.hix = int(r.hi.x);
  a.hiy = int(r.hi.y);
  a.hiz = int(r.hi.z);
  a.rawYm1 = int(dom.raw_size().y - 1);
  a.rawZm1 = int(dom.raw_size().z - 1);
  const Rect3 cr = dom.get_compute_region();
  const Dim3 ce = cr.extent();
  a.wlo[0] = int(cr.lo.x - org.x);
  a.wlo[1] = int(cr.lo.y - org.y);
  a.wlo[2] = int(cr.lo.z - org.z);
  a.wn[0] = int(ce.x);
  a.wn[1] = int(ce.y);
  a.wn[2] = int(ce.z);
  if (kind == StencilKind::Jacobi && sph.enabled) {
    a.hx = int(sph.hot.x - org.x);
    a.hy = int(sph.hot.y - org.y);
    a.hz = int(sph.hot.z - org.z);
    a.cx = int(sph.cold.x - org.x);
    a.cy = int(sph.cold.y - org.y);
    a.cz = int(sph.cold.z - org.z);
    a.r1sq = int((sph.radius + 1) * (sph.radius + 1));
  }
  return a;
}


// z-chunk length for a z-marching launch of `cols` block columns over nz planes with `resident` blocks resident
// at once: maximise (useful planes / planes read) x (blocks / block slots of the rounds), i.e. balance the warm-up
// planes each chunk re-reads (`warm`) against a partly empty last round of blocks.
inline int pick_zchunk(int64_t cols, int nz, int64_t resident, int warm, int minZc = 8) {
  int best = nz;
  double bestEff = -1;
  for (int gz = 1; gz <= nz; ++gz) {
    const int zc = (nz + gz - 1) / gz;
    if (zc < minZc && gz > 1) break;
    const int64_t blocks = cols * ((nz + zc - 1) / zc);
    const int64_t rounds = (blocks + resident - 1) / resident;
    const double fill = double(blocks) / double(rounds * resident);
    const double eff = fill * double(zc) / double(zc + warm);
    if (eff > bestEff + 1e-9) {
      bestEff = eff;
      best = zc;
    }
  }
  return best;
}

// Jacobi: sum order +x,-x,+y,-y,+z,-z (reference bin/jacobi3d.cu:72-83); Astaroth: -x,-y,-z,+x,+y,+z
// (bin/astaroth_sim.cu:72-81); then the exact /6
template <typename T, int KIND>
__device__ __forceinline__ T sum6(T vpx, T vmx, T vpy, T vmy, T vpz, T vmz) {
  T val;
  if (KIND == 0) {
    val = T(0) + vpx;
    val += vmx;
    val += vpy;
    val += vmy;
    val += vpz;
    val += vmz;
  } else {
    val = T(0) + vmx;
    val += vmy;
    val += vmz;
    val += vpx;
    val += vpy;
    val += vpz;
  }
  return div6<T>(val);
}

// per-row-group z part boundaries (plane offsets from the region's first plane) of a lockstep fused sweep (pairs,
// triples): the Jacobi blocks whose rows cross the hot / cold spheres pay the per-cell sphere tests on those planes
// and set the sweep's time (profiles/r5/ak), so the host cuts each group's z range by plane weights
// 1 + w * (the group's rows crossing a sphere at that plane) / rows; on = 0: equal parts
constexpr int kZPartMaxCols = 256, kZPartMaxParts = 4, kLeftMaxBlocks = 256;
struct ZPartBounds {
  int on;
  uint16_t zb[kZPartMaxCols][kZPartMaxParts - 1];
  // lon: block lb's second segment is the leftover (column, plane) slice [l0[lb], l1[lb]) (offsets from the first
  // leftover column), marching down when bit lb of ldir is set (balance_leftover / lockstep_leftover); 0: equal slices
  int lon;
  uint16_t l0[kLeftMaxBlocks], l1[kLeftMaxBlocks];
  uint32_t ldir[kLeftMaxBlocks / 32];
};

// plane weights of row group grp (blocks holding rows [yblk - rowOff, yblk - rowOff + rows), yblk = loy + YO grp):
// 1 + w * (levels of the group's rows crossing a sphere at that plane) / (sum of levels); false: no sphere crossed
template <typename T>
inline bool sphere_group_weights(std::vector<double> &wz, const StencilArgs<T> &a, int64_t grp, int rows, int YO,
                                 int rowOff, float w) {
  const int nz = a.hiz - a.loz;
  wz.assign(static_cast<size_t>(nz), 1.0);
  if (a.r1sq <= 0 || w <= 0) return false;
  auto isqrt_below = [](int d) { // largest h >= 0 with h * h < d (d > 0)
    int h = int(std::sqrt(double(d - 1)));
    while (h > 0 && h * h > d - 1) --h;
    while ((h + 1) * (h + 1) <= d - 1) ++h;
    return h;
  };
  double levelSum = 0;
  for (int r = 0; r < rows; ++r) levelSum += std::min(std::min(r, rows - 1 - r), rowOff);
  bool any = false;
  const int yblk = a.loy + YO * int(grp);
  for (int r = 0; r < rows; ++r) {
    const int y = yblk - rowOff + r;
    const double lw = w * std::min(std::min(r, rows - 1 - r), rowOff) / levelSum;
    if (lw <= 0) continue;
    const int cy[2] = {a.hy, a.cy}, cz[2] = {a.hz, a.cz};
    for (int sidx = 0; sidx < 2; ++sidx) {
      const int d = a.r1sq - (y - cy[sidx]) * (y - cy[sidx]);
      if (d <= 0) continue;
      const int h = isqrt_below(d);
      for (int z = std::max(a.loz, cz[sidx] - h); z <= std::min(a.hiz - 1, cz[sidx] + h); ++z) {
        wz[static_cast<size_t>(z - a.loz)] += lw;
        any = true;
      }
    }
  }
  return any;
}
// fills b for cm row groups of YO output rows, each block holding rows [yblk - rowOff, yblk - rowOff + rows); a row
// r that crosses a sphere adds w * levels(r) / (sum of levels) to the plane's weight, levels(r) = the number of
// updates the row's wave computes per step (min(r, rows - 1 - r, rowOff): the edge rows only load)
template <typename T>
inline void sphere_part_bounds(ZPartBounds &b, const StencilArgs<T> &a, int64_t cm, int P, int rows, int YO,
                               int rowOff, float w) {
  b.on = 0;
  const int nz = a.hiz - a.loz;
  if (a.r1sq <= 0 || w <= 0 || P < 2 || P > kZPartMaxParts || cm > kZPartMaxCols || nz >= 65536) return;
  std::vector<double> wz;
  bool any = false;
  for (int64_t col = 0; col < cm; ++col) {
    any = sphere_group_weights(wz, a, col, rows, YO, rowOff, w) || any;
    double total = 0;
    for (double v : wz) total += v;
    double acc = 0;
    int q = 1;
    for (int z = 0; z < nz && q < P; ++z) {
      acc += wz[static_cast<size_t>(z)];
      while (q < P && acc >= total * q / P) b.zb[col][(q++) - 1] = uint16_t(z + 1);
    }
    while (q < P) b.zb[col][(q++) - 1] = uint16_t(nz);
  }
  b.on = any ? 1 : 0;
}

// Second segments levelled against the lockstep parts (seg 2: block lb = q * cm + col runs part q of column col, then
// a slice of the leftover columns [cm, ncols)). Equal slices leave every block of a sphere-crossing row group its
// parts' extra steps on top: at 512^3 (P = 4 parts of 64 groups + 22 leftover groups) those 72 blocks ran ~20 us
// longer than the rest and set the sweep (profiles/r6/r6r). Here block lb takes leftover planes in order until
// main(lb) + its slice reaches a common level T, the least T that places every plane (bisection): planes weighted as
// the parts are (sphere_group_weights; leftover steps cost `leftw`), each segment start `warm` steps. Columns are
// numbered y-major in x strips (row group = col % gy); b.zb as filled by sphere_part_bounds (b.on), else equal parts.
// block costs (steps) of the lockstep parts: warm + the part's plane weights, block lb = q * cm + col
template <typename T>
inline std::vector<double> lockstep_part_costs(const ZPartBounds &b, const StencilArgs<T> &a, int64_t cm, int P,
                                               int64_t gy, int rows, int YO, int rowOff, float w, int warm) {
  const int64_t nz = a.hiz - a.loz;
  std::vector<double> wz, mainc(static_cast<size_t>(int64_t(P) * cm));
  for (int64_t col = 0; col < cm; ++col) {
    const int64_t grp = col % gy;
    sphere_group_weights(wz, a, grp, rows, YO, rowOff, w);
    for (int q = 0; q < P; ++q) {
      int64_t zlo = int64_t(q) * nz / P, zhi = int64_t(q + 1) * nz / P;
      if (b.on && grp < kZPartMaxCols) {
        zlo = q > 0 ? b.zb[grp][q - 1] : 0;
        zhi = q + 1 < P ? b.zb[grp][q] : nz;
      }
      double c = warm;
      for (int64_t z = zlo; z < zhi; ++z) c += wz[static_cast<size_t>(z)];
      mainc[static_cast<size_t>(q * cm + col)] = c;
    }
  }
  return mainc;
}

// returns the level (steps of the longest block), or -1 where the slices cannot be tabled (b.lon = 0: equal slices)
template <typename T>
inline double balance_leftover(ZPartBounds &b, const StencilArgs<T> &a, int64_t nb, int64_t cm, int P, int64_t ncols,
                               int64_t gy, int rows, int YO, int rowOff, float w, int warm, double leftw) {
  b.lon = 0;
  const int64_t nz = a.hiz - a.loz;
  const int64_t LW = (ncols - cm) * nz;
  if (LW <= 0 || LW > 65535 || nb > kLeftMaxBlocks || nb != int64_t(P) * cm || cm <= 0 || gy <= 0) return -1;
  const std::vector<double> mainc = lockstep_part_costs(b, a, cm, P, gy, rows, YO, rowOff, w, warm);
  std::vector<double> wz, lw(static_cast<size_t>(LW));
  double total = 0;
  for (int64_t col = cm; col < ncols; ++col) {
    sphere_group_weights(wz, a, col % gy, rows, YO, rowOff, w);
    for (int64_t z = 0; z < nz; ++z) {
      lw[static_cast<size_t>((col - cm) * nz + z)] = leftw * wz[static_cast<size_t>(z)];
      total += leftw * wz[static_cast<size_t>(z)];
    }
  }
  // greedy fill at level T; true when every leftover plane found a block
  auto fill = [&](double lvl, bool set) {
    int64_t i = 0;
    for (int64_t lb = 0; lb < nb; ++lb) {
      const int64_t i0 = i;
      double c = mainc[static_cast<size_t>(lb)];
      for (bool started = false; i < LW; started = true, ++i) {
        const double add = lw[static_cast<size_t>(i)] + ((!started || i % nz == 0) ? warm : 0);
        if (c + add > lvl) break;
        c += add;
      }
      if (set) {
        b.l0[lb] = uint16_t(i0);
        b.l1[lb] = uint16_t(i);
      }
    }
    return i >= LW;
  };
  double lo = *std::max_element(mainc.begin(), mainc.end()), hi = lo + total + double(warm) * double(ncols - cm + 1);
  if (!fill(hi, false)) return -1;
  for (int it = 0; it < 48 && hi - lo > 1e-3; ++it) {
    const double mid = 0.5 * (lo + hi);
    (fill(mid, false) ? hi : lo) = mid;
  }
  fill(hi, true);
  // directions as with equal slices: the second segment marches opposite to the block's part
  for (int64_t lb = 0; lb < nb; ++lb) {
    const uint32_t bit = 1u << (lb % 32);
    if (((lb / cm) & 1) == 0)
      b.ldir[lb / 32] |= bit;
    else
      b.ldir[lb / 32] &= ~bit;
  }
  b.lon = 1;
  return hi;
}

// The leftover row groups as a second lockstep phase: G = ncols - cm groups of K parts each, part k of every group
// covering the same planes and marching the same way, so y-adjacent groups' blocks (consecutive blocks, one XCD)
// share their halo rows in L2 as the first phase's parts do; unsynchronised slices re-read them (Astaroth 512^3:
// 241.6 us per triple with 22 leftover groups in slices vs 224.0 with one 2-row group, profiles/r6/r6ab). Blocks are
// binned by the cost of their lockstep part: the latest nb - K G get no second segment, the next G latest the
// thinnest part, ..., and the part heights level every bin at a common T (at least minPlanes planes per part).
// Returns T over the best K (or -1: not tabled; b.lon = 0).
template <typename T>
inline double lockstep_leftover(ZPartBounds &b, const StencilArgs<T> &a, int64_t nb, int64_t cm, int P, int64_t ncols,
                                int64_t gy, int rows, int YO, int rowOff, float w, int warm, int minPlanes) {
  b.lon = 0;
  const int64_t nz = a.hiz - a.loz, G = ncols - cm;
  if (G <= 0 || G * nz > 65535 || nb > kLeftMaxBlocks || nb != int64_t(P) * cm || cm <= 0 || gy <= 0) return -1;
  const std::vector<double> mainc = lockstep_part_costs(b, a, cm, P, gy, rows, YO, rowOff, w, warm);
  std::vector<int64_t> order(static_cast<size_t>(nb));
  for (int64_t i = 0; i < nb; ++i) order[static_cast<size_t>(i)] = i;
  std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
    return mainc[static_cast<size_t>(x)] > mainc[static_cast<size_t>(y)];
  });
  auto late_of = [&](int64_t idle, int64_t k) { return mainc[static_cast<size_t>(order[static_cast<size_t>(idle + k * G)])]; };
  double bestT = -1;
  std::vector<int64_t> bestH;
  int64_t bestK = 0;
  for (int64_t K = 1; K * G <= nb && K * minPlanes <= nz; ++K) {
    const int64_t idle = nb - K * G;
    // bins k = 0 .. K-1, latest first. Parts for the `used` earliest bins (the latest dropped first while a level
    // would leave them fewer than minPlanes planes): h_k = T - late_k - warm, sum h_k = nz
    std::vector<int64_t> h(static_cast<size_t>(K), 0);
    bool ok = false;
    for (int64_t used = K; used >= 1 && !ok; --used) {
      double sum = double(nz);
      for (int64_t k = K - used; k < K; ++k) sum += late_of(idle, k) + warm;
      const double t = sum / double(used);
      if (t - late_of(idle, K - used) - warm < minPlanes) continue;
      int64_t acc = 0;
      for (int64_t k = K - used; k < K; ++k) {
        h[static_cast<size_t>(k)] = std::max<int64_t>(minPlanes, int64_t(std::floor(t - late_of(idle, k) - warm)));
        acc += h[static_cast<size_t>(k)];
      }
      // integer heights summing to nz: pad the earliest bins first, trim the latest first
      for (int64_t k = K - 1; acc < nz; k = k > K - used ? k - 1 : K - 1, ++acc) ++h[static_cast<size_t>(k)];
      for (int64_t k = K - used, guard = 0; acc > nz && guard < 4 * nz; k = k + 1 < K ? k + 1 : K - used, ++guard)
        if (h[static_cast<size_t>(k)] > minPlanes) {
          --h[static_cast<size_t>(k)];
          --acc;
        }
      ok = acc == nz;
    }
    if (!ok) continue;
    double worst = 0;
    for (int64_t i = 0; i < idle; ++i) worst = std::max(worst, mainc[static_cast<size_t>(order[static_cast<size_t>(i)])]);
    for (int64_t k = 0; k < K; ++k)
      worst = std::max(worst, late_of(idle, k) + (h[static_cast<size_t>(k)] ? double(h[static_cast<size_t>(k)] + warm) : 0.0));
    if (bestT < 0 || worst < bestT - 1e-9) {
      bestT = worst;
      bestH = h;
      bestK = K;
    }
  }
  if (bestT < 0) return -1;
  const int64_t K = bestK, idle = nb - K * G;
  for (int64_t i = 0; i < idle; ++i) {
    const int64_t lb = order[static_cast<size_t>(i)];
    b.l0[lb] = b.l1[lb] = 0;
  }
  // parts in z from the earliest bin (the tallest part) on, alternating direction; a bin's blocks take the groups
  // in block order (y-adjacent groups on consecutive blocks)
  int64_t z0 = 0;
  for (int64_t k = K - 1; k >= 0; --k) {
    std::vector<int64_t> bin(order.begin() + idle + k * G, order.begin() + idle + (k + 1) * G);
    std::sort(bin.begin(), bin.end());
    const int64_t hk = bestH[static_cast<size_t>(k)];
    const uint32_t down = ((K - 1 - k) & 1) != 0;
    for (int64_t g = 0; g < G; ++g) {
      const int64_t lb = bin[static_cast<size_t>(g)];
      b.l0[lb] = uint16_t(g * nz + z0);
      b.l1[lb] = uint16_t(g * nz + z0 + hk);
      const uint32_t bit = 1u << (lb % 32);
      b.ldir[lb / 32] = down ? (b.ldir[lb / 32] | bit) : (b.ldir[lb / 32] & ~bit);
    }
    z0 += hk;
  }
  b.lon = 1;
  return bestT;
}

// hot/cold sphere override of the Jacobi app at raw (x, y, z)
template <typename T>
__device__ __forceinline__ T sphere_fix(const StencilArgs<T> &a, int x, int y, int z, T v) {
  if (a.r1sq <= 0) return v;
  const int dh = (x - a.hx) * (x - a.hx) + (y - a.hy) * (y - a.hy) + (z - a.hz) * (z - a.hz);
  const int dc = (x - a.cx) * (x - a.cx) + (y - a.cy) * (y - a.cy) + (z - a.cz) * (z - a.cz);
  return dh < a.r1sq ? T(1) : (dc < a.r1sq ? T(0) : v);
}

} // namespace stencil
