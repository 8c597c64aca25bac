// Two fused 7-point steps per sweep (temporal blocking): dst = S(S(src)) on a region, for gfx950.
//
// A Jacobi/Astaroth step reads 4 B and writes 4 B per cell: at HBM speed that is the whole cost. Fusing two steps
// into one z-march reads the field once and writes it once per TWO steps, and needs one halo exchange of depth 2
// (faces 2, edges 1: the 25-point footprint of S o S) per two steps instead of two exchanges of depth 1. This is
// the "halo multiplier" / deep-halo item of the reference's future-work list (README.md:218-220), built for CDNA4:
//
//   block  = NW waves stacked in y, TY rows per wave, one 64-lane column of 16-B x-chunks (as stencil7_lds_kernel)
//   step t = output plane z (z-march direction dz = +-1):
//     1. load src plane z+3dz (lookahead)          (rows of this wave + the block-edge waves' halo rows)
//     2. u1 = S(src) at plane z+dz for own rows    (y-neighbours of the wave's top/bottom rows: LDS; block edges:
//        plus u1 one cell outside the wave's x range (edge lanes) and, in the block-edge waves, one row outside
//        the block in y (the block halo u1 row), so S(u1) never needs another block's u1
//     3. u2 = S(u1) at plane z from the register window u1(z-dz), u1(z), u1(z+dz) + LDS y-neighbours
//     4. publish src/u1 boundary rows for the next step (double-buffered LDS, one barrier per step)
// Summation order and the /6 are the single-step kernel's, and every u1 value is computed exactly as the single
// step computes it, so S(S(src)) is bitwise equal to two sequential single steps (tests compare with torch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "stencil/rt/hip_check.hpp"
#include "stencil_common.hpp"

namespace stencil {

template <typename T, int TY, int NW, int KIND, bool REMAP, int MINW>
__global__ __launch_bounds__(64 * NW, MINW) void stencil7x2_kernel(StencilArgs<T> a) {
  using VT = typename Vec16<T>::type;
  using NV = typename Vec16<T>::native;
  constexpr int V = Vec16<T>::N;
  static_assert(NW >= 2, "block-edge waves must differ");
  __shared__ VT cs[2][2 * NW][64];     // src rows of plane z+2dz: wave w's top row at 2w, bottom row at 2w+1
  __shared__ VT us[2][2 * NW + 2][64]; // u1 rows of plane z+dz: same slots + block halo rows (2NW above, 2NW+1 below)
  __shared__ T ce[2][2 * NW][2];       // src edge scalars of the published rows: [0] at x-1 (lane 0), [1] at x+V

  const uint32_t nb = uint32_t(a.gx) * a.gy * a.gz;
  const uint32_t lb = REMAP ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int bz = int(lb % uint32_t(a.gz));
  const int by = int((lb / uint32_t(a.gz)) % uint32_t(a.gy));
  const int bx = int(lb / (uint32_t(a.gz) * a.gy));
  const int lane = threadIdx.x;
  const int w = int(threadIdx.y);
  const int c = bx * 64 + lane;
  const bool cvalid = c < a.nchunks;
  const int cl = cvalid ? c : a.nchunks - 1;
  const int xb = a.x0 + cl * V;
  const int yblk = a.loy + NW * TY * by;
  const int ybase = yblk + TY * w;
  const int zs = a.loz + bz * a.zc;
  const int ze = min(zs + a.zc, a.hiz);
  if (yblk >= a.hiy || zs >= ze) return; // block-uniform
  const bool down = ((bz & 1) != 0) != (a.flip != 0);
  const int dz = down ? -1 : 1;
  const int z0 = down ? ze - 1 : zs;
  const int nzs = ze - zs;

  const bool edgeL = lane == 0;
  const bool edgeR = lane == 63 || c + 1 >= a.nchunks;
  const bool fullX = xb >= a.lox && xb + V <= a.hix;
  const bool top = w == 0, bot = w == NW - 1;
  const bool edgeWave = top || bot;
  const int hy1 = top ? yblk - 1 : yblk + NW * TY;     // block halo row (top: above, bottom: below)
  const int hy2 = top ? yblk - 2 : yblk + NW * TY + 1; // its outer neighbour
  const int slotTop = 2 * w, slotBot = 2 * w + 1;
  const int slotAbove = top ? 0 : 2 * (w - 1) + 1, slotBelow = bot ? 0 : 2 * (w + 1);

  auto rowp = [&](int y, int z) -> const T * {
    y = y < 0 ? 0 : (y > a.rawYm1 ? a.rawYm1 : y);
    return a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
  };
  auto ld = [&](const T *p) -> VT { return *reinterpret_cast<const VT *>(p); };
  auto toVT = [&](const T (&o)[V]) -> VT {
    VT v;
    if constexpr (V == 4) {
      v.x = o[0];
      v.y = o[1];
      v.z = o[2];
      v.w = o[3];
    } else {
      v.x = o[0];
      v.y = o[1];
    }
    return v;
  };
  // Sphere membership of a row (raw y, plane P): the y/z part of both squared distances, computed once per row;
  // `hit` is false for the ~97% of rows no sphere reaches, so their cells skip the per-cell test (wave-uniform).
  struct RowSph {
    int dh, dc;
    bool hit;
  };
  auto row_sph = [&](int y, int P) -> RowSph {
    RowSph r{0, 0, false};
    if (KIND == 0 && a.r1sq > 0) {
      r.dh = (y - a.hy) * (y - a.hy) + (P - a.hz) * (P - a.hz);
      r.dc = (y - a.cy) * (y - a.cy) + (P - a.cz) * (P - a.cz);
      r.hit = r.dh < a.r1sq || r.dc < a.r1sq;
    }
    return r;
  };
  auto fix = [&](const RowSph &rs, int x, T v) -> T {
    if (KIND != 0 || !rs.hit) return v;
    const bool hot = (x - a.hx) * (x - a.hx) + rs.dh < a.r1sq;
    const bool cold = (x - a.cx) * (x - a.cx) + rs.dc < a.r1sq;
    return hot ? T(1) : (cold ? T(0) : v);
  };
  // S at the row chunk `cm` (plane P, raw row y): x-neighbours by shuffles (+ the edge scalars at the wave edges)
  auto apply_row = [&](const VT &cm, const VT &up, const VT &dn, const VT &zp, const VT &zm, T eL, T eR,
                       const RowSph &rs, T (&o)[V]) {
    const T sl = shfl_up1<T>(vget<T>(cm, V - 1));
    const T sr = shfl_down1<T>(vget<T>(cm, 0));
    const T left = edgeL ? eL : sl;
    const T right = edgeR ? eR : sr;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const T vpx = e < V - 1 ? vget<T>(cm, e + 1) : right;
      const T vmx = e > 0 ? vget<T>(cm, e - 1) : left;
      o[e] = sum6<T, KIND>(vpx, vmx, vget<T>(dn, e), vget<T>(up, e), vget<T>(zp, e), vget<T>(zm, e));
    }
    if (rs.hit) {
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] = fix(rs, xb + e, o[e]);
    }
  };

  // ---- register windows (one plane of lookahead: every load has a whole step to land) ----
  VT C0[TY], C1[TY], C2[TY], C3[TY]; // src own rows, planes z, z+dz, z+2dz, z+3dz (in flight)
  T C0L[TY], C0R[TY], C1L[TY], C1R[TY], C2L[TY], C2R[TY], C3L[TY], C3R[TY]; // src at x-1 / x+V (edge lanes)
  T C1LL[TY], C1RR[TY], C2LL[TY], C2RR[TY]; // src at x-2 / x+V+1, planes z+dz, z+2dz (in flight)
  VT H0, H1, H2, H3;                        // block halo row hy1, planes z .. z+3dz (edge waves)
  T H1L = T(0), H1R = T(0), H2L = T(0), H2R = T(0), H3L = T(0), H3R = T(0);
  VT G1, G2;                                // row hy2, planes z+dz, z+2dz (in flight)
  VT Ub[TY], Uc[TY], Ua[TY]; // u1 own rows, planes z-dz, z, z+dz
  T UcL[TY], UcR[TY], UaL[TY], UaR[TY];
  VT uH; // u1 block halo row, plane z+dz (edge waves)

  auto zcl = [&](int zz) { return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz); };
  auto load_row = [&](int y, int z, VT &v, T &L, T &R) {
    const T *p = rowp(y, z);
    v = ld(p);
    L = edgeL ? p[-1] : T(0);
    R = edgeR ? p[V] : T(0);
  };
  auto load_outer = [&](int y, int z, T &LL, T &RR) {
    const T *p = rowp(y, z);
    LL = edgeL ? p[-2] : T(0);
    RR = edgeR ? p[V + 1] : T(0);
  };

  // ---- warm-up: src planes z0-2dz .. z0; the loop starts two planes early (u1 only) ----
  {
    const int zA = z0 - 2 * dz, zB = z0 - dz, zC = z0;
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      load_row(ybase + i, zA, C0[i], C0L[i], C0R[i]);
      load_row(ybase + i, zB, C1[i], C1L[i], C1R[i]);
      load_row(ybase + i, zC, C2[i], C2L[i], C2R[i]);
      load_outer(ybase + i, zB, C1LL[i], C1RR[i]);
    }
    if (edgeWave) {
      H0 = ld(rowp(hy1, zA));
      load_row(hy1, zB, H1, H1L, H1R);
      load_row(hy1, zC, H2, H2L, H2R);
      G1 = ld(rowp(hy2, zB));
    }
    cs[0][slotTop][lane] = C1[0];
    cs[0][slotBot][lane] = C1[TY - 1];
    if (edgeL) {
      ce[0][slotTop][0] = C1L[0];
      ce[0][slotBot][0] = C1L[TY - 1];
    }
    if (edgeR) {
      ce[0][slotTop][1] = C1R[0];
      ce[0][slotBot][1] = C1R[TY - 1];
    }
    __syncthreads();
  }

  int buf = 0;
  for (int t = -2; t < nzs; ++t) {
    const int z = z0 + t * dz;
    const int P = z + dz;
    // 1. lookahead loads: src plane z+3dz (+ the outer x scalars and the hy2 row of plane z+2dz)
    {
      const int z3 = zcl(z + 3 * dz), z2 = zcl(z + 2 * dz);
#pragma unroll
      for (int i = 0; i < TY; ++i) {
        load_row(ybase + i, z3, C3[i], C3L[i], C3R[i]);
        load_outer(ybase + i, z2, C2LL[i], C2RR[i]);
      }
      if (edgeWave) {
        load_row(hy1, z3, H3, H3L, H3R);
        G2 = ld(rowp(hy2, z2));
      }
    }
    // src rows at plane z+dz next to this wave's rows (other waves through LDS, block edges from registers)
    const VT cAbove = top ? H1 : cs[buf][slotAbove][lane];
    const VT cBelow = bot ? H1 : cs[buf][slotBelow][lane];
    const T cAboveL = top ? H1L : (edgeL ? ce[buf][slotAbove][0] : T(0));
    const T cAboveR = top ? H1R : (edgeR ? ce[buf][slotAbove][1] : T(0));
    const T cBelowL = bot ? H1L : (edgeL ? ce[buf][slotBelow][0] : T(0));
    const T cBelowR = bot ? H1R : (edgeR ? ce[buf][slotBelow][1] : T(0));

    // 2. u1 at plane z+dz: own rows, their wave-edge scalars, and the block halo row
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      const int y = ybase + i;
      const VT &up = i == 0 ? cAbove : C1[i - 1];
      const VT &dn = i == TY - 1 ? cBelow : C1[i + 1];
      T o[V];
      const RowSph rs = row_sph(y, P);
      apply_row(C1[i], up, dn, down ? C0[i] : C2[i], down ? C2[i] : C0[i], C1L[i], C1R[i], rs, o);
      Ua[i] = toVT(o);
      // one cell outside the wave's x range (meaningful on the edge lanes only; branch-free elsewhere)
      const T upL = i == 0 ? cAboveL : C1L[i - 1], upR = i == 0 ? cAboveR : C1R[i - 1];
      const T dnL = i == TY - 1 ? cBelowL : C1L[i + 1], dnR = i == TY - 1 ? cBelowR : C1R[i + 1];
      UaL[i] = fix(rs, xb - 1,
                   sum6<T, KIND>(vget<T>(C1[i], 0), C1LL[i], dnL, upL, down ? C0L[i] : C2L[i], down ? C2L[i] : C0L[i]));
      UaR[i] = fix(rs, xb + V,
                   sum6<T, KIND>(C1RR[i], vget<T>(C1[i], V - 1), dnR, upR, down ? C0R[i] : C2R[i],
                                 down ? C2R[i] : C0R[i]));
    }
    if (edgeWave) { // u1 of the block halo row (one row outside the block)
      T o[V];
      const VT &up = top ? G1 : C1[TY - 1];
      const VT &dn = top ? C1[0] : G1;
      apply_row(H1, up, dn, down ? H0 : H2, down ? H2 : H0, H1L, H1R, row_sph(hy1, P), o);
      uH = toVT(o);
    }

    // 3. u2 at plane z (once the u1 window is full)
    if (t >= 0) {
      const VT uAbove = top ? us[buf][2 * NW][lane] : us[buf][slotAbove][lane];
      const VT uBelow = bot ? us[buf][2 * NW + 1][lane] : us[buf][slotBelow][lane];
#pragma unroll
      for (int i = 0; i < TY; ++i) {
        const int y = ybase + i;
        const VT &up = i == 0 ? uAbove : Uc[i - 1];
        const VT &dn = i == TY - 1 ? uBelow : Uc[i + 1];
        T o[V];
        apply_row(Uc[i], up, dn, down ? Ub[i] : Ua[i], down ? Ua[i] : Ub[i], UcL[i], UcR[i], row_sph(y, z), o);
        if (cvalid && y < a.hiy) {
          T *dp = a.dst + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
          if (fullX) {
            NV v;
#pragma unroll
            for (int e = 0; e < V; ++e) v[e] = o[e];
            __builtin_nontemporal_store(v, reinterpret_cast<NV *>(dp));
          } else {
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (xb + e >= a.lox && xb + e < a.hix) dp[e] = o[e];
          }
        }
      }
    }

    // 4. publish src plane z+2dz and u1 plane z+dz boundary rows for the next step
    const int nbuf = buf ^ 1;
    cs[nbuf][slotTop][lane] = C2[0];
    cs[nbuf][slotBot][lane] = C2[TY - 1];
    if (edgeL) {
      ce[nbuf][slotTop][0] = C2L[0];
      ce[nbuf][slotBot][0] = C2L[TY - 1];
    }
    if (edgeR) {
      ce[nbuf][slotTop][1] = C2R[0];
      ce[nbuf][slotBot][1] = C2R[TY - 1];
    }
    us[nbuf][slotTop][lane] = Ua[0];
    us[nbuf][slotBot][lane] = Ua[TY - 1];
    if (top) us[nbuf][2 * NW][lane] = uH;
    if (bot) us[nbuf][2 * NW + 1][lane] = uH;
    __syncthreads();
    buf = nbuf;

    // 5. rotate the windows
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      C0[i] = C1[i];
      C0L[i] = C1L[i];
      C0R[i] = C1R[i];
      C1[i] = C2[i];
      C1L[i] = C2L[i];
      C1R[i] = C2R[i];
      C2[i] = C3[i];
      C2L[i] = C3L[i];
      C2R[i] = C3R[i];
      C1LL[i] = C2LL[i];
      C1RR[i] = C2RR[i];
      Ub[i] = Uc[i];
      Uc[i] = Ua[i];
      UcL[i] = UaL[i];
      UcR[i] = UaR[i];
    }
    H0 = H1;
    H1 = H2;
    H2 = H3;
    H1L = H2L;
    H1R = H2R;
    H2L = H3L;
    H2R = H3R;
    G1 = G2;
  }
}

// ---------------------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------------------
static int64_t x2_resident_blocks(const void *kernel, int threads) {
  static std::map<const void *, int64_t> cache;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int dev = 0, perCU = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kernel, threads, 0) != hipSuccess || perCU <= 0) perCU = 1;
  (void)hipGetLastError();
  const int64_t r = int64_t(perCU) * cus;
  cache[kernel] = r;
  return r;
}

bool stencil7x2_supported(const LocalDomain &dom, int64_t qi) {
  if (dom.backend() != Backend::Device) return false;
  const DType dt = dom.dtype(qi);
  const int64_t es = dom.elem_size(qi);
  if (!(dt == DType::F32 || dt == DType::F64 || (dt == DType::Bytes && (es == 4 || es == 8)))) return false;
  const Radius &r = dom.radius();
  for (int s = -1; s <= 1; s += 2)
    if (r.x(s) < 2 || r.y(s) < 2 || r.z(s) < 2) return false;
  const int64_t V = 16 / es;
  const Dim3 p = dom.pitch(qi);
  const int64_t lox = r.x(-1), hix = lox + dom.size().x;
  const int64_t nchunks = (hix - lox + V - 1) / V;
  const bool aligned = (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.curr_data(qi)) + lox * es) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.next_data(qi)) + lox * es) % 16 == 0) &&
                       (p.x * es) % 16 == 0;
  // the edge lanes read x-2 and x+V+1 of their chunk: stay inside the padded row
  return aligned && lox - 2 + dom.pad_x(qi) >= 0 && lox + nchunks * V + 1 < p.x - dom.pad_x(qi);
}

template <typename T, int KIND, int TY, int NW, int MINW>
static void apply_x2_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                       const StencilTune &tune) {
  constexpr int V = Vec16<T>::N;
  StencilArgs<T> a = make_args<T>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  const int rxm = int(dom.radius().x(-1));
  const int off = ((a.lox - rxm) % V + V) % V;
  a.x0 = a.lox - off;
  a.nchunks = (a.hix - a.x0 + V - 1) / V;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = (a.nchunks + 63) / 64;
  a.gy = (ny + NW * TY - 1) / (NW * TY);
  const void *kern = tune.xcdRemap ? (const void *)stencil7x2_kernel<T, TY, NW, KIND, true, MINW>
                                   : (const void *)stencil7x2_kernel<T, TY, NW, KIND, false, MINW>;
  int zc = tune.zchunk;
  if (zc <= 0) {
    // one round of resident blocks; each block re-reads 2 warm-up planes, so keep z-chunks >= 16 planes
    const int64_t cols = int64_t(a.gx) * a.gy;
    const int64_t nzc = std::max<int64_t>(1, x2_resident_blocks(kern, 64 * NW) / cols);
    zc = int(std::max<int64_t>(16, (nz + nzc - 1) / nzc));
  }
  a.zc = zc;
  a.gz = (nz + zc - 1) / zc;
  const uint32_t blocks = uint32_t(a.gx) * a.gy * a.gz;
  dom.set_device();
  if (tune.xcdRemap)
    hipLaunchKernelGGL((stencil7x2_kernel<T, TY, NW, KIND, true, MINW>), dim3(blocks), dim3(64, NW), 0, stream, a);
  else
    hipLaunchKernelGGL((stencil7x2_kernel<T, TY, NW, KIND, false, MINW>), dim3(blocks), dim3(64, NW), 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

void stencil7x2_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune) {
  if (region.empty()) return;
  STENCIL_REQUIRE(stencil7x2_supported(dom, qi),
                  "two-step stencil needs a device fp32/fp64 quantity, face radii >= 2 and the aligned layout");
  const Rect3 cr = dom.get_compute_region();
  STENCIL_REQUIRE(cr.contains(region.lo) && region.hi.x <= cr.hi.x && region.hi.y <= cr.hi.y && region.hi.z <= cr.hi.z,
                  "stencil region " << region << " outside compute region " << cr);
  const bool f32 = dom.elem_size(qi) == 4;
  const bool jac = kind == StencilKind::Jacobi;
  // shapes (rows per lane, waves per block, min waves/SIMD): 1x8 keeps everything in registers at 6 waves/SIMD;
  // 2x4 at 3 waves/SIMD; 2x8 at 4 (spills)
  // shape = rows per lane x waves per block (min waves/SIMD): 1x8 (4), 1x16 (4), 2x4 (3); x2nw == 2 selects 2x4 (2)
  const int shape = tune.x2ty == 2 ? (tune.x2nw == 2 ? 3 : 1) : (tune.x2nw == 16 ? 2 : 0);
#define X2_LAUNCH(TT, K)                                                                                           \
  do {                                                                                                             \
    if (shape == 0)                                                                                                \
      apply_x2_t<TT, K, 1, 8, 4>(dom, qi, region, sph, stream, tune);                                              \
    else if (shape == 1)                                                                                           \
      apply_x2_t<TT, K, 2, 4, 3>(dom, qi, region, sph, stream, tune);                                              \
    else if (shape == 2)                                                                                           \
      apply_x2_t<TT, K, 1, 16, 4>(dom, qi, region, sph, stream, tune);                                             \
    else                                                                                                           \
      apply_x2_t<TT, K, 2, 4, 2>(dom, qi, region, sph, stream, tune);                                              \
  } while (0)
  if (f32) {
    if (jac)
      X2_LAUNCH(float, 0);
    else
      X2_LAUNCH(float, 1);
  } else {
    if (jac)
      X2_LAUNCH(double, 0);
    else
      X2_LAUNCH(double, 1);
  }
#undef X2_LAUNCH
}

} // namespace stencil
