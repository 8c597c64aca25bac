// Three fused 7-point steps per sweep (deeper temporal blocking): dst = S(S(S(src))) on a whole periodic sub-domain
// of 512-cell fp32 rows, for gfx950.
//
// The fused pair (stencil7x2_row_kernel) streams the field once per two steps and sits at ~95 % of a plain copy of
// its access shape (205 us per 512^3 pair, profiles/r4/j). Fewer bytes per step is the only lever left: a triple
// reads and writes the field once per THREE steps (8 B per cell per 3 steps instead of per 2). What it costs is
// compute on the redundant y halo: a block of NW waves (one 512-cell row each, x-neighbours and the x wrap by DPP lane
// rotates exactly as in the pair kernel) holds NW src rows and computes
//   u1 on the inner NW-2 rows, u2 on the inner NW-4, u3 (the output) on the inner NW-6,
// so 12 waves write 6 rows with 10 + 8 + 6 = 24 row updates (4 per output row for 3 steps: 1.33 per row and step,
// against the pair's (10 + 8) / 8 / 2 = 1.13). The round-2 lab triple computed all three levels on every row
// (6 updates per output row: 2.0 per row and step) and was VALU-bound at 134 us per step (profiles/r2/r2_lab_triple.txt);
// here each wave only computes the levels some output row needs (wave-uniform), as the pair's edge waves do.
//
//   step t (output plane z, march direction dz):
//     1. issue the load of src plane z + (3 + PF) dz                      (PF planes of lookahead in registers)
//     2. u1 at plane z+2dz from the src window + LDS y-neighbours          (waves 1 .. NW-2)
//     3. u2 at plane z+dz  from the u1 window (z, z+dz, z+2dz) + LDS       (waves 2 .. NW-3)
//     4. u3 at plane z     from the u2 window (z-dz, z, z+dz) + LDS        (waves 3 .. NW-4)  -> store
//     5. publish src(z+3dz), u1(z+2dz), u2(z+dz) rows into the other LDS buffer; one barrier
// A segment of nzs output planes runs nzs + 4 steps (u3 needs u2 one plane behind it, which needs u1 two planes
// behind). Summation order, the exact /6 and the spheres are those of the single step, every intermediate value is
// computed exactly as the single step computes it (y and z by in-kernel wrap), so S(S(S(src))) is bitwise equal to
// three single steps (tests/test_gpu.py::test_temporal3_matches_three_single_steps).
// Reference step being fused: bin/jacobi3d.cu:40-87 (Jacobi), bin/astaroth_sim.cu:65-83 (Astaroth).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/rt/hip_check.hpp"
#include "stencil_common.hpp"
#include "stencil_wave.hpp"

namespace stencil {

// (column, plane) segment of a block: lockstep parts as the fused pairs (x2_segments), kept local to this file
struct X3Seg {
  uint32_t s, e, s2, e2;
  bool odd;
};
__device__ __forceinline__ X3Seg x3_segments(const StencilArgs<float> &a, uint32_t lb, uint32_t nb, uint32_t ncols,
                                             uint32_t nzt) {
  X3Seg r{0, 0, 0, 0, false};
  if (a.seg == 2) {
    const uint32_t P = uint32_t(a.zparts), cm = nb / P;
    const uint32_t qq = lb / cm, col = lb % cm;
    r.s = col * nzt + qq * nzt / P;
    r.e = col * nzt + (qq + 1) * nzt / P;
    r.odd = (qq & 1) != 0;
    const uint64_t LW = uint64_t(ncols - cm) * nzt;
    r.s2 = cm * nzt + uint32_t(uint64_t(lb) * LW / nb);
    r.e2 = cm * nzt + uint32_t(uint64_t(lb + 1) * LW / nb);
  } else {
    const uint64_t W = uint64_t(ncols) * nzt;
    r.s = uint32_t(uint64_t(lb) * W / nb);
    r.e = uint32_t(uint64_t(lb + 1) * W / nb);
    r.odd = (lb & 1) != 0;
  }
  return r;
}

// Row of the block handled by wave w when StencilArgs::xfast (reused here as "permute waves") is set. The row roles
// carry unequal work (row 0 / 11: none, 1 / 10: u1, 2 / 9: u1 + u2, 3..8: all three); with waves dealt to the four
// SIMDs round-robin (w % 4) or in runs of three (w / 3) this table gives every SIMD 6 row updates per step either way,
// where the identity gives 3 / 9 / 9 / 3 in the second case.
__device__ __forceinline__ int x3_row_of_wave(int w, int permute) {
  constexpr int kPerm[12] = {1, 9, 6, 8, 2, 10, 4, 0, 5, 3, 11, 7};
  return permute ? kPerm[w] : w;
}

template <int NW, int PF, int KIND>
__global__ __launch_bounds__(64 * NW, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void
stencil7x3_row_kernel(StencilArgs<float> a) {
  using T = float;
  using NV = nf4;
  constexpr int V = 4, H = 2, HS = 64 * V;
  constexpr int YO = NW - 6; // output rows per block
  constexpr int NC = 3 + PF; // src planes in registers
  static_assert(NW == 12, "12 waves: 3 per SIMD (168 VGPRs), 3 x 48 KiB of LDS");
  __shared__ NV cs[2][NW][H][64]; // src rows  (plane z+3dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows   (plane z+2dz at publish)
  __shared__ NV vs[2][NW][H][64]; // u2 rows   (plane z+dz at publish)

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(x3_row_of_wave(int(threadIdx.y), a.xfast)); // the wave's block row
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  const X3Seg sg = x3_segments(a, lb, nb, uint32_t(a.gy), nzt);
  const bool lane0 = lane == 0, lane63 = lane == 63;
  // wave-uniform roles: u1 feeds u2 on rows 2..NW-3, which feed u3 on rows 3..NW-4
  const bool needU1 = w >= 1 && w < NW - 1, needU2 = w >= 2 && w < NW - 2, needU3 = w >= 3 && w < NW - 3;
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1;
  const int xb = a.lox + lane * V; // chunk h at xb + h * HS
  const int zwn = a.wn[2], zwlo = a.wlo[2], zwhi = a.wlo[2] + a.wn[2];
  auto zcl = [&](int zz) {
    zz += zz < zwlo ? zwn : 0;
    zz -= zz >= zwhi ? zwn : 0;
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  bool odd = sg.odd;
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t s = pass == 0 ? sg.s : sg.s2;
    const uint32_t e = pass == 0 ? sg.e : sg.e2;
    while (s < e) { // block-uniform
      const uint32_t by = s / nzt;
      const int zo = int(s - by * nzt);
      const int nzs = int(min(nzt - uint32_t(zo), e - s));
      s += uint32_t(nzs);
      const int zs = a.loz + zo;
      const int ze = zs + nzs;
      const bool down = odd != (a.flip != 0);
      odd = !odd;
      const int yblk = a.loy + YO * int(by);
      const int y = yblk - 3 + w;
      if (yblk >= a.hiy) continue;
      const bool outRow = needU3 && y < a.hiy;
      int yw = y < a.wlo[1] ? y + a.wn[1] : (y >= a.wlo[1] + a.wn[1] ? y - a.wn[1] : y);
      yw = yw < 0 ? 0 : (yw > a.rawYm1 ? a.rawYm1 : yw);
      const uint32_t rowoff = uint32_t((yw * int64_t(a.px) + xb) * int64_t(sizeof(T)));
      const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));
      auto planep = [&](int zz) -> const char * {
        return reinterpret_cast<const char *>(a.src + int64_t(zcl(zz)) * a.pxy);
      };
      // spheres (Jacobi): row-level distance terms of plane P, then per-cell tests only on rows that cross a sphere
      struct RowSph {
        int dh, dc;
        bool hit;
      };
      auto row_sph = [&](int P) -> RowSph {
        RowSph r{0, 0, false};
        if (KIND == 0 && a.r1sq > 0) {
          r.dh = (y - a.hy) * (y - a.hy) + (P - a.hz) * (P - a.hz);
          r.dc = (y - a.cy) * (y - a.cy) + (P - a.cz) * (P - a.cz);
          r.hit = r.dh < a.r1sq || r.dc < a.r1sq;
        }
        return r;
      };
      // S of the wave's row (both chunks), x-neighbours and the periodic x wrap by lane rotates
      auto apply_row = [&](const NV(&cm)[H], const NV(&up)[H], const NV(&dn)[H], const NV(&zp)[H], const NV(&zm)[H],
                           const RowSph &rs, NV(&o)[H]) {
        T r3[H], l0[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          r3[h] = rot_prev(cm[h][V - 1]);
          l0[h] = rot_next(cm[h][0]);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const T left = lane0 ? r3[(h + H - 1) % H] : r3[h];
          const T right = lane63 ? l0[(h + 1) % H] : l0[h];
          NV vpx, vmx;
#pragma unroll
          for (int k = 0; k < V; ++k) {
            vpx[k] = k < V - 1 ? cm[h][k + 1] : right;
            vmx[k] = k > 0 ? cm[h][k - 1] : left;
          }
          o[h] = div6v<T, NV, V>(sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]));
        }
        if (KIND == 0 && rs.hit) {
#pragma unroll
          for (int h = 0; h < H; ++h)
#pragma unroll
            for (int k = 0; k < V; ++k) {
              const int x = xb + h * HS + k;
              const bool hot = (x - a.hx) * (x - a.hx) + rs.dh < a.r1sq;
              const bool cold = (x - a.cx) * (x - a.cx) + rs.dc < a.r1sq;
              o[h][k] = hot ? T(1) : (cold ? T(0) : o[h][k]);
            }
        }
      };

      auto march = [&](auto downTag) {
        constexpr bool DOWN = decltype(downTag)::value;
        constexpr int dz = DOWN ? -1 : 1;
        const int z0 = DOWN ? ze - 1 : zs;
        NV C[NC][H];
        NV U1a[H], U1b[H], U1c[H]; // u1 at planes z+2dz (new), z, z+dz
        NV U2a[H], U2b[H], U2c[H]; // u2 at planes z+dz (new), z-dz, z
        auto load_row = [&](int zz, int k) {
          const char *b = planep(zz) + rowoff;
#pragma unroll
          for (int h = 0; h < H; ++h) C[k][h] = *reinterpret_cast<const NV *>(b + h * HS * int(sizeof(T)));
        };
        // step t = -4 starts with src planes z+dz .. z+(NC-1)dz, z = z0 - 4dz, and the src row of its u1 plane
        // (z+2dz: slot 1) published
        {
          const int zw = z0 - 3 * dz;
#pragma unroll
          for (int k = 0; k < NC - 1; ++k) load_row(zw + k * dz, k);
#pragma unroll
          for (int h = 0; h < H; ++h) {
            cs[0][w][h][lane] = C[1][h];
            U1b[h] = U1c[h] = U2b[h] = U2c[h] = C[1][h]; // never read before the warm-up overwrites them
          }
          __syncthreads();
        }
        int buf = 0;
        int t = -4;
        auto step = [&](auto phase) -> bool {
          constexpr int k = decltype(phase)::value;
          // slots: s0 = plane z+dz, s1 = z+2dz, s2 = z+3dz; sn receives z + NC dz (it held plane z)
          constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
          if (t >= nzs) return false;
          const int z = z0 + t * dz;
          load_row(z + NC * dz, sn);
          if (needU1) {
            NV cA[H], cB[H];
#pragma unroll
            for (int h = 0; h < H; ++h) {
              cA[h] = cs[buf][wA][h][lane];
              cB[h] = cs[buf][wB][h][lane];
            }
            apply_row(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], row_sph(z + 2 * dz), U1a);
          }
          if (t >= -2 && needU2) {
            NV uA[H], uB[H];
#pragma unroll
            for (int h = 0; h < H; ++h) {
              uA[h] = us[buf][wA][h][lane];
              uB[h] = us[buf][wB][h][lane];
            }
            apply_row(U1c, uA, uB, DOWN ? U1b : U1a, DOWN ? U1a : U1b, row_sph(z + dz), U2a);
          }
          if (t >= 0 && needU3) {
            NV vA[H], vB[H], o[H];
#pragma unroll
            for (int h = 0; h < H; ++h) {
              vA[h] = vs[buf][wA][h][lane];
              vB[h] = vs[buf][wB][h][lane];
            }
            apply_row(U2c, vA, vB, DOWN ? U2b : U2a, DOWN ? U2a : U2b, row_sph(z), o);
            if (outRow) {
              char *dp = reinterpret_cast<char *>(a.dst + int64_t(z) * a.pxy) + outoff;
#pragma unroll
              for (int h = 0; h < H; ++h) {
                NV *q = reinterpret_cast<NV *>(dp + h * HS * int(sizeof(T)));
                if (a.nt)
                  __builtin_nontemporal_store(o[h], q);
                else
                  *q = o[h];
              }
            }
          }
          const int nbuf = buf ^ 1;
#pragma unroll
          for (int h = 0; h < H; ++h) {
            cs[nbuf][w][h][lane] = C[s2][h];
            if (needU1) us[nbuf][w][h][lane] = U1a[h];
            if (needU2) vs[nbuf][w][h][lane] = U2a[h];
          }
          __syncthreads();
          buf = nbuf;
#pragma unroll
          for (int h = 0; h < H; ++h) {
            U1b[h] = U1c[h];
            U1c[h] = U1a[h];
            U2b[h] = U2c[h];
            U2c[h] = U2a[h];
          }
          ++t;
          return true;
        };
        while (run_phases(step, std::make_integer_sequence<int, NC>{})) {
        }
      };
      if (down)
        march(std::true_type{});
      else
        march(std::false_type{});
    } // segments
  }   // passes
}

template <int NW, int PF, int KIND>
__global__ __launch_bounds__(64 * NW, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void
stencil7x3s_row_kernel(StencilArgs<float> a) {
  using T = float;
  using NV = nf4;
  constexpr int V = 4, H = 2, HS = 64 * V;
  constexpr int YO = NW - 6; // output rows per block
  constexpr int NC = 3 + PF; // src planes in registers (z+2dz .. z+4dz and PF in flight)
  static_assert(NW == 12, "12 waves: 3 per SIMD (168 VGPRs), 3 x 48 KiB of LDS");
  __shared__ NV cs[2][NW][H][64]; // src rows  (plane z+3dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows   (plane z+2dz at publish)
  __shared__ NV vs[2][NW][H][64]; // u2 rows   (plane z+dz at publish)

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(x3_row_of_wave(int(threadIdx.y), a.xfast)); // the wave's block row
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  const X3Seg sg = x3_segments(a, lb, nb, uint32_t(a.gy), nzt);
  const bool lane0 = lane == 0, lane63 = lane == 63;
  // wave-uniform roles: u1 feeds u2 on rows 2..NW-3, which feed u3 on rows 3..NW-4
  const bool needU1 = w >= 1 && w < NW - 1, needU2 = w >= 2 && w < NW - 2, needU3 = w >= 3 && w < NW - 3;
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1;
  const int xb = a.lox + lane * V; // chunk h at xb + h * HS
  const int zwn = a.wn[2], zwlo = a.wlo[2], zwhi = a.wlo[2] + a.wn[2];
  auto zcl = [&](int zz) {
    zz += zz < zwlo ? zwn : 0;
    zz -= zz >= zwhi ? zwn : 0;
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  bool odd = sg.odd;
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t s = pass == 0 ? sg.s : sg.s2;
    const uint32_t e = pass == 0 ? sg.e : sg.e2;
    while (s < e) { // block-uniform
      const uint32_t by = s / nzt;
      const int zo = int(s - by * nzt);
      const int nzs = int(min(nzt - uint32_t(zo), e - s));
      s += uint32_t(nzs);
      const int zs = a.loz + zo;
      const int ze = zs + nzs;
      const bool down = odd != (a.flip != 0);
      odd = !odd;
      const int yblk = a.loy + YO * int(by);
      const int y = yblk - 3 + w;
      if (yblk >= a.hiy) continue;
      const bool outRow = needU3 && y < a.hiy;
      int yw = y < a.wlo[1] ? y + a.wn[1] : (y >= a.wlo[1] + a.wn[1] ? y - a.wn[1] : y);
      yw = yw < 0 ? 0 : (yw > a.rawYm1 ? a.rawYm1 : yw);
      const uint32_t rowoff = uint32_t((yw * int64_t(a.px) + xb) * int64_t(sizeof(T)));
      const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));
      auto planep = [&](int zz) -> const char * {
        return reinterpret_cast<const char *>(a.src + int64_t(zcl(zz)) * a.pxy);
      };
      // spheres (Jacobi): row-level distance terms of plane P, then per-cell tests only on rows that cross a sphere
      struct RowSph {
        int dh, dc;
        bool hit;
      };
      auto row_sph = [&](int P) -> RowSph {
        RowSph r{0, 0, false};
        if (KIND == 0 && a.r1sq > 0) {
          r.dh = (y - a.hy) * (y - a.hy) + (P - a.hz) * (P - a.hz);
          r.dc = (y - a.cy) * (y - a.cy) + (P - a.cz) * (P - a.cz);
          r.hit = r.dh < a.r1sq || r.dc < a.r1sq;
        }
        return r;
      };
      // S of the wave's row (both chunks), x-neighbours and the periodic x wrap by lane rotates
      auto apply_row = [&](const NV(&cm)[H], const NV(&up)[H], const NV(&dn)[H], const NV(&zp)[H], const NV(&zm)[H],
                           const RowSph &rs, NV(&o)[H]) {
        T r3[H], l0[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          r3[h] = rot_prev(cm[h][V - 1]);
          l0[h] = rot_next(cm[h][0]);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const T left = lane0 ? r3[(h + H - 1) % H] : r3[h];
          const T right = lane63 ? l0[(h + 1) % H] : l0[h];
          NV vpx, vmx;
#pragma unroll
          for (int k = 0; k < V; ++k) {
            vpx[k] = k < V - 1 ? cm[h][k + 1] : right;
            vmx[k] = k > 0 ? cm[h][k - 1] : left;
          }
          o[h] = div6v<T, NV, V>(sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]));
        }
        if (KIND == 0 && rs.hit) {
#pragma unroll
          for (int h = 0; h < H; ++h)
#pragma unroll
            for (int k = 0; k < V; ++k) {
              const int x = xb + h * HS + k;
              const bool hot = (x - a.hx) * (x - a.hx) + rs.dh < a.r1sq;
              const bool cold = (x - a.cx) * (x - a.cx) + rs.dc < a.r1sq;
              o[h][k] = hot ? T(1) : (cold ? T(0) : o[h][k]);
            }
        }
      };
      // the same update without branches: the FMA-corrected /6 for every cell, no sphere test, and the smallest |sum|
      // returned, so the caller can redo the row exactly (apply_row) in the rare case it is below 2^-100 (zero sums
      // included) -- three of these per step form one basic block the compiler can interleave
      auto row_fast = [&](const NV(&cm)[H], const NV(&up)[H], const NV(&dn)[H], const NV(&zp)[H], const NV(&zm)[H],
                          NV(&o)[H]) -> T {
        T r3[H], l0[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          r3[h] = rot_prev(cm[h][V - 1]);
          l0[h] = rot_next(cm[h][0]);
        }
        T m = T(1);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const T left = lane0 ? r3[(h + H - 1) % H] : r3[h];
          const T right = lane63 ? l0[(h + 1) % H] : l0[h];
          NV vpx, vmx;
#pragma unroll
          for (int k = 0; k < V; ++k) {
            vpx[k] = k < V - 1 ? cm[h][k + 1] : right;
            vmx[k] = k > 0 ? cm[h][k - 1] : left;
          }
          const NV sm = sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]);
          const NV c = NV(1.0f / 6.0f), six = NV(6.0f);
          const NV q0 = sm * c;
          o[h] = __builtin_elementwise_fma(__builtin_elementwise_fma(-q0, six, sm), c, q0);
          m = __builtin_fminf(m, __builtin_fminf(__builtin_fminf(__builtin_fabsf(sm[0]), __builtin_fabsf(sm[1])),
                                                 __builtin_fminf(__builtin_fabsf(sm[2]), __builtin_fabsf(sm[3]))));
        }
        return m;
      };
      auto sphere_row = [&](const RowSph &rs, NV(&o)[H]) {
        if (KIND == 0 && rs.hit) {
#pragma unroll
          for (int h = 0; h < H; ++h)
#pragma unroll
            for (int k = 0; k < V; ++k) {
              const int x = xb + h * HS + k;
              const bool hot = (x - a.hx) * (x - a.hx) + rs.dh < a.r1sq;
              const bool cold = (x - a.cx) * (x - a.cx) + rs.dc < a.r1sq;
              o[h][k] = hot ? T(1) : (cold ? T(0) : o[h][k]);
            }
        }
      };

      // staggered levels: step t computes u1 at z+3dz, u2 at z+dz and u3 at z-dz (the output), each from values of
      // EARLIER steps only (registers and the LDS rows published one step before), so the three row updates of a
      // step are independent and interleave in one basic block; warm-up 6 steps (u2 from t = -2, u3 from t = 1)
      auto march = [&](auto downTag) {
        constexpr bool DOWN = decltype(downTag)::value;
        constexpr int dz = DOWN ? -1 : 1;
        const int z0 = DOWN ? ze - 1 : zs;
        NV C[NC][H];
        NV U1[4][H]; // u1 at planes z, z+dz, z+2dz, z+3dz (new)
        NV U2[4][H]; // u2 at planes z-2dz, z-dz, z, z+dz (new)
        auto load_row = [&](int zz, int k) {
          const char *b = planep(zz) + rowoff;
#pragma unroll
          for (int h = 0; h < H; ++h) C[k][h] = *reinterpret_cast<const NV *>(b + h * HS * int(sizeof(T)));
        };
        {
          const int zw = z0 - 3 * dz; // z + 2dz at t = -5
#pragma unroll
          for (int k = 0; k < NC - 1; ++k) load_row(zw + k * dz, k);
#pragma unroll
          for (int h = 0; h < H; ++h) {
            cs[0][w][h][lane] = C[1][h];
#pragma unroll
            for (int j = 0; j < 4; ++j) U1[j][h] = U2[j][h] = C[1][h]; // overwritten before any use
          }
          __syncthreads();
        }
        int buf = 0;
        int t = -5;
        const int wl = needU3 ? 3 : (needU2 ? 2 : (needU1 ? 1 : 0)); // levels this wave computes
        auto step = [&](auto phase) -> bool {
          constexpr int k = decltype(phase)::value;
          // slots: s0 = plane z+2dz, s1 = z+3dz, s2 = z+4dz; sn receives z + (NC+1) dz (it held plane z+dz)
          constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
          if (t > nzs) return false;
          const int z = z0 + t * dz;
          load_row(z + (NC + 1) * dz, sn);
          const int lv = min(wl, t >= 1 ? 3 : (t >= -2 ? 2 : 1)); // wave-uniform
          // neighbour rows of the three levels (this step's LDS buffer, published by the previous step)
          auto nb_rows = [&](NV(&lds)[2][NW][H][64], NV(&A)[H], NV(&B)[H]) {
#pragma unroll
            for (int h = 0; h < H; ++h) {
              A[h] = lds[buf][wA][h][lane];
              B[h] = lds[buf][wB][h][lane];
            }
          };
          NV o3[H];
          T m = T(1);
          {
            NV cA[H], cB[H], uA[H], uB[H], vA[H], vB[H];
            if (lv == 3) { // one basic block: u3 at z-dz, u2 at z+dz, u1 at z+3dz, independent of each other
              nb_rows(vs, vA, vB);
              const T m3 = row_fast(U2[1], vA, vB, DOWN ? U2[0] : U2[2], DOWN ? U2[2] : U2[0], o3);
              nb_rows(us, uA, uB);
              const T m2 = row_fast(U1[1], uA, uB, DOWN ? U1[0] : U1[2], DOWN ? U1[2] : U1[0], U2[3]);
              nb_rows(cs, cA, cB);
              const T m1 = row_fast(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], U1[3]);
              m = __builtin_fminf(m3, __builtin_fminf(m2, m1));
            } else if (lv == 2) {
              nb_rows(us, uA, uB);
              nb_rows(cs, cA, cB);
              const T m2 = row_fast(U1[1], uA, uB, DOWN ? U1[0] : U1[2], DOWN ? U1[2] : U1[0], U2[3]);
              const T m1 = row_fast(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], U1[3]);
              m = __builtin_fminf(m2, m1);
            } else if (lv == 1) {
              nb_rows(cs, cA, cB);
              m = row_fast(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], U1[3]);
            }
          }
          const RowSph rs1 = row_sph(z + 3 * dz), rs2 = row_sph(z + dz), rs3 = row_sph(z - dz);
          // wave-uniform (the redo's lane rotates need every lane active): some lane has a |sum| below 2^-100
          if (__builtin_expect(__builtin_amdgcn_ballot_w64(m < 0x1p-100f) != 0, 0)) {
            // some |sum| below 2^-100 (or zero): redo this step's rows with the exact quotient for those cells
            NV A[H], B[H];
            if (lv >= 3) {
              nb_rows(vs, A, B);
              apply_row(U2[1], A, B, DOWN ? U2[0] : U2[2], DOWN ? U2[2] : U2[0], rs3, o3);
            }
            if (lv >= 2) {
              nb_rows(us, A, B);
              apply_row(U1[1], A, B, DOWN ? U1[0] : U1[2], DOWN ? U1[2] : U1[0], rs2, U2[3]);
            }
            if (lv >= 1) {
              nb_rows(cs, A, B);
              apply_row(C[s1], A, B, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], rs1, U1[3]);
            }
          } else {
            if (lv >= 3) sphere_row(rs3, o3);
            if (lv >= 2) sphere_row(rs2, U2[3]);
            if (lv >= 1) sphere_row(rs1, U1[3]);
          }
          if (lv >= 3 && outRow) {
            char *dp = reinterpret_cast<char *>(a.dst + int64_t(z - dz) * a.pxy) + outoff;
#pragma unroll
            for (int h = 0; h < H; ++h) {
              NV *q = reinterpret_cast<NV *>(dp + h * HS * int(sizeof(T)));
              if (a.nt)
                __builtin_nontemporal_store(o3[h], q);
              else
                *q = o3[h];
            }
          }
          const int nbuf = buf ^ 1;
#pragma unroll
          for (int h = 0; h < H; ++h) {
            cs[nbuf][w][h][lane] = C[s2][h];                 // src at z+4dz: next step's u1 plane
            if (needU1) us[nbuf][w][h][lane] = U1[2][h];    // u1 at z+2dz (computed last step): next u2 plane
            if (needU2) vs[nbuf][w][h][lane] = U2[2][h];    // u2 at z (computed last step): next u3 plane
          }
          __syncthreads();
          buf = nbuf;
#pragma unroll
          for (int h = 0; h < H; ++h) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              U1[j][h] = U1[j + 1][h];
              U2[j][h] = U2[j + 1][h];
            }
          }
          ++t;
          return true;
        };
        while (run_phases(step, std::make_integer_sequence<int, NC>{})) {
        }
      };
      if (down)
        march(std::true_type{});
      else
        march(std::false_type{});
    } // segments
  }   // passes
}

// ---------------------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------------------
static int64_t x3_resident_blocks(const void *kernel, int threads) {
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

bool stencil7x3_supported(const LocalDomain &dom, int64_t qi, const Rect3 &region, const StencilTune &tune) {
  if (dom.backend() != Backend::Device || tune.wrap != 7) return false;
  if (!(dom.dtype(qi) == DType::F32 || (dom.dtype(qi) == DType::Bytes && dom.elem_size(qi) == 4))) return false;
  if ((stencil7x2_wrappable_axes(dom, qi, 1) & 7) != 7) return false;
  const Rect3 cr = dom.get_compute_region();
  if (!(region.lo == cr.lo && region.hi == cr.hi)) return false; // every axis wraps at the region's faces
  const Dim3 n = dom.size();
  if (n.x != 512 || n.y < 3 || n.z < 16) return false;
  const int64_t lox = dom.radius().x(-1);
  return (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.curr_data(qi)) + lox * 4) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.next_data(qi)) + lox * 4) % 16 == 0) &&
         (dom.pitch(qi).x * 4) % 16 == 0;
}

template <int KIND, int PF, bool STAG>
static void apply_x3_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                       const StencilTune &tune) {
  constexpr int NW = 12, YO = NW - 6;
  StencilArgs<float> a = make_args<float>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  a.nt = tune.nontemporal ? 1 : 0;
  a.wrapm = 7;
  a.x0 = a.lox;
  a.remap = tune.xcdRemap ? 1 : 0;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = 1;
  a.gy = (ny + YO - 1) / YO;
  const void *kern = STAG ? (const void *)stencil7x3s_row_kernel<NW, PF, KIND>
                          : (const void *)stencil7x3_row_kernel<NW, PF, KIND>;
  const int64_t cols = a.gy;
  const int64_t slots = x3_resident_blocks(kern, 64 * NW);
  a.seg = 1;
  uint32_t blocks = uint32_t(std::max<int64_t>(1, std::min<int64_t>(slots, cols * nz / 24)));
  X2Schedule ls = x2_lockstep_schedule(slots, cols, nz);
  if (tune.x3sched == 1) {
    // lockstep over as many row groups as possible: P parts of cm = min(cols, slots / P) columns, the leftover columns
    // spread over every block as short second segments; P minimises the steps of one block (each segment runs 4
    // warm-up steps). 512^3: 86 row groups -> P = 3 over 85 groups (255 blocks) + one leftover group, where the pairs'
    // quarters leave 22 groups to unsynchronised second segments (FETCH 1.38x the field, profiles/r5/d)
    ls = X2Schedule();
    double best = 1e30;
    for (int64_t P = 2; P <= 8; ++P) {
      const int64_t cm = std::min<int64_t>(cols, slots / P);
      if (cm < 1 || nz / P < 16) continue;
      const int64_t blocksP = P * cm, left = cols - cm;
      const double cost = double(nz) / double(P) + 4 + (left > 0 ? double(left * nz) / double(blocksP) + 4 : 0);
      if (cost < best - 1e-9) {
        best = cost;
        ls.parts = int(P);
        ls.blocks = blocksP;
      }
    }
  }
  if (tune.x2lockstep && ls.parts > 0 && ls.rounds == 1) {
    a.seg = 2;
    a.zparts = ls.parts;
    blocks = uint32_t(ls.blocks);
  }
  a.xfast = tune.x3permute ? 1 : 0;
  dom.set_device();
  if (STAG)
    hipLaunchKernelGGL((stencil7x3s_row_kernel<NW, PF, KIND>), dim3(blocks), dim3(64, NW), 0, stream, a);
  else
    hipLaunchKernelGGL((stencil7x3_row_kernel<NW, PF, KIND>), dim3(blocks), dim3(64, NW), 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

bool stencil7x3_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune) {
  if (!stencil7x3_supported(dom, qi, region, tune)) return false;
  const int pf = tune.x3pf;
  const bool stag = tune.x3stagger;
#define X3_CASE(K, P)                                                                                                  \
  (stag ? apply_x3_t<K, P, true>(dom, qi, region, sph, stream, tune) : apply_x3_t<K, P, false>(dom, qi, region, sph, stream, tune))
  if (kind == StencilKind::Jacobi) {
    if (pf >= 2)
      X3_CASE(0, 2);
    else
      X3_CASE(0, 1);
  } else {
    if (pf >= 2)
      X3_CASE(1, 2);
    else
      X3_CASE(1, 1);
  }
#undef X3_CASE
  return true;
}

} // namespace stencil
