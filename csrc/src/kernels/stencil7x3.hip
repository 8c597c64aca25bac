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
#include <vector>
#include <cmath>

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
__device__ __forceinline__ X3Seg x3_segments(const StencilArgs<float> &a, const ZPartBounds &B, uint32_t lb, uint32_t nb,
                                             uint32_t ncols, uint32_t nzt) {
  X3Seg r{0, 0, 0, 0, false};
  if (a.seg == 2) {
    const uint32_t P = uint32_t(a.zparts), cm = nb / P;
    const uint32_t qq = lb / cm, col = lb % cm;
    uint32_t zlo = qq * nzt / P, zhi = (qq + 1) * nzt / P;
    if (B.on && col < uint32_t(kZPartMaxCols)) {
      zlo = qq > 0 ? uint32_t(B.zb[col][qq - 1]) : 0;
      zhi = qq + 1 < P ? uint32_t(B.zb[col][qq]) : nzt;
    }
    r.s = col * nzt + zlo;
    r.e = col * nzt + zhi;
    // publishing boundary planes (a.pub): the first part marches up from the low z face and the last one down
    // from the high face, so both faces' planes come out in the first steps of the sweep
    r.odd = a.pub != nullptr ? (qq + 1 == P || (qq != 0 && (qq & 1) != 0)) : (qq & 1) != 0;
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

template <int NW, int PF, int KIND, bool CONTIG, int VAR>
__global__ __launch_bounds__(64 * NW, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void
stencil7x3_row_kernel(StencilArgs<float> a, ZPartBounds zbounds) {
  using T = float;
  using NV = nf4;
  constexpr int V = 4, H = 2;
  // CONTIG: a lane holds 8 adjacent cells (chunk h = cells 8 lane + 4h ..): the row's x-neighbours and the periodic
  // wrap are one rotate each way and no lane-0 / lane-63 selects. Otherwise chunk h = cells 256 h + 4 lane .. (every
  // memory op a contiguous 1 KiB; each rotate needs a select between the two chunks at lanes 0 / 63)
  constexpr int CS = CONTIG ? V : 64 * V; // cells between a lane's chunks
  constexpr int LS = CONTIG ? H * V : V;  // cells between adjacent lanes
  // VAR bit 0: publish u1 / u2 rows right after their update (LDS writes spread over the step instead of all before
  // the barrier); bit 1: no scheduling fences between the levels; bit 2: publish the src row right after the u1 update (its load was waited for there); bit 3: every
  // level's LDS reads at the top of the step
  constexpr bool EARLYW = (VAR & 1) != 0, NOSB = (VAR & 2) != 0, EARLYC = (VAR & 4) != 0, HOIST = (VAR & 8) != 0;
  constexpr int YO = NW - 6; // output rows per block
  constexpr int NC = 3 + PF; // src planes in registers
  static_assert(NW == 12, "12 waves: 3 per SIMD (168 VGPRs), 3 x 48 KiB of LDS");
  static_assert(PF == 1 || PF == 2, "slot rotations of 4 or 5 planes (4 unrolled warm-up steps, then the cycle)");
  __shared__ NV cs[2][NW][H][64]; // src rows  (plane z+3dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows   (plane z+2dz at publish)
  __shared__ NV vs[2][NW][H][64]; // u2 rows   (plane z+dz at publish)

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.y)); // the wave's block row (wave-uniform: SGPR)
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  const X3Seg sg = x3_segments(a, zbounds, lb, nb, uint32_t(a.gy), nzt);
  const bool lane0 = lane == 0, lane63 = lane == 63;
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1;
  const int xb = a.lox + lane * LS; // chunk h at xb + h * CS
  const int zwn = a.wn[2], zwlo = a.wlo[2], zwhi = a.wlo[2] + a.wn[2];
  // raw buffer over the source field (offsets from raw [0,0,0] are non-negative and below 4 GiB: checked by the host)
  const __amdgpu_buffer_rsrc_t srcRsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.src), 0, -1, 0x00020000);
  auto zcl = [&](int zz) {
    zz += zz < zwlo ? zwn : 0;
    zz -= zz >= zwhi ? zwn : 0;
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  // The wave's role = the levels its row computes (wave-uniform): 0 on rows 0 / 11 (source rows only), 1 (u1) on 1 /
  // 10, 2 (u1, u2) on 2 / 9, 3 (u1, u2, u3 = output) on 3..8. The whole march is instantiated per role, and the
  // warm-up steps (fewer valid levels) are unrolled separately, so the steady-state step has no role or level
  // branches: per step one tiny-sum test (ballot) and, for Jacobi, one sphere test per level.
  auto body = [&](auto roleTag) {
    constexpr int R = decltype(roleTag)::value;
    bool odd = sg.odd;
    const bool pubOrder = a.pub != nullptr;
    for (int pp = 0; pp < 2; ++pp) {
      // publishing: the leftover row groups' short second segments first (their face planes would otherwise come
      // out last), the main lockstep segment in its fixed direction
      const int pass = pubOrder ? 1 - pp : pp;
      uint32_t s = pass == 0 ? sg.s : sg.s2;
      const uint32_t e = pass == 0 ? sg.e : sg.e2;
      while (s < e) { // block-uniform
        const uint32_t by = s / nzt;
        const int zo = int(s - by * nzt);
        const int nzs = int(min(nzt - uint32_t(zo), e - s));
        s += uint32_t(nzs);
        const int zs = a.loz + zo;
        const int ze = zs + nzs;
        bool down = pass == 0 && sg.odd;
        if (!pubOrder) {
          down = odd != (a.flip != 0);
          odd = !odd;
        }
        const int yblk = a.loy + YO * int(by);
        const int y = yblk - 3 + w;
        if (yblk >= a.hiy) continue;
        const bool outRow = R == 3 && y < a.hiy;
        int yw = y < a.wlo[1] ? y + a.wn[1] : (y >= a.wlo[1] + a.wn[1] ? y - a.wn[1] : y);
        yw = yw < 0 ? 0 : (yw > a.rawYm1 ? a.rawYm1 : yw);
        const uint32_t rowoff = uint32_t((yw * int64_t(a.px) + xb) * int64_t(sizeof(T)));
        const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));

        // spheres (Jacobi): the planes P of this row that cross the hot / cold sphere form two intervals
        // |P - c.z| <= h (h * h < r1sq - dy^2), computed once per segment; per-cell tests only on those planes
        struct RowSph {
          int dh, dc;
          bool hit;
        };
        auto isqrt_below = [](int d) -> int { // largest h >= 0 with h * h < d (d > 0), exact
          int h = int(__builtin_sqrtf(float(d - 1)));
          while (h > 0 && h * h > d - 1) --h;
          while ((h + 1) * (h + 1) <= d - 1) ++h;
          return h;
        };
        int hzlo = 1, hzhi = 0, czlo = 1, czhi = 0; // empty intervals
        if (KIND == 0 && a.r1sq > 0) {
          const int dyh = a.r1sq - (y - a.hy) * (y - a.hy), dyc = a.r1sq - (y - a.cy) * (y - a.cy);
          if (dyh > 0) {
            const int h = isqrt_below(dyh);
            hzlo = a.hz - h;
            hzhi = a.hz + h;
          }
          if (dyc > 0) {
            const int h = isqrt_below(dyc);
            czlo = a.cz - h;
            czhi = a.cz + h;
          }
        }
        auto row_sph = [&](int P) -> RowSph {
          RowSph r{0, 0, false};
          if (KIND == 0) {
            r.hit = (P >= hzlo && P <= hzhi) || (P >= czlo && P <= czhi);
            r.dh = (y - a.hy) * (y - a.hy) + (P - a.hz) * (P - a.hz);
            r.dc = (y - a.cy) * (y - a.cy) + (P - a.cz) * (P - a.cz);
          }
          return r;
        };
        // per-cell tests on the rows that cross a sphere (cheaper variants measured slower: an x interval per row,
        // tests only on the chunk the sphere reaches; profiles/r5/ai, aj, ap). Those rows make their blocks the
        // sweep's longest, which the host evens out with sphere-weighted z parts (x3sphw, profiles/r5/ao)
        auto sphere_row = [&](const RowSph &rs, NV(&o)[H]) {
          if (KIND == 0 && rs.hit) {
            // (x - c)^2 + d < r1sq <=> (x - c)^2 < r1sq - d: the row's bound is one scalar per sphere, the per-cell
            // squared distances loop invariants, so a cell costs a compare and a select per sphere
            const int Dh = a.r1sq - rs.dh, Dc = a.r1sq - rs.dc;
#pragma unroll
            for (int h = 0; h < H; ++h)
#pragma unroll
              for (int k = 0; k < V; ++k) {
                const int x = xb + h * CS + k;
                const bool hot = (x - a.hx) * (x - a.hx) < Dh;
                const bool cold = (x - a.cx) * (x - a.cx) < Dc;
                o[h][k] = hot ? T(1) : (cold ? T(0) : o[h][k]);
              }
          }
        };
        // S of the wave's row (both chunks), x-neighbours and the periodic x wrap by lane rotates. EXACT: the
        // corrected quotient with the true division for |sum| < 2^-100 (div6v); otherwise the FMA-corrected quotient
        // for every cell and the smallest |sum| returned (the caller redoes the step exactly when it is tiny)
        auto row_update = [&](auto exactTag, const NV(&cm)[H], const NV(&up)[H], const NV(&dn)[H], const NV(&zp)[H],
                              const NV(&zm)[H], NV(&o)[H]) -> T {
          constexpr bool EXACT = decltype(exactTag)::value;
          static_assert(H == 2, "two chunks per lane");
          if constexpr (CONTIG) {
            // cells c0..c7 of the lane; left of c0 = c7 of lane - 1 (lane 0: lane 63, the wrap), right of c7 = c0 of
            // lane + 1
            const T L = rot_prev(cm[1][V - 1]), Rr = rot_next(cm[0][0]);
            const NV vmx0 = {L, cm[0][0], cm[0][1], cm[0][2]}, vpx0 = {cm[0][1], cm[0][2], cm[0][3], cm[1][0]};
            const NV vmx1 = {cm[0][3], cm[1][0], cm[1][1], cm[1][2]}, vpx1 = {cm[1][1], cm[1][2], cm[1][3], Rr};
            const NV sm0 = sum6v<T, KIND>(vpx0, vmx0, dn[0], up[0], zp[0], zm[0]);
            const NV sm1 = sum6v<T, KIND>(vpx1, vmx1, dn[1], up[1], zp[1], zm[1]);
            if constexpr (EXACT) {
              // one tiny-sum test for the lane's 8 quotients
              using NV8 = float __attribute__((ext_vector_type(8)));
              const NV8 q = div6v<T, NV8, 2 * V>(__builtin_shufflevector(sm0, sm1, 0, 1, 2, 3, 4, 5, 6, 7));
              o[0] = __builtin_shufflevector(q, q, 0, 1, 2, 3);
              o[1] = __builtin_shufflevector(q, q, 4, 5, 6, 7);
              return T(1);
            } else {
              T m = T(1);
              const NV c = NV(1.0f / 6.0f), six = NV(6.0f);
              const NV q0 = sm0 * c, q1 = sm1 * c;
              o[0] = __builtin_elementwise_fma(__builtin_elementwise_fma(-q0, six, sm0), c, q0);
              o[1] = __builtin_elementwise_fma(__builtin_elementwise_fma(-q1, six, sm1), c, q1);
#pragma unroll
              for (int k = 0; k < V; ++k) m = __builtin_fminf(m, __builtin_fminf(__builtin_fabsf(sm0[k]), __builtin_fabsf(sm1[k])));
              return m;
            }
          }
          // named scalars, not arrays: a select between two array elements became a dynamically indexed private
          // array (scratch stores + loads on every row update, 449 vs 304 us per triple)
          const T r30 = rot_prev(cm[0][V - 1]), r31 = rot_prev(cm[1][V - 1]);
          const T l00 = rot_next(cm[0][0]), l01 = rot_next(cm[1][0]);
          T m = T(1);
#pragma unroll
          for (int h = 0; h < H; ++h) {
            const T left = h == 0 ? (lane0 ? r31 : r30) : (lane0 ? r30 : r31);
            const T right = h == 0 ? (lane63 ? l01 : l00) : (lane63 ? l00 : l01);
            NV vpx, vmx;
#pragma unroll
            for (int k = 0; k < V; ++k) {
              vpx[k] = k < V - 1 ? cm[h][k + 1] : right;
              vmx[k] = k > 0 ? cm[h][k - 1] : left;
            }
            const NV sm = sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]);
            if constexpr (EXACT) {
              o[h] = div6v<T, NV, V>(sm);
            } else {
              const NV c = NV(1.0f / 6.0f), six = NV(6.0f);
              const NV q0 = sm * c;
              o[h] = __builtin_elementwise_fma(__builtin_elementwise_fma(-q0, six, sm), c, q0);
              m = __builtin_fminf(m, __builtin_fminf(__builtin_fminf(__builtin_fabsf(sm[0]), __builtin_fabsf(sm[1])),
                                                     __builtin_fminf(__builtin_fabsf(sm[2]), __builtin_fabsf(sm[3]))));
            }
          }
          return m;
        };

        auto march = [&](auto downTag) {
          constexpr bool DOWN = decltype(downTag)::value;
          constexpr int dz = DOWN ? -1 : 1;
          const int z0 = DOWN ? ze - 1 : zs;
          NV C[NC][H];
          NV U1a[H], U1b[H], U1c[H]; // u1 at planes z+2dz (new), z, z+dz
          NV U2a[H], U2b[H], U2c[H]; // u2 at planes z+dz (new), z-dz, z
          // buffer loads: the plane offset in an SGPR (soffset), the row offset a per-segment constant VGPR. With
          // 64-bit VGPR addresses recomputed every step, the address write landed on registers of the slot's
          // previous load and the compiler waited for every outstanding memory op (s_waitcnt vmcnt(0)) before each
          // step's loads, the previous step's stores included
          auto load_row = [&](int zz, int k) {
            const uint32_t po = uint32_t(zcl(zz)) * uint32_t(a.pxy) * uint32_t(sizeof(T));
#pragma unroll
            for (int h = 0; h < H; ++h)
              C[k][h] = __builtin_bit_cast(
                  NV, __builtin_amdgcn_raw_buffer_load_b128(srcRsrc, rowoff + uint32_t(h * CS * int(sizeof(T))), po, 0));
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
              U1a[h] = U1b[h] = U1c[h] = U2a[h] = U2b[h] = U2c[h] = C[1][h]; // overwritten before any use
            }
            __syncthreads();
          }
          int buf = 0;
          int t = -4;
          // one z step with LV = min(role, levels valid at this step) levels
          auto step = [&](auto phase, auto lvTag) -> bool {
            constexpr int k = decltype(phase)::value;
            constexpr int LV = decltype(lvTag)::value;
            // slots: s0 = plane z+dz, s1 = z+2dz, s2 = z+3dz; sn receives z + NC dz (it held plane z)
            constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
            if (t >= nzs) return false;
            const int z = z0 + t * dz;
            load_row(z + NC * dz, sn);
            NV o[H];
            auto levels = [&](auto exactTag) -> T {
              T m = T(1);
              // every level reads the previous step's rows (buf): no level waits for another's LDS writes, so HOIST
              // issues all of them right after the barrier (one LDS latency per step instead of three)
              NV A1[H], B1[H], A2[H], B2[H], A3[H], B3[H];
              auto rd = [&](NV(&sh)[2][NW][H][64], NV(&A)[H], NV(&B)[H]) {
#pragma unroll
                for (int h = 0; h < H; ++h) {
                  A[h] = sh[buf][wA][h][lane];
                  B[h] = sh[buf][wB][h][lane];
                }
              };
              if constexpr (HOIST) {
                if constexpr (LV >= 1) rd(cs, A1, B1);
                if constexpr (LV >= 2) rd(us, A2, B2);
                if constexpr (LV >= 3) rd(vs, A3, B3);
              }
              if constexpr (LV >= 1) {
                if constexpr (!HOIST) rd(cs, A1, B1);
                m = __builtin_fminf(m, row_update(exactTag, C[s1], A1, B1, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], U1a));
                sphere_row(row_sph(z + 2 * dz), U1a);
                if constexpr (EARLYC)
#pragma unroll
                  for (int h = 0; h < H; ++h) cs[buf ^ 1][w][h][lane] = C[s2][h];
                if constexpr (EARLYW) // publish u1 now (the other buffer: its readers finished last step)
#pragma unroll
                  for (int h = 0; h < H; ++h) us[buf ^ 1][w][h][lane] = U1a[h];
              }
              // (!NOSB) keep each level's LDS reads next to its update: at 144 VGPRs, hoisting all three levels'
              // neighbour rows (48 VGPRs) to the top of the step spilled
              if constexpr (!NOSB) __builtin_amdgcn_sched_barrier(0);
              if constexpr (LV >= 2) {
                if constexpr (!HOIST) rd(us, A2, B2);
                m = __builtin_fminf(m, row_update(exactTag, U1c, A2, B2, DOWN ? U1b : U1a, DOWN ? U1a : U1b, U2a));
                sphere_row(row_sph(z + dz), U2a);
                if constexpr (EARLYW)
#pragma unroll
                  for (int h = 0; h < H; ++h) vs[buf ^ 1][w][h][lane] = U2a[h];
              }
              if constexpr (!NOSB) __builtin_amdgcn_sched_barrier(0);
              if constexpr (LV >= 3) {
                if constexpr (!HOIST) rd(vs, A3, B3);
                m = __builtin_fminf(m, row_update(exactTag, U2c, A3, B3, DOWN ? U2b : U2a, DOWN ? U2a : U2b, o));
                sphere_row(row_sph(z), o);
              }
              return m;
            };
            // exact quotients inline (div6v: the FMA-corrected quotient, a per-lane branch no lane normally takes for
            // |sum| < 2^-100). A branch-free fast pass with a wave-uniform exact redo of the whole step needs more
            // registers (the fast results stay live across the redo: 168 VGPRs + 21 spilled for Jacobi), so not used
            (void)levels(std::true_type{});
            if constexpr (LV >= 3) {
              // unconditional: a row past the region's y end (the last row group) stores into a per-device sink, so
              // every path has the same vector-memory ops and the next step's load wait counts past these stores
              char *dp = outRow ? reinterpret_cast<char *>(a.dst + int64_t(z) * a.pxy) + outoff
                                : a.sink + lane * LS * int(sizeof(T));
#pragma unroll
              for (int h = 0; h < H; ++h) {
                NV *q = reinterpret_cast<NV *>(dp + h * CS * int(sizeof(T)));
                if (a.nt)
                  __builtin_nontemporal_store(o[h], q);
                else
                  *q = o[h];
              }
            }
            const int nbuf = buf ^ 1;
#pragma unroll
            for (int h = 0; h < H; ++h) {
              if constexpr (!EARLYC || LV < 1) cs[nbuf][w][h][lane] = C[s2][h];
              if constexpr (R >= 1 && !EARLYW) us[nbuf][w][h][lane] = U1a[h];
              if constexpr (R >= 2 && !EARLYW) vs[nbuf][w][h][lane] = U2a[h];
            }
            // boundary-plane publication (block-uniform, as the pairs): every wave's stores of output plane z
            // complete before the barrier, then one thread writes the L2 back (release) and counts the block's cells
            const bool pubStep = a.pub != nullptr && t >= 0 && (z < a.pubLo || z >= a.pubHi);
            if (pubStep) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (pubStep && lane == 0 && w == 0) {
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
              const unsigned long long cells =
                  (unsigned long long)(min(YO, a.hiy - yblk)) * (unsigned long long)(a.hix - a.lox);
              __hip_atomic_fetch_add(a.pub, cells, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
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
          using I0 = std::integral_constant<int, 0>;
          using I1 = std::integral_constant<int, 1>;
          using I2 = std::integral_constant<int, 2>;
          using I3 = std::integral_constant<int, 3>;
          using I4 = std::integral_constant<int, 4 % NC>;
          using L1 = std::integral_constant<int, (R < 1 ? R : 1)>;
          using L2 = std::integral_constant<int, (R < 2 ? R : 2)>;
          using LR = std::integral_constant<int, R>;
          // warm-up: t = -4, -3 compute u1 only, t = -2, -1 u1 and u2 (one cycle of the slot rotation)
          step(I0{}, L1{});
          step(I1{}, L1{});
          step(I2{}, L2{});
          step(I3{}, L2{});
          if constexpr (NC == 5)
            while (step(I4{}, LR{}) && step(I0{}, LR{}) && step(I1{}, LR{}) && step(I2{}, LR{}) && step(I3{}, LR{})) {
            }
          else
            while (step(I0{}, LR{}) && step(I1{}, LR{}) && step(I2{}, LR{}) && step(I3{}, LR{})) {
          }
        };
        if (down)
          march(std::true_type{});
        else
          march(std::false_type{});
      } // segments
    }   // passes
  };
  const unsigned long long clk0 = a.clk ? wall_clock64() : 0;
  const int role = (w >= 3 && w < NW - 3) ? 3 : ((w >= 2 && w < NW - 2) ? 2 : ((w >= 1 && w < NW - 1) ? 1 : 0));
  if (role == 3)
    body(std::integral_constant<int, 3>{});
  else if (role == 2)
    body(std::integral_constant<int, 2>{});
  else if (role == 1)
    body(std::integral_constant<int, 1>{});
  else
    body(std::integral_constant<int, 0>{});
  if (a.clk) { // measurement only (StencilTune::blockClock): every wave done, one lane stores the block's interval
    __syncthreads();
    if (lane == 0 && w == 0) {
      a.clk[2 * lb] = clk0;
      a.clk[2 * lb + 1] = wall_clock64();
    }
  }
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

// per-device sink for the stores of rows past a region's y end (2 chunks x 64 lanes x 16 B); allocated by
// stencil7x3_supported (model init), never inside a stream capture
static std::map<int, char *> gX3Sinks;
static std::mutex gX3SinkMu;
static char *x3_sink(int dev, bool create) {
  std::lock_guard<std::mutex> lk(gX3SinkMu);
  char *&p = gX3Sinks[dev];
  if (!p && create) {
    int cur = 0;
    HIP_CHECK(hipGetDevice(&cur));
    HIP_CHECK(hipSetDevice(dev));
    HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&p), 4096));
    HIP_CHECK(hipSetDevice(cur));
  }
  return p;
}

bool stencil7x3_supported(const LocalDomain &dom, int64_t qi, const Rect3 &region, const StencilTune &tune) {
  // x wraps in-kernel (whole 512-cell rows, DPP rotates); y / z either wrap in-kernel too (one GPU: nothing is
  // exchanged) or read 3-deep halos the exchange filled (an axis cut across GPUs / sub-domains)
  if (dom.backend() != Backend::Device || !(tune.wrap & 1)) return false;
  if (!(dom.dtype(qi) == DType::F32 || (dom.dtype(qi) == DType::Bytes && dom.elem_size(qi) == 4))) return false;
  if (!(stencil7x2_wrappable_axes(dom, qi, 1) & 1)) return false;
  const Radius &rad = dom.radius();
  if (!(tune.wrap & 2) && (rad.y(-1) < 3 || rad.y(1) < 3)) return false;
  if (!(tune.wrap & 4) && (rad.z(-1) < 3 || rad.z(1) < 3)) return false;
  const Rect3 cr = dom.get_compute_region();
  if (!(region.lo == cr.lo && region.hi == cr.hi)) return false; // the kernel sweeps whole sub-domains
  const Dim3 n = dom.size();
  if (n.x != 512 || n.y < 3 || n.z < 16) return false;
  if (dom.buffer_bytes(qi) >= (int64_t(1) << 32) - 4096) return false; // 32-bit buffer-load offsets
  (void)x3_sink(dom.gpu(), true);
  const int64_t lox = dom.radius().x(-1);
  return (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.curr_data(qi)) + lox * 4) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.next_data(qi)) + lox * 4) % 16 == 0) &&
         (dom.pitch(qi).x * 4) % 16 == 0;
}

template <int KIND, int PF, bool CONTIG, int VAR>
static void apply_x3_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                       const StencilTune &tune) {
  constexpr int NW = 12, YO = NW - 6;
  StencilArgs<float> a = make_args<float>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  a.nt = tune.nontemporal ? 1 : 0;
  a.wrapm = tune.wrap & 7;
  // an axis read from its halos: no periodic shift (the kernel's row / plane wrap adds / subtracts wn)
  if (!(a.wrapm & 2)) a.wn[1] = 0;
  if (!(a.wrapm & 4)) a.wn[2] = 0;
  a.x0 = a.lox;
  a.remap = tune.xcdRemap ? 1 : 0;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = 1;
  a.gy = (ny + YO - 1) / YO;
  const void *kern = (const void *)stencil7x3_row_kernel<NW, PF, KIND, CONTIG, VAR>;
  const int64_t cols = a.gy;
  const int64_t resident = x3_resident_blocks(kern, 64 * NW);
  // CUs left to the transport kernels running beside the sweep (pipelined triples: the gated exchange)
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dom.gpu()) != hipSuccess) cus = 256;
  const int64_t perCU = std::max<int64_t>(1, resident / std::max(1, cus));
  const int64_t slots = std::max<int64_t>(perCU, resident - perCU * std::min(tune.reserveCUs, cus / 2));
  if (tune.publish) {
    a.pub = reinterpret_cast<unsigned long long *>(tune.publish);
    a.pubLo = a.loz + tune.publishDepth;
    a.pubHi = a.hiz - tune.publishDepth;
    a.flip = 0; // fixed march directions (x3_segments)
  }
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
      if (tune.x3parts > 0 && P != tune.x3parts) continue;
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
  ZPartBounds zb{};
  zb.on = 0;
  if (KIND == 0 && a.seg == 2)
    sphere_part_bounds(zb, a, int64_t(blocks) / a.zparts, a.zparts, NW, YO, 3, tune.x3sphw);
  dom.set_device();
  a.sink = x3_sink(dom.gpu(), false);
  a.clk = reinterpret_cast<unsigned long long *>(tune.blockClock);
  STENCIL_REQUIRE(a.sink, "stencil7x3: no store sink on device " << dom.gpu() << " (stencil7x3_supported first)");
  hipLaunchKernelGGL((stencil7x3_row_kernel<NW, PF, KIND, CONTIG, VAR>), dim3(blocks), dim3(64, NW), 0, stream, a, zb);
  HIP_CHECK(hipGetLastError());
}

bool stencil7x3_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune) {
  if (!stencil7x3_supported(dom, qi, region, tune)) return false;
  // instantiated: x3var 7 (the default) and 0 (r5/s: everything published before the barrier), both layouts, one or
  // two planes of lookahead; r5/v measured 1 / 3 / 5 between them (profiles/r5/v/summary.txt)
  STENCIL_REQUIRE(tune.x3var == 0 || tune.x3var == 7 || tune.x3var == 15,
                  "stencil7x3: x3var " << tune.x3var << " not instantiated (0, 7, 15)");
  STENCIL_REQUIRE(tune.x3pf == 1 || tune.x3pf == 2, "stencil7x3: x3pf " << tune.x3pf << " (1, 2)");
  const bool contig = tune.x3layout == 1, pf2 = tune.x3pf == 2;
  auto go = [&](auto kindTag, auto pfTag) {
    constexpr int K = decltype(kindTag)::value, P = decltype(pfTag)::value;
    if (contig)
      tune.x3var == 7 ? apply_x3_t<K, P, true, 7>(dom, qi, region, sph, stream, tune)
                      : apply_x3_t<K, P, true, 0>(dom, qi, region, sph, stream, tune);
    else if (tune.x3var == 15)
      apply_x3_t<K, P, false, 15>(dom, qi, region, sph, stream, tune);
    else
      tune.x3var == 7 ? apply_x3_t<K, P, false, 7>(dom, qi, region, sph, stream, tune)
                      : apply_x3_t<K, P, false, 0>(dom, qi, region, sph, stream, tune);
  };
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  if (kind == StencilKind::Jacobi)
    pf2 ? go(std::integral_constant<int, 0>{}, P2{}) : go(std::integral_constant<int, 0>{}, P1{});
  else
    pf2 ? go(std::integral_constant<int, 1>{}, P2{}) : go(std::integral_constant<int, 1>{}, P1{});
  return true;
}

} // namespace stencil
