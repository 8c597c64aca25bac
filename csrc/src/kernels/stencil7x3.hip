// Three fused 7-point steps per sweep (deeper temporal blocking): dst = S(S(S(src))) on a whole sub-domain, for
// gfx950. Two kernels share the design below:
//   * stencil7x3_wrap_kernel - whole periodic rows (x wrapped in-kernel, fp32 rows of exactly 512 cells): the
//     x-neighbours and the wrap are DPP lane rotates of the wave's own registers, nothing is read beyond the row (the
//     one-GPU headline);
//   * stencil7x3_xh_kernel - columns with x halos (fp32 x a multiple of 512, fp64 of 256): the same two-chunk lane
//     layout per column of CW cells; only the 3 cells beyond each column end come from outside the wave. The two edge
//     waves (rows 0 and 11, which otherwise only load and publish their source row) carry the column ends of all 12
//     rows - wave 0 the left end, wave 11 the right, lane r = row r: one 16-B load per row and plane (cells x-3 .. x /
//     x+CW-1 .. x+CW+2), u1 at the two cells beyond the end, u2 at the adjacent one, y-neighbours by DPP row shifts -
//     and publish each row's adjacent cell per level through LDS; the output waves read one value per level on lanes
//     0 / 63. So a sub-domain whose x faces come from an exchange (the reference's every-iteration exchange on one
//     GPU, x cut across GPUs, fp64) runs one depth-3 exchange and one read + write of the field per three steps.
//
// The fused pair (stencil7x2_row_kernel) streams the field once per two steps at ~95 % of a plain copy of its access
// shape (205 us per 512^3 pair, profiles/r4/j); a triple reads and writes the field once per THREE steps. What it
// costs is compute on the redundant y halo: a block of 12 waves (one row each) holds 12 src rows and computes
//   u1 on the inner 10 rows, u2 on the inner 8, u3 (the output) on the inner 6,
// i.e. 24 row updates per 6 output rows; each wave only computes the levels some output row needs (wave-uniform).
//
//   step t (output plane z, march direction dz):
//     1. issue the load of src plane z + 4dz                               (one plane of lookahead in registers)
//     2. u1 at plane z+2dz from the src window + LDS y-neighbours          (waves 1 .. 10)   publish src(z+3dz), u1
//     3. u2 at plane z+dz  from the u1 window (z, z+dz, z+2dz) + LDS       (waves 2 .. 9)    publish u2
//     4. u3 at plane z     from the u2 window (z-dz, z, z+dz) + LDS        (waves 3 .. 8)  -> store
//     5. one barrier (every LDS row is written into the other buffer right after its update: the step is bound by
//        the chain LDS write -> barrier -> LDS read -> update, three times per step, profiles/r5/v)
// A segment of nzs output planes runs nzs + 4 steps. Summation order, the exact /6 and the spheres are those of the
// single step, every intermediate value is computed exactly as the single step computes it, so S(S(S(src))) is
// bitwise equal to three single steps (tests/test_gpu.py::test_temporal3_*).
// Reference step being fused: bin/jacobi3d.cu:40-87 (Jacobi), bin/astaroth_sim.cu:65-83 (Astaroth); the exchange the
// XH form reads once per three steps: bin/jacobi3d.cu:291 (dd.exchange() every iteration).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>
#include <vector>
#include <cmath>
#include <cstring>

#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/rt/hip_check.hpp"
#include "stencil_common.hpp"
#include "stencil_wave.hpp"

namespace stencil {

// (column, plane) segment of a block: lockstep parts as the fused pairs (x2_segments), kept local to this file.
// Columns are numbered y-major inside an x strip (col = bx * gy + by); the z-part bounds are per row group (by)
struct X3Seg {
  uint32_t s, e, s2, e2;
  bool odd;  // the first segment's march direction (down unless the sweep flips)
  bool odd2; // the second's
};
template <typename T>
__device__ __forceinline__ X3Seg x3_segments(const StencilArgs<T> &a, const ZPartBounds &B, uint32_t lb, uint32_t nb,
                                             uint32_t ncols, uint32_t gy, uint32_t nzt) {
  X3Seg r{0, 0, 0, 0, false, false};
  if (a.seg == 3) { // rounds of whole column groups (x3_round): parts alternate their z direction as in seg 2
    r.odd = ((lb / (nb / uint32_t(a.zparts))) & 1) != 0;
    r.odd2 = !r.odd;
    return r;
  }
  if (a.seg == 2) {
    const uint32_t P = uint32_t(a.zparts), cm = nb / P;
    const uint32_t qq = lb / cm, col = lb % cm;
    const uint32_t grp = col % gy;
    uint32_t zlo = qq * nzt / P, zhi = (qq + 1) * nzt / P;
    if (B.on && grp < uint32_t(kZPartMaxCols)) {
      zlo = qq > 0 ? uint32_t(B.zb[grp][qq - 1]) : 0;
      zhi = qq + 1 < P ? uint32_t(B.zb[grp][qq]) : nzt;
    }
    r.s = col * nzt + zlo;
    r.e = col * nzt + zhi;
    // publishing boundary planes (a.pub): the first part marches up from the low z face and the last one down
    // from the high face, so both faces' planes come out in the first steps of the sweep
    r.odd = a.pub != nullptr ? (qq + 1 == P || (qq != 0 && (qq & 1) != 0)) : (qq & 1) != 0;
    if (B.lon) { // tabled (balance_leftover / lockstep_leftover)
      r.s2 = cm * nzt + B.l0[lb];
      r.e2 = cm * nzt + B.l1[lb];
      r.odd2 = ((B.ldir[lb >> 5] >> (lb & 31)) & 1) != 0;
    } else {
      const uint64_t LW = uint64_t(ncols - cm) * nzt;
      r.s2 = cm * nzt + uint32_t(uint64_t(lb) * LW / nb);
      r.e2 = cm * nzt + uint32_t(uint64_t(lb + 1) * LW / nb);
      r.odd2 = !r.odd;
    }
  } else {
    const uint64_t W = uint64_t(ncols) * nzt;
    r.s = uint32_t(uint64_t(lb) * W / nb);
    r.e = uint32_t(uint64_t(lb + 1) * W / nb);
    r.odd = (lb & 1) != 0;
    r.odd2 = r.odd;
  }
  return r;
}

// 16 B of the source at byte offset voff + soff (buffer load: the plane offset in an SGPR)
template <typename X>
__device__ __forceinline__ X x3_load16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(X, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

// whole-wave DPP row shifts (16-lane rows; the XH edge waves keep rows 0..11 in lanes 0..11): lane i <- lane i+1 /
// lane i-1 (the lanes shifted in from outside a row are never used)
__device__ __forceinline__ float x3_row_next(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x101, 0xf, 0xf, false));
}
__device__ __forceinline__ float x3_row_prev(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ double x3_row_next(double v) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b), 0x101, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), 0x101, 0xf, 0xf, false);
  return __longlong_as_double(int64_t(uint32_t(lo)) | (int64_t(hi) << 32));
}
__device__ __forceinline__ double x3_row_prev(double v) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b), 0x111, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), 0x111, 0xf, 0xf, false);
  return __longlong_as_double(int64_t(uint32_t(lo)) | (int64_t(hi) << 32));
}

// Columns with x halos (the XH form): every x-neighbour beyond a column end comes from the exchanged halos. BIG:
// fields of 4 GiB or more (a buffer resource per plane); else one resource over the field, the plane in soffset
template <typename T, int KIND, bool BIG, bool PUB>
__global__ __launch_bounds__(64 * 12, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void
stencil7x3_xh_kernel(StencilArgs<T> a, ZPartBounds zbounds) {
  constexpr bool XH = true;
  using NV = typename Vec16<T>::native;
  using P2 = typename Pk<T>::t;
  typedef T E4 __attribute__((ext_vector_type(4)));
  constexpr int NW = 12;              // 3 waves per SIMD (168 VGPRs), 3 x 48 KiB of LDS
  constexpr int V = int(16 / sizeof(T)), H = 2;
  constexpr int CS = 64 * V;          // cells between a lane's two chunks
  constexpr int CW = H * CS;          // cells per column (the whole row when x wraps in-kernel)
  constexpr int YO = NW - 6;          // output rows per block
  constexpr int NC = 4;               // src planes in registers (one plane of lookahead)
  __shared__ NV cs[2][NW][H][64]; // src rows  (plane z+3dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows   (plane z+2dz at publish)
  __shared__ NV vs[2][NW][H][64]; // u2 rows   (plane z+dz at publish)
  // XH: each row's cell just beyond its column end ([0] x-1, [1] x+CW) for the row's own updates: src (z+3dz), u1
  // (z+2dz), u2 (z+dz) at publish, written by the edge waves
  __shared__ T es[2][NW][2], eu[2][NW][2], ev[2][NW][2];

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.y)); // the wave's block row (wave-uniform: SGPR)
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  const uint32_t gy = uint32_t(a.gy);
  const X3Seg sg = x3_segments(a, zbounds, lb, nb, uint32_t(a.gx) * gy, gy, nzt);
  const bool lane0 = lane == 0, lane63 = lane == 63;
  const int side = lane >> 5; // XH: lane 0 reads the left end's cells, lane 63 the right end's
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1;
  const int zwn = a.wn[2], zwlo = a.wlo[2], zwhi = a.wlo[2] + a.wn[2];
  auto zcl = [&](int zz) {
    zz += zz < zwlo ? zwn : 0;
    zz -= zz >= zwhi ? zwn : 0;
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  const __amdgpu_buffer_rsrc_t srcRsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(a.src), 0, -1, 0x00020000);
  auto ywrap = [&](int yy) {
    yy = yy < a.wlo[1] ? yy + a.wn[1] : (yy >= a.wlo[1] + a.wn[1] ? yy - a.wn[1] : yy);
    return yy < 0 ? 0 : (yy > a.rawYm1 ? a.rawYm1 : yy);
  };
  // The wave's role = the levels its row computes (wave-uniform): 0 on rows 0 / 11 (source rows only), 1 (u1) on 1 /
  // 10, 2 (u1, u2) on 2 / 9, 3 (u1, u2, u3 = output) on 3..8. The whole march is instantiated per role, and the
  // warm-up steps (fewer valid levels) are unrolled separately, so the steady-state step has no role or level
  // branches. XH: rows 0 / 11 are role 4, the edge waves: besides their source row, wave 0 computes the left column
  // end of all 12 rows (lane r = row r) and wave 11 the right end - src loads, u1 at the two cells beyond the end, u2
  // at the adjacent one, y-neighbours by DPP row shifts - and publishes each row's adjacent cell per level through
  // LDS. The output waves then carry no edge state: one LDS read per level on lanes 0 / 63.
  auto body = [&](auto roleTag) {
    constexpr int R = decltype(roleTag)::value;
    constexpr int RM = R == 4 ? 0 : R; // levels of the wave's own row
    constexpr bool EDGE = XH && R == 4;
    bool odd = sg.odd;
    const bool pubOrder = PUB; // boundary-plane publication (a.pub, template: no live state otherwise)
    const uint32_t ncols = uint32_t(a.gx) * gy;
    const int npass = XH && a.seg == 3 ? a.zrounds : 2; // rounds: XH only (many columns), fewer SGPRs elsewhere
    for (int pp = 0; pp < npass; ++pp) {
      // publishing: the leftover row groups' short second segments first (their face planes would otherwise come
      // out last), the main lockstep segment in its fixed direction
      const int pass = pubOrder ? 1 - pp : pp;
      uint32_t s = pass == 0 ? sg.s : sg.s2;
      uint32_t e = pass == 0 ? sg.e : sg.e2;
      if (pass == 1 && !pubOrder) odd = sg.odd2;
      if (XH && a.seg == 3) {
        // round pp: column group pp cm + lb % cm, z part lb / cm (every block on y-adjacent columns in step)
        const uint32_t P = uint32_t(a.zparts), cm = nb / P, qq = lb / cm;
        const uint32_t colr = uint32_t(pp) * cm + lb % cm;
        if (colr >= ncols) break;
        s = colr * nzt + qq * nzt / P;
        e = colr * nzt + (qq + 1) * nzt / P;
      }
      while (s < e) { // block-uniform
        const uint32_t col = s / nzt;
        const int zo = int(s - col * nzt);
        const int nzs = int(min(nzt - uint32_t(zo), e - s));
        s += uint32_t(nzs);
        const int bx = XH ? int(col / gy) : 0;
        const int by = int(col - uint32_t(bx) * gy);
        const int zs = a.loz + zo;
        const int ze = zs + nzs;
        bool down = pass == 0 && sg.odd;
        if (!pubOrder) {
          down = odd != (a.flip != 0);
          odd = !odd;
        }
        const int yblk = a.loy + YO * by;
        const int y = yblk - 3 + w;
        if (yblk >= a.hiy) continue;
        const bool outRow = R == 3 && y < a.hiy;
        const int yw = ywrap(y);
        const int xcol = a.x0 + bx * CW; // first cell of the column
        const int xb = xcol + lane * V;  // chunk h at xb + h * CS
        const uint32_t rowoff = uint32_t((yw * int64_t(a.px) + xb) * int64_t(sizeof(T)));
        const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));
        // XH edge waves: lane r holds row r's 4 cells from x-3 (wave 0) / x+CW-1 (wave 11): the two cells beyond the
        // end (e[1], e[2]) and their outer and inner x-neighbours (e[0], e[3])
        const int eside = w == NW - 1 ? 1 : 0;
        const int er = lane < NW ? lane : NW - 1;
        const int ey = yblk - 3 + er;
        const int eyh = (ey - a.hy) * (ey - a.hy), eyc = (ey - a.cy) * (ey - a.cy); // Jacobi spheres, edge lanes
        const uint32_t edgeoff =
            uint32_t((ywrap(ey) * int64_t(a.px) + (eside ? xcol + CW - 1 : xcol - 3)) * int64_t(sizeof(T)));

        // spheres (Jacobi): a cell (x, y, P) is in the hot sphere iff (x - hx)^2 < Dh = yh - (P - hz)^2 with
        // yh = r1sq - (y - hy)^2 (per segment), in the cold one likewise; the row-plane has no sphere cell when both
        // bounds are <= 0 (r1sq = 0: never). Two live scalars per row instead of plane intervals + centres (SGPR
        // pressure: the Jacobi kernels spilled 100-121 SGPRs to VGPR lanes)
        const int yh = a.r1sq - (y - a.hy) * (y - a.hy), yc = a.r1sq - (y - a.cy) * (y - a.cy);
        struct RowSph {
          int Dh, Dc;
          bool hit;
        };
        auto row_sph = [&](int P) -> RowSph {
          RowSph r{0, 0, false};
          if (KIND == 0 && !EDGE) {
            r.Dh = yh - (P - a.hz) * (P - a.hz);
            r.Dc = yc - (P - a.cz) * (P - a.cz);
            r.hit = max(r.Dh, r.Dc) > 0;
          }
          return r;
        };
        // (x - c)^2 < D: the row-plane's bound is one scalar per sphere, the per-cell squared distances loop
        // invariants, so a cell costs a compare and a select per sphere; the blocks of sphere-crossing rows are
        // evened out by sphere-weighted z parts and the leftover plan (x3sphw, x3left)
        auto sph_fix = [&](int dh, int dc, int x, T v) -> T {
          const bool hot = (x - a.hx) * (x - a.hx) < a.r1sq - dh;
          const bool cold = (x - a.cx) * (x - a.cx) < a.r1sq - dc;
          return hot ? T(1) : (cold ? T(0) : v);
        };
        // the chunks (cells xcol + h CS .. + CS - 1 over the wave) a sphere's x range can reach: the 512^3 hot sphere
        // (x 119-221) only touches chunk 0, the cold one (290-392) only chunk 1, so a sphere row tests half the cells
        // (StencilTune.x3sphchunk; 0: every chunk for both spheres). Bits in one SGPR (2h: cold on chunk h, 2h + 1:
        // hot), not booleans (lane masks)
        int sphm = 0;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const int lo = xcol + h * CS, hi = lo + CS - 1;
          sphm |= int(!a.sphchunk || (a.cx - a.sphr <= hi && a.cx + a.sphr >= lo)) << (2 * h);
          sphm |= int(!a.sphchunk || (a.hx - a.sphr <= hi && a.hx + a.sphr >= lo)) << (2 * h + 1);
        }
        sphm = __builtin_amdgcn_readfirstlane(sphm);
        auto sphere_row = [&](const RowSph &rs, NV(&o)[H]) {
          if (KIND == 0 && rs.hit) {
            // cold first, then hot: the hot sphere wins where both hold, as in the single step
#pragma unroll
            for (int h = 0; h < H; ++h) {
              if ((sphm >> (2 * h)) & 1)
#pragma unroll
                for (int k = 0; k < V; ++k) {
                  const int x = xb + h * CS + k;
                  o[h][k] = (x - a.cx) * (x - a.cx) < rs.Dc ? T(0) : o[h][k];
                }
              if ((sphm >> (2 * h + 1)) & 1)
#pragma unroll
                for (int k = 0; k < V; ++k) {
                  const int x = xb + h * CS + k;
                  o[h][k] = (x - a.hx) * (x - a.hx) < rs.Dh ? T(1) : o[h][k];
                }
            }
          }
        };
        // S of the wave's row (both chunks), x-neighbours by lane rotates; at the row / column ends lane 0 and lane
        // 63 take the periodic wrap (whole rows) or ev, their end's cell beyond the column (XH). Exact /6 (div6v)
        auto row_update = [&](const NV(&cm)[H], const NV(&up)[H], const NV(&dn)[H], const NV(&zp)[H], const NV(&zm)[H],
                              T ev, NV(&o)[H]) {
          static_assert(H == 2, "two chunks per lane");
          // named scalars, not arrays: a select between two array elements became a dynamically indexed private
          // array (scratch stores + loads on every row update, 449 vs 304 us per triple)
          const T r30 = rot_prev(cm[0][V - 1]), r31 = rot_prev(cm[1][V - 1]);
          const T l00 = rot_next(cm[0][0]), l01 = rot_next(cm[1][0]);
#pragma unroll
          for (int h = 0; h < H; ++h) {
            const T left = h == 0 ? (lane0 ? (XH ? ev : r31) : r30) : (lane0 ? r30 : r31);
            const T right = h == 0 ? (lane63 ? l01 : l00) : (lane63 ? (XH ? ev : l00) : l01);
            NV vpx, vmx;
#pragma unroll
            for (int k = 0; k < V; ++k) {
              vpx[k] = k < V - 1 ? cm[h][k + 1] : right;
              vmx[k] = k > 0 ? cm[h][k - 1] : left;
            }
            o[h] = div6v<T, NV, V>(sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]));
          }
        };

        auto march = [&](auto downTag) {
          constexpr bool DOWN = decltype(downTag)::value;
          constexpr int dz = DOWN ? -1 : 1;
          const int z0 = DOWN ? ze - 1 : zs;
          NV C[NC][H];
          NV U1a[H], U1b[H], U1c[H]; // u1 at planes z+2dz (new), z, z+dz
          NV U2a[H], U2b[H], U2c[H]; // u2 at planes z+dz (new), z-dz, z
          E4 E[NC];                  // edge waves: the column-end cells of the src window planes
          P2 U1Ea, U1Eb, U1Ec;       // edge waves: u1 at (e[1], e[2]), planes as U1
          // buffer loads: the plane in the resource (SGPRs), the row offset a per-segment constant VGPR. With 64-bit
          // VGPR addresses recomputed every step, the address write landed on registers of the slot's previous load
          // and the compiler waited for every outstanding memory op (s_waitcnt vmcnt(0)) before each step's loads,
          // the previous step's stores included
          auto load_row = [&](int zz, int k) {
            // BIG: a raw buffer over the plane (its base in SGPRs: fields beyond 4 GiB, fp64 1024^3); else one
            // resource over the field, the plane offset in soffset. The row offset a per-segment constant VGPR
            const uint32_t po = BIG ? 0u : uint32_t(zcl(zz)) * uint32_t(a.pxy) * uint32_t(sizeof(T));
            const __amdgpu_buffer_rsrc_t rs =
                BIG ? __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(a.src + int64_t(zcl(zz)) * a.pxy), 0, -1,
                                                        0x00020000)
                    : srcRsrc;
#pragma unroll
            for (int h = 0; h < H; ++h) C[k][h] = x3_load16<NV>(rs, rowoff + uint32_t(h * CS * int(sizeof(T))), po);
            if constexpr (EDGE) {
              if constexpr (sizeof(T) == 4) {
                E[k] = x3_load16<E4>(rs, edgeoff, po);
              } else {
                const NV lo = x3_load16<NV>(rs, edgeoff, po), hi = x3_load16<NV>(rs, edgeoff + 16, po);
                E[k] = E4{lo[0], lo[1], hi[0], hi[1]};
              }
            }
          };
          // the end's cell adjacent to the column in a pair of end cells: x-1 ([1]) or x+CW ([0])
          auto adj = [&](const P2 &p) -> T { return eside ? p[0] : p[1]; };
          // step t = -4 starts with src planes z+dz .. z+3dz, z = z0 - 4dz, and the src row of its u1 plane
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
            if constexpr (EDGE) {
              if (lane < NW) es[0][er][eside] = eside ? E[1][1] : E[1][2];
              U1Ea = U1Eb = U1Ec = P2{T(0), T(0)};
            }
            __syncthreads();
          }
          int buf = 0;
          int t = -4;
          // one z step with LV = min(role, levels valid at this step) levels
          auto step = [&](auto phase, auto lvTag) -> bool {
            constexpr int k = decltype(phase)::value;
            constexpr int LV = decltype(lvTag)::value;
            // slots: s0 = plane z+dz, s1 = z+2dz, s2 = z+3dz; sn receives z + 4dz (it held plane z)
            constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
            if (t >= nzs) return false;
            const int z = z0 + t * dz;
            const int nbuf = buf ^ 1;
            load_row(z + NC * dz, sn);
            NV o[H];
            // every level reads the previous step's rows (buf) and publishes into the other buffer (its readers
            // finished last step) right after its update
            if constexpr (LV >= 1) {
              NV A[H], B[H];
#pragma unroll
              for (int h = 0; h < H; ++h) {
                A[h] = cs[buf][wA][h][lane];
                B[h] = cs[buf][wB][h][lane];
              }
              row_update(C[s1], A, B, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], XH ? es[buf][w][side] : T(0), U1a);
              sphere_row(row_sph(z + 2 * dz), U1a);
#pragma unroll
              for (int h = 0; h < H; ++h) {
                cs[nbuf][w][h][lane] = C[s2][h];
                us[nbuf][w][h][lane] = U1a[h];
              }
            }
            if constexpr (LV >= 2) {
              NV A[H], B[H];
#pragma unroll
              for (int h = 0; h < H; ++h) {
                A[h] = us[buf][wA][h][lane];
                B[h] = us[buf][wB][h][lane];
              }
              row_update(U1c, A, B, DOWN ? U1b : U1a, DOWN ? U1a : U1b, XH ? eu[buf][w][side] : T(0), U2a);
              sphere_row(row_sph(z + dz), U2a);
#pragma unroll
              for (int h = 0; h < H; ++h) vs[nbuf][w][h][lane] = U2a[h];
            }
            if constexpr (LV >= 3) {
              NV A[H], B[H];
#pragma unroll
              for (int h = 0; h < H; ++h) {
                A[h] = vs[buf][wA][h][lane];
                B[h] = vs[buf][wB][h][lane];
              }
              row_update(U2c, A, B, DOWN ? U2b : U2a, DOWN ? U2a : U2b, XH ? ev[buf][w][side] : T(0), o);
              sphere_row(row_sph(z), o);
              // unconditional: a row past the region's y end (the last row group) stores into a per-device sink, so
              // every path has the same vector-memory ops and the next step's load wait counts past these stores
              char *dp = outRow ? reinterpret_cast<char *>(a.dst + int64_t(z) * a.pxy) + outoff
                                : a.sink + lane * V * int(sizeof(T));
#pragma unroll
              for (int h = 0; h < H; ++h) {
                NV *q = reinterpret_cast<NV *>(dp + h * CS * int(sizeof(T)));
                if (a.nt)
                  __builtin_nontemporal_store(o[h], q);
                else
                  *q = o[h];
              }
            }
            if constexpr (LV < 1)
#pragma unroll
              for (int h = 0; h < H; ++h) cs[nbuf][w][h][lane] = C[s2][h];
            if constexpr (EDGE) {
              // u1 at the end cells (e[1], e[2]) of plane z+2dz for every row: x-neighbours in the lane's own load, y
              // the neighbour rows' lanes (row shifts), z the window's other planes
              const E4 &ec = E[s1], &ep = DOWN ? E[s0] : E[s2], &em = DOWN ? E[s2] : E[s0];
              const P2 yb = {x3_row_next(ec[1]), x3_row_next(ec[2])}, ya = {x3_row_prev(ec[1]), x3_row_prev(ec[2])};
              U1Ea = div6v<T, P2, 2>(sum6v<T, KIND>(P2{ec[2], ec[3]}, P2{ec[0], ec[1]}, yb, ya, P2{ep[1], ep[2]},
                                                     P2{em[1], em[2]}));
              // u2 at the adjacent cell of plane z+dz: x-neighbours the far u1 end cell and the row's own first / last
              // u1 cell (published by its wave last step), y the neighbour rows' lanes, z the adjacent u1 cells of the
              // planes before / after
              const T far = eside ? U1Ec[1] : U1Ec[0];
              const T inner = eside ? us[buf][er][H - 1][63][V - 1] : us[buf][er][0][0][0];
              const T vmx = eside ? inner : far, vpx = eside ? far : inner;
              const T ca = adj(U1Ec);
              const T ya2 = x3_row_prev(ca), yb2 = x3_row_next(ca);
              const T za = adj(U1Ea), zb = adj(U1Eb);
              // (a pair: sum6v / div6v map an all -0 sum to +0 exactly as the single step's 0-started sum does)
              T U2E = div6v<T, P2, 2>(sum6v<T, KIND>(P2{vpx, vpx}, P2{vmx, vmx}, P2{yb2, yb2}, P2{ya2, ya2},
                                                      DOWN ? P2{zb, zb} : P2{za, za}, DOWN ? P2{za, za} : P2{zb, zb}))[0];
              if (KIND == 0 && a.r1sq > 0) {
                // spheres at the lane's row (per lane), tested only when some row of the block reaches one
                const int P1 = z + 2 * dz, P2p = z + dz;
                const int dh1 = eyh + (P1 - a.hz) * (P1 - a.hz), dc1 = eyc + (P1 - a.cz) * (P1 - a.cz);
                const int dh2 = eyh + (P2p - a.hz) * (P2p - a.hz), dc2 = eyc + (P2p - a.cz) * (P2p - a.cz);
                if (__builtin_amdgcn_ballot_w64(min(min(dh1, dc1), min(dh2, dc2)) < a.r1sq) != 0) {
                  const int x1 = eside ? xcol + CW : xcol - 2;
                  U1Ea[0] = sph_fix(dh1, dc1, x1, U1Ea[0]);
                  U1Ea[1] = sph_fix(dh1, dc1, x1 + 1, U1Ea[1]);
                  U2E = sph_fix(dh2, dc2, eside ? xcol + CW : xcol - 1, U2E);
                }
              }
              if (lane < NW) {
                es[nbuf][er][eside] = eside ? E[s2][1] : E[s2][2];
                eu[nbuf][er][eside] = adj(U1Ea);
                ev[nbuf][er][eside] = U2E;
              }
            }
            // boundary-plane publication (block-uniform, as the pairs): every wave's stores of output plane z
            // complete before the barrier, then one thread writes the L2 back (release) and counts the block's cells
            const bool pubStep = PUB && t >= 0 && (z < a.pubLo || z >= a.pubHi);
            if (pubStep) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (pubStep && lane == 0 && w == 0) {
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
              const unsigned long long cells =
                  (unsigned long long)(min(YO, a.hiy - yblk)) * (unsigned long long)(XH ? CW : a.hix - a.lox);
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
            if constexpr (EDGE) {
              U1Eb = U1Ec;
              U1Ec = U1Ea;
            }
            ++t;
            return true;
          };
          using I0 = std::integral_constant<int, 0>;
          using I1 = std::integral_constant<int, 1>;
          using I2 = std::integral_constant<int, 2>;
          using I3 = std::integral_constant<int, 3>;
          using L1 = std::integral_constant<int, (RM < 1 ? RM : 1)>;
          using L2 = std::integral_constant<int, (RM < 2 ? RM : 2)>;
          using LR = std::integral_constant<int, RM>;
          // warm-up: t = -4, -3 compute u1 only, t = -2, -1 u1 and u2 (one cycle of the slot rotation)
          step(I0{}, L1{});
          step(I1{}, L1{});
          step(I2{}, L2{});
          step(I3{}, L2{});
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
    body(std::integral_constant<int, 4>{});
  if (a.clk) { // measurement only (StencilTune::blockClock): every wave done, one lane stores the block's interval
    __syncthreads();
    if (lane == 0 && w == 0) {
      a.clk[2 * lb] = clk0;
      a.clk[2 * lb + 1] = wall_clock64();
    }
  }
}

// Whole periodic rows (fp32, 512 cells, x wrapped in-kernel): x-neighbours and the wrap by DPP lane rotates of the
// wave's own registers; the headline kernel (bench.py, one GPU). Kept apart from the XH form: sharing one body cost
// the whole-row instance ~3 % more VALU (window register moves) and 1.2 % of steady-state time (profiles/r6/r6n)
template <int KIND, bool PUB>
__global__ __launch_bounds__(64 * 12, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void
stencil7x3_wrap_kernel(StencilArgs<float> a, ZPartBounds zbounds) {
  constexpr int NW = 12;     // 3 waves per SIMD (168 VGPRs), 3 x 48 KiB of LDS
  using T = float;
  using NV = nf4;
  constexpr int V = 4, H = 2;
  constexpr int CS = 64 * V; // cells between a lane's chunks (chunk h = cells 256 h + 4 lane ..)
  constexpr int LS = V;      // cells between adjacent lanes
  constexpr int YO = NW - 6; // output rows per block
  constexpr int NC = 4;      // src planes in registers (one plane of lookahead)
  __shared__ NV cs[2][NW][H][64]; // src rows  (plane z+3dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows   (plane z+2dz at publish)
  __shared__ NV vs[2][NW][H][64]; // u2 rows   (plane z+dz at publish)

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.y)); // the wave's block row (wave-uniform: SGPR)
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  const X3Seg sg = x3_segments(a, zbounds, lb, nb, uint32_t(a.gy), uint32_t(a.gy), nzt);
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
    const bool pubOrder = PUB; // boundary-plane publication (a.pub, template: no live state otherwise)
    for (int pp = 0; pp < 2; ++pp) {
      // publishing: the leftover row groups' short second segments first (their face planes would otherwise come
      // out last), the main lockstep segment in its fixed direction
      const int pass = pubOrder ? 1 - pp : pp;
      uint32_t s = pass == 0 ? sg.s : sg.s2;
      const uint32_t e = pass == 0 ? sg.e : sg.e2;
      if (pass == 1 && !pubOrder) odd = sg.odd2;
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

        // spheres (Jacobi): a cell (x, y, P) is in the hot sphere iff (x - hx)^2 < Dh = yh - (P - hz)^2 with
        // yh = r1sq - (y - hy)^2 (per segment), in the cold one likewise; the row-plane has no sphere cell when both
        // bounds are <= 0 (r1sq = 0: never)
        const int yh = a.r1sq - (y - a.hy) * (y - a.hy), yc = a.r1sq - (y - a.cy) * (y - a.cy);
        struct RowSph {
          int Dh, Dc;
          bool hit;
        };
        auto row_sph = [&](int P) -> RowSph {
          RowSph r{0, 0, false};
          if (KIND == 0) {
            r.Dh = yh - (P - a.hz) * (P - a.hz);
            r.Dc = yc - (P - a.cz) * (P - a.cz);
            r.hit = max(r.Dh, r.Dc) > 0;
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
            const int Dh = rs.Dh, Dc = rs.Dc;
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
        // S of the wave's row (both chunks), x-neighbours and the periodic x wrap by lane rotates; exact /6 (div6v)
        auto row_update = [&](const NV(&cm)[H], const NV(&up)[H], const NV(&dn)[H], const NV(&zp)[H], const NV(&zm)[H],
                              NV(&o)[H]) -> T {
          static_assert(H == 2, "two chunks per lane");
          // named scalars, not arrays: a select between two array elements became a dynamically indexed private
          // array (scratch stores + loads on every row update, 449 vs 304 us per triple)
          const T r30 = rot_prev(cm[0][V - 1]), r31 = rot_prev(cm[1][V - 1]);
          const T l00 = rot_next(cm[0][0]), l01 = rot_next(cm[1][0]);
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
            o[h] = div6v<T, NV, V>(sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]));
          }
          return T(1);
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
            // every level reads the previous step's rows (buf): no level waits for another's LDS writes; each
            // level's row goes into the other buffer (its readers finished last step) right after its update, the src
            // row right after u1 (its load was waited for there): the step is bound by LDS write -> barrier -> LDS read
            // -> update three times, with only 2-3 waves per SIMD to overlap it (r5: 1381-1392 -> 1431-1443 Gcells/s
            // against publishing everything before the barrier, profiles/r5/v)
            auto levels = [&]() {
              NV A1[H], B1[H], A2[H], B2[H], A3[H], B3[H];
              auto rd = [&](NV(&sh)[2][NW][H][64], NV(&A)[H], NV(&B)[H]) {
#pragma unroll
                for (int h = 0; h < H; ++h) {
                  A[h] = sh[buf][wA][h][lane];
                  B[h] = sh[buf][wB][h][lane];
                }
              };
              if constexpr (LV >= 1) {
                rd(cs, A1, B1);
                (void)row_update(C[s1], A1, B1, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], U1a);
                sphere_row(row_sph(z + 2 * dz), U1a);
#pragma unroll
                for (int h = 0; h < H; ++h) cs[buf ^ 1][w][h][lane] = C[s2][h];
#pragma unroll
                for (int h = 0; h < H; ++h) us[buf ^ 1][w][h][lane] = U1a[h];
              }
              if constexpr (LV >= 2) {
                rd(us, A2, B2);
                (void)row_update(U1c, A2, B2, DOWN ? U1b : U1a, DOWN ? U1a : U1b, U2a);
                sphere_row(row_sph(z + dz), U2a);
#pragma unroll
                for (int h = 0; h < H; ++h) vs[buf ^ 1][w][h][lane] = U2a[h];
              }
              if constexpr (LV >= 3) {
                rd(vs, A3, B3);
                (void)row_update(U2c, A3, B3, DOWN ? U2b : U2a, DOWN ? U2a : U2b, o);
                sphere_row(row_sph(z), o);
              }
            };
            levels();
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
            if constexpr (LV < 1)
#pragma unroll
              for (int h = 0; h < H; ++h) cs[nbuf][w][h][lane] = C[s2][h];
            // boundary-plane publication (block-uniform, as the pairs): every wave's stores of output plane z
            // complete before the barrier, then one thread writes the L2 back (release) and counts the block's cells
            const bool pubStep = PUB && t >= 0 && (z < a.pubLo || z >= a.pubHi);
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
          using L1 = std::integral_constant<int, (R < 1 ? R : 1)>;
          using L2 = std::integral_constant<int, (R < 2 ? R : 2)>;
          using LR = std::integral_constant<int, R>;
          // warm-up: t = -4, -3 compute u1 only, t = -2, -1 u1 and u2 (one cycle of the slot rotation)
          step(I0{}, L1{});
          step(I1{}, L1{});
          step(I2{}, L2{});
          step(I3{}, L2{});
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
template <typename T, int KIND> static const void *x3_wrap_kernel_ptr() {
  if constexpr (std::is_same<T, float>::value)
    return (const void *)stencil7x3_wrap_kernel<KIND, false>;
  else
    return nullptr;
}

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

// the column width of the XH form: two 16-B chunks per lane
static int64_t x3_column_cells(int64_t elemSize) { return 2 * 64 * (16 / elemSize); }

bool stencil7x3_supported(const LocalDomain &dom, int64_t qi, const Rect3 &region, const StencilTune &tune) {
  if (dom.backend() != Backend::Device) return false;
  const int64_t es = dom.elem_size(qi);
  const bool f32 = dom.dtype(qi) == DType::F32 || (dom.dtype(qi) == DType::Bytes && es == 4);
  const bool f64 = dom.dtype(qi) == DType::F64 || (dom.dtype(qi) == DType::Bytes && es == 8);
  if (!f32 && !f64) return false;
  const Radius &rad = dom.radius();
  const Dim3 n = dom.size();
  const int wrapm = tune.wrap & 7;
  if (wrapm & 1) {
    // whole periodic rows: x wraps in-kernel by DPP rotates (fp32, exactly 512 cells)
    if (!f32 || n.x != 512 || !(stencil7x2_wrappable_axes(dom, qi, 1) & 1)) return false;
  } else {
    // x from 3-deep halos, in columns of CW cells
    if (rad.x(-1) < 3 || rad.x(1) < 3 || n.x % x3_column_cells(es) != 0) return false;
  }
  if (!(wrapm & 2) && (rad.y(-1) < 3 || rad.y(1) < 3)) return false;
  if (!(wrapm & 4) && (rad.z(-1) < 3 || rad.z(1) < 3)) return false;
  // S o S o S reaches (1, 2) / (2, 1) cells along two axes and (1, 1, 1) along three: every edge / corner halo whose
  // axes are all read from halos must be exchanged (its extent spans the face depths, LocalDomain::halo_extent)
  for (int i = 0; i < 27; ++i) {
    const Dim3 d = dir_from_index(i);
    const int nzc = (d.x != 0) + (d.y != 0) + (d.z != 0);
    const bool halo = !((d.x != 0 && (wrapm & 1)) || (d.y != 0 && (wrapm & 2)) || (d.z != 0 && (wrapm & 4)));
    if (nzc >= 2 && halo && rad.dir(d) < 1) return false;
  }
  const Rect3 cr = dom.get_compute_region();
  if (!(region.lo == cr.lo && region.hi == cr.hi)) return false; // the kernel sweeps whole sub-domains
  if (n.y < 3 || n.z < 16) return false;
  // 32-bit buffer offsets: within a plane (XH: a resource per plane), within the field (whole rows)
  if (dom.pitch(qi).x * dom.pitch(qi).y * es >= (int64_t(1) << 31)) return false;
  if ((wrapm & 1) && dom.buffer_bytes(qi) >= (int64_t(1) << 32) - 4096) return false;
  (void)x3_sink(dom.gpu(), true);
  const int64_t lox = rad.x(-1);
  return (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.curr_data(qi)) + lox * es) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.next_data(qi)) + lox * es) % 16 == 0) &&
         (dom.pitch(qi).x * es) % 16 == 0;
}

// the lockstep schedule of a triple sweep over cols row groups (columns) of nz planes with `slots` resident blocks
static X2Schedule x3_schedule(int64_t cols, int64_t nz, int64_t slots, const StencilTune &tune) {
  X2Schedule ls = x2_lockstep_schedule(slots, cols, nz);
  if (tune.x3sched == 1) {
    // lockstep over as many row groups as possible: P parts of cm = min(cols, slots / P) columns, the leftover columns
    // as second segments; P minimises the steps of one block (each segment runs 4 warm-up steps). A first guess:
    // x3_plan refines P with the leftover plans (512^3: Jacobi P = 4 over 64 groups + a lockstep phase of the 22
    // others, Astaroth P = 3 over 85 + one 2-row group in slices)
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
  if (tune.x3sched == 1 && cols > slots && !tune.publish) {
    // more row groups than resident blocks (fp64 1024^3 as 4 x 171 groups of 256-cell columns): rounds R of P z
    // parts over cm = ceil(cols / R) groups, every block in step with its y-neighbours in every round; leftover
    // groups as unsynchronised second segments re-fetch their halo rows (fp64 1024^3: 5.1 ms per triple and
    // quantity, profiles/r6/j)
    ls = X2Schedule();
    double best = 1e30;
    for (int64_t R = (cols + slots - 1) / slots; R <= 4 * ((cols + slots - 1) / slots); ++R)
      for (int64_t P = 1; P <= 4; ++P) {
        const int64_t cm = (cols + R - 1) / R;
        if (P * cm > slots || nz / P < 16) continue;
        const double cost = double(R) * (double(nz) / double(P) + 4);
        if (cost < best - 1e-9) {
          best = cost;
          ls.parts = int(P);
          ls.blocks = P * cm;
          ls.rounds = int(R);
        }
      }
  }
  return ls;
}

struct X3Plan {
  int P;
  uint32_t blocks;
  ZPartBounds b;
  double steps; // estimated steps of the longest block
};
// Plans a lockstep (seg 2) triple sweep of a.zparts parts over `blocks` blocks: sphere-weighted z-part bounds (Jacobi)
// and the leftover groups' second segments (StencilTune::x3left); with x3left != 0, x3sched 1 and no fixed x3parts, P
// too: the least estimated steps of the longest block over P = 2 .. 8 and both leftover plans
template <typename T>
static X3Plan x3_plan(const StencilArgs<T> &a, bool jac, int64_t cols, int64_t slots, uint32_t blocks,
                      const StencilTune &tune) {
  constexpr int NW = 12, YO = NW - 6;
  constexpr double kUnsync = 1.2; // a step of an unsynchronised slice vs a lockstep step (profiles/r6/r6ab)
  const int64_t nz = a.hiz - a.loz;
  const float w = jac ? tune.x3sphw : 0.f;
  auto plan = [&](int P, int64_t nbP, ZPartBounds &b) -> double {
    b = ZPartBounds{};
    const int64_t cm = nbP / P;
    if (jac) sphere_part_bounds(b, a, std::min<int64_t>(cm, a.gy), P, NW, YO, 3, w);
    const int mode = tune.x3left;
    ZPartBounds bg = b, bl = b;
    const double tg = mode == 1 || mode == 3
                          ? balance_leftover(bg, a, nbP, cm, P, cols, a.gy, NW, YO, 3, w, 4, mode == 3 ? kUnsync : 1.0)
                          : -1;
    const double tl = mode == 2 || mode == 3 ? lockstep_leftover(bl, a, nbP, cm, P, cols, a.gy, NW, YO, 3, w, 4, 16) : -1;
    if (tl >= 0 && (tg < 0 || tl <= tg)) {
      b = bl;
      return tl;
    }
    if (tg >= 0) {
      b = bg;
      return tg;
    }
    const std::vector<double> mc = lockstep_part_costs(b, a, cm, P, a.gy, NW, YO, 3, w, 4);
    const double left = cols > cm ? double((cols - cm) * nz) * kUnsync / double(nbP) + 4 : 0;
    return *std::max_element(mc.begin(), mc.end()) + left;
  };
  X3Plan pl{a.zparts, blocks, ZPartBounds{}, 0};
  if (tune.x3sched == 1 && tune.x3parts <= 0 && tune.x3left != 0) {
    double best = -1;
    // spheres: only parts the host can weight (P <= kZPartMaxParts); unweighted parts leave the sphere planes to one
    // or two parts (P = 7 with a lockstep second phase: 297 vs 228 us per 512^3 triple, profiles/r6/r6ac)
    const bool sph = jac && a.r1sq > 0 && w > 0;
    for (int P = 2; P <= (sph ? kZPartMaxParts : 8); ++P) {
      const int64_t cm = std::min<int64_t>(cols, slots / P);
      if (cm < 1 || nz / P < 16) continue;
      ZPartBounds b;
      const double t = plan(P, P * cm, b);
      if (best < 0 || t < best - 1e-9) {
        best = t;
        pl = X3Plan{P, uint32_t(P * cm), b, t};
      }
    }
  } else {
    pl.steps = plan(a.zparts, int64_t(blocks), pl.b);
  }
  return pl;
}

template <typename T, int KIND, bool XH>
static void apply_x3_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                       const StencilTune &tune) {
  constexpr int NW = 12, YO = NW - 6;
  StencilArgs<T> a = make_args<T>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  a.nt = tune.nontemporal ? 1 : 0;
  a.wrapm = tune.wrap & 7;
  // an axis read from its halos: no periodic shift (the kernel's row / plane wrap adds / subtracts wn)
  if (!(a.wrapm & 2)) a.wn[1] = 0;
  if (!(a.wrapm & 4)) a.wn[2] = 0;
  a.x0 = a.lox;
  a.remap = tune.xcdRemap ? 1 : 0;
  a.sphchunk = tune.x3sphchunk ? 1 : 0;
  a.sphr = int(sph.radius);
  const int nx = a.hix - a.lox, ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = XH ? int(nx / x3_column_cells(int64_t(sizeof(T)))) : 1;
  a.gy = (ny + YO - 1) / YO;
  const bool big = dom.buffer_bytes(qi) >= (int64_t(1) << 32) - 4096;
  const void *kern = XH ? (big ? (const void *)stencil7x3_xh_kernel<T, KIND, true, false>
                               : (const void *)stencil7x3_xh_kernel<T, KIND, false, false>)
                        : x3_wrap_kernel_ptr<T, KIND>();
  const int64_t cols = int64_t(a.gx) * a.gy;
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
  const X2Schedule ls = x3_schedule(cols, nz, slots, tune);
  if (tune.x2lockstep && ls.parts > 0) {
    a.seg = ls.rounds > 1 ? 3 : 2;
    a.zparts = ls.parts;
    a.zrounds = ls.rounds;
    blocks = uint32_t(ls.blocks);
  }
  // Lockstep parts (seg 2): the z-part bounds (sphere-weighted for Jacobi), the leftover groups' second segments
  // (StencilTune::x3left) and, with the cost model's P, the number of parts are planned per shape on the host
  // (x3_plan) and cached (host work of a few ms would otherwise precede every un-captured launch)
  ZPartBounds zb{};
  if (a.seg == 2) {
    static std::map<std::vector<int64_t>, X3Plan> cache;
    static std::mutex mu;
    int32_t wbits = 0;
    std::memcpy(&wbits, &tune.x3sphw, sizeof(wbits));
    const std::vector<int64_t> key{KIND, a.loy,  a.hiy, a.loz, a.hiz,          a.hy,        a.cy,
                                   a.hz, a.cz,   a.r1sq, int64_t(blocks), a.zparts, cols, a.gy,
                                   wbits, tune.x3left, tune.x3sched, tune.x3parts, slots};
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it == cache.end()) it = cache.emplace(key, x3_plan(a, KIND == 0, cols, slots, blocks, tune)).first;
    a.zparts = it->second.P;
    blocks = it->second.blocks;
    zb = it->second.b;
  }
  dom.set_device();
  a.sink = x3_sink(dom.gpu(), false);
  a.clk = reinterpret_cast<unsigned long long *>(tune.blockClock);
  STENCIL_REQUIRE(a.sink, "stencil7x3: no store sink on device " << dom.gpu() << " (stencil7x3_supported first)");
  if constexpr (XH || !std::is_same<T, float>::value) {
    auto *k = a.pub ? (big ? stencil7x3_xh_kernel<T, KIND, true, true> : stencil7x3_xh_kernel<T, KIND, false, true>)
                    : (big ? stencil7x3_xh_kernel<T, KIND, true, false> : stencil7x3_xh_kernel<T, KIND, false, false>);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64, NW), 0, stream, a, zb);
  } else {
    if (a.pub)
      hipLaunchKernelGGL((stencil7x3_wrap_kernel<KIND, true>), dim3(blocks), dim3(64, NW), 0, stream, a, zb);
    else
      hipLaunchKernelGGL((stencil7x3_wrap_kernel<KIND, false>), dim3(blocks), dim3(64, NW), 0, stream, a, zb);
  }
  HIP_CHECK(hipGetLastError());
}

X3PlanInfo stencil7x3_plan(const Dim3 &size, bool jacobi, const StencilTune &tune, int slots) {
  constexpr int YO = 6;
  StencilArgs<float> a{};
  a.hix = int(size.x);
  a.hiy = int(size.y);
  a.hiz = int(size.z);
  if (jacobi) {
    const Spheres s = Spheres::jacobi(Rect3(Dim3(0, 0, 0), size));
    a.hx = int(s.hot.x);
    a.hy = int(s.hot.y);
    a.hz = int(s.hot.z);
    a.cx = int(s.cold.x);
    a.cy = int(s.cold.y);
    a.cz = int(s.cold.z);
    a.r1sq = int((s.radius + 1) * (s.radius + 1));
  }
  a.gx = 1;
  a.gy = int((size.y + YO - 1) / YO);
  const int64_t cols = a.gy, nz = size.z;
  X3PlanInfo r;
  r.groups = int(cols);
  const X2Schedule ls = x3_schedule(cols, nz, slots, tune);
  r.parts = ls.parts;
  r.blocks = int(ls.blocks);
  r.rounds = ls.rounds;
  if (!tune.x2lockstep || ls.parts <= 0 || ls.rounds > 1) return r;
  a.zparts = ls.parts;
  const X3Plan pl = x3_plan(a, jacobi, cols, slots, uint32_t(ls.blocks), tune);
  r.parts = pl.P;
  r.blocks = int(pl.blocks);
  r.lockstepGroups = int(pl.blocks) / pl.P;
  r.steps = pl.steps;
  r.tabled = pl.b.lon != 0;
  if (pl.b.on)
    for (int g = 0; g < std::min<int>(r.lockstepGroups, kZPartMaxCols); ++g)
      for (int q = 0; q + 1 < pl.P; ++q) r.zb.push_back(pl.b.zb[g][q]);
  if (r.tabled)
    for (uint32_t lb = 0; lb < pl.blocks; ++lb) {
      r.l0.push_back(pl.b.l0[lb]);
      r.l1.push_back(pl.b.l1[lb]);
      r.odd.push_back(int((pl.b.ldir[lb / 32] >> (lb % 32)) & 1));
    }
  return r;
}

bool stencil7x3_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune) {
  if (!stencil7x3_supported(dom, qi, region, tune)) return false;
  const bool jac = kind == StencilKind::Jacobi, xh = !(tune.wrap & 1);
  if (dom.elem_size(qi) == 8) {
    jac ? apply_x3_t<double, 0, true>(dom, qi, region, sph, stream, tune)
        : apply_x3_t<double, 1, true>(dom, qi, region, sph, stream, tune);
  } else if (xh) {
    jac ? apply_x3_t<float, 0, true>(dom, qi, region, sph, stream, tune)
        : apply_x3_t<float, 1, true>(dom, qi, region, sph, stream, tune);
  } else {
    jac ? apply_x3_t<float, 0, false>(dom, qi, region, sph, stream, tune)
        : apply_x3_t<float, 1, false>(dom, qi, region, sph, stream, tune);
  }
  return true;
}

} // namespace stencil
