// Two fused 7-point steps per sweep (temporal blocking): dst = S(S(src)) on a region, for gfx950.
//
// A Jacobi/Astaroth step reads 4 B and writes 4 B per cell: at HBM speed that is the whole cost. Fusing two steps
// into one z-march reads the field once and writes it once per TWO steps, and needs one halo exchange of depth 2
// (faces 2, edges 1: the 25-point footprint of S o S) per two steps instead of two exchanges of depth 1. This is
// the "halo multiplier" / deep-halo item of the reference's future-work list (README.md:218-220), built for CDNA4:
//
//   block  = NW waves stacked in y, one src row per wave (the outer 2 rows on each side are a redundant y halo),
//            one 64-lane column of 16-B x-chunks (as stencil7_lds_kernel)
//   step t = output plane z (z-march direction dz = +-1):
//     1. issue the load of src plane z+(2+PF)dz    (PF planes of lookahead in registers)
//     2. u1 = S(src) at plane z+dz for the wave's row (y-neighbours: adjacent waves through LDS), plus u1 one cell
//        outside the wave's x range on the edge lanes, so S(u1) never needs another wave's registers
//     3. u2 = S(u1) at plane z from the register window u1(z-dz), u1(z), u1(z+dz) + LDS y-neighbours
//     4. publish the src row of plane z+2dz and the u1 row of plane z+dz (double-buffered LDS, one barrier)
// Summation order and the /6 are the single-step kernel's, and every u1 value is computed exactly as the single
// step computes it, so S(S(src)) is bitwise equal to two sequential single steps (tests compare with torch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "stencil/rt/hip_check.hpp"
#include "stencil_common.hpp"
#include "stencil_wave.hpp"

namespace stencil {

// Block = NW waves, ONE src row per wave: the block's src rows are [yblk-2, yblk-2+NW); u1 is valid on the inner
// NW-2 of them and u2 (the output) on the inner NW-4, so the block writes YO = NW-4 rows and every wave runs the
// same code (the two outer rows on each side are a redundant y halo, re-read from L2 by the neighbouring block).
// z: the src window holds planes z .. z+(2+PF)dz; the last PF planes are in flight, so a row load is issued PF
// steps before it is consumed. The march direction is a template argument of the loop body (DOWN), so selecting
// the +z / -z neighbour costs nothing.
// WRAP (in-kernel periodic wrap, StencilTune::wrap): 0 none, 1 y/z only, 2 x too. A template value so that only
// the x-wrap instance pays for separate edge loads (3 loads per row instead of the 2 overlapping 16-B loads the
// compiler forms around the chunk when the edge cells are adjacent to it)
template <typename T, int NW, int PF, int KIND, int WRAP>
// 12 waves: 3 per SIMD, so the register budget is 168 VGPRs (4 waves/SIMD for 8 and 16: 128)
__global__ __launch_bounds__(64 * NW, (NW == 12 ? 3 : 4))
__attribute__((amdgpu_waves_per_eu(NW == 12 ? 3 : 4, NW == 12 ? 3 : 4))) void stencil7x2_kernel(StencilArgs<T> a) {
  using NV = typename Vec16<T>::native;
  using P2 = typename Pk<T>::t;
  constexpr int V = Vec16<T>::N;
  constexpr int YO = NW - 4;
  constexpr int NC = 3 + PF; // src window planes
  static_assert(NW > 4, "a block needs more than its 4 halo rows");
  __shared__ NV cs[2][NW][64]; // src row of every wave, plane z+2dz at publish (= z+dz when read)
  __shared__ NV us[2][NW][64]; // u1 row of every wave, plane z+dz at publish (= z when read)
  __shared__ T ce[2][NW][2];   // src edge scalars of the published rows: [0] at x-1 (lane 0), [1] at x+V

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = int(threadIdx.y);
  // The block's work is a range [s, e) of the linear (column, plane) space, column = bx * gy + by (y-neighbour
  // columns are adjacent, so with the XCD remap their shared halo rows meet in one L2). Chunk mode: one fixed
  // z-chunk. Segment mode (a.seg): gridDim.x = the resident block slots, each takes an equal share, i.e. one or
  // two z segments of about ncols * nz / slots planes: no partly empty last round of blocks, and the fewest
  // 4-plane warm-ups per useful plane.
  // 32-bit block-uniform bookkeeping (the host guarantees ncols * nz < 2^32): every extra live register of the
  // loop around the march would be spilled from the march's hot loop, which uses all 128 VGPRs
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  uint32_t s, e;
  if (a.seg) {
    const uint64_t W = uint64_t(uint32_t(a.gx) * uint32_t(a.gy)) * nzt;
    s = uint32_t(uint64_t(lb) * W / nb);
    e = uint32_t(uint64_t(lb + 1) * W / nb);
  } else {
    const uint32_t col = lb / uint32_t(a.gz);
    s = col * nzt + (lb % uint32_t(a.gz)) * uint32_t(a.zc);
    e = min(s + uint32_t(a.zc), (col + 1) * nzt);
  }
  // alternate the march direction between neighbouring pieces of a column, so the planes two pieces share are
  // read by both at about the same time (warm-up of one, tail of the other)
  bool odd = a.seg ? (lb & 1) != 0 : ((s % nzt) / uint32_t(a.zc) & 1) != 0;
  while (s < e) { // block-uniform
  const uint32_t col = s / nzt;
  const int zo = int(s - col * nzt);
  const int nzs = int(min(nzt - uint32_t(zo), e - s));
  s += uint32_t(nzs);
  // column order: y-major (y-neighbour columns adjacent: their shared halo rows meet in one L2) or x-major (the
  // x-neighbour columns of a row range adjacent: the cells one column's edge lanes read from the next, and with x
  // wrap the far row end, are read by a block of the same XCD at the same time)
  int bx, by;
  if (a.xfast) {
    by = int(col / uint32_t(a.gx));
    bx = int(col - uint32_t(by) * uint32_t(a.gx));
  } else {
    bx = int(col / uint32_t(a.gy));
    by = int(col - uint32_t(bx) * uint32_t(a.gy));
  }
  const int zs = a.loz + zo;
  const int ze = zs + nzs;
  const bool down = odd != (a.flip != 0);
  odd = !odd;
  const int c = bx * 64 + lane;
  const bool cvalid = c < a.nchunks;
  const int cl = cvalid ? c : a.nchunks - 1;
  const int xb = a.x0 + cl * V;
  const int yblk = a.loy + YO * by; // first output row of the block
  const int y = yblk - 2 + w;       // this wave's row
  if (yblk >= a.hiy) continue; // block-uniform

  const bool edgeL = lane == 0;
  const bool edgeR = lane == 63 || c + 1 >= a.nchunks;
  const bool fullX = xb >= a.lox && xb + V <= a.hix;
  const bool outRow = w >= 2 && w < NW - 2 && y < a.hiy && cvalid;
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1; // outer waves: garbage u1, never consumed
  // wave-uniform: u1 only on rows 1 .. NW-2, u2 only on the output rows (see stencil7x2_row_kernel)
  const bool needU1 = w >= 1 && w < NW - 1, needU2 = w >= 2 && w < NW - 2; // edge waves: source rows only

  // y-wrapped rows read their periodic image (one conditional shift: rows reach 2 beyond the region, ny >= 2)
  const int yw =
      (WRAP >= 1 && (a.wrapm & 2)) ? (y < a.wlo[1] ? y + a.wn[1] : (y >= a.wlo[1] + a.wn[1] ? y - a.wn[1] : y)) : y;
  const int yc = yw < 0 ? 0 : (yw > a.rawYm1 ? a.rawYm1 : yw);
  // addresses = wave-uniform plane base (SGPRs) + a 32-bit per-lane byte offset within the plane, so the loads and
  // stores use the saddr + voffset form and each lane holds one offset VGPR instead of 64-bit pointers
  const uint32_t rowoff = uint32_t((yc * int64_t(a.px) + xb) * int64_t(sizeof(T)));
  const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));
  // x wrap: the first interior chunk reads its left edge cells (x-1, x-2) at x-1+nx, x-2+nx, the last one its right
  // edge cells at x+V-nx, x+V+1-nx (the other edge pair of such a lane is never consumed and stays in the row,
  // stencil7x2_wrappable_axes); every other lane reads the edge cells beside its chunk
  int xdelta = 0;
  if (WRAP == 2 && (a.wrapm & 1)) xdelta = xb == a.wlo[0] ? a.wn[0] : (xb + V == a.wlo[0] + a.wn[0] ? -a.wn[0] : 0);
  // byte offset of the edge pointer from (plane base - 64 B): a right-wrap lane's pointer can sit up to 2 cells
  // before raw x = 0 (inside the row's front padding), so on raw row 0 the offset from the plane base is negative;
  // the 64-B bias keeps the unsigned 32-bit offset >= 0 (the front padding is < 64 B)
  const uint32_t edgeoff = uint32_t(int(rowoff) + 64 + xdelta * int(sizeof(T)));
  // z wrap (block-uniform): consumed planes reach 2 beyond the region (one conditional shift, nz >= 2); deeper
  // lookahead planes are never consumed and only need a valid address (the clamp)
  const int zwn = (WRAP >= 1 && (a.wrapm & 4)) ? a.wn[2] : 0, zwlo = a.wlo[2], zwhi = a.wlo[2] + zwn;
  auto zcl = [&](int zz) { // branch-free (zwn = 0: identity shifts), so the unrolled march stays one basic block
    if constexpr (WRAP >= 1) {
      zz += zz < zwlo ? zwn : 0;
      zz -= zz >= zwhi ? zwn : 0;
    }
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  auto planep = [&](int zz) -> const char * { return reinterpret_cast<const char *>(a.src + int64_t(zcl(zz)) * a.pxy); };
  // sphere membership of the row at plane P: y/z part once per row, per-cell test only for the few hit rows
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
  auto fix = [&](const RowSph &rs, int x, T v) -> T {
    const bool hot = (x - a.hx) * (x - a.hx) < a.r1sq - rs.dh;
    const bool cold = (x - a.cx) * (x - a.cx) < a.r1sq - rs.dc;
    return hot ? T(1) : (cold ? T(0) : v);
  };
  // S at this wave's row chunk `cm`: x-neighbours by DPP lane shifts (+ edge scalars at the wave edges)
  auto apply_row = [&](const NV &cm, const NV &up, const NV &dn, const NV &zp, const NV &zm, T eL, T eR,
                       const RowSph &rs) -> NV {
    const T sl = from_prev_lane<T>(cm[V - 1]);
    const T sr = from_next_lane<T>(cm[0]);
    const T left = edgeL ? eL : sl;
    const T right = edgeR ? eR : sr;
    NV vpx, vmx;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      vpx[e] = e < V - 1 ? cm[e + 1] : right;
      vmx[e] = e > 0 ? cm[e - 1] : left;
    }
    NV o = div6v<T, NV, V>(sum6v<T, KIND>(vpx, vmx, dn, up, zp, zm));
    if (KIND == 0 && rs.hit) {
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] = fix(rs, xb + e, o[e]);
    }
    return o;
  };

  auto march = [&](auto downTag) {
    constexpr bool DOWN = decltype(downTag)::value;
    constexpr int dz = DOWN ? -1 : 1;
    const int z0 = DOWN ? ze - 1 : zs;
    // ---- windows: a ring of NC src planes; the step of phase k (t+2 = k mod NC) finds plane z + j dz in slot
    // (k+j) mod NC. The loop is unrolled over the NC phases, so a plane's registers never move while its load is
    // in flight (a register rotation would force a wait on the load right after issuing it). ----
    NV C[NC];             // src rows
    T CL[NC], CR[NC];     // src at x-1 / x+V (edge lanes)
    T LL[NC], RR[NC];     // src at x-2 / x+V+1 (edge lanes)
    NV Ub, Uc, Ua;        // u1 planes z-dz, z, z+dz
    P2 UcE, UaE;          // u1 at (x-1, x+V), planes z and z+dz
    auto load_row = [&](int zz, int k) {
      const char *b = planep(zz);
      const T *p = reinterpret_cast<const T *>(b + rowoff);
      // 16-B aligned (rowoff, the bias and the +-nx shift of whole chunks are): the edge pairs then load as the
      // aligned 16-B vectors around the chunk, as in the copy-halo instance
      const T *pe = WRAP == 2 ? static_cast<const T *>(__builtin_assume_aligned((b - 64) + edgeoff, 16)) : p;
      // every lane loads the edge scalars (in-row addresses, same cache lines as the chunk; only the edge lanes
      // use them): masked loads would sit behind exec branches, and the waitcnt pass, counting the path that skips
      // them, would then wait on this step's own loads and void the lookahead
      C[k] = *reinterpret_cast<const NV *>(p);
      CL[k] = pe[-1];
      CR[k] = pe[V];
      LL[k] = pe[-2];
      RR[k] = pe[V + 1];
    };

    // warm-up: the loop starts two planes early (t = -2: u1 only), window planes z0-2dz .. z0+(NC-2)dz
    {
      const int zw = z0 - 2 * dz;
#pragma unroll
      for (int k = 0; k < NC - 1; ++k) load_row(zw + k * dz, k);
      cs[0][w][lane] = C[1];
      if (edgeL) ce[0][w][0] = CL[1];
      if (edgeR) ce[0][w][1] = CR[1];
      __syncthreads();
    }

    int buf = 0;
    int t = -2;
    auto step = [&](auto phase) -> bool {
      constexpr int k = decltype(phase)::value;
      constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
      if (t >= nzs) return false;
      const int z = z0 + t * dz;
      const int P = z + dz;
      // 1. lookahead load into the slot of the plane that died last step
      load_row(z + (NC - 1) * dz, sn);
      // 2. u1 at plane z+dz (row + the two edge cells as one pair)
      const NV cA = cs[buf][wA][lane], cB = cs[buf][wB][lane];
      const T cAL = ce[buf][wA][0], cAR = ce[buf][wA][1]; // LDS broadcasts
      const T cBL = ce[buf][wB][0], cBR = ce[buf][wB][1];
      if (!needU1) {
        Ua = C[s1]; // never read
        UaE = P2{T(0), T(0)};
      } else {
        const RowSph rs = row_sph(P);
        Ua = apply_row(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], CL[s1], CR[s1], rs);
        const P2 epx = {C[s1][0], RR[s1]}, emx = {LL[s1], C[s1][V - 1]}, epy = {cBL, cBR}, emy = {cAL, cAR};
        const P2 ezp = DOWN ? P2{CL[s0], CR[s0]} : P2{CL[s2], CR[s2]};
        const P2 ezm = DOWN ? P2{CL[s2], CR[s2]} : P2{CL[s0], CR[s0]};
        UaE = div6v<T, P2, 2>(sum6v<T, KIND>(epx, emx, epy, emy, ezp, ezm));
        if (KIND == 0 && rs.hit) {
          UaE[0] = fix(rs, xb - 1, UaE[0]);
          UaE[1] = fix(rs, xb + V, UaE[1]);
        }
      }
      // 3. u2 at plane z
      if (t >= 0 && needU2) {
        const NV uA = us[buf][wA][lane], uB = us[buf][wB][lane];
        const NV o = apply_row(Uc, uA, uB, DOWN ? Ub : Ua, DOWN ? Ua : Ub, UcE[0], UcE[1], row_sph(z));
        if (outRow) {
          T *dp = reinterpret_cast<T *>(reinterpret_cast<char *>(a.dst + int64_t(z) * a.pxy) + outoff);
          if (fullX) {
            if (a.nt)
              __builtin_nontemporal_store(o, reinterpret_cast<NV *>(dp));
            else
              *reinterpret_cast<NV *>(dp) = o;
          } else {
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (xb + e >= a.lox && xb + e < a.hix) dp[e] = o[e];
          }
        }
      }
      // 4. publish src plane z+2dz and u1 plane z+dz
      const int nbuf = buf ^ 1;
      cs[nbuf][w][lane] = C[s2];
      if (edgeL) ce[nbuf][w][0] = CL[s2];
      if (edgeR) ce[nbuf][w][1] = CR[s2];
      if (needU1) us[nbuf][w][lane] = Ua; // the edge waves' u1 is never read
      __syncthreads();
      buf = nbuf;
      // 5. the u1 window (computed values: plain moves)
      Ub = Uc;
      Uc = Ua;
      UcE = UaE;
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
}

// Whole-row variant of the fused pair (fp32, x periodic and wrapped in-kernel, 512 interior cells per row, i.e. the
// one-GPU 512^3 sweep). Each lane holds two 16-B chunks of its row, x = lox + 4*lane and x = lox + 256 + 4*lane, so
// one wave covers the whole row and every x-neighbour - the periodic ones included - is a DPP lane rotate of the
// wave's own registers:
//   left of chunk h  = lane 0 ? (chunk h-1 of lane 63) : (chunk h of lane-1)   -> wave_ror:1 of the chunks' last cells
//   right of chunk h = lane 63 ? (chunk h+1 of lane 0) : (chunk h of lane+1)   -> wave_rol:1 of their first cells
// Against stencil7x2_kernel (one 16-B chunk per lane, two 256-cell columns per row) this drops, per row and plane:
// the two edge-scalar loads (and their far-row-end sectors at the periodic faces: 6 % of the fetched bytes), the
// edge-scalar LDS exchange, the u1 edge-pair computation, and half of the per-step fixed cost (plane addressing,
// sphere tests, loop control, one barrier per 12 rows of 512 cells instead of 256). Each chunk load / store is one
// fully coalesced 1 KB wave instruction. Block, z-march, LDS y-neighbours, summation order, exact /6 and spheres
// are those of stencil7x2_kernel: S(S(src)) is bitwise equal to two single steps.
//
// Ragged rows (RAG: 256 (H-1) < nx < 256 H, e.g. the 645- and 813-cell rows of the 2- and 4-GPU weak-scaling
// ladder): H chunks per lane, the last chunk group partly past the row end. The periodic neighbours of the row ends
// are then not where the rotates put them, so each row application broadcasts the first cell (x = 0) and the last one
// (x = nx-1, lane Lr, element kr of chunk H-1) with v_readlane and selects them in: left of x = 0 on lane 0, right of
// x = nx-1 on lane Lr. Chunks wholly past the row end load the row start (finite values, never selected) and store
// nothing; the partial chunk stores its cells one by one.
//
// Tail rows (TL: 256 H < nx <= 256 H + 64, e.g. the 4-GPU ladder's 813): H = 3 whole chunks per lane and one more
// cell per lane after them (x = 768 + lane, lanes < nx - 768), so a row of up to 832 cells still fits one wave at
// 98 % lane use for 813 (four chunks per lane need 196 KiB of LDS and spill). The tail's x-neighbours are lane
// rotates of the tail (lane 0's left is chunk H-1 of lane 63, the right of chunk H-1 on lane 63 is lane 0's tail);
// the row ends wrap through the broadcast first cell and last tail cell. +12 KiB of LDS for the tail rows.
// (column, plane) segments of one fused-pair block over ncols columns of nzt planes (column c covers [c nzt,
// (c+1) nzt)). seg 2 = lockstep: a.zparts = P blocks per column for the first nb / P columns, each marching one of
// the P z parts, consecutive blocks on y-adjacent columns of one part (one XCD after the remap), so their shared
// y-halo rows meet in L2; the columns left over spread over all blocks as short second segments [s2, e2); parts
// alternate their z direction. seg 1 = balanced split of all (column, plane) pairs; seg 0 = fixed z chunks.
struct X2Segs {
  uint32_t s, e, s2, e2;
  bool odd; // first segment marches down (before the flip)
};
template <typename T>
__device__ __forceinline__ X2Segs x2_segments(const StencilArgs<T> &a, uint32_t lb, uint32_t nb, uint32_t ncols,
                                              uint32_t nzt, const ZPartBounds *B = nullptr, bool useB = true) {
  X2Segs r{0, 0, 0, 0, false};
  if (a.seg == 3) { // rounds (x2_pass): parts alternate their z direction as in seg 2
    r.odd = ((lb / (nb / uint32_t(a.zparts))) & 1) != 0;
    return r;
  }
  if (a.seg == 2) {
    const uint32_t P = uint32_t(a.zparts);
    const uint32_t cm = nb / P;
    // part-major: consecutive blocks take y-adjacent columns of one part (column-major: 1146 vs 1164 Gcells/s, r2s3)
    const uint32_t qq = lb / cm, col = lb % cm;
    uint32_t zlo = qq * nzt / P, zhi = (qq + 1) * nzt / P;
    if (useB && B && B->on && col < uint32_t(kZPartMaxCols)) { // sphere-weighted parts (Jacobi, sphere_part_bounds)
      zlo = qq > 0 ? uint32_t(B->zb[col][qq - 1]) : 0;
      zhi = qq + 1 < P ? uint32_t(B->zb[col][qq]) : nzt;
    }
    r.s = col * nzt + zlo;
    r.e = col * nzt + zhi;
    r.odd = (qq & 1) != 0;
    const uint64_t LW = uint64_t(ncols - cm) * nzt;
    r.s2 = cm * nzt + uint32_t(uint64_t(lb) * LW / nb);
    r.e2 = cm * nzt + uint32_t(uint64_t(lb + 1) * LW / nb);
  } else if (a.seg) {
    const uint64_t W = uint64_t(ncols) * nzt;
    r.s = uint32_t(uint64_t(lb) * W / nb);
    r.e = uint32_t(uint64_t(lb + 1) * W / nb);
    r.odd = (lb & 1) != 0;
  } else {
    const uint32_t col = lb / uint32_t(a.gz);
    r.s = col * nzt + (lb % uint32_t(a.gz)) * uint32_t(a.zc);
    r.e = min(r.s + uint32_t(a.zc), (col + 1) * nzt);
    r.odd = ((r.s % nzt) / uint32_t(a.zc) & 1) != 0;
  }
  return r;
}
// the block's segment of pass p ([s, e) in (column, plane) space); false when it has no more. seg 3 = rounds of
// whole columns (a.zparts rounds): pass p is column p nb + lb, all blocks on adjacent columns in step
template <typename T>
__device__ __forceinline__ bool x2_pass(const StencilArgs<T> &a, const X2Segs &sg, int p, uint32_t lb, uint32_t nb,
                                        uint32_t ncols, uint32_t nzt, uint32_t &s, uint32_t &e) {
  if (a.seg == 3) { // a.zrounds rounds of a.zparts z parts over cm = nb / parts columns each
    const uint32_t P = uint32_t(a.zparts), cm = nb / P, qq = lb / cm;
    const uint32_t col = uint32_t(p) * cm + lb % cm;
    if (p >= a.zrounds || col >= ncols) return false;
    s = col * nzt + qq * nzt / P;
    e = col * nzt + (qq + 1) * nzt / P;
    return true;
  }
  if (p > 1) return false;
  s = p == 0 ? sg.s : sg.s2;
  e = p == 0 ? sg.e : sg.e2;
  return true;
}

template <int NW, int PF, int KIND, int H = 2, bool RAG = false, bool TL = false, bool PUB = false>
__global__ __launch_bounds__(64 * NW, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void
stencil7x2_row_kernel(StencilArgs<float> a, ZPartBounds zbounds) {
  using T = float;
  using NV = nf4;
  constexpr int V = 4;          // H = chunks per lane
  constexpr int HS = 64 * V;    // cells between a lane's chunks
  constexpr int YO = NW - 4;
  constexpr int NC = 3 + PF;
  static_assert(NW == 12 && H <= 3, "3 waves per SIMD: the 168-VGPR budget; 144 KiB of LDS at H = 3");
  static_assert(RAG || TL || H == 2, "unragged rows: 512 cells");
  static_assert(!(RAG && TL), "ragged last chunk or a tail, not both");
  __shared__ NV cs[2][NW][H][64]; // src rows (plane z+2dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows (plane z+dz at publish)
  __shared__ T cst[TL ? 2 : 1][TL ? NW : 1][TL ? 64 : 1]; // tail cells of the src / u1 rows (TL)
  __shared__ T ust[TL ? 2 : 1][TL ? NW : 1][TL ? 64 : 1];

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  // tail rows (three chunks plus a tail cell per lane) are over the 168-VGPR budget with per-cell sphere tests (192,
  // 24 spilled): their wave index, row and per-row sphere x bounds are made wave-uniform (SGPRs; 165, no scratch).
  // Ragged three-chunk rows keep the per-cell test: with the bounds they ran 10 % slower (645x645x323 867-891 vs
  // 972 Gcells/s, same box; the 512-cell kernel with bounds 1047-1052 vs 1142-1157; profiles/r3/s3/ab_sphere.txt)
  const int w = TL ? __builtin_amdgcn_readfirstlane(int(threadIdx.y)) : int(threadIdx.y);
  // raw buffer over the source field: row offsets from raw [0,0,0] are non-negative and the field is below 4 GiB
  // (apply_x2row_t checks)
  const __amdgpu_buffer_rsrc_t srcRsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.src), 0, -1, 0x00020000);
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  // z-march direction alternates between neighbouring segments (their shared boundary planes meet in cache); in the
  // part-major lockstep order it alternates by part, so y-adjacent blocks march together
  const X2Segs sg = x2_segments(a, lb, nb, uint32_t(a.gy), nzt, &zbounds);
  uint32_t s = 0, e = 0;
  bool odd = sg.odd;
  for (int pass = 0; x2_pass(a, sg, pass, lb, nb, uint32_t(a.gy), nzt, s, e); ++pass) {
  while (s < e) { // block-uniform
  const uint32_t by = s / nzt; // one column per row range
  const int zo = int(s - by * nzt);
  const int nzs = int(min(nzt - uint32_t(zo), e - s));
  s += uint32_t(nzs);
  const int zs = a.loz + zo;
  const int ze = zs + nzs;
  const bool down = odd != (a.flip != 0);
  odd = !odd;
  const int xb = a.lox + lane * V; // chunk h at xb + h * HS
  const int yblk = a.loy + YO * int(by);
  const int y = yblk - 2 + w;
  if (yblk >= a.hiy) continue;
  const bool outRow = w >= 2 && w < NW - 2 && y < a.hiy;
  // wave-uniform: u1 is needed on rows 1 .. NW-2 of the block (the y-neighbours of the output rows), u2 only on the
  // output rows; the edge waves only load and publish their source rows
  const bool needU1 = w >= 1 && w < NW - 1, needU2 = w >= 2 && w < NW - 2; // edge waves: source rows only
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1;
  const bool lane0 = lane == 0, lane63 = lane == 63;
  // ragged rows: the last cell x = nx-1 sits in chunk H-1 of lane Lr, element kr
  const int xl = a.hix - a.lox - 1 - HS * (H - 1);
  const int Lr = xl >> 2, kr = xl & 3;
  const bool lastIn = !RAG || lane <= Lr; // chunk H-1 of this lane holds cells of the row
  auto choff = [&](int h) -> int { // byte offset of chunk h from the lane's first chunk
    return (h < H - 1 || lastIn) ? h * HS * int(sizeof(T)) : 0;
  };
  // tail rows: cell x = 256 H + lane on lanes < ntl (the others read the row start: finite, never stored)
  const int ntl = TL ? a.hix - a.lox - HS * H : 0;
  const int Lt = ntl - 1;
  const bool tailIn = lane < ntl;
  const int toff = (tailIn ? HS * H - (V - 1) * lane : -V * lane) * int(sizeof(T)); // from the lane's chunk 0

  const int yw = (a.wrapm & 2) ? (y < a.wlo[1] ? y + a.wn[1] : (y >= a.wlo[1] + a.wn[1] ? y - a.wn[1] : y)) : y;
  const int yc = yw < 0 ? 0 : (yw > a.rawYm1 ? a.rawYm1 : yw);
  const uint32_t rowoff = uint32_t((yc * int64_t(a.px) + xb) * int64_t(sizeof(T)));
  const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));
  const int zwn = (a.wrapm & 4) ? a.wn[2] : 0, zwlo = a.wlo[2], zwhi = a.wlo[2] + zwn;
  auto zcl = [&](int zz) {
    zz += zz < zwlo ? zwn : 0;
    zz -= zz >= zwhi ? zwn : 0;
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  auto planep = [&](int zz) -> const char * { return reinterpret_cast<const char *>(a.src + int64_t(zcl(zz)) * a.pxy); };
  // spheres: a cell (x, y, P) is hot iff (x - hx)^2 < Dh = sqh - (P - hz)^2, sqh = r1sq - (y - hy)^2 (per segment),
  // cold likewise; no sphere cell in the row-plane when both are <= 0 (r1sq = 0: never). Two live scalars per row
  // instead of the centres and r1sq (SGPR pressure: spills to VGPR lanes in the steady loop)
  const int sqh = a.r1sq - (y - a.hy) * (y - a.hy), sqc = a.r1sq - (y - a.cy) * (y - a.cy);
  struct RowSph {
    int Dh, Dc;
    bool hit;
    int hlo, hhi, clo, chi; // TL: the row's hot / cold cells are hlo <= x <= hhi / clo <= x <= chi (wave-uniform)
  };
  // largest s >= 0 with s * s < d (d > 0), exact: float estimate, then integer correction
  auto isqrt_below = [](int d) -> int {
    int s = int(__builtin_sqrtf(float(d - 1)));
    while (s > 0 && s * s > d - 1) --s;
    while ((s + 1) * (s + 1) <= d - 1) ++s;
    return s;
  };
  auto row_sph = [&](int P) -> RowSph {
    RowSph r{0, 0, false, 0, 0, 0, 0};
    if (KIND == 0) {
      r.Dh = sqh - (P - a.hz) * (P - a.hz);
      r.Dc = sqc - (P - a.cz) * (P - a.cz);
      r.hit = max(r.Dh, r.Dc) > 0;
      if constexpr (TL) {
        // (x - hx)^2 < Dh  <=>  |x - hx| <= s with s * s < Dh: bounds instead of per-cell squares
        constexpr int kNone = -(1 << 24); // empty interval: never matches a cell coordinate
        const int sh = r.Dh > 0 ? isqrt_below(r.Dh) : -1;
        const int sc = r.Dc > 0 ? isqrt_below(r.Dc) : -1;
        r.hlo = __builtin_amdgcn_readfirstlane(sh >= 0 ? a.hx - sh : kNone);
        r.hhi = __builtin_amdgcn_readfirstlane(sh >= 0 ? a.hx + sh : kNone);
        r.clo = __builtin_amdgcn_readfirstlane(sc >= 0 ? a.cx - sc : kNone);
        r.chi = __builtin_amdgcn_readfirstlane(sc >= 0 ? a.cx + sc : kNone);
      }
    }
    return r;
  };
  auto fix = [&](const RowSph &rs, int x, T v) -> T {
    bool hot, cold;
    if constexpr (TL) {
      hot = unsigned(x - rs.hlo) <= unsigned(rs.hhi - rs.hlo);
      cold = unsigned(x - rs.clo) <= unsigned(rs.chi - rs.clo);
    } else {
      hot = (x - a.hx) * (x - a.hx) < rs.Dh;
      cold = (x - a.cx) * (x - a.cx) < rs.Dc;
    }
    return hot ? T(1) : (cold ? T(0) : v);
  };
  // S of the wave's row (both chunks), x-neighbours by lane rotates
  // the tail arguments (cmt .. zmt, ot) are the same terms for the tail cell of each row (TL only)
  auto apply_row = [&](const NV (&cm)[H], const NV (&up)[H], const NV (&dn)[H], const NV (&zp)[H], const NV (&zm)[H],
                       const RowSph &rs, NV (&o)[H], T cmt, T upt, T dnt, T zpt, T zmt, T &ot) {
    T r3[H], l0[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      r3[h] = rot_prev(cm[h][V - 1]);
      l0[h] = rot_next(cm[h][0]);
    }
    T first = 0, last = 0; // ragged / tail rows: the cells x = 0 and x = nx-1, broadcast
    if constexpr (RAG) {
      first = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cm[0][0]), 0));
      const T e = kr == 0 ? cm[H - 1][0] : (kr == 1 ? cm[H - 1][1] : (kr == 2 ? cm[H - 1][2] : cm[H - 1][3]));
      last = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), Lr));
    }
    T tp = 0, tn = 0; // tail of lane-1 / lane+1
    if constexpr (TL) {
      first = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cm[0][0]), 0));
      last = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cmt), Lt));
      tp = rot_prev(cmt);
      tn = rot_next(cmt);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const T left = lane0 ? ((RAG || TL) && h == 0 ? last : r3[(h + H - 1) % H]) : r3[h];
      const T right = lane63 ? (TL && h == H - 1 ? tn : l0[(h + 1) % H]) : l0[h];
      NV vpx, vmx;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        vpx[k] = k < V - 1 ? cm[h][k + 1] : right;
        vmx[k] = k > 0 ? cm[h][k - 1] : left;
      }
      if (RAG && h == H - 1) {
#pragma unroll
        for (int k = 0; k < V; ++k) vpx[k] = (lane == Lr && kr == k) ? first : vpx[k];
      }
      o[h] = div6v<T, NV, V>(sum6v<T, KIND>(vpx, vmx, dn[h], up[h], zp[h], zm[h]));
    }
    if constexpr (TL) {
      const T lt = lane0 ? r3[H - 1] : tp;  // lane 0: chunk H-1's last cell on lane 63
      const T rt = lane == Lt ? first : tn; // the last cell of the row wraps to x = 0
      const T s = sum6v<T, KIND>(rt, lt, dnt, upt, zpt, zmt);
      const T c = T(1) / T(6); // exact /6 as div6v, element-wise
      const T q0 = s * c;
      T q = __builtin_fmaf(__builtin_fmaf(-q0, T(6), s), c, q0);
      if (__builtin_expect(__builtin_fabsf(s) < 0x1p-100f, 0) && s != T(0)) q = s / T(6);
      ot = q;
    }
    if (KIND == 0 && rs.hit) {
#pragma unroll
      for (int h = 0; h < H; ++h)
#pragma unroll
        for (int k = 0; k < V; ++k) o[h][k] = fix(rs, xb + h * HS + k, o[h][k]);
      if constexpr (TL) ot = fix(rs, a.lox + HS * H + lane, ot);
    }
  };

  auto march = [&](auto downTag) {
    constexpr bool DOWN = decltype(downTag)::value;
    constexpr int dz = DOWN ? -1 : 1;
    const int z0 = DOWN ? ze - 1 : zs;
    NV C[NC][H];
    NV Ub[H], Uc[H], Ua[H];
    T Ct[NC] = {}, Ubt = 0, Uct = 0, Uat = 0; // tail cells (TL)
    // buffer loads: plane offset in an SGPR, row offset a per-segment VGPR. Recomputing a 64-bit VGPR address every
    // step wrote registers of the slot's previous load, and the compiler then waited for every outstanding memory
    // op (s_waitcnt vmcnt(0), the previous step's stores included) before issuing the step's loads
    auto load_row = [&](int zz, int k) {
      const uint32_t po = uint32_t(zcl(zz)) * uint32_t(a.pxy) * uint32_t(sizeof(T));
#pragma unroll
      for (int h = 0; h < H; ++h)
        C[k][h] = __builtin_bit_cast(NV, __builtin_amdgcn_raw_buffer_load_b128(srcRsrc, rowoff + uint32_t(choff(h)), po, 0));
      if constexpr (TL)
        Ct[k] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(srcRsrc, rowoff + uint32_t(toff), po, 0));
    };
    {
      const int zw = z0 - 2 * dz;
#pragma unroll
      for (int k = 0; k < NC - 1; ++k) load_row(zw + k * dz, k);
#pragma unroll
      for (int h = 0; h < H; ++h) cs[0][w][h][lane] = C[1][h];
      if constexpr (TL) cst[0][w][lane] = Ct[1];
      __syncthreads();
    }
    int buf = 0;
    int t = -2;
    auto step = [&](auto phase) -> bool {
      constexpr int k = decltype(phase)::value;
      constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
      if (t >= nzs) return false;
      const int z = z0 + t * dz;
      const int P = z + dz;
      load_row(z + (NC - 1) * dz, sn);
      if (needU1) {
        NV cA[H], cB[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          cA[h] = cs[buf][wA][h][lane];
          cB[h] = cs[buf][wB][h][lane];
        }
        const T cAt = TL ? cst[buf][wA][TL ? lane : 0] : T(0), cBt = TL ? cst[buf][wB][TL ? lane : 0] : T(0);
        apply_row(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], row_sph(P), Ua, Ct[s1], cAt, cBt,
                  DOWN ? Ct[s0] : Ct[s2], DOWN ? Ct[s2] : Ct[s0], Uat);
        if (a.early) { // block-uniform: publish into the other buffer now (its readers finished last step)
#pragma unroll
          for (int h = 0; h < H; ++h) {
            cs[buf ^ 1][w][h][lane] = C[s2][h];
            us[buf ^ 1][w][h][lane] = Ua[h];
          }
          if constexpr (TL) {
            cst[buf ^ 1][w][lane] = Ct[s2];
            ust[buf ^ 1][w][lane] = Uat;
          }
        }
      } else {
#pragma unroll
        for (int h = 0; h < H; ++h) Ua[h] = C[s1][h]; // never read: the edge waves' u1 feeds no output row
        Uat = Ct[s1];
      }
      if (t >= 0 && needU2) {
        NV uA[H], uB[H], o[H];
        T ot = 0;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          uA[h] = us[buf][wA][h][lane];
          uB[h] = us[buf][wB][h][lane];
        }
        const T uAt = TL ? ust[buf][wA][TL ? lane : 0] : T(0), uBt = TL ? ust[buf][wB][TL ? lane : 0] : T(0);
        apply_row(Uc, uA, uB, DOWN ? Ub : Ua, DOWN ? Ua : Ub, row_sph(z), o, Uct, uAt, uBt, DOWN ? Ubt : Uat,
                  DOWN ? Uat : Ubt, ot);
        if constexpr (TL)
          if (outRow && tailIn)
            *reinterpret_cast<T *>(reinterpret_cast<char *>(a.dst + int64_t(z) * a.pxy) + outoff + toff) = ot;
        if (outRow) {
          char *dp = reinterpret_cast<char *>(a.dst + int64_t(z) * a.pxy) + outoff;
#pragma unroll
          for (int h = 0; h < H; ++h) {
            NV *q = reinterpret_cast<NV *>(dp + h * HS * int(sizeof(T)));
            if (RAG && h == H - 1 && !(lane < Lr || (lane == Lr && kr == V - 1))) {
              if (lane == Lr) { // the partial chunk: cells x .. nx-1
                T *qs = reinterpret_cast<T *>(q);
#pragma unroll
                for (int k = 0; k < V - 1; ++k)
                  if (k <= kr) qs[k] = o[h][k];
              }
            } else if (a.nt) {
              __builtin_nontemporal_store(o[h], q);
            } else {
              *q = o[h];
            }
          }
        }
      }
      const int nbuf = buf ^ 1;
      if (!(a.early && needU1)) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
          cs[nbuf][w][h][lane] = C[s2][h];
          if (needU1) us[nbuf][w][h][lane] = Ua[h]; // the edge waves' u1 is never read
        }
        if constexpr (TL) {
          cst[nbuf][w][lane] = Ct[s2];
          if (needU1) ust[nbuf][w][lane] = Uat;
        }
      }
      // boundary-plane publication (block-uniform): every wave's stores of plane z complete before the barrier,
      // then one thread writes the XCD's L2 back (system-scope release) and counts the block's cells of the plane
      // boundary-plane publication (pipelined pairs): a template parameter, no live state otherwise (SGPR spills)
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
        Ub[h] = Uc[h];
        Uc[h] = Ua[h];
      }
      Ubt = Uct;
      Uct = Uat;
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
  } // passes
}

// Two-chunk columns (512 fp32 / 256 fp64 cells): the whole-row layout of stencil7x2_row_kernel (two 16-B chunks per
// lane, 64 chunks apart, x-neighbours by lane rotates) for rows longer than one wave: a column of CW cells per wave,
// and only the two cells beyond each column end come from outside the wave - a pair left of the column (lane 0 of
// chunk 0) and a pair right of it (lane 63 of chunk 1). Those pairs have one address per wave (a broadcast load each,
// shifted by the period at the wrapped row ends), and the neighbour rows' pairs come through LDS, as the edge scalars
// of stencil7x2_kernel. Taken for x extents that are whole multiples of CW cells (the 1024-wide sub-domains of the
// 8-GPU weak-scaling ladder; fp64 1024-cell rows as 4 columns): per row and plane the edge work and the fixed per-step
// cost of the one-chunk column kernel are paid once per two chunks per lane. Summation order, exact /6 and spheres
// as everywhere: bitwise equal to two single steps.
template <typename T, int NW, int PF, int KIND, int WRAP>
__global__ __launch_bounds__(64 * NW, 3) __attribute__((amdgpu_waves_per_eu(3, 3))) void stencil7x2_col2_kernel(
    StencilArgs<T> a, ZPartBounds zbounds) {
  using NV = typename Vec16<T>::native;
  using P2 = typename Pk<T>::t;
  constexpr int V = int(16 / sizeof(T)), H = 2; // chunks per lane
  constexpr int HS = 64 * V;    // cells between a lane's chunks
  constexpr int CW = H * HS;    // cells per column
  constexpr int YO = NW - 4;
  constexpr int NC = 3 + PF;
  static_assert(NW == 12, "3 waves per SIMD: the 168-VGPR budget");
  __shared__ NV cs[2][NW][H][64]; // src rows (plane z+2dz at publish)
  __shared__ NV us[2][NW][H][64]; // u1 rows (plane z+dz at publish)
  __shared__ T ce[2][NW][2];      // src at x-1 and x+CW of the published rows

  const uint32_t nb = gridDim.x;
  const uint32_t lb = a.remap ? xcd_remap(blockIdx.x, nb) : blockIdx.x;
  const int lane = threadIdx.x;
  const int w = int(threadIdx.y);
  const uint32_t nzt = uint32_t(a.hiz - a.loz);
  // lockstep parts as the whole-row kernel (y-adjacent columns of one 512-cell column strip are consecutive unless
  // xfast): 1024x512x256, 128 columns, marches 2 parts on 256 blocks
  // (no pointer select on the kernel argument: that made the compiler copy it to scratch, 1.5 KB per lane)
  const X2Segs sg = x2_segments(a, lb, nb, uint32_t(a.gx) * uint32_t(a.gy), nzt, &zbounds, a.gx == 1);
  uint32_t s = 0, e = 0;
  bool odd = sg.odd;
  for (int pass = 0; x2_pass(a, sg, pass, lb, nb, uint32_t(a.gx) * uint32_t(a.gy), nzt, s, e); ++pass) {
  while (s < e) { // block-uniform
  const uint32_t col = s / nzt;
  const int zo = int(s - col * nzt);
  const int nzs = int(min(nzt - uint32_t(zo), e - s));
  s += uint32_t(nzs);
  int bx, by;
  if (a.xfast) {
    by = int(col / uint32_t(a.gx));
    bx = int(col - uint32_t(by) * uint32_t(a.gx));
  } else {
    bx = int(col / uint32_t(a.gy));
    by = int(col - uint32_t(bx) * uint32_t(a.gy));
  }
  const int zs = a.loz + zo;
  const int ze = zs + nzs;
  const bool down = odd != (a.flip != 0);
  odd = !odd;
  const int xcol = a.x0 + bx * CW;  // first cell of the column
  const int xb = xcol + lane * V;   // chunk h at xb + h * HS
  const int yblk = a.loy + YO * by;
  const int y = yblk - 2 + w;
  if (yblk >= a.hiy) continue;
  const bool outRow = w >= 2 && w < NW - 2 && y < a.hiy;
  const bool needU1 = w >= 1 && w < NW - 1, needU2 = w >= 2 && w < NW - 2; // edge waves: source rows only
  const int wA = w > 0 ? w - 1 : 0, wB = w < NW - 1 ? w + 1 : NW - 1;
  const bool lane0 = lane == 0, lane63 = lane == 63;

  const int yw =
      (WRAP >= 1 && (a.wrapm & 2)) ? (y < a.wlo[1] ? y + a.wn[1] : (y >= a.wlo[1] + a.wn[1] ? y - a.wn[1] : y)) : y;
  const int yc = yw < 0 ? 0 : (yw > a.rawYm1 ? a.rawYm1 : yw);
  const uint32_t rowoff = uint32_t((yc * int64_t(a.px) + xb) * int64_t(sizeof(T)));
  const uint32_t outoff = uint32_t((y * int64_t(a.px) + xb) * int64_t(sizeof(T)));
  // the edge pairs (x-2, x-1 left of the column; x+CW, x+CW+1 right of it): one address per wave; x wrap moves the
  // left pair of the first column and the right pair of the last one by the period
  int xl = xcol - 2, xr = xcol + CW;
  if (WRAP == 2 && (a.wrapm & 1)) {
    if (xcol == a.wlo[0]) xl += a.wn[0];
    if (xcol + CW == a.wlo[0] + a.wn[0]) xr -= a.wn[0];
  }
  const uint32_t loff = uint32_t((yc * int64_t(a.px) + xl) * int64_t(sizeof(T)));
  const uint32_t roff = uint32_t((yc * int64_t(a.px) + xr) * int64_t(sizeof(T)));
  const int zwn = (WRAP >= 1 && (a.wrapm & 4)) ? a.wn[2] : 0, zwlo = a.wlo[2], zwhi = a.wlo[2] + zwn;
  auto zcl = [&](int zz) {
    if constexpr (WRAP >= 1) {
      zz += zz < zwlo ? zwn : 0;
      zz -= zz >= zwhi ? zwn : 0;
    }
    return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz);
  };
  auto planep = [&](int zz) -> const char * { return reinterpret_cast<const char *>(a.src + int64_t(zcl(zz)) * a.pxy); };
  // hot iff (x - hx)^2 < Dh = sqh - (P - hz)^2 with sqh = r1sq - (y - hy)^2, cold likewise (two live scalars per row:
  // SGPR pressure, see stencil7x2_row_kernel)
  const int sqh = a.r1sq - (y - a.hy) * (y - a.hy), sqc = a.r1sq - (y - a.cy) * (y - a.cy);
  struct RowSph {
    int Dh, Dc;
    bool hit;
  };
  auto row_sph = [&](int P) -> RowSph {
    RowSph r{0, 0, false};
    if (KIND == 0) {
      r.Dh = sqh - (P - a.hz) * (P - a.hz);
      r.Dc = sqc - (P - a.cz) * (P - a.cz);
      r.hit = max(r.Dh, r.Dc) > 0;
    }
    return r;
  };
  auto fix = [&](const RowSph &rs, int x, T v) -> T {
    const bool hot = (x - a.hx) * (x - a.hx) < rs.Dh;
    const bool cold = (x - a.cx) * (x - a.cx) < rs.Dc;
    return hot ? T(1) : (cold ? T(0) : v);
  };
  // S of the wave's column: x-neighbours by lane rotates, eL / eR beyond the column ends
  auto apply_row = [&](const NV (&cm)[H], const NV (&up)[H], const NV (&dn)[H], const NV (&zp)[H], const NV (&zm)[H],
                       T eL, T eR, const RowSph &rs, NV (&o)[H]) {
    T r3[H], l0[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      r3[h] = rot_prev(cm[h][V - 1]);
      l0[h] = rot_next(cm[h][0]);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const T left = lane0 ? (h == 0 ? eL : r3[h - 1]) : r3[h];
      const T right = lane63 ? (h == H - 1 ? eR : l0[h + 1]) : l0[h];
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
        for (int k = 0; k < V; ++k) o[h][k] = fix(rs, xb + h * HS + k, o[h][k]);
    }
  };

  auto march = [&](auto downTag) {
    constexpr bool DOWN = decltype(downTag)::value;
    constexpr int dz = DOWN ? -1 : 1;
    const int z0 = DOWN ? ze - 1 : zs;
    NV C[NC][H];
    P2 EL[NC], ER[NC]; // (x-2, x-1) and (x+CW, x+CW+1) of the column, per window plane
    NV Ub[H], Uc[H], Ua[H];
    P2 UcE, UaE; // u1 at (x-1, x+CW), planes z and z+dz
    auto load_row = [&](int zz, int k) {
      const char *b = planep(zz);
#pragma unroll
      for (int h = 0; h < H; ++h) C[k][h] = *reinterpret_cast<const NV *>(b + rowoff + h * HS * int(sizeof(T)));
      EL[k] = *reinterpret_cast<const P2 *>(b + loff);
      ER[k] = *reinterpret_cast<const P2 *>(b + roff);
    };
    auto publish_src = [&](int bufi, int k) {
#pragma unroll
      for (int h = 0; h < H; ++h) cs[bufi][w][h][lane] = C[k][h];
      if (lane0) {
        ce[bufi][w][0] = EL[k][1];
        ce[bufi][w][1] = ER[k][0];
      }
    };
    {
      const int zw = z0 - 2 * dz;
#pragma unroll
      for (int k = 0; k < NC - 1; ++k) load_row(zw + k * dz, k);
      publish_src(0, 1);
      __syncthreads();
    }
    int buf = 0;
    int t = -2;
    auto step = [&](auto phase) -> bool {
      constexpr int k = decltype(phase)::value;
      constexpr int s0 = k % NC, s1 = (k + 1) % NC, s2 = (k + 2) % NC, sn = (k + NC - 1) % NC;
      if (t >= nzs) return false;
      const int z = z0 + t * dz;
      const int P = z + dz;
      load_row(z + (NC - 1) * dz, sn);
      if (!needU1) {
#pragma unroll
        for (int h = 0; h < H; ++h) Ua[h] = C[s1][h]; // never read
        UaE = P2{T(0), T(0)};
      } else {
        NV cA[H], cB[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          cA[h] = cs[buf][wA][h][lane];
          cB[h] = cs[buf][wB][h][lane];
        }
        const T cAL = ce[buf][wA][0], cAR = ce[buf][wA][1]; // LDS broadcasts
        const T cBL = ce[buf][wB][0], cBR = ce[buf][wB][1];
        const RowSph rs = row_sph(P);
        apply_row(C[s1], cA, cB, DOWN ? C[s0] : C[s2], DOWN ? C[s2] : C[s0], EL[s1][1], ER[s1][0], rs, Ua);
        // u1 just outside the column: (x-1) on lane 0, (x+CW) on lane 63
        const P2 epx = {C[s1][0][0], ER[s1][1]}, emx = {EL[s1][0], C[s1][H - 1][V - 1]}, epy = {cBL, cBR},
                 emy = {cAL, cAR};
        const P2 ezp = DOWN ? P2{EL[s0][1], ER[s0][0]} : P2{EL[s2][1], ER[s2][0]};
        const P2 ezm = DOWN ? P2{EL[s2][1], ER[s2][0]} : P2{EL[s0][1], ER[s0][0]};
        UaE = div6v<T, P2, 2>(sum6v<T, KIND>(epx, emx, epy, emy, ezp, ezm));
        if (KIND == 0 && rs.hit) {
          UaE[0] = fix(rs, xcol - 1, UaE[0]);
          UaE[1] = fix(rs, xcol + CW, UaE[1]);
        }
        if (a.early) { // block-uniform: publish into the other buffer now (its readers finished last step)
          publish_src(buf ^ 1, s2);
#pragma unroll
          for (int h = 0; h < H; ++h) us[buf ^ 1][w][h][lane] = Ua[h];
        }
      }
      if (t >= 0 && needU2) {
        NV uA[H], uB[H], o[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          uA[h] = us[buf][wA][h][lane];
          uB[h] = us[buf][wB][h][lane];
        }
        apply_row(Uc, uA, uB, DOWN ? Ub : Ua, DOWN ? Ua : Ub, UcE[0], UcE[1], row_sph(z), o);
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
      if (!(a.early && needU1)) {
        publish_src(nbuf, s2);
#pragma unroll
        for (int h = 0; h < H; ++h)
          if (needU1) us[nbuf][w][h][lane] = Ua[h]; // the edge waves' u1 is never read
      }
      __syncthreads();
      buf = nbuf;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        Ub[h] = Uc[h];
        Uc[h] = Ua[h];
      }
      UcE = UaE;
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
  } // passes
}

// S o S on a few small boxes (the exterior slabs of an overlapped step: interior sweep during the exchange, these
// after it). One thread per output cell: u2 = S of the six u1 neighbours, each u1 = S of its six src neighbours,
// in the single step's summation order with the exact /6 and the spheres, i.e. the same bits as the sweep kernel
// (whose u1 of a halo cell equals the neighbour's own u1 there, as two single steps with an exchange between).
constexpr int kMaxX2Regions = 8;
struct X2Regions {
  int lo[kMaxX2Regions][3];
  int ext[kMaxX2Regions][3];
  int64_t begin[kMaxX2Regions + 1];
  int n;
};

template <typename T, int KIND>
__global__ __launch_bounds__(256) void stencil7x2_regions_kernel(StencilArgs<T> a, X2Regions rt) {
  const int64_t total = rt.begin[rt.n];
  const int64_t px = a.px, pxy = a.pxy;
  auto ld = [&](int x, int y, int z) -> T {
    return a.src[int64_t(wrap_coord(a, z, 2)) * pxy + int64_t(wrap_coord(a, y, 1)) * px + wrap_coord(a, x, 0)];
  };
  auto u1 = [&](int x, int y, int z) -> T {
    T v;
    if (a.wrapm == 0) {
      const T *p = a.src + int64_t(z) * pxy + int64_t(y) * px + x;
      v = sum6<T, KIND>(p[1], p[-1], p[px], p[-px], p[pxy], p[-pxy]); // sum6 includes the exact /6
    } else {
      v = sum6<T, KIND>(ld(x + 1, y, z), ld(x - 1, y, z), ld(x, y + 1, z), ld(x, y - 1, z), ld(x, y, z + 1),
                        ld(x, y, z - 1));
    }
    return KIND == 0 ? sphere_fix(a, x, y, z, v) : v;
  };
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    int k = 0;
    while (k + 1 < rt.n && rt.begin[k + 1] <= i) ++k;
    const int64_t li = i - rt.begin[k];
    const int nx = rt.ext[k][0], ny = rt.ext[k][1];
    const int x = rt.lo[k][0] + int(li % nx);
    const int y = rt.lo[k][1] + int((li / nx) % ny);
    const int z = rt.lo[k][2] + int(li / (int64_t(nx) * ny));
    const T vpx = u1(x + 1, y, z), vmx = u1(x - 1, y, z), vpy = u1(x, y + 1, z), vmy = u1(x, y - 1, z);
    const T vpz = u1(x, y, z + 1), vmz = u1(x, y, z - 1);
    T v = sum6<T, KIND>(vpx, vmx, vpy, vmy, vpz, vmz);
    if (KIND == 0) v = sphere_fix(a, x, y, z, v);
    a.dst[int64_t(z) * pxy + int64_t(y) * px + x] = v;
  }
}

// S o S on thin slabs (the exterior of an overlapped fused pair: thickness <= NT along axis THIN). A z march over a
// 2-cell slab has too little parallelism and a chunk-per-lane sweep leaves most lanes idle on x slabs, so each wave
// takes a short tile: lanes along axis LANE (60 outputs + a 2-lane halo each side, neighbours by DPP), the slab's
// thin extent plus 2 cells each side in registers, and BC planes (+2 each side) along axis MARCH, all loaded up
// front (one memory round trip per wave). u1 on the tile interior, then u2 on the slab; sums in the reference
// order +x,-x,+y,-y,+z,-z whatever the roles of the axes, exact /6 and spheres as the sweep: the same bits.
constexpr int kThinBC = 4;
struct ThinTable {
  int lo[2][3], hi[2][3]; // raw boxes (up to two slabs of one orientation)
  int wbegin[3];
  int n;
};

template <int THIN, int LANE, int MARCH, int AX, int SGN, typename T, int N0, int N1>
__device__ __forceinline__ T thin_nbr(const T (&v)[N0][N1], int ti, int bi) {
  if constexpr (AX == THIN)
    return v[ti + SGN][bi];
  else if constexpr (AX == MARCH)
    return v[ti][bi + SGN];
  else
    return SGN > 0 ? from_next_lane<T>(v[ti][bi]) : from_prev_lane<T>(v[ti][bi]);
}

template <typename T, int KIND, int THIN, int LANE, int MARCH, int NT>
__global__ __launch_bounds__(256) void stencil7x2_thin_kernel(StencilArgs<T> a, ThinTable tb) {
  constexpr int NTV = NT + 4, NB = kThinBC + 4; // src window: thin cells t0-2 .. t0+NT+1, planes b0-2 .. b0+BC+1
  const int wave = int(blockIdx.x) * 4 + int(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= tb.wbegin[tb.n]) return; // wave-uniform
  const int k = (tb.n > 1 && wave >= tb.wbegin[1]) ? 1 : 0;
  const int lw = wave - tb.wbegin[k];
  const int ng = (tb.hi[k][LANE] - tb.lo[k][LANE] + 59) / 60;
  const int g = lw % ng, bb = lw / ng;
  const int t0 = tb.lo[k][THIN], nt = tb.hi[k][THIN] - t0;
  const int b0 = tb.lo[k][MARCH] + bb * kThinBC;
  const int cl = tb.lo[k][LANE] - 2 + 60 * g + lane;
  const int64_t st[3] = {1, a.px, a.pxy};
  const int rawm1[3] = {int(a.px) - 1, a.rawYm1, a.rawZm1};
  auto clampc = [&](int c, int ax) {
    c = wrap_coord(a, c, ax); // wrapped axes: the periodic image (never the THIN axis of an x slab, see the host)
    return c < 0 ? 0 : (c > rawm1[ax] ? rawm1[ax] : c);
  };
  const T *lp = a.src + int64_t(clampc(cl, LANE)) * st[LANE];
  T v[NTV][NB];
  if constexpr (THIN == 0) {
    // x slabs: each lane's thin window is contiguous in its row. Load it as aligned 16-B vectors (one cache line
    // per row and plane instead of one per value: the lanes sit on 64 different rows) and pick the window out with
    // a wave-uniform offset
    using NV = typename Vec16<T>::native;
    constexpr int V = Vec16<T>::N;
    const int xw = t0 - 2;                                      // first x of the window (raw)
    const int xa = xw - (((xw - a.x0) % V) + V) % V;            // a.x0: a 16-B aligned raw x
    const int off = xw - xa;                                    // 0 .. V-1, wave-uniform
    auto fill = [&](auto offTag) {
      constexpr int O = decltype(offTag)::value;
      constexpr int NL = (NTV + O + V - 1) / V; // vectors covering the window (never past it by a whole vector)
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) {
        const T *pp = lp + int64_t(clampc(b0 - 2 + bi, MARCH)) * st[MARCH] + xa;
        NV w[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) w[j] = *reinterpret_cast<const NV *>(pp + j * V);
#pragma unroll
        for (int ti = 0; ti < NTV; ++ti) v[ti][bi] = w[(ti + O) / V][(ti + O) % V];
      }
    };
    if constexpr (V == 4) {
      switch (off) {
      case 0: fill(std::integral_constant<int, 0>{}); break;
      case 1: fill(std::integral_constant<int, 1>{}); break;
      case 2: fill(std::integral_constant<int, 2>{}); break;
      default: fill(std::integral_constant<int, 3>{}); break;
      }
    } else {
      if (off == 0)
        fill(std::integral_constant<int, 0>{});
      else
        fill(std::integral_constant<int, 1>{});
    }
  } else {
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
      const T *pp = lp + int64_t(clampc(b0 - 2 + bi, MARCH)) * st[MARCH];
#pragma unroll
      for (int ti = 0; ti < NTV; ++ti) v[ti][bi] = pp[int64_t(clampc(t0 - 2 + ti, THIN)) * st[THIN]];
    }
  }
  auto coord = [&](int ax, int ti, int bi) { return ax == THIN ? t0 - 2 + ti : (ax == MARCH ? b0 - 2 + bi : cl); };
  // u1 on thin cells t0-1 .. t0+NT, planes b0-1 .. b0+BC (array index = src index - 1)
  T u[NTV - 2][NB - 2];
#pragma unroll
  for (int ti = 1; ti < NTV - 1; ++ti)
#pragma unroll
    for (int bi = 1; bi < NB - 1; ++bi) {
      T r = sum6<T, KIND>(thin_nbr<THIN, LANE, MARCH, 0, 1>(v, ti, bi), thin_nbr<THIN, LANE, MARCH, 0, -1>(v, ti, bi),
                          thin_nbr<THIN, LANE, MARCH, 1, 1>(v, ti, bi), thin_nbr<THIN, LANE, MARCH, 1, -1>(v, ti, bi),
                          thin_nbr<THIN, LANE, MARCH, 2, 1>(v, ti, bi), thin_nbr<THIN, LANE, MARCH, 2, -1>(v, ti, bi));
      if (KIND == 0) r = sphere_fix(a, coord(0, ti, bi), coord(1, ti, bi), coord(2, ti, bi), r);
      u[ti - 1][bi - 1] = r;
    }
  const bool outLane = lane >= 2 && lane < 62 && cl < tb.hi[k][LANE];
#pragma unroll
  for (int ti = 2; ti < NT + 2; ++ti)
#pragma unroll
    for (int bi = 2; bi < NB - 2; ++bi) {
      const int ui = ti - 1, uj = bi - 1;
      T r = sum6<T, KIND>(thin_nbr<THIN, LANE, MARCH, 0, 1>(u, ui, uj), thin_nbr<THIN, LANE, MARCH, 0, -1>(u, ui, uj),
                          thin_nbr<THIN, LANE, MARCH, 1, 1>(u, ui, uj), thin_nbr<THIN, LANE, MARCH, 1, -1>(u, ui, uj),
                          thin_nbr<THIN, LANE, MARCH, 2, 1>(u, ui, uj), thin_nbr<THIN, LANE, MARCH, 2, -1>(u, ui, uj));
      const int x = coord(0, ti, bi), y = coord(1, ti, bi), z = coord(2, ti, bi);
      if (KIND == 0) r = sphere_fix(a, x, y, z, r);
      if (outLane && ti - 2 < nt && b0 - 2 + bi < tb.hi[k][MARCH])
        a.dst[int64_t(z) * a.pxy + int64_t(y) * a.px + x] = r;
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
  return aligned && lox - 2 + dom.front_slack(qi) >= 0 && lox + nchunks * V + 1 < dom.row_limit(qi);
}

int stencil7x2_wrappable_axes(const LocalDomain &dom, int64_t qi, int x2row) {
  if (!stencil7x2_supported(dom, qi)) return 0;
  const int64_t es = dom.elem_size(qi), V = 16 / es;
  const int64_t lox = dom.radius().x(-1), nx = dom.size().x, lim = dom.row_limit(qi), slack = dom.front_slack(qi);
  // ragged fp32 rows of 257-832 cells: the whole-row kernel wraps x by broadcasting the row-end cells (a ragged last
  // chunk reads at most 3 cells past the row end, inside the padded row; rows of 769-832 end in per-lane tail cells)
  const bool rowX = x2row != 0 && es == 4 && nx > 256 && nx <= 832 && lox + (nx + V - 1) / V * V < lim;
  if (rowX && nx % V != 0) return 1 | (dom.size().y >= 2 ? 2 : 0) | (dom.size().z >= 2 ? 4 : 0);
  // x: whole chunks only (the chunk grid starts at the 16-B aligned lox), at least two, and the last chunk not on
  // lane 0 of its column (a wrap lane shifts both of its edge pairs: its other edge must be the unused one, never a
  // column boundary); the unused edge pair of a wrap lane (x-2 .. x+V+1 shifted by +-nx) must stay in the row
  const bool x = nx % V == 0 && nx >= 2 * V && (nx / V) % 64 != 1 && lox - V - 2 + slack >= 0 &&
                 lox + nx + V + 1 < lim;
  // y / z: one conditional shift maps the 2 cells beyond a face onto the grid
  return (x ? 1 : 0) | (dom.size().y >= 2 ? 2 : 0) | (dom.size().z >= 2 ? 4 : 0);
}

// along wrapped axes the region must be the whole compute region (the kernels wrap at its faces)
static void check_wrap(const LocalDomain &dom, int64_t qi, const Rect3 &region, int wrap, int x2row) {
  if (wrap == 0) return;
  STENCIL_REQUIRE((wrap & ~stencil7x2_wrappable_axes(dom, qi, x2row)) == 0,
                  "in-kernel wrap " << wrap << " not supported by this layout ("
                                    << stencil7x2_wrappable_axes(dom, qi, x2row) << ")");
  const Rect3 cr = dom.get_compute_region();
  const int64_t lo[3] = {region.lo.x, region.lo.y, region.lo.z}, hi[3] = {region.hi.x, region.hi.y, region.hi.z};
  const int64_t clo[3] = {cr.lo.x, cr.lo.y, cr.lo.z}, chi[3] = {cr.hi.x, cr.hi.y, cr.hi.z};
  for (int ax = 0; ax < 3; ++ax)
    STENCIL_REQUIRE(!((wrap >> ax) & 1) || (lo[ax] == clo[ax] && hi[ax] == chi[ax]),
                    "region " << region << " does not span wrapped axis " << ax << " of " << cr);
}

template <typename T, int KIND, int NW, int PF>
static void apply_x2_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                       const StencilTune &tune) {
  constexpr int V = Vec16<T>::N, YO = NW - 4;
  StencilArgs<T> a = make_args<T>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  a.nt = tune.nontemporal ? 1 : 0;
  a.wrapm = tune.wrap;
  a.xfast = tune.x2xfast;
  const int rxm = int(dom.radius().x(-1));
  const int off = ((a.lox - rxm) % V + V) % V;
  a.x0 = a.lox - off;
  a.nchunks = (a.hix - a.x0 + V - 1) / V;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = (a.nchunks + 63) / 64;
  a.gy = (ny + YO - 1) / YO;
  a.remap = tune.xcdRemap ? 1 : 0;
  const void *kern = (const void *)stencil7x2_kernel<T, NW, PF, KIND, 0>;
  const int64_t cols = int64_t(a.gx) * a.gy;
  const int64_t resident = x2_resident_blocks(kern, 64 * NW);
  uint32_t blocks;
  if (tune.x2sched != 0 && tune.zchunk <= 0) {
    // one block per resident slot, but pieces of at least 16 planes (each piece re-reads 4 warm-up planes)
    a.seg = 1;
    a.zc = 1;
    a.gz = 1;
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dom.gpu()) != hipSuccess) cus = 256;
    const int64_t perCU = std::max<int64_t>(1, resident / std::max(1, cus));
    const int64_t slots = std::max<int64_t>(perCU, resident - perCU * std::min(tune.reserveCUs, cus / 2));
    blocks = uint32_t(std::max<int64_t>(1, std::min<int64_t>(slots, cols * nz / 16)));
  } else {
    int zc = tune.zchunk;
    if (zc <= 0) // each z-chunk re-reads 4 warm-up planes (2 src + 2 for u1)
      zc = pick_zchunk(cols, nz, resident, 4, 16);
    a.zc = zc;
    a.gz = (nz + zc - 1) / zc;
    blocks = uint32_t(cols * a.gz);
  }
  dom.set_device();
  if (a.wrapm & 1)
    hipLaunchKernelGGL((stencil7x2_kernel<T, NW, PF, KIND, 2>), dim3(blocks), dim3(64, NW), 0, stream, a);
  else if (a.wrapm)
    hipLaunchKernelGGL((stencil7x2_kernel<T, NW, PF, KIND, 1>), dim3(blocks), dim3(64, NW), 0, stream, a);
  else
    hipLaunchKernelGGL((stencil7x2_kernel<T, NW, PF, KIND, 0>), dim3(blocks), dim3(64, NW), 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

// whole-row kernel: fp32, x wrapped in-kernel, rows starting on a 16-B chunk; H chunks per lane (RAG: rows shorter
// than 256 H cells)
template <int KIND, int PF, int H = 2, bool RAG = false, int NW = 12, bool TL = false>
static bool apply_x2row_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                          const StencilTune &tune) {
  constexpr int YO = NW - 4;
  StencilArgs<float> a = make_args<float>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  const int rxm = int(dom.radius().x(-1));
  const int nx = a.hix - a.lox;
  const bool fitsH = TL ? (nx > 256 * H && nx <= 256 * H + 64) : (RAG ? (nx > 256 * (H - 1) && nx <= 256 * H) : nx == 512);
  if (!(tune.wrap & 1) || !fitsH || (a.lox - rxm) % 4 != 0) return false;
  if (dom.buffer_bytes(qi) >= (int64_t(1) << 32) - 4096) return false; // 32-bit buffer-load offsets
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  a.nt = tune.nontemporal ? 1 : 0;
  a.wrapm = tune.wrap;
  a.early = tune.x2early ? 1 : 0;
  a.x0 = a.lox;
  a.nchunks = 128;
  a.remap = tune.xcdRemap ? 1 : 0;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  if (tune.publish) {
    a.pub = reinterpret_cast<unsigned long long *>(tune.publish);
    a.pubLo = a.loz + tune.publishDepth;
    a.pubHi = a.hiz - tune.publishDepth;
  }
  a.gx = 1;
  a.gy = (ny + YO - 1) / YO;
  const void *kern = (const void *)stencil7x2_row_kernel<NW, PF, KIND, H, RAG, TL>;
  const int64_t cols = a.gy;
  const int64_t resident = x2_resident_blocks(kern, 64 * NW);
  uint32_t blocks;
  if (tune.x2sched != 0 && tune.zchunk <= 0) {
    a.seg = 1;
    a.zc = 1;
    a.gz = 1;
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dom.gpu()) != hipSuccess) cus = 256;
    const int64_t perCU = std::max<int64_t>(1, resident / std::max(1, cus));
    const int64_t slots = std::max<int64_t>(perCU, resident - perCU * std::min(tune.reserveCUs, cus / 2));
    blocks = uint32_t(std::max<int64_t>(1, std::min<int64_t>(slots, cols * nz / 16)));
    // lockstep parts (a.seg = 2, x2_lockstep_schedule): with 8 CUs left to the transports (248 blocks) the balanced
    // split puts y-adjacent blocks 16 planes apart and their halo rows miss L2 (512^3 local interior: 276 vs 237 us
    // at 256 blocks); 813x407x407 (51 row groups) runs 5 parts on 255 blocks
    const X2Schedule ls = x2_lockstep_schedule(slots, cols, nz);
    if (tune.x2lockstep && ls.parts > 0) {
      a.seg = ls.rounds > 1 ? 3 : 2;
      a.zparts = ls.parts;
      a.zrounds = ls.rounds;
      blocks = uint32_t(ls.blocks);
    }
  } else {
    int zc = tune.zchunk;
    if (zc <= 0) zc = pick_zchunk(cols, nz, resident, 4, 16);
    a.zc = zc;
    a.gz = (nz + zc - 1) / zc;
    blocks = uint32_t(cols * a.gz);
  }
  dom.set_device();
  ZPartBounds zb{};
  zb.on = 0;
  if (KIND == 0 && a.seg == 2) sphere_part_bounds(zb, a, int64_t(blocks) / a.zparts, a.zparts, NW, YO, 2, tune.x2sphw);
  if (a.pub)
    hipLaunchKernelGGL((stencil7x2_row_kernel<NW, PF, KIND, H, RAG, TL, true>), dim3(blocks), dim3(64, NW), 0, stream, a,
                       zb);
  else
    hipLaunchKernelGGL((stencil7x2_row_kernel<NW, PF, KIND, H, RAG, TL>), dim3(blocks), dim3(64, NW), 0, stream, a, zb);
  HIP_CHECK(hipGetLastError());
  return true;
}

// two-chunk column kernel: the region's x extent a whole number of CW-cell columns (512 fp32, 256 fp64) starting on
// a 16-B chunk
template <typename T, int KIND, int PF, int WRAP>
static void apply_x2col2_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph,
                           hipStream_t stream, const StencilTune &tune) {
  constexpr int NW = 12, YO = NW - 4, V = int(16 / sizeof(T)), CW = 128 * V;
  StencilArgs<T> a = make_args<T>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  a.nt = tune.nontemporal ? 1 : 0;
  a.wrapm = tune.wrap;
  a.xfast = tune.x2xfast;
  a.remap = tune.xcdRemap ? 1 : 0;
  a.early = tune.x2early ? 1 : 0;
  a.x0 = a.lox; // 16-B aligned (checked by the caller)
  a.nchunks = (a.hix - a.x0) / V;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = (a.hix - a.x0) / CW;
  a.gy = (ny + YO - 1) / YO;
  const void *kern = (const void *)stencil7x2_col2_kernel<T, NW, PF, KIND, WRAP>;
  const int64_t cols = int64_t(a.gx) * a.gy;
  const int64_t resident = x2_resident_blocks(kern, 64 * NW);
  uint32_t blocks;
  if (tune.x2sched != 0 && tune.zchunk <= 0) {
    a.seg = 1;
    a.zc = 1;
    a.gz = 1;
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dom.gpu()) != hipSuccess) cus = 256;
    const int64_t perCU = std::max<int64_t>(1, resident / std::max(1, cus));
    const int64_t slots = std::max<int64_t>(perCU, resident - perCU * std::min(tune.reserveCUs, cus / 2));
    blocks = uint32_t(std::max<int64_t>(1, std::min<int64_t>(slots, cols * nz / 16)));
    // lockstep parts (x2_lockstep_schedule) when y-adjacent columns are consecutive (column index y-major)
    const X2Schedule ls = x2_lockstep_schedule(slots, cols, nz);
    if (tune.x2lockstep && !tune.x2xfast && ls.parts > 0) {
      a.seg = ls.rounds > 1 ? 3 : 2;
      a.zparts = ls.parts;
      a.zrounds = ls.rounds;
      blocks = uint32_t(ls.blocks);
    }
  } else {
    int zc = tune.zchunk;
    if (zc <= 0) zc = pick_zchunk(cols, nz, resident, 4, 16);
    a.zc = zc;
    a.gz = (nz + zc - 1) / zc;
    blocks = uint32_t(cols * a.gz);
  }
  dom.set_device();
  ZPartBounds zb{};
  zb.on = 0;
  if (KIND == 0 && a.seg == 2 && a.gx == 1)
    sphere_part_bounds(zb, a, int64_t(blocks) / a.zparts, a.zparts, NW, YO, 2, tune.x2sphw);
  hipLaunchKernelGGL((stencil7x2_col2_kernel<T, NW, PF, KIND, WRAP>), dim3(blocks), dim3(64, NW), 0, stream, a, zb);
  HIP_CHECK(hipGetLastError());
}

template <typename T, int KIND, int PF>
static void apply_x2col2_wrap(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph,
                              hipStream_t stream, const StencilTune &tune) {
  if (tune.wrap & 1)
    apply_x2col2_t<T, KIND, PF, 2>(dom, qi, region, sph, stream, tune);
  else if (tune.wrap)
    apply_x2col2_t<T, KIND, PF, 1>(dom, qi, region, sph, stream, tune);
  else
    apply_x2col2_t<T, KIND, PF, 0>(dom, qi, region, sph, stream, tune);
}

bool stencil7x2_row_kernel_used(const LocalDomain &dom, int64_t qi, const Rect3 &region, const StencilTune &tune) {
  if (region.empty() || !stencil7x2_supported(dom, qi) || dom.elem_size(qi) != 4 || !tune.x2row || !(tune.wrap & 1))
    return false;
  const Rect3 rr(region.lo - dom.accessor_origin(), region.hi - dom.accessor_origin());
  const int64_t nx = rr.hi.x - rr.lo.x;
  return (nx == 512 || (nx > 256 && nx <= 832)) && (rr.lo.x - dom.radius().x(-1)) % 4 == 0 &&
         dom.buffer_bytes(qi) < (int64_t(1) << 32) - 4096;
}

void stencil7x2_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune) {
  if (region.empty()) return;
  STENCIL_REQUIRE(stencil7x2_supported(dom, qi),
                  "two-step stencil needs a device fp32/fp64 quantity, face radii >= 2 and the aligned layout");
  const Rect3 cr = dom.get_compute_region();
  STENCIL_REQUIRE(cr.contains(region.lo) && region.hi.x <= cr.hi.x && region.hi.y <= cr.hi.y && region.hi.z <= cr.hi.z,
                  "stencil region " << region << " outside compute region " << cr);
  check_wrap(dom, qi, region, tune.wrap, tune.x2row);
  const bool f32 = dom.elem_size(qi) == 4;
  const bool jac = kind == StencilKind::Jacobi;
  if (f32 && tune.x2row) { // whole rows of 512 cells in one wave (x wrapped in-kernel)
    // one plane of lookahead (1-3 measured within noise once the edge waves skip u1 / u2, r2s3; 2 / 3 removed in r6)
    bool done = jac ? apply_x2row_t<0, 1>(dom, qi, region, sph, stream, tune)
                    : apply_x2row_t<1, 1>(dom, qi, region, sph, stream, tune);
    if (done) return;
    const Rect3 rr(region.lo - dom.accessor_origin(), region.hi - dom.accessor_origin());
    const int64_t nx = rr.hi.x - rr.lo.x;
    // ragged periodic rows (x wrapped, 256 < nx <= 768 but not 512): H = 2 / 3 chunks per lane, first / last cell
    // broadcast for the wrap (one plane of lookahead: the 3-chunk window leaves no registers for more). Four chunks
    // per lane (rows of 769-1024) need 10-wave blocks for the LDS and spill at their 168-VGPR budget: 358 vs 668
    // Gcells/s for the column kernel at 813x407x407 (profiles/r2/r2_ragged_shapes.log); 8-wave blocks (2 waves per
    // SIMD, 200 VGPRs, 4 output rows of 8) 597 vs 668 (r2_ragged_h4_8waves.log). Not instantiated.
    if ((tune.wrap & 1) && nx > 256 && nx <= 768) {
      if (nx <= 512)
        done = jac ? apply_x2row_t<0, 1, 2, true>(dom, qi, region, sph, stream, tune)
                   : apply_x2row_t<1, 1, 2, true>(dom, qi, region, sph, stream, tune);
      else
        done = jac ? apply_x2row_t<0, 1, 3, true>(dom, qi, region, sph, stream, tune)
                   : apply_x2row_t<1, 1, 3, true>(dom, qi, region, sph, stream, tune);
      if (done) return;
    }
    // rows of 769-832 cells (the 4-GPU ladder's 813): three chunks per lane plus one tail cell per lane
    if ((tune.wrap & 1) && nx > 768 && nx <= 832) {
      done = jac ? apply_x2row_t<0, 1, 3, false, 12, true>(dom, qi, region, sph, stream, tune)
                 : apply_x2row_t<1, 1, 3, false, 12, true>(dom, qi, region, sph, stream, tune);
      if (done) return;
    }
    STENCIL_REQUIRE(!tune.publish, "boundary-plane publication needs the whole-row kernel");
    // x a whole number of 512-cell columns from a 16-B aligned first cell: the 512-cell column kernel
    if (nx % 512 == 0 && (rr.lo.x - dom.radius().x(-1)) % 4 == 0) {
      // one plane of lookahead (two would spill the Jacobi instance; the row kernel shows no difference)
      jac ? apply_x2col2_wrap<float, 0, 1>(dom, qi, region, sph, stream, tune)
          : apply_x2col2_wrap<float, 1, 1>(dom, qi, region, sph, stream, tune);
      return;
    }
  }
  if (!f32 && tune.x2row && !tune.publish) {
    // fp64: x a whole number of 256-cell columns (two 2-double chunks per lane) from a 16-B aligned first cell
    const Rect3 rr(region.lo - dom.accessor_origin(), region.hi - dom.accessor_origin());
    const int64_t nx = rr.hi.x - rr.lo.x;
    if (nx % 256 == 0 && (rr.lo.x - dom.radius().x(-1)) % 2 == 0) {
      jac ? apply_x2col2_wrap<double, 0, 1>(dom, qi, region, sph, stream, tune)
          : apply_x2col2_wrap<double, 1, 1>(dom, qi, region, sph, stream, tune);
      return;
    }
  }
  STENCIL_REQUIRE(!tune.publish, "boundary-plane publication needs the whole-row kernel");
  // the column kernels wrap x only for whole chunks (ragged periodic rows are the whole-row kernel's)
  STENCIL_REQUIRE(!(tune.wrap & 1) || (stencil7x2_wrappable_axes(dom, qi, 0) & 1),
                  "in-kernel x wrap of a ragged row needs the whole-row kernel (fp32, x2row, 256 < nx < 1024)");
  // one-chunk column kernel: 12 waves (one src row each, 8 output rows) and one plane of z lookahead, the measured best
  // (bench.py 12x3 883-888, 12x1 881-883, 16x2 797-804, 8x2 759-772 Gcells/s, profiles/r1s4_bench_block_shapes.txt;
  // the other shapes were removed in r6)
  if (f32)
    jac ? apply_x2_t<float, 0, 12, 1>(dom, qi, region, sph, stream, tune)
        : apply_x2_t<float, 1, 12, 1>(dom, qi, region, sph, stream, tune);
  else
    jac ? apply_x2_t<double, 0, 12, 1>(dom, qi, region, sph, stream, tune)
        : apply_x2_t<double, 1, 12, 1>(dom, qi, region, sph, stream, tune);
}

template <typename T, int KIND>
static void apply_x2_regions_t(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &rs, const Spheres &sph,
                               hipStream_t stream, int wrap) {
  StencilArgs<T> a = make_args<T>(dom, qi, dom.get_compute_region(), KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth,
                                  sph);
  a.wrapm = wrap;
  const Dim3 org = dom.accessor_origin();
  for (size_t k0 = 0; k0 < rs.size(); k0 += kMaxX2Regions) {
    X2Regions rt{};
    for (size_t k = k0; k < rs.size() && rt.n < kMaxX2Regions; ++k) {
      const Rect3 r(rs[k].lo - org, rs[k].hi - org);
      const Dim3 e = r.extent();
      rt.lo[rt.n][0] = int(r.lo.x);
      rt.lo[rt.n][1] = int(r.lo.y);
      rt.lo[rt.n][2] = int(r.lo.z);
      rt.ext[rt.n][0] = int(e.x);
      rt.ext[rt.n][1] = int(e.y);
      rt.ext[rt.n][2] = int(e.z);
      rt.begin[rt.n + 1] = rt.begin[rt.n] + e.flatten();
      ++rt.n;
    }
    const int64_t total = rt.begin[rt.n];
    if (total == 0) continue;
    const int blocks = int(std::min<int64_t>((total + 255) / 256, 16384));
    hipLaunchKernelGGL((stencil7x2_regions_kernel<T, KIND>), dim3(blocks), dim3(256), 0, stream, a, rt);
    HIP_CHECK(hipGetLastError());
  }
}

void stencil7x2_apply_regions(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &regions, StencilKind kind,
                              const Spheres &sph, hipStream_t stream, int wrap) {
  STENCIL_REQUIRE(stencil7x2_supported(dom, qi), "two-step stencil needs a device fp32/fp64 quantity with depth-2 halos");
  const Rect3 cr = dom.get_compute_region();
  std::vector<Rect3> rs;
  for (const auto &r : regions) {
    if (r.empty()) continue;
    STENCIL_REQUIRE(cr.contains(r.lo) && r.hi.x <= cr.hi.x && r.hi.y <= cr.hi.y && r.hi.z <= cr.hi.z,
                    "stencil region " << r << " outside compute region " << cr);
    rs.push_back(r);
  }
  if (rs.empty()) return;
  dom.set_device();
  const bool f32 = dom.elem_size(qi) == 4;
  STENCIL_REQUIRE((wrap & ~7) == 0, "in-kernel wrap mask " << wrap);  // wrap_coord: any extent
  if (f32)
    kind == StencilKind::Jacobi ? apply_x2_regions_t<float, 0>(dom, qi, rs, sph, stream, wrap)
                                : apply_x2_regions_t<float, 1>(dom, qi, rs, sph, stream, wrap);
  else
    kind == StencilKind::Jacobi ? apply_x2_regions_t<double, 0>(dom, qi, rs, sph, stream, wrap)
                                : apply_x2_regions_t<double, 1>(dom, qi, rs, sph, stream, wrap);
}

template <typename T, int KIND, int THIN, int LANE, int MARCH>
static void launch_thin(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &slabs, const Spheres &sph,
                        hipStream_t stream, int wrap) {
  if (slabs.empty()) return;
  const Dim3 org = dom.accessor_origin();
  ThinTable tb{};
  int maxT = 0;
  for (const Rect3 &g : slabs) {
    const Rect3 r(g.lo - org, g.hi - org);
    const int i = tb.n++;
    const int64_t lo[3] = {r.lo.x, r.lo.y, r.lo.z}, hi[3] = {r.hi.x, r.hi.y, r.hi.z};
    for (int d = 0; d < 3; ++d) {
      tb.lo[i][d] = int(lo[d]);
      tb.hi[i][d] = int(hi[d]);
    }
    maxT = std::max(maxT, int(hi[THIN] - lo[THIN]));
    const int waves = int((hi[LANE] - lo[LANE] + 59) / 60) * int((hi[MARCH] - lo[MARCH] + kThinBC - 1) / kThinBC);
    tb.wbegin[i + 1] = tb.wbegin[i] + waves;
  }
  if (tb.wbegin[tb.n] == 0) return;
  StencilArgs<T> a = make_args<T>(dom, qi, dom.get_compute_region(), KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth,
                                  sph);
  a.x0 = int(dom.radius().x(-1)); // raw x of the first interior cell: 16-B aligned (stencil7x2_supported)
  a.wrapm = wrap;
  const uint32_t blocks = uint32_t((tb.wbegin[tb.n] + 3) / 4);
  if (maxT <= 2)
    hipLaunchKernelGGL((stencil7x2_thin_kernel<T, KIND, THIN, LANE, MARCH, 2>), dim3(blocks), dim3(256), 0, stream, a, tb);
  else
    hipLaunchKernelGGL((stencil7x2_thin_kernel<T, KIND, THIN, LANE, MARCH, 4>), dim3(blocks), dim3(256), 0, stream, a, tb);
  HIP_CHECK(hipGetLastError());
}

template <typename T, int KIND>
static void apply_exterior_t(const LocalDomain &dom, int64_t qi, const Rect3 &c, const Rect3 &in, const Spheres &sph,
                             hipStream_t stream, int wrap, bool zDone) {
  auto nonempty = [](std::initializer_list<Rect3> l) {
    std::vector<Rect3> v;
    for (const Rect3 &r : l)
      if (!r.empty()) v.push_back(r);
    return v;
  };
  // z slabs (whole x-y planes): lanes on x, march in y; y slabs (interior z): lanes on x, march in z; x slabs
  // (interior y, z): lanes on y, march in z
  const auto zs = nonempty({Rect3(c.lo, Dim3(c.hi.x, c.hi.y, in.lo.z)), Rect3(Dim3(c.lo.x, c.lo.y, in.hi.z), c.hi)});
  const auto ys = nonempty({Rect3(Dim3(c.lo.x, c.lo.y, in.lo.z), Dim3(c.hi.x, in.lo.y, in.hi.z)),
                            Rect3(Dim3(c.lo.x, in.hi.y, in.lo.z), Dim3(c.hi.x, c.hi.y, in.hi.z))});
  const auto xs = nonempty({Rect3(Dim3(c.lo.x, in.lo.y, in.lo.z), Dim3(in.lo.x, in.hi.y, in.hi.z)),
                            Rect3(Dim3(in.hi.x, in.lo.y, in.lo.z), Dim3(c.hi.x, in.hi.y, in.hi.z))});
  if (!zDone) launch_thin<T, KIND, 2, 0, 1>(dom, qi, zs, sph, stream, wrap);
  launch_thin<T, KIND, 1, 0, 2>(dom, qi, ys, sph, stream, wrap);
  launch_thin<T, KIND, 0, 1, 2>(dom, qi, xs, sph, stream, wrap);
}

void stencil7x2_apply_exterior(const LocalDomain &dom, int64_t qi, const Rect3 &interior, StencilKind kind,
                               const Spheres &sph, hipStream_t stream, const StencilTune &tune) {
  const Rect3 c = dom.get_compute_region();
  const Rect3 &in = interior;
  if (in.empty()) {
    stencil7x2_apply(dom, qi, c, kind, sph, stream, tune);
    return;
  }
  STENCIL_REQUIRE(stencil7x2_supported(dom, qi), "two-step stencil needs a device fp32/fp64 quantity with depth-2 halos");
  STENCIL_REQUIRE(c.contains(in.lo) && in.hi.x <= c.hi.x && in.hi.y <= c.hi.y && in.hi.z <= c.hi.z,
                  "interior " << in << " outside compute region " << c);
  // a wrapped axis is never cut by the interior: no slab is thin along it (x slabs load unwrapped row windows)
  check_wrap(dom, qi, in, tune.wrap, tune.x2row);
  const Dim3 lo = in.lo - c.lo, hi = c.hi - in.hi;
  if (std::max({lo.x, lo.y, lo.z, hi.x, hi.y, hi.z}) > 4) {
    // thick shells: the thread-per-cell kernel
    std::vector<Rect3> ext = {Rect3(c.lo, Dim3(c.hi.x, c.hi.y, in.lo.z)), Rect3(Dim3(c.lo.x, c.lo.y, in.hi.z), c.hi),
                              Rect3(Dim3(c.lo.x, c.lo.y, in.lo.z), Dim3(c.hi.x, in.lo.y, in.hi.z)),
                              Rect3(Dim3(c.lo.x, in.hi.y, in.lo.z), Dim3(c.hi.x, c.hi.y, in.hi.z)),
                              Rect3(Dim3(c.lo.x, in.lo.y, in.lo.z), Dim3(in.lo.x, in.hi.y, in.hi.z)),
                              Rect3(Dim3(in.hi.x, in.lo.y, in.lo.z), Dim3(c.hi.x, in.hi.y, in.hi.z))};
    stencil7x2_apply_regions(dom, qi, ext, kind, sph, stream, tune.wrap);
    return;
  }
  dom.set_device();
  const bool f32 = dom.elem_size(qi) == 4, jac = kind == StencilKind::Jacobi;
  // z slabs (whole x-y planes) of periodic 512-cell rows: the whole-row kernel, one block per 8 output rows of a
  // slab (fixed z chunk = the slab: every block marches only its slab's planes)
  bool zDone = false;
  if (f32 && tune.x2row && tune.zslabRow && (tune.wrap & 1) && lo.z <= 4 && hi.z <= 4) {
    StencilTune tz = tune;
    tz.x2sched = 0;
    tz.reserveCUs = 0;
    zDone = true;
    for (const Rect3 &r : {Rect3(c.lo, Dim3(c.hi.x, c.hi.y, in.lo.z)), Rect3(Dim3(c.lo.x, c.lo.y, in.hi.z), c.hi)}) {
      if (r.empty()) continue;
      tz.zchunk = int(r.hi.z - r.lo.z);
      stencil7x2_apply(dom, qi, r, kind, sph, stream, tz);
    }
  }
  if (f32)
    jac ? apply_exterior_t<float, 0>(dom, qi, c, in, sph, stream, tune.wrap, zDone)
        : apply_exterior_t<float, 1>(dom, qi, c, in, sph, stream, tune.wrap, zDone);
  else
    jac ? apply_exterior_t<double, 0>(dom, qi, c, in, sph, stream, tune.wrap, zDone)
        : apply_exterior_t<double, 1>(dom, qi, c, in, sph, stream, tune.wrap, zDone);
}

} // namespace stencil
