// 7-point stencil kernels (Jacobi3D / Astaroth proxy) for gfx950. See stencil/kernels/stencil_ops.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>

#include "stencil/domain/packer.hpp"
#include "stencil_common.hpp"
#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/rt/hip_check.hpp"

namespace stencil {

// "no forwarding target" marker of the halo-forwarding offsets (-2^62: far outside any allocation)
constexpr int64_t kNoForward = -(int64_t(1) << 62);

// 2.5D z-march. Lane = one 16-B x-chunk; wave = 64 chunks x TY rows; block = 4 waves stacked in y.
// Per z step a lane issues TY+2 row loads of plane z+1 (plus the two wave-edge scalars), then emits TY rows of
// plane z from registers: x-neighbours by ds_bpermute, y-neighbours from the adjacent rows, z from prev/next.
template <typename T, int TY, int KIND, bool NT, bool REMAP>
__global__ __launch_bounds__(256) void stencil7_kernel(StencilArgs<T> a) {
  using VT = typename Vec16<T>::type;
  constexpr int V = Vec16<T>::N;
  const uint32_t nb = uint32_t(a.gx) * a.gy * a.gz;
  const uint32_t hw = blockIdx.x;
  const uint32_t lb = REMAP ? xcd_remap(hw, nb) : hw;
  // logical order: z-chunk fastest, then y group, then x wave-column
  const int bz = int(lb % uint32_t(a.gz));
  const int by = int((lb / uint32_t(a.gz)) % uint32_t(a.gy));
  const int bx = int(lb / (uint32_t(a.gz) * a.gy));
  const int lane = threadIdx.x;
  const int c = bx * 64 + lane;
  const bool cvalid = c < a.nchunks;
  const int cl = cvalid ? c : a.nchunks - 1;
  const int xb = a.x0 + cl * V;
  const int ybase = a.loy + TY * (by * 4 + int(threadIdx.y));
  const int zs = a.loz + bz * a.zc;
  const int ze = min(zs + a.zc, a.hiz);
  if (ybase >= a.hiy || zs >= ze) return; // wave-uniform

  const bool edgeL = lane == 0;
  const bool edgeR = lane == 63 || c + 1 >= a.nchunks;
  const bool fullX = xb >= a.lox && xb + V <= a.hix;

  auto rowp = [&](int y, int z) -> const T * {
    y = min(y, a.rawYm1);
    return a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
  };
  auto ld = [&](const T *p) -> VT { return *reinterpret_cast<const VT *>(p); };

  VT prev[TY], cur[TY + 2], nxt[TY + 2];
  T curL[TY], curR[TY], nxtL[TY], nxtR[TY];
#pragma unroll
  for (int i = 0; i < TY; ++i) prev[i] = ld(rowp(ybase + i, zs - 1));
#pragma unroll
  for (int i = 0; i < TY + 2; ++i) cur[i] = ld(rowp(ybase - 1 + i, zs));
#pragma unroll
  for (int i = 0; i < TY; ++i) {
    const T *p = rowp(ybase + i, zs);
    curL[i] = edgeL ? p[-1] : T(0);
    curR[i] = edgeR ? p[V] : T(0);
  }

  const int r1sq = a.r1sq;
  for (int z = zs; z < ze; ++z) {
#pragma unroll
    for (int i = 0; i < TY + 2; ++i) nxt[i] = ld(rowp(ybase - 1 + i, z + 1));
    if (z + 1 < ze) {
#pragma unroll
      for (int i = 0; i < TY; ++i) {
        const T *p = rowp(ybase + i, z + 1);
        nxtL[i] = edgeL ? p[-1] : T(0);
        nxtR[i] = edgeR ? p[V] : T(0);
      }
    }

    const int dzh = z - a.hz, dzc = z - a.cz;
#pragma unroll
    for (int i = 1; i <= TY; ++i) {
      const int y = ybase + i - 1;
      const T sl = shfl_up1<T>(vget<T>(cur[i], V - 1));
      const T sr = shfl_down1<T>(vget<T>(cur[i], 0));
      const T left = edgeL ? curL[i - 1] : sl;
      const T right = edgeR ? curR[i - 1] : sr;
      T out[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T vpx = e < V - 1 ? vget<T>(cur[i], e + 1) : right;
        const T vmx = e > 0 ? vget<T>(cur[i], e - 1) : left;
        const T vpy = vget<T>(cur[i + 1], e);
        const T vmy = vget<T>(cur[i - 1], e);
        const T vpz = vget<T>(nxt[i], e);
        const T vmz = vget<T>(prev[i - 1], e);
        T val;
        // leading 0 + as in the reference (keeps the sign of zero identical)
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
        out[e] = div6<T>(val);
      }
      if (KIND == 0 && r1sq > 0) {
        // spheres: only rows whose (y,z) distance is inside the radius can contain sphere cells (wave-uniform)
        const int dyh = y - a.hy, dyc = y - a.cy;
        const int dyzh = dyh * dyh + dzh * dzh;
        const int dyzc = dyc * dyc + dzc * dzc;
        if (dyzh < r1sq || dyzc < r1sq) {
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const int x = xb + e;
            const bool hot = (x - a.hx) * (x - a.hx) < r1sq - dyzh;
            const bool cold = (x - a.cx) * (x - a.cx) < r1sq - dyzc;
            out[e] = hot ? T(1) : (cold ? T(0) : out[e]);
          }
        }
      }
      if (cvalid && y < a.hiy) {
        T *dp = a.dst + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
        if (fullX) {
          using NV = typename Vec16<T>::native;
          NV v;
#pragma unroll
          for (int e = 0; e < V; ++e) v[e] = out[e];
          if (NT)
            __builtin_nontemporal_store(v, reinterpret_cast<NV *>(dp));
          else
            *reinterpret_cast<NV *>(dp) = v;
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (xb + e >= a.lox && xb + e < a.hix) dp[e] = out[e];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TY; ++i) prev[i] = cur[i + 1];
#pragma unroll
    for (int i = 0; i < TY + 2; ++i) cur[i] = nxt[i];
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      curL[i] = nxtL[i];
      curR[i] = nxtR[i];
    }
  }
}

// Forward one output row chunk into the edge/corner halos it feeds (messages with two or three non-zero
// direction components; faces are stored inline by the kernel). sy/sz: wave-uniform y/z slab sides of the row,
// xside/xm: this lane's x slab side and element mask. Store address = own output address + fd[k].
template <typename T, int V>
__device__ __forceinline__ void forward_edges(const StencilArgs<T> &a, T *dp, const T (&out)[V], int xb, bool fullX,
                                              int sy, int sz, int xside, uint32_t xm) {
  using NV = typename Vec16<T>::native;
  for (int kz = 0; kz < 2; ++kz) {
    if (kz && !sz) break;
    const int dz = kz ? sz : 0;
    for (int ky = 0; ky < 2; ++ky) {
      if (ky && !sy) break;
      const int dy = ky ? sy : 0;
      const int k = 13 + 3 * dy + 9 * dz;
      if (dy != 0 && dz != 0 && (a.fmask >> k & 1u)) { // y-z edge: whole row chunk
        T *q = dp + a.fd[k];
        if (fullX) {
          NV v;
#pragma unroll
          for (int e = 0; e < V; ++e) v[e] = out[e];
          *reinterpret_cast<NV *>(q) = v;
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (xb + e >= a.lox && xb + e < a.hix) q[e] = out[e];
        }
      }
      if ((dy | dz) != 0 && xside != 0 && (a.fmask >> (k + xside) & 1u)) { // x-y, x-z edges and corners
        T *q = dp + a.fd[k + xside];
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (xm >> e & 1u) q[e] = out[e];
      }
    }
  }
}

// v3: block = NW waves stacked in y, TY rows per wave, one shared 16-B x-chunk column of 64 lanes. The y-halo rows of
// every wave come from its neighbours through LDS (double-buffered by z parity, one barrier per z step), so HBM
// reads per output row drop from (TY+2)/TY to (NW*TY+2)/(NW*TY).
// PF = z-planes of lookahead: 1 loads plane z+1 while computing plane z (the loads are consumed in the same step,
// so only other waves hide their latency); 2 loads plane z+2, so every load has a whole step to land.
// WRAP: along the axes set in a.wrapm the sub-domain is its own periodic neighbour (StencilTune::wrap): rows and
// planes beyond a face, and the edge scalars of the first / last chunk of a row, are read at their periodic image,
// so those halos need not be exchanged (one conditional shift per access; needs the chunk grid to start at lox and
// whole chunks along x).
template <typename T, int TY, int NW, int KIND, bool NT, bool REMAP, bool FWD, int PF = 1, bool WRAP = false>
__global__ __launch_bounds__(64 * NW, (TY <= 4 && sizeof(T) == 4 ? 4 : 1)) void stencil7_lds_kernel(StencilArgs<T> a) {
  using VT = typename Vec16<T>::type;
  constexpr int V = Vec16<T>::N;
  constexpr int SLOTS = 2 * NW + 2; // per wave: top row, bottom row; plus block halo above and below
  __shared__ VT lds[2][SLOTS][64];
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
  if (yblk >= a.hiy || zs >= ze) return; // block-uniform: every wave of the block leaves together
  // odd z-chunks march downwards: a chunk boundary is then read by both neighbouring chunks at the same time
  // (both start there, or both end there), so the warm-up planes are L2/MALL hits instead of HBM re-reads
  const bool down = ((bz & 1) != 0) != (a.flip != 0);
  const int dz = down ? -1 : 1;
  const int z0 = down ? ze - 1 : zs;
  const int nzs = ze - zs;

  const bool edgeL = lane == 0;
  const bool edgeR = lane == 63 || c + 1 >= a.nchunks;
  const bool fullX = xb >= a.lox && xb + V <= a.hix;
  // forwarding state, all fixed for the whole z-march except the z slab:
  //   x: this lane's slab side, element mask and (for single-cell slabs) the element index; pure-x store offset
  //   y: per row i of the wave, the slab side (wave-uniform) and the pure-y store offset (SGPRs)
  //   edges/corners (several non-zero components) take the general path, only if such messages exist
  int fxside = 0, fxe = -1;
  uint32_t fxm = 0, fxmPure = 0;
  int64_t fxd = 0;
  int fsy[TY];
  int64_t fdy[TY];
  T fxv[TY];
  bool fedges = false;
  if (FWD) {
    if (cvalid) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int x = xb + e;
        if (x >= a.lox && x < a.lox + a.fwm[0]) {
          fxm |= 1u << e;
          fxside = -1;
        }
        if (x >= a.hix - a.fwp[0] && x < a.hix) {
          fxm |= 1u << e;
          fxside = 1;
        }
      }
      if (fxside != 0 && (a.fmask >> (13 + fxside) & 1u)) {
        fxmPure = fxm;
        fxd = a.fd[13 + fxside];
        if (__builtin_popcount(fxm) == 1) fxe = __builtin_ctz(fxm); // only edge lanes get fxe >= 0
      }
    }
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      const int y = ybase + i;
      fsy[i] = y < a.loy + a.fwm[1] ? -1 : (y >= a.hiy - a.fwp[1] ? 1 : 0);
      fdy[i] = (fsy[i] != 0 && (a.fmask >> (13 + 3 * fsy[i]) & 1u)) ? a.fd[13 + 3 * fsy[i]] : kNoForward;
    }
    // any message with two or more non-zero components?
    constexpr uint32_t kFaces = (1u << 4) | (1u << 10) | (1u << 12) | (1u << 14) | (1u << 16) | (1u << 22);
    fedges = (a.fmask & ~kFaces) != 0;
  }
  const int slotTop = 2 * w, slotBot = 2 * w + 1;
  const int slotAbove = w == 0 ? 2 * NW : 2 * (w - 1) + 1;
  const int slotBelow = w == NW - 1 ? 2 * NW + 1 : 2 * (w + 1);

  // periodic images (WRAP): y beyond the region's y faces, z beyond its z faces (then clamped into the allocation:
  // the lookahead planes past the march end are loaded but never used)
  const int ywn = WRAP && (a.wrapm & 2) ? a.wn[1] : 0, ywlo = a.wlo[1], ywhi = a.wlo[1] + ywn;
  const int zwn = WRAP && (a.wrapm & 4) ? a.wn[2] : 0, zwlo = a.wlo[2], zwhi = a.wlo[2] + zwn;
  auto rowp = [&](int y, int z) -> const T * {
    if constexpr (WRAP) {
      y += y < ywlo ? ywn : 0;
      y -= y >= ywhi ? ywn : 0;
      z += z < zwlo ? zwn : 0;
      z -= z >= zwhi ? zwn : 0;
      z = z < 0 ? 0 : (z > a.rawZm1 ? a.rawZm1 : z);
    }
    y = min(y, a.rawYm1);
    return a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
  };
  auto ld = [&](const T *p) -> VT { return *reinterpret_cast<const VT *>(p); };
  // x edge scalars: left of the row's first chunk / right of its last one at the periodic image
  const bool xw = WRAP && (a.wrapm & 1);
  const int offL = -1 + (xw && xb == a.lox ? a.wn[0] : 0);
  const int offR = V - (xw && xb + V == a.hix ? a.wn[0] : 0);

  VT prev[TY], cur[TY], nxt[TY];
  T curL[TY], curR[TY], nxtL[TY], nxtR[TY];
  VT haloN; // block halo row of the next plane (wave 0: above, wave NW-1: below)
  // PF >= 2: planes z+2 .. z+PF in flight (fut[k] = plane z+(k+2)dz)
  constexpr int NF = PF > 1 ? PF - 1 : 1;
  VT fut[NF][TY], futH[NF];
  T futL[NF][TY], futR[NF][TY];
  auto zclamp = [&](int zz) { return zz < 0 ? 0 : (zz > a.rawZm1 ? a.rawZm1 : zz); };
#pragma unroll
  for (int i = 0; i < TY; ++i) prev[i] = ld(rowp(ybase + i, z0 - dz));
#pragma unroll
  for (int i = 0; i < TY; ++i) {
    const T *p = rowp(ybase + i, z0);
    cur[i] = ld(p);
    curL[i] = edgeL ? p[offL] : T(0);
    curR[i] = edgeR ? p[offR] : T(0);
  }
  if (w == 0) lds[0][2 * NW][lane] = ld(rowp(yblk - 1, z0));
  if (w == NW - 1) lds[0][2 * NW + 1][lane] = ld(rowp(yblk + NW * TY, z0));
  lds[0][slotTop][lane] = cur[0];
  lds[0][slotBot][lane] = cur[TY - 1];
  if constexpr (PF >= 2) {
    const int z1 = zclamp(z0 + dz);
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      const T *p = rowp(ybase + i, z1);
      nxt[i] = ld(p);
      nxtL[i] = edgeL ? p[offL] : T(0);
      nxtR[i] = edgeR ? p[offR] : T(0);
    }
    if (w == 0) haloN = ld(rowp(yblk - 1, z1));
    if (w == NW - 1) haloN = ld(rowp(yblk + NW * TY, z1));
#pragma unroll
    for (int k = 0; k + 1 < NF; ++k) {
      const int zk = zclamp(z0 + (k + 2) * dz);
#pragma unroll
      for (int i = 0; i < TY; ++i) {
        const T *p = rowp(ybase + i, zk);
        fut[k][i] = ld(p);
        futL[k][i] = edgeL ? p[offL] : T(0);
        futR[k][i] = edgeR ? p[offR] : T(0);
      }
      if (w == 0) futH[k] = ld(rowp(yblk - 1, zk));
      if (w == NW - 1) futH[k] = ld(rowp(yblk + NW * TY, zk));
    }
  }
  __syncthreads();

  const int r1sq = a.r1sq;
  int buf = 0;
  int z = z0;
  for (int step = 0; step < nzs; ++step, z += dz) {
    if constexpr (PF == 1) {
      const int zn = z + dz;
#pragma unroll
      for (int i = 0; i < TY; ++i) nxt[i] = ld(rowp(ybase + i, zn));
      if (w == 0) haloN = ld(rowp(yblk - 1, zn));
      if (w == NW - 1) haloN = ld(rowp(yblk + NW * TY, zn));
      if (step + 1 < nzs) {
#pragma unroll
        for (int i = 0; i < TY; ++i) {
          const T *p = rowp(ybase + i, zn);
          nxtL[i] = edgeL ? p[offL] : T(0);
          nxtR[i] = edgeR ? p[offR] : T(0);
        }
      }
    } else {
      // plane z+PF (clamped into the allocation at the ends of the march; those values are never used)
      const int zf = zclamp(z + PF * dz);
#pragma unroll
      for (int i = 0; i < TY; ++i) {
        const T *p = rowp(ybase + i, zf);
        fut[NF - 1][i] = ld(p);
        futL[NF - 1][i] = edgeL ? p[offL] : T(0);
        futR[NF - 1][i] = edgeR ? p[offR] : T(0);
      }
      if (w == 0) futH[NF - 1] = ld(rowp(yblk - 1, zf));
      if (w == NW - 1) futH[NF - 1] = ld(rowp(yblk + NW * TY, zf));
    }
    const VT above = lds[buf][slotAbove][lane];
    const VT below = lds[buf][slotBelow][lane];

    const int dzh = z - a.hz, dzc = z - a.cz;
    int fsz = 0;
    int64_t fdz = kNoForward;
    if constexpr (FWD) {
      fsz = z < a.loz + a.fwm[2] ? -1 : (z >= a.hiz - a.fwp[2] ? 1 : 0);
      if (fsz != 0 && (a.fmask >> (13 + 9 * fsz) & 1u)) fdz = a.fd[13 + 9 * fsz];
    }
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      const int y = ybase + i;
      const VT &up = i == 0 ? above : cur[i - 1];
      const VT &dn = i == TY - 1 ? below : cur[i + 1];
      const T sl = shfl_up1<T>(vget<T>(cur[i], V - 1));
      const T sr = shfl_down1<T>(vget<T>(cur[i], 0));
      const T left = edgeL ? curL[i] : sl;
      const T right = edgeR ? curR[i] : sr;
      T out[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T vpx = e < V - 1 ? vget<T>(cur[i], e + 1) : right;
        const T vmx = e > 0 ? vget<T>(cur[i], e - 1) : left;
        const T vpy = vget<T>(dn, e);
        const T vmy = vget<T>(up, e);
        const T vpz = down ? vget<T>(prev[i], e) : vget<T>(nxt[i], e);
        const T vmz = down ? vget<T>(nxt[i], e) : vget<T>(prev[i], e);
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
        out[e] = div6<T>(val);
      }
      if (KIND == 0 && r1sq > 0) {
        const int dyh = y - a.hy, dyc = y - a.cy;
        const int dyzh = dyh * dyh + dzh * dzh;
        const int dyzc = dyc * dyc + dzc * dzc;
        if (dyzh < r1sq || dyzc < r1sq) {
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const int x = xb + e;
            const bool hot = (x - a.hx) * (x - a.hx) < r1sq - dyzh;
            const bool cold = (x - a.cx) * (x - a.cx) < r1sq - dyzc;
            out[e] = hot ? T(1) : (cold ? T(0) : out[e]);
          }
        }
      }
      if (cvalid && y < a.hiy) {
        T *dp = a.dst + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
        if (fullX) {
          using NV = typename Vec16<T>::native;
          NV v;
#pragma unroll
          for (int e = 0; e < V; ++e) v[e] = out[e];
          if (NT)
            __builtin_nontemporal_store(v, reinterpret_cast<NV *>(dp));
          else
            *reinterpret_cast<NV *>(dp) = v;
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (xb + e >= a.lox && xb + e < a.hix) dp[e] = out[e];
        }
        if constexpr (FWD) {
          using NV = typename Vec16<T>::native;
          // pure x: single-cell slabs are stashed (one select, no branch) and stored once per plane below;
          // wider slabs are stored here by the edge lane
          if (fxe >= 0) {
            T v = out[0];
#pragma unroll
            for (int e = 1; e < V; ++e) v = fxe == e ? out[e] : v;
            fxv[i] = v;
          } else if (fxmPure) {
            T *q = dp + fxd;
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (fxmPure >> e & 1u) q[e] = out[e];
          }
          // pure y / pure z: wave-uniform, offsets already in SGPRs
          const bool yrow = fdy[i] != kNoForward, zrow = fdz != kNoForward;
          if (yrow || zrow) {
            NV v;
#pragma unroll
            for (int e = 0; e < V; ++e) v[e] = out[e];
            if (fullX) {
              if (yrow) *reinterpret_cast<NV *>(dp + fdy[i]) = v;
              if (zrow) *reinterpret_cast<NV *>(dp + fdz) = v;
            } else {
#pragma unroll
              for (int e = 0; e < V; ++e)
                if (xb + e >= a.lox && xb + e < a.hix) {
                  if (yrow) dp[fdy[i] + e] = out[e];
                  if (zrow) dp[fdz + e] = out[e];
                }
            }
          }
          if (fedges && ((fsy[i] != 0) + (fsz != 0) + (fxside != 0) >= 2))
            forward_edges<T, V>(a, dp, out, xb, fullX, fsy[i], fsz, fxside, fxm);
        }
      }
    }
    if constexpr (FWD) {
      if (fxe >= 0) { // edge lanes only: the plane's stashed single-cell x messages
        T *q = a.dst + int64_t(z) * a.pxy + int64_t(ybase) * a.px + (xb + fxe) + fxd;
#pragma unroll
        for (int i = 0; i < TY; ++i)
          if (ybase + i < a.hiy) q[int64_t(i) * a.px] = fxv[i];
      }
    }
    // publish plane z+1 boundary rows for the next step
    buf ^= 1;
    lds[buf][slotTop][lane] = nxt[0];
    lds[buf][slotBot][lane] = nxt[TY - 1];
    if (w == 0) lds[buf][2 * NW][lane] = haloN;
    if (w == NW - 1) lds[buf][2 * NW + 1][lane] = haloN;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TY; ++i) {
      prev[i] = cur[i];
      cur[i] = nxt[i];
      curL[i] = nxtL[i];
      curR[i] = nxtR[i];
      if constexpr (PF >= 2) {
        nxt[i] = fut[0][i];
        nxtL[i] = futL[0][i];
        nxtR[i] = futR[0][i];
#pragma unroll
        for (int k = 0; k + 1 < NF; ++k) {
          fut[k][i] = fut[k + 1][i];
          futL[k][i] = futL[k + 1][i];
          futR[k][i] = futR[k + 1][i];
        }
      }
    }
    if constexpr (PF >= 2) {
      haloN = futH[0];
#pragma unroll
      for (int k = 0; k + 1 < NF; ++k) futH[k] = futH[k + 1];
    }
  }
}

// Several thin regions (the exterior slabs) in one launch, one thread per cell.
constexpr int kMaxRegions = 8;
struct RegionTable {
  int lo[kMaxRegions][3];
  int ext[kMaxRegions][3];
  int64_t begin[kMaxRegions + 1];
  int n;
};

template <typename T, int KIND>
__global__ __launch_bounds__(256) void stencil7_regions_kernel(StencilArgs<T> a, RegionTable rt) {
  const int64_t total = rt.begin[rt.n];
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    int k = 0;
    while (k + 1 < rt.n && rt.begin[k + 1] <= i) ++k;
    const int64_t li = i - rt.begin[k];
    const int nx = rt.ext[k][0], ny = rt.ext[k][1];
    const int x = rt.lo[k][0] + int(li % nx);
    const int y = rt.lo[k][1] + int((li / nx) % ny);
    const int z = rt.lo[k][2] + int(li / (int64_t(nx) * ny));
    const T *p = a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + x;
    T val = T(0);
    if (KIND == 0) {
      val += p[1];
      val += p[-1];
      val += p[a.px];
      val += p[-a.px];
      val += p[a.pxy];
      val += p[-a.pxy];
    } else {
      val += p[-1];
      val += p[-a.px];
      val += p[-a.pxy];
      val += p[1];
      val += p[a.px];
      val += p[a.pxy];
    }
    val = div6<T>(val);
    if (KIND == 0 && a.r1sq > 0) {
      const int dh = (x - a.hx) * (x - a.hx) + (y - a.hy) * (y - a.hy) + (z - a.hz) * (z - a.hz);
      const int dc = (x - a.cx) * (x - a.cx) + (y - a.cy) * (y - a.cy) + (z - a.cz) * (z - a.cz);
      val = dh < a.r1sq ? T(1) : (dc < a.r1sq ? T(0) : val);
    }
    a.dst[int64_t(z) * a.pxy + int64_t(y) * a.px + x] = val;
  }
}

// generic scalar fallback (unaligned layouts); also the device reference used by tests
template <typename T, int KIND>
__global__ __launch_bounds__(256) void stencil7_generic_kernel(StencilArgs<T> a) {
  const int64_t nx = a.hix - a.lox, ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  const int64_t total = nx * ny * nz;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int x = a.lox + int(i % nx), y = a.loy + int((i / nx) % ny), z = a.loz + int(i / (nx * ny));
    const T *p = a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + x;
    T val = T(0);
    if (KIND == 0) {
      val += p[1];
      val += p[-1];
      val += p[a.px];
      val += p[-a.px];
      val += p[a.pxy];
      val += p[-a.pxy];
    } else {
      val += p[-1];
      val += p[-a.px];
      val += p[-a.pxy];
      val += p[1];
      val += p[a.px];
      val += p[a.pxy];
    }
    val /= T(6);
    if (KIND == 0 && a.r1sq > 0) {
      const int dh = (x - a.hx) * (x - a.hx) + (y - a.hy) * (y - a.hy) + (z - a.hz) * (z - a.hz);
      const int dc = (x - a.cx) * (x - a.cx) + (y - a.cy) * (y - a.cy) + (z - a.cz) * (z - a.cz);
      if (dh < a.r1sq)
        val = T(1);
      else if (dc < a.r1sq)
        val = T(0);
    }
    a.dst[int64_t(z) * a.pxy + int64_t(y) * a.px + x] = val;
  }
}

// Exterior shell: thin slabs after the exchange. Wave-granular work table:
//   ROW slabs (x-extent >= 8, i.e. y/z faces): one wave = 64 x-chunks of one (y, z) row; 5 coalesced 16-B row loads
//     (centre, y+-1, z+-1) + 2 edge scalars per lane.
//   COL slabs (thin in x, i.e. x faces): one wave = 64 consecutive y of one (x, z); lanes along y, so y-neighbours
//     come from adjacent lanes and each lane touches its own row line once (x+-1 share it).
// a.wrapm: along those axes neighbours beyond a face are read at their periodic image (StencilTune::wrap; x only
// for whole 16-B chunks from the face, stencil7_wrappable_axes).
constexpr int kMaxShell = 8;
struct ShellTable {
  int lo[kMaxShell][3];
  int ext[kMaxShell][3];
  int x0[kMaxShell];      // ROW: raw x of chunk 0
  int nch[kMaxShell];     // ROW: chunks per row
  int col[kMaxShell];     // 1 = COL slab
  int64_t wbegin[kMaxShell + 1];
  int n;
};

template <typename T, int KIND>
__device__ __forceinline__ T finish_cell(const StencilArgs<T> &a, T px, T mx, T py, T my, T pz, T mz, int x, int y,
                                         int z) {
  T val;
  if (KIND == 0) {
    val = T(0) + px;
    val += mx;
    val += py;
    val += my;
    val += pz;
    val += mz;
  } else {
    val = T(0) + mx;
    val += my;
    val += mz;
    val += px;
    val += py;
    val += pz;
  }
  val = div6<T>(val);
  if (KIND == 0 && a.r1sq > 0) {
    const int dh = (x - a.hx) * (x - a.hx) + (y - a.hy) * (y - a.hy) + (z - a.hz) * (z - a.hz);
    const int dc = (x - a.cx) * (x - a.cx) + (y - a.cy) * (y - a.cy) + (z - a.cz) * (z - a.cz);
    val = dh < a.r1sq ? T(1) : (dc < a.r1sq ? T(0) : val);
  }
  return val;
}

template <typename T, int KIND>
__global__ __launch_bounds__(256) void stencil7_shell_kernel(StencilArgs<T> a, ShellTable st) {
  using VT = typename Vec16<T>::type;
  constexpr int V = Vec16<T>::N;
  const int64_t wave = int64_t(blockIdx.x) * 4 + threadIdx.y;
  if (wave >= st.wbegin[st.n]) return; // wave-uniform
  int k = 0;
  while (k + 1 < st.n && st.wbegin[k + 1] <= wave) ++k;
  const int64_t wl = wave - st.wbegin[k];
  const int lane = threadIdx.x;
  const int lx = st.lo[k][0], ly = st.lo[k][1], lz = st.lo[k][2];
  const int ex = st.ext[k][0], ey = st.ext[k][1];
  auto wrapc = [&](int c, int ax) { // one conditional shift (the neighbour of a face cell)
    if ((a.wrapm >> ax) & 1) {
      c += c < a.wlo[ax] ? a.wn[ax] : 0;
      c -= c >= a.wlo[ax] + a.wn[ax] ? a.wn[ax] : 0;
    }
    return c;
  };
  auto at = [&](int x, int y, int z) { return a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + x; };
  if (!st.col[k]) {
    // ROW: wl -> (chunk wave cw, y, z)
    const int cws = (st.nch[k] + 63) / 64;
    const int cw = int(wl % cws);
    const int64_t r = wl / cws;
    const int y = ly + int(r % ey);
    const int z = lz + int(r / ey);
    const int c = cw * 64 + lane;
    const bool valid = c < st.nch[k];
    const int xb = st.x0[k] + (valid ? c : st.nch[k] - 1) * V;
    const T *p = at(xb, y, z);
    const VT cc = *reinterpret_cast<const VT *>(p);
    const VT yp = *reinterpret_cast<const VT *>(at(xb, wrapc(y + 1, 1), z));
    const VT ym = *reinterpret_cast<const VT *>(at(xb, wrapc(y - 1, 1), z));
    const VT zp = *reinterpret_cast<const VT *>(at(xb, y, wrapc(z + 1, 2)));
    const VT zm = *reinterpret_cast<const VT *>(at(xb, y, wrapc(z - 1, 2)));
    const bool eL = lane == 0, eR = lane == 63 || c + 1 >= st.nch[k];
    const bool xw = (a.wrapm & 1) != 0;
    const T le = eL ? p[-1 + (xw && xb == a.wlo[0] ? a.wn[0] : 0)] : T(0);
    const T re = eR ? p[V - (xw && xb + V == a.wlo[0] + a.wn[0] ? a.wn[0] : 0)] : T(0);
    const T sl = shfl_up1<T>(vget<T>(cc, V - 1));
    const T sr = shfl_down1<T>(vget<T>(cc, 0));
    const T left = eL ? le : sl, right = eR ? re : sr;
    if (!valid) return;
    T *dp = a.dst + int64_t(z) * a.pxy + int64_t(y) * a.px + xb;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int x = xb + e;
      if (x < lx || x >= lx + ex) continue;
      const T vpx = e < V - 1 ? vget<T>(cc, e + 1) : right;
      const T vmx = e > 0 ? vget<T>(cc, e - 1) : left;
      dp[e] = finish_cell<T, KIND>(a, vpx, vmx, vget<T>(yp, e), vget<T>(ym, e), vget<T>(zp, e), vget<T>(zm, e), x, y, z);
    }
  } else {
    // COL: wl -> (x, y block, z); lanes along y
    const int ybs = (ey + 63) / 64;
    const int x = lx + int(wl % ex);
    const int64_t r = wl / ex;
    const int yb = int(r % ybs);
    const int z = lz + int(r / ybs);
    const int y = ly + yb * 64 + lane;
    const bool valid = y < ly + ey;
    const int yl = valid ? y : ly + ey - 1;
    const T *p = at(x, yl, z);
    const T c0 = p[0], vpx = *at(wrapc(x + 1, 0), yl, z), vmx = *at(wrapc(x - 1, 0), yl, z);
    const T vpz = *at(x, yl, wrapc(z + 1, 2)), vmz = *at(x, yl, wrapc(z - 1, 2));
    const bool eL = lane == 0, eR = lane == 63 || !(y + 1 < ly + ey);
    const T ue = eL ? *at(x, wrapc(yl - 1, 1), z) : T(0);
    const T de = eR ? *at(x, wrapc(yl + 1, 1), z) : T(0);
    const T su = shfl_up1<T>(c0);   // value of y-1
    const T sd = shfl_down1<T>(c0); // value of y+1
    const T vmy = eL ? ue : su, vpy = eR ? de : sd;
    if (!valid) return;
    a.dst[int64_t(z) * a.pxy + int64_t(y) * a.px + x] = finish_cell<T, KIND>(a, vpx, vmx, vpy, vmy, vpz, vmz, x, y, z);
  }
}

// ---------------------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------------------
template <typename T, int KIND>
static void host_apply(const LocalDomain &dom, const StencilArgs<T> &a) {
  (void)dom;
  for (int z = a.loz; z < a.hiz; ++z)
    for (int y = a.loy; y < a.hiy; ++y)
      for (int x = a.lox; x < a.hix; ++x) {
        const T *p = a.src + int64_t(z) * a.pxy + int64_t(y) * a.px + x;
        T val = T(0);
        if (KIND == 0) {
          val += p[1];
          val += p[-1];
          val += p[a.px];
          val += p[-a.px];
          val += p[a.pxy];
          val += p[-a.pxy];
        } else {
          val += p[-1];
          val += p[-a.px];
          val += p[-a.pxy];
          val += p[1];
          val += p[a.px];
          val += p[a.pxy];
        }
        val /= T(6);
        if (KIND == 0 && a.r1sq > 0) {
          const int dh = (x - a.hx) * (x - a.hx) + (y - a.hy) * (y - a.hy) + (z - a.hz) * (z - a.hz);
          const int dc = (x - a.cx) * (x - a.cx) + (y - a.cy) * (y - a.cy) + (z - a.cz) * (z - a.cz);
          if (dh < a.r1sq)
            val = T(1);
          else if (dc < a.r1sq)
            val = T(0);
        }
        a.dst[int64_t(z) * a.pxy + int64_t(y) * a.px + x] = val;
      }
}

template <typename T, int TY, int KIND>
static void launch_fast(StencilArgs<T> a, const StencilTune &tune, hipStream_t stream) {
  constexpr int V = Vec16<T>::N;
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = (a.nchunks + 63) / 64;
  a.gy = (ny + 4 * TY - 1) / (4 * TY);
  int zc = tune.zchunk;
  if (zc <= 0) {
    // ~2 rounds of resident blocks (4 blocks of 4 waves per CU at <=128 VGPRs) over 256 CUs, z-chunks >= 8 planes
    const int64_t cols = int64_t(a.gx) * a.gy;
    const int64_t targetBlocks = 2048;
    const int64_t nzc = std::max<int64_t>(1, (targetBlocks + cols - 1) / cols);
    zc = int(std::max<int64_t>(8, (nz + nzc - 1) / nzc));
  }
  a.zc = zc;
  a.gz = (nz + zc - 1) / zc;
  (void)V;
  const uint32_t blocks = uint32_t(a.gx) * a.gy * a.gz;
  const dim3 block(64, 4);
  if (tune.nontemporal) {
    if (tune.xcdRemap)
      hipLaunchKernelGGL((stencil7_kernel<T, TY, KIND, true, true>), dim3(blocks), block, 0, stream, a);
    else
      hipLaunchKernelGGL((stencil7_kernel<T, TY, KIND, true, false>), dim3(blocks), block, 0, stream, a);
  } else {
    if (tune.xcdRemap)
      hipLaunchKernelGGL((stencil7_kernel<T, TY, KIND, false, true>), dim3(blocks), block, 0, stream, a);
    else
      hipLaunchKernelGGL((stencil7_kernel<T, TY, KIND, false, false>), dim3(blocks), block, 0, stream, a);
  }
  HIP_CHECK(hipGetLastError());
}

// resident blocks of `kernel` over the whole device (cached per kernel)
static int64_t resident_blocks(const void *kernel, int threads) {
  static std::map<const void *, int64_t> cache;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int dev = 0, perCU = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kernel, threads, 0) != hipSuccess || perCU <= 0) perCU = 2;
  (void)hipGetLastError();
  const int64_t r = int64_t(perCU) * cus;
  cache[kernel] = r;
  return r;
}

template <typename T, int TY, int NW, int KIND, bool WRAP = false>
static void launch_lds(StencilArgs<T> a, const StencilTune &tune, hipStream_t stream) {
  const int ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = (a.nchunks + 63) / 64;
  a.gy = (ny + NW * TY - 1) / (NW * TY);
  int zc = tune.zchunk;
  if (zc <= 0) {
    // Exactly one round of resident blocks (occupancy x CUs): a partial second round leaves most CUs idle at the
    // end (512^3, 2 rows/lane: 1024 blocks at 768 resident ran 20% slower than 768 or 512). z-chunks >= 16
    // planes (the warm-up planes of neighbouring chunks are shared, see kernel).
    const int64_t cols = int64_t(a.gx) * a.gy;
    const void *kern = WRAP      ? (const void *)stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 2, true>
                       : a.fmask ? (const void *)stencil7_lds_kernel<T, TY, NW, KIND, true, true, true>
                       : tune.variant == 2 ? (const void *)stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 2>
                       : tune.variant == 3 ? (const void *)stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 3>
                       : tune.variant == 4 ? (const void *)stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 4>
                                           : (const void *)stencil7_lds_kernel<T, TY, NW, KIND, true, true, false>;
    int64_t targetBlocks = resident_blocks(kern, 64 * NW);
    if (tune.reserveCUs > 0) { // leave that many CUs to the comm stream's kernels (overlapped steps)
      int cus = 256, dev = 0; // the device the launch goes to (the caller set it: dom.set_device())
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
      const int64_t perCU = std::max<int64_t>(1, targetBlocks / std::max(1, cus));
      targetBlocks = std::max<int64_t>(perCU, targetBlocks - perCU * std::min(tune.reserveCUs, cus / 2));
    }
    const int64_t nzc = std::max<int64_t>(1, targetBlocks / cols);
    zc = int(std::max<int64_t>(16, (nz + nzc - 1) / nzc));
  }
  a.zc = zc;
  a.gz = (nz + zc - 1) / zc;
  const uint32_t blocks = uint32_t(a.gx) * a.gy * a.gz;
  const dim3 block(64, NW);
  if (WRAP)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 2, WRAP>), dim3(blocks), block, 0, stream,
                       a);
  else if (a.fmask)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, true, true>), dim3(blocks), block, 0, stream, a);
  else if (tune.variant == 2)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 2>), dim3(blocks), block, 0, stream, a);
  else if (tune.variant == 3)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 3>), dim3(blocks), block, 0, stream, a);
  else if (tune.variant == 4)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, true, false, 4>), dim3(blocks), block, 0, stream, a);
  else if (!tune.nontemporal)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, false, true, false>), dim3(blocks), block, 0, stream, a);
  else if (tune.xcdRemap)
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, true, false>), dim3(blocks), block, 0, stream, a);
  else
    hipLaunchKernelGGL((stencil7_lds_kernel<T, TY, NW, KIND, true, false, false>), dim3(blocks), block, 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

template <typename T, int KIND>
static void apply_t(const LocalDomain &dom, int64_t qi, const Rect3 &region, const Spheres &sph, hipStream_t stream,
                    const StencilTune &tune, const HaloForwarder *fwd) {
  if (region.empty()) return;
  StencilArgs<T> a = make_args<T>(dom, qi, region, KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth, sph);
  a.flip = tune.alternateZ ? (dom.parity() & 1) : 0;
  if (fwd) {
    STENCIL_REQUIRE(region == dom.get_compute_region(), "halo forwarding needs the whole compute region");
    STENCIL_REQUIRE(HaloForwarder::supported(dom, qi), "halo forwarding not supported for this layout");
    const int par = dom.parity();
    for (int k = 0; k < 3; ++k) {
      a.fwm[k] = fwd->wm()[k];
      a.fwp[k] = fwd->wp()[k];
    }
    a.fmask = fwd->mask(par);
    for (int k = 0; k < 27; ++k) a.fd[k] = fwd->delta(par, k);
  }
  if (dom.backend() == Backend::Host) {
    host_apply<T, KIND>(dom, a);
    return;
  }
  constexpr int V = Vec16<T>::N;
  const int rxm = int(dom.radius().x(-1));
  // chunk grid anchored at the (64-B aligned) interior start
  const int off = ((a.lox - rxm) % V + V) % V;
  a.x0 = a.lox - off;
  a.nchunks = (a.hix - a.x0 + V - 1) / V;
  const bool alignedLayout = (reinterpret_cast<uintptr_t>(a.src + a.x0) % 16 == 0) &&
                             (reinterpret_cast<uintptr_t>(a.dst + a.x0) % 16 == 0) && ((a.px * int64_t(sizeof(T))) % 16 == 0);
  // vector loads and the right-edge neighbour stay inside the padded row (LocalDomain keeps >= V+1 tail elements)
  const bool fits = a.x0 + int64_t(a.nchunks) * V < dom.row_limit(qi);
  dom.set_device();
  STENCIL_REQUIRE(!fwd || (alignedLayout && fits), "halo forwarding needs the aligned vector layout");
  if (tune.wrap != 0) {
    // in-kernel periodic wrap: the lookahead-2 LDS kernel (the default shape) reading periodic images
    STENCIL_REQUIRE(fwd == nullptr, "in-kernel wrap and halo forwarding are exclusive");
    STENCIL_REQUIRE((tune.wrap & ~stencil7_wrappable_axes(dom, qi)) == 0,
                    "in-kernel wrap " << tune.wrap << " not supported by this layout (" << stencil7_wrappable_axes(dom, qi)
                                      << ")");
    const Rect3 cr = dom.get_compute_region();
    const int64_t lo[3] = {region.lo.x, region.lo.y, region.lo.z}, hi[3] = {region.hi.x, region.hi.y, region.hi.z};
    const int64_t clo[3] = {cr.lo.x, cr.lo.y, cr.lo.z}, chi[3] = {cr.hi.x, cr.hi.y, cr.hi.z};
    for (int ax = 0; ax < 3; ++ax)
      STENCIL_REQUIRE(!((tune.wrap >> ax) & 1) || (lo[ax] == clo[ax] && hi[ax] == chi[ax]),
                      "region " << region << " does not span wrapped axis " << ax << " of " << cr);
    STENCIL_REQUIRE(alignedLayout && fits && a.x0 == a.lox,
                    "in-kernel wrap needs the aligned vector layout (aligned " << alignedLayout << ", fits " << fits
                                                                               << ", x0 " << a.x0 << ", lox " << a.lox
                                                                               << ", px " << a.px << ", pad "
                                                                               << dom.pad_x(qi) << ", src%64 "
                                                                               << (reinterpret_cast<uintptr_t>(a.src) % 64)
                                                                               << ", nchunks " << a.nchunks << ")");
    a.wrapm = tune.wrap;
    launch_lds<T, 2, 8, KIND, true>(a, tune, stream);
    return;
  }
  if (alignedLayout && fits) {
    if (fwd) {
      // the forwarding epilogue needs registers: 2 rows per lane keeps it spill-free at >= 4 waves/SIMD
      launch_lds<T, 2, 8, KIND>(a, tune, stream);
    } else if (tune.variant == 1) {
      if (tune.ty == 4)
        launch_fast<T, 4, KIND>(a, tune, stream);
      else
        launch_fast<T, 8, KIND>(a, tune, stream);
    } else {
      if (tune.variant >= 2) {
        // deep lookahead keeps PF planes of rows in registers: 1-2 rows per lane only
        if (tune.ty == 1)
          launch_lds<T, 1, 8, KIND>(a, tune, stream);
        else if (tune.nw == 4)
          launch_lds<T, 2, 4, KIND>(a, tune, stream);
        else if (tune.nw == 16)
          launch_lds<T, 2, 16, KIND>(a, tune, stream);
        else
          launch_lds<T, 2, 8, KIND>(a, tune, stream);
      } else if (tune.ty == 8)
        launch_lds<T, 8, 4, KIND>(a, tune, stream);
      else if (tune.ty == 2)
        launch_lds<T, 2, 8, KIND>(a, tune, stream);
      else
        launch_lds<T, 4, 8, KIND>(a, tune, stream);
    }
  } else {
    const int64_t total = Rect3(Dim3(a.lox, a.loy, a.loz), Dim3(a.hix, a.hiy, a.hiz)).extent().flatten();
    const int blocks = int(std::min<int64_t>((total + 255) / 256, 4096));
    hipLaunchKernelGGL((stencil7_generic_kernel<T, KIND>), dim3(blocks), dim3(256), 0, stream, a);
    HIP_CHECK(hipGetLastError());
  }
}

int stencil7_wrappable_axes(const LocalDomain &dom, int64_t qi) {
  if (dom.backend() != Backend::Device) return 0;
  const DType dt = dom.dtype(qi);
  const int64_t es = dom.elem_size(qi);
  if (!(dt == DType::F32 || dt == DType::F64 || (dt == DType::Bytes && (es == 4 || es == 8)))) return 0;
  const int64_t V = 16 / es;
  const int64_t lox = dom.radius().x(-1), nx = dom.size().x;
  const Dim3 p = dom.pitch(qi);
  // the chunk grid starts at lox (16-B aligned) and the vector loads stay inside the padded row (apply_t's `fits`)
  const bool aligned = (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.curr_data(qi)) + lox * es) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.next_data(qi)) + lox * es) % 16 == 0) &&
                       (p.x * es) % 16 == 0;
  if (!aligned || lox + (nx + V - 1) / V * V >= dom.row_limit(qi)) return 0;
  // x: whole chunks (the last chunk's right edge is the face); y / z: one conditional shift per access
  return (nx % V == 0 ? 1 : 0) | 2 | 4;
}

void stencil7_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                    hipStream_t stream, const StencilTune &tune, const HaloForwarder *fwd) {
  STENCIL_REQUIRE(dom.radius().x(-1) >= 1 && dom.radius().x(1) >= 1 && dom.radius().y(-1) >= 1 &&
                      dom.radius().y(1) >= 1 && dom.radius().z(-1) >= 1 && dom.radius().z(1) >= 1,
                  "7-point stencil needs face radii >= 1");
  const Rect3 cr = dom.get_compute_region();
  STENCIL_REQUIRE(region.empty() || (cr.contains(region.lo) && region.hi.all_ge(region.lo) &&
                                     region.hi.x <= cr.hi.x && region.hi.y <= cr.hi.y && region.hi.z <= cr.hi.z),
                  "stencil region " << region << " outside compute region " << cr);
  if (tune.variant == StencilTune::kMfma) {
    STENCIL_REQUIRE(fwd == nullptr, "the MFMA variant does not forward halos");
    STENCIL_REQUIRE(tune.wrap == 0, "the MFMA variant reads halos (no in-kernel wrap)");
    stencil7_mfma_apply(dom, qi, region, kind, sph, stream, tune);
    return;
  }
  const DType dt = dom.dtype(qi);
  const bool f32 = dt == DType::F32 || (dt == DType::Bytes && dom.elem_size(qi) == 4);
  const bool f64 = dt == DType::F64 || (dt == DType::Bytes && dom.elem_size(qi) == 8);
  if (f32) {
    if (kind == StencilKind::Jacobi)
      apply_t<float, 0>(dom, qi, region, sph, stream, tune, fwd);
    else
      apply_t<float, 1>(dom, qi, region, sph, stream, tune, fwd);
  } else if (f64) {
    if (kind == StencilKind::Jacobi)
      apply_t<double, 0>(dom, qi, region, sph, stream, tune, fwd);
    else
      apply_t<double, 1>(dom, qi, region, sph, stream, tune, fwd);
  } else {
    LOG_FATAL("stencil7 supports fp32/fp64 quantities only");
  }
}

template <typename T, int KIND>
static void apply_regions_t(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &regions, const Spheres &sph,
                            hipStream_t stream, int wrap) {
  constexpr int V = Vec16<T>::N;
  StencilArgs<T> a = make_args<T>(dom, qi, dom.get_compute_region(), KIND == 0 ? StencilKind::Jacobi : StencilKind::Astaroth,
                                  sph);
  a.wrapm = wrap;
  const Dim3 org = dom.accessor_origin();
  const int rxm = int(dom.radius().x(-1));
  const bool aligned = (reinterpret_cast<uintptr_t>(a.src + rxm) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(a.dst + rxm) % 16 == 0) && ((a.px * int64_t(sizeof(T))) % 16 == 0);
  std::vector<Rect3> rs;
  for (const auto &r : regions)
    if (!r.empty()) rs.push_back(Rect3(r.lo - org, r.hi - org));
  STENCIL_REQUIRE(wrap == 0 || aligned, "in-kernel wrap of exterior slabs needs the aligned layout");
  if (aligned) {
    for (size_t k0 = 0; k0 < rs.size(); k0 += kMaxShell) {
      ShellTable st{};
      for (size_t k = k0; k < rs.size() && st.n < kMaxShell; ++k) {
        const Rect3 &r = rs[k];
        const Dim3 e = r.extent();
        const int i = st.n;
        st.lo[i][0] = int(r.lo.x);
        st.lo[i][1] = int(r.lo.y);
        st.lo[i][2] = int(r.lo.z);
        st.ext[i][0] = int(e.x);
        st.ext[i][1] = int(e.y);
        st.ext[i][2] = int(e.z);
        int64_t waves;
        if (e.x >= 8) {
          const int off = ((int(r.lo.x) - rxm) % V + V) % V;
          st.x0[i] = int(r.lo.x) - off;
          st.nch[i] = (int(r.hi.x) - st.x0[i] + V - 1) / V;
          st.col[i] = 0;
          waves = int64_t((st.nch[i] + 63) / 64) * e.y * e.z;
        } else {
          st.col[i] = 1;
          waves = int64_t(e.x) * ((e.y + 63) / 64) * e.z;
        }
        st.wbegin[i + 1] = st.wbegin[i] + waves;
        ++st.n;
      }
      const int64_t blocks = (st.wbegin[st.n] + 3) / 4;
      hipLaunchKernelGGL((stencil7_shell_kernel<T, KIND>), dim3(uint32_t(blocks)), dim3(64, 4), 0, stream, a, st);
      HIP_CHECK(hipGetLastError());
    }
    return;
  }
  for (size_t k0 = 0; k0 < rs.size(); k0 += kMaxRegions) {
    RegionTable rt{};
    rt.begin[0] = 0;
    for (size_t k = k0; k < rs.size() && rt.n < kMaxRegions; ++k) {
      const Rect3 &r = rs[k];
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
    if (rt.n == 0) continue;
    const int64_t total = rt.begin[rt.n];
    const int blocks = int(std::min<int64_t>((total + 255) / 256, 8192));
    hipLaunchKernelGGL((stencil7_regions_kernel<T, KIND>), dim3(blocks), dim3(256), 0, stream, a, rt);
    HIP_CHECK(hipGetLastError());
  }
}

void stencil7_apply_regions(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &regions, StencilKind kind,
                            const Spheres &sph, hipStream_t stream, const StencilTune &tune) {
  if (dom.backend() == Backend::Host) {
    STENCIL_REQUIRE(tune.wrap == 0 || dom.backend() == Backend::Device, "in-kernel wrap needs a device sub-domain");
    for (const auto &r : regions) stencil7_apply(dom, qi, r, kind, sph, stream, tune);
    return;
  }
  STENCIL_REQUIRE((tune.wrap & ~stencil7_wrappable_axes(dom, qi)) == 0,
                  "in-kernel wrap " << tune.wrap << " not supported by this layout");
  for (const auto &r : regions) {
    const Rect3 cr = dom.get_compute_region();
    STENCIL_REQUIRE(r.empty() || (cr.contains(r.lo) && r.hi.x <= cr.hi.x && r.hi.y <= cr.hi.y && r.hi.z <= cr.hi.z),
                    "stencil region " << r << " outside compute region " << cr);
  }
  dom.set_device();
  const bool f64 = dom.elem_size(qi) == 8;
  if (!f64)
    kind == StencilKind::Jacobi ? apply_regions_t<float, 0>(dom, qi, regions, sph, stream, tune.wrap)
                                : apply_regions_t<float, 1>(dom, qi, regions, sph, stream, tune.wrap);
  else
    kind == StencilKind::Jacobi ? apply_regions_t<double, 0>(dom, qi, regions, sph, stream, tune.wrap)
                                : apply_regions_t<double, 1>(dom, qi, regions, sph, stream, tune.wrap);
}

// ---------------------------------------------------------------------------------------------------------
// halo forwarder tables
// ---------------------------------------------------------------------------------------------------------
static bool fp_quantity(const LocalDomain &dom, int64_t qi, int64_t *es) {
  const DType dt = dom.dtype(qi);
  *es = dom.elem_size(qi);
  return dt == DType::F32 || dt == DType::F64 || (dt == DType::Bytes && (*es == 4 || *es == 8));
}

bool HaloForwarder::supported(const LocalDomain &dom, int64_t qi) {
  int64_t es = 0;
  if (dom.backend() != Backend::Device || !fp_quantity(dom, qi, &es)) return false;
  const Radius &r = dom.radius();
  const Dim3 sz = dom.size();
  // a cell must not belong to both the low and the high slab of an axis
  if (sz.x < r.x(1) + r.x(-1) || sz.y < r.y(1) + r.y(-1) || sz.z < r.z(1) + r.z(-1)) return false;
  // one 16-B chunk never holds cells of both x slabs
  if (sz.x < 2 * (16 / std::max<int64_t>(es, 1)) + r.x(1) + r.x(-1)) return false;
  // same layout checks as the vector kernel (apply_t)
  const int64_t V = 16 / es;
  const Dim3 p = dom.pitch(qi);
  const int64_t lox = r.x(-1), hix = lox + sz.x;
  const int64_t x0 = lox - ((lox - r.x(-1)) % V + V) % V;
  const int64_t nchunks = (hix - x0 + V - 1) / V;
  const bool aligned = (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.curr_data(qi)) + x0 * es) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(static_cast<const char *>(dom.next_data(qi)) + x0 * es) % 16 == 0) &&
                       (p.x * es) % 16 == 0;
  return aligned && x0 + nchunks * V < dom.row_limit(qi);
}

HaloForwarder::HaloForwarder(const LocalDomain &src, int64_t qi, const std::vector<ForwardTarget> &targets) {
  STENCIL_REQUIRE(supported(src, qi), "halo forwarding not supported for this sub-domain/quantity");
  dev_ = src.gpu();
  n_ = int(targets.size());
  const Radius &r = src.radius();
  // sending along +a feeds the receiver's -a halo (width = face radius on the -a side), and vice versa
  wp_[0] = int(r.x(-1));
  wp_[1] = int(r.y(-1));
  wp_[2] = int(r.z(-1));
  wm_[0] = int(r.x(1));
  wm_[1] = int(r.y(1));
  wm_[2] = int(r.z(1));
  const int64_t es = src.elem_size(qi);
  const int64_t V = 16 / es;
  const Dim3 sp = src.pitch(qi);
  src.set_device();
  for (int par = 0; par < 2; ++par) {
    // all sub-domains swap together: at sender parity `par` every receiver's next buffer is the one that is next
    // (par == current parity) or curr (otherwise) right now
    const bool now = src.parity() == par;
    const char *srcNext = static_cast<const char *>(now ? src.next_data(qi) : src.curr_data(qi));
    std::vector<CopySeg> rest;
    for (const auto &ft : targets) {
      const LocalDomain &d = *ft.dst;
      STENCIL_REQUIRE(d.elem_size(qi) == es, "forward target element size");
      const Dim3 dp = d.pitch(qi);
      const char *dstNext = static_cast<const char *>(d.parity() == par ? d.next_data(qi) : d.curr_data(qi));
      const int64_t byteGap = dstNext - srcNext;
      const int k = int((ft.dir.x + 1) + 3 * (ft.dir.y + 1) + 9 * (ft.dir.z + 1));
      // in-kernel when the receiver shares our pitches (so the offset is constant) and rows keep 16-B alignment
      const bool samePitch = dp.x == sp.x && dp.y == sp.y;
      const bool aligned = byteGap % es == 0 && (ft.dir.x != 0 || ((byteGap / es + ft.offset.x) % V == 0));
      if (samePitch && aligned) {
        mask_[par] |= 1u << k;
        delta_[par][k] = byteGap / es + ft.offset.z * sp.x * sp.y + ft.offset.y * sp.x + ft.offset.x;
      } else {
        build_translate_segs_q(src, d, ft.dir, !now, qi, rest);
      }
    }
    if (!rest.empty()) {
      finalize_segs(rest);
      rest_[par] = make_copy_plan(rest, dev_);
      hasRest_ = true;
    }
  }
}

HaloForwarder::~HaloForwarder() {
  for (auto &p : rest_)
    if (p.dsegs) {
      (void)hipSetDevice(dev_);
      free_copy_plan(p);
    }
}

void HaloForwarder::forward_rest(int parity, hipStream_t stream) const {
  if (rest_[parity].dsegs) copy_plan_device(rest_[parity], stream);
}

// ---------------------------------------------------------------------------------------------------------
// init kernels
// ---------------------------------------------------------------------------------------------------------
template <typename T>
__global__ void fill_region_kernel(T *raw, int64_t px, int64_t pxy, int lox, int loy, int loz, int nx, int ny, int nz,
                                   T v) {
  const int64_t total = int64_t(nx) * ny * nz;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int x = lox + int(i % nx), y = loy + int((i / nx) % ny), z = loz + int(i / (int64_t(nx) * ny));
    raw[int64_t(z) * pxy + int64_t(y) * px + x] = v;
  }
}

template <typename T>
__global__ void astaroth_init_kernel(T *raw, int64_t px, int64_t pxy, int rx, int ry, int rz, int nx, int ny, int nz,
                                     int ox, int oy, int oz, int rxl, int ryl, int rzl, int rxh, int ryh, int rzh,
                                     double period) {
  const int64_t total = int64_t(rx) * ry * rz;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int x = int(i % rx), y = int((i / rx) % ry), z = int(i / (int64_t(rx) * ry));
    T v;
    if (x >= rxl && y >= ryl && z >= rzl && x < rx - rxh && y < ry - ryh && z < rz - rzh) {
      v = T(sin(2 * 3.14159 / period * (ox + x) + 2 * 3.14159 / period * (oy + y) + 2 * 3.14159 / period * (oz + z)));
    } else {
      v = T(-10);
    }
    raw[int64_t(z) * pxy + int64_t(y) * px + x] = v;
    (void)nx;
    (void)ny;
    (void)nz;
  }
}

template <typename T> static void fill_t(const LocalDomain &dom, int64_t qi, const Rect3 &rawRegion, T v, bool curr, hipStream_t s) {
  T *raw = static_cast<T *>(curr ? dom.curr_data(qi) : dom.next_data(qi));
  const Dim3 p = dom.pitch(qi);
  const Dim3 e = rawRegion.extent();
  if (e.flatten() <= 0) return;
  if (dom.backend() == Backend::Host) {
    for (int64_t z = rawRegion.lo.z; z < rawRegion.hi.z; ++z)
      for (int64_t y = rawRegion.lo.y; y < rawRegion.hi.y; ++y)
        for (int64_t x = rawRegion.lo.x; x < rawRegion.hi.x; ++x) raw[z * p.x * p.y + y * p.x + x] = v;
    return;
  }
  dom.set_device();
  const int blocks = int(std::min<int64_t>((e.flatten() + 255) / 256, 8192));
  hipLaunchKernelGGL((fill_region_kernel<T>), dim3(blocks), dim3(256), 0, s, raw, p.x, p.x * p.y, int(rawRegion.lo.x),
                     int(rawRegion.lo.y), int(rawRegion.lo.z), int(e.x), int(e.y), int(e.z), v);
  HIP_CHECK(hipGetLastError());
}

void jacobi_init(const LocalDomain &dom, int64_t qi, const Rect3 &region, hipStream_t stream) {
  const Dim3 org = dom.accessor_origin();
  const Rect3 r(region.lo - org, region.hi - org);
  if (dom.elem_size(qi) == 8)
    fill_t<double>(dom, qi, r, 0.5, true, stream);
  else
    fill_t<float>(dom, qi, r, 0.5f, true, stream);
}

void fill_value(const LocalDomain &dom, int64_t qi, double value, bool curr, hipStream_t stream) {
  const Rect3 r(Dim3(0, 0, 0), dom.raw_size());
  if (dom.elem_size(qi) == 8)
    fill_t<double>(dom, qi, r, value, curr, stream);
  else
    fill_t<float>(dom, qi, r, float(value), curr, stream);
}

template <typename T> static void astaroth_init_t(const LocalDomain &dom, int64_t qi, double period, hipStream_t s) {
  T *raw = static_cast<T *>(dom.curr_data(qi));
  const Dim3 p = dom.pitch(qi), rs = dom.raw_size(), o = dom.origin();
  const Radius &R = dom.radius();
  if (dom.backend() == Backend::Host) {
    for (int64_t z = 0; z < rs.z; ++z)
      for (int64_t y = 0; y < rs.y; ++y)
        for (int64_t x = 0; x < rs.x; ++x) {
          T v;
          if (x >= R.x(-1) && y >= R.y(-1) && z >= R.z(-1) && x < rs.x - R.x(1) && y < rs.y - R.y(1) && z < rs.z - R.z(1))
            v = T(std::sin(2 * 3.14159 / period * double(o.x + x) + 2 * 3.14159 / period * double(o.y + y) +
                           2 * 3.14159 / period * double(o.z + z)));
          else
            v = T(-10);
          raw[z * p.x * p.y + y * p.x + x] = v;
        }
    return;
  }
  dom.set_device();
  const int blocks = int(std::min<int64_t>((rs.flatten() + 255) / 256, 8192));
  hipLaunchKernelGGL((astaroth_init_kernel<T>), dim3(blocks), dim3(256), 0, s, raw, p.x, p.x * p.y, int(rs.x), int(rs.y),
                     int(rs.z), 0, 0, 0, int(o.x), int(o.y), int(o.z), int(R.x(-1)), int(R.y(-1)), int(R.z(-1)),
                     int(R.x(1)), int(R.y(1)), int(R.z(1)), period);
  HIP_CHECK(hipGetLastError());
}

void astaroth_init(const LocalDomain &dom, int64_t qi, double period, hipStream_t stream) {
  if (dom.elem_size(qi) == 8)
    astaroth_init_t<double>(dom, qi, period, stream);
  else
    astaroth_init_t<float>(dom, qi, period, stream);
}

} // namespace stencil
