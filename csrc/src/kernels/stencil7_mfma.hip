// MFMA variant of the 7-point Jacobi step ("an MFMA line-update variant, judged by rocprof
// counters against the VALU variant"). Reference kernel: bin/jacobi3d.cu:40-87.
//
// The x-line update vpx + vmx of a 16 (y) x 16 (x) tile is a product with a banded 0/1 matrix on the matrix cores:
//     Sx[y][n] = sum_k X[y][k] * T[k][n],   T[k][n] = (k == n) || (k == n + 2),   k = x window x0-1 .. x0+18
// with v_mfma_f32_16x16x4_f32 (exact fp32 in/out, 5 K-steps of 4). Every product is exact (x1 or x0) and each output
// has exactly two non-zero terms, so the accumulation order inside the matrix core cannot matter: Sx is the single
// rounding of vpx + vmx, i.e. bitwise the reference's (0 + vpx) + vmx (signed zeros included). The remaining
// +vpy +vmy +vpz +vmz, the exact /6 and the hot/cold spheres run on the VALU in the reference order, so the output is
// bitwise equal to the VALU kernels (tests compare both with the torch oracle).
//
// Honest accounting: the band matrix is 2/16 dense, so a 16x16x4 MFMA (1024 FMAs) delivers 64 useful adds; the VALU
// kernels do the same work with one packed add per two cells. The variant exists to measure that with counters
// (profiles/), not because it is faster: the 7-point stencil is bound by HBM and VALU issue, not by FLOPs. It also
// requires finite inputs (0 x Inf = NaN inside the band product would spread along the 16-wide line).
//
// Layout: block = 4 waves = a 64 (x) x 16 (y) output tile marching in z. A ring of 4 LDS planes (x0-1 .. x0+64 by
// y0-1 .. y0+16) holds z-1, z, z+1 and the plane being loaded; one barrier per plane.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "stencil/rt/hip_check.hpp"
#include "stencil_common.hpp"

namespace stencil {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kTX = 64, kTY = 16;        // output tile per block
constexpr int kLX = kTX + 4;             // LDS row: x0-1 .. x0+64 plus 2 zero columns for the last K-step
constexpr int kLY = kTY + 2;             // rows y0-1 .. y0+16
constexpr int kLoad = kLY * (kTX + 2);   // cells loaded per plane (1188)
constexpr int kPer = (kLoad + 255) / 256; // per thread (5)
constexpr int kRing = 4;
} // namespace

__global__ __launch_bounds__(256) void stencil7_mfma_kernel(StencilArgs<float> a) {
  __shared__ float tile[kRing][kLY][kLX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nb = uint32_t(a.gx) * a.gy * a.gz;
  const uint32_t lb = xcd_remap(blockIdx.x, nb);
  const int bz = int(lb % uint32_t(a.gz));
  const int by = int((lb / uint32_t(a.gz)) % uint32_t(a.gy));
  const int bx = int(lb / (uint32_t(a.gz) * a.gy));
  const int x0 = a.lox + bx * kTX, y0 = a.loy + by * kTY;
  const int zs = a.loz + bz * a.zc, ze = min(zs + a.zc, a.hiz);
  if (zs >= ze) return; // block-uniform

  // zero the two padding columns of every ring slot once (the last K-step reads them with a zero band weight)
  for (int i = tid; i < kRing * kLY * 2; i += 256) {
    const int s = i / (kLY * 2), r = (i / 2) % kLY, c = kTX + 2 + (i & 1);
    tile[s][r][c] = 0.0f;
  }
  // cooperative plane loads: cell i of the plane tile = (row i / 66, col i % 66); clamped to the region's far
  // edges (cells past them only feed outputs that are never stored)
  auto load_plane = [&](int zz, float (&v)[kPer]) {
    const float *pl = a.src + int64_t(zz) * a.pxy;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int idx = tid + 256 * i;
      if (idx < kLoad) {
        const int r = idx / (kTX + 2), c = idx - r * (kTX + 2);
        const int gx = min(x0 - 1 + c, a.hix), gy = min(y0 - 1 + r, a.hiy);
        v[i] = pl[int64_t(gy) * a.px + gx];
      }
    }
  };
  auto store_plane = [&](int slot, const float (&v)[kPer]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int idx = tid + 256 * i;
      if (idx < kLoad) {
        const int r = idx / (kTX + 2), c = idx - r * (kTX + 2);
        tile[slot][r][c] = v[i];
      }
    }
  };
  auto slot_of = [&](int zz) { return (zz - zs + 1) & (kRing - 1); };

  // band weights of this lane's B operand: B[k = 4s + lane/16][n = lane%16]
  float band[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int k = 4 * s + (lane >> 4), n = lane & 15;
    band[s] = (k == n || k == n + 2) ? 1.0f : 0.0f;
  }
  // this lane's outputs (D layout of 16x16x4): rows 4*(lane/16) + r, column lane%16 of the wave's 16x16 subtile
  const int col = 16 * w + (lane & 15) + 1; // LDS column of the output x
  const int ox = x0 + 16 * w + (lane & 15);
  const int oy0 = y0 + 4 * (lane >> 4);

  {
    float v[kPer];
    for (int zz = zs - 1; zz <= zs + 1 && zz <= ze; ++zz) {
      load_plane(zz, v);
      store_plane(slot_of(zz), v);
    }
  }
  __syncthreads();

  for (int z = zs; z < ze; ++z) {
    float pf[kPer];
    const bool more = z + 2 <= ze;
    if (more) load_plane(z + 2, pf); // lands while this plane computes
    const int sm = slot_of(z - 1), s0 = slot_of(z), sp = slot_of(z + 1);
    // x pair on the matrix cores: A[y = lane%16][k = 4s + lane/16] = plane z at (y0 + y, x0 + 16w - 1 + k)
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const float av = tile[s0][1 + (lane & 15)][16 * w + 4 * s + (lane >> 4)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, band[s], acc, 0, 0, 0);
    }
    // y and z neighbours, the exact /6 and the spheres on the VALU (reference order +y, -y, +z, -z)
    const int64_t zoff = int64_t(z) * a.pxy;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int yl = 4 * (lane >> 4) + r; // tile row of the output (LDS row yl + 1)
      float val = acc[r];
      val += tile[s0][yl + 2][col];
      val += tile[s0][yl][col];
      val += tile[sp][yl + 1][col];
      val += tile[sm][yl + 1][col];
      const int oy = oy0 + r;
      val = sphere_fix(a, ox, oy, z, div6<float>(val));
      if (ox < a.hix && oy < a.hiy) a.dst[zoff + int64_t(oy) * a.px + ox] = val;
    }
    if (more) store_plane(slot_of(z + 2), pf); // slot of z-2: last read in the previous step, before the barrier
    __syncthreads();
  }
}

bool stencil7_mfma_supported(const LocalDomain &dom, int64_t qi) {
  if (dom.backend() != Backend::Device) return false;
  const DType dt = dom.dtype(qi);
  return dt == DType::F32 || (dt == DType::Bytes && dom.elem_size(qi) == 4);
}

void stencil7_mfma_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                         hipStream_t stream, const StencilTune &tune) {
  if (region.empty()) return;
  STENCIL_REQUIRE(kind == StencilKind::Jacobi,
                  "the MFMA variant computes the Jacobi order (+x first); Astaroth sums -x, -y first");
  STENCIL_REQUIRE(stencil7_mfma_supported(dom, qi), "the MFMA variant needs a device fp32 quantity");
  StencilArgs<float> a = make_args<float>(dom, qi, region, kind, sph);
  const int nx = a.hix - a.lox, ny = a.hiy - a.loy, nz = a.hiz - a.loz;
  a.gx = (nx + kTX - 1) / kTX;
  a.gy = (ny + kTY - 1) / kTY;
  a.zc = tune.zchunk > 0 ? tune.zchunk : std::max(8, std::min(nz, 32));
  a.gz = (nz + a.zc - 1) / a.zc;
  const uint32_t blocks = uint32_t(a.gx) * a.gy * a.gz;
  dom.set_device();
  hipLaunchKernelGGL(stencil7_mfma_kernel, dim3(blocks), dim3(256), 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

} // namespace stencil
