// Lab for the fused-pair sweep (one 512^3 fp32 Jacobi pair per launch, the bench.py layout, in-kernel x/y/z wrap).
// Kernels come from gen.py: lab_col = stencil7x2_kernel, lab_row = stencil7x2_row_kernel, each with ablation bits
// (ABL: 1 no output stores, 2 no lookahead loads). Prints us per launch and checks that both write the same bits.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "stencil_common.hpp"
#include "stencil_wave.hpp"
namespace stencil {
#include "x2lab_kernel.inc"
}
using namespace stencil;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
template <int ABL, int VAR> void launch(StencilArgs<float> a, int nb) {
  if (VAR == 2) { a.gx = 1; hipLaunchKernelGGL((lab_rownt<12, 3, 0, ABL>), dim3(nb), dim3(64, 12), 0, 0, a); }
  else if (VAR) { a.gx = 1; hipLaunchKernelGGL((lab_row<12, 3, 0, ABL>), dim3(nb), dim3(64, 12), 0, 0, a); }
  else hipLaunchKernelGGL((lab_col<float, 12, 3, 0, 2, ABL>), dim3(nb), dim3(64, 12), 0, 0, a);
}
template <int ABL, int VAR> float run(StencilArgs<float> a, float *b0, float *b1, int nb, int iters) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3 + iters; ++i) {
    if (i == 3) CK(hipEventRecord(e0));
    a.src = (i & 1) ? b1 : b0; a.dst = (i & 1) ? b0 : b1; a.flip = i & 1;
    launch<ABL, VAR>(a, nb);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}
int main() {
  const int n = 512, px = 528, py = n + 4, pz = n + 4;
  const size_t cnt = size_t(px) * py * pz + 64;
  float *m0, *m1, *m2; CK(hipMalloc(&m0, cnt * 4)); CK(hipMalloc(&m1, cnt * 4)); CK(hipMalloc(&m2, cnt * 4));
  std::vector<float> h(cnt);
  for (size_t i = 0; i < cnt; ++i) h[i] = float((i * 2654435761u) % 1000003) / 1000003.f;
  CK(hipMemcpy(m0, h.data(), cnt * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(m1, h.data(), cnt * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(m2, h.data(), cnt * 4, hipMemcpyHostToDevice));
  float *b0 = m0 + 14, *b1 = m1 + 14, *b2 = m2 + 14; // raw x = 2 on a 64-B boundary
  StencilArgs<float> a{};
  a.px = px; a.pxy = int64_t(px) * py;
  a.lox = 2; a.hix = 2 + n; a.loy = 2; a.hiy = 2 + n; a.loz = 2; a.hiz = 2 + n;
  a.x0 = 2; a.nchunks = n / 4; a.rawYm1 = py - 1; a.rawZm1 = pz - 1;
  a.gx = (a.nchunks + 63) / 64; a.gy = (n + 7) / 8; a.gz = 1; a.zc = 1; a.seg = 1; a.remap = 1; a.nt = 1;
  a.hx = 2 + n / 3; a.hy = 2 + n / 2; a.hz = 2 + n / 2; a.cx = 2 + 2 * n / 3; a.cy = a.hy; a.cz = a.hz; a.r1sq = (n / 10 + 1) * (n / 10 + 1);
  a.wrapm = 7; for (int d = 0; d < 3; ++d) { a.wlo[d] = 2; a.wn[d] = n; }
  int per = 0; CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)lab_col<float, 12, 3, 0, 2, 0>, 768, 0));
  const int nb = 256 * per;
  // bitwise check: one launch of each from the same source
  { StencilArgs<float> c = a; c.src = b0; c.dst = b1; launch<0, 0>(c, nb); c.dst = b2; launch<0, 1>(c, nb); CK(hipDeviceSynchronize());
    std::vector<float> o1(cnt), o2(cnt); CK(hipMemcpy(o1.data(), m1, cnt * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(o2.data(), m2, cnt * 4, hipMemcpyDeviceToHost));
    printf("row kernel bitwise equal to column kernel: %s\n", memcmp(o1.data(), o2.data(), cnt * 4) == 0 ? "yes" : "NO"); }
  printf("blocks %d\n", nb);
  const int it = 20;
  { StencilArgs<float> c = a; c.src = b0; c.dst = b1; launch<0, 1>(c, nb); c.dst = b2; launch<0, 2>(c, nb); CK(hipDeviceSynchronize());
    std::vector<float> o1(cnt), o2(cnt); CK(hipMemcpy(o1.data(), m1, cnt * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(o2.data(), m2, cnt * 4, hipMemcpyDeviceToHost));
    printf("nt-load row kernel bitwise equal: %s\n", memcmp(o1.data(), o2.data(), cnt * 4) == 0 ? "yes" : "NO"); }
  for (int rep = 0; rep < 4; ++rep) {
    printf("row        %7.1f us\n", run<0, 1>(a, b0, b1, nb, it));
    printf("row ntload %7.1f us\n", run<0, 2>(a, b0, b1, nb, it));
  }
  return 0;
}
