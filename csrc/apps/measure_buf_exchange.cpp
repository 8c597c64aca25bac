// Calibrate per-pair peer-copy sizes so every transfer takes the same time. Parity: reference
// bin/measure_buf_exchange.cu (4x4 matrix, gradient step gamma=0.2 toward a 4 ms target, clock_block latch so all
// copies start together) — here every visible GPU pair, with a device-side latch kernel spinning on s_memrealtime.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "stencil/rt/argparse.hpp"
#include "stencil/rt/hip_check.hpp"
#include "stencil/topo/gpu_topology.hpp"

using namespace stencil;

__global__ void clock_block(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

int main(int argc, char **argv) {
  double targetMs = 4.0, gamma = 0.2;
  int rounds = 10;
  ArgParser p("peer buffer-size calibration (reference bin/measure_buf_exchange.cu)");
  p.option(&targetMs, "--target-ms", "target ms per copy").option(&gamma, "--gamma", "step").option(&rounds, "--rounds", "rounds");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  const int n = gpu_topo::device_count();
  if (n == 0) return 1;
  std::vector<std::vector<double>> sz(n, std::vector<double>(n, 64.0 * (1 << 20)));
  for (int r = 0; r < rounds; ++r) {
    std::vector<std::vector<double>> ms(n, std::vector<double>(n, 0));
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        if (i != j) gpu_topo::enable_peer(i, j);
        const size_t b = size_t(sz[i][j]);
        char *s = nullptr, *d = nullptr;
        HIP_CHECK(hipSetDevice(i));
        HIP_CHECK(hipMalloc(&s, b));
        HIP_CHECK(hipSetDevice(j));
        HIP_CHECK(hipMalloc(&d, b));
        HIP_CHECK(hipSetDevice(i));
        hipStream_t st;
        HIP_CHECK(hipStreamCreate(&st));
        hipEvent_t a, e;
        HIP_CHECK(hipEventCreate(&a));
        HIP_CHECK(hipEventCreate(&e));
        hipLaunchKernelGGL(clock_block, dim3(1), dim3(1), 0, st, uint64_t(100000)); // 1 ms latch
        HIP_CHECK(hipEventRecord(a, st));
        HIP_CHECK(hipMemcpyPeerAsync(d, j, s, i, b, st));
        HIP_CHECK(hipEventRecord(e, st));
        HIP_CHECK(hipEventSynchronize(e));
        float t = 0;
        HIP_CHECK(hipEventElapsedTime(&t, a, e));
        ms[i][j] = t;
        HIP_CHECK(hipFree(s));
        HIP_CHECK(hipFree(d));
        HIP_CHECK(hipStreamDestroy(st));
      }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) sz[i][j] *= 1.0 + gamma * (targetMs - ms[i][j]) / targetMs;
    std::printf("round %d:", r);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) std::printf(" %d>%d %.2fms/%.1fMiB", i, j, ms[i][j], sz[i][j] / (1 << 20));
    std::printf("\n");
  }
  return 0;
}
