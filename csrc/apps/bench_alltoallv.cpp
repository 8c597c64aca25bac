// Peer-to-peer copy matrices between the GPUs of one process. Parity: reference bin/bench_alltoallv.cu (times
// cudaMemcpyPeerAsync for a stencil comm matrix, all-to-all 8 MiB / 1 GiB, local 1 GiB, local + remote) — here for
// every visible GPU (8 x MI355X over xGMI): hipMemcpyPeerAsync on one stream per (src, dst) pair, all in flight.
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "stencil/rt/argparse.hpp"
#include "stencil/rt/hip_check.hpp"
#include "stencil/topo/gpu_topology.hpp"
#include "stencil/topo/mat2d.hpp"

using namespace stencil;

static double run(const Mat2D<size_t> &bytes, int iters) {
  const int n = int(bytes.rows());
  std::vector<std::vector<char *>> src(n, std::vector<char *>(n, nullptr)), dst(n, std::vector<char *>(n, nullptr));
  std::vector<std::vector<hipStream_t>> st(n, std::vector<hipStream_t>(n, nullptr));
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (!bytes.at(i, j)) continue;
      HIP_CHECK(hipSetDevice(i));
      HIP_CHECK(hipMalloc(&src[i][j], bytes.at(i, j)));
      HIP_CHECK(hipStreamCreateWithFlags(&st[i][j], hipStreamNonBlocking));
      HIP_CHECK(hipSetDevice(j));
      HIP_CHECK(hipMalloc(&dst[i][j], bytes.at(i, j)));
      gpu_topo::enable_peer(i, j);
    }
  auto once = [&] {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (bytes.at(i, j)) {
          HIP_CHECK(hipSetDevice(i));
          HIP_CHECK(hipMemcpyPeerAsync(dst[i][j], j, src[i][j], i, bytes.at(i, j), st[i][j]));
        }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (st[i][j]) HIP_CHECK(hipStreamSynchronize(st[i][j]));
  };
  once();
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < iters; ++k) once();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (src[i][j]) (void)hipFree(src[i][j]);
      if (dst[i][j]) (void)hipFree(dst[i][j]);
      if (st[i][j]) (void)hipStreamDestroy(st[i][j]);
    }
  return el;
}

int main(int argc, char **argv) {
  int iters = 10;
  ArgParser p("peer copy matrices (reference bin/bench_alltoallv.cu)");
  p.option(&iters, "--iters", "iterations");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  const int n = gpu_topo::device_count();
  if (n == 0) {
    std::fprintf(stderr, "no GPU\n");
    return 1;
  }
  std::printf("name,gpus,total_bytes,seconds,GBps\n");
  auto report = [&](const std::string &name, const Mat2D<size_t> &m) {
    size_t tot = 0;
    for (size_t i = 0; i < m.rows(); ++i)
      for (size_t j = 0; j < m.cols(); ++j) tot += m.at(i, j);
    const double t = run(m, iters);
    std::printf("%s,%d,%zu,%e,%.2f\n", name.c_str(), n, tot, t, tot / t / 1e9);
  };
  const size_t MiB = 1 << 20;
  // 2x2x2 stencil of 512^3 fp32 radius 3: face partners 48 MiB, edges 576 KiB, corner 6912 B
  Mat2D<size_t> stencilM(n, n, 0), a2a8(n, n, 0), a2a1g(n, n, 0), local(n, n, 0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      const int d = __builtin_popcount(unsigned(i ^ j));
      if (i != j) stencilM.at(i, j) = d == 1 ? 48 * MiB : (d == 2 ? 576 * 1024 : 6912);
      if (i != j) a2a8.at(i, j) = 8 * MiB;
      if (i != j) a2a1g.at(i, j) = 128 * MiB;
      if (i == j) local.at(i, j) = 1024 * MiB;
    }
  report("stencil-2x2x2-r3-8q", stencilM);
  report("alltoall-8MiB", a2a8);
  report("alltoall-128MiB", a2a1g);
  report("local-1GiB", local);
  return 0;
}
