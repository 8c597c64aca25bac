// Pack/unpack micro-benchmark. Parity: reference bin/bench_pack.cu (LocalDomain 512^3, radius 3, one float,
// 30 x pack() and 30 x unpack() timed with events for +x, +y, +z; prints `ext dir bytes packTime unpackTime`).
#include <chrono>
#include <cstdio>

#include "stencil/domain/packer.hpp"
#include "stencil/rt/argparse.hpp"
#include "stencil/rt/stream.hpp"
#include "stencil/topo/gpu_topology.hpp"

using namespace stencil;

int main(int argc, char **argv) {
  int64_t n = 512;
  int radius = 3, iters = 30, nq = 1;
  ArgParser p("pack/unpack benchmark (reference bin/bench_pack.cu)");
  p.option(&n, "--n", "cube edge").option(&radius, "--radius", "radius").option(&iters, "--iters", "iterations")
      .option(&nq, "--q", "quantities");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  const bool dev = gpu_topo::device_count() > 0;
  LocalDomain ld(Dim3(n, n, n), Dim3(0, 0, 0), dev ? 0 : -1, dev ? Backend::Device : Backend::Host);
  ld.set_radius(radius);
  for (int q = 0; q < nq; ++q) ld.add_data<float>();
  ld.realize();
  Stream s;
  if (dev) s = Stream(0);
  std::printf("ext,dir,bytes,pack_s,unpack_s,pack_GBps,unpack_GBps\n");
  const Dim3 dirs[] = {Dim3(1, 0, 0), Dim3(0, 1, 0), Dim3(0, 0, 1), Dim3(1, 1, 0), Dim3(1, 1, 1)};
  for (const Dim3 &d : dirs) {
    Packer pk(s);
    Unpacker up(s);
    pk.prepare(&ld, {Message{d, 0, 0}});
    up.prepare(&ld, {Message{d, 0, 0}});
    auto timeit = [&](auto &&fn) {
      fn();
      if (dev) {
        Event a(0, true), b(0, true);
        a.record(s);
        for (int i = 0; i < iters; ++i) fn();
        b.record(s);
        b.sync();
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, a, b));
        return double(ms) / 1e3 / iters;
      }
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) fn();
      return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
    };
    const double tp = timeit([&] { pk.pack(); });
    const double tu = timeit([&] { up.unpack(); });
    std::printf("%ld,[%ld;%ld;%ld],%ld,%e,%e,%.2f,%.2f\n", long(n), long(d.x), long(d.y), long(d.z), long(pk.size()), tp,
                tu, pk.size() / tp / 1e9, up.size() / tu / 1e9);
  }
  return 0;
}
