// Point-to-point ping-pong between rank pairs. Parity: reference bin/pingpong.cu (2^min..2^max bytes split over
// concurrent pairs; host-memory MPI). Here: --host uses the native TCP process group (host memory); default uses
// RCCL ncclSend/ncclRecv on device buffers over xGMI between rank r and r + size/2.
#include <chrono>
#include <cstdio>
#include <vector>

#include "stencil/comm/proc_group.hpp"
#include "stencil/comm/rccl_comm.hpp"
#include "stencil/rt/argparse.hpp"
#include "stencil/rt/hip_check.hpp"
#include "stencil/topo/gpu_topology.hpp"

using namespace stencil;

int main(int argc, char **argv) {
  int minP = 10, maxP = 26, iters = 20;
  bool host = false;
  ArgParser p("ping-pong (reference bin/pingpong.cu)");
  p.option(&minP, "--min", "log2 min bytes").option(&maxP, "--max", "log2 max bytes").option(&iters, "--iters", "iters")
      .flag(&host, "--host", "host memory over the TCP process group");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  auto pg = comm::default_group();
  const int n = pg->size(), r = pg->rank();
  if (n < 2 || n % 2) {
    if (r == 0) std::fprintf(stderr, "pingpong needs an even number of ranks\n");
    return 1;
  }
  const int half = n / 2;
  const int peer = r < half ? r + half : r - half;
  const bool leader = r < half;
  rccl::Comm nc = nullptr;
  hipStream_t s = nullptr;
  auto check = [&](const std::string &e) {
    if (!e.empty()) LOG_FATAL("rank " << r << ": " << e);
  };
  if (!host) {
    const int dev = pg->colocated_rank() % std::max(1, gpu_topo::device_count());
    HIP_CHECK(hipSetDevice(dev));
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    rccl::UniqueId id{};
    struct {
      int ok;
      rccl::UniqueId id;
    } boot{1, {}};
    std::string e;
    if (r == 0) {
      e = rccl::get_unique_id(&boot.id);
      boot.ok = e.empty();
    }
    pg->bcast(&boot, sizeof(boot), 0);
    if (!boot.ok) LOG_FATAL("RCCL unique id on rank 0 failed" << (e.empty() ? "" : ": " + e));
    id = boot.id;
    std::vector<rccl::Comm> comms;
    check(rccl::init_ranks(&comms, n, id, {r}, {dev}));
    nc = comms[0];
  }
  if (r == 0) std::printf("mode,bytes,pairs,one_way_s,GBps_per_pair\n");
  for (int lp = minP; lp <= maxP; ++lp) {
    const size_t bytes = size_t(1) << lp;
    std::vector<char> hbuf(bytes);
    char *dbuf = nullptr;
    if (!host) HIP_CHECK(hipMalloc(&dbuf, bytes));
    auto once = [&] {
      if (host) {
        if (leader) {
          pg->send(peer, 7, hbuf.data(), bytes);
          pg->recv(peer, 7, hbuf.data(), bytes);
        } else {
          pg->recv(peer, 7, hbuf.data(), bytes);
          pg->send(peer, 7, hbuf.data(), bytes);
        }
      } else {
        if (leader) {
          check(rccl::send(dbuf, bytes, peer, nc, s));
          check(rccl::recv(dbuf, bytes, peer, nc, s));
        } else {
          check(rccl::recv(dbuf, bytes, peer, nc, s));
          check(rccl::send(dbuf, bytes, peer, nc, s));
        }
        HIP_CHECK(hipStreamSynchronize(s));
      }
    };
    once();
    pg->barrier();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) once();
    const double el = pg->allreduce_max(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    const double oneWay = el / iters / 2;
    if (r == 0) std::printf("%s,%zu,%d,%e,%.3f\n", host ? "tcp-host" : "rccl-device", bytes, half, oneWay, bytes / oneWay / 1e9);
    if (dbuf) HIP_CHECK(hipFree(dbuf));
  }
  rccl::destroy(nc);
  return 0;
}
