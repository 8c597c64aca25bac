#pragma once
// Shared helpers for the C++ apps (method-flag CLI, wall clock, weak-scaling rule).
#include <chrono>
#include <cmath>
#include <string>

#include "stencil/domain/distributed_domain.hpp"
#include "stencil/rt/argparse.hpp"

namespace app {
using namespace stencil;

struct MethodArgs {
  bool staged = false, rccl = false, colo = false, peer = false, kernel = false, trivial = false;
  int interiorAlign = 128; // bytes; the row-start alignment of every interior (LocalDomain::set_interior_align)
  bool sharedHaloLine = false; // LocalDomain::set_shared_halo_line
  bool xFaceLines = false; // TransportOptions::xFaceSectors: same-GPU x faces copied as whole lines
  int xFaceLinesAutoMiB = 128; // TransportOptions::xFaceLinesAutoBytes in MiB (0 = never by themselves)
  void add(ArgParser &p) {
    p.flag(&staged, "--staged,--remote", "host-staged transport (reference CudaMpi)")
        .flag(&rccl, "--rccl,--cuda-aware,--cuda-aware-mpi", "RCCL transport (reference CudaAwareMpi)")
        .flag(&colo, "--colo,--colocated", "HIP-IPC colocated transport")
        .flag(&peer, "--peer", "same-process peer (xGMI) transport")
        .flag(&kernel, "--kernel", "same-GPU kernel transport")
        .flag(&trivial, "--trivial,--naive", "trivial placement")
        .option(&interiorAlign, "--interior-align", "interior row alignment in bytes (64 or 128)")
        .flag(&sharedHaloLine, "--shared-halo-line", "row r's +x and row r+1's -x halo in one 128-B line")
        .flag(&xFaceLines, "--x-face-lines", "same-GPU x faces copied as whole 128-B lines")
        .option(&xFaceLinesAutoMiB, "--x-face-lines-auto", "MiB of x-face lines from which whole lines switch on (0 never)");
  }
  MethodFlags flags() const {
    MethodFlags m = MethodFlags::None;
    if (staged) m |= MethodFlags::Staged;
    if (rccl) m |= MethodFlags::Rccl;
    if (colo) m |= MethodFlags::Colocated;
    if (peer) m |= MethodFlags::PeerCopy;
    if (kernel) m |= MethodFlags::Kernel;
    return any(m) ? m : MethodFlags::All;
  }
  // the transport options these flags set, on top of `o`
  TransportOptions transport(TransportOptions o = {}) const {
    o.xFaceSectors = xFaceLines;
    o.xFaceLinesAutoBytes = int64_t(xFaceLinesAutoMiB) << 20;
    return o;
  }
  PlacementStrategy placement() const { return trivial ? PlacementStrategy::Trivial : PlacementStrategy::NodeAware; }
};

inline double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// reference weak-scaling rule (bin/weak.cu:63-65): size * n^0.33333, rounded
inline int64_t weak_scale(int64_t v, int n) { return int64_t(double(v) * std::pow(double(n), 0.33333) + 0.5); }
} // namespace app
