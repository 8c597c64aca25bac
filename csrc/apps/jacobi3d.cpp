// Jacobi3D weak-scaling app. Parity: reference bin/jacobi3d.cu (flags --staged --colo --peer --kernel --trivial
// --no-overlap --paraview --prefix -n/--iters -q/--period, positionals x y z per GPU, weak scaling by
// numSubdomains^0.33333, CSV `jacobi3d,<methods>,<ranks>,<devCount>,x,y,z,<min s>,<trimean s>`).
// Additions: --rccl, --fp64, --warmup, Gcells/s column.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <iostream>

#include "stencil/models/stencil_model.hpp"
#include "stencil/rt/argparse.hpp"
#include "stencil/rt/statistics.hpp"
#include "stencil/topo/gpu_topology.hpp"

using namespace stencil;

int main(int argc, char **argv) {
  bool staged = false, rccl = false, colo = false, peer = false, kernel = false, trivial = false, noOverlap = false,
       paraview = false, fp64 = false, noWrap = false;
  std::string prefix;
  int iters = 30, period = -1, warmup = 3, temporal = 1;
  int64_t x = 512, y = 512, z = 512;
  ArgParser p("Jacobi3D with hot/cold spheres on a periodic domain (per-GPU size, weak scaled)");
  p.flag(&staged, "--staged", "enable host-staged transport")
      .flag(&rccl, "--rccl", "enable RCCL transport")
      .flag(&colo, "--colo", "enable colocated HIP-IPC transport")
      .flag(&peer, "--peer", "enable same-process peer (xGMI) transport")
      .flag(&kernel, "--kernel", "enable same-GPU kernel transport")
      .flag(&trivial, "--trivial,--naive", "trivial placement")
      .flag(&noOverlap, "--no-overlap", "do not overlap interior compute with the exchange")
      .flag(&paraview, "--paraview", "dump ParaView CSV files")
      .flag(&fp64, "--fp64", "double precision")
      .flag(&noWrap, "--no-wrap", "copy every periodic self-halo instead of reading the periodic image in-kernel")
      .option(&prefix, "--prefix", "ParaView file prefix")
      .option(&iters, "-n,--iters", "iterations")
      .option(&warmup, "--warmup", "untimed warmup iterations")
      .option(&period, "-q,--period", "ParaView dump period")
      .option(&temporal, "--temporal", "steps fused per sweep (2: fused pairs, one depth-2 exchange per pair; 3: fused triples, one depth-3 exchange per three steps)")
      .positional(&x, "x", "per-GPU x")
      .positional(&y, "y", "per-GPU y")
      .positional(&z, "z", "per-GPU z");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;

  auto pg = comm::default_group();
  const int devCount = gpu_topo::device_count();
  const int perRank = devCount > 0 ? std::max(1, devCount / pg->colocated_size()) : 1;
  const int numSubdoms = pg->size() * perRank;
  const double scale = std::pow(double(numSubdoms), 0.33333);
  x = int64_t(double(x) * scale + 0.5);
  y = int64_t(double(y) * scale + 0.5);
  z = int64_t(double(z) * scale + 0.5);

  StencilModelConfig cfg;
  cfg.size = Dim3(x, y, z);
  cfg.kind = StencilKind::Jacobi;
  cfg.radius = 1;
  cfg.fp64 = fp64;
  cfg.temporal = temporal;
  cfg.wrapSelf = !noWrap;
  MethodFlags m = MethodFlags::None;
  if (staged) m |= MethodFlags::Staged;
  if (rccl) m |= MethodFlags::Rccl;
  if (colo) m |= MethodFlags::Colocated;
  if (peer) m |= MethodFlags::PeerCopy;
  if (kernel) m |= MethodFlags::Kernel;
  cfg.methods = any(m) ? m : MethodFlags::All;
  cfg.placement = trivial ? PlacementStrategy::Trivial : PlacementStrategy::NodeAware;
  cfg.overlap = !noOverlap;
  if (period <= 0) period = std::max(1, iters / 10);

  Statistics st;
  {
    StencilModel model(cfg, pg);
    model.init();
    if (paraview) model.domain().write_paraview(prefix + "jacobi3d_init");
    // one timed unit = one sweep: a step, a fused pair or a fused triple (time reported per step)
    const int per = model.steps_per_sweep();
    if (pg->rank() == 0)
      std::fprintf(stderr, "# jacobi3d: %d step(s) per sweep, in-kernel wrap axes %d, overlap %d\n", per,
                   model.wrap_axes(), int(model.overlapping()));
    for (int i = 0; i < warmup; ++i) model.run(per);
    model.synchronize();
    for (int i = 0; i < iters; ++i) {
      pg->barrier();
      auto t0 = std::chrono::steady_clock::now();
      model.run(per);
      model.synchronize();
      double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / per;
      st.insert(pg->allreduce_max(el));
      if (paraview && i % period == 0) model.domain().write_paraview(prefix + "jacobi3d_" + std::to_string(i));
    }
    if (paraview) model.domain().write_paraview(prefix + "jacobi3d_final");
  }
  if (pg->rank() == 0) {
    std::printf("jacobi3d,%s,%d,%d,%ld,%ld,%ld,%e,%e,%.2f\n", to_string(cfg.methods).c_str(), pg->size(), devCount,
                long(x), long(y), long(z), st.min(), st.trimean(), double(x * y * z) / st.trimean() / 1e9);
  }
  return 0;
}
