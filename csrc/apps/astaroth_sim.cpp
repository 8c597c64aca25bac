// Astaroth-like proxy: radius 3 in all 26 directions, several fp32 quantities, 6-neighbour mean.
// Parity: reference bin/astaroth_sim.cu (flags --remote --cuda-aware-mpi --colocated --peer --kernel --trivial
// --x --y --z; sin-wave init, halo -10; interior overlapped with the exchange; 5 iterations). The reference keeps
// one quantity (three commented out); --q defaults to 8 here (BASELINE.json config).
#include <cstdio>

#include "app_common.hpp"
#include "stencil/models/stencil_model.hpp"
#include "stencil/rt/statistics.hpp"

using namespace stencil;

int main(int argc, char **argv) {
  int64_t x = 512, y = 512, z = 512;
  int iters = 5, nq = 8, temporal = 1;
  bool noOverlap = false, weak = false, fp64 = false, noWrap = false, forceOverlap = false;
  int reserve = -1;
  app::MethodArgs ma;
  ArgParser p("Astaroth proxy (reference bin/astaroth_sim.cu)");
  p.option(&x, "--x", "x").option(&y, "--y", "y").option(&z, "--z", "z").option(&iters, "-n,--iters", "iterations")
      .option(&nq, "--q", "quantities")
      .option(&temporal, "--temporal", "steps fused per sweep (1, 2, or 3: fused triples, one depth-3 exchange per three steps)")
      .flag(&noOverlap, "--no-overlap", "no overlap")
      .flag(&forceOverlap, "--overlap", "overlap the interior sweep with the exchange even when every halo is a "
                                        "same-GPU copy (one GPU, --no-wrap: the reference's iteration)")
      .option(&reserve, "--reserve", "CUs the overlapped sweep leaves to the exchange kernels (default 8)")
      .flag(&noWrap, "--no-wrap", "exchange every periodic self-halo each sweep (the reference's per-iteration "
                                  "exchange, bin/astaroth_sim.cu:223-274) instead of reading the periodic image")
      .flag(&weak, "--weak", "treat x,y,z as per-GPU sizes").flag(&fp64, "--fp64", "fp64 quantities");
  ma.add(p);
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  auto pg = comm::default_group();
  if (weak) {
    x = app::weak_scale(x, pg->size());
    y = app::weak_scale(y, pg->size());
    z = app::weak_scale(z, pg->size());
  }
  StencilModelConfig cfg;
  cfg.size = Dim3(x, y, z);
  cfg.kind = StencilKind::Astaroth;
  cfg.radius = 3;
  cfg.allDirections = true;
  cfg.quantities = nq;
  cfg.fp64 = fp64;
  cfg.temporal = temporal;
  cfg.methods = ma.flags();
  cfg.placement = ma.placement();
  cfg.interiorAlign = ma.interiorAlign;
  cfg.sharedHaloLine = ma.sharedHaloLine;
  cfg.transport = ma.transport(cfg.transport);
  cfg.overlap = !noOverlap;
  cfg.autoOverlap = !forceOverlap;
  if (reserve >= 0) cfg.tune.x2reserve = reserve;
  cfg.wrapSelf = !noWrap;
  StencilModel m(cfg, pg);
  m.init();
  const int per = m.steps_per_sweep(); // timed unit = one sweep (1, 2 or 3 steps), reported per step
  if (pg->rank() == 0)
    std::fprintf(stderr, "# astaroth_sim: %d step(s) per sweep, in-kernel wrap axes %d, overlap %d\n", per, m.wrap_axes(),
                 int(m.overlapping()));
  m.run(per);
  m.synchronize();
  Statistics st;
  for (int i = 0; i < iters; ++i) {
    pg->barrier();
    const double t0 = app::now();
    m.run(per);
    m.synchronize();
    st.insert(pg->allreduce_max((app::now() - t0) / per));
  }
  if (pg->rank() == 0)
    std::printf("astaroth,%s,%d,%ld,%ld,%ld,%d,%e,%e,%.3f,%e\n", to_string(cfg.methods).c_str(), pg->size(), long(x),
                long(y), long(z), nq, st.min(), st.trimean(), double(x * y * z) / st.trimean() / 1e9,
                double(m.domain().exchange_bytes_for_method(MethodFlags::All)));
  return 0;
}
