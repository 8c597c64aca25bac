// Exchange-only weak scaling: nIters exchanges (no swap) timed as one block, max over ranks.
// Parity: reference bin/weak_exchange.cu (radius 3, 4 quantities, weak-scaled, MPI_Wtime + Allreduce MAX).
#include <cstdio>

#include "app_common.hpp"

using namespace stencil;

int main(int argc, char **argv) {
  int64_t x = 512, y = 512, z = 512;
  int iters = 30, nq = 4;
  app::MethodArgs ma;
  ArgParser p("exchange-only weak scaling (reference bin/weak_exchange.cu)");
  p.positional(&x, "x", "x").positional(&y, "y", "y").positional(&z, "z", "z").positional(&iters, "iters", "iterations")
      .option(&nq, "--q", "quantities");
  ma.add(p);
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  auto pg = comm::default_group();
  x = app::weak_scale(x, pg->size());
  y = app::weak_scale(y, pg->size());
  z = app::weak_scale(z, pg->size());
  DistributedDomain dd(x, y, z, pg);
  dd.set_radius(3);
  dd.set_methods(ma.flags());
  dd.set_placement(ma.placement());
  dd.set_interior_align(ma.interiorAlign);
  dd.set_shared_halo_line(ma.sharedHaloLine);
  dd.set_transport_options(ma.transport());
  for (int i = 0; i < nq; ++i) dd.add_data<float>("d" + std::to_string(i));
  dd.realize();
  dd.exchange();
  pg->barrier();
  const double t0 = app::now();
  for (int i = 0; i < iters; ++i) dd.exchange();
  const double el = pg->allreduce_max(app::now() - t0);
  const uint64_t bytes = dd.exchange_bytes_for_method(MethodFlags::All);
  if (pg->rank() == 0)
    std::printf("weak_exchange,%s,%d,%ld,%ld,%ld,%d,%e,%e\n", to_string(ma.flags()).c_str(), pg->size(), long(x), long(y),
                long(z), iters, el / iters, double(bytes) * iters / el);
  return 0;
}
