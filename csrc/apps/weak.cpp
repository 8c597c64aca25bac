// Weak / strong scaling exchange driver. Parity: reference bin/weak.cu and bin/strong.cu (positional x y z iters,
// radius 3, 4 float quantities, loop exchange(); swap(); CSV with per-method byte counters and the setup/exchange
// timers). This one binary does both: weak scaling (default) multiplies each axis by ranks^0.33333; --strong keeps
// the global size (the reference's strong.cu printed the label "weak", bin/strong.cu:181).
#include <cstdio>

#include "app_common.hpp"

using namespace stencil;

int main(int argc, char **argv) {
  int64_t x = 512, y = 512, z = 512;
  int iters = 30, nq = 4, radius = 3;
  bool strong = false, fp64 = false;
  app::MethodArgs ma;
  ArgParser p("weak/strong scaling exchange driver (reference bin/weak.cu, bin/strong.cu)");
  p.positional(&x, "x", "x").positional(&y, "y", "y").positional(&z, "z", "z").positional(&iters, "iters", "iterations")
      .option(&nq, "--q", "quantities").option(&radius, "--radius", "radius").flag(&strong, "--strong", "strong scaling")
      .flag(&fp64, "--fp64", "fp64 quantities (BASELINE config: 1024^3/GPU fp64)");
  ma.add(p);
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  auto pg = comm::default_group();
  if (!strong) {
    x = app::weak_scale(x, pg->size());
    y = app::weak_scale(y, pg->size());
    z = app::weak_scale(z, pg->size());
  }
  DistributedDomain dd(x, y, z, pg);
  dd.exchangeStats_ = true;
  dd.set_radius(radius);
  dd.set_methods(ma.flags());
  dd.set_placement(ma.placement());
  dd.set_interior_align(ma.interiorAlign);
  dd.set_shared_halo_line(ma.sharedHaloLine);
  dd.set_transport_options(ma.transport());
  for (int i = 0; i < nq; ++i) {
    if (fp64)
      dd.add_data<double>("d" + std::to_string(i));
    else
      dd.add_data<float>("d" + std::to_string(i));
  }
  dd.realize();
  for (int i = 0; i < iters; ++i) {
    dd.exchange();
    dd.swap();
  }
  if (pg->rank() == 0)
    std::printf("%s,%s,%ld,%ld,%ld,%ld,%lu,%lu,%lu,%lu,%lu,%d,%d,%d,%e,%e,%e,%e,%e,%e,%e,%e,%e\n", strong ? "strong" : "weak",
                to_string(ma.flags()).c_str(), long(x), long(y), long(z), long(x * y * z),
                (unsigned long)dd.exchange_bytes_for_method(MethodFlags::Staged),
                (unsigned long)dd.exchange_bytes_for_method(MethodFlags::Rccl),
                (unsigned long)dd.exchange_bytes_for_method(MethodFlags::Colocated),
                (unsigned long)dd.exchange_bytes_for_method(MethodFlags::PeerCopy),
                (unsigned long)dd.exchange_bytes_for_method(MethodFlags::Kernel), iters, pg->num_nodes(), pg->size(),
                dd.timeMpiTopo_, dd.timeNodeGpus_, dd.timePeerEn_, dd.timePlacement_, dd.timePlan_, dd.timeRealize_,
                dd.timeCreate_, dd.timeExchange_, dd.timeSwap_);
  return 0;
}
