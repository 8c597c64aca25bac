// Halo-exchange bandwidth micro-benchmark. Parity: reference bin/bench_exchange.cu (options --iters --x --y --z --q
// --fr --er --cr; five radius patterns px / x / faces / face&edge / uniform; B/s = aggregate halo bytes over all
// ranks / trimean of exchange()+swap()). Fixes: the recorded time is the max over ranks (reference records rank 0's
// local time, bench_exchange.cu:51); the face&edge pattern sets edges, not corners.
#include <cstdio>
#include <iostream>
#include <sstream>

#include "app_common.hpp"
#include "stencil/rt/statistics.hpp"

using namespace stencil;

static std::pair<Statistics, uint64_t> bench(comm::ProcGroup &pg, int iters, int nq, const Dim3 &ext, const Radius &r,
                                             MethodFlags m, PlacementStrategy pl, bool weak, bool xHaloAlign,
                                             const app::MethodArgs &ma) {
  Dim3 e = ext;
  if (weak) e = Dim3(app::weak_scale(ext.x, pg.size()), app::weak_scale(ext.y, pg.size()), app::weak_scale(ext.z, pg.size()));
  DistributedDomain dd(e.x, e.y, e.z, comm::default_group());
  dd.set_radius(r);
  dd.set_methods(m);
  dd.set_placement(pl);
  dd.set_x_halo_align(xHaloAlign);
  dd.set_interior_align(ma.interiorAlign);
  dd.set_shared_halo_line(ma.sharedHaloLine);
  dd.set_transport_options(ma.transport());
  for (int i = 0; i < nq; ++i) dd.add_data<float>("d" + std::to_string(i));
  dd.realize();
  Statistics st;
  for (int i = 0; i < 2; ++i) {
    dd.exchange();
    dd.swap();
  }
  for (int i = 0; i < iters; ++i) {
    pg.barrier();
    const double t0 = app::now();
    dd.exchange();
    dd.swap();
    st.insert(pg.allreduce_max(app::now() - t0));
  }
  return {st, dd.exchange_bytes_for_method(MethodFlags::All)};
}

int main(int argc, char **argv) {
  int iters = 30, nq = 1;
  int64_t x = 128, y = 128, z = 128, fr = 2, er = 1, cr = 1;
  bool weak = false, xHaloAlign = false;
  app::MethodArgs ma;
  ArgParser p("halo exchange bandwidth (reference bin/bench_exchange.cu)");
  p.option(&iters, "--iters", "iterations").option(&x, "--x", "x").option(&y, "--y", "y").option(&z, "--z", "z")
      .option(&nq, "--q", "quantities").option(&fr, "--fr", "face radius").option(&er, "--er", "edge radius")
      .option(&cr, "--cr", "corner radius").flag(&weak, "--weak", "scale x,y,z by ranks^(1/3)")
      .flag(&xHaloAlign, "--x-halo-align", "x halos inside the interior's first / last 64-B sector");
  ma.add(p);
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  auto pg = comm::default_group();
  const Dim3 ext(x, y, z);
  struct Pat {
    std::string name;
    Radius r;
  };
  std::vector<Pat> pats;
  {
    Radius r = Radius::constant(0);
    r.dir(1, 0, 0) = fr;
    pats.push_back({"px/" + std::to_string(fr), r});
    r.dir(-1, 0, 0) = fr;
    pats.push_back({"x/" + std::to_string(fr), r});
    Radius f = Radius::constant(0);
    f.set_face(fr);
    pats.push_back({"faces/" + std::to_string(fr), f});
    Radius fe = Radius::constant(0);
    fe.set_face(fr);
    fe.set_edge(er);
    pats.push_back({"face&edge/" + std::to_string(fr) + "/" + std::to_string(er), fe});
    Radius fec = Radius::face_edge_corner(fr, er, cr);
    pats.push_back({"fec/" + std::to_string(fr) + "/" + std::to_string(er) + "/" + std::to_string(cr), fec});
    pats.push_back({"uniform/" + std::to_string(fr), Radius::constant(fr)});
  }
  if (pg->rank() == 0) std::printf("name,count,trimean (S),trimean (B/s),stddev,min,avg,max\n");
  for (auto &pt : pats) {
    auto res = bench(*pg, iters, nq, ext, pt.r, ma.flags(), ma.placement(), weak, xHaloAlign, ma);
    if (pg->rank() == 0) {
      std::ostringstream n;
      n << x << "-" << y << "-" << z << "/" << pt.name;
      std::printf("%s,%zu,%e,%e,%e,%e,%e,%e\n", n.str().c_str(), res.first.count(), res.first.trimean(),
                  double(res.second) / res.first.trimean(), res.first.stddev(), res.first.min(), res.first.avg(),
                  res.first.max());
    }
  }
  return 0;
}
