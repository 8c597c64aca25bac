// Native unit tests (ctest). Parity: reference test/test_cpu_*.cpp expectations (radius, mat2d, partition, qap)
// plus host-backend exchange checks. GPU cases run only with --gpu.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <atomic>
#include <cstring>
#include <thread>
#include <functional>
#include <string>
#include <vector>

#include "stencil/comm/rccl_comm.hpp"
#include "stencil/comm/tags.hpp"
#include "stencil/core/array.hpp"
#include "stencil/core/boundary.hpp"
#include "stencil/domain/distributed_domain.hpp"
#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/rt/stream.hpp"
#include "stencil/rt/allocator.hpp"
#include "stencil/rt/build_info.hpp"
#include "stencil/rt/statistics.hpp"
#include "stencil/topo/gpu_topology.hpp"
#include "stencil/topo/partition.hpp"
#include "stencil/topo/qap.hpp"

using namespace stencil;

struct TestCase {
  const char *name;
  bool gpu;
  std::function<void()> fn;
};
static std::vector<TestCase> &registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Reg {
  Reg(const char *n, bool g, std::function<void()> f) { registry().push_back({n, g, f}); }
};
static int g_fail = 0;
#define CHECK(c)                                                                                                   \
  do {                                                                                                             \
    if (!(c)) {                                                                                                    \
      std::fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);                                   \
      ++g_fail;                                                                                                    \
    }                                                                                                              \
  } while (0)
#define TEST(name, gpu) static void name(); static Reg reg_##name(#name, gpu, name); static void name()

TEST(radius_basics, false) {
  Radius r = Radius::constant(0);
  r.set_face(2);
  CHECK(r.x(1) == 2 && r.y(-1) == 2 && r.dir(1, 1, 0) == 0);
  Radius c = Radius::constant(3);
  CHECK(c.dir(1, -1, 1) == 3);
  Radius f = Radius::face_edge_corner(3, 2, 1);
  CHECK(f.dir(0, 0, 0) == 0 && f.dir(1, 0, 0) == 3 && f.dir(1, 1, 0) == 2 && f.dir(1, 1, 1) == 1);
}

TEST(dim3_fixed_bugs, false) {
  CHECK(Dim3(1, 5, 3).max() == 5);
  CHECK(Dim3(1, 2, 3) != Dim3(1, 2, 4));
  CHECK(Dim3(-1, 5, 10).wrap(Dim3(4, 4, 4)) == Dim3(3, 1, 2));
}

TEST(partition_reference_values, false) {
  RankPartition p(Dim3(10, 3, 1), 4);
  CHECK(p.subdomain_size(Dim3(0, 0, 0)) == Dim3(3, 3, 1));
  CHECK(p.subdomain_size(Dim3(3, 0, 0)) == Dim3(2, 3, 1));
  CHECK(p.subdomain_origin(Dim3(3, 0, 0)) == Dim3(8, 0, 0));
  RankPartition q(Dim3(10, 14, 2), 9);
  CHECK(q.subdomain_origin(Dim3(1, 1, 0)) == Dim3(4, 5, 0));
  CHECK(q.subdomain_origin(Dim3(2, 2, 0)) == Dim3(7, 10, 0));
}

TEST(partition_max_link, false) {
  Radius r = Radius::constant(0);
  r.set_face(1);
  const Dim3 c(4, 3, 2);
  // stacked 512^3 cubes on one xGMI node: slabs (one face per link) beat 1x2x4 (two faces on the y link)
  CHECK(NodePartition(Dim3(512, 512, 4096), r, 1, 8, c, PartitionObjective::MaxLink).dim() == Dim3(1, 1, 8));
  CHECK(NodePartition(Dim3(512, 512, 2048), r, 1, 4, c, PartitionObjective::MaxLink).dim() == Dim3(1, 1, 4));
  CHECK(NodePartition::link_cost(Dim3(512, 512, 1024), Dim3(1, 1, 2), r, c).first == 512 * 512 * 2 * 2);
  // the reference rule is unchanged by default
  CHECK(NodePartition(Dim3(1024, 1024, 1024), r, 1, 8, c).dim() == Dim3(1, 2, 4));
}

TEST(qap_reference_values, false) {
  const double inf = INFINITY;
  Mat2D<double> bw = {{inf, 1, 10}, {1, inf, 1}, {10, 1, inf}};
  Mat2D<double> comm = {{0, 10, 1}, {10, 0, 1}, {1, 1, 0}};
  auto f = qap::solve(comm, make_reciprocal(bw));
  CHECK(f[0] == 0 && f[1] == 2 && f[2] == 1);
  Mat2D<double> bw9 = {{900, 75, 64, 64}, {75, 900, 64, 64}, {64, 64, 900, 75}, {64, 64, 75, 900}};
  Mat2D<double> c9 = {{7, 5, 10, 1}, {5, 7, 1, 10}, {10, 1, 7, 5}, {1, 10, 5, 7}};
  auto g = qap::solve(c9, make_reciprocal(bw9));
  CHECK(g[0] == 0 && g[1] == 2 && g[2] == 1 && g[3] == 3);
  auto h = qap::solve_catch(c9, make_reciprocal(bw9));
  CHECK(h[0] == 3 && h[1] == 1 && h[2] == 2 && h[3] == 0);
}

TEST(select_method_ladder, false) {
  PairInfo p;
  p.sameRank = true;
  p.sameDevice = true;
  CHECK(select_method(MethodFlags::All, p) == MethodFlags::Kernel);
  p = PairInfo();
  p.sameHost = true;
  CHECK(select_method(MethodFlags::All, p) == MethodFlags::Rccl);
  p.sharedGpu = true; // RCCL refuses a GPU two ranks drive: only such pairs are staged
  CHECK(select_method(MethodFlags::All, p) == MethodFlags::Staged);
  CHECK(select_method(MethodFlags::Rccl | MethodFlags::Kernel, p) == MethodFlags::Staged);
  p.canAccess = true;
  CHECK(select_method(MethodFlags::All, p) == MethodFlags::Colocated);
  CHECK(select_method(MethodFlags::Kernel, PairInfo()) == MethodFlags::None);
}

TEST(statistics_trimean, false) {
  Statistics s;
  for (int i = 0; i < 8; ++i) s.insert(i);
  CHECK(s.trimean() == (2 + 2 * 4 + 6) / 4.0);
  CHECK(s.med() == 3.5);
}

// encode the global coordinate in the value; after exchange every halo cell must hold its periodic image
static void check_exchange(Backend b, const Radius &r, const Dim3 &sz, std::vector<int> gpus, MethodFlags m) {
  DistributedDomain dd(sz.x, sz.y, sz.z, comm::make_single_group());
  dd.set_backend(b);
  dd.set_radius(r);
  dd.set_gpus(gpus);
  dd.set_methods(m);
  dd.set_plan_file("");
  auto h = dd.add_data<int32_t>("coord");
  dd.realize();
  for (auto &d : dd.domains()) {
    const Dim3 raw = d.raw_size();
    std::vector<int32_t> v(size_t(raw.flatten()), -1);
    const Dim3 org = d.accessor_origin();
    for (int64_t z = 0; z < raw.z; ++z)
      for (int64_t y = 0; y < raw.y; ++y)
        for (int64_t x = 0; x < raw.x; ++x) {
          const Dim3 g = org + Dim3(x, y, z);
          if (d.get_compute_region().contains(g)) v[size_t(x + raw.x * (y + raw.y * z))] = int32_t(g.x + 1000 * g.y + 1000000 * g.z);
        }
    d.region_from_host(Dim3(0, 0, 0), raw, h.id(), v.data());
  }
  dd.exchange();
  for (auto &d : dd.domains()) {
    const Dim3 raw = d.raw_size();
    auto bytes = d.quantity_to_host(h.id());
    const int32_t *v = reinterpret_cast<const int32_t *>(bytes.data());
    const Dim3 org = d.accessor_origin();
    int bad = 0;
    for (int64_t z = 0; z < raw.z; ++z)
      for (int64_t y = 0; y < raw.y; ++y)
        for (int64_t x = 0; x < raw.x; ++x) {
          const Dim3 g = org + Dim3(x, y, z);
          // which halo direction is this cell in?
          const Rect3 cr = d.get_compute_region();
          Dim3 dir(g.x < cr.lo.x ? -1 : (g.x >= cr.hi.x ? 1 : 0), g.y < cr.lo.y ? -1 : (g.y >= cr.hi.y ? 1 : 0),
                   g.z < cr.lo.z ? -1 : (g.z >= cr.hi.z ? 1 : 0));
          if (dir == Dim3(0, 0, 0)) continue;
          const int32_t got = v[size_t(x + raw.x * (y + raw.y * z))];
          // a halo cell in direction dir is filled iff the neighbour on that side sends (radius(dir) != 0) and the
          // cell lies within the face-radius extents
          if (r.dir(dir) == 0) continue;
          const Dim3 w = g.wrap(sz);
          const int32_t want = int32_t(w.x + 1000 * w.y + 1000000 * w.z);
          if (got != want) ++bad;
        }
    CHECK(bad == 0);
  }
}

TEST(host_exchange_uniform, false) { check_exchange(Backend::Host, Radius::constant(2), Dim3(10, 9, 8), {0}, MethodFlags::All); }
TEST(host_exchange_two_subdomains, false) {
  check_exchange(Backend::Host, Radius::constant(1), Dim3(12, 10, 10), {0, 0}, MethodFlags::All);
}
TEST(host_exchange_asymmetric, false) {
  Radius r = Radius::constant(0);
  r.dir(1, 0, 0) = 2;
  r.dir(-1, 0, 0) = 1;
  check_exchange(Backend::Host, r, Dim3(10, 10, 10), {0, 0, 0}, MethodFlags::All);
}
TEST(gpu_exchange_uniform, true) { check_exchange(Backend::Device, Radius::constant(2), Dim3(10, 9, 8), {0}, MethodFlags::All); }
TEST(gpu_exchange_two_subdomains_rccl, true) {
  check_exchange(Backend::Device, Radius::constant(1), Dim3(12, 10, 10), {0, 0}, MethodFlags::Rccl);
}

// reference test/test_cpu_array.cpp / test_cuda_array.cu
TEST(array_host, false) {
  Array<int> a(4, 7);
  CHECK(a.size() == 4 && a[3] == 7);
  Array<int> b = a;
  CHECK(a == b);
  b[0] = 1;
  CHECK(a != b);
  b.resize(6);
  CHECK(b.size() == 6 && b[0] == 1 && b[3] == 7 && b[5] == 0);
  Array<int> c{1, 2, 3};
  Array<int> d(std::move(c));
  CHECK(d.size() == 3 && c.size() == 0 && d[2] == 3);
}

// reference test/test_cpu_tx.cpp:5-9 (tags are distinct); here distinct across kinds and pairs, and overflow-checked
TEST(tags_distinct, false) {
  std::vector<uint32_t> seen;
  const int64_t n = 9;
  for (int k = 0; k < 5; ++k)
    for (int64_t s = 0; s < n; ++s)
      for (int64_t d = 0; d < n; ++d) seen.push_back(comm::make_tag(comm::MsgKind(k), s, d, n));
  std::sort(seen.begin(), seen.end());
  CHECK(std::adjacent_find(seen.begin(), seen.end()) == seen.end());
  for (uint32_t t : seen) CHECK((t & comm::kTagReserved) == 0);
  const uint32_t t = comm::make_tag(comm::MsgKind::IpcCredit, 3, 5, n);
  CHECK(comm::tag_kind(t) == comm::MsgKind::IpcCredit && comm::tag_payload(t) == 3 * 9 + 5);
  bool threw = false;
  try {
    comm::make_tag(comm::MsgKind::Data, 16383, 16383, int64_t(1) << 14);
  } catch (stencil::Error &) {
    threw = true;
  }
  CHECK(!threw);
  threw = false;
  try {
    comm::make_tag(comm::MsgKind::Data, 0, 0, (int64_t(1) << 14) + 1);
  } catch (stencil::Error &) {
    threw = true;
  }
  CHECK(threw);
}

TEST(boundary_flags, false) {
  Boundary b;
  CHECK(b.all_periodic() && b.wraps(Dim3(1, -1, 1)));
  Boundary nx = Boundary::axes(false, true, true);
  CHECK(!nx.all_periodic() && !nx.wraps(Dim3(1, 0, 0)) && nx.wraps(Dim3(0, 1, -1)) && !nx.wraps(Dim3(-1, 1, 0)));
  // 2 sub-domains in x: from idx 1, +x leaves the grid
  CHECK(!nx.reachable(Dim3(1, 0, 0), Dim3(1, 0, 0), Dim3(2, 1, 1)));
  CHECK(nx.reachable(Dim3(0, 0, 0), Dim3(1, 0, 0), Dim3(2, 1, 1)));
  CHECK(nx.reachable(Dim3(1, 0, 0), Dim3(0, 1, 0), Dim3(2, 1, 1)));
  Boundary one;
  one.set_face(0, 0, -1, false);
  CHECK(one.face_periodic(0, 0, 1) && !one.face_periodic(0, 0, -1));
  CHECK(!one.reachable(Dim3(0, 0, 0), Dim3(0, 0, -1), Dim3(1, 1, 3)) && one.reachable(Dim3(0, 0, 2), Dim3(0, 0, 1), Dim3(1, 1, 3)));
}

// non-periodic x: halos across the global x faces are not written (keep the sentinel); everything else wraps
static void check_nonperiodic(Backend b, std::vector<int> gpus) {
  const Dim3 sz(12, 6, 5);
  DistributedDomain dd(sz.x, sz.y, sz.z, comm::make_single_group());
  dd.set_backend(b);
  dd.set_radius(1);
  dd.set_boundary(Boundary::axes(false, true, true));
  dd.set_gpus(gpus);
  dd.set_plan_file("");
  auto h = dd.add_data<int32_t>("coord");
  dd.realize();
  for (auto &d : dd.domains()) {
    const Dim3 raw = d.raw_size();
    std::vector<int32_t> v(size_t(raw.flatten()), -1);
    const Dim3 org = d.accessor_origin();
    for (int64_t z = 0; z < raw.z; ++z)
      for (int64_t y = 0; y < raw.y; ++y)
        for (int64_t x = 0; x < raw.x; ++x) {
          const Dim3 g = org + Dim3(x, y, z);
          if (d.get_compute_region().contains(g)) v[size_t(x + raw.x * (y + raw.y * z))] = int32_t(g.x + 1000 * g.y + 1000000 * g.z);
        }
    d.region_from_host(Dim3(0, 0, 0), raw, h.id(), v.data());
  }
  dd.exchange();
  int bad = 0, untouched = 0;
  for (auto &d : dd.domains()) {
    const Dim3 raw = d.raw_size();
    auto bytes = d.quantity_to_host(h.id());
    const int32_t *v = reinterpret_cast<const int32_t *>(bytes.data());
    const Dim3 org = d.accessor_origin();
    const Rect3 cr = d.get_compute_region();
    for (int64_t z = 1; z < raw.z - 1; ++z)
      for (int64_t y = 1; y < raw.y - 1; ++y)
        for (int64_t x = 0; x < raw.x; ++x) {
          const Dim3 g = org + Dim3(x, y, z);
          if (g.x < cr.lo.x - 1 || g.x > cr.hi.x) continue; // x padding
          if (cr.contains(g)) continue;
          const int32_t got = v[size_t(x + raw.x * (y + raw.y * z))];
          if (g.x < 0 || g.x >= sz.x) {
            untouched += got == -1;
            bad += got != -1;
            continue;
          }
          const Dim3 w = g.wrap(sz);
          bad += got != int32_t(w.x + 1000 * w.y + 1000000 * w.z);
        }
  }
  CHECK(bad == 0);
  CHECK(untouched > 0);
}
TEST(host_exchange_nonperiodic_x, false) { check_nonperiodic(Backend::Host, {0, 0}); }
TEST(gpu_exchange_nonperiodic_x, true) { check_nonperiodic(Backend::Device, {0, 0}); }

TEST(gpu_allocators_array, true) {
  std::vector<float, DeviceAllocator<float>> dv(DeviceAllocator<float>(0));
  dv.reserve(1024);
  CHECK(dv.capacity() >= 1024);
  std::vector<int, ManagedAllocator<int>> mv(16, 3, ManagedAllocator<int>(0));
  int s = 0;
  for (int x : mv) s += x;
  CHECK(s == 48);
  std::vector<char, PinnedAllocator<char>> pv(4096, 1);
  CHECK(pv[4095] == 1);
  Array<double, Mem::Device> a(std::vector<double>{1.0, 2.0, 3.0}, 0);
  auto back = a.to_host();
  CHECK(back.size() == 3 && back[2] == 3.0);
  a.memset(0);
  back = a.to_host();
  CHECK(back[0] == 0.0 && back[2] == 0.0);
}

// the fused pair split as an overlapped step runs it (interior sweep + exterior slabs, thread per cell) must give
// the same bits as one sweep of the whole compute region
static void check_x2_split(StencilKind kind) {
  LocalDomain ld(Dim3(40, 36, 44), Dim3(0, 0, 0), 0, Backend::Device);
  ld.set_radius(Radius::face_edge_corner(2, 1, 0));
  ld.add_data<float>("d");
  ld.realize();
  Stream s(0);
  const Rect3 cr = ld.get_compute_region();
  const Spheres sph = kind == StencilKind::Jacobi ? Spheres::jacobi(Rect3(Dim3(0, 0, 0), Dim3(40, 36, 44))) : Spheres();
  astaroth_init(ld, 0, 10.0, s); // sin-wave interior, -10 halo: every cell distinct enough to catch a wrong read
  const size_t n = size_t(ld.buffer_bytes(0) / 4);
  auto next_to_host = [&]() {
    std::vector<float> h(n);
    s.sync();
    HIP_CHECK(hipMemcpy(h.data(), static_cast<char *>(ld.next_data(0)) - ld.pad_x(0) * 4, n * 4, hipMemcpyDeviceToHost));
    return h;
  };
  fill_value(ld, 0, 0.0, false, s);
  stencil7x2_apply(ld, 0, cr, kind, sph, s);
  const auto whole = next_to_host();
  fill_value(ld, 0, 0.0, false, s);
  Rect3 in = cr;
  in.lo = in.lo + Dim3(2, 2, 2);
  in.hi = in.hi - Dim3(2, 2, 2);
  stencil7x2_apply(ld, 0, in, kind, sph, s);
  std::vector<Rect3> ext;
  ext.push_back(Rect3(Dim3(cr.lo.x, cr.lo.y, cr.lo.z), Dim3(cr.hi.x, cr.hi.y, in.lo.z)));
  ext.push_back(Rect3(Dim3(cr.lo.x, cr.lo.y, in.hi.z), Dim3(cr.hi.x, cr.hi.y, cr.hi.z)));
  ext.push_back(Rect3(Dim3(cr.lo.x, cr.lo.y, in.lo.z), Dim3(cr.hi.x, in.lo.y, in.hi.z)));
  ext.push_back(Rect3(Dim3(cr.lo.x, in.hi.y, in.lo.z), Dim3(cr.hi.x, cr.hi.y, in.hi.z)));
  ext.push_back(Rect3(Dim3(cr.lo.x, in.lo.y, in.lo.z), Dim3(in.lo.x, in.hi.y, in.hi.z)));
  ext.push_back(Rect3(Dim3(in.hi.x, in.lo.y, in.lo.z), Dim3(cr.hi.x, in.hi.y, in.hi.z)));
  stencil7x2_apply_regions(ld, 0, ext, kind, sph, s);
  const auto split = next_to_host();
  int64_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += std::memcmp(&whole[i], &split[i], 4) != 0;
  if (bad) std::fprintf(stderr, "  regions: %lld cells differ\n", (long long)bad);
  CHECK(bad == 0);
  // the overlapped model's exterior (sweep for z/y slabs, lanes-on-rows for x slabs), x slabs 2 and 1 thick
  for (int tx : {2, 1}) {
    fill_value(ld, 0, 0.0, false, s);
    Rect3 in2 = in;
    in2.hi.x = cr.hi.x - tx;
    stencil7x2_apply(ld, 0, in2, kind, sph, s);
    stencil7x2_apply_exterior(ld, 0, in2, kind, sph, s);
    const auto ex = next_to_host();
    int64_t bad2 = 0;
    for (size_t i = 0; i < n; ++i) bad2 += std::memcmp(&whole[i], &ex[i], 4) != 0;
    if (bad2) std::fprintf(stderr, "  exterior (x slab %d): %lld cells differ\n", tx, (long long)bad2);
    CHECK(bad2 == 0);
  }
}
TEST(gpu_x2_split_regions_jacobi, true) { check_x2_split(StencilKind::Jacobi); }
TEST(gpu_x2_split_regions_astaroth, true) { check_x2_split(StencilKind::Astaroth); }

TEST(transport_options_defaults, false) {
  TransportOptions o;
  CHECK(o.inbox == TransportOptions::Inbox::Uncached && o.coloCopy == TransportOptions::Copy::Store &&
        o.peerCopy == TransportOptions::Copy::Store && o.completion == TransportOptions::Completion::Kernel);
  CHECK(std::string(to_string(TransportOptions::Inbox::Coarse)) == "coarse");
  CHECK(std::string(to_string(TransportOptions::Copy::Engine)) == "engine");
  CHECK(std::string(to_string(TransportOptions::Completion::StreamOp)) == "streamop");
  // waitTimeout <= 0 resolves to STENCIL_WAIT_TIMEOUT or 60 s at set_transport_options
  DistributedDomain dd(8, 8, 8, comm::make_single_group());
  dd.set_transport_options(o);
  CHECK(dd.transport_options().waitTimeout > 0);
}

TEST(build_info_embedded, false) {
  const BuildInfo &b = build_info();
  CHECK(!b.gitSha.empty() && b.offloadArch == "gfx950");
  CHECK(b.useRccl == rccl::compiled());
  CHECK(build_info_string().find("git=") != std::string::npos);
}

TEST(rccl_unique_id_or_reason, false) {
  // without a GPU RCCL may refuse; either way the wrapper reports instead of aborting
  rccl::UniqueId id{};
  const std::string e = rccl::get_unique_id(&id);
  CHECK(e.empty() || e.find("nccl") != std::string::npos || e.find("RCCL") != std::string::npos);
}

TEST(numa_cpulist_parse, false) {
  // node 0 exists on every Linux host with sysfs; unknown nodes give nothing
  const auto c0 = gpu_topo::numa_cpus(0);
  CHECK(gpu_topo::numa_cpus(-1).empty() && gpu_topo::numa_cpus(1 << 20).empty());
  for (size_t i = 1; i < c0.size(); ++i) CHECK(c0[i] > c0[i - 1]);
}

TEST(host_self_test_ladder_single_rank, false) {
  // a single rank has no ladder to climb; probe_transports still runs the coordinate oracle on the host backend
  DistributedDomain dd(20, 16, 12, comm::make_single_group());
  dd.set_backend(Backend::Host);
  dd.set_radius(Radius::face_edge_corner(2, 1, 1));
  dd.add_data<float>("d");
  CHECK(dd.probe_transports(MethodFlags::All) == 0);
}

TEST(process_group_bounded_barrier, false) {
  auto g = comm::make_single_group();
  CHECK(g->barrier_for(0.1));
}

TEST(process_group_fork_abandon, false) {
  // two ranks (threads) over TCP: a fork is a separate group; one rank abandons it mid-sequence, the other times out
  // there, and the parent group's collective sequence stays in step (the self-test probe's failure path)
  const int port = comm::find_free_port();
  std::atomic<int> ok{0};
  auto body = [&](int r) {
    auto g = comm::make_tcp_group(r, 2, "127.0.0.1", port, 30.0);
    auto f = g->fork(1.0);
    if (f->size() == 2 && f->rank() == r && f->allreduce_sum_u64(1) == 2) ++ok;
    if (r == 0) {
      bool threw = false;
      try {
        f->barrier(); // rank 1 never joins
      } catch (const std::exception &) {
        threw = true;
      }
      if (threw) ++ok;
    }
    if (g->allreduce_sum_u64(uint64_t(r + 1)) == 3) ++ok;
  };
  std::thread t1(body, 1);
  body(0);
  t1.join();
  CHECK(ok.load() == 5);
}

int main(int argc, char **argv) {
  bool cpu = true, gpu = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--gpu")) gpu = true, cpu = false;
    if (!std::strcmp(argv[i], "--all")) gpu = true, cpu = true;
  }
  int ran = 0;
  for (auto &t : registry()) {
    if ((t.gpu && !gpu) || (!t.gpu && !cpu)) continue;
    const int before = g_fail;
    try {
      t.fn();
    } catch (std::exception &e) {
      std::fprintf(stderr, "  exception: %s\n", e.what());
      ++g_fail;
    }
    std::printf("%s %s\n", g_fail == before ? "PASS" : "FAIL", t.name);
    ++ran;
  }
  std::printf("%d tests, %d failures\n", ran, g_fail);
  return g_fail ? 1 : 0;
}
