// DistributedDomain transport self-test: a coordinate-encoded probe domain run on a forked process group (split out
// of distributed_domain.cpp; called from realize()).
#include "stencil/domain/distributed_domain.hpp"

#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "stencil/rt/hip_check.hpp"
#include "stencil/rt/trace.hpp"

namespace stencil {

// ------------------------------------------------------------------------------------------------
// transport self-test (opt-in): coordinate oracle on a probe domain, ladder Colocated -> Rccl -> Staged
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int32_t kProbePoison = -1;
int32_t probe_key(int64_t gx, int64_t gy, int64_t gz, const Dim3 &L, int32_t offset) {
  return int32_t((gx + L.x * (gy + L.y * gz)) % 1000000007) + offset;
}
} // namespace

int64_t DistributedDomain::probe_transports(MethodFlags m) {
  // same group, radius, boundary, placement, cut costs, devices, backend and transport options; every axis
  // shrunk ~16x (at least 6 cells per stencil reach) so the probe is cheap but spans the same rank pairs
  int64_t rmax = 1;
  for (int i = 0; i < 27; ++i) rmax = std::max<int64_t>(rmax, radius_.dir(dir_from_index(i)));
  auto shrink = [&](int64_t n) { return std::min<int64_t>(n, std::max<int64_t>((n + 15) / 16, 6 * rmax + 2)); };
  // the probe runs on a fork of the group: a rank whose probe fails (an exception anywhere in realize / exchange)
  // abandons the fork mid-sequence and goes straight to the verdict below; the other ranks' next receive on the
  // fork then times out after waitTimeout, they fail too and join the verdict, and this group's own collective
  // sequence never goes out of step
  const double forkTimeout = std::max(1.0, topt_.waitTimeout);
  std::shared_ptr<comm::ProcGroup> grp = pg_->size() > 1 ? pg_->fork(forkTimeout) : pg_;
  int64_t bad = 0;
  {
    DistributedDomain p(shrink(size_.x), shrink(size_.y), shrink(size_.z), grp);
    p.set_radius(radius_);
    p.set_boundary(boundary_);
    p.set_methods(m);
    p.set_placement(strategy_);
    p.set_axis_cost(axisCost_);
    p.set_partition_objective(objective_);
    if (!gpus_.empty()) p.set_gpus(gpus_);
    if (backendSet_) p.set_backend(backend_);
    p.set_transport_options(topt_);
    p.set_plan_file("");
    p.set_x_halo_align(xHaloAlign_);
    p.set_shared_halo_line(sharedHaloLine_);
    p.set_interior_align(interiorAlign_);
    p.add_data(4, "probe", DType::I32);
    try {
      p.realize();
      if (topt_.failProbeRank == rank() && probeFailures_++ == 0) // test hook: this rank's first probe fails alone
        LOG_FATAL("TransportOptions::failProbeRank: probe failure forced on rank " << rank());
      const Dim3 L = p.size();
      for (int it = 0; it < 2; ++it) {
        const int32_t off = 7 * it;
        for (auto &d : p.domains_) {
          const Dim3 raw = d.raw_size(), org = d.accessor_origin();
          std::vector<int32_t> v(size_t(raw.flatten()), kProbePoison);
          const Rect3 cr = d.get_compute_region();
          for (int64_t z = 0; z < raw.z; ++z)
            for (int64_t y = 0; y < raw.y; ++y)
              for (int64_t x = 0; x < raw.x; ++x)
                if (cr.contains(Dim3(org.x + x, org.y + y, org.z + z)))
                  v[size_t(x + raw.x * (y + raw.y * z))] = probe_key(org.x + x, org.y + y, org.z + z, L, off);
          d.region_from_host(Dim3(0, 0, 0), raw, 0, v.data(), true);
          d.region_from_host(Dim3(0, 0, 0), raw, 0, v.data(), false);
        }
        p.exchange();
        for (auto &d : p.domains_) {
          const Dim3 raw = d.raw_size(), org = d.accessor_origin();
          const Rect3 cr = d.get_compute_region();
          const auto bytes = d.region_to_host(Dim3(0, 0, 0), raw, 0, true);
          const int32_t *got = reinterpret_cast<const int32_t *>(bytes.data());
          for (int64_t z = 0; z < raw.z; ++z)
            for (int64_t y = 0; y < raw.y; ++y)
              for (int64_t x = 0; x < raw.x; ++x) {
                const int64_t g[3] = {org.x + x, org.y + y, org.z + z};
                const int64_t lo[3] = {cr.lo.x, cr.lo.y, cr.lo.z}, hi[3] = {cr.hi.x, cr.hi.y, cr.hi.z};
                const int64_t n[3] = {L.x, L.y, L.z};
                int dd[3];
                bool crossesClosed = false;
                for (int a = 0; a < 3; ++a) {
                  dd[a] = g[a] >= hi[a] ? 1 : (g[a] < lo[a] ? -1 : 0);
                  if ((g[a] < 0 || g[a] >= n[a]) &&
                      !boundary_.face_periodic(a == 0 ? dd[a] : 0, a == 1 ? dd[a] : 0, a == 2 ? dd[a] : 0))
                    crossesClosed = true;
                }
                const bool filled = (dd[0] == 0 && dd[1] == 0 && dd[2] == 0) ||
                                    (radius_.dir(Dim3(dd[0], dd[1], dd[2])) != 0 && !crossesClosed);
                const int32_t want =
                    filled ? probe_key(((g[0] % n[0]) + n[0]) % n[0], ((g[1] % n[1]) + n[1]) % n[1],
                                       ((g[2] % n[2]) + n[2]) % n[2], L, off)
                           : kProbePoison;
                bad += got[size_t(x + raw.x * (y + raw.y * z))] != want;
              }
        }
        p.swap();
      }
    } catch (const std::exception &e) {
      LOG_WARN("rank " << rank() << ": transport probe with " << to_string(m) << " failed: " << e.what());
      bad += int64_t(1) << 40;
      p.poison("transport probe failed"); // its destructor must not wait on work stuck behind an absent peer
    }
  } // the probe domain (and its bounded destructor barrier on the fork) is gone before the verdict
  return int64_t(pg_->allreduce_sum_u64(uint64_t(bad)));
}

} // namespace stencil
