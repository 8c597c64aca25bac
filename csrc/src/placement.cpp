#include "stencil/topo/placement.hpp"

#include <algorithm>
#include <sstream>

#include "stencil/rt/logging.hpp"
#include "stencil/topo/qap.hpp"

namespace stencil {

int64_t halo_volume(const Dim3 &dir, const Dim3 &sz, const Radius &radius) {
  Dim3 e;
  e.x = dir.x == 0 ? sz.x : radius.x(int(dir.x));
  e.y = dir.y == 0 ? sz.y : radius.y(int(dir.y));
  e.z = dir.z == 0 ? sz.z : radius.z(int(dir.z));
  return e.flatten();
}

// all-gather a variable-length int list per rank
static std::vector<std::vector<int>> allgather_lists(comm::ProcGroup &pg, const std::vector<int> &mine) {
  int n = int(mine.size());
  std::vector<int> counts(pg.size());
  pg.allgather(&n, sizeof(n), counts.data());
  const int maxN = *std::max_element(counts.begin(), counts.end());
  std::vector<int> padded(maxN, -1), all(size_t(maxN) * pg.size());
  std::copy(mine.begin(), mine.end(), padded.begin());
  if (maxN) pg.allgather(padded.data(), sizeof(int) * maxN, all.data());
  std::vector<std::vector<int>> out(pg.size());
  for (int r = 0; r < pg.size(); ++r) out[r].assign(all.begin() + size_t(r) * maxN, all.begin() + size_t(r) * maxN + counts[r]);
  return out;
}

TrivialPlacement::TrivialPlacement(const Dim3 &size, comm::ProcGroup &pg, const std::vector<int> &rankDevices) {
  auto devs = allgather_lists(pg, rankDevices);
  int64_t num = 0;
  for (auto &d : devs) num += int64_t(d.size());
  part_ = RankPartition(size, num);
  int64_t i = 0;
  for (int r = 0; r < pg.size(); ++r) {
    for (int id = 0; id < int(devs[r].size()); ++id, ++i) {
      SubdomainAssignment a{r, id, devs[r][id]};
      record(part_.dimensionize(i), a);
    }
  }
}

NodeAwarePlacement::NodeAwarePlacement(const Dim3 &size, comm::ProcGroup &pg, const Radius &radius,
                                       const std::vector<int> &rankDevices, const BandwidthFn &bw, const Dim3 &axisCost,
                                       PartitionObjective objective) {
  const int gpusPerRank = int(rankDevices.size());
  STENCIL_REQUIRE(pg.allreduce_min_i64(gpusPerRank) == -pg.allreduce_min_i64(-int64_t(gpusPerRank)),
                  "NodeAware placement requires the same number of GPUs on every rank");

  // number nodes in order of first appearance (rank order)
  std::vector<std::string> nodeNames;
  std::vector<std::vector<int>> nodeRanks;
  for (int r = 0; r < pg.size(); ++r) {
    auto it = std::find(nodeNames.begin(), nodeNames.end(), pg.hostname(r));
    if (it == nodeNames.end()) {
      nodeNames.push_back(pg.hostname(r));
      nodeRanks.push_back({r});
    } else {
      nodeRanks[it - nodeNames.begin()].push_back(r);
    }
  }
  const int numNodes = int(nodeNames.size());
  const int ranksPerNode = int(nodeRanks[0].size());
  for (auto &nr : nodeRanks)
    STENCIL_REQUIRE(int(nr.size()) == ranksPerNode, "NodeAware placement requires the same number of ranks per node");
  const int gpusPerNode = gpusPerRank * ranksPerNode;
  part_ = NodePartition(size, radius, numNodes, gpusPerNode, axisCost, objective);
  const Dim3 dim = part_.dim();
  const int64_t numSub = dim.flatten();

  auto devs = allgather_lists(pg, rankDevices);

  // table[linear global idx] = {rank, id, device}
  std::vector<int> table(size_t(numSub) * 3, -1);
  if (pg.rank() == 0) {
    for (int node = 0; node < numNodes; ++node) {
      const auto &ranks = nodeRanks[node];
      Mat2D<double> bandwidth(gpusPerNode, gpusPerNode, 0.0);
      for (int ci = 0; ci < gpusPerNode; ++ci)
        for (int cj = 0; cj < gpusPerNode; ++cj) {
          const int di = devs[ranks[ci / gpusPerRank]][ci % gpusPerRank];
          const int dj = devs[ranks[cj / gpusPerRank]][cj % gpusPerRank];
          bandwidth.at(ci, cj) = bw(di, dj);
        }
      // halo volume between node-local sub-domains i -> j, summed over every direction that connects them
      Mat2D<double> comm(gpusPerNode, gpusPerNode, 0.0);
      for (int i = 0; i < gpusPerNode; ++i) {
        const Dim3 src = part_.global_idx(node, i);
        const Dim3 sz = part_.subdomain_size(src);
        for (int di = 0; di < 27; ++di) {
          const Dim3 dir = dir_from_index(di);
          if (dir == Dim3(0, 0, 0) || radius.dir(-dir) == 0) continue;
          const Dim3 dst = (src + dir).wrap(dim);
          for (int j = 0; j < gpusPerNode; ++j)
            if (j != i && part_.global_idx(node, j) == dst) comm.at(i, j) += double(halo_volume(-dir, sz, radius));
        }
      }
      const std::vector<size_t> comp = qap::solve(comm, make_reciprocal(bandwidth));
      for (int i = 0; i < gpusPerNode; ++i) {
        const int c = int(comp[i]);
        const int rank = ranks[c / gpusPerRank];
        const int id = c % gpusPerRank;
        const int64_t li = linearize(part_.global_idx(node, i), dim);
        table[li * 3 + 0] = rank;
        table[li * 3 + 1] = id;
        table[li * 3 + 2] = devs[rank][id];
      }
    }
  }
  pg.bcast(table.data(), table.size() * sizeof(int), 0);
  for (int64_t li = 0; li < numSub; ++li) {
    SubdomainAssignment a{table[li * 3 + 0], table[li * 3 + 1], table[li * 3 + 2]};
    STENCIL_REQUIRE(a.rank >= 0, "placement left sub-domain " << li << " unassigned");
    record(dimensionize(li, dim), a);
  }
}

} // namespace stencil
