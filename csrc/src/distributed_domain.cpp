// DistributedDomain implementation: placement, message planning, transport setup and the exchange engine.
// See distributed_domain.hpp for the design; reference call stacks: SURVEY §3.2 (realize) and §3.3 (exchange).
#include "stencil/domain/distributed_domain.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <set>
#include <sstream>
#include <thread>

#include "stencil/comm/rccl_comm.hpp"
#include "stencil/comm/tags.hpp"
#include "stencil/rt/env.hpp"
#include "stencil/rt/hip_check.hpp"
#include "stencil/rt/trace.hpp"
#include "stencil/topo/gpu_topology.hpp"

#include "distributed_domain_impl.hpp"

namespace stencil {


std::string to_string(MethodFlags m) {
  std::string s;
  auto add = [&](MethodFlags f, const char *n) {
    if (m && f) s += (s.empty() ? "" : "/") + std::string(n);
  };
  add(MethodFlags::Staged, "staged");
  add(MethodFlags::Rccl, "rccl");
  add(MethodFlags::Colocated, "colo");
  add(MethodFlags::PeerCopy, "peer");
  add(MethodFlags::Kernel, "kernel");
  return s.empty() ? "none" : s;
}

MethodFlags select_method(MethodFlags flags, const PairInfo &p) {
  auto on = [&](MethodFlags m) { return (int(flags) & int(m)) != 0; };
  if (!p.device) {
    if (p.sameRank && (on(MethodFlags::Kernel) || on(MethodFlags::PeerCopy)))
      return p.sameDevice && on(MethodFlags::Kernel) ? MethodFlags::Kernel : MethodFlags::PeerCopy;
    return on(MethodFlags::Staged) ? MethodFlags::Staged : MethodFlags::None;
  }
  if (on(MethodFlags::Kernel) && p.sameRank && p.sameDevice) return MethodFlags::Kernel;
  if (on(MethodFlags::PeerCopy) && p.sameRank && p.peer) return MethodFlags::PeerCopy;
  if (on(MethodFlags::Colocated) && !p.sameRank && p.sameHost && p.canAccess) return MethodFlags::Colocated;
  if (on(MethodFlags::Rccl) && !p.sharedGpu) return MethodFlags::Rccl;
  if (on(MethodFlags::Staged)) return MethodFlags::Staged;
  if (on(MethodFlags::Rccl) && p.sharedGpu) return MethodFlags::Staged;
  return MethodFlags::None;
}

// ------------------------------------------------------------------------------------------------
// construction / configuration
// ------------------------------------------------------------------------------------------------
DistributedDomain::DistributedDomain(int64_t x, int64_t y, int64_t z, std::shared_ptr<comm::ProcGroup> pg)
    : size_(x, y, z), pg_(pg ? pg : comm::default_group()), impl_(new Impl) {
  radius_ = Radius::constant(0);
#ifdef STENCIL_EXCHANGE_STATS
  exchangeStats_ = STENCIL_EXCHANGE_STATS != 0;
#endif
  topt_.waitTimeout = env_wait_timeout(60.0);
  if (env::get_int("STENCIL_PLAN_FILE", 1) == 0) planPrefix_.clear();
}

void DistributedDomain::set_transport_options(const TransportOptions &o) {
  STENCIL_REQUIRE(!realized_, "set_transport_options after realize");
  topt_ = o;
  if (topt_.waitTimeout <= 0) topt_.waitTimeout = env_wait_timeout(60.0);
}

// whole-line x faces for the translate s -> d: where asked for explicitly, else only on a device whose same-GPU x
// faces reached the auto threshold and only for its same-GPU translates (the threshold was measured there; a
// PeerCopy store across xGMI is left as w-cell pieces)
bool DistributedDomain::x_face_lines(const LocalDomain &s, const LocalDomain &d) const {
  if (topt_.xFaceSectors) return true;
  return s.gpu() == d.gpu() && impl_->xLineDevs.count(s.gpu()) > 0;
}

void DistributedDomain::poison(const std::string &why) {
  if (poisoned_.empty()) poisoned_ = why;
}

DistributedDomain::~DistributedDomain() {
  if (!impl_) return;
  Impl &I = *impl_;
  // a poisoned domain may have work stuck behind a dead peer: do not block on it (the process is going down)
  if (poisoned_.empty()) {
    try {
      for (auto &d : I.devs) {
        (void)HIP_TRY(hipSetDevice(d.dev));
        (void)HIP_TRY(hipStreamSynchronize(d.comm));
      }
      // the Acks no later record consumes: the next IpcEvent domain on this group reuses the channel tags
      if (!drain_ipc_acks(topt_.waitTimeout)) LOG_WARN("IPC-event acks not drained within the wait timeout");
    } catch (...) {
    }
  }
  for (auto &pp : I.pipes) {
    if (pp.sbuf) (void)hipFree(pp.sbuf);
    if (pp.rbuf) (void)hipFree(pp.rbuf);
  }
  for (auto &c : I.chans) {
    if (c.dbuf) (void)hipFree(c.dbuf);
    if (c.hbuf) (void)hipHostFree(c.hbuf);
    if (c.ipcEvent) (void)hipEventDestroy(c.ipcEvent);
    for (auto &r : c.ipcRetired) {
      if (r.fence) (void)hipEventDestroy(r.fence);
      (void)hipEventDestroy(r.event);
    }
    if (c.remoteFlag) (void)hipIpcCloseMemHandle(c.remoteFlag);
    if (c.remoteData) (void)hipIpcCloseMemHandle(c.remoteData);
  }
  // make sure peers closed their mappings of our blocks before freeing them; bounded, so a dead or stalled peer
  // cannot hold this rank in its destructor (the blocks then simply stay allocated until the process exits)
  bool peersDone = true;
  try {
    if (realized_ && pg_->size() > 1) peersDone = pg_->barrier_for(topt_.waitTimeout);
  } catch (...) {
    peersDone = false;
  }
  for (auto &c : I.chans) {
    if (!peersDone) break;
    if (c.ownFlag) (void)hipFree(c.ownFlag);
    if (c.ownData) (void)hipFree(c.ownData);
  }
  for (auto &d : I.devs) {
    d.translate.release();
    d.translateSkip.release();
    d.coloPack.release();
    d.coloPackLocal.release();
    for (int k = 0; k < 2; ++k) {
      d.pipePack[k].release();
      d.pipeUnpack[k].release();
    }
    if (d.syncCounter) (void)hipFree(d.syncCounter);
    if (d.xlog) (void)hipFree(d.xlog);
    d.coloUnpack.release();
    d.rcclPack.release();
    d.rcclUnpack.release();
    d.stagedPack.release();
    d.stagedUnpack.release();
    if (d.nccl) {
      if (poisoned_.empty())
        rccl::destroy(d.nccl);
      else
        rccl::abort(d.nccl);
    }
  }
  if (I.errHost) (void)hipHostFree(I.errHost);
  if (I.doneHost) (void)hipHostFree(I.doneHost);
}

int64_t DistributedDomain::add_data(int64_t elemSize, const std::string &name, DType dtype) {
  STENCIL_REQUIRE(!realized_, "add_data after realize");
  elemSize_.push_back(elemSize);
  names_.push_back(name);
  dtypes_.push_back(dtype);
  return int64_t(elemSize_.size()) - 1;
}


// ------------------------------------------------------------------------------------------------
// RCCL communicator (or the host-staged fallback)
// ------------------------------------------------------------------------------------------------
void DistributedDomain::init_rccl(const std::function<bool(int, int)> &sharedDev) {
  Impl &I = *impl_;
  comm::ProcGroup &pg = *pg_;
  const int myRank = pg.rank();
  int64_t rcclChans = 0;
  for (auto &c : I.chans) rcclChans += c.method == MethodFlags::Rccl;
  if (pg.allreduce_sum_u64(uint64_t(rcclChans)) == 0) return;
  TraceRange trr("rccl init");
  // members: every (rank, device) whose GPU no other rank drives (pairs touching a shared GPU are staged)
  const int nLocal = int(I.devs.size());
  std::vector<int> counts(size_t(pg.size()));
  pg.allgather(&nLocal, sizeof(int), counts.data());
  int maxN = 0;
  for (int c : counts) maxN = std::max(maxN, c);
  std::vector<int> padded(size_t(maxN), -1), allDevs(size_t(maxN) * size_t(pg.size()));
  for (int k = 0; k < nLocal; ++k)
    if (!sharedDev(myRank, I.devs[size_t(k)].dev)) padded[size_t(k)] = I.devs[size_t(k)].dev;
  pg.allgather(padded.data(), sizeof(int) * size_t(maxN), allDevs.data());
  // RCCL rank of (rank r, slot k) = number of members before it
  std::vector<int> ncclRankOf(allDevs.size(), -1);
  int total = 0, root = -1;
  for (int r = 0; r < pg.size(); ++r)
    for (int k = 0; k < maxN; ++k)
      if (allDevs[size_t(r) * size_t(maxN) + size_t(k)] >= 0) {
        ncclRankOf[size_t(r) * size_t(maxN) + size_t(k)] = total++;
        if (root < 0) root = r;
      }
  STENCIL_REQUIRE(root >= 0, "RCCL channels planned but no rank owns an exclusive GPU");

  // every failure is collected and agreed on before anyone falls back, so no rank is left blocked in a
  // communicator the others abandoned. The unique id travels with the root's status.
  std::string why;
  struct {
    int ok;
    rccl::UniqueId id;
  } boot{1, {}};
  if (myRank == root) {
    why = rccl::get_unique_id(&boot.id);
    boot.ok = why.empty();
  }
  pg.bcast(&boot, sizeof(boot), root);
  int ok = boot.ok && !topt_.failRcclInit;
  if (!boot.ok && why.empty()) why = "the root rank could not create an RCCL id";
  if (topt_.failRcclInit) why = "TransportOptions::failRcclInit";
  // local preconditions (the id, the forced-failure hook, every member device selectable) are agreed on BEFORE any
  // rank enters ncclCommInitRank: a rank that would skip or abort creation must not leave the others blocked inside
  // RCCL waiting for it. What remains is a failure inside RCCL itself, reported by the watch thread.
  for (int k = 0; k < nLocal && ok; ++k) {
    if (ncclRankOf[size_t(myRank) * size_t(maxN) + size_t(k)] < 0) continue;
    if (hipSetDevice(I.devs[size_t(k)].dev) != hipSuccess) {
      (void)hipGetLastError();
      ok = 0;
      why = "hipSetDevice(" + std::to_string(I.devs[size_t(k)].dev) + ") before RCCL init";
    }
  }
  if (pg.allreduce_min_i64(ok) != 1) {
    if (ok) why = "another rank cannot create its RCCL communicator";
    ok = 0;
  }
  if (ok) {
    // non-blocking creation polled against the wait timeout: a member that never joins (a rank died or stalled
    // between the bcast and here) costs every other member the timeout and an abort of its communicators, after which
    // the failure is agreed on below like any other -- never a hang inside RCCL
    std::vector<int> ranks, devices, slots;
    for (int k = 0; k < nLocal; ++k) {
      const int nr = ncclRankOf[size_t(myRank) * size_t(maxN) + size_t(k)];
      if (nr < 0) continue;
      ranks.push_back(nr);
      devices.push_back(I.devs[size_t(k)].dev);
      slots.push_back(k);
    }
    std::vector<rccl::Comm> comms;
    const double t0 = now_s();
    why = rccl::init_ranks(&comms, total, boot.id, ranks, devices, topt_.waitTimeout,
                           topt_.stallRcclInitRank == myRank);
    for (size_t j = 0; j < slots.size(); ++j) I.devs[size_t(slots[j])].nccl = comms[j];
    ok = why.empty();
    if (!ok)
      LOG_ERROR("RCCL communicator creation failed after " << now_s() - t0 << " s (" << why << "); plan:\n"
                                                           << plan_summary());
  }
  if (!ok) LOG_WARN("rank " << myRank << ": RCCL unavailable (" << why << ")");
  const bool allOk = pg.allreduce_min_i64(ok) == 1;
  rcclStatus_ = allOk ? "ok" : (ok ? "failed on another rank" : why);
  if (allOk) {
    // translate remote (rank, device) into RCCL ranks
    for (auto &c : I.chans) {
      if (c.method != MethodFlags::Rccl) continue;
      int peer = -1;
      for (int k = 0; k < maxN; ++k)
        if (allDevs[size_t(c.remoteRank) * size_t(maxN) + size_t(k)] == c.remoteDev)
          peer = ncclRankOf[size_t(c.remoteRank) * size_t(maxN) + size_t(k)];
      STENCIL_REQUIRE(peer >= 0, "RCCL peer device not found");
      STENCIL_REQUIRE(I.devs[size_t(I.devIndex[c.localDev])].nccl != nullptr, "RCCL channel on a shared GPU");
      c.ncclPeer = peer;
    }
    I.rccl = true;
    return;
  }
  // fallback: every RCCL channel (and plan entry) becomes host-staged on every rank
  for (auto &d : I.devs)
    if (d.nccl) {
      rccl::abort(d.nccl);
      d.nccl = nullptr;
    }
  if (myRank == 0) LOG_WARN("RCCL communicator creation failed on some rank; RCCL halos are host-staged instead");
  for (auto &c : I.chans)
    if (c.method == MethodFlags::Rccl) c.method = MethodFlags::Staged;
  for (auto &e : plan_)
    if (e.method == MethodFlags::Rccl) e.method = MethodFlags::Staged;
  flags_ = MethodFlags((int(flags_) & ~int(MethodFlags::Rccl)) | int(MethodFlags::Staged));
}

// ------------------------------------------------------------------------------------------------
// realize
// ------------------------------------------------------------------------------------------------
void DistributedDomain::realize() {
  STENCIL_REQUIRE(!realized_, "realize() called twice");
  STENCIL_REQUIRE(!elemSize_.empty(), "add_data() before realize()");
  TraceRange tr0("DistributedDomain::realize");
  Impl &I = *impl_;
  comm::ProcGroup &pg = *pg_;
  const int myRank = pg.rank();
  // setup timers (reference STENCIL_SETUP_STATS, stencil.cu:31-538): max over ranks, or local and collective-free
  // when the option is compiled out
  auto setup_time = [&](double local) { return STENCIL_SETUP_STATS ? pg.allreduce_max(local) : local; };

  if (!backendSet_) backend_ = gpu_topo::device_count() > 0 ? Backend::Device : Backend::Host;
  const bool dev = backend_ == Backend::Device;
  if (selfTest_ && pg.size() > 1) {
    // ladder: as configured -> without Colocated -> without Rccl (host-staged); the last rung always runs
    TraceRange trs("transport self-test");
    std::vector<MethodFlags> ladder{flags_};
    if (flags_ && MethodFlags::Colocated) ladder.push_back(MethodFlags(int(ladder.back()) & ~int(MethodFlags::Colocated)));
    if (ladder.back() && MethodFlags::Rccl)
      ladder.push_back(MethodFlags((int(ladder.back()) & ~int(MethodFlags::Rccl)) | int(MethodFlags::Staged)));
    std::ostringstream rep;
    bool found = false;
    for (size_t k = 0; k < ladder.size() && !found; ++k) {
      const int64_t bad = probe_transports(ladder[k]);
      rep << (k ? "; " : "") << to_string(ladder[k]) << ": " << (bad == 0 ? "ok" : std::to_string(bad) + " bad");
      if (bad == 0) {
        found = true;
        flags_ = ladder[k];
      }
    }
    selfTestReport_ = rep.str();
    if (myRank == 0) LOG_INFO("transport self-test: " << selfTestReport_);
    STENCIL_REQUIRE(found, "no transport set passed the self-test: " << selfTestReport_);
  }
  if (dev) STENCIL_REQUIRE(gpu_topo::device_count() > 0, "Device backend requested but no GPU is visible");

  // ---- node topology / GPU selection (reference stencil.hpp:158-245) ----
  double t0 = now_s();
  const int coloSize = pg.colocated_size();
  const int coloRank = pg.colocated_rank();
  timeMpiTopo_ = setup_time(now_s() - t0);
  t0 = now_s();
  if (gpus_.empty()) {
    if (dev) {
      const int n = gpu_topo::device_count();
      if (coloSize >= n) {
        gpus_ = {coloRank % n};
      } else {
        const int per = n / coloSize;
        for (int i = 0; i < per; ++i) gpus_.push_back(coloRank * per + i);
      }
    } else {
      gpus_ = {0};
    }
  }
  timeNodeGpus_ = setup_time(now_s() - t0);
  t0 = now_s();
  if (dev) {
    for (int a : gpus_)
      for (int b : gpus_)
        if (a != b) gpu_topo::enable_peer(a, b);
  }
  timePeerEn_ = setup_time(now_s() - t0);
  if (dev && topt_.numaAffinity) {
    int node = -2;
    for (int g : gpus_) {
      const int n = gpu_topo::numa_node(g);
      node = node == -2 ? n : (node == n ? node : -1);
    }
    if (node >= 0 && gpu_topo::bind_thread_to_numa(node)) {
      numaNode_ = node;
      LOG_DEBUG("rank " << myRank << " bound to NUMA node " << node << " of its GPU(s)");
    }
  }

  // ---- placement ----
  t0 = now_s();
  {
    TraceRange tr("placement");
    if (strategy_ == PlacementStrategy::NodeAware) {
      BandwidthFn bw = dev ? BandwidthFn([](int a, int b) { return gpu_topo::bandwidth(a, b); })
                           : BandwidthFn([](int a, int b) { return a == b ? 10.0 : 1.0; });
      placement_.reset(new NodeAwarePlacement(size_, pg, radius_, gpus_, bw, axisCost_, objective_));
    } else {
      placement_.reset(new TrivialPlacement(size_, pg, gpus_));
    }
  }
  timePlacement_ = setup_time(now_s() - t0);

  // ---- local domains ----
  t0 = now_s();
  domains_.reserve(gpus_.size());
  for (size_t di = 0; di < gpus_.size(); ++di) {
    const Dim3 idx = placement_->get_idx(myRank, int(di));
    const int device = placement_->get_device(idx);
    domains_.emplace_back(placement_->subdomain_size(idx), placement_->subdomain_origin(idx), dev ? device : -1, backend_);
    LocalDomain &d = domains_.back();
    d.set_radius(radius_);
    d.set_padding(pad_);
    d.set_x_halo_align(xHaloAlign_);
    d.set_shared_halo_line(sharedHaloLine_);
    d.set_interior_align(interiorAlign_);
    d.set_row_pad_lines(rowPadLines_);
    for (size_t q = 0; q < elemSize_.size(); ++q) d.add_data(elemSize_[q], names_[q], dtypes_[q]);
    LOG_INFO("rank " << myRank << " domain " << di << " idx " << idx << " size " << d.size() << " origin " << d.origin()
                     << " device " << device);
  }
  for (auto &d : domains_) d.realize();
  timeRealize_ = setup_time(now_s() - t0);

  // ---- HIP-IPC pre-flight: every rank maps a small uncached block of every co-located rank and reads it back.
  // If any mapping fails anywhere, Colocated is disabled on all ranks (they then agree on RCCL/staged). ----
  if (dev && any_methods(MethodFlags::Colocated) && pg.size() > 1 && pg.colocated_size() > 1 && topt_.ipcProbe) {
    TraceRange trp("ipc probe");
    // up to 3 collective attempts with a growing pause between them (50, 200 ms): a transient open/map failure on a
    // busy node must not cost the transport. Every failed attempt logs the call that failed on this rank.
    bool allOk = false;
    for (int attempt = 0; attempt < 3 && !allOk; ++attempt) {
      if (attempt > 0) std::this_thread::sleep_for(std::chrono::milliseconds(50 * (1 << (2 * (attempt - 1)))));
      int ok = 1;
      const char *failed = "";
      int failedPeer = -1;
      char *blk = nullptr;
      HIP_CHECK(hipSetDevice(gpus_[0]));
      if (hipExtMallocWithFlags((void **)&blk, 256, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        ok = 0;
        failed = "hipExtMallocWithFlags(uncached)";
      }
      hipIpcMemHandle_t mine{};
      if (ok && hipIpcGetMemHandle(&mine, blk) != hipSuccess) {
        (void)hipGetLastError();
        ok = 0;
        failed = "hipIpcGetMemHandle";
      }
      if (ok) {
        const uint64_t tag = 0x57e9c11000000000ull + uint64_t(myRank);
        HIP_CHECK(hipMemcpy(blk, &tag, sizeof(tag), hipMemcpyHostToDevice));
      }
      std::vector<hipIpcMemHandle_t> all(pg.size());
      pg.allgather(&mine, sizeof(mine), all.data());
      std::vector<int> oks(pg.size());
      pg.allgather(&ok, sizeof(int), oks.data());
      for (int r = 0; r < pg.size() && ok; ++r) {
        if (r == myRank || !pg.colocated(r) || !oks[r]) continue;
        char *peer = nullptr;
        if (hipIpcOpenMemHandle((void **)&peer, all[r], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
          (void)hipGetLastError();
          ok = 0;
          failed = "hipIpcOpenMemHandle";
          failedPeer = r;
          break;
        }
        uint64_t got = 0;
        if (hipMemcpy(&got, peer, sizeof(got), hipMemcpyDeviceToHost) != hipSuccess ||
            got != 0x57e9c11000000000ull + uint64_t(r)) {
          (void)hipGetLastError();
          ok = 0;
          failed = "readback of the mapped block";
          failedPeer = r;
        }
        (void)hipIpcCloseMemHandle(peer);
      }
      if (topt_.failIpcProbe) { // rehearses the fallback (tests)
        ok = 0;
        failed = "STENCIL_IPC_PROBE_FAIL";
      }
      if (!ok)
        LOG_INFO("IPC pre-flight attempt " << attempt + 1 << "/3 failed on rank " << myRank << ": " << failed
                                           << (failedPeer >= 0 ? " (peer rank " + std::to_string(failedPeer) + ")" : ""));
      allOk = pg.allreduce_min_i64(ok) == 1;
      pg.barrier(); // peers are done with our block
      if (blk) (void)hipFree(blk);
    }
    if (!allOk) {
      if (myRank == 0) LOG_WARN("HIP IPC between co-located ranks is unavailable; Colocated transport disabled");
      flags_ = MethodFlags(int(flags_) & ~int(MethodFlags::Colocated));
    }
  }

  // ---- physical device identity of every (rank, device ordinal): ranks may number devices differently, and RCCL
  // refuses a communicator in which two ranks drive one GPU. Pairs with an endpoint on a GPU that another rank of
  // the same host also drives never use RCCL (select_method); everything else keeps its transport. ----
  std::map<std::pair<int, int>, bool> sharedDev; // (rank, ordinal) -> GPU driven by another rank too
  if (dev && pg.size() > 1) {
    int nmine = int(gpus_.size()), maxN = 0;
    std::vector<int> counts(pg.size());
    pg.allgather(&nmine, sizeof(int), counts.data());
    for (int c : counts) maxN = std::max(maxN, c);
    struct DevId {
      int64_t ordinal;
      uint64_t bus;
    };
    std::vector<DevId> mine(size_t(maxN), DevId{-1, 0}), all(size_t(maxN) * pg.size());
    for (int k = 0; k < nmine; ++k) {
      char bus[64] = {0};
      HIP_CHECK(hipDeviceGetPCIBusId(bus, sizeof(bus), gpus_[size_t(k)]));
      mine[size_t(k)] = DevId{gpus_[size_t(k)], uint64_t(std::hash<std::string>()(std::string(bus)))};
    }
    pg.allgather(mine.data(), sizeof(DevId) * size_t(maxN), all.data());
    for (int r = 0; r < pg.size(); ++r)
      for (int k = 0; k < counts[r]; ++k) {
        const DevId &a = all[size_t(r) * maxN + k];
        bool sh = false;
        for (int r2 = 0; r2 < pg.size() && !sh; ++r2) {
          if (r2 == r || pg.hostname(r2) != pg.hostname(r)) continue;
          for (int k2 = 0; k2 < counts[r2]; ++k2) sh |= all[size_t(r2) * maxN + k2].bus == a.bus;
        }
        sharedDev[{r, int(a.ordinal)}] = sh;
      }
  }
  auto shared_dev = [&](int r, int ordinal) {
    auto it = sharedDev.find({r, ordinal});
    return it != sharedDev.end() && it->second;
  };

  // ---- plan messages (reference src/stencil.cu:132-239) ----
  t0 = now_s();
  const Dim3 gdim = placement_->dim();
  const int64_t numSub = gdim.flatten();
  auto can_access = [&](int a, int b) {
    if (a == b) return true;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return can != 0;
  };
  bool warnedShared = false;
  auto choose = [&](int srcRank, int srcDev, int dstRank, int dstDev) -> MethodFlags {
    const bool sameRank = srcRank == dstRank;
    PairInfo pi;
    pi.device = dev;
    pi.sameRank = sameRank;
    pi.sameDevice = srcDev == dstDev;
    pi.sameHost = pg.hostname(srcRank) == pg.hostname(dstRank);
    if (dev) {
      pi.peer = sameRank && gpu_topo::peer(srcDev, dstDev);
      pi.canAccess = !sameRank && pi.sameHost && (any_methods(MethodFlags::Colocated)) && can_access(srcDev, dstDev);
      pi.sharedGpu = !sameRank && (shared_dev(srcRank, srcDev) || shared_dev(dstRank, dstDev));
    }
    const MethodFlags m = select_method(flags_, pi);
    if (m == MethodFlags::Staged && pi.sharedGpu && any_methods(MethodFlags::Rccl) && !warnedShared) {
      warnedShared = true;
      LOG_WARN("rank " << srcRank << " dev " << srcDev << " -> rank " << dstRank << " dev " << dstDev
                       << ": a GPU driven by two ranks cannot use RCCL; host-staged for such pairs");
    }
    return m;
  };

  // channel maps: (method, localDom, remoteLinear) -> channel index
  std::map<std::tuple<int, int, int64_t>, int> sendKey, recvKey;
  std::vector<std::tuple<int, int, Dim3>> localTranslates; // (srcDom, dstDom, dir)
  std::map<std::pair<int, int>, std::vector<Message>> pipeMsgs; // PeerCopy over DMA engines: (srcDom, dstDom) -> msgs
  plan_.clear();
  remoteHalo_.assign(domains_.size(), std::array<uint8_t, 27>{});
  for (size_t di = 0; di < domains_.size(); ++di) {
    const Dim3 myIdx = placement_->get_idx(myRank, int(di));
    const int myDev = placement_->get_device(myIdx);
    for (int i = 0; i < 27; ++i) {
      const Dim3 dir = dir_from_index(i);
      if (dir == Dim3(0, 0, 0) || radius_.dir(-dir) == 0) continue;
      // send (nothing crosses a non-periodic face of the global grid)
      if (boundary_.reachable(myIdx, dir, gdim)) {
        const Dim3 dstIdx = (myIdx + dir).wrap(gdim);
        const int dstRank = placement_->get_rank(dstIdx), dstId = placement_->get_subdomain_id(dstIdx),
                  dstDev = placement_->get_device(dstIdx);
        const MethodFlags m = choose(myRank, myDev, dstRank, dstDev);
        if (m == MethodFlags::None) LOG_FATAL("no method available to send " << myIdx << " -> " << dstIdx << " dir " << dir);
        int64_t bytes = 0;
        for (int64_t q = 0; q < domains_[di].num_data(); ++q) bytes += domains_[di].halo_bytes(-dir, q);
        plan_.push_back({m, myIdx, dstIdx, myRank, dstRank, myDev, dstDev, dir, bytes});
        if (m == MethodFlags::PeerCopy && topt_.peerCopy == TransportOptions::Copy::Engine && dstId != int(di) && dev) {
          pipeMsgs[{int(di), dstId}].push_back(Message{dir, int(di), dstId});
        } else if (m == MethodFlags::Kernel || m == MethodFlags::PeerCopy) {
          localTranslates.emplace_back(int(di), dstId, dir);
        } else {
          const auto key = std::make_tuple(int(m), int(di), linearize(dstIdx, gdim));
          auto it = sendKey.find(key);
          int ci;
          if (it == sendKey.end()) {
            ci = int(I.chans.size());
            sendKey[key] = ci;
            Channel c;
            c.method = m;
            c.send = true;
            c.localDom = int(di);
            c.localIdx = myIdx;
            c.remoteIdx = dstIdx;
            c.remoteRank = dstRank;
            c.remoteId = dstId;
            c.remoteDev = dstDev;
            c.localDev = myDev;
            const int64_t sl = linearize(myIdx, gdim), dl = linearize(dstIdx, gdim);
            c.orderKey = sl * numSub + dl;
            c.tag = comm::make_tag(comm::MsgKind::Data, sl, dl, numSub);
            I.chans.push_back(c);
          } else {
            ci = it->second;
          }
          I.chans[ci].msgs.push_back(Message{dir, int(di), dstId});
        }
      }
      // recv
      if (boundary_.reachable(myIdx, -dir, gdim)) {
        const Dim3 srcIdx = (myIdx - dir).wrap(gdim);
        const int srcRank = placement_->get_rank(srcIdx), srcId = placement_->get_subdomain_id(srcIdx),
                  srcDev = placement_->get_device(srcIdx);
        const MethodFlags m = choose(srcRank, srcDev, myRank, myDev);
        if (m == MethodFlags::None) LOG_FATAL("no method available to recv " << srcIdx << " -> " << myIdx);
        // the halo on side -dir is valid after the same-device translate only for Kernel messages
        if (m != MethodFlags::Kernel) remoteHalo_[di][size_t(dir_index(-dir))] = 1;
        if (m == MethodFlags::Kernel || m == MethodFlags::PeerCopy) continue; // written by the sender directly
        const auto key = std::make_tuple(int(m), int(di), linearize(srcIdx, gdim));
        auto it = recvKey.find(key);
        int ci;
        if (it == recvKey.end()) {
          ci = int(I.chans.size());
          recvKey[key] = ci;
          Channel c;
          c.method = m;
          c.send = false;
          c.localDom = int(di);
          c.localIdx = myIdx;
          c.remoteIdx = srcIdx;
          c.remoteRank = srcRank;
          c.remoteId = srcId;
          c.remoteDev = srcDev;
          c.localDev = myDev;
          const int64_t sl = linearize(srcIdx, gdim), dl = linearize(myIdx, gdim);
          c.orderKey = sl * numSub + dl;
          c.tag = comm::make_tag(comm::MsgKind::Data, sl, dl, numSub);
          I.chans.push_back(c);
        } else {
          ci = it->second;
        }
        I.chans[ci].msgs.push_back(Message{dir, srcId, int(di)});
      }
    }
  }
  for (auto &c : I.chans) {
    std::sort(c.msgs.begin(), c.msgs.end());
    c.bytes = packed_size(domains_[c.localDom], c.msgs);
  }
  timePlan_ = setup_time(now_s() - t0);

  // ---- create transports ----
  t0 = now_s();
  TraceRange trc("DistributedDomain::realize: create");
  if (!dev) {
    // host backend: translate + staged only, all executed on the host
    for (const auto &t : localTranslates) {
      const LocalDomain &s = domains_[std::get<0>(t)], &d = domains_[std::get<1>(t)];
      for (int p = 0; p < 2; ++p)
        build_translate(s, d, std::get<2>(t), p == 0, I.hostTranslate.host[p], topt_.xFaceSectors);
    }
    for (auto &c : I.chans) {
      STENCIL_REQUIRE(c.method == MethodFlags::Staged, "host backend supports only Kernel/Staged transports");
      c.hostBuf.resize(size_t(std::max<int64_t>(c.bytes, 1)));
      for (int p = 0; p < 2; ++p) {
        if (c.send)
          build_pack(domains_[c.localDom], c.msgs, c.hostBuf.data(), p == 0, I.hostStagedPack.host[p]);
        else
          build_unpack(domains_[c.localDom], c.msgs, c.hostBuf.data(), p == 0, I.hostStagedUnpack.host[p]);
      }
    }
    I.hostTranslate.upload(-1);
    I.hostStagedPack.upload(-1);
    I.hostStagedUnpack.upload(-1);
  } else {
    // per-device contexts
    for (size_t di = 0; di < domains_.size(); ++di) {
      const int d = domains_[di].gpu();
      if (!I.devIndex.count(d)) {
        I.devIndex[d] = int(I.devs.size());
        I.devs.emplace_back();
        DevCtx &c = I.devs.back();
        c.dev = d;
        c.comm = Stream(d, Priority::HIGH);
        c.done = Event(d);
        c.translated = Event(d);
        if (!I.callerDone) I.callerDone = Event(d);
      }
      I.devs[I.devIndex[d]].doms.push_back(int(di));
      I.ready.emplace_back(d);
      I.readyPending.push_back(false);
    }
    HIP_CHECK(hipHostMalloc((void **)&I.errHost, sizeof(int), hipHostMallocMapped));
    *I.errHost = 0;
    HIP_CHECK(hipHostGetDevicePointer((void **)&I.errDev, I.errHost, 0));
    HIP_CHECK(hipHostMalloc((void **)&I.doneHost, sizeof(uint64_t) * I.devs.size(), hipHostMallocMapped));
    for (size_t k = 0; k < I.devs.size(); ++k) I.doneHost[k] = 0;
    HIP_CHECK(hipHostGetDevicePointer((void **)&I.doneDev, I.doneHost, 0));
    I.nullReady = Event(I.devs[0].dev);

    // RCCL communicator over all (rank, device) pairs, created only if some rank needs it. An init error on any
    // rank (or TransportOptions::failRcclInit) is agreed on collectively and every RCCL channel falls back to the
    // host-staged transport (the reference's ladder also ends at the MPI path, src/stencil.cu:185-194).
    init_rccl(shared_dev);

    // same-process direct stores; x faces as whole lines where asked for or where their lines outgrow the cache
    I.localTranslates = localTranslates;
    {
      std::map<int, int64_t> xLineBytes;
      for (const auto &t : localTranslates) {
        const LocalDomain &s = domains_[std::get<0>(t)];
        const Dim3 dir = std::get<2>(t);
        if (dir.x != 0 && dir.y == 0 && dir.z == 0 && s.gpu() == domains_[std::get<1>(t)].gpu())
          xLineBytes[s.gpu()] += s.size().y * s.size().z * s.num_data() * 192;
      }
      for (auto &kv : xLineBytes)
        if (topt_.xFaceSectors || (topt_.xFaceLinesAutoBytes > 0 && kv.second >= topt_.xFaceLinesAutoBytes))
          I.xLineDevs.insert(kv.first);
      if (!I.xLineDevs.empty() && !topt_.xFaceSectors)
        LOG_DEBUG("x faces as whole lines (auto) on " << I.xLineDevs.size() << " device(s)");
    }
    for (const auto &t : localTranslates) {
      const LocalDomain &s = domains_[std::get<0>(t)], &d = domains_[std::get<1>(t)];
      DevCtx &ctx = I.devs[I.devIndex[s.gpu()]];
      const bool lines = x_face_lines(s, d);
      for (int p = 0; p < 2; ++p) build_translate(s, d, std::get<2>(t), p == 0, ctx.translate.host[p], lines);
      if (d.gpu() != s.gpu()) I.devs[I.devIndex[d.gpu()]].peerWriters.insert(s.gpu());
    }
    for (auto &kv : pipeMsgs) {
      PeerPipe pp;
      pp.srcDom = kv.first.first;
      pp.dstDom = kv.first.second;
      pp.srcDev = domains_[size_t(pp.srcDom)].gpu();
      pp.dstDev = domains_[size_t(pp.dstDom)].gpu();
      pp.msgs = kv.second;
      std::sort(pp.msgs.begin(), pp.msgs.end());
      pp.bytes[0] = pp.bytes[1] = packed_size(domains_[size_t(pp.srcDom)], pp.msgs);
      const size_t nb = size_t(std::max<int64_t>(pp.bytes[0], 1));
      HIP_CHECK(hipSetDevice(pp.srcDev));
      HIP_CHECK(hipMalloc(&pp.sbuf, nb));
      HIP_CHECK(hipSetDevice(pp.dstDev));
      HIP_CHECK(hipMalloc(&pp.rbuf, nb));
      const int k = int(I.pipes.size());
      DevCtx &sc = I.devs[size_t(I.devIndex[pp.srcDev])];
      DevCtx &dc = I.devs[size_t(I.devIndex[pp.dstDev])];
      sc.pipesOut.push_back(k);
      dc.pipesIn.push_back(k);
      for (int p = 0; p < 2; ++p) {
        build_pack(domains_[size_t(pp.srcDom)], pp.msgs, pp.sbuf, p == 0, sc.pipePack[0].host[p]);
        build_unpack(domains_[size_t(pp.dstDom)], pp.msgs, pp.rbuf, p == 0, dc.pipeUnpack[0].host[p]);
      }
      I.pipes.push_back(std::move(pp));
    }
    for (auto &ctx : I.devs) {
      ctx.sharedGpu = shared_dev(myRank, ctx.dev);
      ctx.pipePack[0].upload(ctx.dev);
      ctx.pipeUnpack[0].upload(ctx.dev);
      if (!ctx.pipesOut.empty()) ctx.pipeSent = Event(ctx.dev);
      if (!ctx.pipesIn.empty()) ctx.pipeUnpacked = Event(ctx.dev);
      HIP_CHECK(hipSetDevice(ctx.dev));
      HIP_CHECK(hipMalloc(&ctx.syncCounter, 2 * sizeof(uint32_t)));
      HIP_CHECK(hipMemset(ctx.syncCounter, 0, 2 * sizeof(uint32_t)));
    }
    // copy streams for DMA-engine copies are created on first use (forked_copies): every stream can take a hardware
    // queue, and ranks that share a GPU slow down by orders of magnitude once their queues oversubscribe the
    // device (profiles/r3/cliff/)

    // channel buffers
    for (int ci = 0; ci < int(I.chans.size()); ++ci) {
      Channel &c = I.chans[ci];
      DevCtx &ctx = I.devs[I.devIndex[c.localDev]];
      HIP_CHECK(hipSetDevice(c.localDev));
      const size_t nb = size_t(std::max<int64_t>(c.bytes, 1));
      if (c.method == MethodFlags::Staged) {
        HIP_CHECK(hipMalloc(&c.dbuf, nb));
        // pinned on the GPU's NUMA node when realize() bound this thread there (pages follow the thread's policy)
        HIP_CHECK(hipHostMalloc((void **)&c.hbuf, nb, numaNode_ >= 0 ? hipHostMallocNumaUser : hipHostMallocDefault));
        (c.send ? ctx.stagedSend : ctx.stagedRecv).push_back(ci);
      } else if (c.method == MethodFlags::Rccl) {
        HIP_CHECK(hipMalloc(&c.dbuf, nb));
        (c.send ? ctx.rcclSend : ctx.rcclRecv).push_back(ci);
      } else if (c.method == MethodFlags::Colocated) {
        // flag words (arrival on the receiver, credit on the sender) in uncached memory: polled across processes
        // and GPUs, written remotely
        HIP_CHECK(hipExtMallocWithFlags((void **)&c.ownFlag, 256, hipDeviceMallocUncached));
        HIP_CHECK(hipMemset(c.ownFlag, 0, 256));
        c.slotStride = round_up(int64_t(nb), 256);
        if (!c.send) {
          const size_t dataBytes = size_t(2 * c.slotStride);
          switch (topt_.inbox) {
          case TransportOptions::Inbox::Uncached:
            HIP_CHECK(hipExtMallocWithFlags((void **)&c.ownData, dataBytes, hipDeviceMallocUncached));
            break;
          case TransportOptions::Inbox::Fine:
            HIP_CHECK(hipExtMallocWithFlags((void **)&c.ownData, dataBytes, hipDeviceMallocFinegrained));
            break;
          case TransportOptions::Inbox::Coarse:
            HIP_CHECK(hipMalloc((void **)&c.ownData, dataBytes));
            break;
          }
          HIP_CHECK(hipMemset(c.ownData, 0, dataBytes));
        } else {
          HIP_CHECK(hipMalloc(&c.dbuf, nb)); // Engine copies: the packed message before the DMA copy
        }
        (c.send ? ctx.coloSend : ctx.coloRecv).push_back(ci);
      }
    }
    HIP_CHECK(hipDeviceSynchronize());

    // IPC handshake for colocated channels: every side sends its handles first (non-blocking), then receives.
    // receiver -> sender: {arrival flag block, data block}; sender -> receiver: {credit flag block}
    {
      TraceRange tri("ipc handshake");
      for (auto &c : I.chans) {
        if (c.method != MethodFlags::Colocated) continue;
        hipIpcMemHandle_t h[2] = {};
        HIP_CHECK(hipSetDevice(c.localDev));
        HIP_CHECK(hipIpcGetMemHandle(&h[0], c.ownFlag));
        if (!c.send) HIP_CHECK(hipIpcGetMemHandle(&h[1], c.ownData));
        pg.send(c.remoteRank, retag(c.tag, c.send ? comm::MsgKind::IpcCredit : comm::MsgKind::IpcInbox), h,
                c.send ? sizeof(h[0]) : sizeof(h));
      }
      for (auto &c : I.chans) {
        if (c.method != MethodFlags::Colocated) continue;
        hipIpcMemHandle_t h[2] = {};
        // a sender needs the receiver's flag + data blocks, a receiver the sender's credit block
        pg.recv(c.remoteRank, retag(c.tag, c.send ? comm::MsgKind::IpcInbox : comm::MsgKind::IpcCredit), h,
                c.send ? sizeof(h) : sizeof(h[0]));
        HIP_CHECK(hipSetDevice(c.localDev));
        HIP_CHECK(hipIpcOpenMemHandle((void **)&c.remoteFlag, h[0], hipIpcMemLazyEnablePeerAccess));
        if (c.send) HIP_CHECK(hipIpcOpenMemHandle((void **)&c.remoteData, h[1], hipIpcMemLazyEnablePeerAccess));
      }
      // Completion::IpcEvent: sender -> receiver, the handle of the sender's interprocess event per channel
      if (topt_.completion == TransportOptions::Completion::IpcEvent) {
        for (auto &c : I.chans) {
          if (c.method != MethodFlags::Colocated || !c.send) continue;
          HIP_CHECK(hipSetDevice(c.localDev));
          HIP_CHECK(hipEventCreateWithFlags(&c.ipcEvent, hipEventDisableTiming | hipEventInterprocess));
          hipIpcEventHandle_t h{};
          HIP_CHECK(hipIpcGetEventHandle(&h, c.ipcEvent));
          pg.send(c.remoteRank, retag(c.tag, comm::MsgKind::IpcEvent), &h, sizeof(h));
        }
        for (auto &c : I.chans) {
          if (c.method != MethodFlags::Colocated || c.send) continue;
          hipIpcEventHandle_t h{};
          pg.recv(c.remoteRank, retag(c.tag, comm::MsgKind::IpcEvent), &h, sizeof(h));
          HIP_CHECK(hipSetDevice(c.localDev));
          HIP_CHECK(hipIpcOpenEventHandle(&c.ipcEvent, h));
        }
        I.ipcEvents = true;
        I.ipcEventFirstEpoch = 1;
      }
      pg.barrier();
    }

    // segment lists per device
    for (auto &ctx : I.devs) {
      for (int ci : ctx.coloSend) {
        Channel &c = I.chans[ci];
        const LocalDomain &dom = domains_[c.localDom];
        for (int p = 0; p < 2; ++p) {
          for (int slot = 0; slot < 2; ++slot)
            build_pack(dom, c.msgs, c.remoteData + slot * c.slotStride, p == 0, ctx.coloPack.host[p * 2 + slot]);
          build_pack(dom, c.msgs, c.dbuf, p == 0, ctx.coloPackLocal.host[p]);
        }
      }
      for (int ci : ctx.coloRecv) {
        Channel &c = I.chans[ci];
        const LocalDomain &dom = domains_[c.localDom];
        for (int p = 0; p < 2; ++p)
          for (int slot = 0; slot < 2; ++slot)
            build_unpack(dom, c.msgs, c.ownData + slot * c.slotStride, p == 0, ctx.coloUnpack.host[p * 2 + slot]);
      }
      for (int ci : ctx.rcclSend)
        for (int p = 0; p < 2; ++p)
          build_pack(domains_[I.chans[ci].localDom], I.chans[ci].msgs, I.chans[ci].dbuf, p == 0, ctx.rcclPack.host[p]);
      for (int ci : ctx.rcclRecv)
        for (int p = 0; p < 2; ++p)
          build_unpack(domains_[I.chans[ci].localDom], I.chans[ci].msgs, I.chans[ci].dbuf, p == 0, ctx.rcclUnpack.host[p]);
      for (int ci : ctx.stagedSend)
        for (int p = 0; p < 2; ++p)
          build_pack(domains_[I.chans[ci].localDom], I.chans[ci].msgs, I.chans[ci].dbuf, p == 0, ctx.stagedPack.host[p]);
      for (int ci : ctx.stagedRecv)
        for (int p = 0; p < 2; ++p)
          build_unpack(domains_[I.chans[ci].localDom], I.chans[ci].msgs, I.chans[ci].dbuf, p == 0,
                       ctx.stagedUnpack.host[p]);
      ctx.translate.upload(ctx.dev);
      ctx.coloPack.upload(ctx.dev);
      ctx.coloPackLocal.upload(ctx.dev);
      ctx.coloUnpack.upload(ctx.dev);
      ctx.rcclPack.upload(ctx.dev);
      ctx.rcclUnpack.upload(ctx.dev);
      ctx.stagedPack.upload(ctx.dev);
      ctx.stagedUnpack.upload(ctx.dev);
      // RCCL matching order: canonical (src, dst) sub-domain order on both sides of every pair
      auto byKey = [&](int a, int b) { return I.chans[a].orderKey < I.chans[b].orderKey; };
      std::sort(ctx.rcclSend.begin(), ctx.rcclSend.end(), byKey);
      std::sort(ctx.rcclRecv.begin(), ctx.rcclRecv.end(), byKey);
    }

  }
  // bytes per method (after any RCCL -> staged fallback) and the plan file
  bytesPerMethod_ = {};
  for (const auto &e : plan_) bytesPerMethod_[size_t(method_slot(e.method))] += uint64_t(e.bytes);
  for (int m = 0; m < 5; ++m) bytesPerMethod_[size_t(m)] = pg.allreduce_sum_u64(bytesPerMethod_[size_t(m)]);
  if (!planPrefix_.empty()) {
    std::ofstream f(planPrefix_ + "_" + std::to_string(myRank) + ".txt");
    f << plan_summary();
  }
  timeCreate_ = setup_time(now_s() - t0);
  realized_ = true;
  pg.barrier();
}

std::string DistributedDomain::plan_summary() const {
  std::ostringstream ss;
  ss << "rank=" << rank() << "\n\n== domains ==\n";
  for (size_t di = 0; di < domains_.size(); ++di)
    ss << di << ":dev" << domains_[di].gpu() << ":" << placement_->get_idx(rank(), int(di)) << " sz=" << domains_[di].size()
       << " origin=" << domains_[di].origin() << "\n";
  const MethodFlags order[] = {MethodFlags::Kernel, MethodFlags::PeerCopy, MethodFlags::Colocated, MethodFlags::Rccl,
                               MethodFlags::Staged};
  for (MethodFlags m : order) {
    ss << "\n== " << to_string(m) << " ==\n";
    for (const auto &e : plan_)
      if (e.method == m)
        ss << e.srcIdx << "(r" << e.srcRank << " dev" << e.srcDev << ") -> " << e.dstIdx << "(r" << e.dstRank << " dev"
           << e.dstDev << ") dir=" << e.dir << " " << e.bytes << "B\n";
  }
  ss << "\n== bytes per exchange (all ranks) ==\n";
  for (MethodFlags m : order) ss << to_string(m) << " " << bytesPerMethod_[method_slot(m)] << "\n";
  return ss.str();
}

std::vector<ForwardTarget> DistributedDomain::forward_targets(size_t di) const {
  STENCIL_REQUIRE(realized_, "forward_targets before realize()");
  const Dim3 myIdx = placement_->get_idx(rank(), int(di));
  const Dim3 gdim = placement_->dim();
  const LocalDomain &src = domains_.at(di);
  std::vector<ForwardTarget> out;
  for (const auto &e : plan_) {
    if (e.srcIdx != myIdx || (e.method != MethodFlags::Kernel && e.method != MethodFlags::PeerCopy)) continue;
    const LocalDomain &dst = domains_.at(size_t(placement_->get_subdomain_id(e.dstIdx)));
    // global coordinate of the receiving halo cell = sender's cell - wrap, where wrap = +-global size when the
    // step crosses the periodic boundary
    const Dim3 step = myIdx + e.dir;
    Dim3 wrap(0, 0, 0);
    wrap.x = step.x >= gdim.x ? size_.x : (step.x < 0 ? -size_.x : 0);
    wrap.y = step.y >= gdim.y ? size_.y : (step.y < 0 ? -size_.y : 0);
    wrap.z = step.z >= gdim.z ? size_.z : (step.z < 0 ? -size_.z : 0);
    out.push_back(ForwardTarget{e.dir, &dst, src.accessor_origin() - dst.accessor_origin() - wrap});
  }
  return out;
}

uint64_t DistributedDomain::exchange_bytes_for_method(MethodFlags m) const {
  uint64_t r = 0;
  const MethodFlags all[] = {MethodFlags::Staged, MethodFlags::Rccl, MethodFlags::Colocated, MethodFlags::PeerCopy,
                             MethodFlags::Kernel};
  for (MethodFlags f : all)
    if (m && f) r += bytesPerMethod_[method_slot(f)];
  return r;
}

// ------------------------------------------------------------------------------------------------
// interior / exterior (reference src/stencil.cu:567-666)
// ------------------------------------------------------------------------------------------------
std::vector<Rect3> DistributedDomain::get_interior() const {
  std::vector<Rect3> ret(domains_.size());
  for (size_t di = 0; di < domains_.size(); ++di) {
    const Rect3 com = domains_[di].get_compute_region();
    Rect3 in = com;
    for (int i = 0; i < 27; ++i) {
      const Dim3 d = dir_from_index(i);
      if (d == Dim3(0, 0, 0)) continue;
      const int64_t r = radius_.dir(d);
      if (d.x < 0) in.lo.x = std::max(com.lo.x + r, in.lo.x);
      if (d.x > 0) in.hi.x = std::min(com.hi.x - r, in.hi.x);
      if (d.y < 0) in.lo.y = std::max(com.lo.y + r, in.lo.y);
      if (d.y > 0) in.hi.y = std::min(com.hi.y - r, in.hi.y);
      if (d.z < 0) in.lo.z = std::max(com.lo.z + r, in.lo.z);
      if (d.z > 0) in.hi.z = std::min(com.hi.z - r, in.hi.z);
    }
    ret[di] = in;
  }
  return ret;
}

std::vector<Rect3> DistributedDomain::get_local_interior(int reach) const {
  STENCIL_REQUIRE(realized_, "get_local_interior before realize()");
  std::vector<Rect3> ret(domains_.size());
  for (size_t di = 0; di < domains_.size(); ++di) {
    const Rect3 com = domains_[di].get_compute_region();
    const auto &rh = remoteHalo_[di];
    // shrink[axis][side]: cells to drop at the low (0) / high (1) face of each axis
    int64_t sh[3][2] = {{0, 0}, {0, 0}, {0, 0}};
    auto comp = [](const Dim3 &d, int a) { return a == 0 ? d.x : (a == 1 ? d.y : d.z); };
    // remote faces: the stencil reaches `reach` cells along an axis
    for (int i = 0; i < 27; ++i) {
      const Dim3 d = dir_from_index(i);
      const int nz = (d.x != 0) + (d.y != 0) + (d.z != 0);
      if (nz != 1 || !rh[size_t(i)]) continue;
      for (int a = 0; a < 3; ++a)
        if (comp(d, a) != 0) sh[a][comp(d, a) > 0] = std::max<int64_t>(sh[a][comp(d, a) > 0], std::min<int64_t>(reach, radius_.dir(d)));
    }
    // remote edges / corners: a cell reads them only when it is within reach of all their faces at once, so one
    // shrunk face among them covers the rest; with none, drop every face of the direction (conservative)
    for (int i = 0; i < 27; ++i) {
      const Dim3 d = dir_from_index(i);
      const int nz = (d.x != 0) + (d.y != 0) + (d.z != 0);
      if (nz < 2 || !rh[size_t(i)] || radius_.dir(d) == 0) continue;
      bool covered = false;
      for (int a = 0; a < 3; ++a)
        if (comp(d, a) != 0 && sh[a][comp(d, a) > 0] > 0) covered = true;
      if (covered) continue;
      for (int a = 0; a < 3; ++a)
        if (comp(d, a) != 0) sh[a][comp(d, a) > 0] = std::max<int64_t>(sh[a][comp(d, a) > 0], 1);
    }
    // measurement knob: treat the faces of these axes (mask 1=x, 2=y, 4=z) as remote, so one GPU runs the split
    // (local interior during the transfers, slabs after) of a multi-GPU decomposition
    if (topt_.fakeRemoteAxes != 0)
      for (int a = 0; a < 3; ++a)
        if (topt_.fakeRemoteAxes >> a & 1)
          for (int s = 0; s < 2; ++s) {
            const Dim3 d(a == 0 ? 2 * s - 1 : 0, a == 1 ? 2 * s - 1 : 0, a == 2 ? 2 * s - 1 : 0);
            sh[a][s] = std::max<int64_t>(sh[a][s], std::min<int64_t>(reach, radius_.dir(d)));
          }
    Rect3 in = com;
    in.lo.x += sh[0][0];
    in.hi.x -= sh[0][1];
    in.lo.y += sh[1][0];
    in.hi.y -= sh[1][1];
    in.lo.z += sh[2][0];
    in.hi.z -= sh[2][1];
    if (in.hi.x < in.lo.x || in.hi.y < in.lo.y || in.hi.z < in.lo.z) in = Rect3(com.lo, com.lo);
    ret[di] = in;
  }
  return ret;
}

std::vector<std::vector<Rect3>> DistributedDomain::get_exterior() const {
  std::vector<std::vector<Rect3>> ret(domains_.size());
  const auto ins = get_interior();
  for (size_t di = 0; di < domains_.size(); ++di) {
    const Rect3 &in = ins[di];
    Rect3 c = domains_[di].get_compute_region();
    if (in.hi.x != c.hi.x) {
      ret[di].push_back(Rect3(Dim3(in.hi.x, c.lo.y, c.lo.z), c.hi));
      c.hi.x = in.hi.x;
    }
    if (in.hi.y != c.hi.y) {
      ret[di].push_back(Rect3(Dim3(c.lo.x, in.hi.y, c.lo.z), c.hi));
      c.hi.y = in.hi.y;
    }
    if (in.hi.z != c.hi.z) {
      ret[di].push_back(Rect3(Dim3(c.lo.x, c.lo.y, in.hi.z), c.hi));
      c.hi.z = in.hi.z;
    }
    if (in.lo.x != c.lo.x) {
      ret[di].push_back(Rect3(c.lo, Dim3(in.lo.x, c.hi.y, c.hi.z)));
      c.lo.x = in.lo.x;
    }
    if (in.lo.y != c.lo.y) {
      ret[di].push_back(Rect3(c.lo, Dim3(c.hi.x, in.lo.y, c.hi.z)));
      c.lo.y = in.lo.y;
    }
    if (in.lo.z != c.lo.z) {
      ret[di].push_back(Rect3(c.lo, Dim3(c.hi.x, c.hi.y, in.lo.z)));
      c.lo.z = in.lo.z;
    }
  }
  return ret;
}

} // namespace stencil
