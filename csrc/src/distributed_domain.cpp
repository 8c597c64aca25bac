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

#define RCCL_CHECK(stmt)                                                                                           \
  do {                                                                                                             \
    const std::string _e = (stmt);                                                                                 \
    if (!_e.empty()) LOG_FATAL("RCCL error (" << _e << ") in `" #stmt "`");                                        \
  } while (0)

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

static int method_slot(MethodFlags m) {
  switch (m) {
  case MethodFlags::Staged:
    return 0;
  case MethodFlags::Rccl:
    return 1;
  case MethodFlags::Colocated:
    return 2;
  case MethodFlags::PeerCopy:
    return 3;
  case MethodFlags::Kernel:
    return 4;
  default:
    LOG_FATAL("not a single method: " << int(m));
  }
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------------------------------------
// internal state
// ------------------------------------------------------------------------------------------------

// segment list with up to 4 variants (domain parity x inbox slot), host copies and device copy plans
struct SegList {
  std::vector<CopySeg> host[4];
  CopyPlan plan[4];
  bool empty() const { return host[0].empty() && host[1].empty() && host[2].empty() && host[3].empty(); }
  void upload(int device) {
    for (int v = 0; v < 4; ++v) {
      finalize_segs(host[v]);
      if (device >= 0 && !host[v].empty()) {
        HIP_CHECK(hipSetDevice(device));
        plan[v] = make_copy_plan(host[v], device);
      }
    }
  }
  void run_device(int v, hipStream_t s, int maxBlocks = 0) const { copy_plan_device(plan[v], s, maxBlocks); }
  void run_device_sync(int v, hipStream_t s, int maxBlocks, const FlagSyncArgs &a) const {
    copy_plan_device_sync(plan[v], s, maxBlocks, a);
  }
  void run_host(int v) const { copy_segs_host(host[v]); }
  void release() {
    for (auto &p : plan) free_copy_plan(p);
  }
};

// same (src, dst) pair key, different kind
static uint32_t retag(uint32_t tag, comm::MsgKind kind) {
  return comm::make_tag(kind, comm::tag_payload(tag));
}

struct Channel {
  MethodFlags method = MethodFlags::None;
  bool send = true;
  int localDom = -1;
  Dim3 localIdx, remoteIdx;
  int remoteRank = -1, remoteId = -1, remoteDev = -1;
  int localDev = -1;
  std::vector<Message> msgs; // sorted by dir
  int64_t bytes = 0;         // packed bytes (reference wire layout)
  uint32_t tag = 0;     // host-plane tag (comm::make_tag(Data, src, dst))
  int ncclPeer = -1;    // RCCL rank of the remote (rank, device)
  int64_t orderKey = 0; // canonical (src, dst) order for RCCL matching
  char *dbuf = nullptr; // device staging buffer (Rccl, Staged)
  char *hbuf = nullptr; // pinned host (Staged, device backend)
  std::vector<char> hostBuf; // host backend
  // Colocated (IPC): the receiver owns a flag block [arrived word] and a data block [slot0 | slot1] (memory kind
  // TransportOptions::inbox), the sender a flag block [credit word]; flag blocks are always uncached. remote* are
  // the opened IPC mappings of the peer's blocks. Engine copies stage the packed message in dbuf (sender's GPU).
  char *ownFlag = nullptr, *ownData = nullptr;
  char *remoteFlag = nullptr, *remoteData = nullptr;
  int64_t slotStride = 0;
  // Completion::IpcEvent: the sender's interprocess event (send channel) / the opened peer event (receive channel),
  // the records / waits it has served, and replaced events kept until no wait can still reference them
  hipEvent_t ipcEvent = nullptr;
  int ipcUses = 0;
  std::deque<std::pair<hipEvent_t, uint64_t>> ipcRetired; // (event, epoch it was replaced at)
};

// HIP (ROCm 7.2) refuses hipStreamWaitEvent on an opened interprocess event after 32 records of it ("invalid
// argument" on the 33rd wait; hipEventSynchronize keeps working: `ipc_event_stress`, profiles/r4/ipcevent/). The
// sender therefore replaces a channel's event after this many records and ships the new handle with the Notify.
constexpr int kIpcEventUses = 24;
struct IpcNotify {
  uint64_t epoch = 0;
  uint64_t fresh = 0; // 1: `handle` is the channel's new event from this epoch on
  hipIpcEventHandle_t handle{};
};
// a replaced event is destroyed once this many more exchanges have passed (at most two are ever in flight)
constexpr uint64_t kIpcRetireEpochs = 8;

// PeerCopy over a DMA engine (TransportOptions::peerCopy == Engine): every message from one local sub-domain to
// another (on a peer GPU of this process) is packed into sbuf on the source GPU, copied by hipMemcpyPeerAsync into
// rbuf on the destination GPU and unpacked there (reference PeerCopySender, tx_cuda.cuh:106-170)
struct PeerPipe {
  int srcDom = -1, dstDom = -1, srcDev = -1, dstDev = -1;
  std::vector<Message> msgs; // sorted by dir
  char *sbuf = nullptr, *rbuf = nullptr;
  int64_t bytes[2] = {0, 0}; // packed bytes: all messages / without the directions prepare_skip_wrapped leaves out
};

struct DevCtx {
  int dev = -1;
  Stream comm;
  Event done, translated;
  bool translateEmpty = false; // the last exchange_async translated nothing on this device
  std::vector<int> doms;
  SegList translate;              // Kernel + PeerCopy originating here (variant = parity)
  SegList translateSkip;          // same without the directions crossing Impl::skipAxes (prepare_skip_wrapped)
  std::set<int> peerWriters;      // devices whose translate writes into this device
  std::vector<int> coloSend, coloRecv, rcclSend, rcclRecv, stagedSend, stagedRecv;
  SegList coloPack, coloUnpack;   // variant = parity*2 + slot
  SegList coloPackLocal;          // Engine copies: pack into the channels' local staging buffers (variant = parity)
  // PeerCopy pipes leaving / entering this device ([0] all messages, [1] the prepare_skip_wrapped subset)
  std::vector<int> pipesOut, pipesIn;
  SegList pipePack[2], pipeUnpack[2];
  Event pipeSent, pipeUnpacked;
  // DMA-engine copies to different peers run concurrently: copies on one stream would execute one after another,
  // so each peer's copy is forked onto its own copy stream (copy k of an exchange on copyStreams[k % n]) and joined
  Event copyFork;
  std::vector<Stream> copyStreams;
  std::vector<Event> copyJoin;
  uint32_t *syncCounter = nullptr; // [0] colo send, [1] colo receive: block counters of the fused transport kernels
  bool sharedGpu = false;          // another rank drives this GPU too (fused transport kernels stay capped)
  uint64_t *xlog = nullptr;        // set_transport_log: kTransportLogWords stamps per exchange, a ring of xlogCap
  SegList rcclPack, rcclUnpack;   // variant = parity
  SegList stagedPack, stagedUnpack;
  rccl::Comm nccl = nullptr;
};

struct DistributedDomain::Impl {
  std::vector<Channel> chans;
  std::vector<DevCtx> devs;            // device backend: one per distinct local device
  std::map<int, int> devIndex;         // device id -> index into devs
  std::vector<Event> ready;            // per local domain
  std::vector<bool> readyPending;
  uint64_t epoch = 0;
  int *errHost = nullptr; // host-mapped timeout word
  int *errDev = nullptr;
  uint64_t *doneHost = nullptr; // host-mapped epoch word per device (TransportOptions::spinWait)
  uint64_t *doneDev = nullptr;
  Event nullReady;              // TransportOptions::nullStreamProducers
  // host backend
  SegList hostTranslate, hostStagedPack, hostStagedUnpack;
  bool rccl = false;
  std::vector<std::tuple<int, int, Dim3>> localTranslates; // (srcDom, dstDom, dir) of the Kernel/PeerCopy messages
  std::vector<PeerPipe> pipes;                               // PeerCopy messages over DMA engines (see PeerPipe)
  int skipAxes = 0;                                         // axes translateSkip leaves out (0 = not prepared)
  // exchanges enqueued on a caller stream (single device) vs on the comm stream: each kind waits for the last
  // exchange of the other kind, so the two never race on the IPC inbox slots / flags, and sync_exchange() also
  // waits for (and then checks the timeout word of) the last caller-stream exchange
  Event callerDone;
  bool callerPending = false; // callerDone marks a caller-stream exchange not yet joined by sync_exchange
  bool commPending = false;   // the comm stream holds an exchange (devs[0].done) a caller stream has not waited for
  bool engineRefused = false; // hipMemcpyDeviceToDeviceNoCU not accepted by the runtime (warned once)
  uint64_t *gateCounter = nullptr; // set_send_gate: consumed by the next exchange_async
  uint64_t gateTarget = 0;
  bool ipcEvents = false;            // Completion::IpcEvent events were created by realize()
  uint64_t ipcEventFirstEpoch = 0;  // first exchange in IpcEvent mode since the last set_completion (acks before it
                                    // were never sent)
  int xlogCap = 0;                  // set_transport_log ring size (exchanges)
  uint64_t xlogFirstEpoch = 0;      // first epoch logged since the last set_transport_log
};

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
    for (auto &r : c.ipcRetired) (void)hipEventDestroy(r.first);
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
// segment builders (reference wire layout: messages sorted by dir, each quantity aligned to its element size,
// reference packer.cuh:136-160)
// ------------------------------------------------------------------------------------------------
static void build_pack(const LocalDomain &dom, const std::vector<Message> &msgs, char *buf, bool curr,
                       std::vector<CopySeg> &out) {
  build_pack_segs(dom, msgs, buf, curr, out);
}
static void build_unpack(const LocalDomain &dom, const std::vector<Message> &msgs, char *buf, bool curr,
                         std::vector<CopySeg> &out) {
  build_unpack_segs(dom, msgs, buf, curr, out);
}
static void build_translate(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, bool curr,
                            std::vector<CopySeg> &out, bool xSectors = false) {
  build_translate_segs(src, dst, dir, curr, out, xSectors);
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
    // a communicator that never forms (a rank died between the bcast and here) blocks in RCCL itself: say so
    // with the plan after the wait timeout instead of hanging silently
    std::mutex mu;
    std::condition_variable cv;
    bool initDone = false;
    std::thread watch([&] {
      std::unique_lock<std::mutex> lk(mu);
      if (!cv.wait_for(lk, std::chrono::duration<double>(topt_.waitTimeout), [&] { return initDone; }))
        LOG_ERROR("RCCL communicator creation still running after " << topt_.waitTimeout << " s; plan:\n"
                                                                      << plan_summary());
    });
    std::vector<int> ranks, devices, slots;
    for (int k = 0; k < nLocal; ++k) {
      const int nr = ncclRankOf[size_t(myRank) * size_t(maxN) + size_t(k)];
      if (nr < 0) continue;
      ranks.push_back(nr);
      devices.push_back(I.devs[size_t(k)].dev);
      slots.push_back(k);
    }
    std::vector<rccl::Comm> comms;
    why = rccl::init_ranks(&comms, total, boot.id, ranks, devices);
    for (size_t j = 0; j < slots.size(); ++j) I.devs[size_t(slots[j])].nccl = comms[j];
    {
      std::lock_guard<std::mutex> lk(mu);
      initDone = true;
    }
    cv.notify_all();
    watch.join();
    ok = why.empty();
  }
  if (!ok) LOG_WARN("rank " << myRank << ": RCCL unavailable (" << why << ")");
  if (pg.allreduce_min_i64(ok) == 1) {
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

    // same-process direct stores
    I.localTranslates = localTranslates;
    for (const auto &t : localTranslates) {
      const LocalDomain &s = domains_[std::get<0>(t)], &d = domains_[std::get<1>(t)];
      DevCtx &ctx = I.devs[I.devIndex[s.gpu()]];
      for (int p = 0; p < 2; ++p) build_translate(s, d, std::get<2>(t), p == 0, ctx.translate.host[p], topt_.xFaceSectors);
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

// ------------------------------------------------------------------------------------------------
// exchange
// ------------------------------------------------------------------------------------------------
void DistributedDomain::record_ready(size_t di, hipStream_t s) {
  STENCIL_REQUIRE(realized_, "record_ready before realize");
  if (backend_ != Backend::Device) return;
  impl_->ready.at(di).record(s);
  impl_->readyPending[di] = true;
}

void DistributedDomain::wait_translated(size_t di, hipStream_t s) {
  if (backend_ != Backend::Device) return;
  const DevCtx &ctx = impl_->devs[impl_->devIndex.at(domains_.at(di).gpu())];
  // nothing translated on this device (every same-GPU halo wrapped in-kernel, the rest remote): the caller's stream
  // already orders everything the local interior reads, so skip the cross-stream hop (~10 us per exchange)
  if (ctx.translateEmpty) return;
  ctx.translated.wait_on(s);
}

void DistributedDomain::wait_exchange(size_t di, hipStream_t s) {
  if (backend_ != Backend::Device) return;
  const DevCtx &ctx = impl_->devs[impl_->devIndex.at(domains_.at(di).gpu())];
  ctx.done.wait_on(s);
}

hipStream_t DistributedDomain::comm_stream(size_t di) const {
  if (backend_ != Backend::Device) return nullptr;
  return impl_->devs[impl_->devIndex.at(domains_.at(di).gpu())].comm;
}

void DistributedDomain::sync_exchange() { sync_streams({}); }

void DistributedDomain::sync_streams(const std::vector<hipStream_t> &extra) {
  if (backend_ != Backend::Device) return;
  Impl &I = *impl_;
  STENCIL_REQUIRE(poisoned_.empty(), "halo exchange unusable after an earlier failure: " << poisoned_);
  auto fail = [&](const std::string &why) {
    poison(why);
    for (auto &d : I.devs)
      if (d.nccl) {
        rccl::abort(d.nccl);
        d.nccl = nullptr;
      }
    I.rccl = false;
    LOG_FATAL(why);
  };
  // Every device-side wait of the IPC path is bounded by default (spin kernels stop after waitTimeout and report
  // through errHost), so a blocking synchronize always returns. RCCL operations and command-processor waits are
  // not: then poll the streams, check every communicator's asynchronous error, and give up after the wait timeout
  // with the plan on stderr (a peer that died or never posted its matching send/recv would otherwise block here
  // forever) -- including the caller's compute streams, which join the exchange.
  const bool unbounded = I.rccl || topt_.completion != TransportOptions::Completion::Kernel;
  if (unbounded) {
    const double t0 = now_s();
    auto pending = [&](hipError_t q) {
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        return true;
      }
      HIP_CHECK(q);
      return false;
    };
    auto done = [&]() {
      for (hipStream_t st : extra)
        if (pending(hipStreamQuery(st))) return false;
      for (auto &d : I.devs) {
        HIP_CHECK(hipSetDevice(d.dev));
        if (pending(hipStreamQuery(d.comm))) return false;
      }
      return !(I.callerPending && pending(hipEventQuery(I.callerDone)));
    };
    while (!done()) {
      for (auto &d : I.devs) {
        if (!d.nccl) continue;
        const std::string ae = rccl::async_error(d.nccl);
        if (!ae.empty()) {
          LOG_ERROR("RCCL " << ae << " error on device " << d.dev << "\n"
                                                          << plan_summary());
          fail("halo exchange failed in RCCL (epoch " + std::to_string(I.epoch) + ")");
        }
      }
      if (*I.errHost) break; // a bounded device wait gave up: reported below
      if (now_s() - t0 > topt_.waitTimeout) {
        LOG_ERROR("halo exchange still running after " << topt_.waitTimeout << " s (epoch " << I.epoch
                                                        << "); plan:\n" << plan_summary());
        fail("halo exchange timed out; a peer rank is stalled or dead");
      }
      std::this_thread::yield();
    }
  }
  if (!*I.errHost) {
    for (hipStream_t st : extra) HIP_CHECK(hipStreamSynchronize(st));
    for (auto &d : I.devs) {
      HIP_CHECK(hipSetDevice(d.dev));
      HIP_CHECK(hipStreamSynchronize(d.comm));
    }
    if (I.callerPending) {
      I.callerDone.sync();
      I.callerPending = false;
    }
  }
  if (*I.errHost) {
    const int code = *I.errHost;
    LOG_ERROR("halo exchange timed out waiting for a colocated peer (" << (code == 1 ? "inbox credit" : "arrival")
                                                                      << ", epoch " << I.epoch << "); plan:\n"
                                                                      << plan_summary());
    fail("halo exchange timed out waiting for a colocated peer; a peer rank is stalled or dead");
  }
}

void DistributedDomain::set_colo_copy(TransportOptions::Copy c) {
  if (c == topt_.coloCopy) return;
  if (realized_) sync_exchange(); // the staging buffers and inbox slots of the exchanges in flight
  topt_.coloCopy = c;
  // back to pack-kernel stores with no DMA-engine pipes left: drop the copy streams the engine copies created.
  // Every stream may take a hardware queue of its own, and a process whose streams outnumber its queues
  // multiplexes them (4 ranks sharing one MI355X after a warm-up that tried engine copies: 2.94 ms per step
  // instead of 0.52, profiles/r3/check3)
  if (realized_ && backend_ == Backend::Device && c == TransportOptions::Copy::Store && impl_->pipes.empty())
    for (auto &ctx : impl_->devs) {
      for (auto &s : ctx.copyStreams) s.sync();
      ctx.copyStreams.clear();
      ctx.copyJoin.clear();
      ctx.copyFork = Event();
    }
}

void DistributedDomain::set_transport_options_live(const TransportOptions &o) {
  if (!realized_) {
    set_transport_options(o);
    return;
  }
  STENCIL_REQUIRE(o.inbox == topt_.inbox && o.peerCopy == topt_.peerCopy,
                  "inbox memory and the peer-copy path are fixed at realize()");
  set_colo_copy(o.coloCopy);
  set_completion(o.completion);
  topt_.spinWait = o.spinWait;
  topt_.fuseFlags = o.fuseFlags; // flag words are monotonic epochs: either form continues where the other left off
  topt_.nullStreamProducers = o.nullStreamProducers;
  topt_.jitterUs = o.jitterUs;
  if (o.waitTimeout > 0) topt_.waitTimeout = o.waitTimeout;
  topt_.fakeRemoteAxes = o.fakeRemoteAxes;
}

void DistributedDomain::set_completion(TransportOptions::Completion c) {
  if (c == topt_.completion) return;
  STENCIL_REQUIRE(!realized_ || c != TransportOptions::Completion::IpcEvent || impl_->ipcEvents ||
                      exchange_bytes_for_method(MethodFlags::Colocated) == 0,
                  "Completion::IpcEvent needs its interprocess events: realize() with that completion");
  if (realized_) sync_exchange(); // flag words are monotonic epochs: either method continues where the other left off
  Impl &I = *impl_;
  if (realized_ && topt_.completion == TransportOptions::Completion::IpcEvent && backend_ == Backend::Device) {
    // leaving IpcEvent: take the acknowledgements of the last two exchanges that no later record will consume, so a
    // later switch back finds no stale Ack queued
    for (auto &ctx : I.devs)
      for (int ci : ctx.coloSend) {
        Channel &ch = I.chans[size_t(ci)];
        for (uint64_t e = I.epoch >= 1 ? I.epoch - 1 : 0; e <= I.epoch; ++e) {
          if (e == 0 || e < I.ipcEventFirstEpoch) continue;
          uint64_t acked = 0;
          pg_->recv(ch.remoteRank, retag(ch.tag, comm::MsgKind::Ack), &acked, sizeof(acked));
          STENCIL_REQUIRE(acked == e, "IPC-event ack out of order: got epoch " << acked << ", want " << e);
        }
      }
  }
  topt_.completion = c;
  // every rank switches between the same two exchanges: acknowledgements exist from the next epoch on
  if (c == TransportOptions::Completion::IpcEvent) I.ipcEventFirstEpoch = I.epoch + 1;
}

const char *to_string(TransportOptions::Inbox v) {
  switch (v) {
  case TransportOptions::Inbox::Uncached:
    return "uncached";
  case TransportOptions::Inbox::Fine:
    return "fine";
  case TransportOptions::Inbox::Coarse:
    return "coarse";
  }
  return "?";
}
const char *to_string(TransportOptions::Copy v) { return v == TransportOptions::Copy::Engine ? "engine" : "store"; }
const char *to_string(TransportOptions::Completion v) {
  switch (v) {
  case TransportOptions::Completion::StreamOp:
    return "streamop";
  case TransportOptions::Completion::IpcEvent:
    return "ipcevent";
  default:
    return "kernel";
  }
}

void DistributedDomain::exchange() {
  double t0 = 0;
  if (exchangeStats_) {
    pg_->barrier();
    t0 = now_s();
  }
  exchange_async();
  Impl &I = *impl_;
  if (backend_ == Backend::Device && topt_.spinWait && I.doneHost) {
    // every comm stream ends with a store of this epoch into a host-mapped word; spin (bounded) until all landed,
    // so the synchronize below finds the streams complete instead of sleeping until its wake-up
    for (size_t k = 0; k < I.devs.size(); ++k) {
      HIP_CHECK(hipSetDevice(I.devs[k].dev));
      signal_flags_device({I.doneDev + k}, I.epoch, I.devs[k].comm);
    }
    const double ts = now_s();
    for (size_t k = 0; k < I.devs.size(); ++k)
      while (__atomic_load_n(&I.doneHost[k], __ATOMIC_ACQUIRE) < I.epoch && *I.errHost == 0 &&
             now_s() - ts < topt_.waitTimeout) {
      }
  }
  sync_exchange();
  if (exchangeStats_) timeExchange_ += pg_->allreduce_max(now_s() - t0);
}

int DistributedDomain::self_wrap_axes() const {
  STENCIL_REQUIRE(realized_, "self_wrap_axes before realize");
  const Dim3 gdim = placement_->dim();
  const int64_t n[3] = {gdim.x, gdim.y, gdim.z};
  int m = 0;
  for (int ax = 0; ax < 3; ++ax) {
    const int64_t d[3] = {ax == 0, ax == 1, ax == 2};
    if (n[ax] == 1 && boundary_.face_periodic(int(d[0]), int(d[1]), int(d[2])) &&
        boundary_.face_periodic(-int(d[0]), -int(d[1]), -int(d[2])))
      m |= 1 << ax;
  }
  return m;
}

void DistributedDomain::prepare_skip_wrapped(int axes) {
  STENCIL_REQUIRE(realized_, "prepare_skip_wrapped before realize");
  STENCIL_REQUIRE((axes & ~self_wrap_axes()) == 0,
                  "axes " << axes << " are not self-periodic (self_wrap_axes = " << self_wrap_axes() << ")");
  Impl &I = *impl_;
  if (axes == I.skipAxes || backend_ == Backend::Host) return;
  for (auto &ctx : I.devs) {
    ctx.translateSkip.release();
    ctx.translateSkip = SegList();
  }
  for (const auto &t : I.localTranslates) {
    const Dim3 dir = std::get<2>(t);
    if (((axes & 1) && dir.x != 0) || ((axes & 2) && dir.y != 0) || ((axes & 4) && dir.z != 0)) continue;
    const LocalDomain &sd = domains_[std::get<0>(t)], &dd = domains_[std::get<1>(t)];
    DevCtx &ctx = I.devs[I.devIndex[sd.gpu()]];
    for (int p = 0; p < 2; ++p) build_translate(sd, dd, dir, p == 0, ctx.translateSkip.host[p], topt_.xFaceSectors);
  }
  for (auto &ctx : I.devs) ctx.translateSkip.upload(ctx.dev);
  // PeerCopy pipes: the same subset, packed compactly
  for (auto &ctx : I.devs) {
    ctx.pipePack[1].release();
    ctx.pipePack[1] = SegList();
    ctx.pipeUnpack[1].release();
    ctx.pipeUnpack[1] = SegList();
  }
  for (auto &pp : I.pipes) {
    std::vector<Message> keep;
    for (const Message &mm : pp.msgs) {
      const Dim3 dir = mm.dir;
      if (((axes & 1) && dir.x != 0) || ((axes & 2) && dir.y != 0) || ((axes & 4) && dir.z != 0)) continue;
      keep.push_back(mm);
    }
    pp.bytes[1] = keep.empty() ? 0 : packed_size(domains_[size_t(pp.srcDom)], keep);
    if (keep.empty()) continue;
    DevCtx &sc = I.devs[size_t(I.devIndex[pp.srcDev])];
    DevCtx &dc = I.devs[size_t(I.devIndex[pp.dstDev])];
    for (int p = 0; p < 2; ++p) {
      build_pack(domains_[size_t(pp.srcDom)], keep, pp.sbuf, p == 0, sc.pipePack[1].host[p]);
      build_unpack(domains_[size_t(pp.dstDom)], keep, pp.rbuf, p == 0, dc.pipeUnpack[1].host[p]);
    }
  }
  for (auto &ctx : I.devs) {
    ctx.pipePack[1].upload(ctx.dev);
    ctx.pipeUnpack[1].upload(ctx.dev);
  }
  I.skipAxes = axes;
}

void DistributedDomain::set_transport_log(int exchanges) {
  STENCIL_REQUIRE(realized_, "set_transport_log before realize");
  if (backend_ != Backend::Device) return;
  Impl &I = *impl_;
  sync_exchange();
  for (auto &ctx : I.devs) {
    HIP_CHECK(hipSetDevice(ctx.dev));
    if (ctx.xlog) (void)hipFree(ctx.xlog);
    ctx.xlog = nullptr;
    if (exchanges > 0) {
      const size_t nb = sizeof(uint64_t) * size_t(exchanges) * kTransportLogWords;
      HIP_CHECK(hipMalloc((void **)&ctx.xlog, nb));
      HIP_CHECK(hipMemset(ctx.xlog, 0, nb));
    }
  }
  HIP_CHECK(hipDeviceSynchronize());
  I.xlogCap = std::max(0, exchanges);
  I.xlogFirstEpoch = I.epoch + 1;
}

std::vector<std::array<uint64_t, kTransportLogWords>> DistributedDomain::transport_log(size_t dev) {
  STENCIL_REQUIRE(realized_, "transport_log before realize");
  Impl &I = *impl_;
  std::vector<std::array<uint64_t, kTransportLogWords>> out;
  if (backend_ != Backend::Device || I.xlogCap == 0 || dev >= I.devs.size()) return out;
  sync_exchange();
  DevCtx &ctx = I.devs[dev];
  std::vector<std::array<uint64_t, kTransportLogWords>> ring(size_t(I.xlogCap));
  HIP_CHECK(hipSetDevice(ctx.dev));
  HIP_CHECK(hipMemcpy(ring.data(), ctx.xlog, sizeof(uint64_t) * kTransportLogWords * ring.size(), hipMemcpyDeviceToHost));
  // oldest first: the last min(cap, logged) epochs
  const uint64_t last = I.epoch, first = std::max(I.xlogFirstEpoch, last >= uint64_t(I.xlogCap) ? last - I.xlogCap + 1 : 1);
  for (uint64_t e = first; e <= last && e >= I.xlogFirstEpoch; ++e) out.push_back(ring[size_t((e - 1) % uint64_t(I.xlogCap))]);
  return out;
}

void DistributedDomain::set_send_gate(uint64_t *counter, uint64_t target) {
  STENCIL_REQUIRE(realized_, "set_send_gate before realize");
  impl_->gateCounter = counter;
  impl_->gateTarget = target;
}

bool DistributedDomain::gated_send_supported(int skipAxes) const {
  if (!realized_ || backend_ != Backend::Device) return false;
  const Impl &I = *impl_;
  if (I.devs.size() != 1 || !I.pipes.empty() || I.rccl) return false;
  const DevCtx &ctx = I.devs[0];
  if (skipAxes != 0 && skipAxes != I.skipAxes) return false;
  const SegList &tl = skipAxes != 0 ? ctx.translateSkip : ctx.translate;
  if (!tl.host[0].empty() || !tl.host[1].empty()) return false;
  if (!ctx.stagedSend.empty() || !ctx.stagedRecv.empty() || !ctx.rcclSend.empty() || !ctx.rcclRecv.empty())
    return false;
  return !ctx.coloSend.empty() && topt_.coloCopy == TransportOptions::Copy::Store && topt_.fuseFlags &&
         topt_.completion == TransportOptions::Completion::Kernel;
}

void DistributedDomain::exchange_async(hipStream_t stream, int skipAxes) {
  STENCIL_REQUIRE(realized_, "exchange before realize");
  STENCIL_REQUIRE(poisoned_.empty(), "halo exchange unusable after an earlier failure: " << poisoned_);
  TraceRange tr("DD::exchange()");
  Impl &I = *impl_;
  STENCIL_REQUIRE(skipAxes == 0 || backend_ == Backend::Host || skipAxes == I.skipAxes,
                  "exchange_async(skipAxes=" << skipAxes << ") without prepare_skip_wrapped(" << skipAxes << ")");
  comm::ProcGroup &pg = *pg_;
  const int parity = domains_.empty() ? 0 : domains_[0].parity();
  for (auto &d : domains_) STENCIL_REQUIRE(d.parity() == parity, "local domains out of swap() lockstep");
  ++I.epoch;

  if (backend_ == Backend::Host) {
    {
      TraceRange t("host translate");
      I.hostTranslate.run_host(parity);
    }
    TraceRange t("host staged");
    I.hostStagedPack.run_host(parity);
    for (auto &c : I.chans)
      if (c.send) pg.send(c.remoteRank, c.tag, c.hostBuf.data(), size_t(c.bytes));
    for (auto &c : I.chans)
      if (!c.send) pg.recv(c.remoteRank, c.tag, c.hostBuf.data(), size_t(c.bytes));
    I.hostStagedUnpack.run_host(parity);
    return;
  }

  // a caller-provided stream replaces the comm stream (single device): the exchange is then ordered by that
  // stream alone, with no cross-stream events
  const bool over = stream != nullptr && I.devs.size() == 1;
  auto S = [&](DevCtx &c) -> hipStream_t { return over ? stream : c.comm.get(); };
  // hand-offs between caller-stream and comm-stream exchanges (events are not used while `stream` is being
  // captured into a hipGraph: the graph is ordered by that stream alone)
  bool capturing = false;
  if (over) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_CHECK(hipStreamIsCapturing(stream, &cs));
    capturing = cs != hipStreamCaptureStatusNone;
  }
  if (over && !capturing) {
    HIP_CHECK(hipSetDevice(I.devs[0].dev));
    if (I.commPending) I.devs[0].done.wait_on(stream);
    I.commPending = false;
  } else if (!over && I.callerPending) {
    HIP_CHECK(hipSetDevice(I.devs[0].dev));
    I.callerDone.wait_on(I.devs[0].comm);
  }

  // a producer gate replaces the wait for the producers' kernels (set_send_gate)
  const bool gated = I.gateCounter != nullptr;
  uint64_t *gateCounter = I.gateCounter;
  const uint64_t gateTarget = I.gateTarget;
  I.gateCounter = nullptr;
  if (gated)
    STENCIL_REQUIRE(!over && gated_send_supported(skipAxes), "gated exchange without a fused co-located-only plan");
  // (0) dependencies: the comm streams start after every local domain's producer work
  if (!over && !gated) {
    bool anyMissing = false;
    for (size_t di = 0; di < domains_.size(); ++di) anyMissing |= !I.readyPending[di];
    if (anyMissing && topt_.nullStreamProducers && I.devs.size() == 1) {
      // producers on the null stream / blocking streams: order after them without a host round trip
      HIP_CHECK(hipSetDevice(I.devs[0].dev));
      I.nullReady.record(nullptr);
      I.nullReady.wait_on(S(I.devs[0]));
    } else if (anyMissing) {
      for (auto &d : I.devs) {
        HIP_CHECK(hipSetDevice(d.dev));
        HIP_CHECK(hipDeviceSynchronize());
      }
    }
    for (auto &ctx : I.devs) {
      HIP_CHECK(hipSetDevice(ctx.dev));
      for (size_t di = 0; di < domains_.size(); ++di)
        if (I.readyPending[di]) I.ready[di].wait_on(S(ctx));
    }
    for (size_t di = 0; di < domains_.size(); ++di) I.readyPending[di] = false;
  } else {
    for (size_t di = 0; di < domains_.size(); ++di) I.readyPending[di] = false;
  }

  const int slot = int(I.epoch & 1);
  const int cv = parity * 2 + slot;
  // Colocated completion (TransportOptions::completion): bounded spin / release kernels, or command-processor
  // stream operations on the same flag words
  const bool streamOps = topt_.completion == TransportOptions::Completion::StreamOp;
  // interprocess events + host notify / ack for arrival, credit flags inside the (always fused) transport kernels
  const bool ipcEvt = topt_.completion == TransportOptions::Completion::IpcEvent;
  STENCIL_REQUIRE(!ipcEvt || !capturing, "Completion::IpcEvent exchanges cannot be captured into a hipGraph");
  // Colocated flag waits / signals folded into the pack and unpack kernels (TransportOptions::fuseFlags)
  const bool fused = !streamOps && !ipcEvt && topt_.fuseFlags;
  auto wait_flags = [&](const std::vector<uint64_t *> &flags, uint64_t target, int code, hipStream_t st) {
    if (!streamOps) {
      wait_flags_device(flags, target, I.errDev, code, topt_.waitTimeout, st);
      return;
    }
    for (uint64_t *f : flags) HIP_CHECK(hipStreamWaitValue64(st, f, target, hipStreamWaitValueGte));
  };
  auto signal_flags = [&](const std::vector<uint64_t *> &flags, uint64_t value, hipStream_t st) {
    if (!streamOps) {
      signal_flags_device(flags, value, st);
      return;
    }
    for (uint64_t *f : flags) HIP_CHECK(hipStreamWriteValue64(st, f, value, 0));
  };
  // DMA-engine copy (no CUs); falls back to an ordinary device copy if the runtime refuses the NoCU kind
  auto engine_copy = [&](void *dst, const void *src, size_t n, hipStream_t st) {
    if (!I.engineRefused) {
      const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDeviceNoCU, st);
      if (e == hipSuccess) return;
      (void)hipGetLastError();
      I.engineRefused = true;
      LOG_WARN("hipMemcpyDeviceToDeviceNoCU refused (" << hipGetErrorString(e) << "); engine copies use hipMemcpyDeviceToDevice");
    }
    HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st));
  };
  // run copies[k] (k = 0..n-1) behind the work on `st`, on the device's copy streams when it has them (concurrent
  // DMA engines / links), and make `st` wait for all of them
  auto forked_copies = [&](DevCtx &ctx, hipStream_t st, int n, const std::function<void(int, hipStream_t)> &copy) {
    if (!over && n > 1 && ctx.copyStreams.empty()) { // first engine copies of this device: its copy streams
      ctx.copyFork = Event(ctx.dev);
      for (int k = 0; k < std::min(4, n); ++k) {
        ctx.copyStreams.emplace_back(ctx.dev, Priority::HIGH);
        ctx.copyJoin.emplace_back(ctx.dev);
      }
    }
    const bool fork = !over && ctx.copyStreams.size() > 1 && n > 1;
    if (!fork) {
      for (int k = 0; k < n; ++k) copy(k, st);
      return;
    }
    ctx.copyFork.record(st);
    const int ns = std::min(n, int(ctx.copyStreams.size()));
    for (int j = 0; j < ns; ++j) ctx.copyFork.wait_on(ctx.copyStreams[size_t(j)]);
    for (int k = 0; k < n; ++k) copy(k, ctx.copyStreams[size_t(k % ns)]);
    for (int j = 0; j < ns; ++j) {
      ctx.copyJoin[size_t(j)].record(ctx.copyStreams[size_t(j)]);
      ctx.copyJoin[size_t(j)].wait_on(st);
    }
  };
  // STENCIL_JITTER_US=N: sleep a random 0..N us between transport phases (reference's unused rand_sleep(),
  // packer.cuh:17-20) to shake out ordering assumptions between ranks and streams
  const int jitterUs = topt_.jitterUs;
  auto jitter = [&] {
    if (jitterUs > 0) std::this_thread::sleep_for(std::chrono::microseconds(std::rand() % (jitterUs + 1)));
  };

  // (1) same-process direct stores (Kernel + PeerCopy)
  for (auto &ctx : I.devs) {
    HIP_CHECK(hipSetDevice(ctx.dev));
    TraceRange t("kernel/peer translate");
    const SegList &tl = skipAxes != 0 ? ctx.translateSkip : ctx.translate;
    ctx.translateEmpty = tl.host[parity].empty();
    if (!ctx.translateEmpty) tl.run_device(parity, S(ctx));
    if (!over) ctx.translated.record(S(ctx)); // events only matter across streams
  }

  // (1b) PeerCopy over DMA engines: pack on the source GPU, one peer copy per pipe, unpack on the destination
  //      GPU once the copies into it have landed; a receive buffer is overwritten only after its previous unpack
  if (!I.pipes.empty()) {
    TraceRange t("peer copy (engine)");
    const int pv = skipAxes != 0 ? 1 : 0;
    for (auto &ctx : I.devs) {
      if (ctx.pipesOut.empty()) continue;
      HIP_CHECK(hipSetDevice(ctx.dev));
      ctx.pipePack[pv].run_device(parity, S(ctx), commBlocks_);
      std::set<int> dsts;
      for (int k : ctx.pipesOut) dsts.insert(I.pipes[size_t(k)].dstDev);
      if (!over && I.epoch > 1)
        for (int d : dsts) I.devs[size_t(I.devIndex[d])].pipeUnpacked.wait_on(S(ctx));
      forked_copies(ctx, S(ctx), int(ctx.pipesOut.size()), [&](int j, hipStream_t cs) {
        const PeerPipe &pp = I.pipes[size_t(ctx.pipesOut[size_t(j)])];
        const size_t nb = size_t(pp.bytes[pv]);
        if (nb == 0) return;
        if (pp.srcDev == pp.dstDev && !topt_.peerApiSameDevice)
          engine_copy(pp.rbuf, pp.sbuf, nb, cs);
        else
          HIP_CHECK(hipMemcpyPeerAsync(pp.rbuf, pp.dstDev, pp.sbuf, pp.srcDev, nb, cs));
      });
      if (!over) ctx.pipeSent.record(S(ctx));
    }
    for (auto &ctx : I.devs) {
      if (ctx.pipesIn.empty()) continue;
      HIP_CHECK(hipSetDevice(ctx.dev));
      if (!over) {
        std::set<int> srcs;
        for (int k : ctx.pipesIn) srcs.insert(I.pipes[size_t(k)].srcDev);
        for (int d : srcs) I.devs[size_t(I.devIndex[d])].pipeSent.wait_on(S(ctx));
      }
      ctx.pipeUnpack[pv].run_device(parity, S(ctx), commBlocks_);
      if (!over) ctx.pipeUnpacked.record(S(ctx));
    }
  }

  jitter();
  // (2) colocated sends: wait for inbox credit (slot reuse distance 2), move the packed message into the peer's
  //     inbox over xGMI, then raise the peer's arrival flag.
  //     Store:  the pack kernel stores straight into the IPC-mapped inbox slot.
  //     Engine: pack into the local staging buffer (before the credit wait: it does not touch the inbox), then one
  //             DMA-engine copy per channel into the slot, leaving the CUs to the compute sweep.
  for (auto &ctx : I.devs) {
    if (ctx.coloSend.empty()) continue;
    HIP_CHECK(hipSetDevice(ctx.dev));
    TraceRange t("colo send");
    const bool engine = topt_.coloCopy == TransportOptions::Copy::Engine;
    std::vector<uint64_t *> credits, arrived;
    if (I.epoch > 2)
      for (int ci : ctx.coloSend) credits.push_back(reinterpret_cast<uint64_t *>(I.chans[ci].ownFlag));
    for (int ci : ctx.coloSend) arrived.push_back(reinterpret_cast<uint64_t *>(I.chans[ci].remoteFlag));
    if (ipcEvt) {
      // credit wait fused into the pack (or before the engine copies), then per channel: the receiver's Ack of
      // epoch-2 (its wait on the previous-but-one record is enqueued), record, Notify
      FlagSyncArgs fa;
      fa.err = I.errDev;
      fa.code = 1;
      fa.timeout_s = topt_.waitTimeout;
      fa.sharedGpu = ctx.sharedGpu;
      fa.counter = ctx.syncCounter;
      if (engine) {
        ctx.coloPackLocal.run_device(parity, S(ctx), commBlocks_);
        if (!credits.empty()) wait_flags(credits, I.epoch - 2, 1, S(ctx));
        forked_copies(ctx, S(ctx), int(ctx.coloSend.size()), [&](int k, hipStream_t cs) {
          const Channel &c = I.chans[size_t(ctx.coloSend[size_t(k)])];
          if (c.bytes > 0) engine_copy(c.remoteData + slot * c.slotStride, c.dbuf, size_t(c.bytes), cs);
        });
      } else {
        fa.wait = credits;
        fa.waitTarget = I.epoch - 2;
        if (ctx.xlog) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords;
        ctx.coloPack.run_device_sync(cv, S(ctx), commBlocks_, fa);
      }
      for (int ci : ctx.coloSend) {
        Channel &c = I.chans[size_t(ci)];
        if (I.epoch >= I.ipcEventFirstEpoch + 2) {
          uint64_t acked = 0;
          pg.recv(c.remoteRank, retag(c.tag, comm::MsgKind::Ack), &acked, sizeof(acked));
          STENCIL_REQUIRE(acked == I.epoch - 2, "IPC-event ack out of order: got epoch " << acked << ", want "
                                                                                          << I.epoch - 2);
        }
        IpcNotify msg;
        msg.epoch = I.epoch;
        if (c.ipcUses >= kIpcEventUses) { // a fresh event before HIP's per-event record limit
          c.ipcRetired.emplace_back(c.ipcEvent, I.epoch);
          HIP_CHECK(hipEventCreateWithFlags(&c.ipcEvent, hipEventDisableTiming | hipEventInterprocess));
          HIP_CHECK(hipIpcGetEventHandle(&msg.handle, c.ipcEvent));
          msg.fresh = 1;
          c.ipcUses = 0;
        }
        while (!c.ipcRetired.empty() && I.epoch - c.ipcRetired.front().second >= kIpcRetireEpochs) {
          (void)hipEventDestroy(c.ipcRetired.front().first);
          c.ipcRetired.pop_front();
        }
        HIP_CHECK(hipEventRecord(c.ipcEvent, S(ctx)));
        ++c.ipcUses;
        pg.send(c.remoteRank, retag(c.tag, comm::MsgKind::Notify), &msg, sizeof(msg));
      }
      continue;
    }
    if (!engine && fused) { // one launch: credit wait, pack into the peer slots, arrival flags
      FlagSyncArgs fa;
      fa.wait = credits;
      fa.waitTarget = I.epoch - 2;
      if (gated) {
        fa.gate = {gateCounter};
        fa.gateTarget = gateTarget;
      }
      fa.signal = arrived;
      fa.signalValue = I.epoch;
      fa.counter = ctx.syncCounter;
      fa.err = I.errDev;
      fa.code = 1;
      fa.timeout_s = topt_.waitTimeout;
      fa.sharedGpu = ctx.sharedGpu;
      if (ctx.xlog) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords;
      ctx.coloPack.run_device_sync(cv, S(ctx), commBlocks_, fa);
      continue;
    }
    if (engine) ctx.coloPackLocal.run_device(parity, S(ctx), commBlocks_);
    if (!credits.empty()) wait_flags(credits, I.epoch - 2, 1, S(ctx));
    if (engine) {
      forked_copies(ctx, S(ctx), int(ctx.coloSend.size()), [&](int k, hipStream_t cs) {
        const Channel &c = I.chans[size_t(ctx.coloSend[size_t(k)])];
        if (c.bytes > 0) engine_copy(c.remoteData + slot * c.slotStride, c.dbuf, size_t(c.bytes), cs);
      });
    } else {
      ctx.coloPack.run_device(cv, S(ctx), commBlocks_);
    }
    signal_flags(arrived, I.epoch, S(ctx));
  }

  jitter();
  // (3) RCCL: pack, one group of send/recv over every local device, unpack
  if (I.rccl) {
    TraceRange t("rccl");
    for (auto &ctx : I.devs) {
      if (ctx.rcclSend.empty()) continue;
      HIP_CHECK(hipSetDevice(ctx.dev));
      ctx.rcclPack.run_device(parity, S(ctx), commBlocks_);
    }
    RCCL_CHECK(rccl::group_start());
    for (auto &ctx : I.devs) {
      for (int ci : ctx.rcclSend)
        RCCL_CHECK(rccl::send(I.chans[ci].dbuf, size_t(I.chans[ci].bytes), I.chans[ci].ncclPeer, ctx.nccl, S(ctx)));
      for (int ci : ctx.rcclRecv)
        RCCL_CHECK(rccl::recv(I.chans[ci].dbuf, size_t(I.chans[ci].bytes), I.chans[ci].ncclPeer, ctx.nccl, S(ctx)));
    }
    RCCL_CHECK(rccl::group_end());
    for (auto &ctx : I.devs) {
      if (ctx.rcclRecv.empty()) continue;
      HIP_CHECK(hipSetDevice(ctx.dev));
      ctx.rcclUnpack.run_device(parity, S(ctx), commBlocks_);
    }
  }

  // (4) host-staged fallback (blocks the host)
  {
    bool anyStaged = false;
    for (auto &ctx : I.devs) anyStaged |= !ctx.stagedSend.empty() || !ctx.stagedRecv.empty();
    if (anyStaged) {
      TraceRange t("staged");
      for (auto &ctx : I.devs) {
        if (ctx.stagedSend.empty()) continue;
        HIP_CHECK(hipSetDevice(ctx.dev));
        ctx.stagedPack.run_device(parity, S(ctx), commBlocks_);
        for (int ci : ctx.stagedSend)
          HIP_CHECK(hipMemcpyAsync(I.chans[ci].hbuf, I.chans[ci].dbuf, size_t(I.chans[ci].bytes), hipMemcpyDeviceToHost,
                                   S(ctx)));
      }
      for (auto &ctx : I.devs) {
        if (ctx.stagedSend.empty()) continue;
        HIP_CHECK(hipSetDevice(ctx.dev));
        HIP_CHECK(hipStreamSynchronize(S(ctx)));
        for (int ci : ctx.stagedSend) pg.send(I.chans[ci].remoteRank, I.chans[ci].tag, I.chans[ci].hbuf, size_t(I.chans[ci].bytes));
      }
      for (auto &ctx : I.devs) {
        if (ctx.stagedRecv.empty()) continue;
        HIP_CHECK(hipSetDevice(ctx.dev));
        for (int ci : ctx.stagedRecv) {
          pg.recv(I.chans[ci].remoteRank, I.chans[ci].tag, I.chans[ci].hbuf, size_t(I.chans[ci].bytes));
          HIP_CHECK(hipMemcpyAsync(I.chans[ci].dbuf, I.chans[ci].hbuf, size_t(I.chans[ci].bytes), hipMemcpyHostToDevice,
                                   S(ctx)));
        }
        ctx.stagedUnpack.run_device(parity, S(ctx), commBlocks_);
      }
    }
  }

  jitter();
  // (5) colocated receives: wait for arrival, unpack from our inbox, return the credit to the sender
  for (auto &ctx : I.devs) {
    if (ctx.coloRecv.empty()) continue;
    HIP_CHECK(hipSetDevice(ctx.dev));
    TraceRange t("colo recv");
    std::vector<uint64_t *> arrived, credits;
    for (int ci : ctx.coloRecv) {
      arrived.push_back(reinterpret_cast<uint64_t *>(I.chans[ci].ownFlag));
      credits.push_back(reinterpret_cast<uint64_t *>(I.chans[ci].remoteFlag));
    }
    if (ipcEvt) { // per channel: Notify(epoch) -> wait on the sender's event -> Ack(epoch); unpack + credits
      for (int ci : ctx.coloRecv) {
        Channel &c = I.chans[size_t(ci)];
        IpcNotify msg;
        pg.recv(c.remoteRank, retag(c.tag, comm::MsgKind::Notify), &msg, sizeof(msg));
        STENCIL_REQUIRE(msg.epoch == I.epoch,
                        "IPC-event notify out of order: got epoch " << msg.epoch << ", want " << I.epoch);
        if (msg.fresh) { // the sender replaced its event: open the new one, keep the old until no wait needs it
          c.ipcRetired.emplace_back(c.ipcEvent, I.epoch);
          HIP_CHECK(hipIpcOpenEventHandle(&c.ipcEvent, msg.handle));
        }
        while (!c.ipcRetired.empty() && I.epoch - c.ipcRetired.front().second >= kIpcRetireEpochs) {
          (void)hipEventDestroy(c.ipcRetired.front().first);
          c.ipcRetired.pop_front();
        }
        HIP_CHECK(hipStreamWaitEvent(S(ctx), c.ipcEvent, 0));
        const uint64_t e = I.epoch;
        pg.send(c.remoteRank, retag(c.tag, comm::MsgKind::Ack), &e, sizeof(e));
      }
      FlagSyncArgs fa;
      fa.signal = credits;
      fa.signalValue = I.epoch;
      fa.counter = ctx.syncCounter + 1;
      fa.err = I.errDev;
      fa.code = 2;
      fa.timeout_s = topt_.waitTimeout;
      fa.sharedGpu = ctx.sharedGpu;
      if (ctx.xlog) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords + 4;
      ctx.coloUnpack.run_device_sync(cv, S(ctx), commBlocks_, fa);
      continue;
    }
    // Coarse (L2-cached) inboxes keep the arrival wait in its own kernel: the unpack's dispatch then starts after
    // the wait with the kernel-boundary cache invalidate, where a wait inside the unpack kernel would rely on its
    // in-kernel acquire dropping L2 lines of local coarse-grained memory written over xGMI
    if (fused && topt_.inbox != TransportOptions::Inbox::Coarse) { // one launch: arrival wait, unpack, credits
      FlagSyncArgs fa;
      fa.wait = arrived;
      fa.waitTarget = I.epoch;
      fa.signal = credits;
      fa.signalValue = I.epoch;
      fa.counter = ctx.syncCounter + 1;
      fa.err = I.errDev;
      fa.code = 2;
      fa.timeout_s = topt_.waitTimeout;
      fa.sharedGpu = ctx.sharedGpu;
      if (ctx.xlog) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords + 4;
      ctx.coloUnpack.run_device_sync(cv, S(ctx), commBlocks_, fa);
      continue;
    }
    wait_flags(arrived, I.epoch, 2, S(ctx));
    ctx.coloUnpack.run_device(cv, S(ctx), commBlocks_);
    signal_flags(credits, I.epoch, S(ctx));
  }

  // (6) halos written by peer devices of this process
  for (auto &ctx : I.devs) {
    HIP_CHECK(hipSetDevice(ctx.dev));
    for (int src : ctx.peerWriters) I.devs[I.devIndex[src]].translated.wait_on(S(ctx));
    if (!over) ctx.done.record(S(ctx));
  }
  if (over && !capturing) {
    I.callerDone.record(stream);
    I.callerPending = true;
  } else if (!over) {
    I.commPending = true;
  }
}

void DistributedDomain::swap() {
  double t0 = 0;
  if (exchangeStats_) {
    pg_->barrier();
    t0 = now_s();
  }
  TraceRange tr("swap");
  for (auto &d : domains_) d.swap();
  if (exchangeStats_) timeSwap_ += pg_->allreduce_max(now_s() - t0);
}

} // namespace stencil
