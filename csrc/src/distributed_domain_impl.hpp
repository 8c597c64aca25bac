#pragma once
// DistributedDomain internals shared by its translation units (distributed_domain.cpp: setup and realize;
// distributed_domain_exchange.cpp: the exchange engine). Not installed; private to csrc/src.
#include "stencil/domain/distributed_domain.hpp"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "stencil/comm/rccl_comm.hpp"
#include "stencil/comm/tags.hpp"
#include "stencil/rt/hip_check.hpp"

#define RCCL_CHECK(stmt)                                                                                           \
  do {                                                                                                             \
    const std::string _e = (stmt);                                                                                 \
    if (!_e.empty()) LOG_FATAL("RCCL error (" << _e << ") in `" #stmt "`");                                        \
  } while (0)

namespace stencil {

inline int method_slot(MethodFlags m) {
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

inline double now_s() {
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
inline uint32_t retag(uint32_t tag, comm::MsgKind kind) {
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
  // replaced events, destroyed by DEVICE progress: once the exchange of epoch `fenceEpoch` has been
  // enqueued, an ordinary event `fence` is recorded on the comm stream behind it; the old event is destroyed when
  // `fence` has completed (hipEventQuery), or at teardown after the streams are synchronized. Sender: fenceEpoch =
  // replacement + 1, i.e. behind the pack kernel whose credit wait proves the receiver finished the unpack that
  // followed its last wait on the old event. Receiver: fenceEpoch = replacement (every wait on the old event is
  // already enqueued on this stream).
  struct RetiredEvent {
    hipEvent_t event = nullptr;
    uint64_t fenceEpoch = 0;
    hipEvent_t fence = nullptr;
  };
  std::deque<RetiredEvent> ipcRetired;
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
// fence and destroy the replaced events of channel c whose fence epoch has been reached (see Channel::ipcRetired)
void retire_ipc_events(Channel &c, uint64_t epoch, hipStream_t s);

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
  std::set<int> xLineDevs;          // devices whose same-GPU x faces are copied as whole lines (xFaceSectors, or auto)
};


// ------------------------------------------------------------------------------------------------
// segment builders (reference wire layout: messages sorted by dir, each quantity aligned to its element size,
// reference packer.cuh:136-160)
// ------------------------------------------------------------------------------------------------
inline void build_pack(const LocalDomain &dom, const std::vector<Message> &msgs, char *buf, bool curr,
                       std::vector<CopySeg> &out) {
  build_pack_segs(dom, msgs, buf, curr, out);
}
inline void build_unpack(const LocalDomain &dom, const std::vector<Message> &msgs, char *buf, bool curr,
                         std::vector<CopySeg> &out) {
  build_unpack_segs(dom, msgs, buf, curr, out);
}
inline void build_translate(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, bool curr,
                            std::vector<CopySeg> &out, bool xSectors = false) {
  build_translate_segs(src, dst, dir, curr, out, xSectors);
}

} // namespace stencil
