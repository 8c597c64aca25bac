// DistributedDomain exchange engine: stream bookkeeping, blocking and stream-ordered exchange over every transport,
// completion modes, transport log and swap (split out of distributed_domain.cpp). Reference
// counterparts: DistributedDomain::exchange() and swap() in src/stencil.cu:670-864 and :541-565 (there one
// blocking host loop over the senders / receivers; here one stream-ordered enqueue per device).
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

void retire_ipc_events(Channel &c, uint64_t epoch, hipStream_t s) {
  for (auto &r : c.ipcRetired)
    if (!r.fence && epoch >= r.fenceEpoch) {
      HIP_CHECK(hipEventCreateWithFlags(&r.fence, hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(r.fence, s));
    }
  while (!c.ipcRetired.empty() && c.ipcRetired.front().fence) {
    const hipError_t q = hipEventQuery(c.ipcRetired.front().fence);
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();
      break;
    }
    HIP_CHECK(q);
    (void)hipEventDestroy(c.ipcRetired.front().fence);
    (void)hipEventDestroy(c.ipcRetired.front().event);
    c.ipcRetired.pop_front();
  }
}

// Completion::IpcEvent: the receivers' Acks of the last two exchanges are consumed by no later record. Take them, so
// that neither a switch back to IpcEvent nor another IpcEvent domain on the same group (same channel tags) finds a
// stale Ack queued. timeout_s > 0: poll, give up after that long (teardown); else blocking receives.
bool DistributedDomain::drain_ipc_acks(double timeout_s) {
  Impl &I = *impl_;
  if (!realized_ || backend_ != Backend::Device || topt_.completion != TransportOptions::Completion::IpcEvent)
    return true;
  const double t0 = now_s();
  for (auto &ctx : I.devs)
    for (int ci : ctx.coloSend) {
      Channel &ch = I.chans[size_t(ci)];
      for (uint64_t e = I.epoch >= 1 ? I.epoch - 1 : 0; e <= I.epoch; ++e) {
        if (e == 0 || e < I.ipcEventFirstEpoch) continue;
        uint64_t acked = 0;
        const uint32_t tag = retag(ch.tag, comm::MsgKind::Ack);
        if (timeout_s > 0) {
          while (!pg_->try_recv(ch.remoteRank, tag, &acked, sizeof(acked))) {
            if (now_s() - t0 > timeout_s) return false;
            std::this_thread::sleep_for(std::chrono::microseconds(100));
          }
        } else {
          pg_->recv(ch.remoteRank, tag, &acked, sizeof(acked));
        }
        STENCIL_REQUIRE(acked == e, "IPC-event ack out of order: got epoch " << acked << ", want " << e);
      }
    }
  return true;
}

void DistributedDomain::set_completion(TransportOptions::Completion c) {
  if (c == topt_.completion) return;
  STENCIL_REQUIRE(!realized_ || c != TransportOptions::Completion::IpcEvent || impl_->ipcEvents ||
                      exchange_bytes_for_method(MethodFlags::Colocated) == 0,
                  "Completion::IpcEvent needs its interprocess events: realize() with that completion");
  if (realized_) sync_exchange(); // flag words are monotonic epochs: either method continues where the other left off
  Impl &I = *impl_;
  drain_ipc_acks(0); // leaving IpcEvent: no stale Ack for a later switch back
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
    for (int p = 0; p < 2; ++p) build_translate(sd, dd, dir, p == 0, ctx.translateSkip.host[p], x_face_lines(sd, dd));
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
    if (!ctx.translateEmpty) tl.run_device(parity, S(ctx), translateBlocks_);
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
        if (ctx.xlog && !capturing) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords;
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
          c.ipcRetired.push_back({c.ipcEvent, I.epoch + 1, nullptr});
          HIP_CHECK(hipEventCreateWithFlags(&c.ipcEvent, hipEventDisableTiming | hipEventInterprocess));
          HIP_CHECK(hipIpcGetEventHandle(&msg.handle, c.ipcEvent));
          msg.fresh = 1;
          c.ipcUses = 0;
        }
        retire_ipc_events(c, I.epoch, S(ctx));
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
      if (ctx.xlog && !capturing) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords;
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
    std::vector<rccl::Comm> comms;
    for (auto &ctx : I.devs)
      if (ctx.nccl) comms.push_back(ctx.nccl);
    RCCL_CHECK(rccl::group_end(comms, topt_.waitTimeout));
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
          c.ipcRetired.push_back({c.ipcEvent, I.epoch, nullptr});
          HIP_CHECK(hipIpcOpenEventHandle(&c.ipcEvent, msg.handle));
        }
        retire_ipc_events(c, I.epoch, S(ctx));
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
      if (ctx.xlog && !capturing) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords + 4;
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
      if (ctx.xlog && !capturing) fa.stamps = ctx.xlog + ((I.epoch - 1) % uint64_t(I.xlogCap)) * kTransportLogWords + 4;
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
