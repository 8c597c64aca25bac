// RCCL forwarding layer (see stencil/comm/rccl_comm.hpp).
#include "stencil/comm/rccl_comm.hpp"

#include <chrono>
#include <cstring>
#include <thread>

#if STENCIL_USE_RCCL
#include <rccl/rccl.h>

static_assert(sizeof(ncclUniqueId) == sizeof(stencil::rccl::UniqueId), "ncclUniqueId size");
#endif

namespace stencil {
namespace rccl {

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#if STENCIL_USE_RCCL

static std::string err(const char *what, ncclResult_t r) {
  return r == ncclSuccess ? std::string() : std::string(what) + ": " + ncclGetErrorString(r);
}

// poll until no communicator of `cs` is in progress; ncclInProgress when the deadline passed first
static ncclResult_t settle(const std::vector<Comm> &cs, double timeout) {
  const double t0 = now_s();
  for (;;) {
    ncclResult_t worst = ncclSuccess;
    for (Comm c : cs) {
      if (!c) continue;
      ncclResult_t s = ncclSuccess;
      const ncclResult_t q = ncclCommGetAsyncError(ncclComm_t(c), &s);
      if (q != ncclSuccess) return q;
      if (s != ncclSuccess && s != ncclInProgress) return s;
      if (s == ncclInProgress) worst = ncclInProgress;
    }
    if (worst == ncclSuccess) return ncclSuccess;
    if (timeout > 0 && now_s() - t0 > timeout) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

bool compiled() { return true; }

std::string get_unique_id(UniqueId *id) {
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r == ncclSuccess) std::memcpy(id->bytes, &u, sizeof(u));
  return err("ncclGetUniqueId", r);
}

std::string init_ranks(std::vector<Comm> *comms, int nranks, const UniqueId &id, const std::vector<int> &ranks,
                       const std::vector<int> &devices, double timeout, bool stall) {
  comms->assign(ranks.size(), nullptr);
  if (stall) { // the hook: this rank never enters creation; its peers' polls run into their deadline
    std::this_thread::sleep_for(std::chrono::duration<double>(timeout > 0 ? timeout : 1.0));
    return "ncclCommInitRankConfig timed out (stalled by TransportOptions::stallRcclInitRank)";
  }
  ncclUniqueId u;
  std::memcpy(&u, id.bytes, sizeof(u));
  ncclResult_t r = ncclGroupStart();
  std::string e = err("ncclGroupStart", r);
  for (size_t k = 0; k < ranks.size() && e.empty(); ++k) {
    if (hipSetDevice(devices[k]) != hipSuccess) {
      (void)hipGetLastError();
      e = "hipSetDevice(" + std::to_string(devices[k]) + ")";
      break;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    r = ncclCommInitRankConfig(&c, nranks, u, ranks[k], &cfg);
    (*comms)[k] = c;
    if (r != ncclInProgress) e = err("ncclCommInitRankConfig", r);
  }
  const ncclResult_t re = ncclGroupEnd();
  if (e.empty() && re != ncclInProgress) e = err("ncclGroupEnd", re);
  if (e.empty()) {
    const ncclResult_t s = settle(*comms, timeout);
    if (s == ncclInProgress)
      e = "ncclCommInitRankConfig timed out after " + std::to_string(timeout) + " s (a member never joined)";
    else
      e = err("ncclCommInitRankConfig (asynchronous)", s);
  }
  if (!e.empty()) { // never hand out a half-built communicator: abort every one of the group
    for (Comm &c : *comms)
      if (c) {
        (void)ncclCommAbort(ncclComm_t(c));
        c = nullptr;
      }
  }
  return e;
}

void destroy(Comm c) {
  if (!c) return;
  // a non-blocking communicator: finalize (flush) first, bounded, then free
  if (ncclCommFinalize(ncclComm_t(c)) == ncclInProgress) (void)settle({c}, 10.0);
  (void)ncclCommDestroy(ncclComm_t(c));
}
void abort(Comm c) {
  if (c) (void)ncclCommAbort(ncclComm_t(c));
}

std::string async_error(Comm c) {
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(ncclComm_t(c), &r) != ncclSuccess) return {};
  return r == ncclSuccess || r == ncclInProgress ? std::string() : err("asynchronous", r);
}

std::string group_start() { return err("ncclGroupStart", ncclGroupStart()); }
std::string group_end(const std::vector<Comm> &comms, double timeout) {
  const ncclResult_t r = ncclGroupEnd();
  if (r != ncclInProgress) return err("ncclGroupEnd", r);
  const ncclResult_t s = settle(comms, timeout);
  return s == ncclInProgress ? std::string("ncclGroupEnd: still in progress after the wait timeout")
                             : err("ncclGroupEnd (asynchronous)", s);
}
std::string send(const void *buf, size_t bytes, int peer, Comm c, hipStream_t s) {
  ncclResult_t r = ncclSend(buf, bytes, ncclUint8, peer, ncclComm_t(c), s);
  if (r == ncclInProgress) r = settle({c}, 0);
  return err("ncclSend", r);
}
std::string recv(void *buf, size_t bytes, int peer, Comm c, hipStream_t s) {
  ncclResult_t r = ncclRecv(buf, bytes, ncclUint8, peer, ncclComm_t(c), s);
  if (r == ncclInProgress) r = settle({c}, 0);
  return err("ncclRecv", r);
}

#else // RCCL not compiled in: every entry point reports it, DistributedDomain stages through the host

static const char *kOff = "RCCL not compiled in (STENCIL_USE_RCCL=OFF)";
bool compiled() { return false; }
std::string get_unique_id(UniqueId *) { return kOff; }
std::string init_ranks(std::vector<Comm> *comms, int, const UniqueId &, const std::vector<int> &ranks,
                       const std::vector<int> &, double, bool) {
  comms->assign(ranks.size(), nullptr);
  (void)now_s;
  return kOff;
}
void destroy(Comm) {}
void abort(Comm) {}
std::string async_error(Comm) { return {}; }
std::string group_start() { return kOff; }
std::string group_end(const std::vector<Comm> &, double) { return kOff; }
std::string send(const void *, size_t, int, Comm, hipStream_t) { return kOff; }
std::string recv(void *, size_t, int, Comm, hipStream_t) { return kOff; }

#endif

} // namespace rccl
} // namespace stencil
