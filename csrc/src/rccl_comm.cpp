// RCCL forwarding layer (see stencil/comm/rccl_comm.hpp).
#include "stencil/comm/rccl_comm.hpp"

#include <cstring>

#if STENCIL_USE_RCCL
#include <rccl/rccl.h>

static_assert(sizeof(ncclUniqueId) == sizeof(stencil::rccl::UniqueId), "ncclUniqueId size");
#endif

namespace stencil {
namespace rccl {

#if STENCIL_USE_RCCL

static std::string err(const char *what, ncclResult_t r) {
  return r == ncclSuccess ? std::string() : std::string(what) + ": " + ncclGetErrorString(r);
}

bool compiled() { return true; }

std::string get_unique_id(UniqueId *id) {
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r == ncclSuccess) std::memcpy(id->bytes, &u, sizeof(u));
  return err("ncclGetUniqueId", r);
}

std::string init_ranks(std::vector<Comm> *comms, int nranks, const UniqueId &id, const std::vector<int> &ranks,
                       const std::vector<int> &devices) {
  ncclUniqueId u;
  std::memcpy(&u, id.bytes, sizeof(u));
  comms->assign(ranks.size(), nullptr);
  ncclResult_t r = ncclGroupStart();
  std::string e = err("ncclGroupStart", r);
  for (size_t k = 0; k < ranks.size() && e.empty(); ++k) {
    if (hipSetDevice(devices[k]) != hipSuccess) {
      (void)hipGetLastError();
      e = "hipSetDevice(" + std::to_string(devices[k]) + ")";
      break;
    }
    ncclComm_t c = nullptr;
    r = ncclCommInitRank(&c, nranks, u, ranks[k]);
    (*comms)[k] = c;
    e = err("ncclCommInitRank", r);
  }
  const ncclResult_t re = ncclGroupEnd();
  if (e.empty()) e = err("ncclGroupEnd", re);
  return e;
}

void destroy(Comm c) {
  if (c) (void)ncclCommDestroy(ncclComm_t(c));
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
std::string group_end() { return err("ncclGroupEnd", ncclGroupEnd()); }
std::string send(const void *buf, size_t bytes, int peer, Comm c, hipStream_t s) {
  return err("ncclSend", ncclSend(buf, bytes, ncclUint8, peer, ncclComm_t(c), s));
}
std::string recv(void *buf, size_t bytes, int peer, Comm c, hipStream_t s) {
  return err("ncclRecv", ncclRecv(buf, bytes, ncclUint8, peer, ncclComm_t(c), s));
}

#else // RCCL not compiled in: every entry point reports it, DistributedDomain stages through the host

static const char *kOff = "RCCL not compiled in (STENCIL_USE_RCCL=OFF)";
bool compiled() { return false; }
std::string get_unique_id(UniqueId *) { return kOff; }
std::string init_ranks(std::vector<Comm> *comms, int, const UniqueId &, const std::vector<int> &ranks,
                       const std::vector<int> &) {
  comms->assign(ranks.size(), nullptr);
  return kOff;
}
void destroy(Comm) {}
void abort(Comm) {}
std::string async_error(Comm) { return {}; }
std::string group_start() { return kOff; }
std::string group_end() { return kOff; }
std::string send(const void *, size_t, int, Comm, hipStream_t) { return kOff; }
std::string recv(void *, size_t, int, Comm, hipStream_t) { return kOff; }

#endif

} // namespace rccl
} // namespace stencil
