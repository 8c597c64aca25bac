#pragma once
// Thin RCCL layer: the only place that includes <rccl/rccl.h>. Built with STENCIL_USE_RCCL=ON (CMake, default) it
// forwards to RCCL; with OFF every call reports "RCCL not compiled in" and DistributedDomain plans the host-staged
// transport for GPU-aware remote pairs instead (reference: CMake USE_CUDA_AWARE_MPI, CMakeLists.txt:18,135-141).
// Every function returns an error string ("" on success) instead of aborting, so callers can agree on a fallback.
//
// Communicators are created NON-BLOCKING (ncclConfig_t::blocking = 0) and their creation is polled against a
// deadline: a member that never arrives (a dead or stuck rank) costs the others `timeout` seconds and an abort, not
// a hang inside ncclCommInitRank. Calls on such a communicator may return "in progress"; every entry point below
// settles that (polls ncclCommGetAsyncError) before it returns, so callers see the blocking semantics.
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <string>
#include <vector>

namespace stencil {
namespace rccl {

using Comm = void *; // ncclComm_t

struct UniqueId {
  char bytes[128]; // NCCL_UNIQUE_ID_BYTES
};

bool compiled();
std::string get_unique_id(UniqueId *id);
// one communicator per local device, created in one group: comms[k] gets RCCL rank ranks[k] on device devices[k].
// Gives up after `timeout` seconds (<= 0: no limit): every communicator of the group is aborted, comms[] cleared and
// the error says "timed out". stall (test hook): skip creation entirely and report a timeout after `timeout`
// seconds, as a rank stuck before ncclCommInitRank would leave its peers
std::string init_ranks(std::vector<Comm> *comms, int nranks, const UniqueId &id, const std::vector<int> &ranks,
                       const std::vector<int> &devices, double timeout = 0, bool stall = false);
void destroy(Comm c);
void abort(Comm c);
// "" while healthy (success or still in progress), else the asynchronous error
std::string async_error(Comm c);
std::string group_start();
// ends the group; with non-blocking communicators waits (up to `timeout` s, <= 0: no limit) until every one of
// `comms` has left the in-progress state
std::string group_end(const std::vector<Comm> &comms = {}, double timeout = 0);
std::string send(const void *buf, size_t bytes, int peer, Comm c, hipStream_t s);
std::string recv(void *buf, size_t bytes, int peer, Comm c, hipStream_t s);

} // namespace rccl
} // namespace stencil
