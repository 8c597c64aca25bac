#pragma once
// Thin RCCL layer: the only place that includes <rccl/rccl.h>. Built with STENCIL_USE_RCCL=ON (CMake, default) it
// forwards to RCCL; with OFF every call reports "RCCL not compiled in" and DistributedDomain plans the host-staged
// transport for GPU-aware remote pairs instead (reference: CMake USE_CUDA_AWARE_MPI, CMakeLists.txt:18,135-141).
// Every function returns an error string ("" on success) instead of aborting, so callers can agree on a fallback.
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
// one communicator per local device, created in one group: comms[k] gets RCCL rank ranks[k] on device devices[k]
std::string init_ranks(std::vector<Comm> *comms, int nranks, const UniqueId &id, const std::vector<int> &ranks,
                       const std::vector<int> &devices);
void destroy(Comm c);
void abort(Comm c);
// "" while healthy (success or still in progress), else the asynchronous error
std::string async_error(Comm c);
std::string group_start();
std::string group_end();
std::string send(const void *buf, size_t bytes, int peer, Comm c, hipStream_t s);
std::string recv(void *buf, size_t bytes, int peer, Comm c, hipStream_t s);

} // namespace rccl
} // namespace stencil
