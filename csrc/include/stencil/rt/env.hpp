#pragma once
// The process-level environment variables of the runtime, read in one place. Everything that selects an algorithm,
// a kernel or a transport variant is typed configuration instead (StencilTune, TransportOptions,
// StencilModelConfig) and reaches the runtime through the C++ / Python API and the apps' command lines.
//
//   STENCIL_WAIT_TIMEOUT  seconds before a device-side spin, a host wait on a peer rank or the RCCL watchdog gives up
//                         (default 60; TransportOptions::waitTimeout)
//   STENCIL_COMM_TIMEOUT  receive timeout of the TCP process group (default STENCIL_WAIT_TIMEOUT when set, else 600)
//   STENCIL_LOG_LEVEL     runtime log level 0..5 (default 2 = info)
//   STENCIL_TRACE         1: roctx ranges around realize / exchange / transport phases (rocprofv3 --marker-trace)
//   STENCIL_PLAN_FILE     0: do not write plan_<rank>.txt during realize (reference src/stencil.cu:259-353)
//   STENCIL_HOSTNAME      host name this rank reports (fakes multi-node layouts in tests)
//   STENCIL_AMDSMI        1: also query amd-smi (link weights/bandwidths; off by default: exit-time abort on ROCm 7.2)
//   rendezvous            STENCIL_RANK / STENCIL_WORLD_SIZE / STENCIL_MASTER_ADDR / STENCIL_MASTER_PORT, or torchrun's
//                         RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (+1: torch's store holds MASTER_PORT)
#include <cstdlib>
#include <string>

namespace stencil {
namespace env {

inline const char *raw(const char *name) { return std::getenv(name); }

inline bool has(const char *name) { return raw(name) != nullptr; }

inline long get_int(const char *name, long dflt) {
  const char *e = raw(name);
  return e ? std::atol(e) : dflt;
}

inline double get_double(const char *name, double dflt) {
  const char *e = raw(name);
  return e ? std::atof(e) : dflt;
}

inline std::string get_str(const char *name, const std::string &dflt) {
  const char *e = raw(name);
  return e ? std::string(e) : dflt;
}

} // namespace env

// STENCIL_WAIT_TIMEOUT, or `dflt`
inline double env_wait_timeout(double dflt) { return env::get_double("STENCIL_WAIT_TIMEOUT", dflt); }

} // namespace stencil
