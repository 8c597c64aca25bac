#pragma once
// What this library was built from and with: git revision (cmake/git_sha.cmake) and the compile-time options of
// CMakeLists.txt (reference: CMakeLists.txt:16-35, options and the embedded git hash).
#include <string>

namespace stencil {

struct BuildInfo {
  std::string gitSha;   // "<12-hex>[-dirty]" or "unknown"
  bool useRccl;         // STENCIL_USE_RCCL
  bool setupStats;      // STENCIL_SETUP_STATS
  bool exchangeStats;   // STENCIL_EXCHANGE_STATS (default of DistributedDomain::exchangeStats_)
  int outputLevel;      // STENCIL_OUTPUT_LEVEL
  std::string offloadArch;
};

const BuildInfo &build_info();
std::string build_info_string(); // one line, for app / bench output

} // namespace stencil
