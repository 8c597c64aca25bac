#include "stencil/rt/build_info.hpp"

#include "stencil_git_sha.h" // generated (build dir) by cmake/git_sha.cmake

namespace stencil {

const BuildInfo &build_info() {
  static const BuildInfo b{STENCIL_GIT_SHA, STENCIL_USE_RCCL != 0, STENCIL_SETUP_STATS != 0, STENCIL_EXCHANGE_STATS != 0,
                           STENCIL_OUTPUT_LEVEL, "gfx950"};
  return b;
}

std::string build_info_string() {
  const BuildInfo &b = build_info();
  return "stencil2_amd git=" + b.gitSha + " arch=" + b.offloadArch + " rccl=" + (b.useRccl ? "on" : "off") +
         " setup_stats=" + (b.setupStats ? "on" : "off") + " exchange_stats=" + (b.exchangeStats ? "on" : "off") +
         " log_level=" + std::to_string(b.outputLevel);
}

} // namespace stencil
