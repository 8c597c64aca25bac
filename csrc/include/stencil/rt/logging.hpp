#pragma once
// Leveled logging, format `LEVEL[file:line]{rank} msg` to stderr.
// Parity: reference include/stencil/logging.hpp:8-52 (compile-time levels 0-5, LOG_FATAL exits).
// Addition: the level can be lowered at run time with STENCIL_LOG_LEVEL (0..5).
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <stdexcept>

#ifndef STENCIL_OUTPUT_LEVEL
#define STENCIL_OUTPUT_LEVEL 3
#endif

namespace stencil {
namespace log {
int rank();          // process rank for log tags (set by the process group)
void set_rank(int r);
int runtime_level(); // min(compile level, STENCIL_LOG_LEVEL)
} // namespace log

// Fatal errors throw (so Python callers get an exception) instead of exit()-ing the process.
struct Error : public std::runtime_error {
  using std::runtime_error::runtime_error;
};
} // namespace stencil

#define STENCIL_LOG_IMPL(lvl, name, x)                                                                             \
  do {                                                                                                             \
    if (STENCIL_OUTPUT_LEVEL >= lvl && stencil::log::runtime_level() >= lvl) {                                     \
      std::ostringstream _ss;                                                                                      \
      _ss << name "[" << __FILE__ << ":" << __LINE__ << "]{" << stencil::log::rank() << "} " << x << "\n";          \
      std::cerr << _ss.str();                                                                                      \
    }                                                                                                              \
  } while (0)

#define LOG_SPEW(x) STENCIL_LOG_IMPL(5, "SPEW", x)
#define LOG_DEBUG(x) STENCIL_LOG_IMPL(4, "DEBUG", x)
#define LOG_INFO(x) STENCIL_LOG_IMPL(3, "INFO", x)
#define LOG_WARN(x) STENCIL_LOG_IMPL(2, "WARN", x)
#define LOG_ERROR(x) STENCIL_LOG_IMPL(1, "ERROR", x)
#define LOG_FATAL(x)                                                                                               \
  do {                                                                                                             \
    std::ostringstream _fs;                                                                                        \
    _fs << "FATAL[" << __FILE__ << ":" << __LINE__ << "]{" << stencil::log::rank() << "} " << x;                   \
    std::cerr << _fs.str() << "\n";                                                                               \
    throw stencil::Error(_fs.str());                                                                               \
  } while (0)

#define STENCIL_REQUIRE(cond, msg)                                                                                 \
  do {                                                                                                             \
    if (!(cond)) LOG_FATAL("requirement failed: " #cond ": " << msg);                                              \
  } while (0)
