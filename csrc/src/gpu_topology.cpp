#include "stencil/topo/gpu_topology.hpp"

#include <hip/hip_runtime_api.h>

#include <map>
#include <mutex>

#include "stencil/rt/logging.hpp"

namespace stencil {
namespace gpu_topo {

static constexpr uint32_t kLinkPcie = 2; // HSA_AMD_LINK_INFO_TYPE_PCIE
static constexpr uint32_t kLinkXgmi = 4; // HSA_AMD_LINK_INFO_TYPE_XGMI

int device_count() {
  static int n = [] {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return c;
  }();
  return n;
}

static bool query_link(int a, int b, uint32_t *type, uint32_t *hops) {
  if (a < 0 || b < 0 || a >= device_count() || b >= device_count()) return false;
  if (hipExtGetLinkTypeAndHopCount(a, b, type, hops) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}

double distance(int src, int dst) {
  if (src == dst) return 0.1;
  uint32_t type = 0, hops = 0;
  if (!query_link(src, dst, &type, &hops)) return 1.0; // unknown: treat as uniform mesh
  if (type == kLinkXgmi) return hops <= 1 ? 1.0 : 1.0 + double(hops - 1);
  if (type == kLinkPcie) return 3.0 + double(hops);
  return 6.0;
}

std::vector<LinkInfo> links() {
  std::vector<LinkInfo> out;
  const int n = device_count();
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      LinkInfo li{a, b, "self", 0, distance(a, b)};
      if (a != b) {
        uint32_t t = 0, h = 0;
        if (query_link(a, b, &t, &h)) {
          li.type = t == kLinkXgmi ? "xgmi" : (t == kLinkPcie ? "pcie" : "other");
          li.hops = int(h);
        } else {
          li.type = "unknown";
        }
      }
      out.push_back(li);
    }
  return out;
}

static std::mutex g_mu;
static std::map<std::pair<int, int>, bool> g_peer;

bool enable_peer(int src, int dst) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto key = std::make_pair(src, dst);
  auto it = g_peer.find(key);
  if (it != g_peer.end()) return it->second;
  bool ok = false;
  if (src == dst) {
    ok = src >= 0;
  } else if (src >= 0 && dst >= 0 && src < device_count() && dst < device_count()) {
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, src, dst) == hipSuccess && can) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(src);
      hipError_t e = hipDeviceEnablePeerAccess(dst, 0);
      if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) ok = true;
      (void)hipGetLastError();
      (void)hipSetDevice(prev);
    } else {
      (void)hipGetLastError();
    }
  }
  LOG_DEBUG("peer access " << src << "->" << dst << " = " << ok);
  g_peer[key] = ok;
  return ok;
}

bool peer(int src, int dst) { return enable_peer(src, dst); }

} // namespace gpu_topo
} // namespace stencil
