#include "stencil/topo/gpu_topology.hpp"
#include "stencil/rt/env.hpp"

#include <sched.h>

#include <cctype>
#include <fstream>
#include <sstream>

#include <hip/hip_runtime_api.h>

#include <amd_smi/amdsmi.h>
#include <dlfcn.h>

#include <cstdio>
#include <map>
#include <mutex>

#include "stencil/rt/logging.hpp"

namespace stencil {
namespace gpu_topo {

// ---- amd-smi, resolved with dlopen so the runtime still loads where the library is absent ----
// Opt-in (STENCIL_AMDSMI=1): on the MI355X pool's ROCm 7.2 image a process that has initialised amd-smi next to the
// HIP runtime aborts with glibc "double free or corruption" when it exits (build/bin/jacobi3d 128^3: rc 134 with
// amd-smi, rc 0 without; gpurun_out/d1, r3). Every query the runtime needs has an amd-smi-free source: link type
// and hops from hipExtGetLinkTypeAndHopCount, the NUMA node from sysfs. amd-smi adds the link weights and
// bandwidths of links(); when it is enabled, amdsmi_shut_down runs at exit.
namespace {
amdsmi_status_t (*g_smi_shutdown)() = nullptr;
struct Smi {
  bool ok = false;
  std::vector<amdsmi_processor_handle> byDev; // HIP ordinal -> processor handle (null if unmatched)
  amdsmi_status_t (*link_type)(amdsmi_processor_handle, amdsmi_processor_handle, uint64_t *, amdsmi_link_type_t *) = nullptr;
  amdsmi_status_t (*link_weight)(amdsmi_processor_handle, amdsmi_processor_handle, uint64_t *) = nullptr;
  amdsmi_status_t (*minmax_bw)(amdsmi_processor_handle, amdsmi_processor_handle, uint64_t *, uint64_t *) = nullptr;
  amdsmi_status_t (*numa)(amdsmi_processor_handle, uint32_t *) = nullptr;
  amdsmi_processor_handle handle(int dev) const {
    return ok && dev >= 0 && dev < int(byDev.size()) ? byDev[size_t(dev)] : nullptr;
  }
};

template <typename F> static bool sym(void *lib, const char *name, F *out) {
  *out = reinterpret_cast<F>(dlsym(lib, name));
  return *out != nullptr;
}

const Smi &smi() {
  static Smi s = [] {
    Smi r;
    if (env::get_int("STENCIL_AMDSMI", 0) == 0) return r;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
      (void)hipGetLastError();
      return r;
    }
    void *lib = dlopen("libamd_smi.so", RTLD_NOW | RTLD_LOCAL);
    if (!lib) lib = dlopen("/opt/rocm/lib/libamd_smi.so", RTLD_NOW | RTLD_LOCAL);
    if (!lib) return r;
    amdsmi_status_t (*init)(uint64_t) = nullptr;
    amdsmi_status_t (*sockets)(uint32_t *, amdsmi_socket_handle *) = nullptr;
    amdsmi_status_t (*procs)(amdsmi_socket_handle, uint32_t *, amdsmi_processor_handle *) = nullptr;
    amdsmi_status_t (*bdf)(amdsmi_processor_handle, amdsmi_bdf_t *) = nullptr;
    if (!sym(lib, "amdsmi_init", &init) || !sym(lib, "amdsmi_get_socket_handles", &sockets) ||
        !sym(lib, "amdsmi_get_processor_handles", &procs) || !sym(lib, "amdsmi_get_gpu_device_bdf", &bdf) ||
        !sym(lib, "amdsmi_topo_get_link_type", &r.link_type) || !sym(lib, "amdsmi_topo_get_link_weight", &r.link_weight) ||
        !sym(lib, "amdsmi_get_minmax_bandwidth_between_processors", &r.minmax_bw) ||
        !sym(lib, "amdsmi_topo_get_numa_node_number", &r.numa))
      return r;
    if (init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return r;
    if (sym(lib, "amdsmi_shut_down", &g_smi_shutdown))
      std::atexit([] { (void)g_smi_shutdown(); });
    uint32_t ns = 0;
    if (sockets(&ns, nullptr) != AMDSMI_STATUS_SUCCESS || ns == 0) return r;
    std::vector<amdsmi_socket_handle> sh(ns);
    if (sockets(&ns, sh.data()) != AMDSMI_STATUS_SUCCESS) return r;
    std::map<uint64_t, amdsmi_processor_handle> byBdf; // (domain, bus, device, function) packed
    auto key = [](uint64_t dom, uint64_t bus, uint64_t d, uint64_t f) { return (dom << 16) | (bus << 8) | (d << 3) | f; };
    for (auto s0 : sh) {
      uint32_t np = 0;
      if (procs(s0, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      if (procs(s0, &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
      for (auto p : ph) {
        amdsmi_bdf_t b{};
        if (bdf(p, &b) == AMDSMI_STATUS_SUCCESS)
          byBdf[key(b.domain_number, b.bus_number, b.device_number, b.function_number)] = p;
      }
    }
    r.byDev.assign(size_t(ndev), nullptr);
    int matched = 0;
    for (int d = 0; d < ndev; ++d) {
      char bus[64] = {0};
      if (hipDeviceGetPCIBusId(bus, sizeof(bus), d) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      unsigned dom = 0, b = 0, dv = 0, fn = 0;
      if (std::sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn) != 4) continue;
      auto it = byBdf.find(key(dom, b, dv, fn));
      if (it != byBdf.end()) {
        r.byDev[size_t(d)] = it->second;
        ++matched;
      }
    }
    r.ok = matched > 0;
    LOG_DEBUG("amd-smi: " << byBdf.size() << " GPUs, " << matched << " matched to HIP devices");
    return r;
  }();
  return s;
}
} // namespace

bool smi_available() { return smi().ok; }

int numa_node(int dev) {
  // sysfs: the PCI function's NUMA node (amd-smi only when enabled and sysfs has no answer)
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  std::string b(bus);
  for (auto &c : b) c = char(std::tolower(c));
  std::ifstream f("/sys/bus/pci/devices/" + b + "/numa_node");
  int node = -1;
  if (f >> node && node >= 0) return node;
  const Smi &s = smi();
  amdsmi_processor_handle h = s.handle(dev);
  uint32_t n = 0;
  if (h && s.numa(h, &n) == AMDSMI_STATUS_SUCCESS) return int(n);
  return -1;
}

std::vector<int> numa_cpus(int node) {
  std::vector<int> cpus;
  if (node < 0) return cpus;
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!(f >> list)) return cpus;
  std::stringstream ss(list);
  std::string part;
  while (std::getline(ss, part, ',')) {
    const size_t dash = part.find('-');
    try {
      const int a = std::stoi(part.substr(0, dash));
      const int b = dash == std::string::npos ? a : std::stoi(part.substr(dash + 1));
      for (int c = a; c <= b; ++c) cpus.push_back(c);
    } catch (...) {
      return {};
    }
  }
  return cpus;
}

bool bind_thread_to_numa(int node) {
  const std::vector<int> cpus = numa_cpus(node);
  if (cpus.empty()) return false;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c < CPU_SETSIZE) CPU_SET(c, &set);
  // keep only CPUs this process may use at all (a container / cgroup cpuset may exclude some)
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
    CPU_AND(&set, &set, &allowed);
    if (CPU_COUNT(&set) == 0) return false;
  }
  return sched_setaffinity(0, sizeof(set), &set) == 0;
}

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

// amd-smi link type / hops; false when unavailable
static bool smi_link(int a, int b, amdsmi_link_type_t *type, uint64_t *hops) {
  const Smi &s = smi();
  amdsmi_processor_handle ha = s.handle(a), hb = s.handle(b);
  return ha && hb && s.link_type(ha, hb, hops, type) == AMDSMI_STATUS_SUCCESS;
}

double distance(int src, int dst) {
  if (src == dst) return 0.1;
  {
    amdsmi_link_type_t t{};
    uint64_t h = 0;
    if (smi_link(src, dst, &t, &h)) {
      if (t == AMDSMI_LINK_TYPE_XGMI) return h <= 1 ? 1.0 : 1.0 + double(h - 1);
      if (t == AMDSMI_LINK_TYPE_PCIE) return 3.0 + double(h);
      if (t == AMDSMI_LINK_TYPE_INTERNAL) return 0.5;
    }
  }
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
      LinkInfo li{a, b, "self", 0, distance(a, b), -1, -1, -1, "none"};
      li.source = "none";
      if (a != b) {
        amdsmi_link_type_t st{};
        uint64_t sh = 0;
        uint32_t t = 0, h = 0;
        if (smi_link(a, b, &st, &sh)) {
          li.source = "amd-smi";
          li.type = st == AMDSMI_LINK_TYPE_XGMI ? "xgmi" : (st == AMDSMI_LINK_TYPE_PCIE ? "pcie" : "other");
          li.hops = int(sh);
          const Smi &s = smi();
          uint64_t w = 0, mn = 0, mx = 0;
          if (s.link_weight(s.handle(a), s.handle(b), &w) == AMDSMI_STATUS_SUCCESS) li.weight = int64_t(w);
          if (s.minmax_bw(s.handle(a), s.handle(b), &mn, &mx) == AMDSMI_STATUS_SUCCESS) {
            li.minBwMBs = int64_t(mn);
            li.maxBwMBs = int64_t(mx);
          }
        } else if (query_link(a, b, &t, &h)) {
          li.source = "hip";
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
