#pragma once
// GPU topology: distance/bandwidth between devices and peer-access management.
// Parity: reference include/stencil/gpu_topology.hpp + src/gpu_topology.cpp:17-139
//   (NVML distance: same 0.1, NVLink 1, PCIe levels 2-7; bandwidth = 1/distance; cached enable_peer / peer).
// MI355X: the link type, hop count, link weight and min/max link bandwidth come from amd-smi (libamd_smi, loaded
// at run time, devices matched by PCI address; the analogue of the reference's NVML queries), falling back to
// hipExtGetLinkTypeAndHopCount. A fully connected 8-GPU xGMI node is a uniform mesh: distance 1.0 for every pair,
// 0.1 for self.
#include <cstdint>
#include <string>
#include <vector>

namespace stencil {
namespace gpu_topo {

int device_count(); // 0 when no GPU runtime/device is present

// relative distance between two devices of this node (smaller is closer)
double distance(int src, int dst);
inline double bandwidth(int src, int dst) { return 1.0 / distance(src, dst); }

// try to enable peer access src->dst (cached). Returns whether src can access dst memory.
bool enable_peer(int src, int dst);
// cached answer of enable_peer (enables on first use)
bool peer(int src, int dst);

struct LinkInfo {
  int src, dst;
  std::string type; // "self", "xgmi", "pcie", "unknown"
  int hops;
  double distance;
  int64_t weight = -1;                 // amd-smi link weight (-1: unavailable)
  int64_t minBwMBs = -1, maxBwMBs = -1; // amd-smi min/max io-link bandwidth (MB/s, -1: unavailable)
  std::string source;                  // "amd-smi", "hip" or "none"
};
std::vector<LinkInfo> links();
// NUMA node of a device (amd-smi, else the PCI function's sysfs entry), -1 if unknown
int numa_node(int dev);
// CPUs of a NUMA node (sysfs cpulist), empty if unknown
std::vector<int> numa_cpus(int node);
// restrict the calling thread (and the threads it creates later) to the CPUs of `node` that this process may use;
// false if the node or its CPUs are unknown. Host-staged buffers allocated afterwards are first touched there.
bool bind_thread_to_numa(int node);
// whether the amd-smi library was found and initialised
bool smi_available();

} // namespace gpu_topo
} // namespace stencil
