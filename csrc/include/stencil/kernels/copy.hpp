#pragma once
// Descriptor-driven strided box copies: the single primitive behind pack, unpack, same-GPU translate,
// direct xGMI peer stores and region->host dumps.
//
// Reference equivalents (one CUDA launch per message, make_block_dim shapes, per-element memcpy fallback):
//   grid_pack/pack_kernel        include/stencil/pack_kernel.cuh:5-46
//   unpack/translate/multi_*     include/stencil/copy.cuh:13-145
//   dev_packer_pack_domain       include/stencil/packer.cuh:52-69
//   dev_unpacker_unpack_domain   include/stencil/packer.cuh:233-250
// Here every message x quantity of one exchange step becomes one CopySeg and ONE launch walks them all:
// rows are split into the widest aligned vector unit (16/8/4/2/1 B) so face copies move 1 KiB per wave
// instruction, and the launch is sized for the whole chip (>= 2 waves/SIMD) instead of per-message blocks.
#include <cstdint>
#include <vector>

#include "stencil/core/geometry.hpp"

#if defined(__HIPCC__) || defined(__HIP_PLATFORM_AMD__)
#include <hip/hip_runtime_api.h>
#else
#include <hip/hip_runtime_api.h>
#endif

namespace stencil {

// Address of element (x,y,z) of a strided box: base + x*elem + y*ystride + z*zstride (bytes).
struct StridedBox {
  char *base = nullptr;
  int64_t ystride = 0;
  int64_t zstride = 0;
};

struct CopySeg {
  char *src;
  char *dst;
  int64_t src_ystride, src_zstride;
  int64_t dst_ystride, dst_zstride;
  uint32_t row_units; // vector units per row
  uint32_t ny;        // rows per z-plane
  uint32_t vec;       // bytes per unit (16, 8, 4, 2 or 1)
  uint32_t flags;     // kSegWide: always one unit per item, even for rows of <= kNarrowMaxUnits units
  uint64_t unit_begin; // exclusive prefix sum of units over previous segments
  uint64_t units;      // row_units * ny * nz
  // device plans only: a second copy of the same shape and strides done by the same items (make_copy_plan pairs
  // narrow-row segments, e.g. the +x and -x faces of a periodic self-wrap, whose rows share cache lines)
  char *src2;
  char *dst2;
};

// Build a segment copying a box of extent `ext` elements of `elemSize` bytes.
CopySeg make_copy_seg(const StridedBox &src, const StridedBox &dst, const Dim3 &ext, int64_t elemSize);

// Assign unit_begin prefix sums; returns total units.
uint64_t finalize_segs(std::vector<CopySeg> &segs);

// Host execution (CPU backend and reference for tests).
void copy_segs_host(const std::vector<CopySeg> &segs);

// Device execution plan: the segment list plus a per-block work table built on the host, so every block reads
// its (segment, first item, count) with scalar loads and never searches. Items are whole rows for narrow rows
// (x-faces: <= 4 units per row) and single vector units otherwise.
// Rows of at most this many vector units are copied one row per item (narrow rows, e.g. x faces); wider rows one
// unit per item. make_copy_plan and the kernel's per-row template dispatch share this bound.
constexpr uint32_t kNarrowMaxUnits = 4;
// rows of whole 64-B sectors (x faces widened to sectors): 4 consecutive lanes move one row, so every wave
// instruction reads / writes 16 complete sectors instead of 64 partial ones
constexpr uint32_t kSegWide = 1;
struct CopyWork {
  uint32_t seg;
  uint32_t first;
  uint32_t count;
  uint32_t rows; // 1: items are rows, 0: items are units
};
struct CopyPlan {
  CopySeg *dsegs = nullptr;
  CopyWork *dwork = nullptr;  // entries for one block each (copy_plan_kernel)
  CopyWork *dworkG = nullptr; // entries of 1024 items for the grid-stride kernels (few-CU and fused transport)
  int nsegs = 0;
  int nwork = 0;
  int nworkG = 0;
  int device = -1;
  uint64_t bytes = 0;
};
// build + upload (device must be current). Segments must be finalized.
CopyPlan make_copy_plan(const std::vector<CopySeg> &segs, int device);
// items per work-table entry (= per 256-thread block of copy_plan_kernel) for narrow-row segments (x faces: one row
// per item) and for wide segments (one 16-B unit per item); plans built afterwards use them. Defaults 1024 / 512.
// The grid-stride kernels (copy_plan_device with maxBlocks, copy_plan_device_sync) always use 1024-item entries.
void set_copy_block_items(uint32_t narrow, uint32_t wide);
// row segments of at most maxItems rows (edges) get entries of perEntry rows (plans built afterwards; 4096 / 64)
void set_copy_small_rows(uint32_t maxItems, uint32_t perEntry);
void free_copy_plan(CopyPlan &p);
// maxBlocks > 0: at most that many 1024-thread blocks (one CU each) walk the work table (see copy.hip)
void copy_plan_device(const CopyPlan &p, hipStream_t stream, int maxBlocks = 0);
// one-shot helper (allocates a temporary plan, synchronous)
void copy_segs_device_sync(std::vector<CopySeg> segs, int device);

// ---- cross-process signalling for the IPC transport (device flags, see DistributedDomain colocated path) ----
// Lane i polls *flags[i] (relaxed, system scope, s_sleep back-off) until >= target, then one system-scope
// acquire. A bounded spin: on timeout it stores `code` into *err (host-mapped) and exits, so the grid always drains.
void wait_flags_device(const std::vector<uint64_t *> &flags, uint64_t target, int *err, int code, double timeout_s,
                       hipStream_t stream);
// System-scope release, then lane i stores *flags[i] = value (flags may be IPC-mapped peer memory).
void signal_flags_device(const std::vector<uint64_t *> &flags, uint64_t value, hipStream_t stream);
constexpr int kMaxFlagsPerLaunch = 64;
// Grid cap of the fused wait + copy + signal kernels on a GPU that other ranks drive too: every block spins until
// the peer's flags arrive, and a spinning block holds its CU. Uncapped (one 1024-thread block per CU) two ranks
// sharing a GPU could fill every CU slot with waiting blocks while the peers they wait for cannot start their pack
// kernels: four ranks on one MI355X (1x2x2) deadlocked until the wait timeout (gpurun_out/r3e, r3). 32 CUs still
// move a 2-MiB face in a few us. A GPU this rank drives alone has no such peer on its CUs: there the grid is only
// bounded by the work and the caller's maxBlocks (FlagSyncArgs::sharedGpu = false).
constexpr int kFusedMaxBlocks = 32;
// One fused launch: wait until every `wait` flag >= waitTarget (bounded: on timeout `code` goes to *err), run the
// copy plan on at most maxBlocks 1024-thread blocks (0: up to one per CU), then release-store signalValue into every
// `signal` flag once all blocks are done (`counter`: a zeroed device word, reset by the kernel; one per stream).
struct FlagSyncArgs {
  std::vector<uint64_t *> wait;
  uint64_t waitTarget = 0;
  // producer gate (pipelined pairs): local words, e.g. the boundary-plane counter a stencil sweep that is still
  // running publishes (StencilTune::publish), polled before the copies as well, with their own target
  std::vector<uint64_t *> gate;
  uint64_t gateTarget = 0;
  std::vector<uint64_t *> signal;
  uint64_t signalValue = 0;
  uint32_t *counter = nullptr;
  int *err = nullptr;
  int code = 0;
  double timeout_s = 60;
  bool sharedGpu = true; // another rank drives this GPU: cap the grid at kFusedMaxBlocks
  // STENCIL_EXCHANGE_STATS builds: when non-null, block 0 stores s_memrealtime stamps (100-MHz constant clock) at
  // kernel start, after the flag wait and after its copies into stamps[0..2], and the last block its signal time
  // into stamps[3] (wait vs copy breakdown of the fused transport kernels)
  uint64_t *stamps = nullptr;
};
void copy_plan_device_sync(const CopyPlan &p, hipStream_t stream, int maxBlocks, const FlagSyncArgs &a);

// one wave that keeps the stream busy for `seconds` of the 100-MHz constant clock (tests: work an event is recorded
// behind); 0 = an empty marker kernel
void spin_device(double seconds, hipStream_t stream);

} // namespace stencil
