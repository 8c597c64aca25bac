// Descriptor-driven strided box copies for gfx950 (see stencil/kernels/copy.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "stencil/kernels/copy.hpp"
#include "stencil/rt/hip_check.hpp"

namespace stencil {

static inline bool aligned(uint64_t v, uint32_t a) { return (v & (a - 1)) == 0; }

CopySeg make_copy_seg(const StridedBox &src, const StridedBox &dst, const Dim3 &ext, int64_t elemSize) {
  CopySeg s{};
  s.src = src.base;
  s.dst = dst.base;
  s.src_ystride = src.ystride;
  s.src_zstride = src.zstride;
  s.dst_ystride = dst.ystride;
  s.dst_zstride = dst.zstride;
  const uint64_t rowBytes = uint64_t(ext.x) * uint64_t(elemSize);
  uint32_t vec = 16;
  while (vec > 1) {
    if (aligned(rowBytes, vec) && aligned(uint64_t(uintptr_t(src.base)), vec) &&
        aligned(uint64_t(uintptr_t(dst.base)), vec) && aligned(uint64_t(src.ystride), vec) &&
        aligned(uint64_t(src.zstride), vec) && aligned(uint64_t(dst.ystride), vec) && aligned(uint64_t(dst.zstride), vec))
      break;
    vec >>= 1;
  }
  s.vec = vec;
  s.row_units = uint32_t(rowBytes / vec);
  s.ny = uint32_t(ext.y);
  s.units = (ext.x > 0 && ext.y > 0 && ext.z > 0) ? uint64_t(s.row_units) * uint64_t(ext.y) * uint64_t(ext.z) : 0;
  return s;
}

uint64_t finalize_segs(std::vector<CopySeg> &segs) {
  // drop empty segments, keep order
  segs.erase(std::remove_if(segs.begin(), segs.end(), [](const CopySeg &s) { return s.units == 0; }), segs.end());
  uint64_t acc = 0;
  for (auto &s : segs) {
    s.unit_begin = acc;
    acc += s.units;
  }
  return acc;
}

void copy_segs_host(const std::vector<CopySeg> &segs) {
  for (const auto &s : segs) {
    if (!s.units) continue;
    const uint64_t rowBytes = uint64_t(s.row_units) * s.vec;
    const uint64_t rows = s.units / s.row_units;
    for (uint64_t r = 0; r < rows; ++r) {
      const uint64_t y = r % s.ny, z = r / s.ny;
      std::memmove(s.dst + z * s.dst_zstride + y * s.dst_ystride, s.src + z * s.src_zstride + y * s.src_ystride,
                   rowBytes);
    }
  }
}

template <uint32_t V> struct VecOf;
// clang vector types, not HIP's uint4/uint2 (union structs that SROA will not split: the item arrays below then
// stay a private stack frame)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <> struct VecOf<16> { using T = u32x4; };
template <> struct VecOf<8> { using T = u32x2; };
template <> struct VecOf<4> { using T = uint32_t; };
template <> struct VecOf<2> { using T = uint16_t; };
template <> struct VecOf<1> { using T = uint8_t; };

// One block per work-table entry; the entry and its segment are wave-uniform (scalar loads). Narrow-row segments
// (x-faces) assign one row per item, wide rows one 16-B unit per item, so a y/z face moves 1 KiB per wave
// instruction and the strided x-face rows are spread over every lane. Each thread owns up to kItems items
// (stride 256) and issues all their loads before any store, so the scattered x-face accesses of a thread are in
// flight together instead of one round trip per item.
constexpr uint32_t kItemsMax = 4;

// N = units per item (1 for wide rows, row_units for narrow rows) is a template value: the per-thread register
// arrays are then indexed by constants only and live in VGPRs (with a runtime n guard they stayed a 528-B private
// stack frame: scratch traffic and a scratch setup on every launch).
template <uint32_t V, uint32_t N, bool PAIR>
__device__ __forceinline__ void copy_items(const CopySeg &s, const CopyWork &w, uint32_t tid) {
  using T = typename VecOf<V>::T;
  // items in flight per thread: kItems, fewer when one item's data takes over 16 VGPRs (wide narrow-row pairs),
  // so the 1024-thread form stays within its 128-VGPR budget without spilling
  constexpr uint32_t kRegs = (N * (V < 4 ? 4 : V) / 4) * (PAIR ? 2 : 1);
  constexpr uint32_t kItems = kRegs > 16 ? (kRegs > 32 ? 1 : 2) : kItemsMax;
  const uint32_t ru = s.row_units, ny = s.ny;
  const int64_t sys = s.src_ystride, szs = s.src_zstride, dys = s.dst_ystride, dzs = s.dst_zstride;
  for (uint32_t base = tid; base < w.count; base += 256 * kItems) {
    T v[kItems][N], v2[kItems][PAIR ? N : 1];
    int64_t doff[kItems];
    bool live[kItems];
#pragma unroll
    for (uint32_t k = 0; k < kItems; ++k) {
      const uint32_t it = base + k * 256;
      live[k] = it < w.count;
      const uint32_t item = w.first + (live[k] ? it : 0);
      uint32_t r, c;
      if (w.rows) {
        r = item;
        c = 0;
      } else {
        r = item / ru;
        c = item - r * ru;
      }
      const uint32_t y = r % ny, z = r / ny;
      const int64_t soff = int64_t(z) * szs + int64_t(y) * sys + int64_t(c) * V;
      doff[k] = int64_t(z) * dzs + int64_t(y) * dys + int64_t(c) * V;
      if (live[k]) {
        const T *sp = reinterpret_cast<const T *>(s.src + soff);
#pragma unroll
        for (uint32_t u = 0; u < N; ++u) v[k][u] = sp[u];
        if constexpr (PAIR) {
          const T *sp2 = reinterpret_cast<const T *>(s.src2 + soff);
#pragma unroll
          for (uint32_t u = 0; u < N; ++u) v2[k][u] = sp2[u];
        }
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kItems; ++k)
      if (live[k]) {
        T *dp = reinterpret_cast<T *>(s.dst + doff[k]);
#pragma unroll
        for (uint32_t u = 0; u < N; ++u) dp[u] = v[k][u];
        if constexpr (PAIR) {
          T *dp2 = reinterpret_cast<T *>(s.dst2 + doff[k]);
#pragma unroll
          for (uint32_t u = 0; u < N; ++u) dp2[u] = v2[k][u];
        }
      }
  }
}

template <uint32_t V, bool PAIR> __device__ __forceinline__ void copy_work_v(const CopySeg &s, const CopyWork &w, uint32_t tid) {
  switch (w.rows ? s.row_units : 1u) {
  case 1:
    copy_items<V, 1, PAIR>(s, w, tid);
    break;
  case 2:
    copy_items<V, 2, PAIR>(s, w, tid);
    break;
  case 3:
    copy_items<V, 3, PAIR>(s, w, tid);
    break;
  case 4:
    copy_items<V, 4, PAIR>(s, w, tid);
    break;
  default:
    // make_copy_plan marks a segment as rows only when row_units <= kNarrowMaxUnits: anything else is a planner bug
    __builtin_trap();
  }
  static_assert(kNarrowMaxUnits == 4, "copy_work_v dispatches row widths 1..4");
}

template <bool PAIR> __device__ __forceinline__ void copy_work_t(const CopySeg &s, const CopyWork &w, uint32_t tid) {
  switch (s.vec) {
  case 16:
    copy_work_v<16, PAIR>(s, w, tid);
    break;
  case 8:
    copy_work_v<8, PAIR>(s, w, tid);
    break;
  case 4:
    copy_work_v<4, PAIR>(s, w, tid);
    break;
  case 2:
    copy_work_v<2, PAIR>(s, w, tid);
    break;
  default:
    copy_work_v<1, PAIR>(s, w, tid);
    break;
  }
}

__device__ __forceinline__ void copy_work(const CopySeg &s, const CopyWork &w, uint32_t tid) {
  if (s.src2)
    copy_work_t<true>(s, w, tid);
  else
    copy_work_t<false>(s, w, tid);
}

__global__ __launch_bounds__(256) void copy_plan_kernel(const CopySeg *__restrict__ segs,
                                                        const CopyWork *__restrict__ work) {
  const CopyWork w = work[blockIdx.x];
  copy_work(segs[w.seg], w, threadIdx.x);
}

// Few-CU form (copy_plan_device with maxBlocks): 1024-thread blocks of four independent 256-thread groups, each
// walking the work table with a grid stride. A launch of B blocks then occupies at most B CUs for its whole
// duration, so it can run beside a grid that holds every other CU (an overlapped interior sweep) without taking
// the CUs that grid's blocks need.
__global__ __launch_bounds__(1024) void copy_plan_kernel_narrow(const CopySeg *__restrict__ segs,
                                                                const CopyWork *__restrict__ work, uint32_t nwork) {
  const uint32_t g = threadIdx.x >> 8; // wave-uniform (a group is 4 whole waves)
  for (uint32_t wi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + g); wi < nwork; wi += gridDim.x * 4) {
    const CopyWork w = work[wi];
    copy_work(segs[w.seg], w, threadIdx.x & 255);
  }
}

// Pair narrow-row segments of identical shape and strides: one item then copies the same row of both (the +x and
// -x faces of a periodic self-wrap read and write the first and last line of every row: paired, each line is
// fetched once). Copies in one plan are independent (one launch runs them concurrently anyway), so any pairing
// is valid; the first compatible partner is taken.
static std::vector<CopySeg> pair_narrow_segs(const std::vector<CopySeg> &in) {
  std::vector<CopySeg> out;
  std::vector<bool> used(in.size(), false);
  auto narrow = [](const CopySeg &s) {
    return s.units && s.row_units <= kNarrowMaxUnits && !s.src2 && !(s.flags & kSegWide);
  };
  auto compatible = [&](const CopySeg &a, const CopySeg &b) {
    return narrow(b) && b.vec == a.vec && b.row_units == a.row_units && b.ny == a.ny && b.units == a.units &&
           b.src_ystride == a.src_ystride && b.src_zstride == a.src_zstride && b.dst_ystride == a.dst_ystride &&
           b.dst_zstride == a.dst_zstride;
  };
  // first choice: a partner whose rows write the same 128-B line (shared halo lines: row y's +x halo and row y+1's
  // -x halo), so the line is written once, by one item
  auto sameLine = [](const CopySeg &a, const CopySeg &b) {
    return uintptr_t(a.dst) / 128 == uintptr_t(b.dst) / 128 && uintptr_t(a.dst) + a.row_units * a.vec <= uintptr_t(b.dst) + 128;
  };
  std::vector<long> partner(in.size(), -1);
  for (int pass = 0; pass < 2; ++pass)
    for (size_t i = 0; i < in.size(); ++i) {
      if (used[i] || !narrow(in[i])) continue;
      for (size_t j = i + 1; j < in.size(); ++j) {
        if (used[j] || !compatible(in[i], in[j]) || (pass == 0 && !sameLine(in[i], in[j]))) continue;
        partner[i] = long(j);
        used[i] = used[j] = true;
        break;
      }
    }
  // emitted in the input order (the dispatch order of the work table matters for speed, profiles/r4/ad)
  for (size_t i = 0; i < in.size(); ++i) {
    if (used[i] && partner[i] < 0) continue; // the second half of a pair
    CopySeg a = in[i];
    if (partner[i] >= 0) {
      a.src2 = in[size_t(partner[i])].src;
      a.dst2 = in[size_t(partner[i])].dst;
    }
    out.push_back(a);
  }
  return out;
}

// 512 16-B units per block for wide rows (two per thread) and 1024 rows per block for narrow ones: the 512^3
// radius-2-face self-exchange (bench_exchange config 3) on one MI355X, interleaved over 6 rounds
// (scripts/mi355x/copy_items_probe.py, profiles/r4/x/): wide 1024 -> 512 blocking 280.7-293.1 -> 332.5-345.3 GB/s,
// stream-ordered 438-440 -> 526-537; wide 384 / 640 in between, 128 worse; narrow below 1024 worse (768: 272)
static uint32_t gNarrowBlockItems = 256 * kItemsMax, gWideBlockItems = 512;

static uint32_t gSmallRowSeg = 4096, gSmallRowItems = 64;
void set_copy_small_rows(uint32_t maxItems, uint32_t perEntry) {
  STENCIL_REQUIRE(perEntry >= 1, "items per entry must be positive");
  gSmallRowSeg = maxItems;
  gSmallRowItems = perEntry;
}

void set_copy_block_items(uint32_t narrow, uint32_t wide) {
  STENCIL_REQUIRE(narrow >= 1 && narrow <= 256 * kItemsMax && wide >= 1 && wide <= 256 * kItemsMax,
                  "items per block must be 1.." << 256 * kItemsMax);
  gNarrowBlockItems = narrow;
  gWideBlockItems = wide;
}

// work table of `segs` with at most `narrow` rows / `wide` units per entry
static std::vector<CopyWork> work_table(const std::vector<CopySeg> &segs, uint32_t narrow, uint32_t wide) {
  std::vector<CopyWork> work;
  for (uint32_t si = 0; si < segs.size(); ++si) {
    const CopySeg &s = segs[si];
    if (!s.units) continue;
    const bool rows = s.row_units <= kNarrowMaxUnits && !(s.flags & kSegWide);
    const uint64_t items = rows ? s.units / s.row_units : s.units;
    STENCIL_REQUIRE(items < (1ull << 32), "copy segment too large");
    // small row segments (edges: a few hundred scattered cells) are split finer, so their latency-bound items run
    // on many blocks at once instead of trailing behind the faces in one
    const uint32_t per = rows ? (items <= gSmallRowSeg ? std::min<uint32_t>(narrow, gSmallRowItems) : narrow) : wide;
    for (uint64_t f = 0; f < items; f += per)
      work.push_back({si, uint32_t(f), uint32_t(std::min<uint64_t>(per, items - f)), rows ? 1u : 0u});
  }
  return work;
}

CopyPlan make_copy_plan(const std::vector<CopySeg> &segsIn, int device) {
  CopyPlan p;
  p.device = device;
  std::vector<CopySeg> segs = pair_narrow_segs(segsIn);
  finalize_segs(segs);
  for (const CopySeg &s : segs) p.bytes += s.units * s.vec * (s.src2 ? 2 : 1);
  // one block per entry (copy_plan_kernel): the tuned sizes; grid-stride kernels (few-CU and fused transport
  // kernels) walk entries of 1024 items, four in flight per thread, which their fixed number of groups needs
  const std::vector<CopyWork> work = work_table(segs, gNarrowBlockItems, gWideBlockItems);
  const std::vector<CopyWork> workG = work_table(segs, 256 * kItemsMax, 256 * kItemsMax);
  p.nsegs = int(segs.size());
  p.nwork = int(work.size());
  p.nworkG = int(workG.size());
  if (p.nwork == 0) return p;
  HIP_CHECK(hipMalloc(&p.dsegs, sizeof(CopySeg) * segs.size()));
  HIP_CHECK(hipMemcpy(p.dsegs, segs.data(), sizeof(CopySeg) * segs.size(), hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&p.dwork, sizeof(CopyWork) * work.size()));
  HIP_CHECK(hipMemcpy(p.dwork, work.data(), sizeof(CopyWork) * work.size(), hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&p.dworkG, sizeof(CopyWork) * workG.size()));
  HIP_CHECK(hipMemcpy(p.dworkG, workG.data(), sizeof(CopyWork) * workG.size(), hipMemcpyHostToDevice));
  return p;
}

void free_copy_plan(CopyPlan &p) {
  if (p.dsegs) (void)hipFree(p.dsegs);
  if (p.dwork) (void)hipFree(p.dwork);
  if (p.dworkG) (void)hipFree(p.dworkG);
  p.dsegs = nullptr;
  p.dwork = nullptr;
  p.dworkG = nullptr;
  p.nwork = 0;
  p.nworkG = 0;
}

void copy_plan_device(const CopyPlan &p, hipStream_t stream, int maxBlocks) {
  if (!p.nwork) return;
  if (maxBlocks > 0) {
    const int blocks = std::min(maxBlocks, (p.nworkG + 3) / 4);
    hipLaunchKernelGGL(copy_plan_kernel_narrow, dim3(blocks), dim3(1024), 0, stream, p.dsegs, p.dworkG,
                       uint32_t(p.nworkG));
  } else {
    hipLaunchKernelGGL(copy_plan_kernel, dim3(p.nwork), dim3(256), 0, stream, p.dsegs, p.dwork);
  }
  HIP_CHECK(hipGetLastError());
}

void copy_segs_device_sync(std::vector<CopySeg> segs, int device) {
  finalize_segs(segs);
  // the copy runs on the null stream, which does not order against the non-blocking compute/comm streams: wait for
  // every kernel that may still write the source (e.g. a dump right after StencilModel::run() without synchronize())
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipDeviceSynchronize());
  CopyPlan p = make_copy_plan(segs, device);
  copy_plan_device(p, nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  free_copy_plan(p);
}

// ------------------------------------------------------------------------------------------------
// device flags
// ------------------------------------------------------------------------------------------------
struct FlagList {
  uint64_t *p[kMaxFlagsPerLaunch];
  int n;
};

// lanes i < f.n of the calling wave poll *f.p[i] until >= target (relaxed, system scope, s_sleep back-off); bounded:
// past timeoutTicks of the 100-MHz constant clock the lane stores `code` into *err and gives up
__device__ __forceinline__ void poll_flags(const FlagList &f, uint64_t target, int *err, int code,
                                           uint64_t timeoutTicks, int lane) {
  if (lane < f.n) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      const uint64_t v = __hip_atomic_load(f.p[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v >= target) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeoutTicks) {
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
}

struct FlagSync {
  FlagList wait;        // polled before any copy (n = 0: none)
  uint64_t waitTarget;
  FlagList gate;        // also polled before any copy (producer gate, own target)
  uint64_t gateTarget;
  FlagList signal;      // stored after every block's copies are done
  uint64_t signalValue;
  uint32_t *counter;    // blocks done; 0 at launch, reset by the last block
  int *err;
  int code;
  uint64_t timeoutTicks;
  uint64_t *stamps;     // transport log entry (4 words) or null
};

// Fused transport step (Colocated sends / receives): wait for the peer's flags, run the copy plan, raise the
// peer's flags -- one launch instead of three (each one-wave flag kernel costs ~4.5 us of serial stream time on
// MI355X, profiles/r3/cliff/gaps_mp2x_exchange_loop.txt). Every block waits for itself (the flags are few and
// uncached). The signal follows the classic last-block pattern: each block's thread 0 publishes the block's copies
// with a system-scope release fence and counts itself done; the block that completes the count acquires every
// other block's publication and release-stores the flags.
__global__ __launch_bounds__(1024) void copy_plan_kernel_sync(const CopySeg *__restrict__ segs,
                                                              const CopyWork *__restrict__ work, uint32_t nwork,
                                                              FlagSync fs) {
  // transport log (FlagSyncArgs::stamps): block 0 records start / after the wait / after its copies
  const bool stamp = fs.stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
  const uint64_t tStart = stamp ? __builtin_amdgcn_s_memrealtime() : 0;
  if (fs.wait.n > 0 || fs.gate.n > 0) {
    if (threadIdx.x < 64) {
      poll_flags(fs.wait, fs.waitTarget, fs.err, fs.code, fs.timeoutTicks, int(threadIdx.x));
      poll_flags(fs.gate, fs.gateTarget, fs.err, fs.code, fs.timeoutTicks, int(threadIdx.x));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // the peer's slot writes / reads before our copies
    __syncthreads();
  }
  if (stamp) {
    fs.stamps[0] = tStart;
    fs.stamps[1] = __builtin_amdgcn_s_memrealtime();
  }
  const uint32_t g = threadIdx.x >> 8; // wave-uniform (a group is 4 whole waves)
  for (uint32_t wi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + g); wi < nwork; wi += gridDim.x * 4) {
    const CopyWork w = work[wi];
    copy_work(segs[w.seg], w, threadIdx.x & 255);
  }
  if (fs.signal.n == 0 && fs.stamps == nullptr) return;
  __syncthreads();
  if (stamp) fs.stamps[2] = __builtin_amdgcn_s_memrealtime();
  if (fs.signal.n == 0) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const uint32_t done = __hip_atomic_fetch_add(fs.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      for (int i = 0; i < fs.signal.n; ++i)
        __hip_atomic_store(fs.signal.p[i], fs.signalValue, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(fs.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fs.stamps != nullptr) fs.stamps[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

__global__ void wait_flags_kernel(FlagList f, uint64_t target, int *err, int code, uint64_t timeoutTicks) {
  poll_flags(f, target, err, code, timeoutTicks, int(threadIdx.x));
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
}

__global__ void signal_flags_kernel(FlagList f, uint64_t value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system scope: prior kernels' peer stores are ordered before
  const int i = threadIdx.x;
  if (i < f.n) __hip_atomic_store(f.p[i], value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static FlagList to_list(const std::vector<uint64_t *> &flags) {
  STENCIL_REQUIRE(flags.size() <= size_t(kMaxFlagsPerLaunch), "too many flags in one launch: " << flags.size());
  FlagList f{};
  f.n = int(flags.size());
  for (size_t i = 0; i < flags.size(); ++i) f.p[i] = flags[i];
  return f;
}

void wait_flags_device(const std::vector<uint64_t *> &flags, uint64_t target, int *err, int code, double timeout_s,
                       hipStream_t stream) {
  if (flags.empty()) return;
  const uint64_t ticks = uint64_t(timeout_s * 1e8);
  hipLaunchKernelGGL(wait_flags_kernel, dim3(1), dim3(64), 0, stream, to_list(flags), target, err, code, ticks);
  HIP_CHECK(hipGetLastError());
}

void copy_plan_device_sync(const CopyPlan &p, hipStream_t stream, int maxBlocks, const FlagSyncArgs &a) {
  FlagSync fs{};
  fs.wait = to_list(a.wait);
  fs.waitTarget = a.waitTarget;
  fs.gate = to_list(a.gate);
  fs.gateTarget = a.gateTarget;
  fs.signal = to_list(a.signal);
  fs.signalValue = a.signalValue;
  fs.counter = a.counter;
  fs.err = a.err;
  fs.code = a.code;
  fs.timeoutTicks = uint64_t(a.timeout_s * 1e8);
  fs.stamps = a.stamps;
  STENCIL_REQUIRE(fs.signal.n == 0 || a.counter, "copy_plan_device_sync: signal flags need a block counter");
  // one CU per block (1024 threads): at most maxBlocks and kFusedMaxBlocks (waiting blocks hold their CUs); at
  // least one block, so the flags are waited for and raised even when this device has nothing to copy
  const int shareCap = a.sharedGpu ? kFusedMaxBlocks : (1 << 20);
  const int cap = maxBlocks > 0 ? std::min(maxBlocks, shareCap) : shareCap;
  const int blocks = std::max(1, std::min(cap, (p.nworkG + 3) / 4));
  hipLaunchKernelGGL(copy_plan_kernel_sync, dim3(blocks), dim3(1024), 0, stream, p.dsegs, p.dworkG, uint32_t(p.nworkG),
                     fs);
  HIP_CHECK(hipGetLastError());
}

__global__ void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

void spin_device(double seconds, hipStream_t stream) {
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, stream, uint64_t(seconds * 1e8));
  HIP_CHECK(hipGetLastError());
}

void signal_flags_device(const std::vector<uint64_t *> &flags, uint64_t value, hipStream_t stream) {
  if (flags.empty()) return;
  hipLaunchKernelGGL(signal_flags_kernel, dim3(1), dim3(64), 0, stream, to_list(flags), value);
  HIP_CHECK(hipGetLastError());
}

} // namespace stencil
