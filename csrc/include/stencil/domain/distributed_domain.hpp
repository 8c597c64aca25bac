#pragma once
// DistributedDomain: the public API of the runtime.
// Parity: reference include/stencil/stencil.hpp:29-354 + src/stencil.cu:1-939
//   MethodFlags / set_methods / set_placement / set_gpus / set_radius / add_data<T> / realize / exchange / swap /
//   get_interior / get_exterior / get_compute_region / exchange_bytes_for_method / write_paraview / setup timers.
//
// MI355X-first transport ladder (same priority order as reference src/stencil.cu:163-194):
//   Kernel    same process, same GPU      -> one fused descriptor copy kernel per device (periodic self-wrap and
//                                            co-resident sub-domains), no intermediate buffer
//   PeerCopy  same process, peer GPU      -> the same kernel storing directly into the peer's halo over xGMI
//   Colocated other process, same node    -> HIP IPC: the pack kernel stores into the receiver's (uncached, double
//                                            buffered) inbox over xGMI, device flags signal arrival and credits
//                                            (no host round trip, fixes the reference's missing ack)
//   Rccl      any other rank              -> RCCL ncclSend/ncclRecv grouped per device on a high-priority stream
//   Staged    fallback / CPU backend      -> pack, D2H, TCP (native process group), H2D, unpack
// Exchange is stream-ordered: exchange_async() enqueues everything on per-device comm streams after the events
// given to record_ready(); wait_exchange() makes a compute stream wait for the halos. exchange() keeps the
// reference's blocking semantics.
#include <array>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "stencil/comm/proc_group.hpp"
#include "stencil/core/boundary.hpp"
#include "stencil/domain/local_domain.hpp"
#include "stencil/domain/packer.hpp"
#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/rt/stream.hpp"
#include "stencil/topo/placement.hpp"

namespace stencil {

constexpr int kTransportLogWords = 8; // set_transport_log: stamps per exchange

enum class MethodFlags : int {
  None = 0,
  Staged = 1,    // reference CudaMpi
  Rccl = 2,      // reference CudaAwareMpi (GPU-aware remote path)
  Colocated = 4, // reference CudaMpiColocated
  PeerCopy = 8,  // reference CudaMemcpyPeer
  Kernel = 16,   // reference CudaKernel
  All = 31,
};
inline MethodFlags operator|(MethodFlags a, MethodFlags b) { return MethodFlags(int(a) | int(b)); }
inline MethodFlags &operator|=(MethodFlags &a, MethodFlags b) { return a = a | b; }
inline MethodFlags operator&(MethodFlags a, MethodFlags b) { return MethodFlags(int(a) & int(b)); }
inline bool operator&&(MethodFlags a, MethodFlags b) { return (int(a) & int(b)) != 0; }
inline bool any(MethodFlags a) { return a != MethodFlags::None; }
std::string to_string(MethodFlags m);


// What the planner knows about one (sender, receiver) sub-domain pair when it picks a transport.
struct PairInfo {
  bool device = true;     // device backend (false: host backend, only Kernel/PeerCopy-as-host-copy and Staged)
  bool sameRank = false;  // both sub-domains in this process
  bool sameDevice = false; // same device ordinal (meaningful within one rank)
  bool peer = false;      // same rank, P2P access between the two devices (gpu_topo::peer)
  bool sameHost = false;  // co-located ranks
  bool canAccess = false; // co-located ranks whose devices can map each other's memory (HIP IPC over xGMI)
  bool sharedGpu = false; // different ranks, and an endpoint's GPU is driven by two ranks (RCCL refuses that GPU)
};
// First enabled method whose predicate holds, in the reference's priority order (src/stencil.cu:163-194):
// Kernel > PeerCopy > Colocated > Rccl > Staged. A pair touching a GPU shared by two ranks skips Rccl and takes the
// host-staged path even when Staged is not among `flags` (it is the fallback RCCL itself would need). None = no
// transport (the planner treats that as fatal).
MethodFlags select_method(MethodFlags flags, const PairInfo &p);

// Typed transport configuration (set before realize; the copy path and the completion method can also be switched
// between exchanges with set_colo_copy / set_completion). Replaces the round-1/2 environment knobs.
struct TransportOptions {
  // Memory of a Colocated receiver's data slots (its arrival/credit flag words are always uncached):
  //   Uncached  hipDeviceMallocUncached: every access bypasses the caches (coherent by construction; the unpack
  //             reads the slots from HBM without L2 reuse)
  //   Fine      hipDeviceMallocFinegrained: coherent at system scope, cached with the fine-grained MTYPE
  //   Coarse    hipMalloc: L2-cached; relies on the kernel-boundary cache invalidate of the unpack's dispatch, so
  //             its arrival wait always runs as a separate kernel before the unpack (fuseFlags applies to the
  //             send side only)
  enum class Inbox : int { Uncached = 0, Fine = 1, Coarse = 2 };
  Inbox inbox = Inbox::Uncached;
  // How a packed message reaches another GPU's memory (Colocated: the peer's IPC-mapped inbox; PeerCopy: the peer
  // GPU's halo or receive buffer):
  //   Store   the pack / translate kernel stores straight into the peer memory (CUs issue the xGMI writes)
  //   Engine  pack into a local staging buffer, then hipMemcpyAsync(..., hipMemcpyDeviceToDeviceNoCU) / a peer
  //           copy moves it on a DMA (SDMA) engine and the receiver unpacks (reference tx_cuda.cuh:141-162,
  //           :270-283 use cudaMemcpyPeerAsync). Leaves the CUs to an overlapped interior sweep.
  enum class Copy : int { Store = 0, Engine = 1 };
  Copy coloCopy = Copy::Store;
  Copy peerCopy = Copy::Store;
  // Arrival / credit signalling of the Colocated transport:
  //   Kernel    a one-wave kernel polls the flag word (bounded: stops after waitTimeout and reports) and a one-wave
  //             kernel releases + stores it
  //   StreamOp  hipStreamWaitValue64 / hipStreamWriteValue64 (the command processor waits; no CU is held, but the
  //             wait itself is unbounded: sync_exchange's host watchdog reports a stall)
  //   IpcEvent  the reference's design (tx_cuda.cuh:231-240, :351, :366-372): the sender records an interprocess
  //             event (hipIpcGetEventHandle, opened once by the receiver) after its stores / engine copy and sends a
  //             host Notify(epoch); the receiver, on the notify, orders its unpack with hipStreamWaitEvent on that
  //             event and answers Ack(epoch). Arrival therefore costs a host message per channel per exchange; the
  //             double-buffered inbox keeps its device credit flags (the reference's missing ack),
  //             and a sender records epoch e only after the receiver acknowledged e-2 (an event may only be
  //             re-recorded once the wait that needs the older record has been enqueued). Requires realize() with
  //             this completion (the events are created there); not capturable into a hipGraph.
  enum class Completion : int { Kernel = 0, StreamOp = 1, IpcEvent = 2 };
  Completion completion = Completion::Kernel;
  // Kernel completion: fold the flag waits / signals into the pack and unpack kernels (one launch per side instead
  // of three; copy_plan_device_sync). Engine copies keep a separate credit wait and arrival signal around the copies.
  bool fuseFlags = true;
  // seconds before a device-side spin, a host wait on a peer, or the RCCL watchdog gives up (<= 0: the
  // STENCIL_WAIT_TIMEOUT environment variable, else 60)
  double waitTimeout = 0;
  // measurement hook: get_local_interior treats the faces of these axes (mask 1 = x, 2 = y, 4 = z) as remote, so
  // one GPU runs the overlapped split of a multi-GPU decomposition (the exchange itself is unchanged)
  int fakeRemoteAxes = 0;
  // map every co-located rank's IPC block before planning (up to 3 attempts); Colocated is dropped on all ranks if
  // any mapping fails. failIpcProbe forces that failure (rehearses the fallback).
  bool ipcProbe = true;
  bool failIpcProbe = false;
  // test hook: RCCL communicator creation reports failure on this rank (rehearses the RCCL -> staged fallback)
  bool failRcclInit = false;
  // test hook: this rank never enters RCCL communicator creation and reports a timeout after waitTimeout (a rank
  // stuck before ncclCommInitRank); its peers' non-blocking creation runs into the same deadline and aborts, and the
  // failure is agreed on like any other (-> host-staged)
  int stallRcclInitRank = -1;
  // test hook: PeerCopy engine pipes between sub-domains on the SAME device also go through hipMemcpyPeerAsync
  // (src device == dst device is legal), so the cross-GPU peer-copy call runs on a one-GPU box
  bool peerApiSameDevice = false;
  // test hook: the first transport self-test probe of this rank throws after realize (the other ranks then time out
  // on the probe's forked group; the ladder must go on in step on every rank)
  int failProbeRank = -1;
  // sleep a random 0..jitterUs microseconds between transport phases of every exchange (race canary; reference's
  // unused rand_sleep(), packer.cuh:17-20)
  int jitterUs = 0;
  // blocking exchange(): the last op of every comm stream stores the exchange's epoch into a host-mapped word and
  // the host spins on it (bounded) before the stream synchronize, which then returns at once; false (default):
  // block in hipStreamSynchronize right away. Measured on one MI355X (512^3, faces 2, scripts/mi355x/xchg_latency.py,
  // profiles/r3/xchg_latency_*.json): 45.2 us with the spin vs 37.8 us without -- the extra one-wave signal kernel
  // costs more than the synchronize's wake-up
  bool spinWait = false;
  // blocking exchange() without record_ready(): the producers of the fields are taken to be on the null stream or
  // blocking streams (torch's default stream, synchronous copies) and the comm streams wait for an event recorded on
  // the null stream; false (default): hipDeviceSynchronize, which also covers non-blocking producer streams and
  // measured faster on an idle GPU (37.8 vs 44.2 us per blocking exchange, same probe)
  bool nullStreamProducers = false;
  // device backend: when every GPU of this process sits on one NUMA node, realize() binds the calling thread to that
  // node's CPUs and allocates the host-staged (pinned) buffers there
  bool numaAffinity = true;
  // same-GPU x faces (translates) copied as whole interior-alignment units -- 128-B L2 lines with the default
  // layout, 64-B sectors with interior_align 64 -- (8 / 4 lanes per row, the extra cells land in the receiver's row
  // padding) instead of w-cell pieces of one line per lane (build_translate_segs_q). With 64-B sectors it measured
  // no gain (stream-ordered 26.2 vs 24.9 us for faces 2, 26.8 vs 27.8 us with depth-1 edges)
  bool xFaceSectors = false;
  // ... and switched on automatically for a GPU whose same-GPU x faces cover at least this many bytes of lines per
  // exchange (rows x 1.5 lines of 128 B per face: the read line plus the halo line two rows share; 0 = never). Below
  // the last-level cache's size the repeated exchange stays cache-resident and partial-line halo writes cost
  // nothing (config 3, 512^2 rows x 1 quantity: 353 -> 303 GB/s with whole lines); beyond it they go to HBM as
  // partial-line writes, and whole lines win (config 5a, 1024^2 rows x 4 fp64: 0.69-0.74 -> 0.55-0.57 ms; config 4,
  // 512^2 rows x 8: 68.9 -> 74.1 Gcells/s x 8; profiles/r4/aq/). Crossover (bench_exchange 512^3 radius-2 faces,
  // profiles/r4/au/): 1 quantity = 96 MiB of lines 337 vs 293 GB/s (stay), 2 = 192 MiB 240 vs 338 (switch)
  int64_t xFaceLinesAutoBytes = int64_t(128) << 20;
};
const char *to_string(TransportOptions::Inbox v);
const char *to_string(TransportOptions::Copy v);
const char *to_string(TransportOptions::Completion v);

struct ExchangePlanEntry {
  MethodFlags method;
  Dim3 srcIdx, dstIdx;
  int srcRank, dstRank;
  int srcDev, dstDev;
  Dim3 dir;
  int64_t bytes;
};

// bytes of the aggregated message for sending `dirs` from `dom` (reference wire layout: messages sorted by dir,
// each quantity aligned to its element size; reference packer.cuh:136-160 — pinned by the 264-byte test)
int64_t packed_message_bytes(const LocalDomain &dom, std::vector<Dim3> dirs);

class DistributedDomain {
public:
  DistributedDomain(int64_t x, int64_t y, int64_t z, std::shared_ptr<comm::ProcGroup> pg = nullptr);
  ~DistributedDomain();
  DistributedDomain(const DistributedDomain &) = delete;
  DistributedDomain &operator=(const DistributedDomain &) = delete;

  // ---- configuration (before realize) ----
  void set_radius(int64_t r) { radius_ = Radius::constant(r); }
  void set_radius(const Radius &r) { radius_ = r; }
  const Radius &radius() const { return radius_; }
  // global boundary condition (default periodic everywhere). No message crosses a non-periodic face.
  void set_boundary(const Boundary &b) { boundary_ = b; }
  const Boundary &boundary() const { return boundary_; }
  template <typename T> DataHandle<T> add_data(const std::string &name = "") {
    return DataHandle<T>(add_data(int64_t(sizeof(T)), name, dtype_of<T>()), name);
  }
  int64_t add_data(int64_t elemSize, const std::string &name, DType dtype);
  void set_methods(MethodFlags f) { flags_ = f; }
  MethodFlags methods() const { return flags_; }
  bool any_methods(MethodFlags m) const { return (m && flags_); }
  void set_placement(PlacementStrategy s) { strategy_ = s; }
  // NodeAware partition: relative cost per interface cell of cuts normal to x/y/z (NodePartition; default 1,1,1)
  void set_axis_cost(const Dim3 &c) { axisCost_ = c; }
  const Dim3 &axis_cost() const { return axisCost_; }
  // NodeAware cut rule inside a node (PartitionObjective; default Interface = the reference's greedy rule)
  void set_partition_objective(PartitionObjective o) { objective_ = o; }
  PartitionObjective partition_objective() const { return objective_; }
  void set_gpus(const std::vector<int> &gpus) { gpus_ = gpus; }
  const std::vector<int> &gpus() const { return gpus_; }
  void set_backend(Backend b) { backend_ = b; backendSet_ = true; }
  Backend backend() const { return backend_; }
  // write plan_<rank>.txt during realize (reference src/stencil.cu:259-353); default on, off with STENCIL_PLAN_FILE=0
  void set_plan_file(const std::string &prefix) { planPrefix_ = prefix; }
  void set_padding(bool p) { pad_ = p; }
  // halo-aligned x layout of every local domain (LocalDomain::set_x_halo_align)
  void set_x_halo_align(bool on) { xHaloAlign_ = on; }
  bool x_halo_align() const { return xHaloAlign_; }
  // shared halo lines of every local domain (LocalDomain::set_shared_halo_line)
  void set_shared_halo_line(bool on) { sharedHaloLine_ = on; }
  bool shared_halo_line() const { return sharedHaloLine_; }
  // LocalDomain::set_interior_align of every local domain (128 B default, or 64)
  void set_interior_align(int64_t bytes) { interiorAlign_ = bytes; }
  int64_t interior_align() const { return interiorAlign_; }
  void set_row_pad_lines(int n) { rowPadLines_ = n; } // LocalDomain::set_row_pad_lines of every local domain
  // opt-in self-test ladder run by realize() before planning (multi-rank runs): exchange a coordinate-encoded field
  // on a small probe domain built like this one and check every halo cell on every rank; on any wrong cell or
  // error drop Colocated, then Rccl (-> host-staged), i.e. the reference's always-terminating ladder
  // (src/stencil.cu:163-194). methods() afterwards is the verified set; self_test_report() says what happened.
  void set_self_test(bool on) { selfTest_ = on; }
  const std::string &self_test_report() const { return selfTestReport_; }
  // RCCL communicator creation in realize(): "" (no RCCL channel planned), "ok", or why it failed (the channels then
  // run host-staged)
  const std::string &rccl_status() const { return rcclStatus_; }
  // one probe: wrong halo cells summed over all ranks (0 = the transports of `m` deliver every halo correctly)
  int64_t probe_transports(MethodFlags m);
  // typed transport configuration (before realize)
  void set_transport_options(const TransportOptions &o);
  const TransportOptions &transport_options() const { return topt_; }
  // switch how Colocated messages reach the peer inbox between exchanges (both paths are prepared by realize);
  // waits for the exchanges in flight first
  void set_colo_copy(TransportOptions::Copy c);
  // change the run-time fields (colo copy, completion, spin wait, producer ordering, jitter, timeout) of a realized
  // domain; the allocation-time fields (inbox, peer copy, probes) must stay as realized
  void set_transport_options_live(const TransportOptions &o);
  void set_completion(TransportOptions::Completion c);

  void realize();
  bool realized() const { return realized_; }

  // ---- queries ----
  const Dim3 &size() const { return size_; }
  int rank() const { return pg_->rank(); }
  int world_size() const { return pg_->size(); }
  comm::ProcGroup &group() { return *pg_; }
  std::vector<LocalDomain> &domains() { return domains_; }
  const std::vector<LocalDomain> &domains() const { return domains_; }
  const Dim3 &get_origin(int64_t i) const { return domains_.at(size_t(i)).origin(); }
  Rect3 get_compute_region() const { return Rect3(Dim3(0, 0, 0), size_); }
  std::vector<Rect3> get_interior() const;
  std::vector<std::vector<Rect3>> get_exterior() const;
  // MI355X extension: the part of each local domain's compute region that a stencil reaching `reach` cells along
  // an axis can update from halos filled by the same-device translate (Kernel method) alone, i.e. it is shrunk
  // only at the faces whose halo arrives over IPC / RCCL / staged / peer transports. Safe to compute once
  // wait_translated() has been passed, while those transports are still in flight; the rest (thin slabs at the
  // remote faces) after wait_exchange(). Equals get_compute_region() for a purely same-GPU exchange.
  std::vector<Rect3> get_local_interior(int reach) const;
  const Placement &placement() const { return *placement_; }
  Dim3 subdomain_idx(int64_t di) const { return placement_->get_idx(rank(), int(di)); }
  uint64_t exchange_bytes_for_method(MethodFlags m) const; // summed over all ranks, per exchange
  const std::vector<ExchangePlanEntry> &plan() const { return plan_; }
  std::string plan_summary() const;
  // Direct-store targets of local domain di: every planned message of di whose receiver this process can write
  // (Kernel: same GPU, PeerCopy: P2P-mapped peer GPU), with the raw-coordinate offset into the receiver.
  // Used by the halo-forwarding compute kernels (stencil_ops.hpp HaloForwarder).
  std::vector<ForwardTarget> forward_targets(size_t di) const;
  // true when every message of every rank is Kernel or PeerCopy (a pure in-process exchange)
  bool all_direct() const {
    return exchange_bytes_for_method(MethodFlags::Kernel | MethodFlags::PeerCopy) ==
           exchange_bytes_for_method(MethodFlags::All);
  }

  // ---- exchange ----
  void exchange();       // blocking: returns when every halo of every local domain is valid
  // enqueue on the comm streams; only the staged (host) path blocks the caller. With a single local device a
  // caller stream may be given: the exchange is then enqueued on it. Caller-stream and comm-stream exchanges are
  // ordered against each other by events (the last one of the other kind is waited for), and sync_exchange()
  // also waits for the last caller-stream exchange (except exchanges captured into a hipGraph: the caller orders
  // those by its stream).
  // skipAxes (prepared by prepare_skip_wrapped): leave out the same-process copies of every direction crossing
  // those axes; their halos are then stale and only kernels that wrap in-kernel may run on the result
  void exchange_async(hipStream_t stream = nullptr, int skipAxes = 0);
  // axes (1 = x, 2 = y, 4 = z) along which the decomposition has one sub-domain and the grid is periodic: every
  // sub-domain is its own neighbour there, so a kernel can read the periodic image instead of a copied halo
  int self_wrap_axes() const;
  // build the same-process copy plan used by exchange_async(.., axes) (a subset of self_wrap_axes())
  void prepare_skip_wrapped(int axes);
  // make the next exchange wait for the work currently enqueued on `s` (which touches domain di)
  void record_ready(size_t di, hipStream_t s);
  // make `s` wait until the halos of domain di from the last exchange are written
  void wait_exchange(size_t di, hipStream_t s);
  // make `s` wait until the same-device (Kernel) halo copies of the last exchange_async() are written (the halos
  // get_local_interior() relies on); needs the comm streams, i.e. exchange_async() without a caller stream
  void wait_translated(size_t di, hipStream_t s);
  // block the host until the last exchange is complete (checks device-side timeouts)
  void sync_exchange();
  // block the host until `streams` (e.g. compute streams that joined the exchange) and the last exchange are
  // complete, polling instead of blocking: a transport error (RCCL asynchronous error, device-side timeout word) or
  // no progress within the wait timeout fails with the plan on stderr instead of hanging in hipStreamSynchronize
  void sync_streams(const std::vector<hipStream_t> &streams);
  // non-empty after a fatal exchange error (the domain refuses further exchanges)
  const std::string &poisoned() const { return poisoned_; }
  hipStream_t comm_stream(size_t di) const;
  // confine the pack / unpack kernels of the off-GPU transports (not the same-device translate) to at most n
  // 1024-thread blocks, i.e. n CUs (0 = one block per work item, the whole GPU). Used while an overlapped compute
  // grid holds every other CU: measured on one MI355X (bench_stencil --only ovl) a 4 MiB pack beside the interior
  // sweep costs the pair ~80 us unconfined (its blocks land on CUs the sweep's blocks then wait for) and ~25 us
  // confined to 8 CUs beside a sweep that leaves 8 free.
  void set_comm_max_blocks(int n) { commBlocks_ = n; }
  // the same confinement for the same-device translate (the Kernel method's copy plan): an overlapped single step whose
  // every halo is a same-GPU copy (one GPU, config 4) runs the translate on n CUs beside an interior sweep that leaves
  // n CUs free (0 = the whole GPU, the default)
  void set_translate_max_blocks(int n) { translateBlocks_ = n; }
  // Producer gate for the next exchange_async on the comm stream (pipelined pairs): instead of waiting for the
  // producer's whole kernel (record_ready), the fused co-located pack kernel polls *counter >= target, a word the
  // still-running stencil sweep raises once the boundary planes the exchange reads are written
  // (StencilTune::publish). Valid only where gated_send_supported(skipAxes); consumed by that one exchange.
  void set_send_gate(uint64_t *counter, uint64_t target);
  // every halo of this process's one device leaves through fused pack-kernel stores of the Colocated transport
  // (no same-GPU translate for these skip axes, no DMA-engine pipes, no RCCL / staged channels): the only kind of
  // exchange a producer gate can start early
  bool gated_send_supported(int skipAxes) const;
  void swap();

  // ---- transport log (wait vs copy of the fused co-located kernels) ----
  // keep the last `exchanges` exchanges' device timestamps (s_memrealtime, 100-MHz constant clock) of every fused
  // Colocated pack / unpack kernel: per exchange {send start, send after credit wait, send after copies, send
  // signal, recv start, recv after arrival wait, recv after copies, recv signal}; 0 where no such kernel ran.
  // 0 turns the log off. transport_log(dev) returns the logged exchanges of local device slot `dev`, oldest first.
  void set_transport_log(int exchanges);
  std::vector<std::array<uint64_t, kTransportLogWords>> transport_log(size_t dev = 0);

  // ---- output ----
  void write_paraview(const std::string &prefix, bool zeroNaNs = false);
  // binary checkpoint of every local sub-domain's interior (curr buffers): `prefix_<rank>_<di>.ckpt`, one file per
  // sub-domain with a header (magic, global size, sub-domain index/origin/size, quantity sizes). load_checkpoint
  // validates the header against this domain's decomposition and restores the interiors (halos are re-exchanged).
  // Superset of the reference, which only writes ParaView dumps.
  void save_checkpoint(const std::string &prefix) const;
  void load_checkpoint(const std::string &prefix);

  // ---- setup / exchange timers (max over ranks, seconds), reference stencil.hpp:106-131 ----
  double timeMpiTopo_ = 0, timeNodeGpus_ = 0, timePeerEn_ = 0, timePlacement_ = 0, timePlan_ = 0, timeRealize_ = 0,
         timeCreate_ = 0;
  double timeExchange_ = 0, timeSwap_ = 0;
  bool exchangeStats_ = false; // STENCIL_EXCHANGE_STATS=1: barrier + time every exchange/swap

  struct Impl;

private:
  Dim3 size_;
  std::shared_ptr<comm::ProcGroup> pg_;
  Radius radius_;
  Boundary boundary_;
  std::vector<int> gpus_;
  std::vector<int64_t> elemSize_;
  std::vector<std::string> names_;
  std::vector<DType> dtypes_;
  MethodFlags flags_ = MethodFlags::All;
  PlacementStrategy strategy_ = PlacementStrategy::NodeAware;
  Dim3 axisCost_{1, 1, 1};
  PartitionObjective objective_ = PartitionObjective::Interface;
  int commBlocks_ = 0;
  int translateBlocks_ = 0;
  Backend backend_ = Backend::Device;
  bool backendSet_ = false;
  bool realized_ = false;
  bool pad_ = true;
  bool xHaloAlign_ = false;
  bool sharedHaloLine_ = false;
  int64_t interiorAlign_ = 128;
  int rowPadLines_ = 0;
  TransportOptions topt_;
  bool selfTest_ = false;
  std::string selfTestReport_;
  std::string rcclStatus_;
  int probeFailures_ = 0; // TransportOptions::failProbeRank bookkeeping
  // set when an exchange failed fatally (device wait timed out, RCCL error/timeout): every later exchange refuses to
  // run instead of handing a torn-down transport to the GPU
  std::string poisoned_;
  void poison(const std::string &why);
  void init_rccl(const std::function<bool(int, int)> &sharedDev); // realize(): communicator or staged fallback
  // Completion::IpcEvent: consume the last two exchanges' Acks so a later domain on the same group starts clean.
  // Polls at most timeout_s seconds and returns false if they did not all arrive; timeout_s <= 0 uses the group's
  // blocking receive (bounded by its own wait timeout).
  bool drain_ipc_acks(double timeout_s);
  bool x_face_lines(const LocalDomain &s, const LocalDomain &d) const; // translate s -> d copies x faces as lines
  std::string planPrefix_ = "plan";
  int numaNode_ = -1; // NUMA node the calling thread was bound to in realize() (-1: none)

public:
  int numa_node() const { return numaNode_; }

private:
  std::unique_ptr<Placement> placement_;
  std::vector<LocalDomain> domains_;
  std::vector<ExchangePlanEntry> plan_;
  std::vector<std::array<uint8_t, 27>> remoteHalo_; // per local domain, per halo side: filled by a non-Kernel method
  std::array<uint64_t, 5> bytesPerMethod_{}; // indexed by log2(method)
  std::unique_ptr<Impl> impl_;
};

} // namespace stencil
