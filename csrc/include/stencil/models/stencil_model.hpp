#pragma once
// Iterated 7-point stencil applications on a DistributedDomain: the Jacobi3D and Astaroth-proxy "models".
// Reference apps: bin/jacobi3d.cu:89-385 (hot loop :265-346) and bin/astaroth_sim.cu:150-284.
//
// One step() (overlap mode) is fully stream-ordered, no host synchronisation:
//   compute[d]: interior(curr -> next)                               (overlaps the exchange)
//   comm[dev] : exchange(curr halos) after ready[d] of the previous step -> exterior slabs(curr -> next)
//   compute[d]: wait(exterior done) -> record ready
//   host      : swap curr/next pointers
// The reference instead host-synchronises every compute stream each iteration (jacobi3d.cu:331-337).
#include <map>
#include <memory>
#include <vector>

#include "stencil/domain/distributed_domain.hpp"
#include "stencil/kernels/stencil_ops.hpp"

namespace stencil {

struct StencilModelConfig {
  Dim3 size{512, 512, 512};
  StencilKind kind = StencilKind::Jacobi;
  int64_t radius = 1;          // face radius (Jacobi 1; Astaroth 3 in all 26 directions)
  bool allDirections = false;  // true: radius in all 26 directions (Astaroth), false: faces only (Jacobi)
  int quantities = 1;
  bool fp64 = false;
  MethodFlags methods = MethodFlags::All;
  PlacementStrategy placement = PlacementStrategy::NodeAware;
  // NodeAware cut costs (DistributedDomain::set_axis_cost): x faces count double, so weak-scaled cubes are cut
  // along y and z only (x faces are strided, and whole periodic rows feed the whole-row fused-pair kernels); z cuts
  // cost less than y cuts (contiguous faces, and at these shapes the sweeps are faster with long y than long z).
  // One MI355X, fused pairs, per-GPU shapes of the weak-scaling ladder (profiles/r2/r2_ragged_shapes2.log):
  // N=2 645x645x323 837 vs 645x323x645 790; N=4 813x407x407 664 (either order); N=8 1024x512x256 1000 vs
  // 1024x256x512 972 Gcells/s
  Dim3 axisCost{4, 3, 2};
  PartitionObjective partition = PartitionObjective::Interface; // NodeAware cut rule inside a node
  std::vector<int> gpus;       // empty = automatic
  bool overlap = true;
  // when every halo comes from this GPU (periodic self-wrap / co-resident sub-domains) the exchange is a local
  // HBM copy: overlapping it only adds exterior-slab work that competes for the same bandwidth, so run
  // exchange -> whole-region stencil instead. Off-GPU transports (xGMI/RCCL) keep the overlap.
  bool autoOverlap = true;
  // single stream + kernel-only exchange: capture the step (exchange + stencil) once per buffer parity into a
  // hipGraph and replay it (removes per-kernel launch gaps)
  bool useGraph = true;
  // in-process exchanges only (Kernel/PeerCopy): the stencil kernel stores its boundary outputs straight into the
  // receivers' halos (HaloForwarder), so a step is one kernel per sub-domain and no separate exchange runs.
  // Off by default: on one MI355X the scattered x-face stores cost the kernel more (~+23 us at 512^3) than the
  // separate copy-plan exchange does (~19 us), see BASELINE.md / bench_stencil.
  bool forward = false;
  // steps fused per sweep: 2 = temporal blocking (stencil7x2: one depth-2 exchange and one read+write of the field
  // per two steps, bitwise equal to two single steps); 1 = one exchange + one sweep per step. run(n) advances in
  // fused pairs (a trailing odd step is a single step); step() is always one step.
  int temporal = 1;
  // fused pairs: along axes where the decomposition has one sub-domain (periodic self-neighbour,
  // DistributedDomain::self_wrap_axes) the pair kernels read the periodic image in place of the halo, and the
  // pair's exchange skips those same-GPU copies (on one MI355X at 512^3 the depth-2 self-copy is ~34 us of a ~300 us
  // pair, mostly the strided x faces). Single steps do the same when they do not overlap or forward (the
  // exchange then leaves out every self copy). Off: every halo is copied.
  bool wrapSelf = true;
  int wrapAxesMask = 7;       // axes (1 = x, 2 = y, 4 = z) in-kernel wrap may use at most (experiments restrict it)
  // overlapped single steps with remote halos sweep get_local_interior(1) during the transfers (false: the classic
  // interior / exterior split of the reference, get_interior + get_exterior)
  bool localInterior = true;
  // overlapped fused pairs: where the slabs at the remote faces run at first (set_overlap_mode: 1 beside the
  // interior sweep on the comm stream, 2 after it on the compute stream)
  int overlapMode = 1;
  // halo-aligned x layout (DistributedDomain::set_x_halo_align): x halos share the interior's first / last 64-B
  // sector (x-face copies touch one sector per row end instead of two; every row spans one more sector)
  bool xHaloAlign = false;
  bool sharedHaloLine = false; // DistributedDomain::set_shared_halo_line
  int64_t interiorAlign = 128; // DistributedDomain::set_interior_align (128 B default, or 64)
  int rowPadLines = 0;          // DistributedDomain::set_row_pad_lines (measurement knob)
  TransportOptions transport; // DistributedDomain::set_transport_options
  bool selfTest = false;      // DistributedDomain::set_self_test (multi-rank: verified transport ladder)
  bool setBackend = false;
  Backend backend = Backend::Device;
  StencilTune tune;
  double astarothPeriod = 10.0;
};

class StencilModel {
public:
  explicit StencilModel(const StencilModelConfig &cfg, std::shared_ptr<comm::ProcGroup> pg = nullptr);
  ~StencilModel();

  void init();                  // realize + initial condition; blocks until done
  void step();                  // one iteration, asynchronous
  // `iters` iterations, asynchronous. In hipGraph mode whole blocks of kGraphSteps steps are replayed as one
  // graph (one launch instead of kGraphSteps: the GPU-side gap between graph launches is ~9 us on MI355X).
  void run(int iters);
  static constexpr int kGraphSteps = 16; // even: the block starts and ends on the same buffer parity
  // fused triples: 6 sweeps of 3 steps per block (an even number of sweeps keeps the buffer parity)
  static constexpr int kGraphStepsTriple = 18;
  int graph_steps() const { return triples_ ? kGraphStepsTriple : kGraphSteps; }
  int steps_per_sweep() const { return triples_ ? 3 : (pairs_ ? 2 : 1); }
  void synchronize();           // wait for all enqueued work (and check exchange errors)
  // instantiate run()'s hipGraph blocks for both buffer parities (no work is run); for each length n in `runs`, also one
  // graph per parity holding a whole run(n) (blocks, then the remainder triples / pairs / single steps), which run(n)
  // then replays as one launch: no graph-to-kernel gap before the remainder (~14 us on MI355X, profiles/r6/r6y)
  void prepare(const std::vector<int> &runs = {});
  DistributedDomain &domain() { return *dd_; }
  const StencilModelConfig &config() const { return cfg_; }
  int64_t cells() const { return cfg_.size.flatten(); } // global cells updated per step
  int64_t local_cells() const;
  hipStream_t compute_stream(size_t di) const;
  int64_t steps_done() const { return steps_; }
  const Spheres &spheres() const { return sph_; }
  bool overlapping() const { return overlap_; }
  // fused pairs with remote halos: overlapped (local interior during the transfers, slabs after) and whole-region
  // (exchange, then one sweep) share the wrap mask, so either can run; set_overlap() switches between them (after a
  // synchronize), e.g. to keep whichever the hardware runs faster
  bool can_toggle_overlap() const { return overlapToggle_; }
  void set_overlap(bool on);
  // overlapped pairs, where the slabs at the remote faces run: 1 = on the comm stream right behind the exchange,
  // beside the interior sweep (default); 2 = on the compute stream after the interior sweep (the sweep then shares the
  // GPU with the transport kernels only). 0 = whole-region pairs (set_overlap(false)).
  // 3 = pipelined pairs (can_pipeline()): whole-region sweeps, each publishing its boundary z planes while it runs;
  // the exchange the NEXT pair needs is gated on that publication (DistributedDomain::set_send_gate), so its pack,
  // xGMI stores and unpack run beside the rest of this sweep on the CUs it leaves free, and no sweep is split into
  // interior and slabs. Needs remote halos along z only, the whole-row kernel and fused co-located transports.
  void set_overlap_mode(int mode);
  int overlap_mode() const { return pipelined3_ ? 4 : (pipelined_ ? 3 : (overlap_ ? (slabsAfter_ ? 2 : 1) : 0)); }
  bool can_pipeline() const { return pipeOk_; }
  // 4 = pipelined triples: fused triples that publish their boundary z planes early, each depth-3 exchange gated on
  // them and running beside the rest of the sweep
  bool can_pipeline_triples() const { return pipeOk_ && triplesOk_; }
  // CUs the overlapped sweeps leave to the transport kernels (StencilTune::x2reserve); synchronizes first
  void set_comm_reserve(int cus);
  // the fused triples' lockstep schedule (StencilTune x3sphw / x3left / x3parts: launch geometry only, results are
  // bitwise the same); synchronizes and drops the recorded hipGraphs (run() / prepare() record them again)
  void set_triple_schedule(float sphw, int left, int parts);
  int comm_reserve() const { return cfg_.tune.x2reserve; }
  bool local_interior_steps() const { return localSteps_; } // overlapped single steps on get_local_interior
  bool forwarding() const { return forward_; }
  bool temporal_blocking() const { return pairs_; }
  // three steps per sweep (stencil7x3): temporal >= 3, device sub-domains of 512-cell fp32 rows wrapped in-kernel or of
  // 512-cell fp32 / 256-cell fp64 columns with x halos
  bool temporal_triples() const { return triples_; }
  int wrap_axes() const { return pairTune_.wrap; } // axes the fused pairs wrap in-kernel (mask 1=x 2=y 4=z)
  int step_wrap_axes() const { return stepTune_.wrap; } // same for single steps (stencil7_apply)

private:
  StencilModelConfig cfg_;
  std::unique_ptr<DistributedDomain> dd_;
  std::vector<Stream> compute_;
  std::vector<Event> exteriorDone_;
  std::vector<Rect3> interiors_;     // single steps (get_interior)
  std::vector<Rect3> pairInteriors_; // overlapped fused pairs (get_local_interior, see init)
  std::vector<std::vector<Rect3>> exteriors_;
  Spheres sph_;
  bool overlap_ = true;
  bool graphs_ = false;
  bool forward_ = false;
  bool pairs_ = false; // temporal blocking active
  // fused triples active: three steps per sweep (run() then uses pairs / single steps only for remainders)
  bool triples_ = false;
  bool triplesOk_ = false; // triples possible for whole-region sweeps (triples_ = triplesOk_ && !overlap_)
  bool confinedSelf_ = false; // overlapped single steps with only same-GPU halos: translate on x2reserve CUs
  bool overlapToggle_ = false;
  bool slabsAfter_ = false; // overlap mode 2 (see set_overlap_mode)
  bool pipeOk_ = false;      // overlap mode 3 possible (see init)
  bool pipelined_ = false;   // overlap mode 3
  bool pipelined3_ = false;  // overlap mode 4
  int pubDepth_ = 2;         // boundary z planes a sweep publishes at each face (the exchange's z depth)
  bool lastPublished_ = false; // the last enqueued sweep published its boundary planes into pubCounter_
  uint64_t *pubCounter_ = nullptr; // device word (uncached), cumulative boundary cells published
  uint64_t pubTotal_ = 0;          // its value once every published sweep so far is done
  uint64_t pubCells_ = 0;          // boundary cells one sweep publishes (all quantities)
  StencilTune pairTune_; // cfg_.tune + the in-kernel wrap axes of the fused pairs
  StencilTune stepTune_; // cfg_.tune + the in-kernel wrap axes of single steps
  bool localSteps_ = false;                      // overlapped single steps on the local interior (see init)
  std::vector<Rect3> stepInteriors_;             // get_local_interior(1)
  std::vector<std::vector<Rect3>> stepExteriors_; // the slabs at remote faces
  std::vector<std::vector<std::unique_ptr<HaloForwarder>>> fwd_; // [domain][quantity]
  std::vector<Event> stepDone_;                                    // forwarding with several sub-domains
  hipGraphExec_t graphExec_[2] = {nullptr, nullptr};
  hipGraphExec_t graphBlock_[2] = {nullptr, nullptr}; // kGraphSteps steps starting at parity p
  void enqueue_step(int k = 1); // k = 1: one step; k = 2: a fused pair (temporal blocking)
  void capture_block();         // graphBlock_[current parity] (no work is run)
  struct RunGraph {
    hipGraphExec_t exec = nullptr;
    int sweeps = 0; // buffer swaps of the recorded run
  };
  std::map<std::pair<int, int>, RunGraph> runGraph_; // (steps, starting parity) -> a whole run(steps)
  void capture_run(int n);                           // runGraph_[{n, current parity}] (no work is run)
  void drop_graphs();
  bool pair_ok() const { return pairs_; }
  int64_t steps_ = 0;
};

} // namespace stencil
