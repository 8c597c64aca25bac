#include "stencil/models/stencil_model.hpp"

#include <algorithm>
#include <cstdlib>

#include "stencil/rt/hip_check.hpp"
#include "stencil/rt/trace.hpp"

namespace stencil {

StencilModel::StencilModel(const StencilModelConfig &cfg, std::shared_ptr<comm::ProcGroup> pg) : cfg_(cfg) {
  dd_.reset(new DistributedDomain(cfg.size.x, cfg.size.y, cfg.size.z, pg));
  pubDepth_ = cfg.temporal >= 3 ? 3 : 2;
  Radius r = Radius::constant(0);
  if (cfg.allDirections) {
    r = Radius::constant(cfg.radius);
  } else {
    r.set_face(cfg.radius);
  }
  if (cfg.temporal >= 2) {
    // S o S of a 7-point stencil reaches 2 cells along an axis and 1 cell diagonally (edges), never corners;
    // S o S o S 3 along an axis, (1, 2) / (2, 1) on edges and (1, 1, 1) in corners (an edge / corner halo spans the
    // face depths of its axes, LocalDomain::halo_extent, so a nonzero radius is enough). Corners matter only where x
    // is read from halos (the triples' XH form); wherever x wraps in-kernel their messages are skipped with the other
    // self copies or carry a few hundred bytes
    const int64_t face = cfg.temporal >= 3 ? 3 : 2;
    for (int i = 0; i < 27; ++i) {
      const Dim3 d = dir_from_index(i);
      const int nz = (d.x != 0) + (d.y != 0) + (d.z != 0);
      if (nz == 1) r.dir(d) = std::max<int64_t>(r.dir(d), face);
      if (nz == 2 || (nz == 3 && cfg.temporal >= 3)) r.dir(d) = std::max<int64_t>(r.dir(d), 1);
    }
  }
  dd_->set_radius(r);
  dd_->set_methods(cfg.methods);
  dd_->set_placement(cfg.placement);
  dd_->set_axis_cost(cfg.axisCost);
  dd_->set_partition_objective(cfg.partition);
  if (!cfg.gpus.empty()) dd_->set_gpus(cfg.gpus);
  if (cfg.setBackend) dd_->set_backend(cfg.backend);
  dd_->set_transport_options(cfg.transport);
  dd_->set_x_halo_align(cfg.xHaloAlign);
  dd_->set_shared_halo_line(cfg.sharedHaloLine);
  dd_->set_interior_align(cfg.interiorAlign);
  dd_->set_row_pad_lines(cfg.rowPadLines);
  dd_->set_self_test(cfg.selfTest);
  for (int q = 0; q < cfg.quantities; ++q) {
    const std::string name = cfg.kind == StencilKind::Jacobi && cfg.quantities == 1 ? "d" : "d" + std::to_string(q);
    if (cfg.fp64)
      dd_->add_data<double>(name);
    else
      dd_->add_data<float>(name);
  }
}

StencilModel::~StencilModel() {
  try {
    for (auto &s : compute_) s.sync();
  } catch (...) {
  }
  for (auto &g : graphExec_)
    if (g) (void)hipGraphExecDestroy(g);
  for (auto &g : graphBlock_)
    if (g) (void)hipGraphExecDestroy(g);
  for (auto &kv : runGraph_)
    if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
  if (pubCounter_) (void)hipFree(pubCounter_);
}

int64_t StencilModel::local_cells() const {
  int64_t n = 0;
  for (const auto &d : dd_->domains()) n += d.size().flatten();
  return n;
}

hipStream_t StencilModel::compute_stream(size_t di) const { return compute_.empty() ? nullptr : compute_.at(di).get(); }

void StencilModel::init() {
  TraceRange tr("StencilModel::init");
  cfg_.tune.wrap = 0; // in-kernel wrap axes are the model's decision (pairTune_ / stepTune_ below)
  dd_->realize();
  const Rect3 cReg = dd_->get_compute_region();
  sph_ = cfg_.kind == StencilKind::Jacobi ? Spheres::jacobi(cReg) : Spheres();
  overlap_ = cfg_.overlap;
  if (cfg_.overlap && cfg_.autoOverlap && cfg_.transport.fakeRemoteAxes == 0 &&
      dd_->exchange_bytes_for_method(MethodFlags::Kernel) == dd_->exchange_bytes_for_method(MethodFlags::All))
    overlap_ = false;
  auto &doms0 = dd_->domains();
  forward_ = cfg_.forward && dd_->world_size() == 1 &&
             dd_->all_direct() && !doms0.empty();
  for (const auto &d : doms0)
    for (int64_t q = 0; q < d.num_data() && forward_; ++q) forward_ = HaloForwarder::supported(d, q);
  if (forward_) overlap_ = false; // the halos travel inside the stencil kernel
  pairs_ = cfg_.temporal >= 2 && !forward_ && !doms0.empty();
  // a fused pair computes the intermediate step on the halo ring too, with the sphere test at the halo cell's
  // unwrapped coordinate: across the global periodic boundary that is -1 / L instead of L-1 / 0. The two agree
  // unless a sphere reaches the first or last plane of an axis (only on grids much thinner in y/z than x/10):
  // then run single steps.
  if (pairs_ && sph_.enabled) {
    const Dim3 L = cfg_.size;
    for (const Dim3 &c : {sph_.hot, sph_.cold}) {
      const int64_t cc[3] = {c.x, c.y, c.z}, ll[3] = {L.x, L.y, L.z};
      for (int a = 0; a < 3; ++a)
        if (cc[a] - sph_.radius < 1 || cc[a] + sph_.radius > ll[a] - 2) pairs_ = false;
    }
    if (!pairs_) LOG_WARN("Jacobi spheres reach a periodic face of " << L << ": temporal blocking off");
  }
  for (const auto &d : doms0)
    for (int64_t q = 0; q < d.num_data() && pairs_; ++q) pairs_ = stencil7x2_supported(d, q);
  // Fused pairs overlap against the REMOTE part of the exchange only: the same-device translate (periodic
  // self-wrap, co-resident sub-domains) runs first, then S o S of the local interior (the compute region shrunk
  // only at faces whose halo arrives over IPC / RCCL / staged transports, get_local_interior) while those
  // transports are in flight, then the thin slabs at the remote faces. Measured on one MI355X (512^3,
  // bench_stencil --only ext): with all six faces shrunk the split costs ~90 us of the ~100 us it could hide
  // (interior 308 us + x/y/z slabs 64 us concurrently = 387 us vs 296 us whole), dominated by the x slabs (lanes
  // along strided rows); y/z slabs are row-contiguous. So `auto` overlaps pairs exactly when some halo is remote
  // and no x face is: 2 GPUs (z split) and 4 GPUs (y, z split) of the weak-scaling ladder, not 2x2x2.
  if (pairs_) {
    const auto li = dd_->get_local_interior(2);
    bool remote = false, xcut = false;
    for (size_t di = 0; di < doms0.size(); ++di) {
      const Rect3 c = doms0[di].get_compute_region();
      remote = remote || !(li[di].lo == c.lo && li[di].hi == c.hi);
      xcut = xcut || li[di].lo.x != c.lo.x || li[di].hi.x != c.hi.x;
    }
    if (cfg_.autoOverlap) overlap_ = overlap_ && remote && !xcut;
    // forced overlap without remote halos (one GPU): the classic full split, exercises every slab kernel
    pairInteriors_ = remote ? li : dd_->get_interior();
    for (const auto &r : pairInteriors_) overlap_ = overlap_ && !r.empty();
    // the sweep leaves x2reserve CUs free and the transports' pack/unpack kernels stay on that many CUs
    if (overlap_) dd_->set_comm_max_blocks(cfg_.tune.x2reserve);
  }
  pairTune_ = cfg_.tune;
  pairTune_.wrap = 0;
  // overlapped and whole-region pairs can be switched at run time when both would wrap the same axes: the local
  // interior is shrunk only along axes cut across GPUs, which are never self-wrapped (set_overlap)
  bool sameWrap = true;
  if (pairs_ && cfg_.wrapSelf) {
    int w = dd_->self_wrap_axes() & cfg_.wrapAxesMask;
    for (size_t di = 0; di < doms0.size(); ++di) {
      const auto &d = doms0[di];
      for (int64_t q = 0; q < d.num_data(); ++q) w &= stencil7x2_wrappable_axes(d, q, cfg_.tune.x2row);
    }
    // fused triples where the whole-row kernel cannot wrap x (rows other than 512 fp32 cells: the 1024-wide cbrt
    // shape, fp64): read x from halos (the XH form) and leave the x self copies in the exchange, one per three steps,
    // instead of falling back to pairs that wrap x
    if (cfg_.temporal >= 3 && (w & 1) && doms0[0].backend() == Backend::Device) {
      StencilTune tw = cfg_.tune, th = cfg_.tune;
      tw.wrap = w;
      th.wrap = w & ~1;
      bool withWrap = true, withHalo = true;
      for (const auto &d : doms0)
        for (int64_t q = 0; q < d.num_data(); ++q) {
          withWrap = withWrap && stencil7x3_supported(d, q, d.get_compute_region(), tw);
          withHalo = withHalo && stencil7x3_supported(d, q, d.get_compute_region(), th);
        }
      if (!withWrap && withHalo) w &= ~1;
    }
    int wOn = w;
    for (size_t di = 0; di < doms0.size() && !pairInteriors_.empty(); ++di) {
      // the swept regions must span every wrapped axis (a forced full split cuts all of them)
      const Rect3 c = doms0[di].get_compute_region();
      const Rect3 &r = pairInteriors_[di];
      if (r.lo.x != c.lo.x || r.hi.x != c.hi.x) wOn &= ~1;
      if (r.lo.y != c.lo.y || r.hi.y != c.hi.y) wOn &= ~2;
      if (r.lo.z != c.lo.z || r.hi.z != c.hi.z) wOn &= ~4;
    }
    sameWrap = wOn == w;
    if (overlap_) w = wOn;
    pairTune_.wrap = w;
    if (w != 0) dd_->prepare_skip_wrapped(w);
  }
  if (pairs_ && sameWrap && !pairInteriors_.empty()) {
    const auto li = dd_->get_local_interior(2);
    bool remote = false, ok = true;
    for (size_t di = 0; di < doms0.size(); ++di) {
      const Rect3 c = doms0[di].get_compute_region();
      remote = remote || !(li[di].lo == c.lo && li[di].hi == c.hi);
      ok = ok && !pairInteriors_[di].empty();
    }
    overlapToggle_ = remote && ok && doms0[0].backend() == Backend::Device;
  }
  // pipelined pairs (overlap mode 3): one device, halos remote along z only (every boundary plane an exchange reads
  // is one of the first / last two z planes of the sweep), the whole-row kernel for every quantity, and a plan the
  // producer gate can start (fused co-located stores only; re-checked per pair since the co-located copy can change)
  if (overlapToggle_ && doms0.size() == 1 && doms0[0].backend() == Backend::Device) {
    const auto li = dd_->get_local_interior(2);
    const Rect3 c = doms0[0].get_compute_region();
    bool ok = li[0].lo.x == c.lo.x && li[0].hi.x == c.hi.x && li[0].lo.y == c.lo.y && li[0].hi.y == c.hi.y &&
              dd_->gated_send_supported(pairTune_.wrap) && c.extent().z >= 4 * pubDepth_;
    for (int64_t q = 0; q < doms0[0].num_data() && ok; ++q) ok = stencil7x2_row_kernel_used(doms0[0], q, c, pairTune_);
    if (ok) {
      pipeOk_ = true;
      const Dim3 e = c.extent();
      pubCells_ = uint64_t(e.x) * uint64_t(e.y) * uint64_t(std::min<int64_t>(e.z, 2 * pubDepth_)) *
                  uint64_t(doms0[0].num_data());
      doms0[0].set_device();
      HIP_CHECK(hipExtMallocWithFlags((void **)&pubCounter_, 256, hipDeviceMallocUncached));
      HIP_CHECK(hipMemset(pubCounter_, 0, 256));
      HIP_CHECK(hipDeviceSynchronize());
      if (cfg_.overlapMode == 3 && overlap_) pipelined_ = true;
    }
  }
  // single steps: the self-periodic axes are read in-kernel at their periodic image and their same-GPU copies leave
  // the exchange (a fully periodic sub-domain exchanges nothing; one MI355X at 512^3: the ~25 us copy-plan kernel of
  // a ~225 us step). Overlapped, as for the fused pairs: the same-GPU translate first, the interior shrunk only at
  // faces whose halo arrives from another GPU (get_local_interior) during the remote transfers, the slabs at those
  // faces after them, and the sweep leaves x2reserve CUs to the transports' kernels.
  stepTune_ = cfg_.tune;
  stepTune_.wrap = 0;
  localSteps_ = false;
  const bool stepDevice = !doms0.empty() && doms0[0].backend() == Backend::Device;
  if (!pairs_ && !forward_ && overlap_ && stepDevice && cfg_.wrapSelf && cfg_.tune.variant != StencilTune::kMfma &&
      cfg_.localInterior) {
    const auto li = dd_->get_local_interior(1);
    bool remote = false, ok = true;
    for (size_t di = 0; di < doms0.size(); ++di) {
      const Rect3 c = doms0[di].get_compute_region();
      remote = remote || !(li[di].lo == c.lo && li[di].hi == c.hi);
      ok = ok && !li[di].empty();
    }
    if (remote && ok) {
      localSteps_ = true;
      stepInteriors_ = li;
      stepExteriors_.assign(doms0.size(), {});
      for (size_t di = 0; di < doms0.size(); ++di) {
        const Rect3 c = doms0[di].get_compute_region(), in = li[di];
        for (const Rect3 &r : {Rect3(c.lo, Dim3(c.hi.x, c.hi.y, in.lo.z)), Rect3(Dim3(c.lo.x, c.lo.y, in.hi.z), c.hi),
                               Rect3(Dim3(c.lo.x, c.lo.y, in.lo.z), Dim3(c.hi.x, in.lo.y, in.hi.z)),
                               Rect3(Dim3(c.lo.x, in.hi.y, in.lo.z), Dim3(c.hi.x, c.hi.y, in.hi.z)),
                               Rect3(Dim3(c.lo.x, in.lo.y, in.lo.z), Dim3(in.lo.x, in.hi.y, in.hi.z)),
                               Rect3(Dim3(in.hi.x, in.lo.y, in.lo.z), Dim3(c.hi.x, in.hi.y, in.hi.z))})
          if (!r.empty()) stepExteriors_[di].push_back(r);
      }
      dd_->set_comm_max_blocks(cfg_.tune.x2reserve);
    } else if (!remote && cfg_.autoOverlap) {
      overlap_ = false; // every halo from this GPU: exchange -> whole-region step
    }
  }
  if (!pairs_ && !forward_ && (!overlap_ || localSteps_) && stepDevice && cfg_.wrapSelf &&
      cfg_.tune.variant != StencilTune::kMfma) {
    int w = dd_->self_wrap_axes() & cfg_.wrapAxesMask;
    for (size_t di = 0; di < doms0.size(); ++di) {
      const auto &d = doms0[di];
      for (int64_t q = 0; q < d.num_data(); ++q) w &= stencil7_wrappable_axes(d, q);
      // the swept regions must span every wrapped axis
      const Rect3 c = d.get_compute_region();
      const Rect3 r = localSteps_ ? stepInteriors_[di] : c;
      if (r.lo.x != c.lo.x || r.hi.x != c.hi.x) w &= ~1;
      if (r.lo.y != c.lo.y || r.hi.y != c.hi.y) w &= ~2;
      if (r.lo.z != c.lo.z || r.hi.z != c.hi.z) w &= ~4;
    }
    stepTune_.wrap = w;
    if (w != 0) dd_->prepare_skip_wrapped(w);
  }
  // forced overlap of single steps whose every halo is a same-GPU copy (one GPU with --no-wrap: BASELINE config 4 as
  // the reference runs it, bin/astaroth_sim.cu:223-274): the copy-plan translate runs confined to x2reserve CUs on
  // the comm stream while the interior sweep leaves those CUs free, then the exterior slabs
  confinedSelf_ = !pairs_ && !forward_ && overlap_ && !localSteps_ && stepDevice && cfg_.tune.x2reserve > 0 &&
                  dd_->exchange_bytes_for_method(MethodFlags::Kernel) == dd_->exchange_bytes_for_method(MethodFlags::All);
  if (confinedSelf_) dd_->set_translate_max_blocks(cfg_.tune.x2reserve);
  // overlapped pairs with the slabs after the interior sweep (set_overlap_mode(2)) from the start
  slabsAfter_ = pairs_ && overlap_ && cfg_.overlapMode == 2;
  // fused triples: device sub-domains of whole 512-cell fp32 rows wrapped in-kernel, or of 512-cell fp32 / 256-cell
  // fp64 columns whose x halos come from the exchange (stencil7x3_supported); each other axis wraps in-kernel (its
  // self copies leave the exchange) or reads the 3-deep halos of a depth-3 exchange, one per three steps.
  // Whole regions only, so not beside an overlapped exchange (set_overlap switches between the two). The spheres at
  // least 3 cells from the periodic faces (the intermediate steps evaluate them at unwrapped halo coordinates)
  triples_ = pairs_ && cfg_.temporal >= 3 && stepDevice;
  if (triples_ && sph_.enabled) {
    const Dim3 L = cfg_.size;
    for (const Dim3 &c : {sph_.hot, sph_.cold}) {
      const int64_t cc[3] = {c.x, c.y, c.z}, ll[3] = {L.x, L.y, L.z};
      for (int a = 0; a < 3; ++a)
        if (cc[a] - sph_.radius < 2 || cc[a] + sph_.radius > ll[a] - 3) triples_ = false;
    }
  }
  for (size_t di = 0; di < doms0.size() && triples_; ++di)
    for (int64_t q = 0; triples_ && q < doms0[di].num_data(); ++q)
      triples_ = stencil7x3_supported(doms0[di], q, doms0[di].get_compute_region(), pairTune_);
  triplesOk_ = triples_;
  triples_ = triplesOk_ && !overlap_;
  graphs_ = cfg_.useGraph && !overlap_ && dd_->domains().size() == 1 &&
            dd_->domains()[0].backend() == Backend::Device &&
            dd_->exchange_bytes_for_method(MethodFlags::Kernel) == dd_->exchange_bytes_for_method(MethodFlags::All) &&
            dd_->world_size() == 1;
  interiors_ = dd_->get_interior();
  exteriors_ = dd_->get_exterior();
  auto &doms = dd_->domains();
  for (size_t di = 0; di < doms.size(); ++di) {
    auto &d = doms[di];
    if (d.backend() == Backend::Device) {
      compute_.emplace_back(d.gpu(), Priority::DEFAULT);
      exteriorDone_.emplace_back(d.gpu());
    }
    hipStream_t s = compute_.empty() ? nullptr : compute_.back().get();
    for (int64_t q = 0; q < d.num_data(); ++q) {
      if (cfg_.kind == StencilKind::Jacobi)
        jacobi_init(d, q, d.get_compute_region(), s);
      else
        astaroth_init(d, q, cfg_.astarothPeriod, s);
    }
  }
  synchronize();
  for (size_t di = 0; di < doms.size(); ++di)
    if (!compute_.empty()) dd_->record_ready(di, compute_[di]);
  if (forward_) {
    // from now on the kernels keep the halos current; fill them once for the initial state
    dd_->exchange();
    fwd_.resize(doms.size());
    for (size_t di = 0; di < doms.size(); ++di) {
      const auto targets = dd_->forward_targets(di);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        fwd_[di].emplace_back(new HaloForwarder(doms[di], q, targets));
      stepDone_.emplace_back(doms[di].gpu());
    }
    for (size_t di = 0; di < doms.size(); ++di) stepDone_[di].record(compute_[di]);
  }
}

void StencilModel::step() {
  TraceRange tr("StencilModel::step");
  auto &doms = dd_->domains();
  if (graphs_) {
    const int p = doms[0].parity();
    hipStream_t s = compute_[0].get();
    if (!graphExec_[p]) {
      hipGraph_t g = nullptr;
      HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      enqueue_step();
      HIP_CHECK(hipStreamEndCapture(s, &g));
      HIP_CHECK(hipGraphInstantiate(&graphExec_[p], g, nullptr, nullptr, 0));
      HIP_CHECK(hipGraphDestroy(g));
    }
    HIP_CHECK(hipGraphLaunch(graphExec_[p], s));
    dd_->swap();
    ++steps_;
    return;
  }
  enqueue_step();
  dd_->swap();
  // the next exchange must follow this step's compute; in single-stream mode stream order already guarantees it
  const bool device = !compute_.empty();
  const bool singleStream = device && !overlap_ && !pipelined3_ && doms.size() == 1;
  if (device && !singleStream)
    for (size_t di = 0; di < doms.size(); ++di) dd_->record_ready(di, compute_[di]);
  ++steps_;
}

void StencilModel::run(int iters) {
  TraceRange tr("StencilModel::run");
  auto &doms = dd_->domains();
  if (graphs_ && iters > 0) { // a whole run recorded by prepare({iters})
    auto it = runGraph_.find({iters, doms[0].parity()});
    if (it != runGraph_.end()) {
      for (int k = 0; k < it->second.sweeps; ++k) dd_->swap();
      HIP_CHECK(hipGraphLaunch(it->second.exec, compute_[0].get()));
      steps_ += iters;
      return;
    }
  }
  const int per = steps_per_sweep(), gsteps = graph_steps();
  const int sweeps = gsteps / per; // sweeps per graph block (an even number: the block keeps the parity)
  while (graphs_ && iters >= gsteps) {
    const int p = doms[0].parity();
    hipStream_t s = compute_[0].get();
    if (!graphBlock_[p]) capture_block();
    for (int k = 0; k < sweeps; ++k) dd_->swap();
    HIP_CHECK(hipGraphLaunch(graphBlock_[p], s));
    steps_ += gsteps;
    iters -= gsteps;
  }
  const bool device = !compute_.empty();
  const bool singleStream = device && !overlap_ && !pipelined3_ && doms.size() == 1;
  while (triples_ && iters >= 3) {
    enqueue_step(3);
    dd_->swap();
    if (device && !singleStream)
      for (size_t di = 0; di < doms.size(); ++di) dd_->record_ready(di, compute_[di]);
    steps_ += 3;
    iters -= 3;
  }
  while (pairs_ && iters >= 2) {
    enqueue_step(2);
    dd_->swap();
    if (device && !singleStream)
      for (size_t di = 0; di < doms.size(); ++di) dd_->record_ready(di, compute_[di]);
    steps_ += 2;
    iters -= 2;
  }
  for (int i = 0; i < iters; ++i) step();
}

void StencilModel::capture_block() {
  // records kGraphSteps steps starting at the current buffer parity into graphBlock_[parity]; nothing runs, and
  // the swaps done while recording are undone (an even number of sweeps returns to the same parity anyway)
  auto &doms = dd_->domains();
  const int per = steps_per_sweep(), sweeps = graph_steps() / per;
  const int p = doms[0].parity();
  hipStream_t s = compute_[0].get();
  hipGraph_t g = nullptr;
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < sweeps; ++k) {
    enqueue_step(per);
    dd_->swap(); // pointers only; the captured kernels carry the buffers of each sweep
  }
  HIP_CHECK(hipStreamEndCapture(s, &g));
  HIP_CHECK(hipGraphInstantiate(&graphBlock_[p], g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(g));
}

void StencilModel::capture_run(int n) {
  // the sweeps run(n) enqueues (graph blocks, then triples, pairs, single steps: the same kernels in the same order)
  // recorded as one graph; the swaps done while recording are undone
  auto &doms = dd_->domains();
  const int p = doms[0].parity();
  hipStream_t s = compute_[0].get();
  hipGraph_t g = nullptr;
  int sw = 0;
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int left = n; left > 0;) {
    const int k = triples_ && left >= 3 ? 3 : (pairs_ && left >= 2 ? 2 : 1);
    enqueue_step(k);
    dd_->swap();
    ++sw;
    left -= k;
  }
  HIP_CHECK(hipStreamEndCapture(s, &g));
  RunGraph rg;
  rg.sweeps = sw;
  HIP_CHECK(hipGraphInstantiate(&rg.exec, g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(g));
  if (sw % 2) dd_->swap();
  runGraph_[{n, p}] = rg;
}

void StencilModel::prepare(const std::vector<int> &runs) {
  // instantiate the graph blocks of both buffer parities up front, so the first run() of a timed loop does not pay
  // for stream capture + instantiation (the bench's warm-up may be shorter than one block)
  if (!graphs_) return;
  for (int i = 0; i < 2; ++i) {
    if (!graphBlock_[dd_->domains()[0].parity()]) capture_block();
    for (int n : runs) {
      STENCIL_REQUIRE(n > 0 && n <= 1024, "prepare: run length " << n << " outside [1, 1024]");
      if (!runGraph_.count({n, dd_->domains()[0].parity()})) capture_run(n);
    }
    dd_->swap();
  }
}

void StencilModel::enqueue_step(int k) {
  auto &doms = dd_->domains();
  const bool device = !compute_.empty();
  const bool gateOk = lastPublished_; // the previous sweep published: the next exchange may start on its planes
  lastPublished_ = false;
  if (k == 2 && pipelined_) {
    // pipelined pairs: this pair's exchange was gated on the previous sweep's boundary planes (it ran beside the
    // rest of that sweep); the sweep waits for it, then publishes its own boundary planes for the next exchange
    const bool gate = gateOk && dd_->gated_send_supported(pairTune_.wrap);
    if (gate) dd_->set_send_gate(pubCounter_, pubTotal_);
    dd_->exchange_async(nullptr, pairTune_.wrap);
    dd_->wait_exchange(0, compute_[0]);
    StencilTune ti = pairTune_;
    ti.reserveCUs = cfg_.tune.x2reserve;
    const Rect3 c = doms[0].get_compute_region();
    const bool pub = dd_->gated_send_supported(pairTune_.wrap);
    if (pub) {
      ti.publish = pubCounter_;
      ti.publishDepth = pubDepth_; // the exchange reads this many planes at each z face
      // fixed march directions: the lockstep schedule's outer z parts march away from the domain's z faces, so the
      // boundary planes the next exchange waits for come out at the start of every sweep; the per-pair flip
      // (alternateZ) would write them last on every other pair and leave that exchange nothing to overlap
      ti.alternateZ = false;
    }
    for (int64_t q = 0; q < doms[0].num_data(); ++q)
      stencil7x2_apply(doms[0], q, c, cfg_.kind, sph_, compute_[0].get(), ti);
    if (pub) {
      pubTotal_ += pubCells_;
      lastPublished_ = true;
    }
    return;
  }
  if (k == 2 && overlap_) {
    // temporal blocking, overlapped: interior S o S on the compute stream while the depth-2 exchange runs on the
    // comm stream, then the exterior slabs on the comm stream behind it; the compute stream joins them
    // the interior sweep leaves x2reserve CUs free, so the pack / flag / unpack kernels of the comm stream are
    // not queued behind a grid that holds every CU until it retires
    dd_->exchange_async(nullptr, pairTune_.wrap);
    StencilTune ti = pairTune_;
    ti.reserveCUs = cfg_.tune.x2reserve;
    for (size_t di = 0; di < doms.size(); ++di) {
      dd_->wait_translated(di, compute_[di]);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7x2_apply(doms[di], q, pairInteriors_[di], cfg_.kind, sph_, compute_[di].get(), ti);
    }
    if (slabsAfter_) { // mode 2: the slabs follow the interior sweep on the compute stream, once the halos are in
      for (size_t di = 0; di < doms.size(); ++di) {
        dd_->wait_exchange(di, compute_[di]);
        for (int64_t q = 0; q < doms[di].num_data(); ++q)
          stencil7x2_apply_exterior(doms[di], q, pairInteriors_[di], cfg_.kind, sph_, compute_[di].get(), pairTune_);
      }
      return;
    }
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = dd_->comm_stream(di);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7x2_apply_exterior(doms[di], q, pairInteriors_[di], cfg_.kind, sph_, s, pairTune_);
      exteriorDone_[di].record(s);
      exteriorDone_[di].wait_on(compute_[di]);
    }
    return;
  }
  if (k == 3 && pipelined3_) {
    // pipelined triples (mode 4): as the pipelined pairs, this sweep's exchange was gated on the previous sweep's
    // boundary planes and ran beside the rest of that sweep; the sweep waits for it, leaves x2reserve CUs to the
    // next gated exchange and publishes its own first / last 3 z planes early (fixed march directions)
    const bool gate = gateOk && dd_->gated_send_supported(pairTune_.wrap);
    if (gate) dd_->set_send_gate(pubCounter_, pubTotal_);
    dd_->exchange_async(nullptr, pairTune_.wrap);
    dd_->wait_exchange(0, compute_[0]);
    StencilTune ti = pairTune_;
    ti.reserveCUs = cfg_.tune.x2reserve;
    const Rect3 c = doms[0].get_compute_region();
    const bool pub = dd_->gated_send_supported(pairTune_.wrap);
    if (pub) {
      ti.publish = pubCounter_;
      ti.publishDepth = pubDepth_;
      ti.alternateZ = false;
    }
    for (int64_t q = 0; q < doms[0].num_data(); ++q)
      STENCIL_REQUIRE(stencil7x3_apply(doms[0], q, c, cfg_.kind, sph_, compute_[0].get(), ti),
                      "fused triple not supported for quantity " << q);
    if (pub) {
      pubTotal_ += pubCells_;
      lastPublished_ = true;
    }
    return;
  }
  if (k == 3) {
    // fused triples: one depth-3 exchange (one GPU: every halo is read in-kernel at its periodic image, so it has
    // nothing left to copy and only orders the step), then S o S o S of every sub-domain
    const bool single = device && doms.size() == 1;
    dd_->exchange_async(single ? compute_[0].get() : nullptr, pairTune_.wrap);
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = device ? compute_[di].get() : nullptr;
      if (!single) dd_->wait_exchange(di, s);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        STENCIL_REQUIRE(stencil7x3_apply(doms[di], q, doms[di].get_compute_region(), cfg_.kind, sph_, s, pairTune_),
                        "fused triple not supported for quantity " << q);
    }
    return;
  }
  if (k == 2) {
    // temporal blocking: one depth-2 exchange, then S o S on every sub-domain
    const bool single = device && doms.size() == 1;
    dd_->exchange_async(single ? compute_[0].get() : nullptr, pairTune_.wrap);
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = device ? compute_[di].get() : nullptr;
      if (!single) dd_->wait_exchange(di, s);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7x2_apply(doms[di], q, doms[di].get_compute_region(), cfg_.kind, sph_, s, pairTune_);
    }
    return;
  }
  if (forward_) {
    // step i of a sub-domain overwrites halos its neighbours read in step i-1 and reads halos they write in step
    // i-1: with several sub-domains every stream first joins the previous step of all the others
    const bool multi = doms.size() > 1;
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = compute_[di].get();
      if (multi)
        for (size_t dj = 0; dj < doms.size(); ++dj)
          if (dj != di) stepDone_[dj].wait_on(s);
      for (int64_t q = 0; q < doms[di].num_data(); ++q) {
        const HaloForwarder *f = fwd_[di][size_t(q)].get();
        stencil7_apply(doms[di], q, doms[di].get_compute_region(), cfg_.kind, sph_, s, cfg_.tune, f);
        f->forward_rest(doms[di].parity(), s);
      }
    }
    if (multi)
      for (size_t di = 0; di < doms.size(); ++di) stepDone_[di].record(compute_[di]);
    return;
  }
  if (localSteps_) {
    // single step, overlapped against the remote part of the exchange only (see init)
    dd_->exchange_async(nullptr, stepTune_.wrap);
    StencilTune ti = stepTune_;
    ti.reserveCUs = cfg_.tune.x2reserve;
    for (size_t di = 0; di < doms.size(); ++di) {
      dd_->wait_translated(di, compute_[di]);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply(doms[di], q, stepInteriors_[di], cfg_.kind, sph_, compute_[di].get(), ti);
    }
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = dd_->comm_stream(di);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply_regions(doms[di], q, stepExteriors_[di], cfg_.kind, sph_, s, stepTune_);
      exteriorDone_[di].record(s);
      exteriorDone_[di].wait_on(compute_[di]);
    }
    return;
  }
  if (overlap_) {
    // exchange first: its pack/send kernels (high-priority comm stream) get CUs before the interior sweep fills them
    dd_->exchange_async();
    StencilTune ti = cfg_.tune;
    if (confinedSelf_) ti.reserveCUs = cfg_.tune.x2reserve;
    for (size_t di = 0; di < doms.size(); ++di)
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply(doms[di], q, interiors_[di], cfg_.kind, sph_, device ? compute_[di].get() : nullptr, ti);
    // The exterior slabs only need the halos, not the interior result: run them on the comm stream right behind
    // the exchange; the compute stream then joins the comm stream.
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = device ? dd_->comm_stream(di) : nullptr;
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply_regions(doms[di], q, exteriors_[di], cfg_.kind, sph_, s, cfg_.tune);
      if (device) {
        exteriorDone_[di].record(s);
        exteriorDone_[di].wait_on(compute_[di]);
      }
    }
  } else {
    // one device: enqueue the exchange on the compute stream itself (no cross-stream hand-offs)
    const bool single = device && doms.size() == 1;
    dd_->exchange_async(single ? compute_[0].get() : nullptr, stepTune_.wrap);
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = device ? compute_[di].get() : nullptr;
      if (!single) dd_->wait_exchange(di, s);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply(doms[di], q, doms[di].get_compute_region(), cfg_.kind, sph_, s, stepTune_);
    }
  }
}

void StencilModel::set_overlap(bool on) {
  STENCIL_REQUIRE(overlapToggle_, "set_overlap: this model's pairs cannot switch overlap (no remote halos, or the "
                                  "overlapped sweep would wrap other axes)");
  if (on == overlap_) return;
  synchronize();
  overlap_ = on;
  triples_ = triplesOk_ && !on; // whole-region sweeps: triples where supported
  dd_->set_comm_max_blocks(on ? cfg_.tune.x2reserve : 0);
  // the same-GPU translate stays confined only while an overlapped sweep leaves it those CUs
  dd_->set_translate_max_blocks(on && confinedSelf_ ? cfg_.tune.x2reserve : 0);
}

void StencilModel::set_overlap_mode(int mode) {
  STENCIL_REQUIRE(mode >= 0 && mode <= 4, "overlap mode " << mode);
  STENCIL_REQUIRE(mode != 3 || pipeOk_, "overlap mode 3 (pipelined pairs) is not possible for this model");
  STENCIL_REQUIRE(mode != 4 || can_pipeline_triples(), "overlap mode 4 (pipelined triples) is not possible for this model");
  if (mode == overlap_mode()) return;
  set_overlap(mode != 0 && mode != 4);
  slabsAfter_ = mode == 2;
  pipelined_ = mode == 3;
  pipelined3_ = mode == 4;
  // the gated exchanges of modes 3 / 4 run beside the sweep on the CUs it leaves free
  dd_->set_comm_max_blocks(mode != 0 ? cfg_.tune.x2reserve : 0);
}

void StencilModel::set_comm_reserve(int cus) {
  STENCIL_REQUIRE(cus >= 0 && cus <= 128, "comm reserve " << cus);
  if (cus == cfg_.tune.x2reserve) return;
  synchronize();
  cfg_.tune.x2reserve = cus;
  pairTune_.x2reserve = cus;
  stepTune_.x2reserve = cus;
  if (overlap_ || pipelined3_) dd_->set_comm_max_blocks(cus);
  if (confinedSelf_ && overlap_) dd_->set_translate_max_blocks(cus);
}

void StencilModel::set_triple_schedule(float sphw, int left, int parts) {
  STENCIL_REQUIRE(left >= 0 && left <= 3 && parts >= 0 && parts <= 8 && sphw >= 0, "triple schedule");
  synchronize();
  for (StencilTune *t : {&cfg_.tune, &pairTune_, &stepTune_}) {
    t->x3sphw = sphw;
    t->x3left = left;
    t->x3parts = parts;
  }
  drop_graphs();
}

void StencilModel::drop_graphs() {
  for (auto &g : graphExec_)
    if (g) {
      HIP_CHECK(hipGraphExecDestroy(g));
      g = nullptr;
    }
  for (auto &g : graphBlock_)
    if (g) {
      HIP_CHECK(hipGraphExecDestroy(g));
      g = nullptr;
    }
  for (auto &kv : runGraph_)
    if (kv.second.exec) HIP_CHECK(hipGraphExecDestroy(kv.second.exec));
  runGraph_.clear();
}

void StencilModel::synchronize() {
  // the compute streams join the exchange (wait_exchange / exteriorDone_ / the exchange enqueued on them), so a
  // stalled peer stalls them too: DistributedDomain polls them with its watchdog instead of blocking on them first
  std::vector<hipStream_t> streams;
  for (auto &s : compute_) streams.push_back(s.get());
  if (dd_->realized())
    dd_->sync_streams(streams);
  else
    for (auto &s : compute_) s.sync();
}

} // namespace stencil
