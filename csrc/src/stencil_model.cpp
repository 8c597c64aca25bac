#include "stencil/models/stencil_model.hpp"

#include <cstdlib>

#include "stencil/rt/hip_check.hpp"
#include "stencil/rt/trace.hpp"

namespace stencil {

StencilModel::StencilModel(const StencilModelConfig &cfg, std::shared_ptr<comm::ProcGroup> pg) : cfg_(cfg) {
  dd_.reset(new DistributedDomain(cfg.size.x, cfg.size.y, cfg.size.z, pg));
  if (cfg.allDirections) {
    dd_->set_radius(cfg.radius);
  } else {
    Radius r = Radius::constant(0);
    r.set_face(cfg.radius);
    dd_->set_radius(r);
  }
  dd_->set_methods(cfg.methods);
  dd_->set_placement(cfg.placement);
  if (!cfg.gpus.empty()) dd_->set_gpus(cfg.gpus);
  if (cfg.setBackend) dd_->set_backend(cfg.backend);
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
}

int64_t StencilModel::local_cells() const {
  int64_t n = 0;
  for (const auto &d : dd_->domains()) n += d.size().flatten();
  return n;
}

hipStream_t StencilModel::compute_stream(size_t di) const { return compute_.empty() ? nullptr : compute_.at(di).get(); }

void StencilModel::init() {
  TraceRange tr("StencilModel::init");
  dd_->realize();
  const Rect3 cReg = dd_->get_compute_region();
  sph_ = cfg_.kind == StencilKind::Jacobi ? Spheres::jacobi(cReg) : Spheres();
  overlap_ = cfg_.overlap;
  if (cfg_.overlap && cfg_.autoOverlap &&
      dd_->exchange_bytes_for_method(MethodFlags::Kernel) == dd_->exchange_bytes_for_method(MethodFlags::All))
    overlap_ = false;
  auto &doms0 = dd_->domains();
  forward_ = cfg_.forward && std::getenv("STENCIL_NO_FORWARD") == nullptr && dd_->world_size() == 1 &&
             dd_->all_direct() && !doms0.empty();
  for (const auto &d : doms0)
    for (int64_t q = 0; q < d.num_data() && forward_; ++q) forward_ = HaloForwarder::supported(d, q);
  if (forward_) overlap_ = false; // the halos travel inside the stencil kernel
  graphs_ = cfg_.useGraph && !overlap_ && dd_->domains().size() == 1 &&
            dd_->domains()[0].backend() == Backend::Device &&
            dd_->exchange_bytes_for_method(MethodFlags::Kernel) == dd_->exchange_bytes_for_method(MethodFlags::All) &&
            dd_->world_size() == 1 && std::getenv("STENCIL_NO_GRAPH") == nullptr;
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
  const bool singleStream = device && !overlap_ && doms.size() == 1;
  if (device && !singleStream)
    for (size_t di = 0; di < doms.size(); ++di) dd_->record_ready(di, compute_[di]);
  ++steps_;
}

void StencilModel::run(int iters) {
  TraceRange tr("StencilModel::run");
  auto &doms = dd_->domains();
  while (graphs_ && iters >= kGraphSteps) {
    const int p = doms[0].parity();
    hipStream_t s = compute_[0].get();
    if (!graphBlock_[p]) {
      hipGraph_t g = nullptr;
      HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int k = 0; k < kGraphSteps; ++k) {
        enqueue_step();
        dd_->swap(); // pointers only; the captured kernels carry the buffers of each step
      }
      HIP_CHECK(hipStreamEndCapture(s, &g));
      HIP_CHECK(hipGraphInstantiate(&graphBlock_[p], g, nullptr, nullptr, 0));
      HIP_CHECK(hipGraphDestroy(g));
    } else {
      for (int k = 0; k < kGraphSteps; ++k) dd_->swap();
    }
    HIP_CHECK(hipGraphLaunch(graphBlock_[p], s));
    steps_ += kGraphSteps;
    iters -= kGraphSteps;
  }
  for (int i = 0; i < iters; ++i) step();
}

void StencilModel::enqueue_step() {
  auto &doms = dd_->domains();
  const bool device = !compute_.empty();
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
  if (overlap_) {
    // exchange first: its pack/send kernels (high-priority comm stream) get CUs before the interior sweep fills them
    dd_->exchange_async();
    for (size_t di = 0; di < doms.size(); ++di)
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply(doms[di], q, interiors_[di], cfg_.kind, sph_, device ? compute_[di].get() : nullptr, cfg_.tune);
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
    dd_->exchange_async(single ? compute_[0].get() : nullptr);
    for (size_t di = 0; di < doms.size(); ++di) {
      hipStream_t s = device ? compute_[di].get() : nullptr;
      if (!single) dd_->wait_exchange(di, s);
      for (int64_t q = 0; q < doms[di].num_data(); ++q)
        stencil7_apply(doms[di], q, doms[di].get_compute_region(), cfg_.kind, sph_, s, cfg_.tune);
    }
  }
}

void StencilModel::synchronize() {
  for (auto &s : compute_) s.sync();
  if (dd_->realized()) dd_->sync_exchange();
}

} // namespace stencil
