// pybind11 bindings for stencil2_amd (module stencil2_amd._C).
// Quantity buffers are exported zero-copy as DLPack capsules (kDLROCM device tensors, or kDLCPU for the host
// backend) so Python sees torch tensors aliasing the runtime's halo-padded allocations.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "stencil/comm/proc_group.hpp"
#include "stencil/comm/ipc_event.hpp"
#include "stencil/comm/rccl_comm.hpp"
#include "stencil/domain/distributed_domain.hpp"
#include "stencil/kernels/copy.hpp"
#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/models/stencil_model.hpp"
#include "stencil/rt/build_info.hpp"
#include "stencil/rt/statistics.hpp"
#include "stencil/topo/gpu_topology.hpp"
#include "stencil/topo/partition.hpp"
#include "stencil/topo/placement.hpp"
#include "stencil/topo/qap.hpp"

namespace py = pybind11;
using namespace stencil;

// ---------------- minimal DLPack ABI (v0.8) ----------------
extern "C" {
struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void *data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t *shape;
  int64_t *strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void *manager_ctx;
  void (*deleter)(DLManagedTensor *self);
};
}
static constexpr int32_t kDLCPU = 1, kDLROCM = 10;

struct DLCtx {
  std::shared_ptr<void> keepAlive;
  int64_t shape[3];
  int64_t strides[3];
};

static DLDataType dl_dtype(DType t, int64_t es) {
  switch (t) {
  case DType::F32:
    return {2, 32, 1};
  case DType::F64:
    return {2, 64, 1};
  case DType::F16:
    return {2, 16, 1};
  case DType::BF16:
    return {4, 16, 1};
  case DType::I32:
    return {0, 32, 1};
  case DType::I64:
    return {0, 64, 1};
  case DType::I8:
    return {0, 8, 1};
  case DType::U8:
    return {1, 8, 1};
  case DType::U32:
    return {1, 32, 1};
  case DType::U64:
    return {1, 64, 1};
  default:
    return {1, uint8_t(8 * es), 1};
  }
}

static py::capsule make_capsule(std::shared_ptr<void> keep, const LocalDomain &d, int64_t qi, bool curr) {
  auto *mt = new DLManagedTensor();
  auto *ctx = new DLCtx();
  ctx->keepAlive = std::move(keep);
  const Dim3 raw = d.raw_size(), p = d.pitch(qi);
  ctx->shape[0] = raw.z;
  ctx->shape[1] = raw.y;
  ctx->shape[2] = raw.x;
  ctx->strides[0] = p.x * p.y;
  ctx->strides[1] = p.x;
  ctx->strides[2] = 1;
  mt->dl_tensor.data = curr ? d.curr_data(qi) : d.next_data(qi);
  mt->dl_tensor.device = d.backend() == Backend::Device ? DLDevice{kDLROCM, d.gpu()} : DLDevice{kDLCPU, 0};
  mt->dl_tensor.ndim = 3;
  mt->dl_tensor.dtype = dl_dtype(d.dtype(qi), d.elem_size(qi));
  if (d.dtype(qi) == DType::Bytes && d.elem_size(qi) > 8) {
    // opaque element: expose as bytes with an extra trailing dimension is not expressible in 3D; refuse
    throw std::runtime_error("cannot export opaque element types wider than 8 bytes");
  }
  mt->dl_tensor.shape = ctx->shape;
  mt->dl_tensor.strides = ctx->strides;
  mt->dl_tensor.byte_offset = 0;
  mt->manager_ctx = ctx;
  mt->deleter = [](DLManagedTensor *self) {
    delete static_cast<DLCtx *>(self->manager_ctx);
    delete self;
  };
  return py::capsule(mt, "dltensor", [](PyObject *cap) {
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto *m = static_cast<DLManagedTensor *>(PyCapsule_GetPointer(cap, "dltensor"));
      if (m && m->deleter) m->deleter(m);
    }
  });
}

static Dim3 to_dim3(py::handle h) {
  if (py::isinstance<Dim3>(h)) return h.cast<Dim3>();
  auto t = h.cast<std::vector<int64_t>>();
  if (t.size() != 3) throw std::runtime_error("expected 3 coordinates");
  return Dim3(t[0], t[1], t[2]);
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "stencil2_amd native runtime (HIP/gfx950)";
  py::register_exception<stencil::Error>(m, "StencilError", PyExc_RuntimeError);

  py::class_<Dim3>(m, "Dim3")
      .def(py::init<>())
      .def(py::init<int64_t, int64_t, int64_t>())
      .def_readwrite("x", &Dim3::x)
      .def_readwrite("y", &Dim3::y)
      .def_readwrite("z", &Dim3::z)
      .def("flatten", &Dim3::flatten)
      .def("wrap", &Dim3::wrap)
      .def("max", &Dim3::max)
      .def("min", &Dim3::min)
      .def("__add__", [](const Dim3 &a, const Dim3 &b) { return a + b; })
      .def("__sub__", [](const Dim3 &a, const Dim3 &b) { return a - b; })
      .def("__mul__", [](const Dim3 &a, const Dim3 &b) { return a * b; })
      .def("__mul__", [](const Dim3 &a, int64_t s) { return a * s; })
      .def("__floordiv__", [](const Dim3 &a, const Dim3 &b) { return a / b; })
      .def("__mod__", [](const Dim3 &a, const Dim3 &b) { return a % b; })
      .def("__neg__", [](const Dim3 &a) { return -a; })
      .def("__eq__", [](const Dim3 &a, const Dim3 &b) { return a == b; })
      .def("__ne__", [](const Dim3 &a, const Dim3 &b) { return a != b; })
      .def("__lt__", [](const Dim3 &a, const Dim3 &b) { return a < b; })
      .def("__hash__", [](const Dim3 &a) { return py::hash(py::make_tuple(a.x, a.y, a.z)); })
      .def("__iter__", [](const Dim3 &a) { return py::iter(py::make_tuple(a.x, a.y, a.z)); })
      .def("tolist", [](const Dim3 &a) { return std::vector<int64_t>{a.x, a.y, a.z}; })
      .def("__repr__", [](const Dim3 &a) {
        return "Dim3(" + std::to_string(a.x) + ", " + std::to_string(a.y) + ", " + std::to_string(a.z) + ")";
      });
  py::implicitly_convertible<py::tuple, Dim3>();
  py::implicitly_convertible<py::list, Dim3>();

  py::class_<Rect3>(m, "Rect3")
      .def(py::init<>())
      .def(py::init<Dim3, Dim3>())
      .def_readwrite("lo", &Rect3::lo)
      .def_readwrite("hi", &Rect3::hi)
      .def("extent", &Rect3::extent)
      .def("empty", &Rect3::empty)
      .def("contains", &Rect3::contains)
      .def("__eq__", [](const Rect3 &a, const Rect3 &b) { return a == b; })
      .def("__repr__", [](const Rect3 &r) {
        std::ostringstream s;
        s << "Rect3(" << r.lo << ", " << r.hi << ")";
        return s.str();
      });

  py::class_<Radius>(m, "Radius")
      .def(py::init<>())
      .def_static("constant", &Radius::constant)
      .def_static("face_edge_corner", &Radius::face_edge_corner)
      .def("dir", [](const Radius &r, int x, int y, int z) { return r.dir(x, y, z); })
      .def("set_dir", [](Radius &r, int x, int y, int z, int64_t v) { r.dir(x, y, z) = v; })
      .def("x", &Radius::x)
      .def("y", &Radius::y)
      .def("z", &Radius::z)
      .def("set_face", &Radius::set_face)
      .def("set_edge", &Radius::set_edge)
      .def("set_corner", &Radius::set_corner)
      .def("max", &Radius::max)
      .def("__eq__", [](const Radius &a, const Radius &b) { return a == b; })
      .def("__copy__", [](const Radius &r) { return Radius(r); });
  py::class_<Boundary>(m, "Boundary")
      .def(py::init<>())
      .def_static("periodic", &Boundary::periodic)
      .def_static("axes", &Boundary::axes, py::arg("x"), py::arg("y"), py::arg("z"))
      .def_static("none", &Boundary::none)
      .def("set_face", &Boundary::set_face)
      .def("set_axis", &Boundary::set_axis)
      .def("face_periodic", &Boundary::face_periodic)
      .def("wraps", [](const Boundary &b, int x, int y, int z) { return b.wraps(Dim3(x, y, z)); })
      .def("all_periodic", &Boundary::all_periodic)
      .def("__eq__", [](const Boundary &a, const Boundary &b) { return a == b; });

  py::enum_<MethodFlags>(m, "MethodFlags", py::arithmetic())
      .value("None_", MethodFlags::None)
      .value("Staged", MethodFlags::Staged)
      .value("Rccl", MethodFlags::Rccl)
      .value("Colocated", MethodFlags::Colocated)
      .value("PeerCopy", MethodFlags::PeerCopy)
      .value("Kernel", MethodFlags::Kernel)
      .value("All", MethodFlags::All)
      .def("__or__", [](MethodFlags a, MethodFlags b) { return a | b; })
      .def("__and__", [](MethodFlags a, MethodFlags b) { return a & b; });
  m.def("methods_to_string", [](MethodFlags f) { return to_string(f); });
  m.def(
      "select_method",
      [](MethodFlags flags, bool device, bool same_rank, bool same_device, bool peer, bool same_host, bool can_access,
         bool shared_gpu) {
        PairInfo p;
        p.device = device;
        p.sameRank = same_rank;
        p.sameDevice = same_device;
        p.peer = peer;
        p.sameHost = same_host;
        p.canAccess = can_access;
        p.sharedGpu = shared_gpu;
        return select_method(flags, p);
      },
      py::arg("flags"), py::arg("device") = true, py::arg("same_rank") = false, py::arg("same_device") = false,
      py::arg("peer") = false, py::arg("same_host") = false, py::arg("can_access") = false,
      py::arg("shared_gpu") = false);
  py::enum_<PlacementStrategy>(m, "PlacementStrategy")
      .value("NodeAware", PlacementStrategy::NodeAware)
      .value("Trivial", PlacementStrategy::Trivial);
  py::enum_<Backend>(m, "Backend").value("Host", Backend::Host).value("Device", Backend::Device);
  py::enum_<DType>(m, "DType")
      .value("Bytes", DType::Bytes)
      .value("F32", DType::F32)
      .value("F64", DType::F64)
      .value("I32", DType::I32)
      .value("I64", DType::I64)
      .value("U8", DType::U8)
      .value("I8", DType::I8)
      .value("F16", DType::F16)
      .value("BF16", DType::BF16)
      .value("U32", DType::U32)
      .value("U64", DType::U64);
  py::enum_<StencilKind>(m, "StencilKind").value("Jacobi", StencilKind::Jacobi).value("Astaroth", StencilKind::Astaroth);

  // ---------------- process group ----------------
  py::class_<comm::ProcGroup, std::shared_ptr<comm::ProcGroup>>(m, "ProcGroup")
      .def("rank", &comm::ProcGroup::rank)
      .def("size", &comm::ProcGroup::size)
      .def("hostname", &comm::ProcGroup::hostname)
      .def("barrier", &comm::ProcGroup::barrier, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_max", &comm::ProcGroup::allreduce_max, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_sum", &comm::ProcGroup::allreduce_sum, py::call_guard<py::gil_scoped_release>())
      .def("colocated_ranks", &comm::ProcGroup::colocated_ranks)
      .def("colocated_rank", &comm::ProcGroup::colocated_rank)
      .def("colocated_size", &comm::ProcGroup::colocated_size)
      .def("num_nodes", &comm::ProcGroup::num_nodes)
      .def("send_bytes",
           [](comm::ProcGroup &g, int dst, uint32_t tag, py::bytes b) {
             std::string s = b;
             py::gil_scoped_release r;
             g.send(dst, tag, s.data(), s.size());
           })
      .def("recv_bytes",
           [](comm::ProcGroup &g, int src, uint32_t tag, size_t n) {
             std::string s(n, '\0');
             {
               py::gil_scoped_release r;
               g.recv(src, tag, &s[0], n);
             }
             return py::bytes(s);
           })
      .def("allgather_bytes", [](comm::ProcGroup &g, py::bytes b) {
        std::string s = b;
        std::string out(s.size() * size_t(g.size()), '\0');
        {
          py::gil_scoped_release r;
          g.allgather(s.data(), s.size(), &out[0]);
        }
        py::list l;
        for (int i = 0; i < g.size(); ++i) l.append(py::bytes(out.substr(i * s.size(), s.size())));
        return l;
      });
  m.def("make_single_group", &comm::make_single_group);
  m.def("make_tcp_group", &comm::make_tcp_group, py::arg("rank"), py::arg("size"), py::arg("master_addr"),
        py::arg("master_port"), py::arg("timeout_s") = 600.0, py::call_guard<py::gil_scoped_release>());
  m.def("make_group_from_env", &comm::make_group_from_env, py::call_guard<py::gil_scoped_release>());
  m.def("default_group", &comm::default_group, py::call_guard<py::gil_scoped_release>());
  m.def("set_default_group", &comm::set_default_group);
  m.def("find_free_port", &comm::find_free_port);
  // a one-wave kernel that busy-waits `seconds` on `stream` (tests: hold a stream while host work runs ahead of it)
  m.def(
      "spin_device", [](double seconds, uintptr_t stream) { spin_device(seconds, reinterpret_cast<hipStream_t>(stream)); },
      py::arg("seconds"), py::arg("stream") = 0);
  m.def("set_copy_block_items", &set_copy_block_items, py::arg("narrow"), py::arg("wide"));
  m.def("set_copy_small_rows", &set_copy_small_rows, py::arg("max_items"), py::arg("per_entry"));
  m.def("ipc_event_stress", &ipc_event_stress, py::arg("group"), py::arg("device"), py::arg("n"), py::arg("after"),
        py::call_guard<py::gil_scoped_release>());
  m.def(
      "ipc_event_roundtrip",
      [](std::shared_ptr<comm::ProcGroup> g, int device, double spin) {
        IpcEventReport r;
        {
          py::gil_scoped_release nogil;
          r = ipc_event_roundtrip(*g, device, spin);
        }
        py::dict d;
        d["ok"] = r.ok;
        d["spin_s"] = r.spinS;
        d["waited_s"] = r.waitedS;
        d["error"] = r.error;
        return d;
      },
      py::arg("group"), py::arg("device") = 0, py::arg("spin_s") = 0.2);

  // ---------------- topology / placement ----------------
  m.def("prime_factors", &prime_factors_desc);
  py::class_<RankPartition>(m, "RankPartition")
      .def(py::init<const Dim3 &, int64_t>())
      .def("dim", &RankPartition::dim)
      .def("subdomain_size", &RankPartition::subdomain_size)
      .def("subdomain_origin", &RankPartition::subdomain_origin)
      .def("linearize", &RankPartition::linearize)
      .def("dimensionize", &RankPartition::dimensionize);
  py::enum_<PartitionObjective>(m, "PartitionObjective")
      .value("Interface", PartitionObjective::Interface)
      .value("MaxLink", PartitionObjective::MaxLink);
  py::class_<NodePartition>(m, "NodePartition")
      .def(py::init<const Dim3 &, const Radius &, int64_t, int64_t, const Dim3 &, PartitionObjective>(), py::arg("size"),
           py::arg("radius"), py::arg("nodes"), py::arg("gpus"), py::arg("axis_cost") = Dim3(1, 1, 1),
           py::arg("objective") = PartitionObjective::Interface)
      .def_static("max_link_dims", &NodePartition::max_link_dims, py::arg("size"), py::arg("n"), py::arg("radius"),
                  py::arg("axis_cost") = Dim3(1, 1, 1))
      .def_static("link_cost", &NodePartition::link_cost, py::arg("size"), py::arg("dims"), py::arg("radius"),
                  py::arg("axis_cost") = Dim3(1, 1, 1))
      .def("dim", &NodePartition::dim)
      .def("sys_dim", &NodePartition::sys_dim)
      .def("node_dim", &NodePartition::node_dim)
      .def("subdomain_size", &NodePartition::subdomain_size)
      .def("subdomain_origin", &NodePartition::subdomain_origin)
      .def("global_idx", &NodePartition::global_idx);
  py::class_<Placement>(m, "Placement")
      .def("get_idx", &Placement::get_idx)
      .def("get_rank", &Placement::get_rank)
      .def("get_subdomain_id", &Placement::get_subdomain_id)
      .def("get_device", &Placement::get_device)
      .def("subdomain_size", &Placement::subdomain_size)
      .def("subdomain_origin", &Placement::subdomain_origin)
      .def("dim", &Placement::dim);
  py::class_<TrivialPlacement, Placement>(m, "TrivialPlacement")
      .def(py::init([](const Dim3 &size, std::shared_ptr<comm::ProcGroup> pg, const std::vector<int> &devs) {
             return new TrivialPlacement(size, *pg, devs);
           }),
           py::keep_alive<1, 3>());
  py::class_<NodeAwarePlacement, Placement>(m, "NodeAwarePlacement")
      .def(py::init([](const Dim3 &size, std::shared_ptr<comm::ProcGroup> pg, const Radius &r,
                       const std::vector<int> &devs, std::function<double(int, int)> bw) {
             return new NodeAwarePlacement(size, *pg, r, devs, bw);
           }),
           py::keep_alive<1, 3>());
  m.def("halo_volume", &halo_volume);
  m.def("packed_message_bytes", &packed_message_bytes);
  m.def("qap_solve", [](const std::vector<std::vector<double>> &w, const std::vector<std::vector<double>> &d) {
    Mat2D<double> W, D;
    for (auto &r : w) W.push_back(r);
    for (auto &r : d) D.push_back(r);
    double c = 0;
    auto f = qap::solve(W, D, &c);
    return py::make_tuple(f, c);
  });
  m.def("qap_solve_catch", [](const std::vector<std::vector<double>> &w, const std::vector<std::vector<double>> &d) {
    Mat2D<double> W, D;
    for (auto &r : w) W.push_back(r);
    for (auto &r : d) D.push_back(r);
    double c = 0;
    auto f = qap::solve_catch(W, D, &c);
    return py::make_tuple(f, c);
  });
  m.def("qap_cost", [](const std::vector<std::vector<double>> &w, const std::vector<std::vector<double>> &d,
                       const std::vector<size_t> &f) {
    Mat2D<double> W, D;
    for (auto &r : w) W.push_back(r);
    for (auto &r : d) D.push_back(r);
    return qap::detail::cost(W, D, f);
  });
  m.def("make_reciprocal", [](const std::vector<std::vector<double>> &w) {
    Mat2D<double> W;
    for (auto &r : w) W.push_back(r);
    Mat2D<double> R = make_reciprocal(W);
    std::vector<std::vector<double>> out(R.rows(), std::vector<double>(R.cols()));
    for (size_t i = 0; i < R.rows(); ++i)
      for (size_t j = 0; j < R.cols(); ++j) out[i][j] = R.at(i, j);
    return out;
  });
  m.def("device_count", &gpu_topo::device_count);
  m.def("gpu_distance", &gpu_topo::distance);
  m.def("gpu_bandwidth", &gpu_topo::bandwidth);
  m.def("enable_peer", &gpu_topo::enable_peer);
  m.def("gpu_links", []() {
    py::list l;
    for (auto &li : gpu_topo::links())
      l.append(py::dict(py::arg("src") = li.src, py::arg("dst") = li.dst, py::arg("type") = li.type,
                        py::arg("hops") = li.hops, py::arg("distance") = li.distance, py::arg("weight") = li.weight,
                        py::arg("min_bw_mbs") = li.minBwMBs, py::arg("max_bw_mbs") = li.maxBwMBs,
                        py::arg("source") = li.source));
    return l;
  });
  m.def("gpu_numa_node", &gpu_topo::numa_node);
  m.def("numa_cpus", &gpu_topo::numa_cpus);
  m.def("amdsmi_available", &gpu_topo::smi_available);

  // ---------------- statistics ----------------
  py::class_<Statistics>(m, "Statistics")
      .def(py::init<>())
      .def("insert", &Statistics::insert)
      .def("count", &Statistics::count)
      .def("avg", &Statistics::avg)
      .def("min", &Statistics::min)
      .def("max", &Statistics::max)
      .def("trimean", &Statistics::trimean)
      .def("med", &Statistics::med)
      .def("stddev", &Statistics::stddev);

  // ---------------- LocalDomain (owned by DistributedDomain; exposed by reference) ----------------
  py::class_<LocalDomain>(m, "LocalDomain")
      .def(py::init<const Dim3 &, const Dim3 &, int, Backend>(), py::arg("size"), py::arg("origin"), py::arg("device"),
           py::arg("backend") = Backend::Device)
      .def("add_data",
           [](LocalDomain &d, int64_t es, const std::string &name, DType dt) { return d.add_data(es, name, dt); },
           py::arg("elem_size"), py::arg("name") = "", py::arg("dtype") = DType::Bytes)
      .def("set_radius", py::overload_cast<int64_t>(&LocalDomain::set_radius))
      .def("set_radius", py::overload_cast<const Radius &>(&LocalDomain::set_radius))
      .def("set_padding", &LocalDomain::set_padding)
      .def("set_x_halo_align", &LocalDomain::set_x_halo_align)
      .def("set_shared_halo_line", &LocalDomain::set_shared_halo_line)
      .def("shared_halo_line", &LocalDomain::shared_halo_line)
      .def("row_limit", &LocalDomain::row_limit)
      .def("x_halo_align", &LocalDomain::x_halo_align)
      .def("set_interior_align", &LocalDomain::set_interior_align)
      .def("set_row_pad_lines", &LocalDomain::set_row_pad_lines)
      .def("interior_align", &LocalDomain::interior_align)
      .def("front_slack", &LocalDomain::front_slack)
      .def("realize", &LocalDomain::realize)
      .def("swap", &LocalDomain::swap)
      .def("size", &LocalDomain::size)
      .def("origin", &LocalDomain::origin)
      .def("radius", &LocalDomain::radius)
      .def("gpu", &LocalDomain::gpu)
      .def("backend", &LocalDomain::backend)
      .def("num_data", &LocalDomain::num_data)
      .def("elem_size", &LocalDomain::elem_size)
      .def("dtype", &LocalDomain::dtype)
      .def("name", &LocalDomain::name)
      .def("raw_size", &LocalDomain::raw_size)
      .def("pitch", &LocalDomain::pitch)
      .def("pad_x", &LocalDomain::pad_x)
      .def("get_compute_region", &LocalDomain::get_compute_region)
      .def("get_full_region", &LocalDomain::get_full_region)
      .def("halo_pos", &LocalDomain::halo_pos)
      .def("halo_coords", &LocalDomain::halo_coords)
      .def("halo_extent", py::overload_cast<const Dim3 &>(&LocalDomain::halo_extent, py::const_))
      .def("halo_bytes", &LocalDomain::halo_bytes)
      .def("buffer_bytes", &LocalDomain::buffer_bytes)
      .def("accessor_origin", &LocalDomain::accessor_origin)
      .def("parity", &LocalDomain::parity)
      .def("curr_ptr", [](const LocalDomain &d, int64_t q) { return reinterpret_cast<uintptr_t>(d.curr_data(q)); })
      .def("next_ptr", [](const LocalDomain &d, int64_t q) { return reinterpret_cast<uintptr_t>(d.next_data(q)); })
      .def("region_to_host",
           [](const LocalDomain &d, const Dim3 &pos, const Dim3 &ext, int64_t q, bool curr) {
             auto v = d.region_to_host(pos, ext, q, curr);
             return py::bytes(reinterpret_cast<const char *>(v.data()), v.size());
           },
           py::arg("pos"), py::arg("ext"), py::arg("qi"), py::arg("curr") = true)
      .def("region_from_host",
           [](LocalDomain &d, const Dim3 &pos, const Dim3 &ext, int64_t q, py::bytes b, bool curr) {
             std::string s = b;
             STENCIL_REQUIRE(int64_t(s.size()) == ext.flatten() * d.elem_size(q), "byte count mismatch");
             d.region_from_host(pos, ext, q, s.data(), curr);
           },
           py::arg("pos"), py::arg("ext"), py::arg("qi"), py::arg("data"), py::arg("curr") = true)
      .def("interior_to_host", [](const LocalDomain &d, int64_t q) {
        auto v = d.interior_to_host(q);
        return py::bytes(reinterpret_cast<const char *>(v.data()), v.size());
      })
      .def("quantity_to_host", [](const LocalDomain &d, int64_t q) {
        auto v = d.quantity_to_host(q);
        return py::bytes(reinterpret_cast<const char *>(v.data()), v.size());
      })
      .def("fill_bytes", &LocalDomain::fill_bytes);

  // ---------------- DistributedDomain ----------------
  py::class_<TransportOptions> topt(m, "TransportOptions");
  py::enum_<TransportOptions::Inbox>(topt, "Inbox")
      .value("Uncached", TransportOptions::Inbox::Uncached)
      .value("Fine", TransportOptions::Inbox::Fine)
      .value("Coarse", TransportOptions::Inbox::Coarse);
  py::enum_<TransportOptions::Copy>(topt, "Copy")
      .value("Store", TransportOptions::Copy::Store)
      .value("Engine", TransportOptions::Copy::Engine);
  py::enum_<TransportOptions::Completion>(topt, "Completion")
      .value("Kernel", TransportOptions::Completion::Kernel)
      .value("StreamOp", TransportOptions::Completion::StreamOp)
      .value("IpcEvent", TransportOptions::Completion::IpcEvent);
  topt.def(py::init<>())
      .def_readwrite("inbox", &TransportOptions::inbox)
      .def_readwrite("colo_copy", &TransportOptions::coloCopy)
      .def_readwrite("peer_copy", &TransportOptions::peerCopy)
      .def_readwrite("completion", &TransportOptions::completion)
      .def_readwrite("fuse_flags", &TransportOptions::fuseFlags)
      .def_readwrite("wait_timeout", &TransportOptions::waitTimeout)
      .def_readwrite("fake_remote_axes", &TransportOptions::fakeRemoteAxes)
      .def_readwrite("ipc_probe", &TransportOptions::ipcProbe)
      .def_readwrite("fail_ipc_probe", &TransportOptions::failIpcProbe)
      .def_readwrite("fail_rccl_init", &TransportOptions::failRcclInit)
      .def_readwrite("stall_rccl_init_rank", &TransportOptions::stallRcclInitRank)
      .def_readwrite("fail_probe_rank", &TransportOptions::failProbeRank)
      .def_readwrite("peer_api_same_device", &TransportOptions::peerApiSameDevice)
      .def_readwrite("jitter_us", &TransportOptions::jitterUs)
      .def_readwrite("spin_wait", &TransportOptions::spinWait)
      .def_readwrite("numa_affinity", &TransportOptions::numaAffinity)
      .def_readwrite("x_face_sectors", &TransportOptions::xFaceSectors)
      .def_readwrite("x_face_lines_auto_bytes", &TransportOptions::xFaceLinesAutoBytes)
      .def_readwrite("null_stream_producers", &TransportOptions::nullStreamProducers)
      .def("__repr__", [](const TransportOptions &o) {
        return std::string("TransportOptions(inbox=") + to_string(o.inbox) + ", colo_copy=" + to_string(o.coloCopy) +
               ", peer_copy=" + to_string(o.peerCopy) + ", completion=" + to_string(o.completion) +
               ", wait_timeout=" + std::to_string(o.waitTimeout) + ")";
      });
  m.def("build_info", []() {
    const BuildInfo &b = build_info();
    py::dict d;
    d["git_sha"] = b.gitSha;
    d["use_rccl"] = b.useRccl;
    d["setup_stats"] = b.setupStats;
    d["exchange_stats"] = b.exchangeStats;
    d["output_level"] = b.outputLevel;
    d["offload_arch"] = b.offloadArch;
    return d;
  });
  m.def("build_info_string", &build_info_string);
  m.def("rccl_compiled", &rccl::compiled);
  // host wait policy of this process's HIP device contexts (hipSetDeviceFlags): call before the process first uses
  // the GPU. "spin" busy-waits in synchronize (lowest wake-up latency), "yield", "blocking", "auto" (HIP default)
  m.def("set_device_schedule", [](const std::string &mode) {
    unsigned f = hipDeviceScheduleAuto;
    if (mode == "spin")
      f = hipDeviceScheduleSpin;
    else if (mode == "yield")
      f = hipDeviceScheduleYield;
    else if (mode == "blocking")
      f = hipDeviceScheduleBlockingSync;
    else if (mode != "auto")
      throw std::invalid_argument("schedule mode " + mode);
    const hipError_t e = hipSetDeviceFlags(f);
    if (e != hipSuccess) (void)hipGetLastError();
    return std::string(e == hipSuccess ? "" : hipGetErrorString(e));
  });

  py::class_<ExchangePlanEntry>(m, "ExchangePlanEntry")
      .def_readonly("method", &ExchangePlanEntry::method)
      .def_readonly("src_idx", &ExchangePlanEntry::srcIdx)
      .def_readonly("dst_idx", &ExchangePlanEntry::dstIdx)
      .def_readonly("src_rank", &ExchangePlanEntry::srcRank)
      .def_readonly("dst_rank", &ExchangePlanEntry::dstRank)
      .def_readonly("src_dev", &ExchangePlanEntry::srcDev)
      .def_readonly("dst_dev", &ExchangePlanEntry::dstDev)
      .def_readonly("dir", &ExchangePlanEntry::dir)
      .def_readonly("bytes", &ExchangePlanEntry::bytes);

  py::class_<DistributedDomain, std::shared_ptr<DistributedDomain>>(m, "DistributedDomain")
      .def(py::init([](int64_t x, int64_t y, int64_t z, std::shared_ptr<comm::ProcGroup> pg) {
             py::gil_scoped_release r;
             return std::make_shared<DistributedDomain>(x, y, z, pg);
           }),
           py::arg("x"), py::arg("y"), py::arg("z"), py::arg("group") = nullptr)
      .def("set_radius", py::overload_cast<int64_t>(&DistributedDomain::set_radius))
      .def("set_radius", py::overload_cast<const Radius &>(&DistributedDomain::set_radius))
      .def("set_boundary", &DistributedDomain::set_boundary)
      .def("boundary", &DistributedDomain::boundary)
      .def("radius", &DistributedDomain::radius)
      .def("add_data",
           [](DistributedDomain &d, int64_t es, const std::string &name, DType dt) { return d.add_data(es, name, dt); },
           py::arg("elem_size"), py::arg("name") = "", py::arg("dtype") = DType::Bytes)
      .def("set_methods", &DistributedDomain::set_methods)
      .def("methods", &DistributedDomain::methods)
      .def("set_placement", &DistributedDomain::set_placement)
      .def("set_axis_cost", &DistributedDomain::set_axis_cost)
      .def("set_partition_objective", &DistributedDomain::set_partition_objective)
      .def("partition_objective", &DistributedDomain::partition_objective)
      .def("set_comm_max_blocks", &DistributedDomain::set_comm_max_blocks)
      .def("set_gpus", &DistributedDomain::set_gpus)
      .def("gpus", &DistributedDomain::gpus)
      .def("set_backend", &DistributedDomain::set_backend)
      .def("backend", &DistributedDomain::backend)
      .def("set_plan_file", &DistributedDomain::set_plan_file)
      .def("set_padding", &DistributedDomain::set_padding)
      .def("set_x_halo_align", &DistributedDomain::set_x_halo_align)
      .def("set_shared_halo_line", &DistributedDomain::set_shared_halo_line)
      .def("shared_halo_line", &DistributedDomain::shared_halo_line)
      .def("x_halo_align", &DistributedDomain::x_halo_align)
      .def("set_interior_align", &DistributedDomain::set_interior_align)
      .def("set_row_pad_lines", &DistributedDomain::set_row_pad_lines)
      .def("interior_align", &DistributedDomain::interior_align)
      .def("set_transport_options", &DistributedDomain::set_transport_options)
      .def("transport_options", &DistributedDomain::transport_options)
      .def("set_colo_copy", &DistributedDomain::set_colo_copy, py::call_guard<py::gil_scoped_release>())
      .def("set_completion", &DistributedDomain::set_completion, py::call_guard<py::gil_scoped_release>())
      .def("set_spin_wait", [](DistributedDomain &d, bool on) {
        TransportOptions o = d.transport_options();
        o.spinWait = on;
        d.set_transport_options_live(o);
      })
      .def("set_transport_options_live", &DistributedDomain::set_transport_options_live,
           py::call_guard<py::gil_scoped_release>())
      .def("set_null_stream_producers", [](DistributedDomain &d, bool on) {
        TransportOptions o = d.transport_options();
        o.nullStreamProducers = on;
        d.set_transport_options_live(o);
      })
      .def("set_transport_log", &DistributedDomain::set_transport_log, py::call_guard<py::gil_scoped_release>())
      .def("transport_log", &DistributedDomain::transport_log, py::arg("dev") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("poisoned", &DistributedDomain::poisoned)
      .def("numa_node", &DistributedDomain::numa_node)
      .def("set_self_test", &DistributedDomain::set_self_test)
      .def("self_test_report", &DistributedDomain::self_test_report)
      .def("rccl_status", &DistributedDomain::rccl_status)
      .def("probe_transports", &DistributedDomain::probe_transports, py::call_guard<py::gil_scoped_release>())
      .def_readwrite("exchange_stats", &DistributedDomain::exchangeStats_)
      .def("realize", &DistributedDomain::realize, py::call_guard<py::gil_scoped_release>())
      .def("realized", &DistributedDomain::realized)
      .def("size", &DistributedDomain::size)
      .def("rank", &DistributedDomain::rank)
      .def("world_size", &DistributedDomain::world_size)
      .def("num_domains", [](DistributedDomain &d) { return d.domains().size(); })
      .def("domain", [](DistributedDomain &d, size_t i) -> LocalDomain & { return d.domains().at(i); },
           py::return_value_policy::reference_internal)
      .def("get_origin", &DistributedDomain::get_origin)
      .def("get_compute_region", &DistributedDomain::get_compute_region)
      .def("get_interior", &DistributedDomain::get_interior)
      .def("get_local_interior", &DistributedDomain::get_local_interior, py::arg("reach") = 2)
      .def("get_exterior", &DistributedDomain::get_exterior)
      .def("subdomain_idx", &DistributedDomain::subdomain_idx)
      .def("placement_dim", [](DistributedDomain &d) { return d.placement().dim(); })
      .def("exchange_bytes_for_method", &DistributedDomain::exchange_bytes_for_method)
      .def("plan", &DistributedDomain::plan)
      .def("plan_summary", &DistributedDomain::plan_summary)
      .def("exchange", &DistributedDomain::exchange, py::call_guard<py::gil_scoped_release>())
      .def("exchange_async",
           [](DistributedDomain &d, uintptr_t s, int skip) { d.exchange_async(reinterpret_cast<hipStream_t>(s), skip); },
           py::arg("stream") = 0, py::arg("skip_axes") = 0, py::call_guard<py::gil_scoped_release>())
      .def("self_wrap_axes", &DistributedDomain::self_wrap_axes)
      .def("prepare_skip_wrapped", &DistributedDomain::prepare_skip_wrapped)
      .def("sync_exchange", &DistributedDomain::sync_exchange, py::call_guard<py::gil_scoped_release>())
      .def("record_ready",
           [](DistributedDomain &d, size_t di, uintptr_t s) { d.record_ready(di, reinterpret_cast<hipStream_t>(s)); })
      .def("wait_exchange",
           [](DistributedDomain &d, size_t di, uintptr_t s) { d.wait_exchange(di, reinterpret_cast<hipStream_t>(s)); })
      .def("comm_stream", [](DistributedDomain &d, size_t di) { return reinterpret_cast<uintptr_t>(d.comm_stream(di)); })
      .def("swap", &DistributedDomain::swap)
      .def("write_paraview", &DistributedDomain::write_paraview, py::arg("prefix"), py::arg("zero_nans") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("save_checkpoint", &DistributedDomain::save_checkpoint, py::call_guard<py::gil_scoped_release>())
      .def("load_checkpoint", &DistributedDomain::load_checkpoint, py::call_guard<py::gil_scoped_release>())
      .def("dlpack",
           [](std::shared_ptr<DistributedDomain> self, size_t di, int64_t q, bool curr) {
             return make_capsule(self, self->domains().at(di), q, curr);
           },
           py::arg("domain"), py::arg("qi"), py::arg("curr") = true)
      .def_property_readonly("timers", [](DistributedDomain &d) {
        py::dict t;
        t["mpi_topo"] = d.timeMpiTopo_;
        t["node_gpus"] = d.timeNodeGpus_;
        t["peer_en"] = d.timePeerEn_;
        t["placement"] = d.timePlacement_;
        t["plan"] = d.timePlan_;
        t["realize"] = d.timeRealize_;
        t["create"] = d.timeCreate_;
        t["exchange"] = d.timeExchange_;
        t["swap"] = d.timeSwap_;
        return t;
      });

  // ---------------- kernels ----------------
  m.def("stencil7_apply",
        [](DistributedDomain &dd, size_t di, int64_t q, const Rect3 &region, StencilKind kind, bool spheres,
           uintptr_t stream) {
          const Spheres s = spheres ? Spheres::jacobi(dd.get_compute_region()) : Spheres();
          stencil7_apply(dd.domains().at(di), q, region, kind, s, reinterpret_cast<hipStream_t>(stream));
        },
        py::arg("dd"), py::arg("domain"), py::arg("qi"), py::arg("region"), py::arg("kind"), py::arg("spheres"),
        py::arg("stream") = 0);
  m.def(
      "stencil7x3_apply",
      [](DistributedDomain &dd, size_t di, int64_t q, StencilKind kind, bool spheres, uintptr_t stream,
         const StencilTune &tune) {
        // one fused triple over the sub-domain's compute region (tune.wrap: the axes read in-kernel; 0 = every x / y /
        // z neighbour from the halos); false where stencil7x3_supported refuses
        const Spheres s = spheres ? Spheres::jacobi(dd.get_compute_region()) : Spheres();
        const LocalDomain &d = dd.domains().at(di);
        return stencil7x3_apply(d, q, d.get_compute_region(), kind, s, reinterpret_cast<hipStream_t>(stream), tune);
      },
      py::arg("dd"), py::arg("domain"), py::arg("qi"), py::arg("kind"), py::arg("spheres"), py::arg("stream"),
      py::arg("tune"), py::call_guard<py::gil_scoped_release>());
  m.def("stencil7x2_supported",
        [](DistributedDomain &dd, size_t di, int64_t q) { return stencil7x2_supported(dd.domains().at(di), q); },
        py::arg("dd"), py::arg("domain"), py::arg("qi"));
  m.def("stencil7x2_apply",
        [](DistributedDomain &dd, size_t di, int64_t q, const Rect3 &region, StencilKind kind, bool spheres,
           uintptr_t stream, const StencilTune &tune) {
          STENCIL_REQUIRE(stencil7x2_supported(dd.domains().at(di), q),
                          "fused pairs need a device fp32/fp64 quantity, face radii >= 2 and the aligned layout");
          const Spheres s = spheres ? Spheres::jacobi(dd.get_compute_region()) : Spheres();
          stencil7x2_apply(dd.domains().at(di), q, region, kind, s, reinterpret_cast<hipStream_t>(stream), tune);
        },
        py::arg("dd"), py::arg("domain"), py::arg("qi"), py::arg("region"), py::arg("kind"), py::arg("spheres"),
        py::arg("stream"), py::arg("tune"), py::call_guard<py::gil_scoped_release>());
  py::class_<X3PlanInfo>(m, "X3PlanInfo")
      .def_readonly("parts", &X3PlanInfo::parts)
      .def_readonly("blocks", &X3PlanInfo::blocks)
      .def_readonly("groups", &X3PlanInfo::groups)
      .def_readonly("lockstep_groups", &X3PlanInfo::lockstepGroups)
      .def_readonly("rounds", &X3PlanInfo::rounds)
      .def_readonly("tabled", &X3PlanInfo::tabled)
      .def_readonly("steps", &X3PlanInfo::steps)
      .def_readonly("zb", &X3PlanInfo::zb)
      .def_readonly("l0", &X3PlanInfo::l0)
      .def_readonly("l1", &X3PlanInfo::l1)
      .def_readonly("odd", &X3PlanInfo::odd);
  m.def(
      "stencil7x3_plan",
      [](py::handle size, bool jacobi, py::object tune, int slots) {
        return stencil7x3_plan(to_dim3(size), jacobi, tune.is_none() ? StencilTune() : tune.cast<StencilTune>(), slots);
      },
      py::arg("size"), py::arg("jacobi"), py::arg("tune") = py::none(), py::arg("slots") = 256);
  m.def(
      "x2_lockstep_schedule",
      [](int64_t slots, int64_t cols, int64_t nz) {
        const X2Schedule r = x2_lockstep_schedule(slots, cols, nz);
        return py::make_tuple(r.parts, r.blocks, r.rounds);
      },
      py::arg("slots"), py::arg("cols"), py::arg("nz"),
      "lockstep schedule of the whole-row / two-chunk-column fused pairs: (z parts per row group, blocks, rounds of "
      "whole columns); (0, 0, 1) = balanced split");
  m.def("jacobi_spheres", [](const Rect3 &cReg) {
    Spheres s = Spheres::jacobi(cReg);
    return py::make_tuple(s.hot, s.cold, s.radius);
  });

  // ---------------- models ----------------
  py::class_<StencilTune>(m, "StencilTune")
      .def(py::init<>())
      .def_readwrite("variant", &StencilTune::variant)
      .def_readwrite("ty", &StencilTune::ty)
      .def_readwrite("zchunk", &StencilTune::zchunk)
      .def_readwrite("xcd_remap", &StencilTune::xcdRemap)
      .def_readwrite("nontemporal", &StencilTune::nontemporal)
      .def_readwrite("alternate_z", &StencilTune::alternateZ)
      .def_readwrite("nw", &StencilTune::nw)
      .def_readwrite("x3sched", &StencilTune::x3sched)
      .def_readwrite("x2early", &StencilTune::x2early)
      .def_readwrite("x3parts", &StencilTune::x3parts)
      .def_readwrite("x3sphw", &StencilTune::x3sphw)
      .def_readwrite("x3sphchunk", &StencilTune::x3sphchunk)
      .def_readwrite("x3left", &StencilTune::x3left)
      .def_readwrite("x2sphw", &StencilTune::x2sphw)
      .def_property(
          "block_clock", [](const StencilTune &t) { return reinterpret_cast<uintptr_t>(t.blockClock); },
          [](StencilTune &t, uintptr_t p) { t.blockClock = reinterpret_cast<uint64_t *>(p); })
      .def_readwrite("x2row", &StencilTune::x2row)
      .def_readwrite("x2sched", &StencilTune::x2sched)
      .def_readwrite("x2reserve", &StencilTune::x2reserve)
      .def_readwrite("wrap", &StencilTune::wrap)
      .def_readwrite("x2lockstep", &StencilTune::x2lockstep)
      .def_readwrite("zslab_row", &StencilTune::zslabRow)
      .def_readwrite("x2xfast", &StencilTune::x2xfast);
  py::class_<StencilModelConfig>(m, "StencilModelConfig")
      .def(py::init<>())
      .def_readwrite("size", &StencilModelConfig::size)
      .def_readwrite("kind", &StencilModelConfig::kind)
      .def_readwrite("radius", &StencilModelConfig::radius)
      .def_readwrite("all_directions", &StencilModelConfig::allDirections)
      .def_readwrite("quantities", &StencilModelConfig::quantities)
      .def_readwrite("fp64", &StencilModelConfig::fp64)
      .def_readwrite("methods", &StencilModelConfig::methods)
      .def_readwrite("placement", &StencilModelConfig::placement)
      .def_readwrite("axis_cost", &StencilModelConfig::axisCost)
      .def_readwrite("partition", &StencilModelConfig::partition)
      .def_readwrite("gpus", &StencilModelConfig::gpus)
      .def_readwrite("overlap", &StencilModelConfig::overlap)
      .def_readwrite("auto_overlap", &StencilModelConfig::autoOverlap)
      .def_readwrite("use_graph", &StencilModelConfig::useGraph)
      .def_readwrite("forward", &StencilModelConfig::forward)
      .def_readwrite("temporal", &StencilModelConfig::temporal)
      .def_readwrite("wrap_self", &StencilModelConfig::wrapSelf)
      .def_readwrite("x_halo_align", &StencilModelConfig::xHaloAlign)
      .def_readwrite("shared_halo_line", &StencilModelConfig::sharedHaloLine)
      .def_readwrite("interior_align", &StencilModelConfig::interiorAlign)
      .def_readwrite("row_pad_lines", &StencilModelConfig::rowPadLines)
      .def_readwrite("wrap_axes_mask", &StencilModelConfig::wrapAxesMask)
      .def_readwrite("local_interior", &StencilModelConfig::localInterior)
      .def_readwrite("overlap_mode", &StencilModelConfig::overlapMode)
      .def_readwrite("transport", &StencilModelConfig::transport)
      .def_readwrite("self_test", &StencilModelConfig::selfTest)
      .def_property(
          "backend", [](const StencilModelConfig &c) { return c.backend; },
          [](StencilModelConfig &c, Backend b) {
            c.backend = b;
            c.setBackend = true;
          })
      .def_readwrite("tune", &StencilModelConfig::tune)
      .def_readwrite("astaroth_period", &StencilModelConfig::astarothPeriod);
  py::class_<StencilModel, std::shared_ptr<StencilModel>>(m, "StencilModel")
      .def(py::init([](const StencilModelConfig &c, std::shared_ptr<comm::ProcGroup> pg) {
             py::gil_scoped_release r;
             return std::make_shared<StencilModel>(c, pg);
           }),
           py::arg("config"), py::arg("group") = nullptr)
      .def("init", &StencilModel::init, py::call_guard<py::gil_scoped_release>())
      .def("step", &StencilModel::step, py::call_guard<py::gil_scoped_release>())
      .def("run", &StencilModel::run, py::call_guard<py::gil_scoped_release>())
      .def("prepare", &StencilModel::prepare, py::arg("runs") = std::vector<int>{},
           py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &StencilModel::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("cells", &StencilModel::cells)
      .def("local_cells", &StencilModel::local_cells)
      .def("steps_done", &StencilModel::steps_done)
      .def("overlapping", &StencilModel::overlapping)
      .def("can_toggle_overlap", &StencilModel::can_toggle_overlap)
      .def("set_overlap_mode", &StencilModel::set_overlap_mode, py::call_guard<py::gil_scoped_release>())
      .def("overlap_mode", &StencilModel::overlap_mode)
      .def("can_pipeline", &StencilModel::can_pipeline)
      .def("can_pipeline_triples", &StencilModel::can_pipeline_triples)
      .def("set_comm_reserve", &StencilModel::set_comm_reserve, py::call_guard<py::gil_scoped_release>())
      .def("set_triple_schedule", &StencilModel::set_triple_schedule, py::arg("sphw"), py::arg("left"),
           py::arg("parts"), py::call_guard<py::gil_scoped_release>())
      .def("comm_reserve", &StencilModel::comm_reserve)
      .def("set_overlap", &StencilModel::set_overlap, py::call_guard<py::gil_scoped_release>())
      .def("local_interior_steps", &StencilModel::local_interior_steps)
      .def("forwarding", &StencilModel::forwarding)
      .def("temporal_blocking", &StencilModel::temporal_blocking)
      .def("temporal_triples", &StencilModel::temporal_triples)
      .def("wrap_axes", &StencilModel::wrap_axes)
      .def("step_wrap_axes", &StencilModel::step_wrap_axes)
      .def("compute_stream", [](StencilModel &mdl, size_t di) { return reinterpret_cast<uintptr_t>(mdl.compute_stream(di)); })
      .def("domain",
           [](std::shared_ptr<StencilModel> mdl) {
             // aliasing shared_ptr: the DistributedDomain lives as long as the model
             return std::shared_ptr<DistributedDomain>(mdl, &mdl->domain());
           });
}
