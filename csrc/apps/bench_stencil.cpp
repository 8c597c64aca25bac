// Compute-kernel micro-benchmark: the 7-point Jacobi update on one MI355X against the HBM streaming roofline.
// No reference counterpart as an app (the reference only cites kernel times, bin/astaroth_sim.cu:130-152); this is
// the tuning harness behind the Jacobi3D numbers in BASELINE.md.
// Prints CSV `kernel,variant,ty,zc,us,gcells,eff_TBps` where eff_TBps counts the 8 B/cell minimum traffic.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

#include "stencil/domain/local_domain.hpp"
#include "stencil/domain/packer.hpp"
#include "stencil/kernels/stencil_ops.hpp"
#include "stencil/rt/argparse.hpp"
#include "stencil/rt/stream.hpp"

using namespace stencil;

// streaming roofline: dst = src over n float4, non-temporal stores, grid-stride
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_copy(const f4 *__restrict__ src, f4 *__restrict__ dst, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    f4 v = src[i];
    __builtin_nontemporal_store(v, dst + i);
  }
}
// U independent 16-B loads in flight per lane, contiguous block-sized tiles (each block owns a chunk)
template <int U>
__global__ __launch_bounds__(256) void stream_copy_tiles(const f4 *__restrict__ src, f4 *__restrict__ dst, int64_t n) {
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t beg = int64_t(blockIdx.x) * per, end = beg + per < n ? beg + per : n;
  for (int64_t i = beg + threadIdx.x; i < end; i += 256 * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < end) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < end) __builtin_nontemporal_store(v[u], dst + i + u * 256);
  }
}
// read-only and write-only streams (the two halves of the roofline)
__global__ __launch_bounds__(256) void stream_read(const f4 *__restrict__ src, float *__restrict__ sink, int64_t n) {
  f4 acc = {0, 0, 0, 0};
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) acc += src[i];
  if (acc.x == 1234.5f) sink[0] = acc.y + acc.z + acc.w;
}
__global__ __launch_bounds__(256) void stream_write(f4 *__restrict__ dst, int64_t n) {
  const f4 v = {1, 2, 3, 4};
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
    __builtin_nontemporal_store(v, dst + i);
}

int main(int argc, char **argv) {
  int64_t n = 512;
  int iters = 20, reps = 1;
  std::string only;
  ArgParser p("7-point stencil kernel sweep on one GPU");
  p.option(&n, "--n", "cube edge").option(&iters, "--iters", "timed launches per config")
      .option(&reps, "--reps", "repetitions of the whole sweep (interleaved)")
      .option(&only, "--only", "run only 'lds', 'reg' or 'copy'");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  std::setvbuf(stdout, nullptr, _IOLBF, 0); // progress lines reach a redirected log as they are printed
  LocalDomain ld(Dim3(n, n, n), Dim3(0, 0, 0), 0, Backend::Device);
  ld.set_radius(1);
  ld.add_data<float>("d");
  ld.realize();
  Stream s(0);
  const Rect3 reg = ld.get_compute_region();
  const Spheres sph = Spheres::jacobi(reg);
  jacobi_init(ld, 0, ld.get_full_region(), s);
  s.sync();
  const double cells = double(n) * n * n;

  auto timeit = [&](auto &&fn) {
    for (int i = 0; i < 3; ++i) fn();
    Event a(0, true), b(0, true);
    a.record(s);
    for (int i = 0; i < iters; ++i) fn();
    b.record(s);
    b.sync();
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return double(ms) * 1e3 / iters; // us
  };
  std::printf("kernel,variant,ty,zc,us,gcells,eff_TBps\n");
  if (only.empty() || only == "copy") {
    const int64_t nv = int64_t(n) * n * n / 4;
    for (int blocks : {1024, 2048, 4096, 8192}) {
      const double us = timeit([&] {
        hipLaunchKernelGGL(stream_copy, dim3(blocks), dim3(256), 0, s, (const f4 *)ld.curr_data(0),
                           (f4 *)ld.next_data(0), nv);
      });
      std::printf("copy,%d,0,0,%.2f,%.1f,%.3f\n", blocks, us, cells / us / 1e3, cells * 8 / us / 1e6);
    }
    for (int blocks : {512, 1024, 2048}) {
      const double us4 = timeit([&] {
        hipLaunchKernelGGL(stream_copy_tiles<4>, dim3(blocks), dim3(256), 0, s, (const f4 *)ld.curr_data(0),
                           (f4 *)ld.next_data(0), nv);
      });
      std::printf("copy_tiles4,%d,0,0,%.2f,%.1f,%.3f\n", blocks, us4, cells / us4 / 1e3, cells * 8 / us4 / 1e6);
      const double usr = timeit([&] {
        hipLaunchKernelGGL(stream_read, dim3(blocks), dim3(256), 0, s, (const f4 *)ld.curr_data(0),
                           (float *)ld.next_data(0), nv);
      });
      std::printf("read_only,%d,0,0,%.2f,%.1f,%.3f\n", blocks, usr, cells / usr / 1e3, cells * 4 / usr / 1e6);
      const double usw = timeit([&] {
        hipLaunchKernelGGL(stream_write, dim3(blocks), dim3(256), 0, s, (f4 *)ld.next_data(0), nv);
      });
      std::printf("write_only,%d,0,0,%.2f,%.1f,%.3f\n", blocks, usw, cells / usw / 1e3, cells * 4 / usw / 1e6);
    }
  }
  struct Cfg {
    int variant, ty, zc, nw = 8;
  };
  std::vector<Cfg> cfgs;
  if (only.empty() || only == "lds")
    for (int ty : {2, 4, 8})
      for (int zc : {0, 8, 16, 32, 64}) cfgs.push_back({0, ty, zc});
  if (only.empty() || only == "deep" || only == "lds")
    for (int pf : {2, 3})
      for (int nw : {4, 8, 16})
        for (int zc : {0, 32, 64}) cfgs.push_back({pf, 2, zc, nw});
  if (only.empty() || only == "reg")
    for (int ty : {4, 8})
      for (int zc : {0, 16, 32}) cfgs.push_back({1, ty, zc});
  for (int rep = 0; rep < reps; ++rep)
  if (only.empty() || only == "xchg") {
    // the Kernel-transport exchange of a single self-wrapping sub-domain (one copy-plan launch), all faces and per axis
    const char *names[] = {"xchg_all", "xchg_x", "xchg_y", "xchg_z"};
    for (int mode = 0; mode < 4; ++mode) {
      std::vector<CopySeg> segs;
      for (int ax = 0; ax < 3; ++ax) {
        if (mode != 0 && mode != ax + 1) continue;
        for (int sgn = -1; sgn <= 1; sgn += 2) {
          Dim3 d(0, 0, 0);
          (ax == 0 ? d.x : ax == 1 ? d.y : d.z) = sgn;
          build_translate_segs(ld, ld, d, true, segs);
        }
      }
      finalize_segs(segs);
      CopyPlan cp = make_copy_plan(segs, 0);
      const double us = timeit([&] { copy_plan_device(cp, s); });
      std::printf("%s,0,0,0,%.2f,%.1f,%.3f\n", names[mode], us, double(cp.bytes) / us / 1e3, 2.0 * cp.bytes / us / 1e6);
      free_copy_plan(cp);
    }
  }
  for (int rep = 0; rep < reps; ++rep)
  if (only.empty() || only == "fwd") {
    // halo forwarding onto itself (periodic self-wrap of a single sub-domain): all faces, then each axis alone
    // fwd_xself: x messages stored onto the sender's own output cells (same lines as the main store): separates
    // the instruction cost of the x path from the cost of its scattered halo lines
    const char *names[] = {"fwd_all", "fwd_x", "fwd_y", "fwd_z", "fwd_xself"};
    for (int mode = 0; mode < 5; ++mode)
    for (int zc : {0, 16, 32, 64}) {
      std::vector<ForwardTarget> tg;
      for (int ax = 0; ax < 3; ++ax) {
        if (mode != 0 && mode != ax + 1 && !(mode == 4 && ax == 0)) continue;
        for (int sgn = -1; sgn <= 1; sgn += 2) {
          Dim3 d(0, 0, 0), off(0, 0, 0);
          (ax == 0 ? d.x : ax == 1 ? d.y : d.z) = sgn;
          (ax == 0 ? off.x : ax == 1 ? off.y : off.z) = mode == 4 ? 0 : -sgn * n;
          tg.push_back(ForwardTarget{d, &ld, off});
        }
      }
      HaloForwarder hf(ld, 0, tg);
      StencilTune t;
      t.zchunk = zc;
      const double us = timeit([&] { stencil7_apply(ld, 0, reg, StencilKind::Jacobi, sph, s, t, &hf); });
      std::printf("%s,0,2,%d,%.2f,%.1f,%.3f\n", names[mode], zc, us, cells / us / 1e3, cells * 8 / us / 1e6);
    }
  }
  for (int rep = 0; rep < reps; ++rep)
  if (only.empty() || only == "mfma") {
    // the matrix-core line update (x pair on MFMA) against the VALU single step on the same domain
    for (int zc : {0, 16, 64}) {
      StencilTune t;
      t.variant = StencilTune::kMfma;
      t.zchunk = zc;
      const double us = timeit([&] { stencil7_apply(ld, 0, reg, StencilKind::Jacobi, sph, s, t); });
      std::printf("stencil7_mfma,%d,0,%d,%.2f,%.1f,%.3f\n", StencilTune::kMfma, zc, us, cells / us / 1e3,
                  cells * 8 / us / 1e6);
    }
  }
  if (only == "one") {
    // one launch of each default kernel (single step v2, fused pair, MFMA variant) for counter collection
    StencilTune t;
    timeit([&] { stencil7_apply(ld, 0, reg, StencilKind::Jacobi, sph, s, t); });
    StencilTune tm;
    tm.variant = StencilTune::kMfma;
    timeit([&] { stencil7_apply(ld, 0, reg, StencilKind::Jacobi, sph, s, tm); });
    LocalDomain l2(Dim3(n, n, n), Dim3(0, 0, 0), 0, Backend::Device);
    l2.set_radius(Radius::face_edge_corner(2, 1, 0));
    l2.add_data<float>("d");
    l2.realize();
    jacobi_init(l2, 0, l2.get_full_region(), s);
    timeit([&] { stencil7x2_apply(l2, 0, l2.get_compute_region(), StencilKind::Jacobi, sph, s, t); });
    return 0;
  }
  for (int rep = 0; rep < reps; ++rep)
  if (only == "ext") {
    // overlapped fused pair pieces on a depth-2 domain: whole sweep, interior sweep, exterior (thin-slab kernels)
    LocalDomain l2(Dim3(n, n, n), Dim3(0, 0, 0), 0, Backend::Device);
    l2.set_radius(Radius::face_edge_corner(2, 1, 0));
    l2.add_data<float>("d");
    l2.realize();
    jacobi_init(l2, 0, l2.get_full_region(), s);
    s.sync();
    const Rect3 c = l2.get_compute_region();
    for (int sx : {2, 4}) {
    const Rect3 in(c.lo + Dim3(sx, 2, 2), c.hi - Dim3(sx, 2, 2));
    std::printf("# interior shrink x=%d\n", sx);
    StencilTune t;
    const double whole = timeit([&] { stencil7x2_apply(l2, 0, c, StencilKind::Jacobi, sph, s, t); });
    const double inner = timeit([&] { stencil7x2_apply(l2, 0, in, StencilKind::Jacobi, sph, s, t); });
    const double outer = timeit([&] { stencil7x2_apply_exterior(l2, 0, in, StencilKind::Jacobi, sph, s, t); });
    Stream s2(0, Priority::HIGH);
    Event e(0);
    const double both = timeit([&] {
      e.record(s);
      e.wait_on(s2);
      stencil7x2_apply_exterior(l2, 0, in, StencilKind::Jacobi, sph, s2, t);
      stencil7x2_apply(l2, 0, in, StencilKind::Jacobi, sph, s, t);
      e.record(s2);
      e.wait_on(s);
    });
    std::printf("x2_whole,0,0,0,%.2f,0,0\nx2_interior,0,0,0,%.2f,0,0\nx2_exterior,0,0,0,%.2f,0,0\nx2_int+ext_concurrent,0,0,0,%.2f,0,0\n",
                whole, inner, outer, both);
    }
  }
  for (int rep = 0; rep < reps; ++rep)
  if (only == "ovl") {
    // Remote-halo overlap of a fused pair on ONE GPU, the off-GPU link emulated by host-pinned memory (PCIe, about
    // as slow as one xGMI link): the z faces are "packed" into a pinned buffer, "unpacked" from a device buffer,
    // then the z slabs are computed. seq = pack + unpack + whole sweep on one stream (no overlap); ovl = pack ->
    // unpack -> z slabs on a high-priority stream while the z-shrunk interior sweep runs (reserve r CUs).
    // (CU-masked streams were tried as well: no faster, and one masked configuration hung the run.)
    LocalDomain l2(Dim3(n, n, n), Dim3(0, 0, 0), 0, Backend::Device);
    l2.set_radius(Radius::face_edge_corner(2, 1, 0));
    l2.add_data<float>("d");
    l2.realize();
    jacobi_init(l2, 0, l2.get_full_region(), s);
    s.sync();
    const Rect3 c = l2.get_compute_region();
    const Rect3 in(c.lo + Dim3(0, 0, 2), c.hi - Dim3(0, 0, 2));
    const Dim3 pch = l2.pitch(0);
    const int64_t faceBytes = 2 * pch.x * pch.y * 4; // two planes
    char *hostBuf = nullptr, *devBuf = nullptr;
    HIP_CHECK(hipHostMalloc((void **)&hostBuf, 2 * faceBytes, hipHostMallocDefault));
    HIP_CHECK(hipMalloc((void **)&devBuf, 2 * faceBytes));
    std::vector<CopySeg> packSegs, unpackSegs;
    char *cur = static_cast<char *>(l2.curr_data(0));
    const int64_t zlo = l2.radius().z(-1), nz = l2.size().z;
    for (int k = 0; k < 2; ++k) {
      const int64_t zs = k == 0 ? zlo : zlo + nz - 2;  // interior planes sent
      const int64_t zh = k == 0 ? zlo + nz : zlo - 2;  // halo planes received (periodic self)
      const Dim3 ext(faceBytes / 4, 1, 1);
      packSegs.push_back(make_copy_seg(StridedBox{cur + zs * pch.x * pch.y * 4, 0, 0},
                                       StridedBox{hostBuf + k * faceBytes, 0, 0}, ext, 4));
      unpackSegs.push_back(make_copy_seg(StridedBox{devBuf + k * faceBytes, 0, 0},
                                         StridedBox{cur + zh * pch.x * pch.y * 4, 0, 0}, ext, 4));
    }
    finalize_segs(packSegs);
    finalize_segs(unpackSegs);
    CopyPlan pk = make_copy_plan(packSegs, 0), up = make_copy_plan(unpackSegs, 0);
    StencilTune t;
    Stream hi(0, Priority::HIGH);
    Event e(0), e2(0);
    const double sweep = timeit([&] { stencil7x2_apply(l2, 0, c, StencilKind::Jacobi, sph, s, t); });
    const double packOnly = timeit([&] { copy_plan_device(pk, s); });
    const double seq = timeit([&] {
      copy_plan_device(pk, s);
      copy_plan_device(up, s);
      stencil7x2_apply(l2, 0, c, StencilKind::Jacobi, sph, s, t);
    });
    std::printf("ovl_sweep,0,0,0,%.2f,0,0\novl_pack_pinned,0,0,0,%.2f,0,0\novl_seq,0,0,0,%.2f,0,0\n", sweep, packOnly, seq);
    const double ext = timeit([&] { stencil7x2_apply_exterior(l2, 0, in, StencilKind::Jacobi, sph, s, t); });
    std::printf("ovl_zslabs_alone,0,0,0,%.2f,0,0\n", ext);
    // extAfter: the slabs run on the compute stream after the interior sweep (whole GPU) instead of on the comm
    // stream behind the unpack (few CUs while the sweep holds the rest)
    auto overlapped = [&](hipStream_t cs, hipStream_t ms, int reserve, bool extAfter = false, int lim = 0) {
      StencilTune ti = t;
      ti.reserveCUs = reserve;
      return timeit([&] {
        e.record(s);
        e.wait_on(ms);
        e.wait_on(cs);
        copy_plan_device(pk, ms, lim);
        copy_plan_device(up, ms, lim);
        if (!extAfter) stencil7x2_apply_exterior(l2, 0, in, StencilKind::Jacobi, sph, ms, t);
        stencil7x2_apply(l2, 0, in, StencilKind::Jacobi, sph, cs, ti);
        e2.record(ms);
        e2.wait_on(extAfter ? cs : s);
        if (extAfter) stencil7x2_apply_exterior(l2, 0, in, StencilKind::Jacobi, sph, cs, t);
        e.record(cs);
        e.wait_on(s);
      });
    };
    for (int r : {0, 8, 16})
      std::printf("ovl_reserve%d,0,0,0,%.2f,0,0\n", r, overlapped(s, hi, r));
    for (int r : {0, 4, 8, 16})
      std::printf("ovl_extafter_reserve%d,0,0,0,%.2f,0,0\n", r, overlapped(s, hi, r, true));
    // comm kernels confined to `lim` CUs (copy_plan_device maxBlocks) beside a sweep that leaves `r` CUs free
    for (int lim : {4, 8, 16})
      for (int r : {4, 8, 16}) {
        if (r < lim) continue;
        std::printf("ovl_lim%d_reserve%d,0,0,0,%.2f,0,0\n", lim, r, overlapped(s, hi, r, true, lim));
        std::printf("ovl_lim%d_reserve%d_extcomm,0,0,0,%.2f,0,0\n", lim, r, overlapped(s, hi, r, false, lim));
      }
    {
      const double p8 = timeit([&] { copy_plan_device(pk, s, 8); });
      std::printf("ovl_pack_pinned_lim8,0,0,0,%.2f,0,0\n", p8);
    }
    {
      StencilTune tc = t;
      tc.x2sched = 0; // fixed z-chunks (several rounds of blocks) instead of balanced segments
      const double ch = timeit([&] {
        e.record(s);
        e.wait_on(hi);
        copy_plan_device(pk, hi);
        copy_plan_device(up, hi);
        stencil7x2_apply(l2, 0, in, StencilKind::Jacobi, sph, s, tc);
        e2.record(hi);
        e2.wait_on(s);
        stencil7x2_apply_exterior(l2, 0, in, StencilKind::Jacobi, sph, s, t);
      });
      std::printf("ovl_extafter_chunks,0,0,0,%.2f,0,0\n", ch);
    }
    free_copy_plan(pk);
    free_copy_plan(up);
    HIP_CHECK(hipHostFree(hostBuf));
    HIP_CHECK(hipFree(devBuf));
  }
  for (int rep = 0; rep < reps; ++rep)
  if (only == "x2pp") {
    // the fused pair as the model runs it: ping-pong (swap after every launch), so every launch reads what the
    // previous one wrote; non-temporal stores and the alternating z-march on/off
    LocalDomain l2(Dim3(n, n, n), Dim3(0, 0, 0), 0, Backend::Device);
    l2.set_radius(Radius::face_edge_corner(2, 1, 0));
    l2.add_data<float>("d");
    l2.realize();
    const Rect3 reg2 = l2.get_compute_region();
    jacobi_init(l2, 0, l2.get_full_region(), s);
    fill_value(l2, 0, 0.5, false, s);
    s.sync();
    for (int zc : {-1, 0, 64, 128}) { // -1: fixed auto z-chunks (x2sched 0); 0: balanced segments
      const int nt = 1, alt = 1;
      StencilTune t;
      t.nontemporal = nt;
      t.alternateZ = alt;
      t.zchunk = zc < 0 ? 0 : zc;
      t.x2sched = zc < 0 ? 0 : 1;
      const double us = timeit([&] {
        stencil7x2_apply(l2, 0, reg2, StencilKind::Jacobi, sph, s, t);
        l2.swap();
      }) / 2;
      std::printf("x2pp_nt%d_alt%d,1,1,%d,%.2f,%.1f,%.3f,nw12\n", nt, alt, zc, us, cells / us / 1e3,
                  cells * 8 / us / 1e6);
    }
  }
  for (int rep = 0; rep < reps; ++rep)
  if (only.empty() || only == "x2") {
    // two fused steps per sweep (temporal blocking) on a depth-2 domain; reported per STEP (two steps per launch)
    LocalDomain l2(Dim3(n, n, n), Dim3(0, 0, 0), 0, Backend::Device);
    l2.set_radius(Radius::face_edge_corner(2, 1, 0));
    l2.add_data<float>("d");
    l2.realize();
    const Rect3 reg2 = l2.get_compute_region();
    jacobi_init(l2, 0, l2.get_full_region(), s);
    s.sync();
    for (int zc : {0, 43, 64, 128}) {
      StencilTune t;
      t.zchunk = zc;
      const double us = timeit([&] { stencil7x2_apply(l2, 0, reg2, StencilKind::Jacobi, sph, s, t); }) / 2;
      std::printf("stencil7x2,1,1,%d,%.2f,%.1f,%.3f,nw12\n", zc, us, cells / us / 1e3, cells * 8 / us / 1e6);
    }
  }
  for (int rep = 0; rep < reps; ++rep)
  for (const Cfg &c : cfgs) {
    StencilTune t;
    t.variant = c.variant;
    t.ty = c.ty;
    t.zchunk = c.zc;
    t.nw = c.nw;
    const double us = timeit([&] { stencil7_apply(ld, 0, reg, StencilKind::Jacobi, sph, s, t); });
    std::printf("stencil7,%d,%d,%d,%.2f,%.1f,%.3f,nw%d\n", c.variant, c.ty, c.zc, us, cells / us / 1e3,
                cells * 8 / us / 1e6, c.nw);
  }
  return 0;
}
