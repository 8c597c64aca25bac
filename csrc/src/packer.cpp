// Message packing (see stencil/domain/packer.hpp).
#include "stencil/domain/packer.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>

#include "stencil/rt/hip_check.hpp"

namespace stencil {

static StridedBox dense_box(char *base, const Dim3 &ext, int64_t es) {
  StridedBox b;
  b.base = base;
  b.ystride = ext.x * es;
  b.zstride = ext.x * ext.y * es;
  return b;
}

int64_t packed_size(const LocalDomain &dom, const std::vector<Message> &msgs) {
  int64_t off = 0;
  for (const auto &m : msgs)
    for (int64_t q = 0; q < dom.num_data(); ++q) {
      off = round_up(off, dom.elem_size(q));
      off += dom.halo_bytes(-m.dir, q);
    }
  return off;
}

int64_t packed_message_bytes(const LocalDomain &dom, std::vector<Dim3> dirs) {
  std::sort(dirs.begin(), dirs.end());
  std::vector<Message> msgs;
  for (auto &d : dirs) msgs.push_back(Message{d, 0, 0});
  return packed_size(dom, msgs);
}

// pack: interior slab on the `dir` side -> dense buffer. `curr`: which physical buffer is "curr" in this variant.
void build_pack_segs(const LocalDomain &dom, const std::vector<Message> &msgs, char *buf, bool curr,
                       std::vector<CopySeg> &out) {
  int64_t off = 0;
  for (const auto &m : msgs)
    for (int64_t q = 0; q < dom.num_data(); ++q) {
      const int64_t es = dom.elem_size(q);
      off = round_up(off, es);
      const Dim3 ext = dom.halo_extent(-m.dir);
      out.push_back(make_copy_seg(dom.box(q, curr, dom.halo_pos(m.dir, false)), dense_box(buf + off, ext, es), ext, es));
      off += es * ext.flatten();
    }
}

// unpack: dense buffer -> the -dir halo (message sent along dir lands on our -dir side)
void build_unpack_segs(const LocalDomain &dom, const std::vector<Message> &msgs, char *buf, bool curr,
                         std::vector<CopySeg> &out) {
  int64_t off = 0;
  for (const auto &m : msgs)
    for (int64_t q = 0; q < dom.num_data(); ++q) {
      const int64_t es = dom.elem_size(q);
      off = round_up(off, es);
      const Dim3 ext = dom.halo_extent(-m.dir);
      out.push_back(make_copy_seg(dense_box(buf + off, ext, es), dom.box(q, curr, dom.halo_pos(-m.dir, true)), ext, es));
      off += es * ext.flatten();
    }
}

// An x face (dir = (+-1, 0, 0)) is a strided column of w-cell row pieces: each row touches one line of the source
// and one of the receiver, the latter only partly written. Widened to whole interior-alignment units (S = 128 B / element
// with the default 128-B interior alignment: whole L2 lines; 64 B: sectors) the copy reads the same lines and writes
// whole ones (the extra S - w cells land in the receiver's x padding in front of its -x halo or behind its +x halo,
// which nothing reads). Needs both rows aligned at the interior (the padded layout), interiors a multiple of S long
// and at least S long, and room for the unit in the receiver's row.
static bool widen_x_face(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, int64_t q, Dim3 *sp, Dim3 *dp,
                         Dim3 *ext) {
  if (dir.y != 0 || dir.z != 0 || dir.x == 0) return false;
  const int64_t es = src.elem_size(q);
  const int64_t unit = std::min(src.interior_align(), dst.interior_align());
  // shared halo lines: the unit behind / in front of a row holds the neighbour row's halo too -- never widen into it
  if (es != dst.elem_size(q) || unit % es != 0 || src.x_halo_align() || dst.x_halo_align() || dst.shared_halo_line())
    return false;
  const int64_t S = unit / es, w = ext->x;
  if (w > S || src.size().x % S || dst.size().x % S || src.size().x < S) return false;
  const int64_t srxm = src.radius().x(-1), drxm = dst.radius().x(-1);
  if ((src.pad_x(q) + srxm) % S || (dst.pad_x(q) + drxm) % S) return false; // interiors not sector aligned
  const int64_t dRowEnd = dst.pitch(q).x - dst.pad_x(q);                      // raw x one past the dst row
  if (dir.x > 0) { // +x face -> the receiver's -x halo: sector [nx - S, nx) -> [-S, 0) (global x)
    sp->x -= S - w;
    dp->x -= S - w;
    if (dp->x < -dst.pad_x(q)) return false;
  } else { // -x face -> the receiver's +x halo: [0, S) -> [nx, nx + S)
    if (dp->x + S > dRowEnd) return false;
  }
  ext->x = S;
  return true;
}

// direct translate src interior slab -> dst halo (same process)
void build_translate_segs_q(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, bool curr, int64_t q,
                            std::vector<CopySeg> &out, bool xSectors) {
  const int64_t es = src.elem_size(q);
  Dim3 ext = src.halo_extent(-dir);
  Dim3 sp = src.halo_pos(dir, false), dp = dst.halo_pos(-dir, true);
  Dim3 wsp = sp, wdp = dp, wext = ext;
  const bool wide = xSectors && widen_x_face(src, dst, dir, q, &wsp, &wdp, &wext);
  if (wide) {
    sp = wsp;
    dp = wdp;
    ext = wext;
  }
  if (!wide && dst.shared_halo_line() && dir.x != 0 && dir.y == 0 && dir.z == 0 && ext.y > 1) {
    // shared halo lines: row y's +x halo (written by the dir = -x translate) and row y+1's -x halo (dir = +x) are one
    // line. Split off the row without a partner in this face (the last row of the +x halo column, the first of the
    // -x one) so the remaining rows of the two faces have the same shape and make_copy_plan pairs them row by row:
    // one item then writes both halos of a line (one written line per row instead of two)
    const int64_t lone = dir.x < 0 ? ext.y - 1 : 0, first = dir.x < 0 ? 0 : 1;
    const Dim3 e1(ext.x, ext.y - 1, ext.z), e2(ext.x, 1, ext.z);
    out.push_back(make_copy_seg(src.box(q, curr, sp + Dim3(0, first, 0)), dst.box(q, curr, dp + Dim3(0, first, 0)), e1, es));
    out.push_back(make_copy_seg(src.box(q, curr, sp + Dim3(0, lone, 0)), dst.box(q, curr, dp + Dim3(0, lone, 0)), e2, es));
    return;
  }
  CopySeg sg = make_copy_seg(src.box(q, curr, sp), dst.box(q, curr, dp), ext, es);
  if (wide && sg.vec == 16) sg.flags |= kSegWide;
  out.push_back(sg);
}

void build_translate_segs(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, bool curr,
                          std::vector<CopySeg> &out, bool xSectors) {
  for (int64_t q = 0; q < src.num_data(); ++q) build_translate_segs_q(src, dst, dir, curr, q, out, xSectors);
}


PackerBase::~PackerBase() {
  for (auto &p : plan_) free_copy_plan(p);
  if (buf_) {
    if (device_)
      (void)hipFree(buf_);
    else
      std::free(buf_);
  }
}

void PackerBase::prepare_impl(LocalDomain *dom, std::vector<Message> msgs, bool pack) {
  STENCIL_REQUIRE(dom && dom->realized(), "Packer::prepare needs a realized LocalDomain");
  dom_ = dom;
  std::sort(msgs.begin(), msgs.end());
  msgs_ = msgs;
  size_ = packed_size(*dom, msgs_);
  STENCIL_REQUIRE(size_ > 0, "zero-size packer was prepared");
  device_ = dom->backend() == Backend::Device;
  if (device_) {
    dom->set_device();
    HIP_CHECK(hipMalloc(&buf_, size_t(size_)));
  } else {
    buf_ = static_cast<char *>(std::aligned_alloc(256, size_t(round_up(size_, 256))));
  }
  // variant p: "curr" is the buffer that is current after p swaps from the domain's present parity
  for (int p = 0; p < 2; ++p) {
    const bool currIsCurr = (p == dom->parity());
    segs_[p].clear();
    if (pack)
      build_pack_segs(*dom, msgs_, buf_, currIsCurr, segs_[p]);
    else
      build_unpack_segs(*dom, msgs_, buf_, currIsCurr, segs_[p]);
    finalize_segs(segs_[p]);
    if (device_) plan_[p] = make_copy_plan(segs_[p], dom->gpu());
  }
}

void PackerBase::run() {
  const int p = dom_->parity();
  if (device_) {
    dom_->set_device();
    copy_plan_device(plan_[p], stream_);
  } else {
    copy_segs_host(segs_[p]);
  }
}

} // namespace stencil
